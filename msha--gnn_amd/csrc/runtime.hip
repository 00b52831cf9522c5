// ABI plumbing: version, thread-local error string, dropout mask export.
#include <string>

#include "common.h"

namespace msha {

static thread_local std::string g_last_error;
static const uint64_t* g_rng_counter = nullptr;

const uint64_t* rng_counter() { return g_rng_counter; }

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    return fail(MSHA_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
  }
  return MSHA_OK;
}

__global__ void __launch_bounds__(256) dropout_mask_kernel(Dropout d, int64_t n, uint8_t* keep) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    keep[i] = dropout_factor(d, (uint64_t)i) != 0.f ? 1 : 0;
  }
}

}  // namespace msha

extern "C" int msha_abi_version(void) { return MSHA_ABI_VERSION; }

extern "C" const char* msha_last_error(void) { return msha::g_last_error.c_str(); }

extern "C" int msha_set_rng_counter(const uint64_t* counter) {
  msha::g_rng_counter = counter;
  return MSHA_OK;
}

extern "C" int msha_dropout_keep_mask(uint64_t seed, uint64_t offset, int64_t n, float p,
                                      uint8_t* keep, msha_stream_t stream) {
  MSHA_ARG_CHECK(n >= 0 && (n == 0 || keep != nullptr), "dropout_keep_mask: bad buffer");
  MSHA_ARG_CHECK(p >= 0.f && p <= 1.f, "dropout_keep_mask: p must be in [0, 1]");
  if (n == 0) return MSHA_OK;
  msha::Dropout d = msha::make_dropout(p, seed, offset);
  d.active = true;  // p == 0 still runs the generator: every element kept
  hipLaunchKernelGGL(msha::dropout_mask_kernel, dim3(msha::grid_for(n, 256, 8192)), dim3(256), 0,
                     (hipStream_t)stream, d, n, keep);
  return msha::check_launch("dropout_keep_mask");
}
