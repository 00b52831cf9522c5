// ABI plumbing: version, thread-local error string, dropout mask export.
#include <atomic>
#include <string>

#include "common.h"

namespace msha {

static thread_local std::string g_last_error;

// dropout replay counters, one slot per device (msha_set_rng_counter): a kernel launched
// on a stream of device d reads device d's counter, so two devices (or two processes'
// graphs) never share one
constexpr int kMaxDevices = 64;
static std::atomic<const uint64_t*> g_rng_counter[kMaxDevices];

static int stream_device(hipStream_t s) {
  int dev = -1;
  if (s == nullptr || hipStreamGetDevice(s, &dev) != hipSuccess) {
    if (hipGetDevice(&dev) != hipSuccess) dev = -1;
  }
  return dev;
}

const uint64_t* rng_counter(hipStream_t s) {
  const int dev = stream_device(s);
  return dev >= 0 && dev < kMaxDevices ? g_rng_counter[dev].load(std::memory_order_acquire)
                                       : nullptr;
}

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

// a step's batch copy with the replay counter's increment folded in (msha_feed_step): one
// launch ahead of a graph replay instead of a copy plus the graph's first (add) node
__global__ void __launch_bounds__(256) feed_step_kernel(uint8_t* __restrict__ dst,
                                                       const uint8_t* __restrict__ src,
                                                       int64_t bytes, uint64_t* counter) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nt = (int64_t)gridDim.x * blockDim.x;
  const bool v16 = (((uintptr_t)dst | (uintptr_t)src) & 15) == 0;
  const int64_t n16 = v16 ? bytes / 16 : 0;
  for (int64_t i = t; i < n16; i += nt)
    reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(src)[i];
  for (int64_t i = 16 * n16 + t; i < bytes; i += nt) dst[i] = src[i];
  if (t == 0 && counter != nullptr) *counter += 1;
}

}  // namespace msha

extern "C" int msha_feed_step(void* dst, const void* src, int64_t bytes, uint64_t* counter,
                              msha_stream_t stream) {
  MSHA_ARG_CHECK(bytes >= 0 && (bytes == 0 || (dst != nullptr && src != nullptr)),
                 "feed_step: bad buffers");
  const int64_t units = bytes / 16 + 1;
  hipLaunchKernelGGL(msha::feed_step_kernel, dim3(msha::grid_for(units, 256, 1024)), dim3(256), 0,
                     (hipStream_t)stream, (uint8_t*)dst, (const uint8_t*)src, bytes, counter);
  return msha::check_launch("feed_step");
}

extern "C" int msha_abi_version(void) { return MSHA_ABI_VERSION; }

extern "C" const char* msha_last_error(void) { return msha::g_last_error.c_str(); }

extern "C" int msha_set_rng_counter(int32_t device, const uint64_t* counter) {
  if (device < 0 && hipGetDevice(&device) != hipSuccess)
    return msha::fail(MSHA_ERR_HIP, "set_rng_counter: no current device");
  MSHA_ARG_CHECK(device < msha::kMaxDevices, "set_rng_counter: device index out of range");
  msha::g_rng_counter[device].store(counter, std::memory_order_release);
  return MSHA_OK;
}

extern "C" const uint64_t* msha_get_rng_counter(int32_t device) {
  if (device < 0 && hipGetDevice(&device) != hipSuccess) return nullptr;
  if (device >= msha::kMaxDevices) return nullptr;
  return msha::g_rng_counter[device].load(std::memory_order_acquire);
}

extern "C" int msha_dropout_keep_mask(uint64_t seed, uint64_t offset, int64_t n, float p,
                                      uint8_t* keep, msha_stream_t stream) {
  MSHA_ARG_CHECK(n >= 0 && (n == 0 || keep != nullptr), "dropout_keep_mask: bad buffer");
  MSHA_ARG_CHECK(p >= 0.f && p <= 1.f, "dropout_keep_mask: p must be in [0, 1]");
  if (n == 0) return MSHA_OK;
  msha::Dropout d = msha::make_dropout(p, seed, offset, (hipStream_t)stream);
  d.active = true;  // p == 0 still runs the generator: every element kept
  hipLaunchKernelGGL(msha::dropout_mask_kernel, dim3(msha::grid_for(n, 256, 8192)), dim3(256), 0,
                     (hipStream_t)stream, d, n, keep);
  return msha::check_launch("dropout_keep_mask");
}
