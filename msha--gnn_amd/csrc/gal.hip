// GraphAttentionLayer row-scale kernels (GAT.py:20-35, Ablation.py:100-115).
//
// The reference layer builds an (N, M, 2F) tensor whose two halves are the SAME
// row h_i (GAT.py:24-25), so its score e_ij does not depend on j: the masked
// softmax is exactly mask/deg (1/M on a row without edges), and the layer is
//     out = elu(dropout(mask/deg) * h),     h = input @ W  (N, M)
// One wave per row; each lane owns columns lane, lane+64, ...; membership of a
// column in the row is a binary search in the row's ascending CSR columns.
#include "common.h"

namespace msha {

__device__ __forceinline__ bool row_has(const int32_t* __restrict__ col, int32_t lo, int32_t hi,
                                        int32_t j) {
  while (lo < hi) {
    const int32_t mid = (lo + hi) >> 1;
    const int32_t c = col[mid];
    if (c == j) return true;
    if (c < j) lo = mid + 1; else hi = mid;
  }
  return false;
}

template <bool BWD>
__global__ void __launch_bounds__(256) gal_kernel(const int32_t* __restrict__ rowptr,
                                                  const int32_t* __restrict__ col,
                                                  int64_t n_rows, int64_t n_cols,
                                                  const float* __restrict__ h,
                                                  const float* __restrict__ dout, Dropout dp,
                                                  float* __restrict__ out) {
  const int lane = lane_id();
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  // narrow rows (n_cols <= 32, e.g. the 32 recipients of R15) share a wave: lpr lanes
  // per row, 64 / lpr rows per wave
  int lpr = 64;
  while (lpr > 1 && lpr / 2 >= n_cols) lpr >>= 1;
  const int rpw = 64 / lpr;
  const int sub = lane / lpr, jl = lane % lpr;
  for (int64_t i0 = wave * rpw; i0 < n_rows; i0 += nwaves * rpw) {
    const int64_t i = i0 + sub;
    if (i >= n_rows) continue;
    const int32_t lo = rowptr[i], hi = rowptr[i + 1];
    const int32_t deg = hi - lo;  // virtual full rows have deg == n_cols
    const float inv = deg > 0 ? 1.f / (float)deg : 0.f;
    const bool full = deg == n_cols;
    for (int64_t j = jl; j < n_cols; j += lpr) {
      const int64_t k = i * n_cols + j;
      float a = (full || row_has(col, lo, hi, (int32_t)j)) ? inv : 0.f;
      a *= dropout_factor(dp, (uint64_t)k);
      const float z = a * h[k];
      if (!BWD) {
        out[k] = z > 0.f ? z : expm1f(z);
      } else {
        out[k] = dout[k] * (z > 0.f ? 1.f : __expf(z)) * a;
      }
    }
  }
}

// one wave per 64 / lpr rows (lpr: the kernel's lanes per row)
static dim3 gal_grid(int64_t n_rows, int64_t n_cols) {
  int lpr = 64;
  while (lpr > 1 && lpr / 2 >= n_cols) lpr >>= 1;
  const int64_t rpw = 64 / lpr;
  return dim3(grid_for((n_rows + rpw - 1) / rpw, 4, 1 << 20));
}

static int check(const msha_graph* g, const float* h, const float* o) {
  MSHA_ARG_CHECK(g != nullptr && g->rowptr && g->col, "gal: graph CSR missing");
  MSHA_ARG_CHECK(g->n_rows > 0 && g->n_cols > 0, "gal: bad sizes");
  MSHA_ARG_CHECK(h && o, "gal: null pointer");
  return MSHA_OK;
}

}  // namespace msha

using namespace msha;

extern "C" int msha_gal_fwd(const msha_graph* g, const float* h, float drop_p, uint64_t seed,
                            uint64_t offset, float* out, msha_stream_t stream) {
  if (int rc = check(g, h, out)) return rc;
  MSHA_ARG_CHECK(drop_p >= 0.f && drop_p <= 1.f, "gal_fwd: p must be in [0,1]");
  hipLaunchKernelGGL(gal_kernel<false>, gal_grid(g->n_rows, g->n_cols), dim3(256), 0,
                     (hipStream_t)stream, g->rowptr, g->col, g->n_rows, g->n_cols, h,
                     (const float*)nullptr, make_dropout(drop_p, seed, offset, (hipStream_t)stream), out);
  return check_launch("gal_fwd");
}

extern "C" int msha_gal_bwd(const msha_graph* g, const float* h, const float* dout, float drop_p,
                            uint64_t seed, uint64_t offset, float* dh, msha_stream_t stream) {
  if (int rc = check(g, h, dh)) return rc;
  MSHA_ARG_CHECK(dout != nullptr, "gal_bwd: null dout");
  MSHA_ARG_CHECK(drop_p >= 0.f && drop_p <= 1.f, "gal_bwd: p must be in [0,1]");
  hipLaunchKernelGGL(gal_kernel<true>, gal_grid(g->n_rows, g->n_cols), dim3(256), 0,
                     (hipStream_t)stream, g->rowptr, g->col, g->n_rows, g->n_cols, h, dout,
                     make_dropout(drop_p, seed, offset, (hipStream_t)stream), dh);
  return check_launch("gal_bwd");
}
