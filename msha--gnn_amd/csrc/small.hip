// Projection of a small node table (the recipient side of the MSHA layers: R15 has 32
// recipients): h1 = R @ W1 and its score half er = h1 . a[:F] (Ablation.py:262, :266-267;
// Ours.py:58, :61-62), forward and backward, each in ONE launch.  The tiled GEMMs spend
// one 128-row tile and a serial K loop on these 32 rows (18 us for 0.5 MFLOP), and the
// backward needed three GEMM launches and a column sum.
//
// Forward:  h = X @ W (M x N), el / er = per-head dots of h with al / ar.
// Backward: D = dh + d_el (x) al + d_er (x) ar (the score halves folded in), dX = D @ W^T,
//           dW = X^T @ D, dal / dar[h, f] = sum_m d_el / d_er[m, h] h[m, h F + f].
// One workgroup per output row (forward, dX) or 256-element slice (dW): M <= 256,
// K <= 128, N <= 128, fp32; sums run in index order (deterministic), fp32 fma chains.
#include "common.h"

namespace msha {

constexpr int kSmallThreads = 256;

struct SmallArgs {
  int M, K, N, H, F;
  const float* X;
  const float* W;
  const float* al;
  const float* ar;
  const float* h;
  const float* dh;
  const float* del;
  const float* der;
  float* out_h;
  float* el;
  float* er;
  float* dX;
  float* dW;
  float* dal;
  float* dar;
};

// forward: one workgroup per row i; thread n computes h[i][n] (W columns read straight
// from L2, 8 loads in flight), then the row's per-head score dots from LDS
__global__ void __launch_bounds__(kSmallThreads) small_fwd_kernel(SmallArgs a) {
  __shared__ float xr[128], hr[128];
  const int K = a.K, N = a.N, F = a.F, i = blockIdx.x, t = threadIdx.x;
  if (t < K) xr[t] = a.X[(int64_t)i * K + t];
  __syncthreads();
  if (t < N) {
    float acc = 0.f;
    int k = 0;
    for (; k + 32 <= K; k += 32) {  // 32 loads in flight (8 a round left K = 128 at 16 L2 round trips)
      float w[32];
#pragma unroll
      for (int q = 0; q < 32; ++q) w[q] = a.W[(int64_t)(k + q) * N + t];
#pragma unroll
      for (int q = 0; q < 32; ++q) acc = fmaf(xr[k + q], w[q], acc);
    }
    for (; k < K; ++k) acc = fmaf(xr[k], a.W[(int64_t)k * N + t], acc);
    hr[t] = acc;
    a.out_h[(int64_t)i * N + t] = acc;
  }
  __syncthreads();
  if (t < 2 * a.H) {
    const int side = t / a.H, hh = t - side * a.H;
    const float* v = side == 0 ? a.al : a.ar;
    float* o = side == 0 ? a.el : a.er;
    if (v != nullptr && F % 4 == 0) {
      // the row-score order of the edge kernels (msha_project_scores_row_order, which
      // covers feat % 4 == 0): per 4-element piece last element first, fma downwards;
      // then the pieces' xor tree
      float d[32];  // F / 4 <= 32 pieces
      const int np = F / 4;
      for (int k = 0; k < np; ++k) {
        const float* x = hr + hh * F + 4 * k;
        const float* vv = v + hh * F + 4 * k;
        d[k] = fmaf(x[0], vv[0], fmaf(x[1], vv[1], fmaf(x[2], vv[2], x[3] * vv[3])));
      }
      for (int st = 1; st < np; st <<= 1)
        for (int k = 0; k + st < np; k += 2 * st) d[k] = d[k] + d[k + st];
      o[(int64_t)i * a.H + hh] = d[0];
    } else if (v != nullptr) {
      // any other feat: an fma chain in element order over the whole head
      float d = 0.f;
      for (int f = 0; f < F; ++f) d = fmaf(hr[hh * F + f], v[hh * F + f], d);
      o[(int64_t)i * a.H + hh] = d;
    }
  }
}

__device__ __forceinline__ float small_d(const SmallArgs& a, int i, int n) {
  const int hh = n / a.F;
  float d = a.dh != nullptr ? a.dh[(int64_t)i * a.N + n] : 0.f;
  if (a.del != nullptr) d = fmaf(a.del[i * a.H + hh], a.al[n], d);
  if (a.der != nullptr) d = fmaf(a.der[i * a.H + hh], a.ar[n], d);
  return d;
}

// backward in one launch: blocks [0, M) the rows of dX, blocks [M, M + nbw) 256-element
// slices of dW, the last block dal / dar
__global__ void __launch_bounds__(kSmallThreads) small_bwd_kernel(SmallArgs a, int nbw) {
  __shared__ float dr[128];
  const int M = a.M, K = a.K, N = a.N, F = a.F, H = a.H, t = threadIdx.x;
  const int b = blockIdx.x;
  if (b < M) {
    if (a.dX == nullptr) return;
    if (t < N) dr[t] = small_d(a, b, t);
    __syncthreads();
    if (t < K) {
      const float* wk = a.W + (int64_t)t * N;
      float acc = 0.f;
      int n = 0;
      for (; n + 32 <= N; n += 32) {  // 32 loads in flight
        float w[32];
#pragma unroll
        for (int q = 0; q < 32; ++q) w[q] = wk[n + q];
#pragma unroll
        for (int q = 0; q < 32; ++q) acc = fmaf(dr[n + q], w[q], acc);
      }
      for (; n < N; ++n) acc = fmaf(dr[n], wk[n], acc);
      a.dX[(int64_t)b * K + t] = acc;
    }
    return;
  }
  if (b < M + nbw) {
    if (a.dW == nullptr) return;
    const int e = (b - M) * kSmallThreads + t;
    if (e >= K * N) return;
    const int k = e / N, n = e - k * N;
    float acc = 0.f;
    int i = 0;
    for (; i + 8 <= M; i += 8) {  // 8 rows' loads in flight, added in row order
      float x[8], d[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        x[q] = a.X[(int64_t)(i + q) * K + k];
        d[q] = small_d(a, i + q, n);
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) acc = fmaf(x[q], d[q], acc);
    }
    for (; i < M; ++i) acc = fmaf(a.X[(int64_t)i * K + k], small_d(a, i, n), acc);
    a.dW[e] = acc;
    return;
  }
  for (int e = t; e < 2 * H * F; e += blockDim.x) {
    const int side = e / (H * F), r = e - side * H * F;
    const float* d = side == 0 ? a.del : a.der;
    float* o = side == 0 ? a.dal : a.dar;
    if (d == nullptr || o == nullptr) continue;
    const int hh = r / F;
    float sc = 0.f;
    int i = 0;
    for (; i + 8 <= M; i += 8) {
      float dv[8], hv[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        dv[q] = d[(i + q) * H + hh];
        hv[q] = a.h[(int64_t)(i + q) * N + r];
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) sc = fmaf(dv[q], hv[q], sc);
    }
    for (; i < M; ++i) sc = fmaf(d[i * H + hh], a.h[(int64_t)i * N + r], sc);
    o[r] = sc;
  }
}

}  // namespace msha

using namespace msha;

extern "C" int msha_project_small_supported(int64_t M, int64_t K, int32_t heads, int32_t feat) {
  const int64_t N = (int64_t)heads * feat;
  return M >= 1 && M <= 256 && K >= 1 && K <= 128 && N >= 1 && N <= 128 && feat >= 1;
}

extern "C" int msha_project_small(int64_t M, int64_t K, int32_t heads, int32_t feat,
                                  const float* X, const float* W, const float* al,
                                  const float* ar, float* h, float* el, float* er,
                                  msha_stream_t stream) {
  MSHA_ARG_CHECK(msha_project_small_supported(M, K, heads, feat), "project_small: shape");
  MSHA_ARG_CHECK(X && W && h, "project_small: null pointer");
  MSHA_ARG_CHECK((al == nullptr) == (el == nullptr) && (ar == nullptr) == (er == nullptr),
                 "project_small: score vectors and outputs must be paired");
  SmallArgs a{};
  a.M = (int)M; a.K = (int)K; a.H = heads; a.F = feat; a.N = heads * feat;
  a.X = X; a.W = W; a.al = al; a.ar = ar; a.out_h = h; a.el = el; a.er = er;
  hipLaunchKernelGGL(small_fwd_kernel, dim3(a.M), dim3(kSmallThreads), 0, (hipStream_t)stream,
                     a);
  return check_launch("project_small");
}

extern "C" int msha_project_small_bwd(int64_t M, int64_t K, int32_t heads, int32_t feat,
                                      const float* X, const float* W, const float* al,
                                      const float* ar, const float* h, const float* dh,
                                      const float* d_el, const float* d_er, float* dX,
                                      float* dW, float* dal, float* dar, msha_stream_t stream) {
  MSHA_ARG_CHECK(msha_project_small_supported(M, K, heads, feat), "project_small_bwd: shape");
  MSHA_ARG_CHECK(X && W && h, "project_small_bwd: null pointer");
  MSHA_ARG_CHECK((d_el == nullptr || al != nullptr) && (d_er == nullptr || ar != nullptr),
                 "project_small_bwd: score gradients need their score vectors");
  SmallArgs a{};
  a.M = (int)M; a.K = (int)K; a.H = heads; a.F = feat; a.N = heads * feat;
  a.X = X; a.W = W; a.al = al; a.ar = ar; a.h = h; a.dh = dh; a.del = d_el; a.der = d_er;
  a.dX = dX; a.dW = dW; a.dal = dal; a.dar = dar;
  const int nbw = (a.K * a.N + kSmallThreads - 1) / kSmallThreads;
  hipLaunchKernelGGL(small_bwd_kernel, dim3(a.M + nbw + 1), dim3(kSmallThreads), 0,
                     (hipStream_t)stream, a, nbw);
  return check_launch("project_small_bwd");
}
