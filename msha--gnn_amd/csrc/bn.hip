// BatchNorm1d (training batch statistics / eval running statistics) fused with the
// LeakyReLU that follows it in the MSHA layers' epilogue:
//   Ablation.py:273-274 / Ours.py:100-101:  v_out = lrelu(bn1(v)),  u_out = lrelu(bn2(u))
// on (rows, C) node tables (fp32 or bf16 storage, fp32 arithmetic and statistics).
//
// Forward (training): per-channel mean / biased variance over the rows (Welford per
// thread, Chan combination in a fixed tree inside a block, block partials combined in
// block order: deterministic), running statistics updated as torch does (momentum,
// unbiased variance), y = lrelu(weight * (x - mean) * invstd + bias).
// Backward: dz = dy * lrelu'(z) (z recomputed from x), dbias = sum dz,
// dweight = sum dz * xhat, dx = weight * invstd * (dz - dbias / R - xhat * dweight / R).
// Rows <= kBnSingle: one workgroup does statistics and the elementwise pass in one
// launch (the recipient side v, 32 rows); otherwise partials + finalize + apply.
#include "common.h"

namespace msha {

constexpr int kBnSingle = 256;  // up to this many rows: the one-workgroup path
constexpr int kBnRows = 64;  // rows per partial block (256: 153 blocks at R15's 39k rows,
                             // 16 serial load rounds per thread, 11.5 us)
#ifndef BN_U
#define BN_U 8  // rows per thread whose loads are in flight together
#endif
constexpr int kBnThreads = 256;


// threads: channel c = t % CT (CT = min(C, 256) channels per column tile, blockIdx.y
// tiles), row group rg = t / CT strides the block's rows
template <typename T>
__device__ __forceinline__ Wf block_stats(const T* __restrict__ x, int64_t r0, int64_t r1, int C,
                                          int c, int rg, int RG, Wf* red, int CT, int ci) {
  Wf w{0.f, 0.f, 0.f};
  if (c < C && rg < RG) {
    // BN_U rows loaded before the Welford updates (same order): the loads overlap
    // instead of one memory round trip per row
    int64_t r = r0 + rg;
    for (; r + (BN_U - 1) * RG < r1; r += BN_U * RG) {
      float v[BN_U];
#pragma unroll
      for (int u = 0; u < BN_U; ++u) v[u] = to_f32(x[(r + u * RG) * C + c]);
#pragma unroll
      for (int u = 0; u < BN_U; ++u) {
        w.n += 1.f;
        const float d = v[u] - w.mean;
        w.mean += d / w.n;
        w.m2 += d * (v[u] - w.mean);
      }
    }
    for (; r < r1; r += RG) {
      const float v = to_f32(x[r * C + c]);
      w.n += 1.f;
      const float d = v - w.mean;
      w.mean += d / w.n;
      w.m2 += d * (v - w.mean);
    }
  }
  red[threadIdx.x] = w;
  __syncthreads();
  int p = 1;
  while (p < RG) p <<= 1;
  for (p >>= 1; p >= 1; p >>= 1) {
    if (rg < p && rg + p < RG) red[threadIdx.x] = wf_combine(red[threadIdx.x], red[(rg + p) * CT + ci]);
    __syncthreads();
  }
  return red[ci];
}

struct BnArgs {
  int64_t rows;
  int C;
  float eps, slope, momentum;
  const float* weight;
  const float* bias;
  float* running_mean;
  float* running_var;
  float* mean;    // out (C)
  float* invstd;  // out (C)
};

__device__ __forceinline__ void bn_finalize_channel(const BnArgs& a, int c, Wf w, bool training) {
  if (!training) return;
  const float var = w.n > 0.f ? w.m2 / w.n : 0.f;
  a.mean[c] = w.mean;
  a.invstd[c] = rsqrtf(var + a.eps);
  if (a.running_mean != nullptr) {
    const float unb = w.n > 1.f ? w.m2 / (w.n - 1.f) : var;
    a.running_mean[c] = (1.f - a.momentum) * a.running_mean[c] + a.momentum * w.mean;
    a.running_var[c] = (1.f - a.momentum) * a.running_var[c] + a.momentum * unb;
  }
}

template <typename T>
__device__ __forceinline__ void bn_apply_elem(const BnArgs& a, const T* x, T* y, int64_t i, int c,
                                              float mean, float invstd) {
  const float w = a.weight != nullptr ? a.weight[c] : 1.f;
  const float b = a.bias != nullptr ? a.bias[c] : 0.f;
  const float z = fmaf(w * invstd, to_f32(x[i]) - mean, b);
  y[i] = from_f32<T>(z > 0.f ? z : z * a.slope);
}

// one workgroup: statistics + running update + elementwise (rows <= kBnSingle)
template <typename T>
__global__ void __launch_bounds__(kBnThreads) bn_fwd_small_kernel(BnArgs a, int training,
                                                                 const T* __restrict__ x,
                                                                 T* __restrict__ y) {
  __shared__ Wf red[kBnThreads];
  __shared__ float s_mean[1024], s_inv[1024];
  const int C = a.C;
  for (int c0 = 0; c0 < C; c0 += kBnThreads) {
    const int CT = min(C - c0, kBnThreads);
    const int RG = kBnThreads / CT;
    const int ci = threadIdx.x % CT, rg = threadIdx.x / CT;
    if (training) {
      const Wf w = block_stats(x, 0, a.rows, C, c0 + ci, rg, RG, red, CT, ci);
      if (rg == 0) {
        bn_finalize_channel(a, c0 + ci, w, true);
        s_mean[c0 + ci] = w.mean;
        s_inv[c0 + ci] = rsqrtf((w.n > 0.f ? w.m2 / w.n : 0.f) + a.eps);
      }
    } else if (rg == 0) {
      s_mean[c0 + ci] = a.running_mean[c0 + ci];
      s_inv[c0 + ci] = rsqrtf(a.running_var[c0 + ci] + a.eps);
    }
    __syncthreads();
  }
  const int64_t total = a.rows * C;
  for (int64_t i = threadIdx.x; i < total; i += blockDim.x) {
    const int c = (int)(i % C);
    bn_apply_elem(a, x, y, i, c, s_mean[c], s_inv[c]);
  }
}

template <typename T>
__global__ void __launch_bounds__(kBnThreads) bn_partial_kernel(BnArgs a, const T* __restrict__ x,
                                                               Wf* __restrict__ part) {
  __shared__ Wf red[kBnThreads];
  const int C = a.C;
  const int c0 = blockIdx.y * kBnThreads;
  const int CT = min(C - c0, kBnThreads);
  const int RG = kBnThreads / CT;
  const int ci = threadIdx.x % CT, rg = threadIdx.x / CT;
  const int64_t r0 = (int64_t)blockIdx.x * kBnRows;
  const int64_t r1 = min(a.rows, r0 + kBnRows);
  const Wf w = block_stats(x, r0, r1, C, c0 + ci, rg, RG, red, CT, ci);
  if (rg == 0 && threadIdx.x < CT) part[(int64_t)blockIdx.x * C + c0 + ci] = w;
}

// one wave per channel: lane l Chan-combines partials l, l+64, ... in order, then a
// fixed xor tree across the lanes (deterministic)
__device__ __forceinline__ Wf wf_shfl_xor(Wf w, int o) {
  return Wf{__shfl_xor(w.n, o), __shfl_xor(w.mean, o), __shfl_xor(w.m2, o)};
}

__global__ void __launch_bounds__(256) bn_finalize_kernel(BnArgs a, int nblk,
                                                          const Wf* __restrict__ part) {
  const int c = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const int lane = threadIdx.x & 63;
  if (c >= a.C) return;
  Wf w{0.f, 0.f, 0.f};
  int b = lane;  // partials lane, lane + 64, ... in order, 8 loads in flight at a time
  for (; b + 7 * 64 < nblk; b += 8 * 64) {
    Wf pb[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) pb[q] = part[(int64_t)(b + q * 64) * a.C + c];
#pragma unroll
    for (int q = 0; q < 8; ++q) w = wf_combine(w, pb[q]);
  }
  for (; b < nblk; b += 64) w = wf_combine(w, part[(int64_t)b * a.C + c]);
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) w = wf_combine(w, wf_shfl_xor(w, o));
  if (lane == 0) bn_finalize_channel(a, c, w, true);
}

template <typename T>
__global__ void __launch_bounds__(256) bn_apply_kernel(BnArgs a, int training,
                                                       const T* __restrict__ x, T* __restrict__ y) {
  const int64_t total = a.rows * a.C;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % a.C);
    const float mean = training ? a.mean[c] : a.running_mean[c];
    const float inv = training ? a.invstd[c] : rsqrtf(a.running_var[c] + a.eps);
    bn_apply_elem(a, x, y, i, c, mean, inv);
  }
}

// ---- backward
struct BnBwd {
  int64_t rows;
  int C;
  float slope;
  const float* weight;
  const float* bias;
  const float* mean;
  const float* invstd;
  float* dweight;
  float* dbias;
};

__device__ __forceinline__ void bwd_terms_v(const BnBwd& a, float xv, float gv, int c, float& dz,
                                            float& xhat) {
  const float w = a.weight != nullptr ? a.weight[c] : 1.f;
  const float b = a.bias != nullptr ? a.bias[c] : 0.f;
  xhat = (xv - a.mean[c]) * a.invstd[c];
  const float z = fmaf(w, xhat, b);
  dz = gv * (z > 0.f ? 1.f : a.slope);
}

template <typename T>
__device__ __forceinline__ void bwd_terms(const BnBwd& a, const T* x, const T* dy, int64_t i,
                                          int c, float& dz, float& xhat) {
  bwd_terms_v(a, to_f32(x[i]), to_f32(dy[i]), c, dz, xhat);
}

// per block and channel: (sum dz, sum dz * xhat) over the block's rows, fixed tree
template <typename T>
__device__ __forceinline__ float2 block_bwd_sums(const BnBwd& a, const T* x, const T* dy,
                                                 int64_t r0, int64_t r1, int c, int rg, int RG,
                                                 float2* red, int CT, int ci) {
  float2 s = make_float2(0.f, 0.f);
  if (c < a.C && rg < RG) {
    int64_t r = r0 + rg;
    for (; r + (BN_U - 1) * RG < r1; r += BN_U * RG) {  // loads first, sums in order
      float xv[BN_U], gv[BN_U];
#pragma unroll
      for (int u = 0; u < BN_U; ++u) {
        xv[u] = to_f32(x[(r + u * RG) * a.C + c]);
        gv[u] = to_f32(dy[(r + u * RG) * a.C + c]);
      }
#pragma unroll
      for (int u = 0; u < BN_U; ++u) {
        float dz, xh;
        bwd_terms_v(a, xv[u], gv[u], c, dz, xh);
        s.x += dz;
        s.y = fmaf(dz, xh, s.y);
      }
    }
    for (; r < r1; r += RG) {
      float dz, xh;
      bwd_terms(a, x, dy, r * a.C + c, c, dz, xh);
      s.x += dz;
      s.y = fmaf(dz, xh, s.y);
    }
  }
  red[threadIdx.x] = s;
  __syncthreads();
  int p = 1;
  while (p < RG) p <<= 1;
  for (p >>= 1; p >= 1; p >>= 1) {
    if (rg < p && rg + p < RG) {
      const float2 o = red[(rg + p) * CT + ci];
      red[threadIdx.x].x += o.x;
      red[threadIdx.x].y += o.y;
    }
    __syncthreads();
  }
  return red[ci];
}

template <typename T>
__device__ __forceinline__ void bn_bwd_elem(const BnBwd& a, const T* x, const T* dy, T* dx,
                                            int64_t i, int c, float db, float dw) {
  float dz, xh;
  bwd_terms(a, x, dy, i, c, dz, xh);
  const float w = a.weight != nullptr ? a.weight[c] : 1.f;
  const float invR = 1.f / (float)a.rows;
  dx[i] = from_f32<T>(w * a.invstd[c] * (dz - db * invR - xh * dw * invR));
}

template <typename T>
__global__ void __launch_bounds__(kBnThreads) bn_bwd_small_kernel(BnBwd a, const T* __restrict__ x,
                                                                 const T* __restrict__ dy,
                                                                 T* __restrict__ dx) {
  __shared__ float2 red[kBnThreads];
  __shared__ float s_db[1024], s_dw[1024];
  const int C = a.C;
  for (int c0 = 0; c0 < C; c0 += kBnThreads) {
    const int CT = min(C - c0, kBnThreads);
    const int RG = kBnThreads / CT;
    const int ci = threadIdx.x % CT, rg = threadIdx.x / CT;
    const float2 s = block_bwd_sums(a, x, dy, 0, a.rows, c0 + ci, rg, RG, red, CT, ci);
    if (rg == 0) {
      s_db[c0 + ci] = s.x;
      s_dw[c0 + ci] = s.y;
      if (a.dbias != nullptr) a.dbias[c0 + ci] = s.x;
      if (a.dweight != nullptr) a.dweight[c0 + ci] = s.y;
    }
    __syncthreads();
  }
  const int64_t total = a.rows * C;
  for (int64_t i = threadIdx.x; i < total; i += blockDim.x) {
    const int c = (int)(i % C);
    bn_bwd_elem(a, x, dy, dx, i, c, s_db[c], s_dw[c]);
  }
}

template <typename T>
__global__ void __launch_bounds__(kBnThreads) bn_bwd_partial_kernel(BnBwd a,
                                                                   const T* __restrict__ x,
                                                                   const T* __restrict__ dy,
                                                                   float2* __restrict__ part) {
  __shared__ float2 red[kBnThreads];
  const int C = a.C;
  const int c0 = blockIdx.y * kBnThreads;
  const int CT = min(C - c0, kBnThreads);
  const int RG = kBnThreads / CT;
  const int ci = threadIdx.x % CT, rg = threadIdx.x / CT;
  const int64_t r0 = (int64_t)blockIdx.x * kBnRows;
  const int64_t r1 = min(a.rows, r0 + kBnRows);
  const float2 s = block_bwd_sums(a, x, dy, r0, r1, c0 + ci, rg, RG, red, CT, ci);
  if (rg == 0 && threadIdx.x < CT) part[(int64_t)blockIdx.x * C + c0 + ci] = s;
}

__global__ void __launch_bounds__(256) bn_bwd_finalize_kernel(BnBwd a, int nblk,
                                                              const float2* __restrict__ part,
                                                              float2* __restrict__ tot) {
  const int c = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const int lane = threadIdx.x & 63;
  if (c >= a.C) return;
  float2 s = make_float2(0.f, 0.f);
  for (int b = lane; b < nblk; b += 64) {
    const float2 o = part[(int64_t)b * a.C + c];
    s.x += o.x;
    s.y += o.y;
  }
  s.x = wave_xor_sum<1>(s.x);
  s.y = wave_xor_sum<1>(s.y);
  if (lane != 0) return;
  tot[c] = s;
  if (a.dbias != nullptr) a.dbias[c] = s.x;
  if (a.dweight != nullptr) a.dweight[c] = s.y;
}

template <typename T>
__global__ void __launch_bounds__(256) bn_bwd_apply_kernel(BnBwd a, const float2* __restrict__ tot,
                                                           const T* __restrict__ x,
                                                           const T* __restrict__ dy,
                                                           T* __restrict__ dx) {
  const int64_t total = a.rows * a.C;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % a.C);
    const float2 s = tot[c];
    bn_bwd_elem(a, x, dy, dx, i, c, s.x, s.y);
  }
}

static int64_t bn_blocks(int64_t rows) { return (rows + kBnRows - 1) / kBnRows; }

// per-channel Welford partials of a (rows, C) table, one per kBnRows-row block (the
// model head's u statistics, head.hip); returns the number of partial blocks
int64_t bn_stats_partials(int64_t rows, int C, bool bf, const void* x, void* part,
                          hipStream_t s) {
  BnArgs a{};
  a.rows = rows;
  a.C = C;
  const int64_t nb = bn_blocks(rows);
  const dim3 g((unsigned)nb, (C + kBnThreads - 1) / kBnThreads);
  if (bf)
    hipLaunchKernelGGL(bn_partial_kernel<bf16_t>, g, dim3(kBnThreads), 0, s, a, (const bf16_t*)x,
                       (Wf*)part);
  else
    hipLaunchKernelGGL(bn_partial_kernel<float>, g, dim3(kBnThreads), 0, s, a, (const float*)x,
                       (Wf*)part);
  return nb;
}
int64_t bn_stats_blocks(int64_t rows) { return bn_blocks(rows); }

}  // namespace msha

using namespace msha;

extern "C" size_t msha_bn_workspace_size(int64_t rows, int32_t channels) {
  if (rows <= kBnSingle) return 0;
  const size_t nb = (size_t)bn_blocks(rows);
  const size_t f = nb * (size_t)channels * sizeof(Wf);
  const size_t b = nb * (size_t)channels * sizeof(float2) + (size_t)channels * sizeof(float2);
  return f > b ? f : b;
}

extern "C" int msha_bn_lrelu_fwd(int64_t rows, int32_t channels, int32_t dtype, const void* x,
                                 const float* weight, const float* bias, float eps, float slope,
                                 int32_t training, float momentum, float* running_mean,
                                 float* running_var, float* mean, float* invstd, void* y,
                                 void* ws, size_t ws_bytes, msha_stream_t stream) {
  MSHA_ARG_CHECK(rows > 0 && channels > 0 && channels <= 1024, "bn_lrelu_fwd: bad sizes");
  MSHA_ARG_CHECK(x && y, "bn_lrelu_fwd: null pointer");
  MSHA_ARG_CHECK(dtype == MSHA_DTYPE_F32 || dtype == MSHA_DTYPE_BF16, "bn_lrelu_fwd: bad dtype");
  MSHA_ARG_CHECK(training ? (mean && invstd && (running_mean == nullptr) == (running_var == nullptr))
                          : (running_mean && running_var),
                 "bn_lrelu_fwd: training needs mean/invstd outputs, eval running statistics");
  BnArgs a;
  a.rows = rows; a.C = channels; a.eps = eps; a.slope = slope; a.momentum = momentum;
  a.weight = weight; a.bias = bias; a.running_mean = running_mean; a.running_var = running_var;
  a.mean = mean; a.invstd = invstd;
  hipStream_t s = (hipStream_t)stream;
  const bool bf = dtype == MSHA_DTYPE_BF16;
  if (rows <= kBnSingle || !training) {
    if (rows <= kBnSingle) {
      if (bf)
        hipLaunchKernelGGL(bn_fwd_small_kernel<bf16_t>, dim3(1), dim3(kBnThreads), 0, s, a,
                           training, (const bf16_t*)x, (bf16_t*)y);
      else
        hipLaunchKernelGGL(bn_fwd_small_kernel<float>, dim3(1), dim3(kBnThreads), 0, s, a,
                           training, (const float*)x, (float*)y);
      return check_launch("bn_lrelu_fwd");
    }
  } else {
    MSHA_ARG_CHECK(ws && ws_bytes >= msha_bn_workspace_size(rows, channels),
                   "bn_lrelu_fwd: workspace too small");
    const int64_t nb = bn_blocks(rows);
    const dim3 g(nb, (channels + kBnThreads - 1) / kBnThreads);
    if (bf)
      hipLaunchKernelGGL(bn_partial_kernel<bf16_t>, g, dim3(kBnThreads), 0, s, a,
                         (const bf16_t*)x, (Wf*)ws);
    else
      hipLaunchKernelGGL(bn_partial_kernel<float>, g, dim3(kBnThreads), 0, s, a,
                         (const float*)x, (Wf*)ws);
    hipLaunchKernelGGL(bn_finalize_kernel, dim3((channels + 3) / 4), dim3(256), 0, s, a,
                       (int)nb, (const Wf*)ws);
  }
  const dim3 ga(grid_for(rows * channels, 256, 8192));
  if (bf)
    hipLaunchKernelGGL(bn_apply_kernel<bf16_t>, ga, dim3(256), 0, s, a, training,
                       (const bf16_t*)x, (bf16_t*)y);
  else
    hipLaunchKernelGGL(bn_apply_kernel<float>, ga, dim3(256), 0, s, a, training,
                       (const float*)x, (float*)y);
  return check_launch("bn_lrelu_fwd");
}

extern "C" int msha_bn_lrelu_bwd(int64_t rows, int32_t channels, int32_t dtype, const void* x,
                                 const void* dy, const float* weight, const float* bias,
                                 const float* mean, const float* invstd, float slope, void* dx,
                                 float* dweight, float* dbias, void* ws, size_t ws_bytes,
                                 msha_stream_t stream) {
  MSHA_ARG_CHECK(rows > 0 && channels > 0 && channels <= 1024, "bn_lrelu_bwd: bad sizes");
  MSHA_ARG_CHECK(x && dy && dx && mean && invstd, "bn_lrelu_bwd: null pointer");
  MSHA_ARG_CHECK(dtype == MSHA_DTYPE_F32 || dtype == MSHA_DTYPE_BF16, "bn_lrelu_bwd: bad dtype");
  BnBwd a;
  a.rows = rows; a.C = channels; a.slope = slope; a.weight = weight; a.bias = bias;
  a.mean = mean; a.invstd = invstd; a.dweight = dweight; a.dbias = dbias;
  hipStream_t s = (hipStream_t)stream;
  const bool bf = dtype == MSHA_DTYPE_BF16;
  if (rows <= kBnSingle) {
    if (bf)
      hipLaunchKernelGGL(bn_bwd_small_kernel<bf16_t>, dim3(1), dim3(kBnThreads), 0, s, a,
                         (const bf16_t*)x, (const bf16_t*)dy, (bf16_t*)dx);
    else
      hipLaunchKernelGGL(bn_bwd_small_kernel<float>, dim3(1), dim3(kBnThreads), 0, s, a,
                         (const float*)x, (const float*)dy, (float*)dx);
    return check_launch("bn_lrelu_bwd");
  }
  MSHA_ARG_CHECK(ws && ws_bytes >= msha_bn_workspace_size(rows, channels),
                 "bn_lrelu_bwd: workspace too small");
  const int64_t nb = bn_blocks(rows);
  float2* part = (float2*)ws;
  float2* tot = part + nb * channels;
  const dim3 g(nb, (channels + kBnThreads - 1) / kBnThreads);
  if (bf)
    hipLaunchKernelGGL(bn_bwd_partial_kernel<bf16_t>, g, dim3(kBnThreads), 0, s, a,
                       (const bf16_t*)x, (const bf16_t*)dy, part);
  else
    hipLaunchKernelGGL(bn_bwd_partial_kernel<float>, g, dim3(kBnThreads), 0, s, a,
                       (const float*)x, (const float*)dy, part);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((channels + 3) / 4), dim3(256), 0, s, a,
                     (int)nb, (const float2*)part, tot);
  const dim3 ga(grid_for(rows * channels, 256, 8192));
  if (bf)
    hipLaunchKernelGGL(bn_bwd_apply_kernel<bf16_t>, ga, dim3(256), 0, s, a, (const float2*)tot,
                       (const bf16_t*)x, (const bf16_t*)dy, (bf16_t*)dx);
  else
    hipLaunchKernelGGL(bn_bwd_apply_kernel<float>, ga, dim3(256), 0, s, a, (const float2*)tot,
                       (const float*)x, (const float*)dy, (float*)dx);
  return check_launch("bn_lrelu_bwd");
}
