// The optimizer step of train.py's loop (train.py:207 optim.Adam(lr 1e-3, weight_decay
// 5e-4); :232 optimizer.step()) as one launch over every parameter (include/msha_gnn.h
// msha_adam_step).  torch's fused multi-tensor Adam read each gradient the backward had
// written; here the feature dropout's backward (the only producer of Sfeatures' gradient,
// Ablation.py:296 / Ours.py:161) can be fused into the gradient read instead: the 5M-float
// gradient is never written or re-read.
//
// One thread owns 4 consecutive elements (16-B fp32 / 8-B bf16 pieces of every operand);
// each tensor gets its own range of blocks of a 1-D grid.  Arithmetic follows torch.optim.Adam's
// single-tensor step (grad + wd * p, lerp of the first moment, addcmul of the second,
// addcdiv with step_size = lr / bias_correction1), fp32 per element with the bias
// corrections in double from the step count, as torch computes them on the host.
#include "common.h"

namespace msha {

constexpr int kAdamLeaves = 64;  // completion-ticket leaves (see adam_kernel's end)
constexpr int kAdamLine = 64;    // uint32 words per ticket counter: one 256-B line each

struct AdamBatch {
  msha_adam_tensor t[MSHA_MAX_ADAM];
  double lr, b1, b2, eps, wd;  // torch's Python-float hyperparameters
  int n;
  int first[MSHA_MAX_ADAM + 1];  // blocks [first[i], first[i+1]) update tensor i (1-D grid)
  uint32_t* ticket;     // completion ticket: top counter, then the leaves (workspace, zero between launches)
  const uint64_t* ctr;  // device replay counter (dropout offsets)
};

__device__ __forceinline__ float4 ad_ld4(const void* p, int dt, int64_t q) {
  if (dt == MSHA_DTYPE_BF16) {
    const uint2 w = reinterpret_cast<const uint2*>(p)[q];
    return make_float4(__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u),
                       __uint_as_float(w.y << 16), __uint_as_float(w.y & 0xffff0000u));
  }
  return reinterpret_cast<const float4*>(p)[q];
}
__device__ __forceinline__ void ad_st4(void* p, int dt, int64_t q, float4 v) {
  if (dt == MSHA_DTYPE_BF16)
    reinterpret_cast<uint2*>(p)[q] = make_uint2(pack_bf16x2(v.x, v.y), pack_bf16x2(v.z, v.w));
  else
    reinterpret_cast<float4*>(p)[q] = v;
}
__device__ __forceinline__ float ad_ld(const void* p, int dt, int64_t i) {
  return dt == MSHA_DTYPE_BF16 ? (float)reinterpret_cast<const bf16_t*>(p)[i]
                               : reinterpret_cast<const float*>(p)[i];
}
__device__ __forceinline__ void ad_st(void* p, int dt, int64_t i, float v) {
  if (dt == MSHA_DTYPE_BF16)
    reinterpret_cast<bf16_t*>(p)[i] = (bf16_t)v;
  else
    reinterpret_cast<float*>(p)[i] = v;
}

struct AdamScalars {
  float b1c, b2c, wd, step_size, bc2_sqrt, eps;  // b1c = 1 - beta1, b2c = 1 - beta2
  float b2;
};

// one element: returns the new (param, m, v)
__device__ __forceinline__ void adam_elem(const AdamScalars& a, float g, float& p, float& m,
                                          float& v) {
  g = fmaf(a.wd, p, g);                  // grad.add(param, alpha=wd)
  m = fmaf(a.b1c, g - m, m);             // exp_avg.lerp_(grad, 1 - beta1)
  v = fmaf(a.b2c, g * g, v * a.b2);      // exp_avg_sq.mul_(beta2).addcmul_(g, g, 1 - beta2)
  const float denom = sqrtf(v) / a.bc2_sqrt + a.eps;
  p = p - a.step_size * (m / denom);     // param.addcdiv_(exp_avg, denom, -step_size)
}

// bias corrections of step t (exact integer t) in double, as torch computes them on the
// host: beta ** t by squaring (<= 2 log2 t double multiplies, a few ulps)
__device__ __forceinline__ float2 adam_scalars(const AdamBatch& b, float t) {
  double p1 = 1.0, p2 = 1.0, s1 = b.b1, s2 = b.b2;
  for (uint32_t e = (uint32_t)t; e != 0; e >>= 1) {
    if (e & 1u) {
      p1 *= s1;
      p2 *= s2;
    }
    s1 *= s1;
    s2 *= s2;
  }
  return make_float2((float)(b.lr / (1.0 - p1)), (float)sqrt(1.0 - p2));
}

// One launch (round 5 ran a one-block launch ahead of the update for the scalars: one more
// graph node, ~4 us).  Every thread reads its tensor's step count t - 1 and derives step t's
// scalars itself (as torch's capturable Adam adds 1 first); the last block to finish -- a
// completion ticket in the workspace, zero between launches -- advances every step count.
// The ticket is a relaxed atomic with no fence: each block's step read was consumed by its
// whole update before the block takes its ticket, and nothing else is published through
// it (a device-scope fence per block writes back L2: that form measured 102 us vs 25).
__global__ void __launch_bounds__(256) adam_kernel(AdamBatch b) {
  // the tensor of this block: first[ti] <= blockIdx.x < first[ti + 1] (binary search over
  // the <= 64 boundaries; every block works -- a 2-D grid sized by the largest tensor left
  // ~2k idle blocks per small tensor)
  const int bid = blockIdx.x;
  int lo = 0, hi = b.n;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (b.first[mid] <= bid) lo = mid; else hi = mid;
  }
  const int ti = lo;
  const msha_adam_tensor& T = b.t[ti];
  const int dt = T.dtype;
  const float2 sc = adam_scalars(b, *T.step + 1.f);
  AdamScalars a;  // the scalars torch hands its fp32 kernels
  a.b1c = (float)(1.0 - b.b1);
  a.b2c = (float)(1.0 - b.b2);
  a.b2 = (float)b.b2;
  a.wd = (float)b.wd;
  a.eps = (float)b.eps;
  a.step_size = sc.x;
  a.bc2_sqrt = sc.y;
  Dropout d{};
  d.active = T.drop_p > 0.f;
  uint64_t off = 0;
  if (d.active) {
    d.seed = T.drop_seed;
    d.offset = T.drop_offset;
    d.ctr = b.ctr;
    const double th = (double)T.drop_p * 4294967296.0;
    d.threshold = T.drop_p >= 1.f ? 0xFFFFFFFFu : (uint32_t)(th > 4294967295.0 ? 4294967295.0 : th);
    d.scale = T.drop_p < 1.f ? (float)(1.0 / (1.0 - (double)T.drop_p)) : 0.f;
    off = dropout_offset(d, d.offset);
  }
  const int64_t nthr = (int64_t)(b.first[ti + 1] - b.first[ti]) * blockDim.x;
  const int64_t tid = (int64_t)(bid - b.first[ti]) * blockDim.x + threadIdx.x;
  const int64_t nq = T.n / 4;
  for (int64_t q = tid; q < nq; q += nthr) {
    float4 g = ad_ld4(T.grad, dt, q), p = ad_ld4(T.param, dt, q);
    float4 m = ad_ld4(T.exp_avg, dt, q), v = ad_ld4(T.exp_avg_sq, dt, q);
    if (d.active) {  // the fused dropout backward: msha_segments' flat mask of element 4q + k
      const uint4 w = philox4(d.seed, off, (uint64_t)q);
      g = make_float4(g.x * (w.x >= d.threshold ? d.scale : 0.f),
                      g.y * (w.y >= d.threshold ? d.scale : 0.f),
                      g.z * (w.z >= d.threshold ? d.scale : 0.f),
                      g.w * (w.w >= d.threshold ? d.scale : 0.f));
    }
    adam_elem(a, g.x, p.x, m.x, v.x);
    adam_elem(a, g.y, p.y, m.y, v.y);
    adam_elem(a, g.z, p.z, m.z, v.z);
    adam_elem(a, g.w, p.w, m.w, v.w);
    ad_st4(T.param, dt, q, p);
    ad_st4(T.exp_avg, dt, q, m);
    ad_st4(T.exp_avg_sq, dt, q, v);
  }
  for (int64_t e = 4 * nq + tid; e < T.n; e += nthr) {  // the < 4 tail elements
    float g = ad_ld(T.grad, dt, e), p = ad_ld(T.param, dt, e);
    float m = ad_ld(T.exp_avg, dt, e), v = ad_ld(T.exp_avg_sq, dt, e);
    if (d.active) {
      const uint4 w = philox4(d.seed, off, (uint64_t)e >> 2);
      const uint32_t x = (e & 3) == 0 ? w.x : (e & 3) == 1 ? w.y : (e & 3) == 2 ? w.z : w.w;
      g *= x >= d.threshold ? d.scale : 0.f;
    }
    adam_elem(a, g, p, m, v);
    ad_st(T.param, dt, e, p);
    ad_st(T.exp_avg, dt, e, m);
    ad_st(T.exp_avg_sq, dt, e, v);
  }
  // two-level completion ticket: 64 leaf counters (a 256-B line each) and one top
  // counter -- same-address atomics serialise at the memory side, so 2048 blocks on one
  // counter added ~18 us; here no counter sees more than 64
  __shared__ int s_last;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t leaf = blockIdx.x & (kAdamLeaves - 1);
    const uint32_t in_leaf = (gridDim.x - leaf + kAdamLeaves - 1) / kAdamLeaves;
    const uint32_t leaves = min(gridDim.x, (uint32_t)kAdamLeaves);
    uint32_t* lc = b.ticket + (1 + leaf) * kAdamLine;
    int last = 0;
    if (__hip_atomic_fetch_add(lc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == in_leaf - 1) {
      *lc = 0u;  // every block of this leaf has counted
      last = __hip_atomic_fetch_add(b.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
             leaves - 1;
    }
    s_last = last;
  }
  __syncthreads();
  if (s_last) {
    const bool own = (int)threadIdx.x < b.n;
    const float t = own ? *b.t[threadIdx.x].step + 1.f : 0.f;
    __syncthreads();  // every count read before any is written (tensors may share one)
    if (own) *b.t[threadIdx.x].step = t;
    if (threadIdx.x == 0) *b.ticket = 0u;
  }
}

}  // namespace msha

using namespace msha;

extern "C" int msha_adam_step(int32_t n, const msha_adam_tensor* tensors, double lr,
                              double beta1, double beta2, double eps, double weight_decay,
                              void* ws, msha_stream_t stream) {
  MSHA_ARG_CHECK(n >= 0 && n <= MSHA_MAX_ADAM && (n == 0 || tensors != nullptr),
                 "adam_step: 0..MSHA_MAX_ADAM tensors");
  MSHA_ARG_CHECK(ws != nullptr, "adam_step: needs the msha_adam_workspace_size() workspace");
  MSHA_ARG_CHECK(beta1 >= 0.0 && beta1 < 1.0 && beta2 >= 0.0 && beta2 < 1.0 && eps >= 0.0,
                 "adam_step: bad hyperparameters");
  if (n == 0) return MSHA_OK;
  AdamBatch b{};
  int nblocks = 0;
  for (int i = 0; i < n; ++i) {
    const msha_adam_tensor& t = tensors[i];
    MSHA_ARG_CHECK(t.param && t.grad && t.exp_avg && t.exp_avg_sq && t.step && t.n >= 0,
                   "adam_step: null pointer / bad size");
    MSHA_ARG_CHECK(t.dtype == MSHA_DTYPE_F32 || t.dtype == MSHA_DTYPE_BF16,
                   "adam_step: dtype must be MSHA_DTYPE_F32 or MSHA_DTYPE_BF16");
    MSHA_ARG_CHECK(t.drop_p >= 0.f && t.drop_p <= 1.f, "adam_step: drop_p must be in [0, 1]");
    const uintptr_t am = t.dtype == MSHA_DTYPE_BF16 ? 7 : 15;
    MSHA_ARG_CHECK((((uintptr_t)t.param | (uintptr_t)t.grad | (uintptr_t)t.exp_avg |
                     (uintptr_t)t.exp_avg_sq) & am) == 0,
                   "adam_step: operands must be aligned to 4 elements");
    b.t[i] = t;
    b.first[i] = nblocks;
    nblocks += grid_for(t.n, 256 * 4, 2048);  // 4 elements per thread, grid-stride past 2048
  }
  b.first[n] = nblocks;
  b.lr = lr;
  b.b1 = beta1;
  b.b2 = beta2;
  b.eps = eps;
  b.wd = weight_decay;
  b.n = n;
  hipStream_t s = (hipStream_t)stream;
  b.ctr = rng_counter(s);
  b.ticket = (uint32_t*)ws;
  hipLaunchKernelGGL(adam_kernel, dim3(nblocks), dim3(256), 0, s, b);
  return check_launch("adam_step");
}

extern "C" size_t msha_adam_workspace_size(void) {
  return sizeof(uint32_t) * kAdamLine * (1 + kAdamLeaves);
}
