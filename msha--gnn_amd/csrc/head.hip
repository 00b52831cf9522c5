// Model head: everything between the attention aggregates and the log-probabilities
// (SURVEY.md §8f #3), in three forward and three backward launches.
//
// Reference (per head h, then the model):
//   Ablation.py:273-277 / Ours.py:100-109   v_out = lrelu(bn1(v)), u_out = lrelu(bn2(u)),
//                                           elu(u_out @ v_out.T)              (N, M)
//   Ablation.py:298-301 / Ours.py:163-167   x = dropout(cat_h(...)); elu(out_att(x, adj));
//                                           log_softmax(dim=1)
//   GAT.py:20-35 (out_att)                  elu(dropout(softmax(mask * const)) * (x @ W))
//                                           = elu(dropout(mask / deg) * (x @ W))
// Every step after the BatchNorm statistics is local to a row, so one wave computes a
// whole row of the output from u[i] (H*F values), the tiny v side (lrelu(bn1(v)), M x F
// per head, in LDS transposed so lanes j read consecutive banks) and W (H*M x M, LDS).
//
// Forward launches: u statistics partials (bn.hip), finalize (u channels, one wave each;
// the last block does the whole v side: 32 rows), the row pass.
// Backward: train.py's loss reads 64 rows of the (N, M) output, so dout is zero on all
// other rows; a zero row's only gradient path is BatchNorm's batch terms.
//   rows pass    one wave per contiguous row range: a row whose dout is zero is skipped
//                after one 128-B read; a nonzero row recomputes its forward and
//                accumulates dW, d v_out and the BatchNorm sums (sum dz, sum dz * xhat)
//                in the wave's LDS partials; writes dz of the row (the BN-input side)
//   reduce       the flagged waves' partials added in wave order (deterministic)
//   apply        du for every row (dz of nonzero rows, the batch terms for all), and in
//                block 0 the v side's BatchNorm backward over its M rows
#include "common.h"

namespace msha {

constexpr int kHeadThreads = 256;  // forward row pass: 4 waves per block
constexpr int kHeadBwdWaves = 4096;
constexpr int kHeadRowsPerWave = 32;  // (16 -> 32: R15 row pass + reduce 47.8 -> 45.9 us)
constexpr int kHeadVStage = 4096;  // floats of v staged in LDS by the v-side blocks

struct HeadArgs {
  int64_t N;
  int M, H, F, HF, KX;
  float eps, momentum, slope;
  const int32_t* rowptr;
  const int32_t* col;
  const float* uw[MSHA_HEAD_MAX_HEADS];
  const float* ub[MSHA_HEAD_MAX_HEADS];
  float* urm[MSHA_HEAD_MAX_HEADS];
  float* urv[MSHA_HEAD_MAX_HEADS];
  const float* vw[MSHA_HEAD_MAX_HEADS];
  const float* vb[MSHA_HEAD_MAX_HEADS];
  float* vrm[MSHA_HEAD_MAX_HEADS];
  float* vrv[MSHA_HEAD_MAX_HEADS];
  float* duw[MSHA_HEAD_MAX_HEADS];
  float* dub[MSHA_HEAD_MAX_HEADS];
  float* dvw[MSHA_HEAD_MAX_HEADS];
  float* dvb[MSHA_HEAD_MAX_HEADS];
  int64_t* nbt[2 * MSHA_HEAD_MAX_HEADS];
  const float* W;  // (KX, M)
  Dropout dx, dg;
  float* stats;    // [u mean | u invstd | v mean | v invstd] (HF each) | vo_t (HF x M)
  int slow_bwd;    // head_bwd_rows: the general (LDS partial) form for every shape
};

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// dst[e] = src[e] for e < n by the block's threads, 8 loads in flight per thread before
// their LDS stores (a load -> store per iteration waits out one memory latency each)
template <typename S>
__device__ __forceinline__ void lds_copy(float* dst, const S* __restrict__ src, int n) {
  constexpr int U = 8;
  if constexpr (sizeof(S) == 4) {  // fp32: 16-byte pieces when aligned
    if ((((uintptr_t)src | (uintptr_t)dst) & 15) == 0) {
      const int n4 = n / 4, nt = blockDim.x;
      const float4* s4 = reinterpret_cast<const float4*>(src);
      float4* d4 = reinterpret_cast<float4*>(dst);
      int e0 = threadIdx.x;
      for (; e0 + (U - 1) * nt < n4; e0 += U * nt) {
        float4 v[U];
#pragma unroll
        for (int q = 0; q < U; ++q) v[q] = s4[e0 + q * nt];
#pragma unroll
        for (int q = 0; q < U; ++q) d4[e0 + q * nt] = v[q];
      }
      for (; e0 < n4; e0 += nt) d4[e0] = s4[e0];
      for (int e = 4 * n4 + threadIdx.x; e < n; e += nt) dst[e] = src[e];
      return;
    }
  }
  const int nt = blockDim.x;
  int e0 = threadIdx.x;
  for (; e0 + (U - 1) * nt < n; e0 += U * nt) {
    float v[U];
#pragma unroll
    for (int q = 0; q < U; ++q) v[q] = to_f32(src[e0 + q * nt]);
#pragma unroll
    for (int q = 0; q < U; ++q) dst[e0 + q * nt] = v[q];
  }
  for (; e0 < n; e0 += nt) dst[e0] = to_f32(src[e0]);
}

template <typename T>
__device__ __forceinline__ float4 ld4(const T* p) {
  if constexpr (sizeof(T) == 4) {
    return *reinterpret_cast<const float4*>(p);
  } else {
    const uint2 r = *reinterpret_cast<const uint2*>(p);
    return make_float4(__uint_as_float(r.x << 16), __uint_as_float(r.x & 0xffff0000u),
                       __uint_as_float(r.y << 16), __uint_as_float(r.y & 0xffff0000u));
  }
}
template <typename T>
__device__ __forceinline__ void st4(T* p, float4 v) {
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<float4*>(p) = v;
  } else {
    *reinterpret_cast<uint2*>(p) = make_uint2(pack_bf16x2(v.x, v.y), pack_bf16x2(v.z, v.w));
  }
}

// v of lane ^ o for the row reductions; offset 4 as two DPP moves (row_half_mirror gives
// lane ^ 7 within 8 lanes, quad_perm [3,2,1,0] then ^ 3) instead of an LDS permute
__device__ __forceinline__ float xor_red(float v, int o) {
  if (o == 4) {
    const int x = __builtin_bit_cast(int, v);
    const int m = __builtin_amdgcn_mov_dpp(x, 0x141, 0xF, 0xF, true);
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(m, 0x1B, 0xF, 0xF, true));
  }
  return xor_shfl(v, o);
}

__device__ __forceinline__ float elu1(float z) { return z > 0.f ? z : expm1f(z); }
__device__ __forceinline__ float delu1(float z) { return z > 0.f ? 1.f : __expf(z); }

__device__ __forceinline__ float pw(const float* const* p, int c, int F, float dflt) {
  const float* q = p[c / F];
  return q != nullptr ? q[c % F] : dflt;
}

// ---- finalize: u channels (one wave each) from the partials (blocks [0, nub)); the v
// side (blocks [nub, ...)): 32 channels per block, 8 lanes per channel splitting the M
// rows (Welford per lane, Chan-combined over the 8 lanes in a fixed xor tree), then
// v_out = lrelu(bn1(v)) transposed into stats; block 0 thread 0 advances the BatchNorms'
// num_batches_tracked (training)
template <typename T>
__global__ void __launch_bounds__(256) head_prep_kernel(HeadArgs a, int training, int nbu,
                                                        const Wf* __restrict__ part,
                                                        const T* __restrict__ v, int nub) {
  const int HF = a.HF, F = a.F, M = a.M;
  float* st = a.stats;
  if (training && blockIdx.x == 0 && threadIdx.x == 0)
    for (int k = 0; k < 2 * MSHA_HEAD_MAX_HEADS; ++k)
      if (a.nbt[k] != nullptr) *a.nbt[k] += 1;
  if ((int)blockIdx.x < nub) {
    const int c = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int lane = threadIdx.x & 63;
    if (c >= HF) return;
    if (!training) {
      if (lane == 0) {
        st[c] = pw(a.urm, c, F, 0.f);
        st[HF + c] = rsqrtf(pw(a.urv, c, F, 1.f) + a.eps);
      }
      return;
    }
    Wf w{0.f, 0.f, 0.f};
    // partials lane, lane + 64, ... combined in that order; 8 loads in flight at a time
    // (one dependent L2 round trip per partial was the kernel's time at ~600 partials)
    int b = lane;
    for (; b + 7 * 64 < nbu; b += 8 * 64) {
      Wf pb[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) pb[q] = part[(int64_t)(b + q * 64) * HF + c];
#pragma unroll
      for (int q = 0; q < 8; ++q) w = wf_combine(w, pb[q]);
    }
    for (; b < nbu; b += 64) w = wf_combine(w, part[(int64_t)b * HF + c]);
#pragma unroll
    for (int o = 1; o < 64; o <<= 1)
      w = wf_combine(w, Wf{__shfl_xor(w.n, o), __shfl_xor(w.mean, o), __shfl_xor(w.m2, o)});
    if (lane == 0) {
      const float var = w.n > 0.f ? w.m2 / w.n : 0.f;
      st[c] = w.mean;
      st[HF + c] = rsqrtf(var + a.eps);
      float* rm = a.urm[c / F];
      if (rm != nullptr) {
        float* rv = a.urv[c / F];
        const float unb = w.n > 1.f ? w.m2 / (w.n - 1.f) : var;
        rm[c % F] = (1.f - a.momentum) * rm[c % F] + a.momentum * w.mean;
        rv[c % F] = (1.f - a.momentum) * rv[c % F] + a.momentum * unb;
      }
    }
    return;
  }
  const int c = ((int)blockIdx.x - nub) * 32 + (threadIdx.x >> 3);
  const int g = threadIdx.x & 7;
  const bool live = c < HF;
  float mean = 0.f, inv = 1.f;
  if (training) {
    Wf w{0.f, 0.f, 0.f};
    if (live)
      for (int j = g; j < M; j += 8) {
        const float x = to_f32(v[(int64_t)j * HF + c]);
        w.n += 1.f;
        const float d = x - w.mean;
        w.mean += d / w.n;
        w.m2 += d * (x - w.mean);
      }
#pragma unroll
    for (int o = 1; o < 8; o <<= 1)
      w = wf_combine(w, Wf{__shfl_xor(w.n, o), __shfl_xor(w.mean, o), __shfl_xor(w.m2, o)});
    const float var = w.n > 0.f ? w.m2 / w.n : 0.f;
    mean = w.mean;
    inv = rsqrtf(var + a.eps);
    if (live && g == 0) {
      float* rm = a.vrm[c / F];
      if (rm != nullptr) {
        float* rv = a.vrv[c / F];
        const float unb = w.n > 1.f ? w.m2 / (w.n - 1.f) : var;
        rm[c % F] = (1.f - a.momentum) * rm[c % F] + a.momentum * w.mean;
        rv[c % F] = (1.f - a.momentum) * rv[c % F] + a.momentum * unb;
      }
    }
  } else if (live) {
    mean = pw(a.vrm, c, F, 0.f);
    inv = rsqrtf(pw(a.vrv, c, F, 1.f) + a.eps);
  }
  if (!live) return;
  if (g == 0) {
    st[2 * HF + c] = mean;
    st[3 * HF + c] = inv;
  }
  const float gm = pw(a.vw, c, F, 1.f), bt = pw(a.vb, c, F, 0.f);
  float* vo = st + 4 * HF;
  for (int j = g; j < M; j += 8) {
    const float z = fmaf(gm * inv, to_f32(v[(int64_t)j * HF + c]) - mean, bt);
    vo[(int64_t)c * M + j] = z > 0.f ? z : z * a.slope;  // vo_t[c][j]
  }
}

// block-shared tables of the row passes
struct HeadShared {
  float* vo;  // HF x M
  float* W;   // KX x M
  float* g;   // u BN weight, bias, mean, invstd (HF each)
  float* b;
  float* mu;
  float* su;
};

__device__ __forceinline__ HeadShared head_shared_load(const HeadArgs& a, float* smem) {
  HeadShared s;
  const int HF = a.HF, M = a.M;
  s.vo = smem;
  s.W = s.vo + HF * M;
  s.g = s.W + a.KX * M;
  s.b = s.g + HF;
  s.mu = s.b + HF;
  s.su = s.mu + HF;
  lds_copy(s.vo, a.stats + 4 * HF, HF * M);
  lds_copy(s.W, a.W, a.KX * M);
  for (int c = threadIdx.x; c < HF; c += blockDim.x) {
    s.g[c] = pw(a.uw, c, a.F, 1.f);
    s.b[c] = pw(a.ub, c, a.F, 0.f);
    s.mu[c] = a.stats[c];
    s.su[c] = a.stats[HF + c];
  }
  return s;
}

// forward of one row up to the log-softmax inputs (wave-cooperative).  Leaves in LDS:
// uo (HF: lrelu(bn(u))), xs (KX: dropout(elu(c))), cp (KX: c, when non-null), fl (M:
// row mask); returns per lane the row's y_j = elu(elu(a_j hg_j)) for j = lane + 64 q,
// and hg_j / a_j when asked.
template <typename T, int QM>
__device__ __forceinline__ void head_row_fwd(const HeadArgs& a, const HeadShared& s, int64_t i,
                                             const T* __restrict__ u, float* uo, float* xs,
                                             float* cp, int* fl, float (&y)[QM],
                                             float (&hgv)[QM], float (&av)[QM]) {
  const int lane = threadIdx.x & 63;
  const int HF = a.HF, F = a.F, M = a.M, KX = a.KX;
  const int32_t lo = a.rowptr[i], hi = a.rowptr[i + 1];
  const int deg = hi - lo;
  for (int c = lane; c < HF; c += 64) {
    const float z = fmaf(s.g[c] * s.su[c], to_f32(u[i * HF + c]) - s.mu[c], s.b[c]);
    uo[c] = z > 0.f ? z : z * a.slope;
  }
  for (int j = lane; j < M; j += 64) fl[j] = 0;
  wave_sync();
  for (int e = lane; e < deg; e += 64) fl[a.col[lo + e]] = 1;
  for (int k = lane; k < KX; k += 64) {
    const int h = k / M, j = k - h * M;
    const float* uh = uo + h * F;
    const float* vh = s.vo + (int64_t)h * F * M + j;
    float c = 0.f;
#pragma unroll 8
    for (int f = 0; f < F; ++f) c = fmaf(uh[f], vh[f * M], c);
    if (cp != nullptr) cp[k] = c;
    xs[k] = elu1(c) * dropout_factor4(a.dx, (uint64_t)i * KX + k);
  }
  wave_sync();
  const float inv = deg > 0 ? 1.f / (float)deg : 0.f;
#pragma unroll
  for (int q = 0; q < QM; ++q) {
    const int j = lane + 64 * q;
    y[q] = -INFINITY;
    hgv[q] = 0.f;
    av[q] = 0.f;
    if (j < M) {
      float hg = 0.f;
#pragma unroll 8
      for (int k = 0; k < KX; ++k) hg = fmaf(xs[k], s.W[k * M + j], hg);
      const float at = (fl[j] ? inv : 0.f) * dropout_factor4(a.dg, (uint64_t)i * M + j);
      hgv[q] = hg;
      av[q] = at;
      y[q] = elu1(elu1(at * hg));
    }
  }
}

template <int QM>
__device__ __forceinline__ float row_lse(const float (&y)[QM]) {
  float mx = -INFINITY;
#pragma unroll
  for (int q = 0; q < QM; ++q) mx = fmaxf(mx, y[q]);
  mx = wave_xor_max<1>(mx);
  float sm = 0.f;
#pragma unroll
  for (int q = 0; q < QM; ++q) sm += y[q] == -INFINITY ? 0.f : __expf(y[q] - mx);
  sm = wave_xor_sum<1>(sm);
  return mx + __logf(sm);
}

template <typename T, int QM>
__global__ void __launch_bounds__(kHeadThreads) head_fwd_kernel(HeadArgs a,
                                                                const T* __restrict__ u,
                                                                T* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const HeadShared s = head_shared_load(a, smem);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float* scratch = s.su + a.HF + w * (a.HF + a.KX + a.M);
  float* uo = scratch;
  float* xs = uo + a.HF;
  int* fl = reinterpret_cast<int*>(xs + a.KX);
  __syncthreads();
  const int64_t nwaves = (int64_t)gridDim.x * (kHeadThreads / 64);
  for (int64_t i = (int64_t)blockIdx.x * (kHeadThreads / 64) + w; i < a.N; i += nwaves) {
    float y[QM], hg[QM], at[QM];
    head_row_fwd<T, QM>(a, s, i, u, uo, xs, nullptr, fl, y, hg, at);
    const float lse = row_lse<QM>(y);
#pragma unroll
    for (int q = 0; q < QM; ++q) {
      const int j = lane + 64 * q;
      if (j < a.M) out[i * a.M + j] = from_f32<T>(y[q] - lse);
    }
    wave_sync();  // this row's LDS reads done before the next row's writes
  }
}

// Forward row pass with the small operands in registers (KX = H*M <= 64, F <= 64): lane
// k = (h, j) holds its column of v_out_h (F values), lane j its column of W (KX values).
// A wave takes kHeadBatch consecutive rows at a time, so the batch's rowptr, u rows and
// edge columns are three rounds of loads in flight together (per row they were a chain
// of dependent round trips); per row the LDS traffic is the row's uo and x vectors, read
// as 16-byte broadcasts.
constexpr int kHeadBatch = 16;
#ifndef HD_DBG
#define HD_DBG 0  // diagnostic builds only: 1 no c dots, 2 no tail, 4 no u loads, 8 no masks
#endif

template <typename T, int FV, int KXV>
__global__ void __launch_bounds__(kHeadThreads) head_fwd_reg_kernel(HeadArgs a,
                                                                    const T* __restrict__ u,
                                                                    T* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int R = kHeadBatch;
  const int HF = a.HF, M = a.M;
  float* g = smem;
  float* b = g + HF;
  float* mu = b + HF;
  float* su = mu + HF;
  for (int c = threadIdx.x; c < HF; c += blockDim.x) {
    g[c] = pw(a.uw, c, FV, 1.f);
    b[c] = pw(a.ub, c, FV, 0.f);
    mu[c] = a.stats[c];
    su[c] = a.stats[HF + c];
  }
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float* uo = su + HF + w * (R * HF + R * KXV + R * 64 + 32);
  float* xs = uo + R * HF;
  int* fl = reinterpret_cast<int*>(xs + R * KXV);  // R x M row masks
  int* rps = fl + R * 64;                            // R + 1 rowptr entries
  const int kh = lane < KXV ? lane / M : 0, kj = lane < KXV ? lane - kh * M : 0;
  float vreg[FV], wreg[KXV];
  const float* vo = a.stats + 4 * HF;
#pragma unroll
  for (int f = 0; f < FV; ++f) vreg[f] = lane < KXV ? vo[(int64_t)(kh * FV + f) * M + kj] : 0.f;
  const int rpt = M <= 32 ? 2 : 1;  // rows per tail pass
  const int half = rpt == 2 ? lane >> 5 : 0, jl = rpt == 2 ? lane & 31 : lane;
#pragma unroll
  for (int k = 0; k < KXV; ++k) wreg[k] = jl < M ? a.W[k * M + jl] : 0.f;
  __syncthreads();
  const int64_t nb = (a.N + R - 1) / R;
  const int64_t nwaves = (int64_t)gridDim.x * (kHeadThreads / 64);
  const int q4 = HF / 4;
  for (int64_t bt = (int64_t)blockIdx.x * (kHeadThreads / 64) + w; bt < nb; bt += nwaves) {
    const int64_t r0 = bt * R;
    const int nr = (int)(a.N - r0 < R ? a.N - r0 : R);
    if (lane <= nr) rps[lane] = a.rowptr[r0 + lane];
    // u rows -> lrelu(bn(u)) in LDS; 8 16-byte loads per lane in flight per round
    constexpr int UL = 8;
    for (int eb4 = 0; eb4 < ((HD_DBG & 4) ? 0 : nr * q4); eb4 += 64 * UL) {
      float4 xq[UL];
#pragma unroll
      for (int t = 0; t < UL; ++t) {
        const int e4 = eb4 + 64 * t + lane;
        const int r = e4 / q4, c = 4 * (e4 - r * q4);
        xq[t] = e4 < nr * q4 ? ld4(u + (r0 + r) * HF + c) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int t = 0; t < UL; ++t) {
      const int e4 = eb4 + 64 * t + lane;
      if (e4 >= nr * q4) break;
      const int r = e4 / q4, c = 4 * (e4 - r * q4);
      const float4 x = xq[t];
      const float xv[4] = {x.x, x.y, x.z, x.w};
      float4 o;
      float* ov = reinterpret_cast<float*>(&o);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float z = fmaf(g[c + t] * su[c + t], xv[t] - mu[c + t], b[c + t]);
        ov[t] = z > 0.f ? z : z * a.slope;
      }
      *reinterpret_cast<float4*>(uo + r * HF + c) = o;
      }
    }
    for (int e = lane; e < R * M; e += 64) fl[(e / M) * 64 + e % M] = 0;
    wave_sync();
    const int32_t eb = rps[0], ee = rps[nr];
    for (int32_t e = eb + lane; e < ((HD_DBG & 8) ? eb : ee); e += 64) {  // edges -> row masks
      int r = 0;
      while (rps[r + 1] <= e) ++r;
      fl[r * 64 + a.col[e]] = 1;
    }
    if (lane < KXV && !(HD_DBG & 1)) {
      for (int r = 0; r < nr; ++r) {
        const float4* u4 = reinterpret_cast<const float4*>(uo + r * HF + kh * FV);
        float c = 0.f;
#pragma unroll
        for (int f4 = 0; f4 < FV / 4; ++f4) {
          const float4 q = u4[f4];
          c = fmaf(q.x, vreg[4 * f4], c);
          c = fmaf(q.y, vreg[4 * f4 + 1], c);
          c = fmaf(q.z, vreg[4 * f4 + 2], c);
          c = fmaf(q.w, vreg[4 * f4 + 3], c);
        }
        xs[r * KXV + lane] = elu1(c) * dropout_factor4(a.dx, (uint64_t)(r0 + r) * KXV + lane);
      }
    }
    wave_sync();
    // two rows per pass when a row fits half the wave (M <= 32: lanes 32.. take row r + 1)
    for (int r2 = 0; r2 < ((HD_DBG & 2) ? 0 : nr); r2 += rpt) {
      const int r = r2 + half;
      const bool act = jl < M && r < nr;
      float y = -INFINITY;
      if (act) {
        const float4* x4 = reinterpret_cast<const float4*>(xs + r * KXV);
        float hg = 0.f;
#pragma unroll
        for (int k4 = 0; k4 < KXV / 4; ++k4) {
          const float4 q = x4[k4];
          hg = fmaf(q.x, wreg[4 * k4], hg);
          hg = fmaf(q.y, wreg[4 * k4 + 1], hg);
          hg = fmaf(q.z, wreg[4 * k4 + 2], hg);
          hg = fmaf(q.w, wreg[4 * k4 + 3], hg);
        }
        const int deg = rps[r + 1] - rps[r];
        const float at = (fl[r * 64 + jl] ? (deg > 0 ? 1.f / (float)deg : 0.f) : 0.f) *
                         dropout_factor4(a.dg, (uint64_t)(r0 + r) * M + jl);
        y = elu1(elu1(at * hg));
      }
      float mx = y;
      for (int o = 1; o < 64 / rpt; o <<= 1) mx = fmaxf(mx, xor_red(mx, o));
      float sm = act ? __expf(y - mx) : 0.f;
      for (int o = 1; o < 64 / rpt; o <<= 1) sm += xor_red(sm, o);
      const float lse = mx + __logf(sm);
      if (act) out[(r0 + r) * M + jl] = from_f32<T>(y - lse);
    }
    wave_sync();  // the batch's LDS reads done before the next batch's writes
  }
}

// Forward row pass on the matrix cores for the R15 shape family (H heads x F, M = 16 MB
// recipients): a wave takes 16 rows; both products run transposed so the first one's
// accumulators ARE the second one's B operand (no LDS round trip between them):
//   C_h^T (M x 16) = v_out_h (M x F) @ uo_h^T (F x 16)    A = v_out_h: registers, B = uo (LDS)
//   x^T = dropout(elu(C^T))                                in the accumulators, k = h M + j
//   hg^T (M x 16) = W^T (M x KX) @ x^T (KX x 16)           A = W^T: registers
// v_mfma_f32_16x16x4_f32 (exact fp32).  The second product walks k in the order the first
// one's accumulators hold it (step (c, q): lane group g supplies k = 16 c + 4 g + q), with
// W^T's A operand loaded in the same order.  Each lane then holds 8 of its row's M = 32
// logits (hg^T rows 16 jb + 4 g + q): GAL scale, elu, elu and the row's log_softmax
// (max / sum over its 8 values, then across the 4 lane groups by xor 16 / 32).
template <typename T, int H, int F, int M>
__global__ void __launch_bounds__(kHeadThreads) head_fwd_mfma_kernel(HeadArgs a,
                                                                     const T* __restrict__ u,
                                                                     T* __restrict__ out) {
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  constexpr int HF = H * F, KX = H * M, MB = M / 16, KB = KX / 16, R = 16;
  constexpr int UP = HF + 1;  // padded uo pitch: lanes r16 read rows UP floats apart
  static_assert(M % 16 == 0 && F % 4 == 0, "head mfma shape");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* g_ = smem;
  float* b_ = g_ + HF;
  float* mu = b_ + HF;
  float* su = mu + HF;
  for (int c = threadIdx.x; c < HF; c += blockDim.x) {
    g_[c] = pw(a.uw, c, F, 1.f);
    b_[c] = pw(a.ub, c, F, 0.f);
    mu[c] = a.stats[c];
    su[c] = a.stats[HF + c];
  }
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int g = lane >> 4, r16 = lane & 15;
  float* uo = su + HF + w * (R * UP + R * M + 32);
  int* fl = reinterpret_cast<int*>(uo + R * UP);  // R x M row masks
  int* rps = fl + R * M;                            // R + 1 rowptr entries
  // A operands (constant): v_out_h rows 16 jb + r16 at f = 4 s + g; W rows k = 16 c + 4 g + q
  // at column 16 jb + r16
  const float* vo = a.stats + 4 * HF;
  float A1[H][MB][F / 4], A2[MB][KB][4];
#pragma unroll
  for (int h = 0; h < H; ++h)
#pragma unroll
    for (int jb = 0; jb < MB; ++jb)
#pragma unroll
      for (int s4 = 0; s4 < F / 4; ++s4)
        A1[h][jb][s4] = vo[(h * F + 4 * s4 + g) * M + 16 * jb + r16];
#pragma unroll
  for (int jb = 0; jb < MB; ++jb)
#pragma unroll
    for (int c = 0; c < KB; ++c)
#pragma unroll
      for (int q = 0; q < 4; ++q) A2[jb][c][q] = a.W[(16 * c + 4 * g + q) * M + 16 * jb + r16];
  __syncthreads();
  const int64_t nb = (a.N + R - 1) / R;
  const int64_t nwaves = (int64_t)gridDim.x * (kHeadThreads / 64);
  for (int64_t bt = (int64_t)blockIdx.x * (kHeadThreads / 64) + w; bt < nb; bt += nwaves) {
    const int64_t r0 = bt * R;
    const int nr = (int)(a.N - r0 < R ? a.N - r0 : R);
    if (lane <= nr) rps[lane] = a.rowptr[r0 + lane];
    // u rows -> lrelu(bn(u)) (padded rows; rows past the batch are zero)
    constexpr int Q4 = HF / 4;
    constexpr int UL = (R * Q4 + 63) / 64;
    float4 xq[UL];
#pragma unroll
    for (int t = 0; t < UL; ++t) {
      const int e4 = 64 * t + lane;
      const int r = e4 / Q4, c = 4 * (e4 - r * Q4);
      xq[t] = r < nr ? ld4(u + (r0 + r) * HF + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int t = 0; t < UL; ++t) {
      const int e4 = 64 * t + lane;
      if (e4 >= R * Q4) break;
      const int r = e4 / Q4, c = 4 * (e4 - r * Q4);
      const float xv[4] = {xq[t].x, xq[t].y, xq[t].z, xq[t].w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float z = fmaf(g_[c + k] * su[c + k], xv[k] - mu[c + k], b_[c + k]);
        uo[r * UP + c + k] = r < nr ? (z > 0.f ? z : z * a.slope) : 0.f;
      }
    }
    for (int e = lane; e < R * M; e += 64) fl[e] = 0;
    wave_sync();
    const int32_t eb = rps[0], ee = rps[nr];
    for (int32_t e = eb + lane; e < ee; e += 64) {
      int r = 0;
      while (rps[r + 1] <= e) ++r;
      fl[r * M + a.col[e]] = 1;
    }
    // C_h^T = v_out_h @ uo_h^T
    f32x4 xc[H][MB];
#pragma unroll
    for (int h = 0; h < H; ++h) {
#pragma unroll
      for (int jb = 0; jb < MB; ++jb) xc[h][jb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s4 = 0; s4 < F / 4; ++s4) {
        const float bv = uo[r16 * UP + h * F + 4 * s4 + g];
#pragma unroll
        for (int jb = 0; jb < MB; ++jb)
          xc[h][jb] = __builtin_amdgcn_mfma_f32_16x16x4f32(A1[h][jb][s4], bv, xc[h][jb], 0, 0, 0);
      }
    }
    // x^T = dropout(elu(C^T)); element (row r0 + r16, k = h M + 16 jb + 4 g + q)
    const uint64_t row = (uint64_t)(r0 + r16);
    // (the 4 consecutive elements q of a lane are one 4-aligned group of the mask stream:
    // one generator call for all four)
#pragma unroll
    for (int h = 0; h < H; ++h)
#pragma unroll
      for (int jb = 0; jb < MB; ++jb) {
        const float4 kf = dropout_factors4(a.dx, row * KX + h * M + 16 * jb + 4 * g);
        const float kq[4] = {kf.x, kf.y, kf.z, kf.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) xc[h][jb][q] = elu1(xc[h][jb][q]) * kq[q];
      }
    // hg^T = W^T @ x^T, k in the accumulators' order
    f32x4 hg[MB];
#pragma unroll
    for (int jb = 0; jb < MB; ++jb) hg[jb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < KB; ++c)
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int jb = 0; jb < MB; ++jb)
          hg[jb] = __builtin_amdgcn_mfma_f32_16x16x4f32(A2[jb][c][q], xc[c / MB][c % MB][q],
                                                        hg[jb], 0, 0, 0);
    // GAL scale, elu, elu, log_softmax over the row's M logits
    const bool rv = r16 < nr;
    const int deg = rv ? rps[r16 + 1] - rps[r16] : 1;
    const float inv = deg > 0 ? 1.f / (float)deg : 0.f;
    float y[MB][4];
    float mx = -INFINITY;
#pragma unroll
    for (int jb = 0; jb < MB; ++jb) {
      const float4 kf = dropout_factors4(a.dg, row * M + 16 * jb + 4 * g);
      const float kq[4] = {kf.x, kf.y, kf.z, kf.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = 16 * jb + 4 * g + q;
        const float at = (rv && fl[r16 * M + j] ? inv : 0.f) * kq[q];
        y[jb][q] = elu1(elu1(at * hg[jb][q]));
        mx = fmaxf(mx, y[jb][q]);
      }
    }
    mx = fmaxf(mx, xor_shfl(mx, 16));
    mx = fmaxf(mx, xor_shfl(mx, 32));
    float sm = 0.f;
#pragma unroll
    for (int jb = 0; jb < MB; ++jb)
#pragma unroll
      for (int q = 0; q < 4; ++q) sm += __expf(y[jb][q] - mx);
    sm += xor_shfl(sm, 16);
    sm += xor_shfl(sm, 32);
    const float lse = mx + __logf(sm);
    if (rv) {
#pragma unroll
      for (int jb = 0; jb < MB; ++jb)
        st4(out + (r0 + r16) * M + 16 * jb + 4 * g,
            make_float4(y[jb][0] - lse, y[jb][1] - lse, y[jb][2] - lse, y[jb][3] - lse));
    }
    wave_sync();  // the batch's LDS reads done before the next batch's writes
  }
}

static size_t fwd_mfma_lds(int HF, int M) {
  return sizeof(float) * (4 * (size_t)HF + (kHeadThreads / 64) *
                          (size_t)(16 * (HF + 1) + 16 * M + 32));
}

static size_t fwd_reg_lds(int HF, int KX) {
  return sizeof(float) * (4 * (size_t)HF + (kHeadThreads / 64) *
                          (size_t)(kHeadBatch * (HF + KX + 64) + 32));
}

// ---- backward
struct HeadBwdWs {
  float* part;     // kHeadBwdWaves x PT partials: dW (KX*M) | dvo (HF*M) | sdb (HF) | sdbx (HF)
  int* wflag;      // kHeadBwdWaves
  float* dz;       // N x HF: BN-input-side gradient of nonzero rows
  uint8_t* rflag;  // N
  float* red;      // PT reduced
  uint64_t* wmask; // ceil(N / 64): rows with a nonzero dout, 64 a word (split form)
  float* coef;     // 5 x HF: the apply's u-side coefficients (mean, invstd, w invstd,
                   // sum dz / N, sum dz xhat / N), written by head_bwd_reduce
};

// head_bwd_rows' register form: the shipped shapes (M <= 32, H M <= 64, H F <= 128, F a
// multiple of 64), one 64-column block of the output row
__host__ __device__ inline bool head_bwd_fast(int QM, int M, int KX, int HF, int F, int slow) {
  return !slow && QM == 1 && M <= 32 && KX <= 64 && HF <= 128 && F % 64 == 0;
}
__host__ __device__ inline int64_t head_pt(int HF, int KX, int M) { return (int64_t)KX * M + (int64_t)HF * M + 2 * HF; }

template <typename T, int QM>
__global__ void __launch_bounds__(64) head_bwd_rows_kernel(HeadArgs a, const T* __restrict__ u,
                                                           const T* __restrict__ dout,
                                                           HeadBwdWs ws, int64_t rows_per_wave) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x;
  const int HF = a.HF, M = a.M, KX = a.KX, F = a.F;
  const int64_t PT = head_pt(HF, KX, M);
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_wave;
  const int64_t r1 = r0 + rows_per_wave < a.N ? r0 + rows_per_wave : a.N;
  HeadShared s{};
  float *uo = nullptr, *xs = nullptr, *cp = nullptr, *dcv = nullptr, *dhg = nullptr;
  int* fl = nullptr;
  float *P = nullptr, *PW = nullptr, *Pvo = nullptr, *Pdb = nullptr, *Pdbx = nullptr;
  bool any = false;
  // fast form (the shipped shapes: M <= 32, H M <= 64, H F <= 128, F a multiple of 64):
  // the wave's partials live in registers -- lane k owns W[k][.] and dW[k][.], lane c (and
  // c + 64) owns v_out[c][.] and its partial -- and the per-column vectors travel by
  // v_readlane, so a flagged row costs ~200 VALU instead of ~100 LDS read-modify-write
  // round trips in two serial j loops (the slow form, kept for other shapes)
  const bool fast = head_bwd_fast(QM, M, KX, HF, F, a.slow_bwd);
  // (W and v_out are read from column-major copies in the unused partial area: lane k / c
  // reads consecutive words, conflict free)
  float rPW[32], rPvo[2][32], rPdb[2] = {0.f, 0.f}, rPdbx[2] = {0.f, 0.f};
  float *Wt = nullptr, *vot = nullptr;
#pragma unroll
  for (int j = 0; j < 32; ++j) rPW[j] = rPvo[0][j] = rPvo[1][j] = 0.f;
  // 64 rows per pass: each lane reads one row's dout (all loads in flight together);
  // the nonzero rows are then processed in ascending order
  for (int64_t base = r0; base < r1; base += 64) {
    const int64_t ri = base + lane;
    bool nzl = false;
    if (ri < r1) {
      const T* dr = dout + ri * M;
      int nzi = 0;
      if (M % 4 == 0) {  // 16-byte pieces of the row, 8 in flight
        int j = 0;
        for (; j + 32 <= M; j += 32) {
          float4 q[8];
#pragma unroll
          for (int t = 0; t < 8; ++t) q[t] = ld4(dr + j + 4 * t);
#pragma unroll
          for (int t = 0; t < 8; ++t)
            nzi |= (q[t].x != 0.f) | (q[t].y != 0.f) | (q[t].z != 0.f) | (q[t].w != 0.f);
        }
        for (; j < M; j += 4) {
          const float4 q = ld4(dr + j);
          nzi |= (q.x != 0.f) | (q.y != 0.f) | (q.z != 0.f) | (q.w != 0.f);
        }
      } else {
#pragma unroll 8
        for (int j = 0; j < M; ++j) nzi |= to_f32(dr[j]) != 0.f;
      }
      nzl = nzi != 0;
      ws.rflag[ri] = nzl ? 1 : 0;
    }
    uint64_t mask = __ballot(nzl);
    if (mask != 0ull && !any) {  // first nonzero row of this wave: tables and partials
      any = true;
      s = head_shared_load(a, smem);
      uo = s.su + HF;
      xs = uo + HF;
      cp = xs + KX;
      dcv = cp + KX;
      dhg = dcv + KX;
      fl = reinterpret_cast<int*>(dhg + M);
      P = reinterpret_cast<float*>(fl + M);
      PW = P;
      Pvo = PW + (int64_t)KX * M;
      Pdb = Pvo + (int64_t)HF * M;
      Pdbx = Pdb + HF;
      if (!fast)
        for (int64_t t = lane; t < PT; t += 64) P[t] = 0.f;
      __syncthreads();
      if (fast) {  // Wt[j][k] (32 x 64), vot[j][c] (32 x 128), zero-padded
        Wt = P;
        vot = P + 32 * 64;
        for (int t = lane; t < 32 * 64; t += 64) {
          const int j = t >> 6, k = t & 63;
          Wt[t] = k < KX && j < M ? s.W[k * M + j] : 0.f;
        }
        for (int t = lane; t < 32 * 128; t += 64) {
          const int j = t >> 7, c = t & 127;
          vot[t] = c < HF && j < M ? s.vo[c * M + j] : 0.f;
        }
        __syncthreads();
      }
    }
    while (mask != 0ull) {
    const int bit = __builtin_ctzll(mask);
    mask &= mask - 1ull;
    const int64_t i = base + bit;
    float dov[QM];
#pragma unroll
    for (int q = 0; q < QM; ++q) {
      const int j = lane + 64 * q;
      dov[q] = j < M ? to_f32(dout[i * M + j]) : 0.f;
    }
    float y[QM], hg[QM], at[QM];
    head_row_fwd<T, QM>(a, s, i, u, uo, xs, cp, fl, y, hg, at);
    const float lse = row_lse<QM>(y);
    float sdo = 0.f;
#pragma unroll
    for (int q = 0; q < QM; ++q) sdo += dov[q];
    sdo = wave_xor_sum<1>(sdo);
    if (fast) {
      // lane j < M: this row's gradient at the GAL output column j
      float dh = 0.f;
      if (lane < M) {
        const float dy = dov[0] - __expf(y[0] - lse) * sdo;
        const float z = at[0] * hg[0];
        const float g = elu1(z);
        dh = dy * delu1(g) * delu1(z) * at[0];
      }
      // lane k < KX: dx_k = sum_j dh_j W[k][j]; dW partial += x_k dh_j
      const float xk = lane < KX ? xs[lane] : 0.f;
      float dx = 0.f;
#pragma unroll
      for (int j = 0; j < 32; ++j) {
        const float d = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dh), j));
        dx = fmaf(d, Wt[j * 64 + lane], dx);
        rPW[j] = fmaf(xk, d, rPW[j]);
      }
      float dck = 0.f;
      if (lane < KX) {
        const float keep = dropout_factor4(a.dx, (uint64_t)i * KX + lane);
        dck = dx * keep * delu1(cp[lane]);
      }
      // lanes c, c + 64 < HF (head h = c / F, uniform per half): d u_out[c], its BN input
      // gradient and the v_out / BatchNorm partials
#pragma unroll
      for (int pp = 0; pp < 2; ++pp) {
        const int c = lane + 64 * pp;
        const int hb = (64 * pp / F) * M;  // first lane of this head's dcv
        const float uc = c < HF ? uo[c] : 0.f;
        float duo = 0.f;
#pragma unroll
        for (int j = 0; j < 32; ++j) {
          const float d = j < M ? __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dck),
                                                                          min(hb + j, 63)))
                                : 0.f;
          duo = fmaf(d, vot[j * 128 + c], duo);
          rPvo[pp][j] = fmaf(d, uc, rPvo[pp][j]);
        }
        if (c < HF) {
          const float xhat = (to_f32(u[i * HF + c]) - s.mu[c]) * s.su[c];
          const float zb = fmaf(s.g[c], xhat, s.b[c]);
          const float dz = duo * (zb > 0.f ? 1.f : a.slope);
          rPdb[pp] += dz;
          rPdbx[pp] = fmaf(dz, xhat, rPdbx[pp]);
          ws.dz[i * HF + c] = dz;
        }
      }
      wave_sync();  // uo / xs / cp reads done before the next row's head_row_fwd writes
      continue;
    }
#pragma unroll
    for (int q = 0; q < QM; ++q) {
      const int j = lane + 64 * q;
      if (j < M) {
        // log_softmax, elu, elu, the GAL attention scale
        const float dy = dov[q] - __expf(y[q] - lse) * sdo;
        const float z = at[q] * hg[q];
        const float g = elu1(z);
        dhg[j] = dy * delu1(g) * delu1(z) * at[q];
      }
    }
    wave_sync();
    for (int k = lane; k < KX; k += 64) {
      float dx = 0.f;
      const float xk = xs[k];
#pragma unroll 8
      for (int j = 0; j < M; ++j) {
        const float d = dhg[j];
        dx = fmaf(d, s.W[k * M + j], dx);
        PW[k * M + j] = fmaf(xk, d, PW[k * M + j]);
      }
      const float keep = dropout_factor4(a.dx, (uint64_t)i * KX + k);
      dcv[k] = dx * keep * delu1(cp[k]);
    }
    wave_sync();
    for (int c = lane; c < HF; c += 64) {
      const int h = c / F;
      const float* dch = dcv + h * M;
      const float* voc = s.vo + (int64_t)c * M;
      float* pv = Pvo + (int64_t)c * M;
      const float uc = uo[c];
      float duo = 0.f;
#pragma unroll 8
      for (int j = 0; j < M; ++j) {
        duo = fmaf(dch[j], voc[j], duo);
        pv[j] = fmaf(dch[j], uc, pv[j]);
      }
      const float xhat = (to_f32(u[i * HF + c]) - s.mu[c]) * s.su[c];
      const float zb = fmaf(s.g[c], xhat, s.b[c]);
      const float dz = duo * (zb > 0.f ? 1.f : a.slope);
      Pdb[c] += dz;
      Pdbx[c] = fmaf(dz, xhat, Pdbx[c]);
      ws.dz[i * HF + c] = dz;
    }
    wave_sync();
    }
  }
  if (lane == 0) ws.wflag[blockIdx.x] = any ? 1 : 0;
  if (any) {
    float* dst = ws.part + (int64_t)blockIdx.x * PT;
    if (fast) {  // the register partials in the slow form's layout
      if (lane < KX)
#pragma unroll
        for (int j = 0; j < 32; ++j)
          if (j < M) dst[lane * M + j] = rPW[j];
#pragma unroll
      for (int pp = 0; pp < 2; ++pp) {
        const int c = lane + 64 * pp;
        if (c < HF) {
#pragma unroll
          for (int j = 0; j < 32; ++j)
            if (j < M) dst[(int64_t)KX * M + c * M + j] = rPvo[pp][j];
          dst[(int64_t)KX * M + (int64_t)HF * M + c] = rPdb[pp];
          dst[(int64_t)KX * M + (int64_t)HF * M + HF + c] = rPdbx[pp];
        }
      }
    } else {
      for (int64_t t = lane; t < PT; t += 64) dst[t] = P[t];
    }
  }
}

// Split form of the backward row pass for the shipped shapes (head_bwd_fast): a scan
// launch flags the rows whose dout is nonzero (rflag, and one 64-row bit mask a word),
// then G single-wave blocks take the flagged rows k = b, b + G, ... (ascending row order).
// In the one-launch form a flagged row's wave first scanned its 32 rows behind ~1200
// LDS-heavy waves and then loaded the tables; here the G blocks load the tables while
// locating their rows, and only they hold the LDS image.
template <typename T>
__global__ void __launch_bounds__(256) head_bwd_scan_kernel(const T* __restrict__ dout,
                                                            int64_t N, int M,
                                                            uint8_t* __restrict__ rflag,
                                                            uint64_t* __restrict__ wmask) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  int nzi = 0;
  if (i < N) {
    const T* dr = dout + i * M;
    if (M % 4 == 0) {
      int j = 0;
      for (; j + 32 <= M; j += 32) {
        float4 q[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) q[t] = ld4(dr + j + 4 * t);
#pragma unroll
        for (int t = 0; t < 8; ++t)
          nzi |= (q[t].x != 0.f) | (q[t].y != 0.f) | (q[t].z != 0.f) | (q[t].w != 0.f);
      }
      for (; j < M; j += 4) {
        const float4 q = ld4(dr + j);
        nzi |= (q.x != 0.f) | (q.y != 0.f) | (q.z != 0.f) | (q.w != 0.f);
      }
    } else {
      for (int j = 0; j < M; ++j) nzi |= to_f32(dr[j]) != 0.f;
    }
    rflag[i] = nzi ? 1 : 0;
  }
  const uint64_t bits = __ballot(nzi != 0);
  if ((threadIdx.x & 63) == 0 && i < N) wmask[i >> 6] = bits;
}

// diagnostic build (-DSK_TIMELINE): lane 0 of each rows2 block stamps (wall clock, shader
// clock) pairs at its marks into slot blockIdx.x of the buffer msha_debug_head_timeline
// installs (scripts/head_timeline.py); marks compile to nothing in the shipped build
#ifdef SK_TIMELINE
__device__ uint64_t* g_head_tl = nullptr;
#define HTL_MARK(k)                                                                   \
  do {                                                                                \
    if (g_head_tl != nullptr && (threadIdx.x & 63) == 0 && (k) < 31) {                \
      const int sl_ = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);           \
      g_head_tl[sl_ * 64 + 2 * (k)] = __builtin_amdgcn_s_memrealtime();               \
      g_head_tl[sl_ * 64 + 2 * (k) + 1] = __builtin_amdgcn_s_memtime();               \
    }                                                                                 \
  } while (0)
// head_bwd_apply: slot 1024 + block, lane 0 of thread 0
#define HTL_MARKA(k)                                                                  \
  do {                                                                                \
    if (g_head_tl != nullptr && threadIdx.x == 0 && (k) < 31) {                       \
      g_head_tl[(1024 + blockIdx.x) * 64 + 2 * (k)] = __builtin_amdgcn_s_memrealtime(); \
      g_head_tl[(1024 + blockIdx.x) * 64 + 2 * (k) + 1] = __builtin_amdgcn_s_memtime(); \
    }                                                                                 \
  } while (0)
#else
#define HTL_MARK(k) \
  do {              \
  } while (0)
#define HTL_MARKA(k) \
  do {               \
  } while (0)
#endif

template <typename T>
__global__ void __launch_bounds__(256) head_bwd_rows2_kernel(HeadArgs a, const T* __restrict__ u,
                                                             const T* __restrict__ dout,
                                                             HeadBwdWs ws, int nwords) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int HF = a.HF, M = a.M, KX = a.KX, F = a.F;
  const int64_t PT = head_pt(HF, KX, M);
  // 4 waves a block: they stage the tables together (a one-wave block spent ~12 us of its
  // ~30 us there, its LDS transposes one dependent round trip per element), then each
  // takes the flagged rows slot, slot + 4 G, ... with its own scratch and partial slot
  const int G = (int)gridDim.x, b = (int)blockIdx.x, slot = 4 * b + wv;
  HTL_MARK(0);
  // flagged rows per lane's mask words, and their prefix over the lanes
  const int per = (nwords + 63) / 64;
  const int w0 = lane * per;
  int cnt = 0;
  for (int q0 = 0; q0 < per; q0 += 8) {
    uint64_t mw[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) mw[q] = q0 + q < per && w0 + q0 + q < nwords ? ws.wmask[w0 + q0 + q] : 0ull;
#pragma unroll
    for (int q = 0; q < 8; ++q) cnt += __popcll(mw[q]);
  }
  int incl = cnt;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(incl, o);
    if (lane >= o) incl += y;
  }
  const int nl = __shfl(incl, 63);
  HTL_MARK(1);
  if (4 * b >= nl) {  // (uniform over the block)
    if (lane == 0) ws.wflag[slot] = 0;
    return;
  }
  // the k-th flagged row: the lane whose words hold it walks them, 8 words a round trip
  auto locate = [&](int k) -> int64_t {
    const int L = __builtin_ctzll(__ballot(incl > k));
    int row = 0;
    if (lane == L) {
      int r = k - (incl - cnt);
      for (int q0 = 0; q0 < per; q0 += 8) {
        uint64_t mw[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) mw[q] = q0 + q < per && w0 + q0 + q < nwords ? ws.wmask[w0 + q0 + q] : 0ull;
        bool found = false;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int pc = __popcll(mw[q]);
          if (!found && r < pc) {
            uint64_t m = mw[q];
            for (int t = 0; t < r; ++t) m &= m - 1ull;
            row = (w0 + q0 + q) * 64 + __builtin_ctzll(m);
            found = true;
          }
          if (!found) r -= pc;
        }
        if (found) break;
      }
    }
    return __builtin_amdgcn_readlane(row, L);
  };
  // a row's global inputs, loaded ahead: its GAL adjacency row (rowptr, columns), dout row,
  // u row (lanes c, c + 64).  The first row's loads are in flight while the tables stage.
  struct Pre {
    int32_t lo, hi, col;
    float dov, u0, u1;
  };
  auto prefetch = [&](int64_t i, Pre& p) {
    p.lo = a.rowptr[i];
    p.hi = a.rowptr[i + 1];
    p.dov = lane < M ? to_f32(dout[i * M + lane]) : 0.f;
    p.u0 = lane < HF ? to_f32(u[i * HF + lane]) : 0.f;
    p.u1 = lane + 64 < HF ? to_f32(u[i * HF + 64 + lane]) : 0.f;
    p.col = lane < p.hi - p.lo ? a.col[p.lo + lane] : 0;
  };
  int64_t i_nx = slot < nl ? locate(slot) : 0;
  Pre pre{};
  if (slot < nl) prefetch(i_nx, pre);
  const HeadShared s = head_shared_load(a, smem);
  // W / v_out column-major (lane k / c then reads consecutive words), zero-padded
  float* Wt = s.su + HF;
  float* vot = Wt + 32 * 64;
  float* uo = vot + 32 * 128 + wv * (HF + 3 * KX + 2 * M);  // this wave's scratch
  float* xs = uo + HF;
  float* cp = xs + KX;
  int* fl = reinterpret_cast<int*>(cp + 2 * KX + M);
  __syncthreads();
  for (int t = threadIdx.x; t < 32 * 64; t += 256) {
    const int j = t >> 6, k = t & 63;
    Wt[t] = k < KX && j < M ? s.W[k * M + j] : 0.f;
  }
  for (int t = threadIdx.x; t < 32 * 128; t += 256) {
    const int j = t >> 7, c = t & 127;
    vot[t] = c < HF && j < M ? s.vo[c * M + j] : 0.f;
  }
  __syncthreads();
  HTL_MARK(2);
  if (slot >= nl) {  // (no barrier after this point)
    if (lane == 0) ws.wflag[slot] = 0;
    return;
  }
  float rPW[32], rPvo[2][32], rPdb[2] = {0.f, 0.f}, rPdbx[2] = {0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 32; ++j) rPW[j] = rPvo[0][j] = rPvo[1][j] = 0.f;
  int tlk = 3;
  for (int k = slot; k < nl; k += 4 * G) {
    const int64_t i = i_nx;
    const Pre cur = pre;
    if (k + 4 * G < nl) {  // the next row's loads go out before this row's work
      i_nx = locate(k + 4 * G);
      prefetch(i_nx, pre);
    }
    HTL_MARK(tlk);
    // the row's forward up to the log-softmax inputs (head_row_fwd, QM = 1, on the
    // prefetched inputs)
    const float dov = cur.dov;
    // this lane's x dropout factor (element i KX + lane), used forward and backward
    const float kx = lane < KX ? dropout_factor4(a.dx, (uint64_t)i * KX + lane) : 0.f;
    float y[1], hg[1], at[1];
    {
      const int deg = cur.hi - cur.lo;
#pragma unroll
      for (int pp = 0; pp < 2; ++pp) {
        const int c = lane + 64 * pp;
        if (c < HF) {
          const float z = fmaf(s.g[c] * s.su[c], (pp ? cur.u1 : cur.u0) - s.mu[c], s.b[c]);
          uo[c] = z > 0.f ? z : z * a.slope;
        }
      }
      if (lane < M) fl[lane] = 0;
      wave_sync();
      if (lane < deg) fl[cur.col] = 1;
      if (lane < KX) {
        const int h = lane / M, j = lane - h * M;
        const float* uh = uo + h * F;
        const float* vh = s.vo + (int64_t)h * F * M + j;
        float c = 0.f;
#pragma unroll 8
        for (int f = 0; f < F; ++f) c = fmaf(uh[f], vh[f * M], c);
        cp[lane] = c;
        xs[lane] = elu1(c) * kx;
      }
      wave_sync();
      const float inv = deg > 0 ? 1.f / (float)deg : 0.f;
      y[0] = -INFINITY;
      hg[0] = 0.f;
      at[0] = 0.f;
      if (lane < M) {
        float hv = 0.f;
#pragma unroll 8
        for (int kk = 0; kk < KX; ++kk) hv = fmaf(xs[kk], s.W[kk * M + lane], hv);
        const float av = (fl[lane] ? inv : 0.f) * dropout_factor4(a.dg, (uint64_t)i * M + lane);
        hg[0] = hv;
        at[0] = av;
        y[0] = elu1(elu1(av * hv));
      }
    }
    HTL_MARK(tlk + 1);
    const float lse = row_lse<1>(y);
    const float sdo = wave_xor_sum<1>(dov);
    // lane j < M: this row's gradient at the GAL output column j
    float dh = 0.f;
    if (lane < M) {
      const float dy = dov - __expf(y[0] - lse) * sdo;
      const float z = at[0] * hg[0];
      const float g = elu1(z);
      dh = dy * delu1(g) * delu1(z) * at[0];
    }
    // lane k < KX: dx_k = sum_j dh_j W[k][j]; dW partial += x_k dh_j
    const float xk = lane < KX ? xs[lane] : 0.f;
    float dx = 0.f;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      const float d = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dh), j));
      dx = fmaf(d, Wt[j * 64 + lane], dx);
      rPW[j] = fmaf(xk, d, rPW[j]);
    }
    float dck = 0.f;
    if (lane < KX) dck = dx * kx * delu1(cp[lane]);
    // lanes c, c + 64 < HF (head h = c / F, uniform per half): d u_out[c], its BN input
    // gradient and the v_out / BatchNorm partials
#pragma unroll
    for (int pp = 0; pp < 2; ++pp) {
      const int c = lane + 64 * pp;
      const int hb = (64 * pp / F) * M;  // first lane of this head's dcv
      const float uc = c < HF ? uo[c] : 0.f;
      float duo = 0.f;
#pragma unroll
      for (int j = 0; j < 32; ++j) {
        const float d = j < M ? __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dck),
                                                                        min(hb + j, 63)))
                              : 0.f;
        duo = fmaf(d, vot[j * 128 + c], duo);
        rPvo[pp][j] = fmaf(d, uc, rPvo[pp][j]);
      }
      if (c < HF) {
        const float xhat = ((pp ? cur.u1 : cur.u0) - s.mu[c]) * s.su[c];
        const float zb = fmaf(s.g[c], xhat, s.b[c]);
        const float dz = duo * (zb > 0.f ? 1.f : a.slope);
        rPdb[pp] += dz;
        rPdbx[pp] = fmaf(dz, xhat, rPdbx[pp]);
        ws.dz[i * HF + c] = dz;
      }
    }
    wave_sync();  // uo / xs / cp reads done before the next row's writes
    HTL_MARK(tlk + 2);
    tlk += 3;
  }
  if (lane == 0) ws.wflag[slot] = 1;
  // column-major W / v_out blocks ([j][k], [j][c]: the lanes' stores coalesce; the
  // row-major form put each store's 64 lanes on 64 lines), head_bwd_reduce(tr = 1) maps back
  float* dst = ws.part + (int64_t)slot * PT;
  if (lane < KX)
#pragma unroll
    for (int j = 0; j < 32; ++j)
      if (j < M) dst[j * KX + lane] = rPW[j];
#pragma unroll
  for (int pp = 0; pp < 2; ++pp) {
    const int c = lane + 64 * pp;
    if (c < HF) {
#pragma unroll
      for (int j = 0; j < 32; ++j)
        if (j < M) dst[(int64_t)KX * M + j * HF + c] = rPvo[pp][j];
      dst[(int64_t)KX * M + (int64_t)HF * M + c] = rPdb[pp];
      dst[(int64_t)KX * M + (int64_t)HF * M + HF + c] = rPdbx[pp];
    }
  }
  HTL_MARK(30);
}

// reduced[t] = sum over flagged waves (ascending) of part[w][t]; dW and the u-side
// BatchNorm weight / bias gradients written out
// tr: partials in the split form's layout (W and v_out blocks column-major: [j][k] and
// [j][c], so that its lanes' stores were coalesced); the reduced vector is row-major either way
__global__ void __launch_bounds__(256) head_bwd_reduce_kernel(HeadArgs a, HeadBwdWs ws, int nw,
                                                              float* __restrict__ dW,
                                                              float* __restrict__ dzero,
                                                              int64_t n_zero, int tr) {
  if (blockIdx.x == 0)  // the out_att score vector's (exactly zero) gradient
    for (int64_t e = threadIdx.x; e < n_zero; e += blockDim.x) dzero[e] = 0.f;
  __shared__ int list[kHeadBwdWaves];
  __shared__ int wsum[4];
  // ordered compaction of the wave flags: each thread a contiguous slice of them (its
  // flags loaded together into a bit mask), the slice counts scanned by wave shuffles
  // (a serial scan over 256 counts on one lane was a chain of LDS round trips)
  const int per = (nw + 255) / 256;  // <= kHeadBwdWaves / 256 = 16
  const int b0 = threadIdx.x * per;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t bits = 0;
  for (int q = 0; q < per; ++q)
    if (b0 + q < nw && ws.wflag[b0 + q]) bits |= 1u << q;
  const int c = __popc(bits);
  int x = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  int pos = x - c;
  for (int q = 0; q < w; ++q) pos += wsum[q];
  for (int q = 0; q < per; ++q)
    if ((bits >> q) & 1u) list[pos++] = b0 + q;
  __syncthreads();
  const int nl = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  const int64_t PT = head_pt(a.HF, a.KX, a.M);
  // 64 entries a block, 4 threads an entry: thread quarter w sums list entries
  // [w nl / 4, (w + 1) nl / 4) in order (16 in flight), then the 4 sums add in quarter
  // order (one round of loads per thread at 64 flagged slots instead of four)
  __shared__ float qsum[4][64];
  const int64_t t = (int64_t)blockIdx.x * 64 + lane;
  float sum = 0.f;
  if (t < PT) {
    const int l0 = w * nl / 4, l1 = (w + 1) * nl / 4;
    int l = l0;
    for (; l + 16 <= l1; l += 16) {
      float v[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) v[q] = ws.part[(int64_t)list[l + q] * PT + t];
#pragma unroll
      for (int q = 0; q < 16; ++q) sum += v[q];
    }
    for (; l < l1; ++l) sum += ws.part[(int64_t)list[l] * PT + t];
  }
  qsum[w][lane] = sum;
  __syncthreads();
  if (w != 0 || t >= PT) return;
  sum = ((qsum[0][lane] + qsum[1][lane]) + qsum[2][lane]) + qsum[3][lane];
  const int64_t nW = (int64_t)a.KX * a.M, nV = (int64_t)a.HF * a.M;
  int64_t o = t;
  if (tr && t < nW) {
    o = (t % a.KX) * a.M + t / a.KX;
  } else if (tr && t < nW + nV) {
    const int64_t r = t - nW;
    o = nW + (r % a.HF) * a.M + r / a.HF;
  }
  ws.red[o] = sum;
  if (o < nW) {
    dW[o] = sum;
  } else if (o >= nW + nV) {
    const int64_t r = o - nW - nV;
    const int ch = (int)(r % a.HF);
    const float invN = 1.f / (float)a.N;
    if (r < a.HF) {
      const float* st = a.stats;
      ws.coef[ch] = st[ch];
      ws.coef[a.HF + ch] = st[a.HF + ch];
      ws.coef[2 * a.HF + ch] = pw(a.uw, ch, a.F, 1.f) * st[a.HF + ch];
      ws.coef[3 * a.HF + ch] = sum * invN;
    } else {
      ws.coef[4 * a.HF + ch] = sum * invN;
    }
    float* const* dst = r < a.HF ? a.dub : a.duw;  // sdb = d bias, sdbx = d weight
    float* d = dst[ch / a.F];
    if (d != nullptr) d[ch % a.F] = sum;
  }
}

// du for every row; block 0: the v side's BatchNorm backward (M rows, one thread per
// channel, rows in order)
// du for every row (4 channels per thread); block 0: the v side's BatchNorm backward
// (M rows, one thread per channel, rows in order, v and d v_out staged in LDS)
template <typename T>
__global__ void __launch_bounds__(256) head_bwd_apply_kernel(HeadArgs a, const T* __restrict__ u,
                                                             const T* __restrict__ v,
                                                             HeadBwdWs ws, T* __restrict__ du,
                                                             T* __restrict__ dv) {
  const int HF = a.HF, M = a.M, F = a.F;
  const float* red = ws.red;
  const int64_t nW = (int64_t)a.KX * M, nV = (int64_t)HF * M;
  const float* dvo = red + nW;  // [c][j]
  const float* sdb = red + nW + nV;
  const float* sdbx = sdb + HF;
  const float* st = a.stats;
  HTL_MARKA(0);
  // blocks [0, nvb): the v side's BatchNorm backward, 32 channels a block, 8 row groups a
  // channel (row sums: the 8 groups' partials added in group order through LDS); a single
  // block walking every channel's M rows twice was this kernel's tail (12.6 us at R15)
  const int nvb = (HF + 31) / 32;
  __shared__ float2 vred[8][32];
  if ((int)blockIdx.x < nvb) {
    const int cl = threadIdx.x & 31, g = threadIdx.x >> 5;
    const int c = (int)blockIdx.x * 32 + cl;
    const bool live = c < HF;
    const float mean = live ? st[2 * HF + c] : 0.f, inv = live ? st[3 * HF + c] : 0.f;
    const float gw = live ? pw(a.vw, c, F, 1.f) : 0.f, gb = live ? pw(a.vb, c, F, 0.f) : 0.f;
    constexpr int RJ = 32;  // rows per thread (M <= 256 = 8 RJ)
    float xh[RJ], dz[RJ];
    float db = 0.f, dw = 0.f;
#pragma unroll
    for (int r = 0; r < RJ; ++r) {
      const int j = g + 8 * r;
      xh[r] = 0.f;
      dz[r] = 0.f;
      if (live && j < M) {
        xh[r] = (to_f32(v[(int64_t)j * HF + c]) - mean) * inv;
        dz[r] = dvo[(int64_t)c * M + j] * (fmaf(gw, xh[r], gb) > 0.f ? 1.f : a.slope);
        db += dz[r];
        dw = fmaf(dz[r], xh[r], dw);
      }
    }
    vred[g][cl] = make_float2(db, dw);
    __syncthreads();
    db = 0.f;
    dw = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      db += vred[q][cl].x;
      dw += vred[q][cl].y;
    }
    const float invR = 1.f / (float)M;
#pragma unroll
    for (int r = 0; r < RJ; ++r) {
      const int j = g + 8 * r;
      if (live && j < M)
        dv[(int64_t)j * HF + c] = from_f32<T>(gw * inv * (dz[r] - db * invR - xh[r] * dw * invR));
    }
    if (live && g == 0) {
      float* dwp = a.dvw[c / F];
      float* dbp = a.dvb[c / F];
      if (dwp != nullptr) dwp[c % F] = dw;
      if (dbp != nullptr) dbp[c % F] = db;
    }
    HTL_MARKA(30);
    return;
  }
  __shared__ __attribute__((aligned(16))) float sm[5 * 512];
  const float invN = 1.f / (float)a.N;
  const int q = HF / 4;  // float4 groups per row (HF % 4 == 0, checked by the caller)
  const int64_t total = a.N * q;
  const int64_t stride = (int64_t)(gridDim.x - nvb) * blockDim.x;
  constexpr int U = 8;  // elements per thread whose loads are in flight together
  if (blockDim.x % q == 0) {
    // every element of this thread has the same 4 channels (the grid stride is a multiple
    // of q): their 20 coefficients (written by head_bwd_reduce: mean, invstd, w invstd,
    // sum dz / N, sum dz xhat / N) are 5 float4 loads, in flight with the rows' loads
    const int c = 4 * (int)(threadIdx.x % q);
    const int64_t rs = stride / q;  // rows between a thread's consecutive elements
    const int64_t i00 = ((int64_t)(blockIdx.x - nvb) * blockDim.x + threadIdx.x) / q;
    float4 x[U];
    uint8_t nz[U];
#pragma unroll
    for (int t = 0; t < U; ++t) {
      const int64_t i = i00 + t * rs;
      x[t] = i < a.N ? ld4(u + i * HF + c) : make_float4(0.f, 0.f, 0.f, 0.f);
      nz[t] = i < a.N ? ws.rflag[i] : 0;
    }
    float cm[4], ci[4], cw[4], c1[4], c2[4];
    {
      const float4 k0 = *reinterpret_cast<const float4*>(ws.coef + c);
      const float4 k1 = *reinterpret_cast<const float4*>(ws.coef + HF + c);
      const float4 k2 = *reinterpret_cast<const float4*>(ws.coef + 2 * HF + c);
      const float4 k3 = *reinterpret_cast<const float4*>(ws.coef + 3 * HF + c);
      const float4 k4 = *reinterpret_cast<const float4*>(ws.coef + 4 * HF + c);
      cm[0] = k0.x; cm[1] = k0.y; cm[2] = k0.z; cm[3] = k0.w;
      ci[0] = k1.x; ci[1] = k1.y; ci[2] = k1.z; ci[3] = k1.w;
      cw[0] = k2.x; cw[1] = k2.y; cw[2] = k2.z; cw[3] = k2.w;
      c1[0] = k3.x; c1[1] = k3.y; c1[2] = k3.z; c1[3] = k3.w;
      c2[0] = k4.x; c2[1] = k4.y; c2[2] = k4.z; c2[3] = k4.w;
    }
    HTL_MARKA(1);
    for (int64_t i0 = i00;; ) {
#pragma unroll
      for (int t = 0; t < U; ++t) {
        const int64_t i = i0 + t * rs;
        if (i >= a.N) break;
        const float xs[4] = {x[t].x, x[t].y, x[t].z, x[t].w};
        const float4 d4 = nz[t] ? *reinterpret_cast<const float4*>(ws.dz + i * HF + c)
                                : make_float4(0.f, 0.f, 0.f, 0.f);
        const float dzs[4] = {d4.x, d4.y, d4.z, d4.w};
        float r[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float xh = (xs[k] - cm[k]) * ci[k];
          r[k] = cw[k] * (dzs[k] - c1[k] - xh * c2[k]);
        }
        st4(du + i * HF + c, make_float4(r[0], r[1], r[2], r[3]));
      }
      HTL_MARKA(2);
      i0 += U * rs;
      if (i0 >= a.N) break;
#pragma unroll
      for (int t = 0; t < U; ++t) {
        const int64_t i = i0 + t * rs;
        x[t] = i < a.N ? ld4(u + i * HF + c) : make_float4(0.f, 0.f, 0.f, 0.f);
        nz[t] = i < a.N ? ws.rflag[i] : 0;
      }
    }
    HTL_MARKA(30);
    return;
  }
  // per-channel coefficients in LDS: mean, invstd, w * invstd, sum dz / N, sum dz xhat / N
  float* cf = sm;  // 5 * HF <= 2560 floats
  for (int c = threadIdx.x; c < HF; c += blockDim.x) {
    cf[c] = st[c];
    cf[HF + c] = st[HF + c];
    cf[2 * HF + c] = pw(a.uw, c, F, 1.f) * st[HF + c];
    cf[3 * HF + c] = sdb[c] * invN;
    cf[4 * HF + c] = sdbx[c] * invN;
  }
  __syncthreads();
  for (int64_t e0 = (int64_t)(blockIdx.x - nvb) * blockDim.x + threadIdx.x; e0 < total;
       e0 += U * stride) {
    float4 x[U];
    uint8_t nz[U];
    int64_t ri[U];
    int rc[U];
#pragma unroll
    for (int t = 0; t < U; ++t) {
      const int64_t e = e0 + t * stride;
      // (row, channel) of element e: a 32-bit division where e fits (a 64-bit one is a
      // ~100-instruction sequence, and there is one per float4)
      const int64_t i = e >= total ? 0 : total < (int64_t)INT32_MAX ? (int64_t)((uint32_t)e / (uint32_t)q)
                                                                      : e / q;
      const int c = 4 * (int)(e - i * q);
      ri[t] = i;
      rc[t] = c;
      x[t] = e < total ? ld4(u + i * HF + c) : make_float4(0.f, 0.f, 0.f, 0.f);
      nz[t] = e < total ? ws.rflag[i] : 0;
    }
#pragma unroll
    for (int t = 0; t < U; ++t) {
      const int64_t e = e0 + t * stride;
      if (e >= total) break;
      const int64_t i = ri[t];
      const int c = rc[t];
      const float xs[4] = {x[t].x, x[t].y, x[t].z, x[t].w};
      // dz exists only for the rows the loss reaches (64 of ~39k at R15): read for those
      // alone (a dz pass over every row was a third of the kernel's bytes)
      const float4 d4 = nz[t] ? *reinterpret_cast<const float4*>(ws.dz + i * HF + c)
                              : make_float4(0.f, 0.f, 0.f, 0.f);
      const float dzs[4] = {d4.x, d4.y, d4.z, d4.w};
      float r[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int ch = c + k;
        const float xh = (xs[k] - cf[ch]) * cf[HF + ch];
        r[k] = cf[2 * HF + ch] * (dzs[k] - cf[3 * HF + ch] - xh * cf[4 * HF + ch]);
      }
      st4(du + i * HF + c, make_float4(r[0], r[1], r[2], r[3]));
    }
  }
}

static size_t al256(size_t b) { return (b + 255) & ~(size_t)255; }

static size_t fwd_lds(int HF, int KX, int M) {
  return sizeof(float) * ((size_t)HF * M + (size_t)KX * M + 4 * HF +
                          (kHeadThreads / 64) * (size_t)(HF + KX + M));
}
static size_t bwd_lds(int HF, int KX, int M) {
  // (the partial area also holds head_bwd_rows' fast-form W / v_out copies: 32 x 192)
  const size_t pt = (size_t)head_pt(HF, KX, M) > 32 * 192 ? (size_t)head_pt(HF, KX, M) : 32 * 192;
  return sizeof(float) * ((size_t)HF * M + (size_t)KX * M + 4 * HF + HF + 3 * (size_t)KX + 2 * M + pt);
}

struct HeadLayout {
  size_t part_u, part_b, wflag, dz, rflag, red, wmask, coef, total;
};

// rows per wave and waves of the backward row pass (msha_head_bwd launches exactly these)
// rows per wave of the backward row pass (at least kHeadRowsPerWave; MSHA_HEAD_RPW
// overrides the floor, A/B).  Every wave is a block holding the whole backward LDS
// image, so the floor also sets how many rounds of blocks the row scan takes.
static int64_t head_bwd_rpw(int64_t N) {
  static const int64_t floor_rpw = [] {
    const char* v = getenv("MSHA_HEAD_RPW");
    const int64_t x = v != nullptr && *v ? atoll(v) : 0;
    return x > 0 ? x : (int64_t)kHeadRowsPerWave;
  }();
  int64_t rpw = (N + kHeadBwdWaves - 1) / kHeadBwdWaves;
  return rpw < floor_rpw ? floor_rpw : rpw;
}
static int head_bwd_waves(int64_t N) {
  const int64_t rpw = head_bwd_rpw(N);
  return (int)((N + rpw - 1) / rpw);
}

static HeadLayout head_layout(int64_t N, int M, int H, int F) {
  const int HF = H * F, KX = H * M;
  HeadLayout L{};
  size_t off = 0;
  L.part_u = off;
  const size_t fwd = al256((size_t)bn_stats_blocks(N) * HF * sizeof(Wf));
  // backward regions (the forward's partials are dead by then: they alias); one partial
  // slab per wave the row pass launches (<= kHeadBwdWaves)
  const size_t nw = (size_t)head_bwd_waves(N) > 4 ? (size_t)head_bwd_waves(N) : 4;
  L.part_b = 0;
  off = al256(nw * head_pt(HF, KX, M) * sizeof(float));
  L.wflag = off;
  off += al256(nw * sizeof(int));
  L.dz = off;
  off += al256((size_t)N * HF * sizeof(float));
  L.rflag = off;
  off += al256((size_t)N);
  L.red = off;
  off += al256((size_t)head_pt(HF, KX, M) * sizeof(float));
  L.wmask = off;
  off += al256((size_t)((N + 63) / 64) * sizeof(uint64_t));
  L.coef = off;
  off += al256((size_t)5 * HF * sizeof(float));
  L.total = off > fwd ? off : fwd;
  return L;
}

static int head_check(const msha_graph* g, const msha_head_params* hp, int32_t dtype) {
  MSHA_ARG_CHECK(g != nullptr && g->rowptr && g->col && hp != nullptr, "head: null graph/params");
  MSHA_ARG_CHECK(dtype == MSHA_DTYPE_F32 || dtype == MSHA_DTYPE_BF16, "head: bad dtype");
  MSHA_ARG_CHECK(msha_head_supported(g->n_cols, hp->heads, hp->feat), "head: shape not supported");
  MSHA_ARG_CHECK(g->n_rows > 0, "head: no rows");
  return MSHA_OK;
}

static HeadArgs head_args(const msha_graph* g, const msha_head_params* hp, const float* W,
                          float* stats) {
  HeadArgs a{};
  a.N = g->n_rows;
  a.M = (int)g->n_cols;
  a.H = hp->heads;
  a.F = hp->feat;
  a.HF = a.H * a.F;
  a.KX = a.H * a.M;
  a.eps = hp->eps;
  a.momentum = hp->momentum;
  a.slope = hp->slope;
  a.rowptr = g->rowptr;
  a.col = g->col;
  for (int h = 0; h < MSHA_HEAD_MAX_HEADS; ++h) {
    const bool on = h < hp->heads;
    a.uw[h] = on ? hp->u_weight[h] : nullptr;
    a.ub[h] = on ? hp->u_bias[h] : nullptr;
    a.urm[h] = on ? hp->u_running_mean[h] : nullptr;
    a.urv[h] = on ? hp->u_running_var[h] : nullptr;
    a.vw[h] = on ? hp->v_weight[h] : nullptr;
    a.vb[h] = on ? hp->v_bias[h] : nullptr;
    a.vrm[h] = on ? hp->v_running_mean[h] : nullptr;
    a.vrv[h] = on ? hp->v_running_var[h] : nullptr;
    a.duw[h] = on ? hp->du_weight[h] : nullptr;
    a.dub[h] = on ? hp->du_bias[h] : nullptr;
    a.dvw[h] = on ? hp->dv_weight[h] : nullptr;
    a.dvb[h] = on ? hp->dv_bias[h] : nullptr;
    a.nbt[2 * h] = on ? hp->num_batches_tracked[2 * h] : nullptr;
    a.nbt[2 * h + 1] = on ? hp->num_batches_tracked[2 * h + 1] : nullptr;
  }
  a.W = W;
  a.stats = stats;
  return a;
}

}  // namespace msha

using namespace msha;

extern "C" int msha_head_supported(int64_t n_cols, int32_t heads, int32_t feat) {
  if (heads < 1 || heads > MSHA_HEAD_MAX_HEADS || feat < 1 || n_cols < 1) return 0;
  const int64_t HF = (int64_t)heads * feat, KX = heads * n_cols;
  if (HF > 512 || HF % 4 != 0 || n_cols > 256 || KX > 512) return 0;
  return bwd_lds((int)HF, (int)KX, (int)n_cols) <= 150 * 1024 &&
         fwd_lds((int)HF, (int)KX, (int)n_cols) <= 96 * 1024;
}

extern "C" size_t msha_head_workspace_size(const msha_graph* g, int32_t heads, int32_t feat) {
  if (g == nullptr) return 0;
  return head_layout(g->n_rows, (int)g->n_cols, heads, feat).total;
}

extern "C" int msha_head_fwd(const msha_graph* g, const msha_head_params* hp, int32_t dtype,
                             const void* u, const void* v, const float* W, int32_t training,
                             float p_x, uint64_t seed_x, float p_att, uint64_t seed_att,
                             float* stats, void* out, void* ws, size_t ws_bytes,
                             msha_stream_t stream) {
  if (int rc = head_check(g, hp, dtype)) return rc;
  MSHA_ARG_CHECK(u && v && W && stats && out, "head_fwd: null pointer");
  MSHA_ARG_CHECK(p_x >= 0.f && p_x <= 1.f && p_att >= 0.f && p_att <= 1.f, "head_fwd: bad p");
  const HeadLayout L = head_layout(g->n_rows, (int)g->n_cols, hp->heads, hp->feat);
  MSHA_ARG_CHECK(!training || (ws && ws_bytes >= L.total), "head_fwd: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  HeadArgs a = head_args(g, hp, W, stats);
  a.dx = make_dropout(training ? p_x : 0.f, seed_x, 0, s);
  a.dg = make_dropout(training ? p_att : 0.f, seed_att, 0, s);
  const bool bf = dtype == MSHA_DTYPE_BF16;
  int64_t nbu = 0;
  Wf* part = training ? (Wf*)((char*)ws + L.part_u) : nullptr;
  if (training) nbu = bn_stats_partials(a.N, a.HF, bf, u, part, s);
  const int nub = (a.HF + 3) / 4;
  const dim3 gp(nub + (a.HF + 31) / 32);
  if (bf)
    hipLaunchKernelGGL(head_prep_kernel<bf16_t>, gp, dim3(256), 0, s, a, training, (int)nbu, part,
                       (const bf16_t*)v, nub);
  else
    hipLaunchKernelGGL(head_prep_kernel<float>, gp, dim3(256), 0, s, a, training, (int)nbu, part,
                       (const float*)v, nub);
  const dim3 gr(grid_for(a.N, kHeadThreads / 64, 2048));
  const dim3 grb(grid_for((a.N + kHeadBatch - 1) / kHeadBatch, kHeadThreads / 64, 512));
  // matrix-core path: R15's shape (2 heads x 64, 32 recipients)
#define HEAD_FWD_MFMA(T, H_, F_, M_)                                                      \
  if (a.H == H_ && a.F == F_ && a.M == M_) {                                              \
    hipLaunchKernelGGL((head_fwd_mfma_kernel<T, H_, F_, M_>), grb, dim3(kHeadThreads),    \
                       fwd_mfma_lds(H_ * F_, M_), s, a, (const T*)u, (T*)out);            \
    return check_launch("head_fwd");                                                      \
  }
  if (getenv("MSHA_HEAD_MFMA") == nullptr || atoi(getenv("MSHA_HEAD_MFMA")) != 0) {
    if (bf) {
      HEAD_FWD_MFMA(bf16_t, 2, 64, 32)
    } else {
      HEAD_FWD_MFMA(float, 2, 64, 32)
    }
  }
#undef HEAD_FWD_MFMA
  // register-resident path: KX = H*M of 32 or 64 and F of 16 / 32 / 64
#define HEAD_FWD_REG(T, FV, KXV)                                                          \
  if (a.F == FV && a.KX == KXV) {                                                         \
    hipLaunchKernelGGL((head_fwd_reg_kernel<T, FV, KXV>), grb, dim3(kHeadThreads),        \
                       fwd_reg_lds(a.HF, KXV), s, a, (const T*)u, (T*)out);               \
    return check_launch("head_fwd");                                                      \
  }
  if (a.HF % 4 == 0 && a.HF <= 256 && a.M <= 64) {
    if (bf) {
      HEAD_FWD_REG(bf16_t, 64, 64) HEAD_FWD_REG(bf16_t, 32, 64) HEAD_FWD_REG(bf16_t, 16, 64)
      HEAD_FWD_REG(bf16_t, 64, 32) HEAD_FWD_REG(bf16_t, 32, 32) HEAD_FWD_REG(bf16_t, 16, 32)
    } else {
      HEAD_FWD_REG(float, 64, 64) HEAD_FWD_REG(float, 32, 64) HEAD_FWD_REG(float, 16, 64)
      HEAD_FWD_REG(float, 64, 32) HEAD_FWD_REG(float, 32, 32) HEAD_FWD_REG(float, 16, 32)
    }
  }
#undef HEAD_FWD_REG
  const size_t lds = fwd_lds(a.HF, a.KX, a.M);
#define HEAD_FWD(T, QM)                                                                   \
  hipLaunchKernelGGL((head_fwd_kernel<T, QM>), gr, dim3(kHeadThreads), lds, s, a,         \
                     (const T*)u, (T*)out)
  const int qm = (a.M + 63) / 64;
  if (bf) {
    if (qm == 1) HEAD_FWD(bf16_t, 1); else if (qm == 2) HEAD_FWD(bf16_t, 2); else HEAD_FWD(bf16_t, 4);
  } else {
    if (qm == 1) HEAD_FWD(float, 1); else if (qm == 2) HEAD_FWD(float, 2); else HEAD_FWD(float, 4);
  }
#undef HEAD_FWD
  return check_launch("head_fwd");
}

// rflag / wmask (nullable, together): the row flags of dout already computed by its producer
// (msha_nll_rows_bwd_flags) -- the split row pass then launches no scan of its own
static int head_bwd_impl(const msha_graph* g, const msha_head_params* hp, int32_t dtype,
                         const void* u, const void* v, const float* W, float p_x,
                         uint64_t seed_x, float p_att, uint64_t seed_att, const float* stats,
                         const void* dout, void* du, void* dv, float* dW, float* dzero,
                         int64_t n_zero, void* ws, size_t ws_bytes, const uint8_t* rflag,
                         const uint64_t* wmask, msha_stream_t stream) {
  if (int rc = head_check(g, hp, dtype)) return rc;
  MSHA_ARG_CHECK(u && v && W && stats && dout && du && dv && dW, "head_bwd: null pointer");
  const HeadLayout L = head_layout(g->n_rows, (int)g->n_cols, hp->heads, hp->feat);
  MSHA_ARG_CHECK(ws && ws_bytes >= L.total, "head_bwd: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  HeadArgs a = head_args(g, hp, W, const_cast<float*>(stats));
  a.dx = make_dropout(p_x, seed_x, 0, s);
  a.dg = make_dropout(p_att, seed_att, 0, s);
  char* base = (char*)ws;
  HeadBwdWs w;
  w.part = (float*)(base + L.part_b);
  w.wflag = (int*)(base + L.wflag);
  w.dz = (float*)(base + L.dz);
  w.rflag = (uint8_t*)(base + L.rflag);
  w.red = (float*)(base + L.red);
  w.wmask = (uint64_t*)(base + L.wmask);
  w.coef = (float*)(base + L.coef);
  const int64_t rpw = head_bwd_rpw(a.N);
  const int nw = head_bwd_waves(a.N);
  const bool bf = dtype == MSHA_DTYPE_BF16;
  const size_t lds = bwd_lds(a.HF, a.KX, a.M);
  const int qm = (a.M + 63) / 64;
  static const int slow = [] {
    const char* v = getenv("MSHA_HEAD_BWD_SLOW");
    return v != nullptr && *v ? atoi(v) : 0;
  }();
  a.slow_bwd = slow;
  // the split form (scan + G row blocks) for the shipped shapes; MSHA_HEAD_BWD_SPLIT=0: the
  // one-launch row pass (A/B)
  static const int split_env = [] {
    const char* v = getenv("MSHA_HEAD_BWD_SPLIT");
    return v != nullptr && *v ? atoi(v) : 1;
  }();
  const bool split = split_env != 0 && head_bwd_fast(qm, a.M, a.KX, a.HF, a.F, slow) &&
                     a.N < (int64_t)INT32_MAX / 2;
  int nblk = nw;
  if (split) {
    const int64_t nwords = (a.N + 63) / 64;
    const int g2 = nw / 4 < 64 ? (nw / 4 > 0 ? nw / 4 : 1) : 64;  // 4 slots a block
    nblk = 4 * g2;
    const size_t lds2 = sizeof(float) * ((size_t)a.HF * a.M + (size_t)a.KX * a.M + 4 * (size_t)a.HF +
                                         32 * 192 + 4 * ((size_t)a.HF + 3 * (size_t)a.KX + 2 * (size_t)a.M));
    const dim3 gs((unsigned)((a.N + 255) / 256));
    const bool scan = wmask == nullptr;
    if (!scan) {
      w.rflag = const_cast<uint8_t*>(rflag);
      w.wmask = const_cast<uint64_t*>(wmask);
    }
    if (bf) {
      if (scan)
        hipLaunchKernelGGL(head_bwd_scan_kernel<bf16_t>, gs, dim3(256), 0, s, (const bf16_t*)dout,
                           a.N, a.M, w.rflag, w.wmask);
      hipLaunchKernelGGL(head_bwd_rows2_kernel<bf16_t>, dim3(g2), dim3(256), lds2, s, a,
                         (const bf16_t*)u, (const bf16_t*)dout, w, (int)nwords);
    } else {
      if (scan)
        hipLaunchKernelGGL(head_bwd_scan_kernel<float>, gs, dim3(256), 0, s, (const float*)dout,
                           a.N, a.M, w.rflag, w.wmask);
      hipLaunchKernelGGL(head_bwd_rows2_kernel<float>, dim3(g2), dim3(256), lds2, s, a,
                         (const float*)u, (const float*)dout, w, (int)nwords);
    }
  } else {
#define HEAD_BWD(T, QM)                                                                     \
  hipLaunchKernelGGL((head_bwd_rows_kernel<T, QM>), dim3(nw), dim3(64), lds, s, a,          \
                     (const T*)u, (const T*)dout, w, rpw)
    if (bf) {
      if (qm == 1) HEAD_BWD(bf16_t, 1); else if (qm == 2) HEAD_BWD(bf16_t, 2); else HEAD_BWD(bf16_t, 4);
    } else {
      if (qm == 1) HEAD_BWD(float, 1); else if (qm == 2) HEAD_BWD(float, 2); else HEAD_BWD(float, 4);
    }
#undef HEAD_BWD
  }
  const int64_t PT = head_pt(a.HF, a.KX, a.M);
  hipLaunchKernelGGL(head_bwd_reduce_kernel, dim3((unsigned)((PT + 63) / 64)), dim3(256), 0, s, a,
                     w, nblk, dW, dzero, dzero != nullptr ? n_zero : 0, split ? 1 : 0);
  const dim3 ga((a.HF + 31) / 32 + grid_for(a.N * a.HF / 4, 256 * 8, 1024));
  if (bf)
    hipLaunchKernelGGL(head_bwd_apply_kernel<bf16_t>, ga, dim3(256), 0, s, a, (const bf16_t*)u,
                       (const bf16_t*)v, w, (bf16_t*)du, (bf16_t*)dv);
  else
    hipLaunchKernelGGL(head_bwd_apply_kernel<float>, ga, dim3(256), 0, s, a, (const float*)u,
                       (const float*)v, w, (float*)du, (float*)dv);
  return check_launch("head_bwd");
}

extern "C" int msha_head_bwd(const msha_graph* g, const msha_head_params* hp, int32_t dtype,
                             const void* u, const void* v, const float* W, float p_x,
                             uint64_t seed_x, float p_att, uint64_t seed_att, const float* stats,
                             const void* dout, void* du, void* dv, float* dW, float* dzero,
                             int64_t n_zero, void* ws, size_t ws_bytes, msha_stream_t stream) {
  return head_bwd_impl(g, hp, dtype, u, v, W, p_x, seed_x, p_att, seed_att, stats, dout, du, dv,
                       dW, dzero, n_zero, ws, ws_bytes, nullptr, nullptr, stream);
}

extern "C" int msha_head_bwd_flagged(const msha_graph* g, const msha_head_params* hp,
                                     int32_t dtype, const void* u, const void* v, const float* W,
                                     float p_x, uint64_t seed_x, float p_att, uint64_t seed_att,
                                     const float* stats, const void* dout, const uint8_t* rflag,
                                     const uint64_t* wmask, void* du, void* dv, float* dW,
                                     float* dzero, int64_t n_zero, void* ws, size_t ws_bytes,
                                     msha_stream_t stream) {
  MSHA_ARG_CHECK(rflag != nullptr && wmask != nullptr, "head_bwd_flagged: null row flags");
  return head_bwd_impl(g, hp, dtype, u, v, W, p_x, seed_x, p_att, seed_att, stats, dout, du, dv,
                       dW, dzero, n_zero, ws, ws_bytes, rflag, wmask, stream);
}

// Diagnostic: install (buf != NULL: >= 256 slots x 64 uint64 words, device memory) or
// remove the head_bwd_rows2 timeline buffer; MSHA_ERR_UNSUPPORTED unless built with
// -DSK_TIMELINE (build.py --variant timeline).
extern "C" int msha_debug_head_timeline(void* buf) {
#ifdef SK_TIMELINE
  uint64_t* p = (uint64_t*)buf;
  if (hipMemcpyToSymbol(HIP_SYMBOL(msha::g_head_tl), &p, sizeof(p)) != hipSuccess)
    return msha::fail(MSHA_ERR_HIP, "debug_head_timeline: hipMemcpyToSymbol failed");
  return MSHA_OK;
#else
  (void)buf;
  return msha::fail(MSHA_ERR_UNSUPPORTED, "debug_head_timeline: library built without SK_TIMELINE");
#endif
}
