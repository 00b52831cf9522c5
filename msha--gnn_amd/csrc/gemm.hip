// Feature x W projections on the matrix cores (gfx950 v_mfma_f32_16x16x4_f32).
//
// Reference: every layer projects its features densely before attending --
// Ablation.py:262-263 (h1 = R @ W1, h2 = S @ W2), GAT.py:21 (h = input @ W),
// LLP.py:105-110 (Linear of x_i * x_j).  This is the only MFMA user of the library.
//
// C[m, n] = sum_k A[m, k] * B[k, n], fp32 in / fp32 accumulate: the f32 MFMA is a
// k-ordered fp32 FMA chain (exact f32, no TF32 on gfx950), at the fp32 vector rate.
//
// Tile: 128 x 128 x 32, 256 threads = 4 waves; wave w owns rows [32w, 32w+32) x 128
// columns as 2 x 8 accumulators of 16 x 16.  A is staged m-major ([m][k], rows of
// 34 floats: the 16 rows x 2 k a ds_read_b32 half touches map to banks 2m + k, all
// distinct) and B k-major ([k][n], rows of 144 floats: the two k-rows of a half fall
// in disjoint bank halves), so operand reads and staging writes are conflict free.
//
// A-operand loaders:   strided (any (sAm, sAk): row-major, transposed views)
//                      gather-hadamard A[m, k] = G[gi[m], k] * G[gj[m], k]  (pair scorer)
// Epilogues:           store / split-K slab, bias+relu+dropout+sigmoid (Linear of the
//                      link predictor), and attention-score heads
//                      el[m, h] = sum_f C[m, h*F+f] * al[h, f]  (+ er with ar)
#include <cstring>

#include "common.h"

#ifndef SLAB_U
#define SLAB_U 8
#endif

namespace msha {

constexpr int BM = 128, BN = 128, BK = 32, LDA = BK + 2, LDP = 144;

typedef float f32x4 __attribute__((ext_vector_type(4)));

enum : int { A_STRIDED = 0, A_GATHER_HADAMARD = 1 };
enum : int { EPI_STORE = 0, EPI_ACT = 1, EPI_SCORE = 2 };
enum : int { ACT_BIAS = 1, ACT_RELU = 2, ACT_DROPOUT = 4, ACT_SIGMOID = 8 };

struct GemmArgs {
  int64_t M, N, K;
  const float* A;
  int64_t sAm, sAk;
  const int64_t* gi;  // gather-hadamard rows (A_GATHER_HADAMARD)
  const int64_t* gj;  // nullable: plain gather of gi
  const float* G;
  const float* G2;  // table of the second gather (nullable: G)
  int64_t ldg, ldg2;
  const float* B;
  int64_t sBk, sBn;
  float* C;
  int64_t ldc;
  int64_t k_chunk;  // split-K: K range of blockIdx.z
  float* slab;      // split-K partial output (M x N per split), nullable
  // EPI_ACT
  int act;
  const float* bias;
  Dropout dp;
  // EPI_SCORE
  const float* al;
  const float* ar;
  float* el;
  float* er;
  int H;
  // head-outer operand update (HO_A / HO_B): X[r, c] += de[r, c / hF] * ha[c]
  // (+ de2 * ha2), X the A (r = m, c = k) or B (r = k, c = n) operand
  const float* de;
  const float* ha;
  const float* de2;
  const float* ha2;
  int hH, hF;
};

enum : int { HO_NONE = 0, HO_A = 1, HO_B = 2 };

template <int AMODE>
__device__ __forceinline__ float load_a(const GemmArgs& p, int64_t m, int64_t k) {
  if (m >= p.M || k >= p.K) return 0.f;
  if (AMODE == A_STRIDED) return p.A[m * p.sAm + k * p.sAk];
  const int64_t i = p.gi ? p.gi[m] : m;
  const float x = p.G[i * p.ldg + k];
  if (p.G2 == nullptr && p.gj == nullptr) return x;  // single input (deeper layers)
  const int64_t j = p.gj ? p.gj[m] : m;
  return x * (p.G2 ? p.G2 : p.G)[j * p.ldg2 + k];
}

// Vectorised staging (16-byte loads, prefetched into registers one K-stage ahead)
// for the layouts the library uses: A with k contiguous (row-major X, gathered
// rows) or m contiguous (X^T of a weight gradient); B with n contiguous (W) or
// k contiguous (W^T, nn.Linear weights).  Anything else takes the scalar path.
enum : int { LD_SCALAR = 0, LD_VEC = 1 };

struct Stage {
  float4 a[4];
  float4 b[4];
  uint32_t okmask;  // bit it: a[it] in range, bit 4+it: b[it] in range
  float d1[4], d2[4];  // head-outer update (HO_A / HO_B)
  float4 ha1, ha2;
};

// Branch-free 16-byte loads: an out-of-range element reads a clamped in-range
// address and is zeroed by a select, so the compiler can issue a stage's loads
// back to back and wait for them once (at the LDS store of the next stage).
__device__ __forceinline__ float f4_get(float4 v, int i) {
  return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w;
}

__device__ __forceinline__ float4 sel4(bool ok, float4 v) {
  return ok ? v : make_float4(0.f, 0.f, 0.f, 0.f);
}

// The zeroing select of out-of-range elements is applied in stage_store (after the
// barrier): placed next to the loads, it forces the wait for them before the MFMAs.
template <int AMODE>
__device__ __forceinline__ float4 load_a4_kfast(const GemmArgs& p, int64_t m, int64_t k,
                                                bool& ok) {
  // 4 consecutive k of row m (K % 4 == 0)
  ok = m < p.M && k < p.K;
  const int64_t mc = ok ? m : 0, kc = ok ? k : 0;
  if (AMODE == A_STRIDED) return *reinterpret_cast<const float4*>(p.A + mc * p.sAm + kc);
  const int64_t i = p.gi ? p.gi[mc] : mc;
  const float4 x = *reinterpret_cast<const float4*>(p.G + i * p.ldg + kc);
  if (p.G2 == nullptr && p.gj == nullptr) return x;
  const int64_t j = p.gj ? p.gj[mc] : mc;
  const float4 y = *reinterpret_cast<const float4*>((p.G2 ? p.G2 : p.G) + j * p.ldg2 + kc);
  return make_float4(x.x * y.x, x.y * y.y, x.z * y.z, x.w * y.w);
}

// Head-outer operand update: the loads of de / ha go out with the operand loads
// and the fma is applied in stage_store (after the barrier), so the prefetch stays
// asynchronous.  ha of a thread's 4 columns is the same for all 4 slots `it`.
__device__ __forceinline__ void head_outer_load(const GemmArgs& p, int64_t r, int64_t c,
                                                Stage& st, int it) {
  const int64_t h = c / p.hF;
  st.d1[it] = p.de[r * p.hH + h];
  st.d2[it] = p.de2 != nullptr ? p.de2[r * p.hH + h] : 0.f;
  if (it == 0) {
    st.ha1 = *reinterpret_cast<const float4*>(p.ha + c);
    st.ha2 = p.ha2 != nullptr ? *reinterpret_cast<const float4*>(p.ha2 + c)
                              : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

// AK: A's k is contiguous (else m is); BNF: B's n is contiguous (else k is)
template <int AMODE, int AK, int BNF, int HO = HO_NONE>
__device__ __forceinline__ void stage_load(const GemmArgs& p, Stage& st, int64_t m0, int64_t n0,
                                           int64_t k0, int64_t ke, int tid) {
  uint32_t okm = 0u;
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int idx = tid + 256 * it;
    bool oka, okb;
    if (AK) {  // 128 rows x 8 float4 along k
      const int mm = idx >> 3, kq = idx & 7;
      const int64_t k = k0 + 4 * kq;
      st.a[it] = load_a4_kfast<AMODE>(p, m0 + mm, k < ke ? k : p.K, oka);
      if (HO == HO_A) head_outer_load(p, oka ? m0 + mm : 0, oka ? k : 0, st, it);
    } else {  // 32 k x 32 float4 along m (A[m, k] = A[k * sAk + m])
      const int kk = idx >> 5, mq = idx & 31;
      const int64_t k = k0 + kk, m = m0 + 4 * mq;
      oka = k < ke && m < p.M;
      st.a[it] = *reinterpret_cast<const float4*>(p.A + (oka ? k * p.sAk + m : 0));
    }
    if (BNF) {  // 32 k x 32 float4 along n
      const int kk = idx >> 5, nq = idx & 31;
      const int64_t k = k0 + kk, n = n0 + 4 * nq;
      okb = k < ke && n < p.N;
      st.b[it] = *reinterpret_cast<const float4*>(p.B + (okb ? k * p.sBk + n : 0));
      if (HO == HO_B) head_outer_load(p, okb ? k : 0, okb ? n : 0, st, it);
    } else {  // 128 n x 8 float4 along k (B[k, n] = B[n * sBn + k])
      const int nn = idx >> 3, kq = idx & 7;
      const int64_t k = k0 + 4 * kq, n = n0 + nn;
      okb = k < ke && n < p.N;
      st.b[it] = *reinterpret_cast<const float4*>(p.B + (okb ? n * p.sBn + k : 0));
    }
    okm |= (oka ? 1u : 0u) << it;
    okm |= (okb ? 1u : 0u) << (4 + it);
  }
  st.okmask = okm;
}

template <int AK, int BNF, int HO = HO_NONE>
__device__ __forceinline__ void stage_store(const Stage& st0, float* As, float* Bs, int tid) {
  Stage st;
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    float4 a = st0.a[it], b = st0.b[it];
    if (HO == HO_A) a = f4_fma(st0.d2[it], st0.ha2, f4_fma(st0.d1[it], st0.ha1, a));
    if (HO == HO_B) b = f4_fma(st0.d2[it], st0.ha2, f4_fma(st0.d1[it], st0.ha1, b));
    st.a[it] = sel4((st0.okmask >> it) & 1u, a);
    st.b[it] = sel4((st0.okmask >> (4 + it)) & 1u, b);
  }
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int idx = tid + 256 * it;
    if (AK) {
      const int mm = idx >> 3, kq = idx & 7;
      float* d = As + mm * LDA + 4 * kq;  // 8-byte aligned (LDA even)
      *reinterpret_cast<float2*>(d) = make_float2(st.a[it].x, st.a[it].y);
      *reinterpret_cast<float2*>(d + 2) = make_float2(st.a[it].z, st.a[it].w);
    } else {
      const int kk = idx >> 5, mq = idx & 31;
      As[(4 * mq + 0) * LDA + kk] = st.a[it].x;
      As[(4 * mq + 1) * LDA + kk] = st.a[it].y;
      As[(4 * mq + 2) * LDA + kk] = st.a[it].z;
      As[(4 * mq + 3) * LDA + kk] = st.a[it].w;
    }
    if (BNF) {
      const int kk = idx >> 5, nq = idx & 31;
      *reinterpret_cast<float4*>(Bs + kk * LDP + 4 * nq) = st.b[it];
    } else {
      const int nn = idx >> 3, kq = idx & 7;
      Bs[(4 * kq + 0) * LDP + nn] = st.b[it].x;
      Bs[(4 * kq + 1) * LDP + nn] = st.b[it].y;
      Bs[(4 * kq + 2) * LDP + nn] = st.b[it].z;
      Bs[(4 * kq + 3) * LDP + nn] = st.b[it].w;
    }
  }
}

template <int AMODE>
__device__ __forceinline__ void stage_scalar(const GemmArgs& p, float* As, float* Bs, int64_t m0,
                                             int64_t n0, int64_t k0, int64_t ke, bool a_kfast,
                                             bool b_nfast, int tid) {
#pragma unroll 4
  for (int it = 0; it < (BM * BK) / 256; ++it) {
    const int idx = tid + 256 * it;
    int mm, kk;
    if (a_kfast) { kk = idx % BK; mm = idx / BK; } else { mm = idx % BM; kk = idx / BM; }
    const int64_t k = k0 + kk;
    As[mm * LDA + kk] = k < ke ? load_a<AMODE>(p, m0 + mm, k) : 0.f;
  }
#pragma unroll 4
  for (int it = 0; it < (BK * BN) / 256; ++it) {
    const int idx = tid + 256 * it;
    int nn, kk;
    if (b_nfast) { nn = idx % BN; kk = idx / BN; } else { kk = idx % BK; nn = idx / BK; }
    const int64_t k = k0 + kk, n = n0 + nn;
    Bs[kk * LDP + nn] = (k < ke && n < p.N) ? p.B[k * p.sBk + n * p.sBn] : 0.f;
  }
}

constexpr int TP = BN + 4;  // epilogue staging row pitch (floats)

// VEC = LD_VEC: 16-byte staging with compile-time layouts (AK, BNF); LD_SCALAR:
// element-wise staging for any strides (layouts decided at run time).
template <int AMODE, int EPI, int FEPI, int VEC, int AK, int BNF, int HO = HO_NONE>
__global__ void __launch_bounds__(256) gemm_f32_kernel(GemmArgs p) {
  // one LDS object (operand tiles; reused as the epilogue's C staging)
  __shared__ __attribute__((aligned(16))) float smem[BM * LDA + BK * LDP];
  float* As = smem;
  float* Bs = smem + BM * LDA;
  const int tid = threadIdx.x;
  const int lane = tid & 63, w = tid >> 6;
  const int64_t m0 = (int64_t)blockIdx.x * BM;
  const int64_t n0 = (int64_t)blockIdx.y * BN;
  int64_t kb = 0, ke = p.K;
  if (p.k_chunk > 0) {
    kb = (int64_t)blockIdx.z * p.k_chunk;
    ke = min(p.K, kb + p.k_chunk);
  }
  f32x4 acc[2][8];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[r][c] = f32x4{0.f, 0.f, 0.f, 0.f};

  const bool a_kfast = AMODE != A_STRIDED || p.sAk == 1 || p.sAm != 1;
  const bool b_nfast = p.sBn == 1 || p.sBk != 1;
  Stage st;
  if (VEC == LD_VEC && kb < ke) stage_load<AMODE, AK, BNF, HO>(p, st, m0, n0, kb, ke, tid);
  for (int64_t k0 = kb; k0 < ke; k0 += BK) {
    __syncthreads();
    if (VEC == LD_VEC) {
      stage_store<AK, BNF, HO>(st, As, Bs, tid);
    } else {
      stage_scalar<AMODE>(p, As, Bs, m0, n0, k0, ke, a_kfast, b_nfast, tid);
    }
    __syncthreads();
    // prefetch the next stage into registers while the MFMAs run
    if (VEC == LD_VEC && k0 + BK < ke) stage_load<AMODE, AK, BNF, HO>(p, st, m0, n0, k0 + BK, ke, tid);
    // ---- 8 k-steps of 4: 2 A reads + 8 B reads feed 16 MFMAs
#pragma unroll
    for (int ks = 0; ks < BK / 4; ++ks) {
      const int kr = ks * 4 + (lane >> 4);
      const float a0 = As[(w * 32 + (lane & 15)) * LDA + kr];
      const float a1 = As[(w * 32 + 16 + (lane & 15)) * LDA + kr];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const float b = Bs[kr * LDP + c * 16 + (lane & 15)];
        acc[0][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b, acc[0][c], 0, 0, 0);
        acc[1][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b, acc[1][c], 0, 0, 0);
      }
    }
  }

  // ---- epilogue.  MFMA C/D layout: col = lane & 15, row = (lane >> 4) * 4 + reg.
  // Each wave stages its 16-row halves through LDS, then writes them back in 8 passes
  // of 2 rows: lane l covers columns 4(l & 31) .. +3 of row 2*pass + (l >> 5), so a
  // wave-store is two 512-B row segments (coalesced).  Activation and per-head score
  // dots (an xor tree over the head's F/4 lanes) happen on the way.
  static_assert(4 * 16 * TP <= BM * LDA + BK * LDP, "epilogue staging exceeds LDS");
  __syncthreads();  // all waves are done reading the operand tiles
  float* T = smem + w * (16 * TP);
  float* out = p.C;
  int64_t ldo = p.ldc;
  if (p.slab != nullptr) {
    out = p.slab + (int64_t)blockIdx.z * p.M * p.N;
    ldo = p.N;
  }
  const int c4 = (lane & 31) * 4;  // column (within the tile) of this lane's float4
  const int64_t col = n0 + c4;
  const bool col_ok = col < p.N;
  float4 bia = make_float4(0.f, 0.f, 0.f, 0.f), alv = bia, arv = bia;
  if (EPI == EPI_ACT && (p.act & ACT_BIAS) && col_ok) {
    const float b4[4] = {p.bias[col], col + 1 < p.N ? p.bias[col + 1] : 0.f,
                         col + 2 < p.N ? p.bias[col + 2] : 0.f, col + 3 < p.N ? p.bias[col + 3] : 0.f};
    bia = make_float4(b4[0], b4[1], b4[2], b4[3]);
  }
  if (EPI == EPI_SCORE && p.al && col_ok) alv = *reinterpret_cast<const float4*>(p.al + col);
  if (EPI == EPI_SCORE && p.ar && col_ok) arv = *reinterpret_cast<const float4*>(p.ar + col);
  const bool vec = ((ldo & 3) == 0) && ((((uintptr_t)out) & 15) == 0);
#pragma unroll
  for (int r = 0; r < 2; ++r) {
#pragma unroll
    for (int c = 0; c < 8; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i) T[((lane >> 4) * 4 + i) * TP + c * 16 + (lane & 15)] = acc[r][c][i];
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's staging writes landed
    __builtin_amdgcn_wave_barrier();
#pragma unroll 2
    for (int pass = 0; pass < 8; ++pass) {
      const int rr = 2 * pass + (lane >> 5);
      const int64_t row = m0 + w * 32 + r * 16 + rr;
      float4 v = *reinterpret_cast<const float4*>(T + rr * TP + c4);
      if (EPI == EPI_ACT) {
        uint32_t kb = 0xfu;
        if (p.act & ACT_DROPOUT) {
          kb = 0u;
          const uint64_t off = dropout_offset(p.dp, p.dp.offset);
#pragma unroll 1
          for (int u = 0; u < 4; ++u)
            if (philox_x(p.dp.seed, off, (uint64_t)(row * p.N + col + u)) >= p.dp.threshold)
              kb |= 1u << u;
        }
        float e[4] = {v.x, v.y, v.z, v.w};
        const float bb[4] = {bia.x, bia.y, bia.z, bia.w};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          float x = e[u] + bb[u];
          if (p.act & ACT_RELU) x = fmaxf(x, 0.f);
          if (p.act & ACT_DROPOUT) x *= ((kb >> u) & 1u) ? p.dp.scale : 0.f;
          if (p.act & ACT_SIGMOID) x = 1.f / (1.f + __expf(-x));
          e[u] = x;
        }
        v = make_float4(e[0], e[1], e[2], e[3]);
      }
      if (row < p.M && col_ok) {
        if (vec && col + 3 < p.N) {
          *reinterpret_cast<float4*>(out + row * ldo + col) = v;
        } else {
          const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (col + u < p.N) out[row * ldo + col + u] = e[u];
        }
      }
      if (EPI == EPI_SCORE) {
        // a head covers FE / 4 consecutive lanes of the row's 32 (FE <= 128)
        constexpr int FE = FEPI > 0 ? FEPI : 16;
        float sl = f4_dot(v, alv), sr = f4_dot(v, arv);
#pragma unroll
        for (int o = 1; o < FE / 4; o <<= 1) {
          sl += __shfl_xor(sl, o);
          sr += __shfl_xor(sr, o);
        }
        const int64_t hg = col / FE;
        if ((c4 % FE) == 0 && row < p.M && hg < p.H && col_ok) {
          if (p.el) p.el[row * p.H + hg] = sl;
          if (p.er) p.er[row * p.H + hg] = sr;
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // reads done before the next half overwrites T
    __builtin_amdgcn_wave_barrier();
  }
}

// split-K: C = sum_z slab[z].  A block owns 64 consecutive outputs; its 4 waves add
// the interleaved z-subsets {zg, zg+4, ...} and the 4 partials are added in zg order
// (a fixed order: deterministic).
__global__ void __launch_bounds__(256) slab_reduce_kernel(const float* __restrict__ slab,
                                                          int splits, int64_t M, int64_t N,
                                                          float* __restrict__ C, int64_t ldc,
                                                          float beta) {
  __shared__ float red[256];
  const int64_t total = M * N;
  const int lane = threadIdx.x & 63, zg = threadIdx.x >> 6;
  for (int64_t g = blockIdx.x; g * 64 < total; g += gridDim.x) {
    const int64_t t = g * 64 + lane;
    float s0 = 0.f, s1 = 0.f;
    if (t < total) {
      int z = zg;
      // SLAB_U slab pairs loaded before they are added (same order as one pair per
      // trip): the loads overlap instead of one L2 round trip per slab
      for (; z + 4 + 8 * (SLAB_U - 1) < splits; z += 8 * SLAB_U) {
        float a[SLAB_U], b[SLAB_U];
#pragma unroll
        for (int u = 0; u < SLAB_U; ++u) {
          a[u] = slab[(int64_t)(z + 8 * u) * total + t];
          b[u] = slab[(int64_t)(z + 8 * u + 4) * total + t];
        }
#pragma unroll
        for (int u = 0; u < SLAB_U; ++u) {
          s0 += a[u];
          s1 += b[u];
        }
      }
      for (; z + 4 < splits; z += 8) {
        s0 += slab[(int64_t)z * total + t];
        s1 += slab[(int64_t)(z + 4) * total + t];
      }
      if (z < splits) s0 += slab[(int64_t)z * total + t];
    }
    red[threadIdx.x] = s0 + s1;
    __syncthreads();
    if (zg == 0 && t < total) {
      const float s = (red[lane] + red[64 + lane]) + (red[128 + lane] + red[192 + lane]);
      const int64_t r = t / N, c = t % N;
      C[r * ldc + c] = beta != 0.f ? beta * C[r * ldc + c] + s : s;
    }
    __syncthreads();
  }
}

// out = dh + de (x) a : dh (rows, H*F), de (rows, H), a (H, F)
__global__ void __launch_bounds__(256) add_head_outer_kernel(const float* __restrict__ dh,
                                                             const float* __restrict__ de,
                                                             const float* __restrict__ a,
                                                             const float* __restrict__ de2,
                                                             const float* __restrict__ a2,
                                                             int64_t rows, int H, int F,
                                                             float* __restrict__ out) {
  const int64_t D = (int64_t)H * F;
  const int64_t total = rows * D;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = t / D;
    const int c = (int)(t % D);
    const int h = c / F;
    float v = dh[t] + de[r * H + h] * a[c];
    if (de2) v += de2[r * H + h] * a2[c];
    out[t] = v;
  }
}

static bool aligned16(const void* q) { return ((uintptr_t)q & 15) == 0; }

// 16-byte staging applies when the contiguous dimension of each operand has unit
// stride, its other stride and extent are multiples of 4, and bases are aligned.
template <int AMODE>
static bool vec_ok(const GemmArgs& p) {
  // K % 4 matters only to an operand loaded 4-along-k (k-contiguous); the
  // row-contiguous layouts (X^T, W, dH as B) load one k per float4
  const bool k4 = p.K % 4 == 0;
  bool a_ok;
  if (AMODE == A_GATHER_HADAMARD) {
    a_ok = k4 && aligned16(p.G) && p.ldg % 4 == 0 &&
           (p.G2 == nullptr || (aligned16(p.G2) && p.ldg2 % 4 == 0));
  } else if (p.sAk == 1) {
    a_ok = k4 && aligned16(p.A) && p.sAm % 4 == 0;
  } else if (p.sAm == 1) {
    a_ok = aligned16(p.A) && p.sAk % 4 == 0 && p.M % 4 == 0;
  } else {
    a_ok = false;
  }
  bool b_ok;
  if (p.sBn == 1) b_ok = aligned16(p.B) && p.sBk % 4 == 0 && p.N % 4 == 0;
  else if (p.sBk == 1) b_ok = k4 && aligned16(p.B) && p.sBn % 4 == 0;
  else b_ok = false;
  return a_ok && b_ok;
}

// Gradient of the score vectors of msha_project_scores:
//   out1[h, f] = sum_r s1[r, h] * T[r, h*F + f]   (and out2 with s2)
// A block covers kColsumRows rows: its threads are (row group, float4 column quad),
// each row group strides the block's rows with 16-byte loads; the row groups are
// added in a fixed LDS tree, and a second pass adds the block partials in block
// order (deterministic).
#ifndef CS_U
#define CS_U 8
#endif
#ifndef COLSUM_ROWS
#define COLSUM_ROWS 128
#endif
constexpr int kColsumRows = COLSUM_ROWS;

// N consecutive elements of one row, widened to fp32
template <int N>
struct Fv {
  float v[N];
};
__device__ __forceinline__ Fv<4> fv_load(const float* p, Fv<4>*) {
  const float4 x = *reinterpret_cast<const float4*>(p);
  return Fv<4>{{x.x, x.y, x.z, x.w}};
}
__device__ __forceinline__ Fv<1> fv_load(const float* p, Fv<1>*) { return Fv<1>{{*p}}; }
__device__ __forceinline__ Fv<8> fv_load(const bf16_t* p, Fv<8>*) {
  const Pk<bf16_t> x = pk_load(p);
  Fv<8> r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = x.v[i];
  return r;
}

// grid (row blocks, column tiles of <= 256 vectors); D % N == 0
template <typename T, int N>
__global__ void __launch_bounds__(256) head_colsum_partial_kernel(
    int64_t rows, int H, int F, const float* __restrict__ s1, const float* __restrict__ s2,
    const T* __restrict__ tab, float* __restrict__ part) {
  using VT = Fv<N>;
  __shared__ VT red[2 * 256];
  const int D = H * F, QD = D / N;
  const int QT = QD < 256 ? QD : 256;  // vectors per column tile
  const int RG = 256 / QT;             // row groups
  const int qi = threadIdx.x % QT, rg = threadIdx.x / QT;
  const int q = blockIdx.y * QT + qi;
  const bool live = rg < RG && q < QD;
  const int h = live ? (N * q) / F : 0;
  const int64_t r0 = (int64_t)blockIdx.x * kColsumRows;
  const int64_t r1 = min(rows, r0 + kColsumRows);
  VT a1, a2;
#pragma unroll
  for (int i = 0; i < N; ++i) a1.v[i] = a2.v[i] = 0.f;
  if (live) {
    // CS_U rows loaded before they are accumulated (same order): overlapping loads
    int64_t r = r0 + rg;
    for (; r + (CS_U - 1) * RG < r1; r += CS_U * RG) {
      VT x[CS_U];
      float c1[CS_U], c2[CS_U];
#pragma unroll
      for (int u = 0; u < CS_U; ++u) {
        const int64_t ru = r + u * RG;
        x[u] = fv_load(tab + ru * D + N * q, (VT*)nullptr);
        c1[u] = s1[ru * H + h];
        c2[u] = s2 ? s2[ru * H + h] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < CS_U; ++u)
#pragma unroll
        for (int i = 0; i < N; ++i) {
          a1.v[i] = fmaf(c1[u], x[u].v[i], a1.v[i]);
          a2.v[i] = fmaf(c2[u], x[u].v[i], a2.v[i]);
        }
    }
    for (; r < r1; r += RG) {
      const VT x = fv_load(tab + r * D + N * q, (VT*)nullptr);
      const float c1 = s1[r * H + h];
      const float c2 = s2 ? s2[r * H + h] : 0.f;
#pragma unroll
      for (int i = 0; i < N; ++i) {
        a1.v[i] = fmaf(c1, x.v[i], a1.v[i]);
        a2.v[i] = fmaf(c2, x.v[i], a2.v[i]);
      }
    }
  }
  red[threadIdx.x] = a1;
  red[256 + threadIdx.x] = a2;
  __syncthreads();
  int w = 1;
  while (w < RG) w <<= 1;
  for (w >>= 1; w >= 1; w >>= 1) {  // fixed-order tree over the row groups
    if (rg < w && rg + w < RG) {
      const int i = rg * QT + qi, j = (rg + w) * QT + qi;
#pragma unroll
      for (int e = 0; e < N; ++e) {
        red[i].v[e] += red[j].v[e];
        red[256 + i].v[e] += red[256 + j].v[e];
      }
    }
    __syncthreads();
  }
  // partials transposed, [which][d][block]: the reduce reads each output's blocks
  // contiguously
  if (rg == 0 && q < QD) {
    const int64_t nb = gridDim.x;
#pragma unroll
    for (int e = 0; e < N; ++e) {
      part[((int64_t)0 * D + N * q + e) * nb + blockIdx.x] = red[qi].v[e];
      part[((int64_t)1 * D + N * q + e) * nb + blockIdx.x] = red[256 + qi].v[e];
    }
  }
}

// one wave per output element: lane l adds blocks l, l+64, ... in order, then a
// fixed xor tree across the lanes (deterministic)
__global__ void __launch_bounds__(256) head_colsum_reduce_kernel(int nblk, int D,
                                                                 const float* __restrict__ part,
                                                                 float* __restrict__ out1,
                                                                 float* __restrict__ out2) {
  const int t = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const int lane = threadIdx.x & 63;
  if (t >= 2 * D) return;
  const int which = t / D, d = t % D;
  float* out = which == 0 ? out1 : out2;
  if (out == nullptr) return;
  float s0 = 0.f, s1 = 0.f;
  const float* src = part + ((int64_t)which * D + d) * nblk;
  int b = lane;
  for (; b + 64 < nblk; b += 128) {
    s0 += src[b];
    s1 += src[b + 64];
  }
  if (b < nblk) s0 += src[b];
  float v = s0 + s1;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  if (lane == 0) out[d] = v;
}

template <int AMODE, int EPI, int FEPI>
static void launch(const GemmArgs& p, int splits, hipStream_t s) {
  dim3 grid((unsigned)((p.M + BM - 1) / BM), (unsigned)((p.N + BN - 1) / BN), (unsigned)splits);
  if (!vec_ok<AMODE>(p)) {
    hipLaunchKernelGGL((gemm_f32_kernel<AMODE, EPI, FEPI, LD_SCALAR, 1, 1>), grid, dim3(256), 0, s,
                       p);
    return;
  }
  const bool ak = AMODE != A_STRIDED || p.sAk == 1;
  const bool bn = p.sBn == 1;
  if (AMODE != A_STRIDED || EPI != EPI_STORE) {  // projections / pair scorer: fixed layouts
    if (bn)
      hipLaunchKernelGGL((gemm_f32_kernel<AMODE, EPI, FEPI, LD_VEC, 1, 1>), grid, dim3(256), 0, s,
                         p);
    else
      hipLaunchKernelGGL((gemm_f32_kernel<AMODE, EPI, FEPI, LD_VEC, 1, 0>), grid, dim3(256), 0, s,
                         p);
    return;
  }
  if (ak && bn)
    hipLaunchKernelGGL((gemm_f32_kernel<AMODE, EPI, FEPI, LD_VEC, 1, 1>), grid, dim3(256), 0, s, p);
  else if (ak)
    hipLaunchKernelGGL((gemm_f32_kernel<AMODE, EPI, FEPI, LD_VEC, 1, 0>), grid, dim3(256), 0, s, p);
  else if (bn)
    hipLaunchKernelGGL((gemm_f32_kernel<AMODE, EPI, FEPI, LD_VEC, 0, 1>), grid, dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL((gemm_f32_kernel<AMODE, EPI, FEPI, LD_VEC, 0, 0>), grid, dim3(256), 0, s, p);
}

static GemmArgs base_args(int64_t M, int64_t N, int64_t K) {
  GemmArgs p;
  memset(&p, 0, sizeof(p));
  p.M = M;
  p.N = N;
  p.K = K;
  p.dp = make_dropout(0.f, 0, 0, nullptr);
  return p;
}

}  // namespace msha

using namespace msha;

extern "C" size_t msha_gemm_workspace_size(int64_t M, int64_t N, int32_t splits) {
  if (splits <= 1) return 0;
  return (size_t)splits * (size_t)M * (size_t)N * sizeof(float);
}

template <int HO>
static void launch_ho(const GemmArgs& p, int splits, hipStream_t s) {
  dim3 grid((unsigned)((p.M + BM - 1) / BM), (unsigned)((p.N + BN - 1) / BN), (unsigned)splits);
  const bool ak = p.sAk == 1, bn = p.sBn == 1;
  if (HO == HO_A) {  // A has k contiguous
    if (bn)
      hipLaunchKernelGGL((gemm_f32_kernel<A_STRIDED, EPI_STORE, 0, LD_VEC, 1, 1, HO>), grid,
                         dim3(256), 0, s, p);
    else
      hipLaunchKernelGGL((gemm_f32_kernel<A_STRIDED, EPI_STORE, 0, LD_VEC, 1, 0, HO>), grid,
                         dim3(256), 0, s, p);
  } else {  // B has n contiguous
    if (ak)
      hipLaunchKernelGGL((gemm_f32_kernel<A_STRIDED, EPI_STORE, 0, LD_VEC, 1, 1, HO>), grid,
                         dim3(256), 0, s, p);
    else
      hipLaunchKernelGGL((gemm_f32_kernel<A_STRIDED, EPI_STORE, 0, LD_VEC, 0, 1, HO>), grid,
                         dim3(256), 0, s, p);
  }
}

// shared body of msha_gemm_f32 / msha_gemm_f32_head_outer
static int gemm_run(GemmArgs& p, int ho, float beta, int32_t splits, void* ws, size_t ws_bytes,
                    hipStream_t s) {
  const int64_t M = p.M, N = p.N, K = p.K;
  // dX = (dh + de (x) a) W^T with W^T given as W (N, K) row-major: resident-W kernel
  if (ho == HO_A && beta == 0.f && p.sAk == 1 && p.sAm == K && p.sBk == 1 && p.sBn == K &&
      p.ldc == N &&
      skinny_dx(M, N, K, p.A, p.B, p.C, p.hH, p.hF, p.de, p.ha, p.de2, p.ha2, s))
    return check_launch("gemm_f32");
  if (ho != HO_A && p.slab == nullptr &&
      skinny_wgrad(M, N, K, p.A, p.sAm, p.sAk, p.B, p.sBk, p.sBn, p.C, p.ldc, beta, splits, ws,
                   ws_bytes, p.hH, p.hF, ho == HO_B ? p.de : nullptr, p.ha, p.de2, p.ha2, s))
    return check_launch("gemm_f32");
  auto go = [&](int used) {
    if (ho == HO_A) launch_ho<HO_A>(p, used, s);
    else if (ho == HO_B) launch_ho<HO_B>(p, used, s);
    else launch<A_STRIDED, EPI_STORE, 0>(p, used, s);
  };
  if (splits > 1) {
    MSHA_ARG_CHECK(ws && ws_bytes >= msha_gemm_workspace_size(M, N, splits),
                   "gemm_f32: split-K workspace too small");
    int64_t kc = (K + splits - 1) / splits;
    kc = ((kc + BK - 1) / BK) * BK;
    const int used = (int)((K + kc - 1) / kc);
    p.k_chunk = kc;
    p.slab = (float*)ws;
    go(used);
    const int64_t groups = (M * N + 63) / 64;
    hipLaunchKernelGGL(slab_reduce_kernel, dim3(grid_for(groups, 1, 65535)), dim3(256), 0, s,
                       (const float*)ws, used, M, N, p.C, p.ldc, beta);
  } else {
    go(1);
  }
  return check_launch("gemm_f32");
}

extern "C" int msha_gemm_f32(int64_t M, int64_t N, int64_t K, const float* A, int64_t sAm,
                             int64_t sAk, const float* B, int64_t sBk, int64_t sBn, float* C,
                             int64_t ldc, float beta, int32_t splits, void* ws, size_t ws_bytes,
                             msha_stream_t stream) {
  MSHA_ARG_CHECK(M > 0 && N > 0 && K > 0, "gemm_f32: bad sizes");
  MSHA_ARG_CHECK(A && B && C, "gemm_f32: null pointer");
  MSHA_ARG_CHECK(splits >= 1 && splits <= 65535, "gemm_f32: splits out of range");
  MSHA_ARG_CHECK(splits == 1 || beta == 0.f || beta == 1.f, "gemm_f32: beta must be 0 or 1");
  MSHA_ARG_CHECK(splits > 1 || beta == 0.f, "gemm_f32: beta needs splits > 1");
  GemmArgs p = base_args(M, N, K);
  p.A = A; p.sAm = sAm; p.sAk = sAk;
  p.B = B; p.sBk = sBk; p.sBn = sBn;
  p.C = C; p.ldc = ldc;
  return gemm_run(p, HO_NONE, beta, splits, ws, ws_bytes, (hipStream_t)stream);
}

extern "C" int msha_gemm_f32_head_outer(int64_t M, int64_t N, int64_t K, const float* A,
                                        int64_t sAm, int64_t sAk, const float* B, int64_t sBk,
                                        int64_t sBn, float* C, int64_t ldc, float beta,
                                        int32_t splits, void* ws, size_t ws_bytes,
                                        int32_t operand, int32_t heads, int32_t feat,
                                        const float* de, const float* a, const float* de2,
                                        const float* a2, msha_stream_t stream) {
  MSHA_ARG_CHECK(M > 0 && N > 0 && K > 0, "gemm_f32_head_outer: bad sizes");
  MSHA_ARG_CHECK(A && B && C && de && a && ((de2 == nullptr) == (a2 == nullptr)),
                 "gemm_f32_head_outer: null pointer");
  MSHA_ARG_CHECK(operand == 0 || operand == 1, "gemm_f32_head_outer: operand must be 0 (A) or 1 (B)");
  MSHA_ARG_CHECK(heads > 0 && feat > 0 && feat % 4 == 0,
                 "gemm_f32_head_outer: feat must be a positive multiple of 4");
  MSHA_ARG_CHECK((operand == 0 ? K : N) == (int64_t)heads * feat,
                 "gemm_f32_head_outer: the updated operand's column count must be heads*feat");
  MSHA_ARG_CHECK(splits >= 1 && splits <= 65535, "gemm_f32_head_outer: splits out of range");
  MSHA_ARG_CHECK(splits == 1 || beta == 0.f || beta == 1.f, "gemm_f32_head_outer: beta must be 0 or 1");
  MSHA_ARG_CHECK(splits > 1 || beta == 0.f, "gemm_f32_head_outer: beta needs splits > 1");
  GemmArgs p = base_args(M, N, K);
  p.A = A; p.sAm = sAm; p.sAk = sAk;
  p.B = B; p.sBk = sBk; p.sBn = sBn;
  p.C = C; p.ldc = ldc;
  p.de = de; p.ha = a; p.de2 = de2; p.ha2 = a2; p.hH = heads; p.hF = feat;
  const bool lay = operand == 0 ? sAk == 1 : sBn == 1;
  const bool al = aligned16(a) && (a2 == nullptr || aligned16(a2));
  if (!lay || !al || !vec_ok<A_STRIDED>(p))
    return fail(MSHA_ERR_UNSUPPORTED, "gemm_f32_head_outer: the updated operand needs unit stride "
                                      "along heads*feat and 16-byte aligned, vectorizable operands");
  return gemm_run(p, operand == 0 ? HO_A : HO_B, beta, splits, ws, ws_bytes, (hipStream_t)stream);
}

extern "C" size_t msha_head_outer_colsum_workspace_size(int64_t N) {
  // (T form: 2 x N x 256 block partials; W form: 4 x 128 x 256 -- the larger of the two)
  return N > 0 ? (size_t)4 * (size_t)(N > 128 ? N : 128) * 256 * sizeof(float) : 0;
}

// The projection's weight gradient and score-vector gradients in one pass over the rows
// (Ablation.py:262-267 backward): C = A (B + de (x) a [+ de2 (x) a2]) as
// msha_gemm_f32_head_outer with operand 1, plus cs1[n] = sum_k de[k, n / feat] T[k, n]
// (cs2 with de2) -- msha_head_colsum's outputs -- accumulated by the same launch from a
// table T with B's layout.  Only the resident-accumulator weight-gradient shape (skinny.hip:
// M = N = 128, K >= 4096 rows, fp32); MSHA_ERR_UNSUPPORTED (nothing launched) otherwise,
// and the caller runs the two ops.
extern "C" int msha_gemm_f32_head_outer_colsum(
    int64_t M, int64_t N, int64_t K, const float* A, int64_t sAm, int64_t sAk, const float* B,
    int64_t sBk, int64_t sBn, float* C, int64_t ldc, int32_t splits, void* ws, size_t ws_bytes,
    int32_t heads, int32_t feat, const float* de, const float* a, const float* de2,
    const float* a2, const float* T, float* cs1, float* cs2, void* cs_ws, size_t cs_ws_bytes,
    msha_stream_t stream) {
  MSHA_ARG_CHECK(M > 0 && N > 0 && K > 0, "gemm_f32_head_outer_colsum: bad sizes");
  MSHA_ARG_CHECK(A && B && C && de && a && T && cs1 && ((de2 == nullptr) == (a2 == nullptr)) &&
                     ((de2 == nullptr) == (cs2 == nullptr)),
                 "gemm_f32_head_outer_colsum: null pointer");
  MSHA_ARG_CHECK(heads > 0 && feat > 0 && feat % 4 == 0 && N == (int64_t)heads * feat,
                 "gemm_f32_head_outer_colsum: N must be heads*feat, feat a multiple of 4");
  MSHA_ARG_CHECK(splits >= 1 && splits <= 65535, "gemm_f32_head_outer_colsum: splits out of range");
  MSHA_ARG_CHECK(cs_ws && cs_ws_bytes >= msha_head_outer_colsum_workspace_size(N),
                 "gemm_f32_head_outer_colsum: colsum workspace too small");
  if (!aligned16(a) || (a2 != nullptr && !aligned16(a2)))
    return fail(MSHA_ERR_UNSUPPORTED, "gemm_f32_head_outer_colsum: 16-byte aligned a, a2");
  hipStream_t s = (hipStream_t)stream;
  if (!skinny_wgrad(M, N, K, A, sAm, sAk, B, sBk, sBn, C, ldc, 0.f, splits, ws, ws_bytes, heads,
                    feat, de, a, de2, a2, s, T, (float*)cs_ws, cs1, cs2))
    return fail(MSHA_ERR_UNSUPPORTED, "gemm_f32_head_outer_colsum: shape outside the fused kernel");
  return check_launch("gemm_f32_head_outer_colsum");
}

// (ABI 15) The same outputs where T = X W is the projection's own output (Ablation.py:262,
// h = X @ W): cs1[n] = sum_k de[k, n / feat] (X W)[k, n] = sum_a W[a, n] G[n / feat, a] with
// G = de^T X accumulated from the X rows the weight gradient already streams, so h is never
// read (a third of the pass's bytes).  The sums are the same in real arithmetic; in fp32
// they differ from the T form by h's own rounding.  Two heads, split-bf16 weight-gradient
// kernel only; MSHA_ERR_UNSUPPORTED otherwise (the caller runs the T form).
extern "C" int msha_gemm_f32_head_outer_colsum_w(
    int64_t M, int64_t N, int64_t K, const float* A, int64_t sAm, int64_t sAk, const float* B,
    int64_t sBk, int64_t sBn, float* C, int64_t ldc, int32_t splits, void* ws, size_t ws_bytes,
    int32_t heads, int32_t feat, const float* de, const float* a, const float* de2,
    const float* a2, const float* W, int64_t ldw, float* cs1, float* cs2, void* cs_ws,
    size_t cs_ws_bytes, msha_stream_t stream) {
  MSHA_ARG_CHECK(M > 0 && N > 0 && K > 0, "gemm_f32_head_outer_colsum_w: bad sizes");
  MSHA_ARG_CHECK(A && B && C && de && a && W && cs1 && ((de2 == nullptr) == (a2 == nullptr)) &&
                     ((de2 == nullptr) == (cs2 == nullptr)),
                 "gemm_f32_head_outer_colsum_w: null pointer");
  MSHA_ARG_CHECK(heads > 0 && feat > 0 && feat % 4 == 0 && N == (int64_t)heads * feat && ldw >= N,
                 "gemm_f32_head_outer_colsum_w: N must be heads*feat, feat a multiple of 4, ldw >= N");
  MSHA_ARG_CHECK(splits >= 1 && splits <= 65535, "gemm_f32_head_outer_colsum_w: splits out of range");
  MSHA_ARG_CHECK(cs_ws && cs_ws_bytes >= msha_head_outer_colsum_workspace_size(N),
                 "gemm_f32_head_outer_colsum_w: colsum workspace too small");
  if (!aligned16(a) || (a2 != nullptr && !aligned16(a2)))
    return fail(MSHA_ERR_UNSUPPORTED, "gemm_f32_head_outer_colsum_w: 16-byte aligned a, a2");
  hipStream_t s = (hipStream_t)stream;
  if (!skinny_wgrad(M, N, K, A, sAm, sAk, B, sBk, sBn, C, ldc, 0.f, splits, ws, ws_bytes, heads,
                    feat, de, a, de2, a2, s, nullptr, (float*)cs_ws, cs1, cs2, W, ldw))
    return fail(MSHA_ERR_UNSUPPORTED, "gemm_f32_head_outer_colsum_w: shape outside the fused kernel");
  return check_launch("gemm_f32_head_outer_colsum_w");
}

// every projection path computes its score dots in the row-score order (skinny.hip
// proj_kernel, this file's EPI_SCORE f4_dot + xor tree, gemm_bf16.hip's EPI_SCORE on the
// rounded row, small.hip): 1 for any valid shape
extern "C" int msha_project_scores_row_order(int64_t M, int64_t K, int32_t heads, int32_t feat,
                                             int32_t dtype) {
  if (M <= 0 || K <= 0 || heads <= 0 || feat <= 0) return 0;
  return (dtype == MSHA_DTYPE_F32 || dtype == MSHA_DTYPE_BF16) && feat % 4 == 0 ? 1 : 0;
}

extern "C" int msha_project_scores(int64_t M, int64_t K, int32_t heads, int32_t feat,
                                   const float* X, const float* W, const float* al,
                                   const float* ar, float* h, float* el, float* er,
                                   msha_stream_t stream) {
  MSHA_ARG_CHECK(M > 0 && K > 0 && heads > 0 && feat > 0, "project_scores: bad sizes");
  MSHA_ARG_CHECK(X && W && h, "project_scores: null pointer");
  MSHA_ARG_CHECK((al == nullptr) == (el == nullptr) && (ar == nullptr) == (er == nullptr),
                 "project_scores: score vectors and outputs must be paired");
  const int64_t N = (int64_t)heads * feat;
  GemmArgs p = base_args(M, N, K);
  p.A = X; p.sAm = K; p.sAk = 1;
  p.B = W; p.sBk = N; p.sBn = 1;
  p.C = h; p.ldc = N;
  p.al = al; p.ar = ar; p.el = el; p.er = er; p.H = heads;
  hipStream_t s = (hipStream_t)stream;
  if (skinny_project<float>(M, K, heads, feat, X, W, al, ar, h, el, er, s))
    return check_launch("project_scores");
  if (al == nullptr && ar == nullptr) {
    launch<A_STRIDED, EPI_STORE, 0>(p, 1, s);
  } else if (feat == 4) {
    launch<A_STRIDED, EPI_SCORE, 4>(p, 1, s);
  } else if (feat == 8) {
    launch<A_STRIDED, EPI_SCORE, 8>(p, 1, s);
  } else if (feat == 16) {
    launch<A_STRIDED, EPI_SCORE, 16>(p, 1, s);
  } else if (feat == 32) {
    launch<A_STRIDED, EPI_SCORE, 32>(p, 1, s);
  } else if (feat == 64) {
    launch<A_STRIDED, EPI_SCORE, 64>(p, 1, s);
  } else if (feat == 128) {
    launch<A_STRIDED, EPI_SCORE, 128>(p, 1, s);
  } else {
    return fail(MSHA_ERR_UNSUPPORTED, "project_scores: feat must be 4, 8, 16, 32, 64 or 128 "
                                      "when score vectors are given");
  }
  return check_launch("project_scores");
}

extern "C" int msha_add_head_outer(int64_t rows, int32_t heads, int32_t feat, const float* dh,
                                   const float* de, const float* a, const float* de2,
                                   const float* a2, float* out, msha_stream_t stream) {
  MSHA_ARG_CHECK(rows > 0 && heads > 0 && feat > 0, "add_head_outer: bad sizes");
  MSHA_ARG_CHECK(dh && de && a && out && ((de2 == nullptr) == (a2 == nullptr)),
                 "add_head_outer: null pointer");
  const int64_t total = rows * heads * feat;
  hipLaunchKernelGGL(add_head_outer_kernel, dim3(grid_for(total, 256, 16384)), dim3(256), 0,
                     (hipStream_t)stream, dh, de, a, de2, a2, rows, heads, feat, out);
  return check_launch("add_head_outer");
}

extern "C" int msha_pair_linear(int64_t n_pairs, int64_t K, int64_t N, const float* G,
                                int64_t ldg, const int64_t* gi, const float* G2, int64_t ldg2,
                                const int64_t* gj, int64_t g_rows, int64_t g2_rows,
                                const float* W, const float* bias, int32_t act, float drop_p,
                                uint64_t seed, uint64_t offset, float* out,
                                msha_stream_t stream) {
  MSHA_ARG_CHECK(n_pairs > 0 && K > 0 && N > 0, "pair_linear: bad sizes");
  MSHA_ARG_CHECK(G && W && out, "pair_linear: null pointer");
  MSHA_ARG_CHECK(!(act & ACT_BIAS) || bias, "pair_linear: bias missing");
  GemmArgs p = base_args(n_pairs, N, K);
  p.G = G; p.ldg = ldg; p.gi = gi; p.gj = gj; p.G2 = G2; p.ldg2 = G2 ? ldg2 : ldg;
  p.B = W; p.sBk = 1; p.sBn = K;  // nn.Linear weight (N x K): B[k, n] = W[n, k]
  p.C = out; p.ldc = N;
  p.act = act; p.bias = bias;
  p.dp = make_dropout(drop_p, seed, offset, (hipStream_t)stream);
  if (!p.dp.active) p.act &= ~ACT_DROPOUT;
  if (!skinny_pair_linear(n_pairs, K, N, G, ldg, gi, G2, ldg2, gj, g_rows, g2_rows, W, bias,
                          p.act, p.dp, out, (hipStream_t)stream))
    launch<A_GATHER_HADAMARD, EPI_ACT, 0>(p, 1, (hipStream_t)stream);
  return check_launch("pair_linear");
}

extern "C" size_t msha_head_colsum_workspace_size(int64_t rows, int32_t heads, int32_t feat) {
  if (rows <= 0 || heads <= 0 || feat <= 0) return 0;
  const int64_t nblk = (rows + kColsumRows - 1) / kColsumRows;
  return (size_t)nblk * 2 * (size_t)heads * (size_t)feat * sizeof(float);
}

extern "C" int msha_head_colsum(int64_t rows, int32_t heads, int32_t feat, int32_t dtype,
                                const float* s1, const float* s2, const void* T, float* out1,
                                float* out2, void* ws, size_t ws_bytes, msha_stream_t stream) {
  MSHA_ARG_CHECK(rows > 0 && heads > 0 && feat > 0, "head_colsum: bad sizes");
  MSHA_ARG_CHECK(s1 && T && out1 && ((s2 == nullptr) == (out2 == nullptr)),
                 "head_colsum: null pointer");
  MSHA_ARG_CHECK(ws && ws_bytes >= msha_head_colsum_workspace_size(rows, heads, feat),
                 "head_colsum: workspace too small");
  MSHA_ARG_CHECK(dtype == MSHA_DTYPE_F32 || dtype == MSHA_DTYPE_BF16, "head_colsum: bad dtype");
  const int D = heads * feat;
  const int nblk = (int)((rows + kColsumRows - 1) / kColsumRows);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MSHA_DTYPE_BF16) {
    if (feat % 8 != 0 || !aligned16(T))
      return fail(MSHA_ERR_UNSUPPORTED, "head_colsum: bf16 needs feat % 8 == 0, 16-B aligned T");
    const dim3 grid(nblk, (D / 8 + 255) / 256);
    hipLaunchKernelGGL((head_colsum_partial_kernel<bf16_t, 8>), grid, dim3(256), 0, s, rows,
                       (int)heads, (int)feat, s1, s2, (const bf16_t*)T, (float*)ws);
  } else if (feat % 4 == 0 && aligned16(T)) {
    const dim3 grid(nblk, (D / 4 + 255) / 256);
    hipLaunchKernelGGL((head_colsum_partial_kernel<float, 4>), grid, dim3(256), 0, s, rows,
                       (int)heads, (int)feat, s1, s2, (const float*)T, (float*)ws);
  } else {
    const dim3 grid(nblk, (D + 255) / 256);
    hipLaunchKernelGGL((head_colsum_partial_kernel<float, 1>), grid, dim3(256), 0, s, rows,
                       (int)heads, (int)feat, s1, s2, (const float*)T, (float*)ws);
  }
  hipLaunchKernelGGL(head_colsum_reduce_kernel, dim3((2 * D + 3) / 4), dim3(256), 0, s, nblk,
                     D, (const float*)ws, out1, out2);
  return check_launch("head_colsum");
}
