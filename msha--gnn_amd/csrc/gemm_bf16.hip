// bf16 feature x W projections (config C3) on the gfx950 matrix cores:
// v_mfma_f32_16x16x32_bf16, fp32 accumulation, fp32 score epilogue.
//
// Reference: Ablation.py:262-263 (h1 = R @ W1, h2 = S @ W2), GAT.py:21 (h = x @ W) run
// on a bf16 model; the gradients of those products (dX = dH W^T, dW = X^T dH) with
// the score-vector term dH + de (x) a folded into the operand staging.
//
// Tile 128 x 128 x 64, 4 waves, wave w owns rows [32w, 32w+32) x 128 columns (2 x 8
// accumulators of 16 x 16).  The MFMA lane l (group g = l >> 4, i = l & 15) takes
// the 8 k-slots j of a 32-deep step as k = (j < 4 ? 4g + j : 16 + 4g + j - 4), so:
//   k-contiguous operands (row-major X, W^T, dH) are staged as [row][k] (144-B rows)
//     and read with two ds_read_b64 per fragment (conflict free: rows 36 banks apart);
//   row-contiguous operands (X^T, W, dH as B) are staged as [k][row] (288-B rows, as
//     loaded: 16-B chunks along the row) and read with ds_read_b64_tr_b16, whose 16-lane
//     groups fetch rows 4g + q (+16) of the image and hand lane i column i (the 8 rows
//     of a 32-lane half sit 32 B apart mod 256: conflict free).
// Epilogue: accumulators staged through LDS (fp32), then store fp32 or bf16, the
// per-head score dots el/er in fp32, or a split-K slab (fp32, summed in split order).
#include <cstring>

#include "common.h"

#ifndef SLAB_U
#define SLAB_U 8
#endif

namespace msha {
namespace bfg {

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int PKF = BK + 8;   // [row][k] image pitch (bf16 elements): 144 B
constexpr int PRF = BM + 16;  // [k][row] image pitch: 288 B
constexpr int IMG = 128 * PKF;
static_assert(IMG == BK * PRF, "both operand images take the same LDS");
constexpr int TP = BN + 4;  // epilogue staging pitch (floats)

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

enum : int { EPI_STORE = 0, EPI_ACT = 1, EPI_SCORE = 2 };
enum : int { ACT_BIAS = 1, ACT_RELU = 2, ACT_DROPOUT = 4, ACT_SIGMOID = 8 };
enum : int { HO_NONE = 0, HO_A = 1, HO_B = 2 };

struct Args {
  int64_t M, N, K;
  const bf16_t* A;
  int64_t sAm, sAk;
  const bf16_t* B;
  int64_t sBk, sBn;
  void* C;
  int64_t ldc;
  int c_bf16;
  int64_t k_chunk;
  float* slab;
  const float* al;
  const float* ar;
  float* el;
  float* er;
  int H;
  const float* de;
  const float* ha;
  const float* de2;
  const float* ha2;
  int hH, hF;
  // A as a gather(-hadamard) of table rows: A[m, k] = G[gi[m], k] * G2[gj[m], k]
  // (the fused pair gather of the link scorer, LLP.py:233; G = A, ldg = sAm)
  const int64_t* gi;
  const int64_t* gj;
  const bf16_t* G2;  // NULL: G
  int64_t ldg2;
  bool hadamard;
  // EPI_ACT (nn.Linear of the link predictor): bias, relu, dropout, sigmoid
  int act;
  const float* bias;
  Dropout dp;
};

// One operand's staged 16-byte chunks (4 per thread) + head-outer terms.
struct Stage {
  uint4 x[4];
  uint4 y[4];  // second gathered row of the hadamard A loader
  uint32_t ok;
  float d1[4], d2[4];
  float4 h1[2], h2[2];  // ha / ha2 of the thread's 8 columns (same for all 4 chunks)
};

// KF: the operand's k is contiguous in memory (else its row is).
// rows: M (A) or N (B); srow / sk: element strides; RO: HO on this operand.
template <int KF, bool RO, bool GA = false>
__device__ __forceinline__ void load_operand(const Args& p, const bf16_t* X, int64_t srow,
                                             int64_t sk, int64_t nrows, int64_t r0, int64_t k0,
                                             int64_t ke, int tid, Stage& st) {
  uint32_t ok = 0u;
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int c = tid + 256 * it;
    int64_t row, k;
    if (KF) {
      row = r0 + (c >> 3);
      k = k0 + 8 * (c & 7);
    } else {
      k = k0 + (c >> 4);
      row = r0 + 8 * (c & 15);
    }
    const bool v = row < nrows && k < ke;
    if (GA) {  // KF: rows of the table picked by gi / gj
      const int64_t rr = v ? row : 0, kk = v ? k : 0;
      const int64_t i = p.gi ? p.gi[rr] : rr;
      st.x[it] = *reinterpret_cast<const uint4*>(X + i * srow + kk);
      if (p.hadamard) {
        const int64_t j = p.gj ? p.gj[rr] : rr;
        st.y[it] = *reinterpret_cast<const uint4*>((p.G2 ? p.G2 : X) + j * p.ldg2 + kk);
      }
    } else {
      const int64_t off = v ? (KF ? row * srow + k : k * sk + row) : 0;
      st.x[it] = *reinterpret_cast<const uint4*>(X + off);
    }
    ok |= (v ? 1u : 0u) << it;
    if (RO) {
      // head-outer: KF (A = dH [m][d]): r = row, cols = k..k+7; row-fast (B = dH [k][n]):
      // r = k, cols = row..row+7
      const int64_t r = v ? (KF ? row : k) : 0;
      const int64_t cc = v ? (KF ? k : row) : 0;
      const int64_t h = cc / p.hF;
      st.d1[it] = p.de[r * p.hH + h];
      st.d2[it] = p.de2 != nullptr ? p.de2[r * p.hH + h] : 0.f;
      if (it == 0) {
        st.h1[0] = *reinterpret_cast<const float4*>(p.ha + cc);
        st.h1[1] = *reinterpret_cast<const float4*>(p.ha + cc + 4);
        if (p.ha2 != nullptr) {
          st.h2[0] = *reinterpret_cast<const float4*>(p.ha2 + cc);
          st.h2[1] = *reinterpret_cast<const float4*>(p.ha2 + cc + 4);
        } else {
          st.h2[0] = st.h2[1] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
    }
  }
  st.ok = ok;
}

__device__ __forceinline__ uint4 head_outer8(uint4 x, float d1, float d2, const float4 (&h1)[2],
                                             const float4 (&h2)[2]) {
  const Pk<bf16_t> a = pk_load(reinterpret_cast<const bf16_t*>(&x));
  const float hv1[8] = {h1[0].x, h1[0].y, h1[0].z, h1[0].w, h1[1].x, h1[1].y, h1[1].z, h1[1].w};
  const float hv2[8] = {h2[0].x, h2[0].y, h2[0].z, h2[0].w, h2[1].x, h2[1].y, h2[1].z, h2[1].w};
  Pk<bf16_t> r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = fmaf(d2, hv2[i], fmaf(d1, hv1[i], a.v[i]));
  uint4 o;
  pk_store(reinterpret_cast<bf16_t*>(&o), r);
  return o;
}

__device__ __forceinline__ uint4 hadamard8(uint4 x, uint4 y) {
  const Pk<bf16_t> a = pk_load(reinterpret_cast<const bf16_t*>(&x));
  const Pk<bf16_t> b = pk_load(reinterpret_cast<const bf16_t*>(&y));
  Pk<bf16_t> r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = a.v[i] * b.v[i];
  uint4 o;
  pk_store(reinterpret_cast<bf16_t*>(&o), r);
  return o;
}

template <int KF, bool RO, bool GH = false>
__device__ __forceinline__ void store_operand(const Stage& st, bf16_t* img, int tid,
                                              bool hadamard = false) {
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int c = tid + 256 * it;
    uint4 x = st.x[it];
    if (GH && hadamard) x = hadamard8(x, st.y[it]);
    if (RO) x = head_outer8(x, st.d1[it], st.d2[it], st.h1, st.h2);
    if (!((st.ok >> it) & 1u)) x = make_uint4(0u, 0u, 0u, 0u);
    const int off = KF ? (c >> 3) * PKF + 8 * (c & 7) : (c >> 4) * PRF + 8 * (c & 15);
    *reinterpret_cast<uint4*>(img + off) = x;
  }
}

// MFMA fragment of a 16-row (A) / 16-column (B) tile starting at rt, k-step s
template <int KF>
__device__ __forceinline__ bf16x8 read_frag(const bf16_t* img, int rt, int s, int lane) {
  const int g = lane >> 4, i = lane & 15;
  bf16x4 lo, hi;
  if (KF) {
    const bf16_t* q = img + (rt + i) * PKF + 32 * s + 4 * g;
    lo = *reinterpret_cast<const bf16x4*>(q);
    hi = *reinterpret_cast<const bf16x4*>(q + 16);
  } else {
    const int qq = i >> 2, pp = i & 3;
    const bf16_t* q = img + (32 * s + 4 * g + qq) * PRF + rt + 4 * pp;
    typedef __attribute__((address_space(3))) bf16x4 lds_v4;
    lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4*)(q));
    hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4*)(q + 16 * PRF));
  }
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

template <int EPI, int FEPI, int AK, int BK_, int HO, bool GA = false>
__global__ void __launch_bounds__(256) gemm_bf16_kernel(Args p) {
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * IMG];
  bf16_t* As = smem;
  bf16_t* Bs = smem + IMG;
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

  // A: rows m (sAm), k (sAk); B: rows n (sBn), k (sBk)
  Stage sa, sb;
  if (kb < ke) {
    load_operand<AK, HO == HO_A, GA>(p, p.A, p.sAm, p.sAk, p.M, m0, kb, ke, tid, sa);
    load_operand<BK_, HO == HO_B>(p, p.B, p.sBn, p.sBk, p.N, n0, kb, ke, tid, sb);
  }
  for (int64_t k0 = kb; k0 < ke; k0 += BK) {
    __syncthreads();
    store_operand<AK, HO == HO_A, GA>(sa, As, tid, p.hadamard);
    store_operand<BK_, HO == HO_B>(sb, Bs, tid);
    __syncthreads();
    if (k0 + BK < ke) {
      load_operand<AK, HO == HO_A, GA>(p, p.A, p.sAm, p.sAk, p.M, m0, k0 + BK, ke, tid, sa);
      load_operand<BK_, HO == HO_B>(p, p.B, p.sBn, p.sBk, p.N, n0, k0 + BK, ke, tid, sb);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 a0 = read_frag<AK>(As, w * 32, s, lane);
      const bf16x8 a1 = read_frag<AK>(As, w * 32 + 16, s, lane);
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const bf16x8 b = read_frag<BK_>(Bs, c * 16, s, lane);
        acc[0][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b, acc[0][c], 0, 0, 0);
        acc[1][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b, acc[1][c], 0, 0, 0);
      }
    }
  }

  // ---- epilogue (C/D layout: col = lane & 15, row = (lane >> 4) * 4 + reg).  The
  // 16-row halves are staged through LDS and written back in 4 passes of 4 rows: lane l
  // covers columns 8(l & 15) .. +7 of row 4*pass + (l >> 4) -- a wave-store is four
  // contiguous row segments; per-head score dots reduce over the head's F/8 lanes.
  static_assert(4 * 16 * TP * 4 <= 2 * IMG * 2, "epilogue staging exceeds LDS");
  __syncthreads();
  float* T = reinterpret_cast<float*>(smem) + w * (16 * TP);
  const bool to_slab = p.slab != nullptr;
  const int c8 = (lane & 15) * 8;
  const int64_t col = n0 + c8;
  const bool col_ok = col < p.N;  // N % 8 == 0: the 8 columns are all in or all out
  float al8[8], ar8[8], bi8[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    al8[u] = EPI == EPI_SCORE && p.al && col_ok ? p.al[col + u] : 0.f;
    ar8[u] = EPI == EPI_SCORE && p.ar && col_ok ? p.ar[col + u] : 0.f;
    bi8[u] = EPI == EPI_ACT && (p.act & ACT_BIAS) && col_ok ? p.bias[col + u] : 0.f;
  }
#pragma unroll
  for (int r = 0; r < 2; ++r) {
#pragma unroll
    for (int c = 0; c < 8; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i) T[((lane >> 4) * 4 + i) * TP + c * 16 + (lane & 15)] = acc[r][c][i];
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
#pragma unroll 1
    for (int pass = 0; pass < 4; ++pass) {
      const int rr = 4 * pass + (lane >> 4);
      const int64_t row = m0 + w * 32 + r * 16 + rr;
      const float4 lo = *reinterpret_cast<const float4*>(T + rr * TP + c8);
      const float4 hi = *reinterpret_cast<const float4*>(T + rr * TP + c8 + 4);
      float e[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
      if (EPI == EPI_ACT) {
        uint32_t kb = 0xffu;
        if (p.act & ACT_DROPOUT) {
          kb = 0u;
          const uint64_t off = dropout_offset(p.dp, p.dp.offset);
#pragma unroll 1
          for (int u = 0; u < 8; ++u)
            if (philox_x(p.dp.seed, off, (uint64_t)(row * p.N + col + u)) >= p.dp.threshold)
              kb |= 1u << u;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          float x = e[u] + bi8[u];
          if (p.act & ACT_RELU) x = fmaxf(x, 0.f);
          if (p.act & ACT_DROPOUT) x *= ((kb >> u) & 1u) ? p.dp.scale : 0.f;
          if (p.act & ACT_SIGMOID) x = 1.f / (1.f + __expf(-x));
          e[u] = x;
        }
      }
      if (row < p.M && col_ok) {
        if (to_slab || !p.c_bf16) {
          float* o = to_slab ? p.slab + (int64_t)blockIdx.z * p.M * p.N + row * p.N + col
                             : reinterpret_cast<float*>(p.C) + row * p.ldc + col;
          *reinterpret_cast<float4*>(o) = make_float4(e[0], e[1], e[2], e[3]);
          *reinterpret_cast<float4*>(o + 4) = make_float4(e[4], e[5], e[6], e[7]);
        } else {
          Pk<bf16_t> pk;
#pragma unroll
          for (int u = 0; u < 8; ++u) pk.v[u] = e[u];
          pk_store(reinterpret_cast<bf16_t*>(p.C) + row * p.ldc + col, pk);
        }
      }
      if (EPI == EPI_SCORE) {
        constexpr int FE = FEPI > 0 ? FEPI : 16;  // >= 8: a head covers FE / 8 lanes
        // the stored (bf16-rounded) row in the row-score order of the edge kernels
        // (msha_project_scores_row_order): last element first, fma downwards
        float x8[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) x8[u] = (float)(bf16_t)e[u];
        float sl = x8[7] * al8[7], sr = x8[7] * ar8[7];
#pragma unroll
        for (int u = 6; u >= 0; --u) {
          sl = fmaf(x8[u], al8[u], sl);
          sr = fmaf(x8[u], ar8[u], sr);
        }
#pragma unroll
        for (int o = 1; o < FE / 8; o <<= 1) {
          sl += __shfl_xor(sl, o);
          sr += __shfl_xor(sr, o);
        }
        const int64_t hg = col / FE;
        if ((c8 % FE) == 0 && row < p.M && hg < p.H && col_ok) {
          if (p.el) p.el[row * p.H + hg] = sl;
          if (p.er) p.er[row * p.H + hg] = sr;
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
  }
}

// C = sum_z slab[z] (4 interleaved z-subsets per block, combined in fixed order)
template <typename T>
__global__ void __launch_bounds__(256) slab_reduce_kernel(const float* __restrict__ slab,
                                                          int splits, int64_t M, int64_t N,
                                                          T* __restrict__ C, int64_t ldc) {
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
      C[(t / N) * ldc + t % N] = from_f32<T>(s);
    }
    __syncthreads();
  }
}

static bool al16(const void* q) { return ((uintptr_t)q & 15) == 0; }

template <int EPI, int FEPI, int HO>
static void launch(const Args& p, bool ak, bool bk, int splits, hipStream_t s) {
  const dim3 grid((unsigned)((p.M + BM - 1) / BM), (unsigned)((p.N + BN - 1) / BN),
                  (unsigned)splits);
  if (ak && bk)
    hipLaunchKernelGGL((gemm_bf16_kernel<EPI, FEPI, 1, 1, HO>), grid, dim3(256), 0, s, p);
  else if (ak)
    hipLaunchKernelGGL((gemm_bf16_kernel<EPI, FEPI, 1, 0, HO>), grid, dim3(256), 0, s, p);
  else if (bk)
    hipLaunchKernelGGL((gemm_bf16_kernel<EPI, FEPI, 0, 1, HO>), grid, dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL((gemm_bf16_kernel<EPI, FEPI, 0, 0, HO>), grid, dim3(256), 0, s, p);
}

// operand layout check: one unit stride, the other stride / extent multiples of 8
static int layout_of(int64_t srow, int64_t sk, int64_t rows, int64_t K, const void* base,
                     bool& kfast) {
  if (!al16(base)) return 0;
  if (sk == 1 && srow % 8 == 0 && K % 8 == 0) { kfast = true; return 1; }
  if (srow == 1 && sk % 8 == 0 && rows % 8 == 0) { kfast = false; return 1; }
  return 0;
}

}  // namespace bfg
}  // namespace msha

using namespace msha;
using namespace msha::bfg;

extern "C" size_t msha_gemm_bf16_workspace_size(int64_t M, int64_t N, int32_t splits) {
  if (splits <= 1) return 0;
  return (size_t)splits * (size_t)M * (size_t)N * sizeof(float);
}

extern "C" int msha_gemm_bf16(int64_t M, int64_t N, int64_t K, const void* A, int64_t sAm,
                              int64_t sAk, const void* B, int64_t sBk, int64_t sBn, void* C,
                              int64_t ldc, int32_t c_dtype, int32_t splits, void* ws,
                              size_t ws_bytes, int32_t ho_operand, int32_t heads, int32_t feat,
                              const float* de, const float* a, const float* de2,
                              const float* a2, msha_stream_t stream) {
  MSHA_ARG_CHECK(M > 0 && N > 0 && K > 0, "gemm_bf16: bad sizes");
  MSHA_ARG_CHECK(A && B && C, "gemm_bf16: null pointer");
  MSHA_ARG_CHECK(c_dtype == MSHA_DTYPE_F32 || c_dtype == MSHA_DTYPE_BF16, "gemm_bf16: bad c_dtype");
  MSHA_ARG_CHECK(splits >= 1 && splits <= 65535, "gemm_bf16: splits out of range");
  MSHA_ARG_CHECK(N % 8 == 0 && ldc % 8 == 0 && al16(C), "gemm_bf16: N, ldc must be multiples of 8, C 16-B aligned");
  MSHA_ARG_CHECK(ho_operand >= -1 && ho_operand <= 1, "gemm_bf16: ho_operand must be -1, 0 or 1");
  Args p;
  memset(&p, 0, sizeof(p));
  p.M = M; p.N = N; p.K = K;
  p.A = (const bf16_t*)A; p.sAm = sAm; p.sAk = sAk;
  p.B = (const bf16_t*)B; p.sBk = sBk; p.sBn = sBn;
  p.C = C; p.ldc = ldc; p.c_bf16 = c_dtype == MSHA_DTYPE_BF16;
  bool ak = true, bk = true;
  if (!layout_of(sAm, sAk, M, K, A, ak) || !layout_of(sBn, sBk, N, K, B, bk))
    return fail(MSHA_ERR_UNSUPPORTED, "gemm_bf16: each operand needs one unit stride, the other "
                                      "a multiple of 8, its extent along the unit stride a "
                                      "multiple of 8, and a 16-byte aligned base");
  if (ho_operand >= 0) {
    MSHA_ARG_CHECK(de && a && ((de2 == nullptr) == (a2 == nullptr)), "gemm_bf16: head-outer pointers");
    MSHA_ARG_CHECK(heads > 0 && feat > 0 && feat % 8 == 0, "gemm_bf16: head-outer needs feat % 8 == 0");
    MSHA_ARG_CHECK((ho_operand == 0 ? K : N) == (int64_t)heads * feat,
                   "gemm_bf16: the updated operand's columns must be heads*feat");
    if (ho_operand == 0 ? !ak : bk)
      return fail(MSHA_ERR_UNSUPPORTED, "gemm_bf16: head-outer needs A k-contiguous (operand 0) "
                                        "or B n-contiguous (operand 1)");
    MSHA_ARG_CHECK(al16(a) && (a2 == nullptr || al16(a2)), "gemm_bf16: a / a2 must be 16-B aligned");
    p.de = de; p.ha = a; p.de2 = de2; p.ha2 = a2; p.hH = heads; p.hF = feat;
  }
  hipStream_t s = (hipStream_t)stream;
  int used = 1;
  if (splits > 1) {
    MSHA_ARG_CHECK(ws && ws_bytes >= msha_gemm_bf16_workspace_size(M, N, splits),
                   "gemm_bf16: split-K workspace too small");
    int64_t kc = (K + splits - 1) / splits;
    kc = ((kc + BK - 1) / BK) * BK;
    used = (int)((K + kc - 1) / kc);
    p.k_chunk = kc;
    p.slab = (float*)ws;
  }
  if (ho_operand == 0) launch<EPI_STORE, 0, HO_A>(p, ak, bk, used, s);
  else if (ho_operand == 1) launch<EPI_STORE, 0, HO_B>(p, ak, bk, used, s);
  else launch<EPI_STORE, 0, HO_NONE>(p, ak, bk, used, s);
  if (splits > 1) {
    const dim3 g(grid_for((M * N + 63) / 64, 1, 65535));
    if (p.c_bf16)
      hipLaunchKernelGGL(slab_reduce_kernel<bf16_t>, g, dim3(256), 0, s, (const float*)ws, used,
                         M, N, (bf16_t*)C, ldc);
    else
      hipLaunchKernelGGL(slab_reduce_kernel<float>, g, dim3(256), 0, s, (const float*)ws, used,
                         M, N, (float*)C, ldc);
  }
  return check_launch("gemm_bf16");
}

extern "C" int msha_project_scores_bf16(int64_t M, int64_t K, int32_t heads, int32_t feat,
                                        const void* X, const void* W, const float* al,
                                        const float* ar, void* h, float* el, float* er,
                                        msha_stream_t stream) {
  MSHA_ARG_CHECK(M > 0 && K > 0 && heads > 0 && feat > 0, "project_scores_bf16: bad sizes");
  MSHA_ARG_CHECK(X && W && h, "project_scores_bf16: null pointer");
  MSHA_ARG_CHECK((al == nullptr) == (el == nullptr) && (ar == nullptr) == (er == nullptr),
                 "project_scores_bf16: score vectors and outputs must be paired");
  const int64_t N = (int64_t)heads * feat;
  MSHA_ARG_CHECK(K % 8 == 0 && N % 8 == 0 && al16(X) && al16(W) && al16(h),
                 "project_scores_bf16: K and heads*feat must be multiples of 8, 16-B aligned buffers");
  Args p;
  memset(&p, 0, sizeof(p));
  p.M = M; p.N = N; p.K = K;
  p.A = (const bf16_t*)X; p.sAm = K; p.sAk = 1;
  p.B = (const bf16_t*)W; p.sBk = N; p.sBn = 1;
  p.C = h; p.ldc = N; p.c_bf16 = 1;
  p.al = al; p.ar = ar; p.el = el; p.er = er; p.H = heads;
  hipStream_t s = (hipStream_t)stream;
  if (skinny_project<bf16_t>(M, K, heads, feat, X, W, al, ar, h, el, er, s))
    return check_launch("project_scores_bf16");
  if (al == nullptr && ar == nullptr) {
    launch<EPI_STORE, 0, HO_NONE>(p, true, false, 1, s);
  } else {
    MSHA_ARG_CHECK((al == nullptr || al16(al)) && (ar == nullptr || al16(ar)),
                   "project_scores_bf16: al / ar must be 16-B aligned");
    if (feat == 8) launch<EPI_SCORE, 8, HO_NONE>(p, true, false, 1, s);
    else if (feat == 16) launch<EPI_SCORE, 16, HO_NONE>(p, true, false, 1, s);
    else if (feat == 32) launch<EPI_SCORE, 32, HO_NONE>(p, true, false, 1, s);
    else if (feat == 64) launch<EPI_SCORE, 64, HO_NONE>(p, true, false, 1, s);
    else if (feat == 128) launch<EPI_SCORE, 128, HO_NONE>(p, true, false, 1, s);
    else
      return fail(MSHA_ERR_UNSUPPORTED, "project_scores_bf16: feat must be 8, 16, 32, 64 or 128 "
                                        "when score vectors are given");
  }
  return check_launch("project_scores_bf16");
}

extern "C" int msha_pair_linear_bf16_ex(int64_t n_pairs, int64_t K, int64_t N, const void* G,
                                        int64_t ldg, const int64_t* gi, const void* G2,
                                        int64_t ldg2, const int64_t* gj, const void* W,
                                        const float* bias, int32_t act, float drop_p,
                                        uint64_t seed, uint64_t offset, int32_t out_dtype,
                                        void* out, msha_stream_t stream) {
  MSHA_ARG_CHECK(n_pairs > 0 && K > 0 && N > 0, "pair_linear_bf16: bad sizes");
  MSHA_ARG_CHECK(G && W && out, "pair_linear_bf16: null pointer");
  MSHA_ARG_CHECK(!(act & ACT_BIAS) || bias, "pair_linear_bf16: bias missing");
  MSHA_ARG_CHECK(out_dtype == MSHA_DTYPE_F32 || out_dtype == MSHA_DTYPE_BF16,
                 "pair_linear_bf16: out dtype must be fp32 or bf16");
  MSHA_ARG_CHECK(K % 8 == 0 && N % 8 == 0 && ldg % 8 == 0 && (G2 == nullptr || ldg2 % 8 == 0) &&
                     al16(G) && (G2 == nullptr || al16(G2)) && al16(W) && al16(out),
                 "pair_linear_bf16: K, N, ld multiples of 8 and 16-byte aligned tables");
  Args p;
  memset(&p, 0, sizeof(p));
  p.M = n_pairs; p.N = N; p.K = K;
  p.A = (const bf16_t*)G; p.sAm = ldg; p.sAk = 1;
  p.gi = gi; p.gj = gj; p.G2 = (const bf16_t*)G2; p.ldg2 = G2 ? ldg2 : ldg;
  p.hadamard = G2 != nullptr || gj != nullptr;
  p.B = (const bf16_t*)W; p.sBk = 1; p.sBn = K;  // nn.Linear weight (N x K)
  p.C = out; p.ldc = N; p.c_bf16 = out_dtype == MSHA_DTYPE_BF16;
  p.act = act; p.bias = bias;
  p.dp = make_dropout(drop_p, seed, offset, (hipStream_t)stream);
  if (!p.dp.active) p.act &= ~ACT_DROPOUT;
  if (skinny_pair_linear_bf16(n_pairs, K, N, G, ldg, gi, G2, ldg2, gj, W, bias, p.act, p.dp, out,
                              p.c_bf16 != 0, (hipStream_t)stream))
    return check_launch("pair_linear_bf16");
  const dim3 grid((unsigned)((n_pairs + BM - 1) / BM), (unsigned)((N + BN - 1) / BN), 1);
  hipLaunchKernelGGL((gemm_bf16_kernel<EPI_ACT, 0, 1, 1, HO_NONE, true>), grid, dim3(256), 0,
                     (hipStream_t)stream, p);
  return check_launch("pair_linear_bf16");
}

extern "C" int msha_pair_linear_bf16(int64_t n_pairs, int64_t K, int64_t N, const void* G,
                                     int64_t ldg, const int64_t* gi, const void* G2,
                                     int64_t ldg2, const int64_t* gj, const void* W,
                                     const float* bias, int32_t act, float drop_p, uint64_t seed,
                                     uint64_t offset, float* out, msha_stream_t stream) {
  return msha_pair_linear_bf16_ex(n_pairs, K, N, G, ldg, gi, G2, ldg2, gj, W, bias, act, drop_p,
                                  seed, offset, MSHA_DTYPE_F32, out, stream);
}
