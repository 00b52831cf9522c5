// fp32 weight gradient on the bf16 matrix pipe (split-bf16): dW = X^T D'.
//
// The projections' weight gradient (the autograd of Ablation.py:262-263, h = X @ W):
//   dW[a, n] = sum_r X[r, a] (D[r, n] + d1[r, n / hF] a1[n] + d2[r, n / hF] a2[n])
// over K = 100k .. 1M rows, a, n < 128.  gfx950 has no xf32/TF32, and the exact-fp32 MFMA
// (skinny.hip wgrad_kernel, v_mfma_f32_32x32x2_f32) runs at 1/16 of the bf16 rate: 0.55
// of that peak at bip1m was the whole kernel.  Here every fp32 operand is split into
// three bf16 terms x = x_h + x_m + x_l (both subtractions exact in fp32, |x - sum| <=
// 2^-27 |x|) and the six products whose weight reaches fp32's 2^-24 (lh, hl, mm, mh, hm,
// hh, small first) run as v_mfma_f32_16x16x32_bf16 into fp32 accumulators -- the scheme of
// skinny.hip's pair_x3_kernel and split projection, here for two TRANSPOSED streams:
// both operands are contracted over rows r, and both are row-major in memory, so each
// 64-row tile is staged as [r][a] / [r][n] bf16 images (the rows as loaded: 16-B chunks)
// and read as MFMA fragments with ds_read_b64_tr_b16 (gemm_bf16.hip's operand scheme).
//
// Block = 4 waves, one per SIMD (the six 18 KB images take 110 KB of LDS); wave w owns
// dW rows [32 w, 32 w + 32) x all 128 columns (2 x 8 accumulator tiles of 16 x 16).  Per
// 64-row tile: the next tile's fp32 rows are loaded into registers while this one is
// multiplied; the head-outer term and the optional column sums of the score-vector
// gradients (CS: dal[n] = sum_r d1[r, n / hF] hs[r, n], Ablation.py:266-267 backward)
// are formed while splitting.  Block partials go to the caller's slab and
// skinny.hip's wgrad_reduce_kernel sums them in block order (deterministic).
#include "common.h"

namespace msha {
namespace wx3 {

constexpr int BK = 64;         // rows (the contraction) per tile
constexpr int PRF = 128 + 16;  // image pitch (bf16): 288 B, tr16 reads conflict free
constexpr int IMG = BK * PRF;  // bf16 elements per image
constexpr int kThreads = 256;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_v4;

// MFMA fragment (16 image columns from rt, k-step s of 32 rows) of a [k][col] image:
// lane (g = l >> 4, i = l & 15) takes k slots 4g + j (j < 4) and 16 + 4g + j - 4 (j >= 4)
// of the step -- the same map for both operands, so the k permutation cancels
__device__ __forceinline__ bf16x8 frag(const bf16_t* img, int rt, int s, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const bf16_t* q = img + (32 * s + 4 * g + (i >> 2)) * PRF + rt + 4 * (i & 3);
  const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4*)q);
  const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4*)(q + 16 * PRF));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// 4 fp32 -> their three bf16 terms, 8 bytes each (round to nearest even at every step)
__device__ __forceinline__ void split4(float4 x, uint2& h, uint2& m, uint2& l) {
  const float v[4] = {x.x, x.y, x.z, x.w};
  uint32_t hw[2], mw[2], lw[2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const float a = v[2 * p], b = v[2 * p + 1];
    hw[p] = pack_bf16x2(a, b);
    const float ra = a - __uint_as_float(hw[p] << 16), rb = b - __uint_as_float(hw[p] & 0xffff0000u);
    mw[p] = pack_bf16x2(ra, rb);
    const float sa = ra - __uint_as_float(mw[p] << 16), sb = rb - __uint_as_float(mw[p] & 0xffff0000u);
    lw[p] = pack_bf16x2(sa, sb);
  }
  h = make_uint2(hw[0], hw[1]);
  m = make_uint2(mw[0], mw[1]);
  l = make_uint2(lw[0], lw[1]);
}

template <bool HO, bool CS>
__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(1, 1)))
wgrad_x3_kernel(int M, const float* __restrict__ X, int64_t ldx, const float* __restrict__ D,
                int64_t ldd, const float* __restrict__ d1, const float* __restrict__ a1,
                const float* __restrict__ d2, const float* __restrict__ a2, int hH, int hF,
                float* __restrict__ slab, const float* __restrict__ hs, float* __restrict__ cpart) {
  __shared__ __attribute__((aligned(16))) bf16_t smem[6 * IMG];  // X h m l, D' h m l
  __shared__ float csred[CS ? 2 * 8 * 128 : 1];                   // [which][row lane group][n]
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nb = gridDim.x;
  const int r0 = (int)(((int64_t)blockIdx.x * M) / nb), r1 = (int)(((int64_t)(blockIdx.x + 1) * M) / nb);
  // staging: chunk it of a tile = row (tid >> 5) + 8 it, columns 4 (tid & 31) .. + 3
  const int c4 = 4 * (tid & 31), rs = tid >> 5;
  const int hh = HO ? c4 / hF : 0;
  float4 av1 = make_float4(0.f, 0.f, 0.f, 0.f), av2 = av1;
  if (HO) {
    av1 = *reinterpret_cast<const float4*>(a1 + c4);
    if (d2 != nullptr) av2 = *reinterpret_cast<const float4*>(a2 + c4);
  }
  const rsrc_t r_x = make_rsrc(X, (uint32_t)((int64_t)M * ldx * 4));
  const rsrc_t r_d = make_rsrc(D, (uint32_t)((int64_t)M * ldd * 4));
  const rsrc_t r_e1 = make_rsrc(HO ? d1 : nullptr, HO ? (uint32_t)((int64_t)M * hH * 4) : 0u);
  const rsrc_t r_e2 = make_rsrc(HO ? d2 : nullptr, HO && d2 ? (uint32_t)((int64_t)M * hH * 4) : 0u);
  const rsrc_t r_h = make_rsrc(CS ? hs : nullptr, CS ? (uint32_t)((int64_t)M * ldd * 4) : 0u);
  struct Tile {
    u32x4_t x[8], d[8], h[CS ? 8 : 1];
    float e1[8], e2[8];
  };
  auto load = [&](int rb, Tile& t) {
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int row = rb + rs + 8 * it;
      const uint32_t m = row < r1 ? 0u : kOOB;  // rows past the block's range read 0
      const uint32_t ur = (uint32_t)row;
      t.x[it] = buf_b128(r_x, (ur * (uint32_t)ldx * 4u + 4u * c4) | m);
      t.d[it] = buf_b128(r_d, (ur * (uint32_t)ldd * 4u + 4u * c4) | m);
      if (HO) {
        t.e1[it] = buf_f32(r_e1, (ur * (uint32_t)hH * 4u + 4u * hh) | m);
        t.e2[it] = buf_f32(r_e2, (ur * (uint32_t)hH * 4u + 4u * hh) | m);
      }
      if (CS) t.h[it] = buf_b128(r_h, (ur * (uint32_t)ldd * 4u + 4u * c4) | m);
    }
  };
  float4 cs1 = make_float4(0.f, 0.f, 0.f, 0.f), cs2 = cs1;
  auto stage = [&](const Tile& t) {
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int k = rs + 8 * it;
      float4 x = make_float4(__uint_as_float(t.x[it].x), __uint_as_float(t.x[it].y),
                             __uint_as_float(t.x[it].z), __uint_as_float(t.x[it].w));
      float4 d = make_float4(__uint_as_float(t.d[it].x), __uint_as_float(t.d[it].y),
                             __uint_as_float(t.d[it].z), __uint_as_float(t.d[it].w));
      if (HO) {  // D' = D + d1 a1 + d2 a2 (skinny.hip wgrad_kernel's fma order)
        d.x = fmaf(t.e2[it], av2.x, fmaf(t.e1[it], av1.x, d.x));
        d.y = fmaf(t.e2[it], av2.y, fmaf(t.e1[it], av1.y, d.y));
        d.z = fmaf(t.e2[it], av2.z, fmaf(t.e1[it], av1.z, d.z));
        d.w = fmaf(t.e2[it], av2.w, fmaf(t.e1[it], av1.w, d.w));
      }
      if (CS) {
        const float4 hv = make_float4(__uint_as_float(t.h[it].x), __uint_as_float(t.h[it].y),
                                      __uint_as_float(t.h[it].z), __uint_as_float(t.h[it].w));
        cs1 = make_float4(fmaf(t.e1[it], hv.x, cs1.x), fmaf(t.e1[it], hv.y, cs1.y),
                          fmaf(t.e1[it], hv.z, cs1.z), fmaf(t.e1[it], hv.w, cs1.w));
        cs2 = make_float4(fmaf(t.e2[it], hv.x, cs2.x), fmaf(t.e2[it], hv.y, cs2.y),
                          fmaf(t.e2[it], hv.z, cs2.z), fmaf(t.e2[it], hv.w, cs2.w));
      }
      uint2 h, m, l;
      split4(x, h, m, l);
      bf16_t* p = smem + k * PRF + c4;
      *reinterpret_cast<uint2*>(p) = h;
      *reinterpret_cast<uint2*>(p + IMG) = m;
      *reinterpret_cast<uint2*>(p + 2 * IMG) = l;
      split4(d, h, m, l);
      *reinterpret_cast<uint2*>(p + 3 * IMG) = h;
      *reinterpret_cast<uint2*>(p + 4 * IMG) = m;
      *reinterpret_cast<uint2*>(p + 5 * IMG) = l;
    }
  };

  f32x4 acc[2][8];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[r][c] = f32x4{0.f, 0.f, 0.f, 0.f};

  Tile cur;
  if (r0 < r1) load(r0, cur);
  for (int rb = r0; rb < r1; rb += BK) {
    __syncthreads();  // the previous tile's fragment reads are done
    stage(cur);
    if (rb + BK < r1) load(rb + BK, cur);  // in flight under this tile's MFMAs
    __syncthreads();
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 a[2][3];
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int t = 0; t < 3; ++t) a[r][t] = frag(smem + t * IMG, 32 * w + 16 * r, s, lane);
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        bf16x8 b[3];
#pragma unroll
        for (int t = 0; t < 3; ++t) b[t] = frag(smem + (3 + t) * IMG, 16 * c, s, lane);
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          f32x4 v = acc[r][c];
          v = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[r][2], b[0], v, 0, 0, 0);  // lh
          v = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[r][0], b[2], v, 0, 0, 0);  // hl
          v = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[r][1], b[1], v, 0, 0, 0);  // mm
          v = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[r][1], b[0], v, 0, 0, 0);  // mh
          v = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[r][0], b[1], v, 0, 0, 0);  // hm
          v = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[r][0], b[0], v, 0, 0, 0);  // hh
          acc[r][c] = v;
        }
      }
    }
  }
  // block partial: slab[block][a][n]; C layout col = lane & 15, row = 4 (lane >> 4) + v
  float* out = slab + (int64_t)blockIdx.x * (128 * 128);
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int c = 0; c < 8; ++c)
#pragma unroll
      for (int v = 0; v < 4; ++v)
        out[(32 * w + 16 * r + 4 * (lane >> 4) + v) * 128 + 16 * c + (lane & 15)] = acc[r][c][v];
  if (CS) {  // rows of the block: the 8 row groups of a column, in order
    *reinterpret_cast<float4*>(csred + (0 * 8 + rs) * 128 + c4) = cs1;
    *reinterpret_cast<float4*>(csred + (1 * 8 + rs) * 128 + c4) = cs2;
    __syncthreads();
    for (int i = tid; i < 2 * 128; i += kThreads) {
      const int which = i >> 7, n = i & 127;
      float v = 0.f;
#pragma unroll
      for (int g = 0; g < 8; ++g) v += csred[(which * 8 + g) * 128 + n];
      cpart[((int64_t)which * 128 + n) * nb + blockIdx.x] = v;  // part[which][n][block]
    }
  }
}

}  // namespace wx3

// dW block partials into slab (nb x 128 x 128) for skinny.hip's wgrad_reduce_kernel; 1 =
// launched.  Opt-in (MSHA_WGRAD=x3): measured slower than the exact-fp32 wgrad_kernel at
// bip1m (421 vs 382 us) and R15 (27.5 vs 21 us), profiles/round5_bench_v1/README.md; the
// register-operand split (skinny.hip wgrad_s3_kernel) replaced both.
int wgrad_x3(int64_t K, const float* X, int64_t ldx, const float* D, int64_t ldd, int hH, int hF,
             const float* de, const float* a, const float* de2, const float* a2, float* slab,
             int nb, const float* cs_tab, float* cs_part, hipStream_t s) {
  if (K * ldx * 4 >= (1ll << 31) || K * ldd * 4 >= (1ll << 31)) return 0;
  const dim3 grid(nb), block(wx3::kThreads);
  if (cs_tab != nullptr)
    hipLaunchKernelGGL((wx3::wgrad_x3_kernel<true, true>), grid, block, 0, s, (int)K, X, ldx, D,
                       ldd, de, a, de2, a2, hH, hF, slab, cs_tab, cs_part);
  else if (de != nullptr)
    hipLaunchKernelGGL((wx3::wgrad_x3_kernel<true, false>), grid, block, 0, s, (int)K, X, ldx, D,
                       ldd, de, a, de2, a2, hH, hF, slab, nullptr, nullptr);
  else
    hipLaunchKernelGGL((wx3::wgrad_x3_kernel<false, false>), grid, block, 0, s, (int)K, X, ldx, D,
                       ldd, nullptr, nullptr, nullptr, nullptr, 1, 4, slab, nullptr, nullptr);
  return 1;
}

}  // namespace msha
