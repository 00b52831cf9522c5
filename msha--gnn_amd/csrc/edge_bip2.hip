// Bipartite edge attention on row masks (edge_bip2.hip): the repo's shape, 2 heads x 64.
//
// Every graph the reference trains on has M <= 32 recipient columns (Adjacent/Flow
// 2015-2018, the bip1m stress graph), so a source row's adjacency is one 32-bit column
// mask (msha_graph.rowmask).  These kernels replace the CSR walk of edge_bip.hip (per-group
// binary search, slot records, segmented DPP scans) with two phases per 32-row tile:
//
//   phase A, lane = (row t, head h) = t + 32 h: the row softmax over the 32 columns in
//     registers -- bit j of the mask gates score j, the column scores er_j sit in the
//     lane's own registers, so max, sum and normalisation are straight-line VALU with no
//     cross-lane traffic; the attention stays in the lane's 32-register vector s[].
//   phase B, lane = element (h0 f = l, h1 f = l): each row walks its mask bits (s_ff1 on
//     the wave-uniform mask); the two heads' attention of edge (t, j) comes out of s[j]
//     of lanes t / t + 32 (v_readlane, the vector indexed by the uniform j), so
//     u += att hc_j is one packed FMA against hc_j from LDS, and v_j += att hs_i one packed
//     FMA into the wave's LDS slab.
//
// Reference: Ablation.py:266-274 (OursLayer3 scores, masked softmax, dropout, u = att @ h1,
// v = att.T @ h2), Ours.py:84-86 (the attention export the MSHA layer records).
// Dropout draws the same Philox stream as every other edge kernel: element e * H + h of
// CSR edge e.  Accumulation order: u over the row's edges in column order (= CSR order),
// v over rows in wave order, waves in block order, blocks in order (bip_reduce).
#include "edge_geo.h"

namespace msha {

// block partials -> output (edge_bip.hip bip_reduce_kernel): out[i] = sum_b part[b][i]
int bip_reduce(const float* part, int32_t nb, int32_t stride, int32_t n, int32_t n_t, void* out_t,
               bool bf16, float* out_f, int32_t fblk, hipStream_t s);

namespace bip2 {

typedef float f32x32 __attribute__((ext_vector_type(32)));

constexpr int kF = 64, kD = 128;   // 2 heads x 64: one element of each head per lane
constexpr int kWaves = 8;          // 16.5 KB table + 8 x 16.5 KB slabs
constexpr int kTile = 32;          // rows per tile: phase A lane = row + 32 head
constexpr int kBlk = 8;            // rows per element block (hs one block ahead)
constexpr int kRows = 33;          // LDS table / slab rows: 32 columns + the pair's dummy
constexpr float kLog2e = 1.4426950408889634f;

__device__ __forceinline__ float rdl(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// a lane's two elements (h0 f = l, h1 f = l) of table row r, raw
template <typename T>
__device__ __forceinline__ void ld_pair(rsrc_t rs, uint32_t lane, uint32_t row_soff, uint32_t (&w)[2]) {
  if constexpr (sizeof(T) == 4) {
    w[0] = __builtin_amdgcn_raw_buffer_load_b32(rs, lane * 4u, row_soff, 0);
    w[1] = __builtin_amdgcn_raw_buffer_load_b32(rs, lane * 4u + 256u, row_soff, 0);
  } else {
    w[0] = __builtin_amdgcn_raw_buffer_load_b16(rs, lane * 2u, row_soff, 0);
    w[1] = __builtin_amdgcn_raw_buffer_load_b16(rs, lane * 2u + 128u, row_soff, 0);
  }
}
template <typename T>
__device__ __forceinline__ float2 unpack_pair(const uint32_t (&w)[2]) {
  if constexpr (sizeof(T) == 4) return make_float2(__uint_as_float(w[0]), __uint_as_float(w[1]));
  else return make_float2(__uint_as_float(w[0] << 16), __uint_as_float(w[1] << 16));
}
template <typename T>
__device__ __forceinline__ void st_pair(rsrc_t rs, uint32_t lane, uint32_t row_soff, float2 x) {
  if constexpr (sizeof(T) == 4) {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(x.x), rs, lane * 4u, row_soff, 0);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(x.y), rs, lane * 4u + 256u, row_soff, 0);
  } else {
    __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(uint16_t, (bf16_t)x.x), rs, lane * 2u,
                                          row_soff, 0);
    __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(uint16_t, (bf16_t)x.y), rs,
                                          lane * 2u + 128u, row_soff, 0);
  }
}

__device__ __forceinline__ float2 fma2(float2 a, float2 x, float2 c) {
  return make_float2(fmaf(a.x, x.x, c.x), fmaf(a.y, x.y, c.y));
}

// bit j of m as an all-ones / zero word
__device__ __forceinline__ uint32_t bitmask(uint32_t m, int j) {
  return (uint32_t)(((int32_t)(m << (31 - j))) >> 31);
}

// Phase A: lane (t, h) -> s[j] = attention of (row t, column j, head h) (0 where row t has
// no edge j), lse of (t, h).  elv = el[t][h], flag = virtual full row (score 0 everywhere).
template <bool VIRT>
__device__ __forceinline__ float row_softmax(uint32_t mk, float elv, bool virt, const float* erl,
                                             float slope, f32x32& s) {
  constexpr float NINF = -INFINITY;
  float mx = NINF;
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    float x = elv + erl[2 * j];  // er[j][h]: LDS broadcast reads (no 32-register copy)
    x = fmaxf(x, x * slope);  // lrelu, slope in [0, 1]
    if (VIRT) x = virt ? 0.f : x;
    const uint32_t b = bitmask(mk, j);
    x = __uint_as_float((__float_as_uint(x) & b) | (__float_as_uint(NINF) & ~b));
    s[j] = x;
    mx = fmaxf(mx, x);
  }
  const float m2 = mx == NINF ? 0.f : mx * kLog2e;
  float l = 0.f;
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    const float p = __builtin_amdgcn_exp2f(fmaf(s[j], kLog2e, -m2));
    s[j] = p;
    l += p;
  }
  const float inv = __builtin_amdgcn_rcpf(l);
#pragma unroll
  for (int j = 0; j < 32; ++j) s[j] *= inv;
  return mx == NINF ? NINF : mx + __logf(l);
}

// ------------------------------------------------------------------------ forward ---
template <typename T, bool HS, bool ATTD>
__global__ void __launch_bounds__(kWaves * 64) bip2_fwd_kernel(
    const uint32_t* __restrict__ rowmask, const int32_t* __restrict__ rowptr,
    const uint8_t* __restrict__ rowflag, int32_t n_rows, int32_t M, int32_t n_edges,
    const float* __restrict__ el, const float* __restrict__ er, const T* __restrict__ hc,
    const T* __restrict__ hs, float slope, Dropout dp, T* __restrict__ u,
    float* __restrict__ lse, float* __restrict__ attd, float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) float2 tab[kRows * 64];
  __shared__ __attribute__((aligned(16))) float2 slab[HS ? kWaves : 1][HS ? kRows * 64 : 2];
  __shared__ float ert[64];
  __shared__ uint64_t kw[kWaves][32];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  for (int i = tid; i < kRows * 64; i += kWaves * 64) {  // tab[j][l] = (hc[j][0][l], hc[j][1][l])
    const int j = i >> 6, l = i & 63;
    tab[i] = j < M ? make_float2(to_f32(hc[j * kD + l]), to_f32(hc[j * kD + kF + l]))
                   : make_float2(0.f, 0.f);
  }
  if (tid < 64) ert[tid] = (tid >> 1) < M ? er[tid] : 0.f;
  if (HS)
    for (int i = lane; i < kRows * 64; i += 64) slab[wv][i] = make_float2(0.f, 0.f);
  __syncthreads();

  const int t = lane & 31, h = lane >> 5;
  const float* erl = ert + h;  // er[j][h] = erl[2 j]
  const bool drop = dp.active;
  const uint64_t doff = drop ? dropout_offset(dp, dp.offset) : 0;
  const bool need_rp = ATTD || drop;

  const int64_t Wt = (int64_t)gridDim.x * kWaves, w = (int64_t)blockIdx.x * kWaves + wv;
  const int32_t rb = (int32_t)(w * n_rows / Wt), re = (int32_t)((w + 1) * n_rows / Wt);
  if (rb < re) {
    const rsrc_t r_mask = make_rsrc(rowmask, (uint32_t)re * 4u);
    const rsrc_t r_rp = make_rsrc(need_rp ? rowptr : nullptr, (uint32_t)(re + 1) * 4u);
    const rsrc_t r_flag = make_rsrc(rowflag, (uint32_t)re);
    const rsrc_t r_el = make_rsrc(el, (uint32_t)re * 8u);
    const rsrc_t r_lse = make_rsrc(lse, (uint32_t)re * 8u);
    const rsrc_t r_hs = make_rsrc(HS ? hs : nullptr, (uint32_t)re * kD * (uint32_t)sizeof(T));
    const rsrc_t r_u = make_rsrc(u, (uint32_t)re * kD * (uint32_t)sizeof(T));
    const rsrc_t r_att = make_rsrc(ATTD ? attd : nullptr, (uint32_t)n_edges * 8u);
    constexpr uint32_t RB = kD * sizeof(T);
    const uint32_t v_tl = (uint32_t)t * 4u, v_el = (uint32_t)(t * 2 + h) * 4u;  // (row t, head h)
    const float2* tabl = tab + lane;
    float2* slabl = HS ? &slab[wv][lane] : nullptr;

    // phase-A inputs of a tile (one load each), hs rows of a block (two per row)
    auto load_a = [&](int32_t r0, uint32_t& mk, float& elv, uint32_t& fl, int32_t& rp) {
      mk = __builtin_amdgcn_raw_buffer_load_b32(r_mask, v_tl, (uint32_t)r0 * 4u, 0);
      elv = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r_el, v_el, (uint32_t)r0 * 8u, 0));
      fl = __builtin_amdgcn_raw_buffer_load_b8(r_flag, (uint32_t)t, (uint32_t)r0, 0);
      rp = need_rp ? (int32_t)__builtin_amdgcn_raw_buffer_load_b32(r_rp, v_tl, (uint32_t)r0 * 4u, 0) : 0;
    };
    uint32_t ring[2][kBlk][2];
    auto load_blk = [&](int32_t r0, uint32_t (&rg)[kBlk][2]) {
#pragma unroll
      for (int i = 0; i < kBlk; ++i) {
        if (HS) ld_pair<T>(r_hs, (uint32_t)lane, (uint32_t)(r0 + i) * RB, rg[i]);
        else rg[i][0] = rg[i][1] = 0u;
      }
    };

    uint32_t mk_n, fl_n;
    float el_n;
    int32_t rp_n;
    load_a(rb, mk_n, el_n, fl_n, rp_n);
    load_blk(rb, ring[0]);
    for (int32_t r0 = rb; r0 < re; r0 += kTile) {
      const uint32_t mk = mk_n, fl = fl_n;
      const float elv = el_n;
      const int32_t rp = rp_n;
      load_a(r0 + kTile, mk_n, el_n, fl_n, rp_n);

      // ---- phase A: softmax of (row t, head h) over its mask
      f32x32 s;
      const bool virt = fl != 0;
      float ls;
      if (__builtin_amdgcn_ballot_w64(virt) != 0) ls = row_softmax<true>(mk, elv, virt, erl, slope, s);
      else ls = row_softmax<false>(mk, elv, virt, erl, slope, s);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(ls), r_lse, v_el, (uint32_t)r0 * 8u, 0);
      if (drop || ATTD) {
        // tile edges [E0, E1): rows r0 .. min(re, r0 + 32) - 1 are contiguous in the CSR
        const int tl = min(kTile, re - r0) - 1;
        const int32_t E0 = __builtin_amdgcn_readlane(rp, 0);
        const int32_t E1 = __builtin_amdgcn_readlane(rp + (int32_t)__popc(mk), tl);
        if (drop) {
          // keep bits of the tile's (edge, head) elements, 32 edges x 2 heads per word
          for (int32_t c = 0; c * 32 < E1 - E0; ++c) {
            const int32_t e = E0 + c * 32 + t;
            const bool k = e < E1 && philox_x(dp.seed, doff, (uint64_t)e * 2u + (uint64_t)h) >= dp.threshold;
            const uint64_t word = __builtin_amdgcn_ballot_w64(k);
            if (lane == 0) kw[wv][c & 31] = word;
          }
        }
        int32_t k = 0;
        const int32_t base = rp - E0;
#pragma unroll
        for (int j = 0; j < 32; ++j) {
          const bool bit = (mk >> j) & 1u;
          if (drop) {
            const int32_t idx = min(base + k, 32 * 32 - 1);
            const uint64_t wd = kw[wv][idx >> 5];
            const bool keep = (wd >> ((idx & 31) + 32 * h)) & 1ull;
            s[j] *= keep ? dp.scale : 0.f;
          }
          if (ATTD)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(s[j]), r_att,
                                                  bit ? (uint32_t)(rp + k) * 8u + (uint32_t)h * 4u : kOOB,
                                                  0, 0);
          k += bit ? 1 : 0;
        }
      }

      // ---- phase B: element lanes walk each row's mask
#pragma unroll
      for (int bk = 0; bk < kTile / kBlk; ++bk) {
        load_blk(r0 + (bk + 1) * kBlk, ring[(bk + 1) & 1]);
#pragma unroll
        for (int i = 0; i < kBlk; ++i) {
          const int tr = bk * kBlk + i;
          uint32_t m = (uint32_t)__builtin_amdgcn_readlane((int)mk, tr);
          const float2 hv = unpack_pair<T>(ring[bk & 1][i]);
          float2 acc = make_float2(0.f, 0.f);
          while (m) {
            const int j0 = __builtin_ctz(m);
            m &= m - 1;
            // a row's odd last edge pairs with the dummy column 32: its table row is zero
            // and its slab row is never read, so the (finite) attention read for it is moot
            const int j1 = __builtin_ctzll((uint64_t)m | (1ull << 32));
            m &= m - 1;
            const float s0 = s[j0];
            const float2 a = make_float2(rdl(s0, tr), rdl(s0, tr + 32));
            const float s1 = s[j1 & 31];
            const float2 b = make_float2(rdl(s1, tr), rdl(s1, tr + 32));
            const float2 x0 = tabl[j0 * 64], x1 = tabl[j1 * 64];
            acc = fma2(b, x1, fma2(a, x0, acc));
            if (HS) {
              float2 y0 = slabl[j0 * 64], y1 = slabl[j1 * 64];
              y0 = fma2(a, hv, y0);
              y1 = fma2(b, hv, y1);
              slabl[j0 * 64] = y0;
              slabl[j1 * 64] = y1;
            }
          }
          st_pair<T>(r_u, (uint32_t)lane, (uint32_t)(r0 + tr) * RB, acc);
        }
      }
    }
  }
  if (HS) {
    __syncthreads();
    float* dst = part + (int64_t)blockIdx.x * (M * kD);
    for (int i = tid; i < M * 64; i += kWaves * 64) {  // (column j, element l)
      float2 a = slab[0][i];
#pragma unroll
      for (int q = 1; q < kWaves; ++q) {
        const float2 b = slab[q][i];
        a.x += b.x;
        a.y += b.y;
      }
      const int j = i >> 6, l = i & 63;
      dst[j * kD + l] = a.x;
      dst[j * kD + kF + l] = a.y;
    }
  }
}


// ----------------------------------------------------------------------- backward ---
// Per row i, head h (the autograd of Ablation.py:266-274; Ours.py:84-86 adds coef):
//   g_e  = dU_i . hc_j (+ hs_i . dV_j) (+ coef_i exp(attd_e))
//   D_i  = sum_e attd_e g_e,  ds_e = att_e (keep_e g_e - D_i),  de_e = ds_e lrelu'(pre_e)
//   d_el_i = sum_e de_e,  d_hs_i = sum_e attd_e dV_j,  d_hc_j += attd_e dU_i,  d_er_j += de_e
// Per 32-row tile: phase A (lane = (row, head)) recomputes att from lse (and the keep bits);
// phase B (element lanes) walks each row's mask two edges a step: d_hs in registers, d_hc
// into the wave's slab, and the two edges' per-lane dot partials reduced to g by one
// permlane32 swap per edge, one permlane16 swap per pair and four DPP row rotations -- the
// sums land in the lanes (row t, head h) that phase C reads, written into G[j] by a
// select; phase C (lane = (row, head)) finishes D, de, d_el and the lane's d_er
// accumulators.  d_er is summed over lanes, waves and blocks in order at the end.
constexpr int kWavesB = 7;  // two 16.5 KB tables + 7 x 16.5 KB d_hc slabs
constexpr int kBlkB = 4;    // rows per element block (dU / hs one block ahead)

template <int N>
__device__ __forceinline__ float ror_add(float v) {  // v + v of lane (l + N) % 16 in its row
  // (update_dpp with the add's identity as the old value: folds into one v_add_f32_dpp)
  return v + __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v),
                                                                    0x120 + N, 0xF, 0xF, true));
}
// (x, y) -> x' = [x lanes 0-31, y lanes 0-31], y' = [x lanes 32-63, y lanes 32-63]
__device__ __forceinline__ float swap32_add(float x, float y) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(y), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float swap16_add(float x, float y) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(y), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float swap16(float x) {  // rows 0 <-> 1, 2 <-> 3
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  const int l = threadIdx.x & 63;
  return __uint_as_float((l & 16) ? r[0] : r[1]);
}

template <typename T, bool HS, bool COEF, bool DROP>
__global__ void __launch_bounds__(kWavesB * 64) bip2_bwd_kernel(
    const uint32_t* __restrict__ rowmask, const int32_t* __restrict__ rowptr,
    const uint8_t* __restrict__ rowflag, int32_t n_rows, int32_t M, int32_t n_edges,
    const float* __restrict__ el, const float* __restrict__ er, const T* __restrict__ hc,
    const float* __restrict__ lse, const T* __restrict__ dU, const T* __restrict__ hs,
    const T* __restrict__ dV, const float* __restrict__ row_coef, float slope, Dropout dp,
    float* __restrict__ d_el, T* __restrict__ d_hs, float* __restrict__ part) {
  // hc then dV (one base address, dV at a fixed offset)
  __shared__ __attribute__((aligned(16))) float2 tab[(HS ? 2 : 1) * kRows * 64];
  float2* const tdv = tab + kRows * 64;
  __shared__ __attribute__((aligned(16))) float2 slab[kWavesB][kRows * 64];
  __shared__ float ert[64];
  __shared__ float sder[kWavesB][64];
  __shared__ uint64_t kw[kWavesB][32];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  for (int i = tid; i < kRows * 64; i += kWavesB * 64) {
    const int j = i >> 6, l = i & 63;
    tab[i] = j < M ? make_float2(to_f32(hc[j * kD + l]), to_f32(hc[j * kD + kF + l]))
                   : make_float2(0.f, 0.f);
    if (HS)
      tdv[i] = j < M ? make_float2(to_f32(dV[j * kD + l]), to_f32(dV[j * kD + kF + l]))
                     : make_float2(0.f, 0.f);
  }
  if (tid < 64) ert[tid] = (tid >> 1) < M ? er[tid] : 0.f;
  for (int i = lane; i < kRows * 64; i += 64) slab[wv][i] = make_float2(0.f, 0.f);
  __syncthreads();

  const int t = lane & 31, h = lane >> 5;
  f32x32 derv;  // this lane's d_er (column j, head h) over the wave's rows
#pragma unroll
  for (int j = 0; j < 32; ++j) derv[j] = 0.f;
  const float* erl = ert + h;  // er[j][h] = erl[2 j] (LDS broadcast reads: no 32-register copy)
  const uint64_t doff = DROP ? dropout_offset(dp, dp.offset) : 0;

  const int64_t Wt = (int64_t)gridDim.x * kWavesB, w = (int64_t)blockIdx.x * kWavesB + wv;
  const int32_t rb = (int32_t)(w * n_rows / Wt), re = (int32_t)((w + 1) * n_rows / Wt);
  if (rb < re) {
    const rsrc_t r_mask = make_rsrc(rowmask, (uint32_t)re * 4u);
    const rsrc_t r_rp = make_rsrc(DROP ? rowptr : nullptr, (uint32_t)(re + 1) * 4u);
    const rsrc_t r_flag = make_rsrc(rowflag, (uint32_t)re);
    const rsrc_t r_el = make_rsrc(el, (uint32_t)re * 8u);
    const rsrc_t r_lse = make_rsrc(lse, (uint32_t)re * 8u);
    const rsrc_t r_cf = make_rsrc(COEF ? row_coef : nullptr, (uint32_t)re * 8u);
    const rsrc_t r_del = make_rsrc(d_el, (uint32_t)re * 8u);
    const rsrc_t r_du = make_rsrc(dU, (uint32_t)re * kD * (uint32_t)sizeof(T));
    const rsrc_t r_hs = make_rsrc(HS ? hs : nullptr, (uint32_t)re * kD * (uint32_t)sizeof(T));
    const rsrc_t r_dhs = make_rsrc(HS ? d_hs : nullptr, (uint32_t)re * kD * (uint32_t)sizeof(T));
    constexpr uint32_t RB = kD * sizeof(T);
    const uint32_t v_tl = (uint32_t)t * 4u, v_el = (uint32_t)(t * 2 + h) * 4u;
    const float2* tabl = tab + lane;
    const float2* tdvl = tdv + lane;
    float2* slabl = &slab[wv][lane];

    struct In {
      uint32_t mk, fl;
      float elv, lsv, cf;
      int32_t rp;
    };
    auto load_a = [&](int32_t r0, In& a) {
      a.mk = __builtin_amdgcn_raw_buffer_load_b32(r_mask, v_tl, (uint32_t)r0 * 4u, 0);
      a.elv = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r_el, v_el, (uint32_t)r0 * 8u, 0));
      a.lsv = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r_lse, v_el, (uint32_t)r0 * 8u, 0));
      a.cf = COEF ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r_cf, v_el, (uint32_t)r0 * 8u, 0)) : 0.f;
      a.fl = __builtin_amdgcn_raw_buffer_load_b8(r_flag, (uint32_t)t, (uint32_t)r0, 0);
      a.rp = DROP ? (int32_t)__builtin_amdgcn_raw_buffer_load_b32(r_rp, v_tl, (uint32_t)r0 * 4u, 0) : 0;
    };
    constexpr int NT = HS ? 2 : 1;
    uint32_t ring[2][kBlkB][NT][2];
    auto load_blk = [&](int32_t r0, uint32_t (&rg)[kBlkB][NT][2]) {
#pragma unroll
      for (int i = 0; i < kBlkB; ++i) {
        ld_pair<T>(r_du, (uint32_t)lane, (uint32_t)(r0 + i) * RB, rg[i][0]);
        if (HS) ld_pair<T>(r_hs, (uint32_t)lane, (uint32_t)(r0 + i) * RB, rg[i][NT - 1]);
      }
    };

    In nx;
    load_a(rb, nx);
    load_blk(rb, ring[0]);
    for (int32_t r0 = rb; r0 < re; r0 += kTile) {
      const In cu = nx;
      load_a(r0 + kTile, nx);
      const bool virt = cu.fl != 0;

      // ---- phase A: att = exp(score - lse) on the mask (0 elsewhere); attd with the keep
      f32x32 s, sa;
      const float l2 = cu.lsv * kLog2e;
#pragma unroll
      for (int j = 0; j < 32; ++j) {
        float x = cu.elv + erl[2 * j];
        x = fmaxf(x, x * slope);
        x = virt ? 0.f : x;
        const uint32_t b = bitmask(cu.mk, j);
        const float a = __builtin_amdgcn_exp2f(fmaf(x, kLog2e, -l2));
        s[j] = __uint_as_float(__float_as_uint(a) & b);
      }
      if (DROP) {
        const int tl = min(kTile, re - r0) - 1;
        const int32_t E0 = __builtin_amdgcn_readlane(cu.rp, 0);
        const int32_t E1 = __builtin_amdgcn_readlane(cu.rp + (int32_t)__popc(cu.mk), tl);
        for (int32_t c = 0; c * 32 < E1 - E0; ++c) {
          const int32_t e = E0 + c * 32 + t;
          const bool k = e < E1 && philox_x(dp.seed, doff, (uint64_t)e * 2u + (uint64_t)h) >= dp.threshold;
          const uint64_t word = __builtin_amdgcn_ballot_w64(k);
          if (lane == 0) kw[wv][c & 31] = word;
        }
        int32_t k = 0;
        const int32_t base = cu.rp - E0;
#pragma unroll
        for (int j = 0; j < 32; ++j) {
          const bool bit = (cu.mk >> j) & 1u;
          const int32_t idx = min(base + k, 32 * 32 - 1);
          const uint64_t wd = kw[wv][idx >> 5];
          const bool keep = (wd >> ((idx & 31) + 32 * h)) & 1ull;
          sa[j] = s[j];
          s[j] *= keep ? dp.scale : 0.f;
          k += bit ? 1 : 0;
        }
      }
      f32x32 G;
#pragma unroll
      for (int j = 0; j < 32; ++j) G[j] = 0.f;

      // ---- phase B: element lanes
#pragma unroll
      for (int bk = 0; bk < kTile / kBlkB; ++bk) {
        load_blk(r0 + (bk + 1) * kBlkB, ring[(bk + 1) & 1]);
#pragma unroll
        for (int i = 0; i < kBlkB; ++i) {
          const int tr = bk * kBlkB + i;
          uint32_t m = (uint32_t)__builtin_amdgcn_readlane((int)cu.mk, tr);
          const float2 du = unpack_pair<T>(ring[bk & 1][i][0]);
          const float2 hv = HS ? unpack_pair<T>(ring[bk & 1][i][NT - 1]) : make_float2(0.f, 0.f);
          float2 dhs = make_float2(0.f, 0.f);
          // lanes (tr, h) of G: rows 0 / 2 of the reduced pair hold edge 0's g when tr < 16
          const bool mine = (lane & 31) == tr;
          if (m != 0u && (m & (m - 1u)) == 0u) {
            // a one-edge row: att = 1, so ds = attd g (1 - att) = 0 whatever g is; only the
            // dV / d_hc products remain (the reference's softmax backward gives exactly 0)
            const int j0 = __builtin_ctz(m);
            m = 0u;
            const float s0 = s[j0];
            const float2 a = make_float2(rdl(s0, tr), rdl(s0, tr + 32));
            if (HS) dhs = fma2(a, tdvl[j0 * 64], dhs);
            slabl[j0 * 64] = fma2(a, du, slabl[j0 * 64]);
          }
          while (m) {
            const int j0 = __builtin_ctz(m);
            m &= m - 1;
            // a lone last edge pairs with the dummy column 32 (zero table rows, a slab row
            // never read, G left alone): its attention read is moot
            const int j1 = __builtin_ctzll((uint64_t)m | (1ull << 32));
            const bool two = j1 < 32;
            m &= m - 1;
            const float s0 = s[j0];
            const float2 a = make_float2(rdl(s0, tr), rdl(s0, tr + 32));
            const float s1 = s[j1 & 31];
            const float2 b = make_float2(rdl(s1, tr), rdl(s1, tr + 32));
            const float2 x0 = tabl[j0 * 64], x1 = tabl[j1 * 64];
            float2 p0 = make_float2(du.x * x0.x, du.y * x0.y);
            float2 p1 = make_float2(du.x * x1.x, du.y * x1.y);
            if (HS) {
              const float2 y0 = tdvl[j0 * 64], y1 = tdvl[j1 * 64];
              p0 = fma2(hv, y0, p0);
              p1 = fma2(hv, y1, p1);
              dhs = fma2(b, y1, fma2(a, y0, dhs));
            }
            float2 z0 = slabl[j0 * 64], z1 = slabl[j1 * 64];
            z0 = fma2(a, du, z0);
            z1 = fma2(b, du, z1);
            slabl[j0 * 64] = z0;
            slabl[j1 * 64] = z1;
            // g of (edge 0, 1) x (head 0, 1): lanes 0-15 (e0,h0), 16-31 (e1,h0),
            // 32-47 (e0,h1), 48-63 (e1,h1), every lane of a 16-lane row the row's sum
            float wsum = swap16_add(swap32_add(p0.x, p0.y), swap32_add(p1.x, p1.y));
            wsum = ror_add<8>(wsum);
            wsum = ror_add<4>(wsum);
            wsum = ror_add<2>(wsum);
            wsum = ror_add<1>(wsum);
            const float wsw = swap16(wsum);
            const float g0 = tr < 16 ? wsum : wsw, g1 = tr < 16 ? wsw : wsum;
            const float gj0 = G[j0];
            G[j0] = mine ? g0 : gj0;
            const float gj1 = G[j1 & 31];
            G[j1 & 31] = mine && two ? g1 : gj1;
          }
          if (HS) st_pair<T>(r_dhs, (uint32_t)lane, (uint32_t)(r0 + tr) * RB, dhs);
        }
      }

      // ---- phase C: lane (row, head): D, de, d_el, d_er
      float D = 0.f;
#pragma unroll
      for (int j = 0; j < 32; ++j) {
        if (COEF) {
          const uint32_t b = bitmask(cu.mk, j);
          const float c = cu.cf * __expf(s[j]);
          G[j] += __uint_as_float(__float_as_uint(c) & b);
        }
        D = fmaf(s[j], G[j], D);
      }
      float del = 0.f;
#pragma unroll
      for (int j = 0; j < 32; ++j) {
        // ds = att (keep g - D) = attd g - att D
        const float ds = DROP ? fmaf(s[j], G[j], -sa[j] * D) : s[j] * (G[j] - D);
        const float pre = cu.elv + erl[2 * j];
        float de = ds * (pre > 0.f ? 1.f : slope);
        const uint32_t b = bitmask(cu.mk, j) & (virt ? 0u : ~0u);
        de = __uint_as_float(__float_as_uint(de) & b);
        del += de;
        derv[j] += de;
      }
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(del), r_del, v_el, (uint32_t)r0 * 8u, 0);
    }
  }
  // d_er: lanes (t, h) -> per (j, h) over the wave's rows, then waves in order
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    float v = derv[j];
    v = ror_add<8>(v);
    v = ror_add<4>(v);
    v = ror_add<2>(v);
    v = ror_add<1>(v);
    v += swap16(v);  // both 16-lane rows of each head half
    if (lane == 0) sder[wv][j * 2] = v;
    if (lane == 32) sder[wv][j * 2 + 1] = v;
  }
  __syncthreads();
  const int MD = M * kD, MH = M * 2;
  float* dst = part + (int64_t)blockIdx.x * (((MD + MH) + 3) & ~3);
  for (int i = tid; i < M * 64; i += kWavesB * 64) {
    float2 a = slab[0][i];
#pragma unroll
    for (int q = 1; q < kWavesB; ++q) {
      const float2 b = slab[q][i];
      a.x += b.x;
      a.y += b.y;
    }
    const int j = i >> 6, l = i & 63;
    dst[j * kD + l] = a.x;
    dst[j * kD + kF + l] = a.y;
  }
  for (int i = tid; i < MH; i += kWavesB * 64) {
    float a = sder[0][i];
#pragma unroll
    for (int q = 1; q < kWavesB; ++q) a += sder[q][i];
    dst[MD + i] = a;
  }
}

}  // namespace bip2

bool bip2_ok(const msha_graph* g, int heads, int feat, float slope) {
  static const int env = [] {
    const char* v = getenv("MSHA_BIP2");
    return v != nullptr && *v ? atoi(v) : 1;
  }();
  return env != 0 && heads == 2 && feat == 64 && g->rowmask != nullptr && g->n_cols <= 32 &&
         slope >= 0.f && slope <= 1.f && g->n_rows * (int64_t)bip2::kD * 4 < (1ll << 31) &&
         g->n_edges * 8ll < (1ll << 31);
}

// 1 = launched (forward + the v reduce), 0 = not covered
int bip2_fwd(const msha_graph* g, int dtype, const float* el, const float* er, const void* hc,
             const void* hs, float slope, const Dropout& dp, void* u, float* lse, float* attd,
             void* v, float* part, int nb, hipStream_t s) {
  const dim3 grid(nb), block(bip2::kWaves * 64);
  auto go = [&](auto kern, auto tag) {
    using T = decltype(tag);
    hipLaunchKernelGGL(kern, grid, block, 0, s, g->rowmask, g->rowptr, g->rowflag,
                       (int32_t)g->n_rows, (int32_t)g->n_cols, (int32_t)g->n_edges, el, er,
                       (const T*)hc, (const T*)hs, slope, dp, (T*)u, lse, attd, part);
  };
  const bool bf = dtype == MSHA_DTYPE_BF16;
  const bool H = hs != nullptr, A = attd != nullptr;
#define GO(T_, HS_, A_) go(bip2::bip2_fwd_kernel<T_, HS_, A_>, T_{})
  if (bf) {
    if (H && A) GO(bf16_t, true, true);
    else if (H) GO(bf16_t, true, false);
    else if (A) GO(bf16_t, false, true);
    else GO(bf16_t, false, false);
  } else {
    if (H && A) GO(float, true, true);
    else if (H) GO(float, true, false);
    else if (A) GO(float, false, true);
    else GO(float, false, false);
  }
#undef GO
  if (H) {
    const int32_t MD = (int32_t)(g->n_cols * bip2::kD);
    bip_reduce(part, nb, MD, MD, MD, v, bf, nullptr, 1, s);
  }
  return 1;
}

}  // namespace msha

namespace msha {
int bip2_bwd(const msha_graph* g, int dtype, const float* el, const float* er, const void* hc,
             const float* lse, const void* dU, const void* hs, const void* dV,
             const float* row_coef, float slope, const Dropout& dp, float* d_el, float* d_er,
             void* d_hc, void* d_hs, float* part, int nb, hipStream_t s) {
  const dim3 grid(nb), block(bip2::kWavesB * 64);
  auto go = [&](auto kern, auto tag) {
    using T = decltype(tag);
    hipLaunchKernelGGL(kern, grid, block, 0, s, g->rowmask, g->rowptr, g->rowflag,
                       (int32_t)g->n_rows, (int32_t)g->n_cols, (int32_t)g->n_edges, el, er,
                       (const T*)hc, lse, (const T*)dU, (const T*)hs, (const T*)dV, row_coef,
                       slope, dp, d_el, (T*)d_hs, part);
  };
  const bool bf = dtype == MSHA_DTYPE_BF16;
  const bool H = dV != nullptr, C = row_coef != nullptr, D = dp.active;
#define GO(T_, H_, C_, D_) go(bip2::bip2_bwd_kernel<T_, H_, C_, D_>, T_{})
#define GO4(T_)                                      \
  if (H && C && D) GO(T_, true, true, true);         \
  else if (H && C) GO(T_, true, true, false);        \
  else if (H && D) GO(T_, true, false, true);        \
  else if (H) GO(T_, true, false, false);            \
  else if (C && D) GO(T_, false, true, true);        \
  else if (C) GO(T_, false, true, false);            \
  else if (D) GO(T_, false, false, true);            \
  else GO(T_, false, false, false);
  if (bf) { GO4(bf16_t) } else { GO4(float) }
#undef GO4
#undef GO
  const int32_t MD = (int32_t)(g->n_cols * bip2::kD), MH = (int32_t)(g->n_cols * 2);
  bip_reduce(part, nb, (MD + MH + 3) & ~3, MD + MH, MD, d_hc, bf, d_er, MH, s);
  return 1;
}
}  // namespace msha
