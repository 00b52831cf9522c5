// Bipartite edge attention on the matrix cores (edge_bip3.hip): the repo's shape, M <= 32
// recipient columns, 2 heads x 64 (Adjacent/Flow 2015-2018, the bip1m stress graph).
//
// A wave takes 32-row tiles of its contiguous row range.  Per tile and head the attention
// is a dense 32 x 32 matrix (zero off the row masks), so both aggregates are 32 x 32 x 64
// products on v_mfma_f32_32x32x16_bf16:
//
//   phase A, lane (row t, half c) = t + 32 c: the row softmax over the lane's 16 columns
//     col(c, r) = 4c + (r & 3) + 8 (r >> 2), r = 0..15, both heads (32 registers); the
//     row max and sum meet the partner lane's half with one v_permlane32_swap each.  That
//     column set is the MFMA A operand of att (rows on the lanes) as it stands: k-step s
//     takes r = 8s .. 8s + 7.
//   u = att hc : B = hc, a per-block LDS image of B fragments in the same k order;
//   v += att^T hs : A = att^T from a per-wave LDS image read back with
//     ds_read_b64_tr_b16, B = hs with rows along k, loaded straight from HBM as
//     128-byte row pieces (lane = feature, 8 rows per fragment).  v stays in the MFMA
//     accumulators for the wave's whole row range (no LDS slab): the waves' partials are
//     summed in a fixed order at the end, the blocks' by bip_reduce.
//
// fp32 tables: every operand is split into three bf16 terms x = x_h + x_m + x_l and the six
// products whose weight reaches 2^-24 run (hh, hm, mh, mm, hl, lh; the skinny.hip
// scheme), so the result is fp32-level, not bf16-level.  bf16 tables are exact bf16 and
// the attention (fp32) takes two terms: two products.
//
// Reference: Ablation.py:266-274 (OursLayer3 scores, masked softmax, dropout, u = att @ h1,
// v = att.T @ h2), Ours.py:84-86 (the attention the MSHA layer records).  Dropout draws
// the stream of every other edge kernel: element e * 2 + h of CSR edge e.
#include <algorithm>

#include "edge_geo.h"

// no fp contraction in this file: a product and a later add are not fused differently
// between template variants (u-only and full forwards give the same bits); fmaf is
// written out where a fused multiply-add is meant
#pragma clang fp contract(off)

namespace msha {

int bip_reduce(const float* part, int32_t nb, int32_t stride, int32_t n, int32_t n_t, void* out_t,
               bool bf16, float* out_f, int32_t fblk, hipStream_t s);

namespace bip3 {

// ---- per-wave timeline (diagnostic build, -DSK_TIMELINE; scripts/bip_timeline.py) ------
// Lane 0 of every wave stamps (wall clock at 100 MHz, shader clock) pairs at fixed mark
// indices into its slot of the buffer msha_debug_bip_timeline installs: the forward's
// waves use the first half of the slots, the backward's the second; words 0 / 1 = XCC id
// << 32 | HW_ID and the kernel tag, mark k at words 2 + 2k.  In the shipped build every
// mark compiles to nothing.
constexpr int kTlStride = 64;  // 64-bit words per wave slot
#ifdef SK_TIMELINE
__device__ uint64_t* g_tl = nullptr;
__device__ int64_t g_tl_slots = 0;
struct Tl {
  uint64_t* p;
};
__device__ __forceinline__ Tl tl_open(int bwd, int tag) {
  const int64_t half = g_tl_slots / 2;
  const int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  Tl r{nullptr};
  if (g_tl != nullptr && w < half) r.p = g_tl + (bwd * half + w) * kTlStride;
  if (r.p != nullptr && (threadIdx.x & 63) == 0) {
    const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_ID
    const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
    r.p[0] = ((uint64_t)xcc << 32) | hw;
    r.p[1] = (uint64_t)tag;
  }
  return r;
}
__device__ __forceinline__ void tl_mark(const Tl& r, int k) {
  if (r.p != nullptr && (threadIdx.x & 63) == 0 && 2 * k + 3 < kTlStride) {
    r.p[2 + 2 * k] = __builtin_amdgcn_s_memrealtime();
    r.p[3 + 2 * k] = __builtin_amdgcn_s_memtime();
  }
}
#define B3TL_OPEN(bwd, tag) const ::msha::bip3::Tl tl_ = ::msha::bip3::tl_open(bwd, tag)
#define B3TL_MARK(k) ::msha::bip3::tl_mark(tl_, (k))
#else
#define B3TL_OPEN(bwd, tag) \
  do {                      \
  } while (0)
#define B3TL_MARK(k) \
  do {               \
  } while (0)
#endif
// marks: 0 entry, 1 tables staged, per tile it < kTlTiles kTlPer marks from 2 + kTlPer it,
// then loop end and exit
constexpr int kTlTiles = 4;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) bf16x4 lds_v4;

constexpr int kF = 64, kD = 128;  // 2 heads x 64
constexpr int kWaves = 8;
constexpr int kTile = 32;
constexpr float kLog2e = 1.4426950408889634f;
#ifndef BIP3_PF
#define BIP3_PF 2
#endif
constexpr int kPf = BIP3_PF;  // forward: tiles of hs fragments in flight ahead (1 or 2)

// Static tile split of a block's range [b0, b1) over its n parts (wave pairs forward, waves
// backward): the first half of the parts are the first-dispatched wave of each SIMD, which
// wins the SIMD's issue arbitration by age (bip1m timelines: the second wave's loop runs
// 7-12 % longer on the same tiles), so it takes 1 + skew/1000 shares, the second half
// 1 - skew/1000.  Part k starts at the cumulative weight of parts < k.
__device__ __forceinline__ int32_t skew_split(int32_t b0, int32_t b1, int k, int n, int skew) {
  const int64_t wo = 1000 + skew, wy = 1000 - skew, h = n / 2;
  const int64_t cum = k <= h ? k * wo : h * wo + (k - h) * wy;
  return b0 + (int32_t)((int64_t)(b1 - b0) * cum / (h * (wo + wy)));
}

// column of the lane's r-th attention value (half c)
__device__ __forceinline__ constexpr int col_of(int c, int r) { return 4 * c + (r & 3) + 8 * (r >> 2); }

__device__ __forceinline__ uint32_t bitmask(uint32_t m, int j) {
  return (uint32_t)(((int32_t)(m << (31 - j))) >> 31);
}

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// x -> NT bf16 terms (1: exact bf16 input, 2: hi + mid, 3: hi + mid + lo)
template <int NT>
struct Terms {
  bf16x8 t[NT];
};
template <int NT>
__device__ __forceinline__ Terms<NT> split(const float (&x)[8]) {
  Terms<NT> r;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const bf16_t h = (bf16_t)x[e];
    r.t[0][e] = h;
    if (NT > 1) {
      const float r1 = x[e] - (float)h;
      const bf16_t m = (bf16_t)r1;
      r.t[NT > 1 ? 1 : 0][e] = m;
      if (NT > 2) r.t[NT > 2 ? 2 : 0][e] = (bf16_t)(r1 - (float)m);
    }
  }
  return r;
}

// acc += A B over the kept products of the split terms (NA terms of A, NB of B), the small
// ones first
template <int NA, int NB>
__device__ __forceinline__ f32x16 prod(const bf16x8 (&a)[NA], const bf16x8 (&b)[NB], f32x16 acc) {
  if constexpr (NA == 3 && NB == 3) {
    acc = mfma(a[2], b[0], acc);
    acc = mfma(a[0], b[2], acc);
    acc = mfma(a[1], b[1], acc);
    acc = mfma(a[0], b[1], acc);
    acc = mfma(a[1], b[0], acc);
    acc = mfma(a[0], b[0], acc);
  } else if constexpr (NA == 2 && NB == 1) {
    acc = mfma(a[1], b[0], acc);
    acc = mfma(a[0], b[0], acc);
  } else {
    static_assert(NA == 1 && NB == 1, "term combination");
    acc = mfma(a[0], b[0], acc);
  }
  return acc;
}

// lane l <- (v of lane l & 31, v of lane 32 + (l & 31)): the two halves of a row
__device__ __forceinline__ void halves(float v, float& lo, float& hi) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  lo = __uint_as_float(r[0]);
  hi = __uint_as_float(r[1]);
}

template <typename T>
struct Tab {  // table storage: fp32 -> 3 terms, bf16 -> exact
  static constexpr int NT = sizeof(T) == 4 ? 3 : 1;  // terms of a table operand
  static constexpr int NA = sizeof(T) == 4 ? 3 : 2;  // terms of an attention operand
  static constexpr uint32_t RB = kD * sizeof(T);     // bytes per table row
};

// LDS staging image of a 32-row x 64-feature tile: rows padded by 16 bytes, so the 8 rows
// a B-fragment read walks (one feature each, ds_read2 pairs 1 row apart) sit on
// different banks
#ifndef BIP3_PAD
#define BIP3_PAD 1
#endif
// The second-dispatched wave of each SIMD (waves 4-7) loses the SIMD's issue arbitration by
// age: on the same tiles its loop runs 7-12 % longer (profiles/round6_bip_timeline), and the
// kernel ends with it.  Measured (bip1m, HIP events, scripts/r6/fold.sh, profiles/
// round6_fold_ab): the backward lets the two waves take turns at priority, a tile each
// (BIP3_PRIO_B 2: bf16 205.0 -> 197.4 us over two A/B pairs); giving the forward's waves 0-3
// 5 % more tiles (BIP3_SKEW_F 50) measured within noise over three runs, so it is off.
// 1: waves 4-7 at s_setprio 1 throughout (measured no better: the roles just swap).
#ifndef BIP3_PRIO
#define BIP3_PRIO 0
#endif
#ifndef BIP3_PRIO_F
#define BIP3_PRIO_F BIP3_PRIO  // forward
#endif
#ifndef BIP3_PRIO_B
#define BIP3_PRIO_B 2  // backward
#endif
#ifndef BIP3_APF
#define BIP3_APF 1  // tiles ahead the per-row inputs (mask, el, lse, flag, rowptr) are loaded
#endif
#ifndef BIP3_SKEW_F
#define BIP3_SKEW_F 0  // forward: per-mille extra tiles of the first-dispatched wave pairs
#endif
#ifndef BIP3_SKEW_B
#define BIP3_SKEW_B 0  // backward: per-mille extra tiles of the first-dispatched waves
#endif
#ifndef BIP3_APF_B
#define BIP3_APF_B BIP3_APF  // the same for the backward
#endif
#ifndef BIP3_HSSYNC
#define BIP3_HSSYNC 1  // fp32 backward: hs pieces loaded in their own tile (0: a tile ahead)
#endif
#ifndef BIP3_CLATE
#define BIP3_CLATE 0  // backward: the softmax backward after d_hc / d_hs (A/B knob)
#endif
#ifndef BIP3_HSLATE
#define BIP3_HSLATE 0  // 1 (hs pieces issued after d_hs) failed the 120k-row d_hs check with the padded staging; not understood, off
#endif
template <typename T>
struct Stg {
  static constexpr int P = kF + (BIP3_PAD ? 16 / (int)sizeof(T) : 0);  // row pitch in elements
  static constexpr int N = 32 * P;                    // elements per image
};

// att^T image [term][row 32][col 32] bf16: the 8-byte block cb (columns 4 cb .. 4 cb + 3)
// of row r sits at block cb ^ ((r >> 1) & 7), so the 32 rows' writes of one block spread
// over 16 bank pairs (unswizzled, 64-byte rows put them on 2) and each transposed read of
// 4 rows x 8 blocks still covers 64 distinct banks
__device__ __forceinline__ int img_off(int q, int r, int cb) {
  return (q * 32 + r) * 32 + 4 * (cb ^ ((r >> 1) & 7));
}

// one 8-row x 1-feature fragment of a streamed table, raw (rows along k)
template <typename T>
struct Chunk {
  uint32_t w[8];
};
template <typename T>
__device__ __forceinline__ void load_chunk(rsrc_t rs, uint32_t voff, uint32_t soff, Chunk<T>& c) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if constexpr (sizeof(T) == 4)
      c.w[j] = __builtin_amdgcn_raw_buffer_load_b32(rs, voff, soff + (uint32_t)j * Tab<T>::RB, 0);
    else
      c.w[j] = __builtin_amdgcn_raw_buffer_load_b16(rs, voff, soff + (uint32_t)j * Tab<T>::RB, 0);
  }
}
template <typename T>
__device__ __forceinline__ void chunk_terms(const Chunk<T>& c, bf16x8 (&b)[Tab<T>::NT]) {
  if constexpr (sizeof(T) == 4) {
    float x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = __uint_as_float(c.w[j]);
    const Terms<3> t = split<3>(x);
#pragma unroll
    for (int q = 0; q < 3; ++q) b[q] = t.t[q];
  } else {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    u32x4 p;
#pragma unroll
    for (int q = 0; q < 4; ++q) p[q] = (c.w[2 * q] & 0xffffu) | (c.w[2 * q + 1] << 16);
    b[0] = __builtin_bit_cast(bf16x8, p);
  }
}

// A 32-row x 64-feature output tile (one head) leaves as 16-byte row pieces: the C
// fragments (lane = feature, 16 rows a lane) go into the wave's LDS staging image
// [row][feature] first (st_frag), then whole rows to HBM (flush_rows) -- a quarter of
// the store instructions of writing the fragments' 4- / 2-byte lanes directly
#ifndef BIP3_UST
#define BIP3_UST 1
#endif
#ifndef BIP3_HST  // hs through the same staging image (needs BIP3_UST's image)
#define BIP3_HST 1
#endif
template <typename T>
__device__ __forceinline__ void st_frag(T* st, const f32x16& acc, int n, int t, int c) {
#pragma unroll
  for (int i = 0; i < 16; ++i) st[((i & 3) + 8 * (i >> 2) + 4 * c) * Stg<T>::P + 32 * n + t] = (T)acc[i];
}
template <typename T>
__device__ __forceinline__ void flush_rows(const T* st, rsrc_t rs, int32_t r0, int h, int lane) {
  constexpr int CPR = kF * (int)sizeof(T) / 16;  // 16-byte pieces per row
  constexpr int NP = 32 * CPR / 64;              // pieces per lane
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    const int q = lane + 64 * k, row = q / CPR, pc = q % CPR;
    const u32x4_t v = *reinterpret_cast<const u32x4_t*>(st + row * Stg<T>::P + pc * (16 / (int)sizeof(T)));
    __builtin_amdgcn_raw_buffer_store_b128(
        v, rs, (uint32_t)row * Tab<T>::RB + (uint32_t)(h * kF) * sizeof(T) + (uint32_t)pc * 16u,
        (uint32_t)r0 * Tab<T>::RB, 0);
  }
}

// ------------------------------------------------------------------------ forward ---
// A block's waves come in pairs over one row range, wave w taking head w & 1 (the heads
// are independent from the scores to the aggregates), so a wave holds one head's 16
// attention values per lane, its v accumulators (32 x 64 = 32 registers) and one head's
// streamed hs fragments.
// LDS: B fragments of hc [h][n][s][term][lane] (16 B each), er, per wave the att^T image
// [term][row 32][col 32] bf16 (64-B rows) and 32 dropout keep words.
template <typename T, bool HS, bool ATTD, bool DROP>
__global__ void __launch_bounds__(kWaves * 64) bip3_fwd_kernel(
    const uint32_t* __restrict__ rowmask, const int32_t* __restrict__ rowptr,
    const uint8_t* __restrict__ rowflag, int32_t n_rows, int32_t M, int32_t n_edges,
    const float* __restrict__ el, const float* __restrict__ er, const T* __restrict__ hc,
    const T* __restrict__ hs, float slope, Dropout dp, T* __restrict__ u,
    float* __restrict__ lse, float* __restrict__ attd, float* __restrict__ part) {
  constexpr int NT = Tab<T>::NT, NA = Tab<T>::NA;
  constexpr uint32_t RB = Tab<T>::RB;
  constexpr int TRW = NA * 32 * 32;  // bf16 per wave image
  constexpr int kPairs = kWaves / 2;
  __shared__ bf16x8 bfr[8 * NT * 64];
  __shared__ float ert[64];
  __shared__ __attribute__((aligned(16))) bf16_t trb[HS ? (kWaves * TRW > 16384 ? kWaves * TRW : 16384) : 8];  // >= the 32 KB reduce
  __shared__ uint64_t kw[DROP ? kWaves : 1][32];
  __shared__ __attribute__((aligned(16))) T ust[BIP3_UST ? kWaves : 1][Stg<T>::N];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = wv & 1;
  const int t = lane & 31, c = lane >> 5;
  // forward marks per tile: start, softmax done, attention images written, u out, v issued
  constexpr int kTlPer = 5;
  B3TL_OPEN(0, (int)sizeof(T) + 16 * HS + 32 * ATTD + 64 * DROP);
  B3TL_MARK(0);

  // B fragments of hc: item (h, n, s) x lane (f, c) holds hc[col(s, 8c + j)][h 64 + 32 n + f]
  for (int it = tid; it < 8 * 64; it += kWaves * 64) {
    const int l = it & 63, hns = it >> 6, s = hns & 1, n = (hns >> 1) & 1, hh = hns >> 2;
    const int f = l & 31, cc = l >> 5;
    float x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int col = col_of(cc, 8 * s + j);
      x[j] = col < M ? to_f32(hc[col * kD + hh * kF + 32 * n + f]) : 0.f;
    }
    const Terms<NT> tt = split<NT>(x);
#pragma unroll
    for (int q = 0; q < NT; ++q) bfr[(hns * NT + q) * 64 + l] = tt.t[q];
  }
  if (tid < 64) ert[tid] = (tid >> 1) < M ? er[tid] : 0.f;  // ert[2 j + h] = er[j][h]
  __syncthreads();
  B3TL_MARK(1);

  const uint64_t doff = DROP ? dropout_offset(dp, dp.offset) : 0;
  const int64_t Pt = (int64_t)gridDim.x * kPairs, pw = (int64_t)blockIdx.x * kPairs + (wv >> 1);
  const int32_t n_tiles = (n_rows + kTile - 1) / kTile;
  int32_t tb = (int32_t)(pw * n_tiles / Pt), te = (int32_t)((pw + 1) * n_tiles / Pt);
  if (BIP3_SKEW_F != 0) {  // the block's tiles, the first-dispatched pairs (waves 0-3) more
    const int32_t b0 = (int32_t)((int64_t)blockIdx.x * n_tiles / gridDim.x);
    const int32_t b1 = (int32_t)((int64_t)(blockIdx.x + 1) * n_tiles / gridDim.x);
    tb = skew_split(b0, b1, wv >> 1, kPairs, BIP3_SKEW_F);
    te = skew_split(b0, b1, (wv >> 1) + 1, kPairs, BIP3_SKEW_F);
  }
  const int32_t rb = tb * kTile, re = min(n_rows, te * kTile);

  f32x16 vacc[2];
#pragma unroll
  for (int n = 0; n < 2; ++n)
#pragma unroll
    for (int i = 0; i < 16; ++i) vacc[n][i] = 0.f;

  if (BIP3_PRIO_F == 1 && wv >= 4) __builtin_amdgcn_s_setprio(1);
  if (rb < re) {
    const rsrc_t r_mask = make_rsrc(rowmask, (uint32_t)re * 4u);
    const rsrc_t r_rp = make_rsrc((ATTD || DROP) ? rowptr : nullptr, (uint32_t)(re + 1) * 4u);
    const rsrc_t r_flag = make_rsrc(rowflag, (uint32_t)re);
    const rsrc_t r_el = make_rsrc(el, (uint32_t)re * 8u);
    const rsrc_t r_lse = make_rsrc(lse, (uint32_t)re * 8u);
    const rsrc_t r_hs = make_rsrc(HS ? hs : nullptr, (uint32_t)re * RB);
    const rsrc_t r_u = make_rsrc(u, (uint32_t)re * RB);
    const rsrc_t r_att = make_rsrc(ATTD ? attd : nullptr, (uint32_t)n_edges * 8u);
    bf16_t* const img = trb + (HS ? wv * TRW : 0);
    // hs fragment (n, s) of lane (f, c): rows 16 s + 8 c + j, feature 64 h + 32 n + f
    auto hs_voff = [&](int k) -> uint32_t {
      const int s = k & 1, n = k >> 1;
      return (uint32_t)(16 * s + 8 * c) * RB + (uint32_t)(h * kF + 32 * n + t) * sizeof(T);
    };
    const uint32_t v_eh = (uint32_t)(2 * t + h) * 4u;  // el / lse of (row t, head h)

    struct In {
      uint32_t mk, fl;
      float elv;
      int32_t rp;
    };
    auto load_a = [&](int32_t r0, In& a) {
      a.mk = __builtin_amdgcn_raw_buffer_load_b32(r_mask, (uint32_t)t * 4u, (uint32_t)r0 * 4u, 0);
      a.elv = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r_el, v_eh, (uint32_t)r0 * 8u, 0));
      a.fl = __builtin_amdgcn_raw_buffer_load_b8(r_flag, (uint32_t)t, (uint32_t)r0, 0);
      a.rp = (ATTD || DROP) ? (int32_t)__builtin_amdgcn_raw_buffer_load_b32(r_rp, (uint32_t)t * 4u,
                                                                           (uint32_t)r0 * 4u, 0)
                            : 0;
    };
#if BIP3_HST
    // hs tiles kPf ahead as 16-byte row pieces (lane l, piece k: 16 bytes of row
    // (l + 64 k) / CPR), written to the wave's staging image at use and read back as
    // B fragments: whole 128-byte lines per load instruction
    constexpr int CPR = kF * (int)sizeof(T) / 16, NPc = 32 * CPR / 64;
    struct Ring {
      u32x4_t p[NPc];
    };
    auto load_ring = [&](int32_t r0, Ring& R) {
#pragma unroll
      for (int k = 0; k < NPc; ++k) {
        const int q = lane + 64 * k, row = q / CPR, pc = q % CPR;
        R.p[k] = __builtin_amdgcn_raw_buffer_load_b128(
            r_hs, (uint32_t)row * RB + (uint32_t)(h * kF) * sizeof(T) + (uint32_t)pc * 16u,
            (uint32_t)r0 * RB, 0);
      }
    };
#else
    // hs fragments as loaded (rows along k, 4 / 2 bytes a lane)
    struct Ring {
      Chunk<T> ch[4];
    };
    auto load_ring = [&](int32_t r0, Ring& R) {
#pragma unroll
      for (int k = 0; k < 4; ++k) load_chunk<T>(r_hs, hs_voff(k), (uint32_t)r0 * RB, R.ch[k]);
    };
#endif
    // kPf tiles ahead: ring A holds the even tiles of the range, B the odd ones (the loop
    // below is unrolled by two so both stay statically indexed)
    Ring ringA, ringB;
    if (HS) {
      load_ring(rb, ringA);
      if (kPf > 1) load_ring(rb + kTile, ringB);
    }
    In nx, nx2;
    load_a(rb, nx);
    if (BIP3_APF > 1) load_a(rb + kTile, nx2);

    auto tile = [&](int32_t r0, Ring& ring) {
      // (a compiler barrier: the loop-invariant LDS reads of er and of hc's fragments stay
      // inside the loop instead of being hoisted into registers for the whole range)
      asm volatile("" ::: "memory");
      const int it = (r0 - rb) / kTile;
      const bool tlm = it < kTlTiles;
      if (tlm) B3TL_MARK(2 + kTlPer * it);
      if (BIP3_PRIO_F == 2) {  // the two waves of a SIMD take turns at priority, a tile each
        if (((it + (wv >= 4 ? 1 : 0)) & 1) != 0)
          __builtin_amdgcn_s_setprio(1);
        else
          __builtin_amdgcn_s_setprio(0);
      }
      const In cu = nx;
      if (BIP3_APF > 1) {
        nx = nx2;
        load_a(r0 + 2 * kTile, nx2);
      } else {
        load_a(r0 + kTile, nx);
      }

      // ---- phase A: softmax of (row t, head h) over the lane's 16 columns
      const bool virt = cu.fl != 0;
      float a[16];
      float mx = -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int j = col_of(c, r);
        float x = cu.elv + ert[2 * j + h];
        x = fmaxf(x, x * slope);
        if (virt) x = 0.f;
        const uint32_t b = bitmask(cu.mk, j);
        x = __uint_as_float((__float_as_uint(x) & b) | (__float_as_uint(-INFINITY) & ~b));
        a[r] = x;
        mx = fmaxf(mx, x);
      }
      {
        float lo, hi;
        halves(mx, lo, hi);
        mx = fmaxf(lo, hi);
      }
      const float m2 = mx == -INFINITY ? 0.f : mx * kLog2e;
      float l = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        a[r] = __builtin_amdgcn_exp2f(fmaf(a[r], kLog2e, -m2));
        l += a[r];
      }
      {
        float lo, hi;
        halves(l, lo, hi);
        l = lo + hi;
      }
      const float inv = l > 0.f ? __builtin_amdgcn_rcpf(l) : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) a[r] *= inv;
      if (c == 0) {
        const float ls = mx == -INFINITY ? -INFINITY : mx + __logf(l);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(ls), r_lse, v_eh, (uint32_t)r0 * 8u, 0);
      }
      if (DROP || ATTD) {
        int32_t E0 = 0;
        if (DROP) {
          // keep bits of the tile's edges for head h: 64 edges per word
          const int tl = min(kTile, re - r0) - 1;
          E0 = __builtin_amdgcn_readlane(cu.rp, 0);
          const int32_t E1 = __builtin_amdgcn_readlane(cu.rp + (int32_t)__popc(cu.mk), tl);
          for (int32_t q = 0; q * 64 < E1 - E0; ++q) {
            const int32_t e = E0 + q * 64 + lane;
            const bool k = e < E1 && philox_x(dp.seed, doff, (uint64_t)e * 2u + (uint64_t)h) >= dp.threshold;
            const uint64_t word = __builtin_amdgcn_ballot_w64(k);
            if (lane == 0) kw[DROP ? wv : 0][q & 15] = word;
          }
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int j = col_of(c, r);
          const bool bit = (cu.mk >> j) & 1u;
          const int32_t rank = (int32_t)__popc(cu.mk & ((1u << j) - 1u));
          if (DROP) {
            const int32_t idx = min(cu.rp - E0 + rank, 32 * 32 - 1);
            const uint64_t wd = kw[DROP ? wv : 0][idx >> 6];
            a[r] *= ((wd >> (idx & 63)) & 1ull) ? dp.scale : 0.f;
          }
          if (ATTD)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(a[r]), r_att,
                                                  bit ? (uint32_t)(cu.rp + rank) * 8u + (uint32_t)h * 4u
                                                      : kOOB,
                                                  0, 0);
        }
      }
      if (tlm) B3TL_MARK(3 + kTlPer * it);

      // ---- att as the A operand (rows on the lanes) and the att^T image
      bf16x8 A[2][NA];  // [s][term]
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        float x[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = a[8 * s + j];
        const Terms<NA> p = split<NA>(x);
#pragma unroll
        for (int q = 0; q < NA; ++q) A[s][q] = p.t[q];
      }
      if (HS) {
        // lane (t, c) writes its columns 4c + 8m .. + 3 of row t: image [term][row][col]
#pragma unroll
        for (int q = 0; q < NA; ++q)
#pragma unroll
          for (int m = 0; m < 4; ++m) {
            const int s = m >> 1, o = 4 * (m & 1);
            bf16x4 v4 = {A[s][q][o], A[s][q][o + 1], A[s][q][o + 2], A[s][q][o + 3]};
            *reinterpret_cast<bf16x4*>(img + img_off(q, t, c + 2 * m)) = v4;
          }
      }
      if (tlm) B3TL_MARK(4 + kTlPer * it);

      // ---- u = att hc: C[row][feature], lane = feature, 16 rows per lane
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        asm volatile("" ::: "memory");
        f32x16 acc;
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] = 0.f;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          bf16x8 B[NT];
#pragma unroll
          for (int q = 0; q < NT; ++q) B[q] = bfr[((((h * 2 + n) * 2 + s) * NT) + q) * 64 + lane];
          acc = prod<NA, NT>(A[s], B, acc);
        }
        if (BIP3_UST) {
          st_frag<T>(ust[BIP3_UST ? wv : 0], acc, n, t, c);
        } else {
          const uint32_t vo = (uint32_t)(h * kF + 32 * n + t) * sizeof(T) + (uint32_t)(4 * c) * RB;
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const uint32_t so = (uint32_t)(r0 + (i & 3) + 8 * (i >> 2)) * RB;
            if constexpr (sizeof(T) == 4)
              __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[i]), r_u, vo, so, 0);
            else
              __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(uint16_t, (bf16_t)acc[i]), r_u,
                                                    vo, so, 0);
          }
        }
      }
      if (BIP3_UST) flush_rows<T>(ust[BIP3_UST ? wv : 0], r_u, r0, h, lane);
      if (tlm) B3TL_MARK(5 + kTlPer * it);

      // ---- v += att^T hs: A = att^T (transposed image reads), B = hs rows along k
      if (HS) {
        const int g = lane >> 4, i16 = lane & 15, qq = i16 >> 2, pp = i16 & 3;
#if BIP3_HST
        T* const hsi = ust[BIP3_UST ? wv : 0];  // (after the u rows left it)
#pragma unroll
        for (int k = 0; k < NPc; ++k) {
          const int q = lane + 64 * k, row = q / CPR, pc = q % CPR;
          *reinterpret_cast<u32x4_t*>(hsi + row * Stg<T>::P + pc * (16 / (int)sizeof(T))) = ring.p[k];
        }
        load_ring(r0 + kPf * kTile, ring);
#endif
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int s = k & 1, n = k >> 1;
          bf16x8 B[NT];
#if BIP3_HST
          if constexpr (sizeof(T) == 4) {
            Chunk<T> chk;
#pragma unroll
            for (int j = 0; j < 8; ++j)
              chk.w[j] = __float_as_uint(hsi[(16 * s + 8 * c + j) * Stg<T>::P + 32 * n + t]);
            chunk_terms<T>(chk, B);
          } else {
            const bf16_t* p = reinterpret_cast<const bf16_t*>(hsi) + (16 * s + 8 * c + qq) * Stg<T>::P +
                              32 * n + 16 * (g & 1) + 4 * pp;
            const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4*)p);
            const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4*)(p + 4 * Stg<T>::P));
            B[0] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          }
#else
          chunk_terms<T>(ring.ch[k], B);
          load_chunk<T>(r_hs, hs_voff(k), (uint32_t)(r0 + kPf * kTile) * RB, ring.ch[k]);
#endif
          bf16x8 At[NA];
#pragma unroll
          for (int q = 0; q < NA; ++q) {
            // block rows 16 s + 8 c + {0..3 | 4..7}, columns 16 (g & 1) + 4 pp; the lane
            // gets column 16 (g & 1) + i16 = lane & 31
            const int rr = 16 * s + 8 * c + qq, cb = 4 * (g & 1) + pp;
            const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4*)(img + img_off(q, rr, cb)));
            const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4*)(img + img_off(q, rr + 4, cb)));
            At[q] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          }
          vacc[n] = prod<NA, NT>(At, B, vacc[n]);
        }
      }
      if (tlm) B3TL_MARK(6 + kTlPer * it);
    };
    if (kPf > 1) {
      for (int32_t r0 = rb; r0 < re; r0 += 2 * kTile) {
        tile(r0, ringA);
        if (r0 + kTile < re) tile(r0 + kTile, ringB);
      }
    } else {
      for (int32_t r0 = rb; r0 < re; r0 += kTile) tile(r0, ringA);
    }
  }
  B3TL_MARK(2 + kTlPer * kTlTiles);
  if (HS) {
    // block sum of the waves' v (fixed order): waves 4-7 park theirs in R[w - 4], waves
    // 0-3 add theirs (same head: w and w + 4), then head h = R[h] + R[h + 2]
    static_assert(kWaves == 8, "the reduce below pairs waves w and w + 4");
    float* red = reinterpret_cast<float*>(trb);  // 4 x 32 x 64 floats
    __syncthreads();
    auto slot = [&](int n, int i) -> int { return ((i & 3) + 8 * (i >> 2) + 4 * c) * kF + 32 * n + t; };
    if (wv >= 4) {
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int i = 0; i < 16; ++i) red[(wv - 4) * 32 * kF + slot(n, i)] = vacc[n][i];
    }
    __syncthreads();
    if (wv < 4) {
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          float* q = red + wv * 32 * kF + slot(n, i);
          *q = vacc[n][i] + *q;
        }
    }
    __syncthreads();
    float* dst = part + (int64_t)blockIdx.x * (M * kD);
    for (int i = tid; i < M * kD; i += kWaves * 64) {
      const int j = i / kD, hh = (i / kF) & 1, f = i % kF;
      dst[i] = red[hh * 32 * kF + j * kF + f] + red[(hh + 2) * 32 * kF + j * kF + f];
    }
  }
  B3TL_MARK(3 + kTlPer * kTlTiles);
}

// ----------------------------------------------------------------------- backward ---
// Per row i, head h (the autograd of Ablation.py:266-274; Ours.py:84-86 adds coef):
//   g_ij = dU_i . hc_j + hs_i . dV_j (+ coef_i exp(attd_ij)),  D_i = sum_j attd_ij g_ij,
//   ds_ij = att_ij (keep_ij g_ij - D_i),  de_ij = ds_ij lrelu'(pre_ij),
//   d_el_i = sum_j de_ij,  d_er_j = sum_i de_ij,  d_hs_i = sum_j attd_ij dV_j,
//   d_hc_j = sum_i attd_ij dU_i.
// A block takes one head (blockIdx.x & 1), its 8 waves their own row ranges.  Per 32-row
// tile:
//   phase A (lane (t, c)): att from lse on the lane's 16 columns, the keep bits;
//   G^T = [hc | dV] [dU | hs]^T on the matrix cores (K = 128): A = the block's LDS image of
//     [hc | dV] fragments (column on the lane), B = the rows' dU / hs pieces with the
//     features along k (16-byte loads, one tile ahead).  The accumulator tile has the row
//     on the lane and the columns col(c, r) in its registers: phase A's layout, so phase C
//     needs no lane movement.  The dU pieces also go to the wave's staging image;
//   phase C (lane (t, c)): D, ds, de, d_el (one permlane32 swap per sum), d_er summed over
//     the tile's rows by a recursive-halving exchange into one register per lane;
//   d_hc += attd^T dU (A = the attd^T image, B = dU with the rows along k, read from the
//     staging image), then d_hs = attd dV (A = attd as it stands, B = dV fragments) leaves
//     through the same staging image as 16-byte row pieces.
template <typename T, bool HS, bool COEF, bool DROP>
__global__ void __launch_bounds__(kWaves * 64) bip3_bwd_kernel(
    const uint32_t* __restrict__ rowmask, const int32_t* __restrict__ rowptr,
    const uint8_t* __restrict__ rowflag, int32_t n_rows, int32_t M,
    const float* __restrict__ el, const float* __restrict__ er, const T* __restrict__ hc,
    const float* __restrict__ lse, const T* __restrict__ dU, const T* __restrict__ hs,
    const T* __restrict__ dV, const float* __restrict__ row_coef, float slope, Dropout dp,
    float* __restrict__ d_el, T* __restrict__ d_hs, float* __restrict__ part) {
  constexpr int NT = Tab<T>::NT, NA = Tab<T>::NA;
  constexpr uint32_t RB = Tab<T>::RB;
  constexpr int TRW = NA * 32 * 32;
  constexpr int KS = HS ? 8 : 4;  // k-steps of G (16 features each: dU, then hs)
  constexpr int SGW = Stg<T>::N * (int)sizeof(T) / 2;  // staging image per wave, in bf16 units
  // the end-of-kernel reduce reuses the per-wave images: 4 x 32 x 64 floats
  constexpr int IMG = kWaves * (TRW + SGW) > 16384 ? kWaves * (TRW + SGW) : 16384;
  __shared__ bf16x8 afr[KS * NT * 64];           // [k-step][term][lane]
  __shared__ bf16x8 bdv[HS ? 4 * NT * 64 : 1];   // [n][s][term][lane]
  __shared__ float ert[64];
  __shared__ __attribute__((aligned(16))) bf16_t trb[IMG];
  __shared__ uint64_t kw[DROP ? kWaves : 1][16];
  __shared__ float sder[kWaves][32];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = blockIdx.x & 1;
  const int t = lane & 31, c = lane >> 5;
  // backward marks per tile: start, phase A done, G issued, phase C done, d_hc issued,
  // d_hs out
  constexpr int kTlPer = 6;
  B3TL_OPEN(1, 128 + (int)sizeof(T) + 16 * HS + 32 * COEF + 64 * DROP);
  B3TL_MARK(0);

  // A fragments of [hc | dV] of head h: k-step x lane (j, c) holds the 8 features
  // 16 k' + 8 c .. + 7 of hc[j] (k' = k-step < 4) or dV[j] (k-step - 4)
  for (int it = tid; it < KS * 64; it += kWaves * 64) {
    const int l = it & 63, ks = it >> 6;
    const int j = l & 31, cc = l >> 5;
    const T* src = ks < 4 ? hc : dV;
    const int f0 = h * kF + 16 * (ks & 3) + 8 * cc;
    float x[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) x[q] = j < M ? to_f32(src[j * kD + f0 + q]) : 0.f;
    const Terms<NT> tt = split<NT>(x);
#pragma unroll
    for (int q = 0; q < NT; ++q) afr[(ks * NT + q) * 64 + l] = tt.t[q];
  }
  if (HS) {  // B fragments of dV for d_hs: as the forward's hc image
    for (int it = tid; it < 4 * 64; it += kWaves * 64) {
      const int l = it & 63, ns = it >> 6, s = ns & 1, n = ns >> 1;
      const int f = l & 31, cc = l >> 5;
      float x[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int col = col_of(cc, 8 * s + j);
        x[j] = col < M ? to_f32(dV[col * kD + h * kF + 32 * n + f]) : 0.f;
      }
      const Terms<NT> tt = split<NT>(x);
#pragma unroll
      for (int q = 0; q < NT; ++q) bdv[(ns * NT + q) * 64 + l] = tt.t[q];
    }
  }
  if (tid < 64) ert[tid] = (tid >> 1) < M ? er[tid] : 0.f;
  __syncthreads();
  B3TL_MARK(1);

  const uint64_t doff = DROP ? dropout_offset(dp, dp.offset) : 0;
  const int64_t Wt = (int64_t)(gridDim.x >> 1) * kWaves, w = (int64_t)(blockIdx.x >> 1) * kWaves + wv;
  const int32_t n_tiles = (n_rows + kTile - 1) / kTile;
  int32_t tb = (int32_t)(w * n_tiles / Wt), te = (int32_t)((w + 1) * n_tiles / Wt);
  if (BIP3_SKEW_B != 0) {  // the block's tiles, the first-dispatched waves 0-3 more
    const int64_t nbh = gridDim.x >> 1, bh = blockIdx.x >> 1;
    const int32_t b0 = (int32_t)(bh * n_tiles / nbh), b1 = (int32_t)((bh + 1) * n_tiles / nbh);
    tb = skew_split(b0, b1, wv, kWaves, BIP3_SKEW_B);
    te = skew_split(b0, b1, wv + 1, kWaves, BIP3_SKEW_B);
  }
  const int32_t rb = tb * kTile, re = min(n_rows, te * kTile);

  f32x16 hacc[2];  // d_hc of head h: [n] C[col][feature]
#pragma unroll
  for (int n = 0; n < 2; ++n)
#pragma unroll
    for (int i = 0; i < 16; ++i) hacc[n][i] = 0.f;
  float derv[16];  // d_er of the lane's columns col(c, r) over its rows
#pragma unroll
  for (int r = 0; r < 16; ++r) derv[r] = 0.f;

  if (BIP3_PRIO_B == 1 && wv >= 4) __builtin_amdgcn_s_setprio(1);
  if (rb < re) {
    const rsrc_t r_mask = make_rsrc(rowmask, (uint32_t)re * 4u);
    const rsrc_t r_rp = make_rsrc(DROP ? rowptr : nullptr, (uint32_t)(re + 1) * 4u);
    const rsrc_t r_flag = make_rsrc(rowflag, (uint32_t)re);
    const rsrc_t r_el = make_rsrc(el, (uint32_t)re * 8u);
    const rsrc_t r_lse = make_rsrc(lse, (uint32_t)re * 8u);
    const rsrc_t r_cf = make_rsrc(COEF ? row_coef : nullptr, (uint32_t)re * 8u);
    const rsrc_t r_del = make_rsrc(d_el, (uint32_t)re * 8u);
    const rsrc_t r_du = make_rsrc(dU, (uint32_t)re * RB);
    const rsrc_t r_hs = make_rsrc(HS ? hs : nullptr, (uint32_t)re * RB);
    const rsrc_t r_dhs = make_rsrc(HS ? d_hs : nullptr, (uint32_t)re * RB);
    bf16_t* const img = trb + wv * TRW;
    T* const stg = reinterpret_cast<T*>(trb + kWaves * TRW + wv * SGW);
    const uint32_t v_eh = (uint32_t)(2 * t + h) * 4u;

    struct In {
      uint32_t mk, fl;
      float elv, lsv, cf;
      int32_t rp;
    };
    auto load_a = [&](int32_t r0, In& a) {
      a.mk = __builtin_amdgcn_raw_buffer_load_b32(r_mask, (uint32_t)t * 4u, (uint32_t)r0 * 4u, 0);
      a.elv = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r_el, v_eh, (uint32_t)r0 * 8u, 0));
      a.lsv = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r_lse, v_eh, (uint32_t)r0 * 8u, 0));
      a.cf = COEF ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r_cf, v_eh, (uint32_t)r0 * 8u, 0))
                  : 0.f;
      a.fl = __builtin_amdgcn_raw_buffer_load_b8(r_flag, (uint32_t)t, (uint32_t)r0, 0);
      a.rp = DROP ? (int32_t)__builtin_amdgcn_raw_buffer_load_b32(r_rp, (uint32_t)t * 4u, (uint32_t)r0 * 4u, 0)
                  : 0;
    };
    // G's B pieces: k-step ks of lane (t, c) = features 16 (ks & 3) + 8 c .. + 7 of head h of
    // row t, from dU (ks < 4) or hs
    constexpr int PW = sizeof(T) == 4 ? 8 : 4;  // dwords per piece
    struct Piece {
      uint32_t w[PW];
    };
    auto load_piece = [&](int ks, int32_t r0, Piece& p) {
      const rsrc_t rs = ks < 4 ? r_du : r_hs;
      const uint32_t vo = (uint32_t)t * RB + (uint32_t)(h * kF + 16 * (ks & 3) + 8 * c) * sizeof(T);
      const u32x4_t a = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, (uint32_t)r0 * RB, 0);
      p.w[0] = a.x; p.w[1] = a.y; p.w[2] = a.z; p.w[3] = a.w;
      if constexpr (PW == 8) {
        const u32x4_t b = __builtin_amdgcn_raw_buffer_load_b128(rs, vo + 16u, (uint32_t)r0 * RB, 0);
        p.w[4] = b.x; p.w[5] = b.y; p.w[6] = b.z; p.w[7] = b.w;
      }
    };
    auto piece_terms = [&](const Piece& p, bf16x8 (&b)[NT]) {
      if constexpr (sizeof(T) == 4) {
        float x[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = __uint_as_float(p.w[j]);
        const Terms<3> tt = split<3>(x);
#pragma unroll
        for (int q = 0; q < 3; ++q) b[q] = tt.t[q];
      } else {
        typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
        u32x4v v4 = {p.w[0], p.w[1], p.w[2], p.w[3]};
        b[0] = __builtin_bit_cast(bf16x8, v4);
      }
    };

    // fp32 with BIP3_HSSYNC: only the dU pieces ride one tile ahead; the hs pieces are
    // loaded at the top of their own tile (32 registers fewer through the d_hc / d_hs peak)
    constexpr int KR = (HS && sizeof(T) == 4 && BIP3_HSSYNC) ? 4 : KS;
    Piece ring[KR];
#pragma unroll
    for (int k = 0; k < KR; ++k) load_piece(k, rb, ring[k]);
    In nx, nx2;
    load_a(rb, nx);
    if (BIP3_APF_B > 1) load_a(rb + kTile, nx2);

    for (int32_t r0 = rb; r0 < re; r0 += kTile) {
      asm volatile("" ::: "memory");
      const int it = (r0 - rb) / kTile;
      const bool tlm = it < kTlTiles;
      if (tlm) B3TL_MARK(2 + kTlPer * it);
      if (BIP3_PRIO_B == 2) {  // the two waves of a SIMD take turns at priority, a tile each
        if (((it + (wv >= 4 ? 1 : 0)) & 1) != 0)
          __builtin_amdgcn_s_setprio(1);
        else
          __builtin_amdgcn_s_setprio(0);
      }
      const In cu = nx;
      if (BIP3_APF_B > 1) {
        nx = nx2;
        load_a(r0 + 2 * kTile, nx2);
      } else {
        load_a(r0 + kTile, nx);
      }
      const bool virt = cu.fl != 0;
      Piece hsp[KS - KR > 0 ? KS - KR : 1];
#pragma unroll
      for (int k = 0; k < KS - KR; ++k) load_piece(KR + k, r0, hsp[k]);

      // ---- phase A: att (pre-dropout) on the mask, the keep bits of the lane's columns
      float a[16];
      uint32_t keep = 0xffffu;
      {
        const float l2 = cu.lsv * kLog2e;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int j = col_of(c, r);
          float x = cu.elv + ert[2 * j + h];
          x = fmaxf(x, x * slope);
          x = virt ? 0.f : x;
          const float e = __builtin_amdgcn_exp2f(fmaf(x, kLog2e, -l2));
          a[r] = __uint_as_float(__float_as_uint(e) & bitmask(cu.mk, j));
        }
      }
      if (DROP) {
        const int tl = min(kTile, re - r0) - 1;
        const int32_t E0 = __builtin_amdgcn_readlane(cu.rp, 0);
        const int32_t E1 = __builtin_amdgcn_readlane(cu.rp + (int32_t)__popc(cu.mk), tl);
        for (int32_t q = 0; q * 64 < E1 - E0; ++q) {
          const int32_t e = E0 + q * 64 + lane;
          const bool k = e < E1 && philox_x(dp.seed, doff, (uint64_t)e * 2u + (uint64_t)h) >= dp.threshold;
          const uint64_t word = __builtin_amdgcn_ballot_w64(k);
          if (lane == 0) kw[DROP ? wv : 0][q & 15] = word;
        }
        keep = 0u;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int j = col_of(c, r);
          const int32_t rank = (int32_t)__popc(cu.mk & ((1u << j) - 1u));
          const int32_t idx = min(cu.rp - E0 + rank, 32 * 32 - 1);
          const uint64_t wd = kw[DROP ? wv : 0][idx >> 6];
          keep |= (uint32_t)((wd >> (idx & 63)) & 1ull) << r;
        }
      }
      auto attd_of = [&](int r) -> float {
        return DROP ? (((keep >> r) & 1u) ? a[r] * dp.scale : 0.f) : a[r];
      };
      if (tlm) B3TL_MARK(3 + kTlPer * it);

      // ---- G^T = [hc | dV] [dU | hs]^T: lane (t, c), register r = g of column col(c, r);
      // the dU pieces stay in the staging image [row][feature] for d_hc
      f32x16 G;
#pragma unroll
      for (int i = 0; i < 16; ++i) G[i] = 0.f;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        if (ks & 1) asm volatile("" ::: "memory");  // two k-steps' fragments at a time
        bf16x8 B[NT], Af[NT];
        const Piece& pc = ks < KR ? ring[ks < KR ? ks : 0] : hsp[ks >= KR ? ks - KR : 0];
        piece_terms(pc, B);
        if (ks < 4) {
          uint32_t* q = reinterpret_cast<uint32_t*>(stg + t * Stg<T>::P + 16 * ks + 8 * c);
          *reinterpret_cast<u32x4_t*>(q) = u32x4_t{pc.w[0], pc.w[1], pc.w[2], pc.w[3]};
          if constexpr (PW == 8)
            *reinterpret_cast<u32x4_t*>(q + 4) = u32x4_t{pc.w[4], pc.w[5], pc.w[6], pc.w[7]};
        }
        // the next tile's dU pieces now; its hs pieces after this tile's d_hs (their
        // registers are free through the d_hc / d_hs peak)
        if (ks < KR && (ks < 4 || !BIP3_HSLATE)) load_piece(ks, r0 + kTile, ring[ks < KR ? ks : 0]);
#pragma unroll
        for (int q = 0; q < NT; ++q) Af[q] = afr[(ks * NT + q) * 64 + lane];
        G = prod<NT, NT>(Af, B, G);
      }
      if (tlm) B3TL_MARK(4 + kTlPer * it);

      // ---- phase C: D, ds, de, d_el, d_er (BIP3_CLATE: after d_hc / d_hs, which need only
      // attd, so G's MFMAs complete under them instead of in front of the softmax backward)
      auto phase_c = [&]() {
      float dsum = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float g = G[r];
        if (COEF) {
          const float cx = cu.cf * __expf(attd_of(r));
          g += __uint_as_float(__float_as_uint(cx) & bitmask(cu.mk, col_of(c, r)));
          G[r] = g;
        }
        dsum = fmaf(attd_of(r), g, dsum);
      }
      {
        float lo, hi;
        halves(dsum, lo, hi);
        dsum = lo + hi;
      }
      float de[16];
      float del = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int j = col_of(c, r);
        const float ds = DROP ? fmaf(attd_of(r), G[r], -a[r] * dsum) : a[r] * (G[r] - dsum);
        const float pre = cu.elv + ert[2 * j + h];
        float d = ds * (pre > 0.f ? 1.f : slope);
        d = __uint_as_float(__float_as_uint(d) & bitmask(cu.mk, j) & (virt ? 0u : ~0u));
        de[r] = d;
        del += d;
      }
      {
        float lo, hi;
        halves(del, lo, hi);
        del = lo + hi;
        if (c == 0)
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(del), r_del, v_eh, (uint32_t)r0 * 8u, 0);
      }
      // d_er: per lane (row t of every tile, the lane's 16 columns), summed over the lanes
      // once at the end
#pragma unroll
      for (int r = 0; r < 16; ++r) derv[r] += de[r];
      };
      if (!BIP3_CLATE) phase_c();
      if (tlm) B3TL_MARK(5 + kTlPer * it);

      // ---- attd: A operand of d_hs, and the attd^T image for d_hc
      bf16x8 A[2][NA];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        float x[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = attd_of(8 * s + j);
        const Terms<NA> p = split<NA>(x);
#pragma unroll
        for (int q = 0; q < NA; ++q) A[s][q] = p.t[q];
      }
#pragma unroll
      for (int q = 0; q < NA; ++q)
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const int s = m >> 1, o = 4 * (m & 1);
          bf16x4 v4 = {A[s][q][o], A[s][q][o + 1], A[s][q][o + 2], A[s][q][o + 3]};
          *reinterpret_cast<bf16x4*>(img + img_off(q, t, c + 2 * m)) = v4;
        }

      // ---- d_hc += attd^T dU; B = dU with the rows along k, from the staging image
      {
        const int g = lane >> 4, i16 = lane & 15, qq = i16 >> 2, pp = i16 & 3;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int s = k & 1, n = k >> 1;
          bf16x8 B[NT];
          if constexpr (sizeof(T) == 4) {
            Chunk<T> chk;
#pragma unroll
            for (int j = 0; j < 8; ++j)
              chk.w[j] = __float_as_uint(stg[(16 * s + 8 * c + j) * Stg<T>::P + 32 * n + t]);
            chunk_terms<T>(chk, B);
          } else {
            const bf16_t* p = reinterpret_cast<const bf16_t*>(stg) + (16 * s + 8 * c + qq) * Stg<T>::P +
                              32 * n + 16 * (g & 1) + 4 * pp;
            const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4*)p);
            const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4*)(p + 4 * Stg<T>::P));
            B[0] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          }
          bf16x8 At[NA];
#pragma unroll
          for (int q = 0; q < NA; ++q) {
            const int rr = 16 * s + 8 * c + qq, cb = 4 * (g & 1) + pp;
            const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4*)(img + img_off(q, rr, cb)));
            const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4*)(img + img_off(q, rr + 4, cb)));
            At[q] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          }
          hacc[n] = prod<NA, NT>(At, B, hacc[n]);
        }
      }
      if (tlm) B3TL_MARK(6 + kTlPer * it);

      // ---- d_hs = attd dV (C[row][feature]), out through the staging image
      if (HS) {
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          asm volatile("" ::: "memory");
          f32x16 acc;
#pragma unroll
          for (int i = 0; i < 16; ++i) acc[i] = 0.f;
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            bf16x8 B[NT];
#pragma unroll
            for (int q = 0; q < NT; ++q) B[q] = bdv[(((n * 2 + s) * NT) + q) * 64 + lane];
            acc = prod<NA, NT>(A[s], B, acc);
          }
          st_frag<T>(stg, acc, n, t, c);
        }
        flush_rows<T>(stg, r_dhs, r0, h, lane);
        if (BIP3_HSLATE && KR == KS) {
#pragma unroll
          for (int ks = 4; ks < KS; ++ks) load_piece(ks, r0 + kTile, ring[ks < KR ? ks : 0]);
        }
      }
      if (BIP3_CLATE) phase_c();
      if (tlm) B3TL_MARK(7 + kTlPer * it);
    }
  }
  B3TL_MARK(2 + kTlPer * kTlTiles);
  // block partial [d_hc (M x 128)][d_er (M x 2)] of head h (the other head's slices 0):
  // waves w and w + 4 first, then R0 + R1 + R2 + R3; d_er over the waves in order
  static_assert(kWaves == 8, "the reduce below pairs waves w and w + 4");
  // d_er over the wave's 32 row lanes of each half: xor-butterfly within the 32-lane
  // halves (every lane ends with the sums; lanes 0 / 32 write their half's 16 columns)
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    float v = derv[r];
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) v += xor_shfl(v, o);
    derv[r] = v;
  }
  if (t == 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) sder[wv][col_of(c, r)] = derv[r];
  }
  float* red = reinterpret_cast<float*>(trb);  // 4 x 32 x 64 floats
  __syncthreads();
  auto slot = [&](int n, int i) -> int { return ((i & 3) + 8 * (i >> 2) + 4 * c) * kF + 32 * n + t; };
  if (wv >= 4) {
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int i = 0; i < 16; ++i) red[(wv - 4) * 32 * kF + slot(n, i)] = hacc[n][i];
  }
  __syncthreads();
  if (wv < 4) {
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float* q = red + wv * 32 * kF + slot(n, i);
        *q = hacc[n][i] + *q;
      }
  }
  __syncthreads();
  const int MD = M * kD, MH = M * 2;
  float* dst = part + (int64_t)blockIdx.x * (((MD + MH) + 3) & ~3);
  for (int i = tid; i < MD; i += kWaves * 64) {
    const int j = i / kD, hh = (i / kF) & 1, f = i % kF;
    const int o = j * kF + f;
    dst[i] = hh != h ? 0.f
                     : ((red[o] + red[32 * kF + o]) + red[2 * 32 * kF + o]) + red[3 * 32 * kF + o];
  }
  for (int i = tid; i < MH; i += kWaves * 64) {
    const int j = i >> 1, hh = i & 1;
    float a = 0.f;
    if (hh == h) {
#pragma unroll
      for (int q = 0; q < kWaves; ++q) a += sder[q][j];
    }
    dst[MD + i] = a;
  }
  B3TL_MARK(3 + kTlPer * kTlTiles);
}

}  // namespace bip3

bool bip3_enabled() {
  static const int env = [] {
    const char* v = getenv("MSHA_BIP3");
    return v != nullptr && *v ? atoi(v) : 1;
  }();
  return env != 0;
}

// 1 = launched (forward + the v reduce); the caller checked bip2_ok (2 x 64, M <= 32,
// row masks)
int bip3_fwd(const msha_graph* g, int dtype, const float* el, const float* er, const void* hc,
             const void* hs, float slope, const Dropout& dp, void* u, float* lse, float* attd,
             void* v, float* part, int nb, hipStream_t s) {
  if (!bip3_enabled()) return 0;
  const int32_t n_tiles = (int32_t)((g->n_rows + bip3::kTile - 1) / bip3::kTile);
  // no more blocks than tiles' worth of waves (small graphs: every wave at least one tile)
  const int nbk = (int)std::max<int64_t>(1, std::min<int64_t>(nb, (n_tiles + 3) / 4));  // 4 wave pairs a block
  const dim3 grid(nbk), block(bip3::kWaves * 64);
  auto go = [&](auto kern, auto tag) {
    using T = decltype(tag);
    hipLaunchKernelGGL(kern, grid, block, 0, s, g->rowmask, g->rowptr, g->rowflag,
                       (int32_t)g->n_rows, (int32_t)g->n_cols, (int32_t)g->n_edges, el, er,
                       (const T*)hc, (const T*)hs, slope, dp, (T*)u, lse, attd, part);
  };
  const bool bf = dtype == MSHA_DTYPE_BF16;
  const bool H = hs != nullptr, A = attd != nullptr, D = dp.active;
#define GO(T_, H_, A_, D_) go(bip3::bip3_fwd_kernel<T_, H_, A_, D_>, T_{})
#define GO8(T_)                                 \
  if (H && A && D) GO(T_, true, true, true);    \
  else if (H && A) GO(T_, true, true, false);   \
  else if (H && D) GO(T_, true, false, true);   \
  else if (H) GO(T_, true, false, false);       \
  else if (A && D) GO(T_, false, true, true);   \
  else if (A) GO(T_, false, true, false);       \
  else if (D) GO(T_, false, false, true);       \
  else GO(T_, false, false, false);
  if (bf) { GO8(bf16_t) } else { GO8(float) }
#undef GO8
#undef GO
  if (H) {
    const int32_t MD = (int32_t)(g->n_cols * bip3::kD);
    bip_reduce(part, nbk, MD, MD, MD, v, bf, nullptr, 1, s);
  }
  return 1;
}

// 1 = launched (backward + the d_hc / d_er reduce)
int bip3_bwd(const msha_graph* g, int dtype, const float* el, const float* er, const void* hc,
             const float* lse, const void* dU, const void* hs, const void* dV,
             const float* row_coef, float slope, const Dropout& dp, float* d_el, float* d_er,
             void* d_hc, void* d_hs, float* part, int nb, hipStream_t s) {
  if (!bip3_enabled()) return 0;
  // fp32: with the hs pieces loaded in their own tile (BIP3_HSSYNC) the loop no longer
  // spills and this kernel beats the mask backward of edge_bip2.hip at bip1m (370-377 vs
  // 393-400 us, profiles/round6_bwd32_ab; the spilled form's scratch reloads waited for every
  // outstanding load).  Its dropout variants still spill (the keep words): with dropout the
  // mask kernel runs.  MSHA_BIP3_BWD32 (read per call): 1 forces this kernel, 0 the mask one.
  if (dtype != MSHA_DTYPE_BF16) {
    const char* v = getenv("MSHA_BIP3_BWD32");
    const int force = v != nullptr && *v ? atoi(v) : -1;
    if (force == 0 || (force < 0 && dp.active)) return 0;
  }
  const int32_t n_tiles = (int32_t)((g->n_rows + bip3::kTile - 1) / bip3::kTile);
  // blocks in head pairs (blockIdx.x & 1 = head), each wave at least one tile
  const int64_t pairs = std::max<int64_t>(1, std::min<int64_t>(nb / 2, (n_tiles + bip3::kWaves - 1) / bip3::kWaves));
  const int nbk = (int)(2 * pairs);
  const dim3 grid(nbk), block(bip3::kWaves * 64);
  auto go = [&](auto kern, auto tag) {
    using T = decltype(tag);
    hipLaunchKernelGGL(kern, grid, block, 0, s, g->rowmask, g->rowptr, g->rowflag,
                       (int32_t)g->n_rows, (int32_t)g->n_cols, el, er, (const T*)hc, lse,
                       (const T*)dU, (const T*)hs, (const T*)dV, row_coef, slope, dp, d_el,
                       (T*)d_hs, part);
  };
  const bool bf = dtype == MSHA_DTYPE_BF16;
  const bool H = dV != nullptr, C = row_coef != nullptr, D = dp.active;
#define GO(T_, H_, C_, D_) go(bip3::bip3_bwd_kernel<T_, H_, C_, D_>, T_{})
#define GO8(T_)                                 \
  if (H && C && D) GO(T_, true, true, true);    \
  else if (H && C) GO(T_, true, true, false);   \
  else if (H && D) GO(T_, true, false, true);   \
  else if (H) GO(T_, true, false, false);       \
  else if (C && D) GO(T_, false, true, true);   \
  else if (C) GO(T_, false, true, false);       \
  else if (D) GO(T_, false, false, true);       \
  else GO(T_, false, false, false);
  if (bf) { GO8(bf16_t) } else { GO8(float) }
#undef GO8
#undef GO
  const int32_t MD = (int32_t)(g->n_cols * bip3::kD), MH = (int32_t)(g->n_cols * 2);
  bip_reduce(part, nbk, (MD + MH + 3) & ~3, MD + MH, MD, d_hc, bf, d_er, MH, s);
  return 1;
}

}  // namespace msha

// Diagnostic: install (buf != NULL: slots x 64 uint64 words, device memory; the forward's
// waves take slots [0, slots / 2), the backward's the rest) or remove the per-wave timeline
// of the MFMA bipartite kernels; MSHA_ERR_UNSUPPORTED unless the library was built with
// -DSK_TIMELINE (build.py --variant timeline).
extern "C" int msha_debug_bip_timeline(void* buf, int64_t slots) {
#ifdef SK_TIMELINE
  uint64_t* p = (uint64_t*)buf;
  const int64_t n = buf != nullptr ? slots : 0;
  if (hipMemcpyToSymbol(HIP_SYMBOL(msha::bip3::g_tl), &p, sizeof(p)) != hipSuccess ||
      hipMemcpyToSymbol(HIP_SYMBOL(msha::bip3::g_tl_slots), &n, sizeof(n)) != hipSuccess)
    return msha::fail(MSHA_ERR_HIP, "debug_bip_timeline: hipMemcpyToSymbol failed");
  return MSHA_OK;
#else
  (void)buf;
  (void)slots;
  return msha::fail(MSHA_ERR_UNSUPPORTED, "debug_bip_timeline: library built without SK_TIMELINE");
#endif
}
