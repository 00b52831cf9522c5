// Bipartite small-M edge attention (edge_bip.hip): the repo's own adjacency shape.
//
// Every graph the reference trains on is sources x recipients with M = 32 recipient
// columns (Adjacent/Flow 2015-2018: 39-50k rows of ~2.3 edges; the bip1m stress graph:
// 1M rows).  There the whole column side -- hc (M, H, F), er (M, H), dV -- is 16 KB per
// table, so it lives in LDS for the kernel's lifetime, and the column reductions
//   v_j    = sum_i attd_ij hs_i               (Ablation.py:273, forward)
//   d_hc_j = sum_i attd_ij dU_i,  d_er_j = sum_i de_ij          (its autograd)
// go into per-wave LDS slabs instead of a second CSC pass over the (N, H, F) tables:
// each row's hs_i / dU_i is read from HBM exactly once, next to the row's own work.
// Slabs are summed in wave order per block and the block partials in block order by
// bip_reduce_kernel: deterministic, no atomics.
//
// Layout: a wave walks a contiguous row range in groups of kPD = 8 rows.  Per group one
// buffer load each brings rowptr, the group's <= 256 columns, el / lse / coef and the
// rows' slices of the streamed tables; every global load and store of the loop is an
// unconditional buffer op (masked lanes at kOOB), so the next group's loads are in
// flight while this group runs and the compiler's vmcnt waits stay exact.  A group is cut
// into sub-groups of whole rows whose edges fill <= W = 64 / H slots per head.
//   slot lanes (head-major: lane h W + k = edge k, head h) compute the scores and the row
//     softmax with VALU-only segmented scans (DPP row_shr / row_bcast) and write one
//     record {attd, byte offset of hc_j} per slot to LDS;
//   element lanes (lane l owns elements [l V, l V + V) of the H * F row, V = H F / 64)
//     walk each row's edges: one record read, hc_j from LDS, u_i += attd hc_j in
//     registers, and the column sums v_j += attd hs_i (forward) / d_hc_j += attd dU_i
//     (backward) into the wave's slab, two edges of a row a step (distinct columns: both
//     read before either is written).  Sums land in program order: deterministic.
//     (LDS float atomics for the slab measured 5x slower: 1590 vs ~330 us at bip1m.)
//     d_er_j is one LDS float add per slot.
// Reference: Ablation.py:266-274 (OursLayer3 scores, masked softmax, dropout,
// u = att @ h1, v = att.T @ h2), Ours.py:84-86 (the backward's row coefficients).
#include <atomic>

#include "bip_reduce.h"
#include "edge_geo.h"

namespace msha {
namespace bip {

constexpr int kMaxMD = 4096;  // floats of one (M, H*F) LDS table: M = 32 at H*F = 128
constexpr int kWavesF = 8;    // fwd: 16 KB table + 8 x (16 KB v slab + 1.1 KB) = 153 KB
constexpr int kWavesB = 7;    // bwd: two 16 KB tables + 7 x (d_hc slab + 1.6 KB) = 153 KB
// (MSHA_BIP_SPLIT=1, F = 64 with several heads: head-split, one head per block (grid.y),
// every table 1/H as large, so twice the waves per CU -- see fwd_waves / bwd_waves)

__device__ __forceinline__ int32_t rdlane(int32_t v, int l) {
  return __builtin_amdgcn_readlane(v, l);
}

// V consecutive elements of a table row <-> fp32 registers
template <int V>
__device__ __forceinline__ void ld_row(const float* p, float (&x)[V]) {
  if constexpr (V == 4) {
    const float4 a = *reinterpret_cast<const float4*>(p);
    x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
  } else if constexpr (V == 2) {
    const float2 a = *reinterpret_cast<const float2*>(p);
    x[0] = a.x; x[1] = a.y;
  } else {
    x[0] = *p;
  }
}
template <int V>
__device__ __forceinline__ void ld_row(const bf16_t* p, float (&x)[V]) {
  if constexpr (V == 4) {
    const uint2 a = *reinterpret_cast<const uint2*>(p);
    x[0] = __uint_as_float(a.x << 16); x[1] = __uint_as_float(a.x & 0xffff0000u);
    x[2] = __uint_as_float(a.y << 16); x[3] = __uint_as_float(a.y & 0xffff0000u);
  } else if constexpr (V == 2) {
    const uint32_t a = *reinterpret_cast<const uint32_t*>(p);
    x[0] = __uint_as_float(a << 16); x[1] = __uint_as_float(a & 0xffff0000u);
  } else {
    x[0] = (float)*p;
  }
}
template <int V>
__device__ __forceinline__ void st_row(float* p, const float (&x)[V]) {
  if constexpr (V == 4) *reinterpret_cast<float4*>(p) = make_float4(x[0], x[1], x[2], x[3]);
  else if constexpr (V == 2) *reinterpret_cast<float2*>(p) = make_float2(x[0], x[1]);
  else *p = x[0];
}
template <int V>
__device__ __forceinline__ void st_row(bf16_t* p, const float (&x)[V]) {
  if constexpr (V == 4)
    *reinterpret_cast<uint2*>(p) = make_uint2(pack_bf16x2(x[0], x[1]), pack_bf16x2(x[2], x[3]));
  else if constexpr (V == 2) *reinterpret_cast<uint32_t*>(p) = pack_bf16x2(x[0], x[1]);
  else *p = (bf16_t)x[0];
}
template <int V>
__device__ __forceinline__ void st_residual(bf16_t* p, const float (&x)[V]) {
  float r[V];
#pragma unroll
  for (int v = 0; v < V; ++v) r[v] = x[v] - (float)(bf16_t)x[v];
  st_row<V>(p, r);
}
template <int V>
__device__ __forceinline__ void st_residual(float*, const float (&)[V]) {}

typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));

// V elements of a T table row through a buffer descriptor (masked lanes: offset kOOB,
// read 0 / store dropped), so every load and store of the row loop is unconditional and
// the compiler's vmcnt waits stay exact across iterations
// (soff: a wave-uniform byte offset in the instruction's SGPR field -- no VALU per row)
template <typename T, int V>
__device__ __forceinline__ void bld_row(rsrc_t r, uint32_t off, float (&x)[V], uint32_t soff = 0) {
  constexpr int B = V * (int)sizeof(T);
  uint32_t w[4] = {0, 0, 0, 0};
  if constexpr (B == 16) {
    const u32x4_t a = __builtin_amdgcn_raw_buffer_load_b128(r, off, soff, 0);
    w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
  } else if constexpr (B == 8) {
    const u32x2_t a = __builtin_amdgcn_raw_buffer_load_b64(r, off, soff, 0);
    w[0] = a.x; w[1] = a.y;
  } else if constexpr (B == 4) {
    w[0] = __builtin_amdgcn_raw_buffer_load_b32(r, off, soff, 0);
  } else {
    w[0] = __builtin_amdgcn_raw_buffer_load_b16(r, off, soff, 0);
  }
#pragma unroll
  for (int v = 0; v < V; ++v) {
    if constexpr (sizeof(T) == 4) x[v] = __uint_as_float(w[v]);
    else x[v] = __uint_as_float(v % 2 == 0 ? w[v / 2] << 16 : w[v / 2] & 0xffff0000u);
  }
}
template <typename T, int V>
__device__ __forceinline__ void bst_row(rsrc_t r, uint32_t off, const float (&x)[V],
                                        uint32_t soff = 0) {
  constexpr int B = V * (int)sizeof(T);
  uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
  for (int v = 0; v < V; ++v) {
    if constexpr (sizeof(T) == 4) w[v] = __float_as_uint(x[v]);
  }
  if constexpr (sizeof(T) == 2) {
#pragma unroll
    for (int v = 0; v + 1 < V; v += 2) w[v / 2] = pack_bf16x2(x[v], x[v + 1]);
    if constexpr (V == 1) w[0] = (uint32_t)__builtin_bit_cast(uint16_t, (bf16_t)x[0]);
  }
  if constexpr (B == 16) {
    u32x4_t a;
    a.x = w[0]; a.y = w[1]; a.z = w[2]; a.w = w[3];
    __builtin_amdgcn_raw_buffer_store_b128(a, r, off, soff, 0);
  } else if constexpr (B == 8) {
    u32x2_t a;
    a.x = w[0]; a.y = w[1];
    __builtin_amdgcn_raw_buffer_store_b64(a, r, off, soff, 0);
  } else if constexpr (B == 4) {
    __builtin_amdgcn_raw_buffer_store_b32(w[0], r, off, soff, 0);
  } else {
    __builtin_amdgcn_raw_buffer_store_b16((uint16_t)w[0], r, off, soff, 0);
  }
}

// floats per block partial (16-byte aligned rows: the blocks store float4 pieces)
__host__ __device__ constexpr int32_t part_stride(int32_t n) { return (n + 3) & ~3; }

constexpr int kColPages = 4;  // a group's columns held in registers: 256 edges
constexpr int kNCol = 64 * kColPages;
constexpr int kRec = 72;      // slot records per wave: 64 slots + the pair loop's overrun

// Rows per group: every row's head scalars fit one lane each (PD * H <= 64), and the
// streamed rows of one group (~8 KB over the streamed tables, 8..32 rows) are the bytes a
// wave keeps in flight while it works on the previous group; larger groups also spread
// the group's fixed instructions over more rows.  (8-row groups ran bf16 no faster than
// fp32: rows, not bytes, were in flight.)
#ifndef BIP_GRP_BYTES
#define BIP_GRP_BYTES 8192
#endif
template <int H, int D, typename T, int NT>
constexpr int grp_rows() {
  constexpr int rb = D * (int)sizeof(T) * (NT > 1 ? NT : 1);  // streamed bytes per row
  constexpr int gb = BIP_GRP_BYTES;
  constexpr int want = gb / rb < 8 ? 8 : (gb / rb > 32 ? 32 : gb / rb);
  return want < 64 / H ? want : 64 / H;
}

// a lane's V elements of a table row as loaded (RW 32-bit words; bf16 pairs stay packed
// until their use: half the registers of a prefetched group)
template <int V, typename T>
constexpr int row_words() {
  return V * (int)sizeof(T) / 4 > 0 ? V * (int)sizeof(T) / 4 : 1;
}
template <typename T, int V, int RW>
__device__ __forceinline__ void raw_load(rsrc_t r, uint32_t off, uint32_t soff, uint32_t (&w)[RW]) {
  constexpr int B = V * (int)sizeof(T);
  if constexpr (B == 16) {
    const u32x4_t a = __builtin_amdgcn_raw_buffer_load_b128(r, off, soff, 0);
    w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
  } else if constexpr (B == 8) {
    const u32x2_t a = __builtin_amdgcn_raw_buffer_load_b64(r, off, soff, 0);
    w[0] = a.x; w[1] = a.y;
  } else if constexpr (B == 4) {
    w[0] = __builtin_amdgcn_raw_buffer_load_b32(r, off, soff, 0);
  } else {
    w[0] = __builtin_amdgcn_raw_buffer_load_b16(r, off, soff, 0);
  }
}
template <typename T, int V, int RW>
__device__ __forceinline__ void raw_unpack(const uint32_t (&w)[RW], float (&x)[V]) {
#pragma unroll
  for (int v = 0; v < V; ++v) {
    if constexpr (sizeof(T) == 4) x[v] = __uint_as_float(w[v]);
    else x[v] = __uint_as_float(v % 2 == 0 ? w[v / 2] << 16 : w[v / 2] & 0xffff0000u);
  }
}

// A group: rows [r0, r0 + PD) of the wave's range.  rp lane t (t <= PD) = rowptr[min(r0 +
// t, re)]; colv[p] lane q = column of edge E0 + 64 p + q; s[k] lane t * H + h = row scalar
// k (el / lse / coef) of (row t, head h); flag lane t = rowflag; rows[.][t] = this lane's
// V elements of row r0 + t of the streamed tables (hs, or dU and hs).  Rows past the
// wave's range read 0 (the descriptors end there).
template <int RW, int NT, int NS, int PD>
struct Grp {
  int32_t rp;
  int32_t colv[kColPages];
  float s[NS];
  uint32_t flag;
  uint32_t rows[NT > 0 ? NT : 1][PD][RW];
};

// Per-wave buffer descriptors, bounded at the wave's last row: a row, scalar or flag past
// the range reads 0 and a store there is dropped, with no per-load mask arithmetic; the
// group's row offsets go in the instructions' SGPR offset field.
struct Srcs {
  rsrc_t rp, col, flag, sc[3], t[2];
  uint32_t v_rp, v_col, v_s, v_flag, v_row;  // loop-invariant lane offsets (kOOB = unused lane)
  int32_t re, rp_re;
};

template <int H, int V, int NT, int NS, int PD, typename T, int RW, int HT = H>
__device__ __forceinline__ void load_grp(Grp<RW, NT, NS, PD>& g, const Srcs& S, int32_t r0,
                                         int32_t rp, int lane) {
  // bytes per table row (HT > H: this launch's heads are a slice of HT-head rows)
  constexpr uint32_t RB = 64u * V * (uint32_t)sizeof(T) * HT / H;
  g.rp = rp;
  const int32_t E0 = rdlane(rp, 0);
#pragma unroll
  for (int p = 0; p < kColPages; ++p)
    g.colv[p] = (int32_t)__builtin_amdgcn_raw_buffer_load_b32(S.col, S.v_col + 256u * p,
                                                              (uint32_t)E0 * 4u, 0);
#pragma unroll
  for (int k = 0; k < NS; ++k)
    g.s[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(S.sc[k], S.v_s,
                                                                 (uint32_t)r0 * (4u * HT), 0));
  g.flag = __builtin_amdgcn_raw_buffer_load_b8(S.flag, S.v_flag, (uint32_t)r0, 0);
#pragma unroll
  for (int t = 0; t < PD; ++t) {
    const uint32_t so = (uint32_t)(r0 + t) * RB;
    if (NT > 0) raw_load<T, V, RW>(S.t[0], S.v_row, so, g.rows[0][t]);
    if (NT > 1) raw_load<T, V, RW>(S.t[1], S.v_row, so, g.rows[NT > 1 ? 1 : 0][t]);
  }
}

// rowptr[min(r0 + lane, re)] for lanes <= PD
__device__ __forceinline__ int32_t load_rp(const Srcs& S, int32_t r0, int lane) {
  const int32_t v = (int32_t)__builtin_amdgcn_raw_buffer_load_b32(S.rp, S.v_rp, (uint32_t)r0 * 4u, 0);
  return r0 + lane <= S.re ? v : S.rp_re;
}

__device__ __forceinline__ void make_srcs(Srcs& S, const int32_t* rowptr, const int32_t* col,
                                          const uint8_t* rowflag, int32_t n_edges, int32_t re,
                                          int H, int PD, uint32_t row_bytes, int lane,
                                          int HT = 0, int h0 = 0, uint32_t head_bytes = 0) {
  if (HT == 0) HT = H;
  S.re = re;
  S.rp_re = rowptr[re];
  S.rp = make_rsrc(rowptr, (uint32_t)(re + 1) * 4u);
  S.col = make_rsrc(col, (uint32_t)n_edges * 4u);
  S.flag = make_rsrc(rowflag, (uint32_t)re);
  S.v_rp = (uint32_t)lane * 4u;
  S.v_col = (uint32_t)lane * 4u;
  // row scalar (row t, head h) of lane t H + h at element t HT + h0 + h of an HT-head table
  S.v_s = lane < PD * H ? (uint32_t)((lane / H) * HT + h0 + lane % H) * 4u : kOOB;
  S.v_flag = lane < PD ? (uint32_t)lane : kOOB;
  S.v_row = (uint32_t)lane * row_bytes / 64u + (uint32_t)h0 * head_bytes;
}

// all-reduce over the lanes of one head (lane % H): rotations inside 16-lane rows by
// 8, 4, .. H (DPP row_ror keeps lane % H when H divides the shift), then across rows by
// v_permlane16/32_swap -- VALU only, no LDS round trip
template <int N>
__device__ __forceinline__ float ror16(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x120 + N,
                                                             0xF, 0xF, false));
}
__device__ __forceinline__ float swap16(float v, int lane) {
  const unsigned x = __builtin_bit_cast(unsigned, v);
  const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
  return __builtin_bit_cast(float, (lane & 16) ? r[0] : r[1]);
}
// sum over an aligned group of G lanes: 32 = two 16-lane rows (rotations, then the row
// swap), else the xor tree
template <int G>
__device__ __forceinline__ float lanes_sum(float v, int lane) {
  if constexpr (G == 32 || G == 16) {
    v += ror16<8>(v);
    v += ror16<4>(v);
    v += ror16<2>(v);
    v += ror16<1>(v);
    if (G == 32) v += swap16(v, lane);
    return v;
  } else {
    return group_sum<G>(v);
  }
}

// two dot products per head at once (QH = 32: a head is two 16-lane rows): the rows swap
// so lanes with bit 4 clear collect p0 and the others p1, then one rotation tree per row.
// Lanes (l & 16) == 0 of each head end up with sum(p0), the others with sum(p1).
__device__ __forceinline__ float pair_sum32(float p0, float p1, int lane) {
  const bool hi = (lane & 16) != 0;
  float v = hi ? p1 : p0;
  v += swap16(hi ? p0 : p1, lane);
  v += ror16<8>(v);
  v += ror16<4>(v);
  v += ror16<2>(v);
  v += ror16<1>(v);
  return v;
}

// Slot layout: head-major, W = 64 / H lanes per head; lane h * W + k holds (edge Es + k,
// head h) of a sub-group (<= W edges, whole rows).  A row's slots are a contiguous lane
// segment of its head block, [lane - d, end].
//
// Segmented inclusive scan over that segment, VALU only: DPP row_shr 1/2/4/8 inside
// 16-lane rows, then row_bcast15 (rows 1, 3 take lane 15 / 47) and row_bcast31 (rows 2,
// 3 take lane 31) for the head blocks that span rows -- a source lane contributes only
// when it lies in the lane's own segment (d reaches back to it).
// v of the DPP source lane (CTRL), `old` where the row is masked off (RM) or the source
// lies outside the 16-lane row
template <int CTRL, int RM>
__device__ __forceinline__ float dpp_src(float x, float old) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old),
                                                               __builtin_bit_cast(int, x), CTRL,
                                                               RM, 0xF, false));
}

template <int W, bool MAX>
__device__ __forceinline__ float seg_scan(float v, int lane, int d) {
  const int lr = lane & 15;
  constexpr float idn = MAX ? -INFINITY : 0.f;
  // (max as a select: fmaxf's NaN rules would add two canonicalising moves per step)
  auto op = [](float a, float b) { return MAX ? (a > b ? a : b) : a + b; };
  {
    const float y = dpp_src<0x111, 0xF>(v, idn);
    v = (d >= 1 && lr >= 1) ? op(v, y) : v;
  }
  if constexpr (W > 2) {
    const float y = dpp_src<0x112, 0xF>(v, idn);
    v = (d >= 2 && lr >= 2) ? op(v, y) : v;
  }
  if constexpr (W > 4) {
    const float y = dpp_src<0x114, 0xF>(v, idn);
    v = (d >= 4 && lr >= 4) ? op(v, y) : v;
  }
  if constexpr (W > 8) {
    const float y = dpp_src<0x118, 0xF>(v, idn);
    v = (d >= 8 && lr >= 8) ? op(v, y) : v;
  }
  if constexpr (W >= 32) {
    const float y = dpp_src<0x142, 0xA>(v, idn);
    v = ((lane & 16) && d > lr) ? op(v, y) : v;
  }
  if constexpr (W == 64) {
    const float y = dpp_src<0x143, 0xC>(v, idn);
    v = (lane >= 32 && d > lane - 32) ? op(v, y) : v;
  }
  return v;
}

// keep factor of element e * H + h of the edge-dropout stream (the other edge kernels'
// element order)
__device__ __forceinline__ float slot_keep(const Dropout& dp, uint64_t doff, int64_t elem) {
  if (!dp.active) return 1.f;
  return philox_x(dp.seed, doff, (uint64_t)elem) >= dp.threshold ? dp.scale : 0.f;
}

// the sub-group after t0: rows while their edges fit W slots
template <int W, int PD>
__device__ __forceinline__ int sub_end(int32_t rp, int t0, int lane) {
  const int32_t Es = rdlane(rp, t0);
  const uint64_t fit = __ballot(lane > t0 && lane <= PD && rp - Es <= W);
  return t0 + max(1, (int)__popcll(fit));
}

// Per-slot geometry of a sub-group: its row t (in the group), d = slots back to the
// row's first, the lane holding the row's last slot, the column j.
struct Slot {
  int t, d, endl, j;
  bool valid;
};

// t by binary search over the sub-group's rows [t0, t1) in the rp register (one
// ds_bpermute per halving); colb holds the columns from edge cbase on
template <int H, int PD>
__device__ __forceinline__ Slot slot_geo(int32_t rp, int t0, int t1, int32_t Es, int nEs,
                                         int32_t cbase, const uint8_t* colb, int lane, int M) {
  constexpr int W = 64 / H;
  Slot s;
  const int h = lane / W, k = lane % W;
  const int32_t x = Es + k;
  int t = t0;
#pragma unroll
  for (int st = PD / 2; st >= 1; st >>= 1) {
    const int pr = t + st;
    const int32_t v = __shfl(rp, min(pr, PD));
    t = (pr < t1 && v <= x) ? pr : t;
  }
  s.t = t;
  s.valid = k < nEs;
  const int32_t rs = __shfl(rp, t), re = __shfl(rp, t + 1);
  s.d = x - rs;
  s.endl = h * W + (re - Es) - 1;
  s.j = min((int)colb[(x - cbase) & (kNCol - 1)], M - 1);
  return s;
}

// a sub-group whose edges run past the group's column pages (more than kNCol edges in
// the group): its own page, loaded now
__device__ __forceinline__ int32_t colb_refill(const Srcs& S, uint8_t* colb, int32_t Es,
                                               int lane) {
  colb[lane] = (uint8_t)__builtin_amdgcn_raw_buffer_load_b32(S.col, S.v_col, (uint32_t)Es * 4u, 0);
  return Es;
}

// ------------------------------------------------------------------------ forward ---
// u_i = sum_e attd_e hc_j, lse_i, (ATTD: attd_e), and with HS the block partials of
// v_j = sum_e attd_e hs_i.  attd_e = softmax_row(lrelu(el_i + er_j))_e * keep_e.
// Per sub-group: slot lanes compute scores, the row softmax (segmented max / sum scans)
// and keep bits once, and leave one record {attd, byte offset of hc_j} per slot in LDS.
// Element lanes then walk each row's edges two at a time: the records, hc_j from LDS,
// u += attd hc_j in registers, v_j += attd hs_i into the wave's slab.  The next group's
// loads are in flight meanwhile.
// HT > H: the head-split form -- blockIdx.y picks heads [h0, h0 + H) of HT-head tables
// (strided rows, scalars and attention), so a block holds one head's column table and
// slabs (half the LDS of both heads at HT = 2) and twice the waves fit a CU.
constexpr int kWavesF2 = 16;
template <int H, int HT>
constexpr int fwd_waves() { return HT > H ? kWavesF2 : kWavesF; }
template <int H, int F, typename T, bool HS, bool ATTD, int HT = H>
__global__ void __launch_bounds__((fwd_waves<H, HT>() * 64)) bip_fwd_kernel(
    const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
    const uint8_t* __restrict__ rowflag, int32_t n_rows, int32_t n_cols, int32_t n_edges,
    const float* __restrict__ el, const float* __restrict__ er, const T* __restrict__ hc,
    const T* __restrict__ hs, float slope, Dropout dp, T* __restrict__ u,
    T* __restrict__ u_lo, float* __restrict__ lse, float* __restrict__ attd,
    float* __restrict__ part) {
  constexpr int D = H * F, V = D / 64, WB = fwd_waves<H, HT>(), W = 64 / H;
  constexpr int DT = HT * F;  // floats per table row
  constexpr int MDX = kMaxMD * H / HT;
  constexpr int NT = HS ? 1 : 0;
  constexpr int PD = grp_rows<H, D, T, NT>(), RW = row_words<V, T>();
  constexpr uint32_t RB = (uint32_t)DT * sizeof(T);  // row stride in bytes
  const int h0 = HT > H ? (int)blockIdx.y * H : 0;
  __shared__ __attribute__((aligned(16))) float tab[MDX];
  __shared__ float ert[64];
  __shared__ __attribute__((aligned(16))) float slab[HS ? WB : 1][HS ? MDX : 4];
  __shared__ __attribute__((aligned(16))) float2 rec[WB][kRec];
  __shared__ uint8_t colb[WB][kNCol];
  __shared__ float lses[WB][64];
  const int M = n_cols, MD = M * D;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  for (int i = tid * 4; i < MD; i += WB * 256) {  // this launch's heads of hc (D of DT)
    float x[4];
    ld_row<4>(hc + (i / D) * DT + h0 * F + i % D, x);
    st_row<4>(tab + i, x);
  }
  for (int i = tid; i < M * H; i += WB * 64) ert[i] = er[(i / H) * HT + h0 + i % H];
  if (HS)
    for (int i = lane * 4; i < MD; i += 256)
      *reinterpret_cast<float4*>(&slab[wv][i]) = make_float4(0.f, 0.f, 0.f, 0.f);
  if (lane < kRec - 64) rec[wv][64 + lane] = make_float2(0.f, 0.f);
  __syncthreads();

  const int hl = lane * V / F;  // head of this element lane
  const uint64_t doff = dp.active ? dropout_offset(dp, dp.offset) : 0;
  const int64_t Wt = (int64_t)gridDim.x * WB, w = (int64_t)blockIdx.x * WB + wv;
  const int32_t rb = (int32_t)(w * n_rows / Wt), re = (int32_t)((w + 1) * n_rows / Wt);
  Srcs S;
  make_srcs(S, rowptr, col, rowflag, n_edges, re, H, PD, (uint32_t)D * sizeof(T), lane, HT, h0,
            (uint32_t)F * sizeof(T));
  S.sc[0] = make_rsrc(el, (uint32_t)re * HT * 4u);
  S.t[0] = make_rsrc(HS ? hs : nullptr, (uint32_t)re * RB);
  const rsrc_t r_u = make_rsrc(u, (uint32_t)re * RB);
  const rsrc_t r_ulo = make_rsrc(sizeof(T) == 2 ? u_lo : nullptr, (uint32_t)re * RB);
  const rsrc_t r_lse = make_rsrc(lse, (uint32_t)re * HT * 4u);
  const rsrc_t r_att = make_rsrc(ATTD ? attd : nullptr, (uint32_t)n_edges * HT * 4u);
  const char* tabc = reinterpret_cast<const char*>(tab) + lane * V * 4;
  char* slabc = reinterpret_cast<char*>(&slab[wv][0]) + lane * V * 4;
  const float2* recl = &rec[wv][hl * W];
  const uint32_t v_att0 = (uint32_t)((lane % W) * HT + h0 + lane / W) * 4u;
  if (rb < re) {
    using Gp = Grp<RW, NT, 1, PD>;
    const int ng = (re - rb + PD - 1) / PD;
    Gp nxt;
    load_grp<H, V, NT, 1, PD, T, RW, HT>(nxt, S, rb, load_rp(S, rb, lane), lane);
    int32_t rp_n = load_rp(S, rb + PD, lane);
    for (int gi = 0; gi < ng; ++gi) {
      const int32_t r0 = rb + gi * PD;
      const Gp cur = nxt;  // this group's loads (issued one group ago)
      load_grp<H, V, NT, 1, PD, T, RW, HT>(nxt, S, r0 + PD, rp_n, lane);
      rp_n = load_rp(S, r0 + 2 * PD, lane);

      int32_t srp[PD + 1];
#pragma unroll
      for (int u = 0; u <= PD; ++u) srp[u] = rdlane(cur.rp, u);
      int32_t cbase = srp[0];
#pragma unroll
      for (int p = 0; p < kColPages; ++p) colb[wv][64 * p + lane] = (uint8_t)cur.colv[p];
      const uint64_t vmask = __ballot(lane < PD && cur.flag != 0);
      lses[wv][lane] = -INFINITY;  // rows without edges (and no virtual row)
      for (int t0 = 0; t0 < PD;) {
        const int t1 = sub_end<W, PD>(cur.rp, t0, lane);
        const int32_t Es = rdlane(cur.rp, t0);
        const int nEs = min(W, rdlane(cur.rp, t1) - Es);
        if (Es - cbase + nEs > kNCol) cbase = colb_refill(S, colb[wv], Es, lane);
        // (1) slot lanes: score, row softmax, keep, attention -> records
        {
          const Slot sl = slot_geo<H, PD>(cur.rp, t0, t1, Es, nEs, cbase, colb[wv], lane, M);
          const int h = lane / W, k = lane % W;
          const float elv = __shfl(cur.s[0], sl.t * H + h);
          const bool virt = (vmask >> sl.t) & 1ull;
          const float sc = sl.valid ? (virt ? 0.f : lrelu(elv + ert[sl.j * H + h], slope))
                                    : -INFINITY;
          const float mx = __shfl(seg_scan<W, true>(sc, lane, sl.d), sl.endl);
          const float pe = sl.valid ? __expf(sc - mx) : 0.f;
          const float sm = __shfl(seg_scan<W, false>(pe, lane, sl.d), sl.endl);
          const int64_t elem = (int64_t)(Es + k) * HT + h0 + h;
          const float ad = sl.valid ? pe / sm * slot_keep(dp, doff, elem) : 0.f;
          rec[wv][lane] = make_float2(ad, __int_as_float(sl.j * D * 4));
          if (sl.valid && lane == sl.endl) lses[wv][sl.t * H + h] = mx + __logf(sm);
          if (ATTD)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(ad), r_att,
                                                  sl.valid ? v_att0 : kOOB,
                                                  (uint32_t)Es * (4u * HT), 0);
        }
        // (2) element lanes: per row, its edges' records; u in registers, v slab
#pragma unroll
        for (int t = 0; t < PD; ++t) {
          if (t >= t0 && t < t1) {
            const int32_t q0 = srp[t] - Es, q1 = srp[t + 1] - Es;
            float acc[V], hsr[V];
#pragma unroll
            for (int v = 0; v < V; ++v) acc[v] = 0.f;
            if (HS) raw_unpack<T, V, RW>(cur.rows[0][t], hsr);
            // two edges a step: a row's columns are distinct, so both slab entries are
            // read before either is written (the next step's reads follow these writes)
            for (int32_t q = q0; q < q1; q += 2) {
              const bool two = q + 1 < q1;
              const float2 ra = recl[q], rb2 = recl[q + 1];
              const float a0 = ra.x, a1 = two ? rb2.x : 0.f;
              const int j0 = __float_as_int(ra.y), j1 = __float_as_int(rb2.y);
              float x0[V], x1[V];
              ld_row<V>(reinterpret_cast<const float*>(tabc + j0), x0);
              ld_row<V>(reinterpret_cast<const float*>(tabc + j1), x1);
#pragma unroll
              for (int v = 0; v < V; ++v) acc[v] = fmaf(a1, x1[v], fmaf(a0, x0[v], acc[v]));
              if (HS) {
                float* sp0 = reinterpret_cast<float*>(slabc + j0);
                float* sp1 = reinterpret_cast<float*>(slabc + j1);
                float y0[V], y1[V];
                ld_row<V>(sp0, y0);
                ld_row<V>(sp1, y1);
#pragma unroll
                for (int v = 0; v < V; ++v) {
                  y0[v] = fmaf(a0, hsr[v], y0[v]);
                  y1[v] = fmaf(a1, hsr[v], y1[v]);
                }
                st_row<V>(sp0, y0);
                if (two) st_row<V>(sp1, y1);
              }
            }
            const uint32_t so = (uint32_t)(r0 + t) * RB;
            bst_row<T, V>(r_u, S.v_row, acc, so);
            if (sizeof(T) == 2) {
              float res[V];
#pragma unroll
              for (int v = 0; v < V; ++v) res[v] = acc[v] - (float)(bf16_t)acc[v];
              bst_row<T, V>(r_ulo, S.v_row, res, so);
            }
          }
        }
        t0 = t1;
      }
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(lses[wv][lane]), r_lse, S.v_s,
                                            (uint32_t)r0 * (4u * HT), 0);
    }
  }
  if (HS) {
    __syncthreads();
    float* dst = part + ((int64_t)blockIdx.x * gridDim.y + blockIdx.y) * MD;  // [block][head]
    for (int i = tid * 4; i < MD; i += WB * 256) {
      float4 a = *reinterpret_cast<const float4*>(&slab[0][i]);
#pragma unroll
      for (int q = 1; q < WB; ++q) {
        const float4 b = *reinterpret_cast<const float4*>(&slab[q][i]);
        a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
      }
      *reinterpret_cast<float4*>(dst + i) = a;
    }
  }
}

// ----------------------------------------------------------------------- backward ---
// Per row i, head h (reference: the autograd of Ablation.py:266-274, Ours.py:84-86):
//   g_e  = dU_i . hc_j (+ hs_i . dV_j) (+ coef_i exp(attd_e))
//   D_i  = sum_e attd_e g_e
//   ds_e = att_e (keep_e g_e - D_i),  de_e = ds_e lrelu'(pre_e),  d_el_i = sum_e de_e
//   d_hs_i = sum_e attd_e dV_j;  block partials of d_hc_j = sum attd_e dU_i, d_er_j = sum de_e
// Per sub-group: slot lanes give att, keep and the records; element lanes walk each
// row's edges two at a time (g_e dots reduced together, d_hs in registers, d_hc into the
// wave's slab, g_e back into the record); slot lanes finish D, de, d_el (segmented
// scans) and add de into the wave's d_er slab (one LDS float add per slot).
// (HT > H: the head-split form, as bip_fwd_kernel's; 12 waves (three per SIMD, 168 VGPRs)
// beside the two 8 KB tables of one head, 8 for the bf16 form with hs, which needs ~190)
constexpr int kWavesB2 = 12;
template <int H, int HT, typename T, bool HS>
constexpr int bwd_waves() {
  return HT > H ? (sizeof(T) == 2 && HS ? 8 : kWavesB2) : kWavesB;
}
template <int H, int F, typename T, bool HS, bool COEF, int HT = H>
__global__ void __launch_bounds__((bwd_waves<H, HT, T, HS>() * 64)) bip_bwd_kernel(
    const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
    const uint8_t* __restrict__ rowflag, int32_t n_rows, int32_t n_cols, int32_t n_edges,
    const float* __restrict__ el, const float* __restrict__ er, const T* __restrict__ hc,
    const float* __restrict__ lse, const T* __restrict__ dU, const T* __restrict__ hs,
    const T* __restrict__ dV, const float* __restrict__ row_coef, float slope, Dropout dp,
    float* __restrict__ d_el, T* __restrict__ d_hs, float* __restrict__ part) {
  constexpr int D = H * F, V = D / 64, QH = F / V, WB = bwd_waves<H, HT, T, HS>(), W = 64 / H;
  constexpr int DT = HT * F, MDX = kMaxMD * H / HT;
  constexpr int NT = HS ? 2 : 1;
  constexpr int PD = grp_rows<H, D, T, NT>(), RW = row_words<V, T>();
  constexpr int NS = COEF ? 3 : 2;
  constexpr uint32_t RB = (uint32_t)DT * sizeof(T);  // row stride in bytes
  const int h0 = HT > H ? (int)blockIdx.y * H : 0;
  __shared__ __attribute__((aligned(16))) float tab[HS ? 2 : 1][MDX];  // hc, dV
  __shared__ float ert[64];
  __shared__ __attribute__((aligned(16))) float slab[WB][MDX];  // d_hc
  __shared__ float sder[WB][64];                                  // d_er, lane j * H + h
  __shared__ __attribute__((aligned(16))) float2 rec[WB][kRec];
  __shared__ uint8_t colb[WB][kNCol];
  __shared__ float dels[WB][64];
  const int M = n_cols, MD = M * D, MH = M * H;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  for (int i = tid * 4; i < MD; i += WB * 256) {  // this launch's heads of hc, dV
    const int src = (i / D) * DT + h0 * F + i % D;
    float x[4];
    ld_row<4>(hc + src, x);
    st_row<4>(&tab[0][i], x);
    if (HS) {
      ld_row<4>(dV + src, x);
      st_row<4>(&tab[HS ? 1 : 0][i], x);
    }
  }
  for (int i = tid; i < MH; i += WB * 64) ert[i] = er[(i / H) * HT + h0 + i % H];
  for (int i = lane * 4; i < MD; i += 256)
    *reinterpret_cast<float4*>(&slab[wv][i]) = make_float4(0.f, 0.f, 0.f, 0.f);
  sder[wv][lane] = 0.f;
  if (lane < kRec - 64) rec[wv][64 + lane] = make_float2(0.f, 0.f);
  __syncthreads();

  const int hl = lane * V / F;
  const uint64_t doff = dp.active ? dropout_offset(dp, dp.offset) : 0;
  const int64_t Wt = (int64_t)gridDim.x * WB, w = (int64_t)blockIdx.x * WB + wv;
  const int32_t rb = (int32_t)(w * n_rows / Wt), re = (int32_t)((w + 1) * n_rows / Wt);
  Srcs S;
  make_srcs(S, rowptr, col, rowflag, n_edges, re, H, PD, (uint32_t)D * sizeof(T), lane, HT, h0,
            (uint32_t)F * sizeof(T));
  S.sc[0] = make_rsrc(el, (uint32_t)re * HT * 4u);
  S.sc[1] = make_rsrc(lse, (uint32_t)re * HT * 4u);
  S.sc[2] = make_rsrc(COEF ? row_coef : nullptr, (uint32_t)re * HT * 4u);
  S.t[0] = make_rsrc(dU, (uint32_t)re * RB);
  S.t[1] = make_rsrc(HS ? hs : nullptr, (uint32_t)re * RB);
  const rsrc_t r_dhs = make_rsrc(HS ? d_hs : nullptr, (uint32_t)re * RB);
  const rsrc_t r_del = make_rsrc(d_el, (uint32_t)re * HT * 4u);
  const char* tabc = reinterpret_cast<const char*>(&tab[0][0]) + lane * V * 4;
  const char* tdvc = reinterpret_cast<const char*>(&tab[HS ? 1 : 0][0]) + lane * V * 4;
  char* slabc = reinterpret_cast<char*>(&slab[wv][0]) + lane * V * 4;
  float2* recl = &rec[wv][hl * W];
  if (rb < re) {
    using Gp = Grp<RW, NT, NS, PD>;
    const int ng = (re - rb + PD - 1) / PD;
    Gp nxt;
    load_grp<H, V, NT, NS, PD, T, RW, HT>(nxt, S, rb, load_rp(S, rb, lane), lane);
    int32_t rp_n = load_rp(S, rb + PD, lane);
    for (int gi = 0; gi < ng; ++gi) {
      const int32_t r0 = rb + gi * PD;
      const Gp cur = nxt;
      load_grp<H, V, NT, NS, PD, T, RW, HT>(nxt, S, r0 + PD, rp_n, lane);
      rp_n = load_rp(S, r0 + 2 * PD, lane);

      int32_t srp[PD + 1];
#pragma unroll
      for (int u = 0; u <= PD; ++u) srp[u] = rdlane(cur.rp, u);
      int32_t cbase = srp[0];
#pragma unroll
      for (int p = 0; p < kColPages; ++p) colb[wv][64 * p + lane] = (uint8_t)cur.colv[p];
      const uint64_t vmask = __ballot(lane < PD && cur.flag != 0);
      dels[wv][lane] = 0.f;  // rows without edges (and no virtual row)
      for (int t0 = 0; t0 < PD;) {
        const int t1 = sub_end<W, PD>(cur.rp, t0, lane);
        const int32_t Es = rdlane(cur.rp, t0);
        const int nEs = min(W, rdlane(cur.rp, t1) - Es);
        if (Es - cbase + nEs > kNCol) cbase = colb_refill(S, colb[wv], Es, lane);
        // (1) slot lanes: score, attention, keep -> records
        const Slot sl = slot_geo<H, PD>(cur.rp, t0, t1, Es, nEs, cbase, colb[wv], lane, M);
        const int h = lane / W, k = lane % W;
        const int rsl = sl.t * H + h;
        const bool virt = (vmask >> sl.t) & 1ull;
        // (the row scalars live on lanes t * H + h: every shuffle runs with all lanes
        // active -- ds_bpermute reads 0 from an inactive lane)
        const float elq = __shfl(cur.s[0], rsl), lsq = __shfl(cur.s[1], rsl);
        const float cfq = COEF ? __shfl(cur.s[NS - 1], rsl) : 0.f;
        const float pre = elq + ert[sl.j * H + h];
        const float sc = virt ? 0.f : lrelu(pre, slope);
        const float att = sl.valid ? __expf(sc - lsq) : 0.f;
        const float kf = slot_keep(dp, doff, (int64_t)(Es + k) * HT + h0 + h);
        const float ad = att * kf;
        rec[wv][lane] = make_float2(ad, __int_as_float(sl.j * D * 4));
        // (2) element lanes: g_e (into the record), d_hs, the d_hc slab
#pragma unroll
        for (int t = 0; t < PD; ++t) {
          if (t >= t0 && t < t1) {
            const int32_t q0 = srp[t] - Es, q1 = srp[t + 1] - Es;
            float dUr[V], hsr[V];
            raw_unpack<T, V, RW>(cur.rows[0][t], dUr);
            raw_unpack<T, V, RW>(cur.rows[NT - 1][t], hsr);
            float wacc[V];
#pragma unroll
            for (int v = 0; v < V; ++v) wacc[v] = 0.f;
            for (int32_t q = q0; q < q1; q += 2) {
              const bool two = q + 1 < q1;
              const float2 ra = recl[q], rb2 = recl[q + 1];
              const float a0 = ra.x, a1 = two ? rb2.x : 0.f;
              const int j0 = __float_as_int(ra.y), j1 = __float_as_int(rb2.y);
              float x0[V], x1[V];
              ld_row<V>(reinterpret_cast<const float*>(tabc + j0), x0);
              ld_row<V>(reinterpret_cast<const float*>(tabc + j1), x1);
              float p0 = 0.f, p1 = 0.f;
#pragma unroll
              for (int v = 0; v < V; ++v) {
                p0 = fmaf(dUr[v], x0[v], p0);
                p1 = fmaf(dUr[v], x1[v], p1);
              }
              if (HS) {
                float y0[V], y1[V];
                ld_row<V>(reinterpret_cast<const float*>(tdvc + j0), y0);
                ld_row<V>(reinterpret_cast<const float*>(tdvc + j1), y1);
#pragma unroll
                for (int v = 0; v < V; ++v) {
                  p0 = fmaf(hsr[v], y0[v], p0);
                  p1 = fmaf(hsr[v], y1[v], p1);
                  wacc[v] = fmaf(a1, y1[v], fmaf(a0, y0[v], wacc[v]));
                }
              }
              if constexpr (QH == 32) {
                const float gp = pair_sum32(p0, p1, lane);
                if (lane % 16 == 0 && (two || (lane & 16) == 0))
                  recl[q + ((lane >> 4) & 1)].x = gp;
              } else {
                const float g0 = lanes_sum<QH>(p0, lane), g1 = lanes_sum<QH>(p1, lane);
                if (lane % QH == 0) {
                  recl[q].x = g0;
                  if (two) recl[q + 1].x = g1;
                }
              }
              {
                float* sp0 = reinterpret_cast<float*>(slabc + j0);
                float* sp1 = reinterpret_cast<float*>(slabc + j1);
                float z0[V], z1[V];
                ld_row<V>(sp0, z0);
                ld_row<V>(sp1, z1);
#pragma unroll
                for (int v = 0; v < V; ++v) {
                  z0[v] = fmaf(a0, dUr[v], z0[v]);
                  z1[v] = fmaf(a1, dUr[v], z1[v]);
                }
                st_row<V>(sp0, z0);
                if (two) st_row<V>(sp1, z1);
              }
            }
            if (HS) bst_row<T, V>(r_dhs, S.v_row, wacc, (uint32_t)(r0 + t) * RB);
          }
        }
        // (3) slot lanes: D_i, de_e, d_el_i, the d_er slab
        {
          float g = rec[wv][lane].x;
          if (COEF && sl.valid) g = fmaf(cfq, expf(ad), g);
          const float Dq = __shfl(seg_scan<W, false>(sl.valid ? ad * g : 0.f, lane, sl.d), sl.endl);
          const float ds = att * (g * kf - Dq);
          const float dev = sl.valid && !virt ? ds * (pre > 0.f ? 1.f : slope) : 0.f;
          const float del = seg_scan<W, false>(dev, lane, sl.d);
          if (sl.valid && lane == sl.endl) dels[wv][rsl] = del;
          if (sl.valid)
            __hip_atomic_fetch_add(&sder[wv][sl.j * H + h], dev, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WAVEFRONT);
        }
        t0 = t1;
      }
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(dels[wv][lane]), r_del, S.v_s,
                                            (uint32_t)r0 * (4u * HT), 0);
    }
  }
  __syncthreads();
  // the block's partial: [d_hc: head blk (M D)][d_er: head blk (M H)] over all HT heads,
  // each head block writing its own slices
  const int nh = HT / H, hb = HT > H ? (int)blockIdx.y : 0;
  float* dst = part + (int64_t)blockIdx.x * part_stride(nh * (MD + MH));
  for (int i = tid * 4; i < MD; i += WB * 256) {
    float4 a = *reinterpret_cast<const float4*>(&slab[0][i]);
#pragma unroll
    for (int q = 1; q < WB; ++q) {
      const float4 b = *reinterpret_cast<const float4*>(&slab[q][i]);
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    *reinterpret_cast<float4*>(dst + hb * MD + i) = a;
  }
  for (int i = tid; i < MH; i += WB * 64) {
    float a = sder[0][i];
#pragma unroll
    for (int q = 1; q < WB; ++q) a += sder[q][i];
    dst[nh * MD + hb * MH + i] = a;
  }
}

// out[i] = sum_b part[b][i] in block order: bip_reduce.h (bip_reduce_block).  256 blocks at
// M x H x F = 4096: the whole chip reads the partials (64 blocks of one 64-entry slice each
// ran latency-bound, 6.6 us).
template <typename T>
__global__ void __launch_bounds__(1024) bip_reduce_kernel(BipReduce r) {
  __shared__ float red[64][17];
  bip_reduce_block<T, 1024>(r, blockIdx.x, red);
}

}  // namespace bip

// ---- the reduce launch, or its hand-over to the next Ours-layer launch (bip_reduce.h) ----
namespace {
thread_local int t_defer = 0;         // msha_bip_defer_reduce
thread_local bool t_has = false;      // a reduce is pending
thread_local BipReduce t_pending;
thread_local hipStream_t t_pending_s = nullptr;
}  // namespace

static void bip_reduce_launch(const BipReduce& r, hipStream_t s) {
  if (r.bf16)
    hipLaunchKernelGGL(bip::bip_reduce_kernel<bf16_t>, dim3(r.blocks()), dim3(1024), 0, s, r);
  else
    hipLaunchKernelGGL(bip::bip_reduce_kernel<float>, dim3(r.blocks()), dim3(1024), 0, s, r);
}

void bip_reduce_run(const BipReduce& r, hipStream_t s) { bip_reduce_launch(r, s); }

bool bip_reduce_submit(const BipReduce& r, hipStream_t s) {
  if (t_has) {  // (one at a time: an earlier one not taken runs now)
    bip_reduce_launch(t_pending, t_pending_s);
    t_has = false;
  }
  if (!t_defer) {
    bip_reduce_launch(r, s);
    return false;
  }
  t_pending = r;
  t_pending_s = s;
  t_has = true;
  return true;
}

bool bip_reduce_take(BipReduce& r, hipStream_t s) {
  if (!t_has) return false;
  if (t_pending_s != s) {  // another stream: not fused, run it where it was submitted
    bip_reduce_launch(t_pending, t_pending_s);
    t_has = false;
    return false;
  }
  r = t_pending;
  t_has = false;
  return true;
}

// (edge_bip2.hip) block partials -> v or d_hc + d_er, un-split layout
int bip_reduce(const float* part, int32_t nb, int32_t stride, int32_t n, int32_t n_t, void* out_t,
               bool bf16, float* out_f, int32_t fblk, hipStream_t s) {
  BipReduce r{part, out_t, out_f, nb, stride, n, n_t, n_t, 0, n_t, 0, fblk, 1, bf16 ? 1 : 0};
  bip_reduce_submit(r, s);
  return 1;
}
bool bip2_ok(const msha_graph* g, int heads, int feat, float slope);
int bip2_bwd(const msha_graph* g, int dtype, const float* el, const float* er, const void* hc,
             const float* lse, const void* dU, const void* hs, const void* dV,
             const float* row_coef, float slope, const Dropout& dp, float* d_el, float* d_er,
             void* d_hc, void* d_hs, float* part, int nb, hipStream_t s);
int bip2_fwd(const msha_graph* g, int dtype, const float* el, const float* er, const void* hc,
             const void* hs, float slope, const Dropout& dp, void* u, float* lse, float* attd,
             void* v, float* part, int nb, hipStream_t s);
int bip3_bwd(const msha_graph* g, int dtype, const float* el, const float* er, const void* hc,
             const float* lse, const void* dU, const void* hs, const void* dV,
             const float* row_coef, float slope, const Dropout& dp, float* d_el, float* d_er,
             void* d_hc, void* d_hs, float* part, int nb, hipStream_t s);
int bip3_fwd(const msha_graph* g, int dtype, const float* el, const float* er, const void* hc,
             const void* hs, float slope, const Dropout& dp, void* u, float* lse, float* attd,
             void* v, float* part, int nb, hipStream_t s);

namespace bip {

static int cu_count() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cached[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    cached[dev] = n;
  }
  return cached[dev];
}

}  // namespace bip

static bool bip_shape(int64_t n_cols, int heads, int feat) {
  const int64_t D = (int64_t)heads * feat;
  if (D % 64 != 0 || D > 256 || 64 % heads != 0) return false;
  if (feat % (D / 64) != 0) return false;
  // M <= 32 and M * H <= 64: a row's (edge, head) slots fit one 64-lane sub-group and a
  // group's kPD rows fit the kColPages column pages
  return n_cols <= 32 && n_cols * D <= bip::kMaxMD && n_cols * heads <= 64;
}

}  // namespace msha

using namespace msha;

extern "C" int msha_bip_supported(const msha_graph* g, int32_t heads, int32_t feat,
                                  int32_t dtype) {
  // 32-bit buffer offsets below the kOOB mask bit: every table < 2 GiB
  if (g == nullptr || g->n_rows <= 0 || g->n_cols <= 0 ||
      g->n_rows * (int64_t)heads * feat * 4 >= ((int64_t)1 << 31) ||
      g->n_edges * (int64_t)heads * 4 >= ((int64_t)1 << 31))
    return 0;
  if (dtype != MSHA_DTYPE_F32 && dtype != MSHA_DTYPE_BF16) return 0;
  if (!bip_shape(g->n_cols, heads, feat)) return 0;
  bool ok = false;
#define X(h, f) if (heads == h && feat == f) ok = true;
  MSHA_FOR_EACH_SHAPE(X)
#undef X
  return ok ? 1 : 0;
}

extern "C" size_t msha_bip_workspace_size(const msha_graph* g, int32_t heads, int32_t feat) {
  if (g == nullptr || heads <= 0 || feat <= 0) return 0;
  const size_t rec = (size_t)bip::part_stride((int32_t)(g->n_cols * ((int64_t)heads * feat + heads)));
  return (size_t)bip::cu_count() * rec * sizeof(float) + 256;
}

// the head-split form (one head per block, blockIdx.y) where a head's row slice is 64
// elements: twice the waves per CU, but every row's CSR walk, column bytes and scalar
// control run once per head.  Off by default (MSHA_BIP_SPLIT=1 turns it on): the
// kernels are issue-bound on that per-row control, and the A/B at bip1m fp32 was fwd
// 290 -> 316 us, bwd 466 -> 663 us; R15 bip_fwd + bip_bwd 56 -> 86 us.
static bool bip_split_enabled() {
  static const int on = [] {
    const char* v = getenv("MSHA_BIP_SPLIT");
    return v != nullptr && *v ? atoi(v) : 0;
  }();
  return on != 0;
}

template <int H, int F, typename T>
static void bip_launch_fwd(const msha_graph* g, const float* el, const float* er, const void* hc,
                           const void* hs, float slope, const Dropout& dp, void* u, void* u_lo,
                           float* lse, float* attd, void* v, float* part, int nb, hipStream_t s) {
  constexpr bool kSplit = H > 1 && F == 64;
  const bool split = kSplit && bip_split_enabled();
  auto go = [&](auto kern, dim3 grid, int waves) {
    hipLaunchKernelGGL(kern, grid, dim3(waves * 64), 0, s, g->rowptr, g->col,
                       g->rowflag, (int32_t)g->n_rows, (int32_t)g->n_cols, (int32_t)g->n_edges,
                       el, er, (const T*)hc, (const T*)hs, slope, dp, (T*)u, (T*)u_lo, lse, attd,
                       part);
  };
  const dim3 g1(nb), gs(nb, H);
  constexpr int w1 = bip::kWavesF, ws = bip::kWavesF2;
  if (hs != nullptr) {
    if (split) {
      if constexpr (kSplit) {
        if (attd != nullptr) go(bip::bip_fwd_kernel<1, F, T, true, true, H>, gs, ws);
        else go(bip::bip_fwd_kernel<1, F, T, true, false, H>, gs, ws);
      }
    } else if (attd != nullptr) go(bip::bip_fwd_kernel<H, F, T, true, true>, g1, w1);
    else go(bip::bip_fwd_kernel<H, F, T, true, false>, g1, w1);
    const int32_t MD = (int32_t)(g->n_cols * H * F), MDh = (int32_t)(g->n_cols * F);
    // partials [block][head][column][F] (split) or [block][column][H F]
    const BipReduce r{part, v, nullptr, nb, MD, MD, MD, split ? F : MD, split ? H * F : 0,
                      split ? MDh : MD, split ? F : 0, 1, 1, sizeof(T) == 2 ? 1 : 0};
    bip_reduce_submit(r, s);
  } else if (split) {
    if constexpr (kSplit) {
      if (attd != nullptr) go(bip::bip_fwd_kernel<1, F, T, false, true, H>, gs, ws);
      else go(bip::bip_fwd_kernel<1, F, T, false, false, H>, gs, ws);
    }
  } else if (attd != nullptr) go(bip::bip_fwd_kernel<H, F, T, false, true>, g1, w1);
  else go(bip::bip_fwd_kernel<H, F, T, false, false>, g1, w1);
}

template <int H, int F, typename T>
static void bip_launch_bwd(const msha_graph* g, const float* el, const float* er, const void* hc,
                           const float* lse, const void* dU, const void* hs, const void* dV,
                           const float* row_coef, float slope, const Dropout& dp, float* d_el,
                           float* d_er, void* d_hc, void* d_hs, float* part, int nb,
                           hipStream_t s) {
  constexpr bool kSplit = H > 1 && F == 64;
  const bool split = kSplit && bip_split_enabled();
  auto go = [&](auto kern, dim3 grid, int waves) {
    hipLaunchKernelGGL(kern, grid, dim3(waves * 64), 0, s, g->rowptr, g->col,
                       g->rowflag, (int32_t)g->n_rows, (int32_t)g->n_cols, (int32_t)g->n_edges,
                       el, er, (const T*)hc,
                       lse, (const T*)dU, (const T*)hs, (const T*)dV, row_coef, slope, dp, d_el,
                       (T*)d_hs, part);
  };
  const bool hsb = dV != nullptr, cf = row_coef != nullptr;
  if (split) {
    if constexpr (kSplit) {
      const dim3 gs(nb, H);
      constexpr int w1 = bip::bwd_waves<1, H, T, true>(), w0 = bip::bwd_waves<1, H, T, false>();
      if (hsb && cf) go(bip::bip_bwd_kernel<1, F, T, true, true, H>, gs, w1);
      else if (hsb) go(bip::bip_bwd_kernel<1, F, T, true, false, H>, gs, w1);
      else if (cf) go(bip::bip_bwd_kernel<1, F, T, false, true, H>, gs, w0);
      else go(bip::bip_bwd_kernel<1, F, T, false, false, H>, gs, w0);
    }
  } else {
    const dim3 g1(nb);
    constexpr int w1 = bip::kWavesB;
    if (hsb && cf) go(bip::bip_bwd_kernel<H, F, T, true, true>, g1, w1);
    else if (hsb) go(bip::bip_bwd_kernel<H, F, T, true, false>, g1, w1);
    else if (cf) go(bip::bip_bwd_kernel<H, F, T, false, true>, g1, w1);
    else go(bip::bip_bwd_kernel<H, F, T, false, false>, g1, w1);
  }
  const int32_t MD = (int32_t)(g->n_cols * H * F), MH = (int32_t)(g->n_cols * H);
  const int32_t MDh = (int32_t)(g->n_cols * F), M = (int32_t)g->n_cols;
  // partials [block][d_hc (split: [head][column][F])][d_er (split: [head][column])]
  const BipReduce r{part, d_hc, d_er, nb, bip::part_stride(MD + MH), MD + MH, MD,
                    split ? F : MD, split ? H * F : 0, split ? MDh : MD, split ? F : 0,
                    split ? M : MH, split ? H : 1, sizeof(T) == 2 ? 1 : 0};
  bip_reduce_submit(r, s);
}

extern "C" int msha_bip_attention_fwd(const msha_graph* g, int32_t heads, int32_t feat,
                                      int32_t dtype, const float* el, const float* er,
                                      const void* hc, const void* hs, float neg_slope,
                                      float drop_p, uint64_t seed, uint64_t offset, void* u,
                                      void* u_lo, float* lse, float* attd, void* v, void* ws,
                                      size_t ws_bytes, msha_stream_t stream) {
  MSHA_ARG_CHECK(g != nullptr && g->rowptr != nullptr && (g->n_edges == 0 || g->col != nullptr),
                 "bip_attention_fwd: graph arrays missing");
  MSHA_ARG_CHECK(el && er && hc && u && lse, "bip_attention_fwd: null pointer");
  MSHA_ARG_CHECK((hs == nullptr) == (v == nullptr), "bip_attention_fwd: hs and v go together");
  MSHA_ARG_CHECK(drop_p >= 0.f && drop_p <= 1.f, "bip_attention_fwd: p must be in [0,1]");
  if (!msha_bip_supported(g, heads, feat, dtype))
    return fail(MSHA_ERR_UNSUPPORTED, "bip_attention_fwd: graph/shape not covered (msha_bip_supported)");
  const int nb = bip::cu_count();
  if (hs != nullptr)
    MSHA_ARG_CHECK(ws != nullptr && ws_bytes >= msha_bip_workspace_size(g, heads, feat),
                   "bip_attention_fwd: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const Dropout dp = make_dropout(drop_p, seed, offset, s);
  // the MFMA kernels (edge_bip3.hip) from msha_bip2_bwd_min_rows rows up; below it (the
  // shipped graphs: < 1 tile per wave) the mask forward of edge_bip2.hip
  if (u_lo == nullptr && bip2_ok(g, heads, feat, neg_slope) &&
      ((g->n_rows >= msha_bip2_bwd_min_rows(-1) &&
        bip3_fwd(g, dtype, el, er, hc, hs, neg_slope, dp, u, lse, attd, v, (float*)ws, nb, s)) ||
       bip2_fwd(g, dtype, el, er, hc, hs, neg_slope, dp, u, lse, attd, v, (float*)ws, nb, s)))
    return check_launch("bip_attention_fwd");
  bool done = false;
#define X(h, f)                                                                                  \
  if (heads == h && feat == f) {                                                                 \
    if constexpr ((h * f) % 64 == 0 && h * f <= 256) {                                           \
      if (dtype == MSHA_DTYPE_BF16)                                                              \
        bip_launch_fwd<h, f, bf16_t>(g, el, er, hc, hs, neg_slope, dp, u, u_lo, lse, attd, v,    \
                                     (float*)ws, nb, s);                                         \
      else                                                                                       \
        bip_launch_fwd<h, f, float>(g, el, er, hc, hs, neg_slope, dp, u, nullptr, lse, attd, v,  \
                                    (float*)ws, nb, s);                                          \
      done = true;                                                                               \
    }                                                                                            \
  }
  MSHA_FOR_EACH_SHAPE(X)
#undef X
  if (!done) return fail(MSHA_ERR_UNSUPPORTED, "bip_attention_fwd: unsupported (heads, feat)");
  return check_launch("bip_attention_fwd");
}

static std::atomic<int64_t>& bip2_bwd_cut() {
  static std::atomic<int64_t> cut{[] {
    const char* v = getenv("MSHA_BIP2_BWD_MIN_ROWS");
    return v != nullptr && *v ? (int64_t)atoll(v) : (int64_t)131072;
  }()};
  return cut;
}

// (ABI 16) 1: the block-partial reduce of the next bipartite forward / backward is handed to
// the next Ours-layer launch on the same stream (msha_ours_intra_fwd / stage 1 of
// msha_ours_intra_bwd run it as extra blocks: one graph node fewer each way); 0: back to
// separate launches, and a reduce still pending is launched now
extern "C" int msha_bip_defer_reduce(int32_t on) {
  t_defer = on != 0;
  if (!t_defer && t_has) {
    bip_reduce_launch(t_pending, t_pending_s);
    t_has = false;
    return check_launch("bip_defer_reduce");
  }
  return MSHA_OK;
}

extern "C" int64_t msha_bip2_bwd_min_rows(int64_t rows) {
  return rows >= 0 ? bip2_bwd_cut().exchange(rows) : bip2_bwd_cut().load();
}

extern "C" int msha_bip_attention_bwd(const msha_graph* g, int32_t heads, int32_t feat,
                                      int32_t dtype, const float* el, const float* er,
                                      const void* hc, const float* lse, const void* dU,
                                      const void* hs, const void* dV, const float* row_coef,
                                      float neg_slope, float drop_p, uint64_t seed,
                                      uint64_t offset, float* d_el, float* d_er, void* d_hc,
                                      void* d_hs, void* ws, size_t ws_bytes,
                                      msha_stream_t stream) {
  MSHA_ARG_CHECK(g != nullptr && g->rowptr != nullptr && (g->n_edges == 0 || g->col != nullptr),
                 "bip_attention_bwd: graph arrays missing");
  MSHA_ARG_CHECK(el && er && hc && lse && dU && d_el && d_er && d_hc,
                 "bip_attention_bwd: null pointer");
  MSHA_ARG_CHECK(dV == nullptr || (hs != nullptr && d_hs != nullptr),
                 "bip_attention_bwd: dV needs hs and d_hs");
  MSHA_ARG_CHECK(drop_p >= 0.f && drop_p <= 1.f, "bip_attention_bwd: p must be in [0,1]");
  if (!msha_bip_supported(g, heads, feat, dtype))
    return fail(MSHA_ERR_UNSUPPORTED, "bip_attention_bwd: graph/shape not covered (msha_bip_supported)");
  MSHA_ARG_CHECK(ws != nullptr && ws_bytes >= msha_bip_workspace_size(g, heads, feat),
                 "bip_attention_bwd: workspace too small");
  const int nb = bip::cu_count();
  hipStream_t s = (hipStream_t)stream;
  const Dropout dp = make_dropout(drop_p, seed, offset, s);
  // the MFMA backward (edge_bip3.hip; mask backward edge_bip2.hip with MSHA_BIP3=0) wins on
  // large graphs (bip1m fp32: CSR walk 450 us, mask 380-416, MFMA ~400; bf16 MFMA 204) but
  // not on the shipped ones (R15: MFMA 36.1, mask 36.6, CSR walk 31.6 us; rows per wave too
  // few to amortise the per-block setup and partial epilogue).  MSHA_BIP2_BWD_MIN_ROWS /
  // msha_bip2_bwd_min_rows (per process: tests run small graphs through both) move the
  // cut, for the forward's choice as well.
  if (g->n_rows >= msha_bip2_bwd_min_rows(-1) && bip2_ok(g, heads, feat, neg_slope) &&
      (bip3_bwd(g, dtype, el, er, hc, lse, dU, hs, dV, row_coef, neg_slope, dp, d_el, d_er, d_hc,
                d_hs, (float*)ws, nb, s) ||
       bip2_bwd(g, dtype, el, er, hc, lse, dU, hs, dV, row_coef, neg_slope, dp, d_el, d_er, d_hc,
                d_hs, (float*)ws, nb, s)))
    return check_launch("bip_attention_bwd");
  bool done = false;
#define X(h, f)                                                                                  \
  if (heads == h && feat == f) {                                                                 \
    if constexpr ((h * f) % 64 == 0 && h * f <= 256) {                                           \
      if (dtype == MSHA_DTYPE_BF16)                                                              \
        bip_launch_bwd<h, f, bf16_t>(g, el, er, hc, lse, dU, hs, dV, row_coef, neg_slope, dp,    \
                                     d_el, d_er, d_hc, d_hs, (float*)ws, nb, s);                 \
      else                                                                                       \
        bip_launch_bwd<h, f, float>(g, el, er, hc, lse, dU, hs, dV, row_coef, neg_slope, dp,     \
                                    d_el, d_er, d_hc, d_hs, (float*)ws, nb, s);                  \
      done = true;                                                                               \
    }                                                                                            \
  }
  MSHA_FOR_EACH_SHAPE(X)
#undef X
  if (!done) return fail(MSHA_ERR_UNSUPPORTED, "bip_attention_bwd: unsupported (heads, feat)");
  return check_launch("bip_attention_bwd");
}
