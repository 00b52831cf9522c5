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
// into sub-groups whose (edge, head) pairs fill <= 64 slot lanes: slot lanes compute the
// scores, the row softmax (lane-segmented scans), the keep bits and the attention once;
// element lanes (lane l owns elements [l V, l V + V) of the H * F row, V = H F / 64, so
// a head's dot products reduce over its QH = F / V lanes) then walk each row's edges with
// the attention and hc_j read from LDS.
//
// Reference: Ablation.py:266-274 (OursLayer3 scores, masked softmax, dropout,
// u = att @ h1, v = att.T @ h2), Ours.py:84-86 (the backward's row coefficients).
#include "edge_geo.h"

namespace msha {
namespace bip {

constexpr int kMaxMD = 4096;  // floats of one (M, H*F) LDS table: M = 32 at H*F = 128
constexpr int kWaves = 7;     // fwd: 16 KB table + 7 x (16 KB v slab + scratch) = 156 KB;
                              // bwd: two 16 KB tables + 7 x (d_hc, d_er slabs + scratch)

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
template <typename T, int V>
__device__ __forceinline__ void bld_row(rsrc_t r, uint32_t off, float (&x)[V]) {
  constexpr int B = V * (int)sizeof(T);
  uint32_t w[4] = {0, 0, 0, 0};
  if constexpr (B == 16) {
    const u32x4_t a = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
    w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
  } else if constexpr (B == 8) {
    const u32x2_t a = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
    w[0] = a.x; w[1] = a.y;
  } else if constexpr (B == 4) {
    w[0] = __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
  } else {
    w[0] = __builtin_amdgcn_raw_buffer_load_b16(r, off, 0, 0);
  }
#pragma unroll
  for (int v = 0; v < V; ++v) {
    if constexpr (sizeof(T) == 4) x[v] = __uint_as_float(w[v]);
    else x[v] = __uint_as_float(v % 2 == 0 ? w[v / 2] << 16 : w[v / 2] & 0xffff0000u);
  }
}
template <typename T, int V>
__device__ __forceinline__ void bst_row(rsrc_t r, uint32_t off, const float (&x)[V]) {
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
    __builtin_amdgcn_raw_buffer_store_b128(a, r, off, 0, 0);
  } else if constexpr (B == 8) {
    u32x2_t a;
    a.x = w[0]; a.y = w[1];
    __builtin_amdgcn_raw_buffer_store_b64(a, r, off, 0, 0);
  } else if constexpr (B == 4) {
    __builtin_amdgcn_raw_buffer_store_b32(w[0], r, off, 0, 0);
  } else {
    __builtin_amdgcn_raw_buffer_store_b16((uint16_t)w[0], r, off, 0, 0);
  }
}

constexpr int kPD = 8;        // rows per group
constexpr int kColPages = 4;  // a group's columns: <= kPD * 32 = 256 edges

// A group: rows [r0, r0 + kPD) of the wave's range.  rp lane t = rowptr[min(r0 + t, re)];
// colv[p] lane q = column of edge E0 + 64 p + q; s0/s1/s2 lane t * H + h = el/lse/coef of
// (row t, head h); flag lane t = rowflag; rows[.][t] = this lane's V elements of row
// r0 + t of the streamed tables (hs, or dU and hs).  Rows past the range read as empty.
template <int V, int NT>
struct Grp {
  int32_t rp;
  int32_t colv[kColPages];
  float s0, s1, s2;
  uint32_t flag;
  float rows[NT > 0 ? NT : 1][kPD][V];
};

struct Srcs {
  rsrc_t rp, col, flag, p0, p1, p2, t0, t1;
  int32_t re;
};

__device__ __forceinline__ int32_t load_rp(const Srcs& S, int32_t r0, int lane) {
  return buf_i32(S.rp, (uint32_t)min(r0 + lane, S.re) * 4u);
}

template <int H, int V, int NT, typename T>
__device__ __forceinline__ void load_grp(Grp<V, NT>& g, const Srcs& S, int32_t r0, int32_t rp,
                                         int lane) {
  constexpr int D = 64 * V;
  g.rp = rp;
  const int32_t E0 = rdlane(rp, 0), nE = rdlane(rp, kPD) - E0;
#pragma unroll
  for (int p = 0; p < kColPages; ++p) {
    const int32_t q = 64 * p + lane;
    g.colv[p] = buf_i32(S.col, q < nE ? (uint32_t)(E0 + q) * 4u : kOOB);
  }
  const bool sl = lane < kPD * H && r0 + lane / H < S.re;
  const uint32_t so = sl ? (uint32_t)(r0 * H + lane) * 4u : kOOB;
  g.s0 = buf_f32(S.p0, so);
  g.s1 = buf_f32(S.p1, so);
  g.s2 = buf_f32(S.p2, so);
  g.flag = buf_u8(S.flag, lane < kPD && r0 + lane < S.re ? (uint32_t)(r0 + lane) : kOOB);
#pragma unroll
  for (int t = 0; t < kPD; ++t) {
    const uint32_t ro = r0 + t < S.re ? ((uint32_t)(r0 + t) * D + lane * V) * (uint32_t)sizeof(T)
                                      : kOOB;
    if (NT > 0) bld_row<T, V>(S.t0, ro, g.rows[0][t]);
    if (NT > 1) bld_row<T, V>(S.t1, ro, g.rows[NT > 1 ? 1 : 0][t]);
  }
}

// A sub-group: rows [t0, t1) of a group whose edges fill <= 64 (edge, head) slots (M * H
// <= 64, so one row always fits).  Slot lane k = (edge Es + k / H, head k % H): its row t,
// the row's slot segment [sk, ek) (stride H) and column j.
struct Slot {
  int t, sk, ek;
  int32_t j;
  bool valid;
};

template <int H>
__device__ __forceinline__ Slot slot_of(int32_t rp, int t0, int t1, int32_t Es, int nEs,
                                        int32_t E0, const int32_t* cols, int lane, int M) {
  Slot sl;
  const int q = lane / H, h = lane % H;
  sl.valid = lane < nEs * H;
  int t = t0;
#pragma unroll
  for (int u = 1; u < kPD; ++u)
    if (u > t0 && u < t1) t += rdlane(rp, u) <= Es + q ? 1 : 0;
  sl.t = t;
  sl.sk = (__shfl(rp, t) - Es) * H + h;
  sl.ek = (__shfl(rp, t + 1) - Es) * H;
  sl.j = min(max(cols[(Es - E0 + q) & (64 * kColPages - 1)], 0), M - 1);
  return sl;
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
__device__ __forceinline__ float swap32(float v, int lane) {
  const unsigned x = __builtin_bit_cast(unsigned, v);
  const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  return __builtin_bit_cast(float, lane < 32 ? r[1] : r[0]);
}
template <int H, bool MAX>
__device__ __forceinline__ float head_allreduce(float v, int lane) {
  auto op = [](float a, float b) { return MAX ? fmaxf(a, b) : a + b; };
  if (H <= 8) v = op(v, ror16<8>(v));
  if (H <= 4) v = op(v, ror16<4>(v));
  if (H <= 2) v = op(v, ror16<2>(v));
  if (H <= 1) v = op(v, ror16<1>(v));
  v = op(v, swap16(v, lane));
  return op(v, swap32(v, lane));
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

// segmented reductions over a row's slots (lanes sk, sk + H, ... < ek): every lane ends
// up with its segment's total (doubling toward the segment end, then the head's value)
template <int H>
__device__ __forceinline__ float seg_max(float v, int lane, int sk, int ek) {
#pragma unroll
  for (int o = H; o < 64; o <<= 1) {
    const float w = __shfl_down(v, o);
    if (lane + o < ek) v = fmaxf(v, w);
  }
  return __shfl(v, sk);
}
template <int H>
__device__ __forceinline__ float seg_sum(float v, int lane, int sk, int ek) {
#pragma unroll
  for (int o = H; o < 64; o <<= 1) {
    const float w = __shfl_down(v, o);
    if (lane + o < ek) v += w;
  }
  return __shfl(v, sk);
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

// per-row all-reduce over a sub-group's slot lanes (rows t0 <= r < t1, independent, so
// their chains interleave): rowv[r] = the value of (row r, this lane's head); returns the
// value of this slot's own row
template <int H, bool MAX>
__device__ __forceinline__ float rows_reduce(float x, int slot_t, bool valid, int t0, int t1,
                                             int lane, float (&rowv)[kPD]) {
  const float idn = MAX ? -INFINITY : 0.f;
  float out = idn;
#pragma unroll
  for (int r = 0; r < kPD; ++r) {
    if (r >= t0 && r < t1) {
      const float y = head_allreduce<H, MAX>(valid && slot_t == r ? x : idn, lane);
      rowv[r] = y;
      out = slot_t == r ? y : out;
    }
  }
  return out;
}

// keep factor of element e * H + h = Es * H + k of the edge-dropout stream (the other
// edge kernels' element order)
__device__ __forceinline__ float slot_keep(const Dropout& dp, uint64_t doff, int32_t Es, int H,
                                           int lane) {
  if (!dp.active) return 1.f;
  return philox_x(dp.seed, doff, (uint64_t)Es * H + (uint64_t)lane) >= dp.threshold ? dp.scale
                                                                                    : 0.f;
}

// the sub-group after t0: rows while their edges fit 64 slots
template <int H>
__device__ __forceinline__ int sub_end(int32_t rp, int t0, int lane) {
  const int32_t Es = rdlane(rp, t0);
  const uint64_t fit = __ballot(lane > t0 && lane <= kPD && rp - Es <= 64 / H);
  return t0 + max(1, (int)__popcll(fit));
}

// ------------------------------------------------------------------------ forward ---
// u_i = sum_e attd_e hc_j, lse_i, (ATTD: attd_e), and with HS the block partials of
// v_j = sum_e attd_e hs_i.  attd_e = softmax_row(lrelu(el_i + er_j))_e * keep_e.
// Per sub-group: scores, the row softmax (segmented max / sum across slot lanes) and keep
// bits once per slot; then per row and edge pair independent LDS reads (attention, hc_j)
// and the v slab update.  The next group's loads are in flight meanwhile.
template <int H, int F, typename T, bool HS, bool ATTD>
__global__ void __launch_bounds__(kWaves * 64) bip_fwd_kernel(
    const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
    const uint8_t* __restrict__ rowflag, int32_t n_rows, int32_t n_cols, int32_t n_edges,
    const float* __restrict__ el, const float* __restrict__ er, const T* __restrict__ hc,
    const T* __restrict__ hs, float slope, Dropout dp, T* __restrict__ u,
    T* __restrict__ u_lo, float* __restrict__ lse, float* __restrict__ attd,
    float* __restrict__ part) {
  constexpr int D = H * F, V = D / 64, QH = F / V, PD = kPD, WB = kWaves;
  constexpr int NT = HS ? 1 : 0;
  constexpr int SLAB = HS ? kMaxMD : 0;
  constexpr int NCOL = 64 * kColPages;
  constexpr int NATT = ATTD ? kPD * 64 : 0;  // a group's slots (<= kPD * M * H)
  constexpr int PER_WAVE = SLAB + NCOL + 64 + 64 + NATT;
  __shared__ __attribute__((aligned(16))) float smem[kMaxMD + 64 + WB * PER_WAVE];
  const int M = n_cols, MD = M * D;
  float* tab = smem;
  float* ert = smem + kMaxMD;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  float* slab = smem + kMaxMD + 64 + wv * PER_WAVE;
  int32_t* cols = reinterpret_cast<int32_t*>(slab + SLAB);
  float* scr = reinterpret_cast<float*>(cols + NCOL);
  float* lses = scr + 64;
  float* atts = lses + 64;
  for (int i = tid; i < MD; i += WB * 64) tab[i] = to_f32(hc[i]);
  for (int i = tid; i < M * H; i += WB * 64) ert[i] = er[i];
  if (HS)
    for (int i = lane; i < MD; i += 64) slab[i] = 0.f;
  __syncthreads();

  const int hl = lane * V / F;
  const uint64_t doff = dp.active ? dropout_offset(dp, dp.offset) : 0;
  const int64_t W = (int64_t)gridDim.x * WB, w = (int64_t)blockIdx.x * WB + wv;
  const int32_t rb = (int32_t)(w * n_rows / W), re = (int32_t)((w + 1) * n_rows / W);
  const uint32_t TB = (uint32_t)n_rows * D * (uint32_t)sizeof(T);
  Srcs S;
  S.rp = make_rsrc(rowptr, (uint32_t)(n_rows + 1) * 4u);
  S.col = make_rsrc(col, (uint32_t)n_edges * 4u);
  S.flag = make_rsrc(rowflag, (uint32_t)n_rows);
  S.p0 = make_rsrc(el, (uint32_t)n_rows * H * 4u);
  S.p1 = S.p2 = make_rsrc(nullptr, 0);
  S.t0 = make_rsrc(HS ? hs : nullptr, TB);
  S.t1 = make_rsrc(nullptr, 0);
  S.re = re;
  const rsrc_t r_u = make_rsrc(u, TB);
  const rsrc_t r_ulo = make_rsrc(sizeof(T) == 2 ? u_lo : nullptr, TB);
  const rsrc_t r_lse = make_rsrc(lse, (uint32_t)n_rows * H * 4u);
  const rsrc_t r_att = make_rsrc(ATTD ? attd : nullptr, (uint32_t)n_edges * H * 4u);
  if (rb < re) {
    using Gp = Grp<V, NT>;
    const int ng = (re - rb + PD - 1) / PD;
    Gp nxt;
    load_grp<H, V, NT, T>(nxt, S, rb, load_rp(S, rb, lane), lane);
    int32_t rp_n = load_rp(S, rb + PD, lane);
    for (int gi = 0; gi < ng; ++gi) {
      const int32_t r0 = rb + gi * PD;
      const Gp cur = nxt;  // this group's loads (issued one group ago)
      load_grp<H, V, NT, T>(nxt, S, r0 + PD, rp_n, lane);
      rp_n = load_rp(S, r0 + 2 * PD, lane);

      const int32_t E0 = rdlane(cur.rp, 0);
#pragma unroll
      for (int p = 0; p < kColPages; ++p) cols[64 * p + lane] = cur.colv[p];
      const uint64_t vmask = __ballot(lane < PD && cur.flag != 0);
      lses[lane] = -INFINITY;  // rows without edges (and no virtual row)
      float acc[PD][V];
#pragma unroll
      for (int t = 0; t < PD; ++t)
#pragma unroll
        for (int v = 0; v < V; ++v) acc[t][v] = 0.f;
      for (int t0 = 0; t0 < PD;) {
        const int t1 = sub_end<H>(cur.rp, t0, lane);
        const int32_t Es = rdlane(cur.rp, t0);
        const int nEs = min(64 / H, rdlane(cur.rp, t1) - Es);
        // (1) slot lanes: score, row softmax, keep, attention
        const Slot sl = slot_of<H>(cur.rp, t0, t1, Es, nEs, E0, cols, lane, M);
        {
          const int h = lane % H;
          const float elv = __shfl(cur.s0, sl.t * H + h);
          const bool virt = (vmask >> sl.t) & 1ull;
          const float sc = sl.valid ? (virt ? 0.f : lrelu(elv + ert[sl.j * H + h], slope)) : -INFINITY;
          const float mx = seg_max<H>(sc, lane, sl.sk, sl.ek);
          const float pe = sl.valid ? __expf(sc - mx) : 0.f;
          const float sm = seg_sum<H>(pe, lane, sl.sk, sl.ek);
          const float ad = sl.valid ? pe / sm * slot_keep(dp, doff, Es, H, lane) : 0.f;
          if (sl.valid && lane == sl.sk) lses[sl.t * H + h] = mx + __logf(sm);
          scr[lane] = ad;
          if (ATTD && sl.valid) atts[((Es - E0) * H + lane) & (NATT > 0 ? NATT - 1 : 0)] = ad;
        }
        // (2) element lanes: u_i and the v slab of the sub-group's rows, two edges a step
#pragma unroll
        for (int t = 0; t < PD; ++t) {
          if (t >= t0 && t < t1) {
            const int32_t s = rdlane(cur.rp, t), e1 = rdlane(cur.rp, t + 1);
            for (int32_t e = s; e < e1; e += 2) {
              const bool two = e + 1 < e1;
              const int32_t q0 = e - Es;
              const int32_t j0 = rdlane(sl.j, q0 * H);
              const int32_t j1 = rdlane(sl.j, (two ? q0 + 1 : q0) * H);
              const float a0 = scr[q0 * H + hl];
              const float a1 = two ? scr[(q0 + 1) * H + hl] : 0.f;
              float x0[V], x1[V];
              ld_row<V>(tab + j0 * D + lane * V, x0);
              ld_row<V>(tab + j1 * D + lane * V, x1);
#pragma unroll
              for (int v = 0; v < V; ++v) acc[t][v] = fmaf(a1, x1[v], fmaf(a0, x0[v], acc[t][v]));
              if (HS) {
                float* sp0 = slab + j0 * D + lane * V;
                float y[V];
                ld_row<V>(sp0, y);
#pragma unroll
                for (int v = 0; v < V; ++v) y[v] = fmaf(a0, cur.rows[0][t][v], y[v]);
                st_row<V>(sp0, y);
                if (two) {
                  float* sp1 = slab + j1 * D + lane * V;
                  ld_row<V>(sp1, y);
#pragma unroll
                  for (int v = 0; v < V; ++v) y[v] = fmaf(a1, cur.rows[0][t][v], y[v]);
                  st_row<V>(sp1, y);
                }
              }
            }
          }
        }
        t0 = t1;
      }
      // (3) the group's stores, a fixed set (masked lanes dropped)
#pragma unroll
      for (int t = 0; t < PD; ++t) {
        const uint32_t ro = r0 + t < re ? ((uint32_t)(r0 + t) * D + lane * V) * (uint32_t)sizeof(T)
                                        : kOOB;
        bst_row<T, V>(r_u, ro, acc[t]);
        if (sizeof(T) == 2) {
          float res[V];
#pragma unroll
          for (int v = 0; v < V; ++v) res[v] = acc[t][v] - (float)(bf16_t)acc[t][v];
          bst_row<T, V>(r_ulo, ro, res);
        }
      }
      const bool lr = lane < PD * H && r0 + lane / H < re;
      buf_store_f32(r_lse, lr ? (uint32_t)(r0 * H + lane) * 4u : kOOB, lses[lane]);
      if (ATTD) {
        const int32_t nE = rdlane(cur.rp, PD) - E0;
#pragma unroll
        for (int p = 0; p < (NATT > 0 ? NATT / 64 : 1); ++p) {
          const int32_t sidx = 64 * p + lane;
          buf_store_f32(r_att, sidx < nE * H ? (uint32_t)(E0 * H + sidx) * 4u : kOOB,
                        atts[sidx & (NATT > 0 ? NATT - 1 : 0)]);
        }
      }
    }
  }
  if (HS) {
    __syncthreads();
    float* dst = part + (int64_t)blockIdx.x * MD;
    const float* slabs = smem + kMaxMD + 64;
    for (int i = tid; i < MD; i += WB * 64) {
      float a = slabs[i];
#pragma unroll
      for (int q = 1; q < WB; ++q) a += slabs[q * PER_WAVE + i];
      dst[i] = a;
    }
  }
}

// ----------------------------------------------------------------------- backward ---
// Per row i, head h (reference: the autograd of Ablation.py:266-274, Ours.py:84-86):
//   g_e  = dU_i . hc_j (+ hs_i . dV_j) (+ coef_i exp(attd_e))
//   D_i  = sum_e attd_e g_e
//   ds_e = att_e (keep_e g_e - D_i),  de_e = ds_e lrelu'(pre_e),  d_el_i = sum_e de_e
//   d_hs_i = sum_e attd_e dV_j;  block partials of d_hc_j = sum attd_e dU_i, d_er_j = sum de_e
// Per sub-group: slot lanes give att, keep; element lanes give g_e (dots over the head's
// lanes), d_hs and the d_hc slab; slot lanes finish D, de, d_el (segmented sums) and add
// de into the d_er slab one row at a time (a row's columns are distinct).
template <int H, int F, typename T, bool HS, bool COEF>
__global__ void __launch_bounds__(kWaves * 64) bip_bwd_kernel(
    const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
    const uint8_t* __restrict__ rowflag, int32_t n_rows, int32_t n_cols, int32_t n_edges,
    const float* __restrict__ el, const float* __restrict__ er, const T* __restrict__ hc,
    const float* __restrict__ lse, const T* __restrict__ dU, const T* __restrict__ hs,
    const T* __restrict__ dV, const float* __restrict__ row_coef, float slope, Dropout dp,
    float* __restrict__ d_el, T* __restrict__ d_hs, float* __restrict__ part) {
  constexpr int D = H * F, V = D / 64, QH = F / V, PD = kPD, WB = kWaves;
  constexpr int NT = HS ? 2 : 1;
  constexpr int NCOL = 64 * kColPages;
  constexpr int PER_WAVE = kMaxMD + 64 + NCOL + 3 * 64;  // d_hc, d_er slabs; cols; scratch
  __shared__ __attribute__((aligned(16))) float smem[2 * kMaxMD + 64 + WB * PER_WAVE];
  const int M = n_cols, MD = M * D, MH = M * H;
  float* tab = smem;
  float* tdv = smem + kMaxMD;
  float* ert = smem + 2 * kMaxMD;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  float* slab = smem + 2 * kMaxMD + 64 + wv * PER_WAVE;
  float* sder = slab + kMaxMD;
  int32_t* cols = reinterpret_cast<int32_t*>(sder + 64);
  float* sad = reinterpret_cast<float*>(cols + NCOL);
  float* sg = sad + 64;
  float* dels = sg + 64;
  for (int i = tid; i < MD; i += WB * 64) {
    tab[i] = to_f32(hc[i]);
    if (HS) tdv[i] = to_f32(dV[i]);
  }
  for (int i = tid; i < MH; i += WB * 64) ert[i] = er[i];
  for (int i = lane; i < MD; i += 64) slab[i] = 0.f;
  sder[lane] = 0.f;
  __syncthreads();

  const int hl = lane * V / F;
  const bool lead = lane % QH == 0;
  const uint64_t doff = dp.active ? dropout_offset(dp, dp.offset) : 0;
  const int64_t W = (int64_t)gridDim.x * WB, w = (int64_t)blockIdx.x * WB + wv;
  const int32_t rb = (int32_t)(w * n_rows / W), re = (int32_t)((w + 1) * n_rows / W);
  const uint32_t TB = (uint32_t)n_rows * D * (uint32_t)sizeof(T);
  Srcs S;
  S.rp = make_rsrc(rowptr, (uint32_t)(n_rows + 1) * 4u);
  S.col = make_rsrc(col, (uint32_t)n_edges * 4u);
  S.flag = make_rsrc(rowflag, (uint32_t)n_rows);
  S.p0 = make_rsrc(el, (uint32_t)n_rows * H * 4u);
  S.p1 = make_rsrc(lse, (uint32_t)n_rows * H * 4u);
  S.p2 = make_rsrc(COEF ? row_coef : nullptr, (uint32_t)n_rows * H * 4u);
  S.t0 = make_rsrc(dU, TB);
  S.t1 = make_rsrc(HS ? hs : nullptr, TB);
  S.re = re;
  const rsrc_t r_dhs = make_rsrc(HS ? d_hs : nullptr, TB);
  const rsrc_t r_del = make_rsrc(d_el, (uint32_t)n_rows * H * 4u);
  float der = 0.f;  // d_er of (column lane / H, head lane % H) over the wave's edges
  if (rb < re) {
    using Gp = Grp<V, NT>;
    const int ng = (re - rb + PD - 1) / PD;
    Gp nxt;
    load_grp<H, V, NT, T>(nxt, S, rb, load_rp(S, rb, lane), lane);
    int32_t rp_n = load_rp(S, rb + PD, lane);
    for (int gi = 0; gi < ng; ++gi) {
      const int32_t r0 = rb + gi * PD;
      const Gp cur = nxt;
      load_grp<H, V, NT, T>(nxt, S, r0 + PD, rp_n, lane);
      rp_n = load_rp(S, r0 + 2 * PD, lane);

      const int32_t E0 = rdlane(cur.rp, 0);
#pragma unroll
      for (int p = 0; p < kColPages; ++p) cols[64 * p + lane] = cur.colv[p];
      const uint64_t vmask = __ballot(lane < PD && cur.flag != 0);
      dels[lane] = 0.f;  // rows without edges (and no virtual row)
      float wacc[PD][V];
#pragma unroll
      for (int t = 0; t < PD; ++t)
#pragma unroll
        for (int v = 0; v < V; ++v) wacc[t][v] = 0.f;
      for (int t0 = 0; t0 < PD;) {
        const int t1 = sub_end<H>(cur.rp, t0, lane);
        const int32_t Es = rdlane(cur.rp, t0);
        const int nEs = min(64 / H, rdlane(cur.rp, t1) - Es);
        // (1) slot lanes: score, attention, keep
        const Slot sl = slot_of<H>(cur.rp, t0, t1, Es, nEs, E0, cols, lane, M);
        const int h = lane % H;
        const int rsl = sl.t * H + h;
        const bool virt = (vmask >> sl.t) & 1ull;
        // (the row scalars live on lanes t * H + h, which may be idle slot lanes: every
        // shuffle runs with all lanes active -- ds_bpermute reads 0 from an inactive lane)
        const float elq = __shfl(cur.s0, rsl), lsq = __shfl(cur.s1, rsl);
        const float cfq = COEF ? __shfl(cur.s2, rsl) : 0.f;
        const float pre = elq + ert[sl.j * H + h];
        const float sc = virt ? 0.f : lrelu(pre, slope);
        const float att = sl.valid ? __expf(sc - lsq) : 0.f;
        const float kf = slot_keep(dp, doff, Es, H, lane);
        const float ad = att * kf;
        sad[lane] = ad;
        // (2) element lanes: g_e, d_hs, the d_hc slab
#pragma unroll
        for (int t = 0; t < PD; ++t) {
          if (t >= t0 && t < t1) {
            const int32_t s = rdlane(cur.rp, t), e1 = rdlane(cur.rp, t + 1);
            const float(&dUr)[V] = cur.rows[0][t];
            const float(&hsr)[V] = cur.rows[NT - 1][t];
            for (int32_t e = s; e < e1; e += 2) {
              const bool two = e + 1 < e1;
              const int32_t q0 = e - Es;
              const int32_t j0 = rdlane(sl.j, q0 * H);
              const int32_t j1 = rdlane(sl.j, (two ? q0 + 1 : q0) * H);
              const float a0 = sad[q0 * H + hl];
              const float a1 = two ? sad[(q0 + 1) * H + hl] : 0.f;
              float x0[V], x1[V];
              ld_row<V>(tab + j0 * D + lane * V, x0);
              ld_row<V>(tab + j1 * D + lane * V, x1);
              float p0 = 0.f, p1 = 0.f;
#pragma unroll
              for (int v = 0; v < V; ++v) {
                p0 = fmaf(dUr[v], x0[v], p0);
                p1 = fmaf(dUr[v], x1[v], p1);
              }
              if (HS) {
                float y0[V], y1[V];
                ld_row<V>(tdv + j0 * D + lane * V, y0);
                ld_row<V>(tdv + j1 * D + lane * V, y1);
#pragma unroll
                for (int v = 0; v < V; ++v) {
                  p0 = fmaf(hsr[v], y0[v], p0);
                  p1 = fmaf(hsr[v], y1[v], p1);
                  wacc[t][v] = fmaf(a1, y1[v], fmaf(a0, y0[v], wacc[t][v]));
                }
              }
              if constexpr (QH == 32) {
                const float gp = pair_sum32(p0, p1, lane);
                if (lane % 16 == 0 && (two || (lane & 16) == 0))
                  sg[(q0 + ((lane >> 4) & 1)) * H + hl] = gp;
              } else {
                const float g0 = lanes_sum<QH>(p0, lane), g1 = lanes_sum<QH>(p1, lane);
                if (lead) {
                  sg[q0 * H + hl] = g0;
                  if (two) sg[(q0 + 1) * H + hl] = g1;
                }
              }
              float z[V];
              float* sp0 = slab + j0 * D + lane * V;
              ld_row<V>(sp0, z);
#pragma unroll
              for (int v = 0; v < V; ++v) z[v] = fmaf(a0, dUr[v], z[v]);
              st_row<V>(sp0, z);
              if (two) {
                float* sp1 = slab + j1 * D + lane * V;
                ld_row<V>(sp1, z);
#pragma unroll
                for (int v = 0; v < V; ++v) z[v] = fmaf(a1, dUr[v], z[v]);
                st_row<V>(sp1, z);
              }
            }
          }
        }
        // (3) slot lanes: D_i, de_e, d_el_i, the d_er slab
        {
          float g = sg[lane];
          if (COEF && sl.valid) g = fmaf(cfq, expf(ad), g);
          const float Dq = seg_sum<H>(sl.valid ? ad * g : 0.f, lane, sl.sk, sl.ek);
          const float ds = att * (g * kf - Dq);
          const float dev = sl.valid && !virt ? ds * (pre > 0.f ? 1.f : slope) : 0.f;
          const float del = seg_sum<H>(dev, lane, sl.sk, sl.ek);
          if (sl.valid && lane == sl.sk) dels[rsl] = del;
          // d_er in registers, lane j * H + h (M * H <= 64), edges in order
          for (int q = 0; q < nEs; ++q) {
            const int32_t jq = rdlane(sl.j, q * H);
            float dq = 0.f;
#pragma unroll
            for (int hh = 0; hh < H; ++hh) {
              const float v = __builtin_bit_cast(float, rdlane(__builtin_bit_cast(int32_t, dev), q * H + hh));
              dq = lane % H == hh ? v : dq;
            }
            der += lane / H == jq ? dq : 0.f;
          }
        }
        t0 = t1;
      }
      // (4) the group's stores, a fixed set (masked lanes dropped)
      if (HS) {
#pragma unroll
        for (int t = 0; t < PD; ++t) {
          const uint32_t ro = r0 + t < re
                                  ? ((uint32_t)(r0 + t) * D + lane * V) * (uint32_t)sizeof(T)
                                  : kOOB;
          bst_row<T, V>(r_dhs, ro, wacc[t]);
        }
      }
      const bool lr = lane < PD * H && r0 + lane / H < re;
      buf_store_f32(r_del, lr ? (uint32_t)(r0 * H + lane) * 4u : kOOB, dels[lane]);
    }
  }
  sder[lane] = der;
  __syncthreads();
  float* dst = part + (int64_t)blockIdx.x * (MD + MH);
  const float* base = smem + 2 * kMaxMD + 64;
  for (int i = tid; i < MD + MH; i += WB * 64) {
    const int o = i < MD ? i : kMaxMD + (i - MD);
    float a = base[o];
#pragma unroll
    for (int q = 1; q < WB; ++q) a += base[q * PER_WAVE + o];
    dst[i] = a;
  }
}

// out[i] = sum_b part[b][i] in block order (i < n_t -> out_t as T, else out_f fp32).
// A block owns 16 consecutive entries; its 64 streams (lane / 16 of each wave, wave-major)
// sum contiguous block ranges (every load of a stream in flight at once), then the
// stream sums add in stream order.  256 blocks at M x H x F = 4096: the whole chip reads
// the partials (64 blocks of one 64-entry slice each ran latency-bound, 6.6 us).
template <typename T>
__global__ void __launch_bounds__(1024) bip_reduce_kernel(const float* __restrict__ part,
                                                          int32_t nb, int32_t stride,
                                                          int32_t n_t, T* __restrict__ out_t,
                                                          float* __restrict__ out_f) {
  __shared__ float red[64][17];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = lane & 15, st = wv * 4 + (lane >> 4);  // entry in the slice, stream
  const int i = blockIdx.x * 16 + c;
  const int per = (nb + 63) / 64;
  const int b0 = st * per, b1 = min(nb, b0 + per);
  float a = 0.f;
  if (i < stride)
    for (int b = b0; b < b1; ++b) a += part[(int64_t)b * stride + i];
  red[st][c] = a;
  __syncthreads();
  if (threadIdx.x < 16 && i < stride) {
    float sum = red[0][c];
#pragma unroll 8
    for (int q = 1; q < 64; ++q) sum += red[q][c];
    if (i < n_t) out_t[i] = from_f32<T>(sum);
    else out_f[i - n_t] = sum;
  }
}

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
  const size_t rec = (size_t)g->n_cols * ((size_t)heads * feat + heads);
  return (size_t)bip::cu_count() * rec * sizeof(float) + 256;
}

template <int H, int F, typename T>
static void bip_launch_fwd(const msha_graph* g, const float* el, const float* er, const void* hc,
                           const void* hs, float slope, const Dropout& dp, void* u, void* u_lo,
                           float* lse, float* attd, void* v, float* part, int nb, hipStream_t s) {
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(nb), dim3(bip::kWaves * 64), 0, s, g->rowptr, g->col,
                       g->rowflag, (int32_t)g->n_rows, (int32_t)g->n_cols, (int32_t)g->n_edges,
                       el, er, (const T*)hc, (const T*)hs, slope, dp, (T*)u, (T*)u_lo, lse, attd,
                       part);
  };
  if (hs != nullptr) {
    if (attd != nullptr) go(bip::bip_fwd_kernel<H, F, T, true, true>);
    else go(bip::bip_fwd_kernel<H, F, T, true, false>);
    const int32_t MD = (int32_t)(g->n_cols * H * F);
    hipLaunchKernelGGL(bip::bip_reduce_kernel<T>, dim3((MD + 15) / 16), dim3(1024), 0, s, part,
                       nb, MD, MD, (T*)v, (float*)nullptr);
  } else {
    if (attd != nullptr) go(bip::bip_fwd_kernel<H, F, T, false, true>);
    else go(bip::bip_fwd_kernel<H, F, T, false, false>);
  }
}

template <int H, int F, typename T>
static void bip_launch_bwd(const msha_graph* g, const float* el, const float* er, const void* hc,
                           const float* lse, const void* dU, const void* hs, const void* dV,
                           const float* row_coef, float slope, const Dropout& dp, float* d_el,
                           float* d_er, void* d_hc, void* d_hs, float* part, int nb,
                           hipStream_t s) {
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(nb), dim3(bip::kWaves * 64), 0, s, g->rowptr, g->col,
                       g->rowflag, (int32_t)g->n_rows, (int32_t)g->n_cols, (int32_t)g->n_edges,
                       el, er, (const T*)hc,
                       lse, (const T*)dU, (const T*)hs, (const T*)dV, row_coef, slope, dp, d_el,
                       (T*)d_hs, part);
  };
  const bool hsb = dV != nullptr, cf = row_coef != nullptr;
  if (hsb && cf) go(bip::bip_bwd_kernel<H, F, T, true, true>);
  else if (hsb) go(bip::bip_bwd_kernel<H, F, T, true, false>);
  else if (cf) go(bip::bip_bwd_kernel<H, F, T, false, true>);
  else go(bip::bip_bwd_kernel<H, F, T, false, false>);
  const int32_t MD = (int32_t)(g->n_cols * H * F), MH = (int32_t)(g->n_cols * H);
  hipLaunchKernelGGL(bip::bip_reduce_kernel<T>, dim3((MD + MH + 15) / 16), dim3(1024), 0, s, part,
                     nb, MD + MH, MD, (T*)d_hc, d_er);
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
