// Fused edge-softmax + attention-weighted aggregation for gfx950.
//
// Reference op chain (dense in the reference, sparse here):
//   Ablation.py:266-267  e12 = lrelu(cat(h1_j, h2_i) @ a)        -> el_i + er_j per edge
//   Ablation.py:268-271  where(adj>0, e12, -9e15); softmax; dropout -> segmented softmax
//   Ablation.py:274      u = att @ h1                             -> CSR gather-aggregate
//   Ablation.py:273      v = att.t() @ h2                         -> CSC aggregate
//   + the autograd backward of all of the above.
//
// Layout of work on a 64-lane wavefront (one CSR row per wave at a time):
//   score layout  : lane = e_s * H + h_s   (CE = 64/H edges x H heads per chunk)
//   gather layout : lane = g_e * NQ + q    (NQ = H*F/4 float4 quads per feature row,
//                                           EPI = 64/NQ edges per wave-instruction,
//                                           16 B per lane, whole rows per instruction)
// Scores/softmax statistics live in the score layout and reach the gather lanes
// through ds_bpermute (__shfl).  The forward is single-pass (online softmax with
// per-head rescale of the accumulators) and stores only log-sum-exp per
// (row, head); the backward recomputes the attention from it and uses
// sum_e att_e * g_e = dU_i . u_i (FlashAttention's "D" identity), so the row
// pass needs no second sweep over the gathered rows.
#include <stdlib.h>

#include <cstdlib>

#include "common.h"
#include "edge_geo.h"

#ifndef COLS_EH
#define COLS_EH 1
#endif
#ifndef DE_SLOT_MIN_BYTES
#define DE_SLOT_MIN_BYTES (192ll << 20)
#endif
#ifndef COLS_WIDE_UG
#define COLS_WIDE_UG 4  // wide-row column pass: edges whose dU rows are in flight together
#endif
#ifndef COLS_EPI_BUF
#define COLS_EPI_BUF 1  // the buffer-load batch above for EPI > 1 too
#endif
#ifndef COLS_NARROW_UG
#define COLS_NARROW_UG 8  // gather instructions in flight together when EPI > 1
#endif
#ifndef COLS_NG
#define COLS_NG 2  // slot groups whose loads are in flight together in the column pass
#endif

namespace msha {

// ------------------------------------------------------------------ forward ---
// EPL = edges per lane in the score layout: a chunk covers EPL * 64/H edges, so the
// per-chunk max / sum reductions, the accumulator rescale and the loop overhead are
// amortised over EPL times as many edges (the bf16 kernel is issue-bound).
template <int H, int F, typename T, int EPL>
__global__ void __launch_bounds__(256) edge_attn_fwd_kernel(
    const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
    const uint8_t* __restrict__ rowflag, int64_t n_rows, const float* __restrict__ el,
    const float* __restrict__ er, const T* __restrict__ hc, float slope, Dropout dp,
    T* __restrict__ u, T* __restrict__ u_lo, float* __restrict__ lse, float* __restrict__ attd) {
  using G = Geo<H, F, T>;
  constexpr int CEL = EPL * G::CE;  // edges per chunk
  const int lane = lane_id();
  const int e_s = lane / H, h_s = lane % H;
  const int g_e = G::QPL == 1 ? lane / G::NQ : 0;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;

  // Software pipeline (the kernel is latency-bound per row: rowptr -> col -> er ->
  // gathers): the next row's bounds, flag, el and first two chunks' columns are loaded
  // while this row runs, and inside a row the columns two chunks ahead and the er one
  // chunk ahead are in flight during the current chunk's gathers.
  int64_t row = wave;
  if (row >= n_rows) return;
  int32_t start = rowptr[row], end = rowptr[row + 1];
  bool virt = rowflag != nullptr && rowflag[row] != 0;
  float elh = el[row * H + h_s];
  int32_t j0[EPL], j1[EPL];
#pragma unroll
  for (int t = 0; t < EPL; ++t) {
    const int32_t e0 = start + t * G::CE + e_s, e1 = e0 + CEL;
    j0[t] = e0 < end ? col[e0] : 0;
    j1[t] = e1 < end ? col[e1] : 0;
  }
  while (true) {
    const int64_t nrow = row + nwaves;
    const bool has_next = nrow < n_rows;
    const int32_t nstart = has_next ? rowptr[nrow] : 0;
    const int32_t nend = has_next ? rowptr[nrow + 1] : 0;
    float m = -INFINITY, l = 0.f;
    Pk<T> acc[G::QPL];
#pragma unroll
    for (int k = 0; k < G::QPL; ++k) acc[k] = pk_zero<T>();
    float erv[EPL];
#pragma unroll
    for (int t = 0; t < EPL; ++t)
      erv[t] = start + t * G::CE + e_s < end ? er[(int64_t)j0[t] * H + h_s] : 0.f;

    for (int32_t cs = start; cs < end; cs += CEL) {
      int32_t j[EPL], j2[EPL];
      float ern[EPL], sc[EPL];
      bool valid[EPL];
      float smax = -INFINITY;
#pragma unroll
      for (int t = 0; t < EPL; ++t) {
        const int32_t e = cs + t * G::CE + e_s;
        valid[t] = e < end;
        j[t] = j0[t];
        j2[t] = e + 2 * CEL < end ? col[e + 2 * CEL] : 0;
        ern[t] = e + CEL < end ? er[(int64_t)j1[t] * H + h_s] : 0.f;
        sc[t] = valid[t] ? (virt ? 0.f : lrelu(elh + erv[t], slope)) : -INFINITY;
        smax = fmaxf(smax, sc[t]);
      }
      const float mn = fmaxf(m, wave_xor_max<H>(smax));
      const float alpha = __expf(m - mn);
      float w[EPL], psum = 0.f;
#pragma unroll
      for (int t = 0; t < EPL; ++t) {
        const float pe = valid[t] ? __expf(sc[t] - mn) : 0.f;
        psum += pe;
        w[t] = valid[t] ? pe * dropout_factor(dp, (uint64_t)(cs + t * G::CE + e_s) * H + h_s)
                        : 0.f;
      }
      l = fmaf(l, alpha, wave_xor_sum<H>(psum));
      m = mn;
#pragma unroll
      for (int k = 0; k < G::QPL; ++k) {
        const int hd = quad_of<G>(lane, k) / G::QH;
        acc[k] = pk_scale(acc[k], __shfl(alpha, hd));
      }
      const int nvalid = min(CEL, (int)(end - cs));
#pragma unroll
      for (int g = 0; g < CEL; g += G::EPI) {
        if (g >= nvalid) break;
        const int t = g / G::CE;        // half of the chunk (compile time)
        const int ei = g % G::CE + g_e;  // edge slot inside that half
        const int32_t jq = __shfl(j[t], ei * H);
#pragma unroll
        for (int k = 0; k < G::QPL; ++k) {
          const int q = quad_of<G>(lane, k);
          const float wq = __shfl(w[t], ei * H + q / G::QH);
          if (g + g_e < nvalid)
            acc[k] = pk_fma(wq, pk_load(hc + (int64_t)jq * G::D + G::V * q), acc[k]);
        }
      }
#pragma unroll
      for (int t = 0; t < EPL; ++t) {
        j0[t] = j1[t];
        j1[t] = j2[t];
        erv[t] = ern[t];
      }
    }
    // the next row's first loads go out before this row's epilogue
    bool nvirt = false;
    float nelh = 0.f;
    if (has_next) {
      nvirt = rowflag != nullptr && rowflag[nrow] != 0;
      nelh = el[nrow * H + h_s];
#pragma unroll
      for (int t = 0; t < EPL; ++t) {
        const int32_t e0 = nstart + t * G::CE + e_s, e1 = e0 + CEL;
        j0[t] = e0 < nend ? col[e0] : 0;
        j1[t] = e1 < nend ? col[e1] : 0;
      }
    }
    if (G::EPI > 1) {
#pragma unroll
      for (int o = G::NQ; o < 64; o <<= 1) acc[0] = pk_xor_add(acc[0], o);
    }
#pragma unroll
    for (int k = 0; k < G::QPL; ++k) {
      const int q = quad_of<G>(lane, k);
      const float lk = __shfl(l, q / G::QH);
      const float inv = lk > 0.f ? 1.f / lk : 0.f;
      if (g_e == 0) {
        const Pk<T> uk = pk_scale(acc[k], inv);
        pk_store(u + row * G::D + G::V * q, uk);
        if (sizeof(T) == 2 && u_lo != nullptr) pk_store(u_lo + row * G::D + G::V * q, pk_residual(uk));
      }
    }
    const float lse_h = l > 0.f ? m + __logf(l) : -INFINITY;
    if (lane < H) lse[row * H + lane] = lse_h;
    if (attd != nullptr) {
      for (int32_t cs = start; cs < end; cs += G::CE) {
        const int32_t e = cs + e_s;
        if (e < end) {
          const float sv = virt ? 0.f : lrelu(elh + er[(int64_t)col[e] * H + h_s], slope);
          attd[(int64_t)e * H + h_s] =
              __expf(sv - lse_h) * dropout_factor(dp, (uint64_t)e * H + h_s);
        }
      }
    }
    if (!has_next) break;
    row = nrow;
    start = nstart;
    end = nend;
    virt = nvirt;
    elh = nelh;
  }
}

// ------------------------------------------------------ forward, batched gathers ---
// Rows of at most 64 16-byte pieces (QPL == 1: every C4/R15 shape).  The same values in
// the same order as edge_attn_fwd_kernel (bitwise-identical u / lse), but every memory
// op of the chunk loop goes through a buffer descriptor (a masked lane reads 0), so the
// loop body is straight-line: the NGI gathers of a chunk leave back to back before the
// chunk's scores are reduced, and the compiler's vmcnt waits count them down instead of
// draining after each one (a divergent branch around a load forces vmcnt(0), which
// serialised the gathers of edge_attn_fwd_kernel to one in flight per wave).
// Issue order per chunk c: gathers(c), er(c+1), col(c+2); the softmax of c uses er(c),
// issued a chunk earlier, so it runs while the gathers are in flight.
// Row bounds are wave-uniform (readfirstlane): scalar loads and scalar loop control.
// Needs every table below 2 GiB (the dispatcher checks and otherwise runs the above).
//
// RT (row terms for the backward's d_el, large graphs): with c_ij = lrelu'(el_i + er_j)
// (1 or slope), the kernel also accumulates uc_i = sum_j c_ij attd_ij hc_j (fp32, N x D)
// and qc_i = sum_j c_ij att_ij (N x H, pre-dropout probabilities), by the same online
// rescale as u and l.  Then d_el_i = dU_i . uc_i - D_i qc_i per head (D_i = dU_i . u_i),
// which is sum_j de_ij rearranged: the fused backward needs no per-edge de crossing
// from CSC to CSR order (bwd_row_stats_kernel<RT> finishes d_el in its row pass).
template <int H, int F, typename T, int EPL, bool RT = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(FWD_WPE)))
edge_attn_fwd_bat_kernel(
    const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
    const uint8_t* __restrict__ rowflag, int32_t n_rows, int32_t n_cols, int32_t n_edges,
    const float* __restrict__ el, const float* __restrict__ er, const T* __restrict__ hc,
    float slope, Dropout dp, T* __restrict__ u, T* __restrict__ u_lo, float* __restrict__ lse,
    float* __restrict__ attd, float* __restrict__ uc, float* __restrict__ qc) {
  using G = Geo<H, F, T>;
  static_assert(G::QPL == 1, "batched forward: one 16-byte piece per lane");
  constexpr int CEL = EPL * G::CE;    // edges per chunk
  constexpr int NGI = CEL / G::EPI;   // gather instructions per chunk
  const int lane = lane_id();
  const int e_s = lane / H, h_s = lane % H;
  const int g_e = lane / G::NQ, q = lane % G::NQ;
  const rsrc_t r_col = make_rsrc(col, (uint32_t)n_edges * 4u);
  const rsrc_t r_er = make_rsrc(er, (uint32_t)n_cols * (4u * H));
  const rsrc_t r_hc = make_rsrc(hc, (uint32_t)n_cols * (uint32_t)(G::D * sizeof(T)));
  const uint32_t q_off = 16u * q;
  const int wave0 = __builtin_amdgcn_readfirstlane((int)(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6));
  const int nwaves = (int)(((int64_t)gridDim.x * blockDim.x) >> 6);

  // a wave walks rows row, row + nwaves, ... (one row when the grid covers them all);
  // the next row's bounds, flag, el and first columns load before this row's epilogue,
  // unconditionally (the last row reloads its own: no branch around the loads)
  int row = wave0;
  if (row >= n_rows) return;
  int32_t start = __builtin_amdgcn_readfirstlane(rowptr[row]);
  int32_t end = __builtin_amdgcn_readfirstlane(rowptr[row + 1]);
  bool virt = rowflag != nullptr && rowflag[row] != 0;
  float elh = el[(int64_t)row * H + h_s];
  int32_t j0[EPL], j1[EPL];
#pragma unroll
  for (int t = 0; t < EPL; ++t) {
    const int32_t e0 = start + t * G::CE + e_s, e1 = e0 + CEL;
    j0[t] = buf_i32(r_col, e0 < end ? (uint32_t)e0 * 4u : kOOB);
    j1[t] = buf_i32(r_col, e1 < end ? (uint32_t)e1 * 4u : kOOB);
  }
  while (true) {
    float erv[EPL];
#pragma unroll
    for (int t = 0; t < EPL; ++t)
      erv[t] = buf_f32(r_er, start + t * G::CE + e_s < end
                                 ? (uint32_t)j0[t] * (4u * H) + 4u * h_s : kOOB);
    float m = -INFINITY, l = 0.f, lc = 0.f;
    Pk<T> acc = pk_zero<T>(), accc = pk_zero<T>();
    float sc_keep[EPL];  // the last chunk's scores (record mode, one-chunk rows)
    for (int32_t cs = start; cs < end; cs += CEL) {
      const int nvalid = min(CEL, (int)(end - cs));
      // (1) this chunk's gathers, all in flight together
      u32x4_t raw[NGI];
#pragma unroll
      for (int gi = 0; gi < NGI; ++gi) {
        const int g = gi * G::EPI;
        const int t = g / G::CE;
        const int ei = g % G::CE + g_e;
        const int32_t jq = __shfl(j0[t], ei * H);
        raw[gi] = buf_b128(r_hc, g + g_e < nvalid
                                     ? (uint32_t)jq * (uint32_t)(G::D * sizeof(T)) + q_off
                                     : kOOB);
      }
      // (2) er one chunk ahead, col two chunks ahead
      float ern[EPL];
      int32_t j2[EPL];
#pragma unroll
      for (int t = 0; t < EPL; ++t) {
        const int32_t e1 = cs + CEL + t * G::CE + e_s, e2 = e1 + CEL;
        ern[t] = buf_f32(r_er, e1 < end ? (uint32_t)j1[t] * (4u * H) + 4u * h_s : kOOB);
        j2[t] = buf_i32(r_col, e2 < end ? (uint32_t)e2 * 4u : kOOB);
      }
      // (3) the chunk's online softmax (score layout), while the gathers fly
      float sc[EPL], cf[EPL], smax = -INFINITY;
      uint64_t cpos[EPL];  // RT: ballot of pre > 0 over the score lanes (edge * H + head)
      bool valid[EPL];
#pragma unroll
      for (int t = 0; t < EPL; ++t) {
        valid[t] = cs + t * G::CE + e_s < end;
        const float pre = elh + erv[t];
        sc[t] = valid[t] ? (virt ? 0.f : lrelu(pre, slope)) : -INFINITY;
        cf[t] = pre > 0.f ? 1.f : slope;  // the column pass's lrelu' (virtual rows: unused)
        if (RT) cpos[t] = __ballot(pre > 0.f);
        smax = fmaxf(smax, sc[t]);
        sc_keep[t] = sc[t];
      }
      const float mn = fmaxf(m, wave_xor_max<H>(smax));
      const float alpha = __expf(m - mn);
      float w[EPL], psum = 0.f, pcsum = 0.f;
#pragma unroll
      for (int t = 0; t < EPL; ++t) {
        const float pe = valid[t] ? __expf(sc[t] - mn) : 0.f;
        psum += pe;
        if (RT) pcsum = fmaf(pe, cf[t], pcsum);
        w[t] = valid[t] ? pe * dropout_factor(dp, (uint64_t)(cs + t * G::CE + e_s) * H + h_s)
                        : 0.f;
      }
      l = fmaf(l, alpha, wave_xor_sum<H>(psum));
      if (RT) lc = fmaf(lc, alpha, wave_xor_sum<H>(pcsum));
      m = mn;
      const float alpha_q = __shfl(alpha, q / G::QH);
      acc = pk_scale(acc, alpha_q);
      if (RT) accc = pk_scale(accc, alpha_q);
      // (4) accumulate in gather order (masked lanes carry w = 0 and a zero row)
#pragma unroll
      for (int gi = 0; gi < NGI; ++gi) {
        const int g = gi * G::EPI;
        const int t = g / G::CE;
        const int ei = g % G::CE + g_e;
        const float wq = __shfl(w[t], ei * H + q / G::QH);
        const Pk<T> xr = pk_from_raw(raw[gi], (T*)nullptr);
        acc = pk_fma(wq, xr, acc);
        if (RT) {  // lrelu' of this gather lane's (edge, head) from the ballot: no shuffle
          const float c = (cpos[t] >> (ei * H + q / G::QH)) & 1ull ? 1.f : slope;
          accc = pk_fma(wq * c, xr, accc);
        }
      }
#pragma unroll
      for (int t = 0; t < EPL; ++t) {
        j0[t] = j1[t];
        j1[t] = j2[t];
        erv[t] = ern[t];
      }
    }
    const int nrow_raw = row + nwaves;
    const bool has_next = nrow_raw < n_rows;
    const int nrow = has_next ? nrow_raw : row;
    const int32_t nstart = __builtin_amdgcn_readfirstlane(rowptr[nrow]);
    const int32_t nend = __builtin_amdgcn_readfirstlane(rowptr[nrow + 1]);
    const bool nvirt = rowflag != nullptr && rowflag[nrow] != 0;
    const float nelh = el[(int64_t)nrow * H + h_s];
    int32_t nj0[EPL], nj1[EPL];
#pragma unroll
    for (int t = 0; t < EPL; ++t) {
      const int32_t e0 = nstart + t * G::CE + e_s, e1 = e0 + CEL;
      nj0[t] = buf_i32(r_col, e0 < nend ? (uint32_t)e0 * 4u : kOOB);
      nj1[t] = buf_i32(r_col, e1 < nend ? (uint32_t)e1 * 4u : kOOB);
    }
    if (G::EPI > 1) {
#pragma unroll
      for (int o = G::NQ; o < 64; o <<= 1) acc = pk_xor_add(acc, o);
      if (RT) {
#pragma unroll
        for (int o = G::NQ; o < 64; o <<= 1) accc = pk_xor_add(accc, o);
      }
    }
    const float lk = __shfl(l, q / G::QH);
    const float inv = lk > 0.f ? 1.f / lk : 0.f;
    if (g_e == 0) {
      const Pk<T> uk = pk_scale(acc, inv);
      pk_store(u + (int64_t)row * G::D + G::V * q, uk);
      // bf16 tables: the rounding residual too, so the backward's D = dU . u is exact
      if (sizeof(T) == 2 && u_lo != nullptr)
        pk_store(u_lo + (int64_t)row * G::D + G::V * q, pk_residual(uk));
      if (RT) {  // uc in fp32 for either table type
        const Pk<T> ck = pk_scale(accc, inv);
        float* dst = uc + (int64_t)row * G::D + G::V * q;
#pragma unroll
        for (int v = 0; v < G::V; v += 4)
          *reinterpret_cast<float4*>(dst + v) = make_float4(ck.v[v], ck.v[v + 1], ck.v[v + 2], ck.v[v + 3]);
      }
    }
    const float lse_h = l > 0.f ? m + __logf(l) : -INFINITY;
    if (lane < H) lse[(int64_t)row * H + lane] = lse_h;
    if (RT && lane < H) qc[(int64_t)row * H + lane] = l > 0.f ? lc / l : 0.f;
    if (attd != nullptr && end - start <= CEL) {
      // one chunk (every R15 row): its scores are still in registers -- the same values
      // the reload below would recompute, without the col -> er round trips
#pragma unroll
      for (int t = 0; t < EPL; ++t) {
        const int32_t e = start + t * G::CE + e_s;
        if (e < end)
          attd[(int64_t)e * H + h_s] =
              __expf(sc_keep[t] - lse_h) * dropout_factor(dp, (uint64_t)e * H + h_s);
      }
    } else if (attd != nullptr) {
      for (int32_t cs = start; cs < end; cs += G::CE) {
        const int32_t e = cs + e_s;
        if (e < end) {
          const float sv = virt ? 0.f : lrelu(elh + er[(int64_t)col[e] * H + h_s], slope);
          attd[(int64_t)e * H + h_s] =
              __expf(sv - lse_h) * dropout_factor(dp, (uint64_t)e * H + h_s);
        }
      }
    }
    if (!has_next) break;
    row = nrow;
    start = nstart;
    end = nend;
    virt = nvirt;
    elh = nelh;
#pragma unroll
    for (int t = 0; t < EPL; ++t) {
      j0[t] = nj0[t];
      j1[t] = nj1[t];
    }
  }
}

// er_j = hc_j . a_r of one head from its QH 16-byte pieces, in the forward's order
// (pk_dot per piece, then the xor tree of group_sum<QH>)
template <int NV, typename T>
__device__ __forceinline__ float head_score(const Pk<T> (&hv)[NV], const float* __restrict__ a) {
  float d[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    Pk<T> ak;
#pragma unroll
    for (int v = 0; v < Pk<T>::V; v += 4) {
      const float4 a4 = *reinterpret_cast<const float4*>(a + Pk<T>::V * k + v);
      ak.v[v] = a4.x; ak.v[v + 1] = a4.y; ak.v[v + 2] = a4.z; ak.v[v + 3] = a4.w;
    }
    d[k] = pk_dot(hv[k], ak);
  }
#pragma unroll
  for (int o = 1; o < NV; o <<= 1)
#pragma unroll
    for (int k = 0; k < NV; k += 2 * o) d[k] = d[k] + d[k + o];
  return d[0];
}

// --------------------------------------------------------------- backward rows ---
// The gather-group loops unroll fully for fp32 and by BWR_UNR_BF16 for bf16 tables: the
// kernel is latency-bound (R15 rows hold ~2.3 edges, so the first group is usually the
// only one), and the fully unrolled bf16 v-branch variant held 129 VGPRs (3 waves/SIMD,
// 2x the fp32 time) for groups it rarely runs.
#ifndef BWR_UNR_BF16
#define BWR_UNR_BF16 2
#endif
template <int H, int F, typename T, bool DV>
__global__ void __launch_bounds__(256) edge_attn_bwd_rows_kernel(
    const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
    const uint8_t* __restrict__ rowflag, int64_t n_rows, const float* __restrict__ el,
    const float* __restrict__ er, const T* __restrict__ hc, const float* __restrict__ lse,
    const T* __restrict__ u, const T* __restrict__ u_lo, const T* __restrict__ dU,
    const T* __restrict__ hs, const T* __restrict__ dV, const float* __restrict__ row_coef,
    float slope, Dropout dp,
    float* __restrict__ d_el, float* __restrict__ de, float* __restrict__ attd, int ld,
    T* __restrict__ d_hs) {
  using G = Geo<H, F, T>;
  constexpr int UNR = sizeof(T) == 2 ? BWR_UNR_BF16 : G::CE / G::EPI;
  const int lane = lane_id();
  const int e_s = lane / H, h_s = lane % H;
  const int g_e = G::QPL == 1 ? lane / G::NQ : 0;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  // lane (in the gather layout) holding the first chunk of head h_s, and its slot
  const int dsrc_k = (h_s * G::QH) / 64;
  const int dsrc_l = (h_s * G::QH) % 64;

  // same software pipeline as the forward: next row's bounds during this row, the
  // main loop's columns two chunks ahead and er one chunk ahead
  int64_t row = wave;
  if (row >= n_rows) return;
  int32_t start = rowptr[row], end = rowptr[row + 1];
  int32_t j0 = start + e_s < end ? col[start + e_s] : 0;
  int32_t j1 = start + G::CE + e_s < end ? col[start + G::CE + e_s] : 0;
  while (true) {
    const int64_t nrow = row + nwaves;
    const bool has_next = nrow < n_rows;
    const int32_t nstart = has_next ? rowptr[nrow] : 0;
    const int32_t nend = has_next ? rowptr[nrow + 1] : 0;
    const bool virt = rowflag != nullptr && rowflag[row] != 0;
    const float elh = el[row * H + h_s];
    const float lseh = lse[row * H + h_s];
    Pk<T> dUq[G::QPL], hsq[G::QPL];
    float dpart[G::QPL];
#pragma unroll
    for (int k = 0; k < G::QPL; ++k) {
      const int q = quad_of<G>(lane, k);
      dUq[k] = pk_load(dU + row * G::D + G::V * q);
      dpart[k] = pk_dot(dUq[k], pk_load(u + row * G::D + G::V * q));
      if (sizeof(T) == 2 && u_lo != nullptr)
        dpart[k] += pk_dot(dUq[k], pk_load(u_lo + row * G::D + G::V * q));
      hsq[k] = pk_zero<T>();
    }
    if (DV) {
      // w_i = sum_e attd_e dV[j]   (== d hs_i of the v-branch)
      Pk<T> wacc[G::QPL];
#pragma unroll
      for (int k = 0; k < G::QPL; ++k) wacc[k] = pk_zero<T>();
      for (int32_t cs = start; cs < end; cs += G::CE) {
        const int32_t e = cs + e_s;
        const bool valid = e < end;
        const int32_t j = valid ? col[e] : 0;
        float w = 0.f;
        if (valid) {
          const float s = virt ? 0.f : lrelu(elh + er[(int64_t)j * H + h_s], slope);
          w = __expf(s - lseh) * dropout_factor(dp, (uint64_t)e * H + h_s);
        }
        const int nvalid = min(G::CE, (int)(end - cs));
#pragma unroll UNR
        for (int g = 0; g < G::CE; g += G::EPI) {
          if (g >= nvalid) break;
          const int ei = g + g_e;
          const int32_t jq = __shfl(j, ei * H);
#pragma unroll
          for (int k = 0; k < G::QPL; ++k) {
            const int q = quad_of<G>(lane, k);
            const float wq = __shfl(w, ei * H + q / G::QH);
            if (ei < nvalid)
              wacc[k] = pk_fma(wq, pk_load(dV + (int64_t)jq * G::D + G::V * q), wacc[k]);
          }
        }
      }
      if (G::EPI > 1) {
#pragma unroll
        for (int o = G::NQ; o < 64; o <<= 1) wacc[0] = pk_xor_add(wacc[0], o);
      }
#pragma unroll
      for (int k = 0; k < G::QPL; ++k) {
        const int q = quad_of<G>(lane, k);
        if (g_e == 0) pk_store(d_hs + row * G::D + G::V * q, wacc[k]);
        hsq[k] = pk_load(hs + row * G::D + G::V * q);
        dpart[k] += pk_dot(hsq[k], wacc[k]);
      }
    }
    // D_h = dU_i.u_i (+ hs_i.w_i) per head, delivered to the score layout
    float Ds = 0.f;
#pragma unroll
    for (int k = 0; k < G::QPL; ++k) {
      const float dk = group_sum<G::QH>(dpart[k]);
      const float cand = __shfl(dk, dsrc_l);
      if (k == dsrc_k) Ds = cand;
    }
    // Ours.py:84-86: SUM_county adds sum_j exp(attd_ij) for batch rows, so those rows'
    // attention gets the extra gradient coef * exp(attd) (row_coef = dL/dSUM terms)
    const float coef = row_coef != nullptr ? row_coef[row * H + h_s] : 0.f;
    if (__ballot(coef != 0.f)) {
      float t = 0.f;
      for (int32_t cs = start; cs < end; cs += G::CE) {
        const int32_t e = cs + e_s;
        if (e < end) {
          const float s = virt ? 0.f : lrelu(elh + er[(int64_t)col[e] * H + h_s], slope);
          const float ad = __expf(s - lseh) * dropout_factor(dp, (uint64_t)e * H + h_s);
          t += ad * expf(ad);
        }
      }
      Ds += coef * wave_xor_sum<H>(t);
    }
    float del = 0.f;
    float erv = start + e_s < end ? er[(int64_t)j0 * H + h_s] : 0.f;
    for (int32_t cs = start; cs < end; cs += G::CE) {
      const int32_t e = cs + e_s;
      const bool valid = e < end;
      const int32_t j = j0;
      float pre = 0.f, att = 0.f, dropf = 0.f;
      if (valid) {
        pre = elh + erv;
        const float s = virt ? 0.f : lrelu(pre, slope);
        att = __expf(s - lseh);
        dropf = dropout_factor(dp, (uint64_t)e * H + h_s);
      }
      const int nvalid = min(G::CE, (int)(end - cs));
      float gsum = 0.f;
#pragma unroll UNR
      for (int g = 0; g < G::CE; g += G::EPI) {
        if (g >= nvalid) break;
        const int ei = g + g_e;
        const int32_t jq = __shfl(j, ei * H);
        const bool mine = e_s >= g && e_s < g + G::EPI;
        const int srcl = G::QPL == 1 ? ((e_s - g) & (G::EPI - 1)) * G::NQ + h_s * G::QH : dsrc_l;
#pragma unroll
        for (int k = 0; k < G::QPL; ++k) {
          const int q = quad_of<G>(lane, k);
          float t = 0.f;
          if (ei < nvalid) {
            t = pk_dot(dUq[k], pk_load(hc + (int64_t)jq * G::D + G::V * q));
            if (DV) t += pk_dot(hsq[k], pk_load(dV + (int64_t)jq * G::D + G::V * q));
          }
          t = group_sum<G::QH>(t);
          const float cand = __shfl(t, srcl);
          if (mine && (G::QPL == 1 || k == dsrc_k)) gsum = cand;
        }
      }
      // prefetch after the gathers: they are not queued behind these loads
      const int32_t j2 = e + 2 * G::CE < end ? col[e + 2 * G::CE] : 0;
      const float ern = e + G::CE < end ? er[(int64_t)j1 * H + h_s] : 0.f;
      if (valid) {
        if (coef != 0.f) gsum += coef * expf(att * dropf);
        const float ds = att * (gsum * dropf - Ds);
        const float dev = virt ? 0.f : ds * (pre > 0.f ? 1.f : slope);
        de[(int64_t)e * ld + h_s] = dev;
        attd[(int64_t)e * ld + h_s] = att * dropf;
        del += dev;
      }
      j0 = j1;
      j1 = j2;
      erv = ern;
    }
    if (has_next) {
      j0 = nstart + e_s < nend ? col[nstart + e_s] : 0;
      j1 = nstart + G::CE + e_s < nend ? col[nstart + G::CE + e_s] : 0;
    }
    del = wave_xor_sum<H>(del);
    if (lane < H) d_el[row * H + lane] = del;
    if (!has_next) break;
    row = nrow;
    start = nstart;
    end = nend;
  }
}

// ------------------------------------------------------- column (CSC) aggregate ---
// Whole columns write the table type T directly; chunks of multi-chunk columns
// write fp32 partials that csc_combine adds in chunk order.
template <int H, int F, typename T, bool HASX>
__global__ void __launch_bounds__(256) csc_aggregate_kernel(
    const int32_t* __restrict__ chunk_col, const int32_t* __restrict__ chunk_start,
    const int32_t* __restrict__ chunk_end, int64_t n_chunks, const int32_t* __restrict__ colptr,
    const int32_t* __restrict__ csc_row, const int32_t* __restrict__ csc_eid,
    const float* __restrict__ w, const float* __restrict__ x, int ld, const T* __restrict__ table,
    T* __restrict__ out, float* __restrict__ out_x, float* __restrict__ part,
    float* __restrict__ part_x) {
  using G = Geo<H, F, T>;
  const int lane = lane_id();
  const int e_s = lane / H, h_s = lane % H;
  const int g_e = G::QPL == 1 ? lane / G::NQ : 0;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;

  for (int64_t c = wave; c < n_chunks; c += nwaves) {
    const int32_t jc = chunk_col[c], s0 = chunk_start[c], s1 = chunk_end[c];
    const bool whole = s0 == colptr[jc] && s1 == colptr[jc + 1];
    Pk<T> acc[G::QPL];
#pragma unroll
    for (int k = 0; k < G::QPL; ++k) acc[k] = pk_zero<T>();
    float xacc = 0.f;
    for (int32_t cs = s0; cs < s1; cs += G::CE) {
      const int32_t slot = cs + e_s;
      const bool valid = slot < s1;
      const int32_t i = valid ? csc_row[slot] : 0;
      // csc_eid NULL: slot order is the edge order (the CSR-as-CSC view of a graph)
      const int64_t eid = valid ? (csc_eid != nullptr ? (int64_t)csc_eid[slot] : slot) : 0;
      const float wv = valid ? w[eid * ld + h_s] : 0.f;
      if (HASX && valid) xacc += x[eid * ld + h_s];
      const int nvalid = min(G::CE, (int)(s1 - cs));
#pragma unroll
      for (int g = 0; g < G::CE; g += G::EPI) {
        if (g >= nvalid) break;
        const int ei = g + g_e;
        const int32_t iq = __shfl(i, ei * H);
#pragma unroll
        for (int k = 0; k < G::QPL; ++k) {
          const int q = quad_of<G>(lane, k);
          const float wq = __shfl(wv, ei * H + q / G::QH);
          if (ei < nvalid) acc[k] = pk_fma(wq, pk_load(table + (int64_t)iq * G::D + G::V * q), acc[k]);
        }
      }
    }
    if (G::EPI > 1) {
#pragma unroll
      for (int o = G::NQ; o < 64; o <<= 1) acc[0] = pk_xor_add(acc[0], o);
    }
#pragma unroll
    for (int k = 0; k < G::QPL; ++k) {
      if (g_e != 0) continue;
      const int q = quad_of<G>(lane, k);
      if (whole) {
        pk_store(out + (int64_t)jc * G::D + G::V * q, acc[k]);
      } else {
        float* dst = part + c * G::D + G::V * q;
#pragma unroll
        for (int i = 0; i < G::V; i += 4)
          *reinterpret_cast<float4*>(dst + i) =
              make_float4(acc[k].v[i], acc[k].v[i + 1], acc[k].v[i + 2], acc[k].v[i + 3]);
      }
    }
    if (HASX) {
      xacc = wave_xor_sum<H>(xacc);
      if (lane < H) (whole ? out_x + (int64_t)jc * H : part_x + c * H)[lane] = xacc;
    }
  }
}

// multi-chunk columns: add the chunk partials.  Block = one column x a tile of 256
// output elements (D table columns then H x-sums); its 16 waves stride the column's
// chunks (wave g takes chunks g, g+16, ...) and the 16 partial sums are added in a
// fixed LDS tree (deterministic).
constexpr int kCombineWaves = 16;

template <typename T>
__global__ void __launch_bounds__(1024) csc_combine_kernel(
    const int32_t* __restrict__ multi_col, const int32_t* __restrict__ multi_first,
    const int32_t* __restrict__ multi_count, int64_t n_multi, int D, int H,
    const float* __restrict__ part, const float* __restrict__ part_x, T* __restrict__ out,
    float* __restrict__ out_x) {
  __shared__ float red[kCombineWaves][256];
  const int W = D + (part_x != nullptr ? H : 0);
  const int64_t mi = blockIdx.x;
  const int e0 = blockIdx.y * 256;
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int32_t jc = multi_col[mi], first = multi_first[mi], cnt = multi_count[mi];
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  auto ld = [&](int64_t c, int q) {
    const int e = e0 + lane + 64 * q;
    return e < D ? part[c * D + e] : (e < W ? part_x[c * H + (e - D)] : 0.f);
  };
  int k = g;
  // 4 chunk partials per lane loaded before they are added (same order per lane)
  for (; k + 3 * kCombineWaves < cnt; k += 4 * kCombineWaves) {
    float v[4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int q = 0; q < 4; ++q) v[u][q] = ld(first + k + u * kCombineWaves, q);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] += v[u][q];
  }
  for (; k < cnt; k += kCombineWaves) {
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] += ld(first + k, q);
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) red[g][lane + 64 * q] = acc[q];
  __syncthreads();
  for (int w = kCombineWaves / 2; w >= 1; w >>= 1) {
    if (g < w) {
#pragma unroll
      for (int q = 0; q < 4; ++q) red[g][lane + 64 * q] += red[g + w][lane + 64 * q];
    }
    __syncthreads();
  }
  if (g == 0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = e0 + lane + 64 * q;
      if (e < D) out[(int64_t)jc * D + e] = from_f32<T>(red[0][lane + 64 * q]);
      else if (e < W) out_x[(int64_t)jc * H + (e - D)] = red[0][lane + 64 * q];
    }
  }
}

// ------------------------------------------------ fused backward (u only) ---
// Column-major backward for u = drop(att) @ hc (no v branch, no row coefficients).
// The row pass of the split backward gathers hc[j] only for g_ij = dU_i . hc_j and
// the column pass gathers dU[i]; a column owns hc_j, so one pass over the CSC gets
// g_ij from the dU[i] gather it does anyway: per edge one 16-B/lane gather instead
// of two, and no (de, attd) record written and re-read.  Three launches:
//   row_stats : rec_i = (el_i, lse_i, D_i = dU_i . u_i)  per head   (N x 3H fp32)
//   cols      : d_hc[j] = sum attd_ij dU_i, d_er[j] = sum de_ij, de_ij -> edge order
//   row_sum   : d_el[i] = sum_j de_ij                                (CSR order)
// Every value is computed with the same operands in the same order as
// edge_attn_bwd_rows + csc_aggregate: the results are bitwise identical.
// Row statistics: RPW rows per wave trip (EPI rows per load instruction, all loads of
// the trip issued before the first use), D_i = dU_i . u_i per head in group_sum order.
// Row record stride in floats: the 3H values padded to a power of two (H = 8: 32 floats,
// one 128-B line), so a record never straddles a line and a CSC slot's record gather
// touches exactly one (the unpadded 96-B record straddled two lines half the time).
#ifndef REC_PAD
#define REC_PAD 1
#endif
__host__ __device__ constexpr int rec_stride(int H) {
  int s = 1;
  while (s < 3 * H) s <<= 1;
  return REC_PAD ? s : 3 * H;
}
// the padded record also carries the row's virtual flag (float 0 / 1 at 3H): the column
// pass reads it from the record line it fetches anyway instead of a random byte gather
__host__ __device__ constexpr bool rec_has_flag(int H) { return rec_stride(H) > 3 * H; }

// RT: the forward's row terms are given (uc, qc; see edge_attn_fwd_bat_kernel), so the
// same pass also finishes d_el_i = dU_i . uc_i - D_i qc_i (0 on virtual rows) and the
// column pass stores no per-edge de (no row sum follows).
template <int H, int F, typename T, bool RT = false>
__global__ void __launch_bounds__(256) bwd_row_stats_kernel(
    int64_t n_rows, const float* __restrict__ el, const float* __restrict__ lse,
    const T* __restrict__ u, const T* __restrict__ u_lo, const T* __restrict__ dU,
    float* __restrict__ rec, const float* __restrict__ uc, const float* __restrict__ qc,
    const uint8_t* __restrict__ rowflag, float* __restrict__ d_el) {
  using G = Geo<H, F, T>;
  constexpr int UNR = G::QPL == 1 ? 4 : 1;        // load groups per trip
  constexpr int RPW = G::EPI * UNR;               // rows per trip
  const int lane = lane_id();
  const int r_s = G::QPL == 1 ? lane / G::NQ : 0;  // row slot of this lane in a group
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t r0 = wave * RPW; r0 < n_rows; r0 += nwaves * RPW) {
    Pk<T> a[UNR][G::QPL], b[UNR][G::QPL];
    const bool lo = sizeof(T) == 2 && u_lo != nullptr;
#pragma unroll
    for (int g = 0; g < UNR; ++g) {
      const int64_t row = min(r0 + g * G::EPI + r_s, n_rows - 1);
#pragma unroll
      for (int k = 0; k < G::QPL; ++k) {
        const int q = quad_of<G>(lane, k);
        a[g][k] = pk_load(dU + row * G::D + G::V * q);
        b[g][k] = pk_load(u + row * G::D + G::V * q);
      }
    }
#pragma unroll
    for (int g = 0; g < UNR; ++g) {
      const int64_t row = r0 + g * G::EPI + r_s;
#pragma unroll
      for (int k = 0; k < G::QPL; ++k) {
        const int q = quad_of<G>(lane, k);
        float dot = pk_dot(a[g][k], b[g][k]);
        if (lo) {  // bf16: u = hi + lo (the forward's rounding residual)
          const int64_t rr = min(row, n_rows - 1);
          dot += pk_dot(a[g][k], pk_load(u_lo + rr * G::D + G::V * q));
        }
        const float dk = group_sum<G::QH>(dot);
        float dc = 0.f;
        if (RT) {  // dU_i . uc_i over the head's pieces (uc is fp32 for either table type)
          const int64_t rr = min(row, n_rows - 1);
          const float* cp = uc + rr * G::D + G::V * q;
          float cv = 0.f;
#pragma unroll
          for (int v = G::V - 4; v >= 0; v -= 4) {
            const float4 c4 = *reinterpret_cast<const float4*>(cp + v);
            cv = fmaf(a[g][k].v[v + 3], c4.w, cv);
            cv = fmaf(a[g][k].v[v + 2], c4.z, cv);
            cv = fmaf(a[g][k].v[v + 1], c4.y, cv);
            cv = fmaf(a[g][k].v[v], c4.x, cv);
          }
          dc = group_sum<G::QH>(cv);
        }
        // the head's first chunk lane writes D; el and lse ride along
        if (q % G::QH == 0 && row < n_rows) {
          const int h = q / G::QH;
          float* r = rec + row * rec_stride(H);
          r[h] = el[row * H + h];
          r[H + h] = lse[row * H + h];
          r[2 * H + h] = dk;
          if (rec_has_flag(H) && h == 0)
            r[3 * H] = rowflag != nullptr && rowflag[row] != 0 ? 1.f : 0.f;
          if (RT) {
            const bool virt = rowflag != nullptr && rowflag[row] != 0;
            d_el[row * H + h] = virt ? 0.f : fmaf(-dk, qc[row * H + h], dc);
          }
        }
      }
    }
  }
}

// RSC (row scores, recomputed): er_j = hc_j . a_r in the gather-layout forward's order
// instead of reading er (a separate instantiation: the extra registers stay out of the
// er-reading kernel)
template <int H, int F, typename T, bool BUF, bool RSC = false>
__global__ void __launch_bounds__(256) bwd_cols_kernel(
    const int32_t* __restrict__ chunk_col, const int32_t* __restrict__ chunk_start,
    const int32_t* __restrict__ chunk_end, int64_t n_chunks, const int32_t* __restrict__ colptr,
    const int32_t* __restrict__ csc_row, const int32_t* __restrict__ csc_eid, int64_t n_rows,
    const uint8_t* __restrict__ rowflag, const float* __restrict__ rec,
    const float* __restrict__ er, const float* __restrict__ ar, const T* __restrict__ hc,
    const T* __restrict__ dU, float slope, Dropout dp, bool slot_de, float* __restrict__ de,
    T* __restrict__ d_hc, float* __restrict__ d_er, float* __restrict__ part,
    float* __restrict__ part_x) {
  using G = Geo<H, F, T>;
  const int lane = lane_id();
  const int e_s = lane / H, h_s = lane % H;
  const int g_e = G::QPL == 1 ? lane / G::NQ : 0;
  const int dsrc_k = (h_s * G::QH) / 64;
  const int dsrc_l = (h_s * G::QH) % 64;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;

  // software pipeline: the next chunk's plan entry during this chunk; CSC slot rows
  // two slot-groups ahead, issued after each group's gathers
  int64_t c = wave;
  if (c >= n_chunks) return;
  int32_t jc = chunk_col[c], s0 = chunk_start[c], s1 = chunk_end[c];
  int32_t i0 = s0 + e_s < s1 ? csc_row[s0 + e_s] : 0;
  int32_t i1 = s0 + G::CE + e_s < s1 ? csc_row[s0 + G::CE + e_s] : 0;
  while (true) {
    const int64_t nc = c + nwaves;
    const bool has_next = nc < n_chunks;
    const int32_t njc = has_next ? chunk_col[nc] : 0;
    const int32_t ns0 = has_next ? chunk_start[nc] : 0;
    const int32_t ns1 = has_next ? chunk_end[nc] : 0;
    const bool whole = s0 == colptr[jc] && s1 == colptr[jc + 1];
    Pk<T> hcq[G::QPL], acc[G::QPL];
#pragma unroll
    for (int k = 0; k < G::QPL; ++k) {
      hcq[k] = pk_load(hc + (int64_t)jc * G::D + G::V * quad_of<G>(lane, k));
      acc[k] = pk_zero<T>();
    }
    float erh;
    if (RSC && G::QPL == 1) {  // er_j from hc_j in the row-score forward's order
      const int q = lane % G::NQ;
      Pk<T> aq;
#pragma unroll
      for (int v = 0; v < G::V; ++v) aq.v[v] = ar[G::V * q + v];
      erh = __shfl(group_sum<G::QH>(pk_dot(hcq[0], aq)), h_s * G::QH);
    } else {
      erh = er[(int64_t)jc * H + h_s];
    }
    float xacc = 0.f;
    for (int32_t cs = s0; cs < s1; cs += G::CE) {
      const int32_t slot = cs + e_s;
      const bool valid = slot < s1;
      const int32_t i = i0;
      const int64_t eid = valid ? (int64_t)csc_eid[slot] : 0;
      float pre = 0.f, att = 0.f, dropf = 0.f, Dsi = 0.f;
      bool virt = false;
      if (valid) {
        const float* r = rec + (int64_t)i * rec_stride(H);
        virt = rowflag != nullptr && rowflag[i] != 0;
        pre = r[h_s] + erh;
        const float sv = virt ? 0.f : lrelu(pre, slope);
        att = __expf(sv - r[H + h_s]);
        Dsi = r[2 * H + h_s];
        dropf = dropout_factor(dp, (uint64_t)eid * H + h_s);
      }
      const float wv = att * dropf;
      const int nvalid = min(G::CE, (int)(s1 - cs));
      float gsum = 0.f;
      if constexpr (BUF && (G::EPI == 1 || COLS_EPI_BUF)) {
        // UG gather instructions (EPI edges each; one edge per instruction on wide rows)
        // load their dU rows through the buffer descriptor -- a slot past the chunk
        // reads 0, so its fma adds 0 and its dot is 0, as the skipped branch below --
        // before any is used, then are consumed in slot order: the same operations in
        // the same order as below, with UG instructions in flight instead of one (a load
        // under "if (ei < nvalid)" drained the queue after every instruction)
        constexpr int UG = G::EPI == 1 ? COLS_WIDE_UG : COLS_NARROW_UG;
        const rsrc_t r_dU = make_rsrc(dU, (uint32_t)(n_rows * G::D * sizeof(T)));
#pragma unroll
        for (int g0 = 0; g0 < G::CE; g0 += UG * G::EPI) {
          if (g0 >= nvalid) break;
          // raw 16-B pieces in flight (a bf16 piece widens to 8 floats only at its use)
          u32x4_t dl[UG][G::QPL];
#pragma unroll
          for (int u = 0; u < UG; ++u) {
            const int g = g0 + u * G::EPI;
            if (g >= G::CE) break;
            const int ei = g + g_e;
            const int32_t iq = __shfl(i, ei * H);
#pragma unroll
            for (int k = 0; k < G::QPL; ++k) {
              const int q = quad_of<G>(lane, k);
              const uint32_t off = ei < nvalid
                  ? (uint32_t)iq * (uint32_t)(G::D * sizeof(T)) + (uint32_t)(G::V * q * sizeof(T))
                  : kOOB;
              dl[u][k] = buf_b128(r_dU, off);
            }
          }
#pragma unroll
          for (int u = 0; u < UG; ++u) {
            const int g = g0 + u * G::EPI;
            if (g >= G::CE || g >= nvalid) break;
            const int ei = g + g_e;
            const bool mine = e_s >= g && e_s < g + G::EPI;
            const int srcl =
                G::QPL == 1 ? ((e_s - g) & (G::EPI - 1)) * G::NQ + h_s * G::QH : dsrc_l;
#pragma unroll
            for (int k = 0; k < G::QPL; ++k) {
              const int q = quad_of<G>(lane, k);
              const float wq = __shfl(wv, ei * H + q / G::QH);
              const Pk<T> dUi = pk_from_raw(dl[u][k], (T*)nullptr);
              acc[k] = pk_fma(wq, dUi, acc[k]);
              float t = pk_dot(dUi, hcq[k]);
              t = group_sum<G::QH>(t);
              const float cand = __shfl(t, srcl);
              if (mine && (G::QPL == 1 || k == dsrc_k)) gsum = cand;
            }
          }
        }
      } else {
#pragma unroll
      for (int g = 0; g < G::CE; g += G::EPI) {
        if (g >= nvalid) break;
        const int ei = g + g_e;
        const int32_t iq = __shfl(i, ei * H);
        const bool mine = e_s >= g && e_s < g + G::EPI;
        const int srcl = G::QPL == 1 ? ((e_s - g) & (G::EPI - 1)) * G::NQ + h_s * G::QH : dsrc_l;
#pragma unroll
        for (int k = 0; k < G::QPL; ++k) {
          const int q = quad_of<G>(lane, k);
          const float wq = __shfl(wv, ei * H + q / G::QH);
          float t = 0.f;
          if (ei < nvalid) {
            const Pk<T> dUi = pk_load(dU + (int64_t)iq * G::D + G::V * q);
            acc[k] = pk_fma(wq, dUi, acc[k]);
            t = pk_dot(dUi, hcq[k]);
          }
          t = group_sum<G::QH>(t);
          const float cand = __shfl(t, srcl);
          if (mine && (G::QPL == 1 || k == dsrc_k)) gsum = cand;
        }
      }
      }
      const int32_t sl2 = slot + 2 * G::CE;
      const int32_t i2 = sl2 < s1 ? csc_row[sl2] : 0;
      if (valid) {
        const float ds = att * (gsum * dropf - Dsi);
        const float dev = virt ? 0.f : ds * (pre > 0.f ? 1.f : slope);
        if (de != nullptr) de[(slot_de ? (int64_t)slot : eid) * H + h_s] = dev;
        xacc += dev;
      }
      i0 = i1;
      i1 = i2;
    }
    if (has_next) {
      const int32_t a0 = ns0 + e_s, a1 = ns0 + G::CE + e_s;
      i0 = a0 < ns1 ? csc_row[a0] : 0;
      i1 = a1 < ns1 ? csc_row[a1] : 0;
    }
    if (G::EPI > 1) {
#pragma unroll
      for (int o = G::NQ; o < 64; o <<= 1) acc[0] = pk_xor_add(acc[0], o);
    }
#pragma unroll
    for (int k = 0; k < G::QPL; ++k) {
      if (g_e != 0) continue;
      const int q = quad_of<G>(lane, k);
      if (whole) {
        pk_store(d_hc + (int64_t)jc * G::D + G::V * q, acc[k]);
      } else {
        float* dst = part + c * G::D + G::V * q;
#pragma unroll
        for (int v = 0; v < G::V; v += 4)
          *reinterpret_cast<float4*>(dst + v) =
              make_float4(acc[k].v[v], acc[k].v[v + 1], acc[k].v[v + 2], acc[k].v[v + 3]);
      }
    }
    xacc = wave_xor_sum<H>(xacc);
    if (lane < H) (whole ? d_er + (int64_t)jc * H : part_x + c * H)[lane] = xacc;
    if (!has_next) break;
    c = nc;
    jc = njc;
    s0 = ns0;
    s1 = ns1;
  }
}

// Head-per-lane variant of the column pass for narrow heads (F * sizeof(T) <= 64 B):
// lane = (slot e_s, head h_s) holds that head's F features of dU[i] (QH 16-B loads at
// stride QH * 16 B; the edge's H lanes together cover its whole row), so the score,
// the dot dU_i[h] . hc_j[h], the weight and the accumulation all stay in the lane: no
// per-edge shuffles; the CE slot lanes are combined once per chunk.  Memory ops go
// through buffer descriptors (masked lanes read 0 / drop their store), so the slot
// loop is branch-free and its waits exact; two slot groups per trip, each group's
// CSC rows loaded two groups ahead into the register it just consumed.
// Needs every table below 2 GiB (msha_edge_attention_bwd_fused checks).
template <int H, int F, typename T, bool RSC = false>
__global__ void __launch_bounds__(256) bwd_cols_eh_kernel(
    const int32_t* __restrict__ chunk_col, const int32_t* __restrict__ chunk_start,
    const int32_t* __restrict__ chunk_end, int64_t n_chunks, const int32_t* __restrict__ colptr,
    const int32_t* __restrict__ csc_row, const int32_t* __restrict__ csc_eid, int64_t n_edges,
    const uint8_t* __restrict__ rowflag, int64_t n_rows, const float* __restrict__ rec,
    const float* __restrict__ er, const float* __restrict__ ar, const T* __restrict__ hc,
    const T* __restrict__ dU, float slope, Dropout dp, bool slot_de, float* __restrict__ de,
    T* __restrict__ d_hc, float* __restrict__ d_er, float* __restrict__ part,
    float* __restrict__ part_x) {
  using G = Geo<H, F, T>;
  constexpr int NV = G::QH;  // 16-B pieces per head
  constexpr int NG = COLS_NG;
  const int lane = lane_id();
  const int e_s = lane / H, h_s = lane % H;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const rsrc_t r_row = make_rsrc(csc_row, (uint32_t)(n_edges * 4));
  const rsrc_t r_eid = make_rsrc(csc_eid, (uint32_t)(n_edges * 4));
  const rsrc_t r_flag = make_rsrc(rowflag, (uint32_t)n_rows);
  const rsrc_t r_rec = make_rsrc(rec, (uint32_t)(n_rows * 4 * rec_stride(H)));
  const rsrc_t r_dU = make_rsrc(dU, (uint32_t)(n_rows * G::D * sizeof(T)));
  const rsrc_t r_de = make_rsrc(de, (uint32_t)(n_edges * 4 * H));
  const uint32_t h_off = h_s * F * sizeof(T);
  // the CSR edge id serves the dropout stream and an edge-ordered de only: otherwise its
  // load stays off the memory system (kOOB)
  const bool need_eid = dp.active || (de != nullptr && !slot_de);

  int64_t c = wave;
  if (c >= n_chunks) return;
  int32_t jc = chunk_col[c], s0 = chunk_start[c], s1 = chunk_end[c];
  int32_t ii[NG];
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const int32_t a = s0 + g * G::CE + e_s;
    ii[g] = buf_i32(r_row, a < s1 ? (uint32_t)a * 4u : kOOB);
  }
  while (true) {
    const int64_t nc = c + nwaves;
    const bool has_next = nc < n_chunks;
    const int32_t njc = has_next ? chunk_col[nc] : 0;
    const int32_t ns0 = has_next ? chunk_start[nc] : 0;
    const int32_t ns1 = has_next ? chunk_end[nc] : 0;
    const bool whole = s0 == colptr[jc] && s1 == colptr[jc + 1];
    Pk<T> hcv[NV], acc[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      hcv[k] = pk_load(hc + (int64_t)jc * G::D + h_s * F + G::V * k);
      acc[k] = pk_zero<T>();
    }
    const float er_tab = RSC ? 0.f : er[(int64_t)jc * H + h_s];
    float xacc = 0.f;
    // one trip = COLS_NG slot groups: every group's loads leave before the first
    // group's compute and de store (the compiler may not hoist a buffer load above a
    // buffer store), then the groups are consumed in slot order
    for (int32_t cs = s0; cs < s1; cs += NG * G::CE) {
      Pk<T> dUv[NG][NV];
      int32_t eid[NG];
      float r_el[NG], r_lse[NG], Dsi[NG];
      uint32_t vflag[NG];
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        const bool valid = cs + g * G::CE + e_s < s1;
        const uint32_t row_off = valid ? (uint32_t)ii[g] * (G::D * sizeof(T)) + h_off : kOOB;
#pragma unroll
        for (int k = 0; k < NV; ++k)
          dUv[g][k] = pk_load_buf(r_dU, row_off + (valid ? k * 16u : 0u), (T*)nullptr);
        eid[g] = buf_i32(r_eid, valid && need_eid ? (uint32_t)(cs + g * G::CE + e_s) * 4u : kOOB);
        const uint32_t rec_off = valid ? (uint32_t)ii[g] * (4u * rec_stride(H)) + h_s * 4u : kOOB;
        r_el[g] = buf_f32(r_rec, rec_off);
        r_lse[g] = buf_f32(r_rec, valid ? rec_off + 4u * H : kOOB);
        Dsi[g] = buf_f32(r_rec, valid ? rec_off + 8u * H : kOOB);
        if constexpr (rec_has_flag(H))
          vflag[g] = __float_as_uint(buf_f32(r_rec, valid ? rec_off - h_s * 4u + 12u * H : kOOB));
        else
          vflag[g] = buf_u8(r_flag, valid ? (uint32_t)ii[g] : kOOB);
      }
      // CSC rows of the next trip
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        const int32_t a = cs + (NG + g) * G::CE + e_s;
        ii[g] = buf_i32(r_row, a < s1 ? (uint32_t)a * 4u : kOOB);
      }
      // er_j: from hc_j in the row-score forward's order when a_r is given, recomputed
      // per trip AFTER the trip's loads are in flight (computed before the loop, the wait
      // for hc_j / a_r put one memory latency in front of every chunk's loads); the empty
      // asm keeps it from being hoisted back out of the loop
      float erh = er_tab;
      if (RSC) {
        Pk<T> hv[NV];
#pragma unroll
        for (int k = 0; k < NV; ++k) {
          hv[k] = hcv[k];
#pragma unroll
          for (int v = 0; v < G::V; ++v) asm volatile("" : "+v"(hv[k].v[v]));
        }
        erh = head_score<NV>(hv, ar + h_s * F);
      }
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        const int32_t slot = cs + g * G::CE + e_s;
        const bool valid = slot < s1;
        const bool virt = vflag[g] != 0;
        const float pre = r_el[g] + erh;
        const float sv = virt ? 0.f : lrelu(pre, slope);
        const float att = __expf(sv - r_lse[g]);
        const float dropf = dropout_factor(dp, (uint64_t)eid[g] * H + h_s);
        const float wv = valid ? att * dropf : 0.f;
        // dU_i[h] . hc_j[h] in group_sum's order over the head's pieces
        float d[NV];
#pragma unroll
        for (int k = 0; k < NV; ++k) {
          d[k] = pk_dot(dUv[g][k], hcv[k]);
          acc[k] = pk_fma(wv, dUv[g][k], acc[k]);
        }
#pragma unroll
        for (int o = 1; o < NV; o <<= 1)
#pragma unroll
          for (int k = 0; k < NV; k += 2 * o) d[k] = d[k] + d[k + o];
        const float ds = att * (d[0] * dropf - Dsi[g]);
        const float dev = virt ? 0.f : ds * (pre > 0.f ? 1.f : slope);
#ifndef DIAG_NO_DE
        const uint32_t at = slot_de ? (uint32_t)slot : (uint32_t)eid[g];
        buf_store_f32(r_de, valid ? at * (4u * H) + h_s * 4u : kOOB, dev);
#endif
        xacc += valid ? dev : 0.f;
      }
    }
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int32_t a = ns0 + g * G::CE + e_s;
      ii[g] = buf_i32(r_row, a < ns1 ? (uint32_t)a * 4u : kOOB);
    }
#pragma unroll
    for (int k = 0; k < NV; ++k)
#pragma unroll
      for (int o = H; o < 64; o <<= 1) acc[k] = pk_xor_add(acc[k], o);
    if (e_s == 0) {
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        if (whole) {
          pk_store(d_hc + (int64_t)jc * G::D + h_s * F + G::V * k, acc[k]);
        } else {
          float* dst = part + c * G::D + h_s * F + G::V * k;
#pragma unroll
          for (int v = 0; v < G::V; v += 4)
            *reinterpret_cast<float4*>(dst + v) =
                make_float4(acc[k].v[v], acc[k].v[v + 1], acc[k].v[v + 2], acc[k].v[v + 3]);
        }
      }
    }
    xacc = wave_xor_sum<H>(xacc);
    if (lane < H) (whole ? d_er + (int64_t)jc * H : part_x + c * H)[lane] = xacc;
    if (!has_next) break;
    c = nc;
    jc = njc;
    s0 = ns0;
    s1 = ns1;
  }
}

// d_el[i] = sum over the row's edges of de.  Lane = (row slot, head): 64/H rows per
// wave, each lane walking its row's edges with independent loads.  The sum keeps
// bwd_rows' order (lane e_s of a CE-edge chunk accumulates edges e_s, e_s + CE, ...;
// then the xor tree over e_s), so the result is the same bits.
template <int H>
__global__ void __launch_bounds__(256) bwd_row_sum_kernel(
    const int32_t* __restrict__ rowptr, int64_t n_rows, const float* __restrict__ de,
    const int32_t* __restrict__ slot_of, float* __restrict__ d_el) {
  constexpr int CE = 64 / H;
  const int lane = lane_id();
  const int r_s = lane / H, h_s = lane % H;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t r0 = wave * CE; r0 < n_rows; r0 += nwaves * CE) {
    const int64_t row = r0 + r_s;
    if (row >= n_rows) continue;
    const int32_t start = rowptr[row], end = rowptr[row + 1];
    float p[CE];
#pragma unroll
    for (int k = 0; k < CE; ++k) p[k] = 0.f;
    for (int32_t cs = start; cs < end; cs += CE) {
      float v[CE];
      int32_t at[CE];
#pragma unroll
      for (int k = 0; k < CE; ++k)
        at[k] = slot_of == nullptr ? cs + k : (cs + k < end ? slot_of[cs + k] : 0);
#pragma unroll
      for (int k = 0; k < CE; ++k)
        v[k] = cs + k < end ? de[(int64_t)at[k] * H + h_s] : 0.f;
#pragma unroll
      for (int k = 0; k < CE; ++k)
        if (cs + k < end) p[k] += v[k];
    }
    // the xor tree of wave_xor_sum<H> over the CE edge slots
#pragma unroll
    for (int o = 1; o < CE; o <<= 1) {
#pragma unroll
      for (int k = 0; k < CE; ++k)
        if ((k & o) == 0 && (k & (2 * o - 1)) == 0) p[k] = p[k] + p[k + o];
    }
    d_el[row * H + h_s] = p[0];
  }
}

// ------------------------------------------------------------------- dispatch ---
static bool shape_supported(int H, int F) {
#define X(h, f) if (H == h && F == f) return true;
  MSHA_FOR_EACH_SHAPE(X)
#undef X
  return false;
}

// integer tuning knob from the environment (A/B measurements; default = shipped choice)
static int env_int(const char* name, int def) {
  const char* v = getenv(name);
  return v != nullptr && *v ? atoi(v) : def;
}

// one wave per row (or chunk), 4 waves per block; grid-stride beyond the cap
static dim3 wave_grid(int64_t items) { return dim3(grid_for(items, 4, 1 << 20)); }

static int check_graph(const msha_graph* g, bool need_csc) {
  MSHA_ARG_CHECK(g != nullptr, "graph descriptor is NULL");
  MSHA_ARG_CHECK(g->n_rows > 0 && g->n_cols > 0 && g->n_edges >= 0, "graph: bad sizes");
  MSHA_ARG_CHECK(g->rowptr && (g->n_edges == 0 || g->col), "graph: CSR arrays missing");
  if (need_csc) {
    MSHA_ARG_CHECK(g->colptr && (g->n_edges == 0 || g->csc_row), "graph: CSC arrays missing");
    MSHA_ARG_CHECK(g->n_chunks >= g->n_cols && g->chunk_col && g->chunk_start && g->chunk_end,
                   "graph: CSC chunk plan missing (need >= 1 chunk per column)");
    MSHA_ARG_CHECK(g->n_multi == 0 || (g->multi_col && g->multi_first && g->multi_count),
                   "graph: multi-chunk column list missing");
  }
  return MSHA_OK;
}

}  // namespace msha

using namespace msha;

extern "C" int msha_edge_attention_supported(int32_t heads, int32_t feat) {
  return shape_supported(heads, feat) ? 1 : 0;
}

static bool dtype_ok(int32_t dtype, int32_t feat) {
  return dtype == MSHA_DTYPE_F32 || (dtype == MSHA_DTYPE_BF16 && feat % 8 == 0);
}

// the batched-gather forward applies: one piece per lane, every table addressable by
// 32-bit offsets
// MSHA_FWD_WAVES caps the forward's grid (waves then walk rows with the next row
// prefetched); default: short rows (mean degree <= FWD_SHORT_DEG) walk ~FWD_SHORT_RPW rows
// per wave
static dim3 fwd_grid(const msha_graph* g) {
  int64_t cap = env_int("MSHA_FWD_WAVES", -1);
  if (cap < 0)
    cap = g->n_edges <= (int64_t)FWD_SHORT_DEG * g->n_rows ? g->n_rows / FWD_SHORT_RPW : 0;
  return wave_grid(cap > 0 && cap < g->n_rows ? cap : g->n_rows);
}

static bool fwd_bat_ok(const msha_graph* g, int heads, int feat, int32_t dtype) {
  const int64_t lim = (int64_t)1 << 31;
  const int64_t esz = dtype == MSHA_DTYPE_BF16 ? 2 : 4;
  return env_int("MSHA_FWD_BAT", 1) != 0 && (int64_t)heads * feat * esz <= 1024 &&
         g->n_rows < lim && g->n_edges * 4 < lim && g->n_cols * 4 * heads < lim &&
         g->n_cols * heads * feat * esz < lim;
}

extern "C" int msha_edge_attention_rowterms_preferred(const msha_graph* g, int32_t heads,
                                                      int32_t feat, int32_t dtype) {
  if (g == nullptr || !shape_supported(heads, feat) || !dtype_ok(dtype, feat)) return 0;
  if (!fwd_bat_ok(g, heads, feat, dtype)) return 0;
  // MSHA_ROWTERMS: 1 = always, 0 = never.  Default: once the per-edge de would leave the
  // Infinity Cache (syn2m: fp32 step 11.70 -> 10.94 ms, bf16 7.34 -> 7.04 ms), and for
  // fp32 tables also on graphs whose rows average >= FWD_SHORT_DEG edges (C4: 0.507 ->
  // 0.494 ms).  Short rows (R15, ~2.3 edges) keep the de row sum: there the row terms'
  // extra forward work costs more (forward 48 -> 68 us) than the row sum they save.
  const int knob = env_int("MSHA_ROWTERMS", -1);
  if (knob >= 0) return knob != 0;
  if (g->n_edges * 4 * (int64_t)heads >= DE_SLOT_MIN_BYTES) return 1;
  return dtype == MSHA_DTYPE_F32 && g->n_edges >= (int64_t)FWD_SHORT_DEG * g->n_rows ? 1 : 0;
}

extern "C" int msha_edge_attention_fwd(const msha_graph* g, int32_t heads, int32_t feat,
                                       int32_t dtype, const float* el, const float* er,
                                       const void* hc, float neg_slope, float drop_p,
                                       uint64_t seed, uint64_t offset, void* u, void* u_lo,
                                       float* lse, float* attd, msha_stream_t stream) {
  return msha_edge_attention_fwd_ex(g, heads, feat, dtype, el, er, hc, neg_slope, drop_p, seed,
                                    offset, u, u_lo, lse, attd, nullptr, nullptr, stream);
}

extern "C" int msha_edge_attention_fwd_ex(const msha_graph* g, int32_t heads, int32_t feat,
                                          int32_t dtype, const float* el, const float* er,
                                          const void* hc, float neg_slope, float drop_p,
                                          uint64_t seed, uint64_t offset, void* u, void* u_lo,
                                          float* lse, float* attd, float* uc, float* qc,
                                          msha_stream_t stream) {
  if (int rc = check_graph(g, false)) return rc;
  MSHA_ARG_CHECK(el && er && hc && u && lse, "edge_attention_fwd: null pointer");
  MSHA_ARG_CHECK(drop_p >= 0.f && drop_p <= 1.f, "edge_attention_fwd: p must be in [0,1]");
  MSHA_ARG_CHECK((uc == nullptr) == (qc == nullptr), "edge_attention_fwd: uc and qc go together");
  if (!shape_supported(heads, feat) || !dtype_ok(dtype, feat))
    return fail(MSHA_ERR_UNSUPPORTED, "edge_attention_fwd: unsupported (heads, feat, dtype)");
  hipStream_t s = (hipStream_t)stream;
  const Dropout dp = make_dropout(drop_p, seed, offset, s);
  const bool bat = fwd_bat_ok(g, heads, feat, dtype);
  if (uc != nullptr && !bat)
    return fail(MSHA_ERR_UNSUPPORTED, "edge_attention_fwd: row terms need the batched forward");
  if (bat) {
    const dim3 grid = fwd_grid(g);
    // short rows (mean degree <= FWD_SHORT_DEG: R15, bip1m): the gather-layout forward
    // with FWD_SHORT_CEL-edge chunks (MSHA_FWD_GL=0: the batched kernel, A/B)
    const bool short_rows = g->n_edges <= (int64_t)FWD_SHORT_DEG * g->n_rows;
    if (short_rows && env_int("MSHA_FWD_GL", 1) != 0 &&
        launch_fwd_gl(g, heads, feat, dtype, el, er, nullptr, hc, neg_slope, dp, u, u_lo, lse,
                      attd, uc, qc, true, grid, s))
      return check_launch("edge_attention_fwd");
#define XB(h, f)                                                                               \
    if (heads == h && feat == f) {                                                             \
      if (dtype == MSHA_DTYPE_BF16) {                                                          \
        if constexpr (f % 8 == 0 && h * f * 2 <= 1024) {                                       \
          auto kern = uc != nullptr                                                            \
              ? edge_attn_fwd_bat_kernel<h, f, bf16_t, fwd_epl<h, f, bf16_t>(), true>          \
              : edge_attn_fwd_bat_kernel<h, f, bf16_t, fwd_epl<h, f, bf16_t>(), false>;        \
          hipLaunchKernelGGL(kern, grid, dim3(256), 0, s, g->rowptr, g->col, g->rowflag,       \
                             (int32_t)g->n_rows, (int32_t)g->n_cols, (int32_t)g->n_edges, el,  \
                             er, (const bf16_t*)hc, neg_slope, dp, (bf16_t*)u,                 \
                             (bf16_t*)u_lo, lse, attd, uc, qc);                                \
        }                                                                                      \
      } else {                                                                                 \
        if constexpr (h * f * 4 <= 1024) {                                                     \
          auto kern = uc != nullptr                                                            \
              ? edge_attn_fwd_bat_kernel<h, f, float, fwd_epl<h, f, float>(), true>            \
              : edge_attn_fwd_bat_kernel<h, f, float, fwd_epl<h, f, float>(), false>;          \
          hipLaunchKernelGGL(kern, grid, dim3(256), 0, s, g->rowptr, g->col, g->rowflag,       \
                             (int32_t)g->n_rows, (int32_t)g->n_cols, (int32_t)g->n_edges, el,  \
                             er, (const float*)hc, neg_slope, dp, (float*)u, (float*)nullptr,  \
                             lse, attd, uc, qc);                                               \
        }                                                                                      \
      }                                                                                        \
    }
    MSHA_FOR_EACH_SHAPE(XB)
#undef XB
    return check_launch("edge_attention_fwd");
  }
#define X(h, f)                                                                                \
  if (heads == h && feat == f) {                                                               \
    if (dtype == MSHA_DTYPE_BF16) {                                                            \
      if constexpr (f % 8 == 0)                                                                \
        hipLaunchKernelGGL((edge_attn_fwd_kernel<h, f, bf16_t, fwd_epl<h, f, bf16_t>()>),      \
                           wave_grid(g->n_rows), dim3(256), 0, s, g->rowptr, g->col,           \
                           g->rowflag, g->n_rows, el, er, (const bf16_t*)hc, neg_slope, dp,    \
                           (bf16_t*)u, (bf16_t*)u_lo, lse, attd);                              \
    } else {                                                                                   \
      hipLaunchKernelGGL((edge_attn_fwd_kernel<h, f, float, fwd_epl<h, f, float>()>),          \
                         wave_grid(g->n_rows), dim3(256), 0, s, g->rowptr, g->col, g->rowflag, \
                         g->n_rows, el, er, (const float*)hc, neg_slope, dp, (float*)u,        \
                         (float*)nullptr, lse, attd);                                          \
    }                                                                                          \
  }
  MSHA_FOR_EACH_SHAPE(X)
#undef X
  return check_launch("edge_attention_fwd");
}

template <typename T>
static void launch_bwd_rows(const msha_graph* g, int heads, int feat, const float* el,
                            const float* er, const void* hc, const float* lse, const void* u,
                            const void* u_lo, const void* dU, const void* hs, const void* dV, const float* row_coef,
                            float neg_slope, const Dropout& dp, float* d_el, float* de,
                            float* attd, int ld, void* d_hs, hipStream_t s) {
#define X(h, f)                                                                                  \
  if (heads == h && feat == f) {                                                                 \
    if constexpr (f % Pk<T>::V == 0) {                                                           \
      if (dV)                                                                                    \
        hipLaunchKernelGGL((edge_attn_bwd_rows_kernel<h, f, T, true>), wave_grid(g->n_rows),     \
                           dim3(256), 0, s, g->rowptr, g->col, g->rowflag, g->n_rows, el, er,    \
                           (const T*)hc, lse, (const T*)u, (const T*)u_lo, (const T*)dU,         \
                           (const T*)hs,                                                         \
                           (const T*)dV, row_coef, neg_slope, dp, d_el, de, attd, ld, (T*)d_hs); \
      else                                                                                       \
        hipLaunchKernelGGL((edge_attn_bwd_rows_kernel<h, f, T, false>), wave_grid(g->n_rows),    \
                           dim3(256), 0, s, g->rowptr, g->col, g->rowflag, g->n_rows, el, er,    \
                           (const T*)hc, lse, (const T*)u, (const T*)u_lo, (const T*)dU,         \
                           (const T*)hs,                                                         \
                           (const T*)dV, row_coef, neg_slope, dp, d_el, de, attd, ld, (T*)d_hs); \
    }                                                                                            \
  }
  MSHA_FOR_EACH_SHAPE(X)
#undef X
}

extern "C" int msha_edge_attention_bwd_rows(const msha_graph* g, int32_t heads, int32_t feat,
                                            int32_t dtype, const float* el, const float* er,
                                            const void* hc, const float* lse, const void* u,
                                            const void* u_lo, const void* dU, const void* hs,
                                            const void* dV,
                                            const float* row_coef, float neg_slope,
                                            float drop_p, uint64_t seed, uint64_t offset,
                                            float* d_el, float* de, float* attd,
                                            int32_t edge_ld, void* d_hs, msha_stream_t stream) {
  if (int rc = check_graph(g, false)) return rc;
  MSHA_ARG_CHECK(el && er && hc && lse && u && dU && d_el && de && attd,
                 "edge_attention_bwd_rows: null pointer");
  MSHA_ARG_CHECK(dV == nullptr || (hs && d_hs), "edge_attention_bwd_rows: dV needs hs and d_hs");
  MSHA_ARG_CHECK(drop_p >= 0.f && drop_p <= 1.f, "edge_attention_bwd_rows: p must be in [0,1]");
  const int ld = edge_ld > 0 ? edge_ld : heads;
  MSHA_ARG_CHECK(ld >= heads, "edge_attention_bwd_rows: edge_ld < heads");
  if (!shape_supported(heads, feat) || !dtype_ok(dtype, feat))
    return fail(MSHA_ERR_UNSUPPORTED, "edge_attention_bwd_rows: unsupported (heads, feat, dtype)");
  hipStream_t s = (hipStream_t)stream;
  const Dropout dp = make_dropout(drop_p, seed, offset, s);
  // short rows (R15, bip1m): the gather-layout row pass (MSHA_BWD_GL=0: this file's, A/B)
  const bool short_rows = g->n_edges <= (int64_t)FWD_SHORT_DEG * g->n_rows;
  if (short_rows && env_int("MSHA_BWD_GL", 1) != 0 && fwd_bat_ok(g, heads, feat, dtype) &&
      launch_bwd_rows_gl(g, heads, feat, dtype, el, er, hc, lse, u,
                         dtype == MSHA_DTYPE_BF16 ? u_lo : nullptr, dU, hs, dV, row_coef,
                         neg_slope, dp, d_el, de, attd, ld, d_hs, fwd_grid(g), s))
    return check_launch("edge_attention_bwd_rows");
  if (dtype == MSHA_DTYPE_BF16)
    launch_bwd_rows<bf16_t>(g, heads, feat, el, er, hc, lse, u, u_lo, dU, hs, dV, row_coef,
                            neg_slope,
                            dp, d_el, de, attd, ld, d_hs, s);
  else
    launch_bwd_rows<float>(g, heads, feat, el, er, hc, lse, u, nullptr, dU, hs, dV, row_coef,
                           neg_slope,
                           dp, d_el, de, attd, ld, d_hs, s);
  return check_launch("edge_attention_bwd_rows");
}

extern "C" size_t msha_csc_aggregate_workspace_size(const msha_graph* g, int32_t heads,
                                                    int32_t feat) {
  if (g == nullptr || heads <= 0 || feat <= 0) return 0;
  const size_t per = (size_t)heads * (size_t)feat + (size_t)heads;
  return (size_t)g->n_chunks * per * sizeof(float) + 256;
}

template <typename T>
static void launch_csc(const msha_graph* g, int heads, int feat, const float* w, const float* x,
                       int ld, const void* table, void* out, float* out_x, float* part,
                       float* part_x, hipStream_t s) {
#define X(h, f)                                                                                 \
  if (heads == h && feat == f) {                                                                \
    if constexpr (f % Pk<T>::V == 0) {                                                          \
      if (x)                                                                                    \
        hipLaunchKernelGGL((csc_aggregate_kernel<h, f, T, true>), wave_grid(g->n_chunks),       \
                           dim3(256), 0, s, g->chunk_col, g->chunk_start, g->chunk_end,         \
                           g->n_chunks, g->colptr, g->csc_row, g->csc_eid, w, x, ld,            \
                           (const T*)table, (T*)out, out_x, part, part_x);                      \
      else                                                                                      \
        hipLaunchKernelGGL((csc_aggregate_kernel<h, f, T, false>), wave_grid(g->n_chunks),      \
                           dim3(256), 0, s, g->chunk_col, g->chunk_start, g->chunk_end,         \
                           g->n_chunks, g->colptr, g->csc_row, g->csc_eid, w, x, ld,            \
                           (const T*)table, (T*)out, out_x, part, part_x);                      \
    }                                                                                           \
  }
  MSHA_FOR_EACH_SHAPE(X)
#undef X
  if (g->n_multi > 0) {
    const int64_t D = (int64_t)heads * feat;
    const int64_t W = D + (x ? heads : 0);
    hipLaunchKernelGGL(csc_combine_kernel<T>, dim3(g->n_multi, (W + 255) / 256),
                       dim3(64 * kCombineWaves), 0, s, g->multi_col, g->multi_first,
                       g->multi_count, g->n_multi, (int)D, heads, part, x ? part_x : nullptr,
                       (T*)out, out_x);
  }
}

extern "C" int msha_csc_aggregate(const msha_graph* g, int32_t heads, int32_t feat,
                                  int32_t dtype, const float* w, const float* x, int32_t edge_ld,
                                  const void* table, void* out, float* out_x, void* ws,
                                  size_t ws_bytes, msha_stream_t stream) {
  if (int rc = check_graph(g, true)) return rc;
  MSHA_ARG_CHECK(w && table && out, "csc_aggregate: null pointer");
  MSHA_ARG_CHECK(x == nullptr || out_x != nullptr, "csc_aggregate: x needs out_x");
  if (!shape_supported(heads, feat) || !dtype_ok(dtype, feat))
    return fail(MSHA_ERR_UNSUPPORTED, "csc_aggregate: unsupported (heads, feat, dtype)");
  const int64_t D = (int64_t)heads * feat;
  float* part = nullptr;
  float* part_x = nullptr;
  if (g->n_multi > 0) {
    MSHA_ARG_CHECK(ws != nullptr && ws_bytes >= msha_csc_aggregate_workspace_size(g, heads, feat),
                   "csc_aggregate: workspace too small");
    part = (float*)ws;
    part_x = part + g->n_chunks * D;
  }
  hipStream_t s = (hipStream_t)stream;
  const int ld = edge_ld > 0 ? edge_ld : heads;
  MSHA_ARG_CHECK(ld >= heads, "csc_aggregate: edge_ld < heads");
  if (dtype == MSHA_DTYPE_BF16)
    launch_csc<bf16_t>(g, heads, feat, w, x, ld, table, out, out_x, part, part_x, s);
  else
    launch_csc<float>(g, heads, feat, w, x, ld, table, out, out_x, part, part_x, s);
  return check_launch("csc_aggregate");
}

extern "C" size_t msha_edge_attention_bwd_fused_workspace_size(const msha_graph* g,
                                                               int32_t heads, int32_t feat) {
  if (g == nullptr || heads <= 0 || feat <= 0) return 0;
  const size_t rec = ((size_t)g->n_rows * rec_stride(heads) * sizeof(float) + 255) & ~(size_t)255;
  return rec + msha_csc_aggregate_workspace_size(g, heads, feat);
}

template <typename T>
static void launch_bwd_fused(const msha_graph* g, int heads, int feat, const float* el,
                             const float* er, const float* ar, const void* hc, const float* lse, const void* u,
                             const void* u_lo, const void* dU, float neg_slope, const Dropout& dp, float* d_el,
                             float* d_er, void* d_hc, float* de, float* rec, float* part,
                             float* part_x, const float* uc, const float* qc, hipStream_t s) {
  const bool rt = uc != nullptr;  // row terms: d_el in the row pass, no de, no row sum
  if (rt) de = nullptr;
  // the buffer-descriptor kernel addresses each table with 32-bit byte offsets
  const int64_t lim = (int64_t)1 << 31;
  // de in CSC slot order (contiguous writes, gathered by the row sum) once it outgrows
  // the Infinity Cache; below that the cache absorbs the scattered 4H-byte writes and
  // the CSR-order row sum reads it contiguously (measured: syn100k's 64 MB de is faster
  // in edge order, syn2m's 1.28 GB in slot order)
  const bool slot_de = g->csr_slot != nullptr && g->n_edges * 4 * (int64_t)heads >= DE_SLOT_MIN_BYTES;
  // MSHA_COLS_NOBUF=1 forces the pointer-load column pass (what tables of 2 GiB or more
  // take) so tests cover it at small sizes; read per call, so a test can flip it
  const char* nobuf = getenv("MSHA_COLS_NOBUF");
  const bool buf_ok = !(nobuf != nullptr && *nobuf == '1') &&
                      g->n_rows * (int64_t)heads * feat * (int64_t)sizeof(T) < lim &&
                      g->n_edges * 4 * (int64_t)heads < lim && g->n_rows * 4 * rec_stride(heads) < lim;
#define X(h, f)                                                                                \
  if (heads == h && feat == f) {                                                               \
    if constexpr (f % Pk<T>::V == 0) {                                                         \
      auto row_stats = rt ? bwd_row_stats_kernel<h, f, T, true>                                \
                          : bwd_row_stats_kernel<h, f, T, false>;                              \
      hipLaunchKernelGGL(row_stats,                                                            \
                         wave_grid(g->n_rows / 8 + 1), dim3(256), 0, s, g->n_rows, el, lse,   \
                         (const T*)u, (const T*)u_lo, (const T*)dU, rec, uc, qc, g->rowflag,  \
                         d_el);                                                                \
      if (f * sizeof(T) <= 64 && COLS_EH && buf_ok)                                            \
        hipLaunchKernelGGL((ar != nullptr ? bwd_cols_eh_kernel<h, f, T, true>                 \
                                           : bwd_cols_eh_kernel<h, f, T, false>),               \
                           wave_grid(g->n_chunks), dim3(256), 0,                                \
                           s, g->chunk_col, g->chunk_start, g->chunk_end, g->n_chunks,         \
                           g->colptr, g->csc_row, g->csc_eid, g->n_edges, g->rowflag,          \
                           g->n_rows, rec, er, ar, (const T*)hc, (const T*)dU, neg_slope, dp,  \
                           slot_de, de,                                                        \
                           (T*)d_hc, d_er, part, part_x);                                      \
      else                                                                                     \
      {                                                                                        \
        auto kern = ar != nullptr                                                              \
            ? (buf_ok ? bwd_cols_kernel<h, f, T, true, true> : bwd_cols_kernel<h, f, T, false, true>) \
            : (buf_ok ? bwd_cols_kernel<h, f, T, true> : bwd_cols_kernel<h, f, T, false>);     \
        hipLaunchKernelGGL(kern, wave_grid(g->n_chunks), dim3(256), 0,                         \
                           s, g->chunk_col, g->chunk_start, g->chunk_end, g->n_chunks,         \
                           g->colptr, g->csc_row, g->csc_eid, g->n_rows, g->rowflag, rec, er,  \
                           ar, (const T*)hc, (const T*)dU, neg_slope, dp, slot_de,             \
                           de, (T*)d_hc, d_er,                                                 \
                           part, part_x);                                                      \
      }                                                                                        \
      if (!rt)                                                                                 \
        hipLaunchKernelGGL((bwd_row_sum_kernel<h>), wave_grid(g->n_rows), dim3(256), 0, s,     \
                           g->rowptr, g->n_rows, de, slot_de ? g->csr_slot : nullptr, d_el);  \
    }                                                                                          \
  }
  MSHA_FOR_EACH_SHAPE(X)
#undef X
  if (g->n_multi > 0) {
    const int64_t D = (int64_t)heads * feat;
    hipLaunchKernelGGL(csc_combine_kernel<T>, dim3(g->n_multi, (D + heads + 255) / 256),
                       dim3(64 * kCombineWaves), 0, s, g->multi_col, g->multi_first,
                       g->multi_count, g->n_multi, (int)D, heads, part, part_x, (T*)d_hc, d_er);
  }
}

extern "C" int msha_edge_attention_bwd_fused(const msha_graph* g, int32_t heads, int32_t feat,
                                             int32_t dtype, const float* el, const float* er,
                                             const void* hc, const float* lse, const void* u,
                                             const void* u_lo, const void* dU, float neg_slope,
                                             float drop_p,
                                             uint64_t seed, uint64_t offset, float* d_el,
                                             float* d_er, void* d_hc, float* de, void* ws,
                                             size_t ws_bytes, msha_stream_t stream) {
  return msha_edge_attention_bwd_fused_ex(g, heads, feat, dtype, el, er, hc, lse, u, u_lo, dU,
                                          neg_slope, drop_p, seed, offset, nullptr, nullptr,
                                          d_el, d_er, d_hc, de, ws, ws_bytes, stream);
}

extern "C" int msha_edge_attention_bwd_fused_ex(
    const msha_graph* g, int32_t heads, int32_t feat, int32_t dtype, const float* el,
    const float* er, const void* hc, const float* lse, const void* u, const void* u_lo,
    const void* dU, float neg_slope, float drop_p, uint64_t seed, uint64_t offset,
    const float* uc, const float* qc, float* d_el, float* d_er, void* d_hc, float* de, void* ws,
    size_t ws_bytes, msha_stream_t stream) {
  if (int rc = check_graph(g, true)) return rc;
  MSHA_ARG_CHECK(el && er && hc && lse && u && dU && d_el && d_er && d_hc,
                 "edge_attention_bwd_fused: null pointer");
  MSHA_ARG_CHECK((uc == nullptr) == (qc == nullptr), "edge_attention_bwd_fused: uc and qc go together");
  MSHA_ARG_CHECK(g->n_edges == 0 || ((de || uc) && g->csc_eid),
                 "edge_attention_bwd_fused: needs de scratch (or row terms) and csc_eid");
  MSHA_ARG_CHECK(drop_p >= 0.f && drop_p <= 1.f, "edge_attention_bwd_fused: p must be in [0,1]");
  if (!shape_supported(heads, feat) || !dtype_ok(dtype, feat))
    return fail(MSHA_ERR_UNSUPPORTED, "edge_attention_bwd_fused: unsupported (heads, feat, dtype)");
  MSHA_ARG_CHECK(ws != nullptr &&
                     ws_bytes >= msha_edge_attention_bwd_fused_workspace_size(g, heads, feat),
                 "edge_attention_bwd_fused: workspace too small");
  const int64_t D = (int64_t)heads * feat;
  float* rec = (float*)ws;
  const size_t rec_bytes = ((size_t)g->n_rows * rec_stride(heads) * sizeof(float) + 255) & ~(size_t)255;
  float* part = (float*)((char*)ws + rec_bytes);
  float* part_x = part + g->n_chunks * D;
  hipStream_t s = (hipStream_t)stream;
  const Dropout dp = make_dropout(drop_p, seed, offset, s);
  if (dtype == MSHA_DTYPE_BF16)
    launch_bwd_fused<bf16_t>(g, heads, feat, el, er, nullptr, hc, lse, u, u_lo, dU, neg_slope, dp,
                             d_el, d_er, d_hc, de, rec, part, part_x, uc, qc, s);
  else
    launch_bwd_fused<float>(g, heads, feat, el, er, nullptr, hc, lse, u, nullptr, dU, neg_slope, dp,
                            d_el, d_er, d_hc, de, rec, part, part_x, uc, qc, s);
  return check_launch("edge_attention_bwd_fused");
}

// ---------------------------------------------------- scores from the gathered row ---
extern "C" int msha_edge_attention_row_scores_supported(const msha_graph* g, int32_t heads,
                                                        int32_t feat, int32_t dtype) {
  if (g == nullptr || !shape_supported(heads, feat) || !dtype_ok(dtype, feat)) return 0;
  return fwd_bat_ok(g, heads, feat, dtype) ? 1 : 0;
}

// MSHA_ROW_SCORES: 1 = whenever supported, 0 = never (A/B).  Default: whenever supported.
// fp32: C4 forward 174 -> 149 us, syn2m 3900 -> 3652 us.  bf16: in round 3 the C4 forward
// (3.2 MB er, L2-resident) ran slower on row scores (98 -> 111 us) and took them only
// once the er table outgrew an XCD's L2; on the round-4 gather-layout forward they win
// there too (C4 bf16 forward 101 -> 94 us, step 0.325 -> 0.318 ms,
// profiles/round4_rs_bf16_ab/), and the er gather's extra traffic is gone.
#ifndef RS_BF16_MIN_BYTES
#define RS_BF16_MIN_BYTES 0ll
#endif
extern "C" int msha_edge_attention_row_scores_preferred(const msha_graph* g, int32_t heads,
                                                        int32_t feat, int32_t dtype) {
  if (!msha_edge_attention_row_scores_supported(g, heads, feat, dtype)) return 0;
  const int knob = env_int("MSHA_ROW_SCORES", -1);
  if (knob >= 0) return knob != 0;
  if (dtype == MSHA_DTYPE_F32) return 1;
  return g->n_cols * 4 * (int64_t)heads >= RS_BF16_MIN_BYTES ? 1 : 0;
}

extern "C" int msha_edge_attention_fwd_rs(const msha_graph* g, int32_t heads, int32_t feat,
                                          int32_t dtype, const float* el, const float* ar,
                                          const void* hc, float neg_slope, float drop_p,
                                          uint64_t seed, uint64_t offset, void* u, void* u_lo,
                                          float* lse, float* uc, float* qc,
                                          msha_stream_t stream) {
  if (int rc = check_graph(g, false)) return rc;
  MSHA_ARG_CHECK(el && ar && hc && u && lse, "edge_attention_fwd_rs: null pointer");
  MSHA_ARG_CHECK(drop_p >= 0.f && drop_p <= 1.f, "edge_attention_fwd_rs: p must be in [0,1]");
  MSHA_ARG_CHECK((uc == nullptr) == (qc == nullptr), "edge_attention_fwd_rs: uc and qc go together");
  MSHA_ARG_CHECK(((uintptr_t)ar & 15) == 0, "edge_attention_fwd_rs: a_r must be 16-byte aligned");
  if (!msha_edge_attention_row_scores_supported(g, heads, feat, dtype))
    return fail(MSHA_ERR_UNSUPPORTED, "edge_attention_fwd_rs: unsupported (heads, feat, dtype, sizes)");
  hipStream_t s = (hipStream_t)stream;
  const Dropout dp = make_dropout(drop_p, seed, offset, s);
  const bool short_rows = g->n_edges <= (int64_t)FWD_SHORT_DEG * g->n_rows;
  if (!launch_fwd_gl(g, heads, feat, dtype, el, nullptr, ar, hc, neg_slope, dp, u, u_lo, lse,
                     nullptr, uc, qc, short_rows, fwd_grid(g), s))
    return fail(MSHA_ERR_UNSUPPORTED, "edge_attention_fwd_rs: shape not compiled");
  return check_launch("edge_attention_fwd_rs");
}

extern "C" int msha_edge_attention_bwd_fused_rs(
    const msha_graph* g, int32_t heads, int32_t feat, int32_t dtype, const float* el,
    const float* ar, const void* hc, const float* lse, const void* u, const void* u_lo,
    const void* dU, float neg_slope, float drop_p, uint64_t seed, uint64_t offset,
    const float* uc, const float* qc, float* d_el, float* d_er, void* d_hc, float* de, void* ws,
    size_t ws_bytes, msha_stream_t stream) {
  if (int rc = check_graph(g, true)) return rc;
  MSHA_ARG_CHECK(el && ar && hc && lse && u && dU && d_el && d_er && d_hc,
                 "edge_attention_bwd_fused_rs: null pointer");
  MSHA_ARG_CHECK((uc == nullptr) == (qc == nullptr), "edge_attention_bwd_fused_rs: uc and qc go together");
  MSHA_ARG_CHECK(g->n_edges == 0 || ((de || uc) && g->csc_eid),
                 "edge_attention_bwd_fused_rs: needs de scratch (or row terms) and csc_eid");
  MSHA_ARG_CHECK(drop_p >= 0.f && drop_p <= 1.f, "edge_attention_bwd_fused_rs: p must be in [0,1]");
  MSHA_ARG_CHECK(((uintptr_t)ar & 15) == 0, "edge_attention_bwd_fused_rs: a_r must be 16-byte aligned");
  if (!msha_edge_attention_row_scores_supported(g, heads, feat, dtype))
    return fail(MSHA_ERR_UNSUPPORTED, "edge_attention_bwd_fused_rs: unsupported (heads, feat, dtype, sizes)");
  MSHA_ARG_CHECK(ws != nullptr &&
                     ws_bytes >= msha_edge_attention_bwd_fused_workspace_size(g, heads, feat),
                 "edge_attention_bwd_fused_rs: workspace too small");
  const int64_t D = (int64_t)heads * feat;
  float* rec = (float*)ws;
  const size_t rec_bytes = ((size_t)g->n_rows * rec_stride(heads) * sizeof(float) + 255) & ~(size_t)255;
  float* part = (float*)((char*)ws + rec_bytes);
  float* part_x = part + g->n_chunks * D;
  hipStream_t s = (hipStream_t)stream;
  const Dropout dp = make_dropout(drop_p, seed, offset, s);
  if (dtype == MSHA_DTYPE_BF16)
    launch_bwd_fused<bf16_t>(g, heads, feat, el, nullptr, ar, hc, lse, u, u_lo, dU, neg_slope, dp,
                             d_el, d_er, d_hc, de, rec, part, part_x, uc, qc, s);
  else
    launch_bwd_fused<float>(g, heads, feat, el, nullptr, ar, hc, lse, u, nullptr, dU, neg_slope, dp,
                            d_el, d_er, d_hc, de, rec, part, part_x, uc, qc, s);
  return check_launch("edge_attention_bwd_fused_rs");
}
