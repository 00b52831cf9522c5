// Row half of the edge-attention backward for short rows, gather layout
// (msha_edge_attention_bwd_rows on graphs whose rows average <= FWD_SHORT_DEG edges:
// R15 and the repo-shape bip1m graph, ~2.3 edges per row).
//
// Reference: the autograd of Ablation.py:266-274 (OursLayer3: scores, masked softmax,
// dropout, u = att @ h1 and v = att.T @ h2), and of Ours.py:84-86 (SUM_county's sum of
// exp(attention_inter) over the batch rows: the row coefficients).  Per row i, head h:
//   D_i  = dU_i . u_i (+ hs_i . w_i, w_i = sum_e attd_e dV_j = d_hs_i)
//          (+ coef_i sum_e attd_e exp(attd_e))
//   g_e  = dU_i . hc_j (+ hs_i . dV_j) (+ coef_i exp(attd_e))
//   ds_e = att_e (drop_e g_e - D_i),  de_e = ds_e lrelu'(pre_e),  d_el_i = sum_e de_e
// written as de / attd records (ld floats per edge) for the column pass
// (msha_csc_aggregate) and d_el, d_hs.
//
// edge_attn_bwd_rows_kernel walks one row per wave with the score layout's 64 / H edge
// slots (R15: 32 slots of masked gathers for 2.3 edges) and branchy pointer loads.  Here
// a chunk is NGI gather instructions of EPI edge slots each (CEL = NGI * EPI edges,
// FWD_SHORT_CEL = 4), every load of a chunk goes out at once through buffer descriptors
// (masked slots read 0), and the first chunk's gathers (hc_j, dV_j, er_j and the dropout
// bits) are loaded once for both passes over the row.
#include "edge_geo.h"

namespace msha {

template <int H, int F, typename T, int NGI, bool DV>
__global__ void __launch_bounds__(256) edge_attn_bwd_rows_gl_kernel(
    const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
    const uint8_t* __restrict__ rowflag, int32_t n_rows, int32_t n_cols, int32_t n_edges,
    const float* __restrict__ el, const float* __restrict__ er, const T* __restrict__ hc,
    const float* __restrict__ lse, const T* __restrict__ u, const T* __restrict__ u_lo,
    const T* __restrict__ dU, const T* __restrict__ hs, const T* __restrict__ dV,
    const float* __restrict__ row_coef, float slope, Dropout dp, float* __restrict__ d_el,
    float* __restrict__ de, float* __restrict__ attd, int ld, T* __restrict__ d_hs) {
  using G = Geo<H, F, T>;
  static_assert(G::QPL == 1, "gather-layout backward: one 16-byte piece per lane");
  constexpr int CEL = NGI * G::EPI;
  constexpr int NB = (CEL * H + 63) / 64;
  const int lane = lane_id();
  const int g_e = lane / G::NQ, q = lane % G::NQ;
  const int hq = q / G::QH;
  const bool lead = q % G::QH == 0;  // one lane per (edge slot, head) writes
  const uint32_t RB = (uint32_t)(G::D * sizeof(T));
  const rsrc_t r_col = make_rsrc(col, (uint32_t)n_edges * 4u);
  const rsrc_t r_er = make_rsrc(er, (uint32_t)n_cols * (4u * H));
  const rsrc_t r_hc = make_rsrc(hc, (uint32_t)n_cols * RB);
  const rsrc_t r_dV = make_rsrc(DV ? dV : nullptr, (uint32_t)n_cols * RB);
  const uint32_t q_off = 16u * q;
  const int wave0 = __builtin_amdgcn_readfirstlane((int)(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6));
  const int nwaves = (int)(((int64_t)gridDim.x * blockDim.x) >> 6);

  // one chunk's gathered operands (edge slot gi * EPI + g_e of the chunk)
  struct Chunk {
    u32x4_t h[NGI], v[NGI];
    float er[NGI];
    uint64_t kb[NB];
  };
  auto load_cols = [&](int32_t cs, int32_t end, int32_t (&j)[NGI]) {
#pragma unroll
    for (int gi = 0; gi < NGI; ++gi) {
      const int32_t e = cs + gi * G::EPI + g_e;
      j[gi] = buf_i32(r_col, e < end ? (uint32_t)e * 4u : kOOB);
    }
  };
  auto load_chunk = [&](int32_t cs, int32_t end, const int32_t (&j)[NGI], Chunk& c) {
#pragma unroll
    for (int gi = 0; gi < NGI; ++gi) {
      const bool valid = cs + gi * G::EPI + g_e < end;
      const uint32_t off = valid ? (uint32_t)j[gi] * RB + q_off : kOOB;
      c.h[gi] = buf_b128(r_hc, off);
      if (DV) c.v[gi] = buf_b128(r_dV, off);
      c.er[gi] = buf_f32(r_er, valid ? (uint32_t)j[gi] * (4u * H) + 4u * hq : kOOB);
    }
    if (dp.active) {  // lanes edge * H + head of NB ballots (the forward's element order)
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const int idx = b * 64 + lane;
        c.kb[b] = __ballot(idx < CEL * H &&
                           dropout_factor(dp, (uint64_t)(cs + idx / H) * H + (idx % H)) != 0.f);
      }
    }
  };
  auto drop_of = [&](const Chunk& c, int gi) -> float {
    if (!dp.active) return 1.f;
    const int bit = (gi * G::EPI + g_e) * H + hq;
    return (c.kb[bit >> 6] >> (bit & 63)) & 1ull ? dp.scale : 0.f;
  };

  int row = wave0;
  if (row >= n_rows) return;
  int32_t start = __builtin_amdgcn_readfirstlane(rowptr[row]);
  int32_t end = __builtin_amdgcn_readfirstlane(rowptr[row + 1]);
  int32_t jc[NGI];
  load_cols(start, end, jc);
  while (true) {
    const bool virt = rowflag != nullptr && rowflag[row] != 0;
    const float elq = el[(int64_t)row * H + hq];
    const float lseq = lse[(int64_t)row * H + hq];
    const float coef = row_coef != nullptr ? row_coef[(int64_t)row * H + hq] : 0.f;
    const int64_t roff = (int64_t)row * G::D + G::V * q;
    const Pk<T> dUq = pk_load(dU + roff);
    float dpart = pk_dot(dUq, pk_load(u + roff));
    if (sizeof(T) == 2 && u_lo != nullptr) dpart += pk_dot(dUq, pk_load(u_lo + roff));
    Pk<T> hsq = pk_zero<T>();
    if (DV) hsq = pk_load(hs + roff);
    Chunk c0;
    load_chunk(start, end, jc, c0);
    // the next row's bounds and first columns while this row runs
    const int nrow_raw = row + nwaves;
    const bool has_next = nrow_raw < n_rows;
    const int nrow = has_next ? nrow_raw : row;
    const int32_t nstart = __builtin_amdgcn_readfirstlane(rowptr[nrow]);
    const int32_t nend = __builtin_amdgcn_readfirstlane(rowptr[nrow + 1]);
    int32_t njc[NGI];
    load_cols(nstart, nend, njc);

    // pass A: w_i = sum_e attd_e dV_j (the v branch) and the row coefficient's sum
    const bool any_coef = __ballot(coef != 0.f) != 0;
    Pk<T> wacc = pk_zero<T>();
    float tco = 0.f;
    if (DV || any_coef) {
      for (int32_t cs = start; cs < end; cs += CEL) {
        Chunk c = c0;  // a copy, not a pointer: the chunk stays in registers
        if (cs != start) {
          int32_t j[NGI];
          load_cols(cs, end, j);
          load_chunk(cs, end, j, c);
        }
#pragma unroll
        for (int gi = 0; gi < NGI; ++gi) {
          const bool valid = cs + gi * G::EPI + g_e < end;
          const float s = virt ? 0.f : lrelu(elq + c.er[gi], slope);
          const float ad = valid ? __expf(s - lseq) * drop_of(c, gi) : 0.f;
          if (DV) wacc = pk_fma(ad, pk_from_raw(c.v[gi], (T*)nullptr), wacc);
          if (any_coef) tco += ad * expf(ad);
        }
      }
      if (G::EPI > 1) {
#pragma unroll
        for (int o = G::NQ; o < 64; o <<= 1) {
          if (DV) wacc = pk_xor_add(wacc, o);
          if (any_coef) tco += xor_shfl(tco, o);
        }
      }
      if (DV) {
        if (g_e == 0) pk_store(d_hs + roff, wacc);
        dpart += pk_dot(hsq, wacc);
      }
    }
    // D_i per head (replicated over the head's lanes)
    float Dq = group_sum<G::QH>(dpart);
    if (any_coef) Dq += coef * tco;

    // pass B: the per-edge score gradients
    float del = 0.f;
    for (int32_t cs = start; cs < end; cs += CEL) {
      Chunk c = c0;
      if (cs != start) {
        int32_t j[NGI];
        load_cols(cs, end, j);
        load_chunk(cs, end, j, c);
      }
#pragma unroll
      for (int gi = 0; gi < NGI; ++gi) {
        const int32_t e = cs + gi * G::EPI + g_e;
        const bool valid = e < end;
        const float pre = elq + c.er[gi];
        const float s = virt ? 0.f : lrelu(pre, slope);
        const float att = valid ? __expf(s - lseq) : 0.f;
        const float dropf = drop_of(c, gi);
        float t = pk_dot(dUq, pk_from_raw(c.h[gi], (T*)nullptr));
        if (DV) t += pk_dot(hsq, pk_from_raw(c.v[gi], (T*)nullptr));
        float g = group_sum<G::QH>(t);
        if (any_coef && valid) g += coef * expf(att * dropf);
        const float ds = att * (g * dropf - Dq);
        const float dev = virt ? 0.f : ds * (pre > 0.f ? 1.f : slope);
        if (lead && valid) {
          de[(int64_t)e * ld + hq] = dev;
          attd[(int64_t)e * ld + hq] = att * dropf;
        }
        del += valid ? dev : 0.f;
      }
    }
#pragma unroll
    for (int o = G::NQ; o < 64; o <<= 1) del += xor_shfl(del, o);
    if (g_e == 0 && lead) d_el[(int64_t)row * H + hq] = del;
    if (!has_next) break;
    row = nrow;
    start = nstart;
    end = nend;
#pragma unroll
    for (int gi = 0; gi < NGI; ++gi) jc[gi] = njc[gi];
  }
}

template <int H, int F, typename T>
static void launch_bwd_gl_shape(const msha_graph* g, const float* el, const float* er,
                                const void* hc, const float* lse, const void* u,
                                const void* u_lo, const void* dU, const void* hs,
                                const void* dV, const float* row_coef, float slope,
                                const Dropout& dp, float* d_el, float* de, float* attd, int ld,
                                void* d_hs, dim3 grid, hipStream_t s) {
  constexpr int NGI = gl_ngi_short<H, F, T>();
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, dim3(256), 0, s, g->rowptr, g->col, g->rowflag,
                       (int32_t)g->n_rows, (int32_t)g->n_cols, (int32_t)g->n_edges, el, er,
                       (const T*)hc, lse, (const T*)u, (const T*)u_lo, (const T*)dU,
                       (const T*)hs, (const T*)dV, row_coef, slope, dp, d_el, de, attd, ld,
                       (T*)d_hs);
  };
  if (dV != nullptr) go(edge_attn_bwd_rows_gl_kernel<H, F, T, NGI, true>);
  else go(edge_attn_bwd_rows_gl_kernel<H, F, T, NGI, false>);
}

int launch_bwd_rows_gl(const msha_graph* g, int heads, int feat, int32_t dtype, const float* el,
                       const float* er, const void* hc, const float* lse, const void* u,
                       const void* u_lo, const void* dU, const void* hs, const void* dV,
                       const float* row_coef, float slope, const Dropout& dp, float* d_el,
                       float* de, float* attd, int ld, void* d_hs, dim3 grid, hipStream_t s) {
  int done = 0;
#define XG(h, f)                                                                              \
  if (heads == h && feat == f) {                                                              \
    if (dtype == MSHA_DTYPE_BF16) {                                                           \
      if constexpr (f % 8 == 0 && h * f * 2 <= 1024) {                                        \
        launch_bwd_gl_shape<h, f, bf16_t>(g, el, er, hc, lse, u, u_lo, dU, hs, dV, row_coef,  \
                                          slope, dp, d_el, de, attd, ld, d_hs, grid, s);      \
        done = 1;                                                                             \
      }                                                                                       \
    } else {                                                                                  \
      if constexpr (h * f * 4 <= 1024) {                                                      \
        launch_bwd_gl_shape<h, f, float>(g, el, er, hc, lse, u, nullptr, dU, hs, dV, row_coef, \
                                         slope, dp, d_el, de, attd, ld, d_hs, grid, s);       \
        done = 1;                                                                             \
      }                                                                                       \
    }                                                                                         \
  }
  MSHA_FOR_EACH_SHAPE(XG)
#undef XG
  return done;
}

}  // namespace msha
