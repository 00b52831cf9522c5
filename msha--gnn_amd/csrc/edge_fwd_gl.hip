// The gather-layout edge forward (edge_fwd_gl.hip): see the kernel's comment.  Split
// from edge_attention.hip so its instantiations compile in parallel with the rest.
#include "edge_geo.h"

namespace msha {

// ------------------------------------------------------- forward, gather layout ---
// One 16-byte piece per lane (QPL == 1), softmax in the gather layout: lane = edge slot
// g_e x piece q, every (edge, head) score replicated over the head's QH lanes; a chunk
// is NGI gather instructions (CEL = NGI * EPI edges).  The chunk max / sum reduce the
// NGI slots in registers and the EPI edge slots by xor over g_e, so no weight is
// shuffled to the gather lanes, and the chunk length is free of the 64 / H score lanes
// of edge_attn_fwd_bat_kernel: short rows (R15, bip1m: ~2.3 edges) take CEL = 4, where
// the score layout issued 32 edge slots of masked gathers per row.
// Columns are loaded in the gather layout, two chunks ahead; dropout keep bits are
// drawn one Philox call per (edge, head) on lanes edge * H + head of NB ballots (the
// score layout's lanes and element order) and reach the gather lanes by ballot.
//
// RS ("row scores"): every caller of the u-only path scores the gathered table itself,
// er_j = hc_j . a_r per head (Ablation.py:266-267: a[:F] against h1_j, the row u
// aggregates).  Given a_r, er_j comes from the row the gather lanes already hold -- V
// fmas per lane and the xor tree over the head's QH lanes (DPP) -- instead of a 4H-byte
// per-edge gather of an (M, H) table that costs a whole cache line per edge once the
// table outgrows L2 (syn2m: 64 MB er, 40M edges).  The fused backward's column pass
// recomputes er_j from hc_j in the same order (same bits).  Without RS er is gathered
// per edge in the gather layout (the QH lanes of a head read the same word).
// ATTD: also the post-dropout attention (E, H) (the v-branch and the Ours layer read
// it): from the scores still in registers for one-chunk rows, else a second pass over
// the row's columns and er (not with RS).
// RT: the row terms uc, qc of the fused backward (see edge_attn_fwd_bat_kernel).
template <int H, int F, typename T, int NGI, bool RT, bool RS, bool ATTD, bool PF>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(FWD_WPE)))
edge_attn_fwd_gl_kernel(
    const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
    const uint8_t* __restrict__ rowflag, int32_t n_rows, int32_t n_cols, int32_t n_edges,
    const float* __restrict__ el, const float* __restrict__ er, const float* __restrict__ ar,
    const T* __restrict__ hc, float slope, Dropout dp, T* __restrict__ u, T* __restrict__ u_lo,
    float* __restrict__ lse, float* __restrict__ attd, float* __restrict__ uc,
    float* __restrict__ qc) {
  using G = Geo<H, F, T>;
  static_assert(G::QPL == 1, "gather-layout forward: one 16-byte piece per lane");
  static_assert(!(RS && ATTD), "the attention export recomputes scores from er");
  constexpr int CEL = NGI * G::EPI;         // edges per chunk
  constexpr int NB = (CEL * H + 63) / 64;   // dropout ballots per chunk
  const int lane = lane_id();
  const int g_e = lane / G::NQ, q = lane % G::NQ;  // gather layout
  const int hq = q / G::QH;                        // head of this lane's piece
  const rsrc_t r_col = make_rsrc(col, (uint32_t)n_edges * 4u);
  const rsrc_t r_hc = make_rsrc(hc, (uint32_t)n_cols * (uint32_t)(G::D * sizeof(T)));
  const rsrc_t r_er = make_rsrc(RS ? nullptr : er, (uint32_t)n_cols * (4u * H));
  const uint32_t q_off = 16u * q;
  const int wave0 = __builtin_amdgcn_readfirstlane((int)(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6));
  const int nwaves = (int)(((int64_t)gridDim.x * blockDim.x) >> 6);
  // this lane's piece of a_r ((H, F) fp32: piece q covers elements q*V .. q*V + V - 1)
  Pk<T> arq = pk_zero<T>();
  if (RS) {
#pragma unroll
    for (int v = 0; v < G::V; v += 4) {
      const float4 a4 = *reinterpret_cast<const float4*>(ar + G::V * q + v);
      arq.v[v] = a4.x; arq.v[v + 1] = a4.y; arq.v[v + 2] = a4.z; arq.v[v + 3] = a4.w;
    }
  }
  // columns of a chunk.  Long chunks (whole score-layout chunks, CEL = SL * 64 / H): SL
  // words per lane in the score layout (lane e_s * H + h_s holds edge t * CE + e_s), the
  // gather lanes fetch theirs by ds_bpermute -- SL loads instead of NGI; short chunks:
  // one word per gather instruction in the gather layout (slot gi * EPI + g_e).  Past
  // the row: 0.
  constexpr bool SLC = CEL % G::CE == 0;
  constexpr int NJ = SLC ? CEL / G::CE : NGI;
  const int e_s = lane / H;
  auto load_cols = [&](int32_t cs, int32_t end, int32_t (&j)[NJ]) {
#pragma unroll
    for (int k = 0; k < NJ; ++k) {
      const int32_t e = SLC ? cs + k * G::CE + e_s : cs + k * G::EPI + g_e;
      j[k] = buf_i32(r_col, e < end ? (uint32_t)e * 4u : kOOB);
    }
  };
  auto col_of = [&](const int32_t (&j)[NJ], int gi) -> int32_t {
    if constexpr (SLC) {
      const int g = gi * G::EPI;
      return __shfl(j[g / G::CE], (g % G::CE + g_e) * H);
    } else {
      return j[gi];
    }
  };

  int row = wave0;
  if (row >= n_rows) return;
  int32_t start = __builtin_amdgcn_readfirstlane(rowptr[row]);
  int32_t end = __builtin_amdgcn_readfirstlane(rowptr[row + 1]);
  bool virt = rowflag != nullptr && rowflag[row] != 0;
  float elq = el[(int64_t)row * H + hq];
  // one chunk's gathers (and er), all in flight together; slots past the row read 0
  auto gather = [&](int32_t cs, int32_t end, const int32_t (&j)[NJ], u32x4_t (&raw)[NGI],
                    float (&erq)[NGI]) {
    const int nvalid = min(CEL, (int)(end - cs));
#pragma unroll
    for (int gi = 0; gi < NGI; ++gi) {
      const bool valid = gi * G::EPI + g_e < nvalid;
      const int32_t jj = col_of(j, gi);
      raw[gi] = buf_b128(r_hc, valid ? (uint32_t)jj * (uint32_t)(G::D * sizeof(T)) + q_off
                                     : kOOB);
      if (!RS) erq[gi] = buf_f32(r_er, valid ? (uint32_t)jj * (4u * H) + 4u * hq : kOOB);
    }
  };
  int32_t jc[NJ], jn[NJ];
  load_cols(start, end, jc);
  load_cols(start + CEL, end, jn);
  while (true) {
    float m = -INFINITY, l = 0.f, lc = 0.f;
    Pk<T> acc = pk_zero<T>(), accc = pk_zero<T>();
    float sc_keep[NGI];   // ATTD: the scores of a one-chunk row
    uint64_t kb_keep[NB];
    // PF (long rows): chunk c + 1's gathers leave before chunk c's scores are reduced
    // (two chunks in flight per wave); otherwise each chunk's gathers leave at its start
    u32x4_t raw[NGI];
    float erq[NGI];
    if (PF) gather(start, end, jc, raw, erq);
    for (int32_t cs = start; cs < end; cs += CEL) {
      const int nvalid = min(CEL, (int)(end - cs));
      // (1) the gathers: this chunk's, or (prefetch) the next chunk's
      u32x4_t rawn[NGI];
      float erqn[NGI];
      if (PF) gather(cs + CEL, end, jn, rawn, erqn);
      else gather(cs, end, jc, raw, erq);
      // columns two chunks ahead
      int32_t jnn[NJ];
      load_cols(cs + 2 * CEL, end, jnn);
      // (2) dropout keep bits of the chunk, while the gathers fly: ballot b, lane l holds
      // edge (b * 64 + l) / H, head (b * 64 + l) % H of the chunk
      uint64_t kb[NB];
      if (dp.active) {
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          const int idx = b * 64 + lane;
          const int32_t e = cs + idx / H;
          kb[b] = __ballot(idx < CEL * H &&
                           dropout_factor(dp, (uint64_t)e * H + (idx % H)) != 0.f);
        }
      }
      // (3) scores (gather layout)
      float sc[NGI], pre[NGI];
      float smax = -INFINITY;
#pragma unroll
      for (int gi = 0; gi < NGI; ++gi) {
        float erv;
        if (RS) {
          const Pk<T> xr = pk_from_raw(raw[gi], (T*)nullptr);
          erv = group_sum<G::QH>(pk_dot(xr, arq));
        } else {
          erv = erq[gi];
        }
        pre[gi] = elq + erv;
        const bool valid = gi * G::EPI + g_e < nvalid;
        sc[gi] = valid ? (virt ? 0.f : lrelu(pre[gi], slope)) : -INFINITY;
        smax = fmaxf(smax, sc[gi]);
        if (ATTD) sc_keep[gi] = sc[gi];
      }
#pragma unroll
      for (int o = G::NQ; o < 64; o <<= 1) smax = fmaxf(smax, xor_shfl(smax, o));
      const float mn = fmaxf(m, smax);
      const float alpha = __expf(m - mn);
      float w[NGI], psum = 0.f, pcsum = 0.f;
#pragma unroll
      for (int gi = 0; gi < NGI; ++gi) {
        const float pe = __expf(sc[gi] - mn);  // masked slots: exp(-inf) = 0
        psum += pe;
        if (RT) pcsum = fmaf(pe, pre[gi] > 0.f ? 1.f : slope, pcsum);
        w[gi] = pe;
        if (dp.active) {
          const int bit = (gi * G::EPI + g_e) * H + hq;  // < CEL * H
          w[gi] = (kb[bit >> 6] >> (bit & 63)) & 1ull ? pe * dp.scale : 0.f;
        }
      }
      if (ATTD && dp.active) {
#pragma unroll
        for (int b = 0; b < NB; ++b) kb_keep[b] = kb[b];
      }
#pragma unroll
      for (int o = G::NQ; o < 64; o <<= 1) psum += xor_shfl(psum, o);
      l = fmaf(l, alpha, psum);
      if (RT) {
#pragma unroll
        for (int o = G::NQ; o < 64; o <<= 1) pcsum += xor_shfl(pcsum, o);
        lc = fmaf(lc, alpha, pcsum);
      }
      m = mn;
      acc = pk_scale(acc, alpha);
      if (RT) accc = pk_scale(accc, alpha);
      // (4) accumulate in gather order (masked slots carry w = 0 and a zero row)
#pragma unroll
      for (int gi = 0; gi < NGI; ++gi) {
        const Pk<T> xr = pk_from_raw(raw[gi], (T*)nullptr);
        acc = pk_fma(w[gi], xr, acc);
        if (RT) accc = pk_fma(w[gi] * (pre[gi] > 0.f ? 1.f : slope), xr, accc);
      }
#pragma unroll
      for (int k = 0; k < NJ; ++k) {
        jc[k] = jn[k];
        jn[k] = jnn[k];
      }
      if (PF) {
#pragma unroll
        for (int gi = 0; gi < NGI; ++gi) {
          raw[gi] = rawn[gi];
          if (!RS) erq[gi] = erqn[gi];
        }
      }
    }
    // the next row's bounds, flag, el and first columns before this row's epilogue
    const int nrow_raw = row + nwaves;
    const bool has_next = nrow_raw < n_rows;
    const int nrow = has_next ? nrow_raw : row;
    const int32_t nstart = __builtin_amdgcn_readfirstlane(rowptr[nrow]);
    const int32_t nend = __builtin_amdgcn_readfirstlane(rowptr[nrow + 1]);
    const bool nvirt = rowflag != nullptr && rowflag[nrow] != 0;
    const float nelq = el[(int64_t)nrow * H + hq];
    int32_t njc[NJ], njn[NJ];
    load_cols(nstart, nend, njc);
    load_cols(nstart + CEL, nend, njn);
    if (G::EPI > 1) {
#pragma unroll
      for (int o = G::NQ; o < 64; o <<= 1) acc = pk_xor_add(acc, o);
      if (RT) {
#pragma unroll
        for (int o = G::NQ; o < 64; o <<= 1) accc = pk_xor_add(accc, o);
      }
    }
    const float inv = l > 0.f ? 1.f / l : 0.f;  // l, m: this lane's head (replicated)
    const float lse_q = l > 0.f ? m + __logf(l) : -INFINITY;
    if (g_e == 0) {
      const Pk<T> uk = pk_scale(acc, inv);
      pk_store(u + (int64_t)row * G::D + G::V * q, uk);
      if (sizeof(T) == 2 && u_lo != nullptr)
        pk_store(u_lo + (int64_t)row * G::D + G::V * q, pk_residual(uk));
      if (RT) {
        const Pk<T> ck = pk_scale(accc, inv);
        float* dst = uc + (int64_t)row * G::D + G::V * q;
#pragma unroll
        for (int v = 0; v < G::V; v += 4)
          *reinterpret_cast<float4*>(dst + v) = make_float4(ck.v[v], ck.v[v + 1], ck.v[v + 2], ck.v[v + 3]);
      }
      if (q % G::QH == 0) {
        lse[(int64_t)row * H + hq] = lse_q;
        if (RT) qc[(int64_t)row * H + hq] = l > 0.f ? lc / l : 0.f;
      }
    }
    if (ATTD && attd != nullptr) {
      const bool lead = q % G::QH == 0;  // one lane per (edge slot, head) writes
      if (end - start <= CEL) {
        // one chunk (nearly every R15 / bip1m row): its scores are still in registers
#pragma unroll
        for (int gi = 0; gi < NGI; ++gi) {
          const int32_t e = start + gi * G::EPI + g_e;
          const int bit = (gi * G::EPI + g_e) * H + hq;
          const float dropf = !dp.active ? 1.f
                              : ((kb_keep[bit >> 6] >> (bit & 63)) & 1ull ? dp.scale : 0.f);
          if (lead && e < end) attd[(int64_t)e * H + hq] = __expf(sc_keep[gi] - lse_q) * dropf;
        }
      } else {
        for (int32_t cs = start; cs < end; cs += CEL) {
#pragma unroll
          for (int gi = 0; gi < NGI; ++gi) {
            const int32_t e = cs + gi * G::EPI + g_e;
            if (lead && e < end) {
              const float sv = virt ? 0.f : lrelu(elq + er[(int64_t)col[e] * H + hq], slope);
              attd[(int64_t)e * H + hq] =
                  __expf(sv - lse_q) * dropout_factor(dp, (uint64_t)e * H + hq);
            }
          }
        }
      }
    }
    if (!has_next) break;
    row = nrow;
    start = nstart;
    end = nend;
    virt = nvirt;
    elq = nelq;
#pragma unroll
    for (int k = 0; k < NJ; ++k) {
      jc[k] = njc[k];
      jn[k] = njn[k];
    }
  }
}

template <int H, int F, typename T, int NGI, bool PF>
static void launch_gl_shape(const msha_graph* g, const float* el, const float* er,
                            const float* ar, const void* hc, float slope, const Dropout& dp,
                            void* u, void* u_lo, float* lse, float* attd, float* uc, float* qc,
                            dim3 grid, hipStream_t s) {
  const bool rs = ar != nullptr, rt = uc != nullptr, at = attd != nullptr;
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, dim3(256), 0, s, g->rowptr, g->col, g->rowflag,
                       (int32_t)g->n_rows, (int32_t)g->n_cols, (int32_t)g->n_edges, el, er, ar,
                       (const T*)hc, slope, dp, (T*)u, (T*)u_lo, lse, attd, uc, qc);
  };
  if (rs) {
    if (rt) go(edge_attn_fwd_gl_kernel<H, F, T, NGI, true, true, false, PF>);
    else go(edge_attn_fwd_gl_kernel<H, F, T, NGI, false, true, false, PF>);
  } else if (at) {
    go(edge_attn_fwd_gl_kernel<H, F, T, NGI, false, false, true, PF>);
  } else if (rt) {
    go(edge_attn_fwd_gl_kernel<H, F, T, NGI, true, false, false, PF>);
  } else {
    go(edge_attn_fwd_gl_kernel<H, F, T, NGI, false, false, false, PF>);
  }
}

int launch_fwd_gl(const msha_graph* g, int heads, int feat, int32_t dtype, const float* el,
                  const float* er, const float* ar, const void* hc, float slope,
                  const Dropout& dp, void* u, void* u_lo, float* lse, float* attd, float* uc,
                  float* qc, bool short_rows, dim3 grid, hipStream_t s) {
  // row scores have no attention export; the er-table long-row forward is the batched
  // kernel of edge_attention.hip; row terms and the attention export never go together
  if ((ar != nullptr && attd != nullptr) || (ar == nullptr && !short_rows) ||
      (uc != nullptr && attd != nullptr))
    return 0;
  int done = 0;
#define XG(h, f)                                                                              \
  if (heads == h && feat == f) {                                                              \
    if (dtype == MSHA_DTYPE_BF16) {                                                           \
      if constexpr (f % 8 == 0 && h * f * 2 <= 1024) {                                        \
        if (short_rows)                                                                       \
          launch_gl_shape<h, f, bf16_t, gl_ngi_short<h, f, bf16_t>(), false>(                        \
              g, el, er, ar, hc, slope, dp, u, u_lo, lse, attd, uc, qc, grid, s);             \
        else                                                                                  \
          launch_gl_shape<h, f, bf16_t, gl_ngi_long<h, f, bf16_t>(), GL_PREFETCH_BF16>(                         \
              g, el, er, ar, hc, slope, dp, u, u_lo, lse, attd, uc, qc, grid, s);             \
        done = 1;                                                                             \
      }                                                                                       \
    } else {                                                                                  \
      if constexpr (h * f * 4 <= 1024) {                                                      \
        if (short_rows)                                                                       \
          launch_gl_shape<h, f, float, gl_ngi_short<h, f, float>(), false>(                          \
              g, el, er, ar, hc, slope, dp, u, nullptr, lse, attd, uc, qc, grid, s);          \
        else                                                                                  \
          launch_gl_shape<h, f, float, gl_ngi_long<h, f, float>(), GL_PREFETCH_F32>(                           \
              g, el, er, ar, hc, slope, dp, u, nullptr, lse, attd, uc, qc, grid, s);          \
        done = 1;                                                                             \
      }                                                                                       \
    }                                                                                         \
  }
  MSHA_FOR_EACH_SHAPE(XG)
#undef XG
  return done;
}

}  // namespace msha
