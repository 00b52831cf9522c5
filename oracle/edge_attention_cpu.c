/*
 * CPU restatement (plain C + OpenMP) of the fused edge-softmax + aggregate path.
 * TEST INFRASTRUCTURE / CPU BASELINE ONLY -- never linked into the product.
 *
 * Restates, per CSR row i and head h (Ablation.py:266-274 of the reference):
 *   s_e = lrelu(el[i,h] + er[j,h])                 (Ablation.py:266-267)
 *   att = softmax over the row's edges             (Ablation.py:268-270)
 *   u_i = sum_e att_e hc[j]                        (Ablation.py:274)
 *   v_j = sum_e att_e hs[i]   (optional: att_out + oracle_csc_aggregate, Ablation.py:273)
 * and the autograd backward (d_el, d_er, d_hc; with the v branch also the hs . dV term of
 * g_e and d_hs_i = sum_e att_e dV[j]).  Column sums use the CSC view.
 * Pinned to the reference through gnn_oracle.py (tests/test_oracle_golden.py) by
 * tests/test_oracle_c.py.
 *
 * Built twice (oracle/build_oracle.py): REAL = float (libmsha_oracle.so, the CPU
 * baseline) and REAL = double with the suffix _f64 (libmsha_oracle64.so, the fp64
 * checker of the full-size parity tests).
 */
#include <stdint.h>
#include <stdlib.h>
#include <tgmath.h>

#ifndef REAL
#define REAL float
#endif
#ifndef SFX
#define SFX(name) name
#endif

typedef REAL real;

static inline real lrelu(real x, real s) { return x > 0 ? x : x * s; }

void SFX(oracle_edge_attention_fwd)(int64_t n_rows, const int32_t* rowptr, const int32_t* col, int H,
                               int F, const real* el, const real* er, const real* hc,
                               real slope, real* u, real* lse, real* att_out) {
  const int D = H * F;
#pragma omp parallel for schedule(dynamic, 256)
  for (int64_t i = 0; i < n_rows; ++i) {
    const int32_t a = rowptr[i], b = rowptr[i + 1];
    real* ui = u + i * D;
    for (int k = 0; k < D; ++k) ui[k] = (real)0;
    for (int h = 0; h < H; ++h) {
      real m = -(real)INFINITY;
      for (int32_t e = a; e < b; ++e) {
        const real s = lrelu(el[i * H + h] + er[(int64_t)col[e] * H + h], slope);
        if (s > m) m = s;
      }
      real l = (real)0;
      for (int32_t e = a; e < b; ++e) {
        const real s = lrelu(el[i * H + h] + er[(int64_t)col[e] * H + h], slope);
        const real p = exp(s - m);
        l += p;
        const real* hj = hc + (int64_t)col[e] * D + h * F;
        for (int f = 0; f < F; ++f) ui[h * F + f] += p * hj[f];
      }
      const real inv = l > (real)0 ? (real)1 / l : (real)0;
      for (int f = 0; f < F; ++f) ui[h * F + f] *= inv;
      lse[i * H + h] = l > (real)0 ? m + log(l) : -(real)INFINITY;
      if (att_out)
        for (int32_t e = a; e < b; ++e)
          att_out[(int64_t)e * H + h] =
              exp(lrelu(el[i * H + h] + er[(int64_t)col[e] * H + h], slope) - m) * inv;
    }
  }
}

/* row half of the backward: d_el, per-edge de and att (for the column half); with the v
 * branch (hs, dV non-NULL) g_e gains hs_i . dV_j and d_hs_i = sum_e att_e dV_j, so
 * D_i = sum_e att_e g_e = dU_i . u_i + hs_i . d_hs_i */
void SFX(oracle_edge_attention_bwd_rows)(int64_t n_rows, const int32_t* rowptr, const int32_t* col,
                                    int H, int F, const real* el, const real* er,
                                    const real* hc, const real* lse, const real* u,
                                    const real* dU, const real* hs, const real* dV,
                                    real slope, real* d_el, real* de, real* att_out,
                                    real* d_hs) {
  const int D = H * F;
#pragma omp parallel for schedule(dynamic, 256)
  for (int64_t i = 0; i < n_rows; ++i) {
    const int32_t a = rowptr[i], b = rowptr[i + 1];
    for (int h = 0; h < H; ++h) {
      const real* dui = dU + i * D + h * F;
      const real* hsi = hs ? hs + i * D + h * F : NULL;
      real Dh = (real)0;
      for (int f = 0; f < F; ++f) Dh += dui[f] * u[i * D + h * F + f];
      if (hsi) {
        real* dhs = d_hs + i * D + h * F;
        for (int f = 0; f < F; ++f) dhs[f] = (real)0;
        for (int32_t e = a; e < b; ++e) {
          const real att = exp(lrelu(el[i * H + h] + er[(int64_t)col[e] * H + h], slope) -
                               lse[i * H + h]);
          const real* vj = dV + (int64_t)col[e] * D + h * F;
          for (int f = 0; f < F; ++f) dhs[f] += att * vj[f];
        }
        for (int f = 0; f < F; ++f) Dh += hsi[f] * dhs[f];
      }
      real acc = (real)0;
      for (int32_t e = a; e < b; ++e) {
        const real pre = el[i * H + h] + er[(int64_t)col[e] * H + h];
        const real att = exp(lrelu(pre, slope) - lse[i * H + h]);
        const real* hj = hc + (int64_t)col[e] * D + h * F;
        real g = (real)0;
        for (int f = 0; f < F; ++f) g += dui[f] * hj[f];
        if (hsi) {
          const real* vj = dV + (int64_t)col[e] * D + h * F;
          for (int f = 0; f < F; ++f) g += hsi[f] * vj[f];
        }
        const real d = att * (g - Dh) * (pre > (real)0 ? (real)1 : slope);
        de[(int64_t)e * H + h] = d;
        att_out[(int64_t)e * H + h] = att;
        acc += d;
      }
      d_el[i * H + h] = acc;
    }
  }
}

/* column half: out[j] = sum_e w[e] table[row(e)], out_x[j] = sum_e x[e] */
void SFX(oracle_csc_aggregate)(int64_t n_cols, const int32_t* colptr, const int32_t* csc_row,
                          const int32_t* csc_eid, int H, int F, const real* w, const real* x,
                          const real* table, real* out, real* out_x) {
  const int D = H * F;
#pragma omp parallel for schedule(dynamic, 64)
  for (int64_t j = 0; j < n_cols; ++j) {
    real* oj = out + j * D;
    for (int k = 0; k < D; ++k) oj[k] = (real)0;
    for (int h = 0; h < H; ++h) {
      real xs = (real)0;
      for (int32_t s = colptr[j]; s < colptr[j + 1]; ++s) {
        const int64_t e = csc_eid[s];
        const real* ti = table + (int64_t)csc_row[s] * D + h * F;
        const real ww = w[e * H + h];
        for (int f = 0; f < F; ++f) oj[h * F + f] += ww * ti[f];
        if (x) xs += x[e * H + h];
      }
      if (out_x) out_x[j * H + h] = xs;
    }
  }
}

int SFX(oracle_num_threads)(void) {
#ifdef _OPENMP
  extern int omp_get_max_threads(void);
  return omp_get_max_threads();
#else
  return 1;
#endif
}
