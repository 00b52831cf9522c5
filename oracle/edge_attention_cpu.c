/*
 * CPU restatement (plain C + OpenMP) of the fused edge-softmax + aggregate path.
 * TEST INFRASTRUCTURE / CPU BASELINE ONLY -- never linked into the product.
 *
 * Restates, per CSR row i and head h (Ablation.py:266-274 of the reference):
 *   s_e = lrelu(el[i,h] + er[j,h])                 (Ablation.py:266-267)
 *   att = softmax over the row's edges             (Ablation.py:268-270)
 *   u_i = sum_e att_e hc[j]                        (Ablation.py:274)
 * and the autograd backward (d_el, d_er, d_hc).  Column sums use the CSC view.
 * Pinned to the reference through gnn_oracle.py (tests/test_oracle_golden.py) by
 * tests/test_oracle_c.py.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

static inline float lrelu(float x, float s) { return x > 0.f ? x : x * s; }

void oracle_edge_attention_fwd(int64_t n_rows, const int32_t* rowptr, const int32_t* col, int H,
                               int F, const float* el, const float* er, const float* hc,
                               float slope, float* u, float* lse) {
  const int D = H * F;
#pragma omp parallel for schedule(dynamic, 256)
  for (int64_t i = 0; i < n_rows; ++i) {
    const int32_t a = rowptr[i], b = rowptr[i + 1];
    float* ui = u + i * D;
    for (int k = 0; k < D; ++k) ui[k] = 0.f;
    for (int h = 0; h < H; ++h) {
      float m = -INFINITY;
      for (int32_t e = a; e < b; ++e) {
        const float s = lrelu(el[i * H + h] + er[(int64_t)col[e] * H + h], slope);
        if (s > m) m = s;
      }
      float l = 0.f;
      for (int32_t e = a; e < b; ++e) {
        const float s = lrelu(el[i * H + h] + er[(int64_t)col[e] * H + h], slope);
        const float p = expf(s - m);
        l += p;
        const float* hj = hc + (int64_t)col[e] * D + h * F;
        for (int f = 0; f < F; ++f) ui[h * F + f] += p * hj[f];
      }
      const float inv = l > 0.f ? 1.f / l : 0.f;
      for (int f = 0; f < F; ++f) ui[h * F + f] *= inv;
      lse[i * H + h] = l > 0.f ? m + logf(l) : -INFINITY;
    }
  }
}

/* row half of the backward: d_el, per-edge de and att (for the column half) */
void oracle_edge_attention_bwd_rows(int64_t n_rows, const int32_t* rowptr, const int32_t* col,
                                    int H, int F, const float* el, const float* er,
                                    const float* hc, const float* lse, const float* u,
                                    const float* dU, float slope, float* d_el, float* de,
                                    float* att_out) {
  const int D = H * F;
#pragma omp parallel for schedule(dynamic, 256)
  for (int64_t i = 0; i < n_rows; ++i) {
    const int32_t a = rowptr[i], b = rowptr[i + 1];
    for (int h = 0; h < H; ++h) {
      const float* dui = dU + i * D + h * F;
      float Dh = 0.f;
      for (int f = 0; f < F; ++f) Dh += dui[f] * u[i * D + h * F + f];
      float acc = 0.f;
      for (int32_t e = a; e < b; ++e) {
        const float pre = el[i * H + h] + er[(int64_t)col[e] * H + h];
        const float att = expf(lrelu(pre, slope) - lse[i * H + h]);
        const float* hj = hc + (int64_t)col[e] * D + h * F;
        float g = 0.f;
        for (int f = 0; f < F; ++f) g += dui[f] * hj[f];
        const float d = att * (g - Dh) * (pre > 0.f ? 1.f : slope);
        de[(int64_t)e * H + h] = d;
        att_out[(int64_t)e * H + h] = att;
        acc += d;
      }
      d_el[i * H + h] = acc;
    }
  }
}

/* column half: out[j] = sum_e w[e] table[row(e)], out_x[j] = sum_e x[e] */
void oracle_csc_aggregate(int64_t n_cols, const int32_t* colptr, const int32_t* csc_row,
                          const int32_t* csc_eid, int H, int F, const float* w, const float* x,
                          const float* table, float* out, float* out_x) {
  const int D = H * F;
#pragma omp parallel for schedule(dynamic, 64)
  for (int64_t j = 0; j < n_cols; ++j) {
    float* oj = out + j * D;
    for (int k = 0; k < D; ++k) oj[k] = 0.f;
    for (int h = 0; h < H; ++h) {
      float xs = 0.f;
      for (int32_t s = colptr[j]; s < colptr[j + 1]; ++s) {
        const int64_t e = csc_eid[s];
        const float* ti = table + (int64_t)csc_row[s] * D + h * F;
        const float ww = w[e * H + h];
        for (int f = 0; f < F; ++f) oj[h * F + f] += ww * ti[f];
        if (x) xs += x[e * H + h];
      }
      if (out_x) out_x[j * H + h] = xs;
    }
  }
}

int oracle_num_threads(void) {
#ifdef _OPENMP
  extern int omp_get_max_threads(void);
  return omp_get_max_threads();
#else
  return 1;
#endif
}
