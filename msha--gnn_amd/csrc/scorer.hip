// Link scoring: LinkPredictor (LLP.py:86-115) with the caller's pair gather
// (LLP.py:233: predictor(h[source_index], h[recipient_index])) fused in.
//
//   'inner':  out[b] = sigmoid(sum_f x_i[b,f] * x_j[b,f])           (LLP.py:112-113,115)
//   'mlp'  :  out[b] = sigmoid(dropout(relu((x_i*x_j) @ W0^T + b0)))  (LLP.py:107-111,115)
//             -> msha_pair_linear (gemm.hip, MFMA); the last Linear is never applied in
//                the reference, so the output is (B, hidden).
// x_i = G[gi[b]], x_j = G2[gj[b]] (gi/gj NULL: row b of the table itself).
// Inner mode is memory bound: one wave scores 64 / (F/4) pairs per instruction with
// 16-byte gathers and a reduction over F/4 lanes.
#include "common.h"

namespace msha {

__device__ __forceinline__ float sigmoidf_(float z) { return 1.f / (1.f + __expf(-z)); }

// One pass over a pair batch's row indices (LLP.py:233, h[source_index]): flags[0] = 1
// when an index lies outside [-rows, rows) (torch's h[idx] raises), flags[1] = 1 when
// one is negative inside it (torch wraps it to rows + idx).  One global OR per wave.
__global__ void __launch_bounds__(256) pair_index_check_kernel(
    int64_t n, const int64_t* __restrict__ gi, int64_t rows_i, const int64_t* __restrict__ gj,
    int64_t rows_j, int32_t* __restrict__ flags) {
  bool oob = false, neg = false;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n;
       t += (int64_t)gridDim.x * blockDim.x) {
    if (gi != nullptr) {
      const int64_t v = gi[t];
      oob |= v >= rows_i || v < -rows_i;
      neg |= v < 0;
    }
    if (gj != nullptr) {
      const int64_t v = gj[t];
      oob |= v >= rows_j || v < -rows_j;
      neg |= v < 0;
    }
  }
  const uint64_t bo = __ballot(oob), bn = __ballot(neg);
  if (lane_id() == 0) {
    if (bo) atomicOr(flags, 1);
    if (bn) atomicOr(flags + 1, 1);
  }
}

// rows_i / rows_j bound the gathered rows (INT64_MAX: unchecked); a pair with an index
// outside [0, rows) scores NaN and sets *err (nullable) instead of reading past the table.
template <typename T>
__global__ void __launch_bounds__(256) pair_inner_kernel(
    int64_t n_pairs, int F, const T* __restrict__ G, int64_t ldg,
    const int64_t* __restrict__ gi, const T* __restrict__ G2, int64_t ldg2,
    const int64_t* __restrict__ gj, int64_t rows_i, int64_t rows_j, int32_t* __restrict__ err,
    float* __restrict__ out) {
  constexpr int V = Pk<T>::V;          // elements per 16-byte lane chunk
  const int lane = lane_id();
  const int QP = F / V;                // lanes per pair
  const int PPW = 64 / QP;             // pairs per wave-instruction
  const int slot = lane / QP, q = lane % QP;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  constexpr int UNROLL = 4;
  for (int64_t b0 = wave * PPW * UNROLL; b0 < n_pairs; b0 += nwaves * PPW * UNROLL) {
    float acc[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int64_t b = b0 + u * PPW + slot;
      acc[u] = 0.f;
      if (b < n_pairs && slot < PPW) {
        const int64_t i = gi ? gi[b] : b;
        const int64_t j = gj ? gj[b] : b;
        if ((uint64_t)i < (uint64_t)rows_i && (uint64_t)j < (uint64_t)rows_j) {
          acc[u] = pk_dot(pk_load(G + i * ldg + V * q), pk_load(G2 + j * ldg2 + V * q));
        } else {
          acc[u] = __builtin_nanf("");
          if (err != nullptr && q == 0) atomicOr(err, 1);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      float v = acc[u];
      for (int o = 1; o < QP; o <<= 1) v += __shfl_xor(v, o);
      const int64_t b = b0 + u * PPW + slot;
      if (q == 0 && slot < PPW && b < n_pairs) out[b] = sigmoidf_(v);
    }
  }
}

// d/dz of sigmoid for the inner product, then dx_i = dz * x_j, dx_j = dz * x_i
__global__ void __launch_bounds__(256) pair_inner_bwd_kernel(
    int64_t n_pairs, int F, const float* __restrict__ G, int64_t ldg,
    const int64_t* __restrict__ gi, const float* __restrict__ G2, int64_t ldg2,
    const int64_t* __restrict__ gj, const float* __restrict__ s, const float* __restrict__ dout,
    float* __restrict__ dxi, float* __restrict__ dxj) {
  const int64_t total = n_pairs * F;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = t / F;
    const int f = (int)(t % F);
    const int64_t i = gi ? gi[b] : b;
    const int64_t j = gj ? gj[b] : b;
    const float sb = s[b];
    const float dz = dout[b] * sb * (1.f - sb);
    dxi[t] = dz * G2[j * ldg2 + f];
    dxj[t] = dz * G[i * ldg + f];
  }
}

// mlp layer y = [sigmoid](drop(relu(z))): dz = dout * [s(1-s)] * [kept & z > 0] * scale.
// With the sigmoid, kept & z > 0  <=>  y > 0.5; without it  <=>  y > 0.
__global__ void __launch_bounds__(256) pair_mlp_dz_kernel(int64_t n, const float* __restrict__ s,
                                                          const float* __restrict__ dout,
                                                          float scale, int sigmoid,
                                                          float* __restrict__ dz) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n;
       t += (int64_t)gridDim.x * blockDim.x) {
    const float sv = s[t];
    if (sigmoid)
      dz[t] = sv > 0.5f ? dout[t] * sv * (1.f - sv) * scale : 0.f;
    else
      dz[t] = sv > 0.f ? dout[t] * scale : 0.f;
  }
}

// x = x_i * x_j (materialised for the weight gradient), or its backward
__global__ void __launch_bounds__(256) pair_hadamard_kernel(
    int64_t n_pairs, int F, const float* __restrict__ G, int64_t ldg,
    const int64_t* __restrict__ gi, const float* __restrict__ G2, int64_t ldg2,
    const int64_t* __restrict__ gj, const float* __restrict__ dx, float* __restrict__ x_or_dxi,
    float* __restrict__ dxj) {
  const int64_t total = n_pairs * F;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = t / F;
    const int f = (int)(t % F);
    const float xi = G[(gi ? gi[b] : b) * ldg + f];
    const float xj = G2[(gj ? gj[b] : b) * ldg2 + f];
    if (dx == nullptr) {
      x_or_dxi[t] = xi * xj;
    } else {
      x_or_dxi[t] = dx[t] * xj;
      dxj[t] = dx[t] * xi;
    }
  }
}

// any other predictor string (LLP.py:104-115 takes neither branch): y = sigmoid(x_i * x_j)
// elementwise, shape (B, F); backward dx_i = dy y (1 - y) x_j, dx_j = dy y (1 - y) x_i
__global__ void __launch_bounds__(256) pair_hadamard_sigmoid_kernel(
    int64_t n_pairs, int F, const float* __restrict__ G, int64_t ldg,
    const int64_t* __restrict__ gi, const float* __restrict__ G2, int64_t ldg2,
    const int64_t* __restrict__ gj, const float* __restrict__ y, const float* __restrict__ dy,
    float* __restrict__ y_or_dxi, float* __restrict__ dxj) {
  const int64_t total = n_pairs * F;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = t / F;
    const int f = (int)(t % F);
    const float xi = G[(gi ? gi[b] : b) * ldg + f];
    const float xj = G2[(gj ? gj[b] : b) * ldg2 + f];
    if (dy == nullptr) {
      y_or_dxi[t] = sigmoidf_(xi * xj);
    } else {
      const float yt = y[t];
      const float dz = dy[t] * yt * (1.f - yt);
      y_or_dxi[t] = dz * xj;
      dxj[t] = dz * xi;
    }
  }
}

}  // namespace msha

using namespace msha;

extern "C" int msha_pair_hadamard_sigmoid(int64_t n_pairs, int32_t feat, const float* G,
                                          int64_t ldg, const int64_t* gi, const float* G2,
                                          int64_t ldg2, const int64_t* gj, const float* y,
                                          const float* dy, float* y_or_dxi, float* dxj,
                                          msha_stream_t stream) {
  MSHA_ARG_CHECK(n_pairs >= 0 && feat > 0 && G && G2 && y_or_dxi,
                 "pair_hadamard_sigmoid: bad arguments");
  MSHA_ARG_CHECK(dy == nullptr || (y != nullptr && dxj != nullptr),
                 "pair_hadamard_sigmoid: the backward needs y and dxj");
  if (n_pairs == 0) return MSHA_OK;
  hipLaunchKernelGGL(pair_hadamard_sigmoid_kernel, dim3(grid_for(n_pairs * feat, 256, 16384)),
                     dim3(256), 0, (hipStream_t)stream, n_pairs, (int)feat, G, ldg, gi, G2, ldg2,
                     gj, y, dy, y_or_dxi, dxj);
  return check_launch("pair_hadamard_sigmoid");
}

extern "C" int msha_pair_index_check(int64_t n_pairs, const int64_t* gi, int64_t g_rows,
                                     const int64_t* gj, int64_t g2_rows, int32_t* flags,
                                     msha_stream_t stream) {
  MSHA_ARG_CHECK(n_pairs >= 0 && flags != nullptr, "pair_index_check: bad arguments");
  MSHA_ARG_CHECK((gi == nullptr || g_rows >= 0) && (gj == nullptr || g2_rows >= 0),
                 "pair_index_check: negative row count");
  if (n_pairs == 0 || (gi == nullptr && gj == nullptr)) return MSHA_OK;
  hipLaunchKernelGGL(pair_index_check_kernel, dim3(grid_for(n_pairs, 256, 4096)), dim3(256), 0,
                     (hipStream_t)stream, n_pairs, gi, g_rows, gj, g2_rows, flags);
  return check_launch("pair_index_check");
}

template <typename T>
static int pair_inner_launch(const char* name, int vmax, int64_t n_pairs, int32_t feat,
                             const void* G, int64_t ldg, const int64_t* gi, const void* G2,
                             int64_t ldg2, const int64_t* gj, int64_t g_rows, int64_t g2_rows,
                             int32_t* err, float* out, msha_stream_t stream) {
  constexpr int V = Pk<T>::V;
  MSHA_ARG_CHECK(n_pairs >= 0 && feat >= V && feat <= vmax && (feat & (feat - 1)) == 0,
                 "pair_inner_fwd: feat must be a power of two in [16 B, 64 lanes x 16 B]");
  MSHA_ARG_CHECK(G && G2 && out, "pair_inner_fwd: null pointer");
  MSHA_ARG_CHECK(ldg % V == 0 && ldg2 % V == 0 && ((uintptr_t)G % 16) == 0 &&
                     ((uintptr_t)G2 % 16) == 0,
                 "pair_inner_fwd: tables must be 16-byte aligned with 16-byte rows pitch");
  if (n_pairs == 0) return MSHA_OK;
  if (gi == nullptr) g_rows = INT64_MAX;  // row b of the table itself: the caller's count
  if (gj == nullptr) g2_rows = INT64_MAX;
  const int ppw = 64 / (feat / V) * 4;
  hipLaunchKernelGGL(pair_inner_kernel<T>, dim3(grid_for((n_pairs + ppw - 1) / ppw, 4, 1 << 20)),
                     dim3(256), 0, (hipStream_t)stream, n_pairs, (int)feat, (const T*)G, ldg, gi,
                     (const T*)G2, ldg2, gj, g_rows, g2_rows, err, out);
  return check_launch(name);
}

extern "C" int msha_pair_inner_fwd(int64_t n_pairs, int32_t feat, const float* G, int64_t ldg,
                                   const int64_t* gi, const float* G2, int64_t ldg2,
                                   const int64_t* gj, float* out, msha_stream_t stream) {
  return pair_inner_launch<float>("pair_inner_fwd", 256, n_pairs, feat, G, ldg, gi, G2, ldg2, gj,
                                  INT64_MAX, INT64_MAX, nullptr, out, stream);
}

extern "C" int msha_pair_inner_fwd_bf16(int64_t n_pairs, int32_t feat, const void* G,
                                        int64_t ldg, const int64_t* gi, const void* G2,
                                        int64_t ldg2, const int64_t* gj, float* out,
                                        msha_stream_t stream) {
  return pair_inner_launch<bf16_t>("pair_inner_fwd_bf16", 512, n_pairs, feat, G, ldg, gi, G2,
                                   ldg2, gj, INT64_MAX, INT64_MAX, nullptr, out, stream);
}

extern "C" int msha_pair_inner_fwd_ex(int64_t n_pairs, int32_t feat, int32_t dtype, const void* G,
                                      int64_t ldg, const int64_t* gi, int64_t g_rows,
                                      const void* G2, int64_t ldg2, const int64_t* gj,
                                      int64_t g2_rows, int32_t* err, float* out,
                                      msha_stream_t stream) {
  MSHA_ARG_CHECK(dtype == MSHA_DTYPE_F32 || dtype == MSHA_DTYPE_BF16,
                 "pair_inner_fwd_ex: dtype must be MSHA_DTYPE_F32 or MSHA_DTYPE_BF16");
  MSHA_ARG_CHECK((gi == nullptr || g_rows >= 0) && (gj == nullptr || g2_rows >= 0),
                 "pair_inner_fwd_ex: negative row count");
  if (dtype == MSHA_DTYPE_BF16)
    return pair_inner_launch<bf16_t>("pair_inner_fwd_ex", 512, n_pairs, feat, G, ldg, gi, G2, ldg2,
                                     gj, g_rows, g2_rows, err, out, stream);
  return pair_inner_launch<float>("pair_inner_fwd_ex", 256, n_pairs, feat, G, ldg, gi, G2, ldg2,
                                  gj, g_rows, g2_rows, err, out, stream);
}

extern "C" int msha_pair_inner_bwd(int64_t n_pairs, int32_t feat, const float* G, int64_t ldg,
                                   const int64_t* gi, const float* G2, int64_t ldg2,
                                   const int64_t* gj, const float* s, const float* dout,
                                   float* dxi, float* dxj, msha_stream_t stream) {
  MSHA_ARG_CHECK(n_pairs >= 0 && feat > 0, "pair_inner_bwd: bad sizes");
  MSHA_ARG_CHECK(G && G2 && s && dout && dxi && dxj, "pair_inner_bwd: null pointer");
  if (n_pairs == 0) return MSHA_OK;
  hipLaunchKernelGGL(pair_inner_bwd_kernel, dim3(grid_for(n_pairs * feat, 256, 16384)),
                     dim3(256), 0, (hipStream_t)stream, n_pairs, (int)feat, G, ldg, gi, G2, ldg2,
                     gj, s, dout, dxi, dxj);
  return check_launch("pair_inner_bwd");
}

extern "C" int msha_pair_mlp_dz(int64_t n, const float* s, const float* dout, float drop_p,
                                int32_t sigmoid, float* dz, msha_stream_t stream) {
  MSHA_ARG_CHECK(n >= 0 && s && dout && dz, "pair_mlp_dz: bad arguments");
  MSHA_ARG_CHECK(drop_p >= 0.f && drop_p < 1.f, "pair_mlp_dz: p must be in [0, 1)");
  if (n == 0) return MSHA_OK;
  const float scale = drop_p > 0.f ? (float)(1.0 / (1.0 - (double)drop_p)) : 1.f;
  hipLaunchKernelGGL(pair_mlp_dz_kernel, dim3(grid_for(n, 256, 16384)), dim3(256), 0,
                     (hipStream_t)stream, n, s, dout, scale, (int)sigmoid, dz);
  return check_launch("pair_mlp_dz");
}

extern "C" int msha_pair_hadamard(int64_t n_pairs, int32_t feat, const float* G, int64_t ldg,
                                  const int64_t* gi, const float* G2, int64_t ldg2,
                                  const int64_t* gj, const float* dx, float* x_or_dxi,
                                  float* dxj, msha_stream_t stream) {
  MSHA_ARG_CHECK(n_pairs >= 0 && feat > 0 && G && G2 && x_or_dxi,
                 "pair_hadamard: bad arguments");
  MSHA_ARG_CHECK(dx == nullptr || dxj != nullptr, "pair_hadamard: dx needs dxj");
  if (n_pairs == 0) return MSHA_OK;
  hipLaunchKernelGGL(pair_hadamard_kernel, dim3(grid_for(n_pairs * feat, 256, 16384)),
                     dim3(256), 0, (hipStream_t)stream, n_pairs, (int)feat, G, ldg, gi, G2, ldg2,
                     gj, dx, x_or_dxi, dxj);
  return check_launch("pair_hadamard");
}
