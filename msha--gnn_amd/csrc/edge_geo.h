// Work geometry shared by the edge-attention kernels (edge_attention.hip,
// edge_fwd_gl.hip): one CSR row (or CSC chunk) per 64-lane wave, node-table rows read as
// 16-byte pieces.
#pragma once

#include "common.h"

#ifndef FWD_EPL
#define FWD_EPL 2
#endif
#ifndef FWD_EPL_BF16
#define FWD_EPL_BF16 2
#endif
#ifndef GL_EPL_BF16
#define GL_EPL_BF16 1  // the gather-layout forward's long chunks, bf16 tables (CEL 8)
#endif
#ifndef GL_EPL_F32
#define GL_EPL_F32 1  // fp32 tables: CEL 8 with the prefetch (CEL 16 without it)
#endif
// the gather-layout forward's long rows issue the next chunk's gathers before this
// chunk's softmax (syn2m forward: bf16 2460 -> 2262 us, fp32 at CEL 8 3728 -> 3649 us; fp32
// at CEL 16 lost a wave per SIMD to the second buffer and ran slower, 3961 us)
#ifndef GL_PREFETCH_BF16
#define GL_PREFETCH_BF16 1
#endif
#ifndef GL_PREFETCH_F32
#define GL_PREFETCH_F32 1
#endif
#ifndef FWD_WPE
#define FWD_WPE 1
#endif
#ifndef FWD_SHORT_DEG
#define FWD_SHORT_DEG 8
#endif
#ifndef FWD_SHORT_RPW
#define FWD_SHORT_RPW 5  // rows per wave on short-row graphs (A/B: MSHA_FWD_WAVES)
#endif
#ifndef FWD_SHORT_CEL
#define FWD_SHORT_CEL 4  // edges per chunk of the gather-layout forward on short rows
#endif

namespace msha {

template <int H, int F, typename T>
struct Geo {
  static constexpr int V = Pk<T>::V;        // elements per 16-byte chunk (4 fp32 / 8 bf16)
  static constexpr int D = H * F;
  static constexpr int NQ = D / V;          // chunks per feature row
  static constexpr int QPL = NQ > 64 ? NQ / 64 : 1;
  static constexpr int EPI = NQ >= 64 ? 1 : 64 / NQ;
  static constexpr int CE = 64 / H;
  static constexpr int QH = F / V;          // chunks per head
  static_assert(F % V == 0, "feat must be a multiple of the 16-byte chunk");
  static_assert(H >= 1 && H <= 64 && (64 % H) == 0, "heads must divide 64");
  static_assert(CE % EPI == 0, "score chunk must cover whole gather groups");
  static_assert(QH <= 64 && (64 % QH) == 0, "chunks per head must divide 64");
};

// chunk index (within the feature row) owned by this lane for slot k
template <class G>
__device__ __forceinline__ int quad_of(int lane, int k) {
  return G::QPL == 1 ? (lane % G::NQ) : (lane + 64 * k);
}

// Compiled (heads, feat) set.  Extend here (and in msha_edge_attention_supported).
#define MSHA_FOR_EACH_SHAPE(X) \
  X(1, 8) X(1, 16) X(1, 32) X(1, 64) X(1, 128) \
  X(2, 8) X(2, 16) X(2, 32) X(2, 64) X(2, 128) \
  X(4, 8) X(4, 16) X(4, 32) X(4, 64) X(4, 128) \
  X(8, 8) X(8, 16) X(8, 32) X(8, 64) X(8, 128)

// edges per lane of the forward's score layout (2: amortise the per-chunk reductions
// where a chunk is short and the gathers are single 16-byte pieces per lane)
template <int H, int F, typename T>
constexpr int fwd_epl() {
  using G = Geo<H, F, T>;
  return (G::QPL == 1 && G::CE <= 16) ? (sizeof(T) == 2 ? FWD_EPL_BF16 : FWD_EPL) : 1;
}

// gather instructions per chunk of the gather-layout forward: long rows as many edges
// as the score layout's chunk (CEL = EPL * 64 / H), short rows FWD_SHORT_CEL
template <int H, int F, typename T>
constexpr int gl_ngi_long() {
  using G = Geo<H, F, T>;
  constexpr int epl = (G::QPL == 1 && G::CE <= 16) ? (sizeof(T) == 2 ? GL_EPL_BF16 : GL_EPL_F32) : 1;
  return epl * G::CE / G::EPI;
}
template <int H, int F, typename T>
constexpr int gl_ngi_short() {
  using G = Geo<H, F, T>;
  return FWD_SHORT_CEL / G::EPI > 0 ? FWD_SHORT_CEL / G::EPI : 1;
}

// edge_fwd_gl.hip: the gather-layout forward (1 = launched).  rs: er from the gathered
// row with a_r (er unused); otherwise er gathered per edge.  short_rows picks the chunk.
int launch_fwd_gl(const msha_graph* g, int heads, int feat, int32_t dtype, const float* el,
                  const float* er, const float* ar, const void* hc, float slope,
                  const Dropout& dp, void* u, void* u_lo, float* lse, float* attd, float* uc,
                  float* qc, bool short_rows, dim3 grid, hipStream_t s);

// edge_bwd_gl.hip: the gather-layout row half of the backward for short rows (1 =
// launched).
int launch_bwd_rows_gl(const msha_graph* g, int heads, int feat, int32_t dtype, const float* el,
                       const float* er, const void* hc, const float* lse, const void* u,
                       const void* u_lo, const void* dU, const void* hs, const void* dV,
                       const float* row_coef, float slope, const Dropout& dp, float* d_el,
                       float* de, float* attd, int ld, void* d_hs, dim3 grid, hipStream_t s);

}  // namespace msha
