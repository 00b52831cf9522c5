// Batched 2-D segment copies (include/msha_gnn.h msha_segments): the per-head parameter
// packing of the MSHA layers and the models' feature dropout, each one launch where
// torch issued a cat / stack / sum / contiguous copy or a dropout per tensor.
#include "common.h"

namespace msha {

struct SegBatch {
  msha_segment s[MSHA_MAX_SEGMENTS];
  const uint64_t* ctr;  // device replay counter (dropout offsets)
};

__global__ void __launch_bounds__(256) segments_kernel(SegBatch sb) {
  const msha_segment& g = sb.s[blockIdx.y];
  const int64_t total = g.rows * g.cols;
  Dropout d{};
  d.active = g.p > 0.f;
  if (d.active) {
    d.seed = g.seed;
    d.offset = g.offset;
    d.ctr = sb.ctr;
    const double t = (double)g.p * 4294967296.0;
    d.threshold = g.p >= 1.f ? 0xFFFFFFFFu : (uint32_t)(t > 4294967295.0 ? 4294967295.0 : t);
    d.scale = g.p < 1.f ? (float)(1.0 / (1.0 - (double)g.p)) : 0.f;
  }
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / g.cols, c = e - r * g.cols;
    float v = 0.f;
    if (g.a != nullptr) {
      v = g.a[r * g.lda + c];
      if (g.b != nullptr) v += g.b[r * g.ldb + c];
    }
    g.dst[r * g.ldd + c] = v * dropout_factor(d, (uint64_t)e);
  }
}

}  // namespace msha

using namespace msha;

extern "C" int msha_segments(int32_t n, const msha_segment* segs, msha_stream_t stream) {
  MSHA_ARG_CHECK(n >= 0 && n <= MSHA_MAX_SEGMENTS && (n == 0 || segs != nullptr),
                 "segments: 0..32 segments");
  if (n == 0) return MSHA_OK;
  SegBatch sb{};
  int64_t mx = 1;
  for (int i = 0; i < n; ++i) {
    const msha_segment& g = segs[i];
    MSHA_ARG_CHECK(g.dst != nullptr && g.rows >= 0 && g.cols >= 0, "segments: bad segment");
    MSHA_ARG_CHECK(g.p >= 0.f && g.p <= 1.f, "segments: p must be in [0, 1]");
    sb.s[i] = g;
    if (g.rows * g.cols > mx) mx = g.rows * g.cols;
  }
  hipStream_t s = (hipStream_t)stream;
  sb.ctr = rng_counter(s);
  const dim3 grid(grid_for(mx, 256 * 4, 1024), n);
  hipLaunchKernelGGL(segments_kernel, grid, dim3(256), 0, s, sb);
  return check_launch("segments");
}
