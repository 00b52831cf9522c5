// Batched 2-D segment copies (include/msha_gnn.h msha_segments): the per-head parameter
// packing of the MSHA layers, the models' feature dropout and the bf16 models' dtype
// casts, each one launch where torch issued a cat / stack / sum / contiguous copy, a
// dropout or a .to(dtype) per tensor.
#include "common.h"

namespace msha {

struct SegBatch {
  msha_segment s[MSHA_MAX_SEGMENTS];
  const uint64_t* ctr;  // device replay counter (dropout offsets)
};

__device__ __forceinline__ float keep4(const Dropout& d, uint64_t e, uint4 w) {
  const uint32_t x = (e & 3) == 0 ? w.x : (e & 3) == 1 ? w.y : (e & 3) == 2 ? w.z : w.w;
  return x >= d.threshold ? d.scale : 0.f;
}

// element loads / stores in a segment's storage type (fp32 arithmetic, bf16 rounded once)
__device__ __forceinline__ float seg_ld(const void* p, int dt, int64_t i) {
  return dt == MSHA_DTYPE_BF16 ? (float)reinterpret_cast<const bf16_t*>(p)[i]
                               : reinterpret_cast<const float*>(p)[i];
}
__device__ __forceinline__ void seg_st(void* p, int dt, int64_t i, float v) {
  if (dt == MSHA_DTYPE_BF16)
    reinterpret_cast<bf16_t*>(p)[i] = (bf16_t)v;
  else
    reinterpret_cast<float*>(p)[i] = v;
}
// 4 consecutive elements (element 4q .. 4q + 3): 16 B fp32 / 8 B bf16
__device__ __forceinline__ float4 seg_ld4(const void* p, int dt, int64_t q) {
  if (dt == MSHA_DTYPE_BF16) {
    const uint2 w = reinterpret_cast<const uint2*>(p)[q];
    return make_float4(__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u),
                       __uint_as_float(w.y << 16), __uint_as_float(w.y & 0xffff0000u));
  }
  return reinterpret_cast<const float4*>(p)[q];
}
__device__ __forceinline__ void seg_st4(void* p, int dt, int64_t q, float4 v) {
  if (dt == MSHA_DTYPE_BF16)
    reinterpret_cast<uint2*>(p)[q] = make_uint2(pack_bf16x2(v.x, v.y), pack_bf16x2(v.z, v.w));
  else
    reinterpret_cast<float4*>(p)[q] = v;
}

__global__ void __launch_bounds__(256) segments_kernel(SegBatch sb) {
  const msha_segment& g = sb.s[blockIdx.y];
  const int64_t total = g.rows * g.cols;
  const int adt = g.a_dtype, ddt = g.dst_dtype;
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
  const uint64_t off = d.active ? dropout_offset(d, d.offset) : 0;
  const int64_t nthr = (int64_t)gridDim.x * blockDim.x;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // 4-element pieces: 16 B (fp32) / 8 B (bf16) aligned in every operand
  const uintptr_t amask = adt == MSHA_DTYPE_BF16 ? 7 : 15, dmask = ddt == MSHA_DTYPE_BF16 ? 7 : 15;
  const bool flat = g.lda == g.cols && g.ldd == g.cols && (g.b == nullptr || g.ldb == g.cols) &&
                    total % 4 == 0 && (((uintptr_t)g.a | (uintptr_t)g.b) & amask) == 0 &&
                    ((uintptr_t)g.dst & dmask) == 0;
  if (flat) {  // contiguous table: 4 elements per thread, one generator block per 4
    for (int64_t q = tid; q < total / 4; q += nthr) {
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (g.a != nullptr) {
        v = seg_ld4(g.a, adt, q);
        if (g.b != nullptr) {
          const float4 w = seg_ld4(g.b, adt, q);
          v = make_float4(v.x + w.x, v.y + w.y, v.z + w.z, v.w + w.w);
        }
      }
      if (d.active) {
        const uint4 w = philox4(d.seed, off, (uint64_t)q);
        v = make_float4(v.x * (w.x >= d.threshold ? d.scale : 0.f),
                        v.y * (w.y >= d.threshold ? d.scale : 0.f),
                        v.z * (w.z >= d.threshold ? d.scale : 0.f),
                        v.w * (w.w >= d.threshold ? d.scale : 0.f));
      }
      seg_st4(g.dst, ddt, q, v);
    }
    return;
  }
  for (int64_t e = tid; e < total; e += nthr) {
    const int64_t r = e / g.cols, c = e - r * g.cols;
    float v = 0.f;
    if (g.a != nullptr) {
      v = seg_ld(g.a, adt, r * g.lda + c);
      if (g.b != nullptr) v += seg_ld(g.b, adt, r * g.ldb + c);
    }
    if (d.active) v *= keep4(d, (uint64_t)e, philox4(d.seed, off, (uint64_t)e >> 2));
    seg_st(g.dst, ddt, r * g.ldd + c, v);
  }
}

__global__ void __launch_bounds__(256) keep_mask4_kernel(Dropout d, int64_t n, uint8_t* keep) {
  const uint64_t off = dropout_offset(d, d.offset);
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x)
    keep[e] = keep4(d, (uint64_t)e, philox4(d.seed, off, (uint64_t)e >> 2)) != 0.f ? 1 : 0;
}

__global__ void __launch_bounds__(256) keep_mask_word_kernel(Dropout d, int64_t n, int word,
                                                             uint8_t* keep) {
  const uint64_t off = dropout_offset(d, d.offset);
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const uint4 w = philox4(d.seed, off, (uint64_t)e);
    const uint32_t x = word == 0 ? w.x : word == 1 ? w.y : word == 2 ? w.z : w.w;
    keep[e] = x >= d.threshold ? 1 : 0;
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
    MSHA_ARG_CHECK((g.a_dtype == MSHA_DTYPE_F32 || g.a_dtype == MSHA_DTYPE_BF16) &&
                       (g.dst_dtype == MSHA_DTYPE_F32 || g.dst_dtype == MSHA_DTYPE_BF16),
                   "segments: dtypes must be MSHA_DTYPE_F32 or MSHA_DTYPE_BF16");
    sb.s[i] = g;
    if (g.rows * g.cols > mx) mx = g.rows * g.cols;
  }
  hipStream_t s = (hipStream_t)stream;
  sb.ctr = rng_counter(s);
  const dim3 grid(grid_for(mx, 256 * 4, 1024), n);
  hipLaunchKernelGGL(segments_kernel, grid, dim3(256), 0, s, sb);
  return check_launch("segments");
}

extern "C" int msha_dropout_keep_mask4(uint64_t seed, uint64_t offset, int64_t n, float p,
                                       uint8_t* keep, msha_stream_t stream) {
  MSHA_ARG_CHECK(n >= 0 && (n == 0 || keep != nullptr), "dropout_keep_mask4: bad buffer");
  MSHA_ARG_CHECK(p >= 0.f && p <= 1.f, "dropout_keep_mask4: p must be in [0, 1]");
  if (n == 0) return MSHA_OK;
  Dropout d = make_dropout(p, seed, offset, (hipStream_t)stream);
  d.active = true;
  hipLaunchKernelGGL(keep_mask4_kernel, dim3(grid_for(n, 256, 8192)), dim3(256), 0,
                     (hipStream_t)stream, d, n, keep);
  return check_launch("dropout_keep_mask4");
}

extern "C" int msha_dropout_keep_mask_word(uint64_t seed, uint64_t offset, int64_t n, float p,
                                           int32_t word, uint8_t* keep, msha_stream_t stream) {
  MSHA_ARG_CHECK(n >= 0 && (n == 0 || keep != nullptr), "dropout_keep_mask_word: bad buffer");
  MSHA_ARG_CHECK(p >= 0.f && p <= 1.f, "dropout_keep_mask_word: p must be in [0, 1]");
  MSHA_ARG_CHECK(word >= 0 && word < 4, "dropout_keep_mask_word: word must be 0..3");
  if (n == 0) return MSHA_OK;
  Dropout d = make_dropout(p, seed, offset, (hipStream_t)stream);
  d.active = true;
  hipLaunchKernelGGL(keep_mask_word_kernel, dim3(grid_for(n, 256, 8192)), dim3(256), 0,
                     (hipStream_t)stream, d, n, word, keep);
  return check_launch("dropout_keep_mask_word");
}
