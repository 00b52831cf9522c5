// Block partials of the bipartite kernels -> their outputs (v; d_hc + d_er), shared by the
// standalone reduce launch (edge_bip.hip bip_reduce_kernel) and the launches that carry it
// as extra blocks (ours.hip: the Ours layer's prep / finish kernels -- one graph node fewer
// each way on the shipped graphs).
//
// out[i] = sum_b part[b][i] in block order (i < n_t -> out_t as T, else out_f fp32).  A
// reduce block owns 16 consecutive entries; 64 streams (entry c = lane & 15, stream =
// 4 wave + lane / 16 over 16 waves of work) sum contiguous block ranges, then the stream
// sums add in stream order.  A launch of NT < 1024 threads runs the 16 waves' work as
// 1024 / NT rounds per thread: the same sums in the same order, so the same bits.
#pragma once

#include "common.h"

namespace msha {

struct BipReduce {
  const float* part;
  void* out_t;
  float* out_f;
  int32_t nb, stride, n, n_t;
  int32_t seg, seg_stride, blk, blk_off, fblk, fstride;
  int32_t bf16;
  int32_t blocks() const { return (n + 15) / 16; }
};

template <typename T, int NT>
__device__ __forceinline__ void bip_reduce_block(const BipReduce& r, int blk_id,
                                                 float (*red)[17]) {
  static_assert(1024 % NT == 0 && NT >= 64, "whole waves");
  const int i0 = blk_id * 16;
  const int per = (r.nb + 63) / 64;
#pragma unroll
  for (int k = 0; k < 1024 / NT; ++k) {
    const int t = (int)threadIdx.x + k * NT;
    const int lane = t & 63, wv = t >> 6;
    const int c = lane & 15, st = wv * 4 + (lane >> 4);
    const int i = i0 + c;
    const int b0 = st * per, b1 = min(r.nb, b0 + per);
    float a = 0.f;
    if (i < r.n)
      for (int b = b0; b < b1; ++b) a += r.part[(int64_t)b * r.stride + i];
    red[st][c] = a;
  }
  __syncthreads();
  const int c = threadIdx.x;
  const int i = i0 + c;
  if (c < 16 && i < r.n) {
    float sum = red[0][c];
#pragma unroll 8
    for (int q = 1; q < 64; ++q) sum += red[q][c];
    // (a head-split launch's partials are [head blk][column seg]: entry i lands at column
    // (i % blk) / seg, head i / blk of the HT-head table)
    if (i < r.n_t)
      reinterpret_cast<T*>(r.out_t)[((i % r.blk) / r.seg) * r.seg_stride + (i / r.blk) * r.blk_off +
                                    i % r.seg] = from_f32<T>(sum);
    else
      r.out_f[((i - r.n_t) % r.fblk) * r.fstride + (i - r.n_t) / r.fblk] = sum;
  }
}

// The host side (edge_bip.hip): launch the reduce now, or -- between
// msha_bip_defer_reduce(1) and the next Ours-layer launch that takes it -- hand it over.
// Returns true when deferred.
bool bip_reduce_submit(const BipReduce& r, hipStream_t s);
// the pending reduce of this host thread, removed: true when there was one submitted on
// stream s (one submitted on another stream is launched there instead, false)
bool bip_reduce_take(BipReduce& r, hipStream_t s);
// the standalone reduce launch
void bip_reduce_run(const BipReduce& r, hipStream_t s);

}  // namespace msha
