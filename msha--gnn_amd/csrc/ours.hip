// Full MSHA layer (Ours.OursLayer, Ours.py:54-109): the intra-source attention of a
// batch of sources over their city / province groups, coupled to the inter
// attention through the joint normaliser SUM_county (Ours.py:84-90).
//
// Reference (dense): for a batch of B sources (source_index),
//   e3_b  = lrelu(h2_b . (a3[:F] + a3[F:]))           constant along n (Ours.py:74-75)
//   att3  = where(city_adj[src] > 0, e3, -9e15)        (B, N)          (Ours.py:81)
//   SUM_b = sum_n exp(att3) + sum_n exp(att4) + sum_j exp(attd_inter[src_b, j])
//         (no max subtraction; the last term runs over ALL M columns, post-dropout)
//   att3  = dropout(exp(att3) / SUM), att4 likewise    (Ours.py:87-90)
//   IntraNC = att3^T @ h2[src] + att4^T @ h2[src]      (N, F)          (Ours.py:99)
//   u = lrelu(bn2(att_inter @ h1 + IntraNC))           (Ours.py:101)
// Here the masks are group ids (same city <=> same id): the (B, N) tensors are
// never built.  Per batch entry b: c3 = |city group|, so sum_n exp(att3) = c3 E3.
//
// Kernels:  prep (wave per b): e3/e4, the inter term I_b, SUM_b, weights w3/w4
//           fwd  (wave per node n): ballot-match the batch against n's groups and
//                gather-aggregate the matching h2 rows (dropout per (b, n))
//           bwd_gather (wave per (b, kind)): G_b = sum_{n in group} drop * dU_n
//           bwd_finish (one workgroup): scalar chain, deterministic per-row sums
#include <atomic>
#include <cstdlib>

#include "bip_reduce.h"
#include "common.h"

namespace msha {

constexpr int kMaxD = 512;  // heads * feat
constexpr int kOursMB = 4;  // forward: batch matches whose loads are in flight together

struct OursArgs {
  int64_t B, N, M;
  int H, F;
  const int64_t* src;
  const int32_t* gid3;
  const int32_t* gptr3;
  const int32_t* gmem3;
  const int32_t* gid4;
  const int32_t* gptr4;
  const int32_t* gmem4;
  const void* h2;    // (N, H, F), fp32 or bf16 (the kernels' T)
  const float* a3s;  // (H, F) = a3[:F] + a3[F:]
  const float* a4s;
  float slope;
  Dropout dp;  // edge dropout: offset; intra att3/att4: see intra_keep_bits
};

enum { BS_PRE3 = 0, BS_PRE4, BS_E3, BS_E4, BS_SUM, BS_W3, BS_W4, BS_I, BS_N };

template <typename T>
__device__ __forceinline__ float ldt(const void* p, int64_t i) {
  return to_f32(reinterpret_cast<const T*>(p)[i]);
}

// Intra dropout of (batch entry b, node n), idx = b * N + n: one Philox4x32-10 block per
// head pair j = h / 2, keyed (seed; counter {idx, offset + 1 + j}); word 2 (h % 2) + kind
// keeps att3 (kind 0) / att4 (kind 1) of head h.  One generator call covers both kinds of
// two heads (msha_dropout_keep_mask_word exports the words for tests).
__device__ __forceinline__ uint32_t intra_word(const uint4& w, int h, int kind) {
  const int t = 2 * (h & 1) + kind;
  return t == 0 ? w.x : t == 1 ? w.y : t == 2 ? w.z : w.w;
}
__device__ __forceinline__ float intra_drop(const Dropout& d, int kind, int h, uint64_t idx) {
  if (!d.active) return 1.f;
  const uint4 w = philox4(d.seed, dropout_offset(d, d.offset + 1 + (uint64_t)(h >> 1)), idx);
  return intra_word(w, h, kind) >= d.threshold ? d.scale : 0.f;
}
// keep bits (bit h) of both kinds for heads h < min(H, 32)
__device__ __forceinline__ void intra_keep_bits(const Dropout& d, int H, uint64_t idx,
                                                uint32_t& kb3, uint32_t& kb4) {
  kb3 = kb4 = 0u;
  const uint64_t off = dropout_offset(d, d.offset + 1);
  for (int h = 0; h < H && h < 32; h += 2) {
    const uint4 w = philox4(d.seed, off + (uint64_t)(h >> 1), idx);
    kb3 |= (w.x >= d.threshold ? 1u : 0u) << h;
    kb4 |= (w.y >= d.threshold ? 1u : 0u) << h;
    if (h + 1 < H) {
      kb3 |= (w.z >= d.threshold ? 1u : 0u) << (h + 1);
      kb4 |= (w.w >= d.threshold ? 1u : 0u) << (h + 1);
    }
  }
}

// ---------------------------------------------------------------------- prep ---
// Blocks from nprep on run the bipartite forward's block-partial reduce of v (handed over by
// msha_bip_defer_reduce; bip_reduce.h), which needs nothing prep computes: one launch
// instead of two.
template <typename T>
__global__ void __launch_bounds__(256) ours_prep_kernel(
    OursArgs a, const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
    const uint8_t* __restrict__ rowflag, const float* __restrict__ el,
    const float* __restrict__ er, const float* __restrict__ lse, float* __restrict__ bstat,
    BipReduce rd, int nprep) {
  if ((int)blockIdx.x >= nprep) {
    __shared__ float red[64][17];
    bip_reduce_block<T, 256>(rd, (int)blockIdx.x - nprep, red);
    return;
  }
  const int lane = lane_id();
  const int64_t b = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (b >= a.B) return;
  const int64_t i = a.src[b];
  const int H = a.H, F = a.F;
  const int32_t start = rowptr[i], end = rowptr[i + 1];
  const bool virt = rowflag != nullptr && rowflag[i] != 0;
  const float c3 = (float)(a.gptr3[a.gid3[i] + 1] - a.gptr3[a.gid3[i]]);
  const float c4 = (float)(a.gptr4[a.gid4[i] + 1] - a.gptr4[a.gid4[i]]);
  for (int h = 0; h < H; ++h) {
    float p3 = 0.f, p4 = 0.f;
    for (int f = lane; f < F; f += 64) {
      const float x = ldt<T>(a.h2, (i * H + h) * F + f);
      p3 = fmaf(x, a.a3s[h * F + f], p3);
      p4 = fmaf(x, a.a4s[h * F + f], p4);
    }
    p3 = wave_xor_sum<1>(p3);
    p4 = wave_xor_sum<1>(p4);
    // I_b = sum over ALL M columns of exp(post-dropout inter attention): non-edges
    // hold attention 0 -> exp(0) = 1 each
    float I = 0.f;
    for (int32_t e = start + lane; e < end; e += 64) {
      const float s = virt ? 0.f : lrelu(el[i * H + h] + er[(int64_t)col[e] * H + h], a.slope);
      const float att = __expf(s - lse[i * H + h]) * dropout_factor(a.dp, (uint64_t)e * H + h);
      I += expf(att);
    }
    I = wave_xor_sum<1>(I) + (float)(a.M - (end - start));
    const float E3 = expf(lrelu(p3, a.slope)), E4 = expf(lrelu(p4, a.slope));
    const float sum = (c3 * E3 + c4 * E4) + I;
    if (lane == 0) {
      float* o = bstat + (b * H + h) * BS_N;
      o[BS_PRE3] = p3; o[BS_PRE4] = p4; o[BS_E3] = E3; o[BS_E4] = E4;
      o[BS_SUM] = sum; o[BS_W3] = E3 / sum; o[BS_W4] = E4 / sum; o[BS_I] = I;
    }
  }
}

// ---------------------------------------------------------------- forward ---
// u_out[n] = u_in[n] + sum_{b: city(src_b) = city(n)} drop * w3_b h2[src_b]
//                    + sum_{b: prov(src_b) = prov(n)} drop * w4_b h2[src_b]
template <typename T, int KD>
__global__ void __launch_bounds__(256) ours_fwd_kernel(OursArgs a, const float* __restrict__ bstat,
                                                       const T* __restrict__ u_in,
                                                       T* __restrict__ u_out) {
  const int lane = lane_id();
  const int D = a.H * a.F;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  if (a.B <= 64) {
    // one batch chunk (train.py's 64 flows): lane b's source and its groups load once per
    // wave; a wave walks nodes n, n + nwaves, ... with the next node's group ids and u_in
    // loaded before this node's matches are gathered.  Same sums in the same order.
    const bool bvalid = lane < a.B;
    const int64_t ib = bvalid ? a.src[lane] : 0;
    const int32_t bg3 = bvalid ? a.gid3[ib] : 0, bg4 = bvalid ? a.gid4[ib] : 0;
    int64_t n = wave;
    if (n >= a.N) return;
    int32_t g3 = a.gid3[n], g4 = a.gid4[n];
    float uin[KD];
#pragma unroll
    for (int k = 0; k < KD; ++k) {
      const int d = lane + 64 * k;
      uin[k] = d < D ? to_f32(u_in[n * D + d]) : 0.f;
    }
    while (true) {
      const int64_t nn = n + nwaves;
      const bool has_next = nn < a.N;
      int32_t ng3 = 0, ng4 = 0;
      float nuin[KD];
      if (has_next) {
        ng3 = a.gid3[nn];
        ng4 = a.gid4[nn];
      }
#pragma unroll
      for (int k = 0; k < KD; ++k) {
        const int d = lane + 64 * k;
        nuin[k] = has_next && d < D ? to_f32(u_in[nn * D + d]) : 0.f;
      }
      float acc3[KD], acc4[KD];
#pragma unroll
      for (int k = 0; k < KD; ++k) acc3[k] = acc4[k] = 0.f;
      const uint64_t bal3 = __ballot(bvalid && bg3 == g3);
      const uint64_t bal4 = __ballot(bvalid && bg4 == g4);
      uint32_t kb3 = 0xffffffffu, kb4 = 0xffffffffu;
      if (a.dp.active && (bal3 | bal4)) intra_keep_bits(a.dp, a.H, (uint64_t)lane * a.N + n, kb3, kb4);
      // matches in bit order, kOursMB at a time: the batch's weight and h2 loads leave
      // together (an unused slot repeats the first match's addresses), then the fmas run
      // in bit order for the used slots only
      constexpr int MB = kOursMB;
      for (int kind = 0; kind < 2; ++kind) {
        uint64_t bal = kind == 0 ? bal3 : bal4;
        const uint32_t kbk = kind == 0 ? kb3 : kb4;
        while (bal) {
          int bits[MB];
#pragma unroll
          for (int q = 0; q < MB; ++q) {
            bits[q] = bal ? __ffsll((long long)bal) - 1 : -1;
            bal &= bal - 1;
          }
          float wv[MB][KD], xv[MB][KD];
#pragma unroll
          for (int q = 0; q < MB; ++q) {
            const int bit = bits[q] >= 0 ? bits[q] : bits[0];
            const int64_t ibb = __shfl(ib, bit);
            const uint32_t kbits = __shfl(kbk, bit);
#pragma unroll
            for (int k = 0; k < KD; ++k) {
              const int d = min(lane + 64 * k, D - 1);
              const int h = d / a.F;
              float drop = 1.f;
              if (a.dp.active)
                drop = h < 32 ? (((kbits >> h) & 1u) ? a.dp.scale : 0.f)
                              : intra_drop(a.dp, kind, h, (uint64_t)bit * a.N + n);
              wv[q][k] = bstat[((int64_t)bit * a.H + h) * BS_N + (kind == 0 ? BS_W3 : BS_W4)] * drop;
              xv[q][k] = ldt<T>(a.h2, ibb * D + d);
            }
          }
#pragma unroll
          for (int q = 0; q < MB; ++q) {
            if (bits[q] < 0) break;
#pragma unroll
            for (int k = 0; k < KD; ++k) {
              if (kind == 0) acc3[k] = fmaf(wv[q][k], xv[q][k], acc3[k]);
              else acc4[k] = fmaf(wv[q][k], xv[q][k], acc4[k]);
            }
          }
        }
      }
#pragma unroll
      for (int k = 0; k < KD; ++k) {
        const int d = lane + 64 * k;
        if (d < D) u_out[n * D + d] = from_f32<T>(uin[k] + (acc3[k] + acc4[k]));
      }
      if (!has_next) break;
      n = nn;
      g3 = ng3;
      g4 = ng4;
#pragma unroll
      for (int k = 0; k < KD; ++k) uin[k] = nuin[k];
    }
    return;
  }
  for (int64_t n = wave; n < a.N; n += nwaves) {
    const int32_t g3 = a.gid3[n], g4 = a.gid4[n];
    float acc3[KD], acc4[KD];
#pragma unroll
    for (int k = 0; k < KD; ++k) acc3[k] = acc4[k] = 0.f;
    for (int64_t base = 0; base < a.B; base += 64) {
      const int64_t b = base + lane;
      const bool valid = b < a.B;
      const int64_t ib = valid ? a.src[b] : 0;
      uint64_t bal3 = __ballot(valid && a.gid3[ib] == g3);
      uint64_t bal4 = __ballot(valid && a.gid4[ib] == g4);
      // keep bits of (b = base + lane, n) for every head, drawn lane-parallel once per
      // chunk (bit h of kb3 / kb4); heads >= 32 fall back to a per-use draw
      uint32_t kb3 = 0xffffffffu, kb4 = 0xffffffffu;
      if (a.dp.active && (bal3 | bal4)) intra_keep_bits(a.dp, a.H, (uint64_t)b * a.N + n, kb3, kb4);
      for (int kind = 0; kind < 2; ++kind) {
        uint64_t bal = kind == 0 ? bal3 : bal4;
        while (bal) {
          const int bit = __ffsll((long long)bal) - 1;
          bal &= bal - 1;
          const int64_t bb = base + bit;
          const int64_t ibb = __shfl(ib, bit);
          const uint32_t kbits = __shfl(kind == 0 ? kb3 : kb4, bit);
#pragma unroll
          for (int k = 0; k < KD; ++k) {
            const int d = lane + 64 * k;
            if (d < D) {
              const int h = d / a.F;
              float drop = 1.f;
              if (a.dp.active)
                drop = h < 32 ? (((kbits >> h) & 1u) ? a.dp.scale : 0.f)
                              : intra_drop(a.dp, kind, h, (uint64_t)bb * a.N + n);
              const float w = bstat[(bb * a.H + h) * BS_N + (kind == 0 ? BS_W3 : BS_W4)] * drop;
              const float x = ldt<T>(a.h2, ibb * D + d);
              if (kind == 0) acc3[k] = fmaf(w, x, acc3[k]); else acc4[k] = fmaf(w, x, acc4[k]);
            }
          }
        }
      }
    }
#pragma unroll
    for (int k = 0; k < KD; ++k) {
      const int d = lane + 64 * k;
      if (d < D) u_out[n * D + d] = from_f32<T>(to_f32(u_in[n * D + d]) + (acc3[k] + acc4[k]));
    }
  }
}

// Batch of <= 64 sources with D <= 256 (train.py's 64 flows): the batch's h2 rows (fp32,
// B x D) and intra weights w3 / w4 (B x H) are staged in LDS once per block, so a node's
// matches read LDS instead of a dependent global round trip each (the global-gather form
// above took 43 us at the 2015 graph: ~5 nodes per wave, one L2 latency chain per node).
// A persistent grid walks the nodes; the next node's group ids and u_in are loaded before
// this node's matches run.  Same sums in the same order as ours_fwd_kernel.  Blocks of 8
// waves, 4 per CU (4 x 34 KB of LDS at B 64, D 128): ~5 nodes per wave at the 2015 graph
// (2 blocks of 4 waves per CU left each wave ~19 dependent node steps: 60 us vs 43 us
// for the global-gather form).
constexpr int kOursFwdWaves = 8;
template <typename T, int KD, bool PACK>
__global__ void __launch_bounds__(64 * kOursFwdWaves)
__attribute__((amdgpu_waves_per_eu(KD >= 4 ? 4 : 8))) ours_fwd_lds_kernel(OursArgs a,
                                                           const float* __restrict__ bstat,
                                                           const T* __restrict__ u_in,
                                                           T* __restrict__ u_out) {
  extern __shared__ __attribute__((aligned(16))) float sx[];  // [B][D], then w3 [B][H], w4
  const int lane = lane_id(), wv = threadIdx.x >> 6;
  const int D = a.H * a.F, H = a.H;
  const int B = (int)a.B;
  float* w3s = sx + B * D;
  float* w4s = w3s + B * H;
  {  // every row this wave stages, loads first: one gather latency, not one per row
    constexpr int RPW = 64 / kOursFwdWaves;  // B <= 64
    int64_t ib[RPW];
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      const int b = wv + kOursFwdWaves * r;
      ib[r] = b < B ? a.src[b] : 0;
    }
    float xv[RPW][KD];
#pragma unroll
    for (int r = 0; r < RPW; ++r)
#pragma unroll
      for (int k = 0; k < KD; ++k) {
        const int d = lane + 64 * k;
        xv[r][k] = d < D ? ldt<T>(a.h2, ib[r] * D + d) : 0.f;
      }
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      const int b = wv + kOursFwdWaves * r;
#pragma unroll
      for (int k = 0; k < KD; ++k) {
        const int d = lane + 64 * k;
        if (b < B && d < D) sx[b * D + d] = xv[r][k];
      }
    }
  }
  for (int i = threadIdx.x; i < B * H; i += 64 * kOursFwdWaves) {
    w3s[i] = bstat[(int64_t)i * BS_N + BS_W3];
    w4s[i] = bstat[(int64_t)i * BS_N + BS_W4];
  }
  const bool bvalid = lane < B;
  const int64_t ib = bvalid ? a.src[lane] : 0;
  const int32_t bg3 = bvalid ? a.gid3[ib] : 0, bg4 = bvalid ? a.gid4[ib] : 0;
  __syncthreads();
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  int64_t n = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (n >= a.N) return;
  int hk[KD];
#pragma unroll
  for (int k = 0; k < KD; ++k) hk[k] = min(lane + 64 * k, D - 1) / a.F;
  if (PACK && a.dp.active) {
    // Intra dropout: the keep bits of a (batch entry, node) pair are needed only where the
    // entry's group matches the node's (~3 of 64 entries per node at the 2015 graph), but a
    // per-node draw costs the whole wave one Philox block per head pair.  So the matched
    // pairs of consecutive nodes are packed into groups of <= 64 (one lane each, in node
    // then entry order), one draw covers a group, and each node's matches read their
    // words from LDS at (group base + rank of the entry among the node's matches).  Same
    // draws, same sums in the same order as the per-node form below.
    uint16_t* pl = reinterpret_cast<uint16_t*>(w4s + B * H) + wv * 64;
    uint2* kw = reinterpret_cast<uint2*>(
                    reinterpret_cast<uint16_t*>(w4s + B * H) + kOursFwdWaves * 64 +
                    ((B * D) & 1) * 2) + wv * 64;  // 8-B aligned: sx + w3s + w4s is 4 (B D + 2 B H) B
    const uint64_t lt = (1ull << lane) - 1ull;
    for (int64_t c0 = n; c0 < a.N; c0 += 64 * nwaves) {
      // this wave's next <= 64 nodes c0 + k nwaves: group ids one per lane
      const int kc = (int)min<int64_t>(64, (a.N - c0 + nwaves - 1) / nwaves);
      const int64_t nl = c0 + (int64_t)lane * nwaves;
      const int32_t cg3 = lane < kc ? a.gid3[nl] : -1, cg4 = lane < kc ? a.gid4[nl] : -1;
      float uin[KD];
#pragma unroll
      for (int k = 0; k < KD; ++k) {
        const int d = lane + 64 * k;
        uin[k] = d < D ? to_f32(u_in[c0 * D + d]) : 0.f;
      }
      int k0 = 0;
      while (k0 < kc) {
        int cnt = 0, k1 = k0;
        for (; k1 < kc; ++k1) {
          const int32_t g3 = __builtin_amdgcn_readlane(cg3, k1);
          const int32_t g4 = __builtin_amdgcn_readlane(cg4, k1);
          const uint64_t bal = __ballot(bvalid && (bg3 == g3 || bg4 == g4));
          const int c = __popcll(bal);
          if (k1 > k0 && cnt + c > 64) break;
          if ((bal >> lane) & 1ull) pl[cnt + __popcll(bal & lt)] = (uint16_t)(((k1 - k0) << 6) | lane);
          cnt += c;
        }
        __builtin_amdgcn_wave_barrier();
        if (lane < cnt) {
          const int q = pl[lane];
          const int64_t node = c0 + (int64_t)(k0 + (q >> 6)) * nwaves;
          uint32_t kb3, kb4;
          intra_keep_bits(a.dp, H, (uint64_t)(q & 63) * a.N + node, kb3, kb4);
          kw[lane] = make_uint2(kb3, kb4);
        }
        __builtin_amdgcn_wave_barrier();
        int base = 0;
        for (int kk = k0; kk < k1; ++kk) {
          const int64_t nd = c0 + (int64_t)kk * nwaves;
          const bool has_next = kk + 1 < kc;
          float nuin[KD];
#pragma unroll
          for (int k = 0; k < KD; ++k) {
            const int d = lane + 64 * k;
            nuin[k] = has_next && d < D ? to_f32(u_in[(nd + nwaves) * D + d]) : 0.f;
          }
          const int32_t g3 = __builtin_amdgcn_readlane(cg3, kk);
          const int32_t g4 = __builtin_amdgcn_readlane(cg4, kk);
          const uint64_t bal3 = __ballot(bvalid && bg3 == g3);
          const uint64_t bal4 = __ballot(bvalid && bg4 == g4);
          const uint64_t ball = bal3 | bal4;
          float acc3[KD], acc4[KD];
#pragma unroll
          for (int k = 0; k < KD; ++k) acc3[k] = acc4[k] = 0.f;
          for (int kind = 0; kind < 2; ++kind) {
            uint64_t bal = kind == 0 ? bal3 : bal4;
            const float* ws = kind == 0 ? w3s : w4s;
            while (bal) {
              const int bit0 = __ffsll((long long)bal) - 1;
              bal &= bal - 1;
              const bool two = bal != 0;
              const int bit1 = two ? __ffsll((long long)bal) - 1 : bit0;
              if (two) bal &= bal - 1;
              const int bits[2] = {bit0, bit1};
              float wv2[2][KD], xv2[2][KD];
#pragma unroll
              for (int q = 0; q < 2; ++q) {
                const int bit = bits[q];
                const uint2 kwd = kw[base + __popcll(ball & ((1ull << bit) - 1ull))];
                const uint32_t kbits = kind == 0 ? kwd.x : kwd.y;
#pragma unroll
                for (int k = 0; k < KD; ++k) {
                  const int d = min(lane + 64 * k, D - 1);
                  const int h = hk[k];
                  const float drop = h < 32 ? (((kbits >> h) & 1u) ? a.dp.scale : 0.f)
                                            : intra_drop(a.dp, kind, h, (uint64_t)bit * a.N + nd);
                  wv2[q][k] = ws[bit * H + h] * drop;
                  xv2[q][k] = sx[bit * D + d];
                }
              }
#pragma unroll
              for (int q = 0; q < 2; ++q) {
                if (q == 1 && !two) break;
#pragma unroll
                for (int k = 0; k < KD; ++k) {
                  if (kind == 0) acc3[k] = fmaf(wv2[q][k], xv2[q][k], acc3[k]);
                  else acc4[k] = fmaf(wv2[q][k], xv2[q][k], acc4[k]);
                }
              }
            }
          }
          base += __popcll(ball);
#pragma unroll
          for (int k = 0; k < KD; ++k) {
            const int d = lane + 64 * k;
            if (d < D) u_out[nd * D + d] = from_f32<T>(uin[k] + (acc3[k] + acc4[k]));
            uin[k] = nuin[k];
          }
        }
        // the next group's pair list overwrites this one's: every lane is past its reads
        __builtin_amdgcn_wave_barrier();
        k0 = k1;
      }
    }
    return;
  }
  int32_t g3 = a.gid3[n], g4 = a.gid4[n];
  float uin[KD];
#pragma unroll
  for (int k = 0; k < KD; ++k) {
    const int d = lane + 64 * k;
    uin[k] = d < D ? to_f32(u_in[n * D + d]) : 0.f;
  }
  while (true) {
    const int64_t nn = n + nwaves;
    const bool has_next = nn < a.N;
    const int32_t ng3 = has_next ? a.gid3[nn] : 0, ng4 = has_next ? a.gid4[nn] : 0;
    float nuin[KD];
#pragma unroll
    for (int k = 0; k < KD; ++k) {
      const int d = lane + 64 * k;
      nuin[k] = has_next && d < D ? to_f32(u_in[nn * D + d]) : 0.f;
    }
    float acc3[KD], acc4[KD];
#pragma unroll
    for (int k = 0; k < KD; ++k) acc3[k] = acc4[k] = 0.f;
    const uint64_t bal3 = __ballot(bvalid && bg3 == g3);
    const uint64_t bal4 = __ballot(bvalid && bg4 == g4);
    uint32_t kb3 = 0xffffffffu, kb4 = 0xffffffffu;
    if (a.dp.active && (bal3 | bal4)) intra_keep_bits(a.dp, a.H, (uint64_t)lane * a.N + n, kb3, kb4);
    for (int kind = 0; kind < 2; ++kind) {
      uint64_t bal = kind == 0 ? bal3 : bal4;
      const uint32_t kbk = kind == 0 ? kb3 : kb4;
      const float* ws = kind == 0 ? w3s : w4s;
      // matches two at a time: both matches' LDS reads leave before the first fma (the
      // sums stay in bit order); the keep bits come by readlane (the match index is
      // wave-uniform), not a bpermute round trip through LDS
      while (bal) {
        const int bit0 = __ffsll((long long)bal) - 1;
        bal &= bal - 1;
        const bool two = bal != 0;
        const int bit1 = two ? __ffsll((long long)bal) - 1 : bit0;
        if (two) bal &= bal - 1;
        const int bits[2] = {bit0, bit1};
        float wv2[2][KD], xv2[2][KD];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int bit = bits[q];
          const uint32_t kbits = __builtin_amdgcn_readlane(kbk, bit);
#pragma unroll
          for (int k = 0; k < KD; ++k) {
            const int d = min(lane + 64 * k, D - 1);
            const int h = hk[k];
            float drop = 1.f;
            if (a.dp.active)
              drop = h < 32 ? (((kbits >> h) & 1u) ? a.dp.scale : 0.f)
                            : intra_drop(a.dp, kind, h, (uint64_t)bit * a.N + n);
            wv2[q][k] = ws[bit * H + h] * drop;
            xv2[q][k] = sx[bit * D + d];
          }
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          if (q == 1 && !two) break;
#pragma unroll
          for (int k = 0; k < KD; ++k) {
            if (kind == 0) acc3[k] = fmaf(wv2[q][k], xv2[q][k], acc3[k]);
            else acc4[k] = fmaf(wv2[q][k], xv2[q][k], acc4[k]);
          }
        }
      }
    }
#pragma unroll
    for (int k = 0; k < KD; ++k) {
      const int d = lane + 64 * k;
      if (d < D) u_out[n * D + d] = from_f32<T>(uin[k] + (acc3[k] + acc4[k]));
    }
    if (!has_next) break;
    n = nn;
    g3 = ng3;
    g4 = ng4;
#pragma unroll
    for (int k = 0; k < KD; ++k) uin[k] = nuin[k];
  }
}

// ----------------------------------------------------------- backward: gather ---
// Gp[b, kind, c] = sum_{n in chunk c of group(kind, src_b)} drop(kind, b, n) * dU[n]
// (chunks of kGatherChunk members, ascending), then G[b, kind] = sum_c Gp[b, kind, c]
// in chunk order: one wave per (b, kind, chunk) keeps thousands of members in flight.
constexpr int kGatherChunk = 64;  // one member per lane for the keep-bit draw

// bf16 tables: a lane takes two adjacent elements per 4-byte load (EL = 2), so a wave
// reads a 128-element row slice per instruction as the fp32 kernel does; every element's
// sum over the members keeps its order (same bits as one element per lane).
template <typename T, int KD>
__global__ void __launch_bounds__(256) ours_bwd_gather_kernel(OursArgs a,
                                                              const T* __restrict__ dU,
                                                              int nck, float* __restrict__ Gp) {
  constexpr int EL = (sizeof(T) == 2 && KD > 1) ? 2 : 1;  // elements per lane per slot
  constexpr int KE = KD / EL;                              // slots per lane
  const int lane = lane_id();
  const int D = a.H * a.F;
  const int64_t wv = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (wv >= 2 * a.B * nck) return;
  const int c = (int)(wv % nck);
  const int64_t bk = wv / nck;
  const int64_t b = bk >> 1;
  const int kind = (int)(bk & 1);
  const int64_t i = a.src[b];
  const int32_t* gptr = kind == 0 ? a.gptr3 : a.gptr4;
  const int32_t* gmem = kind == 0 ? a.gmem3 : a.gmem4;
  const int32_t grp = kind == 0 ? a.gid3[i] : a.gid4[i];
  const int32_t m0 = gptr[grp] + c * kGatherChunk;
  const int32_t m1 = min(gptr[grp + 1], m0 + kGatherChunk);
  float acc[KE][EL];
#pragma unroll
  for (int k = 0; k < KE; ++k)
#pragma unroll
    for (int e = 0; e < EL; ++e) acc[k][e] = 0.f;
  // members of this chunk: lane j draws the keep bits of (b, member j) for every head
  const int cnt = m1 - m0;  // <= kGatherChunk == 64
  const int64_t nj = lane < cnt ? (int64_t)gmem[m0 + lane] : 0;
  uint32_t kbits = 0xffffffffu;
  if (a.dp.active) {
    uint32_t k3, k4;
    intra_keep_bits(a.dp, a.H, (uint64_t)b * a.N + nj, k3, k4);
    kbits = kind == 0 ? k3 : k4;
  }
  // GU members' rows are loaded before they are accumulated (in member order, as one
  // at a time): GU gathers in flight per wave instead of one
  constexpr int GU = 8;
  for (int t0 = 0; t0 < cnt; t0 += GU) {
    float v[GU][KE][EL];
    int64_t nn[GU];
    uint32_t kk[GU];
#pragma unroll
    for (int u = 0; u < GU; ++u) {
      nn[u] = __shfl(nj, t0 + u);  // lanes past cnt hold member 0: a valid row, unused
      kk[u] = __shfl(kbits, t0 + u);
#pragma unroll
      for (int k = 0; k < KE; ++k) {
        const int d = (lane + 64 * k) * EL;
        if constexpr (EL == 2) {
          const uint32_t w = d < D ? *reinterpret_cast<const uint32_t*>(dU + nn[u] * D + d) : 0u;
          v[u][k][0] = __uint_as_float(w << 16);
          v[u][k][1] = __uint_as_float(w & 0xffff0000u);
        } else {
          v[u][k][0] = d < D ? to_f32(dU[nn[u] * D + d]) : 0.f;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < GU; ++u) {
      if (t0 + u >= cnt) break;
#pragma unroll
      for (int k = 0; k < KE; ++k) {
#pragma unroll
        for (int e = 0; e < EL; ++e) {
          const int d = (lane + 64 * k) * EL + e;
          if (d < D) {
            const int h = d / a.F;
            float drop = 1.f;
            if (a.dp.active)
              drop = h < 32 ? (((kk[u] >> h) & 1u) ? a.dp.scale : 0.f)
                            : intra_drop(a.dp, kind, h, (uint64_t)b * a.N + nn[u]);
            acc[k][e] = fmaf(drop, v[u][k][e], acc[k][e]);
          }
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < KE; ++k)
#pragma unroll
    for (int e = 0; e < EL; ++e) {
      const int d = (lane + 64 * k) * EL + e;
      if (d < D) Gp[(bk * nck + c) * D + d] = acc[k][e];
    }
}

// (also zero-fills row_coef (nz floats), which the finish kernel after it writes at the
// batch rows: one launch fewer than a separate fill)
__global__ void __launch_bounds__(256) ours_bwd_gather_reduce_kernel(int64_t B, int D, int nck,
                                                                     const float* __restrict__ Gp,
                                                                     float* __restrict__ G,
                                                                     float* __restrict__ zf,
                                                                     int64_t nz) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nz;
       t += (int64_t)gridDim.x * blockDim.x)
    zf[t] = 0.f;
  const int64_t total = 2 * B * D;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t bk = t / D;
    const int d = (int)(t % D);
    float s = 0.f;
    int c = 0;
    for (; c + 7 < nck; c += 8) {  // 8 chunk partials loaded, then added in order
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = Gp[(bk * nck + c + u) * D + d];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; c < nck; ++c) s += Gp[(bk * nck + c) * D + d];
    G[t] = s;
  }
}

// ------------------------------------------------------------ backward: finish ---
// mode 0 (before the inter row backward):
//   per (b, h): dw3 = G3 . h2_b, dw4 = G4 . h2_b; through w = E/SUM, SUM = c3E3 + c4E4 + I,
//   E = exp(lrelu(pre)): bgrad = {dpre3, dpre4, dI}; row_coef[src, h] = sum_b dI (per row,
//   batch order) -- the extra gradient sum_j exp(attd_ij) puts on the inter attention;
//   da3s[h, f] = sum_b dpre3 h2_b, da4s likewise.
// mode 1 (after it): d_hs[src_b] += w3 G3 + w4 G4 + dpre3 a3s + dpre4 a4s (per row,
//   batch order).  One workgroup (B is a mini-batch, train.py:33, 64 flows): the dots
//   and the sums over b run a wave per output with lanes across f / b and a fixed xor
//   tree; the batch sources sit in LDS for the repeated-source scans.
constexpr int kFinishLds = 2048;
constexpr int kFinishKB = 8;  // items per wave whose loads are issued together
constexpr int kFinishBg = 4096;  // floats of bgrad staged in LDS between the mode-0 phases

// Mode 1's blocks from nwork on run the bipartite backward's block-partial reduce of d_hc /
// d_er (handed over by msha_bip_defer_reduce; bip_reduce.h; independent of d_hs): one
// launch instead of two.
template <typename T>
__global__ void __launch_bounds__(1024) ours_bwd_finish_kernel(
    OursArgs a, int mode, const float* __restrict__ bstat, const float* __restrict__ G,
    float* __restrict__ bgrad, float* __restrict__ row_coef, float* __restrict__ da3s,
    float* __restrict__ da4s, T* __restrict__ d_hs, BipReduce rd, int nwork) {
  if ((int)blockIdx.x >= nwork) {
    __shared__ float red[64][17];
    bip_reduce_block<T, 1024>(rd, (int)blockIdx.x - nwork, red);
    return;
  }
  __shared__ int64_t s_src[kFinishLds];
  __shared__ int32_t s_next[kFinishLds];  // next batch entry with the same source, -1 = none
  __shared__ int32_t s_first[kFinishLds];  // first batch entry of its source
  __shared__ float s_bg[kFinishBg];         // mode 0: bgrad between the phases
  const int H = a.H, F = a.F, D = H * F;
  const int64_t B = a.B;
  const bool in_lds = B <= kFinishLds;
  // Mode 0 is one workgroup walking a chain of dependent phases; the loads that depend on
  // no phase are issued here, so their latencies (the group-size lookups are two deep)
  // overlap the batch-source staging instead of adding to the chain: the scalar chain's
  // per-(b, h) statistics and group sizes (a thread per item), and the h2 values of the
  // da3s / da4s sums (a wave per output, a lane per batch entry).
  const int nwv = (int)blockDim.x >> 6, lid = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const bool pre2 = mode == 0 && B * H <= (int64_t)blockDim.x;
  const bool pre4 = mode == 0 && B <= 64 && D <= nwv * kFinishKB;
  float pS = 0.f, pE3 = 0.f, pE4 = 0.f, pP3 = 0.f, pP4 = 0.f, pc3 = 0.f, pc4 = 0.f;
  if (pre2 && threadIdx.x < B * H) {
    const int64_t b = threadIdx.x / H;
    const int64_t i = a.src[b];
    const float* st = bstat + (int64_t)threadIdx.x * BS_N;
    pS = st[BS_SUM];
    pE3 = st[BS_E3];
    pE4 = st[BS_E4];
    pP3 = st[BS_PRE3];
    pP4 = st[BS_PRE4];
    const int32_t g3 = a.gid3[i], g4 = a.gid4[i];
    pc3 = (float)(a.gptr3[g3 + 1] - a.gptr3[g3]);
    pc4 = (float)(a.gptr4[g4 + 1] - a.gptr4[g4]);
  }
  float px[kFinishKB];
#pragma unroll
  for (int k = 0; k < kFinishKB; ++k) px[k] = 0.f;
  if (pre4 && lid < B) {
    const int64_t ib = a.src[lid];
#pragma unroll
    for (int k = 0; k < kFinishKB; ++k) {
      const int t = wid + k * nwv;
      if (t < D) px[k] = ldt<T>(a.h2, ib * D + t);
    }
  }
  const bool bg_lds = mode == 0 && B * H * 4 <= kFinishBg;
  float* const bg = bg_lds ? s_bg : bgrad;
  if (in_lds)
    for (int64_t t = threadIdx.x; t < B; t += blockDim.x) {
      s_src[t] = a.src[t];
      s_first[t] = 1;
      s_next[t] = INT32_MAX;
    }
  __syncthreads();
  if (in_lds) {
    // every (b, q) pair of the batch at once (one LDS min per match), instead of a
    // serial scan per entry: next = the smallest later entry with b's source
    // (32-bit index math here and below: B <= kFinishLds, B * H < 2^31 (check()); a
    // 64-bit division is a ~100-instruction sequence and these phases are issue-bound)
    const int Bi = (int)B;
    for (int t = threadIdx.x; t < Bi * Bi; t += blockDim.x) {
      const int b = t / Bi, q = t - b * Bi;
      if (q != b && s_src[q] == s_src[b]) {
        if (q < b) s_first[b] = 0;
        else atomicMin(&s_next[b], (int32_t)q);
      }
    }
    __syncthreads();
  }
  auto SRC = [&](int64_t b) { return in_lds ? s_src[b] : a.src[b]; };
  // batch entries of b's source in batch order (b first): the per-row sums below
  auto is_first = [&](int64_t b) {
    if (in_lds) return s_first[b] != 0;
    const int64_t i = a.src[b];
    for (int64_t q = 0; q < b; ++q)
      if (a.src[q] == i) return false;
    return true;
  };
  auto next_same = [&](int64_t q) -> int64_t {
    if (in_lds) return s_next[q] == INT32_MAX ? -1 : s_next[q];
    const int64_t i = a.src[q];
    for (int64_t r = q + 1; r < B; ++r)
      if (a.src[r] == i) return r;
    return -1;
  };
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if (mode == 0) {
    // dots dw3 = G3 . h2_b, dw4 = G4 . h2_b: a wave per (b, h), lanes across f, kFinishKB
    // items' loads in flight together; parked in bgrad[.., 0..1]
    const int64_t nt = B * H;
    for (int64_t t0 = wv; t0 < nt; t0 += (int64_t)nw * kFinishKB) {
      float d3[kFinishKB], d4[kFinishKB];
#pragma unroll
      for (int k = 0; k < kFinishKB; ++k) d3[k] = d4[k] = 0.f;
      for (int f0 = 0; f0 < F; f0 += 64) {
        const int f = f0 + lane;
        float x[kFinishKB], g3[kFinishKB], g4[kFinishKB];
#pragma unroll
        for (int k = 0; k < kFinishKB; ++k) {
          const int64_t t = t0 + (int64_t)k * nw;
          const bool ok = t < nt && f < F;
          const int ti = ok ? (int)t : 0;
          const int64_t b = ti / H;
          const int h = ti - (int)b * H;
          x[k] = ok ? ldt<T>(a.h2, SRC(b) * D + h * F + f) : 0.f;
          g3[k] = ok ? G[(b * 2 + 0) * D + h * F + f] : 0.f;
          g4[k] = ok ? G[(b * 2 + 1) * D + h * F + f] : 0.f;
        }
#pragma unroll
        for (int k = 0; k < kFinishKB; ++k) {
          d3[k] = fmaf(g3[k], x[k], d3[k]);
          d4[k] = fmaf(g4[k], x[k], d4[k]);
        }
      }
#pragma unroll
      for (int k = 0; k < kFinishKB; ++k) {
        const float dw3 = wave_xor_sum<1>(d3[k]);
        const float dw4 = wave_xor_sum<1>(d4[k]);
        const int64_t t = t0 + (int64_t)k * nw;
        if (lane == 0 && t < nt) {
          bg[t * 4 + 0] = dw3;
          bg[t * 4 + 1] = dw4;
        }
      }
    }
    __syncthreads();
    // the scalar chain, a thread per (b, h) (its dependent group-size loads overlap
    // across threads; on one lane per wave they ran one item after another)
    for (int64_t t = threadIdx.x; t < nt; t += blockDim.x) {
      const int64_t b = (int)t / H;
      const int h = (int)t - (int)b * H;
      const float dw3 = bg[t * 4 + 0], dw4 = bg[t * 4 + 1];
      float sum, E3, E4, c3, c4, p3, p4;
      if (pre2) {
        sum = pS, E3 = pE3, E4 = pE4, c3 = pc3, c4 = pc4, p3 = pP3, p4 = pP4;
      } else {
        const int64_t i = SRC(b);
        const float* st = bstat + (b * H + h) * BS_N;
        sum = st[BS_SUM], E3 = st[BS_E3], E4 = st[BS_E4];
        c3 = (float)(a.gptr3[a.gid3[i] + 1] - a.gptr3[a.gid3[i]]);
        c4 = (float)(a.gptr4[a.gid4[i] + 1] - a.gptr4[a.gid4[i]]);
        p3 = st[BS_PRE3], p4 = st[BS_PRE4];
      }
      const float dsum = -(dw3 * E3 + dw4 * E4) / (sum * sum);
      const float dE3 = dw3 / sum + dsum * c3;
      const float dE4 = dw4 / sum + dsum * c4;
      float* o = bg + t * 4;
      o[0] = dE3 * E3 * (p3 > 0.f ? 1.f : a.slope);
      o[1] = dE4 * E4 * (p4 > 0.f ? 1.f : a.slope);
      o[2] = dsum;
      o[3] = 0.f;
    }
    __syncthreads();
    if (bg_lds)  // the (B, H, 4) output, for mode 1
      for (int64_t t = threadIdx.x; t < nt * 4; t += blockDim.x) bgrad[t] = s_bg[t];
    for (int64_t t = threadIdx.x; t < B * H; t += blockDim.x) {
      const int64_t b = (int)t / H;
      const int h = (int)t - (int)b * H;
      if (!is_first(b)) continue;
      float s = 0.f;
      for (int64_t q = b; q >= 0; q = next_same(q)) s += bg[(q * H + h) * 4 + 2];
      row_coef[SRC(b) * H + h] = s;
    }
    // da3s[t] = sum_b dpre3_b h2_b[t] (da4s): a wave per output, lanes across b,
    // kFinishKB outputs' loads in flight together
    for (int64_t t0 = wv; t0 < (int64_t)D; t0 += (int64_t)nw * kFinishKB) {
      float s3[kFinishKB], s4[kFinishKB];
#pragma unroll
      for (int k = 0; k < kFinishKB; ++k) s3[k] = s4[k] = 0.f;
      for (int64_t b = lane; b < B; b += 64) {
        const int64_t ib = SRC(b);
        float x[kFinishKB], w3[kFinishKB], w4[kFinishKB];
#pragma unroll
        for (int k = 0; k < kFinishKB; ++k) {
          const int64_t t = t0 + (int64_t)k * nw;
          const bool ok = t < D;
          const int h = ok ? (int)t / F : 0;
          // (pre4: one pass, t0 = wave, b = lane: the values loaded at entry)
          x[k] = pre4 ? px[k] : ok ? ldt<T>(a.h2, ib * D + t) : 0.f;
          w3[k] = ok ? bg[(b * H + h) * 4 + 0] : 0.f;
          w4[k] = ok ? bg[(b * H + h) * 4 + 1] : 0.f;
        }
#pragma unroll
        for (int k = 0; k < kFinishKB; ++k) {
          s3[k] = fmaf(w3[k], x[k], s3[k]);
          s4[k] = fmaf(w4[k], x[k], s4[k]);
        }
      }
#pragma unroll
      for (int k = 0; k < kFinishKB; ++k) {
        const float r3 = wave_xor_sum<1>(s3[k]);
        const float r4 = wave_xor_sum<1>(s4[k]);
        const int64_t t = t0 + (int64_t)k * nw;
        if (lane == 0 && t < D) {
          da3s[t] = r3;
          da4s[t] = r4;
        }
      }
    }
  } else {
    // mode 1 runs on a grid: block k takes items [k, k + nwork, ...) * blockDim.x
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < B * D;
         t += (int64_t)nwork * blockDim.x) {
      const int64_t b = t / D;
      const int d = (int)(t % D);
      const int h = d / F;
      const int64_t i = SRC(b);
      if (!is_first(b)) continue;
      float s = 0.f;
      for (int64_t q = b; q >= 0; q = next_same(q)) {
        const float* st = bstat + (q * H + h) * BS_N;
        const float* gq = bgrad + (q * H + h) * 4;
        s += st[BS_W3] * G[(q * 2 + 0) * D + d] + st[BS_W4] * G[(q * 2 + 1) * D + d] +
             gq[0] * a.a3s[d] + gq[1] * a.a4s[d];
      }
      d_hs[i * D + d] = from_f32<T>(to_f32(d_hs[i * D + d]) + s);
    }
  }
}

static int check(const msha_graph* g, const msha_groups* grp, int64_t B, const int64_t* src,
                 int32_t heads, int32_t feat) {
  MSHA_ARG_CHECK(g && g->rowptr && g->col && g->n_rows > 0 && g->n_cols > 0,
                 "ours: graph CSR missing");
  MSHA_ARG_CHECK(grp && grp->gid3 && grp->gptr3 && grp->gmem3 && grp->gid4 && grp->gptr4 &&
                     grp->gmem4 && grp->n_nodes == g->n_rows,
                 "ours: group CSR missing or not over the graph's rows");
  MSHA_ARG_CHECK(B >= 0 && (B == 0 || src), "ours: batch missing");
  MSHA_ARG_CHECK(B * (int64_t)heads < INT32_MAX, "ours: batch * heads must be < 2^31");
  MSHA_ARG_CHECK(heads > 0 && feat > 0 && heads * feat <= kMaxD, "ours: heads*feat must be <= 512");
  return MSHA_OK;
}

static int ours_cu_count() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cached[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    cached[dev] = n;
  }
  return cached[dev];
}

static OursArgs make_args(const msha_graph* g, const msha_groups* grp, int64_t B,
                          const int64_t* src, int32_t heads, int32_t feat, const void* h2,
                          const float* a3s, const float* a4s, float slope, float drop_p,
                          uint64_t seed, uint64_t offset, hipStream_t s) {
  OursArgs a;
  a.B = B; a.N = g->n_rows; a.M = g->n_cols; a.H = heads; a.F = feat; a.src = src;
  a.gid3 = grp->gid3; a.gptr3 = grp->gptr3; a.gmem3 = grp->gmem3;
  a.gid4 = grp->gid4; a.gptr4 = grp->gptr4; a.gmem4 = grp->gmem4;
  a.h2 = h2; a.a3s = a3s; a.a4s = a4s; a.slope = slope;
  a.dp = make_dropout(drop_p, seed, offset, s);
  return a;
}

}  // namespace msha

using namespace msha;

// the intra-dropout draw form of ours_fwd_lds_kernel: packed (default; MSHA_OURS_PACK_DRAWS=0
// starts the process with the per-node form), switchable for A/B runs and the bitwise test
static std::atomic<int>& ours_pack_flag() {
  static std::atomic<int> f([] {
    const char* v = getenv("MSHA_OURS_PACK_DRAWS");
    return v == nullptr || atoi(v) != 0 ? 1 : 0;
  }());
  return f;
}

extern "C" int32_t msha_ours_pack_draws(int32_t mode) {
  if (mode < 0) return ours_pack_flag().load();
  return ours_pack_flag().exchange(mode != 0 ? 1 : 0);
}

template <typename T>
static void launch_fwd(const OursArgs& a, const msha_graph* g, int64_t B, const float* el,
                       const float* er, const float* lse, const void* u_inter, float* bstat,
                       void* u_out, hipStream_t s) {
  // the bipartite forward's v reduce, when it was handed over, rides along as extra blocks
  BipReduce rd{};
  const bool fuse = bip_reduce_take(rd, s);
  const int nprep = B > 0 ? (int)grid_for(B, 4) : 0;
  if (fuse && rd.bf16 != (sizeof(T) == 2 ? 1 : 0)) {  // (not this launch's table type)
    bip_reduce_run(rd, s);
    rd = BipReduce{};
  }
  const int nred = fuse && rd.part != nullptr ? rd.blocks() : 0;
  if (nprep + nred > 0)
    hipLaunchKernelGGL(ours_prep_kernel<T>, dim3(nprep + nred), dim3(256), 0, s, a, g->rowptr,
                       g->col, g->rowflag, el, er, lse, bstat, rd, nprep);
  const int D = a.H * a.F;
  if (B > 0 && B <= 64 && D <= 256) {
    // the batch staged in LDS (ours_fwd_lds_kernel): a persistent grid, four blocks per CU
    // + the dropout path's per-wave pair list (64 x u16) and keep words (64 x uint2, 8-B
    // aligned: see the kernel)
    const size_t lds = (size_t)B * (D + 2 * a.H) * sizeof(float) + 4 +
                       kOursFwdWaves * 64 * (sizeof(uint16_t) + sizeof(uint2));
    const dim3 grid(grid_for(g->n_rows, kOursFwdWaves, 4 * ours_cu_count()));
    const bool pk = a.dp.active && msha_ours_pack_draws(-1) != 0;
#define FWDL(kd)                                                                                 \
  hipLaunchKernelGGL((pk ? ours_fwd_lds_kernel<T, kd, true> : ours_fwd_lds_kernel<T, kd, false>), grid, \
                     dim3(64 * kOursFwdWaves), lds, s, a, (const float*)bstat, (const T*)u_inter,     \
                     (T*)u_out)
    if (D <= 64) FWDL(1);
    else if (D <= 128) FWDL(2);
    else FWDL(4);
#undef FWDL
    return;
  }
  // B <= 64: waves walk ~4 nodes each (the batch's groups load once per wave, the next
  // node's loads overlap this node's gathers); otherwise one node per wave
  const dim3 grid(grid_for(g->n_rows, 4, B <= 64 ? 2048 : 1 << 16));
#define FWD(kd) hipLaunchKernelGGL((ours_fwd_kernel<T, kd>), grid, dim3(256), 0, s, a, \
                                   (const float*)bstat, (const T*)u_inter, (T*)u_out)
  if (D <= 64) FWD(1);
  else if (D <= 128) FWD(2);
  else if (D <= 256) FWD(4);
  else FWD(8);
#undef FWD
}

extern "C" int msha_ours_intra_fwd(const msha_graph* g, const msha_groups* grp, int64_t B,
                                   const int64_t* src, int32_t heads, int32_t feat, int32_t dtype,
                                   const void* h2, const float* a3s, const float* a4s,
                                   const float* el, const float* er, const float* lse,
                                   const void* u_inter, float neg_slope, float drop_p,
                                   uint64_t seed, uint64_t offset, float* bstat, void* u_out,
                                   msha_stream_t stream) {
  if (int rc = check(g, grp, B, src, heads, feat)) return rc;
  MSHA_ARG_CHECK(h2 && a3s && a4s && el && er && lse && u_inter && bstat && u_out,
                 "ours_intra_fwd: null pointer");
  MSHA_ARG_CHECK(dtype == MSHA_DTYPE_F32 || dtype == MSHA_DTYPE_BF16, "ours_intra_fwd: bad dtype");
  hipStream_t s = (hipStream_t)stream;
  const OursArgs a = make_args(g, grp, B, src, heads, feat, h2, a3s, a4s, neg_slope, drop_p,
                               seed, offset, s);
  if (dtype == MSHA_DTYPE_BF16)
    launch_fwd<bf16_t>(a, g, B, el, er, lse, u_inter, bstat, u_out, s);
  else
    launch_fwd<float>(a, g, B, el, er, lse, u_inter, bstat, u_out, s);
  return check_launch("ours_intra_fwd");
}

extern "C" size_t msha_ours_workspace_size(const msha_groups* grp, int64_t B, int32_t heads,
                                           int32_t feat) {
  if (grp == nullptr || B <= 0) return 0;
  const int64_t maxg = grp->max_group > 0 ? grp->max_group : grp->n_nodes;
  const int64_t nck = (maxg + kGatherChunk - 1) / kGatherChunk;
  return (size_t)(2 * B * nck) * (size_t)heads * (size_t)feat * sizeof(float);
}

template <typename T>
static void launch_bwd(const OursArgs& a, int stage, int64_t B, int nck, int heads, int feat,
                       const float* bstat, const void* dU, float* G, float* bgrad,
                       float* row_coef, float* da3s, float* da4s, void* d_hs, float* Gp,
                       hipStream_t s) {
  if (stage == 0) {
    const int D = heads * feat;
    const dim3 grid(grid_for(2 * B * nck, 4));
#define GATHER(kd) hipLaunchKernelGGL((ours_bwd_gather_kernel<T, kd>), grid, dim3(256), 0, s, a, \
                                      (const T*)dU, nck, Gp)
    if (D <= 64) GATHER(1);
    else if (D <= 128) GATHER(2);
    else if (D <= 256) GATHER(4);
    else GATHER(8);
#undef GATHER
    hipLaunchKernelGGL(ours_bwd_gather_reduce_kernel,
                       dim3(grid_for(2 * B * heads * feat, 256, 4096)), dim3(256), 0, s, B,
                       heads * feat, nck, (const float*)Gp, G, row_coef, a.N * heads);
    hipLaunchKernelGGL(ours_bwd_finish_kernel<T>, dim3(1), dim3(1024), 0, s, a, 0, bstat,
                       (const float*)G, bgrad, row_coef, da3s, da4s, (T*)nullptr, BipReduce{}, 1);
  } else {
    // mode 1 (d_hs of the batch rows) is independent per (b, d): one thread per item
    // on a grid (single workgroup: ~20 us, grid: 13 us at B = 64, D = 128)
    // + the bipartite backward's d_hc / d_er reduce, when it was handed over
    BipReduce rd{};
    const bool fuse = bip_reduce_take(rd, s);
    const int nwork = (int)grid_for(B * heads * feat, 1024, 256);
    if (fuse && rd.bf16 != (sizeof(T) == 2 ? 1 : 0)) {  // (not this launch's table type)
      bip_reduce_run(rd, s);
      rd = BipReduce{};
    }
    const int nred = fuse && rd.part != nullptr ? rd.blocks() : 0;
    hipLaunchKernelGGL(ours_bwd_finish_kernel<T>, dim3(nwork + nred), dim3(1024), 0, s, a, 1, bstat,
                       (const float*)G, bgrad, (float*)nullptr, (float*)nullptr,
                       (float*)nullptr, (T*)d_hs, rd, nwork);
  }
}

extern "C" int msha_ours_intra_bwd(const msha_graph* g, const msha_groups* grp, int64_t B,
                                   const int64_t* src, int32_t heads, int32_t feat, int32_t dtype,
                                   const void* h2, const float* a3s, const float* a4s,
                                   const float* bstat, const void* dU, int32_t stage,
                                   float neg_slope, float drop_p, uint64_t seed,
                                   uint64_t offset, float* G, float* bgrad, float* row_coef,
                                   float* da3s, float* da4s, void* d_hs, void* ws,
                                   size_t ws_bytes, msha_stream_t stream) {
  if (int rc = check(g, grp, B, src, heads, feat)) return rc;
  MSHA_ARG_CHECK(stage == 0 || stage == 1, "ours_intra_bwd: stage must be 0 or 1");
  MSHA_ARG_CHECK(dtype == MSHA_DTYPE_F32 || dtype == MSHA_DTYPE_BF16, "ours_intra_bwd: bad dtype");
  MSHA_ARG_CHECK(h2 && a3s && a4s && bstat && G && bgrad, "ours_intra_bwd: null pointer");
  MSHA_ARG_CHECK(stage == 1 || (dU && row_coef && da3s && da4s), "ours_intra_bwd: stage 0 outputs");
  MSHA_ARG_CHECK(stage == 0 || d_hs, "ours_intra_bwd: stage 1 needs d_hs");
  hipStream_t s = (hipStream_t)stream;
  const OursArgs a = make_args(g, grp, B, src, heads, feat, h2, a3s, a4s, neg_slope, drop_p,
                               seed, offset, s);
  if (B == 0) {
    if (stage == 0) {
      if (hipMemsetAsync(da3s, 0, sizeof(float) * heads * feat, s) != hipSuccess ||
          hipMemsetAsync(da4s, 0, sizeof(float) * heads * feat, s) != hipSuccess ||
          hipMemsetAsync(row_coef, 0, sizeof(float) * a.N * heads, s) != hipSuccess)
        return check_launch("ours_intra_bwd memset");
    }
    return MSHA_OK;
  }
  int nck = 0;
  float* Gp = nullptr;
  if (stage == 0) {
    const int maxg = grp->max_group > 0 ? grp->max_group : (int)g->n_rows;
    nck = (maxg + kGatherChunk - 1) / kGatherChunk;
    MSHA_ARG_CHECK(ws && ws_bytes >= msha_ours_workspace_size(grp, B, heads, feat),
                   "ours_intra_bwd: workspace too small");
    Gp = (float*)ws;
  }
  if (dtype == MSHA_DTYPE_BF16)
    launch_bwd<bf16_t>(a, stage, B, nck, heads, feat, bstat, dU, G, bgrad, row_coef, da3s, da4s,
                       d_hs, Gp, s);
  else
    launch_bwd<float>(a, stage, B, nck, heads, feat, bstat, dU, G, bgrad, row_coef, da3s, da4s,
                      d_hs, Gp, s);
  return check_launch("ours_intra_bwd");
}
