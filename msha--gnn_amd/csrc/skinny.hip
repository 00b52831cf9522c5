// Skinny projections of the hot path on the gfx950 matrix cores.
//
// Reference: Ablation.py:262-263 (h1 = R @ W1, h2 = S @ W2), GAT.py:21 (h = x @ W):
// a tall node table (100k+ rows) times a small weight (K, N <= 128), and the weight
// gradient dW = X^T (dh + de (x) a) of the same product, a reduction over all rows.
// The tiled GEMMs of gemm.hip / gemm_bf16.hip re-stage W through LDS for every
// 128-row tile behind two block barriers per k-stage; these kernels keep the skinny
// operand resident instead:
//
//   proj_kernel   W sits in LDS for the whole (persistent) block; each wave streams
//                 16-row tiles of X straight from HBM into MFMA A registers (the next
//                 tile's loads in flight during this tile's MFMAs) and runs with no
//                 block barrier after the W load.  The k order of a lane's A values
//                 is permuted (lane group g takes k = g*K/4 + s at step s) so each lane
//                 reads K/4 contiguous elements of its row with 16-byte loads; W's LDS
//                 image is laid out in the same permuted order.
//   wgrad_kernel  one wave accumulates the whole 128 x 128 dW of its row range in 256
//                 accumulator registers with v_mfma_f32_32x32x2_f32: per two rows a
//                 lane loads one float4 of X and one of dh (+ de (x) a folded in), whose
//                 4 elements feed 4 row (column) blocks, so the operands need no LDS at
//                 all; the 4 row quarters of a block add their tiles pairwise through
//                 LDS and the block writes one partial, reduced over blocks in block
//                 order.
//
// Both are deterministic (fixed summation orders); numerics are the fp32 MFMA's exact
// fma chain (fp32) or fp32 accumulation of bf16 products (bf16).
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "common.h"

namespace msha {
namespace sk {

// ---- per-wave timeline of the skinny kernels (diagnostic build, -DSK_TIMELINE) ---------
// Lane 0 of every wave records into slot (global wave id) of a host-set buffer: word 0 =
// XCC id << 32 | HW_ID (SIMD, CU, SE of the wave), word 1 = kernel tag, then (wall clock
// at 100 MHz, shader clock) pairs at the kernel's marks.  scripts/skinny_timeline.py reads
// them back.  In the shipped build every mark compiles to nothing.
constexpr int kTlStride = 64;  // 64-bit words per wave slot
#ifdef SK_TIMELINE
__device__ uint64_t* g_tl_buf = nullptr;
__device__ int64_t g_tl_slots = 0;
struct Tl {
  uint64_t* p;
  int k;
};
__device__ __forceinline__ void tl_mark(Tl& r) {
  if (r.p != nullptr && (threadIdx.x & 63) == 0 && r.k + 1 < kTlStride) {
    r.p[r.k] = __builtin_amdgcn_s_memrealtime();
    r.p[r.k + 1] = __builtin_amdgcn_s_memtime();
  }
  r.k += 2;
}
__device__ __forceinline__ Tl tl_open(int tag) {
  const int64_t slot = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  Tl r{nullptr, 2};
  if (g_tl_buf != nullptr && slot < g_tl_slots) r.p = g_tl_buf + slot * kTlStride;
  if (r.p != nullptr && (threadIdx.x & 63) == 0) {
    const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_ID
    const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
    r.p[0] = ((uint64_t)xcc << 32) | hw;
    r.p[1] = (uint64_t)tag;
  }
  tl_mark(r);
  return r;
}
#define TL_OPEN(tag) ::msha::sk::Tl tl_ = ::msha::sk::tl_open(tag)
#define TL_MARK() ::msha::sk::tl_mark(tl_)
#else
#define TL_OPEN(tag) \
  do {               \
  } while (0)
#define TL_MARK() \
  do {            \
  } while (0)
#endif

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kProjWaves = 8;  // 2 waves per SIMD

template <typename T, int K, int N>
struct ProjGeo {
  static constexpr bool F32 = sizeof(T) == 4;
  static constexpr int NB = N / 16;                    // 16-column MFMA blocks
  static constexpr int KL = K / 4;                     // k per lane group (g = lane >> 4)
  static constexpr int NLD = KL * (int)sizeof(T) / 16; // 16-B A loads per lane per tile
  static constexpr int S = F32 ? KL : KL / 8;          // MFMA steps per tile
  // W image: fp32 [k'][n] with k' = 4 s + g (pitch N + 16: the 4 groups' rows of a read
  // sit 16 banks apart); bf16 [n][k] (pitch K + 8 elements, one ds_read_b128 per lane)
  static constexpr int PW = F32 ? N + 16 : K + 8;
  static constexpr int WROWS = F32 ? K : N;
  static constexpr int WBYTES = WROWS * PW * (int)sizeof(T);
  static constexpr int TPS = N + 4;                    // fp32 staging pitch of a tile
  static constexpr int SBYTES = 16 * TPS * 4;
  static constexpr int EPL = 16 / (int)sizeof(T);      // output elements per lane store
  static constexpr int LPR = N / EPL;                  // lanes per output row
  static constexpr int RPP = 64 / LPR;                 // rows per store pass
  static_assert(K % 64 == 0 && N % 16 == 0 && N <= 128 && K <= 128, "skinny projection shape");
  static_assert(64 % LPR == 0, "a row must map onto whole lanes");
};

// Fill the fp32 W image [k'][n] (k' = 4 (k % KL) + k / KL, pitch PW) from a row-major
// (N, K) matrix M[n][k] (B[k][n] = M[n][k]).  A lane reads 16 B of one row n (4
// consecutive k) and writes them to 4 image rows: a wave's 64 stores of one element
// index fall in 8 banks (8-way).  One element per lane in M's order (k fastest) put every
// lane of a wave on 2 banks (32-way), ~7 us of LDS time per block at K = N = 128.
// Every piece a thread copies is loaded before the first is written (one HBM round trip
// for the whole fill instead of one per piece).
template <int PIECES, int NT>
struct Pieces {
  static constexpr int IT = (PIECES + NT - 1) / NT;
  static __device__ __forceinline__ bool ok(int idx) { return PIECES % NT == 0 || idx < PIECES; }
  uint4 v[IT];
  // buffer loads (a piece past the end reads 0): unlike plain loads of a __restrict__
  // pointer, the compiler keeps them where they are written, ahead of later loads
  __device__ __forceinline__ void load(const void* src, int tid) {
    const rsrc_t r = make_rsrc(src, PIECES * 16u);
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const u32x4_t x = buf_b128(r, ok(tid + NT * i) ? 16u * (tid + NT * i) : kOOB);
      v[i] = make_uint4(x[0], x[1], x[2], x[3]);
    }
  }
};

template <int K, int N, int NT>
using WPieces = Pieces<K * N / 4, NT>;
template <int K, int N, int NT>
__device__ __forceinline__ void transpose_store(float* Wl, const WPieces<K, N, NT>& p, int tid) {
  using Gm = ProjGeo<float, K, N>;
#pragma unroll
  for (int i = 0; i < p.IT; ++i) {
    const int idx = tid + NT * i;
    if (p.ok(idx)) {
      const int n = idx / (K / 4), k4 = idx % (K / 4);
      const uint4 v = p.v[i];
      const uint32_t e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = 4 * k4 + j;
        Wl[(4 * (k % Gm::KL) + k / Gm::KL) * Gm::PW + n] = __uint_as_float(e[j]);
      }
    }
  }
}
template <int K, int N, int NT>
__device__ __forceinline__ void transpose_fill(float* Wl, const float* __restrict__ M, int tid) {
  WPieces<K, N, NT> p;
  p.load(M, tid);
  transpose_store<K, N, NT>(Wl, p, tid);
}

// Line-major k order (PROJ_LINE=1): slot i of a lane group g holds the row's
// columns [16 i + 4 g, +4) (fp32) / [32 i + 8 g, +8) (bf16), so one 16-byte load per lane
// reads 64 contiguous bytes of each of the tile's 16 rows and slots 2j, 2j + 1 -- reloaded
// together -- complete one 128-byte line.  PROJ_LINE=0: lane group g holds the row's
// g-th K/4 quarter (every slot load touches 4 lines per row, 16 bytes of each, and a
// slot-by-slot reload fetched each line from L2 once per slot).  The fp32 W image rows
// follow the k order; the bf16 image stays [n][k] and only the read offsets move.
// Measured 1-2 % at C4 / bip1m, and it changes the bf16 projection's summation order
// (ablation3's bf16 gradient check sits at its reference-bf16 bar): off by default; the
// fp32 projection runs the split-bf16 form below, whose rows are line-major anyway.
#ifndef PROJ_LINE
#define PROJ_LINE 0
#endif
template <int KL>
__host__ __device__ constexpr int proj_img_row(int k) {  // fp32 image row of column k
  return PROJ_LINE ? 4 * (4 * (k / 16) + k % 4) + (k % 16) / 4 : 4 * (k % KL) + k / KL;
}

struct Split3 {
  bf16x8 h, m, l;
};
__device__ __forceinline__ Split3 split3(const float (&x)[8]) {
  Split3 r;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const bf16_t h = (bf16_t)x[e];
    const float r1 = x[e] - (float)h;
    const bf16_t m = (bf16_t)r1;
    const float r2 = r1 - (float)m;
    r.h[e] = h;
    r.m[e] = m;
    r.l[e] = (bf16_t)r2;
  }
  return r;
}
// fp32 projections on the split-bf16 products (PROJ_X3=1, default; see pair_x3_kernel for
// the error argument): W is held as three bf16 [n][k] images, each k-chunk of 32 runs six
// v_mfma_f32_16x16x32_bf16 per column block instead of eight v_mfma_f32_16x16x4_f32, the
// rows are read line-major (step s of lane group g: columns [32 s + 8 g, +8), two slots
// per step, reloaded right after the step).  PROJ_X3=0: the exact-fp32 MFMA.
#ifndef PROJ_X3
#define PROJ_X3 1
#endif

// proj_kernel's block: PROJ_WPS waves per SIMD when the resident W and one staging
// tile per wave fit the 160 KB of LDS, the staging tile narrowed to column halves when
// the whole-width one would not fit (a head must not straddle the halves), else 2.
// 2, 3 and 4 waves per SIMD measured the same at C4 (42.5 / 43.6 / 46.5 us fp32).
#ifndef PROJ_WPS
#define PROJ_WPS 2
#endif
template <typename T, int K, int N, int FE, bool SPLIT = false>
struct ProjStage {
  using G = ProjGeo<T, K, N>;
  static constexpr int kLds = 160 * 1024;
  static constexpr bool HALF_OK = (FE == 0 || FE <= N / 2) && (N / 2) % (16 / (int)sizeof(T)) == 0 &&
                                  64 % ((N / 2) / (16 / (int)sizeof(T))) == 0;
  // split-bf16 W images (fp32 only, when they fit beside the narrowest staging tiles)
  static constexpr int XPW = K + 8;                     // bf16 image pitch
  static constexpr int XIMG = N * XPW;                  // elements per image
  // the split form runs 3 waves per SIMD (C4 34.2 vs 36.4 us, 1M rows 264 vs 279 us at 2);
  // the exact-fp32 and bf16 forms PROJ_WPS (R15 fp32: 20.5 us at 2, 23.3 at 3)
  static constexpr bool X3 = SPLIT && sizeof(T) == 4 && PROJ_X3 &&
                             3 * XIMG * 2 + 12 * 16 * ((HALF_OK ? N / 2 : N) + 4) * 4 + 8 * N <= kLds;
  static constexpr int WB = X3 ? 3 * XIMG * 2 : G::WBYTES;  // W image bytes
  static constexpr int bytes(int waves, int sw) { return WB + waves * 16 * (sw + 4) * 4 + 8 * N; }
  static constexpr int W3 = 4 * (X3 ? 3 : PROJ_WPS);
  static constexpr bool FULL3 = bytes(W3, N) <= kLds;
  static constexpr bool HALF3 = !FULL3 && HALF_OK && bytes(W3, N / 2) <= kLds;
  static constexpr int WAVES = FULL3 || HALF3 ? W3 : kProjWaves;
  static constexpr int SW = HALF3 ? N / 2 : N;          // staged columns per pass
  static constexpr int TPS = SW + 4;
  static constexpr int SBYTES = 16 * TPS * 4;
  static constexpr int LPR = SW / G::EPL;                // lanes per staged row
  static constexpr int RPP = 64 / LPR;                   // rows per store pass
  // column parts per tail tile: 4, or fewer when a head (FE columns) would straddle them
  // or a part's staged row would cover fewer than 4 lanes
  static constexpr bool part_ok(int pt) { return N / pt >= 4 * G::EPL && (FE == 0 || FE <= N / pt); }
  static constexpr int PT = part_ok(4) ? 4 : part_ok(2) ? 2 : 1;
  static_assert(bytes(WAVES, SW) <= kLds, "proj_kernel LDS");
};

template <typename T, int K, int N, int FE, bool SPLIT>
__global__ void __launch_bounds__((64 * ProjStage<T, K, N, FE, SPLIT>::WAVES)) proj_kernel(
    int M, const T* __restrict__ X, const T* __restrict__ W, const float* __restrict__ al,
    const float* __restrict__ ar, T* __restrict__ h, float* __restrict__ el,
    float* __restrict__ er, int H) {
  using G = ProjGeo<T, K, N>;
  using S = ProjStage<T, K, N, FE, SPLIT>;
  constexpr int kWaves = S::WAVES;
  constexpr bool X3 = S::X3;
  // W image | per-wave staging tiles | score vectors al, ar (read in the epilogue)
  __shared__ __attribute__((aligned(16))) char smem[S::WB + kWaves * S::SBYTES + 8 * N];
  T* Wl = reinterpret_cast<T*>(smem);
  float* als = reinterpret_cast<float*>(smem + S::WB + kWaves * S::SBYTES);
  float* ars = als + N;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar loop control
  const int g = lane >> 4, r16 = lane & 15;
  constexpr uint32_t kSlotB = PROJ_LINE ? 64u : 16u;      // bytes between a lane's slots
  constexpr int kStepK = PROJ_LINE ? 32 : 8;              // bf16 k advance per MFMA step
  static_assert(!PROJ_LINE || G::NLD % 2 == 0, "line-major slots come in pairs");
  // byte offset of slot i from the lane's base (X3: step i / 2's 32 bytes, two halves)
  auto slot_b = [&](int i) -> uint32_t { return X3 ? 128u * (i >> 1) + 16u * (i & 1) : kSlotB * i; };
  TL_OPEN(1);  // marks: entry, W resident, per item (start, MFMAs done), exit

  // Work items of a wave, in order: whole 16-row tiles gw, gw + nw, ... for the R rounds
  // every wave completes, then the tail: the L tiles left over are cut into PT column
  // parts each (PT L items), one per wave in the same SIMD-spreading order, so the last
  // round costs 1 / PT of a tile instead of leaving 1 - L / (SIMDs) of the SIMDs idle.
  // The first pass of waves covers every SIMD once (wave w & 3 of each block) before
  // any SIMD takes a second wave's share.
  const int nblk = gridDim.x;
  const int gw = (w >> 2) * (nblk * 4) + blockIdx.x * 4 + (w & 3);
  const int nw = nblk * kWaves;
  const int tiles = (M + 15) / 16;
  constexpr int PT = S::PT;
  const int R = tiles / nw;
  const int units = PT * (tiles - R * nw);
  const int n_items = R + (gw < units ? (units - gw + nw - 1) / nw : 0);
  // item k -> (tile, first column block)
  auto item_tile = [&](int k) -> int { return k < R ? gw + k * nw : R * nw + (gw + (k - R) * nw) / PT; };
  auto item_cb = [&](int k) -> int { return k < R ? 0 : ((gw + (k - R) * nw) % PT) * (G::NB / PT); };

  // buffer-descriptor loads: a row past M (or an item past the last) reads 0 without a
  // branch, so the prefetch is unconditional and the waits on it stay exact (a load
  // under "if (t + nw < tiles)" made the join wait on the tile just issued)
  const rsrc_t r_x = make_rsrc(X, (uint32_t)((int64_t)M * K * sizeof(T)));
  auto tile_off = [&](int t) -> uint32_t {
    const int row = t * 16 + r16;
    return row < M ? (uint32_t)row * (K * (uint32_t)sizeof(T)) +
                         (uint32_t)(X3 ? 32 * g : PROJ_LINE ? 16 * g : g * G::KL * (int)sizeof(T))
                   : kOOB;
  };
  // ---- W -> LDS once per block.  W's pieces load first, then the first item's rows:
  // the W stores wait for W alone (vmcnt counts in order), so the block barrier is not
  // held by the rows' HBM burst (every wave's first tile at once, ~16 MB at C4), whose
  // latency hides under the W copy and the first steps instead.  (A load -> store loop
  // paid one HBM round trip per W piece: ~4 us of a 40 us launch.)
  Pieces<K * N * (int)sizeof(T) / 16, 64 * kWaves> wp;
  wp.load(W, tid);
  static_assert(N <= 64 * kWaves, "one score-vector element per thread");
  const uint32_t aoff = tid < N ? 4u * tid : kOOB;
  const float alv = FE > 0 ? buf_f32(make_rsrc(al, 4u * N), aoff) : 0.f;
  const float arv = FE > 0 ? buf_f32(make_rsrc(ar, 4u * N), aoff) : 0.f;
  asm volatile("" ::: "memory");  // keep the row loads behind W's
  u32x4_t buf[G::NLD];
  {
    const uint32_t off = n_items > 0 ? tile_off(item_tile(0)) : kOOB;
#pragma unroll
    for (int i = 0; i < G::NLD; ++i) buf[i] = buf_b128(r_x, off + slot_b(i));
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < wp.IT; ++i) {
    const int idx = tid + 64 * kWaves * i;
    if (!wp.ok(idx)) continue;
    if constexpr (X3) {  // W[k][4 n4 .. +3] -> the three bf16 images at [n][k]
      const int k = idx / (N / 4), n4 = idx % (N / 4);
      const uint32_t e4[4] = {wp.v[i].x, wp.v[i].y, wp.v[i].z, wp.v[i].w};
      bf16_t* Wx = reinterpret_cast<bf16_t*>(Wl);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float x = __uint_as_float(e4[j]);
        const bf16_t hb = (bf16_t)x;
        const float r1 = x - (float)hb;
        const bf16_t mb = (bf16_t)r1;
        const int o = (4 * n4 + j) * S::XPW + k;
        Wx[o] = hb;
        Wx[S::XIMG + o] = mb;
        Wx[2 * S::XIMG + o] = (bf16_t)(r1 - (float)mb);
      }
    } else if constexpr (G::F32) {
      const int k = idx / (N / 4), n4 = idx % (N / 4);
      const int kr = proj_img_row<G::KL>(k);
      *reinterpret_cast<uint4*>(reinterpret_cast<float*>(Wl) + kr * G::PW + 4 * n4) = wp.v[i];
    } else {
      const int k = idx / (N / 8), n8 = idx % (N / 8);
      const uint32_t e2[4] = {wp.v[i].x, wp.v[i].y, wp.v[i].z, wp.v[i].w};
      uint16_t* Wt = reinterpret_cast<uint16_t*>(Wl);
#pragma unroll
      for (int e = 0; e < 8; ++e)
        Wt[(8 * n8 + e) * G::PW + k] = (uint16_t)(e2[e >> 1] >> (16 * (e & 1)));
    }
  }
  if (FE > 0 && tid < N) {  // (a null al / ar reads 0: an empty descriptor)
    als[tid] = alv;
    ars[tid] = arv;
  }
  __syncthreads();
  TL_MARK();
  if (n_items == 0) {
    TL_MARK();
    return;
  }

  float* Tw = reinterpret_cast<float*>(smem + S::WB) + w * 16 * S::TPS;
  // A register i of a tile feeds steps [i SPL, (i + 1) SPL): once they have issued, it is
  // reloaded with the next item's (one register buffer, a whole tile of lead time)
  constexpr int SPL = G::S / G::NLD;
  // one item: NBP column blocks from cb0 -- MFMAs over the resident W (B operands of
  // step s + 1 read from LDS while step s's MFMAs issue), then the epilogue.  A column
  // block's accumulation and a head's score dot are the same operations in the same
  // order whichever item holds them, so a part's values are the whole tile's bits.
  // (Running an item's epilogue inside the next item's MFMA steps instead -- two
  // accumulator sets -- raised the MFMA share of the steady state from ~78 % to ~85 %
  // but not the launch: 42.2 vs 40.6 us at C4, the last item's epilogue and the start
  // dominate.  The two waves of a SIMD already overlap one's epilogue with the other's
  // MFMAs.)
  // slot reloads: one slot after its last step (PROJ_LINE=0), or the two slots of a line
  // after the second one's last step
  auto reload = [&](int s, u32x4_t* cur, uint32_t noff) {
    if (!PROJ_LINE) {
      if ((s + 1) % SPL == 0) cur[s / SPL] = buf_b128(r_x, noff + 16u * (s / SPL));
    } else if ((s + 1) % (2 * SPL) == 0) {
      const int i = s / SPL - 1;
      cur[i] = buf_b128(r_x, noff + 64u * i);
      cur[i + 1] = buf_b128(r_x, noff + 64u * (i + 1));
    }
  };
  auto tile = [&](auto nbp_c, int t, int cb0, u32x4_t* cur, uint32_t noff) {
    constexpr int NBP = decltype(nbp_c)::value;
    TL_MARK();
    f32x4 acc[NBP];
#pragma unroll
    for (int c = 0; c < NBP; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (X3) {
      constexpr int XI = S::XIMG;
      const bf16_t* Wb = reinterpret_cast<const bf16_t*>(Wl) + (r16 + cb0 * 16) * S::XPW + 8 * g;
      // the six products of a column block, small terms first
      auto six = [&](f32x4& ac, const Split3& a, const bf16_t* wc) {
        const bf16x8 hb = *reinterpret_cast<const bf16x8*>(wc);
        const bf16x8 mb = *reinterpret_cast<const bf16x8*>(wc + XI);
        const bf16x8 lb = *reinterpret_cast<const bf16x8*>(wc + 2 * XI);
        ac = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.l, hb, ac, 0, 0, 0);
        ac = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, lb, ac, 0, 0, 0);
        ac = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.m, mb, ac, 0, 0, 0);
        ac = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, mb, ac, 0, 0, 0);
        ac = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.m, hb, ac, 0, 0, 0);
        ac = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, hb, ac, 0, 0, 0);
      };
#pragma unroll
      for (int st = 0; st < K / 32; ++st) {
        float x[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          x[e] = __uint_as_float(cur[2 * st][e]);
          x[4 + e] = __uint_as_float(cur[2 * st + 1][e]);
        }
        __builtin_amdgcn_sched_barrier(0);
        cur[2 * st] = buf_b128(r_x, noff + slot_b(2 * st));  // both slots free: next item's
        cur[2 * st + 1] = buf_b128(r_x, noff + slot_b(2 * st + 1));
        __builtin_amdgcn_sched_barrier(0);
        const Split3 a = split3(x);
        const bf16_t* ws = Wb + 32 * st;
        // column blocks in pairs: a block's dependent MFMAs alternate with its partner's
#pragma unroll
        for (int c = 0; c + 1 < NBP; c += 2) {
          const bf16_t* w0 = ws + c * 16 * S::XPW;
          const bf16_t* w1 = w0 + 16 * S::XPW;
          const bf16x8 h0 = *reinterpret_cast<const bf16x8*>(w0);
          const bf16x8 h1 = *reinterpret_cast<const bf16x8*>(w1);
          const bf16x8 m0 = *reinterpret_cast<const bf16x8*>(w0 + XI);
          const bf16x8 m1 = *reinterpret_cast<const bf16x8*>(w1 + XI);
          const bf16x8 l0 = *reinterpret_cast<const bf16x8*>(w0 + 2 * XI);
          const bf16x8 l1 = *reinterpret_cast<const bf16x8*>(w1 + 2 * XI);
          acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.l, h0, acc[c], 0, 0, 0);
          acc[c + 1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.l, h1, acc[c + 1], 0, 0, 0);
          acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, l0, acc[c], 0, 0, 0);
          acc[c + 1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, l1, acc[c + 1], 0, 0, 0);
          acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.m, m0, acc[c], 0, 0, 0);
          acc[c + 1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.m, m1, acc[c + 1], 0, 0, 0);
          acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, m0, acc[c], 0, 0, 0);
          acc[c + 1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, m1, acc[c + 1], 0, 0, 0);
          acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.m, h0, acc[c], 0, 0, 0);
          acc[c + 1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.m, h1, acc[c + 1], 0, 0, 0);
          acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, h0, acc[c], 0, 0, 0);
          acc[c + 1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, h1, acc[c + 1], 0, 0, 0);
        }
        if constexpr (NBP % 2 == 1) six(acc[NBP - 1], a, ws + (NBP - 1) * 16 * S::XPW);
      }
    } else if constexpr (G::F32) {
      const float* Wf = reinterpret_cast<const float*>(Wl) + g * G::PW + r16 + cb0 * 16;
      float bc[NBP], bn[NBP];
#pragma unroll
      for (int c = 0; c < NBP; ++c) bc[c] = Wf[c * 16];
#pragma unroll
      for (int s = 0; s < G::S; ++s) {
        if (s + 1 < G::S) {
#pragma unroll
          for (int c = 0; c < NBP; ++c) bn[c] = Wf[4 * (s + 1) * G::PW + c * 16];
        }
        // keep step s + 1's LDS reads ahead of step s's MFMAs (the scheduler would
        // otherwise sink each read to just before its MFMA and wait on it there)
        __builtin_amdgcn_sched_barrier(0);
        const float a = __uint_as_float(cur[s >> 2][s & 3]);
#pragma unroll
        for (int c = 0; c < NBP; ++c)
          acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bc[c], acc[c], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        reload(s, cur, noff);
#pragma unroll
        for (int c = 0; c < NBP; ++c) bc[c] = bn[c];
      }
    } else {
      const bf16_t* Wb = reinterpret_cast<const bf16_t*>(Wl) + (r16 + cb0 * 16) * G::PW +
                         (PROJ_LINE ? 8 * g : g * G::KL);
      bf16x8 bc[NBP], bn[NBP];
#pragma unroll
      for (int c = 0; c < NBP; ++c) bc[c] = *reinterpret_cast<const bf16x8*>(Wb + c * 16 * G::PW);
#pragma unroll
      for (int s = 0; s < G::S; ++s) {
        if (s + 1 < G::S) {
#pragma unroll
          for (int c = 0; c < NBP; ++c)
            bn[c] = *reinterpret_cast<const bf16x8*>(Wb + c * 16 * G::PW + kStepK * (s + 1));
        }
        __builtin_amdgcn_sched_barrier(0);
        const bf16x8 a = __builtin_bit_cast(bf16x8, cur[s]);
#pragma unroll
        for (int c = 0; c < NBP; ++c)
          acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bc[c], acc[c], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        reload(s, cur, noff);
#pragma unroll
        for (int c = 0; c < NBP; ++c) bc[c] = bn[c];
      }
    }
    TL_MARK();
    // ---- epilogue: stage the 16 x 16 NBP item (MFMA C layout: col = lane & 15, row =
    // 4 (lane >> 4) + reg), SWE columns at a time, then whole-row segments per wave
    // store + score dots
    constexpr int SWE = NBP * 16 < S::SW ? NBP * 16 : S::SW;
    constexpr int LPR = SWE / G::EPL, RPP = 64 / LPR, TPS = SWE + 4;
    static_assert(64 % LPR == 0 && 16 % RPP == 0 && (FE == 0 || SWE % FE == 0), "proj staging");
    const int cl = (lane % LPR) * G::EPL;  // first staged column of this lane
#pragma unroll
    for (int hf = 0; hf < NBP * 16 / SWE; ++hf) {
#pragma unroll
      for (int c = 0; c < SWE / 16; ++c)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          Tw[(4 * g + i) * TPS + c * 16 + r16] = acc[hf * (SWE / 16) + c][i];
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's staging writes landed
      __builtin_amdgcn_wave_barrier();
      const int col = cb0 * 16 + hf * SWE + cl;
#pragma unroll
      for (int pass = 0; pass < 16 / RPP; ++pass) {
        const int rr = pass * RPP + lane / LPR;
        const int row = t * 16 + rr;
        float e[G::EPL];
#pragma unroll
        for (int u = 0; u < G::EPL; u += 4) {
          const float4 v = *reinterpret_cast<const float4*>(Tw + rr * TPS + cl + u);
          e[u] = v.x; e[u + 1] = v.y; e[u + 2] = v.z; e[u + 3] = v.w;
        }
        if (row < M) {
          if constexpr (G::F32) {
            *reinterpret_cast<float4*>(reinterpret_cast<float*>(h) + (int64_t)row * N + col) =
                make_float4(e[0], e[1], e[2], e[3]);
          } else {
            *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(h) + (int64_t)row * N + col) =
                make_uint4(pack_bf16x2(e[0], e[1]), pack_bf16x2(e[2], e[3]),
                           pack_bf16x2(e[4], e[5]), pack_bf16x2(e[6], e[7]));
          }
        }
        if constexpr (FE > 0) {
          // the score dots of the STORED row (bf16 tables: the rounded values) in the
          // order the gather-layout edge kernels recompute er_j = h_j . a_r from a gathered
          // 16-byte piece (pk_dot: last element first, then fma downwards; then the xor
          // tree over the head's pieces below): el / er are the same bits as that
          // recomputation (msha_project_scores_row_order)
          float av[G::EPL], rv[G::EPL], x[G::EPL];
#pragma unroll
          for (int u = 0; u < G::EPL; u += 4) {
            const float4 a4 = *reinterpret_cast<const float4*>(als + col + u);
            const float4 r4 = *reinterpret_cast<const float4*>(ars + col + u);
            av[u] = a4.x; av[u + 1] = a4.y; av[u + 2] = a4.z; av[u + 3] = a4.w;
            rv[u] = r4.x; rv[u + 1] = r4.y; rv[u + 2] = r4.z; rv[u + 3] = r4.w;
          }
#pragma unroll
          for (int j = 0; j < G::EPL; ++j) x[j] = G::F32 ? e[j] : (float)(bf16_t)e[j];
          float sl = x[G::EPL - 1] * av[G::EPL - 1], sr = x[G::EPL - 1] * rv[G::EPL - 1];
#pragma unroll
          for (int j = G::EPL - 2; j >= 0; --j) {
            sl = fmaf(x[j], av[j], sl);
            sr = fmaf(x[j], rv[j], sr);
          }
#pragma unroll
          for (int o = 1; o < FE / G::EPL; o <<= 1) {
            sl += __shfl_xor(sl, o);
            sr += __shfl_xor(sr, o);
          }
          if (col % FE == 0 && row < M) {
            if (el != nullptr) el[(int64_t)row * H + col / FE] = sl;
            if (er != nullptr) er[(int64_t)row * H + col / FE] = sr;
          }
        }
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);  // staging reads done before the next writes
      __builtin_amdgcn_wave_barrier();
    }
  };
  // past the last item the prefetch reads 0 (kOOB)
  auto next_off = [&](int k) -> uint32_t { return k + 1 < n_items ? tile_off(item_tile(k + 1)) : kOOB; };
  for (int k = 0; k < R; ++k)
    tile(std::integral_constant<int, G::NB>{}, item_tile(k), 0, buf, next_off(k));
  for (int k = R; k < n_items; ++k)
    tile(std::integral_constant<int, G::NB / PT>{}, item_tile(k), item_cb(k), buf, next_off(k));
  TL_MARK();
}

// ------------------------------------------------------ pair linear (LLP 'mlp') ---
// out[p, n] = act(sum_k G[gi[p], k] G2[gj[p], k] Wlin[n, k] + b[n]) for the link scorer
// (LLP.py:104-115 with the caller's gather LLP.py:233): the projection's structure with
// the A rows gathered and multiplied (x_i (.) x_j) at the MFMA step, nn.Linear's W
// transposed into the resident LDS image, and the activation epilogue of gemm.hip
// (same bits: bias, ReLU, dropout keyed on p * N + n, sigmoid).  Row indices are
// loaded one tile ahead of the row gathers they address; rows past the batch clamp to
// its last pair (valid addresses, never stored), so the prefetch needs no branch.
enum : int { SK_BIAS = 1, SK_RELU = 2, SK_DROPOUT = 4, SK_SIGMOID = 8 };  // gemm.hip ACT_*

template <int K, int N>
__global__ void __launch_bounds__(64 * kProjWaves) pair_kernel(
    int M, const float* __restrict__ G, int64_t ldg, const int64_t* __restrict__ gi,
    const float* __restrict__ G2, int64_t ldg2, const int64_t* __restrict__ gj,
    const float* __restrict__ Wlin, const float* __restrict__ bias, int act, Dropout dp,
    float* __restrict__ out) {
  using Gm = ProjGeo<float, K, N>;
  __shared__ __attribute__((aligned(16))) char smem[Gm::WBYTES + kProjWaves * Gm::SBYTES];
  float* Wl = reinterpret_cast<float*>(smem);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;

  // ---- B[k][n] = Wlin[n][k] -> the projection's W image [k'][n], k' = 4 (k % KL) + k / KL
  transpose_fill<K, N, 64 * kProjWaves>(Wl, Wlin, tid);
  __syncthreads();

  float* Tw = reinterpret_cast<float*>(smem + Gm::WBYTES) + w * 16 * Gm::TPS;
  const int cl = (lane % Gm::LPR) * Gm::EPL;
  float bv[Gm::EPL];
#pragma unroll
  for (int u = 0; u < Gm::EPL; ++u) bv[u] = (act & SK_BIAS) ? bias[cl + u] : 0.f;
  const uint64_t doff = (act & SK_DROPOUT) ? dropout_offset(dp, dp.offset) : 0;

  const int nblk = gridDim.x;
  const int gw = (w >> 2) * (nblk * 4) + blockIdx.x * 4 + (w & 3);
  const int nw = nblk * kProjWaves;
  const int tiles = (M + 15) / 16;
  if (gw >= tiles) return;

  auto load_idx = [&](int t, int64_t& a, int64_t& b) {
    const int row = min(t * 16 + r16, M - 1);
    a = gi[row];
    b = gj[row];
  };
  auto load_rows = [&](int64_t a, int64_t b, u32x4_t* ri, u32x4_t* rj) {
    const float* pa = G + a * ldg + g * Gm::KL;
    const float* pb = G2 + b * ldg2 + g * Gm::KL;
#pragma unroll
    for (int i = 0; i < Gm::NLD; ++i) {
      ri[i] = *reinterpret_cast<const u32x4_t*>(pa + 4 * i);
      rj[i] = *reinterpret_cast<const u32x4_t*>(pb + 4 * i);
    }
  };
  auto tile = [&](int t, const u32x4_t* ci, const u32x4_t* cj) {
    f32x4 acc[Gm::NB];
#pragma unroll
    for (int c = 0; c < Gm::NB; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
    const float* Wf = Wl + g * Gm::PW + r16;
    float bc[Gm::NB], bn[Gm::NB];
#pragma unroll
    for (int c = 0; c < Gm::NB; ++c) bc[c] = Wf[c * 16];
#pragma unroll
    for (int s = 0; s < Gm::S; ++s) {
      if (s + 1 < Gm::S) {
#pragma unroll
        for (int c = 0; c < Gm::NB; ++c) bn[c] = Wf[4 * (s + 1) * Gm::PW + c * 16];
      }
      __builtin_amdgcn_sched_barrier(0);
      const float a = __uint_as_float(ci[s >> 2][s & 3]) * __uint_as_float(cj[s >> 2][s & 3]);
#pragma unroll
      for (int c = 0; c < Gm::NB; ++c)
        acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bc[c], acc[c], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int c = 0; c < Gm::NB; ++c) bc[c] = bn[c];
    }
#pragma unroll
    for (int c = 0; c < Gm::NB; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i) Tw[(4 * g + i) * Gm::TPS + c * 16 + r16] = acc[c][i];
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int pass = 0; pass < 16 / Gm::RPP; ++pass) {
      const int rr = pass * Gm::RPP + lane / Gm::LPR;
      const int row = t * 16 + rr;
      const float4 v = *reinterpret_cast<const float4*>(Tw + rr * Gm::TPS + cl);
      float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float x = e[u] + bv[u];
        if (act & SK_RELU) x = fmaxf(x, 0.f);
        if (act & SK_DROPOUT)
          x *= philox_x(dp.seed, doff, (uint64_t)row * N + cl + u) >= dp.threshold ? dp.scale
                                                                                   : 0.f;
        if (act & SK_SIGMOID) x = 1.f / (1.f + __expf(-x));
        e[u] = x;
      }
      if (row < M)
        *reinterpret_cast<float4*>(out + (int64_t)row * N + cl) = make_float4(e[0], e[1], e[2], e[3]);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
  };
  u32x4_t ai[Gm::NLD], aj[Gm::NLD], bi[Gm::NLD], bj[Gm::NLD];
  int64_t xa, xb;
  load_idx(gw, xa, xb);
  load_rows(xa, xb, ai, aj);
  load_idx(gw + nw, xa, xb);
  for (int t = gw; t < tiles; t += 2 * nw) {
    load_rows(xa, xb, bi, bj);  // tile t + nw (clamped: valid rows, never stored)
    load_idx(t + 2 * nw, xa, xb);
    __builtin_amdgcn_sched_barrier(0);
    tile(t, ai, aj);
    if (t + nw >= tiles) break;
    load_rows(xa, xb, ai, aj);  // tile t + 2 nw
    load_idx(t + 3 * nw, xa, xb);
    __builtin_amdgcn_sched_barrier(0);
    tile(t + nw, bi, bj);
  }
}

// The fp32 pair scorer with ONE register set of rows (pair_kernel holds two: the tile in
// use and the next one, 128 VGPRs of rows at K = 128, which left it at 2 waves per SIMD
// with a spill).  A lane's row registers ci[i] / cj[i] feed steps [i SPL, (i + 1) SPL);
// once those MFMAs have issued, slot i is reloaded with the NEXT tile's rows, so the next
// tile's gathers are in flight under the rest of this tile (7/8 of a tile of lead for the
// first slot).  The next tile's pair indices are loaded a whole tile earlier still.
//   The waits must stay exact for that lead to exist, which decides the memory ops:
//   - row gathers are buffer loads at 32-bit offsets from the table base (plain 64-bit
//     loads let the register allocator rotate the row registers through copies at the
//     loop latch, each copy waiting on its load);
//   - the epilogue writes the MFMA C layout (row 4 g + i, column 16 c + r16) with
//     buffer stores through a per-tile descriptor that ends at the batch's last row, so
//     rows past it drop without a branch: every tile issues the same count of stores
//     and the compiler's vmcnt at the next tile's first use counts them (a branch
//     around the stores made it assume none and wait for every reload);
//   - no staging tile: the LDS holds W alone, so WPS waves per SIMD fit.
//   - line-major k: slot i of lane group g holds columns [16 i + 4 g, +4), so one load
//     instruction reads 64 contiguous bytes of each of its 16 rows and slots 2j, 2j + 1
//     (reloaded together) cover one 128-byte line.  (pair_kernel's k = g K/4 + s puts a
//     lane group's 16 bytes of a slot in a different line for each g: reloaded a slot at
//     a time, every line came from L2 eight times.)  The W image rows follow the same
//     k order.
// The host picks this kernel when both tables fit a buffer window (msha_pair_linear's
// table_rows: rows x ldg x 4 < 4 GiB); the descriptors end at the tables' ends, so an
// index past them reads zeros instead of faulting.  Same activation bits and dropout
// keys (p * N + n) as pair_kernel; the k order differs, so the sums round differently.
#ifndef PAIR32_WPS
#define PAIR32_WPS 3
#endif
template <int K, int N, int WPS>
__global__ void __launch_bounds__(256 * WPS) pair_roll_kernel(
    int M, const float* __restrict__ G, int64_t ldg, const int64_t* __restrict__ gi,
    const float* __restrict__ G2, int64_t ldg2, const int64_t* __restrict__ gj,
    const float* __restrict__ Wlin, const float* __restrict__ bias, int act, Dropout dp,
    float* __restrict__ out, uint32_t bytes_a, uint32_t bytes_b) {
  using Gm = ProjGeo<float, K, N>;
  constexpr int kWaves = 4 * WPS;
  constexpr int SPL = Gm::S / Gm::NLD;  // MFMA steps fed by one 16-byte row register
  __shared__ __attribute__((aligned(16))) float Wl[Gm::WBYTES / 4];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;

  {  // B[k][n] = Wlin[n][k] -> image row 4 s + g for k = 16 (s / 4) + 4 g + s % 4
    WPieces<K, N, 64 * kWaves> p;
    p.load(Wlin, tid);
#pragma unroll
    for (int i = 0; i < p.IT; ++i) {
      const int idx = tid + 64 * kWaves * i;
      if (p.ok(idx)) {
        const int n = idx / (K / 4), k4 = idx % (K / 4);
        const uint32_t e[4] = {p.v[i].x, p.v[i].y, p.v[i].z, p.v[i].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int k = 4 * k4 + j;
          const int row = 4 * (4 * (k / 16) + k % 4) + (k % 16) / 4;
          Wl[row * Gm::PW + n] = __uint_as_float(e[j]);
        }
      }
    }
  }
  __syncthreads();

  float bv[Gm::NB];
#pragma unroll
  for (int c = 0; c < Gm::NB; ++c) bv[c] = (act & SK_BIAS) ? bias[c * 16 + r16] : 0.f;
  const uint64_t doff = (act & SK_DROPOUT) ? dropout_offset(dp, dp.offset) : 0;

  const int nblk = gridDim.x;
  const int gw = (w >> 2) * (nblk * 4) + blockIdx.x * 4 + (w & 3);
  const int nw = nblk * kWaves;
  const int tiles = (M + 15) / 16;
  if (gw >= tiles) return;

  // the tables (G / G2 are non-null: checked on the host; make_rsrc's null test would put
  // the descriptor in VGPRs and waterfall every load)
  const rsrc_t r_a = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(G), 0, bytes_a, 0x00020000);
  const rsrc_t r_b = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(G2), 0, bytes_b, 0x00020000);
  // rows past the batch (and tiles past the last) clamp to the last pair: valid
  // addresses, never stored, so every reload is unconditional
  auto load_idx = [&](int t, int64_t& a, int64_t& b) {
    const int row = min(t * 16 + r16, M - 1);
    a = gi[row];
    b = gj[row];
  };
  // byte offsets of this lane's first 4 columns of the two rows (< 4 GiB: the host's check).
  // An index outside [0, rows) maps past the window (reads zeros); the test also keeps
  // the index's high word live, so the register allocator does not put the offset into
  // the dead high half of the NEXT index load's destination (a write that would wait on
  // that load: vmcnt(0) at every tile start)
  // (the row counts behind the windows: an index at or past them, or negative, reads
  // zeros instead of wrapping its byte offset past 4 GiB back into the table)
  const uint64_t rows_a = ((uint64_t)bytes_a - 4 * K) / (4 * (uint64_t)ldg) + 1;
  const uint64_t rows_b = ((uint64_t)bytes_b - 4 * K) / (4 * (uint64_t)ldg2) + 1;
  auto offset_a = [&](int64_t a) -> uint32_t {
    return (uint64_t)a >= rows_a ? 0xFFFFFFF0u : (uint32_t)((a * ldg + 4 * g) * 4);
  };
  auto offset_b = [&](int64_t b) -> uint32_t {
    return (uint64_t)b >= rows_b ? 0xFFFFFFF0u : (uint32_t)((b * ldg2 + 4 * g) * 4);
  };
  auto mfma_tile = [&](int t, u32x4_t* ci, u32x4_t* cj, uint32_t na, uint32_t nb) {
    f32x4 acc[Gm::NB];
#pragma unroll
    for (int c = 0; c < Gm::NB; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
    const float* Wf = Wl + g * Gm::PW + r16;
    float bc[Gm::NB], bn[Gm::NB];
#pragma unroll
    for (int c = 0; c < Gm::NB; ++c) bc[c] = Wf[c * 16];
#pragma unroll
    for (int s = 0; s < Gm::S; ++s) {
      if (s + 1 < Gm::S) {
#pragma unroll
        for (int c = 0; c < Gm::NB; ++c) bn[c] = Wf[4 * (s + 1) * Gm::PW + c * 16];
      }
      __builtin_amdgcn_sched_barrier(0);
      const float a = __uint_as_float(ci[s / 4][s % 4]) * __uint_as_float(cj[s / 4][s % 4]);
#pragma unroll
      for (int c = 0; c < Gm::NB; ++c)
        acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bc[c], acc[c], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if ((s + 1) % (2 * SPL) == 0) {  // the two slots of one 128-byte line
        const int i = s / SPL - 1;
        ci[i] = buf_b128(r_a, na + 64u * i);
        ci[i + 1] = buf_b128(r_a, na + 64u * (i + 1));
        cj[i] = buf_b128(r_b, nb + 64u * i);
        cj[i + 1] = buf_b128(r_b, nb + 64u * (i + 1));
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int c = 0; c < Gm::NB; ++c) bc[c] = bn[c];
    }
    // ---- epilogue on the C layout: element (row t 16 + 4 g + i, column 16 c + r16)
    const int rows = min(16, M - t * 16);
    const rsrc_t r_o = make_rsrc(out + (int64_t)t * 16 * N, (uint32_t)(rows * N * 4));
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = t * 16 + 4 * g + i;
#pragma unroll
      for (int c = 0; c < Gm::NB; ++c) {
        float x = acc[c][i] + bv[c];
        if (act & SK_RELU) x = fmaxf(x, 0.f);
        if (act & SK_DROPOUT)
          x *= philox_x(dp.seed, doff, (uint64_t)row * N + c * 16 + r16) >= dp.threshold
                   ? dp.scale
                   : 0.f;
        if (act & SK_SIGMOID) x = 1.f / (1.f + __expf(-x));
        buf_store_f32(r_o, (uint32_t)(((4 * g + i) * N + c * 16 + r16) * 4), x);
      }
    }
  };

  u32x4_t ci[Gm::NLD], cj[Gm::NLD];
  int64_t xa, xb;
  load_idx(gw, xa, xb);
  {
    const uint32_t oa = offset_a(xa), ob = offset_b(xb);
    // in slot order, as the loop reloads them: the wait counts at the loop head merge
    // this path's (a reordered prologue let slot 0 look like one of the last loads and
    // the loop then waited for nearly every reload at each tile start)
#pragma unroll
    for (int i = 0; i < Gm::NLD; i += 2) {
      ci[i] = buf_b128(r_a, oa + 64u * i);
      ci[i + 1] = buf_b128(r_a, oa + 64u * (i + 1));
      cj[i] = buf_b128(r_b, ob + 64u * i);
      cj[i + 1] = buf_b128(r_b, ob + 64u * (i + 1));
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  load_idx(gw + nw, xa, xb);
  for (int t = gw; t < tiles; t += nw) {
    // the next tile's row offsets (its indices were loaded one tile ago), then the
    // indices of the tile after it
    const uint32_t oa = offset_a(xa), ob = offset_b(xb);
    load_idx(t + 2 * nw, xa, xb);
    __builtin_amdgcn_sched_barrier(0);
    mfma_tile(t, ci, cj, oa, ob);
  }
}

// ------------------------------------------- fp32 pair scorer on split bf16 MFMA ---
// The same resident-W rolling-row structure with the fp32 products computed on the bf16
// matrix pipe (16x the fp32 MFMA rate): every fp32 operand is split into three bf16
// terms, x = x_h + x_m + x_l (x_h = bf16(x), x_m = bf16(x - x_h), x_l = bf16(x - x_h -
// x_m); both subtractions exact in fp32, |x - sum| <= 2^-27 |x|), and each k-chunk runs
// the six products whose weight reaches fp32's 2^-24: hh, hm, mh, mm, hl, lh (the dropped
// ml, lm, ll are <= 2^-26 |x w| each).  Each bf16 x bf16 product is exact in fp32 and the
// MFMA accumulates in fp32, so a score carries fp32-level error (the same order as the
// exact-fp32 MFMA's; tests/test_gpu_kernels.py holds both kernels to 1e-5 of fp64).
// Cost per 32-wide k-chunk and 16 x 16 block: 6 x 16 cycles on the bf16 pipe against
// 8 x 32 cycles of v_mfma_f32_16x16x4_f32.  The hadamard x_i * x_j is rounded to fp32
// first (the reference's fp32 product), then split.  W is split once into three bf16
// [n][k] images (3 x 34 KB at K = N = 128).  Rows: line-major, step s of lane group g
// reads columns [32 s + 8 g, +8) -- 32 contiguous bytes, a full 128-byte line per row
// per step -- and both of a step's slots are reloaded with the next tile's rows right
// after that step's MFMAs.
#ifndef PAIR_X3_WPS
#define PAIR_X3_WPS 3
#endif
template <int K, int N>
struct X3Geo {
  static constexpr int NB = N / 16;    // 16-column MFMA blocks
  static constexpr int S = K / 32;     // k-chunks (MFMA steps)
  static constexpr int PW = K + 8;     // image pitch (bf16 elements)
  static constexpr int IMG = N * PW;   // elements per image
  static_assert(K % 64 == 0 && N % 32 == 0 && K <= 128 && N <= 128, "x3 pair shape");
};
template <int K, int N, int WPS>
__global__ void __launch_bounds__(256 * WPS) pair_x3_kernel(
    int M, const float* __restrict__ G, int64_t ldg, const int64_t* __restrict__ gi,
    const float* __restrict__ G2, int64_t ldg2, const int64_t* __restrict__ gj,
    const float* __restrict__ Wlin, const float* __restrict__ bias, int act, Dropout dp,
    float* __restrict__ out, uint32_t bytes_a, uint32_t bytes_b) {
  using Gx = X3Geo<K, N>;
  constexpr int kWaves = 4 * WPS;
  __shared__ __attribute__((aligned(16))) bf16_t Wl[3 * Gx::IMG];  // hi | mid | lo
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;

  {  // W (N, K) row-major fp32 -> three bf16 [n][k] images
    WPieces<K, N, 64 * kWaves> p;
    p.load(Wlin, tid);
#pragma unroll
    for (int i = 0; i < p.IT; ++i) {
      const int idx = tid + 64 * kWaves * i;
      if (p.ok(idx)) {
        const int n = idx / (K / 4), k4 = idx % (K / 4);
        const float x[4] = {__uint_as_float(p.v[i].x), __uint_as_float(p.v[i].y),
                            __uint_as_float(p.v[i].z), __uint_as_float(p.v[i].w)};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const bf16_t h = (bf16_t)x[j];
          const float r1 = x[j] - (float)h;
          const bf16_t m = (bf16_t)r1;
          const int o = n * Gx::PW + 4 * k4 + j;
          Wl[o] = h;
          Wl[Gx::IMG + o] = m;
          Wl[2 * Gx::IMG + o] = (bf16_t)(r1 - (float)m);
        }
      }
    }
  }
  __syncthreads();

  float bv[Gx::NB];
#pragma unroll
  for (int c = 0; c < Gx::NB; ++c) bv[c] = (act & SK_BIAS) ? bias[c * 16 + r16] : 0.f;
  const uint64_t doff = (act & SK_DROPOUT) ? dropout_offset(dp, dp.offset) : 0;

  const int nblk = gridDim.x;
  const int gw = (w >> 2) * (nblk * 4) + blockIdx.x * 4 + (w & 3);
  const int nw = nblk * kWaves;
  const int tiles = (M + 15) / 16;
  if (gw >= tiles) return;

  // (G / G2 non-null, host-checked: a null test would put the descriptors in VGPRs)
  const rsrc_t r_a = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(G), 0, bytes_a, 0x00020000);
  const rsrc_t r_b = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(G2), 0, bytes_b, 0x00020000);
  auto load_idx = [&](int t, int64_t& a, int64_t& b) {
    const int row = min(t * 16 + r16, M - 1);
    a = gi[row];
    b = gj[row];
  };
  // this lane's first 8 columns of each row (index outside [0, rows): past the window;
  // the test keeps the index's high word live, see pair_roll_kernel)
  const uint64_t rows_a = ((uint64_t)bytes_a - 4 * K) / (4 * (uint64_t)ldg) + 1;
  const uint64_t rows_b = ((uint64_t)bytes_b - 4 * K) / (4 * (uint64_t)ldg2) + 1;
  auto offset_a = [&](int64_t a) -> uint32_t {
    return (uint64_t)a >= rows_a ? 0xFFFFFFF0u : (uint32_t)((a * ldg + 8 * g) * 4);
  };
  auto offset_b = [&](int64_t b) -> uint32_t {
    return (uint64_t)b >= rows_b ? 0xFFFFFFF0u : (uint32_t)((b * ldg2 + 8 * g) * 4);
  };
  // slot 2 s + j: step s's columns [32 s + 8 g + 4 j, +4) at byte 128 s + 16 j
  auto slot_off = [](int i) -> uint32_t { return 128u * (i >> 1) + 16u * (i & 1); };
  constexpr int NS = 2 * Gx::S;  // 16-byte slots per lane and row
  auto mfma_tile = [&](int t, u32x4_t* ci, u32x4_t* cj, uint32_t na, uint32_t nb) {
    f32x4 acc[Gx::NB];
#pragma unroll
    for (int c = 0; c < Gx::NB; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
    const bf16_t* Wb = Wl + r16 * Gx::PW + 8 * g;
#pragma unroll
    for (int s = 0; s < Gx::S; ++s) {
      float x[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        x[e] = __uint_as_float(ci[2 * s][e]) * __uint_as_float(cj[2 * s][e]);
        x[4 + e] = __uint_as_float(ci[2 * s + 1][e]) * __uint_as_float(cj[2 * s + 1][e]);
      }
      __builtin_amdgcn_sched_barrier(0);
      // both of this step's slots are free: the next tile's rows go out now
      ci[2 * s] = buf_b128(r_a, na + slot_off(2 * s));
      ci[2 * s + 1] = buf_b128(r_a, na + slot_off(2 * s + 1));
      cj[2 * s] = buf_b128(r_b, nb + slot_off(2 * s));
      cj[2 * s + 1] = buf_b128(r_b, nb + slot_off(2 * s + 1));
      __builtin_amdgcn_sched_barrier(0);
      const Split3 a = split3(x);
      // column blocks in pairs (dependent MFMAs two apart); per pair the B terms in the
      // order h (hh, mh, lh), m (hm, mm), l (hl)
#pragma unroll
      for (int c = 0; c < Gx::NB; c += 2) {
        const bf16_t* w0 = Wb + c * 16 * Gx::PW + 32 * s;
        const bf16_t* w1 = w0 + 16 * Gx::PW;
        const bf16x8 h0 = *reinterpret_cast<const bf16x8*>(w0);
        const bf16x8 h1 = *reinterpret_cast<const bf16x8*>(w1);
        const bf16x8 m0 = *reinterpret_cast<const bf16x8*>(w0 + Gx::IMG);
        const bf16x8 m1 = *reinterpret_cast<const bf16x8*>(w1 + Gx::IMG);
        const bf16x8 l0 = *reinterpret_cast<const bf16x8*>(w0 + 2 * Gx::IMG);
        const bf16x8 l1 = *reinterpret_cast<const bf16x8*>(w1 + 2 * Gx::IMG);
        acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.l, h0, acc[c], 0, 0, 0);
        acc[c + 1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.l, h1, acc[c + 1], 0, 0, 0);
        acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, l0, acc[c], 0, 0, 0);
        acc[c + 1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, l1, acc[c + 1], 0, 0, 0);
        acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.m, m0, acc[c], 0, 0, 0);
        acc[c + 1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.m, m1, acc[c + 1], 0, 0, 0);
        acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, m0, acc[c], 0, 0, 0);
        acc[c + 1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, m1, acc[c + 1], 0, 0, 0);
        acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.m, h0, acc[c], 0, 0, 0);
        acc[c + 1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.m, h1, acc[c + 1], 0, 0, 0);
        acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, h0, acc[c], 0, 0, 0);
        acc[c + 1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, h1, acc[c + 1], 0, 0, 0);
      }
    }
    // ---- epilogue on the C layout: element (row t 16 + 4 g + i, column 16 c + r16)
    const int rows = min(16, M - t * 16);
    const rsrc_t r_o = make_rsrc(out + (int64_t)t * 16 * N, (uint32_t)(rows * N * 4));
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = t * 16 + 4 * g + i;
#pragma unroll
      for (int c = 0; c < Gx::NB; ++c) {
        float x = acc[c][i] + bv[c];
        if (act & SK_RELU) x = fmaxf(x, 0.f);
        if (act & SK_DROPOUT)
          x *= philox_x(dp.seed, doff, (uint64_t)row * N + c * 16 + r16) >= dp.threshold
                   ? dp.scale
                   : 0.f;
        if (act & SK_SIGMOID) x = 1.f / (1.f + __expf(-x));
        buf_store_f32(r_o, (uint32_t)(((4 * g + i) * N + c * 16 + r16) * 4), x);
      }
    }
  };

  u32x4_t ci[NS], cj[NS];
  int64_t xa, xb;
  load_idx(gw, xa, xb);
  {
    const uint32_t oa = offset_a(xa), ob = offset_b(xb);
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      ci[i] = buf_b128(r_a, oa + slot_off(i));
      cj[i] = buf_b128(r_b, ob + slot_off(i));
      if (i & 1) __builtin_amdgcn_sched_barrier(0);
    }
  }
  load_idx(gw + nw, xa, xb);
  for (int t = gw; t < tiles; t += nw) {
    const uint32_t oa = offset_a(xa), ob = offset_b(xb);
    load_idx(t + 2 * nw, xa, xb);
    __builtin_amdgcn_sched_barrier(0);
    mfma_tile(t, ci, cj, oa, ob);
  }
}

// bf16 tables (config C5): the same structure on v_mfma_f32_16x16x32_bf16.  The hadamard
// is rounded to bf16 before the MFMA, as a bf16 x_i * x_j is in PyTorch (and as the
// tiled bf16 GEMM's gather-hadamard loader does); nn.Linear's (N, K) weight is already
// the [n][k] image the bf16 B operand reads.  Scores out in fp32 or bf16 (OB).
// 3 waves per SIMD: 588 -> 540 us per 4M pairs (gather-bound: more loads in flight); a
// one-register-set rolling reload measured slower (576 us at 3, 631 at 2 waves per SIMD)
#ifndef PAIR_WPS
#define PAIR_WPS 3
#endif
constexpr int kPairWaves = 4 * PAIR_WPS;  // pair_bf16_kernel block (waves per SIMD x 4)
template <int K, int N, bool OB>
__global__ void __launch_bounds__(64 * kPairWaves) pair_bf16_kernel(
    int M, const bf16_t* __restrict__ G, int64_t ldg, const int64_t* __restrict__ gi,
    const bf16_t* __restrict__ G2, int64_t ldg2, const int64_t* __restrict__ gj,
    const bf16_t* __restrict__ Wlin, const float* __restrict__ bias, int act, Dropout dp,
    void* __restrict__ out) {
  using Gm = ProjGeo<bf16_t, K, N>;
  __shared__ __attribute__((aligned(16))) char smem[Gm::WBYTES + kPairWaves * Gm::SBYTES];
  bf16_t* Wl = reinterpret_cast<bf16_t*>(smem);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;

  // (a batched fill, as proj_kernel's, spills here at 3 waves per SIMD)
  for (int idx = tid; idx < N * K / 8; idx += 64 * kPairWaves) {
    const int n = idx / (K / 8), k8 = idx % (K / 8);
    *reinterpret_cast<uint4*>(Wl + n * Gm::PW + 8 * k8) =
        *reinterpret_cast<const uint4*>(Wlin + (int64_t)n * K + 8 * k8);
  }
  __syncthreads();

  float* Tw = reinterpret_cast<float*>(smem + Gm::WBYTES) + w * 16 * Gm::TPS;
  const int cl = (lane % Gm::LPR) * Gm::EPL;
  float bv[Gm::EPL];
#pragma unroll
  for (int u = 0; u < Gm::EPL; ++u) bv[u] = (act & SK_BIAS) ? bias[cl + u] : 0.f;
  const uint64_t doff = (act & SK_DROPOUT) ? dropout_offset(dp, dp.offset) : 0;

  const int nblk = gridDim.x;
  const int gw = (w >> 2) * (nblk * 4) + blockIdx.x * 4 + (w & 3);
  const int nw = nblk * kPairWaves;
  const int tiles = (M + 15) / 16;
  if (gw >= tiles) return;

  auto load_idx = [&](int t, int64_t& a, int64_t& b) {
    const int row = min(t * 16 + r16, M - 1);
    a = gi[row];
    b = gj[row];
  };
  auto load_rows = [&](int64_t a, int64_t b, u32x4_t* ri, u32x4_t* rj) {
    const bf16_t* pa = G + a * ldg + g * Gm::KL;
    const bf16_t* pb = G2 + b * ldg2 + g * Gm::KL;
#pragma unroll
    for (int i = 0; i < Gm::NLD; ++i) {
      ri[i] = *reinterpret_cast<const u32x4_t*>(pa + 8 * i);
      rj[i] = *reinterpret_cast<const u32x4_t*>(pb + 8 * i);
    }
  };
  auto tile = [&](int t, const u32x4_t* ci, const u32x4_t* cj) {
    f32x4 acc[Gm::NB];
#pragma unroll
    for (int c = 0; c < Gm::NB; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
    const bf16_t* Wb = Wl + r16 * Gm::PW + g * Gm::KL;
#pragma unroll
    for (int s = 0; s < Gm::S; ++s) {
      bf16x8 bc[Gm::NB];
#pragma unroll
      for (int c = 0; c < Gm::NB; ++c)
        bc[c] = *reinterpret_cast<const bf16x8*>(Wb + c * 16 * Gm::PW + 8 * s);
      // x_i (.) x_j rounded to bf16
      const Pk<bf16_t> xa = pk_from_raw(ci[s], (bf16_t*)nullptr);
      const Pk<bf16_t> xb = pk_from_raw(cj[s], (bf16_t*)nullptr);
      bf16x8 a;
#pragma unroll
      for (int e = 0; e < 8; ++e) a[e] = (bf16_t)(xa.v[e] * xb.v[e]);
#pragma unroll
      for (int c = 0; c < Gm::NB; ++c)
        acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bc[c], acc[c], 0, 0, 0);
    }
#pragma unroll
    for (int c = 0; c < Gm::NB; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i) Tw[(4 * g + i) * Gm::TPS + c * 16 + r16] = acc[c][i];
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int pass = 0; pass < 16 / Gm::RPP; ++pass) {
      const int rr = pass * Gm::RPP + lane / Gm::LPR;
      const int row = t * 16 + rr;
      float e[Gm::EPL];
#pragma unroll
      for (int u = 0; u < Gm::EPL; u += 4) {
        const float4 v = *reinterpret_cast<const float4*>(Tw + rr * Gm::TPS + cl + u);
        e[u] = v.x; e[u + 1] = v.y; e[u + 2] = v.z; e[u + 3] = v.w;
      }
#pragma unroll
      for (int u = 0; u < Gm::EPL; ++u) {
        float x = e[u] + bv[u];
        if (act & SK_RELU) x = fmaxf(x, 0.f);
        if (act & SK_DROPOUT)
          x *= philox_x(dp.seed, doff, (uint64_t)row * N + cl + u) >= dp.threshold ? dp.scale
                                                                                   : 0.f;
        if (act & SK_SIGMOID) x = 1.f / (1.f + __expf(-x));
        e[u] = x;
      }
      if (row < M) {
        if constexpr (OB) {
          *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(out) + (int64_t)row * N + cl) =
              make_uint4(pack_bf16x2(e[0], e[1]), pack_bf16x2(e[2], e[3]),
                         pack_bf16x2(e[4], e[5]), pack_bf16x2(e[6], e[7]));
        } else {
          float* o = reinterpret_cast<float*>(out) + (int64_t)row * N + cl;
          *reinterpret_cast<float4*>(o) = make_float4(e[0], e[1], e[2], e[3]);
          *reinterpret_cast<float4*>(o + 4) = make_float4(e[4], e[5], e[6], e[7]);
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
  };
  u32x4_t ai[Gm::NLD], aj[Gm::NLD], bi[Gm::NLD], bj[Gm::NLD];
  int64_t xa, xb;
  load_idx(gw, xa, xb);
  load_rows(xa, xb, ai, aj);
  load_idx(gw + nw, xa, xb);
  for (int t = gw; t < tiles; t += 2 * nw) {
    load_rows(xa, xb, bi, bj);
    load_idx(t + 2 * nw, xa, xb);
    __builtin_amdgcn_sched_barrier(0);
    tile(t, ai, aj);
    if (t + nw >= tiles) break;
    load_rows(xa, xb, ai, aj);
    load_idx(t + 3 * nw, xa, xb);
    __builtin_amdgcn_sched_barrier(0);
    tile(t + nw, bi, bj);
  }
}

// ------------------------------------------------ input gradient of the projection ---
// dX = (dh + d1 (x) a1 [+ d2 (x) a2]) W^T (msha_gemm_f32_head_outer, operand 0; the
// backward of Ablation.py:262 / Ours.py:58 for the source table): the projection's
// structure with W^T resident (W (N, K) row-major transposed at the fill, as pair_kernel
// does with nn.Linear's weight) and the head-outer term folded into the A operand at the
// MFMA step, in the tiled kernel's fma order fma(d2, a2, fma(d1, a1, x)).  a1 / a2 sit in
// LDS; a lane's KL contiguous columns span at most two heads (hF >= KL / 2), whose d1 /
// d2 values load with the tile.  Tiles, prefetch and epilogue as proj_kernel.
template <int K, int N>
__global__ void __launch_bounds__(64 * kProjWaves) dx_kernel(
    int M, const float* __restrict__ Dh, const float* __restrict__ Wt,
    const float* __restrict__ d1, const float* __restrict__ a1, const float* __restrict__ d2,
    const float* __restrict__ a2, int hH, int hF, float* __restrict__ out) {
  using Gm = ProjGeo<float, K, N>;
  __shared__ __attribute__((aligned(16))) char smem[Gm::WBYTES + kProjWaves * Gm::SBYTES + 8 * K];
  float* Wl = reinterpret_cast<float*>(smem);
  float* a1s = reinterpret_cast<float*>(smem + Gm::WBYTES + kProjWaves * Gm::SBYTES);
  float* a2s = a1s + K;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;

  // B[k][n] = W[n][k] -> the projection's W image [k'][n], k' = 4 (k % KL) + k / KL.
  // W's pieces (and a1, a2) load before the first item's rows, so the block barrier
  // waits for W alone (vmcnt counts in order) while the rows' burst is in flight.
  WPieces<K, N, 64 * kProjWaves> wp;
  wp.load(Wt, tid);
  static_assert(K <= 64 * kProjWaves, "one score-vector element per thread");
  const uint32_t aoff = tid < K ? 4u * tid : kOOB;
  const float a1v = buf_f32(make_rsrc(a1, 4u * K), aoff);
  const float a2v = buf_f32(make_rsrc(a2, 4u * K), aoff);  // (a null a2 reads 0)
  asm volatile("" ::: "memory");  // keep the row loads behind W's
  float* Tw = reinterpret_cast<float*>(smem + Gm::WBYTES) + w * 16 * Gm::TPS;
  // items as proj_kernel: R whole-tile rounds, then the leftover tiles in PT column parts
  constexpr int PT = 4;
  const int nblk = gridDim.x;
  const int gw = (w >> 2) * (nblk * 4) + blockIdx.x * 4 + (w & 3);
  const int nw = nblk * kProjWaves;
  const int tiles = (M + 15) / 16;
  const int R = tiles / nw;
  const int units = PT * (tiles - R * nw);
  const int n_items = R + (gw < units ? (units - gw + nw - 1) / nw : 0);
  auto item_tile = [&](int k) -> int { return k < R ? gw + k * nw : R * nw + (gw + (k - R) * nw) / PT; };
  auto item_cb = [&](int k) -> int { return k < R ? 0 : ((gw + (k - R) * nw) % PT) * (Gm::NB / PT); };

  const rsrc_t r_x = make_rsrc(Dh, (uint32_t)((int64_t)M * K * 4));
  const rsrc_t r_d1 = make_rsrc(d1, (uint32_t)((int64_t)M * hH * 4));
  const rsrc_t r_d2 = make_rsrc(d2, d2 != nullptr ? (uint32_t)((int64_t)M * hH * 4) : 0u);
  const int h0 = (g * Gm::KL) / hF;  // first head of this lane's columns
  struct Tile {
    u32x4_t x[Gm::NLD];
    float e1[2], e2[2];
  };
  auto load_tile = [&](int t, Tile& b) {
    const int row = t * 16 + r16;
    const uint32_t off = row < M ? (uint32_t)row * (K * 4u) + (uint32_t)(g * Gm::KL * 4) : kOOB;
#pragma unroll
    for (int i = 0; i < Gm::NLD; ++i) b.x[i] = buf_b128(r_x, off + 16u * i);
    const uint32_t eo = row < M ? (uint32_t)row * (uint32_t)hH * 4u + 4u * h0 : kOOB;
#pragma unroll
    for (int j = 0; j < 2; ++j) {  // a second head only when hF < KL (reads 0 otherwise)
      const uint32_t o = (j == 0 || hF < Gm::KL) ? eo + 4u * j : kOOB;
      b.e1[j] = buf_f32(r_d1, o);
      b.e2[j] = buf_f32(r_d2, o);
    }
  };
  auto tile = [&](auto nbp_c, int t, int cb0, const Tile& cur) {
    constexpr int NBP = decltype(nbp_c)::value;
    f32x4 acc[NBP];
#pragma unroll
    for (int c = 0; c < NBP; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
    const float* Wf = Wl + g * Gm::PW + r16 + cb0 * 16;
    const float* a1l = a1s + g * Gm::KL;
    const float* a2l = a2s + g * Gm::KL;
    float bc[NBP], bn[NBP];
#pragma unroll
    for (int c = 0; c < NBP; ++c) bc[c] = Wf[c * 16];
#pragma unroll
    for (int s = 0; s < Gm::S; ++s) {
      if (s + 1 < Gm::S) {
#pragma unroll
        for (int c = 0; c < NBP; ++c) bn[c] = Wf[4 * (s + 1) * Gm::PW + c * 16];
      }
      const int hi = s >= hF ? 1 : 0;
      const float av1 = a1l[s], av2 = a2l[s];
      __builtin_amdgcn_sched_barrier(0);
      const float x = __uint_as_float(cur.x[s >> 2][s & 3]);
      const float a = fmaf(cur.e2[hi], av2, fmaf(cur.e1[hi], av1, x));
#pragma unroll
      for (int c = 0; c < NBP; ++c)
        acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bc[c], acc[c], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int c = 0; c < NBP; ++c) bc[c] = bn[c];
    }
    constexpr int SWE = NBP * 16, LPR = SWE / 4, RPP = 64 / LPR, TPS = SWE + 4;
    static_assert(64 % LPR == 0 && 16 % RPP == 0, "dx staging");
    const int cl = (lane % LPR) * 4;
#pragma unroll
    for (int c = 0; c < NBP; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i) Tw[(4 * g + i) * TPS + c * 16 + r16] = acc[c][i];
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int pass = 0; pass < 16 / RPP; ++pass) {
      const int rr = pass * RPP + lane / LPR;
      const int row = t * 16 + rr;
      const float4 v = *reinterpret_cast<const float4*>(Tw + rr * TPS + cl);
      if (row < M) *reinterpret_cast<float4*>(out + (int64_t)row * N + cb0 * 16 + cl) = v;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
  };
  // two tile buffers, alternating: item k + 1's loads fly during item k (past the last
  // item they read 0)
  auto run = [&](int k, Tile& cur) {
    if (k < R)
      tile(std::integral_constant<int, Gm::NB>{}, item_tile(k), 0, cur);
    else
      tile(std::integral_constant<int, Gm::NB / PT>{}, item_tile(k), item_cb(k), cur);
  };
  auto next_tile = [&](int k) -> int { return k < n_items ? item_tile(k) : tiles; };
  Tile ta, tb;
  load_tile(next_tile(0), ta);  // (no items: rows past M, reads 0)
  transpose_store<K, N, 64 * kProjWaves>(Wl, wp, tid);
  if (tid < K) {
    a1s[tid] = a1v;
    a2s[tid] = a2v;
  }
  __syncthreads();
  if (n_items == 0) return;
  for (int k = 0; k < n_items; k += 2) {
    load_tile(next_tile(k + 1), tb);
    __builtin_amdgcn_sched_barrier(0);
    run(k, ta);
    if (k + 1 >= n_items) break;
    load_tile(next_tile(k + 2), ta);
    __builtin_amdgcn_sched_barrier(0);
    run(k + 1, tb);
  }
}

// ------------------------------------------------------------- weight gradient ---
// dW[a, n] = sum_r X[r, a] * (D[r, n] + d1[r, n / hF] a1[n] + d2[r, n / hF] a2[n]),
// a, n < 128.  A wave owns one column half nh (64 columns) of dW for a row range:
// 4 x 2 blocks of 32 x 32 (128 accumulator registers, so two waves fit a SIMD).  Lane
// l = (i = l & 31, q = l >> 5) of a two-row step takes row r + q: X[r+q, 4i .. 4i+3]
// -> A of row blocks t = 0..3 (dW row 4i + t), D'[r+q, 64 nh + 2i .. +1] -> B of
// column blocks u = 0..1 (dW column 64 nh + 2i + u).  v_mfma_f32_32x32x2_f32, k = q.
// Block = 8 waves: column half nh = w & 1, row quarter w >> 1 of the block's rows.
// CS (the projection's score-vector gradients, Ablation.py:266-267 backward): the same
// rows also give dal[n] = sum_r d1[r, n / hF] hs[r, n] (and dar with d2) -- one 8-byte
// load of the forward's h per lane and row next to D's, 4 fmas -- written as per-block
// partials part[which][n][block] for head_colsum_reduce_kernel (gemm.hip), instead of a
// second pass over h (msha_head_colsum).
constexpr int kWgWaves = 8;
#ifndef WG_PD
#define WG_PD 2
#endif
constexpr int kWgPD = WG_PD;  // two-row steps per load batch (two batches in flight)
constexpr int kWgPitch = 132;
constexpr int kWgImage = 128 * kWgPitch;  // floats of one 128 x 128 LDS tile image

template <bool HO, bool CS>
__global__ void __launch_bounds__(64 * kWgWaves) __attribute__((amdgpu_waves_per_eu(2, 2)))
wgrad_kernel(int M, const float* __restrict__ X, int64_t ldx, const float* __restrict__ D,
             int64_t ldd, const float* __restrict__ d1, const float* __restrict__ a1,
             const float* __restrict__ d2, const float* __restrict__ a2, int hH, int hF,
             float* __restrict__ slab, const float* __restrict__ hs, float* __restrict__ cpart) {
  static_assert(!CS || HO, "the score-vector gradients need the head terms");
  __shared__ __attribute__((aligned(16))) float red[2 * kWgImage];
  __shared__ float csred[CS ? 4 * 2 * 128 : 1];  // [row quarter][which][column]
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar loop control
  const int nh = w & 1, rq = w >> 1;
  const int i32 = lane & 31, q = lane >> 5;
  const int nq = gridDim.x * (kWgWaves / 2);  // row slices
  const int gs = blockIdx.x * (kWgWaves / 2) + rq;
  const int r0 = __builtin_amdgcn_readfirstlane((int)(((int64_t)gs * M) / nq));
  const int r1 = __builtin_amdgcn_readfirstlane((int)(((int64_t)(gs + 1) * M) / nq));
  const int c0 = 64 * nh + 2 * i32;  // this lane's two dW columns
  const int hh = HO ? c0 / hF : 0;
  TL_OPEN(2);  // marks: entry, row loop start, row loop done, block sum done, exit
  float2 av1 = make_float2(0.f, 0.f), av2 = av1;
  if (HO) {
    av1 = *reinterpret_cast<const float2*>(a1 + c0);
    if (d2 != nullptr) av2 = *reinterpret_cast<const float2*>(a2 + c0);
  }
  f32x16 acc[4][2];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[t][u][v] = 0.f;

  // buffer-descriptor loads (32-bit offsets, rows past r1 read 0): the load batches
  // are branch-free, so their waits stay exact and no 64-bit address math is carried
  const rsrc_t r_x = make_rsrc(X, (uint32_t)((int64_t)M * ldx * 4));
  const rsrc_t r_d = make_rsrc(D, (uint32_t)((int64_t)M * ldd * 4));
  const rsrc_t r_e1 = make_rsrc(HO ? d1 : nullptr, HO ? (uint32_t)((int64_t)M * hH * 4) : 0u);
  const rsrc_t r_e2 = make_rsrc(HO ? d2 : nullptr, HO && d2 ? (uint32_t)((int64_t)M * hH * 4) : 0u);
  const rsrc_t r_h = make_rsrc(CS ? hs : nullptr, CS ? (uint32_t)((int64_t)M * ldd * 4) : 0u);
  float2 cs1 = make_float2(0.f, 0.f), cs2 = cs1;  // CS: this lane's rows' dal, dar terms
  const uint32_t sx = (uint32_t)ldx * 4u, sd = (uint32_t)ldd * 4u, se = (uint32_t)hH * 4u;
  const uint32_t ox = 16u * i32, od = 4u * c0, oe = 4u * hh;
  struct Batch {
    u32x4_t x[kWgPD];
    float d0[kWgPD], d1v[kWgPD];
    float e1[kWgPD], e2[kWgPD];
    float h0[CS ? kWgPD : 1], h1[CS ? kWgPD : 1];
  };
  auto load = [&](int rb, Batch& b) {
#pragma unroll
    for (int p = 0; p < kWgPD; ++p) {
      const int row = rb + 2 * p + q;
      const bool ok = row < r1;
      const uint32_t ur = (uint32_t)row;
      // a masked row's offsets are kOOB (+ small): past every descriptor's range
      const uint32_t m = ok ? 0u : kOOB;
      b.x[p] = buf_b128(r_x, (ur * sx + ox) | m);
      const auto dd = __builtin_amdgcn_raw_buffer_load_b64(r_d, (ur * sd + od) | m, 0, 0);
      b.d0[p] = __uint_as_float(dd[0]);
      b.d1v[p] = __uint_as_float(dd[1]);
      if (HO) {
        b.e1[p] = buf_f32(r_e1, (ur * se + oe) | m);
        b.e2[p] = buf_f32(r_e2, (ur * se + oe) | m);
      }
      if (CS) {  // (h has D's row pitch: the host checks)
        const auto hv = __builtin_amdgcn_raw_buffer_load_b64(r_h, (ur * sd + od) | m, 0, 0);
        b.h0[p] = __uint_as_float(hv[0]);
        b.h1[p] = __uint_as_float(hv[1]);
      }
    }
  };
  auto compute = [&](int rb, const Batch& cb) {
#pragma unroll
    for (int p = 0; p < kWgPD; ++p) {
      float d[2] = {cb.d0[p], cb.d1v[p]};
      if (HO) {
        d[0] = fmaf(cb.e2[p], av2.x, fmaf(cb.e1[p], av1.x, d[0]));
        d[1] = fmaf(cb.e2[p], av2.y, fmaf(cb.e1[p], av1.y, d[1]));
      }
      if (CS) {
        cs1.x = fmaf(cb.e1[p], cb.h0[p], cs1.x);
        cs1.y = fmaf(cb.e1[p], cb.h1[p], cs1.y);
        cs2.x = fmaf(cb.e2[p], cb.h0[p], cs2.x);
        cs2.y = fmaf(cb.e2[p], cb.h1[p], cs2.y);
      }
      const float xa[4] = {__uint_as_float(cb.x[p].x), __uint_as_float(cb.x[p].y),
                           __uint_as_float(cb.x[p].z), __uint_as_float(cb.x[p].w)};
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int u = 0; u < 2; ++u)
          acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x2f32(xa[t], d[u], acc[t][u], 0, 0, 0);
    }
  };
  // double-buffered loads in two named batches (no register copy between them: a
  // "cur = next" copy made the compiler wait for the loads it had just issued): batch
  // B's loads leave before batch A's MFMAs (kWgPD x 8 MFMAs of 64 cycles) and vice
  // versa, and the other wave of the SIMD covers the rest.
  constexpr int R = 2 * kWgPD;
  Batch ba, bb;
  load(r0, ba);
  TL_MARK();
  for (int rb = r0; rb < r1; rb += 2 * R) {
    // sched_barrier: the scheduler may not sink a batch's loads below the other
    // batch's MFMAs (it did, and the loop then waited on loads just issued)
    load(rb + R, bb);  // past r1: masked (reads 0, adds 0)
    __builtin_amdgcn_sched_barrier(0);
    compute(rb, ba);
    __builtin_amdgcn_sched_barrier(0);
    load(rb + 2 * R, ba);
    __builtin_amdgcn_sched_barrier(0);
    compute(rb + R, bb);
    __builtin_amdgcn_sched_barrier(0);
  }
  TL_MARK();
  // ---- block sum, pairwise: quarters 2, 3 park their tiles in LDS images 0, 1; quarters
  // 0, 1 add them in; quarter 1 parks its sum in image 0; quarter 0 adds it and stores
  // the block's partial straight from its accumulators.  Order (q0 + q2) + (q1 + q3).
  // Every read of a tile is issued before its adds (16 in flight): the earlier in-place
  // read-add-write per element serialised one LDS round trip per element (7 us a launch).
  // 32x32 C layout: reg v of lane l is row 8 (v / 4) + 4 (l >> 5) + (v % 4), col l & 31
  auto row_of = [&](int t, int v) { return 4 * (8 * (v >> 2) + 4 * q + (v & 3)) + t; };
  auto park = [&](int img) {
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int v = 0; v < 16; ++v)
        *reinterpret_cast<float2*>(red + img * kWgImage + row_of(t, v) * kWgPitch + c0) =
            make_float2(acc[t][0][v], acc[t][1][v]);
  };
  auto absorb = [&](int img) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      float2 o[16];
#pragma unroll
      for (int v = 0; v < 16; ++v)
        o[v] = *reinterpret_cast<const float2*>(red + img * kWgImage + row_of(t, v) * kWgPitch + c0);
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        acc[t][0][v] += o[v].x;
        acc[t][1][v] += o[v].y;
      }
    }
  };
  if (CS) {  // the two row parities of the lane pair, then the quarters via LDS
    cs1.x += __shfl_xor(cs1.x, 32);
    cs1.y += __shfl_xor(cs1.y, 32);
    cs2.x += __shfl_xor(cs2.x, 32);
    cs2.y += __shfl_xor(cs2.y, 32);
    if (q == 0) {
      *reinterpret_cast<float2*>(csred + (rq * 2 + 0) * 128 + c0) = cs1;
      *reinterpret_cast<float2*>(csred + (rq * 2 + 1) * 128 + c0) = cs2;
    }
  }
  if (rq >= 2) park(rq - 2);
  __syncthreads();
  if (rq < 2) absorb(rq);
  __syncthreads();
  if (rq == 1) park(0);
  __syncthreads();
  TL_MARK();
  if (CS && rq == 0 && q == 0) {  // quarters in order; part[which][n][block]
    const int nb = gridDim.x;
#pragma unroll
    for (int which = 0; which < 2; ++which)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        float v = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) v += csred[(k * 2 + which) * 128 + c0 + u];
        cpart[((int64_t)which * 128 + c0 + u) * nb + blockIdx.x] = v;
      }
  }
  if (rq == 0) {
    absorb(0);
    float* out = slab + (int64_t)blockIdx.x * (128 * 128);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int v = 0; v < 16; ++v)  // a row's 32 lanes write 256 contiguous bytes
        *reinterpret_cast<float2*>(out + row_of(t, v) * 128 + c0) =
            make_float2(acc[t][0][v], acc[t][1][v]);
  }
  TL_MARK();
}

// C[a, n] (= or +=) sum over blocks b of slab[b, a, n], b ascending within each of 32
// interleaved groups, the groups added in a fixed LDS tree.  Block = 32 groups x 8
// float4 columns (128 contiguous bytes per group); grid = 128 * 128 / 32 blocks.  With
// nb <= 256 every load of a thread is in flight at once (one HBM round trip; the
// earlier 16-group layout took two and ran latency-bound at ~5 us).
constexpr int kWrGroups = 32, kWrCols = 8, kWrRB = 8;
template <typename TC>
__global__ void __launch_bounds__(256) wgrad_reduce_kernel(const float* __restrict__ slab, int nb,
                                                           TC* __restrict__ C, int64_t ldc,
                                                           float beta, const float* __restrict__ cpart,
                                                           float* __restrict__ cs1,
                                                           float* __restrict__ cs2) {
  __shared__ float4 part[256];
  if (blockIdx.x >= 128 * 128 / (4 * kWrCols)) {
    // the CS partials of wgrad_kernel (part[which][n][block]): one wave per output, lane
    // l adds blocks l, l + 64, ... in order, then a fixed xor tree (head_colsum_reduce's
    // order)
    const int t = (int)((blockIdx.x - 128 * 128 / (4 * kWrCols)) * 4 + (threadIdx.x >> 6));
    const int lane = threadIdx.x & 63, which = t / 128, d = t % 128;
    float* out = which == 0 ? cs1 : cs2;
    if (t >= 256 || out == nullptr) return;
    const float* src = cpart + ((int64_t)which * 128 + d) * nb;
    float s0 = 0.f, s1 = 0.f;
    int b = lane;
    for (; b + 64 < nb; b += 128) {
      s0 += src[b];
      s1 += src[b + 64];
    }
    if (b < nb) s0 += src[b];
    float v = s0 + s1;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    if (lane == 0) out[d] = v;
    return;
  }
  const int zq = threadIdx.x / kWrCols, cq = threadIdx.x % kWrCols;
  const int f4 = blockIdx.x * kWrCols + cq;  // float4 index in the 128 x 128 tile
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int b0 = zq; b0 < nb; b0 += kWrGroups * kWrRB) {
    float4 v[kWrRB];
#pragma unroll
    for (int j = 0; j < kWrRB; ++j) {
      const int b = b0 + kWrGroups * j;
      v[j] = b < nb ? reinterpret_cast<const float4*>(slab + (int64_t)b * (128 * 128))[f4]
                    : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int j = 0; j < kWrRB; ++j)
      if (b0 + kWrGroups * j < nb) s = make_float4(s.x + v[j].x, s.y + v[j].y, s.z + v[j].z, s.w + v[j].w);
  }
  part[threadIdx.x] = s;
  __syncthreads();
  for (int o = kWrGroups / 2; o >= 1; o >>= 1) {
    if (zq < o) {
      const float4 v = part[threadIdx.x + kWrCols * o];
      float4& d = part[threadIdx.x];
      d = make_float4(d.x + v.x, d.y + v.y, d.z + v.z, d.w + v.w);
    }
    __syncthreads();
  }
  if (zq == 0) {
    const float4 r = part[cq];
    const int a = f4 >> 5, c4 = (f4 & 31) * 4;
    const float e[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      TC* dst = C + a * ldc + c4 + u;
      float v = e[u];
      if (beta != 0.f) v += beta * to_f32(*dst);
      *dst = from_f32<TC>(v);
    }
  }
}


// ------------------------------------------- weight gradient, split-bf16 in registers ---
// The same dW as wgrad_kernel on the bf16 matrix pipe.  Every fp32 operand is split into
// three bf16 terms x = x_h + x_m + x_l (|x - sum| <= 2^-27 |x|) and the six products whose
// weight reaches fp32's 2^-24 (lh, hl, mm, mh, hm, hh, small first) run as
// v_mfma_f32_32x32x16_bf16: 16x the exact-fp32 MFMA's rate, so the six cost 3/8 of one
// exact product.  Unlike wgrad_x3.hip (both operands staged as bf16 LDS images and read
// back with transposed LDS reads, one block of six 18 KB images per CU) no operand is
// transposed: a 16-row step's k index is (row group q = lane >> 5, j < 8), so lane
// (i = lane & 31, q) loads float4 X[r + 8q + j][4i .. 4i + 3] and D[r + 8q + j][4i .. 4i + 3]
// for j < 8, and component t of its eight X float4s IS its A fragment of the 32 x 32 tile
// of dW rows {4i + t}, component u of its D' float4s its B fragment of dW columns {4i + u}.
// One wave per SIMD owns the whole 128 x 128 dW of its row range (16 tiles, 256
// accumulator registers, so X is read once).  X is double-buffered a step ahead; D, e and
// h (CS) are reloaded for the next step as soon as this step's B terms and column sums
// have consumed them, and the B terms (split once per step) wait in LDS, each lane reading
// back its own 16 B, so their registers go to the loads in flight.  The four waves of a
// block add their tiles through four 32-row LDS images per pass ((w0 + w2) + (w1 + w3),
// wgrad_kernel's order) into the same slab / partials.
constexpr int kWsWaves = 4;
constexpr int kWsImg = 32 * kWgPitch;  // floats of one 32-row LDS image of the block sum

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
// two fp32 -> their three packed bf16 terms: v_cvt_pk_bf16_f32 (RNE) + v_pk_add_f32 for the
// exact residuals, 9 instructions a pair
__device__ __forceinline__ uint32_t pk_bf16(f32x2 v) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2));
}
__device__ __forceinline__ f32x2 unpk_bf16(uint32_t b) {
  return f32x2{__uint_as_float(b << 16), __uint_as_float(b & 0xffff0000u)};
}
__device__ __forceinline__ void split3x8(const f32x2 (&v)[4], bf16x8& h, bf16x8& m, bf16x8& l) {
  uint32_t hw[4], mw[4], lw[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    hw[p] = pk_bf16(v[p]);
    const f32x2 r = v[p] - unpk_bf16(hw[p]);
    mw[p] = pk_bf16(r);
    lw[p] = pk_bf16(r - unpk_bf16(mw[p]));
  }
  h = __builtin_bit_cast(bf16x8, make_uint4(hw[0], hw[1], hw[2], hw[3]));
  m = __builtin_bit_cast(bf16x8, make_uint4(mw[0], mw[1], mw[2], mw[3]));
  l = __builtin_bit_cast(bf16x8, make_uint4(lw[0], lw[1], lw[2], lw[3]));
}

template <bool HO, int CSM>
__global__ void __launch_bounds__(64 * kWsWaves) __attribute__((amdgpu_waves_per_eu(1, 1)))
wgrad_s3_kernel(int M, const float* __restrict__ X, int64_t ldx, const float* __restrict__ D,
                int64_t ldd, const float* __restrict__ d1, const float* __restrict__ a1,
                const float* __restrict__ d2, const float* __restrict__ a2, int hH, int hF,
                float* __restrict__ slab, const float* __restrict__ hs, float* __restrict__ cpart) {
  // CSM: the score-vector gradients' column sums -- 0 none; 1 cs[n] = sum_r e[r, n / hF]
  // T[r, n] from a table T (= h); 2 (two heads) G[head][a] = sum_r e[r, head] X[r, a] from
  // the X rows already in registers (dal = G W: wgrad_gw_kernel), so h is never read
  constexpr bool CS = CSM == 1, GS = CSM == 2;
  static_assert(CSM == 0 || HO, "the score-vector gradients need the head terms");
  // the B terms [wave][u][term][lane] (48 KB) during the loop; the block sum's four 32-row
  // images (68 KB) after it
  __shared__ __attribute__((aligned(16))) float red[kWsWaves * kWsImg];
  __shared__ __attribute__((aligned(16))) float csred[CS ? kWsWaves * 2 * 128 : GS ? kWsWaves * 4 * 128 : 4];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i32 = lane & 31, q = lane >> 5;
  const int nq = gridDim.x * kWsWaves;
  const int gs = blockIdx.x * kWsWaves + w;
  const int r0 = __builtin_amdgcn_readfirstlane((int)(((int64_t)gs * M) / nq));
  const int r1 = __builtin_amdgcn_readfirstlane((int)(((int64_t)(gs + 1) * M) / nq));
  const int c4 = 4 * i32;  // this lane's four dW columns (and X columns)
  const int hh = HO ? c4 / hF : 0;
  TL_OPEN(3);  // marks: entry, row loop start, row loop done, block sum done, exit
  float av1[4] = {0.f, 0.f, 0.f, 0.f}, av2[4] = {0.f, 0.f, 0.f, 0.f};
  if (HO) {
    const float4 v1 = *reinterpret_cast<const float4*>(a1 + c4);
    av1[0] = v1.x, av1[1] = v1.y, av1[2] = v1.z, av1[3] = v1.w;
    if (d2 != nullptr) {
      const float4 v2 = *reinterpret_cast<const float4*>(a2 + c4);
      av2[0] = v2.x, av2[1] = v2.y, av2[2] = v2.z, av2[3] = v2.w;
    }
  }
  f32x16 acc[4][4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[t][u][v] = 0.f;
  // descriptors end at the wave's last row: rows past r1 read 0 and add nothing, with no
  // per-lane mask (the offsets are one VGPR per stream + a scalar row term)
  const uint32_t sx = (uint32_t)ldx * 4u, sd = (uint32_t)ldd * 4u, se = (uint32_t)hH * 4u;
  const rsrc_t r_x = make_rsrc(X, (uint32_t)r1 * sx);
  const rsrc_t r_d = make_rsrc(D, (uint32_t)r1 * sd);
  const rsrc_t r_e1 = make_rsrc(HO ? d1 : nullptr, HO ? (uint32_t)r1 * se : 0u);
  const rsrc_t r_e2 = make_rsrc(HO ? d2 : nullptr, HO && d2 ? (uint32_t)r1 * se : 0u);
  const rsrc_t r_h = make_rsrc(CS ? hs : nullptr, CS ? (uint32_t)r1 * sd : 0u);
  const uint32_t vx = 8u * q * sx + 16u * i32, vd = 8u * q * sd + 16u * i32, ve = 8u * q * se + 4u * hh;
  auto roff = [&](int rb, int j, uint32_t stride, uint32_t v) -> uint32_t {
    return v + (uint32_t)(rb + j) * stride;
  };
  u32x4_t xa[8], xb[8], dv[8], hv[CS ? 8 : 1];
  float e1[8], e2[8];             // this lane's head's e of the step's rows
  f32x2 eg1[GS ? 8 : 1], eg2[GS ? 8 : 1];  // GS: both heads' e of the rows
  float g1[GS ? 2 : 1][4], g2[GS ? 2 : 1][4];
  if (GS)
#pragma unroll
    for (int hd = 0; hd < 2; ++hd)
#pragma unroll
      for (int t = 0; t < 4; ++t) g1[hd][t] = g2[hd][t] = 0.f;
  const uint32_t veg = 8u * q * se;
  auto load_x = [&](int rb, u32x4_t(&x)[8]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = buf_b128(r_x, roff(rb, j, sx, vx));
  };
  auto load_d = [&](int rb) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      dv[j] = buf_b128(r_d, roff(rb, j, sd, vd));
      if (GS) {  // (se = 8: both heads of a row in one load)
        const auto a = __builtin_amdgcn_raw_buffer_load_b64(r_e1, roff(rb, j, se, veg), 0, 0);
        const auto b = __builtin_amdgcn_raw_buffer_load_b64(r_e2, roff(rb, j, se, veg), 0, 0);
        eg1[j] = f32x2{__uint_as_float(a[0]), __uint_as_float(a[1])};
        eg2[j] = f32x2{__uint_as_float(b[0]), __uint_as_float(b[1])};
      } else if (HO) {
        e1[j] = buf_f32(r_e1, roff(rb, j, se, ve));
        e2[j] = buf_f32(r_e2, roff(rb, j, se, ve));
      }
      if (CS) hv[j] = buf_b128(r_h, roff(rb, j, sd, vd));
    }
  };
  float cs1[4] = {0.f, 0.f, 0.f, 0.f}, cs2[4] = {0.f, 0.f, 0.f, 0.f};
  // this wave's B terms of the step, [u][term][lane] (16 B each): parked in LDS so their 48
  // registers go to the loads in flight; each lane reads back its own
  bf16x8* bst = reinterpret_cast<bf16x8*>(red) + w * (4 * 3 * 64) + lane;
  auto step = [&](const u32x4_t(&x)[8], int rb_next) {
    if (GS)  // G += e^T X over this step's rows (before load_d replaces e)
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const float xv = __uint_as_float(x[j][t]);
          g1[0][t] = fmaf(eg1[j].x, xv, g1[0][t]);
          g1[1][t] = fmaf(eg1[j].y, xv, g1[1][t]);
          g2[0][t] = fmaf(eg2[j].x, xv, g2[0][t]);
          g2[1][t] = fmaf(eg2[j].y, xv, g2[1][t]);
        }
    if (CS) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float h = __uint_as_float(hv[j][u]);
          cs1[u] = fmaf(e1[j], h, cs1[u]);
          cs2[u] = fmaf(e2[j], h, cs2[u]);
        }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      f32x2 dd[4];
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        f32x2 d = {__uint_as_float(dv[2 * p][u]), __uint_as_float(dv[2 * p + 1][u])};
        if (HO) {
          const f32x2 e1p = GS ? f32x2{hh ? eg1[2 * p].y : eg1[2 * p].x, hh ? eg1[2 * p + 1].y : eg1[2 * p + 1].x}
                               : f32x2{e1[2 * p], e1[2 * p + 1]};
          const f32x2 e2p = GS ? f32x2{hh ? eg2[2 * p].y : eg2[2 * p].x, hh ? eg2[2 * p + 1].y : eg2[2 * p + 1].x}
                               : f32x2{e2[2 * p], e2[2 * p + 1]};
          d = e2p * av2[u] + (e1p * av1[u] + d);  // wgrad_kernel's order, two rows at once
        }
        dd[p] = d;
      }
      bf16x8 th, tm, tl;
      split3x8(dd, th, tm, tl);
      bst[(u * 3 + 0) * 64] = th;
      bst[(u * 3 + 1) * 64] = tm;
      bst[(u * 3 + 2) * 64] = tl;
    }
    __builtin_amdgcn_sched_barrier(0);
    load_d(rb_next);  // the next step's D', e, h: in flight under this step's MFMAs
    __builtin_amdgcn_sched_barrier(0);
    // the next tile's B terms are read from LDS under the current tile's six MFMAs
    bf16x8 bh = bst[0], bm = bst[64], bl = bst[128];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      __builtin_amdgcn_sched_barrier(0);  // one tile row's A terms live at a time
      f32x2 xs[4];
#pragma unroll
      for (int p = 0; p < 4; ++p) xs[p] = f32x2{__uint_as_float(x[2 * p][t]), __uint_as_float(x[2 * p + 1][t])};
      bf16x8 ah, am, al;
      split3x8(xs, ah, am, al);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const bf16x8 ch = bh, cm = bm, cl = bl;
        if (t < 3 || u < 3) {
          const int nu = (u + 1) & 3;
          bh = bst[(nu * 3 + 0) * 64];
          bm = bst[(nu * 3 + 1) * 64];
          bl = bst[(nu * 3 + 2) * 64];
        }
        __builtin_amdgcn_sched_barrier(0);  // the reads leave before these MFMAs
        // one accumulation chain per tile (32x32x16 bf16 issues back to back on one
        // accumulator): lh, hl, mm, mh, hm, hh -- the small products first
        acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, ch, acc[t][u], 0, 0, 0);
        acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, cl, acc[t][u], 0, 0, 0);
        acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, cm, acc[t][u], 0, 0, 0);
        acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, ch, acc[t][u], 0, 0, 0);
        acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, cm, acc[t][u], 0, 0, 0);
        acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, ch, acc[t][u], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  load_x(r0, xa);
  load_d(r0);
  TL_MARK();
  for (int rb = r0; rb < r1; rb += 32) {
    load_x(rb + 16, xb);  // past r1: reads 0
    __builtin_amdgcn_sched_barrier(0);
    step(xa, rb + 16);
    __builtin_amdgcn_sched_barrier(0);
    load_x(rb + 32, xa);
    __builtin_amdgcn_sched_barrier(0);
    step(xb, rb + 32);
    __builtin_amdgcn_sched_barrier(0);
  }
  TL_MARK();
  if (CS) {  // the two row groups of the lane pair, then the waves via LDS
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      cs1[u] += __shfl_xor(cs1[u], 32);
      cs2[u] += __shfl_xor(cs2[u], 32);
    }
    if (q == 0) {
      *reinterpret_cast<float4*>(csred + (w * 2 + 0) * 128 + c4) = make_float4(cs1[0], cs1[1], cs1[2], cs1[3]);
      *reinterpret_cast<float4*>(csred + (w * 2 + 1) * 128 + c4) = make_float4(cs2[0], cs2[1], cs2[2], cs2[3]);
    }
  }
  if (GS) {  // the two row groups of the lane pair, then the waves via LDS: [w][which][head][a]
#pragma unroll
    for (int hd = 0; hd < 2; ++hd)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        g1[hd][t] += __shfl_xor(g1[hd][t], 32);
        g2[hd][t] += __shfl_xor(g2[hd][t], 32);
      }
    if (q == 0)
#pragma unroll
      for (int hd = 0; hd < 2; ++hd) {
        *reinterpret_cast<float4*>(csred + ((w * 2 + 0) * 2 + hd) * 128 + c4) =
            make_float4(g1[hd][0], g1[hd][1], g1[hd][2], g1[hd][3]);
        *reinterpret_cast<float4*>(csred + ((w * 2 + 1) * 2 + hd) * 128 + c4) =
            make_float4(g2[hd][0], g2[hd][1], g2[hd][2], g2[hd][3]);
      }
  }
  // ---- block sum, 32 dW rows a pass: every wave parks its slice in its own image, then
  // all four store (w0 + w2) + (w1 + w3) (wgrad_kernel's order), 512 contiguous bytes a
  // row.  C layout: reg v of lane l is tile row 8 (v / 4) + 4 (l >> 5) + (v % 4), column
  // l & 31 -> dW row 4 m + t (pass v / 4), columns 4 (l & 31) + u
  float* out = slab + (int64_t)blockIdx.x * (128 * 128);
  float* img = red + w * kWsImg;
#pragma unroll
  for (int pass = 0; pass < 4; ++pass) {
    __syncthreads();  // the B slots (pass 0) / the previous pass's images are free
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int vv = 0; vv < 4; ++vv) {
        const int v = 4 * pass + vv;
        const int row = 4 * (4 * q + vv) + t;  // row within the pass's 32
        *reinterpret_cast<float4*>(img + row * kWgPitch + c4) =
            make_float4(acc[t][0][v], acc[t][1][v], acc[t][2][v], acc[t][3][v]);
      }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 32 * 32 / (64 * kWsWaves); ++k) {
      const int f = tid + k * 64 * kWsWaves;
      const int row = f >> 5, col = (f & 31) * 4;
      const float4 x0 = *reinterpret_cast<const float4*>(red + 0 * kWsImg + row * kWgPitch + col);
      const float4 x1 = *reinterpret_cast<const float4*>(red + 1 * kWsImg + row * kWgPitch + col);
      const float4 x2 = *reinterpret_cast<const float4*>(red + 2 * kWsImg + row * kWgPitch + col);
      const float4 x3 = *reinterpret_cast<const float4*>(red + 3 * kWsImg + row * kWgPitch + col);
      // row r of the pass is dW row 4 (8 pass + r / 4 ... ): rows 32 pass .. 32 pass + 31
      *reinterpret_cast<float4*>(out + (32 * pass + row) * 128 + col) =
          make_float4((x0.x + x2.x) + (x1.x + x3.x), (x0.y + x2.y) + (x1.y + x3.y),
                      (x0.z + x2.z) + (x1.z + x3.z), (x0.w + x2.w) + (x1.w + x3.w));
    }
  }
  TL_MARK();
  if (GS && w == 0 && q == 0) {  // waves in order; part[which][head][a][block]
    const int nb = gridDim.x;
#pragma unroll
    for (int wh = 0; wh < 4; ++wh)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        float v = 0.f;
#pragma unroll
        for (int k = 0; k < kWsWaves; ++k) v += csred[(k * 4 + wh) * 128 + c4 + t];
        cpart[((int64_t)wh * 128 + c4 + t) * nb + blockIdx.x] = v;
      }
  }
  if (CS && w == 0 && q == 0) {  // waves in order; part[which][n][block]
    const int nb = gridDim.x;
#pragma unroll
    for (int which = 0; which < 2; ++which)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float v = 0.f;
#pragma unroll
        for (int k = 0; k < kWsWaves; ++k) v += csred[(k * 2 + which) * 128 + c4 + u];
        cpart[((int64_t)which * 128 + c4 + u) * nb + blockIdx.x] = v;
      }
  }
  TL_MARK();
}

// The G-based column sums (wgrad_s3_kernel CSM 2): block (which, head) sums its G[a] over
// the row blocks (nb <= 256; a wave per 32 a, lane l takes blocks l, l + 64, .. in order,
// then a fixed xor tree), then
// cs_which[head * hF + f] = sum_a W[a][head * hF + f] G[a]: a wave per 16 a, lanes over f
// (coalesced W rows), the four waves' partials added in wave order.
__global__ void __launch_bounds__(256) wgrad_gw_kernel(const float* __restrict__ cpart, int nb,
                                                       const float* __restrict__ W, int64_t ldw,
                                                       int hF, float* __restrict__ cs1,
                                                       float* __restrict__ cs2) {
  __shared__ float G[128];
  __shared__ float part[4][256];
  const int which = blockIdx.x >> 1, hd = blockIdx.x & 1;
  float* out = which == 0 ? cs1 : cs2;
  if (out == nullptr) return;  // (block-uniform)
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const float* src = cpart + (int64_t)(which * 2 + hd) * 128 * nb;
  {  // wave wv: a in [32 wv, 32 wv + 32); every load in flight at once (nb <= 256)
    float v[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      const float* r = src + (int64_t)(32 * wv + k) * nb;
      float s = 0.f;
#pragma unroll
      for (int c = 0; c < 4; ++c) {  // unconditional loads (clamped), masked adds
        const int b = lane + 64 * c;
        const float x = r[b < nb ? b : nb - 1];
        s += b < nb ? x : 0.f;
      }
      v[k] = s;
    }
#pragma unroll
    for (int k = 0; k < 32; ++k) {
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) v[k] += __shfl_xor(v[k], o);
      if (lane == 0) G[32 * wv + k] = v[k];
    }
  }
  __syncthreads();
  for (int f0 = 0; f0 < hF; f0 += 256) {
    for (int f = f0 + lane; f < f0 + 256 && f < hF; f += 64) {
      const int n = hd * hF + f;
      float v = 0.f;
#pragma unroll 8
      for (int a = 32 * wv; a < 32 * wv + 32; ++a) v = fmaf(W[(int64_t)a * ldw + n], G[a], v);
      part[wv][f - f0] = v;
    }
    __syncthreads();
    for (int f = f0 + (int)threadIdx.x; f < f0 + 256 && f < hF; f += 256)
      out[hd * hF + f] = ((part[0][f - f0] + part[1][f - f0]) + part[2][f - f0]) + part[3][f - f0];
    __syncthreads();
  }
}

}  // namespace sk

// ------------------------------------------------------------------ dispatch ---
// Environment knob MSHA_SKINNY=0 routes every call to the tiled GEMMs (A/B runs).
static bool skinny_enabled() {
  static const int on = [] {
    const char* v = getenv("MSHA_SKINNY");
    return v != nullptr && *v ? atoi(v) : 1;
  }();
  return on != 0;
}

static int proj_grid(int64_t M, int waves = sk::kProjWaves) {
  const int64_t tiles = (M + 15) / 16;
  const int64_t blocks = (tiles + waves - 1) / waves;
  return (int)(blocks < 256 ? blocks : 256);  // one 8-wave block per CU
}

// Returns 1 when it launched, 0 when the shape is not covered (caller falls back).
template <typename T>
int skinny_project(int64_t M, int64_t K, int heads, int feat, const void* X, const void* W,
                   const float* al, const float* ar, void* h, float* el, float* er,
                   hipStream_t s) {
  const int64_t N = (int64_t)heads * feat;
  if (!skinny_enabled() || M < 1024 || M * K * (int64_t)sizeof(T) >= (1ll << 31)) return 0;
  if (((uintptr_t)X | (uintptr_t)W | (uintptr_t)h) & 15) return 0;
  const bool score = al != nullptr || ar != nullptr;
  const int minfe = 16 / (int)sizeof(T);
  if (score && (feat < minfe || N % feat != 0)) return 0;
  // fp32: the split-bf16 form from 64k rows (1M rows: 292 vs 368 us, C4's 100k: 36.6 vs
  // 39.4 us); below it the three-image W fill outweighs the faster steps (R15's 39k rows:
  // 24.9 vs 20.8 us), so the exact-fp32 MFMA runs there
  constexpr bool kF32 = std::is_same<T, float>::value;
  const bool split = kF32 && M >= 65536;
#define SKP(k, n, fe)                                                                           \
  if (K == k && N == n && (score ? feat == fe : fe == 0)) {                                    \
    if (split) {                                                                                \
      constexpr int wv = sk::ProjStage<T, k, n, fe, kF32>::WAVES;                               \
      hipLaunchKernelGGL((sk::proj_kernel<T, k, n, fe, kF32>), dim3(proj_grid(M, wv)),         \
                         dim3(64 * wv), 0, s, (int)M, (const T*)X, (const T*)W, al, ar, (T*)h,  \
                         el, er, heads);                                                        \
      return 1;                                                                                 \
    }                                                                                           \
    constexpr int wv = sk::ProjStage<T, k, n, fe, false>::WAVES;                                \
    hipLaunchKernelGGL((sk::proj_kernel<T, k, n, fe, false>), dim3(proj_grid(M, wv)), dim3(64 * wv), \
                       0, s, (int)M, (const T*)X, (const T*)W, al, ar, (T*)h, el, er, heads);   \
    return 1;                                                                                   \
  }
#define SKP_N(k, n) SKP(k, n, 0) SKP(k, n, 16) SKP(k, n, 32) SKP(k, n, 64) SKP(k, n, n)
  SKP_N(128, 128)
  SKP_N(64, 128)
  SKP(128, 64, 0) SKP(128, 64, 16) SKP(128, 64, 32) SKP(128, 64, 64)
  SKP(64, 64, 0) SKP(64, 64, 16) SKP(64, 64, 32) SKP(64, 64, 64)
#undef SKP_N
#undef SKP
  return 0;
}
template int skinny_project<float>(int64_t, int64_t, int, int, const void*, const void*,
                                   const float*, const float*, void*, float*, float*, hipStream_t);
template int skinny_project<bf16_t>(int64_t, int64_t, int, int, const void*, const void*,
                                    const float*, const float*, void*, float*, float*, hipStream_t);

// pair linear on the resident-W kernels: fp32, both gathers given, K and N in {64, 128},
// 16-byte aligned rows; 0 = not covered (the caller runs the tiled GEMM).  Tables with
// known row counts inside a 4 GiB buffer window take pair_roll_kernel.
int skinny_pair_linear(int64_t P, int64_t K, int64_t N, const float* G, int64_t ldg,
                       const int64_t* gi, const float* G2, int64_t ldg2, const int64_t* gj,
                       int64_t g_rows, int64_t g2_rows, const float* W, const float* bias,
                       int act, const Dropout& dp, float* out, hipStream_t s) {
  if (!skinny_enabled() || P < 1024 || P >= (1ll << 31) || gi == nullptr || gj == nullptr) return 0;
  if (G2 == nullptr) { G2 = G; ldg2 = ldg; g2_rows = g_rows; }
  if (ldg % 4 || ldg2 % 4 || (((uintptr_t)G | (uintptr_t)G2 | (uintptr_t)out | (uintptr_t)W) & 15))
    return 0;
  // MSHA_PAIR_ROLL: 2 (default) split-bf16 pair_x3_kernel, 1 the exact-fp32 rolling
  // pair_roll_kernel, 0 always the two-register-set pair_kernel
  static const int roll_env = [] {
    const char* v = getenv("MSHA_PAIR_ROLL");
    return v != nullptr && *v ? atoi(v) : 2;
  }();
  // table bytes up to the last row's K columns (the kernel reads no further)
  auto span = [&](int64_t rows, int64_t ld) -> int64_t { return rows > 0 ? ((rows - 1) * ld + K) * 4 : -1; };
  const int64_t ba = span(g_rows, ldg), bb = span(g2_rows, ldg2);
  const bool roll = roll_env && ba > 0 && bb > 0 && ba <= 0xFFFFFFFFll && bb <= 0xFFFFFFFFll &&
                    P * N * 4 < (1ll << 31);
  const dim3 grid(proj_grid(P)), block(64 * sk::kProjWaves);
  constexpr int rw = 4 * PAIR32_WPS, xw = 4 * PAIR_X3_WPS;
  const dim3 rgrid(proj_grid(P, rw)), rblock(64 * rw);
  const dim3 xgrid(proj_grid(P, xw)), xblock(64 * xw);
#define SKPL(k, n)                                                                              \
  if (K == k && N == n) {                                                                       \
    if (roll && roll_env == 2)                                                                  \
      hipLaunchKernelGGL((sk::pair_x3_kernel<k, n, PAIR_X3_WPS>), xgrid, xblock, 0, s, (int)P,  \
                         G, ldg, gi, G2, ldg2, gj, W, bias, act, dp, out, (uint32_t)ba,         \
                         (uint32_t)bb);                                                         \
    else if (roll)                                                                              \
      hipLaunchKernelGGL((sk::pair_roll_kernel<k, n, PAIR32_WPS>), rgrid, rblock, 0, s, (int)P, \
                         G, ldg, gi, G2, ldg2, gj, W, bias, act, dp, out, (uint32_t)ba,         \
                         (uint32_t)bb);                                                         \
    else                                                                                        \
      hipLaunchKernelGGL((sk::pair_kernel<k, n>), grid, block, 0, s, (int)P, G, ldg, gi, G2,   \
                         ldg2, gj, W, bias, act, dp, out);                                      \
    return 1;                                                                                   \
  }
  SKPL(128, 128) SKPL(64, 128) SKPL(128, 64) SKPL(64, 64)
#undef SKPL
  return 0;
}

int skinny_pair_linear_bf16(int64_t P, int64_t K, int64_t N, const void* G, int64_t ldg,
                            const int64_t* gi, const void* G2, int64_t ldg2, const int64_t* gj,
                            const void* W, const float* bias, int act, const Dropout& dp,
                            void* out, bool out_bf16, hipStream_t s) {
  if (!skinny_enabled() || P < 1024 || P >= (1ll << 31) || gi == nullptr || gj == nullptr) return 0;
  if (G2 == nullptr) { G2 = G; ldg2 = ldg; }
  if (ldg % 8 || ldg2 % 8 || (((uintptr_t)G | (uintptr_t)G2 | (uintptr_t)W | (uintptr_t)out) & 15))
    return 0;
  const dim3 grid(proj_grid(P, sk::kPairWaves)), block(64 * sk::kPairWaves);
#define SKPB(k, n)                                                                              \
  if (K == k && N == n) {                                                                       \
    if (out_bf16)                                                                               \
      hipLaunchKernelGGL((sk::pair_bf16_kernel<k, n, true>), grid, block, 0, s, (int)P,        \
                         (const bf16_t*)G, ldg, gi, (const bf16_t*)G2, ldg2, gj,               \
                         (const bf16_t*)W, bias, act, dp, out);                                 \
    else                                                                                        \
      hipLaunchKernelGGL((sk::pair_bf16_kernel<k, n, false>), grid, block, 0, s, (int)P,       \
                         (const bf16_t*)G, ldg, gi, (const bf16_t*)G2, ldg2, gj,               \
                         (const bf16_t*)W, bias, act, dp, out);                                 \
    return 1;                                                                                   \
  }
  SKPB(128, 128) SKPB(64, 128) SKPB(128, 64) SKPB(64, 64)
#undef SKPB
  return 0;
}

// dX (M x N) = (dh + d1 (x) a1 [+ d2 (x) a2]) W^T with W (N, K) row-major (the
// projection's input gradient): K, N in {64, 128}, hF >= 16 dividing K, C row-major
// (ldc = N); 0 = not covered (the caller runs the tiled head-outer GEMM)
int skinny_dx(int64_t M, int64_t N, int64_t K, const float* Dh, const float* W, float* C,
              int hH, int hF, const float* d1, const float* a1, const float* d2, const float* a2,
              hipStream_t s) {
  if (!skinny_enabled() || M < 1024 || M * K * 4 >= (1ll << 31) || M * hH * 4 >= (1ll << 31))
    return 0;
  if (hF < 16 || K % hF != 0 || (int64_t)hH * hF != K || d1 == nullptr || a1 == nullptr) return 0;
  if (((uintptr_t)Dh | (uintptr_t)C | (uintptr_t)W) & 15) return 0;
  const dim3 grid(proj_grid(M)), block(64 * sk::kProjWaves);
#define SKDX(k, n)                                                                              \
  if (K == k && N == n) {                                                                       \
    hipLaunchKernelGGL((sk::dx_kernel<k, n>), grid, block, 0, s, (int)M, Dh, W, d1, a1, d2, a2, \
                       hH, hF, C);                                                              \
    return 1;                                                                                   \
  }
  SKDX(128, 128) SKDX(64, 128) SKDX(128, 64) SKDX(64, 64)
#undef SKDX
  return 0;
}

// dW (128 x 128, fp32) = X^T D' over K rows: A = X^T given as (A, sAm = 1, sAk = ldx),
// B = D' = D (+ head outer) given as (B, sBk = ldd, sBn = 1).  Uses the caller's split-K
// workspace (splits x 128 x 128 fp32) for the block partials; 0 = not covered.
int wgrad_x3(int64_t K, const float* X, int64_t ldx, const float* D, int64_t ldd, int hH, int hF,
             const float* de, const float* a, const float* de2, const float* a2, float* slab,
             int nb, const float* cs_tab, float* cs_part, hipStream_t s);

// The fp32 weight gradient's kernel: MSHA_WGRAD=s3 (split-bf16, register operands, at any
// size), x3 (split-bf16 through LDS images, wgrad_x3.hip) or fp32 (exact-fp32 MFMA,
// wgrad_kernel); unset: s3 from MSHA_WGRAD_S3_MIN_ROWS (131,072) rows, fp32 below.
// Switchable at run time (msha_wgrad_kernel) for A/B runs and tests.
static std::atomic<int>& wgrad_mode() {
  static std::atomic<int> m([] {
    const char* v = getenv("MSHA_WGRAD");
    if (v == nullptr || !*v) return 0;
    return strcmp(v, "x3") == 0 ? 2 : strcmp(v, "fp32") == 0 ? 1 : strcmp(v, "s3") == 0 ? 3 : 0;
  }());
  return m;
}

int skinny_wgrad(int64_t M, int64_t N, int64_t K, const float* A, int64_t sAm, int64_t sAk,
                 const float* B, int64_t sBk, int64_t sBn, float* C, int64_t ldc, float beta,
                 int32_t splits, void* ws, size_t ws_bytes, int hH, int hF, const float* de,
                 const float* a, const float* de2, const float* a2, hipStream_t s,
                 const float* cs_tab, float* cs_part, float* cs_out1, float* cs_out2,
                 const float* cs_w, int64_t ldw) {
  if (!skinny_enabled() || M != 128 || N != 128 || sAm != 1 || sBn != 1) return 0;
  if (K < 4096 || K >= (1ll << 31) || splits < 16) return 0;
  if (sAk % 4 || sBk % 4 || ((uintptr_t)A | (uintptr_t)B) & 15) return 0;
  if (de != nullptr && (hF % 4 || ((uintptr_t)a & 15) || (a2 && ((uintptr_t)a2 & 15)))) return 0;
  const size_t per = (size_t)128 * 128 * sizeof(float);
  int64_t nb = (int64_t)(ws_bytes / per);
  if (nb > splits) nb = splits;
  if (nb > 256) nb = 256;
  if (nb < 16 || ws == nullptr) return 0;
  if (cs_tab != nullptr && (de == nullptr || cs_part == nullptr || cs_out1 == nullptr ||
                          (de2 != nullptr) != (cs_out2 != nullptr) || ((uintptr_t)cs_tab & 7)))
    return 0;
  float* slab = (float*)ws;
  // below ~128k rows a wave of the split kernel has too few 16-row steps to repay its
  // fixed costs (C4 100k rows: 46 vs 43 us): the exact-fp32 kernel runs there
  static const int64_t s3_min = [] {
    const char* v = getenv("MSHA_WGRAD_S3_MIN_ROWS");
    return v != nullptr && *v ? (int64_t)atoll(v) : (int64_t)131072;
  }();
  const int req = wgrad_mode().load();  // 3: the split kernel whatever the rows
  const int mode = req == 3 ? 0 : req == 0 && K < s3_min ? 1 : req;
  const bool small = K * sAk * 4 < (1ll << 31) && K * sBk * 4 < (1ll << 31);
  if (cs_w != nullptr) {
    // the column sums from G = e^T X and W (two heads, split-bf16 kernel only)
    if (mode != 0 || !small || hH != 2 || de == nullptr || cs_part == nullptr || cs_out1 == nullptr ||
        (de2 != nullptr) != (cs_out2 != nullptr) || ldw < 128)
      return 0;
    hipLaunchKernelGGL((sk::wgrad_s3_kernel<true, 2>), dim3((unsigned)nb), dim3(64 * sk::kWsWaves), 0, s,
                       (int)K, A, sAk, B, sBk, de, a, de2, a2, hH, hF, slab, nullptr, cs_part);
    hipLaunchKernelGGL(sk::wgrad_reduce_kernel<float>, dim3(128 * 128 / (4 * sk::kWrCols)), dim3(256), 0,
                       s, (const float*)slab, (int)nb, C, ldc, beta, (const float*)nullptr,
                       (float*)nullptr, (float*)nullptr);
    hipLaunchKernelGGL(sk::wgrad_gw_kernel, dim3(de2 != nullptr ? 4 : 2), dim3(256), 0, s,
                       (const float*)cs_part, (int)nb, cs_w, ldw, hF, cs_out1, cs_out2);
    return 1;
  }
  if (mode == 0 && small) {
    // split-bf16, register operands (wgrad_s3_kernel): same slab / partial layout
    if (cs_tab != nullptr)
      hipLaunchKernelGGL((sk::wgrad_s3_kernel<true, 1>), dim3((unsigned)nb), dim3(64 * sk::kWsWaves), 0,
                         s, (int)K, A, sAk, B, sBk, de, a, de2, a2, hH, hF, slab, cs_tab, cs_part);
    else if (de != nullptr)
      hipLaunchKernelGGL((sk::wgrad_s3_kernel<true, 0>), dim3((unsigned)nb), dim3(64 * sk::kWsWaves), 0,
                         s, (int)K, A, sAk, B, sBk, de, a, de2, a2, hH, hF, slab, nullptr, nullptr);
    else
      hipLaunchKernelGGL((sk::wgrad_s3_kernel<false, 0>), dim3((unsigned)nb), dim3(64 * sk::kWsWaves),
                         0, s, (int)K, A, sAk, B, sBk, nullptr, nullptr, nullptr, nullptr, 1, 4, slab,
                         nullptr, nullptr);
  } else if (mode == 2 &&
             wgrad_x3(K, A, sAk, B, sBk, hH, hF, de, a, de2, a2, slab, (int)nb, cs_tab, cs_part, s)) {
    // split-bf16 (wgrad_x3.hip): same slab / partial layout
  } else if (cs_tab != nullptr)
    hipLaunchKernelGGL((sk::wgrad_kernel<true, true>), dim3((unsigned)nb), dim3(64 * sk::kWgWaves), 0, s,
                       (int)K, A, sAk, B, sBk, de, a, de2, a2, hH, hF, slab, cs_tab, cs_part);
  else if (de != nullptr)
    hipLaunchKernelGGL((sk::wgrad_kernel<true, false>), dim3((unsigned)nb), dim3(64 * sk::kWgWaves), 0, s,
                       (int)K, A, sAk, B, sBk, de, a, de2, a2, hH, hF, slab, nullptr, nullptr);
  else
    hipLaunchKernelGGL((sk::wgrad_kernel<false, false>), dim3((unsigned)nb), dim3(64 * sk::kWgWaves), 0, s,
                       (int)K, A, sAk, B, sBk, nullptr, nullptr, nullptr, nullptr, 1, 4, slab, nullptr,
                       nullptr);
  // (+ 64 blocks of one wave per output for the CS partials)
  hipLaunchKernelGGL(sk::wgrad_reduce_kernel<float>,
                     dim3(128 * 128 / (4 * sk::kWrCols) + (cs_tab != nullptr ? 2 * 128 / 4 : 0)),
                     dim3(256), 0, s, (const float*)slab, (int)nb, C, ldc, beta,
                     (const float*)cs_part, cs_out1, cs_out2);
  return 1;
}

}  // namespace msha

// Diagnostic: install (buf != NULL) or remove the per-wave timeline buffer of the skinny
// kernels (slots x 64 uint64 words, device memory); MSHA_ERR_UNSUPPORTED unless the library
// was built with -DSK_TIMELINE (build.py --variant timeline).
// (ABI 15) the fp32 weight-gradient kernel: 0 auto (split-bf16 registers from 131,072 rows,
// exact fp32 below), 1 exact fp32, 2 split-bf16 LDS images, 3 split-bf16 registers at any
// size; returns the previous mode, mode < 0 only queries
extern "C" int32_t msha_wgrad_kernel(int32_t mode) {
  if (mode < 0 || mode > 3) return msha::wgrad_mode().load();
  return msha::wgrad_mode().exchange(mode);
}

extern "C" int msha_debug_timeline(void* buf, int64_t slots) {
#ifdef SK_TIMELINE
  uint64_t* p = (uint64_t*)buf;
  const int64_t n = buf != nullptr ? slots : 0;
  if (hipMemcpyToSymbol(HIP_SYMBOL(msha::sk::g_tl_buf), &p, sizeof(p)) != hipSuccess ||
      hipMemcpyToSymbol(HIP_SYMBOL(msha::sk::g_tl_slots), &n, sizeof(n)) != hipSuccess)
    return msha::fail(MSHA_ERR_HIP, "debug_timeline: hipMemcpyToSymbol failed");
  return MSHA_OK;
#else
  (void)buf;
  (void)slots;
  return msha::fail(MSHA_ERR_UNSUPPORTED, "debug_timeline: library built without SK_TIMELINE");
#endif
}
