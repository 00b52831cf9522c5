// Shared device/host helpers for the MSHA-GNN gfx950 library.
//
// Everything here is written for CDNA4 (gfx950): 64-lane wavefronts, 64-bit
// ballots, xor-shuffles lowered to ds_swizzle / DPP by hipcc.  No CUDA shims.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "../../include/msha_gnn.h"

namespace msha {

constexpr int kWave = 64;

// ---- error plumbing (thread-local last error, no exceptions across the ABI) ----
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
int check_launch(const char* what);

#define MSHA_ARG_CHECK(cond, msg)                              \
  do {                                                        \
    if (!(cond)) return ::msha::fail(MSHA_ERR_ARG, (msg));    \
  } while (0)

// ---- wave helpers ----
__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }

// v of lane ^ o.  Offsets 1, 2 (quad_perm) and 8 (row_ror:8 inside a 16-lane row) are
// DPP moves on the VALU; 16 and 32 are gfx950's v_permlane16/32_swap (VALU, no LDS
// round trip); the rest go through ds_bpermute.  The same values either way.
// permlaneN_swap(x, x) exchanges the odd N-lane blocks of its first operand with the
// even blocks of its second, so its two results hold x[l] and x[l ^ N] in some order:
// lane l takes the one from the other block.
#ifndef XOR_DPP
#define XOR_DPP 1
#endif
#ifndef XOR_PERMLANE
#define XOR_PERMLANE 0  // measured neutral-to-slower; kept for A/B
#endif
__device__ __forceinline__ float xor_shfl(float v, int o) {
  if (XOR_DPP) {
    const int x = __builtin_bit_cast(int, v);
    if (o == 1) return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, true));
    if (o == 2) return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, true));
    if (o == 8) return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(x, 0x128, 0xF, 0xF, true));
  }
  if (XOR_PERMLANE && (o == 16 || o == 32)) {
    const unsigned x = __builtin_bit_cast(unsigned, v);
    const int l = (int)(threadIdx.x & (kWave - 1));
    if (o == 32) {
      const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
      return __builtin_bit_cast(float, l < 32 ? r[1] : r[0]);
    }
    const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    return __builtin_bit_cast(float, (l & 16) ? r[0] : r[1]);
  }
  return __shfl_xor(v, o);
}

template <int FIRST>
__device__ __forceinline__ float wave_xor_max(float v) {
#pragma unroll
  for (int o = FIRST; o < kWave; o <<= 1) v = fmaxf(v, xor_shfl(v, o));
  return v;
}

template <int FIRST>
__device__ __forceinline__ float wave_xor_sum(float v) {
#pragma unroll
  for (int o = FIRST; o < kWave; o <<= 1) v += xor_shfl(v, o);
  return v;
}

// sum over an aligned group of G consecutive lanes (G power of two); all lanes get it
template <int G>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = 1; o < G; o <<= 1) v += xor_shfl(v, o);
  return v;
}

__device__ __forceinline__ float4 f4_scale(float4 a, float s) {
  return make_float4(a.x * s, a.y * s, a.z * s, a.w * s);
}
__device__ __forceinline__ float4 f4_fma(float s, float4 a, float4 c) {
  return make_float4(fmaf(s, a.x, c.x), fmaf(s, a.y, c.y), fmaf(s, a.z, c.z), fmaf(s, a.w, c.w));
}
__device__ __forceinline__ float f4_dot(float4 a, float4 b) {
  return fmaf(a.x, b.x, fmaf(a.y, b.y, fmaf(a.z, b.z, a.w * b.w)));
}
__device__ __forceinline__ float4 f4_xor_add(float4 v, int o) {
  return make_float4(v.x + __shfl_xor(v.x, o), v.y + __shfl_xor(v.y, o),
                     v.z + __shfl_xor(v.z, o), v.w + __shfl_xor(v.w, o));
}

__device__ __forceinline__ float lrelu(float x, float slope) { return x > 0.f ? x : x * slope; }

// ---- node-table storage types: fp32 or bf16 (MSHA_DTYPE_*), fp32 arithmetic ----
typedef __bf16 bf16_t;

// 16 bytes of a table row held as fp32 in registers: 4 fp32 or 8 bf16 elements
template <typename T>
struct Pk {
  static constexpr int V = 16 / (int)sizeof(T);
  float v[V];
};

template <typename T>
__device__ __forceinline__ Pk<T> pk_zero() {
  Pk<T> r;
#pragma unroll
  for (int i = 0; i < Pk<T>::V; ++i) r.v[i] = 0.f;
  return r;
}

__device__ __forceinline__ Pk<float> pk_load(const float* p) {
  const float4 x = *reinterpret_cast<const float4*>(p);
  Pk<float> r;
  r.v[0] = x.x; r.v[1] = x.y; r.v[2] = x.z; r.v[3] = x.w;
  return r;
}
__device__ __forceinline__ Pk<bf16_t> pk_load(const bf16_t* p) {
  const uint4 x = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {x.x, x.y, x.z, x.w};
  Pk<bf16_t> r;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    r.v[2 * i] = __uint_as_float(w[i] << 16);
    r.v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
  return r;
}
__device__ __forceinline__ void pk_store(float* p, const Pk<float>& a) {
  *reinterpret_cast<float4*>(p) = make_float4(a.v[0], a.v[1], a.v[2], a.v[3]);
}
// round-to-nearest-even (v_cvt_pk_bf16_f32)
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  const bf16_t l = (bf16_t)lo, h = (bf16_t)hi;
  return (uint32_t)__builtin_bit_cast(uint16_t, l) | ((uint32_t)__builtin_bit_cast(uint16_t, h) << 16);
}
__device__ __forceinline__ void pk_store(bf16_t* p, const Pk<bf16_t>& a) {
  *reinterpret_cast<uint4*>(p) = make_uint4(pack_bf16x2(a.v[0], a.v[1]), pack_bf16x2(a.v[2], a.v[3]),
                                            pack_bf16x2(a.v[4], a.v[5]), pack_bf16x2(a.v[6], a.v[7]));
}
template <typename T>
__device__ __forceinline__ Pk<T> pk_fma(float s, const Pk<T>& a, Pk<T> c) {
#pragma unroll
  for (int i = 0; i < Pk<T>::V; ++i) c.v[i] = fmaf(s, a.v[i], c.v[i]);
  return c;
}
template <typename T>
__device__ __forceinline__ Pk<T> pk_scale(Pk<T> a, float s) {
#pragma unroll
  for (int i = 0; i < Pk<T>::V; ++i) a.v[i] *= s;
  return a;
}
template <typename T>
__device__ __forceinline__ float pk_dot(const Pk<T>& a, const Pk<T>& b) {
  float r = a.v[Pk<T>::V - 1] * b.v[Pk<T>::V - 1];
#pragma unroll
  for (int i = Pk<T>::V - 2; i >= 0; --i) r = fmaf(a.v[i], b.v[i], r);
  return r;
}
// what a bf16 store of `a` rounds away: a - bf16(a) (round-to-nearest-even), exact in
// fp32; stored as bf16 itself, hi + lo carries ~16 mantissa bits.  fp32 tables: zero.
__device__ __forceinline__ Pk<bf16_t> pk_residual(const Pk<bf16_t>& a) {
  Pk<bf16_t> r;
#pragma unroll
  for (int i = 0; i < Pk<bf16_t>::V; ++i) r.v[i] = a.v[i] - (float)(bf16_t)a.v[i];
  return r;
}
__device__ __forceinline__ Pk<float> pk_residual(const Pk<float>&) { return pk_zero<float>(); }

template <typename T>
__device__ __forceinline__ Pk<T> pk_xor_add(Pk<T> a, int o) {
#pragma unroll
  for (int i = 0; i < Pk<T>::V; ++i) a.v[i] += xor_shfl(a.v[i], o);
  return a;
}

// ---- buffer (descriptor) memory ops: 32-bit byte offsets, hardware range check ----
// A lane whose offset is past the descriptor's byte count reads 0 and its store is
// dropped, so "load or 0" and masked stores need no branch: the loop bodies stay
// straight-line and the compiler's vmcnt waits stay exact (a divergent branch around
// a load makes the count path-dependent and forces vmcnt(0)).
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr uint32_t kOOB = 0x80000000u;  // offset of a masked lane (descriptors < 2 GiB)

__device__ __forceinline__ rsrc_t make_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, p ? bytes : 0, 0x00020000);
}
__device__ __forceinline__ float buf_f32(rsrc_t r, uint32_t off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
__device__ __forceinline__ int32_t buf_i32(rsrc_t r, uint32_t off) {
  return (int32_t)__builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
}
__device__ __forceinline__ uint32_t buf_u8(rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b8(r, off, 0, 0);
}
__device__ __forceinline__ void buf_store_f32(rsrc_t r, uint32_t off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, off, 0, 0);
}
__device__ __forceinline__ u32x4_t buf_b128(rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
}
// 16 raw bytes -> fp32 lanes (kept raw in registers while in flight: a bf16 piece
// widens only at its use, so a batch of loads costs 4 VGPRs each)
__device__ __forceinline__ Pk<float> pk_from_raw(u32x4_t x, float*) {
  Pk<float> p;
  p.v[0] = __uint_as_float(x.x); p.v[1] = __uint_as_float(x.y);
  p.v[2] = __uint_as_float(x.z); p.v[3] = __uint_as_float(x.w);
  return p;
}
__device__ __forceinline__ Pk<bf16_t> pk_from_raw(u32x4_t x, bf16_t*) {
  const uint32_t w[4] = {x.x, x.y, x.z, x.w};
  Pk<bf16_t> p;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    p.v[2 * i] = __uint_as_float(w[i] << 16);
    p.v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
  return p;
}
__device__ __forceinline__ Pk<float> pk_load_buf(rsrc_t r, uint32_t off, float* t) {
  return pk_from_raw(buf_b128(r, off), t);
}
__device__ __forceinline__ Pk<bf16_t> pk_load_buf(rsrc_t r, uint32_t off, bf16_t* t) {
  return pk_from_raw(buf_b128(r, off), t);
}

__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(bf16_t x) { return (float)x; }
template <typename T>
__device__ __forceinline__ T from_f32(float x) { return (T)x; }

// ---- counter-based dropout (Philox4x32-10) ----
// keep(i) = philox(seed; counter = {i, offset}).x >= p * 2^32.  Deterministic per
// element index, so forward and backward regenerate the same mask without storing it.
__host__ __device__ __forceinline__ uint32_t mulhi32(uint32_t a, uint32_t b) {
  return (uint32_t)(((uint64_t)a * (uint64_t)b) >> 32);
}

__host__ __device__ __forceinline__ uint32_t philox_x(uint64_t seed, uint64_t offset,
                                                      uint64_t idx) {
  uint32_t c0 = (uint32_t)idx, c1 = (uint32_t)(idx >> 32);
  uint32_t c2 = (uint32_t)offset, c3 = (uint32_t)(offset >> 32);
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = mulhi32(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
    const uint32_t hi1 = mulhi32(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
    c0 = hi1 ^ c1 ^ k0;
    c1 = lo1;
    c2 = hi0 ^ c3 ^ k1;
    c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c0;
}

// all four words of the same Philox4x32-10 block: word t of block q keys element 4q + t
// of the flat-table dropout masks (msha_segments), one generator call per 4 elements
__host__ __device__ __forceinline__ uint4 philox4(uint64_t seed, uint64_t offset, uint64_t q) {
  uint32_t c0 = (uint32_t)q, c1 = (uint32_t)(q >> 32);
  uint32_t c2 = (uint32_t)offset, c3 = (uint32_t)(offset >> 32);
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = mulhi32(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
    const uint32_t hi1 = mulhi32(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
    c0 = hi1 ^ c1 ^ k0;
    c1 = lo1;
    c2 = hi0 ^ c3 ^ k1;
    c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return make_uint4(c0, c1, c2, c3);
}

struct Dropout {
  uint64_t seed, offset;
  uint32_t threshold;  // drop when philox < threshold
  float scale;         // 1 / (1 - p)
  bool active;
  const uint64_t* ctr;  // device replay counter (msha_set_rng_counter), nullable
};

// the replay counter installed for the device of `s` (runtime.hip, one slot per device):
// read by the kernels at draw time
const uint64_t* rng_counter(hipStream_t s);

inline Dropout make_dropout(float p, uint64_t seed, uint64_t offset, hipStream_t s) {
  Dropout d;
  d.seed = seed;
  d.offset = offset;
  d.ctr = rng_counter(s);
  d.active = p > 0.f;
  double t = (double)p * 4294967296.0;
  d.threshold = p >= 1.f ? 0xFFFFFFFFu : (uint32_t)(t > 4294967295.0 ? 4294967295.0 : t);
  d.scale = p > 0.f && p < 1.f ? (float)(1.0 / (1.0 - (double)p)) : (p >= 1.f ? 0.f : 1.f);
  return d;
}

// Philox offset of a draw: the call's offset, plus (replay counter << 32) when a device
// counter is installed, so a captured HIP graph draws fresh masks on every replay
__device__ __forceinline__ uint64_t dropout_offset(const Dropout& d, uint64_t offset) {
  return d.ctr != nullptr ? offset + (*d.ctr << 32) : offset;
}

__device__ __forceinline__ float dropout_factor(const Dropout& d, uint64_t idx) {
  if (!d.active) return 1.f;
  return philox_x(d.seed, dropout_offset(d, d.offset), idx) >= d.threshold ? d.scale : 0.f;
}

// the four-words-per-call stream (element e = word e % 4 of block e / 4, as the flat-table
// masks): dropout_factor4 for one element, dropout_factors4 for the 4-aligned group from e4
__device__ __forceinline__ float dropout_factor4(const Dropout& d, uint64_t idx) {
  if (!d.active) return 1.f;
  const uint4 w = philox4(d.seed, dropout_offset(d, d.offset), idx >> 2);
  const uint32_t x = (idx & 3) == 0 ? w.x : (idx & 3) == 1 ? w.y : (idx & 3) == 2 ? w.z : w.w;
  return x >= d.threshold ? d.scale : 0.f;
}
__device__ __forceinline__ float4 dropout_factors4(const Dropout& d, uint64_t e4) {
  if (!d.active) return make_float4(1.f, 1.f, 1.f, 1.f);
  const uint4 w = philox4(d.seed, dropout_offset(d, d.offset), e4 >> 2);
  return make_float4(w.x >= d.threshold ? d.scale : 0.f, w.y >= d.threshold ? d.scale : 0.f,
                     w.z >= d.threshold ? d.scale : 0.f, w.w >= d.threshold ? d.scale : 0.f);
}

// skinny.hip: resident-W projection and whole-tile weight gradient (1 = launched,
// 0 = shape not covered: the caller runs its tiled GEMM)
template <typename T>
int skinny_project(int64_t M, int64_t K, int heads, int feat, const void* X, const void* W,
                   const float* al, const float* ar, void* h, float* el, float* er,
                   hipStream_t s);
int skinny_pair_linear(int64_t P, int64_t K, int64_t N, const float* G, int64_t ldg,
                       const int64_t* gi, const float* G2, int64_t ldg2, const int64_t* gj,
                       int64_t g_rows, int64_t g2_rows, const float* W, const float* bias, int act, const Dropout& dp, float* out,
                       hipStream_t s);
int skinny_pair_linear_bf16(int64_t P, int64_t K, int64_t N, const void* G, int64_t ldg,
                            const int64_t* gi, const void* G2, int64_t ldg2, const int64_t* gj,
                            const void* W, const float* bias, int act, const Dropout& dp,
                            void* out, bool out_bf16, hipStream_t s);
int skinny_dx(int64_t M, int64_t N, int64_t K, const float* Dh, const float* W, float* C,
              int hH, int hF, const float* d1, const float* a1, const float* d2, const float* a2,
              hipStream_t s);
// cs_tab (optional): also cs_out1[n] = sum_r de[r, n / hF] cs_tab[r, n] (cs_out2 with de2)
// through the per-block partials in cs_part (2 x N x 256 floats); cs_tab has B's row pitch.
// cs_w (optional, instead of cs_tab, where cs_tab = A^T-rows x cs_w): the same sums as
// (de^T X) cs_w from the rows already loaded (two heads; partials 4 x 128 x 256 floats)
int skinny_wgrad(int64_t M, int64_t N, int64_t K, const float* A, int64_t sAm, int64_t sAk,
                 const float* B, int64_t sBk, int64_t sBn, float* C, int64_t ldc, float beta,
                 int32_t splits, void* ws, size_t ws_bytes, int hH, int hF, const float* de,
                 const float* a, const float* de2, const float* a2, hipStream_t s,
                 const float* cs_tab = nullptr, float* cs_part = nullptr,
                 float* cs_out1 = nullptr, float* cs_out2 = nullptr,
                 const float* cs_w = nullptr, int64_t ldw = 0);

// Welford triple (count, mean, M2) and Chan's combination (bn.hip, head.hip)
struct Wf {
  float n, mean, m2;
};

__host__ __device__ __forceinline__ Wf wf_combine(Wf a, Wf b) {
  if (b.n == 0.f) return a;
  if (a.n == 0.f) return b;
  const float n = a.n + b.n;
  const float d = b.mean - a.mean;
  Wf r;
  r.n = n;
  r.mean = a.mean + d * (b.n / n);
  r.m2 = a.m2 + b.m2 + d * d * (a.n * b.n / n);
  return r;
}

// bn.hip: Welford partials per 256-row block of a (rows, C) table (Wf, block-major)
int64_t bn_stats_partials(int64_t rows, int C, bool bf, const void* x, void* part, hipStream_t s);
int64_t bn_stats_blocks(int64_t rows);

inline int grid_for(int64_t work_items, int per_block, int cap = 1 << 20) {
  int64_t g = (work_items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

}  // namespace msha
