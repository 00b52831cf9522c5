// The training loss on gathered rows (train.py:227-229: F.nll_loss(output[source_index],
// recipient_index), mean reduction) and its backward, in one launch each.  In torch this
// is a row gather, the nll forward, and in the backward a ones fill, the nll backward, a
// zero fill of the (N, M) gradient and an index backward (sort + scatter-add): ~12
// launches around a 64-row batch.
//
//   forward   loss = -(1/B) sum_b logp[rows[b], cols[b]]   (b ascending, fp32)
//   backward  dlogp = 0 except dlogp[rows[b], cols[b]] += -g / B   (b ascending; repeated
//             (row, col) pairs accumulate as index backward does)
// An entry outside the (N, M) table (torch raises on such an index) is never read or
// written: the forward returns NaN instead, as it does for an empty batch (torch's mean
// over zero elements), and the backward skips it.
// The backward zero-fills row ranges per block (16-byte stores); each block then adds the
// batch entries that fall in its own rows in batch order (one lane, the batch staged
// through LDS), so the result is deterministic and no two blocks touch the same row.
#include "common.h"

namespace msha {

constexpr int kLossThreads = 256;
constexpr int kLossRowsPerBlock = 64;

template <typename T>
__global__ void __launch_bounds__(kLossThreads) nll_rows_fwd_kernel(
    int64_t N, int64_t M, int64_t B, const int64_t* __restrict__ rows,
    const int64_t* __restrict__ cols, const T* __restrict__ logp, int64_t ld,
    float* __restrict__ loss) {
  __shared__ float part[kLossThreads];
  float s = 0.f;
  // thread t adds entries t, t + 256, ... in order; the partials then add in a fixed tree
  for (int64_t b = threadIdx.x; b < B; b += kLossThreads) {
    const int64_t r = rows[b], c = cols[b];
    s += (r >= 0 && r < N && c >= 0 && c < M) ? to_f32(logp[r * ld + c]) : __builtin_nanf("");
  }
  part[threadIdx.x] = s;
  __syncthreads();
  for (int o = kLossThreads / 2; o >= 1; o >>= 1) {
    if ((int)threadIdx.x < o) part[threadIdx.x] += part[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) loss[0] = B > 0 ? -part[0] / (float)B : __builtin_nanf("");
}

// With rflag / wmask (msha_nll_rows_bwd_flags) each block also flags its rows whose gradient
// is nonzero -- one byte a row and one 64-row bit mask a word (a block's 64 rows are one
// word) -- the row scan the model head's backward would otherwise launch over the same
// gradient (head.hip head_bwd_scan_kernel: same test, value != 0 after the adds).
static_assert(kLossRowsPerBlock == 64, "one wmask word per block");
template <typename T>
__global__ void __launch_bounds__(kLossThreads) nll_rows_bwd_kernel(
    int64_t N, int64_t M, int64_t B, const int64_t* __restrict__ rows,
    const int64_t* __restrict__ cols, const float* __restrict__ gloss, T* __restrict__ dlogp,
    int64_t ld, uint8_t* __restrict__ rflag, uint64_t* __restrict__ wmask) {
  const int64_t r0 = (int64_t)blockIdx.x * kLossRowsPerBlock;
  const int64_t r1 = min(N, r0 + kLossRowsPerBlock);
  T* base = dlogp + r0 * ld;
  const int n = (int)((r1 - r0) * ld);  // <= 64 rows: 32-bit index math
  constexpr int kv = 16 / (int)sizeof(T);
  if (ld == M && ((uintptr_t)base % 16) == 0) {
    // the block's rows are one contiguous span: 16-byte zero stores (the scalar loop with
    // 64-bit div / mod took 11 us for the 5 MB gradient of the 2015 graph)
    const int nv = n / kv;
    for (int q = threadIdx.x; q < nv; q += kLossThreads)
      reinterpret_cast<uint4*>(base)[q] = make_uint4(0u, 0u, 0u, 0u);
    for (int e = nv * kv + threadIdx.x; e < n; e += kLossThreads) base[e] = from_f32<T>(0.f);
  } else {
    const int m = (int)M, l = (int)ld;
    for (int e = threadIdx.x; e < (int)(r1 - r0) * m; e += kLossThreads)
      base[(e / m) * l + e % m] = from_f32<T>(0.f);
  }
  // the batch entries in this block's rows, added in batch order by one lane; the batch
  // comes through LDS a chunk at a time (a serial loop over global loads cost ~0.5 us per
  // entry in every block)
  __shared__ int32_t br[kLossThreads], bc[kLossThreads];
  __shared__ uint64_t whit[kLossThreads / 64];
  const float v = B > 0 ? -gloss[0] / (float)B : 0.f;
  for (int64_t b0 = 0; b0 < B; b0 += kLossThreads) {
    __syncthreads();  // (the fill above / the previous chunk's reads)
    const int64_t b = b0 + threadIdx.x;
    int32_t rr = -1, cc = 0;
    if (b < B) {
      const int64_t r = rows[b], c = cols[b];
      if (r >= r0 && r < r1 && c >= 0 && c < M) {
        rr = (int32_t)(r - r0);
        cc = (int32_t)c;
      }
    }
    br[threadIdx.x] = rr;
    bc[threadIdx.x] = cc;
    // which of the chunk's entries fall in this block's rows (one mask per wave): the lane
    // then visits those alone, in batch order (its scan over every entry was ~2 us a block)
    const uint64_t hit = __ballot(rr >= 0);
    if ((threadIdx.x & 63) == 0) whit[threadIdx.x >> 6] = hit;
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
      for (int w = 0; w < kLossThreads / 64; ++w) {
        for (uint64_t m = whit[w]; m != 0ull; m &= m - 1ull) {
          const int q = w * 64 + __builtin_ctzll(m);
          T* p = base + (int64_t)br[q] * ld + bc[q];
          *p = from_f32<T>(to_f32(*p) + v);
        }
      }
    }
  }
  if (wmask != nullptr) {
    __syncthreads();  // (lane 0's adds)
    if (threadIdx.x < 64) {
      const int64_t i = r0 + threadIdx.x;
      int nz = 0;
      if (i < r1) {
        const T* dr = dlogp + i * ld;
        for (int j = 0; j < (int)M; ++j) nz |= to_f32(dr[j]) != 0.f;
        rflag[i] = nz ? 1 : 0;
      }
      const uint64_t bits = __ballot(nz != 0);
      if (threadIdx.x == 0) wmask[blockIdx.x] = bits;
    }
  }
}

}  // namespace msha

using namespace msha;

extern "C" int msha_nll_rows_fwd(int64_t N, int64_t M, int64_t B, const int64_t* rows,
                                 const int64_t* cols, int32_t dtype, const void* logp, int64_t ld,
                                 float* loss, msha_stream_t stream) {
  MSHA_ARG_CHECK(B >= 0 && loss != nullptr && (B == 0 || (rows && cols && logp)),
                 "nll_rows_fwd: null pointer");
  MSHA_ARG_CHECK(N > 0 && M > 0 && ld >= M, "nll_rows_fwd: bad sizes");
  MSHA_ARG_CHECK(dtype == MSHA_DTYPE_F32 || dtype == MSHA_DTYPE_BF16, "nll_rows_fwd: bad dtype");
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MSHA_DTYPE_BF16)
    hipLaunchKernelGGL(nll_rows_fwd_kernel<bf16_t>, dim3(1), dim3(kLossThreads), 0, s, N, M, B,
                       rows, cols, (const bf16_t*)logp, ld, loss);
  else
    hipLaunchKernelGGL(nll_rows_fwd_kernel<float>, dim3(1), dim3(kLossThreads), 0, s, N, M, B,
                       rows, cols, (const float*)logp, ld, loss);
  return check_launch("nll_rows_fwd");
}

extern "C" int msha_nll_rows_bwd_flags(int64_t N, int64_t M, int64_t B, const int64_t* rows,
                                       const int64_t* cols, const float* gloss, int32_t dtype,
                                       void* dlogp, int64_t ld, uint8_t* rflag, uint64_t* wmask,
                                       msha_stream_t stream) {
  MSHA_ARG_CHECK(N > 0 && M > 0 && B >= 0 && ld >= M, "nll_rows_bwd: bad sizes");
  MSHA_ARG_CHECK(dlogp && gloss && (B == 0 || (rows && cols)), "nll_rows_bwd: null pointer");
  MSHA_ARG_CHECK(dtype == MSHA_DTYPE_F32 || dtype == MSHA_DTYPE_BF16, "nll_rows_bwd: bad dtype");
  MSHA_ARG_CHECK((rflag == nullptr) == (wmask == nullptr), "nll_rows_bwd: rflag and wmask go together");
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((unsigned)((N + kLossRowsPerBlock - 1) / kLossRowsPerBlock));
  if (dtype == MSHA_DTYPE_BF16)
    hipLaunchKernelGGL(nll_rows_bwd_kernel<bf16_t>, grid, dim3(kLossThreads), 0, s, N, M, B,
                       rows, cols, gloss, (bf16_t*)dlogp, ld, rflag, wmask);
  else
    hipLaunchKernelGGL(nll_rows_bwd_kernel<float>, grid, dim3(kLossThreads), 0, s, N, M, B, rows,
                       cols, gloss, (float*)dlogp, ld, rflag, wmask);
  return check_launch("nll_rows_bwd");
}

extern "C" int msha_nll_rows_bwd(int64_t N, int64_t M, int64_t B, const int64_t* rows,
                                 const int64_t* cols, const float* gloss, int32_t dtype,
                                 void* dlogp, int64_t ld, msha_stream_t stream) {
  return msha_nll_rows_bwd_flags(N, M, B, rows, cols, gloss, dtype, dlogp, ld, nullptr, nullptr,
                                 stream);
}
