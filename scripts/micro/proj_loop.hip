// Microbenchmark (not part of the library): the skinny projection's inner loop alone --
// per k-step one A VGPR, 8 B operands read from an LDS image in MFMA-operand order, 8
// v_mfma_f32_16x16x4_f32 into 8 accumulators -- at 1, 2 and 4 waves per SIMD, with the B
// reads from LDS or from registers, to find the loop's own MFMA-pipe ceiling.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <bool LDSB, int STEPS_AHEAD>
__global__ void __launch_bounds__(512) loop_kernel(float* out, int tiles) {
  __shared__ float Wl[128 * 128];
  for (int i = threadIdx.x; i < 128 * 128; i += blockDim.x) Wl[i] = (float)(i % 13) * 0.01f;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const float* Wf = Wl + lane;
  f32x4 acc[8];
  for (int c = 0; c < 8; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  float a0 = lane * 0.001f;
  for (int t = 0; t < tiles; ++t) {
    float bc[8], bn[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) bc[c] = LDSB ? Wf[c * 64] : a0 + c;
#pragma unroll
    for (int s = 0; s < 32; ++s) {
      if (LDSB && s + 1 < 32) {
#pragma unroll
        for (int c = 0; c < 8; ++c) bn[c] = Wf[((s + 1) * 8 + c) * 64];
      }
      __builtin_amdgcn_sched_barrier(0);
      const float a = a0 + s;
#pragma unroll
      for (int c = 0; c < 8; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bc[c], acc[c], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (LDSB) {
#pragma unroll
        for (int c = 0; c < 8; ++c) bc[c] = bn[c];
      }
    }
    a0 += 1e-3f;
  }
  float s = 0.f;
  for (int c = 0; c < 8; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <bool LDSB>
static void run(const char* name, int blocks, int threads, int tiles, float* out) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL((loop_kernel<LDSB, 1>), dim3(blocks), dim3(threads), 0, 0, out, tiles);
  (void)hipEventRecord(a);
  hipLaunchKernelGGL((loop_kernel<LDSB, 1>), dim3(blocks), dim3(threads), 0, 0, out, tiles);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  const double flop = 2.0 * 16 * 128 * 128 * (double)tiles * blocks * (threads / 64);
  printf("%-8s blocks %4d x %3d thr (%d waves/SIMD), %d tiles/wave: %8.1f us  %6.1f TFLOP/s\n",
         name, blocks, threads, blocks / 256 * threads / 256, tiles, ms * 1e3,
         flop / (ms * 1e-3) / 1e12);
}

int main() {
  float* out;
  (void)hipMalloc(&out, 4096 * 512 * sizeof(float));
  for (int tiles : {3, 24}) {
    run<true>("lds-B", 256, 256, tiles, out);
    run<true>("lds-B", 256, 512, tiles, out);
    run<true>("lds-B", 512, 512, tiles, out);
    run<false>("reg-B", 256, 256, tiles, out);
    run<false>("reg-B", 256, 512, tiles, out);
  }
  return 0;
}
