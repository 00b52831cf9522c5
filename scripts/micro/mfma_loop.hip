// Microbenchmark (not part of the library): the fp32 GEMM's inner MFMA loop alone
// (LDS operand reads + 16 v_mfma_f32_16x16x4_f32 per k-step), to separate the loop's
// issue efficiency from the global-load / barrier structure of gemm_f32_kernel.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int LDA = 34, LDP = 144;

__global__ void __launch_bounds__(256) loop_kernel(float* out, int iters) {
  __shared__ float smem[128 * LDA + 32 * LDP];
  float* As = smem;
  float* Bs = smem + 128 * LDA;
  for (int i = threadIdx.x; i < 128 * LDA + 32 * LDP; i += 256) smem[i] = (float)(i % 7) * 0.1f;
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  f32x4 acc[2][8];
  for (int r = 0; r < 2; ++r)
    for (int c = 0; c < 8; ++c) acc[r][c] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const int kr = ks * 4 + (lane >> 4);
      const float a0 = As[(w * 32 + (lane & 15)) * LDA + kr];
      const float a1 = As[(w * 32 + 16 + (lane & 15)) * LDA + kr];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const float b = Bs[kr * LDP + c * 16 + (lane & 15)];
        acc[0][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b, acc[0][c], 0, 0, 0);
        acc[1][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b, acc[1][c], 0, 0, 0);
      }
    }
  }
  float s = 0.f;
  for (int r = 0; r < 2; ++r)
    for (int c = 0; c < 8; ++c) s += acc[r][c][0] + acc[r][c][1] + acc[r][c][2] + acc[r][c][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
  float* out;
  hipMalloc(&out, 4096 * 256 * sizeof(float));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int blocks : {256, 512, 782, 1024, 2048}) {
    const int iters = 64;
    hipLaunchKernelGGL(loop_kernel, dim3(blocks), dim3(256), 0, 0, out, iters);
    hipEventRecord(a);
    hipLaunchKernelGGL(loop_kernel, dim3(blocks), dim3(256), 0, 0, out, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double flop = 2.0 * blocks * 128.0 * 128.0 * 32.0 * iters;
    printf("blocks %d: %.1f us, %.1f TFLOP/s\n", blocks, ms * 1e3, flop / (ms * 1e-3) / 1e12);
  }
  return 0;
}
