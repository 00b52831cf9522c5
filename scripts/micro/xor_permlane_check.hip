// Checks common.h's xor_shfl (DPP / v_permlane16/32_swap / ds_bpermute paths) against
// __shfl_xor for every offset, on random bit patterns incl. NaN/denormal payloads.
// Build: hipcc --offload-arch=gfx950 -O3 -I msha--gnn_amd/csrc scripts/micro/xor_permlane_check.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "common.h"

__global__ void k(const float* a, float* got, float* want) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const float v = a[t];
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const int o = 1 << j;
    got[t * 6 + j] = msha::xor_shfl(v, o);
    want[t * 6 + j] = __shfl_xor(v, o);
  }
}

int main() {
  const int n = 256 * 64;
  float *a, *g, *w;
  if (hipMallocManaged(&a, n * 4) || hipMallocManaged(&g, n * 24) || hipMallocManaged(&w, n * 24))
    return 2;
  srand(1);
  for (int i = 0; i < n; ++i) {
    unsigned u = ((unsigned)rand() << 16) ^ (unsigned)rand();
    memcpy(&a[i], &u, 4);
  }
  hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, a, g, w);
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  int bad = 0;
  for (int i = 0; i < n * 6; ++i) bad += memcmp(&g[i], &w[i], 4) != 0;
  printf("xor_shfl vs __shfl_xor: %d mismatches of %d\n", bad, n * 6);
  return bad ? 1 : 0;
}
