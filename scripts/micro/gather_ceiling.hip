// Random row-gather ceiling on one MI355X: how fast can a wave-per-segment kernel
// read uniformly random ROW_BYTES rows of a large table (the access pattern of the
// edge kernels on a cache-busting graph)?  Each wave reads SEG consecutive indices,
// gathers those rows 16 B per lane (16 loads in flight per lane) and sums them; one float per wave is written.
// Bandwidth counts the index bytes and the gathered row bytes.
//   hipcc -O3 --offload-arch=gfx950 gather_ceiling.hip -o gather_ceiling
//   ./gather_ceiling [table_MB]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

template <int ROW_BYTES>
__global__ void __launch_bounds__(256) gather(const float4* __restrict__ table,
                                              const int* __restrict__ idx, long n_idx,
                                              float* __restrict__ out) {
  constexpr int LPR = ROW_BYTES / 16;  // lanes per row
  constexpr int RPI = 64 / LPR;        // rows per wave-instruction
  constexpr int NL = 16;               // independent 16-B loads in flight per lane
  constexpr int SEG = NL * RPI;        // rows per wave step
  const int lane = threadIdx.x & 63;
  const long wave = (blockIdx.x * (long)blockDim.x + threadIdx.x) >> 6;
  const long nwaves = (gridDim.x * (long)blockDim.x) >> 6;
  float acc = 0.f;
  for (long s = wave * SEG; s < n_idx; s += nwaves * SEG) {
    const int my = lane < SEG && s + lane < n_idx ? idx[s + lane] : 0;
    float4 v[NL];
#pragma unroll
    for (int g = 0; g < NL; ++g) {
      const int r = __shfl(my, g * RPI + lane / LPR);
      v[g] = table[(long)r * LPR + lane % LPR];
    }
#pragma unroll
    for (int g = 0; g < NL; ++g) acc += v[g].x + v[g].y + v[g].z + v[g].w;
  }
  if (acc == 1234.5f) out[wave] = acc;  // keep the loads alive
}

template <int RB>
static void run(long table_bytes, int grid, long n_idx, int* d_idx, float4* d_table,
                float* d_out, long n_rows_table) {
  std::vector<int> h(n_idx);
  srand(7);
  for (long i = 0; i < n_idx; ++i)
    h[i] = (int)(((long)rand() * RAND_MAX + rand()) % (table_bytes / RB));
  CHECK(hipMemcpy(d_idx, h.data(), n_idx * 4, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int it = 0; it < 3; ++it)
    hipLaunchKernelGGL(gather<RB>, grid, 256, 0, 0, d_table, d_idx, n_idx, d_out);
  CHECK(hipEventRecord(a));
  const int reps = 10;
  for (int it = 0; it < reps; ++it)
    hipLaunchKernelGGL(gather<RB>, grid, 256, 0, 0, d_table, d_idx, n_idx, d_out);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const double us = ms * 1e3 / reps;
  const double bytes = (double)n_idx * (RB + 4);
  printf("row %4d B  table %6ld MB  grid %6d  %8.1f us  %7.1f GB/s\n", RB, table_bytes >> 20,
         grid, us, bytes / us / 1e3);
}

int main(int argc, char** argv) {
  const long table_mb = argc > 1 ? atol(argv[1]) : 1024;
  const long table_bytes = table_mb << 20;
  const long n_idx = 40l << 20;
  float4* d_table;
  int* d_idx;
  float* d_out;
  CHECK(hipMalloc(&d_table, table_bytes));
  CHECK(hipMemset(d_table, 0, table_bytes));
  CHECK(hipMalloc(&d_idx, n_idx * 4));
  CHECK(hipMalloc(&d_out, 1 << 24));
  for (int grid : {256 * 8, 256 * 32}) {
    run<256>(table_bytes, grid, n_idx, d_idx, d_table, d_out, 0);
    run<512>(table_bytes, grid, n_idx, d_idx, d_table, d_out, 0);
    run<1024>(table_bytes, grid, n_idx, d_idx, d_table, d_out, 0);
  }
  return 0;
}
