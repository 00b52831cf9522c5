// Graph ingestion on the GPU: flow counts -> dense adjacency, column
// normalisation, and the `adj > 0` mask -> CSR + CSC (with virtual full rows).
//
// Reference: dataset.py:279-296 (inter_adjacent), model.py:95-100
// (normalize_adjacency_matrix), Ablation.py:268 / GAT.py:30 (the mask).
// All passes are deterministic (no float atomics; integer atomics only where
// the result is order independent).
#include <algorithm>

#include "common.h"

namespace msha {

constexpr int kRowBlock = 256;  // rows per column-count block
constexpr int kScanItems = 4;
constexpr int kScanThreads = 1024;
constexpr int kScanTile = kScanItems * kScanThreads;

// ------------------------------------------------------------ flow counts ---
__global__ void __launch_bounds__(256) count_flows_kernel(const int64_t* __restrict__ src,
                                                          const int64_t* __restrict__ dst,
                                                          int64_t n_flows, int64_t n_rows,
                                                          int64_t n_cols, int32_t* counts) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n_flows;
       k += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = src[k], r = dst[k];
    if (s >= 0 && s < n_rows && r >= 0 && r < n_cols) atomicAdd(&counts[s * n_cols + r], 1);
  }
}

__global__ void __launch_bounds__(256) counts_to_float_kernel(const int32_t* __restrict__ c,
                                                              int64_t n, float* __restrict__ out) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n;
       k += (int64_t)gridDim.x * blockDim.x)
    out[k] = (float)c[k];
}

// ----------------------------------------------------------- normalisation ---
// Column sums: block b sums rows [b*kRowBlock, ...) of every column in row order,
// then one thread per column adds the block partials in block order.
__global__ void __launch_bounds__(256) colsum_partial_kernel(const float* __restrict__ adj,
                                                             int64_t n_rows, int64_t n_cols,
                                                             float* __restrict__ part) {
  const int64_t r0 = (int64_t)blockIdx.x * kRowBlock;
  const int64_t r1 = min(n_rows, r0 + kRowBlock);
  for (int64_t j = threadIdx.x; j < n_cols; j += blockDim.x) {
    float s = 0.f;
    for (int64_t i = r0; i < r1; ++i) s += adj[i * n_cols + j];
    part[blockIdx.x * n_cols + j] = s;
  }
}

__global__ void __launch_bounds__(256) colscale_kernel(const float* __restrict__ part, int nblk,
                                                       int64_t n_cols, float* __restrict__ d,
                                                       float* __restrict__ bad) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n_cols;
       j += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int b = 0; b < nblk; ++b) s += part[(int64_t)b * n_cols + j];
    const float dj = 1.0f / sqrtf(s);  // == torch.pow(s, -0.5) on CPU (1/sqrt in fp32)
    d[j] = dj;
    if (!isfinite(dj)) *bad = 1.0f;  // any writer stores the same value
  }
}

__global__ void __launch_bounds__(256) scale_cols_kernel(const float* __restrict__ adj,
                                                         int64_t n_rows, int64_t n_cols,
                                                         const float* __restrict__ d,
                                                         const float* __restrict__ bad,
                                                         float* __restrict__ out) {
  const bool nan_all = *bad != 0.f;
  const int64_t n = n_rows * n_cols;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n;
       k += (int64_t)gridDim.x * blockDim.x) {
    const float dj = d[k % n_cols];
    out[k] = nan_all ? __builtin_nanf("") : (adj[k] * dj) * dj;
  }
}

// ------------------------------------------------------------- mask -> CSR ---
// One wave per row: degree via 64-column ballots.  Empty rows become virtual
// full rows (degree n_cols, rowflag 1).
__global__ void __launch_bounds__(256) row_count_kernel(const float* __restrict__ adj,
                                                        int64_t n_rows, int64_t n_cols,
                                                        int32_t* __restrict__ rowcnt,
                                                        uint8_t* __restrict__ rowflag) {
  const int lane = lane_id();
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) / kWave;
  for (int64_t i = wave; i < n_rows; i += nwaves) {
    int deg = 0;
    for (int64_t c = 0; c < n_cols; c += kWave) {
      const int64_t j = c + lane;
      const bool e = j < n_cols && adj[i * n_cols + j] > 0.f;
      deg += __popcll(__ballot(e));
    }
    if (lane == 0) {
      rowcnt[i] = deg > 0 ? deg : (int32_t)n_cols;
      rowflag[i] = deg > 0 ? 0 : 1;
    }
  }
}

__global__ void __launch_bounds__(256) col_count_partial_kernel(const float* __restrict__ adj,
                                                                int64_t n_rows, int64_t n_cols,
                                                                const uint8_t* __restrict__ rowflag,
                                                                int32_t* __restrict__ part) {
  const int64_t r0 = (int64_t)blockIdx.x * kRowBlock;
  const int64_t r1 = min(n_rows, r0 + kRowBlock);
  for (int64_t j = threadIdx.x; j < n_cols; j += blockDim.x) {
    int c = 0;
    for (int64_t i = r0; i < r1; ++i) c += (rowflag[i] || adj[i * n_cols + j] > 0.f) ? 1 : 0;
    part[blockIdx.x * n_cols + j] = c;
  }
}

// per column: exclusive prefix over row blocks (in place) and the column total
__global__ void __launch_bounds__(256) col_block_scan_kernel(int32_t* __restrict__ part, int nblk,
                                                             int64_t n_cols,
                                                             int32_t* __restrict__ colcnt) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n_cols;
       j += (int64_t)gridDim.x * blockDim.x) {
    int run = 0;
    for (int b = 0; b < nblk; ++b) {
      const int v = part[(int64_t)b * n_cols + j];
      part[(int64_t)b * n_cols + j] = run;
      run += v;
    }
    colcnt[j] = run;
  }
}

// ---- exclusive scan of int32 counts into an (n+1)-long offset array ----
__device__ __forceinline__ int block_exclusive_scan(int v, int* sh, int& total) {
  // sh: kScanThreads/64 ints
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(incl, o);
    if (lane >= o) incl += t;
  }
  if (lane == 63) sh[w] = incl;
  __syncthreads();
  if (w == 0) {
    int s = lane < (kScanThreads / 64) ? sh[lane] : 0;
    int si = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(si, o);
      if (lane >= o) si += t;
    }
    if (lane < (kScanThreads / 64)) sh[lane] = si - s;
    if (lane == (kScanThreads / 64) - 1) sh[kScanThreads / 64] = si;
  }
  __syncthreads();
  const int res = sh[w] + incl - v;
  total = sh[kScanThreads / 64];
  __syncthreads();
  return res;
}

__global__ void __launch_bounds__(kScanThreads) scan_tiles_kernel(const int32_t* __restrict__ in,
                                                                  int64_t n,
                                                                  int32_t* __restrict__ out,
                                                                  int32_t* __restrict__ tile_sums) {
  __shared__ int sh[kScanThreads / 64 + 1];
  const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
  int v[kScanItems];
  int s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    v[k] = base + k < n ? in[base + k] : 0;
    s += v[k];
  }
  int total;
  int run = block_exclusive_scan(s, sh, total);
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    if (base + k < n) out[base + k] = run;
    run += v[k];
  }
  if (threadIdx.x == 0) tile_sums[blockIdx.x] = total;
}

// single block: exclusive scan of the tile sums (any count, chunked with a carry);
// writes the grand total to out[n]
__global__ void __launch_bounds__(kScanThreads) scan_sums_kernel(int32_t* __restrict__ sums,
                                                                 int64_t ntiles,
                                                                 int32_t* __restrict__ out,
                                                                 int64_t n) {
  __shared__ int sh[kScanThreads / 64 + 1];
  int carry = 0;
  for (int64_t c = 0; c < ntiles; c += kScanThreads) {
    const int64_t k = c + threadIdx.x;
    const int v = k < ntiles ? sums[k] : 0;
    int total;
    const int ex = block_exclusive_scan(v, sh, total);
    if (k < ntiles) sums[k] = carry + ex;
    carry += total;
  }
  if (threadIdx.x == 0) out[n] = carry;
}

__global__ void __launch_bounds__(256) scan_add_kernel(int32_t* __restrict__ out, int64_t n,
                                                       const int32_t* __restrict__ sums) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n;
       k += (int64_t)gridDim.x * blockDim.x)
    out[k] += sums[k / kScanTile];
}

static size_t scan_ws_ints(int64_t n) { return (size_t)((n + kScanTile - 1) / kScanTile) + 1; }

static void exclusive_scan(const int32_t* in, int64_t n, int32_t* out, int32_t* ws,
                           hipStream_t s) {
  const int64_t ntiles = std::max<int64_t>(1, (n + kScanTile - 1) / kScanTile);
  hipLaunchKernelGGL(scan_tiles_kernel, dim3((unsigned)ntiles), dim3(kScanThreads), 0, s, in, n,
                     out, ws);
  hipLaunchKernelGGL(scan_sums_kernel, dim3(1), dim3(kScanThreads), 0, s, ws, ntiles, out, n);
  hipLaunchKernelGGL(scan_add_kernel, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s, out, n, ws);
}

// ------------------------------------------------------------ CSR / CSC fill ---
__global__ void __launch_bounds__(256) csr_fill_kernel(const float* __restrict__ adj,
                                                       int64_t n_rows, int64_t n_cols,
                                                       const int32_t* __restrict__ rowptr,
                                                       const uint8_t* __restrict__ rowflag,
                                                       int32_t* __restrict__ col) {
  const int lane = lane_id();
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) / kWave;
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  for (int64_t i = wave; i < n_rows; i += nwaves) {
    int32_t pos = rowptr[i];
    const bool virt = rowflag[i] != 0;
    for (int64_t c = 0; c < n_cols; c += kWave) {
      const int64_t j = c + lane;
      const bool e = j < n_cols && (virt || adj[i * n_cols + j] > 0.f);
      const uint64_t b = __ballot(e);
      if (e) col[pos + __popcll(b & lt)] = (int32_t)j;
      pos += __popcll(b);
    }
  }
}

__device__ __forceinline__ int32_t edge_id(const int32_t* __restrict__ rowptr,
                                           const int32_t* __restrict__ col, int64_t i, int32_t j) {
  int32_t lo = rowptr[i], hi = rowptr[i + 1];
  while (lo < hi) {  // first position with col >= j (columns ascend within a row)
    const int32_t mid = (lo + hi) >> 1;
    if (col[mid] < j) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__global__ void __launch_bounds__(256) csc_fill_kernel(const float* __restrict__ adj,
                                                       int64_t n_rows, int64_t n_cols,
                                                       const int32_t* __restrict__ rowptr,
                                                       const int32_t* __restrict__ col,
                                                       const int32_t* __restrict__ colptr,
                                                       const uint8_t* __restrict__ rowflag,
                                                       const int32_t* __restrict__ part,
                                                       int32_t* __restrict__ csc_row,
                                                       int32_t* __restrict__ csc_eid) {
  const int64_t r0 = (int64_t)blockIdx.x * kRowBlock;
  const int64_t r1 = min(n_rows, r0 + kRowBlock);
  for (int64_t j = threadIdx.x; j < n_cols; j += blockDim.x) {
    int32_t slot = colptr[j] + part[blockIdx.x * n_cols + j];
    for (int64_t i = r0; i < r1; ++i) {
      const bool virt = rowflag[i] != 0;
      if (virt || adj[i * n_cols + j] > 0.f) {
        csc_row[slot] = (int32_t)i;
        csc_eid[slot] = virt ? rowptr[i] + (int32_t)j : edge_id(rowptr, col, i, (int32_t)j);
        ++slot;
      }
    }
  }
}

struct GraphWs {
  int32_t* rowcnt;  // n_rows
  int32_t* colcnt;  // n_cols
  int32_t* part;    // nblk * n_cols
  int32_t* scan;    // scan workspace
  int nblk;
};

static size_t graph_ws_layout(int64_t n_rows, int64_t n_cols, void* base, GraphWs* w) {
  const int nblk = (int)((n_rows + kRowBlock - 1) / kRowBlock);
  const size_t scan_n = std::max(scan_ws_ints(n_rows), scan_ws_ints(n_cols));
  size_t off = 0;
  auto take = [&](size_t ints) {
    size_t o = off;
    off += ((ints * 4 + 255) / 256) * 256;
    return o;
  };
  const size_t o_row = take((size_t)n_rows), o_col = take((size_t)n_cols),
               o_part = take((size_t)nblk * (size_t)n_cols), o_scan = take(scan_n);
  if (w) {
    char* b = (char*)base;
    w->rowcnt = (int32_t*)(b + o_row);
    w->colcnt = (int32_t*)(b + o_col);
    w->part = (int32_t*)(b + o_part);
    w->scan = (int32_t*)(b + o_scan);
    w->nblk = nblk;
  }
  return off;
}

// one lane per row: OR of the row's columns (n_cols <= 32)
__global__ void __launch_bounds__(256) rowmask_kernel(const int32_t* __restrict__ rowptr,
                                                      const int32_t* __restrict__ col,
                                                      int64_t n_rows, uint32_t* __restrict__ out) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= n_rows) return;
  uint32_t m = 0;
  for (int32_t e = rowptr[r], e1 = rowptr[r + 1]; e < e1; ++e) m |= 1u << (col[e] & 31);
  out[r] = m;
}

}  // namespace msha

using namespace msha;

extern "C" int msha_graph_rowmask(const msha_graph* g, uint32_t* rowmask, msha_stream_t stream) {
  MSHA_ARG_CHECK(g != nullptr && rowmask != nullptr && g->rowptr != nullptr,
                 "graph_rowmask: null pointer");
  MSHA_ARG_CHECK(g->n_rows > 0 && g->n_cols > 0 && g->n_cols <= 32 && g->n_rows < (1ll << 31),
                 "graph_rowmask: needs 1 <= n_cols <= 32");
  MSHA_ARG_CHECK(g->n_edges == 0 || g->col != nullptr, "graph_rowmask: col missing");
  hipLaunchKernelGGL(rowmask_kernel, dim3((unsigned)((g->n_rows + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, g->rowptr, g->col, g->n_rows, rowmask);
  return check_launch("graph_rowmask");
}

extern "C" int msha_inter_adjacency(const int64_t* source, const int64_t* recipient,
                                    int64_t n_flows, int64_t n_rows, int64_t n_cols, float* adj,
                                    int32_t* counts_ws, msha_stream_t stream) {
  MSHA_ARG_CHECK(n_rows > 0 && n_cols > 0 && n_flows >= 0, "inter_adjacency: bad sizes");
  MSHA_ARG_CHECK(adj && counts_ws && (n_flows == 0 || (source && recipient)),
                 "inter_adjacency: null pointer");
  hipStream_t s = (hipStream_t)stream;
  const int64_t n = n_rows * n_cols;
  if (hipMemsetAsync(counts_ws, 0, (size_t)n * sizeof(int32_t), s) != hipSuccess)
    return check_launch("inter_adjacency memset");
  if (n_flows > 0)
    hipLaunchKernelGGL(count_flows_kernel, dim3(grid_for(n_flows, 256, 8192)), dim3(256), 0, s,
                       source, recipient, n_flows, n_rows, n_cols, counts_ws);
  hipLaunchKernelGGL(counts_to_float_kernel, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s,
                     counts_ws, n, adj);
  return check_launch("inter_adjacency");
}

extern "C" int msha_normalize_adjacency(const float* adj, int64_t n_rows, int64_t n_cols,
                                        float* out, float* col_ws, msha_stream_t stream) {
  MSHA_ARG_CHECK(n_rows > 0 && n_cols > 0, "normalize_adjacency: bad sizes");
  MSHA_ARG_CHECK(adj && out && col_ws, "normalize_adjacency: null pointer");
  hipStream_t s = (hipStream_t)stream;
  const int nblk = (int)((n_rows + kRowBlock - 1) / kRowBlock);
  // col_ws: [d (n_cols)] [bad flag] ; partials live in `out` until the final pass
  // (nblk * n_cols <= n_rows * n_cols always holds).
  float* part = out;
  float* d = col_ws;
  float* bad = col_ws + n_cols;
  if (hipMemsetAsync(bad, 0, sizeof(float), s) != hipSuccess)
    return check_launch("normalize memset");
  hipLaunchKernelGGL(colsum_partial_kernel, dim3(nblk), dim3(256), 0, s, adj, n_rows, n_cols, part);
  hipLaunchKernelGGL(colscale_kernel, dim3(grid_for(n_cols, 256, 4096)), dim3(256), 0, s, part,
                     nblk, n_cols, d, bad);
  hipLaunchKernelGGL(scale_cols_kernel, dim3(grid_for(n_rows * n_cols, 256, 8192)), dim3(256), 0,
                     s, adj, n_rows, n_cols, d, bad, out);
  return check_launch("normalize_adjacency");
}

extern "C" size_t msha_graph_workspace_size(int64_t n_rows, int64_t n_cols) {
  if (n_rows <= 0 || n_cols <= 0) return 0;
  return graph_ws_layout(n_rows, n_cols, nullptr, nullptr);
}

extern "C" int msha_graph_count(const float* adj, int64_t n_rows, int64_t n_cols,
                                int32_t* rowptr, int32_t* colptr, uint8_t* rowflag, void* ws,
                                size_t ws_bytes, msha_stream_t stream) {
  MSHA_ARG_CHECK(n_rows > 0 && n_cols > 0 && n_rows < (1ll << 31) && n_cols < (1ll << 31),
                 "graph_count: bad sizes");
  MSHA_ARG_CHECK(adj && rowptr && colptr && rowflag && ws, "graph_count: null pointer");
  MSHA_ARG_CHECK(ws_bytes >= msha_graph_workspace_size(n_rows, n_cols),
                 "graph_count: workspace too small");
  GraphWs w;
  graph_ws_layout(n_rows, n_cols, ws, &w);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(row_count_kernel, dim3(grid_for(n_rows * kWave, 256, 16384)), dim3(256), 0,
                     s, adj, n_rows, n_cols, w.rowcnt, rowflag);
  hipLaunchKernelGGL(col_count_partial_kernel, dim3(w.nblk), dim3(256), 0, s, adj, n_rows, n_cols,
                     rowflag, w.part);
  hipLaunchKernelGGL(col_block_scan_kernel, dim3(grid_for(n_cols, 256, 4096)), dim3(256), 0, s,
                     w.part, w.nblk, n_cols, w.colcnt);
  exclusive_scan(w.rowcnt, n_rows, rowptr, w.scan, s);
  exclusive_scan(w.colcnt, n_cols, colptr, w.scan, s);
  return check_launch("graph_count");
}

extern "C" int msha_graph_fill(const float* adj, int64_t n_rows, int64_t n_cols,
                               const int32_t* rowptr, const int32_t* colptr,
                               const uint8_t* rowflag, int32_t* col, int32_t* csc_row,
                               int32_t* csc_eid, void* ws, size_t ws_bytes,
                               msha_stream_t stream) {
  MSHA_ARG_CHECK(n_rows > 0 && n_cols > 0, "graph_fill: bad sizes");
  MSHA_ARG_CHECK(adj && rowptr && colptr && rowflag && col && ws, "graph_fill: null pointer");
  MSHA_ARG_CHECK(ws_bytes >= msha_graph_workspace_size(n_rows, n_cols),
                 "graph_fill: workspace too small (pass the msha_graph_count workspace)");
  GraphWs w;
  graph_ws_layout(n_rows, n_cols, ws, &w);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(csr_fill_kernel, dim3(grid_for(n_rows * kWave, 256, 16384)), dim3(256), 0, s,
                     adj, n_rows, n_cols, rowptr, rowflag, col);
  if (csc_row && csc_eid)
    hipLaunchKernelGGL(csc_fill_kernel, dim3(w.nblk), dim3(256), 0, s, adj, n_rows, n_cols, rowptr,
                       col, colptr, rowflag, w.part, csc_row, csc_eid);
  return check_launch("graph_fill");
}
