/*
 * msha_gnn.h -- C ABI of the MI355X (gfx950) MSHA-GNN attention library.
 *
 * The reference (Sienna12321/MSHA--GNN @ 2025-01-17) has no FFI: its hot path is
 * the Python nn.Module surface that train.py / LLP.py call, computed by dense
 * ATen ops.  Each entry point below replaces one dense op chain of that surface;
 * the comment on each cites the reference lines it stands in for.  The Python
 * host layer (msha--gnn_amd/) binds these with ctypes.
 *
 * Conventions
 *   - All pointers are DEVICE pointers to caller-owned, contiguous buffers; the
 *     library never allocates.  Temporary space is passed in as a workspace whose
 *     size a *_workspace_size() query returns.
 *   - Every call is stream-ordered and asynchronous on `stream` (a hipStream_t;
 *     NULL = the legacy default stream).  No host synchronisation, no global
 *     mutable state: calls are re-entrant and graph-capturable.
 *   - Return 0 (MSHA_OK) or a negative MSHA_ERR_* code; msha_last_error() gives a
 *     thread-local message.  No C++ exception crosses the ABI.
 *   - Floating-point buffers are fp32 unless stated.  Node tables are row-major
 *     (rows, heads, feat) with the head index outer; per-edge arrays are
 *     (edges, heads) in CSR edge order.
 *   - Graph = the mask `adj > 0` of an (n_rows x n_cols) adjacency as CSR
 *     (row-major edge order == torch.nonzero order).  A row without edges is
 *     stored as a VIRTUAL FULL ROW (all n_cols columns, rowflag = 1): the
 *     reference's softmax of an all -9e15 row is uniform over every column
 *     (Ablation.py:268-270), and so is the GAL's mask/deg (GAT.py:29-31).
 */
#ifndef MSHA_GNN_H_
#define MSHA_GNN_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MSHA_ABI_VERSION 16

#if defined(__GNUC__) || defined(__clang__)
#define MSHA_API __attribute__((visibility("default")))
#else
#define MSHA_API
#endif

enum {
  MSHA_OK = 0,
  MSHA_ERR_ARG = -1,         /* bad size / null pointer / unsupported shape */
  MSHA_ERR_UNSUPPORTED = -2, /* shape combination without a compiled kernel */
  MSHA_ERR_HIP = -3          /* a HIP runtime call failed (see msha_last_error) */
};

typedef void* msha_stream_t; /* hipStream_t */

/* Storage type of node-feature tables (h, u, v, dU, dV, dh): fp32, or bf16 with
 * fp32 arithmetic (loads widen, stores round to nearest even).  Scores, softmax
 * statistics, per-edge values and their gradients are always fp32. */
enum { MSHA_DTYPE_F32 = 0, MSHA_DTYPE_BF16 = 1 };

/* Graph descriptor.  Built by msha_graph_count / msha_graph_fill from a dense
 * adjacency, or by the caller from its own CSR.  The CSC view and the column
 * chunk plan are needed only by msha_csc_aggregate. */
typedef struct msha_graph {
  int64_t n_rows, n_cols, n_edges;
  const int32_t* rowptr;  /* n_rows + 1 */
  const int32_t* col;     /* n_edges, column of each edge */
  const uint8_t* rowflag; /* n_rows, 1 = virtual full row (nullable: none) */
  const int32_t* colptr;  /* n_cols + 1 (CSC) */
  const int32_t* csc_row; /* n_edges, source row of each CSC slot */
  const int32_t* csc_eid; /* n_edges, CSR edge id of each CSC slot (NULL: the slot IS the
                           * edge id -- a CSR presented as a CSC, msha_csc_aggregate only) */
  /* CSC work split: chunk c covers CSC slots [chunk_start[c], chunk_end[c]) of
   * column chunk_col[c]; a column with more than one chunk is listed in
   * multi_col with its first chunk and chunk count (partials summed in order). */
  int64_t n_chunks;
  const int32_t* chunk_col;
  const int32_t* chunk_start;
  const int32_t* chunk_end;
  int64_t n_multi;
  const int32_t* multi_col;
  const int32_t* multi_first;
  const int32_t* multi_count;
  /* n_edges, CSC slot of each CSR edge (the inverse of csc_eid; nullable).  When set,
   * msha_edge_attention_bwd_fused may keep its per-edge de scratch in CSC slot order
   * (large graphs): the column pass writes it contiguously and the row pass gathers it
   * through this map (ABI 3). */
  const int32_t* csr_slot;
  /* n_rows, graphs with n_cols <= 32 (ABI 13; nullable): bit j of rowmask[i] is set when
   * row i has an edge to column j (virtual full rows: every column).  Built from the CSR
   * by msha_graph_rowmask; the bipartite kernels walk these masks instead of col. */
  const uint32_t* rowmask;
} msha_graph;

/* Same-group adjacency of the full MSHA layer (city and province, dataset.py:260-277
 * builds them as dense N x N masks): group id per node, and per group the sorted
 * member list (CSR: gptr over gmem). */
typedef struct msha_groups {
  int64_t n_nodes;
  const int32_t* gid3;  /* n_nodes: city group of each node */
  const int32_t* gptr3; /* n_city_groups + 1 */
  const int32_t* gmem3; /* n_nodes: members, grouped, ascending */
  const int32_t* gid4;  /* province */
  const int32_t* gptr4;
  const int32_t* gmem4;
  int64_t max_group; /* largest group (either kind): sizes the backward's chunking */
} msha_groups;

MSHA_API int msha_abi_version(void);
MSHA_API const char* msha_last_error(void);
/* Diagnostic (ABI 9): per-wave timeline of the skinny projection / weight-gradient kernels
 * into a device buffer of `slots` x 64 uint64 words (NULL: off).  Only a library built with
 * -DSK_TIMELINE records (build.py --variant timeline); otherwise MSHA_ERR_UNSUPPORTED. */
MSHA_API int msha_debug_timeline(void* buf, int64_t slots);
/* Diagnostic: the model head's split backward row pass (head_bwd_rows2) stamps per-block
 * marks into buf (>= 2048 x 64 uint64, device memory; NULL removes it).  Same build
 * condition as msha_debug_timeline. */
MSHA_API int msha_debug_head_timeline(void* buf);
/* Diagnostic: the MFMA bipartite kernels (edge_bip3.hip) stamp per-wave marks into buf
 * (slots x 64 uint64 words, device memory: forward waves in the first half of the slots,
 * backward waves in the second; NULL removes it).  Same build condition. */
MSHA_API int msha_debug_bip_timeline(void* buf, int64_t slots);

/* ---------------------------------------------------------------- dropout --- */
/* Dropout under HIP-graph replay.  Every dropout draw of the library is Philox4x32-10
 * keyed on (seed, offset, element); seeds are kernel arguments, so a captured graph
 * would replay the same masks.  With a device counter installed here (a uint64 in
 * device memory, NULL = none), each draw adds (*counter << 32) to its offset, read on
 * the device at draw time: the caller increments *counter inside the captured region
 * and every replay draws fresh masks.  One slot per device: a launch on a stream of
 * device d uses device d's counter (device < 0: the current device).  Set it before the
 * launches it should apply to (launch-time snapshot of the pointer, not the value). */
MSHA_API int msha_set_rng_counter(int32_t device, const uint64_t* counter);
/* the counter installed for `device` (< 0: current device), NULL if none */
MSHA_API const uint64_t* msha_get_rng_counter(int32_t device);
/* (ABI 15) A replayed step's feed: copies `bytes` from src to dst (device memory) and adds 1
 * to *counter (NULL: no counter) in ONE stream-ordered launch, so a graph whose counter
 * increment is left to its feed (msha_gnn_amd.step.GraphedStep.replay(feed=...)) starts
 * with its first kernel instead of an add node. */
MSHA_API int msha_feed_step(void* dst, const void* src, int64_t bytes, uint64_t* counter,
                            msha_stream_t stream);

/* keep[i] = 1 iff element i survives F.dropout(p) under (seed, offset).  The
 * kernels below draw exactly these masks (stream-ordered Philox4x32-10), which
 * is how tests inject the same mask into the CPU oracle. */
MSHA_API int msha_dropout_keep_mask(uint64_t seed, uint64_t offset, int64_t n, float p, uint8_t* keep,
                           msha_stream_t stream);

/* ------------------------------------------------------- graph ingestion --- */
/* dataset.py:279-288 (HigherDataset.inter_adjacent): adj[source[k], recipient[k]] += 1.
 * Counts are accumulated exactly in int32 (workspace: n_rows*n_cols int32). */
MSHA_API int msha_inter_adjacency(const int64_t* source, const int64_t* recipient, int64_t n_flows,
                         int64_t n_rows, int64_t n_cols, float* adj, int32_t* counts_ws,
                         msha_stream_t stream);

/* model.py:95-100 (normalize_adjacency_matrix): out = (adj * d) * d, d = colsum^-1/2;
 * a zero column sum spreads NaN to every entry, as the reference's two mm's do.
 * Workspace: n_cols + 1 floats. */
MSHA_API int msha_normalize_adjacency(const float* adj, int64_t n_rows, int64_t n_cols, float* out,
                             float* col_ws, msha_stream_t stream);

/* Ablation.py:268 / GAT.py:30 mask `adj > 0` -> CSR + CSC.  Two phases: count
 * (row/column degrees incl. virtual rows, rowptr/colptr scans), then the caller
 * reads rowptr[n_rows] (= n_edges), allocates, and fills.  Deterministic:
 * CSC slots of a column are in ascending row order. */
MSHA_API size_t msha_graph_workspace_size(int64_t n_rows, int64_t n_cols);
MSHA_API int msha_graph_count(const float* adj, int64_t n_rows, int64_t n_cols, int32_t* rowptr,
                     int32_t* colptr, uint8_t* rowflag, void* ws, size_t ws_bytes,
                     msha_stream_t stream);
/* rowmask[i] = OR over row i's CSR edges of (1 << col) for a graph with n_cols <= 32
 * (g->rowptr, g->col; g->rowmask is not read).  ABI 13. */
MSHA_API int msha_graph_rowmask(const msha_graph* g, uint32_t* rowmask, msha_stream_t stream);
MSHA_API int msha_graph_fill(const float* adj, int64_t n_rows, int64_t n_cols, const int32_t* rowptr,
                    const int32_t* colptr, const uint8_t* rowflag, int32_t* col,
                    int32_t* csc_row, int32_t* csc_eid, void* ws, size_t ws_bytes,
                    msha_stream_t stream);

/* --------------------------------------------------------- attention core --- */
/* Fused edge score + per-row segmented softmax + attention-weighted gather.
 * Replaces Ablation.py:266-271,274 (OursLayer3: e12 = lrelu(cat(h1_j,h2_i) @ a),
 * where/softmax/dropout, u = att @ h1), per head h:
 *   s_e   = lrelu(el[i,h] + er[j,h], neg_slope)      (0 on virtual rows)
 *   att_e = softmax over row i of s
 *   u[i]  = sum_e dropout(att_e) * hc[j]             hc: (n_cols, heads, feat)
 * Outputs u (n_rows, heads, feat), lse (n_rows, heads) = log-sum-exp of the row's
 * scores (the backward recomputes att from it) and, if attd != NULL, the
 * post-dropout attention (n_edges, heads).  u_lo (nullable, bf16 tables only): the
 * rounding residual of the bf16 u (u32 - bf16(u32), stored bf16); the backward's
 * D = dU . u then reads u + u_lo, so a degree-1 row's d_el stays ~0 instead of
 * carrying the 2^-9 rounding of u.
 * Supported (heads, feat): heads in {1,2,4,8}, feat in {8,16,32,64,128} (see
 * msha_edge_attention_supported).  dtype (MSHA_DTYPE_*) is the storage type of the
 * tables hc / u (and hs, dU, dV, d_hs, table, out below); fp32 arithmetic either way. */
MSHA_API int msha_edge_attention_supported(int32_t heads, int32_t feat);
MSHA_API int msha_edge_attention_fwd(const msha_graph* g, int32_t heads, int32_t feat,
                                     int32_t dtype, const float* el, const float* er,
                                     const void* hc, float neg_slope, float drop_p,
                                     uint64_t seed, uint64_t offset, void* u, void* u_lo,
                                     float* lse, float* attd, msha_stream_t stream);
/* The same forward that also writes the row terms of the fused backward (ABI 8), with
 * c_ij = lrelu'(el_i + er_j) (1 when > 0, else neg_slope):
 *   uc (n_rows, heads, feat) fp32 = sum_j c_ij attd_ij hc[j]   (attd: post-dropout)
 *   qc (n_rows, heads)       fp32 = sum_j c_ij att_ij          (att: pre-dropout)
 * so d_el_i = dU_i . uc_i - D_i qc_i (D_i = dU_i . u_i) needs no per-edge de in CSR
 * order.  uc and qc together or both NULL (= msha_edge_attention_fwd).  Needs the
 * batched forward (MSHA_ERR_UNSUPPORTED otherwise); msha_edge_attention_rowterms_preferred
 * says whether a graph should use them (once the per-edge de of
 * msha_edge_attention_bwd_fused would leave the Infinity Cache, and for fp32 tables on
 * graphs whose rows average >= 8 edges). */
MSHA_API int msha_edge_attention_rowterms_preferred(const msha_graph* g, int32_t heads,
                                                    int32_t feat, int32_t dtype);
MSHA_API int msha_edge_attention_fwd_ex(const msha_graph* g, int32_t heads, int32_t feat,
                                        int32_t dtype, const float* el, const float* er,
                                        const void* hc, float neg_slope, float drop_p,
                                        uint64_t seed, uint64_t offset, void* u, void* u_lo,
                                        float* lse, float* attd, float* uc, float* qc,
                                        msha_stream_t stream);

/* Row half of the backward (autograd of the chain above; Ablation.py:266-274):
 *   g_e  = dU[i]·hc[j] (+ dV[j]·hs[i] when dV != NULL: the v = att^T @ h2 branch,
 *          Ablation.py:273)
 *   ds_e = att_e * (drop(g_e) - sum_row att*drop(g)),  de_e = ds_e * lrelu'(pre_e)
 * Writes d_el (n_rows, heads) = row sums of de, de (n_edges, heads), attd
 * (n_edges, heads) = post-dropout attention, and d_hs (n_rows, heads, feat) =
 * sum_e attd_e dV[j] when dV != NULL.  The column half (d_er, d_hc) is
 * msha_csc_aggregate over (attd, de).  row_coef (n_rows, heads), nullable: an extra
 * gradient row_coef[i] * exp(attd_e) on the attention of row i -- the full MSHA
 * layer's normaliser sums exp(attention_inter) of its batch rows (Ours.py:84-86).
 * edge_ld: floats between consecutive edges in de / attd (0 = heads); with
 * edge_ld = 2*heads and attd = de + heads the two share one 2H-float record per edge,
 * which msha_csc_aggregate then reads as one 64-B segment (w = attd, x = de).
 * u_lo: the forward's u_lo (nullable; bf16 tables). */
MSHA_API int msha_edge_attention_bwd_rows(const msha_graph* g, int32_t heads, int32_t feat,
                                          int32_t dtype, const float* el, const float* er,
                                          const void* hc, const float* lse, const void* u,
                                          const void* u_lo, const void* dU, const void* hs, const void* dV,
                                          const float* row_coef, float neg_slope, float drop_p,
                                          uint64_t seed, uint64_t offset, float* d_el, float* de,
                                          float* attd, int32_t edge_ld, void* d_hs,
                                          msha_stream_t stream);

/* Bipartite small-M attention (ABI 11): the repo's own adjacency shape, N sources x
 * M recipients with M * heads * feat <= 4096 (M = 32 at 2 heads x 64: every shipped
 * year).  The column side (hc, er, dV) stays in LDS and the column reductions run in
 * per-wave LDS slabs beside the row work, so one launch (+ a block-partial reduce)
 * replaces msha_edge_attention_fwd + msha_csc_aggregate (v) and one replaces
 * msha_edge_attention_bwd_rows + msha_csc_aggregate (d_hc, d_er).  Deterministic (wave
 * and block order), no atomics; the rows of g must have distinct columns (every CSR the
 * library builds does).  Reference: Ablation.py:266-274, Ours.py:84-86.
 *   fwd: u, lse, attd (nullable), v = attd^T hs (hs, v: both or neither).  u_lo as in
 *        msha_edge_attention_fwd.  Same dropout stream (element e * heads + h).
 *   bwd: d_el, d_er, d_hc, and with dV: d_hs = attd dV (hs, dV, d_hs together);
 *        row_coef (nullable) as in msha_edge_attention_bwd_rows.  No u / u_lo needed:
 *        D_i = sum_e attd_e g_e.
 * ws: msha_bip_workspace_size bytes (block partials; fwd needs it only with hs). */
MSHA_API int msha_bip_supported(const msha_graph* g, int32_t heads, int32_t feat, int32_t dtype);
MSHA_API size_t msha_bip_workspace_size(const msha_graph* g, int32_t heads, int32_t feat);
MSHA_API int msha_bip_attention_fwd(const msha_graph* g, int32_t heads, int32_t feat,
                                    int32_t dtype, const float* el, const float* er,
                                    const void* hc, const void* hs, float neg_slope,
                                    float drop_p, uint64_t seed, uint64_t offset, void* u,
                                    void* u_lo, float* lse, float* attd, void* v, void* ws,
                                    size_t ws_bytes, msha_stream_t stream);
MSHA_API int msha_bip_attention_bwd(const msha_graph* g, int32_t heads, int32_t feat,
                                    int32_t dtype, const float* el, const float* er,
                                    const void* hc, const float* lse, const void* dU,
                                    const void* hs, const void* dV, const float* row_coef,
                                    float neg_slope, float drop_p, uint64_t seed,
                                    uint64_t offset, float* d_el, float* d_er, void* d_hc,
                                    void* d_hs, void* ws, size_t ws_bytes,
                                    msha_stream_t stream);
/* The source-row count from which msha_bip_attention_fwd / _bwd take the MFMA row-mask
 * kernels (graphs with msha_graph.rowmask, 2 heads x 64; below it the mask forward and the
 * CSR-walk backward; default 131072, or MSHA_BIP2_BWD_MIN_ROWS): rows >= 0 sets it for
 * the process and returns the previous value, rows < 0 only returns it. */
MSHA_API int64_t msha_bip2_bwd_min_rows(int64_t rows);
/* (ABI 15) The Ours intra forward's dropout draws: mode 1 packs the matched (batch entry,
 * node) pairs of consecutive nodes into one Philox draw per <= 64 pairs (default), mode 0
 * draws per node for the whole batch (MSHA_OURS_PACK_DRAWS=0 starts with it); both give
 * the same bits.  Returns the previous mode; mode < 0 only queries. */
MSHA_API int32_t msha_ours_pack_draws(int32_t mode);
/* (ABI 15) The fp32 weight gradient's kernel (projection backward, dW = X^T D'): mode 0 =
 * auto (default: from 131,072 rows -- MSHA_WGRAD_S3_MIN_ROWS -- the operands split into
 * three bf16 terms in registers, six products on the bf16 MFMA; the exact-fp32 MFMA below),
 * 1 = exact-fp32 MFMA, 2 = split-bf16 through LDS images, 3 = the register split at any
 * size (MSHA_WGRAD=fp32 / x3 / s3 start the process with 1 / 2 / 3).  Returns the previous
 * mode; mode < 0 only queries. */
MSHA_API int32_t msha_wgrad_kernel(int32_t mode);

/* Column-side (transposed) aggregate over the CSC view:
 *   out[j]   = sum_{e in col j} w[e] * table[row(e)]   (per head; table (n_rows,heads,feat))
 *   out_x[j] = sum_{e in col j} x[e]                   (when x != NULL)
 * Forward v = attd^T @ h2 (Ablation.py:273) and backward d_hc = attd^T @ dU,
 * d_er = colsum(de).  With heads = 1 and w = the adjacency values it is the GCN
 * SpMM adj^T @ support (model.py:37); on a CSR-as-CSC view (colptr = rowptr,
 * csc_row = col, csc_eid = NULL, chunks over rows) it is adj @ support.
 * edge_ld: floats between consecutive edges in w / x (0 = heads).
 * Long columns are split into chunks whose partial sums are added in a fixed order:
 * deterministic, no atomics. */
MSHA_API size_t msha_csc_aggregate_workspace_size(const msha_graph* g, int32_t heads, int32_t feat);
MSHA_API int msha_csc_aggregate(const msha_graph* g, int32_t heads, int32_t feat, int32_t dtype,
                                const float* w, const float* x, int32_t edge_ld,
                                const void* table, void* out, float* out_x, void* ws,
                                size_t ws_bytes, msha_stream_t stream);

/* Fused backward of u = drop(att) @ hc alone (no v branch, no row coefficients):
 * the same d_el, d_er, d_hc as msha_edge_attention_bwd_rows + msha_csc_aggregate,
 * bitwise, from one pass over the CSC (the column owns hc_j, so dU_i . hc_j comes from
 * the dU[i] gather the column pass makes anyway) plus two light row passes.
 * Replaces the reference's autograd of Ablation.py:266-274 for that case.
 * de (n_edges, heads) fp32: scratch (left holding de in CSR edge order, or in CSC slot
 * order when g->csr_slot is set and de exceeds 192 MB).
 * ws: msha_edge_attention_bwd_fused_workspace_size bytes.  Needs the CSC view with
 * csc_eid.  u_lo: the forward's u_lo (nullable; bf16 tables). */
MSHA_API size_t msha_edge_attention_bwd_fused_workspace_size(const msha_graph* g,
                                                             int32_t heads, int32_t feat);
MSHA_API int msha_edge_attention_bwd_fused(const msha_graph* g, int32_t heads, int32_t feat,
                                           int32_t dtype, const float* el, const float* er,
                                           const void* hc, const float* lse, const void* u,
                                           const void* u_lo, const void* dU, float neg_slope,
                                           float drop_p,
                                           uint64_t seed, uint64_t offset, float* d_el,
                                           float* d_er, void* d_hc, float* de, void* ws,
                                           size_t ws_bytes, msha_stream_t stream);
/* The same with the forward's row terms (uc, qc from msha_edge_attention_fwd_ex, same
 * dropout seed/offset): d_el is finished in the row-statistics pass, the column pass
 * stores no de and no row sum runs (de may be NULL).  uc = qc = NULL: the call above. */
MSHA_API int msha_edge_attention_bwd_fused_ex(
    const msha_graph* g, int32_t heads, int32_t feat, int32_t dtype, const float* el,
    const float* er, const void* hc, const float* lse, const void* u, const void* u_lo,
    const void* dU, float neg_slope, float drop_p, uint64_t seed, uint64_t offset,
    const float* uc, const float* qc, float* d_el, float* d_er, void* d_hc, float* de, void* ws,
    size_t ws_bytes, msha_stream_t stream);

/* Scores from the gathered row (ABI 9).  Every caller of the u = att @ hc path scores
 * the gathered table itself: er[j,h] = hc[j,h,:] . a_r[h,:] (Ablation.py:266-267 --
 * a[:F] against h1_j, the rows u aggregates).  Given a_r ((heads, feat) fp32, 16-byte
 * aligned) instead of er, the forward computes er_j from the row its gather lanes hold
 * (no per-edge er gather: a 4*heads-byte piece that costs a cache line per edge once
 * the er table leaves L2) and the fused backward's column pass recomputes it from hc_j
 * in the same order, so both passes see the same scores bit for bit.  The outputs and
 * their meaning are those of msha_edge_attention_fwd_ex (without attd) and
 * msha_edge_attention_bwd_fused_ex; d_er is still the gradient w.r.t. er (the caller
 * routes it to whatever produced er = hc . a_r).  Supported where
 * msha_edge_attention_row_scores_supported says so (one 16-byte piece per lane:
 * heads*feat*sizeof <= 1024 B; tables under 2 GiB); MSHA_ERR_UNSUPPORTED otherwise. */
MSHA_API int msha_edge_attention_row_scores_supported(const msha_graph* g, int32_t heads,
                                                      int32_t feat, int32_t dtype);
/* whether the library's default is to use them (wherever supported, fp32 and bf16,
 * since round 4); MSHA_ROW_SCORES=0/1 in the environment forces it */
MSHA_API int msha_edge_attention_row_scores_preferred(const msha_graph* g, int32_t heads,
                                                      int32_t feat, int32_t dtype);
MSHA_API int msha_edge_attention_fwd_rs(const msha_graph* g, int32_t heads, int32_t feat,
                                        int32_t dtype, const float* el, const float* ar,
                                        const void* hc, float neg_slope, float drop_p,
                                        uint64_t seed, uint64_t offset, void* u, void* u_lo,
                                        float* lse, float* uc, float* qc, msha_stream_t stream);
MSHA_API int msha_edge_attention_bwd_fused_rs(
    const msha_graph* g, int32_t heads, int32_t feat, int32_t dtype, const float* el,
    const float* ar, const void* hc, const float* lse, const void* u, const void* u_lo,
    const void* dU, float neg_slope, float drop_p, uint64_t seed, uint64_t offset,
    const float* uc, const float* qc, float* d_el, float* d_er, void* d_hc, float* de, void* ws,
    size_t ws_bytes, msha_stream_t stream);

/* ----------------------------------------------- GraphAttentionLayer (GAL) --- */
/* GAT.py:20-35 / Ablation.py:100-115.  The layer's score is constant along a row
 * (it concatenates h_i with itself), so its attention is mask/deg (uniform on
 * virtual rows) and the layer is out = elu(dropout(mask/deg) * h), h (n_rows, n_cols).
 * The bwd returns dh = dout * elu'(z) * dropout(mask/deg). */
MSHA_API int msha_gal_fwd(const msha_graph* g, const float* h, float drop_p, uint64_t seed,
                 uint64_t offset, float* out, msha_stream_t stream);
MSHA_API int msha_gal_bwd(const msha_graph* g, const float* h, const float* dout, float drop_p,
                 uint64_t seed, uint64_t offset, float* dh, msha_stream_t stream);

/* ------------------------------------------------ projections (MFMA, fp32) --- */
/* Ablation.py:262-263 (h1 = R @ W1, h2 = S @ W2), GAT.py:21 (h = input @ W) and the
 * gradients of those products.  C = A @ B with arbitrary element strides
 * (A[m,k] = A[m*sAm + k*sAk], B[k,n] = B[k*sBk + n*sBn]), C row-major with ldc.
 * v_mfma_f32_16x16x4_f32: exact fp32 FMA chains.  splits > 1 splits K over
 * workgroups (for long reductions such as dW = X^T dH over all rows); partial
 * slabs are added in split order (deterministic) and beta (0 or 1) selects
 * C = sum or C += sum.  Workspace: msha_gemm_workspace_size(M, N, splits). */
MSHA_API size_t msha_gemm_workspace_size(int64_t M, int64_t N, int32_t splits);
MSHA_API int msha_gemm_f32(int64_t M, int64_t N, int64_t K, const float* A, int64_t sAm,
                           int64_t sAk, const float* B, int64_t sBk, int64_t sBn, float* C,
                           int64_t ldc, float beta, int32_t splits, void* ws, size_t ws_bytes,
                           msha_stream_t stream);

/* msha_gemm_f32 with the backward of msha_project_scores folded into one operand's
 * loads: operand 0 (A, M x K, K = heads*feat, sAk = 1) or 1 (B, K x N, N = heads*feat,
 * sBn = 1) is read as X + de (x) a [+ de2 (x) a2], i.e. X[r, c] + de[r, c/feat] a[c].
 * dX = (dh + de (x) a) W^T and dW = X^T (dh + de (x) a) without materialising the sum
 * (replaces msha_add_head_outer + msha_gemm_f32).  MSHA_ERR_UNSUPPORTED when the
 * operands cannot take the 16-byte path (then use those two calls). */
MSHA_API int msha_gemm_f32_head_outer(int64_t M, int64_t N, int64_t K, const float* A,
                                      int64_t sAm, int64_t sAk, const float* B, int64_t sBk,
                                      int64_t sBn, float* C, int64_t ldc, float beta,
                                      int32_t splits, void* ws, size_t ws_bytes, int32_t operand,
                                      int32_t heads, int32_t feat, const float* de,
                                      const float* a, const float* de2, const float* a2,
                                      msha_stream_t stream);

/* The projection's whole parameter backward in one pass over the rows (replaces
 * msha_gemm_f32_head_outer with operand 1 + msha_head_colsum, Ablation.py:262-267
 * backward): C = A (B + de (x) a [+ de2 (x) a2]) (dW = X^T dh'), and
 * cs1[n] = sum_k de[k, n / feat] T[k, n], cs2 likewise with de2 (d_al, d_ar with T the
 * forward's h), T laid out as B (row pitch sBk, unit column stride).  beta = 0.  Only
 * the resident-accumulator weight-gradient shape (M = N = 128, K >= 4096, splits >= 16);
 * MSHA_ERR_UNSUPPORTED (nothing launched) otherwise.  cs_ws: at least
 * msha_head_outer_colsum_workspace_size(N) bytes; ws as msha_gemm_f32. */
MSHA_API size_t msha_head_outer_colsum_workspace_size(int64_t N);
MSHA_API int msha_gemm_f32_head_outer_colsum(
    int64_t M, int64_t N, int64_t K, const float* A, int64_t sAm, int64_t sAk, const float* B,
    int64_t sBk, int64_t sBn, float* C, int64_t ldc, int32_t splits, void* ws, size_t ws_bytes,
    int32_t heads, int32_t feat, const float* de, const float* a, const float* de2,
    const float* a2, const float* T, float* cs1, float* cs2, void* cs_ws, size_t cs_ws_bytes,
    msha_stream_t stream);
/* (ABI 15) The same, where T is the projection's own output X W (Ablation.py:262, h = X @ W;
 * A = X^T): cs1[n] = sum_a W[a, n] G[n / feat, a] with G = de^T X accumulated from the rows
 * the weight gradient already reads, so T is never read.  Equal in real arithmetic; in fp32
 * it differs from the T form by T's own rounding.  heads == 2 and the split-bf16
 * weight-gradient kernel (msha_wgrad_kernel mode 0) only; MSHA_ERR_UNSUPPORTED otherwise. */
MSHA_API int msha_gemm_f32_head_outer_colsum_w(
    int64_t M, int64_t N, int64_t K, const float* A, int64_t sAm, int64_t sAk, const float* B,
    int64_t sBk, int64_t sBn, float* C, int64_t ldc, int32_t splits, void* ws, size_t ws_bytes,
    int32_t heads, int32_t feat, const float* de, const float* a, const float* de2,
    const float* a2, const float* W, int64_t ldw, float* cs1, float* cs2, void* cs_ws,
    size_t cs_ws_bytes, msha_stream_t stream);

/* Projection with the attention-score halves fused into its epilogue:
 *   h = X @ W  (M x heads*feat),  el[m,h] = h[m,h,:] . al[h,:],  er[m,h] = h[m,h,:] . ar[h,:]
 * Replaces Ablation.py:262-267's projection + the (N, M, 2F) score tensor: the
 * score of edge (i, j) is lrelu(el_i + er_j).  al/el and ar/er are optional pairs;
 * feat must be 4, 8, 16, 32, 64 or 128 when a score vector is given. */
/* 1 when msha_project_scores(_bf16) / msha_project_small at this shape compute el / er
 * from the STORED h in the order the row-score edge kernels recompute er_j = h_j . a_r
 * from a gathered row (per 16-byte piece: last element first, fma downwards; then the
 * xor tree over the head's pieces): er is then bit-identical to that recomputation and
 * msha_edge_attention_bwd_fused_ex may read it in place of msha_edge_attention_bwd_fused_rs
 * (ABI 9: every projection path; feat a multiple of 4). */
MSHA_API int msha_project_scores_row_order(int64_t M, int64_t K, int32_t heads, int32_t feat,
                                           int32_t dtype);
MSHA_API int msha_project_scores(int64_t M, int64_t K, int32_t heads, int32_t feat,
                                 const float* X, const float* W, const float* al,
                                 const float* ar, float* h, float* el, float* er,
                                 msha_stream_t stream);

/* bf16 projections (config C3: the same model in bf16), v_mfma_f32_16x16x32_bf16 with
 * fp32 accumulation.  A, B bf16 with element strides as msha_gemm_f32; each operand
 * needs one unit stride (its extent along it a multiple of 8; the other stride a
 * multiple of 8; 16-byte aligned base), else MSHA_ERR_UNSUPPORTED.  C (ldc, N
 * multiples of 8) is fp32 or bf16 (c_dtype).  ho_operand 0 / 1 reads A / B as
 * X + de (x) a [+ de2 (x) a2] (as msha_gemm_f32_head_outer; feat % 8 == 0, A
 * k-contiguous / B n-contiguous), -1 = none.  splits > 1: deterministic split-K with
 * an fp32 slab workspace of msha_gemm_bf16_workspace_size(M, N, splits) bytes. */
MSHA_API size_t msha_gemm_bf16_workspace_size(int64_t M, int64_t N, int32_t splits);
MSHA_API int msha_gemm_bf16(int64_t M, int64_t N, int64_t K, const void* A, int64_t sAm,
                            int64_t sAk, const void* B, int64_t sBk, int64_t sBn, void* C,
                            int64_t ldc, int32_t c_dtype, int32_t splits, void* ws,
                            size_t ws_bytes, int32_t ho_operand, int32_t heads, int32_t feat,
                            const float* de, const float* a, const float* de2, const float* a2,
                            msha_stream_t stream);
/* msha_project_scores on bf16 X (M x K) and W (K x heads*feat): h bf16, el / er fp32
 * from the fp32 accumulators.  K, heads*feat multiples of 8. */
MSHA_API int msha_project_scores_bf16(int64_t M, int64_t K, int32_t heads, int32_t feat,
                                      const void* X, const void* W, const float* al,
                                      const float* ar, void* h, float* el, float* er,
                                      msha_stream_t stream);

/* out = dh + de (x) a [+ de2 (x) a2]  (rows x heads*feat; de (rows, heads), a (heads, feat)):
 * the gradient reaching h through el = h . a (the backward of msha_project_scores). */
MSHA_API int msha_add_head_outer(int64_t rows, int32_t heads, int32_t feat, const float* dh,
                                 const float* de, const float* a, const float* de2,
                                 const float* a2, float* out, msha_stream_t stream);

/* Gradient of the score vectors of msha_project_scores (el = h . al):
 * out1[h, f] = sum_r s1[r, h] h[r, h, f] (and out2 with s2); deterministic row-block
 * partials.  Workspace: msha_head_colsum_workspace_size(rows, heads, feat). */
MSHA_API size_t msha_head_colsum_workspace_size(int64_t rows, int32_t heads, int32_t feat);
MSHA_API int msha_head_colsum(int64_t rows, int32_t heads, int32_t feat, int32_t dtype,
                              const float* s1, const float* s2, const void* T, float* out1,
                              float* out2, void* ws, size_t ws_bytes, msha_stream_t stream);

/* bf16 link scoring (config C5 names a bf16 embedding table): msha_pair_inner_fwd and
 * msha_pair_linear on bf16 tables G / G2 (and a bf16 nn.Linear weight W); fp32
 * products and accumulation, fp32 scores out.  feat / K, N multiples of 8. */
MSHA_API int msha_pair_inner_fwd_bf16(int64_t n_pairs, int32_t feat, const void* G, int64_t ldg,
                                      const int64_t* gi, const void* G2, int64_t ldg2,
                                      const int64_t* gj, float* out, msha_stream_t stream);
MSHA_API int msha_pair_linear_bf16(int64_t n_pairs, int64_t K, int64_t N, const void* G,
                                   int64_t ldg, const int64_t* gi, const void* G2, int64_t ldg2,
                                   const int64_t* gj, const void* W, const float* bias,
                                   int32_t act, float drop_p, uint64_t seed, uint64_t offset,
                                   float* out, msha_stream_t stream);
/* The same with the output dtype chosen (MSHA_DTYPE_F32 or MSHA_DTYPE_BF16): a bf16
 * LinkPredictor in PyTorch returns bf16 scores, and the (n_pairs, N) output is the
 * dominant byte stream of the scorer.  The epilogue (bias, ReLU, dropout, sigmoid) runs
 * in fp32 and rounds once. */
MSHA_API int msha_pair_linear_bf16_ex(int64_t n_pairs, int64_t K, int64_t N, const void* G,
                                      int64_t ldg, const int64_t* gi, const void* G2,
                                      int64_t ldg2, const int64_t* gj, const void* W,
                                      const float* bias, int32_t act, float drop_p,
                                      uint64_t seed, uint64_t offset, int32_t out_dtype,
                                      void* out, msha_stream_t stream);

/* ------------------------------------------------- BatchNorm + LeakyReLU --- */
/* Ablation.py:273-274 / Ours.py:100-101 epilogue: y = lrelu(bn(x)) on (rows, channels)
 * tables (dtype fp32 / bf16; weight, bias, statistics fp32; weight / bias nullable =
 * 1 / 0).  training != 0: batch statistics (mean, invstd = 1/sqrt(var_biased + eps)
 * written to mean / invstd), running_mean / running_var (nullable pair) updated with
 * momentum and the unbiased variance, as torch.nn.BatchNorm1d; training == 0: the
 * running statistics normalise.  Deterministic (fixed-order Welford / Chan combines).
 * Backward (training statistics): dx, dweight = sum dz xhat, dbias = sum dz with
 * dz = dy lrelu'(z).  Workspace: msha_bn_workspace_size(rows, channels) (0 for
 * rows <= 256: one workgroup). */
MSHA_API size_t msha_bn_workspace_size(int64_t rows, int32_t channels);
MSHA_API int msha_bn_lrelu_fwd(int64_t rows, int32_t channels, int32_t dtype, const void* x,
                               const float* weight, const float* bias, float eps, float slope,
                               int32_t training, float momentum, float* running_mean,
                               float* running_var, float* mean, float* invstd, void* y,
                               void* ws, size_t ws_bytes, msha_stream_t stream);
MSHA_API int msha_bn_lrelu_bwd(int64_t rows, int32_t channels, int32_t dtype, const void* x,
                               const void* dy, const float* weight, const float* bias,
                               const float* mean, const float* invstd, float slope, void* dx,
                               float* dweight, float* dbias, void* ws, size_t ws_bytes,
                               msha_stream_t stream);

/* ----------------------------------------------------------- link scoring --- */
/* LLP.py:104-115 LinkPredictor with the caller's gather (LLP.py:233) fused:
 * x_i = G[gi[b]], x_j = G2[gj[b]] (gi / gj NULL: row b).
 * 'mlp' layer: out = act((x_i * x_j) @ W^T + bias), W an nn.Linear weight (N x K);
 * with G2 == NULL and gj == NULL the input is x_i alone (deeper predictor layers);
 * act bits: 1 bias, 2 relu, 4 dropout(drop_p, seed, offset), 8 sigmoid.
 * g_rows / g2_rows: the row counts of G / G2 (every gi / gj index below them; 0 =
 * unknown).  Known counts whose tables fit 4 GiB select the gather kernel with 32-bit
 * buffer offsets (an index outside [0, rows) then reads zeros: negative indices are not
 * wrapped as torch indexing would wrap them, so callers pass valid indices). */
MSHA_API int msha_pair_linear(int64_t n_pairs, int64_t K, int64_t N, const float* G, int64_t ldg,
                              const int64_t* gi, const float* G2, int64_t ldg2,
                              const int64_t* gj, int64_t g_rows, int64_t g2_rows,
                              const float* W, const float* bias, int32_t act,
                              float drop_p, uint64_t seed, uint64_t offset, float* out,
                              msha_stream_t stream);
/* 'inner': out[b] = sigmoid(sum_f x_i[b,f] x_j[b,f]); feat a power of two in [4, 256]. */
MSHA_API int msha_pair_inner_fwd(int64_t n_pairs, int32_t feat, const float* G, int64_t ldg,
                                 const int64_t* gi, const float* G2, int64_t ldg2,
                                 const int64_t* gj, float* out, msha_stream_t stream);
/* 'inner' with the gathered tables' row counts (ABI 14): a pair whose gi / gj index lies
 * outside [0, g_rows) / [0, g2_rows) scores NaN and sets *err = 1 (err nullable) instead
 * of reading past the table.  dtype MSHA_DTYPE_F32 (feat in [4, 256]) or
 * MSHA_DTYPE_BF16 (feat in [8, 512]); replaces the gather of LLP.py:233 + LLP.py:112-115. */
MSHA_API int msha_pair_inner_fwd_ex(int64_t n_pairs, int32_t feat, int32_t dtype, const void* G,
                                    int64_t ldg, const int64_t* gi, int64_t g_rows,
                                    const void* G2, int64_t ldg2, const int64_t* gj,
                                    int64_t g2_rows, int32_t* err, float* out,
                                    msha_stream_t stream);
/* Index validation of a pair batch before a fused gather (LLP.py:233: torch's h[idx]
 * raises for idx outside [-rows, rows) and wraps a negative idx to rows + idx): flags[0]
 * is set to 1 when any gi (gj) lies outside [-g_rows, g_rows) ([-g2_rows, g2_rows)),
 * flags[1] when any is negative.  flags (2 x int32, device) are OR-ed into, never
 * cleared: the caller zeroes them.  gi / gj nullable. */
MSHA_API int msha_pair_index_check(int64_t n_pairs, const int64_t* gi, int64_t g_rows,
                                   const int64_t* gj, int64_t g2_rows, int32_t* flags,
                                   msha_stream_t stream);
/* backward of 'inner' given its output s: dx_i = dout*s*(1-s)*x_j, dx_j = ...*x_i */
MSHA_API int msha_pair_inner_bwd(int64_t n_pairs, int32_t feat, const float* G, int64_t ldg,
                                 const int64_t* gi, const float* G2, int64_t ldg2,
                                 const int64_t* gj, const float* s, const float* dout,
                                 float* dxi, float* dxj, msha_stream_t stream);
/* backward through y = [sigmoid](dropout(relu(z))) given its output y: dz */
MSHA_API int msha_pair_mlp_dz(int64_t n, const float* s, const float* dout, float drop_p,
                              int32_t sigmoid, float* dz, msha_stream_t stream);
/* x = x_i * x_j (dx == NULL), or dx_i = dx * x_j, dx_j = dx * x_i */
MSHA_API int msha_pair_hadamard(int64_t n_pairs, int32_t feat, const float* G, int64_t ldg,
                                const int64_t* gi, const float* G2, int64_t ldg2,
                                const int64_t* gj, const float* dx, float* x_or_dxi, float* dxj,
                                msha_stream_t stream);

/* LinkPredictor with a predictor string other than 'mlp' / 'inner' (LLP.py:104-115 takes
 * neither branch): y = sigmoid(x_i * x_j), (B, F).  dy == NULL: forward into y_or_dxi;
 * else the backward from the forward's y: dx_i into y_or_dxi, dx_j into dxj. */
MSHA_API int msha_pair_hadamard_sigmoid(int64_t n_pairs, int32_t feat, const float* G,
                                        int64_t ldg, const int64_t* gi, const float* G2,
                                        int64_t ldg2, const int64_t* gj, const float* y,
                                        const float* dy, float* y_or_dxi, float* dxj,
                                        msha_stream_t stream);

/* ----------------------------------------------- full MSHA layer (Ours.py) --- */
/* Intra-source attention of a batch (Ours.py:71-101) on top of the inter forward:
 *   e3_b = lrelu(h2[src_b] . a3s), E3 = exp(e3_b); e4/E4 with a4s (a3s = a3[:F] + a3[F:])
 *   SUM_b = |city(src_b)| E3 + |prov(src_b)| E4 + sum_j exp(attd[src_b, j]) (all M columns)
 *   u_out[n] = u_inter[n] + sum_{b: same city} drop E3/SUM h2[src_b]
 *                         + sum_{b: same province} drop E4/SUM h2[src_b]
 * (per head; heads*feat <= 512).  el/er/lse are the inter forward's.  bstat (B, heads, 8)
 * keeps the per-batch statistics for the backward.  Dropout of att3/att4 uses Philox
 * offsets offset+1+2h / offset+2+2h on the dense (B, N) index. */
MSHA_API int msha_ours_intra_fwd(const msha_graph* g, const msha_groups* grp, int64_t B,
                                 const int64_t* src, int32_t heads, int32_t feat, int32_t dtype,
                                 const void* h2, const float* a3s, const float* a4s,
                                 const float* el, const float* er, const float* lse,
                                 const void* u_inter, float neg_slope, float drop_p,
                                 uint64_t seed, uint64_t offset, float* bstat, void* u_out,
                                 msha_stream_t stream);
/* Backward, two stages around msha_edge_attention_bwd_rows:
 *   stage 0: G (B, 2, heads*feat) = group sums of dropout * dU; bgrad (B, heads, 4);
 *            row_coef (n_rows, heads; written in full) = dL/dSUM at the batch rows, 0
 *            elsewhere;
 *            da3s, da4s (heads, feat).
 *   stage 1: d_hs[src_b] += the intra gradient of h2's batch rows.
 * Per-row sums follow batch order (deterministic).  Stage 0 needs a workspace of
 * msha_ours_workspace_size(grp, B, heads, feat) bytes (chunked group sums). */
MSHA_API size_t msha_ours_workspace_size(const msha_groups* grp, int64_t B, int32_t heads,
                                         int32_t feat);
MSHA_API int msha_ours_intra_bwd(const msha_graph* g, const msha_groups* grp, int64_t B,
                                 const int64_t* src, int32_t heads, int32_t feat, int32_t dtype,
                                 const void* h2, const float* a3s, const float* a4s,
                                 const float* bstat, const void* dU, int32_t stage,
                                 float neg_slope, float drop_p, uint64_t seed, uint64_t offset,
                                 float* G, float* bgrad, float* row_coef, float* da3s,
                                 float* da4s, void* d_hs, void* ws, size_t ws_bytes,
                                 msha_stream_t stream);


/* ---- Model head (Ablation.py:273-277 + :298-301, Ours.py:100-109
 * + :163-167): for every row i of the source side
 *   u_out_h = lrelu(bn2_h(u[:, h]))       v_out_h = lrelu(bn1_h(v[:, h]))   (per head h)
 *   x[i]    = dropout(cat_h elu(u_out_h[i] @ v_out_h^T), p_x)               (H*M values)
 *   out[i]  = log_softmax(elu(elu(dropout(mask_i / deg_i, p_att) * (x[i] @ W))))
 * i.e. the heads' BatchNorm + LeakyReLU epilogue, u_out @ v_out.T, elu, the heads'
 * concatenation, the model's dropout, the GraphAttentionLayer out_att (its score is
 * constant along a row: attention = mask / deg, 1/M on a virtual full row), the model's
 * elu and log_softmax, in three launches (u statistics partials, statistics finalize +
 * the whole v side, one row pass).  u (N, H, F) and v (M, H, F) are the attention
 * aggregates (dtype storage, fp32 arithmetic), W the out_att weight (H*M, M) fp32,
 * out (N, M) log-probabilities (dtype).  training: batch statistics, running statistics
 * updated as nn.BatchNorm1d (momentum, unbiased variance; the num_batches_tracked
 * counters given are advanced on the device); otherwise running statistics and no dropout.  Dropout: Philox keyed on
 * (seed_x, element i*H*M + k) and (seed_att, element i*M + j), offset 0.
 * stats (4, H*F) fp32 out: u mean, u invstd, v mean, v invstd (the backward's input).
 *
 * Backward (training statistics): given dout (N, M), writes du (N, H, F), dv (M, H, F),
 * dW (H*M, M) fp32 and the per-head BatchNorm weight / bias gradients, and zeroes
 * dzero[0 .. n_zero) (nullable: the out_att score vector's gradient, which is exactly 0).  Rows whose dout
 * is all zero (train.py's nll on out[source_index] touches 64 rows) contribute only
 * through the BatchNorm batch terms and cost one row read.  Deterministic: per-wave
 * partials over ascending row ranges, added in wave order.
 * Limits: heads <= 8, heads*feat <= 512, n_cols <= 256, heads*n_cols <= 512,
 * msha_head_supported() for the LDS budget (backward row pass <= 150 KB per wave). */
#define MSHA_HEAD_MAX_HEADS 8
typedef struct msha_head_params {
  int32_t heads, feat;
  float eps, momentum, slope;                     /* BatchNorm eps / momentum, lrelu slope */
  const float* u_weight[MSHA_HEAD_MAX_HEADS];     /* bn2 of head h (u side), feat each */
  const float* u_bias[MSHA_HEAD_MAX_HEADS];
  float* u_running_mean[MSHA_HEAD_MAX_HEADS];
  float* u_running_var[MSHA_HEAD_MAX_HEADS];
  const float* v_weight[MSHA_HEAD_MAX_HEADS];     /* bn1 of head h (v side) */
  const float* v_bias[MSHA_HEAD_MAX_HEADS];
  float* v_running_mean[MSHA_HEAD_MAX_HEADS];
  float* v_running_var[MSHA_HEAD_MAX_HEADS];
  float* du_weight[MSHA_HEAD_MAX_HEADS];          /* backward outputs (nullable) */
  float* du_bias[MSHA_HEAD_MAX_HEADS];
  float* dv_weight[MSHA_HEAD_MAX_HEADS];
  float* dv_bias[MSHA_HEAD_MAX_HEADS];
  int64_t* num_batches_tracked[2 * MSHA_HEAD_MAX_HEADS]; /* nullable; +1 per training forward */
} msha_head_params;
MSHA_API int msha_head_supported(int64_t n_cols, int32_t heads, int32_t feat);
MSHA_API size_t msha_head_workspace_size(const msha_graph* g, int32_t heads, int32_t feat);
MSHA_API int msha_head_fwd(const msha_graph* g, const msha_head_params* hp, int32_t dtype,
                           const void* u, const void* v, const float* W, int32_t training,
                           float p_x, uint64_t seed_x, float p_att, uint64_t seed_att,
                           float* stats, void* out, void* ws, size_t ws_bytes,
                           msha_stream_t stream);
MSHA_API int msha_head_bwd(const msha_graph* g, const msha_head_params* hp, int32_t dtype,
                           const void* u, const void* v, const float* W, float p_x,
                           uint64_t seed_x, float p_att, uint64_t seed_att, const float* stats,
                           const void* dout, void* du, void* dv, float* dW, float* dzero,
                           int64_t n_zero, void* ws, size_t ws_bytes, msha_stream_t stream);
/* (ABI 16) msha_head_bwd with dout's row flags already computed by its producer
 * (msha_nll_rows_bwd_flags: rflag[i] = row i of dout has a nonzero, wmask[w] bit k = rflag[64w
 * + k]): the backward's own row scan is skipped.  Same outputs, bit for bit. */
MSHA_API int msha_head_bwd_flagged(const msha_graph* g, const msha_head_params* hp,
                                   int32_t dtype, const void* u, const void* v, const float* W,
                                   float p_x, uint64_t seed_x, float p_att, uint64_t seed_att,
                                   const float* stats, const void* dout, const uint8_t* rflag,
                                   const uint64_t* wmask, void* du, void* dv, float* dW,
                                   float* dzero, int64_t n_zero, void* ws, size_t ws_bytes,
                                   msha_stream_t stream);


/* ---- Training loss on gathered rows (train.py:227-229): F.nll_loss(logp[rows], cols),
 * mean reduction, and its backward, one launch each (ABI 8).  logp (N, M) row stride ld,
 * fp32 or bf16 (dtype); rows, cols int64 (B).
 *   msha_nll_rows_fwd: loss[0] = -(1/B) sum_b logp[rows[b], cols[b]]  (fp32)
 *   msha_nll_rows_bwd: dlogp = 0 except dlogp[rows[b], cols[b]] += -gloss[0] / B for b in
 *                      order (repeated pairs accumulate); gloss is a device scalar.
 * An entry outside [0, N) x [0, M) is never read or written (torch raises on it): the
 * forward returns NaN for it (and for B = 0, torch's mean over nothing), the backward
 * skips it.  (ABI 9: the forward takes N, M.) */
MSHA_API int msha_nll_rows_fwd(int64_t N, int64_t M, int64_t B, const int64_t* rows,
                               const int64_t* cols, int32_t dtype, const void* logp, int64_t ld,
                               float* loss, msha_stream_t stream);
MSHA_API int msha_nll_rows_bwd(int64_t N, int64_t M, int64_t B, const int64_t* rows,
                               const int64_t* cols, const float* gloss, int32_t dtype,
                               void* dlogp, int64_t ld, msha_stream_t stream);
/* (ABI 16) the backward that also flags dlogp's nonzero rows for the model head's backward
 * (msha_head_bwd_flagged): rflag (N bytes), wmask (ceil(N / 64) words), both or neither. */
/* (ABI 16) on = 1: the block-partial reduce of the next msha_bip_attention_fwd / _bwd on this
 * host thread is handed to the next msha_ours_intra_fwd / stage 1 of msha_ours_intra_bwd on
 * the same stream, which runs it as extra blocks of its own launch (one graph node fewer each
 * way).  on = 0: separate launches again; a reduce still pending is launched now.  The
 * outputs (v; d_hc, d_er) are complete once the taking launch (or the on = 0 call) is
 * enqueued. */
MSHA_API int msha_bip_defer_reduce(int32_t on);
MSHA_API int msha_nll_rows_bwd_flags(int64_t N, int64_t M, int64_t B, const int64_t* rows,
                                     const int64_t* cols, const float* gloss, int32_t dtype,
                                     void* dlogp, int64_t ld, uint8_t* rflag, uint64_t* wmask,
                                     msha_stream_t stream);

/* ---- Batched segment copies: the models' per-head parameter packing (Ablation.py:262-267,
 * Ours.py:58-75 read W1/W2/a/a3/a4 of every head; one launch stacks them, one scatters
 * their gradients back) and the feature dropout of Sfeatures / Rfeatures
 * (Ablation.py:296-297, Ours.py:161-162) in one launch forward and one backward.
 * For every segment:  dst[r*ldd + c] = (a[r*lda + c] (+ b[r*ldb + c])) * keep(r*cols + c)
 * for r < rows, c < cols; a NULL `a` writes zeros; keep is the dropout factor (0 or
 * 1/(1-p)) when p > 0, else 1: element e = r*cols + c keeps iff word e % 4 of the
 * Philox4x32-10 block (seed; counter {e / 4, offset}) is >= p * 2^32 (one generator call
 * per four elements; msha_dropout_keep_mask4 writes the same mask). */
#define MSHA_MAX_SEGMENTS 32
typedef struct msha_segment {
  const void* a;
  const void* b;
  void* dst;
  int64_t rows, cols, lda, ldb, ldd;
  float p;
  uint64_t seed, offset;
  /* storage types (MSHA_DTYPE_*) of a and b (shared) and of dst; arithmetic is fp32 and
   * a bf16 dst is rounded once (nearest-even), so a segment is also a dtype cast (the
   * bf16 models' parameter / gradient / running-statistics conversions, ABI 8) */
  int32_t a_dtype, dst_dtype;
} msha_segment;
MSHA_API int msha_segments(int32_t n, const msha_segment* segs, msha_stream_t stream);
MSHA_API int msha_dropout_keep_mask4(uint64_t seed, uint64_t offset, int64_t n, float p,
                                     uint8_t* keep, msha_stream_t stream);
/* keep[i] = word `word` (0..3) of the Philox4x32-10 block (seed; counter {i, offset}) >=
 * p * 2^32: the Ours intra masks (att3 / att4 of head h, batch entry b, node n: offset
 * drop_offset + 1 + h / 2, word 2 (h % 2) + kind, i = b * n_nodes + n), for tests. */
MSHA_API int msha_dropout_keep_mask_word(uint64_t seed, uint64_t offset, int64_t n, float p,
                                         int32_t word, uint8_t* keep, msha_stream_t stream);


/* ---- Optimizer step (train.py:207,232: optim.Adam(lr, weight_decay) ... step()) ------ */
/* torch.optim.Adam's update (L2 weight decay, no amsgrad / maximize) for up to
 * MSHA_MAX_ADAM tensors in ONE launch, per element (fp32 arithmetic, bias corrections in
 * double as torch computes them from its step count):
 *   g  = grad (* keep * 1/(1-p) when drop_p > 0) + weight_decay * param
 *   m  = m + (1 - beta1) (g - m);  v = beta2 v + (1 - beta2) g^2
 *   t  = *step + 1;  param -= lr / (1 - beta1^t) * m / (sqrt(v) / sqrt(1 - beta2^t) + eps)
 * in one launch whose last block advances *step (capturable: the step lives on the
 * device, as torch's capturable Adam keeps it).  param, grad, exp_avg, exp_avg_sq share `dtype` (bf16 state for bf16
 * parameters, as torch keeps it), contiguous, n elements.  drop_p > 0 fuses a dropout
 * backward into the gradient read: grad is then the dropout's OUTPUT gradient and keep is
 * msha_segments' flat mask (element e: word e % 4 of the Philox4x32-10 block (drop_seed;
 * counter {e / 4, drop_offset})), so the parameter's own gradient never exists (the
 * feature dropout of Sfeatures, Ablation.py:296, Ours.py:161).  ws: device scratch of
 * msha_adam_workspace_size() bytes, ZERO-FILLED before its first use (the launch's
 * completion ticket, back at zero when the launch ends; stream-ordered reuse). */
#define MSHA_MAX_ADAM 64
typedef struct msha_adam_tensor {
  void* param;
  const void* grad;
  void* exp_avg;
  void* exp_avg_sq;
  float* step;
  int64_t n;
  int32_t dtype;
  float drop_p;
  uint64_t drop_seed, drop_offset;
} msha_adam_tensor;
MSHA_API size_t msha_adam_workspace_size(void);
MSHA_API int msha_adam_step(int32_t n, const msha_adam_tensor* tensors, double lr,
                            double beta1, double beta2, double eps, double weight_decay,
                            void* ws, msha_stream_t stream);

/* ---- Projection of a small node table in one workgroup (the recipient side: R15 has 32
 * recipients; Ablation.py:262, :266-267): h = X @ W (M x N, N = heads*feat) with optional
 * per-head score halves el = h . al, er = h . ar; backward with D = dh + d_el (x) al +
 * d_er (x) ar: dX = D @ W^T, dW = X^T @ D, dal / dar[h, f] = sum_m d_el / d_er[m, h]
 * h[m, h*feat + f] -- one launch each (any output pointer may be NULL).  fp32, M <= 256,
 * K <= 128, heads*feat <= 128 (msha_project_small_supported). */
MSHA_API int msha_project_small_supported(int64_t M, int64_t K, int32_t heads, int32_t feat);
MSHA_API int msha_project_small(int64_t M, int64_t K, int32_t heads, int32_t feat,
                                const float* X, const float* W, const float* al,
                                const float* ar, float* h, float* el, float* er,
                                msha_stream_t stream);
MSHA_API int msha_project_small_bwd(int64_t M, int64_t K, int32_t heads, int32_t feat,
                                    const float* X, const float* W, const float* al,
                                    const float* ar, const float* h, const float* dh,
                                    const float* d_el, const float* d_er, float* dX, float* dW,
                                    float* dal, float* dar, msha_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* MSHA_GNN_H_ */
