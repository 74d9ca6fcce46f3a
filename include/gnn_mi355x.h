/*
 * gnn_mi355x.h -- C-ABI of the MI355X (gfx950) message-passing aggregation library
 * (libgnn_mi355x.so, built from graphneuralnetwork_amd/csrc/ *.hip).
 *
 * Every entry point:
 *   - takes plain device pointers, sizes and a hipStream_t passed as `void*`
 *     (NULL = the null stream); no torch / C++ types cross this boundary;
 *   - never allocates device memory: buffers (outputs, workspaces) are owned and
 *     preallocated by the caller;
 *   - never synchronises the host, except the once-per-graph builders that size their
 *     outputs (gnn_gcn_adjacency_build, gnn_spmm_tasks_build, gnn_column_order,
 *     gnn_xcd_hub_plan_build, gnn_cover_*), which say so;
 *   - enqueues its kernels on `stream` and returns 0 on success, a positive
 *     hipError_t on a launch/runtime failure, or a negative GNN_E_* code when an
 *     argument is rejected before anything is launched. It never throws.
 *
 * Layout conventions (DESIGN.md "Data layout in HBM"):
 *   CSR graph   rowptr int64 [n_rows+1], col int32 [nnz], val fp32 [nnz]
 *               (row = destination/output node, col = source/gathered node,
 *               exactly torch.spmm(adj, X)'s orientation: Y[i] = sum_j adj[i,j] X[j]).
 *   features    fp32 row-major, row stride `ld*` in elements (ld >= feat).
 *
 * Each function names the reference call site it replaces (file:line under
 * kaddly/GraphNeuralNetwork).
 */
#ifndef GNN_MI355X_H_
#define GNN_MI355X_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- error codes (negative = argument rejected, nothing launched) ---- */
#define GNN_OK 0
#define GNN_E_ARG (-1)        /* null pointer / negative size / bad stride          */
#define GNN_E_ALIGN (-2)      /* a pointer is not aligned as the layout requires    */
#define GNN_E_UNSUPPORTED (-3) /* shape outside what the library implements         */
#define GNN_E_EMPTY (-4)      /* random.choices on an empty neighbour set (the reference's
                                 IndexError: Cannot choose from an empty sequence)      */
#define GNN_E_RAGGED (-5)     /* index maps of unequal length (the reference's torch.tensor
                                 ValueError)                                           */
#define GNN_E_NOMEM (-6)      /* host allocation failed                                 */
#define GNN_E_COMM (-7)       /* RCCL not found in the process, or its call failed      */

/* ---- epilogue flags ---- */
#define GNN_EPI_RELU 1u /* y = max(y, 0) after the bias add                          */
#define GNN_EPI_ELU 2u  /* y = y > 0 ? y : expm1(y)   (F.elu, alpha = 1)             */
#define GNN_EPI_ACCUMULATE 4u /* SpMM only: y = y_old + A.X (+ bias) (act) -- second pass
                                 of a split (interior + halo) aggregation             */
#define GNN_EPI_SKIP_EMPTY 8u /* gnn_spmm_csr_tasks_f32 only: rows of a task without edges
                                 are left unwritten (an accumulate pass with no bias /
                                 activation: their output is unchanged anyway)        */

/* Library version, e.g. 100 for 0.1.0. */
int gnn_version(void);

/* Human-readable text for a return code of this library (GNN_E_* or hipError_t). */
const char* gnn_error_string(int code);

/* Build provenance: sha256 (16 hex) of the sources, headers, export map and compile flags the
 * library was built from (graphneuralnetwork_amd/build.py lib_source_stamp). The Python loader
 * refuses a library whose stamp differs from the tree it is loaded from. */
const char* gnn_build_stamp(void);

/* The -D defines of a tuning-variant build (build.build_variant); "" for the product library. */
const char* gnn_build_defines(void);

/*
 * GCN aggregation: Y[r, :] = sum_{e in row r} val[e] * X[col[e], :] (+ bias) (epilogue)
 *
 * Replaces `torch.spmm(adj, support)` + `output + self.bias` at
 * GCN/GCN.py:43-45 (Graph_conv_layer.forward).
 *
 * Rows are scheduled by a row-class plan (gnn_spmm_plan_* below):
 *   small rows (degree <= 1)       small_row/small_col/small_val[n_small]: the
 *                                  single edge resolved (col -1 = no edge);
 *                                  packed many rows per wavefront;
 *   mid rows (1 < degree <= seg_len) mid_row[n_mid]: one wavefront per row;
 *   long rows (degree > seg_len)   long_row[n_long], long_seg_ptr[n_long+1],
 *                                  segments seg_row/seg_begin[n_seg] (segment s
 *                                  ends at min(seg_begin+seg_len, rowptr[row+1])),
 *                                  reduced into partial[n_seg * feat] and merged
 *                                  in a fixed order.
 * mid_row == NULL means "no plan": every row is reduced by one wavefront
 * (n_seg / n_long / n_small are then ignored).
 * flags: GNN_EPI_* ; bias may be NULL.
 */
int gnn_spmm_csr_f32(const int64_t* rowptr, const int32_t* col, const float* val, int64_t n_rows,
                     const float* x, int64_t ldx, int64_t feat, const float* bias, float* y,
                     int64_t ldy, int64_t seg_len, const int32_t* seg_row, const int64_t* seg_begin,
                     int64_t n_seg, const int32_t* long_row, const int32_t* long_seg_ptr,
                     int64_t n_long, const int32_t* small_row, const int32_t* small_col,
                     const float* small_val, int64_t n_small, const int32_t* mid_row,
                     int64_t n_mid, float* partial, uint32_t flags, void* stream);

/*
 * gnn_spmm_csr_f32 with hub staging (same aggregation, same plan arguments).
 * The K highest-degree columns of X ("hubs") are copied by the caller into one
 * compact table xh [K, ldh] (gnn_gather_rows_f32 with the hub id list) once per
 * call, and the column array is the graph's hub-remapped copy col_hub: a
 * hub column c with rank k is stored as -1-k, every other column as itself.
 * Hub gathers then hit a few MiB-GiB of contiguous rows instead of rows spread
 * over the whole of X (address-translation reach and Infinity Cache locality).
 * small_col keeps the unremapped ids. Results equal gnn_spmm_csr_f32's.
 * Replaces the same call site: GCN/GCN.py:43-45.
 */
int gnn_spmm_csr_hub_f32(const int64_t* rowptr, const int32_t* col_hub, const float* val,
                         int64_t n_rows, const float* x, int64_t ldx, const float* xh,
                         int64_t ldh, int64_t feat, const float* bias, float* y, int64_t ldy,
                         int64_t seg_len, const int32_t* seg_row, const int64_t* seg_begin,
                         int64_t n_seg, const int32_t* long_row, const int32_t* long_seg_ptr,
                         int64_t n_long, const int32_t* small_row, const int32_t* small_col,
                         const float* small_val, int64_t n_small, const int32_t* mid_row,
                         int64_t n_mid, float* partial, uint32_t flags, void* stream);

/*
 * The same aggregation with short rows in packed row tasks (replaces the same call site,
 * GCN/GCN.py:43-45). task_row int32 [2 * n_task] holds [begin, end) ranges of
 * consecutive rows (at most 63 rows each; every row of a task has degree <= seg_len and
 * is in no other list); one wavefront streams a task's edges, its edge slots taking
 * cost-balanced sub-ranges of the rows, so the rowptr -> col -> X chain is paid once per
 * task instead of once per row. mid_row lists the other rows of degree <= seg_len (one
 * wavefront each), seg_* / long_* the long rows as in gnn_spmm_csr_f32. xh / ldh: the
 * optional hub table (col < 0 names row -1-col of xh, as gnn_spmm_csr_hub_f32; NULL: none).
 * flags: GNN_EPI_* including GNN_EPI_SKIP_EMPTY. Needs feat % 4 == 0 (a row of feat <= 32
 * is held by feat / 4 lanes, 64 / (feat / 4) edge slots per wavefront: the narrow classifier
 * widths), 16-B aligned x / xh / y / bias / partial and ldx, ldh, ldy multiples of 4
 * (else GNN_E_UNSUPPORTED). Each row's sum runs in edge order: deterministic. A task
 * outside the contract (no row, more than 63 rows, rows outside [0, n_rows)) is skipped by
 * the kernel (its rows are left unwritten, nothing is read out of bounds): validate a task
 * list once with gnn_spmm_tasks_check.
 */
int gnn_spmm_csr_tasks_f32(const int64_t* rowptr, const int32_t* col, const float* val,
                           int64_t n_rows, const float* x, int64_t ldx, const float* xh,
                           int64_t ldh, int64_t feat, const float* bias, float* y, int64_t ldy,
                           int64_t seg_len, const int32_t* seg_row, const int64_t* seg_begin,
                           int64_t n_seg, const int32_t* long_row, const int32_t* long_seg_ptr,
                           int64_t n_long, const int32_t* mid_row, int64_t n_mid,
                           const int32_t* task_row, int64_t n_task, float* partial,
                           uint32_t flags, void* stream);

/*
 * Validates a task list of gnn_spmm_csr_tasks_f32 on the device: *err (device int32, zeroed by
 * the caller) gets bit 1 for a task with no row, more than 63 rows or rows outside
 * [0, n_rows), bit 2 for a task that starts before the previous one ends (tasks must be
 * ascending and disjoint). No host sync.
 */
int gnn_spmm_tasks_check(const int32_t* task_row, int64_t n_task, int64_t n_rows, int32_t* err,
                         void* stream);

/*
 * In-degree of every column of a CSR (deg[c] = number of entries with column c, uint32,
 * device), the histogram of gnn_hub_plan_build: LDS-privatised counts for the hottest ids, so
 * the hub columns' counters do not serialise. A column id outside [0, n_cols) sets
 * *err_flag |= 1 (not counted). No host sync. (graph.degree_order's in-degree.)
 */
int gnn_in_degree_u32(const int32_t* col, int64_t nnz, int64_t n_cols, uint32_t* deg,
                      int32_t* err_flag, void* stream);

/*
 * Hub-staging plan for gnn_spmm_csr_hub_f32 / gnn_gat_csr_hub_f32 (built once per graph
 * and hub count k, 1 <= k <= n_cols):
 *   hub_ids[r] (int64 [k]) = the column of in-degree rank r (degree descending, ties by
 *                            ascending column id: deterministic);
 *   col_hub[e] (int32 [nnz]) = -1 - rank(col[e]) for a hub column, col[e] otherwise.
 * A column id outside [0, n_cols) sets *err_flag |= 1 (device int32) and is copied as is.
 * workspace: gnn_hub_plan_workspace_bytes(n_cols) bytes of device memory.
 * New in this library (the reference has no such plan); it serves GCN/GCN.py:43-45 and
 * GAT/models/layers.py:22-37 / :94-131 through the two hub kernels.
 */
int64_t gnn_hub_plan_workspace_bytes(int64_t n_cols);
int gnn_hub_plan_build(const int32_t* col, int64_t nnz, int64_t n_cols, int64_t k,
                       int64_t* hub_ids, int32_t* col_hub, int32_t* err_flag, void* workspace,
                       int64_t workspace_bytes, void* stream);

/*
 * Schedule builders of the default aggregation path (csrc/plan_build.hip). Each one returns
 * the arrays the Python builder named in brackets makes, bit for bit; they synchronise the
 * stream to size their stages (once per graph, never per forward). New in this library: the
 * reference has no plans; they serve GCN/GCN.py:43-45 through the SpMM entries above.
 *
 * gnn_spmm_tasks_build (graph.task_ranges): the packed row tasks of gnn_spmm_csr_tasks_f32 --
 *   maximal runs of consecutive rows of degree <= max_deg, cut every 63 rows and where the
 *   (edges + rows) prefix inside the run crosses a multiple of `cost` (>= 1). *n_task (host)
 *   receives the task count; the [begin, end) pairs go to task_row (int32 [2 * cap_tasks],
 *   device) when task_row is non-null and n_task <= cap_tasks (else GNN_E_ARG with *n_task
 *   set: call again with room for it; n_rows pairs always suffice). Ascending, disjoint,
 *   1..63 rows each (gnn_spmm_tasks_check accepts them). Pass min(max_deg, seg_len).
 *   workspace: gnn_spmm_tasks_workspace_bytes(n_rows) bytes of device memory.
 */
int64_t gnn_spmm_tasks_workspace_bytes(int64_t n_rows);
int gnn_spmm_tasks_build(const int64_t* rowptr, int64_t n_rows, int64_t max_deg, int64_t cost,
                         int32_t* task_row, int64_t cap_tasks, int64_t* n_task, void* workspace,
                         int64_t workspace_bytes, void* stream);

/*
 * gnn_column_order (graph.degree_order(g, rows=False, prefix)): the column relabelling of the
 * column-degree order A P^T. perm[i] (int64 [n_cols]) = the old id of new column i: in-degree
 * descending, ties by ascending id; with 0 <= prefix < n_cols only the first `prefix` ids are
 * ranked and the rest follow in ascending id order (prefix < 0: all ranked). inv[perm[i]] = i;
 * col_out[e] = inv[col[e]] (col_out may be col). Y = (A P^T)(P X) = A X with every row's sum
 * in its CSR order: bit-identical. A column id outside [0, n_cols) -> GNN_E_ARG.
 * workspace: gnn_column_order_workspace_bytes(n_cols) bytes of device memory.
 */
int64_t gnn_column_order_workspace_bytes(int64_t n_cols);
int gnn_column_order(const int32_t* col, int64_t nnz, int64_t n_cols, int64_t prefix,
                     int64_t* perm, int64_t* inv, int32_t* col_out, void* workspace,
                     int64_t workspace_bytes, void* stream);

/*
 * gnn_xcd_hub_plan_build / _fill (graph.xcd_hub_coo + from_coo): the XCD-sliced hub staging
 * of gnn_spmm_csr_hub_f32 / gnn_spmm_csr_tasks_f32 for a column array renamed by
 * gnn_hub_plan_build (col_hub; k hub ranks). The hub ranks are dealt to S = 8 * phases slices
 * in groups of G = 4 consecutive ranks (rank r in slice (r / 4) % S; G = 1 when the item ranks
 * number fewer than 4 S). For every row of degree >= min_deg (>= 2 with small_item >= 2), the edges to
 * the item_k hottest ranks (item_k <= 0: all k) that fall in one slice form a group; groups of
 * >= 2 edges (and, with small_item, rows of degree >= min_deg or groups of >= small_item edges)
 * are cut into ceil(m / chunk) balanced items. Pass 1 ("items") reduces each item into a
 * partial row at a position laid out so that workgroup w (4 waves) holds items of slice
 * w % 8 only; pass 2 ("rest") is every row's unmoved edges in CSR order followed by one edge
 * -1 - (k + position) of value 1.0 per item of the row.
 *   build: counts[4] (host) = n_items, n_pos, nnz_items, nnz_rest; n_items == 0 means no
 *          row has two hub edges in one slice (no plan). chunk >= 4, k >= S, item_k >= S,
 *          8 * phases <= 1024, else GNN_E_ARG.
 *   fill:  with the same workspace, rowptr, col_hub, n_rows, nnz, k, phases and the counts:
 *          items CSR (rowptr int64 [n_pos + 1], col int32 / val fp32 [nnz_items]; a pad
 *          position holds two zero-valued edges of its slice), pos_row (int64 [n_pos]: the
 *          graph row of each position, pads 0) and rest CSR (rowptr int64 [n_rows + 1],
 *          col int32 / val fp32 [nnz_rest]). All device memory.
 * workspace: gnn_xcd_hub_plan_workspace_bytes(n_rows, nnz) bytes of device memory.
 */
int64_t gnn_xcd_hub_plan_workspace_bytes(int64_t n_rows, int64_t nnz);
/* The slice group G the builder was compiled with (4): a caller that needs another grouping
 * builds the arrays itself (graph.xcd_hub_coo restates them). */
int64_t gnn_xcd_slice_group(void);
int gnn_xcd_hub_plan_build(const int64_t* rowptr, const int32_t* col_hub, int64_t n_rows,
                           int64_t nnz, int64_t k, int64_t min_deg, int64_t chunk, int64_t phases,
                           int64_t item_k, int64_t small_item, int64_t* counts, void* workspace,
                           int64_t workspace_bytes, void* stream);
int gnn_xcd_hub_plan_fill(const void* workspace, const int64_t* rowptr, const int32_t* col_hub,
                          const float* val, int64_t n_rows, int64_t nnz, int64_t k, int64_t phases,
                          const int64_t* counts, int64_t* items_rowptr, int32_t* items_col,
                          float* items_val, int64_t* pos_row, int64_t* rest_rowptr,
                          int32_t* rest_col, float* rest_val, void* stream);

/*
 * Edge-cut cover exchange of the N-rank SpMM (distributed.build_cover_exchange; csrc/
 * cover_build.hip), rank `rank` of `world` (<= 64), row blocks bounds[0..world] (host int64,
 * bounds[0] = 0, bounds[world] = n_rows, non-decreasing). Rank p owns rows [b_p, b_{p+1}) of
 * the CSR and of X; each cut edge (i, j) is covered by shipping X_j to p (a feature row) or by
 * the owner q of j computing the partial row sum over its columns (a partial row), per the
 * greedy rule documented there. New in this library (the reference is single-device); it
 * shards GCN/GCN.py:43-45 across ranks with gnn_halo_alltoallv_f32 + the SpMM entries.
 *   gnn_cover_build: counts (host int64 [4 + 3 world]) = interior nnz, requested feature rows,
 *     halo_x nnz, partial rows received, then per peer q: feature rows asked of q, partial
 *     rows asked of q, partial edges handed to q. Synchronises the stream. A column id
 *     outside [0, n_rows) in this rank's rows -> GNN_E_ARG.
 *   gnn_cover_fill (same workspace and arguments + the counts): the interior CSR (local rows x
 *     local columns), xcols (the requested global ids, ascending = grouped by owner), halo_x CSR
 *     (local rows x positions in xcols), the partial edges (pe_i global row, pe_j global
 *     column, pe_v value; grouped by owner q, then row, CSR order inside a row) and halo_p CSR
 *     (local rows x partial-row index, values 1.0).
 *   Handshake (the caller's collectives): all-to-all of the 3 per-peer counts, then
 *     all-to-all-v of xcols (-> the rows this rank sends, minus b_p) and of pe_i / pe_j / pe_v.
 *   gnn_cover_send_partials: from the received partial edges (recv_edges[q] from peer q, host),
 *     the CSR of the partial rows this rank computes for its peers: n_p_send rows (the sum of
 *     the partial rows peers asked of it; another total -> GNN_E_ARG) x local columns.
 * workspaces: gnn_cover_workspace_bytes(n_rows, local nnz, b_{p+1} - b_p, world),
 * gnn_cover_send_workspace_bytes(received partial edges) bytes of device memory.
 */
int64_t gnn_cover_workspace_bytes(int64_t n_rows, int64_t nnz_local, int64_t n_own, int32_t world);
int gnn_cover_build(const int64_t* rowptr, const int32_t* col, int64_t n_rows,
                    const int64_t* bounds, int32_t rank, int32_t world, int64_t* counts,
                    void* workspace, int64_t workspace_bytes, void* stream);
int gnn_cover_fill(const void* workspace, const int64_t* rowptr, const int32_t* col,
                   const float* val, int64_t n_rows, const int64_t* bounds, int32_t rank,
                   int32_t world, const int64_t* counts, int64_t* int_rowptr, int32_t* int_col,
                   float* int_val, int64_t* xcols, int64_t* hx_rowptr, int32_t* hx_col,
                   float* hx_val, int64_t* pe_i, int64_t* pe_j, float* pe_v, int64_t* hp_rowptr,
                   int32_t* hp_col, float* hp_val, void* stream);
int64_t gnn_cover_send_workspace_bytes(int64_t n_edges);
int gnn_cover_send_partials(const int64_t* pe_i, const int64_t* pe_j, const float* pe_v,
                            const int64_t* recv_edges, int32_t world, int64_t r0, int64_t n_own,
                            int64_t n_p_send, int64_t* sp_rowptr, int32_t* sp_col, float* sp_val,
                            void* workspace, int64_t workspace_bytes, void* stream);


/*
 * Row-class plan for gnn_spmm_csr_f32 / gnn_gat_csr_f32 (built once per graph).
 *
 * gnn_spmm_plan_count: classifies the rows and writes four int64 counters into
 *   `counts_dev` (device memory, [4]: n_long, n_seg, n_small, n_mid). The caller
 *   reads them back once (the only host round-trip of a plan: once per graph,
 *   never per forward).
 * gnn_spmm_plan_fill: fills the lists (ascending row order) for those counts.
 *   `scratch` needs gnn_spmm_plan_scratch_bytes(n_rows) bytes and must be the
 *   buffer passed to gnn_spmm_plan_count.
 */
int64_t gnn_spmm_plan_scratch_bytes(int64_t n_rows);
int gnn_spmm_plan_count(const int64_t* rowptr, int64_t n_rows, int64_t seg_len,
                        int64_t* counts_dev, void* scratch, void* stream);
int gnn_spmm_plan_fill(const int64_t* rowptr, const int32_t* col, const float* val, int64_t n_rows,
                       int64_t seg_len, int32_t* seg_row, int64_t* seg_begin, int32_t* long_row,
                       int32_t* long_seg_ptr, int32_t* small_row, int32_t* small_col,
                       float* small_val, int32_t* mid_row, void* scratch, void* stream);

/*
 * GAT attention logits for all heads: el[n,h] = a_src[h,:] . Wh[n, h*fh:(h+1)*fh],
 * er[n,h] = a_dst[h,:] . Wh[n, h*fh:(h+1)*fh]  (a_src/a_dst: [heads*fh]).
 *
 * Replaces the a-products of GAT/models/layers.py:25-26 (dense: a[:F] pairs with
 * the row node, a[F:] with the column node) and :105-108 (sparse: a[:, :F] / a[:, F:]).
 */
int gnn_gat_logits_f32(const float* wh, int64_t ldw, int64_t n_rows, int64_t heads, int64_t fh,
                       const float* a_src, const float* a_dst, float* el, float* er, int64_t lde,
                       void* stream);

/*
 * GCN feature transform on the matrix cores: y[n, :fout] = x[n, :k] @ w^T with w the
 * nn.Linear weight [fout, k] (row-major), fp32 in / fp32 accumulate
 * (v_mfma_f32_16x16x4_f32). Replaces `support = self.dense(X_input)` at GCN/GCN.py:42
 * (inference path). Shapes covered: gnn_gcn_transform_supported(k, fout) != 0
 * (k in {16, 32, 64, 128, 256}; fout 64, 128 or 256);
 * other shapes return GNN_E_UNSUPPORTED (the caller uses a library GEMM). x, w, y
 * 16-B aligned, ldx and ldy multiples of 4 (else GNN_E_ALIGN).
 */
int gnn_gcn_transform_supported(int64_t k, int64_t fout);

/*
 * Arithmetic of the transform entries (gnn_gcn_transform_f32 / _rows_f32, gnn_linear_relu_f32
 * / _cls_f32) at k >= 128, process-wide: mode 1 (the default) forms every fp32 product from
 * bf16 MFMAs -- x and w split into three bf16 pieces each (v = v0 + v1 + v2 to 2^-24
 * relative), the six piece products down to order 2^-16 accumulated in fp32 by
 * v_mfma_f32_16x16x32_bf16 -- an error per product of a few fp32 ulps (tested against the
 * fp32 path and a float64 product); mode 0: v_mfma_f32_16x16x4_f32 (a k-ordered fp32 fmaf
 * chain). k < 128 always takes mode 0; the GAT projection (gnn_gat_project_f32 / _rows_f32)
 * follows the same mode at k = 64. Returns the previous mode, GNN_E_ARG for another value.
 * gnn_transform_get_precision returns the current mode.
 */
int gnn_transform_set_precision(int mode);
int gnn_transform_get_precision(void);
int gnn_gcn_transform_f32(const float* x, int64_t ldx, int64_t n_rows, int64_t k, const float* w,
                          int64_t fout, float* y, int64_t ldy, void* stream);

/*
 * y = dropout(act(x @ w^T + bias)): the dense half of a Graph_conv_layer trained as
 * (A X) W^T + b -- the same layer as GCN/GCN.py:42-45's A (X W^T) + b, reassociated where
 * in_features <= out_features (graphneuralnetwork_amd/ops.py _GcnLayerFn) -- with the ReLU
 * and Dropout that follow it in GCN_Model (GCN/GCN.py:12-14) in the store epilogue. bias: fp32
 * [fout], 16-B aligned (GNN_E_ALIGN), or NULL; act = ReLU when relu != 0; dropout: element
 * (i, c) is kept iff (h >> 8) / 2^24 >= drop_p for h = the 32-bit hash of (drop_seed, i, c)
 * (oracle/spmm_oracle.c oracle_hash3 restates it), kept values scaled by 1 / (1 - drop_p)
 * (inverted dropout, as F.dropout); drop_p in [0, 1) (GNN_E_ARG), 0 = no dropout. Shapes,
 * alignment, arithmetic and return codes as gnn_gcn_transform_f32.
 */
int gnn_gcn_transform_epi_f32(const float* x, int64_t ldx, int64_t n_rows, int64_t k,
                              const float* w, int64_t fout, const float* bias, int32_t relu,
                              float drop_p, uint64_t drop_seed, float* y, int64_t ldy,
                              void* stream);

/*
 * The same product with the output rows scattered: y[y_row[i], :fout] = x[i, :k] @ w^T for
 * i < n_rows (y has n_y rows; x is read in order). With y_row = a degree order's inv (old ->
 * new id) it writes the support of GCN/GCN.py:42 directly in the row order the
 * column-degree-ordered graph A P^T reads it (A P^T . P (X W^T) = A . X W^T:
 * Graph_conv_layer's output rows stay in the original order), so the SpMM gathers its hub
 * rows from the first rows of y with no staging copy. Rows whose id is outside [0, n_y) are
 * not stored and set *err_flag = 1. y_row must not repeat an id (a permutation or another
 * injective map): two rows stored to one output row leave either. Same shapes, alignment and
 * return codes as gnn_gcn_transform_f32.
 */
int gnn_gcn_transform_rows_f32(const float* x, int64_t ldx, int64_t n_rows, int64_t k,
                               const float* w, int64_t fout, float* y, int64_t ldy,
                               const int64_t* y_row, int64_t n_y, int32_t* err_flag,
                               void* stream);

/*
 * Feature row normalisation, bit-exact with the reference loader: normalize_features
 * (GCN/data_utils.py:39-51) then torch.Tensor(features.toarray()) (:81-83). rowsum = the
 * first nonzero of the row plus numpy's float32 pairwise sum of the others (scipy's csr
 * sum = np.add.reduceat); r = rowsum ** -1 in float64, inf -> 0; y = fp32(r * x) in
 * float64, +0.0 where x == 0 or r == 0. x [n_rows, ldx], y [n_rows, ldy] must not
 * overlap; n_cols <= 16384 (else GNN_E_UNSUPPORTED).
 */
int gnn_normalize_features_f32(const float* x, int64_t ldx, int64_t n_rows, int64_t n_cols,
                               float* y, int64_t ldy, void* stream);

/*
 * The same product with a ReLU epilogue: y = max(x @ w^T, 0). Replaces the SageLayer's
 * F.relu(self.weight(torch.cat([self_feats, aggregate_feats], dim=1))) at
 * GraphSAGE/GraphSAGE.py:18-20 (inference; x = the [M, 2F] cat buffer). Same shapes,
 * alignment and return codes as gnn_gcn_transform_f32.
 */
int gnn_linear_relu_f32(const float* x, int64_t ldx, int64_t n_rows, int64_t k, const float* w,
                        int64_t fout, float* y, int64_t ldy, void* stream);

/*
 * gnn_linear_relu_f32 over rows [0, min(*live, n_rows)) only: *live is a DEVICE int64 (a
 * frontier size written by gnn_sample_layers, never read back by the host), n_rows the
 * capacity of x / y. Rows from *live on are neither read nor written. live must not be NULL.
 */
int gnn_linear_relu_live_f32(const float* x, int64_t ldx, int64_t n_rows, const int64_t* live,
                             int64_t k, const float* w, int64_t fout, float* y, int64_t ldy,
                             void* stream);

/*
 * The last SageLayer with the GraphSAGE classifier fused into its epilogue:
 *   y = max(x @ w^T, 0)                      GraphSAGE/GraphSAGE.py:18-20 (the embedding)
 *   logits[n, c] = y[n, :] . wd[c, :] + bd[c]  GraphSAGE.py:51-52 (self.dense, nn.Linear)
 * for c < n_cls <= 4 (wd [n_cls, fout] row-major, bd nullable = no bias; logits row pitch
 * ldl >= n_cls). The per-row sums run in a fixed order (deterministic). Shapes, alignment
 * and return codes as gnn_gcn_transform_f32; GNN_E_ARG for n_cls outside [1, 4].
 */
int gnn_linear_relu_cls_f32(const float* x, int64_t ldx, int64_t n_rows, int64_t k,
                            const float* w, int64_t fout, float* y, int64_t ldy, const float* wd,
                            const float* bd, int64_t n_cls, float* logits, int64_t ldl,
                            void* stream);

/*
 * GAT feature transform on the matrix cores with the attention logits fused:
 *   wh[n, :] = x[n, :k] @ w[k, fout]   (w row-major [k, fout], all heads side by side)
 *   el[n, h] = a_src[h*fh:(h+1)*fh] . wh[n, h*fh:(h+1)*fh], er likewise with a_dst
 * Replaces torch.mm(h, self.W) + the a-products of GAT/models/layers.py:23-26 /
 * :97-108 for the inference path (v_mfma_f32_16x16x4_f32, exact f32; the logits are
 * computed as x (w A) with A the block-diagonal a_src / a_dst matrix, so they match
 * gnn_gat_logits_f32 on wh to fp32 rounding, not bitwise). Shapes:
 * gnn_gat_project_supported(k, fout, fh) != 0 (k in {16,32,64,128,256}, fout in
 * {16,32,64} with (k/4)*(fout/16) <= 64, heads = fout/fh <= 8); otherwise
 * GNN_E_UNSUPPORTED. x / wh rows 16-B aligned (GNN_E_ALIGN). w2_scratch: unused (may be
 * null; each workgroup folds the logit weights w A itself, one launch in all), kept so that
 * existing callers link.
 */
int gnn_gat_project_supported(int64_t k, int64_t fout, int64_t fh);
int gnn_gat_project_f32(const float* x, int64_t ldx, int64_t n_rows, int64_t k, const float* w,
                        int64_t fout, const float* a_src, const float* a_dst, int64_t heads,
                        int64_t fh, float* wh, int64_t ldwh, float* el, float* er, int64_t lde,
                        float* w2_scratch, void* stream);

/*
 * The same with the column side scattered: wh and er of node n go to row col_row[n], el stays
 * at row n -- the operands of the aggregation over a column-degree-ordered graph A P^T
 * (col_row = the order's inv; GAT/models/layers.py:23-26 unchanged in value). el and er must
 * be separate [n_rows, lde] buffers. Rows whose col_row id is outside [0, n_rows) are not
 * stored; col_row must not repeat an id (a permutation).
 */
int gnn_gat_project_rows_f32(const float* x, int64_t ldx, int64_t n_rows, int64_t k,
                             const float* w, int64_t fout, const float* a_src,
                             const float* a_dst, int64_t heads, int64_t fh, float* wh,
                             int64_t ldwh, float* el, float* er, int64_t lde,
                             const int64_t* col_row, float* w2_scratch, void* stream);

/*
 * GAT edge-softmax + neighbour aggregation over CSR, all heads in one pass:
 *   out[i, h*fh+f] = act( sum_{j in row i} p_ijh * Wh[j, h*fh+f] / sum_j p_ijh )
 * mode 0 (dense layer, GAT/models/layers.py:22-37):
 *     p_ijh = exp(LeakyReLU(el_ih + er_jh) - max_j(...))   -- softmax(dim=1)
 *     rows with no edge -> empty_row_fill[h*fh+f] (the reference's uniform
 *     average over all N rows; NULL -> NaN)
 * mode 1 (sparse layer, GAT/models/layers.py:94-131):
 *     p_ijh = exp(-LeakyReLU(el_ih + er_jh))  -- no max subtraction (reference arithmetic)
 *     rows with no edge -> 0/0 = NaN (the reference then fails its isnan assert)
 * dropout_p > 0 (training) drops numerator weights with a hash RNG keyed by
 * (dropout_seed, edge, head) and rescales by 1/(1-p), as F.dropout does.
 * Rows are scheduled by the row-class plan of gnn_spmm_plan_* (small rows packed,
 * mid rows one wave each, long rows in segments with
 * partial[n_seg * (heads*fh + 2*heads)] merged by the log-sum-exp rule);
 * mid_row == NULL: no plan, one wave per row. short_row[n_short] (nullable when
 * n_short == 0): rows taken out of the mid list for the short-row path (64/LPR rows
 * per wave, lane-private softmax; any degree >= 1 is correct, it pays for deg <= 8).
 * flags: GNN_EPI_ELU for concat=True.
 * stats (nullable, [n_rows, heads]): per-(row, head) log-sum-exp of the attention
 * logits (dense: max + log sum exp; sparse: log sum exp(-LeakyReLU)), -inf for an
 * edgeless row -- saved by training forwards for gnn_gat_backward_*.
 */
int gnn_gat_csr_f32(const int64_t* rowptr, const int32_t* col, int64_t n_rows, const float* wh,
                    int64_t ldw, int64_t heads, int64_t fh, const float* el, const float* er,
                    int64_t lde, float negative_slope, int32_t mode, const float* empty_row_fill,
                    float dropout_p, uint64_t dropout_seed, float* out, int64_t ldo,
                    int64_t seg_len, const int32_t* seg_row, const int64_t* seg_begin,
                    int64_t n_seg, const int32_t* long_row, const int32_t* long_seg_ptr,
                    int64_t n_long, const int32_t* small_row, const int32_t* small_col,
                    int64_t n_small, const int32_t* mid_row, int64_t n_mid,
                    const int32_t* short_row, int64_t n_short, float* partial,
                    float* stats, uint32_t flags, void* stream);

/*
 * gnn_gat_csr_f32 with hub staging (same outputs, bit for bit): col_hub is the graph's
 * hub-remapped column array (hub column of rank k stored as -1-k, as for
 * gnn_spmm_csr_hub_f32) and whh [K, ldwh] / erh [K, ldeh] hold the Wh rows and er
 * entries of the K hub columns, copied by the caller (gnn_gather_rows_f32) per call.
 * small_col keeps the unremapped ids. Replaces the same call sites as gnn_gat_csr_f32.
 */
int gnn_gat_csr_hub_f32(const int64_t* rowptr, const int32_t* col_hub, int64_t n_rows,
                        const float* wh, int64_t ldw, int64_t heads, int64_t fh, const float* el,
                        const float* er, int64_t lde, float negative_slope, int32_t mode,
                        const float* empty_row_fill, float dropout_p, uint64_t dropout_seed,
                        float* out, int64_t ldo, int64_t seg_len, const int32_t* seg_row,
                        const int64_t* seg_begin, int64_t n_seg, const int32_t* long_row,
                        const int32_t* long_seg_ptr, int64_t n_long, const int32_t* small_row,
                        const int32_t* small_col, int64_t n_small, const int32_t* mid_row,
                        int64_t n_mid, const int32_t* short_row, int64_t n_short, float* partial,
                        float* stats, uint32_t flags, void* stream, const float* whh,
                        int64_t ldwh, const float* erh, int64_t ldeh);

/*
 * gnn_gat_csr_hub_f32 with the hub tables optional (whh / erh both NULL: no staging, col plain)
 * and an optional a_dst [heads * fh] (the vector er = Wh . a_dst was computed with,
 * GAT/models/layers.py:26-27 / :106): with it the kernels recompute er_j from the Wh_j rows they
 * gather (one-chunk rows, short rows, one-edge rows) instead of loading er -- the er gathers were
 * 0.17 of 0.78 ms at cfg3. er must still be given (the other row paths read it). Outputs equal
 * to the er-gathering form up to the rounding of er's dot products.
 */
int gnn_gat_csr_ex_f32(const int64_t* rowptr, const int32_t* col, int64_t n_rows,
                       const float* wh, int64_t ldw, int64_t heads, int64_t fh, const float* el,
                       const float* er, int64_t lde, float negative_slope, int32_t mode,
                       const float* empty_row_fill, float dropout_p, uint64_t dropout_seed,
                       float* out, int64_t ldo, int64_t seg_len, const int32_t* seg_row,
                       const int64_t* seg_begin, int64_t n_seg, const int32_t* long_row,
                       const int32_t* long_seg_ptr, int64_t n_long, const int32_t* small_row,
                       const int32_t* small_col, int64_t n_small, const int32_t* mid_row,
                       int64_t n_mid, const int32_t* short_row, int64_t n_short, float* partial,
                       float* stats, uint32_t flags, void* stream, const float* whh,
                       int64_t ldwh, const float* erh, int64_t ldeh, const float* a_dst);

/*
 * The same layer with the low-degree rows as packed row tasks (the package's default at fh % 4
 * == 0): task_row [2 n_task] = [begin, end) ranges of <= 63 consecutive rows of degree <= the
 * plan's threshold (edgeless and one-edge rows included; gnn_spmm_tasks_build builds them),
 * mid_row = the rows above the threshold up to seg_len, segments / long rows as above; there is
 * no small / short class. One wave streams a task's edges with a lane-private online softmax per
 * row (same weights and ELU, rounding of a streamed softmax). whh / erh: hub tables (column
 * c < 0 reads row -1-c) or NULL. GNN_E_UNSUPPORTED unless fh % 4 == 0, <= 256 features per
 * group of 8 heads and 16-B aligned rows.
 */
int gnn_gat_csr_tasks_f32(const int64_t* rowptr, const int32_t* col, int64_t n_rows,
                          const float* wh, int64_t ldw, int64_t heads, int64_t fh, const float* el,
                          const float* er, int64_t lde, float negative_slope, int32_t mode,
                          const float* empty_row_fill, float dropout_p, uint64_t dropout_seed,
                          float* out, int64_t ldo, int64_t seg_len, const int32_t* seg_row,
                          const int64_t* seg_begin, int64_t n_seg, const int32_t* long_row,
                          const int32_t* long_seg_ptr, int64_t n_long, const int32_t* mid_row,
                          int64_t n_mid, const int32_t* task_row, int64_t n_task, float* partial,
                          float* stats, uint32_t flags, void* stream, const float* whh,
                          int64_t ldwh, const float* erh, int64_t ldeh);

/*
 * y[n, fout] = x[n, k] w^T (w [fout, k], nn.Linear's layout), fp32, with one side narrow: the
 * classifier layer of GCN_Model in training (GCN/GCN.py:16-17, 42: support = H W^T with 7
 * classes padded to 8, and its backward dH = dS W), where a library GEMM spends 1.6x the HBM
 * time. gnn_linear_small_supported(k, fout): 1 = fout <= 16 and k in {16, 32, 64, 128, 256}
 * (v_mfma_f32_16x16x4_f32: exact fp32 products, fp32 accumulation); 2 = k <= 16 and fout in
 * {64, 128, 256} (fp32 FMAs in k order); 0 = not covered (GNN_E_UNSUPPORTED). x, y 16-B
 * aligned, ldx and ldy multiples of 4 (GNN_E_ALIGN).
 */
int gnn_linear_small_supported(int64_t k, int64_t fout);
int gnn_linear_small_f32(const float* x, int64_t ldx, int64_t n_rows, int64_t k, const float* w,
                         int64_t fout, float* y, int64_t ldy, void* stream);

/*
 * Weight gradients of the training step (GCN/train_eval.py:43-48 through GCN/GCN.py:42,
 * GAT/train_eval.py:75-76 through GAT/models/layers.py:23): C = A^T B summed over the n rows
 * (A [n, m], B [n, k], row strides lda / ldb), written as C [m, k] (trans_c = 0, row stride
 * ldc >= k) or C^T [k, m] (trans_c = 1, ldc >= m); with d != NULL also dsum[k] = the column sums
 * of D [n, k] (the bias gradient, read in the same pass; d == b with ldd == ldb sums B's own
 * loads, no third read, at the split-bf16 wide shapes). Per block of rows the products are
 * accumulated in row order (fp32 FMAs; fp32 or split-bf16 MFMAs at the wide shapes, per
 * gnn_transform_set_precision), the block partials summed in block order (deterministic).
 * gnn_gemm_tn_supported(m, k): 1 = a wide shape (m, k) in {(128,128), (64,64), (128,64),
 * (64,128), (8,64), (16,64)}: 16-B aligned rows, strides multiples of 4 (GNN_E_ALIGN); 2 = a
 * narrow one (k <= 16, m <= 128: a classifier layer's dW, e.g. k = 7 for 7 classes): any row
 * stride, 4-B aligned; 0 = not covered. workspace: gnn_gemm_tn_workspace_bytes(n, m, k) bytes
 * of device memory.
 */
int gnn_gemm_tn_supported(int64_t m, int64_t k);
int64_t gnn_gemm_tn_workspace_bytes(int64_t n, int64_t m, int64_t k);
int gnn_gemm_tn_f32(const float* a, int64_t lda, const float* b, int64_t ldb, int64_t n,
                    int64_t m, int64_t k, float* c, int64_t ldc, int32_t trans_c, const float* d,
                    int64_t ldd, float* dsum, void* workspace, int64_t workspace_bytes,
                    void* stream);

/*
 * The same reduction over B' = B . [H > 0] * scale (elementwise; H [n, k], row stride ldh,
 * 16-B aligned): C = A^T B' (or its transpose) and, when dsum != NULL, dsum = the column sums
 * of B'. The weight and bias gradients of a Graph_conv_layer whose ReLU and Dropout
 * (GCN/GCN.py:12-14) ran in its transform's epilogue (gnn_gcn_transform_epi_f32) with output
 * H: the upstream gradient B passes exactly where H > 0, scaled by 1 / (1 - p) -- no separate
 * ReLU / dropout backward pass. gnn_gemm_tn_masked_supported(m, k): 1 for (m, k) in {(128,128),
 * (64,64), (128,64), (64,128)} in the split-bf16 arithmetic (gnn_transform_set_precision 1),
 * else 0 (GNN_E_UNSUPPORTED: the caller masks B itself and calls gnn_gemm_tn_f32). Workspace,
 * alignment and determinism as gnn_gemm_tn_f32.
 */
int gnn_gemm_tn_masked_supported(int64_t m, int64_t k);
int gnn_gemm_tn_masked_f32(const float* a, int64_t lda, const float* b, int64_t ldb,
                           const float* h, int64_t ldh, float scale, int64_t n, int64_t m,
                           int64_t k, float* c, int64_t ldc, int32_t trans_c, float* dsum,
                           void* workspace, int64_t workspace_bytes, void* stream);

/*
 * Column mean of x[n_rows, feat] (double accumulation, deterministic): the dense
 * GAT layer's output for an edgeless row (uniform softmax over all N nodes,
 * GAT/models/layers.py:29-32). scratch: gnn_col_mean_scratch_bytes(n_rows, feat).
 */
int64_t gnn_col_mean_scratch_bytes(int64_t n_rows, int64_t feat);
int gnn_col_mean_f32(const float* x, int64_t ldx, int64_t n_rows, int64_t feat, float* out,
                     void* scratch, void* stream);

/*
 * GAT backward (training through GraphAttentionLayer / SpGraphAttentionLayer;
 * replaces ATen autograd of GAT/models/layers.py:22-37 and
 * SpecialSpmmFunction.backward, layers.py:54-64). With per head
 *   out_i = sum_j m_ij a_ij Wh_j, a_ij = exp(z_ij - lse_i), z = +-LeakyReLU(el_i + er_j):
 * prep : dout = dy * ELU'(out) (elu != 0; out recovered from y), D_i = dout_i . out_i
 *        (dout [n, heads*fh], D [n, heads]);
 * edges: over CSR rows (plan segments + `rows` = every other row), per edge e and head:
 *        w_edge[e,h] = m a, ds_edge[e,h] = a (m dout_i.Wh_j - D_i) dz/ds, del[i,h] = sum_e ds
 *        (del_part [n_seg, heads] workspace for long rows);
 * nodes: over the transposed CSR (rowptr_t, src_t = source row, eid_t = CSR edge id)
 *        with its own plan: dwh[j] = sum_e w_edge[e,h] dout_i + der_j a_dst + del_j a_src,
 *        der[j,h] = sum_e ds_edge[e,h] (part [n_seg_t, heads*fh + heads] workspace);
 *        any head count (der is reduced 8 heads per pass inside the kernel).
 * The dropout mask is recomputed from (dropout_seed, edge, head) exactly as the forward drew it.
 */
int gnn_gat_backward_prep_f32(const float* dy, const float* y, int64_t ldo, int64_t n_rows,
                              int64_t heads, int64_t fh, int32_t elu, float* dout, float* D,
                              void* stream);
int gnn_gat_backward_edges_f32(const int64_t* rowptr, const int32_t* col, int64_t n_rows,
                               const float* wh, int64_t ldw, int64_t heads, int64_t fh,
                               const float* el, const float* er, const float* lse,
                               const float* dout, const float* D, float negative_slope,
                               int32_t mode, float dropout_p, uint64_t dropout_seed,
                               float* w_edge, float* ds_edge, float* del, int64_t seg_len,
                               const int32_t* seg_row, const int64_t* seg_begin, int64_t n_seg,
                               const int32_t* long_row, const int32_t* long_seg_ptr,
                               int64_t n_long, const int32_t* rows, int64_t n_rows_list,
                               float* del_part, void* stream);
int gnn_gat_backward_nodes_f32(const int64_t* rowptr_t, const int32_t* src_t,
                               const int64_t* eid_t, int64_t n_nodes, int64_t heads, int64_t fh,
                               const float* dout, const float* w_edge, const float* ds_edge,
                               const float* del, const float* a_src, const float* a_dst,
                               float* dwh, float* der, int64_t seg_len, const int32_t* seg_row,
                               const int64_t* seg_begin, int64_t n_seg, const int32_t* long_row,
                               const int32_t* long_seg_ptr, int64_t n_long, const int32_t* rows,
                               int64_t n_rows_list, float* part, void* stream);
/*
 * GAT backward, two passes with recomputation (what ops.gat_backward runs; the three passes
 * above remain for the shapes these refuse with GNN_E_UNSUPPORTED):
 * rows : over CSR rows, the prep fused in: dout (as prep), del (as edges), and per row
 *        nstat[i][h] = {el_ih, lse_ih, D_ih, 0} ([n, heads, 4], 16-B aligned); no per-edge
 *        output. Rows: plan segments + `rows` (one wave each) + `short_rows` (8 per wave; the
 *        low-degree rows), every row exactly once. a_dst (nullable, [heads * fh]): er_j
 *        recomputed from the gathered Wh_j row (fh / VW <= 4) instead of loaded from er.
 *        Unsupported: 2 heads*fh + heads > 1152, or
 *        short rows with 8 (2 heads*fh + heads) > 1152.
 * nodes_recompute: over the transposed CSR: per edge (i -> j) a_ij, g_ij = dout_i . Wh_j, w_ij,
 *        ds_ij recomputed from dout_i, nstat_i and node j's own Wh_j / er_j; dwh, der as nodes.
 *        eid_t is read only when dropout_p > 0. Rows: plan segments + `rows` + `short_rows`
 *        (one per lane group). Unsupported: fh / VW lanes per head not a power of two (VW = 4
 *        when fh % 4 == 0 and 16-B aligned, else 1), heads*fh above 256 VW.
 */
int gnn_gat_backward_rows_f32(const int64_t* rowptr, const int32_t* col, int64_t n_rows,
                              const float* wh, int64_t ldw, int64_t heads, int64_t fh,
                              const float* el, const float* er, const float* lse, const float* dy,
                              const float* y, int64_t ldo, int32_t elu, float negative_slope,
                              int32_t mode, float dropout_p, uint64_t dropout_seed, float* dout,
                              float* nstat, float* del, int64_t seg_len, const int32_t* seg_row,
                              const int64_t* seg_begin, int64_t n_seg, const int32_t* long_row,
                              const int32_t* long_seg_ptr, int64_t n_long, const int32_t* rows,
                              int64_t n_rows_list, const int32_t* short_rows, int64_t n_short,
                              float* del_part, const float* a_dst, void* stream);
/*
 * rows_ex: the same, with dy the gradient of dropout(y) taken by gnn_dropout_rows_f32 (key =
 * the row, p = dy_dropout_p, seed = dy_dropout_seed; GAT/models/GAT.py:17 after the heads):
 * the prep applies that mask to dy, so the separate backward of the dropout is not run.
 * dy_dropout_p > 0 needs ldo == heads*fh and the coalesced prep (fh % 4 == 0, fh / 4 a power of
 * two <= 64, 16-B aligned operands), else GNN_E_UNSUPPORTED (mask dy first, then call rows).
 */
int gnn_gat_backward_rows_ex_f32(const int64_t* rowptr, const int32_t* col, int64_t n_rows,
                                 const float* wh, int64_t ldw, int64_t heads, int64_t fh,
                                 const float* el, const float* er, const float* lse,
                                 const float* dy, const float* y, int64_t ldo, int32_t elu,
                                 float negative_slope, int32_t mode, float dropout_p,
                                 uint64_t dropout_seed, float* dout, float* nstat, float* del,
                                 int64_t seg_len, const int32_t* seg_row, const int64_t* seg_begin,
                                 int64_t n_seg, const int32_t* long_row,
                                 const int32_t* long_seg_ptr, int64_t n_long, const int32_t* rows,
                                 int64_t n_rows_list, const int32_t* short_rows, int64_t n_short,
                                 float* del_part, const float* a_dst, float dy_dropout_p,
                                 uint64_t dy_dropout_seed, void* stream);
int gnn_gat_backward_nodes_recompute_f32(
    const int64_t* rowptr_t, const int32_t* src_t, const int64_t* eid_t, int64_t n_nodes,
    int64_t heads, int64_t fh, const float* dout, const float* nstat, const float* wh,
    int64_t ldw, const float* er, const float* del, const float* a_src, const float* a_dst,
    float negative_slope, int32_t mode, float dropout_p, uint64_t dropout_seed, float* dwh,
    float* der, int64_t seg_len, const int32_t* seg_row, const int64_t* seg_begin, int64_t n_seg,
    const int32_t* long_row, const int32_t* long_seg_ptr, int64_t n_long, const int32_t* rows,
    int64_t n_rows_list, const int32_t* short_rows, int64_t n_short, float* part, void* stream);

/* ---- GraphSAGE aggregation modes ---- */
#define GNN_SAGE_MEAN 0   /* torch.mean(neigh_feat, dim=1)               -> fp32 out  */
#define GNN_SAGE_ARGMAX 1 /* torch.argmax(neigh_feat, dim=1): first max,
                             NaN counts as the maximum                   -> int64 out */
#define GNN_SAGE_SUM 2    /* neighbor_feature.sum(dim=1)                  -> fp32 out
                             (GraphSAGE_Pytorch/models/Aggregator.py:21-22)          */
#define GNN_SAGE_MAXPOOL 3 /* value max-pool, torch.max(neigh, dim=1).values -> fp32 out:
                             north_star "mean/max-pool"; the value that
                             GraphSAGE_Pytorch/models/Aggregator.py:23-24 reaches for
                             (there it gets the namedtuple and fails). A NaN in the
                             slice propagates.                                       */
#define GNN_SAGE_ARGMAX_F32 4 /* the GNN_SAGE_ARGMAX index stored as fp32 (exact below
                             2^24): the SageLayer's torch.cat([self, argmax]) promotion,
                             GraphSAGE/GraphSAGE.py:17 -- gnn_sage_gather_concat_* only */

/*
 * GraphSAGE Aggregator over a pre-gathered neighbour tensor
 *   neigh[m, j, f] at neigh + m*ld_m + j*ld_k + f   (m < M, j < k, f < feat)
 * Replaces Aggregator(neigh_feat, agg_func) at GraphSAGE/graph_utils.py:4-11.
 * Also NeighborAggregator.forward 'mean' / 'sum' (GraphSAGE_Pytorch/models/Aggregator.py:18-22).
 * out: fp32 [M, ldo] (MEAN, SUM) or int64 [M, ldo] (ARGMAX). k == 0 -> GNN_E_UNSUPPORTED.
 */
int gnn_sage_aggregate_f32(const float* neigh, int64_t ld_k, int64_t ld_m, int64_t M, int64_t k,
                           int64_t feat, int32_t mode, void* out, int64_t ldo, void* stream);

/*
 * Fused gather + Aggregator: out[m] = Aggregator(table[idx[m, 0..k)]) without
 * materialising the [M, k, feat] tensor the reference builds with
 * torch.embedding (GraphSAGE/GraphSAGE.py:47-49 + graph_utils.py:6,8).
 * idx int64 [M, ldi]; an index outside [0, n_table) sets *err_flag (device int32,
 * OR-ed with 1) and is skipped -- the caller raises IndexError like torch.embedding.
 */
int gnn_sage_gather_aggregate_f32(const float* table, int64_t ldt, int64_t n_table,
                                  const int64_t* idx, int64_t ldi, int64_t M, int64_t k,
                                  int64_t feat, int32_t mode, void* out, int64_t ldo,
                                  int32_t* err_flag, void* stream);

/*
 * Both halves of the SageLayer input cat[self, agg] in ONE launch (GraphSAGE/GraphSAGE.py:17
 * with the torch.embedding gathers of :47-49 and Aggregator, graph_utils.py:6):
 *   self_out[m, :] = table[self_idx[m], :]
 *   out[m, :]      = reduce_j table[idx[m * ldi + j], :]   (mode GNN_SAGE_MEAN / SUM / MAXPOOL)
 * self_out and out may be the two column halves of one [M, 2F] buffer. An index outside
 * [0, n_table) sets *err_flag |= 1 and reads nothing. k == 0 -> GNN_E_UNSUPPORTED.
 * mode GNN_SAGE_ARGMAX_F32: out holds the argmax index as fp32 (the cat's promotion).
 */
int gnn_sage_gather_concat_f32(const float* table, int64_t ldt, int64_t n_table,
                               const int64_t* self_idx, const int64_t* idx, int64_t ldi,
                               int64_t M, int64_t k, int64_t feat, int32_t mode, float* self_out,
                               int64_t ld_self, float* out, int64_t ldo, int32_t* err_flag,
                               void* stream);

/*
 * gnn_sage_gather_concat_f32 over rows [0, min(*live, M)) (live: a DEVICE int64 row count,
 * NULL = M): a sampled batch's layer runs on its buffers' capacity M without the host reading
 * the frontier size first. Rows from *live on are neither read nor written.
 */
int gnn_sage_gather_concat_live_f32(const float* table, int64_t ldt, int64_t n_table,
                                    const int64_t* self_idx, const int64_t* idx, int64_t ldi,
                                    int64_t M, const int64_t* live, int64_t k, int64_t feat,
                                    int32_t mode, float* self_out, int64_t ld_self, float* out,
                                    int64_t ldo, int32_t* err_flag, void* stream);

/*
 * One fused GraphSAGE inference layer (MEAN, not gcn):
 *   out[m] = relu(W . cat[self[m], mean_j table[nbr_idx[m, j]]])
 * Replaces SageLayer.forward(self, Aggregator(neigh, 'MEAN')) -- GraphSAGE/GraphSAGE.py:15-20,
 * graph_utils.py:6 -- plus the torch.embedding gathers of its inputs (GraphSAGE.py:47-49).
 * self[m] = self_src[self_idx[m]] (self_idx int64 [M], rows of a [n_self, lds] matrix) or,
 * with self_idx NULL, row m of self_src. nbr_idx int64 [M, ldi], k >= 1 neighbours per row;
 * table [n_table, ldt]. W fp32 [out_features, 2*feat] row-major (nn.Linear's weight).
 * out fp32 [M, ldo]. Shapes: gnn_sage_layer_supported(feat, out_features) != 0; 16-B
 * aligned rows. An index out of range sets *err_flag (the caller raises IndexError).
 * One persistent launch: gathers into an LDS tile, then v_mfma_f32_16x16x4_f32.
 */
int gnn_sage_layer_supported(int64_t feat, int64_t out_features);
int gnn_sage_layer_f32(const float* table, int64_t ldt, int64_t n_table, const float* self_src,
                       int64_t lds, int64_t n_self, const int64_t* self_idx,
                       const int64_t* nbr_idx, int64_t ldi, int64_t M, int64_t k, int64_t feat,
                       const float* w, int64_t out_features, float* out, int64_t ldo,
                       int32_t* err_flag, void* stream);

/*
 * Row gather out[i, :] = x[idx[i], :] (torch.embedding at GraphSAGE/GraphSAGE.py:47-48;
 * also packs halo send buffers for the multi-GPU edge-cut). Out-of-range index ->
 * *err_flag |= 1, row skipped.
 */
int gnn_gather_rows_f32(const float* x, int64_t ldx, int64_t n_x, const int64_t* idx, int64_t n,
                        int64_t feat, float* out, int64_t ldo, int32_t* err_flag, void* stream);

/*
 * Hashed element dropout fused with a row gather, replacing F.dropout(x, p, training) at
 * GAT/models/GAT.py:15,17 in training (and its backward): r = idx ? idx[i] : i,
 * out[i, c] = x[r, c] / (1 - p) when the (seed, key, c) hash clears p (common.hpp
 * dropout_keep; key = r if key_by_source else i), else 0. No mask is stored: the backward
 * re-derives it from the seed. 0 <= p < 1; x == out only without idx. Out-of-range index ->
 * *err_flag |= 1, row skipped.
 */
int gnn_dropout_rows_f32(const float* x, int64_t ldx, int64_t n_x, const int64_t* idx,
                         int32_t key_by_source, int64_t n, int64_t feat, float p, uint64_t seed,
                         float* out, int64_t ldo, int32_t* err_flag, void* stream);

/*
 * GraphSAGE neighbour sampling for a frontier (GraphSAGE/data_utils.py:89-94):
 *   out[i, 0..k) = k neighbours of nodes[i] in the CSR (rowptr, col):
 *     deg >  k: k distinct neighbours (random.sample), Floyd's algorithm;
 *     deg <= k: k draws with replacement (random.choices);
 *     deg == 0: row of -1 and *err_flag |= 1 (the reference raises IndexError);
 *   node id outside [0, n_graph): row of -1, *err_flag |= 2.
 * Draws come from a counter-based hash RNG keyed by (seed, i, draw), i = the position
 * in `nodes`: a frontier is reproducible for a given seed, and a node listed twice
 * draws independently. Callers derive `seed` per (batch seed, layer) with a hash
 * (sampler.stream_seed), never seed + layer. k <= 256.
 */
int gnn_sample_neighbors(const int64_t* rowptr, const int32_t* col, int64_t n_graph,
                         const int64_t* nodes, int64_t n, int64_t k, uint64_t seed, int64_t* out,
                         int32_t* err_flag, void* stream);

/*
 * Batch frontier (sampler.sample_batch): the sorted distinct ids of two id lists and the
 * position of listed ids among them -- collate_fn's set union and index remap
 * (GraphSAGE/data_utils.py:100-116), i.e. torch.unique(cat[a, b]) + torch.searchsorted.
 * A node bitmap marked with atomics and an exclusive scan of its word popcounts; no sort.
 *   gnn_frontier_build: clears the bitmap, marks ids_a and ids_b (an id outside
 *     [0, n_nodes) sets *err_flag |= 2), scans; writes the distinct count to *count
 *     (device int64). n_a + n_b < 2^32.
 *   gnn_frontier_emit:  frontier[0 .. count) = the distinct ids, ascending.
 *   gnn_frontier_rank:  pos[i] = position of ids[i] in the frontier (ids must be marked;
 *     an id outside [0, n_nodes) gives -1).
 * workspace: gnn_frontier_workspace_bytes(n_nodes) bytes, kept between the three calls.
 */
int64_t gnn_frontier_workspace_bytes(int64_t n_nodes);
int gnn_frontier_build(const int64_t* ids_a, int64_t n_a, const int64_t* ids_b, int64_t n_b,
                       int64_t n_nodes, void* workspace, int64_t workspace_bytes, int64_t* count,
                       int32_t* err_flag, void* stream);
int gnn_frontier_emit(int64_t n_nodes, const void* workspace, int64_t* frontier, void* stream);
int gnn_frontier_rank(const int64_t* ids, int64_t n, int64_t n_nodes, const void* workspace,
                      int64_t* pos, void* stream);

/*
 * The whole L-hop mini-batch of sampler.sample_batch in one call, with no host round trip
 * between hops (get_layer_adj_nodes + collate_fn's maps, GraphSAGE/data_utils.py:82-162):
 * S_0 = seeds; for i < L: nbrs[i] = gnn_sample_neighbors(S_i, fanouts[i], layer_seeds[i]) (with
 * append_self the node itself as column fanouts[i], data_utils.py:95-96); for i < L-1:
 * S_{i+1} = sorted distinct ids of S_i and nbrs[i] (layers[i+1]), center_maps[i] / neigh_maps[i]
 * = positions of S_i / nbrs[i] in S_{i+1}. Every list length lives on the device: stat (device
 * int64 [L + 1]) receives |S_i| in stat[i] and the error bits in the low word of stat[L]
 * (1 = a node without neighbours, 2 = a node id out of range, 4 = a frontier larger than its
 * buffer, 8 = an unsampled id reached the frontier, 16 = internal: the frontier scan's
 * look-back gave up), so the caller reads everything with ONE
 * copy at the end. Host arrays: fanouts, layer_seeds, caps [L] (caps[i] = rows of the S_i /
 * nbrs[i] / map buffers, caps[0] = n_seeds; caps[i+1] >= min(n_graph, caps[i] (1 + ld_i)) never
 * overflows), layers, nbrs, center_maps, neigh_maps (device pointers; layers[0] unused).
 * nbrs[i] / neigh_maps[i] rows have ld_i = fanouts[i] + append_self ids. fanouts[i] <= 64
 * (GNN_E_UNSUPPORTED above: use the step-by-step calls). The same draws, frontiers and maps as
 * the step-by-step calls. Launches: 2 L - 1 (L = 1: 2) -- each hop's draw also sets the
 * frontier flags of its ids, one scan per hop builds S_{i+1} (decoupled look-back over the
 * flags, which it clears), and the next hop's draw computes the maps and the previous hop's
 * error bits.
 * Workspace: gnn_sample_layers_workspace_bytes(n_graph) bytes, ZERO-FILLED before its first
 * use; every call leaves it zero-filled again. One workspace per stream (calls sharing one
 * must be ordered).
 */
int64_t gnn_sample_layers_workspace_bytes(int64_t n_graph);
int gnn_sample_layers(const int64_t* rowptr, const int32_t* col, int64_t n_graph,
                      const int64_t* seeds, int64_t n_seeds, int32_t n_layers,
                      const int64_t* fanouts, const uint64_t* layer_seeds, int32_t append_self,
                      int64_t* const* layers, const int64_t* caps, int64_t* const* nbrs,
                      int64_t* const* center_maps, int64_t* const* neigh_maps, int64_t* stat,
                      void* workspace, int64_t workspace_bytes, void* stream);

/*
 * Reference GCN adjacency on the device: D^-1/2 (max(A, A^T) + I)^T D^-1/2 as fp32 CSR
 * (GCN/data_utils.py:32-35 symmetrise, :78 + sp.eye, :54-60 normalize_adj, :63-70 fp32),
 * from a directed edge list (src -> dst, int64, duplicates allowed). Bit-identical to
 * the scipy pipeline (float64 normalisation). Two calls:
 *   gnn_gcn_adjacency_build: sorts / reduces in `workspace`
 *     (gnn_gcn_adjacency_workspace_bytes(n_edges, n_nodes) bytes) and returns nnz in
 *     *nnz_out (host). An endpoint outside [0, n_nodes) -> GNN_E_ARG.
 *   gnn_gcn_adjacency_fill: writes rowptr [n_nodes+1], col [nnz], val [nnz] from the
 *     same workspace.
 * Unlike the aggregation entry points these SYNCHRONISE `stream` between stages
 * (graph construction runs once per graph).
 */
int64_t gnn_gcn_adjacency_workspace_bytes(int64_t n_edges, int64_t n_nodes);
int gnn_gcn_adjacency_build(const int64_t* src, const int64_t* dst, int64_t n_edges,
                            int64_t n_nodes, void* workspace, int64_t workspace_bytes,
                            int64_t* nnz_out, void* stream);
int gnn_gcn_adjacency_fill(const void* workspace, int64_t n_edges, int64_t n_nodes, int64_t nnz,
                           int64_t* rowptr, int32_t* col, float* val, void* stream);

/* ---- CPython-exact host sampler (pysample.cpp; host memory, no stream) ----
 * Bit-exact restatement of the reference's host-side GraphSAGE sampling, which draws
 * from CPython's global `random` and iterates Python sets:
 *   gnn_pyadj_build      adj_lists of read_pubmed_data (GraphSAGE/data_utils.py:29-37):
 *                        for each pair t in order, adj[src[t]].add(dst[t]);
 *                        adj[dst[t]].add(src[t]). Writes each node's neighbours in the
 *                        iteration order of its Python set: rowptr [n_nodes+1],
 *                        nbr [<= 2 n_pairs]. Ids in [0, n_nodes) (else GNN_E_ARG).
 *   gnn_py_layer_sample  get_layer_adj_nodes(nodes, adj_lists, num_layers, num_neighs,
 *                        is_gcn) (data_utils.py:82-124) with the neighbour order
 *                        (rowptr, nbr) = list(adj_lists[v]). mt_state is CPython's
 *                        random.getstate()[1] (624 MT words + position, 625 uint32),
 *                        advanced in place exactly as the reference advances it.
 *                        On success *result holds the maps; read them with
 *                        gnn_py_layer_result_shape (dims = {L, pad_len, width}) and
 *                        gnn_py_layer_result_copy (neigh_map [L, pad_len, width],
 *                        center_map [L, pad_len], the torch.tensor()s of collate_fn,
 *                        data_utils.py:158-160), then gnn_py_layer_result_free.
 *                        GNN_E_EMPTY: a sampled node has no neighbours (IndexError).
 *   gnn_pyset_order / gnn_pyset_union_order: iteration order of set(keys) and of
 *                        set(a).union(set(b)) (test hooks for the set restatement).
 * Keys are node ids in [0, 2^61 - 1). */
int gnn_pyadj_build(const int64_t* src, const int64_t* dst, int64_t n_pairs, int64_t n_nodes,
                    int64_t* rowptr, int64_t* nbr);
int gnn_py_layer_sample(const int64_t* rowptr, const int64_t* nbr, int64_t n_nodes,
                        const int64_t* nodes, int64_t n_batch, int32_t num_layers,
                        int64_t num_neighs, int32_t is_gcn, uint32_t* mt_state, void** result);
int gnn_py_layer_result_shape(const void* result, int64_t* dims);
int gnn_py_layer_result_copy(const void* result, int64_t* neigh_map, int64_t* center_map);
void gnn_py_layer_result_free(void* result);
int gnn_pyset_order(const int64_t* keys, int64_t n, int64_t* out, int64_t* n_out);
int gnn_pyset_union_order(const int64_t* a, int64_t na, const int64_t* b, int64_t nb,
                          int64_t* out, int64_t* n_out);

/* ---- developer entry (not part of the drop-in surface) ----
 * gnn_dev_spmm_variant_f32: gnn_spmm_csr_f32 at feat == 128 with a compile-time
 * kernel variant (0 shipped: U=4, non-temporal Y stores; 1 U=8; 2 U=2; 3 U=4 and 4 U=8
 * with the neighbour rows staged through LDS by LDS-DMA; 7 U=4 with plain Y stores) and
 * no epilogue, for interleaved A/B timing (tools/spmm_ab.py). */
int gnn_dev_spmm_variant_f32(const int64_t* rowptr, const int32_t* col, const float* val,
                             int64_t n_rows, const float* x, int64_t ldx, int64_t feat,
                             const float* bias, float* y, int64_t ldy, int64_t seg_len,
                             const int32_t* seg_row, const int64_t* seg_begin, int64_t n_seg,
                             const int32_t* long_row, const int32_t* long_seg_ptr, int64_t n_long,
                             const int32_t* small_row, const int32_t* small_col,
                             const float* small_val, int64_t n_small, const int32_t* mid_row,
                             int64_t n_mid, float* partial, int32_t variant, void* stream);

/*
 * Edge-cut halo exchange (SURVEY 8(b) gnn_halo_alltoallv; the all-to-all-v that
 * distributed.EdgeCutSpmm / EdgeCutGat run through torch.distributed on the nccl = RCCL
 * backend). Rank p sends send_rows[q] rows of row_floats floats to every rank q (blocks
 * in peer order, contiguous in `send`) and receives recv_rows[q] rows from each into `recv`,
 * with ncclAllToAllv on the caller's communicator `comm` (an ncclComm_t) and HIP stream.
 * send_rows / recv_rows are host arrays [world]. The library does not link RCCL:
 * ncclAllToAllv is resolved from the process at the first call (the global scope, then an
 * already-loaded librccl.so / librccl.so.1; an RCCL not yet loaded is never loaded here, it
 * could not own `comm`), so it is the same RCCL that made `comm`; gnn_halo_rccl_path writes
 * that library's path. No host sync. Returns GNN_E_COMM when no loaded RCCL exports
 * ncclAllToAllv or its call fails, GNN_E_UNSUPPORTED when rows * row_floats or the running
 * offsets would exceed 2^62 elements.
 */
int gnn_halo_alltoallv_f32(const float* send, const int64_t* send_rows, float* recv,
                           const int64_t* recv_rows, int64_t row_floats, int64_t world,
                           void* comm, void* stream);
int gnn_halo_rccl_path(char* buf, int64_t len);

#ifdef __cplusplus
}
#endif

#endif /* GNN_MI355X_H_ */
