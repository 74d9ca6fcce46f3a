/*
 * capi_gcn_spmm.c -- the GCN aggregation of bench.py's cfg2 step driven from plain C through
 * include/gnn_mi355x.h only: no Python, no torch. What INTEGRATION.md sketches, end to end:
 *
 *   edges -> gnn_gcn_adjacency_build/_fill         the reference's normalised adjacency
 *         -> gnn_column_order                      column-degree order A P^T
 *         -> gnn_gather_rows_f32                   X' = P X (the support in that order)
 *         -> gnn_hub_plan_build                    hub ranks (the first K rows of X')
 *         -> gnn_xcd_hub_plan_build/_fill          XCD-sliced items + rest
 *         -> gnn_spmm_plan_count/_fill, gnn_spmm_tasks_build
 *         -> gnn_spmm_csr_f32 (pass 1), gnn_spmm_csr_tasks_f32 (pass 2)
 *
 * with ops.py's default knobs (XCD_MIN_DEG 128, XCD_CHUNK 128, TASK_MAX_DEG 128, TASK_COST
 * 128, seg_len = max(64, 192 KiB / 4F), K = min(n, 262144, 128 MiB / 4F)). The output must
 * equal ops.spmm_forward(column_order(g).graph, X[perm]) bit for bit
 * (tests/test_capi_program_gpu.py).
 *
 *   capi_gcn_spmm <edges.bin> <x.bin> <y.bin> <n_nodes> <n_edges> <feat>
 *     edges.bin: int64 src[n_edges] then int64 dst[n_edges]; x.bin: fp32 [n_nodes, feat];
 *     y.bin (written): fp32 [n_nodes, feat] = A X, rows in the original order.
 * Exit status 0 on success; a failing call prints its name and the library's error string.
 */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/gnn_mi355x.h"

static hipStream_t S;

#define CHECK(call)                                                                       \
  do {                                                                                    \
    int rc_ = (int)(call);                                                                \
    if (rc_ != 0) {                                                                       \
      fprintf(stderr, "%s:%d %s -> %d (%s)\n", __FILE__, __LINE__, #call, rc_,            \
              gnn_error_string(rc_));                                                     \
      exit(1);                                                                            \
    }                                                                                     \
  } while (0)

static void* dmalloc(size_t bytes) {
  void* p = NULL;
  CHECK(hipMalloc(&p, bytes ? bytes : 16));
  return p;
}
static void h2d(void* d, const void* h, size_t b) { CHECK(hipMemcpy(d, h, b, hipMemcpyHostToDevice)); }
static void d2h(void* h, const void* d, size_t b) { CHECK(hipMemcpy(h, d, b, hipMemcpyDeviceToHost)); }
static void* hmalloc(size_t b) {
  void* p = malloc(b ? b : 16);
  if (!p) {
    fprintf(stderr, "host allocation of %zu bytes failed\n", b);
    exit(1);
  }
  return p;
}

static void read_file(const char* path, void* dst, size_t bytes) {
  FILE* f = fopen(path, "rb");
  if (!f || fread(dst, 1, bytes, f) != bytes) {
    fprintf(stderr, "cannot read %zu bytes from %s\n", bytes, path);
    exit(1);
  }
  fclose(f);
}

/* row-class plan of a CSR (graph.RowSplitPlan) */
typedef struct {
  int64_t seg_len, n_long, n_seg, n_small, n_mid;
  int32_t *seg_row, *long_row, *long_seg_ptr, *small_row, *small_col, *mid_row;
  int64_t* seg_begin;
  float* small_val;
} Plan;

static Plan row_plan(const int64_t* rowptr, const int32_t* col, const float* val, int64_t n,
                     int64_t seg_len) {
  Plan p;
  memset(&p, 0, sizeof p);
  p.seg_len = seg_len;
  void* scratch = dmalloc((size_t)gnn_spmm_plan_scratch_bytes(n));
  int64_t* counts = (int64_t*)dmalloc(4 * sizeof(int64_t));
  CHECK(hipMemset(counts, 0, 4 * sizeof(int64_t)));
  CHECK(gnn_spmm_plan_count(rowptr, n, seg_len, counts, scratch, S));
  int64_t c[4];
  CHECK(hipStreamSynchronize(S));
  d2h(c, counts, sizeof c);
  p.n_long = c[0], p.n_seg = c[1], p.n_small = c[2], p.n_mid = c[3];
  p.seg_row = (int32_t*)dmalloc(p.n_seg * 4);
  p.seg_begin = (int64_t*)dmalloc(p.n_seg * 8);
  p.long_row = (int32_t*)dmalloc(p.n_long * 4);
  p.long_seg_ptr = (int32_t*)dmalloc((p.n_long + 1) * 4);
  p.small_row = (int32_t*)dmalloc(p.n_small * 4);
  p.small_col = (int32_t*)dmalloc(p.n_small * 4);
  p.small_val = (float*)dmalloc(p.n_small * 4);
  p.mid_row = (int32_t*)dmalloc(p.n_mid * 4);
  CHECK(gnn_spmm_plan_fill(rowptr, col, val, n, seg_len, p.n_seg ? p.seg_row : NULL,
                           p.n_seg ? p.seg_begin : NULL, p.n_long ? p.long_row : NULL,
                           p.long_seg_ptr, p.n_small ? p.small_row : NULL,
                           p.n_small ? p.small_col : NULL, p.n_small ? p.small_val : NULL,
                           p.n_mid ? p.mid_row : NULL, scratch, S));
  CHECK(hipStreamSynchronize(S));
  hipFree(scratch);
  hipFree(counts);
  return p;
}

int main(int argc, char** argv) {
  if (argc != 7) {
    fprintf(stderr, "usage: %s edges.bin x.bin y.bin n_nodes n_edges feat\n", argv[0]);
    return 2;
  }
  const int64_t n = atoll(argv[4]), m = atoll(argv[5]), F = atoll(argv[6]);
  CHECK(hipStreamCreate(&S));

  /* ---- the reference adjacency (GCN/data_utils.py) ---- */
  int64_t* h_edges = (int64_t*)hmalloc((size_t)m * 16);
  read_file(argv[1], h_edges, (size_t)m * 16);
  int64_t* src = (int64_t*)dmalloc((size_t)m * 8);
  int64_t* dst = (int64_t*)dmalloc((size_t)m * 8);
  h2d(src, h_edges, (size_t)m * 8);
  h2d(dst, h_edges + m, (size_t)m * 8);
  free(h_edges);
  int64_t ws_bytes = gnn_gcn_adjacency_workspace_bytes(m, n);
  void* ws = dmalloc((size_t)ws_bytes);
  int64_t nnz = 0;
  CHECK(gnn_gcn_adjacency_build(src, dst, m, n, ws, ws_bytes, &nnz, S));
  int64_t* rowptr = (int64_t*)dmalloc((size_t)(n + 1) * 8);
  int32_t* col = (int32_t*)dmalloc((size_t)nnz * 4);
  float* val = (float*)dmalloc((size_t)nnz * 4);
  CHECK(gnn_gcn_adjacency_fill(ws, m, n, nnz, rowptr, col, val, S));
  CHECK(hipStreamSynchronize(S));
  hipFree(ws);
  hipFree(src);
  hipFree(dst);

  /* ---- column-degree order: A P^T, X' = P X ---- */
  int64_t* perm = (int64_t*)dmalloc((size_t)n * 8);
  int64_t* inv = (int64_t*)dmalloc((size_t)n * 8);
  int32_t* col_ord = (int32_t*)dmalloc((size_t)nnz * 4);
  ws_bytes = gnn_column_order_workspace_bytes(n);
  ws = dmalloc((size_t)ws_bytes);
  CHECK(gnn_column_order(col, nnz, n, -1, perm, inv, col_ord, ws, ws_bytes, S));
  CHECK(hipStreamSynchronize(S));
  hipFree(ws);
  float* h_x = (float*)hmalloc((size_t)n * F * 4);
  read_file(argv[2], h_x, (size_t)n * F * 4);
  float* x = (float*)dmalloc((size_t)n * F * 4);
  float* xo = (float*)dmalloc((size_t)n * F * 4);
  h2d(x, h_x, (size_t)n * F * 4);
  free(h_x);
  int32_t* err = (int32_t*)dmalloc(4);
  CHECK(hipMemset(err, 0, 4));
  CHECK(gnn_gather_rows_f32(x, F, n, perm, n, F, xo, F, err, S));

  /* ---- hub ranks and the XCD-sliced plan ---- */
  const int64_t seg = (192 * 1024) / (4 * F) > 64 ? (192 * 1024) / (4 * F) : 64;
  int64_t k = (int64_t)(128 << 20) / (4 * F);
  if (k < 64) k = 64;
  if (k > 262144) k = 262144;
  if (k > n) k = n;
  const int64_t chunk = seg < 128 ? seg : 128;
  int64_t* hub_ids = (int64_t*)dmalloc((size_t)k * 8);
  int32_t* col_hub = (int32_t*)dmalloc((size_t)nnz * 4);
  ws_bytes = gnn_hub_plan_workspace_bytes(n);
  ws = dmalloc((size_t)ws_bytes);
  CHECK(gnn_hub_plan_build(col_ord, nnz, n, k, hub_ids, col_hub, err, ws, ws_bytes, S));
  CHECK(hipStreamSynchronize(S));
  hipFree(ws);
  int64_t c[4];
  ws_bytes = gnn_xcd_hub_plan_workspace_bytes(n, nnz);
  ws = dmalloc((size_t)ws_bytes);
  CHECK(gnn_xcd_hub_plan_build(rowptr, col_hub, n, nnz, k, 128, chunk, 1, 0, 0, c, ws, ws_bytes, S));
  if (c[0] == 0) {
    fprintf(stderr, "no XCD items on this graph\n");
    return 1;
  }
  const int64_t n_pos = c[1];
  int64_t* irp = (int64_t*)dmalloc((size_t)(n_pos + 1) * 8);
  int32_t* icol = (int32_t*)dmalloc((size_t)c[2] * 4);
  float* ival = (float*)dmalloc((size_t)c[2] * 4);
  int64_t* pos_row = (int64_t*)dmalloc((size_t)n_pos * 8);
  int64_t* rrp = (int64_t*)dmalloc((size_t)(n + 1) * 8);
  int32_t* rcol = (int32_t*)dmalloc((size_t)c[3] * 4);
  float* rval = (float*)dmalloc((size_t)c[3] * 4);
  CHECK(gnn_xcd_hub_plan_fill(ws, rowptr, col_hub, val, n, nnz, k, 1, c, irp, icol, ival, pos_row,
                              rrp, rcol, rval, S));
  CHECK(hipStreamSynchronize(S));
  hipFree(ws);

  /* hub ranks are X' rows 0..k-1 (the column order): read them in place (XcdHubPlan.direct):
     items -1-rank -> rank; rest -1-rank -> rank, partial refs -1-(k + pos) -> -1-pos */
  int32_t* h = (int32_t*)hmalloc((size_t)(c[2] > c[3] ? c[2] : c[3]) * 4);
  d2h(h, icol, (size_t)c[2] * 4);
  for (int64_t e = 0; e < c[2]; ++e) h[e] = -1 - h[e];
  h2d(icol, h, (size_t)c[2] * 4);
  d2h(h, rcol, (size_t)c[3] * 4);
  for (int64_t e = 0; e < c[3]; ++e) {
    const int64_t v = h[e];
    h[e] = (int32_t)(v >= 0 ? v : (v >= -k ? -1 - v : v + k));
  }
  h2d(rcol, h, (size_t)c[3] * 4);
  free(h);

  /* ---- pass 1: every item into its partial row (plain kernel, mid-row class) ---- */
  Plan p1 = row_plan(irp, icol, ival, n_pos, seg);
  if (p1.n_seg || p1.n_small) {
    fprintf(stderr, "item rows outside the mid-row class\n");
    return 1;
  }
  float* part = (float*)dmalloc((size_t)n_pos * F * 4);
  CHECK(gnn_spmm_csr_f32(irp, icol, ival, n_pos, xo, F, F, NULL, part, F, p1.seg_len, NULL, NULL, 0,
                         NULL, p1.long_seg_ptr, 0, NULL, NULL, NULL, 0,
                         p1.n_mid ? p1.mid_row : p1.long_seg_ptr, p1.n_mid, NULL, 0, S));

  /* ---- pass 2: the rest as packed row tasks + mid rows + long-row segments ---- */
  Plan p2 = row_plan(rrp, rcol, rval, n, seg);
  const int64_t max_deg = seg < 128 ? seg : 128;
  int64_t* h_rp = (int64_t*)hmalloc((size_t)(n + 1) * 8);
  d2h(h_rp, rrp, (size_t)(n + 1) * 8);
  int32_t* h_mid = (int32_t*)hmalloc((size_t)n * 4);
  int64_t n_mid = 0;
  for (int64_t r = 0; r < n; ++r) {
    const int64_t d = h_rp[r + 1] - h_rp[r];
    if (d > max_deg && d <= seg) h_mid[n_mid++] = (int32_t)r;
  }
  int32_t* mid = (int32_t*)dmalloc((size_t)n_mid * 4);
  h2d(mid, h_mid, (size_t)n_mid * 4);
  free(h_mid);
  free(h_rp);
  int32_t* task_row = (int32_t*)dmalloc((size_t)n * 8);
  int64_t n_task = 0;
  ws_bytes = gnn_spmm_tasks_workspace_bytes(n);
  ws = dmalloc((size_t)ws_bytes);
  CHECK(gnn_spmm_tasks_build(rrp, n, max_deg, 128, task_row, n, &n_task, ws, ws_bytes, S));
  CHECK(gnn_spmm_tasks_check(task_row, n_task, n, err, S));
  float* partial = p2.n_seg ? (float*)dmalloc((size_t)p2.n_seg * F * 4) : NULL;
  float* y = (float*)dmalloc((size_t)n * F * 4);
  CHECK(gnn_spmm_csr_tasks_f32(rrp, rcol, rval, n, xo, F, part, F, F, NULL, y, F, p2.seg_len,
                               p2.n_seg ? p2.seg_row : NULL, p2.n_seg ? p2.seg_begin : NULL, p2.n_seg,
                               p2.n_long ? p2.long_row : NULL, p2.long_seg_ptr, p2.n_long,
                               n_mid ? mid : p2.long_seg_ptr, n_mid, n_task ? task_row : NULL,
                               n_task, partial, 0, S));
  CHECK(hipStreamSynchronize(S));
  int32_t herr = 0;
  d2h(&herr, err, 4);
  if (herr) {
    fprintf(stderr, "device error flag %d\n", herr);
    return 1;
  }

  float* h_y = (float*)hmalloc((size_t)n * F * 4);
  d2h(h_y, y, (size_t)n * F * 4);
  FILE* f = fopen(argv[3], "wb");
  if (!f || fwrite(h_y, 4, (size_t)n * F, f) != (size_t)n * F) {
    fprintf(stderr, "cannot write %s\n", argv[3]);
    return 1;
  }
  fclose(f);
  printf("{\"nnz\": %lld, \"k\": %lld, \"items\": %lld, \"positions\": %lld, \"tasks\": %lld, "
         "\"mid\": %lld, \"segments\": %lld}\n",
         (long long)nnz, (long long)k, (long long)c[0], (long long)n_pos, (long long)n_task,
         (long long)n_mid, (long long)p2.n_seg);
  return 0;
}
