// hub.hip -- hub-staging plan for the SpMM / GAT aggregations (built once per graph and K).
//
// The gathers of gnn_spmm_csr_hub_f32 / gnn_gat_csr_hub_f32 read the K columns of highest
// in-degree ("hubs") from a compact per-call table instead of from X. This file builds
// the plan those kernels consume:
//   hub_ids[r]  = the column of rank r (degree descending, ties by ascending column id:
//                 a stable radix sort, so the plan is deterministic);
//   col_hub[e]  = -1 - rank(col[e]) for a hub column, col[e] otherwise.
// Steps: in-degree histogram (uint32 atomics, LDS-privatised for the hot ids) -> keys ~deg, values id -> rocPRIM
// radix_sort_pairs -> rank scatter -> column rename. No host synchronisation.
#include <cstring>  // rocprim's texture_cache_iterator calls host memset
#include <rocprim/rocprim.hpp>

#include "common.hpp"

namespace gnn {

// In-degree histogram. The hub columns take most edges and, in a degree-ordered graph, are the
// smallest ids: one global atomic per edge serialises on their counters (2.57 ms for the 20M
// edges of cfg3, profiles/r04e_cfg3_kernel_stats.csv). Each workgroup therefore counts the
// columns below kHubHotCols in LDS over a grid-stride range and adds its non-zero counts once.
constexpr int kHubHotCols = 8192;  // 32 KiB of LDS
constexpr int kHubDegBlocks = 512;

__global__ __launch_bounds__(256) void hub_degree_kernel(const int32_t* __restrict__ col,
                                                         int64_t nnz, int64_t n_cols,
                                                         uint32_t* __restrict__ deg,
                                                         int32_t* __restrict__ err) {
  __shared__ uint32_t hot[kHubHotCols];
  for (int i = threadIdx.x; i < kHubHotCols; i += blockDim.x) hot[i] = 0;
  __syncthreads();
  for (int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; e < nnz;
       e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int32_t c = col[e];
    if (c < 0 || c >= n_cols) {
      atomicOr(err, 1);
      continue;
    }
    if (c < kHubHotCols)
      atomicAdd(hot + c, 1u);  // LDS
    else
      atomicAdd(deg + c, 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kHubHotCols && i < n_cols; i += blockDim.x)
    if (hot[i]) atomicAdd(deg + i, hot[i]);
}

// deg -> ~deg in place (ascending sort of ~deg = descending degree), id = column, rank = -1
__global__ void hub_keys_kernel(uint32_t* deg_key, int64_t n_cols, int32_t* __restrict__ id,
                                int32_t* __restrict__ rank) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n_cols;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    deg_key[i] = ~deg_key[i];
    id[i] = static_cast<int32_t>(i);
    rank[i] = -1;
  }
}

__global__ void hub_rank_kernel(const int32_t* __restrict__ sorted_id, int64_t k,
                                int64_t* __restrict__ hub_ids, int32_t* __restrict__ rank) {
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; r < k;
       r += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int32_t c = sorted_id[r];
    hub_ids[r] = c;
    rank[c] = static_cast<int32_t>(r);
  }
}

__global__ void hub_rename_kernel(const int32_t* __restrict__ col, int64_t nnz,
                                  const int32_t* __restrict__ rank, int64_t n_cols,
                                  int32_t* __restrict__ col_hub) {
  for (int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; e < nnz;
       e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int32_t c = col[e];
    const int32_t r = (c >= 0 && c < n_cols) ? rank[c] : -1;
    col_hub[e] = r >= 0 ? -1 - r : c;
  }
}

static unsigned grid_for_n(int64_t n) {
  const int64_t b = (n + 255) / 256;
  return static_cast<unsigned>(b < 1 ? 1 : (b > 65536 ? 65536 : b));
}

static int64_t align256(int64_t v) { return (v + 255) / 256 * 256; }

static size_t hub_sort_temp_bytes(int64_t n_cols) {
  size_t t = 0;
  (void)rocprim::radix_sort_pairs(nullptr, t, static_cast<uint32_t*>(nullptr),
                                  static_cast<uint32_t*>(nullptr), static_cast<int32_t*>(nullptr),
                                  static_cast<int32_t*>(nullptr), static_cast<size_t>(n_cols));
  return t;
}

}  // namespace gnn

using namespace gnn;

extern "C" int64_t gnn_hub_plan_workspace_bytes(int64_t n_cols) {
  if (n_cols < 0) return GNN_E_ARG;
  const int64_t n = n_cols > 0 ? n_cols : 1;
  return 5 * align256(4 * n) + 256 + static_cast<int64_t>(hub_sort_temp_bytes(n)) + 256;
}

extern "C" int gnn_hub_plan_build(const int32_t* col, int64_t nnz, int64_t n_cols, int64_t k,
                                  int64_t* hub_ids, int32_t* col_hub, int32_t* err_flag,
                                  void* workspace, int64_t workspace_bytes, void* stream) {
  if (nnz < 0 || n_cols < 1 || k < 1 || k > n_cols || !hub_ids || !err_flag || !workspace ||
      (nnz > 0 && (!col || !col_hub)))
    return GNN_E_ARG;
  if (n_cols > 0x7fffffffLL) return GNN_E_UNSUPPORTED;
  if (workspace_bytes < gnn_hub_plan_workspace_bytes(n_cols)) return GNN_E_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  char* p = static_cast<char*>(workspace);
  const int64_t seg = align256(4 * n_cols);
  uint32_t* deg = reinterpret_cast<uint32_t*>(p);
  uint32_t* key_out = reinterpret_cast<uint32_t*>(p + seg);
  int32_t* id_in = reinterpret_cast<int32_t*>(p + 2 * seg);
  int32_t* id_out = reinterpret_cast<int32_t*>(p + 3 * seg);
  int32_t* rank = reinterpret_cast<int32_t*>(p + 4 * seg);
  void* temp = p + 5 * seg + 256;
  size_t tb = static_cast<size_t>(workspace_bytes - (5 * seg + 256));
  hipError_t e = hipMemsetAsync(deg, 0, 4 * n_cols, s);
  if (e != hipSuccess) return static_cast<int>(e);
  if (nnz > 0)
    hipLaunchKernelGGL(hub_degree_kernel,
                       dim3(grid_for_n(nnz) < kHubDegBlocks ? grid_for_n(nnz) : kHubDegBlocks),
                       dim3(256), 0, s, col, nnz, n_cols, deg, err_flag);
  hipLaunchKernelGGL(hub_keys_kernel, dim3(grid_for_n(n_cols)), dim3(256), 0, s, deg, n_cols,
                     id_in, rank);
  e = rocprim::radix_sort_pairs(temp, tb, deg, key_out, id_in, id_out,
                                static_cast<size_t>(n_cols), 0, 32, s);
  if (e != hipSuccess) return static_cast<int>(e);
  hipLaunchKernelGGL(hub_rank_kernel, dim3(grid_for_n(k)), dim3(256), 0, s, id_out, k, hub_ids,
                     rank);
  if (nnz > 0)
    hipLaunchKernelGGL(hub_rename_kernel, dim3(grid_for_n(nnz)), dim3(256), 0, s, col, nnz, rank,
                       n_cols, col_hub);
  return launch_status();
}

extern "C" int gnn_in_degree_u32(const int32_t* col, int64_t nnz, int64_t n_cols, uint32_t* deg,
                                 int32_t* err_flag, void* stream) {
  if (nnz < 0 || n_cols < 1 || !deg || !err_flag || (nnz > 0 && !col)) return GNN_E_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipError_t e = hipMemsetAsync(deg, 0, 4 * n_cols, s);
  if (e != hipSuccess) return static_cast<int>(e);
  if (nnz > 0)
    hipLaunchKernelGGL(hub_degree_kernel,
                       dim3(grid_for_n(nnz) < kHubDegBlocks ? grid_for_n(nnz) : kHubDegBlocks),
                       dim3(256), 0, s, col, nnz, n_cols, deg, err_flag);
  return launch_status();
}
