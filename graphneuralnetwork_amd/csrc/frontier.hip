// frontier.hip -- the GraphSAGE batch frontier on gfx950: the sorted set of distinct node
// ids of one or more id lists, and the position of any listed id inside it.
//
// Device counterpart of collate_fn's set union and index remap (GraphSAGE/data_utils.py:
// 100-116: layer_nodes.union(...), then unique_nodes[...] lookups); in sampler.sample_batch
// it replaces torch.unique(cat[seeds, nb0]) + torch.searchsorted. No sort: a node bitmap
// (one bit per graph node) is marked with atomicOr, an exclusive scan of the per-word
// popcounts gives every word's first position, and
//   frontier[pre[w] + j]  = the j-th set bit of word w   (ascending ids = torch.unique order)
//   pos(v)                = pre[v / 32] + popcount(bits[v / 32] & ((1 << v % 32) - 1))
// Cost: O(n_nodes / 32) words + O(listed ids), against a radix sort of the listed ids.
#include <cstring>  // rocprim's texture_cache_iterator calls host memset
#include <rocprim/rocprim.hpp>

#include "common.hpp"

namespace gnn {

__global__ void frontier_mark_kernel(const int64_t* __restrict__ ids, int64_t n, int64_t n_nodes,
                                     uint32_t* __restrict__ bits, int32_t* __restrict__ err) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t v = ids[i];
    if (v < 0 || v >= n_nodes) {
      atomicOr(err, 2);
      continue;
    }
    atomicOr(bits + (v >> 5), 1u << (v & 31));
  }
}

__global__ void frontier_popc_kernel(const uint32_t* __restrict__ bits, int64_t n_words,
                                     uint32_t* __restrict__ cnt) {
  for (int64_t w = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; w < n_words;
       w += static_cast<int64_t>(gridDim.x) * blockDim.x)
    cnt[w] = static_cast<uint32_t>(__popc(bits[w]));
}

__global__ void frontier_count_kernel(const uint32_t* __restrict__ cnt,
                                      const uint32_t* __restrict__ pre, int64_t n_words,
                                      int64_t* __restrict__ count) {
  if (blockIdx.x == 0 && threadIdx.x == 0) count[0] = static_cast<int64_t>(pre[n_words - 1]) + cnt[n_words - 1];
}

__global__ void frontier_emit_kernel(const uint32_t* __restrict__ bits,
                                     const uint32_t* __restrict__ pre, int64_t n_words,
                                     int64_t* __restrict__ out) {
  for (int64_t w = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; w < n_words;
       w += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    uint32_t b = bits[w];
    int64_t o = pre[w];
    while (b) {
      const int t = __ffs(b) - 1;
      out[o++] = w * 32 + t;
      b &= b - 1;
    }
  }
}

__global__ void frontier_rank_kernel(const int64_t* __restrict__ ids, int64_t n, int64_t n_nodes,
                                     const uint32_t* __restrict__ bits,
                                     const uint32_t* __restrict__ pre, int64_t* __restrict__ pos) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t v = ids[i];
    if (v < 0 || v >= n_nodes) {
      pos[i] = -1;
      continue;
    }
    const int64_t w = v >> 5;
    pos[i] = static_cast<int64_t>(pre[w]) + __popc(bits[w] & ((1u << (v & 31)) - 1u));
  }
}

static unsigned fr_grid(int64_t n) {
  const int64_t b = (n + 255) / 256;
  return static_cast<unsigned>(b < 1 ? 1 : (b > 65536 ? 65536 : b));
}

static int64_t fr_align(int64_t v) { return (v + 255) / 256 * 256; }

static size_t fr_scan_temp(int64_t n_words) {
  size_t t = 0;
  (void)rocprim::exclusive_scan(nullptr, t, static_cast<uint32_t*>(nullptr),
                                static_cast<uint32_t*>(nullptr), 0u,
                                static_cast<size_t>(n_words), rocprim::plus<uint32_t>());
  return t;
}

struct FrontierWs {
  uint32_t* bits;
  uint32_t* cnt;
  uint32_t* pre;
  void* temp;
  size_t temp_bytes;
};

static FrontierWs fr_layout(void* ws, int64_t n_nodes, int64_t ws_bytes) {
  const int64_t n_words = (n_nodes + 31) / 32;
  const int64_t seg = fr_align(4 * n_words);
  char* p = static_cast<char*>(ws);
  FrontierWs f;
  f.bits = reinterpret_cast<uint32_t*>(p);
  f.cnt = reinterpret_cast<uint32_t*>(p + seg);
  f.pre = reinterpret_cast<uint32_t*>(p + 2 * seg);
  f.temp = p + 3 * seg;
  f.temp_bytes = ws_bytes > 3 * seg ? static_cast<size_t>(ws_bytes - 3 * seg) : 0;
  return f;
}

}  // namespace gnn

using namespace gnn;

extern "C" int64_t gnn_frontier_workspace_bytes(int64_t n_nodes) {
  if (n_nodes < 1) return GNN_E_ARG;
  const int64_t n_words = (n_nodes + 31) / 32;
  return 3 * fr_align(4 * n_words) + static_cast<int64_t>(fr_scan_temp(n_words)) + 256;
}

extern "C" int gnn_frontier_build(const int64_t* ids_a, int64_t n_a, const int64_t* ids_b,
                                  int64_t n_b, int64_t n_nodes, void* workspace,
                                  int64_t workspace_bytes, int64_t* count, int32_t* err_flag,
                                  void* stream) {
  if (n_a < 0 || n_b < 0 || n_nodes < 1 || !workspace || !count || !err_flag ||
      (n_a > 0 && !ids_a) || (n_b > 0 && !ids_b))
    return GNN_E_ARG;
  if (n_a + n_b > 0xffffffffLL) return GNN_E_UNSUPPORTED;  // 32-bit word prefixes
  if (workspace_bytes < gnn_frontier_workspace_bytes(n_nodes)) return GNN_E_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t n_words = (n_nodes + 31) / 32;
  FrontierWs f = fr_layout(workspace, n_nodes, workspace_bytes);
  hipError_t e = hipMemsetAsync(f.bits, 0, 4 * n_words, s);
  if (e != hipSuccess) return static_cast<int>(e);
  if (n_a > 0)
    hipLaunchKernelGGL(frontier_mark_kernel, dim3(fr_grid(n_a)), dim3(256), 0, s, ids_a, n_a,
                       n_nodes, f.bits, err_flag);
  if (n_b > 0)
    hipLaunchKernelGGL(frontier_mark_kernel, dim3(fr_grid(n_b)), dim3(256), 0, s, ids_b, n_b,
                       n_nodes, f.bits, err_flag);
  hipLaunchKernelGGL(frontier_popc_kernel, dim3(fr_grid(n_words)), dim3(256), 0, s, f.bits,
                     n_words, f.cnt);
  e = rocprim::exclusive_scan(f.temp, f.temp_bytes, f.cnt, f.pre, 0u,
                              static_cast<size_t>(n_words), rocprim::plus<uint32_t>(), s);
  if (e != hipSuccess) return static_cast<int>(e);
  hipLaunchKernelGGL(frontier_count_kernel, dim3(1), dim3(64), 0, s, f.cnt, f.pre, n_words, count);
  return launch_status();
}

extern "C" int gnn_frontier_emit(int64_t n_nodes, const void* workspace, int64_t* frontier,
                                 void* stream) {
  if (n_nodes < 1 || !workspace || !frontier) return GNN_E_ARG;
  const int64_t n_words = (n_nodes + 31) / 32;
  FrontierWs f = fr_layout(const_cast<void*>(workspace), n_nodes, 0);
  hipLaunchKernelGGL(frontier_emit_kernel, dim3(fr_grid(n_words)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), f.bits, f.pre, n_words, frontier);
  return launch_status();
}

extern "C" int gnn_frontier_rank(const int64_t* ids, int64_t n, int64_t n_nodes,
                                 const void* workspace, int64_t* pos, void* stream) {
  if (n < 0 || n_nodes < 1 || !workspace || (n > 0 && (!ids || !pos))) return GNN_E_ARG;
  if (n == 0) return GNN_OK;
  FrontierWs f = fr_layout(const_cast<void*>(workspace), n_nodes, 0);
  hipLaunchKernelGGL(frontier_rank_kernel, dim3(fr_grid(n)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), ids, n, n_nodes, f.bits, f.pre, pos);
  return launch_status();
}
