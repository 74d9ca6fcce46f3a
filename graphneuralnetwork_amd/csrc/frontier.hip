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
#include "sample_kernels.hpp"

namespace gnn {

// Marking a power-law frontier: the hub ids appear thousands of times and share a few bitmap
// words (the degree order puts every hub in the first words), and every thread of the launch is
// in flight at once, so a global atomicOr per listed id serialises on those words (rocprofv3:
// 190 us to mark the 213K ids of a cfg4 batch, profiles/r04c_sample_kernel_stats.csv). Each
// workgroup therefore ORs the ids below kHotIds into an LDS copy of the first words and folds
// it into the global bitmap once at the end (one atomic per non-zero word and workgroup); ids
// above it are rare per word and go straight to a global atomic, skipped when a read already
// shows the bit (bits are only ever set during a build, so a stale read costs an extra atomic,
// never a missed one).
constexpr int kHotWords = 2048;                 // 8 KiB of LDS per workgroup
constexpr int64_t kHotIds = 32 * kHotWords;     // ids 0 .. 65535
constexpr int kMarkBlocks = 256;                // workgroups of a mark launch (grid-stride)

__device__ __forceinline__ void mark_bit(uint32_t* bits, int64_t v) {
  uint32_t* w = bits + (v >> 5);
  const uint32_t m = 1u << (v & 31);
  if ((__builtin_nontemporal_load(w) & m) == 0) atomicOr(w, m);
}

// ids a[0 .. na) then b[0 .. nb) (one grid-stride range); sets *err |= errbit for an id outside
// [0, n_nodes)
__device__ __forceinline__ void mark_lists(const int64_t* __restrict__ a, int64_t na,
                                           const int64_t* __restrict__ b, int64_t nb,
                                           int64_t n_nodes, uint32_t* __restrict__ bits,
                                           int32_t* __restrict__ err, int32_t errbit) {
  __shared__ uint32_t hot[kHotWords];
  for (int i = threadIdx.x; i < kHotWords; i += blockDim.x) hot[i] = 0;
  __syncthreads();
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < na + nb;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t v = i < na ? a[i] : b[i - na];
    if (v < 0 || v >= n_nodes) {
      atomicOr(err, errbit);
      continue;
    }
    if (v < kHotIds)
      atomicOr(hot + (v >> 5), 1u << (v & 31));  // LDS atomic, on this CU
    else
      mark_bit(bits, v);
  }
  __syncthreads();
  const int64_t words = (n_nodes + 31) / 32;
  for (int i = threadIdx.x; i < kHotWords && i < words; i += blockDim.x)
    if (hot[i]) atomicOr(bits + i, hot[i]);
}

static unsigned mark_grid(int64_t n) {
  const int64_t b = (n + 255) / 256;
  return static_cast<unsigned>(b < 1 ? 1 : (b > kMarkBlocks ? kMarkBlocks : b));
}

__global__ __launch_bounds__(256) void frontier_mark_kernel(const int64_t* __restrict__ a,
                                                             int64_t na,
                                                             const int64_t* __restrict__ b,
                                                             int64_t nb, int64_t n_nodes,
                                                             uint32_t* __restrict__ bits,
                                                             int32_t* __restrict__ err) {
  mark_lists(a, na, b, nb, n_nodes, bits, err, 2);
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

// ---- the fused L-hop batch (gnn_sample_layers): list lengths read from the device ----------
// error bits beyond the sampler's (kSampleErrEmpty / kSampleErrRange)
constexpr int32_t kBatchErrOverflow = 4;  // a frontier larger than its buffer (cannot happen
                                          // with the caller's bounds; checked anyway)
constexpr int32_t kBatchErrMark = 8;      // a listed id outside [0, n_nodes) (a failed draw)

// rows of list a (a_n rows, live count *a_dev) and of list b (b_rows rows of b_ld ids, live
// rows *b_dev) in one grid: b's ids are the a rows' sampled neighbours
__global__ __launch_bounds__(256) void batch_mark_kernel(
    const int64_t* __restrict__ a, int64_t a_n, const int64_t* __restrict__ a_dev,
    const int64_t* __restrict__ b, int64_t b_rows, const int64_t* __restrict__ b_dev,
    int64_t b_ld, int64_t n_nodes, uint32_t* __restrict__ bits, int32_t* __restrict__ err) {
  mark_lists(a, live_rows(a_n, a_dev), b, live_rows(b_rows, b_dev) * b_ld, n_nodes, bits, err,
             kBatchErrMark);
}

// frontier[0 .. count) = the set bits in ascending order, *count = their number (clamped to cap)
__global__ void batch_emit_kernel(const uint32_t* __restrict__ bits, const uint32_t* __restrict__ pre,
                                  int64_t n_words, int64_t cap, int64_t* __restrict__ out,
                                  int64_t* __restrict__ count, int32_t* __restrict__ err) {
  const int64_t t0 = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t0 == 0) {
    const int64_t total = static_cast<int64_t>(pre[n_words - 1]) + __popc(bits[n_words - 1]);
    if (total > cap) atomicOr(err, kBatchErrOverflow);
    count[0] = total < cap ? total : cap;
  }
  for (int64_t w = t0; w < n_words; w += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    uint32_t b = bits[w];
    int64_t o = pre[w];
    while (b) {
      const int t = __ffs(b) - 1;
      if (o < cap) out[o] = w * 32 + t;
      ++o;
      b &= b - 1;
    }
  }
}

// positions of the a ids and the b ids (as batch_mark_kernel's lists) in the frontier
__global__ void batch_rank_kernel(const int64_t* __restrict__ a, int64_t a_n,
                                  const int64_t* __restrict__ a_dev, const int64_t* __restrict__ b,
                                  int64_t b_rows, const int64_t* __restrict__ b_dev, int64_t b_ld,
                                  int64_t n_nodes, const uint32_t* __restrict__ bits,
                                  const uint32_t* __restrict__ pre, int64_t* __restrict__ pos_a,
                                  int64_t* __restrict__ pos_b) {
  const int64_t na = live_rows(a_n, a_dev), nb = live_rows(b_rows, b_dev) * b_ld;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < na + nb;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t v = i < na ? a[i] : b[i - na];
    int64_t p = -1;
    if (v >= 0 && v < n_nodes) {
      const int64_t w = v >> 5;
      p = static_cast<int64_t>(pre[w]) + __popc(bits[w] & ((1u << (v & 31)) - 1u));
    }
    if (i < na)
      pos_a[i] = p;
    else
      pos_b[i - na] = p;
  }
}

__global__ void batch_init_kernel(int64_t* __restrict__ stat, int n_layers, int64_t n_seeds) {
  const int i = threadIdx.x;
  if (i <= n_layers) stat[i] = i == 0 ? n_seeds : 0;  // sizes |S_i|, then the error word
}

static unsigned fr_grid(int64_t n) {
  const int64_t b = (n + 255) / 256;
  return static_cast<unsigned>(b < 1 ? 1 : (b > 65536 ? 65536 : b));
}

static int64_t fr_align(int64_t v) { return (v + 255) / 256 * 256; }

struct PopcOp {
  __host__ __device__ uint32_t operator()(uint32_t w) const {
#if defined(__HIP_DEVICE_COMPILE__)
    return static_cast<uint32_t>(__popc(w));
#else
    return static_cast<uint32_t>(__builtin_popcount(w));
#endif
  }
};

static auto popc_iter(const uint32_t* bits) { return rocprim::make_transform_iterator(bits, PopcOp()); }

static size_t fr_scan_temp(int64_t n_words) {
  size_t t = 0, t2 = 0;
  (void)rocprim::exclusive_scan(nullptr, t, static_cast<uint32_t*>(nullptr),
                                static_cast<uint32_t*>(nullptr), 0u,
                                static_cast<size_t>(n_words), rocprim::plus<uint32_t>());
  // the fused batch sampler scans the word popcounts straight from the bitmap
  (void)rocprim::exclusive_scan(nullptr, t2, popc_iter(nullptr), static_cast<uint32_t*>(nullptr),
                                0u, static_cast<size_t>(n_words), rocprim::plus<uint32_t>());
  return t > t2 ? t : t2;
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
  if (n_a + n_b > 0)
    hipLaunchKernelGGL(frontier_mark_kernel, dim3(mark_grid(n_a + n_b)), dim3(256), 0, s, ids_a,
                       n_a, ids_b, n_b, n_nodes, f.bits, err_flag);
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

extern "C" int gnn_sample_layers(const int64_t* rowptr, const int32_t* col, int64_t n_graph,
                                 const int64_t* seeds, int64_t n_seeds, int32_t n_layers,
                                 const int64_t* fanouts, const uint64_t* layer_seeds,
                                 int32_t append_self, int64_t* const* layers, const int64_t* caps,
                                 int64_t* const* nbrs, int64_t* const* center_maps,
                                 int64_t* const* neigh_maps, int64_t* stat, void* workspace,
                                 int64_t workspace_bytes, void* stream) {
  if (n_layers < 1 || n_layers > 64 || n_seeds < 1 || n_graph < 1 || !rowptr || !col || !seeds ||
      !fanouts || !layer_seeds || !caps || !nbrs || !stat || !workspace)
    return GNN_E_ARG;
  if (n_layers > 1 && (!layers || !center_maps || !neigh_maps)) return GNN_E_ARG;
  if (workspace_bytes < gnn_frontier_workspace_bytes(n_graph)) return GNN_E_ARG;
  if (caps[0] != n_seeds) return GNN_E_ARG;
  for (int i = 0; i < n_layers; ++i) {
    if (fanouts[i] < 1 || fanouts[i] > kMaxFanout || caps[i] < 1 || !nbrs[i]) return GNN_E_ARG;
    const int64_t ld = fanouts[i] + (append_self ? 1 : 0);
    if (caps[i] > (INT64_C(1) << 40) / ld) return GNN_E_UNSUPPORTED;
    if (i + 1 < n_layers) {
      if (!layers[i + 1] || !center_maps[i] || !neigh_maps[i] || caps[i + 1] < 1)
        return GNN_E_ARG;
      if (caps[i] * (ld + 1) > 0xffffffffLL) return GNN_E_UNSUPPORTED;  // 32-bit word prefixes
    }
  }
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t n_words = (n_graph + 31) / 32;
  FrontierWs f = fr_layout(workspace, n_graph, workspace_bytes);
  int32_t* err = reinterpret_cast<int32_t*>(stat + n_layers);  // low word of the last entry
  // n_layers + 1 <= 65 entries (sizes, then the error word): one workgroup of 128 threads
  hipLaunchKernelGGL(batch_init_kernel, dim3(1), dim3(128), 0, s, stat, n_layers, n_seeds);
  for (int i = 0; i < n_layers; ++i) {
    const int64_t* nodes = i == 0 ? seeds : layers[i];
    const int64_t* n_dev = stat + i;
    const int k = static_cast<int>(fanouts[i]);
    const int64_t ld = k + (append_self ? 1 : 0);
    launch_sample(rowptr, col, n_graph, nodes, caps[i], n_dev, k, ld, append_self != 0,
                  layer_seeds[i], nbrs[i], err, s);
    if (i + 1 == n_layers) break;
    // S_{i+1} = sorted distinct ids of S_i and its sampled neighbours, and the maps into it
    hipError_t e = hipMemsetAsync(f.bits, 0, 4 * n_words, s);
    if (e != hipSuccess) return static_cast<int>(e);
    const int64_t listed = caps[i] * (ld + 1);
    hipLaunchKernelGGL(batch_mark_kernel, dim3(mark_grid(listed)), dim3(256), 0, s, nodes, caps[i],
                       n_dev, nbrs[i], caps[i], n_dev, ld, n_graph, f.bits, err);
    e = rocprim::exclusive_scan(f.temp, f.temp_bytes, popc_iter(f.bits), f.pre, 0u,
                                static_cast<size_t>(n_words), rocprim::plus<uint32_t>(), s);
    if (e != hipSuccess) return static_cast<int>(e);
    hipLaunchKernelGGL(batch_emit_kernel, dim3(fr_grid(n_words)), dim3(256), 0, s, f.bits, f.pre,
                       n_words, caps[i + 1], layers[i + 1], stat + i + 1, err);
    hipLaunchKernelGGL(batch_rank_kernel, dim3(fr_grid(listed)), dim3(256), 0, s, nodes, caps[i],
                       n_dev, nbrs[i], caps[i], n_dev, ld, n_graph, f.bits, f.pre, center_maps[i],
                       neigh_maps[i]);
  }
  return launch_status();
}
