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

static inline int64_t fr_align_bytes(int64_t v) { return (v + 255) / 256 * 256; }

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
constexpr int32_t kBatchErrInternal = 16; // the frontier scan's look-back did not complete

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

// ---- the 3-launch L-hop batch (gnn_sample_layers) -------------------------------------------
// The frontier marks are byte flags (flags[v] = 1, plain stores: idempotent, no atomics), set by
// the hop's sampling kernel itself. One scan kernel per hop transition turns them into the
// frontier: a workgroup per tile of 512 words (32 flags per word); each tile publishes its
// count in ONE 8-byte agent-scope atomic word {tag, kind, value} and takes as its prefix the
// sum of every earlier tile's count (independent loads, no chain); it writes the frontier ids, the word
// prefixes / bitmaps the position lookups need, and clears the flags it read (the workspace
// is left all-zero for the next call: no memset). The next hop's sampling kernel also ranks the
// previous hop's lists (its extra workgroups) and derives the previous hop's sampler errors.
// For L = 2 ([25, 10]): sample + mark, scan + emit, sample + rank = 3 launches.
// 8192-word tiles (1024 threads x 8 words, 39 tiles at 10M nodes) were slower: 0.107 vs 0.083 ms per
// cfg4 batch (the dense hub tiles' emission on few workgroups)
#ifndef GNN_SCAN_WPT
// words per thread: 512-word tiles (611 at 10M nodes); in one process 4 / 2 / 1 words gave
// 57.1 / 55.4 / 61.8 us per pending cfg4 batch (profiles/r05s_scan_wpt_ab.log)
#define GNN_SCAN_WPT 2
#endif
constexpr int kScanThreads = 256;
constexpr int kScanWpt = GNN_SCAN_WPT;  // words per thread
constexpr int kScanWaves = kScanThreads / 64;
constexpr int kScanTileWords = kScanThreads * kScanWpt;
constexpr uint64_t kTileAgg = 1;  // kind of a published tile count

struct SampleWs {
  uint8_t* flags;   // [32 * n_words] (zero between calls)
  uint32_t* bits;   // [n_words] flag bitmap of the marked words (written where non-zero)
  uint32_t* pre;    // [n_words] frontier position of each marked word's first id
  uint64_t* tile;   // [n_tiles] look-back words {tag:30 | kind:2 | value:32}
  uint64_t* ctl;    // [0] tag base (bumped by L per call), [1] tile ticket of the next scan
};

static int64_t sw_tiles(int64_t n_words) { return (n_words + kScanTileWords - 1) / kScanTileWords; }

static int64_t sw_bytes(int64_t n_graph, SampleWs* w, char* base) {
  const int64_t n_words = (n_graph + 31) / 32;
  int64_t off = 0;
  auto take = [&](int64_t bytes) {
    char* p = base ? base + off : nullptr;
    off += fr_align_bytes(bytes);
    return p;
  };
  char* f = take(32 * n_words);
  char* b = take(4 * n_words);
  char* pr = take(4 * n_words);
  char* t = take(8 * sw_tiles(n_words));
  char* c = take(64);
  if (w) {
    w->flags = reinterpret_cast<uint8_t*>(f);
    w->bits = reinterpret_cast<uint32_t*>(b);
    w->pre = reinterpret_cast<uint32_t*>(pr);
    w->tile = reinterpret_cast<uint64_t*>(t);
    w->ctl = reinterpret_cast<uint64_t*>(c);
  }
  return off;
}

struct HopArgs {
  const int64_t* rowptr;
  const int32_t* col;
  int64_t n_graph;
  // this hop's draw: rows [0, live) of nodes, live = min(*n_dev, cap) (n_dev NULL: cap)
  const int64_t* nodes;
  int64_t cap;
  const int64_t* n_dev;
  int k;
  int64_t ld;
  bool self;
  uint64_t seed;
  int64_t* out;
  int32_t* err;        // stat[L]'s low word
  bool own_err;        // the last hop: the sampler records its own errors
  uint8_t* flags;      // non-NULL: mark (a scan follows)
  // first launch: stat[0..L] and the control words
  int64_t* stat;
  int n_layers;
  int64_t n_seeds;
  uint64_t* ctl;       // non-NULL: reset the next scan's tile ticket (and, first launch, bump the tag)
  bool first;
  // the previous hop's lists to rank (NULL: none)
  const int64_t* p_nodes;
  int64_t p_cap;
  const int64_t* p_dev;
  const int64_t* p_nbrs;
  int64_t p_ld;
  const uint32_t* bits;
  const uint32_t* pre;
  int64_t* p_cmap;
  int64_t* p_nmap;
  int64_t sample_blocks;
};

template <int LPN>
__global__ __launch_bounds__(256) void batch_hop_kernel(HopArgs A) {
  if (blockIdx.x == 0 && threadIdx.x == 0 && A.ctl != nullptr) {
    if (A.first) A.ctl[0] += static_cast<uint64_t>(A.n_layers);  // this call's scan tags
    A.ctl[1] = 0;                                                 // the next scan's tickets
  }
  if (A.first && blockIdx.x == 0 && threadIdx.x <= A.n_layers)
    A.stat[threadIdx.x] = threadIdx.x == 0 ? A.n_seeds : 0;      // sizes, then the error word
  if (static_cast<int64_t>(blockIdx.x) < A.sample_blocks) {
    const int64_t wave = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
    const int64_t live = live_rows(A.cap, A.n_dev);
    int32_t* err = A.own_err ? A.err : nullptr;
    if (A.flags)
      sample_lane_wave<LPN, true>(A.rowptr, A.col, A.n_graph, A.nodes, live, wave, A.k, A.ld,
                                  A.self, A.seed, A.out, err, A.flags);
    else
      sample_lane_wave<LPN, false>(A.rowptr, A.col, A.n_graph, A.nodes, live, wave, A.k, A.ld,
                                   A.self, A.seed, A.out, err, nullptr);
    return;
  }
  if (A.p_nodes == nullptr) return;
  // positions of the previous hop's nodes and neighbour ids in the frontier just built, and
  // that hop's sampler errors, derived from its lists (its draw ran with err == NULL):
  // node outside [0, n) -> 2 | 8, node without neighbours -> 1, listed id outside -> 8
  const int64_t live = live_rows(A.p_cap, A.p_dev);
  const int64_t total = live * (1 + A.p_ld);
  const int64_t stride = (static_cast<int64_t>(gridDim.x) - A.sample_blocks) * blockDim.x;
  int32_t e = 0;
  for (int64_t t = (static_cast<int64_t>(blockIdx.x) - A.sample_blocks) * blockDim.x + threadIdx.x;
       t < total; t += stride) {
    const bool node = t < live;
    const int64_t v = node ? A.p_nodes[t] : A.p_nbrs[t - live];
    int64_t p = -1;
    if (v >= 0 && v < A.n_graph) {
      const int64_t w = v >> 5;
      p = static_cast<int64_t>(A.pre[w]) + __popc(A.bits[w] & ((1u << (v & 31)) - 1u));
      if (node && A.rowptr[v + 1] == A.rowptr[v]) e |= kSampleErrEmpty;
    } else {
      e |= node ? (kSampleErrRange | kBatchErrMark) : kBatchErrMark;
    }
    if (node)
      A.p_cmap[t] = p;
    else
      A.p_nmap[t - live] = p;
  }
  if (e) atomicOr(A.err, e);
}

__device__ __forceinline__ uint64_t tile_word(uint64_t tag, uint64_t kind, uint32_t v) {
  return (tag << 34) | (kind << 32) | v;
}

// frontier = the flagged ids in ascending order (out[0 .. min(total, cap)), *count), the word
// prefixes and bitmaps of the flagged words, flags cleared; one workgroup per tile, tiles taken
// by ticket (ctl[1], reset by the launch before) so that a tile waits only on tiles that an
// earlier-started workgroup holds
__global__ __launch_bounds__(kScanThreads) void batch_scan_kernel(uint8_t* __restrict__ flags,
                                                         int64_t n_words, uint32_t* __restrict__ bits,
                                                         uint32_t* __restrict__ pre,
                                                         uint64_t* __restrict__ tile_st,
                                                         uint64_t* __restrict__ ctl, int tag_off,
                                                         int64_t cap, int64_t* __restrict__ out,
                                                         int64_t* __restrict__ count,
                                                         int32_t* __restrict__ err) {
  __shared__ int64_t s_tile;
  __shared__ uint32_t s_wave[kScanWaves];
  __shared__ uint32_t s_prefix;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (tid == 0)
    s_tile = static_cast<int64_t>(__hip_atomic_fetch_add(ctl + 1, uint64_t(1), __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT));
  __syncthreads();
  const int64_t tile = s_tile;
  if (tile >= (n_words + kScanTileWords - 1) / kScanTileWords) {  // tickets not reset: never
    if (tid == 0) atomicOr(err, kBatchErrInternal);                // writes out of range
    return;
  }
  const uint64_t tag = (ctl[0] + static_cast<uint64_t>(static_cast<int64_t>(tag_off))) & 0x3fffffffull;
  const int64_t w0 = tile * kScanTileWords + tid * kScanWpt;
  uint32_t mask[kScanWpt];
  uint32_t cnt = 0;
#pragma unroll
  for (int q = 0; q < kScanWpt; ++q) {
    const int64_t w = w0 + q;
    mask[q] = 0;
    if (w < n_words) {
      const uint4* f = reinterpret_cast<const uint4*>(flags + 32 * w);
      const uint4 a = f[0], b = f[1];
      const uint32_t d[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
      uint32_t m = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
#pragma unroll
        for (int bb = 0; bb < 4; ++bb)
          m |= ((d[j] >> (8 * bb)) & 0xffu ? 1u : 0u) << (4 * j + bb);
      }
      mask[q] = m;
      cnt += __popc(m);
    }
  }
  // block-wide exclusive scan of the thread counts
  uint32_t incl = cnt;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  if (lane == 63) s_wave[wid] = incl;
  __syncthreads();
  uint32_t wave_off = 0, agg = 0;
#pragma unroll
  for (int q = 0; q < kScanWaves; ++q) {
    wave_off += q < wid ? s_wave[q] : 0;
    agg += s_wave[q];
  }
  const uint32_t excl = wave_off + incl - cnt;
  // publish the tile's count; the prefix is the sum of EVERY earlier tile's count, loaded 8
  // windows of 64 at a time (independent loads: one round trip, not one per window as a
  // nearest-inclusive-prefix look-back takes -- 306 tiles at 10M nodes made that a chain of
  // up to 5 dependent agent-scope loads, 20 us per scan)
  if (wid == 0) {
    if (lane == 0)
      __hip_atomic_store(tile_st + tile, tile_word(tag, kTileAgg, agg), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    uint32_t part = 0;
    uint32_t polls = 0;  // every wave leaves: a tile that never publishes is an error
    bool failed = false;
    for (int64_t j0 = 0; j0 < tile && !failed; j0 += 64 * 8) {
      uint64_t sw[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int64_t j = j0 + q * 64 + lane;
        sw[q] = j < tile ? __hip_atomic_load(tile_st + j, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT)
                         : tile_word(tag, kTileAgg, 0);
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int64_t j = j0 + q * 64 + lane;
        while (__ballot((sw[q] >> 34) != tag)) {  // a tile of this window has not published
          if (++polls > (1u << 22)) {
            failed = true;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          if ((sw[q] >> 34) != tag)
            sw[q] = __hip_atomic_load(tile_st + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        part += static_cast<uint32_t>(sw[q]);
      }
    }
    if (failed && lane == 0) atomicOr(err, kBatchErrInternal);
    uint32_t prefix = part;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) prefix += __shfl_xor(prefix, o, 64);
    if (lane == 0) {
      s_prefix = prefix;
      if ((tile + 1) * kScanTileWords >= n_words) {  // the last tile: the frontier size
        const int64_t total = static_cast<int64_t>(prefix) + agg;
        if (total > cap) atomicOr(err, kBatchErrOverflow);
        count[0] = total < cap ? total : cap;
      }
    }
  }
  __syncthreads();
  uint32_t o = s_prefix + excl;
#pragma unroll
  for (int q = 0; q < kScanWpt; ++q) {
    uint32_t m = mask[q];
    if (m == 0) continue;
    const int64_t w = w0 + q;
    bits[w] = m;
    pre[w] = o;
    uint4* f = reinterpret_cast<uint4*>(flags + 32 * w);
    f[0] = make_uint4(0, 0, 0, 0);
    f[1] = make_uint4(0, 0, 0, 0);
    while (m) {
      const int t = __ffs(m) - 1;
      if (o < cap) out[o] = w * 32 + t;
      ++o;
      m &= m - 1;
    }
  }
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

extern "C" int64_t gnn_sample_layers_workspace_bytes(int64_t n_graph) {
  if (n_graph < 1) return GNN_E_ARG;
  return sw_bytes(n_graph, nullptr, nullptr);
}

template <int LPN>
static void launch_hop(HopArgs A, int64_t rank_blocks, hipStream_t s) {
  const int64_t per_block = 4 * (kWave / LPN);  // 4 waves of 64 / LPN nodes
  A.sample_blocks = (A.cap + per_block - 1) / per_block;
  hipLaunchKernelGGL(batch_hop_kernel<LPN>, dim3(static_cast<unsigned>(A.sample_blocks + rank_blocks)),
                     dim3(256), 0, s, A);
}

static void launch_hop_k(const HopArgs& A, int64_t rank_blocks, hipStream_t s) {
  if (A.k <= 16)
    launch_hop<16>(A, rank_blocks, s);
  else if (A.k <= 32)
    launch_hop<32>(A, rank_blocks, s);
  else
    launch_hop<64>(A, rank_blocks, s);
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
  if (workspace_bytes < gnn_sample_layers_workspace_bytes(n_graph)) return GNN_E_ARG;
  if (caps[0] != n_seeds) return GNN_E_ARG;
  for (int i = 0; i < n_layers; ++i) {
    if (fanouts[i] < 1 || caps[i] < 1 || !nbrs[i]) return GNN_E_ARG;
    if (fanouts[i] > 64) return GNN_E_UNSUPPORTED;  // the lane sampler's widest group
    const int64_t ld = fanouts[i] + (append_self ? 1 : 0);
    if (caps[i] > (INT64_C(1) << 40) / ld) return GNN_E_UNSUPPORTED;
    if (i + 1 < n_layers) {
      if (!layers[i + 1] || !center_maps[i] || !neigh_maps[i] || caps[i + 1] < 1)
        return GNN_E_ARG;
      if (caps[i] * (ld + 1) > 0xffffffffLL) return GNN_E_UNSUPPORTED;  // 32-bit prefixes
    }
  }
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t n_words = (n_graph + 31) / 32;
  SampleWs w;
  sw_bytes(n_graph, &w, static_cast<char*>(workspace));
  int32_t* err = reinterpret_cast<int32_t*>(stat + n_layers);  // low word of the last entry
  if (n_layers == 1) {  // one hop: no frontier; the sizes / error word first
    hipLaunchKernelGGL(batch_init_kernel, dim3(1), dim3(128), 0, s, stat, n_layers, n_seeds);
    launch_sample(rowptr, col, n_graph, seeds, n_seeds, nullptr, static_cast<int>(fanouts[0]),
                  fanouts[0] + (append_self ? 1 : 0), append_self != 0, layer_seeds[0], nbrs[0],
                  err, s);
    return launch_status();
  }
  const int64_t rank_blocks = 512;  // grid-stride over the ranked lists
  for (int i = 0; i < n_layers; ++i) {
    HopArgs A{};
    A.rowptr = rowptr;
    A.col = col;
    A.n_graph = n_graph;
    A.nodes = i == 0 ? seeds : layers[i];
    A.cap = caps[i];
    A.n_dev = i == 0 ? nullptr : stat + i;
    A.k = static_cast<int>(fanouts[i]);
    A.ld = fanouts[i] + (append_self ? 1 : 0);
    A.self = append_self != 0;
    A.seed = layer_seeds[i];
    A.out = nbrs[i];
    A.err = err;
    A.own_err = i + 1 == n_layers;
    A.flags = i + 1 < n_layers ? w.flags : nullptr;
    A.stat = stat;
    A.n_layers = n_layers;
    A.n_seeds = n_seeds;
    A.ctl = w.ctl;
    A.first = i == 0;
    if (i > 0) {  // rank hop i - 1's lists in the frontier S_i the scan just built
      A.p_nodes = i == 1 ? seeds : layers[i - 1];
      A.p_cap = caps[i - 1];
      A.p_dev = i == 1 ? nullptr : stat + i - 1;
      A.p_nbrs = nbrs[i - 1];
      A.p_ld = fanouts[i - 1] + (append_self ? 1 : 0);
      A.bits = w.bits;
      A.pre = w.pre;
      A.p_cmap = center_maps[i - 1];
      A.p_nmap = neigh_maps[i - 1];
    }
    launch_hop_k(A, i > 0 ? rank_blocks : 0, s);
    if (i + 1 == n_layers) break;
    // S_{i+1} = the flagged ids of S_i and nbrs[i] (tag i of this call's L)
    hipLaunchKernelGGL(batch_scan_kernel, dim3(static_cast<unsigned>(sw_tiles(n_words))),
                       dim3(kScanThreads),
                       0, s, w.flags, n_words, w.bits, w.pre, w.tile, w.ctl, i + 1 - n_layers,
                       caps[i + 1], layers[i + 1], stat + i + 1, err);
  }
  return launch_status();
}
