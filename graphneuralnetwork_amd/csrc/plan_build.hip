// plan_build.hip -- device builders of the SpMM schedules of the default aggregation path,
// so that a C caller reaches the path bench.py times without the Python package:
//
//   gnn_spmm_tasks_build   packed row tasks of gnn_spmm_csr_tasks_f32 (graph.task_ranges)
//   gnn_column_order       the column-degree relabelling A P^T (graph.degree_order(rows=False))
//   gnn_xcd_hub_plan_*     the XCD-sliced hub items + rest lists (graph.xcd_hub_coo)
//
// Each restates the torch builder of graph.py step by step with rocPRIM scans, selects,
// stable radix sorts and run-length encodes, and produces the same arrays bit for bit
// (tests/test_plan_build_gpu.py compares them). They run once per graph: the builders
// synchronise their stream to size the next stage, never per forward.
#include <cstring>  // rocprim's texture_cache_iterator calls host memset

#include <rocprim/rocprim.hpp>

#include "common.hpp"

extern "C" int gnn_in_degree_u32(const int32_t* col, int64_t nnz, int64_t n_cols, uint32_t* deg,
                                 int32_t* err_flag, void* stream);

namespace gnn {
namespace pb {

constexpr int kT = 256;
constexpr int kTaskRows = 63;  // spmm.hip kTaskRows
constexpr int kXcds = 8;       // graph.XCDS: workgroup w runs on XCD w % 8
constexpr int kWaves = 4;      // graph.SPMM_WAVES_PER_WG
constexpr int64_t kMaxSlices = 1024;
// Hub rank r belongs to slice (r / G) % S (graph.XCD_SLICE_GROUP): G = 4 consecutive ranks, 2 KiB
// of X at F = 128, stay together. With G = 1 an XCD's hub rows sit 4 KiB apart and the step
// is 2.8 % slower at cfg2 (tools/slice_group_ab.py, profiles/r04sg_slice_group_ab.log). G drops
// to 1 when fewer than S * G ranks may form items.
#ifndef GNN_XCD_SLICE_GROUP
#define GNN_XCD_SLICE_GROUP 4
#endif
constexpr int64_t kSliceGroup = GNN_XCD_SLICE_GROUP;

static inline unsigned grid(int64_t n) { return static_cast<unsigned>((n + kT - 1) / kT); }
static inline int64_t up(int64_t v) { return (v + 255) / 256 * 256; }

static unsigned bits_for(uint64_t max_value) {  // bits to hold values < max_value
  unsigned b = 1;
  while (b < 64 && (static_cast<uint64_t>(1) << b) < max_value) ++b;
  return b;
}

static int sync_read(const int64_t* dev, int64_t* host, int64_t count, hipStream_t s) {
  hipError_t e = hipMemcpyAsync(host, dev, count * sizeof(int64_t), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  return e == hipSuccess ? GNN_OK : static_cast<int>(e);
}

// bump allocator over the caller's workspace (256-byte aligned pieces)
struct Carve {
  char* p;
  int64_t used = 0;
  template <class T> T* take(int64_t n) {
    T* r = reinterpret_cast<T*>(p ? p + used : nullptr);
    used += up(n * static_cast<int64_t>(sizeof(T)));
    return r;
  }
};

typedef rocprim::counting_iterator<int64_t> Count;

// ------------------------------------------------------------------------- packed tasks
struct TaskCost {  // (edges + 1) of a row of degree <= max_deg, 0 for the others
  const int64_t* rp;
  int64_t n, max_deg;
  __host__ __device__ int64_t operator()(int64_t i) const {
    if (i >= n) return 0;
    const int64_t d = rp[i + 1] - rp[i];
    return d <= max_deg ? d + 1 : 0;
  }
};
struct RunHead {  // i at the first row of a run of packable rows, else -1
  const int64_t* rp;
  int64_t max_deg;
  __host__ __device__ int64_t operator()(int64_t i) const {
    const bool p = rp[i + 1] - rp[i] <= max_deg;
    const bool pp = i > 0 && rp[i] - rp[i - 1] <= max_deg;
    return (p && !pp) ? i : -1;
  }
};
struct Bit0 {
  const uint8_t* f;
  __host__ __device__ bool operator()(int64_t i) const { return (f[i] & 1) != 0; }
};
struct NotSentinel {
  __host__ __device__ bool operator()(uint64_t v) const { return v != ~0ull; }
};

// flags[i]: bit 0 = a task boundary (a task starts here, or the row is not packable),
// bit 1 = a task starts here. Same rule as graph.task_ranges.
__global__ void task_flags_kernel(const int64_t* __restrict__ rp, int64_t n, int64_t max_deg,
                                  int64_t cost, const int64_t* __restrict__ excl,
                                  const int64_t* __restrict__ first, uint8_t* __restrict__ flags) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t f = 1;
  if (rp[i + 1] - rp[i] <= max_deg) {
    const int64_t f0 = first[i];
    bool start = i == f0 || (i - f0) % kTaskRows == 0;
    if (!start) start = (excl[i] - excl[f0]) / cost != (excl[i - 1] - excl[f0]) / cost;
    f = start ? 3 : 0;
  }
  flags[i] = f;
}

// pair j of the boundary list: (begin, next boundary) when B[j] starts a task, else sentinel
__global__ void task_pairs_kernel(const int64_t* __restrict__ bounds, const int64_t* __restrict__ nb_dev,
                                  const uint8_t* __restrict__ flags, int64_t n,
                                  uint64_t* __restrict__ pairs) {
  const int64_t j = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const int64_t nb = *nb_dev;
  uint64_t v = ~0ull;
  if (j < nb) {
    const int64_t b = bounds[j];
    if (flags[b] & 2) {
      const int64_t e = j + 1 < nb ? bounds[j + 1] : n;
      v = static_cast<uint64_t>(static_cast<uint32_t>(b)) | (static_cast<uint64_t>(e) << 32);
    }
  }
  pairs[j] = v;
}

struct TaskWs {
  int64_t* excl;
  int64_t* first;
  uint8_t* flags;
  int64_t* bounds;
  uint64_t* pairs;
  int64_t* cnt;  // [2]: boundaries, tasks
  void* temp;
  size_t temp_bytes;
  int64_t bytes;
};

static size_t task_temp_bytes(int64_t n) {
  size_t a = 0, b = 0, c = 0, d = 0;
  const auto cost_it = rocprim::make_transform_iterator(Count(0), TaskCost{nullptr, 0, 0});
  const auto head_it = rocprim::make_transform_iterator(Count(0), RunHead{nullptr, 0});
  const auto flag_it = rocprim::make_transform_iterator(Count(0), Bit0{nullptr});
  (void)rocprim::exclusive_scan(nullptr, a, cost_it, static_cast<int64_t*>(nullptr), int64_t(0),
                                static_cast<size_t>(n), rocprim::plus<int64_t>());
  (void)rocprim::inclusive_scan(nullptr, b, head_it, static_cast<int64_t*>(nullptr),
                                static_cast<size_t>(n), rocprim::maximum<int64_t>());
  (void)rocprim::select(nullptr, c, Count(0), flag_it, static_cast<int64_t*>(nullptr),
                        static_cast<int64_t*>(nullptr), static_cast<size_t>(n));
  (void)rocprim::select(nullptr, d, static_cast<uint64_t*>(nullptr), static_cast<uint64_t*>(nullptr),
                        static_cast<int64_t*>(nullptr), static_cast<size_t>(n), NotSentinel{});
  size_t m = a > b ? a : b;
  m = m > c ? m : c;
  m = m > d ? m : d;
  return m + 256;
}

static TaskWs task_carve(void* ws, int64_t n) {
  Carve c{static_cast<char*>(ws)};
  TaskWs w{};
  const int64_t m = n > 0 ? n : 1;
  w.excl = c.take<int64_t>(m);
  w.first = c.take<int64_t>(m);
  w.flags = c.take<uint8_t>(m);
  w.bounds = c.take<int64_t>(m);
  w.pairs = c.take<uint64_t>(m);
  w.cnt = c.take<int64_t>(2);
  w.temp_bytes = task_temp_bytes(m);
  w.temp = c.take<char>(static_cast<int64_t>(w.temp_bytes));
  w.bytes = c.used;
  return w;
}

// ------------------------------------------------------------------------- column order
__global__ void order_keys_kernel(const uint32_t* __restrict__ deg, int64_t n,
                                  uint32_t* __restrict__ key, int64_t* __restrict__ ids) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  key[i] = ~deg[i];  // ascending key = descending degree; the stable sort keeps ids ascending
  ids[i] = i;
}
__global__ void order_mark_kernel(const int64_t* __restrict__ perm, int64_t prefix,
                                  uint8_t* __restrict__ in_prefix) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t < prefix) in_prefix[perm[t]] = 1;
}
struct NotMarked {
  const uint8_t* f;
  __host__ __device__ bool operator()(int64_t i) const { return f[i] == 0; }
};
__global__ void order_inv_kernel(const int64_t* __restrict__ perm, int64_t n, int64_t* __restrict__ inv) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t < n) inv[perm[t]] = t;
}
__global__ void order_rename_kernel(const int32_t* __restrict__ col, int64_t nnz,
                                    const int64_t* __restrict__ inv, int32_t* __restrict__ out) {
  const int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (e < nnz) out[e] = static_cast<int32_t>(inv[col[e]]);
}

struct OrderWs {
  uint32_t* deg;
  uint32_t* key0;
  uint32_t* key1;
  int64_t* ids;
  uint8_t* mark;
  int64_t* cnt;
  int32_t* err;
  void* temp;
  size_t temp_bytes;
  int64_t bytes;
};

static size_t order_temp_bytes(int64_t n) {
  size_t a = 0, b = 0;
  (void)rocprim::radix_sort_pairs(nullptr, a, static_cast<uint32_t*>(nullptr),
                                  static_cast<uint32_t*>(nullptr), static_cast<int64_t*>(nullptr),
                                  static_cast<int64_t*>(nullptr), static_cast<size_t>(n), 0, 32);
  const auto keep_it = rocprim::make_transform_iterator(Count(0), NotMarked{nullptr});
  (void)rocprim::select(nullptr, b, Count(0), keep_it, static_cast<int64_t*>(nullptr),
                        static_cast<int64_t*>(nullptr), static_cast<size_t>(n));
  return (a > b ? a : b) + 256;
}

static OrderWs order_carve(void* ws, int64_t n) {
  Carve c{static_cast<char*>(ws)};
  OrderWs w{};
  w.deg = c.take<uint32_t>(n);
  w.key0 = c.take<uint32_t>(n);
  w.key1 = c.take<uint32_t>(n);
  w.ids = c.take<int64_t>(n);
  w.mark = c.take<uint8_t>(n);
  w.cnt = c.take<int64_t>(1);
  w.err = c.take<int32_t>(1);
  w.temp_bytes = order_temp_bytes(n);
  w.temp = c.take<char>(static_cast<int64_t>(w.temp_bytes));
  w.bytes = c.used;
  return w;
}

// ------------------------------------------------------------------------- XCD hub plan
// State kept in the workspace from gnn_xcd_hub_plan_build to gnn_xcd_hub_plan_fill.
// hdr: [0] selected edges, [1] groups, [2] items, [3] moved edges, [4] positions,
//      [5] slice group G (ranks r of slice (r / G) % S), [8 ..] phase bases (phases + 1)
struct XcdWs {
  int64_t* hdr;
  int32_t* row_e;      // [E] row of each edge
  uint64_t* key0;      // [E] (row, slice) keys; after the sort: the unique keys
  uint64_t* key1;      // [E] sorted keys
  int64_t* eid0;       // [E] selected edge ids
  int64_t* eid1;       // [E] selected edge ids in (row, slice) order
  uint32_t* gcnt;      // [E] edges per (row, slice) group
  int64_t* gstart;     // [E + 1] first sorted edge of each group
  int64_t* nch;        // [E + 1] chunks (items) of each group, 0 when not moved
  int64_t* ibase;      // [E + 1] first item of each group
  uint32_t* it_slice;  // [I] slice of each item
  uint32_t* it_slice2; // [I] sorted by slice
  int64_t* it_idx0;    // [I] iota, then the rank of the item inside its slice
  int64_t* it_idx1;    // [I] items in slice order
  int64_t* it_row;     // [I] graph row of each item
  int64_t* it_e0;      // [I] first sorted edge of each item
  int32_t* it_cnt;     // [I] edges of each item
  int64_t* it_pos;     // [I] position (pass-1 row) of each item
  int64_t* row_delta;  // [N] items - moved edges per row
  int64_t* first_item; // [N] first item of each row
  uint8_t* moved_e;    // [E] edge moved to an item
  int64_t* kpre;       // [E + 1] exclusive prefix of the kept edges
  int64_t* cstart;     // [S] first slice-sorted item of each slice
  int64_t* cend;       // [S]
  void* temp;
  size_t temp_bytes;
  int64_t bytes;
};

struct EligOp {  // hub edge of the item_k hottest, in a row of degree >= min_row_deg
  const int64_t* rp;
  const int32_t* col;
  const int32_t* row_e;
  int64_t ik, min_row_deg;
  __host__ __device__ bool operator()(int64_t e) const {
    const int32_t c = col[e];
    if (c >= 0 || static_cast<int64_t>(c) < -ik) return false;
    const int32_t r = row_e[e];
    return rp[r + 1] - rp[r] >= min_row_deg;
  }
};
struct GroupCount {
  const uint32_t* gcnt;
  int64_t g;
  __host__ __device__ int64_t operator()(int64_t i) const { return i < g ? gcnt[i] : 0; }
};
struct Arr64 {
  const int64_t* a;
  int64_t n;
  __host__ __device__ int64_t operator()(int64_t i) const { return i < n ? a[i] : 0; }
};
struct KeptOp {
  const uint8_t* moved;
  int64_t n;
  __host__ __device__ int64_t operator()(int64_t e) const { return e < n ? 1 - moved[e] : 0; }
};
struct RestCount {
  const int64_t* rp;
  const int64_t* delta;
  int64_t n;
  __host__ __device__ int64_t operator()(int64_t r) const {
    return r < n ? rp[r + 1] - rp[r] + delta[r] : 0;
  }
};

// the item at pass-1 position p (or -1: a pad), by the layout of graph.xcd_hub_coo: the j-th
// item of slice s (phase s / 8) sits at base[phase] + ((j / W) * 8 + s % 8) * W + j % W
struct PosMap {
  const int64_t* base;  // [phases + 1]
  const int64_t* cstart;
  const int64_t* cend;
  const int64_t* by_slice;
  int64_t phases;
  __host__ __device__ int64_t item(int64_t p, int64_t* phase_out) const {
    int64_t ph = 0;
    while (ph + 1 < phases && base[ph + 1] <= p) ++ph;
    if (phase_out) *phase_out = ph;
    const int64_t local = p - base[ph];
    const int64_t rw = local / kWaves;
    const int64_t s = ph * kXcds + rw % kXcds;
    const int64_t j = (rw / kXcds) * kWaves + local % kWaves;
    return j < cend[s] - cstart[s] ? by_slice[cstart[s] + j] : -1;
  }
};
struct PosCount {
  PosMap m;
  const int32_t* it_cnt;
  int64_t n_pos;
  __host__ __device__ int64_t operator()(int64_t p) const {
    if (p >= n_pos) return 0;
    const int64_t it = m.item(p, nullptr);
    return it >= 0 ? it_cnt[it] : 2;
  }
};

__global__ void edge_row_kernel(const int64_t* __restrict__ rp, int64_t n, int64_t nnz,
                                int32_t* __restrict__ row_e) {
  const int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (e >= nnz) return;
  int64_t lo = 0, hi = n;  // last row r with rp[r] <= e
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) >> 1;
    if (rp[mid] <= e) lo = mid; else hi = mid;
  }
  row_e[e] = static_cast<int32_t>(lo);
}

__global__ void xcd_group_kernel(int64_t* __restrict__ hdr, int64_t gsz) {
  if (blockIdx.x == 0 && threadIdx.x == 0) hdr[5] = gsz;
}

__global__ void xcd_keys_kernel(const int64_t* __restrict__ eid, const int64_t* __restrict__ hdr,
                                const int32_t* __restrict__ col, const int32_t* __restrict__ row_e,
                                int64_t S, uint64_t* __restrict__ key) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= hdr[0]) return;
  const int64_t e = eid[t];
#ifdef GNN_XCD_SLICE_SNAKE  // A/B only: groups dealt back and forth (0..S-1, S-1..0, ...)
  const int64_t q = (-1 - static_cast<int64_t>(col[e])) / hdr[5];
  const int64_t s = (q / S) % 2 ? S - 1 - q % S : q % S;
#else
  const int64_t s = ((-1 - static_cast<int64_t>(col[e])) / hdr[5]) % S;
#endif
  key[t] = static_cast<uint64_t>(row_e[e]) * static_cast<uint64_t>(S) + static_cast<uint64_t>(s);
}

__global__ void xcd_groups_kernel(const uint64_t* __restrict__ ukey, const uint32_t* __restrict__ gcnt,
                                  int64_t G, const int64_t* __restrict__ rp, int64_t S,
                                  int64_t min_deg, int64_t small_item, int64_t chunk,
                                  int64_t* __restrict__ nch, int64_t* __restrict__ hdr) {
  const int64_t g = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (g >= G) return;
  const int64_t m = gcnt[g];
  const int64_t r = static_cast<int64_t>(ukey[g] / static_cast<uint64_t>(S));
  bool moved = m >= 2;  // a one-edge item saves nothing
  if (moved && small_item > 0) moved = rp[r + 1] - rp[r] >= min_deg || m >= small_item;
  nch[g] = moved ? (m + chunk - 1) / chunk : 0;
  if (moved) atomicAdd(reinterpret_cast<unsigned long long*>(hdr + 3),
                       static_cast<unsigned long long>(m));
}

__global__ void xcd_items_kernel(const uint64_t* __restrict__ ukey, const uint32_t* __restrict__ gcnt,
                                 int64_t G, int64_t S, const int64_t* __restrict__ nch,
                                 const int64_t* __restrict__ ibase, const int64_t* __restrict__ gstart,
                                 uint32_t* __restrict__ it_slice, int64_t* __restrict__ it_row,
                                 int64_t* __restrict__ it_e0, int32_t* __restrict__ it_cnt,
                                 int64_t* __restrict__ row_delta) {
  const int64_t g = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (g >= G) return;
  const int64_t nc = nch[g];
  if (nc == 0) return;
  const int64_t m = gcnt[g];
  const uint64_t k = ukey[g];
  const int64_t r = static_cast<int64_t>(k / static_cast<uint64_t>(S));
  const uint32_t s = static_cast<uint32_t>(k % static_cast<uint64_t>(S));
  // chunk ci holds the edges with pos * nc / m == ci: pos in [ceil(ci m / nc), ceil((ci+1) m / nc))
  for (int64_t ci = 0; ci < nc; ++ci) {
    const int64_t it = ibase[g] + ci;
    const int64_t a = (ci * m + nc - 1) / nc, b = ((ci + 1) * m + nc - 1) / nc;
    it_slice[it] = s;
    it_row[it] = r;
    it_e0[it] = gstart[g] + a;
    it_cnt[it] = static_cast<int32_t>(b - a);
  }
  // rows own consecutive groups; one atomic per group
  atomicAdd(reinterpret_cast<unsigned long long*>(row_delta + r),
            static_cast<unsigned long long>(nc - m));
}

__global__ void xcd_moved_kernel(const int64_t* __restrict__ eid1, int64_t n_sel,
                                 const int64_t* __restrict__ gstart, const int64_t* __restrict__ nch,
                                 int64_t G, uint8_t* __restrict__ moved_e) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= n_sel) return;
  int64_t lo = 0, hi = G;  // last group g with gstart[g] <= t
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) >> 1;
    if (gstart[mid] <= t) lo = mid; else hi = mid;
  }
  if (nch[lo] > 0) moved_e[eid1[t]] = 1;
}

__global__ void iota_kernel(int64_t* __restrict__ a, int64_t n) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) a[i] = i;
}

__global__ void xcd_slice_bounds_kernel(const uint32_t* __restrict__ s2, int64_t I,
                                        int64_t* __restrict__ cstart, int64_t* __restrict__ cend) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= I) return;
  const uint32_t s = s2[t];
  if (t == 0 || s2[t - 1] != s) cstart[s] = t;
  if (t == I - 1 || s2[t + 1] != s) cend[s] = t + 1;
}

__global__ void xcd_rank_kernel(const uint32_t* __restrict__ s2, const int64_t* __restrict__ by_slice,
                                int64_t I, const int64_t* __restrict__ cstart,
                                int64_t* __restrict__ rank) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t < I) rank[by_slice[t]] = t - cstart[s2[t]];
}

// one thread: per-phase extents (the largest slice of the phase, rounded up to W) -> bases
__global__ void xcd_bases_kernel(const int64_t* __restrict__ cstart, const int64_t* __restrict__ cend,
                                 int64_t phases, int64_t* __restrict__ hdr) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  int64_t b = 0;
  hdr[8] = 0;
  for (int64_t p = 0; p < phases; ++p) {
    int64_t mx = 0;
    for (int x = 0; x < kXcds; ++x) {
      const int64_t s = p * kXcds + x;
      const int64_t c = cend[s] - cstart[s];
      mx = c > mx ? c : mx;
    }
    b += (mx + kWaves - 1) / kWaves * kWaves * kXcds;
    hdr[9 + p] = b;
  }
  hdr[4] = b;
}

__global__ void xcd_pos_kernel(const uint32_t* __restrict__ it_slice, const int64_t* __restrict__ rank,
                               int64_t I, const int64_t* __restrict__ hdr, int64_t* __restrict__ it_pos) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= I) return;
  const int64_t s = it_slice[i], j = rank[i];
  it_pos[i] = hdr[8 + s / kXcds] + ((j / kWaves) * kXcds + s % kXcds) * kWaves + j % kWaves;
}

__global__ void xcd_first_item_kernel(const int64_t* __restrict__ it_row, int64_t I,
                                      int64_t* __restrict__ first_item) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= I) return;
  if (i == 0 || it_row[i - 1] != it_row[i]) first_item[it_row[i]] = i;
}

__global__ void xcd_fill_items_kernel(PosMap pm, const int64_t* __restrict__ hdr, int64_t n_pos,
                                      const int64_t* __restrict__ irp,
                                      const int64_t* __restrict__ it_e0, const int32_t* __restrict__ it_cnt,
                                      const int64_t* __restrict__ it_row, const int64_t* __restrict__ eid1,
                                      const int32_t* __restrict__ col, const float* __restrict__ val,
                                      int32_t* __restrict__ icol, float* __restrict__ ival,
                                      int64_t* __restrict__ pos_row) {
  const int64_t p = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (p >= n_pos) return;
  int64_t ph = 0;
  const int64_t it = pm.item(p, &ph);
  const int64_t o = irp[p];
  if (it >= 0) {
    const int64_t e0 = it_e0[it];
    for (int32_t q = 0; q < it_cnt[it]; ++q) {
      const int64_t e = eid1[e0 + q];
      icol[o + q] = col[e];
      ival[o + q] = val[e];
    }
    pos_row[p] = it_row[it];
  } else {  // a pad: two zero-valued edges to a row of its own slice
    const int64_t pc = -1 - (ph * kXcds + ((p - pm.base[ph]) / kWaves) % kXcds) * hdr[5];
    icol[o] = static_cast<int32_t>(pc);
    icol[o + 1] = static_cast<int32_t>(pc);
    ival[o] = 0.f;
    ival[o + 1] = 0.f;
    pos_row[p] = 0;
  }
}

__global__ void xcd_fill_kept_kernel(const int64_t* __restrict__ rp, const int32_t* __restrict__ row_e,
                                     int64_t nnz, const uint8_t* __restrict__ moved_e,
                                     const int64_t* __restrict__ kpre, const int64_t* __restrict__ rrp,
                                     const int32_t* __restrict__ col, const float* __restrict__ val,
                                     int32_t* __restrict__ rcol, float* __restrict__ rval) {
  const int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (e >= nnz || moved_e[e]) return;
  const int64_t r = row_e[e];
  const int64_t o = rrp[r] + kpre[e] - kpre[rp[r]];
  rcol[o] = col[e];
  rval[o] = val[e];
}

__global__ void xcd_fill_refs_kernel(const int64_t* __restrict__ rp, const int64_t* __restrict__ it_row,
                                     const int64_t* __restrict__ it_pos, int64_t I, int64_t k,
                                     const int64_t* __restrict__ first_item,
                                     const int64_t* __restrict__ kpre, const int64_t* __restrict__ rrp,
                                     int32_t* __restrict__ rcol, float* __restrict__ rval) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= I) return;
  const int64_t r = it_row[i];
  const int64_t kept = kpre[rp[r + 1]] - kpre[rp[r]];
  const int64_t o = rrp[r] + kept + (i - first_item[r]);
  rcol[o] = static_cast<int32_t>(-1 - (k + it_pos[i]));
  rval[o] = 1.f;
}

static size_t xcd_temp_bytes(int64_t E, int64_t N, int64_t I) {
  size_t t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const auto elig_it = rocprim::make_transform_iterator(Count(0), EligOp{nullptr, nullptr, nullptr, 0, 0});
  (void)rocprim::select(nullptr, t[0], Count(0), elig_it, static_cast<int64_t*>(nullptr),
                        static_cast<int64_t*>(nullptr), static_cast<size_t>(E));
  (void)rocprim::radix_sort_pairs(nullptr, t[1], static_cast<uint64_t*>(nullptr),
                                  static_cast<uint64_t*>(nullptr), static_cast<int64_t*>(nullptr),
                                  static_cast<int64_t*>(nullptr), static_cast<size_t>(E), 0, 64);
  (void)rocprim::run_length_encode(nullptr, t[2], static_cast<uint64_t*>(nullptr),
                                   static_cast<unsigned int>(E), static_cast<uint64_t*>(nullptr),
                                   static_cast<uint32_t*>(nullptr), static_cast<int64_t*>(nullptr));
  const auto gc_it = rocprim::make_transform_iterator(Count(0), GroupCount{nullptr, 0});
  (void)rocprim::exclusive_scan(nullptr, t[3], gc_it, static_cast<int64_t*>(nullptr), int64_t(0),
                                static_cast<size_t>(E + 1), rocprim::plus<int64_t>());
  const auto a_it = rocprim::make_transform_iterator(Count(0), Arr64{nullptr, 0});
  const size_t big = static_cast<size_t>((E > N ? E : N) + 1);
  (void)rocprim::exclusive_scan(nullptr, t[4], a_it, static_cast<int64_t*>(nullptr), int64_t(0), big,
                                rocprim::plus<int64_t>());
  (void)rocprim::radix_sort_pairs(nullptr, t[5], static_cast<uint32_t*>(nullptr),
                                  static_cast<uint32_t*>(nullptr), static_cast<int64_t*>(nullptr),
                                  static_cast<int64_t*>(nullptr), static_cast<size_t>(I), 0, 32);
  const auto k_it = rocprim::make_transform_iterator(Count(0), KeptOp{nullptr, 0});
  (void)rocprim::exclusive_scan(nullptr, t[6], k_it, static_cast<int64_t*>(nullptr), int64_t(0),
                                static_cast<size_t>(E + 1), rocprim::plus<int64_t>());
  const auto r_it = rocprim::make_transform_iterator(Count(0), RestCount{nullptr, nullptr, 0});
  (void)rocprim::exclusive_scan(nullptr, t[7], r_it, static_cast<int64_t*>(nullptr), int64_t(0),
                                static_cast<size_t>(N + 1), rocprim::plus<int64_t>());
  size_t m = 0;
  for (size_t v : t) m = v > m ? v : m;
  // the position scan (PosCount) has the transform-scan shape of the ones above, at most
  // 8 * I + 32 * phases elements: query it at that bound too
  size_t p = 0;
  const auto p_it = rocprim::make_transform_iterator(
      Count(0), PosCount{PosMap{nullptr, nullptr, nullptr, nullptr, 0}, nullptr, 0});
  (void)rocprim::exclusive_scan(nullptr, p, p_it, static_cast<int64_t*>(nullptr), int64_t(0),
                                static_cast<size_t>(8 * I + kWaves * kXcds * kMaxSlices + 1),
                                rocprim::plus<int64_t>());
  m = p > m ? p : m;
  return m + 256;
}

static XcdWs xcd_carve(void* ws, int64_t E, int64_t N) {
  const int64_t e = E > 0 ? E : 1, n = N > 0 ? N : 1, I = e / 2 + 1;
  Carve c{static_cast<char*>(ws)};
  XcdWs w{};
  w.hdr = c.take<int64_t>(16 + kMaxSlices);
  w.row_e = c.take<int32_t>(e);
  w.key0 = c.take<uint64_t>(e);
  w.key1 = c.take<uint64_t>(e);
  w.eid0 = c.take<int64_t>(e);
  w.eid1 = c.take<int64_t>(e);
  w.gcnt = c.take<uint32_t>(e);
  w.gstart = c.take<int64_t>(e + 1);
  w.nch = c.take<int64_t>(e + 1);
  w.ibase = c.take<int64_t>(e + 1);
  w.it_slice = c.take<uint32_t>(I);
  w.it_slice2 = c.take<uint32_t>(I);
  w.it_idx0 = c.take<int64_t>(I);
  w.it_idx1 = c.take<int64_t>(I);
  w.it_row = c.take<int64_t>(I);
  w.it_e0 = c.take<int64_t>(I);
  w.it_cnt = c.take<int32_t>(I);
  w.it_pos = c.take<int64_t>(I);
  w.row_delta = c.take<int64_t>(n);
  w.first_item = c.take<int64_t>(n);
  w.moved_e = c.take<uint8_t>(e);
  w.kpre = c.take<int64_t>(e + 1);
  w.cstart = c.take<int64_t>(kMaxSlices);
  w.cend = c.take<int64_t>(kMaxSlices);
  w.temp_bytes = xcd_temp_bytes(e, n, I);
  w.temp = c.take<char>(static_cast<int64_t>(w.temp_bytes));
  w.bytes = c.used;
  return w;
}

#define PB_TRY(x)                                       \
  do {                                                  \
    hipError_t e_ = (x);                                \
    if (e_ != hipSuccess) return static_cast<int>(e_);  \
  } while (0)

}  // namespace pb
}  // namespace gnn

using namespace gnn;
using namespace gnn::pb;

// ============================================================================ packed tasks
extern "C" int64_t gnn_spmm_tasks_workspace_bytes(int64_t n_rows) {
  if (n_rows < 0) return GNN_E_ARG;
  return task_carve(nullptr, n_rows).bytes;
}

extern "C" int gnn_spmm_tasks_build(const int64_t* rowptr, int64_t n_rows, int64_t max_deg,
                                    int64_t cost, int32_t* task_row, int64_t cap_tasks,
                                    int64_t* n_task, void* workspace, int64_t workspace_bytes,
                                    void* stream) {
  if (n_rows < 0 || !n_task || cost < 1 || cap_tasks < 0 || (n_rows > 0 && (!rowptr || !workspace)))
    return GNN_E_ARG;
  if (n_rows > 0x7fffffffLL) return GNN_E_UNSUPPORTED;  // int32 task bounds
  *n_task = 0;
  if (n_rows == 0) return GNN_OK;
  if (workspace_bytes < gnn_spmm_tasks_workspace_bytes(n_rows)) return GNN_E_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  TaskWs w = task_carve(workspace, n_rows);
  const size_t n = static_cast<size_t>(n_rows);
  size_t tb = w.temp_bytes;
  const auto cost_it = rocprim::make_transform_iterator(Count(0), TaskCost{rowptr, n_rows, max_deg});
  PB_TRY(rocprim::exclusive_scan(w.temp, tb, cost_it, w.excl, int64_t(0), n, rocprim::plus<int64_t>(), s));
  tb = w.temp_bytes;
  const auto head_it = rocprim::make_transform_iterator(Count(0), RunHead{rowptr, max_deg});
  PB_TRY(rocprim::inclusive_scan(w.temp, tb, head_it, w.first, n, rocprim::maximum<int64_t>(), s));
  hipLaunchKernelGGL(task_flags_kernel, dim3(grid(n_rows)), dim3(kT), 0, s, rowptr, n_rows, max_deg,
                     cost, w.excl, w.first, w.flags);
  tb = w.temp_bytes;
  const auto flag_it = rocprim::make_transform_iterator(Count(0), Bit0{w.flags});
  PB_TRY(rocprim::select(w.temp, tb, Count(0), flag_it, w.bounds, w.cnt, n, s));
  hipLaunchKernelGGL(task_pairs_kernel, dim3(grid(n_rows)), dim3(kT), 0, s, w.bounds, w.cnt, w.flags,
                     n_rows, w.pairs);
  tb = w.temp_bytes;
  PB_TRY(rocprim::select(w.temp, tb, w.pairs, reinterpret_cast<uint64_t*>(w.excl), w.cnt + 1, n,
                         NotSentinel{}, s));
  int64_t nt = 0;
  int rc = sync_read(w.cnt + 1, &nt, 1, s);
  if (rc != GNN_OK) return rc;
  *n_task = nt;
  if (!task_row) return launch_status();
  if (nt > cap_tasks) return GNN_E_ARG;  // *n_task says how many pairs to make room for
  if (nt > 0)
    PB_TRY(hipMemcpyAsync(task_row, w.excl, static_cast<size_t>(nt) * 8, hipMemcpyDeviceToDevice, s));
  return launch_status();
}

// ============================================================================ column order
extern "C" int64_t gnn_column_order_workspace_bytes(int64_t n_cols) {
  if (n_cols < 1) return GNN_E_ARG;
  return order_carve(nullptr, n_cols).bytes;
}

extern "C" int gnn_column_order(const int32_t* col, int64_t nnz, int64_t n_cols, int64_t prefix,
                                int64_t* perm, int64_t* inv, int32_t* col_out, void* workspace,
                                int64_t workspace_bytes, void* stream) {
  if (nnz < 0 || n_cols < 1 || !perm || !inv || !workspace || (nnz > 0 && (!col || !col_out)))
    return GNN_E_ARG;
  if (n_cols > 0x7fffffffLL) return GNN_E_UNSUPPORTED;  // int32 column ids
  if (workspace_bytes < gnn_column_order_workspace_bytes(n_cols)) return GNN_E_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  OrderWs w = order_carve(workspace, n_cols);
  PB_TRY(hipMemsetAsync(w.err, 0, sizeof(int32_t), s));
  if (nnz == 0) PB_TRY(hipMemsetAsync(w.deg, 0, static_cast<size_t>(n_cols) * 4, s));
  if (nnz > 0) {
    const int rc = gnn_in_degree_u32(col, nnz, n_cols, w.deg, w.err, stream);
    if (rc != GNN_OK) return rc;
    int64_t herr = 0;
    PB_TRY(hipMemcpyAsync(&herr, w.err, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    PB_TRY(hipStreamSynchronize(s));
    if (herr) return GNN_E_ARG;  // a column id outside [0, n_cols)
  }
  const size_t n = static_cast<size_t>(n_cols);
  hipLaunchKernelGGL(order_keys_kernel, dim3(grid(n_cols)), dim3(kT), 0, s, w.deg, n_cols, w.key0, w.ids);
  size_t tb = w.temp_bytes;
  PB_TRY(rocprim::radix_sort_pairs(w.temp, tb, w.key0, w.key1, w.ids, perm, n, 0, 32, s));
  if (prefix >= 0 && prefix < n_cols) {
    // the ids after the prefix in ascending order (graph.degree_order's default tail)
    PB_TRY(hipMemsetAsync(w.mark, 0, n, s));
    if (prefix > 0)
      hipLaunchKernelGGL(order_mark_kernel, dim3(grid(prefix)), dim3(kT), 0, s, perm, prefix, w.mark);
    tb = w.temp_bytes;
    const auto keep_it = rocprim::make_transform_iterator(Count(0), NotMarked{w.mark});
    PB_TRY(rocprim::select(w.temp, tb, Count(0), keep_it, perm + prefix, w.cnt, n, s));
  }
  hipLaunchKernelGGL(order_inv_kernel, dim3(grid(n_cols)), dim3(kT), 0, s, perm, n_cols, inv);
  if (nnz > 0)
    hipLaunchKernelGGL(order_rename_kernel, dim3(grid(nnz)), dim3(kT), 0, s, col, nnz, inv, col_out);
  return launch_status();
}

// ============================================================================ XCD hub plan
// the compile-time slice group G of this builder (graph.XCD_SLICE_GROUP must agree for the
// package to use it; a different Python value selects the torch builder, which honours it)
extern "C" int64_t gnn_xcd_slice_group(void) { return kSliceGroup; }

extern "C" int64_t gnn_xcd_hub_plan_workspace_bytes(int64_t n_rows, int64_t nnz) {
  if (n_rows < 1 || nnz < 0) return GNN_E_ARG;
  return xcd_carve(nullptr, nnz, n_rows).bytes;
}

extern "C" int gnn_xcd_hub_plan_build(const int64_t* rowptr, const int32_t* col_hub,
                                      int64_t n_rows, int64_t nnz, int64_t k, int64_t min_deg,
                                      int64_t chunk, int64_t phases, int64_t item_k,
                                      int64_t small_item, int64_t* counts, void* workspace,
                                      int64_t workspace_bytes, void* stream) {
  if (n_rows < 1 || nnz < 0 || !rowptr || !counts || !workspace || (nnz > 0 && !col_hub))
    return GNN_E_ARG;
  const int64_t S = kXcds * phases;
  const int64_t ik = item_k > 0 && item_k < k ? item_k : k;
  if (chunk < 4 || phases < 1 || S > kMaxSlices || k < S || ik < S || (small_item != 0 && small_item < 2))
    return GNN_E_ARG;  // graph.xcd_hub_coo's ValueErrors
  if (n_rows > 0x7fffffffLL || nnz > 0xffffffffLL) return GNN_E_UNSUPPORTED;
  if (workspace_bytes < gnn_xcd_hub_plan_workspace_bytes(n_rows, nnz)) return GNN_E_ARG;
  for (int i = 0; i < 4; ++i) counts[i] = 0;
  if (nnz == 0) return GNN_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  XcdWs w = xcd_carve(workspace, nnz, n_rows);
  PB_TRY(hipMemsetAsync(w.hdr, 0, (16 + kMaxSlices) * sizeof(int64_t), s));
  const int64_t gsz = kSliceGroup > 1 && ik >= S * kSliceGroup ? kSliceGroup : 1;
  hipLaunchKernelGGL(xcd_group_kernel, dim3(1), dim3(64), 0, s, w.hdr, gsz);
  hipLaunchKernelGGL(edge_row_kernel, dim3(grid(nnz)), dim3(kT), 0, s, rowptr, n_rows, nnz, w.row_e);
  // 1. the hub edges that may form items, by (row, slice), CSR order kept inside a group
  size_t tb = w.temp_bytes;
  const auto elig_it = rocprim::make_transform_iterator(
      Count(0), EligOp{rowptr, col_hub, w.row_e, ik, small_item > 0 ? 2 : min_deg});
  PB_TRY(rocprim::select(w.temp, tb, Count(0), elig_it, w.eid0, w.hdr, static_cast<size_t>(nnz), s));
  int64_t n_sel = 0;
  int rc = sync_read(w.hdr, &n_sel, 1, s);
  if (rc != GNN_OK) return rc;
  if (n_sel == 0) return launch_status();
  hipLaunchKernelGGL(xcd_keys_kernel, dim3(grid(n_sel)), dim3(kT), 0, s, w.eid0, w.hdr, col_hub,
                     w.row_e, S, w.key0);
  tb = w.temp_bytes;
  const unsigned kbits = bits_for(static_cast<uint64_t>(n_rows) * static_cast<uint64_t>(S));
  PB_TRY(rocprim::radix_sort_pairs(w.temp, tb, w.key0, w.key1, w.eid0, w.eid1,
                                   static_cast<size_t>(n_sel), 0, kbits, s));
  // 2. groups = (row, slice) runs; moved groups of >= 2 edges are cut into balanced chunks
  tb = w.temp_bytes;
  PB_TRY(rocprim::run_length_encode(w.temp, tb, w.key1, static_cast<unsigned int>(n_sel), w.key0,
                                    w.gcnt, w.hdr + 1, s));
  int64_t G = 0;
  if ((rc = sync_read(w.hdr + 1, &G, 1, s)) != GNN_OK) return rc;
  hipLaunchKernelGGL(xcd_groups_kernel, dim3(grid(G)), dim3(kT), 0, s, w.key0, w.gcnt, G, rowptr, S,
                     min_deg, small_item, chunk, w.nch, w.hdr);
  tb = w.temp_bytes;
  const auto gc_it = rocprim::make_transform_iterator(Count(0), GroupCount{w.gcnt, G});
  PB_TRY(rocprim::exclusive_scan(w.temp, tb, gc_it, w.gstart, int64_t(0), static_cast<size_t>(G + 1),
                                 rocprim::plus<int64_t>(), s));
  tb = w.temp_bytes;
  const auto nch_it = rocprim::make_transform_iterator(Count(0), Arr64{w.nch, G});
  PB_TRY(rocprim::exclusive_scan(w.temp, tb, nch_it, w.ibase, int64_t(0), static_cast<size_t>(G + 1),
                                 rocprim::plus<int64_t>(), s));
  PB_TRY(hipMemcpyAsync(w.hdr + 2, w.ibase + G, sizeof(int64_t), hipMemcpyDeviceToDevice, s));
  int64_t h[4];
  if ((rc = sync_read(w.hdr, h, 4, s)) != GNN_OK) return rc;
  const int64_t I = h[2], n_moved = h[3];
  if (I == 0) return launch_status();  // no row has two hub edges in one slice
  // 3. items: slice, row, edge range; per-row deltas; moved-edge marks
  PB_TRY(hipMemsetAsync(w.row_delta, 0, static_cast<size_t>(n_rows) * 8, s));
  hipLaunchKernelGGL(xcd_items_kernel, dim3(grid(G)), dim3(kT), 0, s, w.key0, w.gcnt, G, S, w.nch,
                     w.ibase, w.gstart, w.it_slice, w.it_row, w.it_e0, w.it_cnt, w.row_delta);
  PB_TRY(hipMemsetAsync(w.moved_e, 0, static_cast<size_t>(nnz), s));
  hipLaunchKernelGGL(xcd_moved_kernel, dim3(grid(n_sel)), dim3(kT), 0, s, w.eid1, n_sel, w.gstart,
                     w.nch, G, w.moved_e);
  // 4. rank of each item inside its slice (stable: item order), positions per phase
  hipLaunchKernelGGL(iota_kernel, dim3(grid(I)), dim3(kT), 0, s, w.it_idx0, I);
  tb = w.temp_bytes;
  PB_TRY(rocprim::radix_sort_pairs(w.temp, tb, w.it_slice, w.it_slice2, w.it_idx0, w.it_idx1,
                                   static_cast<size_t>(I), 0, bits_for(static_cast<uint64_t>(S)), s));
  PB_TRY(hipMemsetAsync(w.cstart, 0, kMaxSlices * 8, s));
  PB_TRY(hipMemsetAsync(w.cend, 0, kMaxSlices * 8, s));
  hipLaunchKernelGGL(xcd_slice_bounds_kernel, dim3(grid(I)), dim3(kT), 0, s, w.it_slice2, I, w.cstart,
                     w.cend);
  hipLaunchKernelGGL(xcd_rank_kernel, dim3(grid(I)), dim3(kT), 0, s, w.it_slice2, w.it_idx1, I,
                     w.cstart, w.it_idx0);
  hipLaunchKernelGGL(xcd_bases_kernel, dim3(1), dim3(64), 0, s, w.cstart, w.cend, phases, w.hdr);
  hipLaunchKernelGGL(xcd_pos_kernel, dim3(grid(I)), dim3(kT), 0, s, w.it_slice, w.it_idx0, I, w.hdr,
                     w.it_pos);
  hipLaunchKernelGGL(xcd_first_item_kernel, dim3(grid(I)), dim3(kT), 0, s, w.it_row, I, w.first_item);
  tb = w.temp_bytes;
  const auto k_it = rocprim::make_transform_iterator(Count(0), KeptOp{w.moved_e, nnz});
  PB_TRY(rocprim::exclusive_scan(w.temp, tb, k_it, w.kpre, int64_t(0), static_cast<size_t>(nnz + 1),
                                 rocprim::plus<int64_t>(), s));
  int64_t n_pos = 0;
  if ((rc = sync_read(w.hdr + 4, &n_pos, 1, s)) != GNN_OK) return rc;
  counts[0] = I;
  counts[1] = n_pos;
  counts[2] = n_moved + 2 * (n_pos - I);  // item edges + two per pad position
  counts[3] = nnz - n_moved + I;          // kept edges + one partial ref per item
  return launch_status();
}

extern "C" int gnn_xcd_hub_plan_fill(const void* workspace, const int64_t* rowptr,
                                     const int32_t* col_hub, const float* val, int64_t n_rows,
                                     int64_t nnz, int64_t k, int64_t phases, const int64_t* counts,
                                     int64_t* items_rowptr, int32_t* items_col, float* items_val,
                                     int64_t* pos_row, int64_t* rest_rowptr, int32_t* rest_col,
                                     float* rest_val, void* stream) {
  if (!workspace || !rowptr || !col_hub || !val || !counts || n_rows < 1 || nnz < 1 || phases < 1 ||
      kXcds * phases > kMaxSlices)
    return GNN_E_ARG;
  const int64_t I = counts[0], n_pos = counts[1];
  if (I < 1 || n_pos < I || !items_rowptr || !items_col || !items_val || !pos_row || !rest_rowptr ||
      !rest_col || !rest_val)
    return GNN_E_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  XcdWs w = xcd_carve(const_cast<void*>(workspace), nnz, n_rows);
  const PosMap pm{w.hdr + 8, w.cstart, w.cend, w.it_idx1, phases};
  size_t tb = w.temp_bytes;
  const auto p_it = rocprim::make_transform_iterator(Count(0), PosCount{pm, w.it_cnt, n_pos});
  PB_TRY(rocprim::exclusive_scan(w.temp, tb, p_it, items_rowptr, int64_t(0),
                                 static_cast<size_t>(n_pos + 1), rocprim::plus<int64_t>(), s));
  hipLaunchKernelGGL(xcd_fill_items_kernel, dim3(grid(n_pos)), dim3(kT), 0, s, pm, w.hdr, n_pos,
                     items_rowptr,
                     w.it_e0, w.it_cnt, w.it_row, w.eid1, col_hub, val, items_col, items_val, pos_row);
  tb = w.temp_bytes;
  const auto r_it = rocprim::make_transform_iterator(Count(0), RestCount{rowptr, w.row_delta, n_rows});
  PB_TRY(rocprim::exclusive_scan(w.temp, tb, r_it, rest_rowptr, int64_t(0),
                                 static_cast<size_t>(n_rows + 1), rocprim::plus<int64_t>(), s));
  hipLaunchKernelGGL(xcd_fill_kept_kernel, dim3(grid(nnz)), dim3(kT), 0, s, rowptr, w.row_e, nnz,
                     w.moved_e, w.kpre, rest_rowptr, col_hub, val, rest_col, rest_val);
  hipLaunchKernelGGL(xcd_fill_refs_kernel, dim3(grid(I)), dim3(kT), 0, s, rowptr, w.it_row, w.it_pos,
                     I, k, w.first_item, w.kpre, rest_rowptr, rest_col, rest_val);
  return launch_status();
}
