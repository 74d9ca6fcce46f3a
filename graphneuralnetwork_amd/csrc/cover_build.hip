// cover_build.hip -- the edge-cut cover exchange of the N-rank SpMM built on the device, so a C
// caller can set up the multi-GPU path (distributed.build_cover_exchange) without Python.
//
// Rank p owns rows [b_p, b_{p+1}) of A and of X. Every edge (i, j) of its rows whose column j
// belongs to another rank q (a cut edge) is covered EITHER by shipping X_j from q to p (column
// cover) OR by q computing the partial row sum s_qi = sum_{j in q} A_ij X_j (row cover), per
// the greedy rule of distributed.build_cover_exchange:
//   part  = cnt(i, q) > cnt(j)            (edges of the pair (row i, owner q) vs edges of column j)
//   part  = any part over the pair        (a row already shipped as a partial takes all its edges)
//   part &= no non-part edge on column j  (a column already shipped serves all its edges)
// gnn_cover_build computes it with dense per-(q, row) and per-column arrays (atomics for the
// counts, benign same-value stores for the flags), rocPRIM scans / selects / one stable sort;
// gnn_cover_fill writes the CSR pieces and the request lists; after the caller's handshake
// (all-to-all of the per-peer counts, all-to-all-v of the requests) gnn_cover_send_partials
// builds the partial-sum CSR this rank computes for its peers. The arrays equal the torch
// builder's (tests/test_cover_build_gpu.py).
#include <cstring>  // rocprim's texture_cache_iterator calls host memset

#include <rocprim/rocprim.hpp>

#include "common.hpp"

namespace gnn {
namespace cb {

constexpr int kT = 256;
constexpr int kMaxWorld = 64;

static inline unsigned grid(int64_t n) { return static_cast<unsigned>((n + kT - 1) / kT); }
static inline int64_t up(int64_t v) { return (v + 255) / 256 * 256; }

struct Bounds {  // row boundaries by value (no host-to-device copy of a caller's array)
  int64_t b[kMaxWorld + 1];
  int world;
  __host__ __device__ int owner(int64_t c) const {  // last q with b[q] <= c
    int lo = 0, hi = world;
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (b[mid] <= c) lo = mid; else hi = mid;
    }
    return lo;
  }
};

struct Carve {
  char* p;
  int64_t used = 0;
  template <class T> T* take(int64_t n) {
    T* r = reinterpret_cast<T*>(p ? p + used : nullptr);
    used += up((n > 0 ? n : 1) * static_cast<int64_t>(sizeof(T)));
    return r;
  }
};

typedef rocprim::counting_iterator<int64_t> Count;

// edge classes
constexpr uint8_t kInterior = 0, kFeature = 1, kPartial = 2;

struct CoverWs {
  int32_t* e_row;    // [E] local row of each local edge
  uint8_t* e_cls;    // [E]
  int32_t* cnt_pair; // [W * n_own] cut edges per (owner q, row), q-major
  uint8_t* hp;       // [W * n_own] pair takes partials (after the first refinement)
  uint8_t* pk;       // [W * n_own] pair ships a partial row (final)
  int32_t* cnt_col;  // [n] cut edges per column
  uint8_t* hx;       // [n] column shipped as a feature row
  int64_t* kpre;     // [E + 1] interior edges before each edge
  int64_t* xpre;     // [E + 1] feature-covered edges before each edge
  int64_t* xrank;    // [n + 1] requested columns before each column
  int64_t* pscan;    // [W * n_own + 1] partial rows before each pair
  int64_t* p_idx0;   // [E] partial edges (local edge ids), edge order
  int64_t* p_idx1;   // [E] sorted by (q, row)
  uint64_t* p_key0;  // [E]
  uint64_t* p_key1;  // [E]
  int64_t* hp_cnt;   // [n_own + 1] partial rows per row (halo_p degrees)
  int64_t* qb;       // [2 W] first / end of each owner's partial edges in sorted order
  int64_t* cnt;      // [4] select counts
  int32_t* err;      // [1] a column id outside [0, n_rows)
  int64_t* out;      // [4 + 3 W] the counts handed back (one host read)
  void* temp;
  size_t temp_bytes;
  int64_t bytes;
};

struct ClsIs {
  const uint8_t* c;
  uint8_t v;
  int64_t n;
  __host__ __device__ int64_t operator()(int64_t e) const { return e < n && c[e] == v ? 1 : 0; }
};
struct ByteAt {
  const uint8_t* f;
  int64_t n;
  __host__ __device__ int64_t operator()(int64_t i) const { return i < n ? f[i] : 0; }
};
struct ClsFlag {
  const uint8_t* c;
  uint8_t v;
  __host__ __device__ bool operator()(int64_t e) const { return c[e] == v; }
};
struct Arr {
  const int64_t* a;
  int64_t n;
  __host__ __device__ int64_t operator()(int64_t i) const { return i < n ? a[i] : 0; }
};

static size_t cover_temp_bytes(int64_t E, int64_t n, int64_t P, int64_t n_own) {
  size_t t[6] = {0, 0, 0, 0, 0, 0};
  const auto c_it = rocprim::make_transform_iterator(Count(0), ClsIs{nullptr, 0, 0});
  (void)rocprim::exclusive_scan(nullptr, t[0], c_it, static_cast<int64_t*>(nullptr), int64_t(0),
                                static_cast<size_t>(E + 1), rocprim::plus<int64_t>());
  const auto b_it = rocprim::make_transform_iterator(Count(0), ByteAt{nullptr, 0});
  const size_t big = static_cast<size_t>((n > P ? n : P) + 1);
  (void)rocprim::exclusive_scan(nullptr, t[1], b_it, static_cast<int64_t*>(nullptr), int64_t(0), big,
                                rocprim::plus<int64_t>());
  const auto f_it = rocprim::make_transform_iterator(Count(0), ClsFlag{nullptr, 0});
  (void)rocprim::select(nullptr, t[2], Count(0), f_it, static_cast<int64_t*>(nullptr),
                        static_cast<int64_t*>(nullptr), static_cast<size_t>(E > n ? E : n));
  (void)rocprim::radix_sort_pairs(nullptr, t[3], static_cast<uint64_t*>(nullptr),
                                  static_cast<uint64_t*>(nullptr), static_cast<int64_t*>(nullptr),
                                  static_cast<int64_t*>(nullptr), static_cast<size_t>(E), 0, 64);
  const auto a_it = rocprim::make_transform_iterator(Count(0), Arr{nullptr, 0});
  (void)rocprim::exclusive_scan(nullptr, t[4], a_it, static_cast<int64_t*>(nullptr), int64_t(0),
                                static_cast<size_t>(n_own + 1), rocprim::plus<int64_t>());
  // the select of requested columns runs over hx (ByteAt-shaped flags)
  const auto h_it = rocprim::make_transform_iterator(Count(0), ByteAt{nullptr, 0});
  (void)rocprim::select(nullptr, t[5], Count(0), h_it, static_cast<int64_t*>(nullptr),
                        static_cast<int64_t*>(nullptr), static_cast<size_t>(n));
  size_t m = 0;
  for (size_t v : t) m = v > m ? v : m;
  return m + 256;
}

static CoverWs cover_carve(void* ws, int64_t E, int64_t n, int64_t n_own, int world) {
  Carve c{static_cast<char*>(ws)};
  CoverWs w{};
  const int64_t P = n_own * world;
  w.e_row = c.take<int32_t>(E);
  w.e_cls = c.take<uint8_t>(E);
  w.cnt_pair = c.take<int32_t>(P);
  w.hp = c.take<uint8_t>(P);
  w.pk = c.take<uint8_t>(P);
  w.cnt_col = c.take<int32_t>(n);
  w.hx = c.take<uint8_t>(n);
  w.kpre = c.take<int64_t>(E + 1);
  w.xpre = c.take<int64_t>(E + 1);
  w.xrank = c.take<int64_t>(n + 1);
  w.pscan = c.take<int64_t>(P + 1);
  w.p_idx0 = c.take<int64_t>(E);
  w.p_idx1 = c.take<int64_t>(E);
  w.p_key0 = c.take<uint64_t>(E);
  w.p_key1 = c.take<uint64_t>(E);
  w.hp_cnt = c.take<int64_t>(n_own + 1);
  w.qb = c.take<int64_t>(2 * kMaxWorld);
  w.cnt = c.take<int64_t>(4);
  w.err = c.take<int32_t>(1);
  w.out = c.take<int64_t>(4 + 3 * static_cast<int64_t>(world));
  w.temp_bytes = cover_temp_bytes(E, n, P, n_own);
  w.temp = c.take<char>(static_cast<int64_t>(w.temp_bytes));
  w.bytes = c.used;
  return w;
}

// the counts gnn_cover_build hands back (see there), one lane per owner q
__global__ void cover_counts_kernel(const int64_t* __restrict__ kpre, const int64_t* __restrict__ xpre,
                                    const int64_t* __restrict__ xrank, const int64_t* __restrict__ pscan,
                                    const int64_t* __restrict__ qb, int64_t E, int64_t n_rows, int64_t P,
                                    int64_t n_own, Bounds B, int64_t* __restrict__ out) {
  const int q = threadIdx.x;
  const int W = B.world;
  if (q == 0) {
    out[0] = kpre[E];
    out[1] = xrank[n_rows];
    out[2] = xpre[E];
    out[3] = pscan[P];
  }
  if (q < W) {
    out[4 + q] = xrank[B.b[q + 1]] - xrank[B.b[q]];
    out[4 + W + q] = pscan[(q + 1) * n_own] - pscan[q * n_own];
    out[4 + 2 * W + q] = qb[kMaxWorld + q] - qb[q];
  }
}

// local edge t (global e0 + t): its row, its class (interior / cut), the cut counts
__global__ void cover_count_kernel(const int64_t* __restrict__ rp, const int32_t* __restrict__ col,
                                   int64_t r0, int64_t n_own, int64_t e0, int64_t E, Bounds B,
                                   int32_t* __restrict__ e_row, uint8_t* __restrict__ e_cls,
                                   int32_t* __restrict__ cnt_pair, int32_t* __restrict__ cnt_col,
                                   int32_t* __restrict__ err) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= E) return;
  const int64_t e = e0 + t;
  int64_t lo = 0, hi = n_own;  // last local row r with rp[r0 + r] <= e
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) >> 1;
    if (rp[r0 + mid] <= e) lo = mid; else hi = mid;
  }
  e_row[t] = static_cast<int32_t>(lo);
  const int64_t c = col[e];
  if (c < 0 || c >= B.b[B.world]) {  // counted as interior so no later pass indexes with it
    atomicOr(err, 1);
    e_cls[t] = kInterior;
    return;
  }
  if (c >= r0 && c < r0 + n_own) {
    e_cls[t] = kInterior;
    return;
  }
  e_cls[t] = kFeature;  // refined below
  const int q = B.owner(c);
  atomicAdd(cnt_pair + q * n_own + lo, 1);
  atomicAdd(cnt_col + c, 1);
}

// pass 1: the greedy rule marks pairs that take partials
__global__ void cover_rule_kernel(const int32_t* __restrict__ col, int64_t e0, int64_t E, int64_t n_own,
                                  Bounds B, const int32_t* __restrict__ e_row,
                                  const uint8_t* __restrict__ e_cls, const int32_t* __restrict__ cnt_pair,
                                  const int32_t* __restrict__ cnt_col, uint8_t* __restrict__ hp) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= E || e_cls[t] == kInterior) return;
  const int64_t c = col[e0 + t];
  const int64_t p = B.owner(c) * n_own + e_row[t];
  if (cnt_pair[p] > cnt_col[c]) hp[p] = 1;
}

// pass 2: an edge whose pair does not ship a partial marks its column as shipped
__global__ void cover_cols_kernel(const int32_t* __restrict__ col, int64_t e0, int64_t E, int64_t n_own,
                                  Bounds B, const int32_t* __restrict__ e_row,
                                  const uint8_t* __restrict__ e_cls, const uint8_t* __restrict__ hp,
                                  uint8_t* __restrict__ hx) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= E || e_cls[t] == kInterior) return;
  const int64_t c = col[e0 + t];
  if (!hp[B.owner(c) * n_own + e_row[t]]) hx[c] = 1;
}

// pass 3: final class of each cut edge (a shipped column serves every edge of it)
__global__ void cover_final_kernel(const int32_t* __restrict__ col, int64_t e0, int64_t E, int64_t n_own,
                                   Bounds B, const int32_t* __restrict__ e_row,
                                   uint8_t* __restrict__ e_cls, const uint8_t* __restrict__ hp,
                                   const uint8_t* __restrict__ hx, uint8_t* __restrict__ pk) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= E || e_cls[t] == kInterior) return;
  const int64_t c = col[e0 + t];
  const int64_t p = B.owner(c) * n_own + e_row[t];
  const bool part = hp[p] && !hx[c];
  e_cls[t] = part ? kPartial : kFeature;
  if (part) pk[p] = 1;
}

__global__ void cover_pkeys_kernel(const int64_t* __restrict__ idx, const int64_t* __restrict__ n_dev,
                                   const int32_t* __restrict__ col, int64_t e0, int64_t n_own,
                                   Bounds B, const int32_t* __restrict__ e_row,
                                   uint64_t* __restrict__ key) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= *n_dev) return;
  const int64_t t = idx[i];
  key[i] = static_cast<uint64_t>(B.owner(col[e0 + t])) * static_cast<uint64_t>(n_own) +
           static_cast<uint64_t>(e_row[t]);
}

// owner ranges of the sorted partial edges
__global__ void cover_qbounds_kernel(const uint64_t* __restrict__ key, int64_t np, int64_t n_own,
                                     int64_t* __restrict__ qb) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= np) return;
  const int64_t q = static_cast<int64_t>(key[i] / static_cast<uint64_t>(n_own));
  if (i == 0 || key[i - 1] / static_cast<uint64_t>(n_own) != static_cast<uint64_t>(q)) qb[q] = i;
  if (i == np - 1 || key[i + 1] / static_cast<uint64_t>(n_own) != static_cast<uint64_t>(q))
    qb[kMaxWorld + q] = i + 1;
}

// partial rows per row of this rank (the rows of halo_p)
__global__ void cover_hp_count_kernel(const uint8_t* __restrict__ pk, int64_t n_own, int world,
                                      int64_t* __restrict__ hp_cnt) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (r >= n_own) return;
  int64_t c = 0;
  for (int q = 0; q < world; ++q) c += pk[q * n_own + r];
  hp_cnt[r] = c;
}

// ---- fill
__global__ void cover_fill_edges_kernel(const int32_t* __restrict__ col, const float* __restrict__ val,
                                        int64_t e0, int64_t E, int64_t r0,
                                        const int32_t* __restrict__ e_row, const uint8_t* __restrict__ e_cls,
                                        const int64_t* __restrict__ kpre, const int64_t* __restrict__ xpre,
                                        const int64_t* __restrict__ xrank, int32_t* __restrict__ int_col,
                                        float* __restrict__ int_val, int32_t* __restrict__ hx_col,
                                        float* __restrict__ hx_val) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= E) return;
  const int64_t c = col[e0 + t];
  if (e_cls[t] == kInterior) {
    int_col[kpre[t]] = static_cast<int32_t>(c - r0);
    int_val[kpre[t]] = val[e0 + t];
  } else if (e_cls[t] == kFeature) {
    hx_col[xpre[t]] = static_cast<int32_t>(xrank[c]);
    hx_val[xpre[t]] = val[e0 + t];
  }
}

__global__ void cover_fill_rowptr_kernel(const int64_t* __restrict__ rp, int64_t r0, int64_t n_own,
                                         int64_t e0, const int64_t* __restrict__ kpre,
                                         const int64_t* __restrict__ xpre, int64_t* __restrict__ int_rp,
                                         int64_t* __restrict__ hx_rp) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (r > n_own) return;
  const int64_t t = rp[r0 + r] - e0;  // the edges are in row order: a row's first edge
  int_rp[r] = kpre[t];
  hx_rp[r] = xpre[t];
}

__global__ void cover_fill_pedges_kernel(const int64_t* __restrict__ idx, int64_t np,
                                         const int32_t* __restrict__ col, const float* __restrict__ val,
                                         int64_t e0, int64_t r0, const int32_t* __restrict__ e_row,
                                         int64_t* __restrict__ pe_i, int64_t* __restrict__ pe_j,
                                         float* __restrict__ pe_v) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= np) return;
  const int64_t t = idx[i];
  pe_i[i] = r0 + e_row[t];
  pe_j[i] = col[e0 + t];
  pe_v[i] = val[e0 + t];
}

__global__ void cover_fill_halo_p_kernel(const uint8_t* __restrict__ pk, const int64_t* __restrict__ pscan,
                                         int64_t n_own, int world, const int64_t* __restrict__ hp_rp,
                                         int32_t* __restrict__ hpc, float* __restrict__ hpv) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (r >= n_own) return;
  int64_t o = hp_rp[r];
  for (int q = 0; q < world; ++q) {  // ascending owner = ascending partial-row index
    const int64_t p = q * n_own + r;
    if (pk[p]) {
      hpc[o] = static_cast<int32_t>(pscan[p]);
      hpv[o] = 1.f;
      ++o;
    }
  }
}

// ---- partial rows this rank computes for its peers
struct Offsets {
  int64_t o[kMaxWorld + 1];
  int world;
  __host__ __device__ int peer(int64_t t) const {
    int lo = 0, hi = world;
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (o[mid] <= t) lo = mid; else hi = mid;
    }
    return lo;
  }
};
struct SlotHead {  // 1 where a new (peer, row) slot starts
  const int64_t* pe_i;
  Offsets O;
  __host__ __device__ int64_t operator()(int64_t t) const {
    return t == 0 || O.peer(t) != O.peer(t - 1) || pe_i[t] != pe_i[t - 1] ? 1 : 0;
  }
};
__global__ void send_p_fill_kernel(const int64_t* __restrict__ slot_incl, const int64_t* __restrict__ pe_i,
                                   const int64_t* __restrict__ pe_j, const float* __restrict__ pe_v,
                                   int64_t m, Offsets O, int64_t r0, int64_t n_own,
                                   int64_t* __restrict__ sp_rp, int32_t* __restrict__ sp_col,
                                   float* __restrict__ sp_val, int32_t* __restrict__ err) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= m) return;
  const bool head = t == 0 || O.peer(t) != O.peer(t - 1) || pe_i[t] != pe_i[t - 1];
  if (head) sp_rp[slot_incl[t] - 1] = t;
  if (t == m - 1) sp_rp[slot_incl[t]] = m;
  const int64_t c = pe_j[t] - r0;
  if (c < 0 || c >= n_own) {
    atomicOr(err, 1);
    sp_col[t] = 0;
  } else {
    sp_col[t] = static_cast<int32_t>(c);
  }
  sp_val[t] = pe_v[t];
}

#define CB_TRY(x)                                       \
  do {                                                  \
    hipError_t e_ = (x);                                \
    if (e_ != hipSuccess) return static_cast<int>(e_);  \
  } while (0)

static int sync_read(const int64_t* dev, int64_t* host, int64_t count, hipStream_t s) {
  hipError_t e = hipMemcpyAsync(host, dev, count * sizeof(int64_t), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  return e == hipSuccess ? GNN_OK : static_cast<int>(e);
}

static bool read_bounds(const int64_t* bounds, int32_t world, int64_t n_rows, Bounds* B) {
  if (!bounds || world < 1 || world > kMaxWorld) return false;
  B->world = world;
  for (int q = 0; q <= world; ++q) {
    B->b[q] = bounds[q];
    if (q > 0 && B->b[q] < B->b[q - 1]) return false;
  }
  return B->b[0] == 0 && B->b[world] == n_rows;
}

}  // namespace cb
}  // namespace gnn

using namespace gnn;
using namespace gnn::cb;

extern "C" int64_t gnn_cover_workspace_bytes(int64_t n_rows, int64_t nnz_local, int64_t n_own,
                                             int32_t world) {
  if (n_rows < 1 || nnz_local < 0 || n_own < 0 || world < 1 || world > kMaxWorld) return GNN_E_ARG;
  return cover_carve(nullptr, nnz_local, n_rows, n_own, world).bytes;
}

extern "C" int gnn_cover_build(const int64_t* rowptr, const int32_t* col, int64_t n_rows,
                               const int64_t* bounds, int32_t rank, int32_t world, int64_t* counts,
                               void* workspace, int64_t workspace_bytes, void* stream) {
  Bounds B;
  if (!rowptr || !counts || !workspace || n_rows < 1 || !read_bounds(bounds, world, n_rows, &B) ||
      rank < 0 || rank >= world)
    return GNN_E_ARG;
  if (n_rows > 0x7fffffffLL) return GNN_E_UNSUPPORTED;
  const int64_t r0 = B.b[rank], n_own = B.b[rank + 1] - r0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  int64_t e01[2];
  CB_TRY(hipMemcpyAsync(&e01[0], rowptr + r0, 8, hipMemcpyDeviceToHost, s));
  CB_TRY(hipMemcpyAsync(&e01[1], rowptr + r0 + n_own, 8, hipMemcpyDeviceToHost, s));
  CB_TRY(hipStreamSynchronize(s));
  const int64_t e0 = e01[0], E = e01[1] - e01[0];
  if (E > 0 && !col) return GNN_E_ARG;
  if (workspace_bytes < gnn_cover_workspace_bytes(n_rows, E, n_own, world)) return GNN_E_ARG;
  for (int i = 0; i < 4 + 3 * world; ++i) counts[i] = 0;
  CoverWs w = cover_carve(workspace, E, n_rows, n_own, world);
  const int64_t P = n_own * world;
  CB_TRY(hipMemsetAsync(w.cnt_pair, 0, static_cast<size_t>(P) * 4, s));
  CB_TRY(hipMemsetAsync(w.hp, 0, static_cast<size_t>(P), s));
  CB_TRY(hipMemsetAsync(w.pk, 0, static_cast<size_t>(P), s));
  CB_TRY(hipMemsetAsync(w.cnt_col, 0, static_cast<size_t>(n_rows) * 4, s));
  CB_TRY(hipMemsetAsync(w.hx, 0, static_cast<size_t>(n_rows), s));
  CB_TRY(hipMemsetAsync(w.qb, 0, 2 * kMaxWorld * 8, s));
  CB_TRY(hipMemsetAsync(w.cnt, 0, 4 * 8, s));
  CB_TRY(hipMemsetAsync(w.err, 0, 4, s));
  if (E > 0) {
    hipLaunchKernelGGL(cover_count_kernel, dim3(grid(E)), dim3(kT), 0, s, rowptr, col, r0, n_own, e0,
                       E, B, w.e_row, w.e_cls, w.cnt_pair, w.cnt_col, w.err);
    int32_t herr = 0;
    CB_TRY(hipMemcpyAsync(&herr, w.err, 4, hipMemcpyDeviceToHost, s));
    CB_TRY(hipStreamSynchronize(s));
    if (herr) return GNN_E_ARG;  // a column id outside [0, n_rows)
    hipLaunchKernelGGL(cover_rule_kernel, dim3(grid(E)), dim3(kT), 0, s, col, e0, E, n_own, B, w.e_row,
                       w.e_cls, w.cnt_pair, w.cnt_col, w.hp);
    hipLaunchKernelGGL(cover_cols_kernel, dim3(grid(E)), dim3(kT), 0, s, col, e0, E, n_own, B, w.e_row,
                       w.e_cls, w.hp, w.hx);
    hipLaunchKernelGGL(cover_final_kernel, dim3(grid(E)), dim3(kT), 0, s, col, e0, E, n_own, B,
                       w.e_row, w.e_cls, w.hp, w.hx, w.pk);
  }
  // edge prefixes of the interior and the feature-covered classes (their CSR offsets)
  size_t tb = w.temp_bytes;
  const auto k_it = rocprim::make_transform_iterator(Count(0), ClsIs{w.e_cls, kInterior, E});
  CB_TRY(rocprim::exclusive_scan(w.temp, tb, k_it, w.kpre, int64_t(0), static_cast<size_t>(E + 1),
                                 rocprim::plus<int64_t>(), s));
  tb = w.temp_bytes;
  const auto x_it = rocprim::make_transform_iterator(Count(0), ClsIs{w.e_cls, kFeature, E});
  CB_TRY(rocprim::exclusive_scan(w.temp, tb, x_it, w.xpre, int64_t(0), static_cast<size_t>(E + 1),
                                 rocprim::plus<int64_t>(), s));
  // requested columns (ascending global ids = grouped by owner) and their ranks
  tb = w.temp_bytes;
  const auto h_it = rocprim::make_transform_iterator(Count(0), ByteAt{w.hx, n_rows});
  CB_TRY(rocprim::exclusive_scan(w.temp, tb, h_it, w.xrank, int64_t(0), static_cast<size_t>(n_rows + 1),
                                 rocprim::plus<int64_t>(), s));
  // partial rows: one per (owner, row) pair with a partial edge, in (owner, row) order
  tb = w.temp_bytes;
  const auto p_it = rocprim::make_transform_iterator(Count(0), ByteAt{w.pk, P});
  CB_TRY(rocprim::exclusive_scan(w.temp, tb, p_it, w.pscan, int64_t(0), static_cast<size_t>(P + 1),
                                 rocprim::plus<int64_t>(), s));
  // partial edges: edge order, then a stable sort by (owner, row)
  int64_t np = 0;
  if (E > 0) {
    tb = w.temp_bytes;
    const auto f_it = rocprim::make_transform_iterator(Count(0), ClsFlag{w.e_cls, kPartial});
    CB_TRY(rocprim::select(w.temp, tb, Count(0), f_it, w.p_idx0, w.cnt, static_cast<size_t>(E), s));
    int rc = sync_read(w.cnt, &np, 1, s);
    if (rc != GNN_OK) return rc;
  }
  if (np > 0) {
    hipLaunchKernelGGL(cover_pkeys_kernel, dim3(grid(np)), dim3(kT), 0, s, w.p_idx0, w.cnt, col, e0,
                       n_own, B, w.e_row, w.p_key0);
    unsigned bits = 1;
    while (bits < 64 && (static_cast<uint64_t>(1) << bits) < static_cast<uint64_t>(P)) ++bits;
    tb = w.temp_bytes;
    CB_TRY(rocprim::radix_sort_pairs(w.temp, tb, w.p_key0, w.p_key1, w.p_idx0, w.p_idx1,
                                     static_cast<size_t>(np), 0, bits, s));
    hipLaunchKernelGGL(cover_qbounds_kernel, dim3(grid(np)), dim3(kT), 0, s, w.p_key1, np, n_own, w.qb);
  }
  if (n_own > 0)
    hipLaunchKernelGGL(cover_hp_count_kernel, dim3(grid(n_own)), dim3(kT), 0, s, w.pk, n_own, world,
                       w.hp_cnt);
  // counts: [0] interior nnz, [1] requested columns, [2] halo_x nnz, [3] partial rows,
  // [4 + q] feature rows asked of q, [4 + W + q] partial rows asked of q, [4 + 2W + q] their edges
  // -- gathered on the device and read back once (4 W + 6 separate reads before)
  hipLaunchKernelGGL(cover_counts_kernel, dim3(1), dim3(kMaxWorld), 0, s, w.kpre, w.xpre, w.xrank,
                     w.pscan, w.qb, E, n_rows, P, n_own, B, w.out);
  int rc = sync_read(w.out, counts, 4 + 3 * static_cast<int64_t>(world), s);
  if (rc != GNN_OK) return rc;
  return launch_status();
}

extern "C" int gnn_cover_fill(const void* workspace, const int64_t* rowptr, const int32_t* col,
                              const float* val, int64_t n_rows, const int64_t* bounds, int32_t rank,
                              int32_t world, const int64_t* counts, int64_t* int_rowptr,
                              int32_t* int_col, float* int_val, int64_t* xcols, int64_t* hx_rowptr,
                              int32_t* hx_col, float* hx_val, int64_t* pe_i, int64_t* pe_j,
                              float* pe_v, int64_t* hp_rowptr, int32_t* hp_col, float* hp_val,
                              void* stream) {
  Bounds B;
  if (!workspace || !rowptr || !counts || n_rows < 1 || !read_bounds(bounds, world, n_rows, &B) ||
      rank < 0 || rank >= world || !int_rowptr || !hx_rowptr || !hp_rowptr)
    return GNN_E_ARG;
  const int64_t r0 = B.b[rank], n_own = B.b[rank + 1] - r0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  int64_t e01[2];
  CB_TRY(hipMemcpyAsync(&e01[0], rowptr + r0, 8, hipMemcpyDeviceToHost, s));
  CB_TRY(hipMemcpyAsync(&e01[1], rowptr + r0 + n_own, 8, hipMemcpyDeviceToHost, s));
  CB_TRY(hipStreamSynchronize(s));
  const int64_t e0 = e01[0], E = e01[1] - e01[0];
  CoverWs w = cover_carve(const_cast<void*>(workspace), E, n_rows, n_own, world);
  int64_t np = 0;
  for (int q = 0; q < world; ++q) np += counts[4 + 2 * world + q];
  if ((counts[0] && (!int_col || !int_val)) || (counts[1] && !xcols) ||
      (counts[2] && (!hx_col || !hx_val)) || (np && (!pe_i || !pe_j || !pe_v)) ||
      (counts[3] && (!hp_col || !hp_val)))
    return GNN_E_ARG;
  hipLaunchKernelGGL(cover_fill_rowptr_kernel, dim3(grid(n_own + 1)), dim3(kT), 0, s, rowptr, r0, n_own,
                     e0, w.kpre, w.xpre, int_rowptr, hx_rowptr);
  if (E > 0)
    hipLaunchKernelGGL(cover_fill_edges_kernel, dim3(grid(E)), dim3(kT), 0, s, col, val, e0, E, r0,
                       w.e_row, w.e_cls, w.kpre, w.xpre, w.xrank, int_col, int_val, hx_col, hx_val);
  if (counts[1] > 0) {
    size_t tb = w.temp_bytes;
    const auto h_it = rocprim::make_transform_iterator(Count(0), ByteAt{w.hx, n_rows});
    CB_TRY(rocprim::select(w.temp, tb, Count(0), h_it, xcols, w.cnt + 1, static_cast<size_t>(n_rows), s));
  }
  if (np > 0)
    hipLaunchKernelGGL(cover_fill_pedges_kernel, dim3(grid(np)), dim3(kT), 0, s, w.p_idx1, np, col, val,
                       e0, r0, w.e_row, pe_i, pe_j, pe_v);
  size_t tb = w.temp_bytes;
  const auto a_it = rocprim::make_transform_iterator(Count(0), Arr{w.hp_cnt, n_own});
  CB_TRY(rocprim::exclusive_scan(w.temp, tb, a_it, hp_rowptr, int64_t(0), static_cast<size_t>(n_own + 1),
                                 rocprim::plus<int64_t>(), s));
  if (n_own > 0 && counts[3] > 0)
    hipLaunchKernelGGL(cover_fill_halo_p_kernel, dim3(grid(n_own)), dim3(kT), 0, s, w.pk, w.pscan, n_own,
                       world, hp_rowptr, hp_col, hp_val);
  return launch_status();
}

extern "C" int64_t gnn_cover_send_workspace_bytes(int64_t n_edges) {
  if (n_edges < 0) return GNN_E_ARG;
  size_t t = 0;
  const auto h_it = rocprim::make_transform_iterator(Count(0), SlotHead{nullptr, Offsets{}});
  (void)rocprim::inclusive_scan(nullptr, t, h_it, static_cast<int64_t*>(nullptr),
                                static_cast<size_t>(n_edges > 0 ? n_edges : 1), rocprim::plus<int64_t>());
  return up((n_edges > 0 ? n_edges : 1) * 8) + 256 + up(static_cast<int64_t>(t) + 256);
}

extern "C" int gnn_cover_send_partials(const int64_t* pe_i, const int64_t* pe_j, const float* pe_v,
                                       const int64_t* recv_edges, int32_t world, int64_t r0,
                                       int64_t n_own, int64_t n_p_send, int64_t* sp_rowptr,
                                       int32_t* sp_col, float* sp_val, void* workspace,
                                       int64_t workspace_bytes, void* stream) {
  if (!recv_edges || world < 1 || world > kMaxWorld || r0 < 0 || n_own < 0 || n_p_send < 0 ||
      !sp_rowptr || !workspace)
    return GNN_E_ARG;
  Offsets O;
  O.world = world;
  O.o[0] = 0;
  for (int q = 0; q < world; ++q) {
    if (recv_edges[q] < 0) return GNN_E_ARG;
    O.o[q + 1] = O.o[q] + recv_edges[q];
  }
  const int64_t m = O.o[world];
  if (workspace_bytes < gnn_cover_send_workspace_bytes(m)) return GNN_E_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (m == 0) {
    if (n_p_send != 0) return GNN_E_ARG;
    CB_TRY(hipMemsetAsync(sp_rowptr, 0, 8, s));
    return launch_status();
  }
  if (!pe_i || !pe_j || !pe_v || !sp_col || !sp_val) return GNN_E_ARG;
  char* p = static_cast<char*>(workspace);
  int64_t* slot = reinterpret_cast<int64_t*>(p);
  int32_t* err = reinterpret_cast<int32_t*>(p + up(m * 8));
  void* temp = p + up(m * 8) + 256;
  size_t tb = static_cast<size_t>(workspace_bytes - up(m * 8) - 256);
  CB_TRY(hipMemsetAsync(err, 0, 4, s));
  const auto h_it = rocprim::make_transform_iterator(Count(0), SlotHead{pe_i, O});
  CB_TRY(rocprim::inclusive_scan(temp, tb, h_it, slot, static_cast<size_t>(m), rocprim::plus<int64_t>(), s));
  int64_t n_slots = 0;
  int rc = sync_read(slot + m - 1, &n_slots, 1, s);
  if (rc != GNN_OK) return rc;
  if (n_slots != n_p_send) return GNN_E_ARG;  // the handshake's partial-row count disagrees
  hipLaunchKernelGGL(send_p_fill_kernel, dim3(grid(m)), dim3(kT), 0, s, slot, pe_i, pe_j, pe_v, m, O, r0,
                     n_own, sp_rowptr, sp_col, sp_val, err);
  int32_t herr = 0;
  CB_TRY(hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, s));
  CB_TRY(hipStreamSynchronize(s));
  if (herr) return GNN_E_ARG;  // a column outside this rank's rows
  return launch_status();
}
