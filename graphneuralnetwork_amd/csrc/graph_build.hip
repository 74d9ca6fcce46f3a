// graph_build.hip -- the reference GCN adjacency, built on the device.
//
// Restates GCN/data_utils.py as sort / reduce passes over int64 edge keys
// key = row * n + col (rocPRIM device radix sort + reduce-by-key):
//
//   A     = coo(ones(E), (src, dst)), duplicates summed            (:32-33)
//   A_sym = A + A^T.(A^T > A) - A.(A^T > A) = elementwise max(A, A^T)  (:35)
//   A_til = A_sym + I   (float64, sp.eye)                          (:78)
//   d     = rowsum(A_til)^-1/2, inf -> 0                          (:55-57)
//   A_hat[i, j] = (A_til[j, i] * d[i]) * d[j]  -> fp32 CSR       (:60, :63-70)
//
// All values are small integers until the normalisation, so every sum is exact
// in float64 and the result is bit-identical to scipy's (checked against the
// reference-generated fixtures, tests/test_graph_build_gpu.py). Reductions use
// rocPRIM's deterministic reduce-by-key. The builder synchronises its stream
// between stages to size the next one: it runs once per graph, never per forward.
#include <cstring>  // rocprim's texture_cache_iterator calls host memset

#include <rocprim/rocprim.hpp>

#include "common.hpp"

namespace gnn {

struct BuildWs {
  uint64_t* k0;
  uint64_t* k1;
  double* v0;
  double* v1;
  int64_t* count;  // [4] device counters
  int32_t* err;
  void* temp;
  size_t temp_bytes;
  int64_t cap;
};

struct RowOfKey {
  uint64_t n;
  __host__ __device__ uint64_t operator()(uint64_t k) const { return k / n; }
};

static int64_t align_up(int64_t v, int64_t a) { return (v + a - 1) / a * a; }

static int64_t build_capacity(int64_t n_edges, int64_t n_nodes) { return 2 * n_edges + n_nodes; }

static unsigned key_bits(int64_t n) {
  const unsigned __int128 m = static_cast<unsigned __int128>(n) * static_cast<unsigned __int128>(n);
  unsigned b = 1;
  while (b < 64 && (static_cast<unsigned __int128>(1) << b) < m) ++b;
  return b;
}

// rocPRIM temporary storage needed by the largest pass (queried with null storage)
static size_t temp_bytes_for(int64_t cap, int64_t n) {
  size_t a = 0, b = 0, c = 0, d = 0;
  const unsigned bits = key_bits(n > 1 ? n : 2);
  (void)rocprim::radix_sort_keys(nullptr, a, static_cast<uint64_t*>(nullptr), static_cast<uint64_t*>(nullptr),
                           static_cast<size_t>(cap), 0, bits);
  (void)rocprim::radix_sort_pairs(nullptr, b, static_cast<uint64_t*>(nullptr),
                            static_cast<uint64_t*>(nullptr), static_cast<double*>(nullptr),
                            static_cast<double*>(nullptr), static_cast<size_t>(cap), 0, bits);
  (void)rocprim::deterministic_reduce_by_key(nullptr, c, static_cast<uint64_t*>(nullptr),
                                       static_cast<double*>(nullptr), static_cast<size_t>(cap),
                                       static_cast<uint64_t*>(nullptr), static_cast<double*>(nullptr),
                                       static_cast<int64_t*>(nullptr), rocprim::plus<double>());
  (void)rocprim::reduce_by_key(nullptr, d, static_cast<uint64_t*>(nullptr), static_cast<double*>(nullptr),
                         static_cast<size_t>(cap), static_cast<uint64_t*>(nullptr),
                         static_cast<double*>(nullptr), static_cast<int64_t*>(nullptr),
                         rocprim::maximum<double>());
  size_t e = 0;
  auto rows = rocprim::make_transform_iterator(static_cast<uint64_t*>(nullptr),
                                               RowOfKey{static_cast<uint64_t>(n > 1 ? n : 2)});
  (void)rocprim::deterministic_reduce_by_key(nullptr, e, rows, static_cast<double*>(nullptr),
                                             static_cast<size_t>(cap),
                                             static_cast<uint64_t*>(nullptr),
                                             static_cast<double*>(nullptr),
                                             static_cast<int64_t*>(nullptr), rocprim::plus<double>(),
                                             rocprim::equal_to<uint64_t>());
  size_t m = a;
  if (b > m) m = b;
  if (c > m) m = c;
  if (d > m) m = d;
  if (e > m) m = e;
  return m + (1u << 20);
}

static BuildWs carve(void* ws, int64_t n_edges, int64_t n_nodes) {
  BuildWs w{};
  w.cap = build_capacity(n_edges, n_nodes);
  char* p = static_cast<char*>(ws);
  const int64_t kb = align_up(w.cap * 8, 256);
  w.k0 = reinterpret_cast<uint64_t*>(p);
  p += kb;
  w.k1 = reinterpret_cast<uint64_t*>(p);
  p += kb;
  w.v0 = reinterpret_cast<double*>(p);
  p += kb;
  w.v1 = reinterpret_cast<double*>(p);
  p += kb;
  w.count = reinterpret_cast<int64_t*>(p);
  p += 256;
  w.err = reinterpret_cast<int32_t*>(p);
  p += 256;
  w.temp = p;
  w.temp_bytes = temp_bytes_for(w.cap, n_nodes);
  return w;
}

__global__ void make_keys_kernel(const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                 int64_t n_edges, int64_t n, uint64_t* __restrict__ keys,
                                 double* __restrict__ ones, int32_t* __restrict__ err) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n_edges) return;
  const int64_t s = src[i], d = dst[i];
  if (s < 0 || s >= n || d < 0 || d >= n) {
    atomicOr(err, 1);
    keys[i] = 0;
  } else {
    keys[i] = static_cast<uint64_t>(s) * static_cast<uint64_t>(n) + static_cast<uint64_t>(d);
  }
  ones[i] = 1.0;
}

// append the transpose of the U unique keys (same values) after them
__global__ void append_transpose_kernel(uint64_t* __restrict__ keys, double* __restrict__ vals,
                                        const int64_t* __restrict__ count, int64_t n) {
  const int64_t u = count[0];
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= u) return;
  const uint64_t k = keys[i];
  const uint64_t r = k / static_cast<uint64_t>(n), c = k % static_cast<uint64_t>(n);
  keys[u + i] = c * static_cast<uint64_t>(n) + r;
  vals[u + i] = vals[i];
}

// append the n diagonal keys (value 1.0) after the U keys
__global__ void append_diag_kernel(uint64_t* __restrict__ keys, double* __restrict__ vals,
                                   const int64_t* __restrict__ count, int64_t n) {
  const int64_t u = count[0];
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  keys[u + i] = static_cast<uint64_t>(i) * static_cast<uint64_t>(n + 1);
  vals[u + i] = 1.0;
}

// d[i] = rowsum[i]^-1/2 (inf -> 0), in place
__global__ void inv_sqrt_kernel(double* __restrict__ d, int64_t n) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double r = d[i];
  const double v = pow(r, -0.5);  // numpy's np.power(rowsum, -0.5)
  d[i] = isinf(v) ? 0.0 : v;
}

// transpose + normalise: output row = col c, gathered col = row r,
// value (A_til[r, c] * d[c]) * d[r]   (scipy's ((A D)^T D) rounding order)
__global__ void normalise_transpose_kernel(const uint64_t* __restrict__ keys_in,
                                           double* __restrict__ vals, const double* __restrict__ d,
                                           uint64_t* __restrict__ keys_out,
                                           const int64_t* __restrict__ count, int64_t n) {
  const int64_t u = count[0];
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= u) return;
  const uint64_t k = keys_in[i];
  const uint64_t r = k / static_cast<uint64_t>(n), c = k % static_cast<uint64_t>(n);
  vals[i] = (vals[i] * d[c]) * d[r];
  keys_out[i] = c * static_cast<uint64_t>(n) + r;
}

__global__ void emit_csr_kernel(const uint64_t* __restrict__ keys, const double* __restrict__ vals,
                                int64_t nnz, int64_t n, int64_t* __restrict__ rowptr,
                                int32_t* __restrict__ col, float* __restrict__ val) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= nnz) return;
  const uint64_t k = keys[i];
  const int64_t r = static_cast<int64_t>(k / static_cast<uint64_t>(n));
  col[i] = static_cast<int32_t>(k % static_cast<uint64_t>(n));
  val[i] = static_cast<float>(vals[i]);
  // every row holds its diagonal entry, so each row has a first element
  if (i == 0 || static_cast<int64_t>(keys[i - 1] / static_cast<uint64_t>(n)) != r) rowptr[r] = i;
  if (i == nnz - 1) rowptr[n] = nnz;
}

static inline unsigned grid_for(int64_t n) { return static_cast<unsigned>((n + 255) / 256); }

static int read_count(const int64_t* dev, int64_t* host, hipStream_t s) {
  hipError_t e = hipMemcpyAsync(host, dev, sizeof(int64_t), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  return e == hipSuccess ? GNN_OK : static_cast<int>(e);
}

}  // namespace gnn

using namespace gnn;

extern "C" int64_t gnn_gcn_adjacency_workspace_bytes(int64_t n_edges, int64_t n_nodes) {
  if (n_edges < 0 || n_nodes < 1) return GNN_E_ARG;
  const int64_t cap = build_capacity(n_edges, n_nodes);
  return 4 * align_up(cap * 8, 256) + 512 +
         static_cast<int64_t>(temp_bytes_for(cap, n_nodes)) + 256;
}

extern "C" int gnn_gcn_adjacency_build(const int64_t* src, const int64_t* dst, int64_t n_edges,
                                       int64_t n_nodes, void* workspace, int64_t workspace_bytes,
                                       int64_t* nnz_out, void* stream) {
  if (n_edges < 0 || n_nodes < 1 || !workspace || !nnz_out || (n_edges > 0 && (!src || !dst)))
    return GNN_E_ARG;
  if (n_nodes > 0x7fffffffLL || static_cast<__int128>(n_nodes) * n_nodes > (static_cast<__int128>(1) << 63))
    return GNN_E_UNSUPPORTED;
  if (workspace_bytes < gnn_gcn_adjacency_workspace_bytes(n_edges, n_nodes)) return GNN_E_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  BuildWs w = carve(workspace, n_edges, n_nodes);
  const int64_t n = n_nodes;
  const unsigned bits = key_bits(n > 1 ? n : 2);
  hipError_t e = hipMemsetAsync(w.err, 0, sizeof(int32_t), s);
  if (e != hipSuccess) return static_cast<int>(e);
  int64_t u = 0;
  int rc;
  size_t tb = w.temp_bytes;
  if (n_edges > 0) {
    // A: duplicate edges summed
    hipLaunchKernelGGL(make_keys_kernel, dim3(grid_for(n_edges)), dim3(256), 0, s, src, dst,
                       n_edges, n, w.k0, w.v1, w.err);
    e = rocprim::radix_sort_keys(w.temp, tb, w.k0, w.k1, static_cast<size_t>(n_edges), 0, bits, s);
    if (e != hipSuccess) return static_cast<int>(e);
    tb = w.temp_bytes;
    e = rocprim::deterministic_reduce_by_key(w.temp, tb, w.k1, w.v1, static_cast<size_t>(n_edges),
                                             w.k0, w.v0, w.count, rocprim::plus<double>(),
                                             rocprim::equal_to<uint64_t>(), s);
    if (e != hipSuccess) return static_cast<int>(e);
    if ((rc = read_count(w.count, &u, s)) != GNN_OK) return rc;
    int32_t herr = 0;
    e = hipMemcpy(&herr, w.err, sizeof(int32_t), hipMemcpyDeviceToHost);
    if (e != hipSuccess) return static_cast<int>(e);
    if (herr) return GNN_E_ARG;  // an endpoint outside [0, n)
    // A_sym = max(A, A^T)
    hipLaunchKernelGGL(append_transpose_kernel, dim3(grid_for(u)), dim3(256), 0, s, w.k0, w.v0,
                       w.count, n);
    tb = w.temp_bytes;
    e = rocprim::radix_sort_pairs(w.temp, tb, w.k0, w.k1, w.v0, w.v1, static_cast<size_t>(2 * u), 0,
                                  bits, s);
    if (e != hipSuccess) return static_cast<int>(e);
    tb = w.temp_bytes;
    e = rocprim::reduce_by_key(w.temp, tb, w.k1, w.v1, static_cast<size_t>(2 * u), w.k0, w.v0,
                               w.count, rocprim::maximum<double>(), rocprim::equal_to<uint64_t>(), s);
    if (e != hipSuccess) return static_cast<int>(e);
    if ((rc = read_count(w.count, &u, s)) != GNN_OK) return rc;
  } else {
    e = hipMemsetAsync(w.count, 0, sizeof(int64_t), s);
    if (e != hipSuccess) return static_cast<int>(e);
  }
  // + I (float64): diagonal keys appended, then one sorted sum
  hipLaunchKernelGGL(append_diag_kernel, dim3(grid_for(n)), dim3(256), 0, s, w.k0, w.v0, w.count, n);
  tb = w.temp_bytes;
  e = rocprim::radix_sort_pairs(w.temp, tb, w.k0, w.k1, w.v0, w.v1, static_cast<size_t>(u + n), 0,
                                bits, s);
  if (e != hipSuccess) return static_cast<int>(e);
  tb = w.temp_bytes;
  e = rocprim::deterministic_reduce_by_key(w.temp, tb, w.k1, w.v1, static_cast<size_t>(u + n), w.k0,
                                           w.v0, w.count, rocprim::plus<double>(),
                                           rocprim::equal_to<uint64_t>(), s);
  if (e != hipSuccess) return static_cast<int>(e);
  int64_t nnz = 0;
  if ((rc = read_count(w.count, &nnz, s)) != GNN_OK) return rc;
  // rowsum per row (every row present: it holds its diagonal) -> d = rowsum^-1/2 in v1[0..n)
  auto rows = rocprim::make_transform_iterator(w.k0, RowOfKey{static_cast<uint64_t>(n)});
  tb = w.temp_bytes;
  e = rocprim::deterministic_reduce_by_key(w.temp, tb, rows, w.v0, static_cast<size_t>(nnz), w.k1,
                                           w.v1, w.count + 1, rocprim::plus<double>(),
                                           rocprim::equal_to<uint64_t>(), s);
  if (e != hipSuccess) return static_cast<int>(e);
  hipLaunchKernelGGL(inv_sqrt_kernel, dim3(grid_for(n)), dim3(256), 0, s, w.v1, n);
  // transpose + normalise, then sort by the new (row, col)
  hipLaunchKernelGGL(normalise_transpose_kernel, dim3(grid_for(nnz)), dim3(256), 0, s, w.k0, w.v0,
                     w.v1, w.k1, w.count, n);
  tb = w.temp_bytes;
  e = rocprim::radix_sort_pairs(w.temp, tb, w.k1, w.k0, w.v0, w.v1, static_cast<size_t>(nnz), 0,
                                bits, s);
  if (e != hipSuccess) return static_cast<int>(e);
  *nnz_out = nnz;
  return launch_status();
}

extern "C" int gnn_gcn_adjacency_fill(const void* workspace, int64_t n_edges, int64_t n_nodes,
                                      int64_t nnz, int64_t* rowptr, int32_t* col, float* val,
                                      void* stream) {
  if (!workspace || n_nodes < 1 || nnz < n_nodes || !rowptr || !col || !val) return GNN_E_ARG;
  BuildWs w = carve(const_cast<void*>(workspace), n_edges, n_nodes);
  hipLaunchKernelGGL(emit_csr_kernel, dim3(grid_for(nnz)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), w.k0, w.v1, nnz, n_nodes, rowptr, col, val);
  return launch_status();
}
