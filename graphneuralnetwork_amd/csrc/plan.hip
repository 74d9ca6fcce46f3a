// plan.hip -- row-split plan for power-law CSR graphs (built once per graph).
//
// A "long row" has degree > seg_len. The plan lists, in ascending row order,
// every long row and the seg_len-edge segments it is cut into, so that the
// aggregation kernels can give each segment its own wavefront (spmm.hip,
// gat.hip). Three launches, all deterministic (ordered block scans, no atomics):
//   count: per-block (n_long, n_seg) over 4096-row tiles
//   scan : one workgroup turns the per-block counts into exclusive offsets
//          and the two totals (written to the caller's counts_dev[2])
//   fill : every block re-derives its rows' counts, scans them inside the
//          block and writes seg_row / seg_begin / long_row / long_seg_ptr.
#include "common.hpp"

namespace gnn {

constexpr int kPlanThreads = 256;
constexpr int kPlanRowsPerThread = 16;
constexpr int64_t kPlanRowsPerBlock = kPlanThreads * kPlanRowsPerThread;

static inline int64_t plan_blocks(int64_t n_rows) {
  return (n_rows + kPlanRowsPerBlock - 1) / kPlanRowsPerBlock;
}

__device__ __forceinline__ void thread_counts(const int64_t* __restrict__ rowptr, int64_t n_rows,
                                              int64_t seg_len, int64_t r0, int64_t& nl,
                                              int64_t& ns) {
  nl = 0;
  ns = 0;
  for (int i = 0; i < kPlanRowsPerThread; ++i) {
    const int64_t r = r0 + i;
    if (r >= n_rows) break;
    const int64_t d = rowptr[r + 1] - rowptr[r];
    if (d > seg_len) {
      nl += 1;
      ns += (d + seg_len - 1) / seg_len;
    }
  }
}

// Exclusive scan of one int64 per thread over a 256-thread block. Returns the
// exclusive prefix; *total receives the block sum. `lds` holds >= 4 int64.
__device__ int64_t block_exclusive_scan(int64_t v, int64_t* lds, int64_t* total) {
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  int64_t inc = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int64_t t = __shfl_up(inc, off, 64);
    if (lane >= off) inc += t;
  }
  if (lane == 63) lds[wid] = inc;
  __syncthreads();
  int64_t wave_off = 0, tot = 0;
  for (int w = 0; w < kPlanThreads / 64; ++w) {
    if (w < wid) wave_off += lds[w];
    tot += lds[w];
  }
  __syncthreads();
  *total = tot;
  return wave_off + inc - v;
}

__global__ __launch_bounds__(kPlanThreads) void plan_count_kernel(const int64_t* __restrict__ rowptr,
                                                                  int64_t n_rows, int64_t seg_len,
                                                                  int64_t* __restrict__ blk_cnt) {
  __shared__ int64_t lds[8];
  const int64_t r0 = blockIdx.x * kPlanRowsPerBlock + threadIdx.x * kPlanRowsPerThread;
  int64_t nl, ns, tl, ts;
  thread_counts(rowptr, n_rows, seg_len, r0, nl, ns);
  block_exclusive_scan(nl, lds, &tl);
  block_exclusive_scan(ns, lds + 4, &ts);
  if (threadIdx.x == 0) {
    blk_cnt[2 * blockIdx.x] = tl;
    blk_cnt[2 * blockIdx.x + 1] = ts;
  }
}

// Single workgroup: blk_off[2b..] = exclusive prefix of blk_cnt, counts[0..1] = totals.
__global__ __launch_bounds__(kPlanThreads) void plan_scan_kernel(const int64_t* __restrict__ blk_cnt,
                                                                 int64_t nblk,
                                                                 int64_t* __restrict__ blk_off,
                                                                 int64_t* __restrict__ totals,
                                                                 int64_t* __restrict__ counts_out) {
  __shared__ int64_t lds[8];
  const int64_t per = (nblk + kPlanThreads - 1) / kPlanThreads;
  const int64_t b0 = threadIdx.x * per;
  int64_t sl = 0, ss = 0;
  for (int64_t b = b0; b < b0 + per && b < nblk; ++b) {
    sl += blk_cnt[2 * b];
    ss += blk_cnt[2 * b + 1];
  }
  int64_t tl, ts;
  int64_t ol = block_exclusive_scan(sl, lds, &tl);
  int64_t os = block_exclusive_scan(ss, lds + 4, &ts);
  for (int64_t b = b0; b < b0 + per && b < nblk; ++b) {
    blk_off[2 * b] = ol;
    blk_off[2 * b + 1] = os;
    ol += blk_cnt[2 * b];
    os += blk_cnt[2 * b + 1];
  }
  if (threadIdx.x == 0) {
    totals[0] = tl;
    totals[1] = ts;
    counts_out[0] = tl;
    counts_out[1] = ts;
  }
}

__global__ __launch_bounds__(kPlanThreads) void plan_fill_kernel(
    const int64_t* __restrict__ rowptr, int64_t n_rows, int64_t seg_len,
    const int64_t* __restrict__ blk_off, const int64_t* __restrict__ totals,
    int32_t* __restrict__ seg_row, int64_t* __restrict__ seg_begin, int32_t* __restrict__ long_row,
    int32_t* __restrict__ long_seg_ptr) {
  __shared__ int64_t lds[8];
  const int64_t r0 = blockIdx.x * kPlanRowsPerBlock + threadIdx.x * kPlanRowsPerThread;
  int64_t nl, ns, tl, ts;
  thread_counts(rowptr, n_rows, seg_len, r0, nl, ns);
  int64_t ol = block_exclusive_scan(nl, lds, &tl) + blk_off[2 * blockIdx.x];
  int64_t os = block_exclusive_scan(ns, lds + 4, &ts) + blk_off[2 * blockIdx.x + 1];
  for (int i = 0; i < kPlanRowsPerThread; ++i) {
    const int64_t r = r0 + i;
    if (r >= n_rows) break;
    const int64_t b = rowptr[r];
    const int64_t d = rowptr[r + 1] - b;
    if (d <= seg_len) continue;
    long_row[ol] = static_cast<int32_t>(r);
    long_seg_ptr[ol] = static_cast<int32_t>(os);
    ++ol;
    for (int64_t e = 0; e < d; e += seg_len) {
      seg_row[os] = static_cast<int32_t>(r);
      seg_begin[os] = b + e;
      ++os;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) long_seg_ptr[totals[0]] = static_cast<int32_t>(totals[1]);
}

}  // namespace gnn

using namespace gnn;

extern "C" int64_t gnn_spmm_plan_scratch_bytes(int64_t n_rows) {
  if (n_rows < 0) return GNN_E_ARG;
  return (4 * plan_blocks(n_rows) + 2) * static_cast<int64_t>(sizeof(int64_t));
}

extern "C" int gnn_spmm_plan_count(const int64_t* rowptr, int64_t n_rows, int64_t seg_len,
                                   int64_t* counts_dev, void* scratch, void* stream) {
  if (rowptr == nullptr || counts_dev == nullptr || scratch == nullptr || n_rows < 0 ||
      seg_len < 1)
    return GNN_E_ARG;
  if (n_rows > 0x7fffffffLL) return GNN_E_UNSUPPORTED;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t nblk = plan_blocks(n_rows);
  int64_t* blk_cnt = static_cast<int64_t*>(scratch);
  int64_t* blk_off = blk_cnt + 2 * nblk;
  int64_t* totals = blk_off + 2 * nblk;
  if (nblk == 0) {
    hipError_t e = hipMemsetAsync(counts_dev, 0, 2 * sizeof(int64_t), s);
    if (e == hipSuccess) e = hipMemsetAsync(totals, 0, 2 * sizeof(int64_t), s);
    return e == hipSuccess ? GNN_OK : static_cast<int>(e);
  }
  hipLaunchKernelGGL(plan_count_kernel, dim3(static_cast<unsigned>(nblk)), dim3(kPlanThreads), 0,
                     s, rowptr, n_rows, seg_len, blk_cnt);
  hipLaunchKernelGGL(plan_scan_kernel, dim3(1), dim3(kPlanThreads), 0, s, blk_cnt, nblk, blk_off,
                     totals, counts_dev);
  return launch_status();
}

extern "C" int gnn_spmm_plan_fill(const int64_t* rowptr, int64_t n_rows, int64_t seg_len,
                                  int32_t* seg_row, int64_t* seg_begin, int32_t* long_row,
                                  int32_t* long_seg_ptr, void* scratch, void* stream) {
  if (rowptr == nullptr || scratch == nullptr || long_seg_ptr == nullptr || n_rows < 0 ||
      seg_len < 1)
    return GNN_E_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t nblk = plan_blocks(n_rows);
  int64_t* blk_off = static_cast<int64_t*>(scratch) + 2 * nblk;
  int64_t* totals = blk_off + 2 * nblk;
  if (nblk == 0) {
    hipError_t e = hipMemsetAsync(long_seg_ptr, 0, sizeof(int32_t), s);
    return e == hipSuccess ? GNN_OK : static_cast<int>(e);
  }
  hipLaunchKernelGGL(plan_fill_kernel, dim3(static_cast<unsigned>(nblk)), dim3(kPlanThreads), 0, s,
                     rowptr, n_rows, seg_len, blk_off, totals, seg_row, seg_begin, long_row,
                     long_seg_ptr);
  return launch_status();
}

extern "C" int gnn_version(void) { return 100; }

extern "C" const char* gnn_error_string(int code) {
  switch (code) {
    case GNN_OK: return "success";
    case GNN_E_ARG: return "gnn: invalid argument (null pointer, negative size or bad stride)";
    case GNN_E_ALIGN: return "gnn: misaligned pointer";
    case GNN_E_UNSUPPORTED: return "gnn: shape not supported by this library";
    default: break;
  }
  if (code > 0) return hipGetErrorString(static_cast<hipError_t>(code));
  return "gnn: unknown error";
}
