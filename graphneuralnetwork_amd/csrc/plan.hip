// plan.hip -- row-class plan for power-law CSR graphs (built once per graph).
//
// Every row falls in exactly one class, by degree d and the segment length L:
//   small  d <= 1  : its single edge (col, val) is resolved here, so the
//                    aggregation kernels pack many such rows per wavefront
//                    (44% of the rows of the 1M-node R-MAT graph are self-loop only);
//   mid    1 < d <= L : one wavefront per row, from a compact row list;
//   long   d > L   : cut into ceil(d / L) segments, one wavefront each, merged
//                    by a fix-up (the 187k-degree hub of the 10M-node graph).
// The lists are in ascending row order. Three launches, deterministic (ordered
// block scans, no atomics):
//   count: per-block class counts over 4096-row tiles
//   scan : one workgroup turns them into exclusive offsets + totals
//          (written to the caller's counts_dev[4] = n_long, n_seg, n_small, n_mid)
//   fill : every block re-derives its rows' classes, scans inside the block
//          and writes the lists.
#include "common.hpp"

namespace gnn {

constexpr int kPlanThreads = 256;
constexpr int kPlanRowsPerThread = 16;
constexpr int64_t kPlanRowsPerBlock = kPlanThreads * kPlanRowsPerThread;
constexpr int kClasses = 4;  // long rows, segments, small rows, mid rows

static inline int64_t plan_blocks(int64_t n_rows) {
  return (n_rows + kPlanRowsPerBlock - 1) / kPlanRowsPerBlock;
}

__device__ __forceinline__ void thread_counts(const int64_t* __restrict__ rowptr, int64_t n_rows,
                                              int64_t seg_len, int64_t r0,
                                              int64_t (&cnt)[kClasses]) {
#pragma unroll
  for (int k = 0; k < kClasses; ++k) cnt[k] = 0;
  for (int i = 0; i < kPlanRowsPerThread; ++i) {
    const int64_t r = r0 + i;
    if (r >= n_rows) break;
    const int64_t d = rowptr[r + 1] - rowptr[r];
    if (d > seg_len) {
      cnt[0] += 1;
      cnt[1] += (d + seg_len - 1) / seg_len;
    } else if (d <= 1) {
      cnt[2] += 1;
    } else {
      cnt[3] += 1;
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
  __shared__ int64_t lds[4 * kClasses];
  const int64_t r0 = blockIdx.x * kPlanRowsPerBlock + threadIdx.x * kPlanRowsPerThread;
  int64_t cnt[kClasses];
  thread_counts(rowptr, n_rows, seg_len, r0, cnt);
#pragma unroll
  for (int k = 0; k < kClasses; ++k) {
    int64_t t;
    block_exclusive_scan(cnt[k], lds + 4 * k, &t);
    if (threadIdx.x == 0) blk_cnt[kClasses * blockIdx.x + k] = t;
  }
}

// Single workgroup: blk_off = exclusive prefix of blk_cnt per class; totals / counts_out.
__global__ __launch_bounds__(kPlanThreads) void plan_scan_kernel(const int64_t* __restrict__ blk_cnt,
                                                                 int64_t nblk,
                                                                 int64_t* __restrict__ blk_off,
                                                                 int64_t* __restrict__ totals,
                                                                 int64_t* __restrict__ counts_out) {
  __shared__ int64_t lds[4 * kClasses];
  const int64_t per = (nblk + kPlanThreads - 1) / kPlanThreads;
  const int64_t b0 = threadIdx.x * per;
#pragma unroll
  for (int k = 0; k < kClasses; ++k) {
    int64_t sum = 0;
    for (int64_t b = b0; b < b0 + per && b < nblk; ++b) sum += blk_cnt[kClasses * b + k];
    int64_t tot;
    int64_t off = block_exclusive_scan(sum, lds + 4 * k, &tot);
    for (int64_t b = b0; b < b0 + per && b < nblk; ++b) {
      blk_off[kClasses * b + k] = off;
      off += blk_cnt[kClasses * b + k];
    }
    if (threadIdx.x == 0) {
      totals[k] = tot;
      counts_out[k] = tot;
    }
  }
}

__global__ __launch_bounds__(kPlanThreads) void plan_fill_kernel(
    const int64_t* __restrict__ rowptr, const int32_t* __restrict__ col,
    const float* __restrict__ val, int64_t n_rows, int64_t seg_len,
    const int64_t* __restrict__ blk_off, const int64_t* __restrict__ totals,
    int32_t* __restrict__ seg_row, int64_t* __restrict__ seg_begin, int32_t* __restrict__ long_row,
    int32_t* __restrict__ long_seg_ptr, int32_t* __restrict__ small_row,
    int32_t* __restrict__ small_col, float* __restrict__ small_val, int32_t* __restrict__ mid_row) {
  __shared__ int64_t lds[4 * kClasses];
  const int64_t r0 = blockIdx.x * kPlanRowsPerBlock + threadIdx.x * kPlanRowsPerThread;
  int64_t cnt[kClasses], off[kClasses];
  thread_counts(rowptr, n_rows, seg_len, r0, cnt);
#pragma unroll
  for (int k = 0; k < kClasses; ++k) {
    int64_t t;
    off[k] = block_exclusive_scan(cnt[k], lds + 4 * k, &t) + blk_off[kClasses * blockIdx.x + k];
  }
  for (int i = 0; i < kPlanRowsPerThread; ++i) {
    const int64_t r = r0 + i;
    if (r >= n_rows) break;
    const int64_t b = rowptr[r];
    const int64_t d = rowptr[r + 1] - b;
    if (d > seg_len) {
      long_row[off[0]] = static_cast<int32_t>(r);
      long_seg_ptr[off[0]] = static_cast<int32_t>(off[1]);
      ++off[0];
      for (int64_t e = 0; e < d; e += seg_len) {
        seg_row[off[1]] = static_cast<int32_t>(r);
        seg_begin[off[1]] = b + e;
        ++off[1];
      }
    } else if (d <= 1) {
      small_row[off[2]] = static_cast<int32_t>(r);
      small_col[off[2]] = d == 1 ? col[b] : -1;
      small_val[off[2]] = d == 1 ? val[b] : 0.f;
      ++off[2];
    } else {
      mid_row[off[3]] = static_cast<int32_t>(r);
      ++off[3];
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) long_seg_ptr[totals[0]] = static_cast<int32_t>(totals[1]);
}

}  // namespace gnn

using namespace gnn;

extern "C" int64_t gnn_spmm_plan_scratch_bytes(int64_t n_rows) {
  if (n_rows < 0) return GNN_E_ARG;
  return (2 * kClasses * plan_blocks(n_rows) + kClasses) * static_cast<int64_t>(sizeof(int64_t));
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
  int64_t* blk_off = blk_cnt + kClasses * nblk;
  int64_t* totals = blk_off + kClasses * nblk;
  if (nblk == 0) {
    hipError_t e = hipMemsetAsync(counts_dev, 0, kClasses * sizeof(int64_t), s);
    if (e == hipSuccess) e = hipMemsetAsync(totals, 0, kClasses * sizeof(int64_t), s);
    return e == hipSuccess ? GNN_OK : static_cast<int>(e);
  }
  hipLaunchKernelGGL(plan_count_kernel, dim3(static_cast<unsigned>(nblk)), dim3(kPlanThreads), 0,
                     s, rowptr, n_rows, seg_len, blk_cnt);
  hipLaunchKernelGGL(plan_scan_kernel, dim3(1), dim3(kPlanThreads), 0, s, blk_cnt, nblk, blk_off,
                     totals, counts_dev);
  return launch_status();
}

extern "C" int gnn_spmm_plan_fill(const int64_t* rowptr, const int32_t* col, const float* val,
                                  int64_t n_rows, int64_t seg_len, int32_t* seg_row,
                                  int64_t* seg_begin, int32_t* long_row, int32_t* long_seg_ptr,
                                  int32_t* small_row, int32_t* small_col, float* small_val,
                                  int32_t* mid_row, void* scratch, void* stream) {
  if (rowptr == nullptr || scratch == nullptr || long_seg_ptr == nullptr || n_rows < 0 ||
      seg_len < 1)
    return GNN_E_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t nblk = plan_blocks(n_rows);
  int64_t* blk_off = static_cast<int64_t*>(scratch) + kClasses * nblk;
  int64_t* totals = blk_off + kClasses * nblk;
  if (nblk == 0) {
    hipError_t e = hipMemsetAsync(long_seg_ptr, 0, sizeof(int32_t), s);
    return e == hipSuccess ? GNN_OK : static_cast<int>(e);
  }
  hipLaunchKernelGGL(plan_fill_kernel, dim3(static_cast<unsigned>(nblk)), dim3(kPlanThreads), 0, s,
                     rowptr, col, val, n_rows, seg_len, blk_off, totals, seg_row, seg_begin,
                     long_row, long_seg_ptr, small_row, small_col, small_val, mid_row);
  return launch_status();
}

extern "C" int gnn_version(void) { return 100; }

extern "C" const char* gnn_error_string(int code) {
  switch (code) {
    case GNN_OK: return "success";
    case GNN_E_ARG: return "gnn: invalid argument (null pointer, negative size or bad stride)";
    case GNN_E_ALIGN: return "gnn: misaligned pointer";
    case GNN_E_UNSUPPORTED: return "gnn: shape not supported by this library";
    case GNN_E_EMPTY: return "Cannot choose from an empty sequence";
    case GNN_E_RAGGED: return "gnn: index maps of unequal length (ragged nested sequence)";
    case GNN_E_NOMEM: return "gnn: host allocation failed";
    case GNN_E_COMM: return "gnn: RCCL not found in the process, or its call failed";
    default: break;
  }
  if (code > 0) return hipGetErrorString(static_cast<hipError_t>(code));
  return "gnn: unknown error";
}
