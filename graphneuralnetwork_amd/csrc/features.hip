// features.hip -- GCN feature row normalisation, bit-exact with the reference loader.
//
// Replaces normalize_features (GCN/data_utils.py:39-51) as load_cora applies it
// (features = normalize_features(features); torch.Tensor(features.toarray()),
// GCN/data_utils.py:81-83):
//   rowsum_i = scipy's csr sum over the row's stored (nonzero) values = np.add.reduceat:
//              the first value plus numpy's float32 pairwise sum of the rest;
//   r_i      = rowsum_i ** -1 in float64, inf -> 0;
//   y_ij     = fp32(r_i * x_ij) in float64, and +0.0 where x_ij == 0 or r_i == 0 (the sparse
//              product drops exact zeros, so toarray() reads +0.0 there).
//
// One wave per row (1-wave workgroups, grid-stride over rows). The row's nonzeros are
// compacted into LDS in column order (ballot + popcount prefix per 64-column chunk), lane 0
// evaluates numpy's pairwise tree over them with an explicit stack, and all lanes write the
// scaled row. A preprocessing op (once per dataset): written for exactness, not speed.
#include "common.hpp"

namespace gnn {

constexpr int64_t kFeatMaxCols = 16384;  // LDS: one float per column (64 KiB)

// numpy 2.x FLOAT_pairwise_sum over a[0..n): < 8 values left to right from -0.0; <= 128
// values in 8 strided accumulators ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) then the tail;
// longer runs split at n/2 rounded down to a multiple of 8 (left + right).
__device__ float np_pairwise_leaf(const float* a, int64_t n) {
  if (n < 8) {
    float res = -0.0f;
    for (int64_t i = 0; i < n; ++i) res += a[i];
    return res;
  }
  float r[8];
  for (int j = 0; j < 8; ++j) r[j] = a[j];
  int64_t i = 8;
  for (; i < n - (n % 8); i += 8)
    for (int j = 0; j < 8; ++j) r[j] += a[i + j];
  float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res += a[i];
  return res;
}

__device__ float np_pairwise(const float* a, int64_t n) {
  if (n <= 128) return np_pairwise_leaf(a, n);
  // post-order walk of the split tree: depth <= log2(kFeatMaxCols / 128) + 1
  int64_t off[16], cnt[16];
  int stage[16];
  float left[16];
  int sp = 0;
  off[0] = 0;
  cnt[0] = n;
  stage[0] = 0;
  float ret = 0.f;
  while (sp >= 0) {
    if (stage[sp] == 0 && cnt[sp] <= 128) {  // a leaf: its sum goes to the parent
      ret = np_pairwise_leaf(a + off[sp], cnt[sp]);
      --sp;
      continue;
    }
    int64_t n2 = cnt[sp] / 2;
    n2 -= n2 % 8;
    if (stage[sp] == 0) {  // descend left
      stage[sp] = 1;
      off[sp + 1] = off[sp];
      cnt[sp + 1] = n2;
    } else if (stage[sp] == 1) {  // left done: descend right
      left[sp] = ret;
      stage[sp] = 2;
      off[sp + 1] = off[sp] + n2;
      cnt[sp + 1] = cnt[sp] - n2;
    } else {  // both done
      ret = left[sp] + ret;
      --sp;
      continue;
    }
    ++sp;
    stage[sp] = 0;
  }
  return ret;
}

__global__ __launch_bounds__(kWave) void normalize_features_kernel(const float* __restrict__ x,
                                                                   int64_t ldx, int64_t n_rows,
                                                                   int64_t n_cols,
                                                                   float* __restrict__ y,
                                                                   int64_t ldy) {
  extern __shared__ float nzv[];
  const int lane = threadIdx.x;
  const uint64_t below = (1ull << lane) - 1ull;
  for (int64_t row = blockIdx.x; row < n_rows; row += gridDim.x) {
    const float* xr = x + row * ldx;
    int nnz = 0;
    for (int64_t c0 = 0; c0 < n_cols; c0 += kWave) {
      const int64_t c = c0 + lane;
      const float v = c < n_cols ? xr[c] : 0.f;
      const bool nz = v != 0.f;  // -0.0 is not stored by sp.csr_matrix either
      const uint64_t m = __ballot(nz);
      if (nz) nzv[nnz + __popcll(m & below)] = v;
      nnz += __popcll(m);
    }
    __syncthreads();  // the compacted row is complete before lane 0 reads it
    double r = 0.0;
    if (lane == 0 && nnz > 0) {
      const float s = nnz == 1 ? nzv[0] : nzv[0] + np_pairwise(nzv + 1, nnz - 1);
      r = 1.0 / static_cast<double>(s);
      if (isinf(r)) r = 0.0;
    }
    r = __shfl(r, 0, kWave);
    __syncthreads();  // lane 0 is done with nzv before the next row overwrites it
    float* yr = y + row * ldy;
    for (int64_t c0 = 0; c0 < n_cols; c0 += kWave) {
      const int64_t c = c0 + lane;
      if (c < n_cols) {
        const float v = xr[c];
        yr[c] = (v == 0.f || r == 0.0) ? 0.f : static_cast<float>(r * static_cast<double>(v));
      }
    }
  }
}

}  // namespace gnn

using namespace gnn;

extern "C" int gnn_normalize_features_f32(const float* x, int64_t ldx, int64_t n_rows,
                                          int64_t n_cols, float* y, int64_t ldy, void* stream) {
  if (n_rows < 0 || n_cols < 0 || ldx < n_cols || ldy < n_cols) return GNN_E_ARG;
  if (n_cols > kFeatMaxCols) return GNN_E_UNSUPPORTED;
  if (n_rows == 0 || n_cols == 0) return GNN_OK;
  if (!x || !y) return GNN_E_ARG;
  // x and y must not overlap (x is re-read after the row's sum, while y is written)
  const float* x_end = x + (n_rows - 1) * ldx + n_cols;
  const float* y_end = y + (n_rows - 1) * ldy + n_cols;
  if (x < y_end && y < x_end) return GNN_E_ARG;
  const int64_t grid = n_rows < 8192 ? n_rows : 8192;
  hipLaunchKernelGGL(normalize_features_kernel, dim3(static_cast<unsigned>(grid)), dim3(kWave),
                     static_cast<size_t>(n_cols) * sizeof(float), static_cast<hipStream_t>(stream),
                     x, ldx, n_rows, n_cols, y, ldy);
  return launch_status();
}
