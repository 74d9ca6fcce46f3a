// transform.hip -- the GCN feature transform on the matrix cores: Y = X W^T (fp32).
//
// Replaces `support = self.dense(X_input)` (nn.Linear, no bias) at GCN/GCN.py:42, the
// dense half of Graph_conv_layer.forward, for the inference path (no autograd).
// Shapes: X [n, K] row-major, W [FO, K] (nn.Linear's [out, in]), Y [n, FO].
//
// One workgroup = 4 waves; the X tile (64 rows x K) is staged in LDS once by all four
// waves with fully coalesced 16-B loads (the next tile is prefetched into registers
// while the MFMAs run) and each wave computes all 64 rows for its FO/4 output columns
// with v_mfma_f32_16x16x4_f32 (exact f32 products, f32 accumulation). W stays in
// registers for the whole launch (persistent grid). Operands are arranged as in
// project.hip: D = W_blk X_tile^T, so a lane's four accumulators are four consecutive
// columns of one Y row (16-B stores), and the K axis is permuted so that lane quarter q
// owns k in [q*S, q*S + S): its X values are one contiguous run of an LDS row (float4
// reads, rows padded by 4 floats so the 16 rows of a read hit distinct banks).
#include "common.hpp"

namespace gnn {

constexpr int kTfWaves = 4;
constexpr int kTfBlock = kTfWaves * kWave;
constexpr int kTfRows = 64;  // rows per tile (4 MFMA row blocks)
using tf32x4 = __attribute__((ext_vector_type(4))) float;

template <int K, int CB>
__global__ __launch_bounds__(kTfBlock) void gcn_transform_kernel(const float* __restrict__ x,
                                                                 int64_t ldx, int64_t n_rows,
                                                                 const float* __restrict__ w,
                                                                 float* __restrict__ y,
                                                                 int64_t ldy) {
  constexpr int S = K / 4;           // MFMA k-steps
  constexpr int FO = kTfWaves * CB * 16;
  constexpr int LDA = K + 4;         // padded LDS row (floats)
  constexpr int V4 = kTfRows * K / 4;  // float4s per tile
  constexpr int NV = V4 / kTfBlock;    // per thread
  static_assert(V4 % kTfBlock == 0, "tile must split evenly over the workgroup");
  __shared__ float xt[kTfRows * LDA];
  const int lane = threadIdx.x & (kWave - 1);
  const int wv = threadIdx.x >> 6;
  const int q = lane >> 4, r = lane & 15;

  // A fragments: W[c0 + r][q*S + s] for this wave's CB column blocks, resident
  float wa[CB][S];
#pragma unroll
  for (int cb = 0; cb < CB; ++cb) {
    const float* wr = w + static_cast<int64_t>((wv * CB + cb) * 16 + r) * K + q * S;
#pragma unroll
    for (int v = 0; v < S / 4; ++v) {
      const float4 t = *reinterpret_cast<const float4*>(wr + 4 * v);
      wa[cb][4 * v] = t.x;
      wa[cb][4 * v + 1] = t.y;
      wa[cb][4 * v + 2] = t.z;
      wa[cb][4 * v + 3] = t.w;
    }
  }

  const int64_t n_tiles = (n_rows + kTfRows - 1) / kTfRows;
  float4 pre[NV];
  auto fetch = [&](int64_t g) {
    const int64_t r0 = g * kTfRows;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int e = v * kTfBlock + static_cast<int>(threadIdx.x);
      const int rr = e / (K / 4), c4 = e - rr * (K / 4);
      pre[v] = (g < n_tiles && r0 + rr < n_rows)
                   ? *reinterpret_cast<const float4*>(x + (r0 + rr) * ldx + 4 * c4)
                   : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  fetch(blockIdx.x);
  for (int64_t g = blockIdx.x; g < n_tiles; g += gridDim.x) {  // uniform over the block
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int e = v * kTfBlock + static_cast<int>(threadIdx.x);
      const int rr = e / (K / 4), c4 = e - rr * (K / 4);
      *reinterpret_cast<float4*>(xt + rr * LDA + 4 * c4) = pre[v];
    }
    __syncthreads();
    fetch(g + gridDim.x);
    const int64_t row0 = g * kTfRows;
#pragma unroll
    for (int rb = 0; rb < kTfRows / 16; ++rb) {
      float xb[S];
      const float* xr = xt + (rb * 16 + r) * LDA + q * S;
#pragma unroll
      for (int v = 0; v < S / 4; ++v) {
        const float4 t = *reinterpret_cast<const float4*>(xr + 4 * v);
        xb[4 * v] = t.x;
        xb[4 * v + 1] = t.y;
        xb[4 * v + 2] = t.z;
        xb[4 * v + 3] = t.w;
      }
      tf32x4 acc[CB];
#pragma unroll
      for (int cb = 0; cb < CB; ++cb) acc[cb] = tf32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < S; ++s) {
#pragma unroll
        for (int cb = 0; cb < CB; ++cb)
          acc[cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[cb][s], xb[s], acc[cb], 0, 0, 0);
      }
      // acc[cb][i] = Y[row0 + 16 rb + r][(wv*CB + cb)*16 + 4q + i]
      const int64_t orow = row0 + rb * 16 + r;
      if (orow < n_rows) {
#pragma unroll
        for (int cb = 0; cb < CB; ++cb)
          *reinterpret_cast<float4*>(y + orow * ldy + (wv * CB + cb) * 16 + 4 * q) =
              make_float4(acc[cb][0], acc[cb][1], acc[cb][2], acc[cb][3]);
      }
    }
    __syncthreads();  // the next tile overwrites xt
  }
  (void)FO;
}

template <int K, int CB>
static int launch_transform(const float* x, int64_t ldx, int64_t n_rows, const float* w,
                            float* y, int64_t ldy, hipStream_t s) {
  const int64_t tiles = (n_rows + kTfRows - 1) / kTfRows;
#ifndef GNN_TF_GRID
#define GNN_TF_GRID 512  // persistent grid: 2 workgroups per CU
#endif
  const int64_t grid = tiles < GNN_TF_GRID ? tiles : GNN_TF_GRID;
  hipLaunchKernelGGL((gcn_transform_kernel<K, CB>), dim3(static_cast<unsigned>(grid)),
                     dim3(kTfBlock), 0, s, x, ldx, n_rows, w, y, ldy);
  return launch_status();
}

template <int K>
static int dispatch_transform(int64_t fout, const float* x, int64_t ldx, int64_t n_rows,
                              const float* w, float* y, int64_t ldy, hipStream_t s) {
  if (fout == 64) return launch_transform<K, 1>(x, ldx, n_rows, w, y, ldy, s);
  if constexpr (K <= 128)
    if (fout == 128) return launch_transform<K, 2>(x, ldx, n_rows, w, y, ldy, s);
  if constexpr (K <= 64)
    if (fout == 256) return launch_transform<K, 4>(x, ldx, n_rows, w, y, ldy, s);
  return GNN_E_UNSUPPORTED;
}

}  // namespace gnn

using namespace gnn;

extern "C" int gnn_gcn_transform_supported(int64_t k, int64_t fout) {
  const bool kk = k == 16 || k == 32 || k == 64 || k == 128 || k == 256;
  if (!kk) return 0;
  if (fout == 64) return 1;
  if (fout == 128) return k <= 128;
  if (fout == 256) return k <= 64;
  return 0;
}

extern "C" int gnn_gcn_transform_f32(const float* x, int64_t ldx, int64_t n_rows, int64_t k,
                                     const float* w, int64_t fout, float* y, int64_t ldy,
                                     void* stream) {
  if (n_rows < 0 || ldx < k || ldy < fout) return GNN_E_ARG;
  if (!gnn_gcn_transform_supported(k, fout)) return GNN_E_UNSUPPORTED;
  if (n_rows == 0) return GNN_OK;
  if (!x || !w || !y) return GNN_E_ARG;
  if (ldx % 4 || ldy % 4 || !aligned_to(x, 16) || !aligned_to(y, 16) || !aligned_to(w, 16))
    return GNN_E_ALIGN;
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (k) {
    case 16: return dispatch_transform<16>(fout, x, ldx, n_rows, w, y, ldy, s);
    case 32: return dispatch_transform<32>(fout, x, ldx, n_rows, w, y, ldy, s);
    case 64: return dispatch_transform<64>(fout, x, ldx, n_rows, w, y, ldy, s);
    case 128: return dispatch_transform<128>(fout, x, ldx, n_rows, w, y, ldy, s);
    default: return dispatch_transform<256>(fout, x, ldx, n_rows, w, y, ldy, s);
  }
}
