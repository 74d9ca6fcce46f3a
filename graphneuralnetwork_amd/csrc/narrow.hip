// narrow.hip -- the classifier-width products of a GCN layer in training: y = x w^T with one
// side narrow.
//
// GCN_Model's last Graph_conv_layer (GCN/GCN.py:16-17: num_hidden -> num_classes, 7 classes at
// cfg2, zero-padded to 8 by ops._GcnLayerFn) computes support = H W^T (GCN/GCN.py:42) in its
// forward and dH = dS W in its backward: [n, 128] x [128, 8] and [n, 8] x [8, 128]. Both are
// HBM-bound (one [n, 128] pass); the library GEMM took 0.146 ms for each at 1M rows.
//
// gnn_linear_small_f32 (fout <= 16, k in {16, 32, 64, 128, 256}): one wave per 16 rows,
// v_mfma_f32_16x16x4_f32 (exact fp32 products, fp32 accumulation). Lane (i, q) = (l & 15, l >> 4)
// loads x[row0 + i][16 t + 4 q .. + 3] for every t (16 rows x 64 B contiguous per load), and
// the k order of MFMA step (t, c) is k = 16 t + 4 q + c, so the A fragment is the lane's own
// float4 component c; the B fragment w[j][16 t + 4 q + c] (j = l & 15) stays resident. The
// 16 x 16 result holds rows 4 q + r of output column j in lane (j, q).
// (k <= 16, fout in {64, 128, 256}): fout / 4 lanes per row, each owning 4 output columns whose
// k weights stay resident; the row's k inputs are read as 16-B pieces (the same for its
// lanes), four rows per lane in flight; fp32 FMAs in k order; 16-B coalesced stores.
#include "common.hpp"

namespace gnn {

constexpr int kSmallBlock = 256;
#ifndef GNN_SMALL_IN_R
#define GNN_SMALL_IN_R 8  // wave steps of the broadcast kernel in flight (tools/small_ab.py,
                          // profiles/r06t_small_ab.log: 8 -> 0.121 ms, 4 -> 0.173, 2 -> 0.135)
#endif
#ifndef GNN_SMALL_IN_NT
#define GNN_SMALL_IN_NT 1  // A/B: nontemporal (streamed) stores of the broadcast kernel
#endif
constexpr int64_t kSmallGrid = 2048;  // persistent: 8 workgroups (32 waves) per CU

template <int K>
__global__ __launch_bounds__(kSmallBlock) void linear_small_out_kernel(
    const float* __restrict__ x, int64_t ldx, int64_t n, const float* __restrict__ w, int fo,
    float* __restrict__ y, int64_t ldy) {
  constexpr int T = K / 16;
  using fx4 = __attribute__((ext_vector_type(4))) float;
  const int lane = threadIdx.x & (kWave - 1);
  const int i = lane & 15, q = lane >> 4;
  float wf[T][4];
#pragma unroll
  for (int t = 0; t < T; ++t)
#pragma unroll
    for (int c = 0; c < 4; ++c) wf[t][c] = i < fo ? w[static_cast<int64_t>(i) * K + 16 * t + 4 * q + c] : 0.f;
  const int64_t waves = static_cast<int64_t>(gridDim.x) * (kSmallBlock / kWave);
  const int64_t n_grp = (n + 15) / 16;
  for (int64_t g = static_cast<int64_t>(blockIdx.x) * (kSmallBlock / kWave) + (threadIdx.x >> 6);
       g < n_grp; g += waves) {
    const int64_t row = g * 16 + i;
    float4 xv[T];
#pragma unroll
    for (int t = 0; t < T; ++t)
      xv[t] = row < n ? *reinterpret_cast<const float4*>(x + row * ldx + 16 * t + 4 * q)
                      : make_float4(0.f, 0.f, 0.f, 0.f);
    fx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < T; ++t) {
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[t].x, wf[t][0], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[t].y, wf[t][1], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[t].z, wf[t][2], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[t].w, wf[t][3], acc, 0, 0, 0);
    }
    if (i < fo) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t orow = g * 16 + 4 * q + r;
        if (orow < n) y[orow * ldy + i] = acc[r];
      }
    }
  }
}

template <int FO, int K4>
__global__ __launch_bounds__(kSmallBlock) void linear_small_in_kernel(
    const float* __restrict__ x, int64_t ldx, int64_t n, int k, const float* __restrict__ w,
    float* __restrict__ y, int64_t ldy) {
  constexpr int LPR = FO / 4;             // lanes per row
  constexpr int RPW = kWave / LPR;        // rows per wave step
  constexpr int R = GNN_SMALL_IN_R;       // wave steps per iteration: their loads issued together
  const int lane = threadIdx.x & (kWave - 1);
  const int sub = lane % LPR, grp = lane / LPR;
  // K4 = ceil(k / 4) float4s of a row are read (ldx >= 4 K4: a multiple of 4 >= k)
  float4 wc[4 * K4];  // w[4 sub .. + 3][kk] for kk < k, zero beyond
#pragma unroll
  for (int kk = 0; kk < 4 * K4; ++kk) {
    const bool ok = kk < k;
    wc[kk] = make_float4(ok ? w[static_cast<int64_t>(4 * sub) * k + kk] : 0.f,
                         ok ? w[static_cast<int64_t>(4 * sub + 1) * k + kk] : 0.f,
                         ok ? w[static_cast<int64_t>(4 * sub + 2) * k + kk] : 0.f,
                         ok ? w[static_cast<int64_t>(4 * sub + 3) * k + kk] : 0.f);
  }
  const int64_t waves = static_cast<int64_t>(gridDim.x) * (kSmallBlock / kWave);
  const int64_t wave = static_cast<int64_t>(blockIdx.x) * (kSmallBlock / kWave) + (threadIdx.x >> 6);
  for (int64_t r0 = wave * RPW * R; r0 < n; r0 += waves * RPW * R) {
    float4 xv[R][K4];
#pragma unroll
    for (int s = 0; s < R; ++s) {
      const int64_t row = r0 + s * RPW + grp;
#pragma unroll
      for (int c = 0; c < K4; ++c)  // the row's k inputs (the same 16-B pieces for its LPR lanes)
        xv[s][c] = row < n ? *reinterpret_cast<const float4*>(x + row * ldx + 4 * c)
                           : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int s = 0; s < R; ++s) {
      const int64_t row = r0 + s * RPW + grp;
      float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int kk = 0; kk < 4 * K4; ++kk) {
        const float v = kk < k ? xv[s][kk / 4][kk % 4] : 0.f;  // columns >= k: never used
        o.x = fmaf(v, wc[kk].x, o.x);
        o.y = fmaf(v, wc[kk].y, o.y);
        o.z = fmaf(v, wc[kk].z, o.z);
        o.w = fmaf(v, wc[kk].w, o.w);
      }
      if (row < n) {  // streamed out: nothing reads y back in this kernel
        if (GNN_SMALL_IN_NT)
          __builtin_nontemporal_store(f4{o.x, o.y, o.z, o.w},
                                      reinterpret_cast<f4*>(y + row * ldy + 4 * sub));
        else
          *reinterpret_cast<float4*>(y + row * ldy + 4 * sub) = o;
      }
    }
  }
}

}  // namespace gnn

using namespace gnn;

template <int K4>
static void launch_small_in(dim3 grid, hipStream_t s, const float* x, int64_t ldx, int64_t n,
                            int k, const float* w, int64_t fout, float* y, int64_t ldy) {
  const dim3 blk(kSmallBlock);
  if (fout == 64)
    hipLaunchKernelGGL((linear_small_in_kernel<64, K4>), grid, blk, 0, s, x, ldx, n, k, w, y, ldy);
  else if (fout == 128)
    hipLaunchKernelGGL((linear_small_in_kernel<128, K4>), grid, blk, 0, s, x, ldx, n, k, w, y, ldy);
  else
    hipLaunchKernelGGL((linear_small_in_kernel<256, K4>), grid, blk, 0, s, x, ldx, n, k, w, y, ldy);
}

// 1: fout <= 16, k in {16, 32, 64, 128, 256} (the MFMA row kernel); 2: k <= 16, fout in
// {64, 128, 256} (the broadcast kernel); 0: not covered
extern "C" int gnn_linear_small_supported(int64_t k, int64_t fout) {
  const bool kp = k == 16 || k == 32 || k == 64 || k == 128 || k == 256;
  if (fout >= 1 && fout <= 16 && kp) return 1;
  if (k >= 1 && k <= 16 && (fout == 64 || fout == 128 || fout == 256)) return 2;
  return 0;
}

// y[n, fout] = x[n, k] w^T (w [fout, k] row-major, nn.Linear's layout), fp32. x and y 16-B
// aligned with row strides multiples of 4 floats (GNN_E_ALIGN).
extern "C" int gnn_linear_small_f32(const float* x, int64_t ldx, int64_t n_rows, int64_t k,
                                    const float* w, int64_t fout, float* y, int64_t ldy,
                                    void* stream) {
  const int kind = gnn_linear_small_supported(k, fout);
  if (!kind) return GNN_E_UNSUPPORTED;
  if (n_rows < 0 || ldx < k || ldy < fout) return GNN_E_ARG;
  if (n_rows == 0) return GNN_OK;
  if (!x || !w || !y) return GNN_E_ARG;
  if (!aligned_to(x, 16) || !aligned_to(y, 16) || ldx % 4 || ldy % 4) return GNN_E_ALIGN;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t waves_needed =
      kind == 1 ? (n_rows + 15) / 16 : (n_rows * fout / 4 + 4 * kWave - 1) / (4 * kWave);
  const int64_t blocks = (waves_needed + 3) / 4;
  const dim3 grid(static_cast<unsigned>(blocks < kSmallGrid ? blocks : kSmallGrid)), blk(kSmallBlock);
  if (kind == 1) {
    const int fo = static_cast<int>(fout);
    switch (k) {
      case 16: hipLaunchKernelGGL((linear_small_out_kernel<16>), grid, blk, 0, s, x, ldx, n_rows, w, fo, y, ldy); break;
      case 32: hipLaunchKernelGGL((linear_small_out_kernel<32>), grid, blk, 0, s, x, ldx, n_rows, w, fo, y, ldy); break;
      case 64: hipLaunchKernelGGL((linear_small_out_kernel<64>), grid, blk, 0, s, x, ldx, n_rows, w, fo, y, ldy); break;
      case 128: hipLaunchKernelGGL((linear_small_out_kernel<128>), grid, blk, 0, s, x, ldx, n_rows, w, fo, y, ldy); break;
      case 256: hipLaunchKernelGGL((linear_small_out_kernel<256>), grid, blk, 0, s, x, ldx, n_rows, w, fo, y, ldy); break;
      default: return GNN_E_UNSUPPORTED;
    }
    return launch_status();
  }
  const int kk = static_cast<int>(k);
  switch ((kk + 3) / 4) {
    case 1: launch_small_in<1>(grid, s, x, ldx, n_rows, kk, w, fout, y, ldy); break;
    case 2: launch_small_in<2>(grid, s, x, ldx, n_rows, kk, w, fout, y, ldy); break;
    case 3: launch_small_in<3>(grid, s, x, ldx, n_rows, kk, w, fout, y, ldy); break;
    default: launch_small_in<4>(grid, s, x, ldx, n_rows, kk, w, fout, y, ldy); break;
  }
  return launch_status();
}
