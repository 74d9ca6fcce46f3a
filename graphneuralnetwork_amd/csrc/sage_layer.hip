// sage_layer.hip -- one GraphSAGE inference layer fused on gfx950:
//   out[m] = relu(W . cat[self[m], mean_j table[nbr[m, j]]])
//
// Replaces, at inference, SageLayer.forward(self_feats, Aggregator(neigh_feats, 'MEAN'))
// (GraphSAGE/GraphSAGE.py:15-20, graph_utils.py:6) together with the torch.embedding
// gathers that produce its inputs (GraphSAGE.py:47-49, data_utils.py:161-162). The
// unfused path is three launches (centre-row gather, gather-mean, hipBLASLt K=2F GEMM)
// and runs the GEMM only after the last gather; here one persistent launch does both:
//
//   gather phase: the 32-row tile [self | mean of k neighbours] is built in LDS (F/4 lanes
//     per row, 16-B loads, the k neighbour loads of a row in flight together);
//   MFMA phase:   Y_tile = W . tile^T on v_mfma_f32_16x16x4_f32 (exact f32 products, f32
//     accumulation) with W resident in registers for the whole launch, ReLU epilogue,
//     16-B stores. Operands are arranged as in transform.hip (lane quarter q owns the k
//     range [q*S, q*S + S) of the 2F-long rows).
//
// Two workgroups per CU alternate: one gathers (HBM-bound) while the other runs its MFMAs.
#include "common.hpp"

namespace gnn {

constexpr int kSlWaves = 8;
constexpr int kSlBlock = kSlWaves * kWave;
constexpr int kSlRows = 32;  // rows per tile: 2 MFMA row blocks
#ifndef GNN_SL_U
#define GNN_SL_U 4           // neighbour loads in flight per lane (8 spills at 4 waves/SIMD)
#endif
#ifndef GNN_SL_GRID
#define GNN_SL_GRID 512      // persistent grid: 2 workgroups per CU
#endif
using sl32x4 = __attribute__((ext_vector_type(4))) float;

template <int F, int H>
__global__ __launch_bounds__(kSlBlock) __attribute__((amdgpu_waves_per_eu(H == 128 ? 4 : 2))) void sage_layer_kernel(
    const float* __restrict__ table, int64_t ldt, int64_t n_table,
    const float* __restrict__ self_src, int64_t lds, int64_t n_self,
    const int64_t* __restrict__ self_idx, const int64_t* __restrict__ nbr, int64_t ldi,
    int64_t M, int64_t k, const float* __restrict__ w, float* __restrict__ out, int64_t ldo,
    int32_t* __restrict__ err) {
  constexpr int K = 2 * F;
  constexpr int S = K / 4;                    // MFMA k-steps
  constexpr int CB = H / (kSlWaves * 16);     // 16-column blocks per wave
  static_assert(CB >= 1 && CB * kSlWaves * 16 == H, "H must be a multiple of 128");
  constexpr int LDA = K + 4;                  // padded LDS row (floats)
  constexpr int LPR = F / 4;                  // lanes per row in the gather phase
  constexpr int RPW = kWave / LPR;            // rows per wave instruction
  constexpr int RW = kSlRows / kSlWaves;      // tile rows per wave
  static_assert(RW % RPW == 0, "tile rows must split evenly over the half-waves");
  constexpr int U = GNN_SL_U;
  __shared__ float xt[kSlRows * LDA];
  const int lane = threadIdx.x & (kWave - 1);
  const int wv = threadIdx.x >> 6;
  const int q = lane >> 4, r = lane & 15;
  const int sub = lane % LPR, grp = lane / LPR;

  float wa[CB][S];  // W[(wv*CB + cb)*16 + r][q*S + s], resident
#pragma unroll
  for (int cb = 0; cb < CB; ++cb) {
    const float* wr = w + static_cast<int64_t>((wv * CB + cb) * 16 + r) * K + q * S;
#pragma unroll
    for (int v = 0; v < S / 4; ++v) {
      const f4 t = *reinterpret_cast<const f4*>(wr + 4 * v);
      wa[cb][4 * v] = t.x;
      wa[cb][4 * v + 1] = t.y;
      wa[cb][4 * v + 2] = t.z;
      wa[cb][4 * v + 3] = t.w;
    }
  }
  const int64_t n_tiles = (M + kSlRows - 1) / kSlRows;
  for (int64_t t = blockIdx.x; t < n_tiles; t += gridDim.x) {  // uniform over the block
    const int64_t m0 = t * kSlRows;
    // ---- gather phase: [self | mean] rows of the tile into LDS. A lane group owns IT rows
    // of the wave's RW; the self rows and U neighbours of every owned row are in flight
    // together (IT x U 16-B loads per lane).
    constexpr int IT = RW / RPW;
    f4 sv[IT], acc[IT];
    int64_t mr[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      mr[it] = m0 + wv * RW + it * RPW + grp;
      sv[it] = vzero<4>();
      acc[it] = vzero<4>();
      if (mr[it] < M) {
        const float* srow = nullptr;
        if (self_idx) {
          const int64_t s = self_idx[mr[it]];
          if (s >= 0 && s < n_self) srow = self_src + s * lds;
          else if (sub == 0) atomicOr(err, 1);
        } else {
          srow = self_src + mr[it] * lds;
        }
        if (srow) sv[it] = vload<4>(srow + 4 * sub);
      }
    }
    for (int64_t j0 = 0; j0 < k; j0 += U) {
      f4 xv[IT][U];
#pragma unroll
      for (int it = 0; it < IT; ++it) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int64_t j = j0 + u;
          xv[it][u] = vzero<4>();
          if (j < k && mr[it] < M) {
            const int64_t c = nbr[mr[it] * ldi + j];
            if (c >= 0 && c < n_table) xv[it][u] = vload<4>(table + c * ldt + 4 * sub);
            else if (sub == 0) atomicOr(err, 1);
          }
        }
      }
#pragma unroll
      for (int it = 0; it < IT; ++it) {
#pragma unroll
        for (int u = 0; u < U; ++u) acc[it] += xv[it][u];
      }
    }
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int lr = wv * RW + it * RPW + grp;
      *reinterpret_cast<f4*>(xt + lr * LDA + 4 * sub) = sv[it];
      *reinterpret_cast<f4*>(xt + lr * LDA + F + 4 * sub) = acc[it] / static_cast<float>(k);
    }
    __syncthreads();
    // ---- MFMA phase: Y = W . tile^T, ReLU, 16-B stores. The two 16-row blocks and the
    // two halves of the k range accumulate in four independent chains (a single chain of
    // dependent MFMAs would wait out the full MFMA latency at every step).
    constexpr int NRB = kSlRows / 16;
    constexpr int HS = S / 8;  // float4 steps per k half
    sl32x4 d[NRB][2][CB];
#pragma unroll
    for (int rb = 0; rb < NRB; ++rb)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int cb = 0; cb < CB; ++cb) d[rb][h][cb] = sl32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int v = 0; v < HS; ++v) {
      f4 xb[NRB][2];
#pragma unroll
      for (int rb = 0; rb < NRB; ++rb)
#pragma unroll
        for (int h = 0; h < 2; ++h)
          xb[rb][h] = *reinterpret_cast<const f4*>(xt + (rb * 16 + r) * LDA + q * S +
                                                   4 * (h * HS + v));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int rb = 0; rb < NRB; ++rb)
#pragma unroll
            for (int cb = 0; cb < CB; ++cb)
              d[rb][h][cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                  wa[cb][4 * (h * HS + v) + i], xb[rb][h][i], d[rb][h][cb], 0, 0, 0);
    }
#pragma unroll
    for (int rb = 0; rb < NRB; ++rb) {
      // d[rb][0][cb][i] + d[rb][1][cb][i] = Y[m0 + 16 rb + r][(wv*CB + cb)*16 + 4q + i]
      const int64_t orow = m0 + rb * 16 + r;
      if (orow < M) {
#pragma unroll
        for (int cb = 0; cb < CB; ++cb) {
          const sl32x4 y = d[rb][0][cb] + d[rb][1][cb];
          *reinterpret_cast<f4*>(out + orow * ldo + (wv * CB + cb) * 16 + 4 * q) =
              f4{fmaxf(y[0], 0.f), fmaxf(y[1], 0.f), fmaxf(y[2], 0.f), fmaxf(y[3], 0.f)};
        }
      }
    }
    __syncthreads();  // the next tile overwrites xt
  }
}

template <int F, int H>
static int launch_sage_layer(const float* table, int64_t ldt, int64_t n_table,
                             const float* self_src, int64_t lds, int64_t n_self,
                             const int64_t* self_idx, const int64_t* nbr, int64_t ldi, int64_t M,
                             int64_t k, const float* w, float* out, int64_t ldo, int32_t* err,
                             hipStream_t s) {
  const int64_t tiles = (M + kSlRows - 1) / kSlRows;
  const int64_t grid = tiles < GNN_SL_GRID ? tiles : GNN_SL_GRID;
  hipLaunchKernelGGL((sage_layer_kernel<F, H>), dim3(static_cast<unsigned>(grid)), dim3(kSlBlock),
                     0, s, table, ldt, n_table, self_src, lds, n_self, self_idx, nbr, ldi, M, k, w,
                     out, ldo, err);
  return launch_status();
}

}  // namespace gnn

using namespace gnn;

extern "C" int gnn_sage_layer_supported(int64_t feat, int64_t out_features) {
  return (feat == 64 || feat == 128) && (out_features == 128 || out_features == 256);
}

extern "C" int gnn_sage_layer_f32(const float* table, int64_t ldt, int64_t n_table,
                                  const float* self_src, int64_t lds, int64_t n_self,
                                  const int64_t* self_idx, const int64_t* nbr_idx, int64_t ldi,
                                  int64_t M, int64_t k, int64_t feat, const float* w,
                                  int64_t out_features, float* out, int64_t ldo,
                                  int32_t* err_flag, void* stream) {
  if (M < 0 || k < 0 || n_table < 0 || n_self < 0) return GNN_E_ARG;
  if (!gnn_sage_layer_supported(feat, out_features)) return GNN_E_UNSUPPORTED;
  if (M == 0) return GNN_OK;
  if (k == 0) return GNN_E_UNSUPPORTED;  // torch.mean over no neighbour is NaN: unfused path
  if (!table || !self_src || !nbr_idx || !w || !out || !err_flag) return GNN_E_ARG;
  if (ldt < feat || lds < feat || ldi < k || ldo < out_features) return GNN_E_ARG;
  if (ldt % 4 || lds % 4 || ldo % 4 || !aligned_to(table, 16) || !aligned_to(self_src, 16) ||
      !aligned_to(w, 16) || !aligned_to(out, 16))
    return GNN_E_ALIGN;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (feat == 128)
    return out_features == 128
               ? launch_sage_layer<128, 128>(table, ldt, n_table, self_src, lds, n_self, self_idx,
                                             nbr_idx, ldi, M, k, w, out, ldo, err_flag, s)
               : launch_sage_layer<128, 256>(table, ldt, n_table, self_src, lds, n_self, self_idx,
                                             nbr_idx, ldi, M, k, w, out, ldo, err_flag, s);
  return out_features == 128
             ? launch_sage_layer<64, 128>(table, ldt, n_table, self_src, lds, n_self, self_idx,
                                          nbr_idx, ldi, M, k, w, out, ldo, err_flag, s)
             : launch_sage_layer<64, 256>(table, ldt, n_table, self_src, lds, n_self, self_idx,
                                          nbr_idx, ldi, M, k, w, out, ldo, err_flag, s);
}
