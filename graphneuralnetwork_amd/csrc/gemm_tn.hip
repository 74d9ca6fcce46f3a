// gemm_tn.hip -- the weight gradients of the training step: C = A^T B over a long row axis.
//
// Replaces the autograd GEMMs of nn.Linear inside the reference's training loops
// (GCN/train_eval.py:43-48 through Graph_conv_layer's `self.dense`, GCN/GCN.py:42: dW = dS^T X;
// GAT/train_eval.py:75-76 through `torch.mm(h, self.W)`, GAT/models/layers.py:23: dW = h^T dWh),
// and the bias gradient db = column sums of dY (GCN/GCN.py:45). A [n, M], B [n, K] with n the
// node count (1M-10M) and M, K <= 128: a tall-skinny reduction with a tiny output, where a
// library GEMM parallelises badly (hipBLASLt: 1.81 ms for 1M x 128 x 128 at cfg2, 7 % of HBM).
//
// Each workgroup reduces a contiguous block of rows: 32-row tiles of A and B are staged in LDS
// with coalesced 16-B loads (the next tile is loaded into registers while this one is
// multiplied), and thread (tm, tk) accumulates its TM x TK patch of the outer products in fp32
// registers, in row order. The per-workgroup partials go to a workspace and a second kernel sums
// them in workgroup order: deterministic, no atomics. That FMA kernel serves M = 8; M, K >= 64
// run gemm_tn_mfma_kernel below (the same staging, fp32 MFMA products).
// Optional: dsum[k] = sum_i D[i, k] (a third [n, K] operand, accumulated while its tiles pass).
#include "common.hpp"

namespace gnn {

constexpr int kTnThreads = 256;
constexpr int kTnRows = 32;  // rows per LDS tile

template <int M, int K>
struct TnShape {
  // the 256 threads tile the M x K output as (M / TM) x (K / TK)
  static constexpr int TM = M >= 128 ? 8 : (M >= 64 ? 4 : 1);
  static constexpr int TK = (M / TM) * (K / 8) == kTnThreads ? 8
                          : (M / TM) * (K / 4) == kTnThreads ? 4
                          : (M / TM) * (K / 2) == kTnThreads ? 2 : 1;
  static_assert((M / TM) * (K / TK) == kTnThreads, "unsupported (M, K)");
  static constexpr int A4 = M / 4, B4 = K / 4;  // float4s per row
};

template <int M, int K, bool DSUM>
__global__ __launch_bounds__(kTnThreads) void gemm_tn_partial_kernel(
    const float* __restrict__ a, int64_t lda, const float* __restrict__ b, int64_t ldb,
    const float* __restrict__ d, int64_t ldd, int64_t n, int64_t rows_per_block,
    float* __restrict__ part) {
  using S = TnShape<M, K>;
  constexpr int TM = S::TM, TK = S::TK, A4 = S::A4, B4 = S::B4;
  constexpr int NA = (kTnRows * A4 + kTnThreads - 1) / kTnThreads;  // float4s per thread per tile
  constexpr int NB = (kTnRows * B4 + kTnThreads - 1) / kTnThreads;
  __shared__ float4 sa[kTnRows * A4];
  __shared__ float4 sb[kTnRows * B4];
  const int t = threadIdx.x;
  const int tm = t / (K / TK), tk = t % (K / TK);
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_block;
  const int64_t r1 = min(n, r0 + rows_per_block);
  float acc[TM][TK];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TK; ++j) acc[i][j] = 0.f;
  float4 ds[NB];  // DSUM: this thread's running sums of the D float4s it stages
#pragma unroll
  for (int q = 0; q < NB; ++q) ds[q] = make_float4(0.f, 0.f, 0.f, 0.f);

  auto load = [&](int64_t row0, float4 (&va)[NA], float4 (&vb)[NB], float4 (&vd)[NB]) {
#pragma unroll
    for (int q = 0; q < NA; ++q) {
      const int i = t + q * kTnThreads;
      const int64_t row = row0 + i / A4;
      va[q] = (i < kTnRows * A4 && row < r1)
                  ? *reinterpret_cast<const float4*>(a + row * lda + 4 * (i % A4))
                  : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      const int i = t + q * kTnThreads;
      const int64_t row = row0 + i / B4;
      const bool ok = i < kTnRows * B4 && row < r1;
      vb[q] = ok ? *reinterpret_cast<const float4*>(b + row * ldb + 4 * (i % B4))
                 : make_float4(0.f, 0.f, 0.f, 0.f);
      if constexpr (DSUM)
        vd[q] = ok ? *reinterpret_cast<const float4*>(d + row * ldd + 4 * (i % B4))
                   : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };

  float4 va[NA], vb[NB], vd[NB];
  load(r0, va, vb, vd);
  for (int64_t row0 = r0; row0 < r1; row0 += kTnRows) {
    __syncthreads();  // the previous tile's readers are done
#pragma unroll
    for (int q = 0; q < NA; ++q) {
      const int i = t + q * kTnThreads;
      if (i < kTnRows * A4) sa[i] = va[q];
    }
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      const int i = t + q * kTnThreads;
      if (i < kTnRows * B4) sb[i] = vb[q];
      if constexpr (DSUM) {
        ds[q].x += vd[q].x;
        ds[q].y += vd[q].y;
        ds[q].z += vd[q].z;
        ds[q].w += vd[q].w;
      }
    }
    __syncthreads();
    if (row0 + kTnRows < r1) load(row0 + kTnRows, va, vb, vd);  // next tile in flight
    const int nr = static_cast<int>(min(static_cast<int64_t>(kTnRows), r1 - row0));
    for (int r = 0; r < nr; ++r) {
      float x[TM], y[TK];
      const float* ar = reinterpret_cast<const float*>(sa + r * A4) + tm * TM;
      const float* br = reinterpret_cast<const float*>(sb + r * B4) + tk * TK;
#pragma unroll
      for (int i = 0; i < TM; ++i) x[i] = ar[i];
#pragma unroll
      for (int j = 0; j < TK; ++j) y[j] = br[j];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TK; ++j) acc[i][j] = fmaf(x[i], y[j], acc[i][j]);
    }
  }
  float* pc = part + static_cast<int64_t>(blockIdx.x) * (M * K + (DSUM ? K : 0));
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TK; ++j) pc[(tm * TM + i) * K + tk * TK + j] = acc[i][j];
  if constexpr (DSUM) {
    // every thread stages the same float4 columns of D in every tile (i % B4 is fixed per q):
    // the threads holding column group c are t = c + B4 * s; sum them in a fixed order via LDS
    __syncthreads();
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      const int i = t + q * kTnThreads;
      if (i < kTnRows * B4) sb[i] = ds[q];
    }
    __syncthreads();
    if (t < B4) {
      float4 s4 = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int i = t; i < kTnRows * B4; i += B4) {
        s4.x += sb[i].x;
        s4.y += sb[i].y;
        s4.z += sb[i].z;
        s4.w += sb[i].w;
      }
      pc[M * K + 4 * t] = s4.x;
      pc[M * K + 4 * t + 1] = s4.y;
      pc[M * K + 4 * t + 2] = s4.z;
      pc[M * K + 4 * t + 3] = s4.w;
    }
  }
}

// The same partials on the fp32 MFMA (v_mfma_f32_32x32x2_f32: exact fp32, a k-ordered fmaf
// chain, 64 FLOP/clk/SIMD; the FMA kernel above is VALU-bound at ~53 TF/s). The tiles are
// staged exactly as above (each element loaded once, coalesced, the next tile in flight); rows
// are padded by 32 floats so that the two lane halves of an operand read (rows r, r + 1) hit
// disjoint banks. For a row pair, lane l holds A[i = l & 31][k = l >> 5] and B[k][j = l & 31]
// (cdna_hip_programming.md: the 32x32x2 f32 operand maps): wave (h, s) multiplies A's 32-column
// block h into every 32-column block of B (K / 32 accumulator tiles) over the tile's row pairs
// s, s + S, ... (S = 4 / (M / 32)); the S partials are summed in s order through LDS.
typedef float f16x __attribute__((ext_vector_type(16)));

template <int M, int K, bool DSUM>
__global__ __launch_bounds__(kTnThreads) void gemm_tn_mfma_kernel(
    const float* __restrict__ a, int64_t lda, const float* __restrict__ b, int64_t ldb,
    const float* __restrict__ d, int64_t ldd, int64_t n, int64_t rows_per_block,
    float* __restrict__ part) {
  constexpr int A4 = M / 4, B4 = K / 4;
  constexpr int PA = M + 32, PB = K + 32;  // padded LDS row pitches (floats)
  constexpr int NA = (kTnRows * A4 + kTnThreads - 1) / kTnThreads;
  constexpr int NB = (kTnRows * B4 + kTnThreads - 1) / kTnThreads;
  constexpr int QA = M / 32, QB = K / 32;
  constexpr int S = 4 / QA;  // row-pair streams per tile
  __shared__ float4 sa[kTnRows * PA / 4];
  __shared__ float4 sb[kTnRows * PB / 4];
  __shared__ float red[S > 1 ? M * K : 1];
  const int t = threadIdx.x;
  const int lane = t & 63, w = t >> 6;
  const int h = w % QA, s = w / QA;
  const int i = lane & 31, kk = lane >> 5;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_block;
  const int64_t r1 = min(n, r0 + rows_per_block);
  f16x acc[QB];
#pragma unroll
  for (int q = 0; q < QB; ++q) acc[q] = f16x(0.f);
  float4 ds[NB];
#pragma unroll
  for (int q = 0; q < NB; ++q) ds[q] = make_float4(0.f, 0.f, 0.f, 0.f);

  auto load = [&](int64_t row0, float4 (&va)[NA], float4 (&vb)[NB], float4 (&vd)[NB]) {
#pragma unroll
    for (int q = 0; q < NA; ++q) {
      const int e = t + q * kTnThreads;
      const int64_t row = row0 + e / A4;
      va[q] = (e < kTnRows * A4 && row < r1)
                  ? *reinterpret_cast<const float4*>(a + row * lda + 4 * (e % A4))
                  : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      const int e = t + q * kTnThreads;
      const int64_t row = row0 + e / B4;
      const bool ok = e < kTnRows * B4 && row < r1;
      vb[q] = ok ? *reinterpret_cast<const float4*>(b + row * ldb + 4 * (e % B4))
                 : make_float4(0.f, 0.f, 0.f, 0.f);
      if constexpr (DSUM)
        vd[q] = ok ? *reinterpret_cast<const float4*>(d + row * ldd + 4 * (e % B4))
                   : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };

  // one register set: tile k + 1's loads in flight during tile k's MFMAs (two sets, tile k + 2
  // in flight as well, took 184 VGPRs + 128 AGPRs at 128 x 128: one wave per SIMD)
  float4 va[NA], vb[NB], vd[NB];
  load(r0, va, vb, vd);
  const float* saf = reinterpret_cast<const float*>(sa);
  const float* sbf = reinterpret_cast<const float*>(sb);
  for (int64_t row0 = r0; row0 < r1; row0 += kTnRows) {
    __syncthreads();  // the previous tile's readers are done
#pragma unroll
    for (int q = 0; q < NA; ++q) {
      const int e = t + q * kTnThreads;
      if (e < kTnRows * A4) sa[(e / A4) * (PA / 4) + e % A4] = va[q];
    }
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      const int e = t + q * kTnThreads;
      if (e < kTnRows * B4) sb[(e / B4) * (PB / 4) + e % B4] = vb[q];
      if constexpr (DSUM) {
        ds[q].x += vd[q].x;
        ds[q].y += vd[q].y;
        ds[q].z += vd[q].z;
        ds[q].w += vd[q].w;
      }
    }
    __syncthreads();
    if (row0 + kTnRows < r1) load(row0 + kTnRows, va, vb, vd);  // next tile in flight
    const int np = static_cast<int>((min(static_cast<int64_t>(kTnRows), r1 - row0) + 1) / 2);
    for (int p = s; p < np; p += S) {  // rows past r1 were staged as zeros
      const int r = 2 * p + kk;
      const float av = saf[r * PA + 32 * h + i];
#pragma unroll
      for (int q = 0; q < QB; ++q)
        acc[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, sbf[r * PB + 32 * q + i], acc[q], 0, 0, 0);
    }
  }
  float* pc = part + static_cast<int64_t>(blockIdx.x) * (M * K + (DSUM ? K : 0));
  // the S row-pair streams' partials, summed in s order: s = S - 1 stores, ..., s = 0 writes
  for (int tt = S - 1; tt >= 0; --tt) {
    if (s == tt) {
#pragma unroll
      for (int q = 0; q < QB; ++q) {
#pragma unroll
        for (int rg = 0; rg < 16; ++rg) {
          const int m = 32 * h + (rg & 3) + 8 * (rg >> 2) + 4 * kk, nn = 32 * q + i;
          float v = acc[q][rg];
          if (tt < S - 1) v += red[m * K + nn];
          if (tt > 0)
            red[m * K + nn] = v;
          else
            pc[m * K + nn] = v;
        }
      }
    }
    __syncthreads();
  }
  if constexpr (DSUM) {
    // as the FMA kernel: the threads holding column group c (t = c + B4 * j) summed in order
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      const int e = t + q * kTnThreads;
      if (e < kTnRows * B4) sb[e] = ds[q];
    }
    __syncthreads();
    if (t < B4) {
      float4 s4 = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int e = t; e < kTnRows * B4; e += B4) {
        s4.x += sb[e].x;
        s4.y += sb[e].y;
        s4.z += sb[e].z;
        s4.w += sb[e].w;
      }
      pc[M * K + 4 * t] = s4.x;
      pc[M * K + 4 * t + 1] = s4.y;
      pc[M * K + 4 * t + 2] = s4.z;
      pc[M * K + 4 * t + 3] = s4.w;
    }
  }
}

// The same partials from bf16 MFMAs on three-piece splits (common.hpp split3: each fp32 operand
// = v0 + v1 + v2 in bf16, the six piece products down to order 2^-16 summed in fp32 -- the
// transforms' "X6" arithmetic, error per product at fp32 rounding). v_mfma_f32_32x32x16_bf16
// takes 16 node rows per instruction: lane l holds A[rows 16 s + 8 (l >> 5) + j][column l & 31]
// for j = 0..7 (cdna_hip_programming.md, the bf16 A / B lane maps), so each lane reads a
// column strip of the staged tile: 8 ds_read_b32 down the rows, which the row pitch M + 4
// (8 rows apart = 32 banks apart) keeps conflict-free for the two lane halves; the strips are
// split in registers. 6 x 32 cycles per 16 rows x 32 x 32 outputs against 8 x 64 on the f32
// MFMA: the kernel is left paced by its HBM reads. C/D lane map as the f32 form's.
#ifndef GNN_TN_X6_2X2
#define GNN_TN_X6_2X2 1  // 128 x 128 outputs as 2 x 2 blocks of 32 x 32 per wave (0: 1 x 4;
                         // tools/tn_ab.py, profiles/r06v_tn_ab.log: DB 0.282 vs 0.325 ms,
                         // masked 0.331 vs 0.352 at 1M rows)
#endif
// DB: D is B (dsum = the column sums of B, taken from B's own staged loads: no third read --
// the bias gradient next to dW = dY^T Z of a layer trained as (A X) W^T + b).
// MB: D is a mask H and the kernel multiplies B' = B . [H > 0] * mscale (elementwise, at
// staging), dsum from B' -- dW, db of that layer when its ReLU and Dropout ran in the
// transform's epilogue (H = their output: H > 0 exactly where the gradient passes).
template <int M, int K, bool DSUM, bool DB = false, bool MB = false>
__global__ __launch_bounds__(kTnThreads, 2) void gemm_tn_x6_kernel(
    const float* __restrict__ a, int64_t lda, const float* __restrict__ b, int64_t ldb,
    const float* __restrict__ d, int64_t ldd, int64_t n, int64_t rows_per_block,
    float* __restrict__ part, float mscale) {
  constexpr int A4 = M / 4, B4 = K / 4;
  constexpr int PA = M + 4, PB = K + 4;  // padded LDS row pitches (floats)
  constexpr int NA = (kTnRows * A4 + kTnThreads - 1) / kTnThreads;
  constexpr int NB = (kTnRows * B4 + kTnThreads - 1) / kTnThreads;
  constexpr int QA = M / 32, QB = K / 32;
  constexpr int S = 4 / QA;  // k-step streams per tile
  // the 4 waves' share of the QA x QB output blocks: one A block x all B blocks each, or (T22,
  // M = K = 128) 2 x 2 blocks each -- every wave then splits 2 + 2 strips per step, not 1 + 4
  constexpr bool T22 = GNN_TN_X6_2X2 != 0 && QA == 4 && QB == 4;
  constexpr int WH = T22 ? 2 : 1, WQ = T22 ? 2 : QB;
  __shared__ float4 sa[kTnRows * PA / 4];
  __shared__ float4 sb[kTnRows * PB / 4];
  __shared__ float red[S > 1 ? M * K : 1];
  const int t = threadIdx.x;
  const int lane = t & 63, w = t >> 6;
  const int s = T22 ? 0 : w / QA;
  const int hb = T22 ? 2 * (w & 1) : w % QA;  // this wave's first A block
  const int qb = T22 ? 2 * (w >> 1) : 0;      // and first B block
  const int i = lane & 31, kh = lane >> 5;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_block;
  const int64_t r1 = min(n, r0 + rows_per_block);
  f16x acc[WH][WQ];
#pragma unroll
  for (int hi = 0; hi < WH; ++hi)
#pragma unroll
    for (int q = 0; q < WQ; ++q) acc[hi][q] = f16x(0.f);
  float4 ds[NB];
#pragma unroll
  for (int q = 0; q < NB; ++q) ds[q] = make_float4(0.f, 0.f, 0.f, 0.f);

  constexpr int ND = DB || (!DSUM && !MB) ? 1 : NB;  // D's float4s in flight (none when D is B)
  auto load = [&](int64_t row0, float4 (&va)[NA], float4 (&vb)[NB], float4 (&vd)[ND]) {
#pragma unroll
    for (int q = 0; q < NA; ++q) {
      const int e = t + q * kTnThreads;
      const int64_t row = row0 + e / A4;
      va[q] = (e < kTnRows * A4 && row < r1)
                  ? *reinterpret_cast<const float4*>(a + row * lda + 4 * (e % A4))
                  : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      const int e = t + q * kTnThreads;
      const int64_t row = row0 + e / B4;
      const bool ok = e < kTnRows * B4 && row < r1;
      vb[q] = ok ? *reinterpret_cast<const float4*>(b + row * ldb + 4 * (e % B4))
                 : make_float4(0.f, 0.f, 0.f, 0.f);
      if constexpr ((DSUM || MB) && !DB)
        vd[q] = ok ? *reinterpret_cast<const float4*>(d + row * ldd + 4 * (e % B4))
                   : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };

  float4 va[NA], vb[NB], vd[ND];
  load(r0, va, vb, vd);
  const float* saf = reinterpret_cast<const float*>(sa);
  const float* sbf = reinterpret_cast<const float*>(sb);
  for (int64_t row0 = r0; row0 < r1; row0 += kTnRows) {
    __syncthreads();  // the previous tile's readers are done
#pragma unroll
    for (int q = 0; q < NA; ++q) {
      const int e = t + q * kTnThreads;
      if (e < kTnRows * A4) sa[(e / A4) * (PA / 4) + e % A4] = va[q];
    }
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      const int e = t + q * kTnThreads;
      if constexpr (MB) {  // after the wait for the tile: no stall on the prefetch
        const float4 h = vd[q];
        vb[q].x = h.x > 0.f ? vb[q].x * mscale : 0.f;
        vb[q].y = h.y > 0.f ? vb[q].y * mscale : 0.f;
        vb[q].z = h.z > 0.f ? vb[q].z * mscale : 0.f;
        vb[q].w = h.w > 0.f ? vb[q].w * mscale : 0.f;
      }
      if (e < kTnRows * B4) sb[(e / B4) * (PB / 4) + e % B4] = vb[q];
      if constexpr (DSUM) {
        const float4 dv = DB || MB ? vb[q] : vd[ND == 1 ? 0 : q];
        ds[q].x += dv.x;
        ds[q].y += dv.y;
        ds[q].z += dv.z;
        ds[q].w += dv.w;
      }
    }
    __syncthreads();
    if (row0 + kTnRows < r1) load(row0 + kTnRows, va, vb, vd);  // next tile in flight
    const int nsteps = static_cast<int>((min(static_cast<int64_t>(kTnRows), r1 - row0) + 15) / 16);
    for (int st = s; st < nsteps; st += S) {  // rows past r1 were staged as zeros
      const int rb = 16 * st + 8 * kh;
      bf16x8 ap[WH][3];
#pragma unroll
      for (int hi = 0; hi < WH; ++hi)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          __bf16 x0, x1, x2;
          split3(saf[(rb + j) * PA + 32 * (hb + hi) + i], x0, x1, x2);
          ap[hi][0][j] = x0;
          ap[hi][1][j] = x1;
          ap[hi][2][j] = x2;
        }
#pragma unroll
      for (int q = 0; q < WQ; ++q) {
        bf16x8 b0, b1, b2;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          __bf16 y0, y1, y2;
          split3(sbf[(rb + j) * PB + 32 * (qb + q) + i], y0, y1, y2);
          b0[j] = y0;
          b1[j] = y1;
          b2[j] = y2;
        }
#pragma unroll
        for (int hi = 0; hi < WH; ++hi) {
          const bf16x8 a0 = ap[hi][0], a1 = ap[hi][1], a2 = ap[hi][2];
          f16x c = acc[hi][q];  // smallest terms first
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b0, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b2, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, c, 0, 0, 0);
          acc[hi][q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, c, 0, 0, 0);
        }
      }
    }
  }
  float* pc = part + static_cast<int64_t>(blockIdx.x) * (M * K + (DSUM ? K : 0));
  for (int tt = S - 1; tt >= 0; --tt) {  // the S streams' partials, summed in s order
    if (s == tt) {
#pragma unroll
      for (int hi = 0; hi < WH; ++hi)
#pragma unroll
        for (int q = 0; q < WQ; ++q) {
#pragma unroll
          for (int rg = 0; rg < 16; ++rg) {
            const int m = 32 * (hb + hi) + (rg & 3) + 8 * (rg >> 2) + 4 * kh;
            const int nn = 32 * (qb + q) + i;
            float v = acc[hi][q][rg];
            if (tt < S - 1) v += red[m * K + nn];
            if (tt > 0)
              red[m * K + nn] = v;
            else
              pc[m * K + nn] = v;
          }
        }
    }
    __syncthreads();
  }
  if constexpr (DSUM) {
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      const int e = t + q * kTnThreads;
      if (e < kTnRows * B4) sb[e] = ds[q];
    }
    __syncthreads();
    if (t < B4) {
      float4 s4 = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int e = t; e < kTnRows * B4; e += B4) {
        s4.x += sb[e].x;
        s4.y += sb[e].y;
        s4.z += sb[e].z;
        s4.w += sb[e].w;
      }
      pc[M * K + 4 * t] = s4.x;
      pc[M * K + 4 * t + 1] = s4.y;
      pc[M * K + 4 * t + 2] = s4.z;
      pc[M * K + 4 * t + 3] = s4.w;
    }
  }
}

// Narrow outputs (K <= 16, M <= 128: the classifier layers' weight gradients, e.g.
// GCN_Model's last Graph_conv_layer(128, 7) dW = dS^T X, or a 1-head out_att with 7 classes),
// where a library GEMM took 1.4-2.1 ms at 1M rows. No LDS tiles: each wave walks chunks of 64
// rows; lane l holds row l's B (and D) values in registers (K scalar loads), and for each row of
// the chunk the wave reads A's row coalesced (lane = column m, MP = 1 or 2 columns per lane) and
// takes that row's K B values by v_readlane, so every product is one v_fma with a uniform
// operand. The 4 waves of a workgroup are summed in wave order through LDS (deterministic),
// the workgroup partials by gemm_tn_reduce_kernel.
constexpr int kNarrowK = 16, kNarrowM = 128;
#ifndef GNN_TN_NARROW_MFMA
#define GNN_TN_NARROW_MFMA 1  // A/B: 0 = the FMA row walk for M in {64, 128} too
#endif
constexpr int kNarrowRowsInFlight = 16;

template <bool DSUM, int MP>
__global__ __launch_bounds__(kTnThreads) void gemm_tn_narrow_kernel(
    const float* __restrict__ a, int64_t lda, const float* __restrict__ b, int64_t ldb,
    const float* __restrict__ d, int64_t ldd, int64_t n, int64_t rows_per_block, int M, int K,
    float* __restrict__ part) {
  __shared__ float red[kTnThreads / kWave][kNarrowM * kNarrowK + kNarrowK];
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x >> 6;
  constexpr int W = kTnThreads / kWave;
  const int MK = M * K;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_block;
  const int64_t r1 = min(n, r0 + rows_per_block);
  float acc[MP][kNarrowK];
#pragma unroll
  for (int p = 0; p < MP; ++p)
#pragma unroll
    for (int k = 0; k < kNarrowK; ++k) acc[p][k] = 0.f;
  float dacc[DSUM ? kNarrowK : 1];
#pragma unroll
  for (int k = 0; k < (DSUM ? kNarrowK : 1); ++k) dacc[k] = 0.f;
  for (int64_t base = r0 + static_cast<int64_t>(w) * kWave; base < r1; base += W * kWave) {
    const int64_t row = base + lane;
    const bool ok = row < r1;
    float brow[kNarrowK];
#pragma unroll
    for (int k = 0; k < kNarrowK; ++k) {
      brow[k] = (ok && k < K) ? b[row * ldb + k] : 0.f;
      if constexpr (DSUM) dacc[k] += (ok && k < K) ? d[row * ldd + k] : 0.f;
    }
    const int nr = static_cast<int>(min(static_cast<int64_t>(kWave), r1 - base));
    for (int rr = 0; rr < nr; rr += kNarrowRowsInFlight) {
      float av[kNarrowRowsInFlight][MP];
#pragma unroll
      for (int u = 0; u < kNarrowRowsInFlight; ++u)
#pragma unroll
        for (int p = 0; p < MP; ++p) {
          const int m = lane + kWave * p;
          av[u][p] = (rr + u < nr && m < M) ? a[(base + rr + u) * lda + m] : 0.f;
        }
#pragma unroll
      for (int u = 0; u < kNarrowRowsInFlight; ++u) {
        const int src = (rr + u) & (kWave - 1);  // wave-uniform
#pragma unroll
        for (int k = 0; k < kNarrowK; ++k) {
          if (k < K) {  // uniform
            const float bk =
                __int_as_float(__builtin_amdgcn_readlane(__float_as_int(brow[k]), src));
#pragma unroll
            for (int p = 0; p < MP; ++p) acc[p][k] = fmaf(av[u][p], bk, acc[p][k]);
          }
        }
      }
    }
  }
  // this wave's partial -> LDS; workgroup sum in wave order
#pragma unroll
  for (int p = 0; p < MP; ++p) {
    const int m = lane + kWave * p;
    if (m < M)
#pragma unroll
      for (int k = 0; k < kNarrowK; ++k)
        if (k < K) red[w][m * K + k] = acc[p][k];
  }
  if constexpr (DSUM) {
#pragma unroll
    for (int k = 0; k < kNarrowK; ++k) {
      float v = dacc[k];
#pragma unroll
      for (int o = 1; o < kWave; o <<= 1) v += __shfl_xor(v, o, kWave);
      if (lane == 0 && k < K) red[w][MK + k] = v;
    }
  }
  __syncthreads();
  float* pc = part + static_cast<int64_t>(blockIdx.x) * (MK + (DSUM ? K : 0));
  for (int e = threadIdx.x; e < MK + (DSUM ? K : 0); e += kTnThreads) {
    float v = red[0][e];
#pragma unroll
    for (int q = 1; q < W; ++q) v += red[q][e];
    pc[e] = v;
  }
}

// Tiny outputs (M * K <= 32: the a-vector gradients of a 1-head out_att, [del | der]^T Wh with
// M = 2): lane = row, every lane accumulates all M x K products of its rows in registers, the
// wave's lanes are summed by an xor tree and the 4 waves in order through LDS.
constexpr int kTinyOut = 32;

// The same narrow partials on the matrix cores for M in {64, 128} with 16-B aligned A rows
// (GCN_Model's classifier layer: dW = dS^T H, M = 128, K = 8): v_mfma_f32_16x16x4_f32 contracts
// 4 rows per instruction. Lane (i, q) = (l & 15, l >> 4) loads A[row0 + q][64 h + 4 i .. + 3]
// (a row's 256 B per 16 lanes) and B[row0 + q][i] (i < K); MFMA (h, c) takes component c of
// A's float4 h as its A operand, so its output rows are m = 64 h + 4 i' + c. G row groups of 4
// per wave step are loaded before their MFMAs. fp32 products, fp32 accumulation.
constexpr int kNarrowGroups = 4;
template <int M, bool DSUM>
__global__ __launch_bounds__(kTnThreads) void gemm_tn_narrow_mfma_kernel(
    const float* __restrict__ a, int64_t lda, const float* __restrict__ b, int64_t ldb,
    const float* __restrict__ d, int64_t ldd, int64_t n, int64_t rows_per_block, int K,
    float* __restrict__ part) {
  constexpr int H = M / 64, G = kNarrowGroups, W = kTnThreads / kWave;
  using fx4 = __attribute__((ext_vector_type(4))) float;
  __shared__ float red[W][M * kNarrowK + kNarrowK];
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x >> 6;
  const int i = lane & 15, q = lane >> 4;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_block;
  const int64_t r1 = min(n, r0 + rows_per_block);
  fx4 acc[H][4];
#pragma unroll
  for (int h = 0; h < H; ++h)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[h][c] = fx4{0.f, 0.f, 0.f, 0.f};
  float dacc = 0.f;
  for (int64_t base = r0 + static_cast<int64_t>(w) * (4 * G); base < r1; base += W * 4 * G) {
    float4 av[G][H];
    float bv[G];
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
      const int64_t row = base + 4 * gi + q;
      const bool ok = row < r1;
#pragma unroll
      for (int h = 0; h < H; ++h)
        av[gi][h] = ok ? *reinterpret_cast<const float4*>(a + row * lda + 64 * h + 4 * i)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
      bv[gi] = (ok && i < K) ? b[row * ldb + i] : 0.f;
      if constexpr (DSUM) dacc += (ok && i < K) ? d[row * ldd + i] : 0.f;
    }
#pragma unroll
    for (int gi = 0; gi < G; ++gi)
#pragma unroll
      for (int h = 0; h < H; ++h) {
        acc[h][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[gi][h].x, bv[gi], acc[h][0], 0, 0, 0);
        acc[h][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[gi][h].y, bv[gi], acc[h][1], 0, 0, 0);
        acc[h][2] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[gi][h].z, bv[gi], acc[h][2], 0, 0, 0);
        acc[h][3] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[gi][h].w, bv[gi], acc[h][3], 0, 0, 0);
      }
  }
  // D of MFMA (h, c): lane (j = l & 15, q) holds rows 4 q + r, i.e. m = 64 h + 4 (4 q + r) + c
  const int MK = M * K;
  if (i < K) {
#pragma unroll
    for (int h = 0; h < H; ++h)
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) red[w][(64 * h + 4 * (4 * q + r) + c) * K + i] = acc[h][c][r];
  }
  if constexpr (DSUM) {  // the 4 row lanes of column i, in lane order
    dacc += __shfl_xor(dacc, 16, kWave);
    dacc += __shfl_xor(dacc, 32, kWave);
    if (q == 0 && i < K) red[w][MK + i] = dacc;
  }
  __syncthreads();
  float* pc = part + static_cast<int64_t>(blockIdx.x) * (MK + (DSUM ? K : 0));
  for (int e = threadIdx.x; e < MK + (DSUM ? K : 0); e += kTnThreads) {
    float v = red[0][e];
#pragma unroll
    for (int ww = 1; ww < W; ++ww) v += red[ww][e];
    pc[e] = v;
  }
}

template <bool DSUM>
__global__ __launch_bounds__(kTnThreads) void gemm_tn_tiny_kernel(
    const float* __restrict__ a, int64_t lda, const float* __restrict__ b, int64_t ldb,
    const float* __restrict__ d, int64_t ldd, int64_t n, int64_t rows_per_block, int M, int K,
    float* __restrict__ part) {
  __shared__ float red[kTnThreads / kWave][kTinyOut + kNarrowK];
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x >> 6;
  const int MK = M * K;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_block;
  const int64_t r1 = min(n, r0 + rows_per_block);
  float acc[kTinyOut], dacc[DSUM ? kNarrowK : 1];
#pragma unroll
  for (int o = 0; o < kTinyOut; ++o) acc[o] = 0.f;
#pragma unroll
  for (int k = 0; k < (DSUM ? kNarrowK : 1); ++k) dacc[k] = 0.f;
  for (int64_t row = r0 + threadIdx.x; row < r1; row += kTnThreads) {
    float av[kTinyOut], bv[kNarrowK];
#pragma unroll
    for (int m = 0; m < kTinyOut; ++m) av[m] = m < M ? a[row * lda + m] : 0.f;
#pragma unroll
    for (int k = 0; k < kNarrowK; ++k) {
      bv[k] = k < K ? b[row * ldb + k] : 0.f;
      if constexpr (DSUM) dacc[k] += k < K ? d[row * ldd + k] : 0.f;
    }
#pragma unroll
    for (int o = 0; o < kTinyOut; ++o)
      if (o < MK) acc[o] = fmaf(av[o / K < kTinyOut ? o / K : 0], bv[(o % K) & (kNarrowK - 1)],
                                acc[o]);
  }
#pragma unroll
  for (int o = 0; o < kTinyOut + (DSUM ? kNarrowK : 0); ++o) {
    if (o >= kTinyOut && o - kTinyOut >= K) continue;
    if (o < kTinyOut && o >= MK) continue;
    float v = o < kTinyOut ? acc[o] : (DSUM ? dacc[(o - kTinyOut) & (kNarrowK - 1)] : 0.f);
#pragma unroll
    for (int q = 1; q < kWave; q <<= 1) v += __shfl_xor(v, q, kWave);
    if (lane == 0) red[w][o < kTinyOut ? o : MK + (o - kTinyOut)] = v;
  }
  __syncthreads();
  float* pc = part + static_cast<int64_t>(blockIdx.x) * (MK + (DSUM ? K : 0));
  for (int e = threadIdx.x; e < MK + (DSUM ? K : 0); e += kTnThreads) {
    float v = red[0][e];
#pragma unroll
    for (int q = 1; q < kTnThreads / kWave; ++q) v += red[q][e];
    pc[e] = v;
  }
}

static bool tn_narrow(int64_t m, int64_t k) {
  return m >= 1 && k >= 1 && m <= kNarrowM && k <= kNarrowK;
}

// out[e] = the sum over the blocks' partials in a fixed order (e < M*K: C, then dsum). A
// workgroup takes 64 consecutive elements; its 4 waves sum the partials g, g + 4, g + 8, ...
// (coalesced 256-B rows of the partial array, 8 loads in flight per lane) and the 4 wave sums
// are added in wave order. (One thread per element walking all 512 partials took 127 us.)
constexpr int kTnRedGroups = 4;
__global__ __launch_bounds__(256) void gemm_tn_reduce_kernel(const float* __restrict__ part,
                                                             int64_t blocks, int64_t stride,
                                                             int64_t mk, int64_t k,
                                                             float* __restrict__ c, int64_t ldc,
                                                             int trans_c,
                                                             float* __restrict__ dsum) {
  __shared__ float sred[kTnRedGroups][64];
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int64_t e = static_cast<int64_t>(blockIdx.x) * 64 + lane;
  float s = 0.f;
  if (e < stride) {
    int64_t j = g;
    for (; j + 7 * kTnRedGroups < blocks; j += 8 * kTnRedGroups) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(j + u * kTnRedGroups) * stride + e];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; j < blocks; j += kTnRedGroups) s += part[j * stride + e];
  }
  sred[g][lane] = s;
  __syncthreads();
  if (g != 0 || e >= stride) return;
  s = sred[0][lane];
#pragma unroll
  for (int q = 1; q < kTnRedGroups; ++q) s += sred[q][lane];
  if (e >= mk)
    dsum[e - mk] = s;
  else if (trans_c)
    c[(e % k) * ldc + e / k] = s;  // C^T: [k, m]
  else
    c[(e / k) * ldc + e % k] = s;
}

constexpr int64_t kTnBlocks = 512;  // 2 workgroups per CU
#ifndef GNN_TN_X6  // A/B: 0 = the f32 MFMA kernel in either arithmetic mode
#define GNN_TN_X6 1
#endif

static int64_t tn_blocks(int64_t n) {
  const int64_t by_rows = (n + 4 * kTnRows - 1) / (4 * kTnRows);  // >= 4 tiles per block
  return by_rows < kTnBlocks ? (by_rows < 1 ? 1 : by_rows) : kTnBlocks;
}

template <int M, int K>
static int launch_tn(const float* a, int64_t lda, const float* b, int64_t ldb, const float* d,
                     int64_t ldd, int64_t n, float* c, int64_t ldc, int trans_c, float* dsum,
                     float* part, hipStream_t s, const float* mask = nullptr, int64_t ldm = 0,
                     float mscale = 1.f) {
  const int64_t blocks = tn_blocks(n);
  int64_t rpb = (n + blocks - 1) / blocks;
  rpb = (rpb + kTnRows - 1) / kTnRows * kTnRows;
  const int64_t stride = M * K + (d || (mask && dsum) ? K : 0);
#ifndef GNN_TN_FMA  // A/B: the FMA kernel at every shape
  constexpr bool mfma = M >= 64 && K >= 32;
#else
  constexpr bool mfma = false;
#endif
  if constexpr (mfma) {
    if (GNN_TN_X6 != 0 && g_tf_x6 != 0) {  // the transforms' arithmetic mode (set_precision)
      const dim3 grid(static_cast<unsigned>(blocks)), blk(kTnThreads);
      if (mask)  // B' = B . [mask > 0] * mscale (gnn_gemm_tn_masked_f32)
        if (dsum)
          hipLaunchKernelGGL((gemm_tn_x6_kernel<M, K, true, false, true>), grid, blk, 0, s, a,
                             lda, b, ldb, mask, ldm, n, rpb, part, mscale);
        else
          hipLaunchKernelGGL((gemm_tn_x6_kernel<M, K, false, false, true>), grid, blk, 0, s, a,
                             lda, b, ldb, mask, ldm, n, rpb, part, mscale);
      else if (d && d == b && ldd == ldb)  // dsum of B itself: B's loads serve both
        hipLaunchKernelGGL((gemm_tn_x6_kernel<M, K, true, true>), grid, blk, 0, s, a, lda, b, ldb,
                           d, ldd, n, rpb, part, 1.f);
      else if (d)
        hipLaunchKernelGGL((gemm_tn_x6_kernel<M, K, true>), grid, blk, 0, s, a, lda, b, ldb, d,
                           ldd, n, rpb, part, 1.f);
      else
        hipLaunchKernelGGL((gemm_tn_x6_kernel<M, K, false>), grid, blk, 0, s, a, lda, b, ldb, d,
                           ldd, n, rpb, part, 1.f);
    } else if (d) {
      hipLaunchKernelGGL((gemm_tn_mfma_kernel<M, K, true>), dim3(static_cast<unsigned>(blocks)),
                         dim3(kTnThreads), 0, s, a, lda, b, ldb, d, ldd, n, rpb, part);
    } else {
      hipLaunchKernelGGL((gemm_tn_mfma_kernel<M, K, false>), dim3(static_cast<unsigned>(blocks)),
                         dim3(kTnThreads), 0, s, a, lda, b, ldb, d, ldd, n, rpb, part);
    }
  } else if (d) {
    hipLaunchKernelGGL((gemm_tn_partial_kernel<M, K, true>), dim3(static_cast<unsigned>(blocks)),
                       dim3(kTnThreads), 0, s, a, lda, b, ldb, d, ldd, n, rpb, part);
  } else {
    hipLaunchKernelGGL((gemm_tn_partial_kernel<M, K, false>), dim3(static_cast<unsigned>(blocks)),
                       dim3(kTnThreads), 0, s, a, lda, b, ldb, d, ldd, n, rpb, part);
  }
  hipLaunchKernelGGL(gemm_tn_reduce_kernel, dim3(static_cast<unsigned>((stride + 63) / 64)),
                     dim3(256), 0, s, part, blocks, stride, static_cast<int64_t>(M * K),
                     static_cast<int64_t>(K), c, ldc, trans_c, dsum);
  return launch_status();
}

}  // namespace gnn

using namespace gnn;

static bool tn_wide(int64_t m, int64_t k) {
  return (m == 128 && k == 128) || (m == 64 && k == 64) || (m == 128 && k == 64) ||
         (m == 64 && k == 128) || (m == 8 && k == 64) || (m == 16 && k == 64);
}

// 1: a wide shape (16-B aligned rows, strides multiples of 4 floats); 2: a narrow one (K <= 16,
// M <= 128; any row stride, 4-B aligned); 0: not covered
extern "C" int gnn_gemm_tn_supported(int64_t m, int64_t k) {
  return tn_wide(m, k) ? 1 : (tn_narrow(m, k) ? 2 : 0);
}

// the narrow / tiny kernels are latency-bound row walks: 4x the workgroups (32 waves per CU)
static int64_t tn_blocks_for(int64_t n, int64_t m, int64_t k) {
  if (tn_wide(m, k)) return tn_blocks(n);
  const int64_t by_rows = (n + 2 * kTnRows - 1) / (2 * kTnRows);
  return by_rows < 4 * kTnBlocks ? (by_rows < 1 ? 1 : by_rows) : 4 * kTnBlocks;
}

extern "C" int64_t gnn_gemm_tn_workspace_bytes(int64_t n, int64_t m, int64_t k) {
  if (n < 0 || m < 1 || k < 1) return GNN_E_ARG;
  return tn_blocks_for(n, m, k) * (m * k + k) * static_cast<int64_t>(sizeof(float));
}

// C[m, k] = A^T B = sum_i A[i, :]^T B[i, :] (A [n, m], B [n, k], row strides lda / ldb), stored
// as C (trans_c = 0, row stride ldc >= k) or as C^T [k, m] (trans_c = 1, ldc >= m); when
// d != NULL also dsum[k] = sum_i D[i, :] (D [n, k]). fp32, deterministic. Shapes: (m, k) in
// gnn_gemm_tn_supported; rows 16-B aligned (row strides multiples of 4 floats).
extern "C" int gnn_gemm_tn_f32(const float* a, int64_t lda, const float* b, int64_t ldb, int64_t n,
                               int64_t m, int64_t k, float* c, int64_t ldc, int32_t trans_c,
                               const float* d, int64_t ldd, float* dsum, void* workspace,
                               int64_t workspace_bytes, void* stream) {
  if (n < 0 || !a || !b || !c || !workspace || lda < m || ldb < k) return GNN_E_ARG;
  if (trans_c ? ldc < m : ldc < k) return GNN_E_ARG;
  if (d && (!dsum || ldd < k)) return GNN_E_ARG;
  if (!gnn_gemm_tn_supported(m, k)) return GNN_E_UNSUPPORTED;
  if (workspace_bytes < gnn_gemm_tn_workspace_bytes(n, m, k)) return GNN_E_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  float* part = static_cast<float*>(workspace);
  const int tc = trans_c ? 1 : 0;
  if (!tn_wide(m, k)) {  // narrow: any row stride
    if (!aligned_to(a, 4) || !aligned_to(b, 4) || (d && !aligned_to(d, 4))) return GNN_E_ALIGN;
    const int64_t blocks = tn_blocks_for(n, m, k);
    int64_t rpb = (n + blocks - 1) / blocks;
    rpb = (rpb + kTnRows - 1) / kTnRows * kTnRows;
    const int M = static_cast<int>(m), K = static_cast<int>(k);
    const dim3 grid(static_cast<unsigned>(blocks)), blk(kTnThreads);
    if (m * k <= kTinyOut) {
      if (d)
        hipLaunchKernelGGL((gemm_tn_tiny_kernel<true>), grid, blk, 0, s, a, lda, b, ldb, d, ldd,
                           n, rpb, M, K, part);
      else
        hipLaunchKernelGGL((gemm_tn_tiny_kernel<false>), grid, blk, 0, s, a, lda, b, ldb, d, ldd,
                           n, rpb, M, K, part);
    } else if (GNN_TN_NARROW_MFMA && (m == 64 || m == 128) && aligned_to(a, 16) && lda % 4 == 0) {
      if (m == 128 && d)
        hipLaunchKernelGGL((gemm_tn_narrow_mfma_kernel<128, true>), grid, blk, 0, s, a, lda, b,
                           ldb, d, ldd, n, rpb, K, part);
      else if (m == 128)
        hipLaunchKernelGGL((gemm_tn_narrow_mfma_kernel<128, false>), grid, blk, 0, s, a, lda, b,
                           ldb, d, ldd, n, rpb, K, part);
      else if (d)
        hipLaunchKernelGGL((gemm_tn_narrow_mfma_kernel<64, true>), grid, blk, 0, s, a, lda, b,
                           ldb, d, ldd, n, rpb, K, part);
      else
        hipLaunchKernelGGL((gemm_tn_narrow_mfma_kernel<64, false>), grid, blk, 0, s, a, lda, b,
                           ldb, d, ldd, n, rpb, K, part);
    } else if (m > kWave) {
      if (d)
        hipLaunchKernelGGL((gemm_tn_narrow_kernel<true, 2>), grid, blk, 0, s, a, lda, b, ldb, d,
                           ldd, n, rpb, M, K, part);
      else
        hipLaunchKernelGGL((gemm_tn_narrow_kernel<false, 2>), grid, blk, 0, s, a, lda, b, ldb, d,
                           ldd, n, rpb, M, K, part);
    } else {
      if (d)
        hipLaunchKernelGGL((gemm_tn_narrow_kernel<true, 1>), grid, blk, 0, s, a, lda, b, ldb, d,
                           ldd, n, rpb, M, K, part);
      else
        hipLaunchKernelGGL((gemm_tn_narrow_kernel<false, 1>), grid, blk, 0, s, a, lda, b, ldb, d,
                           ldd, n, rpb, M, K, part);
    }
    const int64_t stride = m * k + (d ? k : 0);
    hipLaunchKernelGGL(gemm_tn_reduce_kernel, dim3(static_cast<unsigned>((stride + 63) / 64)),
                       dim3(256), 0, s, part, blocks, stride, m * k, k, c, ldc, tc, dsum);
    return launch_status();
  }
  if (!aligned_to(a, 16) || !aligned_to(b, 16) || (d && !aligned_to(d, 16)) || lda % 4 ||
      ldb % 4 || (d && ldd % 4))
    return GNN_E_ALIGN;
  if (m == 128 && k == 128)
    return launch_tn<128, 128>(a, lda, b, ldb, d, ldd, n, c, ldc, tc, dsum, part, s);
  if (m == 64 && k == 64)
    return launch_tn<64, 64>(a, lda, b, ldb, d, ldd, n, c, ldc, tc, dsum, part, s);
  if (m == 128 && k == 64)
    return launch_tn<128, 64>(a, lda, b, ldb, d, ldd, n, c, ldc, tc, dsum, part, s);
  if (m == 64 && k == 128)
    return launch_tn<64, 128>(a, lda, b, ldb, d, ldd, n, c, ldc, tc, dsum, part, s);
  if (m == 16 && k == 64)  // [del | der] against Wh: both GAT a-vector gradients in one pass
    return launch_tn<16, 64>(a, lda, b, ldb, d, ldd, n, c, ldc, tc, dsum, part, s);
  return launch_tn<8, 64>(a, lda, b, ldb, d, ldd, n, c, ldc, tc, dsum, part, s);
}

// C = A^T B' with B' = B . [H > 0] * scale elementwise (H [n, k], row stride ldh), and dsum = the
// column sums of B' when dsum != NULL: dW and db of a GCN layer whose ReLU and Dropout ran in its
// transform's store epilogue (gnn_gcn_transform_epi_f32), H being that output -- the gradient
// passes exactly where H > 0, scaled by 1 / (1 - p). Wide shapes with m, k >= 64 in the
// split-bf16 arithmetic only (gnn_gemm_tn_masked_supported); the workspace as gnn_gemm_tn_f32's.
extern "C" int gnn_gemm_tn_masked_supported(int64_t m, int64_t k) {
  return GNN_TN_X6 != 0 && g_tf_x6 != 0 && tn_wide(m, k) && m >= 64 && k >= 64;
}

extern "C" int gnn_gemm_tn_masked_f32(const float* a, int64_t lda, const float* b, int64_t ldb,
                                      const float* h, int64_t ldh, float scale, int64_t n,
                                      int64_t m, int64_t k, float* c, int64_t ldc, int32_t trans_c,
                                      float* dsum, void* workspace, int64_t workspace_bytes,
                                      void* stream) {
  if (n < 0 || !a || !b || !h || !c || !workspace || lda < m || ldb < k || ldh < k)
    return GNN_E_ARG;
  if (trans_c ? ldc < m : ldc < k) return GNN_E_ARG;
  if (!gnn_gemm_tn_masked_supported(m, k)) return GNN_E_UNSUPPORTED;
  if (workspace_bytes < gnn_gemm_tn_workspace_bytes(n, m, k)) return GNN_E_ARG;
  if (!aligned_to(a, 16) || !aligned_to(b, 16) || !aligned_to(h, 16) || lda % 4 || ldb % 4 ||
      ldh % 4)
    return GNN_E_ALIGN;
  hipStream_t s = static_cast<hipStream_t>(stream);
  float* part = static_cast<float*>(workspace);
  const int tc = trans_c ? 1 : 0;
  if (m == 128 && k == 128)
    return launch_tn<128, 128>(a, lda, b, ldb, nullptr, 0, n, c, ldc, tc, dsum, part, s, h, ldh,
                               scale);
  if (m == 64 && k == 64)
    return launch_tn<64, 64>(a, lda, b, ldb, nullptr, 0, n, c, ldc, tc, dsum, part, s, h, ldh,
                             scale);
  if (m == 128 && k == 64)
    return launch_tn<128, 64>(a, lda, b, ldb, nullptr, 0, n, c, ldc, tc, dsum, part, s, h, ldh,
                              scale);
  return launch_tn<64, 128>(a, lda, b, ldb, nullptr, 0, n, c, ldc, tc, dsum, part, s, h, ldh,
                            scale);
}
