// transform.hip -- the GCN feature transform on the matrix cores: Y = X W^T (fp32).
//
// Replaces `support = self.dense(X_input)` (nn.Linear, no bias) at GCN/GCN.py:42, the
// dense half of Graph_conv_layer.forward (with the layer's bias, and GCN_Model's ReLU and
// Dropout, in the store epilogue -- gnn_gcn_transform_epi_f32 -- when training runs the layer
// as (A X) W^T + b); with the ReLU epilogue (gnn_linear_relu_f32) the SageLayer's
// relu(weight(cat[self, agg])) at GraphSAGE/GraphSAGE.py:18-20.
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
#include <type_traits>

#include "common.hpp"

extern "C" int gnn_gcn_transform_supported(int64_t k, int64_t fout);

namespace gnn {

constexpr int kTfWaves = 4;

struct RowIdx {  // the optional output-row scatter (gcn_transform_kernel y_row)
  const int64_t* row;
  int64_t n_y;
  int32_t* err;
  // optional device row count: rows [0, min(*live, n_rows)) are computed (a sampled batch's
  // frontier size, never read back to the host; n_rows is then the buffer's capacity)
  const int64_t* live = nullptr;
};
// the optional classifier epilogue (gnn_linear_relu_cls_f32): logits = y wd^T + bd
constexpr int kMaxCls = 4;
struct Classifier {
  const float* wd;  // [n_cls, FO] (nn.Linear weight)
  const float* bd;  // [n_cls] or null
  float* logits;    // [n_rows, ldl]
  int64_t ldl;
  int n_cls;
};
// the optional store epilogue of the plain mode: y = dropout(act(x w^T + bias)) -- a GCN layer
// trained as (A X) W^T + b with GCN_Model's ReLU and Dropout after it (gnn_gcn_transform_epi_f32)
struct TfEpi {
  const float* bias = nullptr;  // [fout] or null
  float drop_p = 0.f;           // element (row, col) kept iff dropout_keep(seed, row, col0 + col, p)
  float drop_scale = 1.f;       // 1 / (1 - p)
  uint64_t seed = 0;
  int col0 = 0;                 // column offset of this launch (the two-launch 256 split)
  TfEpi shifted(int c) const {
    TfEpi e = *this;
    if (e.bias) e.bias += c;
    e.col0 += c;
    return e;
  }
};
// kernel epilogue modes
constexpr int kTfPlain = 0, kTfScatter = 1, kTfClassify = 2;
using tf32x4 = __attribute__((ext_vector_type(4))) float;
// split3 / swz6 / x6_pitch (fp32 products from bf16 MFMAs): common.hpp

#ifndef GNN_TF_SINGLE_BUFFER
#define GNN_TF_SINGLE_BUFFER 0  // A/B: the round-2 one-buffer tile loop (two barriers per tile)
#endif
#ifndef GNN_TF_X6_PIPE
#define GNN_TF_X6_PIPE 0  // A/B: X6 fragments of k-step s + 1 read during step s's MFMAs
#endif
#ifndef GNN_TF_K256_CB2
#define GNN_TF_K256_CB2 0  // A/B: K = 256 -> 128 as 4 waves x 2 column blocks
#endif
#ifndef GNN_TF_ONE256
#define GNN_TF_ONE256 1  // 0 = A/B: 256 output columns at K >= 128 as two 128-column launches
#endif
#ifndef GNN_TF_PREFETCH
#define GNN_TF_PREFETCH 1  // X tiles in flight in registers ahead of the one being multiplied
#endif

// NW waves per workgroup, each owning CB 16-column blocks of W (FO = NW * CB * 16); a tile is
// TR rows of X (TR = 16, 32 or 64: small launches use short tiles so that every CU gets work).
// K = 256 (the SageLayer's cat[self, agg]) runs 8 waves x 1 block: its 64 W values per lane
// stay resident, the X fragment is read from LDS in chunks of XC k-steps, and the tile's
// 16-row blocks run as independent MFMA chains (one chain of 64 dependent MFMAs per wave
// would leave the matrix core waiting on its own results).
// Tiles are double-buffered in LDS (TileLds layout: no bank conflicts on the fragment
// reads): tile g+1 is loaded into registers during tile g's MFMAs and written to the other
// buffer before tile g's epilogue, so one barrier per tile separates the two.
// y_row (optional): X row i goes to output row y_row[i] -- the support written in another
// row order (a degree-ordered graph's, graph.degree_order) while X is read in order; ids
// outside [0, n_y) are not stored and raise *err. The stores are scattered 64-B row pieces
// (fire and forget); a gather on the X side would put the index load in front of every tile.
// MODE kTfClassify (the GraphSAGE classifier fused into the last SageLayer's GEMM,
// GraphSAGE.py:51-52): each lane dots its 4 * CB output columns of a row with the classifier
// weights, the 4 lane quarters are summed by shuffles and the NW waves' partials through LDS
// (fixed order, deterministic), + bias: logits[row, c] for c < n_cls <= 4.
template <int K, int CB, int NW, bool RELU, int TR, int MODE, bool X6 = false>
__global__ __launch_bounds__(NW * kWave) void gcn_transform_kernel(
    const float* __restrict__ x, int64_t ldx, int64_t n_rows, const float* __restrict__ w,
    float* __restrict__ y, int64_t ldy, const int64_t* __restrict__ y_row, int64_t n_y,
    int32_t* __restrict__ err, Classifier cls, const int64_t* __restrict__ live,
    TfEpi epi) {
  if (live != nullptr) {  // uniform: every wave reads the same count
    const int64_t l = *live;
    n_rows = l < n_rows ? (l > 0 ? l : 0) : n_rows;
  }
  constexpr bool SCATTER = MODE == kTfScatter;
  constexpr bool CLS = MODE == kTfClassify;
  constexpr int kTfBlock = NW * kWave;
  constexpr int S = K / 4;           // MFMA k-steps
  constexpr int XC = S <= 32 ? S : 16;  // k-steps of X held in registers at a time
  constexpr int RB0 = CB == 1 && S > 32 ? 4 : 1;
  constexpr int RB = RB0 < TR / 16 ? RB0 : TR / 16;  // 16-row blocks computed together
  constexpr int LDA = 4 * TileLds<K>::L4;  // LDS row pitch (floats)
  constexpr int V4 = TR * K / 4;       // float4s per tile
  constexpr int NV = (V4 + kTfBlock - 1) / kTfBlock;  // per thread
  constexpr int NBUF = GNN_TF_SINGLE_BUFFER ? 1 : 2;
  static_assert(S % XC == 0 && XC % 4 == 0, "X chunks of whole float4s");
  constexpr int S32 = K / 32;  // X6: bf16 MFMA k-steps (32 k each, 8 per lane quarter)
  constexpr int P6 = x6_pitch<K>();
  constexpr int PLANE = TR * P6;  // bytes per bf16 plane
  static_assert(!X6 || (K >= 64 && K % 64 == 0), "X6 tiles: K in {64, 128, 256}");
  __shared__ float xt[NBUF][X6 ? 3 * PLANE / 4 : TR * LDA];
  __shared__ float part[CLS ? 2 : 1][CLS ? NW * TR * kMaxCls : 1];  // per-wave logit partials
  const int lane = threadIdx.x & (kWave - 1);
  const int wv = threadIdx.x >> 6;
  const int q = lane >> 4, r = lane & 15;
  float wd[CLS ? CB : 1][4][kMaxCls];  // classifier weights of this lane's output columns
  if constexpr (CLS) {
#pragma unroll
    for (int cb = 0; cb < CB; ++cb)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int c = 0; c < kMaxCls; ++c)
          wd[cb][i][c] = c < cls.n_cls ? cls.wd[c * (NW * CB * 16) + (wv * CB + cb) * 16 + 4 * q + i]
                                       : 0.f;
  }

  // A fragments: W[c0 + r][q*S + s] for this wave's CB column blocks, resident
  float wa[X6 ? 1 : CB][X6 ? 1 : S];
  // X6: the bf16 pieces of W[c0 + r][q*K/4 + 8s + j] (j < 8) for k-step s, resident
  bf16x8 wb[X6 ? CB : 1][X6 ? S32 : 1][3];
#pragma unroll
  for (int cb = 0; cb < CB; ++cb) {
    const float* wr = w + static_cast<int64_t>((wv * CB + cb) * 16 + r) * K + q * S;
#pragma unroll
    for (int v = 0; v < S / 4; ++v) {
      const float4 t = *reinterpret_cast<const float4*>(wr + 4 * v);
      if constexpr (X6) {
        const float tv[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          __bf16 a, b, c;
          split3(tv[i], a, b, c);
          wb[cb][v / 2][0][(v & 1) * 4 + i] = a;
          wb[cb][v / 2][1][(v & 1) * 4 + i] = b;
          wb[cb][v / 2][2][(v & 1) * 4 + i] = c;
        }
      } else {
        wa[cb][4 * v] = t.x;
        wa[cb][4 * v + 1] = t.y;
        wa[cb][4 * v + 2] = t.z;
        wa[cb][4 * v + 3] = t.w;
      }
    }
  }

  const int64_t n_tiles = (n_rows + TR - 1) / TR;
  // PF tiles in flight in registers: tile it + PF is requested while tile it is multiplied
  // (slot it % PF; the loop is unrolled by PF so every slot index is a constant)
  constexpr int PF = GNN_TF_PREFETCH;
  static_assert(PF >= 1 && PF <= 4 && (PF == 1 || NBUF == 2), "prefetch depth 1..4");
  float4 pre[PF][NV];
  // Tile loads through a buffer descriptor of the tile's rows: the hardware range check
  // returns 0 for rows past the end (and for a tile past the last), so the loads need no
  // per-lane branch. Under such a branch the compiler cannot count the outstanding loads at
  // the join and waits for all of them (s_waitcnt vmcnt(0)), which exposed the next tile's
  // whole load latency instead of hiding it under this tile's MFMAs.
  auto fetch = [&](float4 (&p)[NV], int64_t g) {
    const int64_t r0 = g * TR;
    const int64_t live = g < n_tiles ? (n_rows - r0 < TR ? n_rows - r0 : TR) : 0;
    const float* base = x + (live > 0 ? r0 : 0) * ldx;
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(base), 0, static_cast<int>(live * ldx * 4), 0x00020000);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int e = v * kTfBlock + static_cast<int>(threadIdx.x);
      const int rr = e / (K / 4), c4 = e - rr * (K / 4);
      const int off = e < V4 ? (rr * static_cast<int>(ldx) + 4 * c4) * 4 : 0x7ffffff0;
      p[v] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0));
    }
  };
  constexpr bool kFullTile = NV * kTfBlock == V4;  // every thread stages NV float4s
  auto stage = [&](float* buf, const float4 (&p)[NV]) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int e = v * kTfBlock + static_cast<int>(threadIdx.x);
      if (kFullTile || e < V4) {
        const int rr = e / (K / 4), c4 = e - rr * (K / 4);
        if constexpr (X6) {  // 4 floats -> 4 bf16 of each plane (8 B), chunk c4 / 2 swizzled
          const float tv[4] = {p[v].x, p[v].y, p[v].z, p[v].w};
          bf16x4 p0, p1, p2;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            __bf16 a, b, c;
            split3(tv[i], a, b, c);
            p0[i] = a;
            p1[i] = b;
            p2[i] = c;
          }
          char* base = reinterpret_cast<char*>(buf) + rr * P6 +
                       16 * ((c4 >> 1) ^ swz6<K>(rr)) + 8 * (c4 & 1);
          *reinterpret_cast<bf16x4*>(base) = p0;
          *reinterpret_cast<bf16x4*>(base + PLANE) = p1;
          *reinterpret_cast<bf16x4*>(base + 2 * PLANE) = p2;
        } else {
          *reinterpret_cast<float4*>(buf + rr * LDA + 4 * (c4 ^ TileLds<K>::swz(rr))) = p[v];
        }
      }
    }
  };
  fetch(pre[0], blockIdx.x);
  if (NBUF == 2) {
    stage(xt[0], pre[0]);
    __syncthreads();
  }
#pragma unroll
  for (int f = 1; f < PF; ++f) fetch(pre[f], blockIdx.x + static_cast<int64_t>(f) * gridDim.x);
  int it = 0;
  auto body = [&](auto slot, int64_t g) {  // one tile; uniform over the block
    constexpr int SL = decltype(slot)::value;  // this tile's register slot (already staged)
    constexpr int SN = (SL + 1) % PF;          // the next tile's
    const float* cur = xt[NBUF == 2 ? (it & 1) : 0];
    if (NBUF == 1) {
      stage(xt[0], pre[0]);
      __syncthreads();
    }
    const int64_t row0 = g * TR;
    // output rows of this lane's rows, requested first: the epilogue's wait for them then does
    // not also wait for the prefetch issued after them (the counter retires in order)
    int64_t dst[TR / 16];
#pragma unroll
    for (int j = 0; j < TR / 16; ++j) {
      const int64_t orow = row0 + j * 16 + r;
      dst[j] = orow;
      if constexpr (SCATTER) dst[j] = y_row[orow < n_rows ? orow : n_rows - 1];
    }
    // tile it + PF into the slot this tile left, in flight during the next PF tiles' MFMAs
    fetch(pre[SL], g + static_cast<int64_t>(PF) * gridDim.x);
    // keep the loads here: left to itself the scheduler sinks them to their use in stage(),
    // after the MFMAs, and the tile waits for its own prefetch
    __builtin_amdgcn_sched_barrier(0);
    tf32x4 acc[TR / 16][CB];
    if constexpr (X6) {
#pragma unroll
      for (int j = 0; j < TR / 16; ++j) {
#pragma unroll
        for (int cb = 0; cb < CB; ++cb) acc[j][cb] = tf32x4{0.f, 0.f, 0.f, 0.f};
        const int rr = j * 16 + r;
        const char* xr = reinterpret_cast<const char*>(cur) + rr * P6;
#if GNN_TF_X6_PIPE
        // the next k-step's three fragments are read while this step's MFMAs run
        bf16x8 fr[2][3];
        auto rd = [&](int s6, bf16x8 (&f)[3]) {
          const char* xp = xr + 16 * ((q * S32 + s6) ^ swz6<K>(rr));
          f[0] = *reinterpret_cast<const bf16x8*>(xp);
          f[1] = *reinterpret_cast<const bf16x8*>(xp + PLANE);
          f[2] = *reinterpret_cast<const bf16x8*>(xp + 2 * PLANE);
        };
        rd(0, fr[0]);
#endif
#pragma unroll
        for (int s6 = 0; s6 < S32; ++s6) {
#if GNN_TF_X6_PIPE
          if (s6 + 1 < S32) rd(s6 + 1, fr[(s6 + 1) & 1]);
          const bf16x8 x0 = fr[s6 & 1][0], x1 = fr[s6 & 1][1], x2 = fr[s6 & 1][2];
#else
          const char* xp = xr + 16 * ((q * S32 + s6) ^ swz6<K>(rr));
          const bf16x8 x0 = *reinterpret_cast<const bf16x8*>(xp);
          const bf16x8 x1 = *reinterpret_cast<const bf16x8*>(xp + PLANE);
          const bf16x8 x2 = *reinterpret_cast<const bf16x8*>(xp + 2 * PLANE);
#endif
#pragma unroll
          for (int cb = 0; cb < CB; ++cb) {  // smallest terms first
            tf32x4 a = acc[j][cb];
            a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[cb][s6][0], x2, a, 0, 0, 0);
            a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[cb][s6][1], x1, a, 0, 0, 0);
            a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[cb][s6][2], x0, a, 0, 0, 0);
            a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[cb][s6][0], x1, a, 0, 0, 0);
            a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[cb][s6][1], x0, a, 0, 0, 0);
            acc[j][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[cb][s6][0], x0, a, 0, 0, 0);
          }
        }
      }
    } else
#pragma unroll
    for (int rb0 = 0; rb0 < TR / 16; rb0 += RB) {
#pragma unroll
      for (int j = 0; j < RB; ++j)
#pragma unroll
        for (int cb = 0; cb < CB; ++cb) acc[rb0 + j][cb] = tf32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c0 = 0; c0 < S; c0 += XC) {
        float xb[RB][XC];
#pragma unroll
        for (int j = 0; j < RB; ++j) {
          const int rr = (rb0 + j) * 16 + r;
          const float* xr = cur + rr * LDA;
#pragma unroll
          for (int v = 0; v < XC / 4; ++v) {
            const int c4 = (q * S + c0) / 4 + v;
            const float4 t =
                *reinterpret_cast<const float4*>(xr + 4 * (c4 ^ TileLds<K>::swz(rr)));
            xb[j][4 * v] = t.x;
            xb[j][4 * v + 1] = t.y;
            xb[j][4 * v + 2] = t.z;
            xb[j][4 * v + 3] = t.w;
          }
        }
#pragma unroll
        for (int s = 0; s < XC; ++s) {
#pragma unroll
          for (int j = 0; j < RB; ++j)
#pragma unroll
            for (int cb = 0; cb < CB; ++cb)
              acc[rb0 + j][cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[cb][c0 + s], xb[j][s],
                                                                      acc[rb0 + j][cb], 0, 0, 0);
        }
      }
    }
    // the next tile goes to the other buffer while the last MFMAs drain (nobody reads it:
    // the barrier that ended the previous tile saw every wave's reads of it complete)
    __builtin_amdgcn_sched_barrier(0);  // ... and the staging (which waits for them) after the MFMAs
    if (NBUF == 2) stage(xt[(it + 1) & 1], pre[SN]);
#pragma unroll
    for (int j = 0; j < TR / 16; ++j) {
      // acc[j][cb][i] = Y[row0 + 16 j + r][(wv*CB + cb)*16 + 4q + i]
      const int64_t orow = dst[j];
      const bool ok = !SCATTER || (orow >= 0 && orow < n_y);
      if (SCATTER && !ok && row0 + j * 16 + r < n_rows && q == 0 && wv == 0) atomicOr(err, 1);
      if (row0 + j * 16 + r < n_rows && ok) {
#pragma unroll
        for (int cb = 0; cb < CB; ++cb) {
          float4 o = make_float4(acc[j][cb][0], acc[j][cb][1], acc[j][cb][2], acc[j][cb][3]);
          const int col = (wv * CB + cb) * 16 + 4 * q;
          if (epi.bias != nullptr) {  // uniform: the layer's bias (gnn_gcn_transform_epi_f32)
            const float4 bv = *reinterpret_cast<const float4*>(epi.bias + col);
            o.x += bv.x;
            o.y += bv.y;
            o.z += bv.z;
            o.w += bv.w;
          }
          if constexpr (RELU) {
            o.x = fmaxf(o.x, 0.f);
            o.y = fmaxf(o.y, 0.f);
            o.z = fmaxf(o.z, 0.f);
            o.w = fmaxf(o.w, 0.f);
          }
          if (epi.drop_p > 0.f) {  // uniform: inverted dropout, one hash per element
            const int c = epi.col0 + col;
            o.x = dropout_keep(epi.seed, orow, c, epi.drop_p) ? o.x * epi.drop_scale : 0.f;
            o.y = dropout_keep(epi.seed, orow, c + 1, epi.drop_p) ? o.y * epi.drop_scale : 0.f;
            o.z = dropout_keep(epi.seed, orow, c + 2, epi.drop_p) ? o.z * epi.drop_scale : 0.f;
            o.w = dropout_keep(epi.seed, orow, c + 3, epi.drop_p) ? o.w * epi.drop_scale : 0.f;
          }
          *reinterpret_cast<float4*>(y + orow * ldy + (wv * CB + cb) * 16 + 4 * q) = o;
        }
      }
      if constexpr (CLS) {  // every lane, rows past n_rows included (their sums go unused)
        float pc[kMaxCls];
#pragma unroll
        for (int c = 0; c < kMaxCls; ++c) pc[c] = 0.f;
#pragma unroll
        for (int cb = 0; cb < CB; ++cb)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float v = RELU ? fmaxf(acc[j][cb][i], 0.f) : acc[j][cb][i];
#pragma unroll
            for (int c = 0; c < kMaxCls; ++c) pc[c] = fmaf(v, wd[cb][i][c], pc[c]);
          }
#pragma unroll
        for (int c = 0; c < kMaxCls; ++c) {
          pc[c] += __shfl_xor(pc[c], 16, kWave);
          pc[c] += __shfl_xor(pc[c], 32, kWave);
        }
        if (q == 0) {
#pragma unroll
          for (int c = 0; c < kMaxCls; ++c)
            part[it & 1][(wv * TR + j * 16 + r) * kMaxCls + c] = pc[c];
        }
      }
    }
    __syncthreads();  // one barrier per tile: the staged next tile is complete, this one free
    if constexpr (CLS) {
      // the waves' partials of this tile, summed in wave order (the buffer of parity it & 1 is
      // written again two tiles on, after the next tile's barrier)
      const int t = static_cast<int>(threadIdx.x);
      if (t < TR * kMaxCls) {
        const int rr = t / kMaxCls, c = t - rr * kMaxCls;
        if (c < cls.n_cls && row0 + rr < n_rows) {
          float v = 0.f;
#pragma unroll
          for (int wq = 0; wq < NW; ++wq) v += part[it & 1][(wq * TR + rr) * kMaxCls + c];
          if (cls.bd) v += cls.bd[c];
          cls.logits[(row0 + rr) * cls.ldl + c] = v;
        }
      }
    }
  };
  for (int64_t g = blockIdx.x; g < n_tiles;) {  // unrolled by PF: constant slot indices
    body(std::integral_constant<int, 0>{}, g);
    g += gridDim.x;
    ++it;
    if constexpr (PF > 1) {
      if (g >= n_tiles) break;
      body(std::integral_constant<int, 1 % PF>{}, g);
      g += gridDim.x;
      ++it;
    }
    if constexpr (PF > 2) {
      if (g >= n_tiles) break;
      body(std::integral_constant<int, 2 % PF>{}, g);
      g += gridDim.x;
      ++it;
    }
    if constexpr (PF > 3) {
      if (g >= n_tiles) break;
      body(std::integral_constant<int, 3 % PF>{}, g);
      g += gridDim.x;
      ++it;
    }
  }
}

// transform precision (gnn_transform_set_precision): 1 = fp32 products from bf16 MFMAs (X6,
// K >= 128), 0 = v_mfma_f32_16x16x4_f32 (a k-ordered fp32 fmaf chain)
int g_tf_x6 = 1;

template <int K, int CB, int NW, bool RELU, int TR, bool X6>
static void launch_transform_kernel(dim3 grid, const float* x, int64_t ldx, int64_t n_rows,
                                    const float* w, float* y, int64_t ldy, const RowIdx& ri,
                                    const Classifier& cls, const TfEpi& epi, hipStream_t s) {
  if (ri.row != nullptr)  // a template flag: no index loads in the in-order kernel
    hipLaunchKernelGGL((gcn_transform_kernel<K, CB, NW, RELU, TR, kTfScatter, X6>), grid,
                       dim3(NW * kWave), 0, s, x, ldx, n_rows, w, y, ldy, ri.row, ri.n_y, ri.err,
                       cls, ri.live, epi);
  else if (RELU && cls.logits != nullptr)  // the classifier epilogue: SageLayer GEMMs only
    hipLaunchKernelGGL((gcn_transform_kernel<K, CB, NW, RELU, TR, RELU ? kTfClassify : kTfPlain,
                                             X6>),
                       grid, dim3(NW * kWave), 0, s, x, ldx, n_rows, w, y, ldy, ri.row, ri.n_y,
                       ri.err, cls, ri.live, epi);
  else
    hipLaunchKernelGGL((gcn_transform_kernel<K, CB, NW, RELU, TR, kTfPlain, X6>), grid,
                       dim3(NW * kWave), 0, s, x, ldx, n_rows, w, y, ldy, ri.row, ri.n_y, ri.err,
                       cls, ri.live, epi);
}

template <int K, int CB, int NW, bool RELU, int TR>
static int launch_transform_tr(const float* x, int64_t ldx, int64_t n_rows, const float* w,
                               float* y, int64_t ldy, const RowIdx& ri, const Classifier& cls,
                               const TfEpi& epi, hipStream_t s) {
  const int64_t tiles = (n_rows + TR - 1) / TR;
#ifndef GNN_TF_GRID
#define GNN_TF_GRID 512  // persistent grid: 2 workgroups per CU
#endif
  constexpr int64_t kGrid = GNN_TF_GRID * kTfWaves / NW;  // 8-wave workgroups: 1 per CU
  const int64_t grid = tiles < kGrid ? tiles : kGrid;
  const dim3 g(static_cast<unsigned>(grid));
  // X6 tiles: 3 bf16 planes, at most 32 rows; 2 blocks of K = 256 pieces (192 VGPRs) spill
  if constexpr (K >= 128 && TR <= 32 && !(K == 256 && CB == 2)) {
    if (g_tf_x6) {
      launch_transform_kernel<K, CB, NW, RELU, TR, true>(g, x, ldx, n_rows, w, y, ldy, ri, cls, epi, s);
      return launch_status();
    }
  }
  launch_transform_kernel<K, CB, NW, RELU, TR, false>(g, x, ldx, n_rows, w, y, ldy, ri, cls, epi, s);
  return launch_status();
}

#ifndef GNN_TF_MIN_TR
#define GNN_TF_MIN_TR 16  // A/B: 64 = always the round-2 64-row tiles
#endif
#ifndef GNN_TF_TR64_MAX_K
#define GNN_TF_TR64_MAX_K 64  // K above this: at most 32-row tiles
#endif
// Tile rows: 16 or 32 when 64-row tiles would leave CUs without a tile (< 2 tiles per
// resident workgroup slot): the fixed cost of a small launch is its first tile. K >= 128 runs
// 32-row tiles at every size: in one process (tools/transform_tile_ab.py,
// profiles/r03m_transform_tile_ab2.log) 32 vs 64 rows: K = 256 -> 128 at 62,479 / 200K / 1M
// rows 40.7 / 111.8 / 524 vs 44.3 / 124.5 / 559 us, K = 128 -> 128 at 1M / 10M rows 299 /
// 2891 vs 307 / 2932 us; K = 64 -> 64 keeps 64 rows (95 vs 113 us at 1M).
template <int K, int CB, int NW, bool RELU>
static int launch_transform(const float* x, int64_t ldx, int64_t n_rows, const float* w,
                            float* y, int64_t ldy, const RowIdx& ri, const Classifier& cls, const TfEpi& epi, hipStream_t s) {
  constexpr int64_t slots = GNN_TF_GRID * kTfWaves / NW;
#ifdef GNN_TF_TR32_ROWS  // A/B: 16-row tiles below GNN_TF_TR16_ROWS, 32-row below this
#ifndef GNN_TF_TR16_ROWS
#define GNN_TF_TR16_ROWS (32 * 2 * slots)
#endif
  if (n_rows < GNN_TF_TR16_ROWS) return launch_transform_tr<K, CB, NW, RELU, 16>(x, ldx, n_rows, w, y, ldy, ri, cls, epi, s);
  if (n_rows < GNN_TF_TR32_ROWS) return launch_transform_tr<K, CB, NW, RELU, 32>(x, ldx, n_rows, w, y, ldy, ri, cls, epi, s);
#endif
  // X6 at K = 256: 16-row tiles at every size (in one process, tools/transform_x6_ab.py,
  // profiles/r03x_transform_x6_ab.log: 62K / 200K x 256 -> 128 30.9 / 79.9 vs 32.9 / 89.7 us
  // with 32-row tiles; K = 128 keeps 32: 1M x 128 -> 128 205 vs 211 us)
  if (GNN_TF_MIN_TR <= 16 &&
      (n_rows < 32 * 2 * slots || (K == 256 && g_tf_x6 && !(CB == 2 && K == 256))))
    return launch_transform_tr<K, CB, NW, RELU, 16>(x, ldx, n_rows, w, y, ldy, ri, cls, epi, s);
  if (GNN_TF_MIN_TR <= 32 && (K > GNN_TF_TR64_MAX_K || n_rows < 64 * 2 * slots))
    return launch_transform_tr<K, CB, NW, RELU, 32>(x, ldx, n_rows, w, y, ldy, ri, cls, epi, s);
  if constexpr (K <= GNN_TF_TR64_MAX_K || GNN_TF_MIN_TR > 32)
    return launch_transform_tr<K, CB, NW, RELU, 64>(x, ldx, n_rows, w, y, ldy, ri, cls, epi, s);
  return launch_transform_tr<K, CB, NW, RELU, 32>(x, ldx, n_rows, w, y, ldy, ri, cls, epi, s);
}

template <int K, bool RELU>
static int dispatch_transform(int64_t fout, const float* x, int64_t ldx, int64_t n_rows,
                              const float* w, float* y, int64_t ldy, const RowIdx& ri,
                              const Classifier& cls, const TfEpi& epi, hipStream_t s) {
  if (fout == 64) return launch_transform<K, 1, kTfWaves, RELU>(x, ldx, n_rows, w, y, ldy, ri, cls, epi, s);
  if (fout == 128) {
    if constexpr (K <= 128 || GNN_TF_K256_CB2)
      return launch_transform<K, 2, kTfWaves, RELU>(x, ldx, n_rows, w, y, ldy, ri, cls, epi, s);
    else
      return launch_transform<K, 1, 8, RELU>(x, ldx, n_rows, w, y, ldy, ri, cls, epi, s);
  }
  if (fout == 256) {
    if constexpr (K <= 64) {
      return launch_transform<K, 4, kTfWaves, RELU>(x, ldx, n_rows, w, y, ldy, ri, cls, epi, s);
    } else if (K == 256 && g_tf_x6 && cls.logits == nullptr) {
      // X6 at K = 256: the 2-block tile does not fit the registers, so two launches of the
      // 1-block kernel, one per half of W's rows (X read twice; memory-bound either way)
      const int rc = dispatch_transform<K, RELU>(128, x, ldx, n_rows, w, y, ldy, ri, cls, epi, s);
      if (rc != GNN_OK) return rc;
      return dispatch_transform<K, RELU>(128, x, ldx, n_rows, w + 128 * K, y + 128, ldy, ri, cls,
                                        epi.shifted(128), s);
    } else if constexpr (GNN_TF_ONE256) {
      // one launch, 8 waves x 2 column blocks (128 W values per lane resident, 200 VGPRs):
      // X read and staged once for all 256 columns. In one process (tools/transform_tile_ab.py,
      // profiles/r03o_transform_one256_ab.log): 10M x 256 -> 256 9.63 ms (136 TF/s) vs 10.57
      // as two launches vs 9.95 hipBLASLt; 1M x 128 -> 256 0.545 vs 0.618 vs 0.628 ms
      return launch_transform<K, 2, 8, RELU>(x, ldx, n_rows, w, y, ldy, ri, cls, epi, s);
    } else {
      // A/B: two launches of the 128-column kernel, one per half of W's rows (X read twice)
      if (cls.logits != nullptr) return GNN_E_UNSUPPORTED;
      const int rc = dispatch_transform<K, RELU>(128, x, ldx, n_rows, w, y, ldy, ri, cls, epi, s);
      if (rc != GNN_OK) return rc;
      return dispatch_transform<K, RELU>(128, x, ldx, n_rows, w + 128 * K, y + 128, ldy, ri, cls,
                                        epi.shifted(128), s);
    }
  }
  return GNN_E_UNSUPPORTED;
}

template <bool RELU>
static int transform_entry(const float* x, int64_t ldx, int64_t n_rows, int64_t k,
                           const float* w, int64_t fout, float* y, int64_t ldy,
                           void* stream, const RowIdx& ri = RowIdx{nullptr, 0, nullptr},
                           const Classifier& cls = Classifier{nullptr, nullptr, nullptr, 0, 0},
                           const TfEpi& epi = TfEpi{}) {
  if (n_rows < 0 || ldx < k || ldy < fout) return GNN_E_ARG;
  if (ri.row != nullptr && (ri.err == nullptr || ri.n_y < 0)) return GNN_E_ARG;
  if (!gnn_gcn_transform_supported(k, fout)) return GNN_E_UNSUPPORTED;
  if (n_rows == 0) return GNN_OK;
  if (!x || !w || !y) return GNN_E_ARG;
  if (ldx % 4 || ldy % 4 || !aligned_to(x, 16) || !aligned_to(y, 16) || !aligned_to(w, 16))
    return GNN_E_ALIGN;
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (k) {
    case 16: return dispatch_transform<16, RELU>(fout, x, ldx, n_rows, w, y, ldy, ri, cls, epi, s);
    case 32: return dispatch_transform<32, RELU>(fout, x, ldx, n_rows, w, y, ldy, ri, cls, epi, s);
    case 64: return dispatch_transform<64, RELU>(fout, x, ldx, n_rows, w, y, ldy, ri, cls, epi, s);
    case 128: return dispatch_transform<128, RELU>(fout, x, ldx, n_rows, w, y, ldy, ri, cls, epi, s);
    default: return dispatch_transform<256, RELU>(fout, x, ldx, n_rows, w, y, ldy, ri, cls, epi, s);
  }
}

}  // namespace gnn

using namespace gnn;

extern "C" int gnn_transform_set_precision(int mode) {
  if (mode != 0 && mode != 1) return GNN_E_ARG;
  const int prev = g_tf_x6;
  g_tf_x6 = mode;
  return prev;
}

extern "C" int gnn_transform_get_precision(void) { return g_tf_x6; }

extern "C" int gnn_gcn_transform_supported(int64_t k, int64_t fout) {
  const bool kk = k == 16 || k == 32 || k == 64 || k == 128 || k == 256;
  if (!kk) return 0;
  return fout == 64 || fout == 128 || fout == 256;
}

extern "C" int gnn_gcn_transform_f32(const float* x, int64_t ldx, int64_t n_rows, int64_t k,
                                     const float* w, int64_t fout, float* y, int64_t ldy,
                                     void* stream) {
  return transform_entry<false>(x, ldx, n_rows, k, w, fout, y, ldy, stream);
}

// y = dropout(act(x w^T + bias)) (bias [fout] 16-B aligned or null; act = ReLU if relu;
// element (i, c) kept iff dropout_keep(seed, i, c, drop_p), kept values scaled by 1/(1 - p)):
// the transform of a GCN layer trained as (A X) W^T + b with GCN_Model's ReLU and Dropout in
// its store epilogue (graphneuralnetwork_amd/ops.py _GcnLayerFn)
extern "C" int gnn_gcn_transform_epi_f32(const float* x, int64_t ldx, int64_t n_rows, int64_t k,
                                         const float* w, int64_t fout, const float* bias,
                                         int32_t relu, float drop_p, uint64_t drop_seed, float* y,
                                         int64_t ldy, void* stream) {
  if (!(drop_p >= 0.f && drop_p < 1.f)) return GNN_E_ARG;
  if (bias && !aligned_to(bias, 16)) return GNN_E_ALIGN;
  TfEpi epi;
  epi.bias = bias;
  epi.drop_p = drop_p;
  epi.drop_scale = 1.f / (1.f - drop_p);
  epi.seed = drop_seed;
  const RowIdx ri{nullptr, 0, nullptr};
  const Classifier cls{nullptr, nullptr, nullptr, 0, 0};
  return relu ? transform_entry<true>(x, ldx, n_rows, k, w, fout, y, ldy, stream, ri, cls, epi)
              : transform_entry<false>(x, ldx, n_rows, k, w, fout, y, ldy, stream, ri, cls, epi);
}

extern "C" int gnn_gcn_transform_rows_f32(const float* x, int64_t ldx, int64_t n_rows,
                                          int64_t k, const float* w, int64_t fout, float* y,
                                          int64_t ldy, const int64_t* y_row, int64_t n_y,
                                          int32_t* err_flag, void* stream) {
  if (n_rows > 0 && !y_row) return GNN_E_ARG;
  if (n_rows > 0 && n_y == 0) return GNN_E_ARG;  // every id would be out of range
  return transform_entry<false>(x, ldx, n_rows, k, w, fout, y, ldy, stream,
                                RowIdx{y_row, n_y, err_flag});
}

extern "C" int gnn_linear_relu_f32(const float* x, int64_t ldx, int64_t n_rows, int64_t k,
                                   const float* w, int64_t fout, float* y, int64_t ldy,
                                   void* stream) {
  return transform_entry<true>(x, ldx, n_rows, k, w, fout, y, ldy, stream);
}

extern "C" int gnn_linear_relu_live_f32(const float* x, int64_t ldx, int64_t n_rows,
                                        const int64_t* live, int64_t k, const float* w,
                                        int64_t fout, float* y, int64_t ldy, void* stream) {
  if (n_rows > 0 && !live) return GNN_E_ARG;
  RowIdx ri{nullptr, 0, nullptr};
  ri.live = live;
  return transform_entry<true>(x, ldx, n_rows, k, w, fout, y, ldy, stream, ri);
}

extern "C" int gnn_linear_relu_cls_f32(const float* x, int64_t ldx, int64_t n_rows, int64_t k,
                                       const float* w, int64_t fout, float* y, int64_t ldy,
                                       const float* wd, const float* bd, int64_t n_cls,
                                       float* logits, int64_t ldl, void* stream) {
  if (n_cls < 1 || n_cls > kMaxCls || ldl < n_cls) return GNN_E_ARG;
  if (n_rows > 0 && (!wd || !logits)) return GNN_E_ARG;
  return transform_entry<true>(x, ldx, n_rows, k, w, fout, y, ldy, stream,
                               RowIdx{nullptr, 0, nullptr},
                               Classifier{wd, bd, logits, ldl, static_cast<int>(n_cls)});
}
