// project.hip -- GAT feature transform on the matrix cores, attention logits fused.
//
// Replaces, for the inference path of every attention layer,
//   Wh = torch.mm(h, W)                        GAT/models/layers.py:23 / :97 (all heads at
//                                              once: W = [W_1 | ... | W_H], GAT.py:16)
//   el = a[:F].Wh_i,  er = a[F:].Wh_j          layers.py:25-26 / :105-108
// with ONE pass over h: each wave computes a 16-row x 16*NT-column tile of Wh with
// v_mfma_f32_16x16x4_f32 (exact f32 in / f32 accumulate; gfx950 has no xf32), W held
// in registers for the whole launch, Wh stored straight from the accumulator layout
// (16 lanes = 64 contiguous bytes of a row). The logits ride along as one more
// 16-column MFMA tile: [el | er] = X (W A) with A the block-diagonal [fout, 2 heads]
// matrix of a_src / a_dst, folded into W once per workgroup (W2 = W A in LDS, computed by
// the workgroup itself: no separate launch).
//
// MFMA operand maps (16x16x4 f32): lane l holds A[l & 15][k = l >> 4] and
// B[k = l >> 4][l & 15]; C/D: col = l & 15, row = 4 * (l >> 4) + reg. The kernel
// computes the transposed tile D = W^T X^T (A = W^T, B = X^T) so that a lane's four
// accumulators are four consecutive columns of one Wh row (16-B stores). The K axis is
// permuted so that lane quarter q owns k in [q*S, q*S + S): its X values for all S
// steps are one contiguous run of h's row, read as float4s from an LDS copy of the
// wave's 16 rows that was loaded with fully coalesced 16-B-per-lane global loads.
#include "common.hpp"

namespace gnn {

constexpr int kProjWaves = 4;
constexpr int kProjBlock = kProjWaves * kWave;
#ifndef GNN_PROJ_G
#define GNN_PROJ_G 1  // 16-row blocks per wave per iteration (independent MFMA chains x G)
#endif
constexpr int kProjG = GNN_PROJ_G;
using f32x4 = __attribute__((ext_vector_type(4))) float;

// w2[k][c] = W[k, head c] . a_src[head c] (c < heads), W[k, head c-heads] . a_dst[head
// c-heads] (heads <= c < 2 heads), 0 beyond: the logits as a [K, 16] weight tile.
// (w and a read from the workgroup's LDS copies: wl = W [K, fout], al = [a_src | a_dst])
__device__ __forceinline__ float logit_weight(const float* wl, int kk, int fout, const float* al,
                                              int heads, int fh, int c) {
  float v = 0.f;
  if (c < 2 * heads) {
    const int h = c < heads ? c : c - heads;
    const float* av = al + (c < heads ? 0 : fout) + h * fh;
    const float* wr = wl + kk * fout + h * fh;
    for (int f = 0; f < fh; ++f) v = fmaf(wr[f], av[f], v);
  }
  return v;
}

// The A tile's LDS image (row pitch and xor swizzle per K): TileLds in common.hpp.
template <int K> using ProjLds = TileLds<K>;

// Each wave stages and reads only its own A tile, so the tile hand-off needs the wave's LDS
// stores to land before its reads (and its reads before the next tile's stores), not a
// workgroup barrier: the four waves then drift apart and one's global loads overlap
// another's MFMAs. GNN_PROJ_BLOCK_SYNC=1 restores the round-2 __syncthreads (A/B).
#ifndef GNN_PROJ_BLOCK_SYNC
#define GNN_PROJ_BLOCK_SYNC 0
#endif
#ifndef GNN_PROJ_DEPTH
#define GNN_PROJ_DEPTH 1  // A tiles in flight per wave (A/B: 2 and 3 slower, profiles/r03e_proj_ab2.log)
#endif
__device__ __forceinline__ void proj_tile_sync() {
#if GNN_PROJ_BLOCK_SYNC
  __syncthreads();
#else
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#endif
}

// X6 (K = 64; the kernel takes 64 and 128): the products from bf16 MFMAs with three-piece fp32 splits (common.hpp
// split3): W and the logit tile split once into registers, each wave's X tile split while it
// is staged into three bf16 LDS planes, six v_mfma_f32_16x16x32_bf16 per 32-long k-step.
template <int K, int NT, bool COLROW, bool X6 = false>
__global__ __launch_bounds__(kProjBlock) void gat_project_kernel(
    const float* __restrict__ x, int64_t ldx, int64_t n_rows, const float* __restrict__ w,
    const float* __restrict__ a_src, const float* __restrict__ a_dst, int fh, int heads,
    float* __restrict__ wh, int64_t ldwh,
    float* __restrict__ el, float* __restrict__ er, int64_t lde,
    const int64_t* __restrict__ col_row) {
  constexpr int S = K / 4;   // MFMA k-steps
  constexpr int FO = 16 * NT;
  constexpr int LDA = 4 * ProjLds<K>::L4;  // LDS row (floats), see ProjLds
  constexpr int G = kProjG;
  constexpr int S32 = K / 32;
  constexpr int P6 = x6_pitch<K>();
  constexpr int PLANE = 16 * G * P6;  // bytes per bf16 plane of a wave's tile
  static_assert(!X6 || K == 64 || K == 128, "X6 projection: K in {64, 128}");
  __shared__ float atile[kProjWaves][X6 ? 3 * PLANE / 4 : 16 * G * LDA];
  const int lane = threadIdx.x & (kWave - 1);
  const int q = lane >> 4, r = lane & 15;
  const bool vec_logits = heads % 4 == 0 && lde % 4 == 0 &&
                          ((reinterpret_cast<uintptr_t>(el) | reinterpret_cast<uintptr_t>(er)) & 15) == 0;

  // Logit weights as one more 16-column tile (w2 = W A, folded here per workgroup):
  // [el | er] = X w2 comes out of the same MFMA k-loop as Wh = X W.
  // W and a are copied to LDS first (independent loads, one round trip), the fold reads them
  // there (a loop of dependent global loads per entry would stall every workgroup's start)
  __shared__ float w2s[K * 16];
  __shared__ float wl[K * FO];
  __shared__ float al[2 * FO];
  for (int e = threadIdx.x; e < K * FO; e += kProjBlock) wl[e] = w[e];
  for (int e = threadIdx.x; e < 2 * FO; e += kProjBlock) al[e] = e < FO ? a_src[e] : a_dst[e - FO];
  __syncthreads();
  for (int e = threadIdx.x; e < K * 16; e += kProjBlock)
    w2s[e] = logit_weight(wl, e >> 4, FO, al, heads, fh, e & 15);
  __syncthreads();
#ifdef GNN_PROJ_B_LDS
  // B fragments read from LDS at every step (fewer VGPRs, more waves per SIMD)
  __shared__ float ws[K * FO];
  for (int e = threadIdx.x; e < K * FO; e += kProjBlock) ws[e] = w[e];
  __syncthreads();
#else
  float b[X6 ? 1 : NT][X6 ? 1 : S];  // B fragments: W[q*S + s][16t + r], resident
  float b2[X6 ? 1 : S];
  bf16x8 bx[X6 ? NT + 1 : 1][X6 ? S32 : 1][3];  // X6: pieces of W[q*S + 8 s6 + j][16t + r]
  if constexpr (X6) {
#pragma unroll
    for (int t = 0; t <= NT; ++t)  // t == NT: the logit tile w2
#pragma unroll
      for (int s6 = 0; s6 < S32; ++s6)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int k = q * S + 8 * s6 + j;
          const float v = t < NT ? wl[k * FO + 16 * t + r] : w2s[k * 16 + r];
          __bf16 p0, p1, p2;
          split3(v, p0, p1, p2);
          bx[t][s6][0][j] = p0;
          bx[t][s6][1][j] = p1;
          bx[t][s6][2][j] = p2;
        }
  } else {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int s = 0; s < S; ++s) b[t][s] = wl[(q * S + s) * FO + 16 * t + r];
  }
  __syncthreads();
  if constexpr (!X6) {
#pragma unroll
    for (int s = 0; s < S; ++s) b2[s] = w2s[(q * S + s) * 16 + r];
  }
#endif

  // A tiles are staged through LDS: a coalesced 16-B-per-lane copy of the wave's 16 rows,
  // then each lane reads its row's quarter (row l & 15, k in [q*S, q*S + S)) as float4s
  float* at = atile[threadIdx.x >> 6];
  const int64_t n_groups = (n_rows + 16 * G * kProjWaves - 1) / (16 * G * kProjWaves);
  constexpr int V4 = 16 * G * K / 4;              // float4s in the wave's tile
  constexpr int NV = (V4 + kWave - 1) / kWave;    // per lane
  // DEPTH tiles in flight per wave (registers): a tile's loads are issued DEPTH groups
  // before its MFMAs, so the HBM latency (several microseconds under load) is covered by
  // DEPTH tiles of MFMA work, not one
  constexpr int DEPTH = K >= 128 ? 1 : GNN_PROJ_DEPTH;  // K >= 128: 64+ VGPRs per tile
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  float4 pre[DEPTH][NV];
  // COLROW: the column-order ids of a tile's output rows travel with its X loads (requested a
  // tile ahead, like them): a plain load of them after the MFMAs is where the compiler would
  // put it, and its wait would also wait for the refill issued before -- the next tile's whole
  // latency, once per tile
  int64_t cidx[DEPTH][G];
  auto fetch_ids = [&](int64_t (&dst)[G], int64_t g) {
    if constexpr (COLROW) {
      const int64_t r0 = (g * kProjWaves + wave) * 16 * G;
      const int64_t live =
          (g < n_groups && r0 < n_rows) ? (n_rows - r0 < 16 * G ? n_rows - r0 : 16 * G) : 0;
      const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<int64_t*>(col_row + (live > 0 ? r0 : 0)), 0, static_cast<int>(live * 8),
          0x00020000);
#pragma unroll
      for (int j = 0; j < G; ++j)
        dst[j] = __builtin_bit_cast(int64_t,
                                    __builtin_amdgcn_raw_buffer_load_b64(rsrc, (16 * j + r) * 8, 0, 0));
    }
  };
  // The wave's tile rows through a buffer descriptor: the range check returns 0 past the last
  // row, so the loads carry no per-lane branch (under one, the compiler cannot count them and
  // waits for all outstanding loads -- the prefetch -- before the MFMAs; transform.hip).
  auto fetch = [&](float4 (&dst)[NV], int64_t g) {
    const int64_t r0 = (g * kProjWaves + wave) * 16 * G;
    const int64_t live =
        (g < n_groups && r0 < n_rows) ? (n_rows - r0 < 16 * G ? n_rows - r0 : 16 * G) : 0;
    const float* base = x + (live > 0 ? r0 : 0) * ldx;
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(base), 0, static_cast<int>(live * ldx * 4), 0x00020000);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int e = v * kWave + lane;
      const int rr = e / (K / 4), c4 = e - rr * (K / 4);
      const int off = e < V4 ? (rr * static_cast<int>(ldx) + 4 * c4) * 4 : 0x7ffffff0;
      dst[v] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0));
    }
  };
  constexpr bool kFullTile = NV * kWave == V4;
  auto tile = [&](int64_t g, float4 (&src)[NV], int64_t (&ids)[G]) {
    const int64_t row0 = (g * kProjWaves + (threadIdx.x >> 6)) * 16 * G;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int e = v * kWave + lane;
      if (kFullTile || e < V4) {
        const int rr = e / (K / 4), c4 = e - rr * (K / 4);
        if constexpr (X6) {
          const float tv[4] = {src[v].x, src[v].y, src[v].z, src[v].w};
          bf16x4 p0, p1, p2;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            __bf16 u0, u1, u2;
            split3(tv[i], u0, u1, u2);
            p0[i] = u0;
            p1[i] = u1;
            p2[i] = u2;
          }
          char* base = reinterpret_cast<char*>(at) + rr * P6 + 16 * ((c4 >> 1) ^ swz6<K>(rr)) +
                       8 * (c4 & 1);
          *reinterpret_cast<bf16x4*>(base) = p0;
          *reinterpret_cast<bf16x4*>(base + PLANE) = p1;
          *reinterpret_cast<bf16x4*>(base + 2 * PLANE) = p2;
        } else {
          *reinterpret_cast<float4*>(at + rr * LDA + 4 * (c4 ^ ProjLds<K>::swz(rr))) = src[v];
        }
      }
    }
    proj_tile_sync();
    int64_t crow_pre[G];
#pragma unroll
    for (int j = 0; j < G; ++j) crow_pre[j] = COLROW ? ids[j] : row0 + 16 * j + r;
    fetch(src, g + DEPTH * static_cast<int64_t>(gridDim.x));  // refill this slot
    fetch_ids(ids, g + DEPTH * static_cast<int64_t>(gridDim.x));
    __builtin_amdgcn_sched_barrier(0);  // issued here, not sunk to the next tile's staging
    float a[X6 ? 1 : G][X6 ? 1 : S];
    if constexpr (!X6)
#pragma unroll
    for (int j = 0; j < G; ++j)
#pragma unroll
      for (int v = 0; v < S / 4; ++v) {
        const int rr = j * 16 + r;
        const float4 t4 = *reinterpret_cast<const float4*>(
            at + rr * LDA + 4 * ((q * (S / 4) + v) ^ ProjLds<K>::swz(rr)));
        a[j][4 * v] = t4.x;
        a[j][4 * v + 1] = t4.y;
        a[j][4 * v + 2] = t4.z;
        a[j][4 * v + 3] = t4.w;
      }
    f32x4 acc[G][NT], acc2[G];
#pragma unroll
    for (int j = 0; j < G; ++j) {
      acc2[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[j][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if constexpr (X6) {
#pragma unroll
      for (int j = 0; j < G; ++j) {
        const int rr = j * 16 + r;
#pragma unroll
        for (int s6 = 0; s6 < S32; ++s6) {
          const char* xp = reinterpret_cast<const char*>(at) + rr * P6 +
                           16 * ((q * S32 + s6) ^ swz6<K>(rr));
          const bf16x8 x0 = *reinterpret_cast<const bf16x8*>(xp);
          const bf16x8 x1 = *reinterpret_cast<const bf16x8*>(xp + PLANE);
          const bf16x8 x2 = *reinterpret_cast<const bf16x8*>(xp + 2 * PLANE);
#pragma unroll
          for (int t = 0; t <= NT; ++t) {  // smallest terms first; t == NT: the logit tile
            f32x4 c = t < NT ? acc[j][t] : acc2[j];
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bx[t][s6][0], x2, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bx[t][s6][1], x1, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bx[t][s6][2], x0, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bx[t][s6][0], x1, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bx[t][s6][1], x0, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bx[t][s6][0], x0, c, 0, 0, 0);
            if (t < NT)
              acc[j][t] = c;
            else
              acc2[j] = c;
          }
        }
      }
    } else {
#pragma unroll
    for (int s = 0; s < S; ++s) {
#pragma unroll
      for (int j = 0; j < G; ++j) {
#ifdef GNN_PROJ_B_LDS
#pragma unroll
        for (int t = 0; t < NT; ++t)
          acc[j][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(ws[(q * S + s) * FO + 16 * t + r],
                                                           a[j][s], acc[j][t], 0, 0, 0);
        acc2[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(w2s[(q * S + s) * 16 + r], a[j][s],
                                                       acc2[j], 0, 0, 0);
#else
#pragma unroll
        for (int t = 0; t < NT; ++t)
          acc[j][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[t][s], a[j][s], acc[j][t], 0, 0, 0);
        acc2[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(b2[s], a[j][s], acc2[j], 0, 0, 0);
#endif
      }
    }
    }
    // Operands are swapped (D = W^T X^T), so acc[j][t][i] is Wh[row0 + 16j + r][16t + 4q + i]:
    // one 16-B store per tile, 4 lanes = 64 contiguous bytes of a row; acc2[j][i] is column
    // 4q + i of [el | er] for row 16j + r
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const int64_t orow = row0 + 16 * j + r;
      // col_row: Wh and er are the column side of the aggregation -- rows in the column
      // order of a degree-ordered graph; el (the row side) stays in place (a template flag:
      // the index load and range check cost 10 % of the in-order launch when compiled in,
      // profiles/r03i_proj_colrow_ab.log). Resolved outside the row guard below, so the
      // compiler keeps the index load where it was issued, ahead of the MFMAs.
      int64_t crow = orow;
      bool cok = true;
      if constexpr (COLROW) {
        crow = crow_pre[j];
        cok = crow >= 0 && crow < n_rows;  // an id out of range is not stored
        crow = cok ? crow : 0;
      }
      if (orow < n_rows) {
#pragma unroll
        for (int t = 0; t < NT; ++t)
          if (cok)
            *reinterpret_cast<float4*>(wh + crow * ldwh + 16 * t + 4 * q) =
                make_float4(acc[j][t][0], acc[j][t][1], acc[j][t][2], acc[j][t][3]);
        if (vec_logits) {  // heads % 4 == 0: quarter q holds 4 whole logits of el or er
          const int c = 4 * q;
          if (c < 2 * heads && (c < heads || cok))
            *reinterpret_cast<float4*>(c < heads ? el + orow * lde + c
                                                 : er + crow * lde + c - heads) =
                make_float4(acc2[j][0], acc2[j][1], acc2[j][2], acc2[j][3]);
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int c = 4 * q + i;
            if (c < heads)
              el[orow * lde + c] = acc2[j][i];
            else if (c < 2 * heads && cok)
              er[crow * lde + c - heads] = acc2[j][i];
          }
        }
      }
    }
    proj_tile_sync();  // the next group overwrites the A tile
  };
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) {
    fetch(pre[d], blockIdx.x + d * static_cast<int64_t>(gridDim.x));
    fetch_ids(cidx[d], blockIdx.x + d * static_cast<int64_t>(gridDim.x));
  }
  for (int64_t g = blockIdx.x; g < n_groups; g += DEPTH * static_cast<int64_t>(gridDim.x)) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {  // uniform over the block
      const int64_t gg = g + d * static_cast<int64_t>(gridDim.x);
      if (gg < n_groups) tile(gg, pre[d], cidx[d]);
    }
  }
}

template <int K, int NT>
static int launch_project(const float* x, int64_t ldx, int64_t n_rows, const float* w,
                          const float* a_src, const float* a_dst, int fh, int heads, float* wh,
                          int64_t ldwh, float* el, float* er, int64_t lde,
                          const int64_t* col_row, hipStream_t s) {
  const int64_t groups = (n_rows + 16 * kProjG * kProjWaves - 1) / (16 * kProjG * kProjWaves);
#ifndef GNN_PROJ_GRID
// 512 = the resident workgroups at 2 waves/SIMD (144 VGPRs): A/B at cfg3 with isolated
// variant libraries (tools/project_ab.py, profiles/r02zl_project_ab.log) 0.135 ms vs 0.139-0.147
// at 1024; G = 2 row blocks per wave (10 MFMA chains) 0.152-0.157, W from LDS 0.153-0.156
#define GNN_PROJ_GRID 512
#endif
  const int64_t grid = groups < GNN_PROJ_GRID ? groups : GNN_PROJ_GRID;  // W resident across groups
  const dim3 g(static_cast<unsigned>(grid));
  // X6 at K = 64 only: in one process (tools/transform_prec_ab.py,
  // profiles/r03z_transform_prec_ab.log) 1M x 64 -> 8 x 8 112.5 vs 130.4 us in order, 145.5 vs
  // 142.0 with the rows scattered by a random permutation; 1M x 128 -> 4 x 8 138.6 vs 139.2
  if constexpr (K == 64) {
    if (g_tf_x6) {  // the transforms' arithmetic (gnn_transform_set_precision)
      if (col_row != nullptr)
        hipLaunchKernelGGL((gat_project_kernel<K, NT, true, true>), g, dim3(kProjBlock), 0, s, x,
                           ldx, n_rows, w, a_src, a_dst, fh, heads, wh, ldwh, el, er, lde, col_row);
      else
        hipLaunchKernelGGL((gat_project_kernel<K, NT, false, true>), g, dim3(kProjBlock), 0, s, x,
                           ldx, n_rows, w, a_src, a_dst, fh, heads, wh, ldwh, el, er, lde, col_row);
      return launch_status();
    }
  }
  if (col_row != nullptr)
    hipLaunchKernelGGL((gat_project_kernel<K, NT, true>), g, dim3(kProjBlock), 0, s, x, ldx,
                       n_rows, w, a_src, a_dst, fh, heads, wh, ldwh, el, er, lde, col_row);
  else
    hipLaunchKernelGGL((gat_project_kernel<K, NT, false>), g, dim3(kProjBlock), 0, s, x, ldx,
                       n_rows, w, a_src, a_dst, fh, heads, wh, ldwh, el, er, lde, col_row);
  return launch_status();
}

template <int K>
static int dispatch_project_nt(int64_t fout, const float* x, int64_t ldx, int64_t n_rows,
                               const float* w, const float* a_src, const float* a_dst, int fh,
                               int heads, float* wh,
                               int64_t ldwh, float* el, float* er, int64_t lde,
                               const int64_t* col_row, hipStream_t s) {
  // B fragments live in registers: (K / 4) * NT <= 64
  if (fout == 16) return launch_project<K, 1>(x, ldx, n_rows, w, a_src, a_dst, fh, heads, wh, ldwh, el, er, lde, col_row, s);
  if constexpr (K <= 128)
    if (fout == 32) return launch_project<K, 2>(x, ldx, n_rows, w, a_src, a_dst, fh, heads, wh, ldwh, el, er, lde, col_row, s);
  if constexpr (K <= 64)
    if (fout == 64) return launch_project<K, 4>(x, ldx, n_rows, w, a_src, a_dst, fh, heads, wh, ldwh, el, er, lde, col_row, s);
  return GNN_E_UNSUPPORTED;
}

}  // namespace gnn

using namespace gnn;

extern "C" int gnn_gat_project_supported(int64_t k, int64_t fout, int64_t fh) {
  const bool kk = k == 16 || k == 32 || k == 64 || k == 128 || k == 256;
  if (!kk || fh < 1 || fout % fh || fout / fh > 8) return 0;  // [el | er] fits one tile
  if (fout == 16) return 1;
  if (fout == 32) return k <= 128;
  if (fout == 64) return k <= 64;
  return 0;
}

static int project_entry(const float* x, int64_t ldx, int64_t n_rows, int64_t k,
                         const float* w, int64_t fout, const float* a_src, const float* a_dst,
                         int64_t heads, int64_t fh, float* wh, int64_t ldwh, float* el,
                         float* er, int64_t lde, const int64_t* col_row, float* w2_scratch,
                         void* stream) {
  if (n_rows < 0 || heads < 1 || fh < 1 || heads * fh != fout || ldx < k || ldwh < fout ||
      lde < heads)
    return GNN_E_ARG;
  if (!gnn_gat_project_supported(k, fout, fh)) return GNN_E_UNSUPPORTED;
  if (n_rows == 0) return GNN_OK;
  if (!x || !w || !a_src || !a_dst || !wh || !el || !er) return GNN_E_ARG;
  if (ldx % 4 || ldwh % 4 || !aligned_to(x, 16) || !aligned_to(wh, 16)) return GNN_E_ALIGN;
  (void)w2_scratch;  // the logit weights are folded inside the kernel (kept for the ABI)
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int h = static_cast<int>(heads);
  const int f = static_cast<int>(fh);
  switch (k) {
    case 16: return dispatch_project_nt<16>(fout, x, ldx, n_rows, w, a_src, a_dst, f, h, wh, ldwh, el, er, lde, col_row, s);
    case 32: return dispatch_project_nt<32>(fout, x, ldx, n_rows, w, a_src, a_dst, f, h, wh, ldwh, el, er, lde, col_row, s);
    case 64: return dispatch_project_nt<64>(fout, x, ldx, n_rows, w, a_src, a_dst, f, h, wh, ldwh, el, er, lde, col_row, s);
    case 128: return dispatch_project_nt<128>(fout, x, ldx, n_rows, w, a_src, a_dst, f, h, wh, ldwh, el, er, lde, col_row, s);
    default: return dispatch_project_nt<256>(fout, x, ldx, n_rows, w, a_src, a_dst, f, h, wh, ldwh, el, er, lde, col_row, s);
  }
}

extern "C" int gnn_gat_project_f32(const float* x, int64_t ldx, int64_t n_rows, int64_t k,
                                   const float* w, int64_t fout, const float* a_src,
                                   const float* a_dst, int64_t heads, int64_t fh, float* wh,
                                   int64_t ldwh, float* el, float* er, int64_t lde,
                                   float* w2_scratch, void* stream) {
  return project_entry(x, ldx, n_rows, k, w, fout, a_src, a_dst, heads, fh, wh, ldwh, el, er,
                       lde, nullptr, w2_scratch, stream);
}

extern "C" int gnn_gat_project_rows_f32(const float* x, int64_t ldx, int64_t n_rows, int64_t k,
                                        const float* w, int64_t fout, const float* a_src,
                                        const float* a_dst, int64_t heads, int64_t fh,
                                        float* wh, int64_t ldwh, float* el, float* er,
                                        int64_t lde, const int64_t* col_row,
                                        float* w2_scratch, void* stream) {
  if (n_rows > 0 && col_row == nullptr) return GNN_E_ARG;
  return project_entry(x, ldx, n_rows, k, w, fout, a_src, a_dst, heads, fh, wh, ldwh, el, er,
                       lde, col_row, w2_scratch, stream);
}
