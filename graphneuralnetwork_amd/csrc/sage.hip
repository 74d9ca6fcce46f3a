// sage.hip -- GraphSAGE neighbour aggregation + row gathers on gfx950.
//
// Replaces
//   Aggregator(neigh_feat, 'MEAN' | 'MAX')         GraphSAGE/graph_utils.py:4-11
//     MEAN -> torch.mean(neigh_feat, dim=1)         (fp32 [M, F])
//     MAX  -> torch.argmax(neigh_feat, dim=1)       (int64 [M, F]: FIRST maximal position,
//                                                    a NaN counts as the maximum)
//   value max-pool (north_star "mean/max-pool")     torch.max(neigh, dim=1).values, the
//     value NeighborAggregator 'max' reaches for      (GraphSAGE_Pytorch/models/Aggregator.py:23-24):
//                                                    fp32 [M, F], a NaN in the slice propagates
//   torch.embedding(feats_data, index_map)          GraphSAGE/GraphSAGE.py:47-49,
//                                                    GraphSAGE/data_utils.py:161-162
// Two input forms:
//   pre-gathered  neigh_feat [M, k, F] (the layer-0 tensor collate_fn builds);
//   fused gather  table [n, F] + index map [M, k] int64: the (M, k, F) tensor the
//                 reference materialises with torch.embedding is never written --
//                 every neighbour row is read once from the table and reduced in
//                 registers (K7/K8 + K9 of SURVEY 2.3).
// One wavefront per output row m: EPI = 64/LPR neighbour slots x LPR feature
// lanes x VW-wide loads, U slot loads in flight; the slot partials are combined
// with xor-shuffles. For argmax the combine uses the total order
// (NaN first, larger value, smaller index), so the result is exactly torch's
// regardless of the reduction tree.
#include "common.hpp"

namespace gnn {

constexpr int kSageBlock = 256;
#ifndef GNN_SAGE_U
// neighbour-slot loads in flight per lane. A/B (tools/lib_ab.py --op sage, 10M-row table,
// k = 10, profiles/r01h_sage_u_ab.log): 2: 37.1 us, 4: 35.5, 8: 33.7, 16: 45.8
#define GNN_SAGE_U 8
#endif
#ifndef GNN_SAGE_LDS_PAD
#define GNN_SAGE_LDS_PAD 0  // A/B: dynamic LDS per workgroup to cap workgroups per CU
#endif
constexpr int kSageWaves = kSageBlock / kWave;

// kArgmaxF: the argmax index stored as fp32 (exact below 2^24) -- what the SageLayer's
// torch.cat([self_feats, argmax]) promotes it to (GraphSAGE/GraphSAGE.py:17, graph_utils.py:8)
enum SageMode : int32_t { kMean = 0, kArgmax = 1, kSum = 2, kMaxPool = 3, kArgmaxF = 4 };

// torch.max's value rule: a NaN on either side wins, else the larger value
__device__ __forceinline__ float nanmax(float a, float b) { return (a > b || a != a) ? a : b; }

template <int VW>
__device__ __forceinline__ typename Vec<VW>::T vnanmax(typename Vec<VW>::T a, typename Vec<VW>::T b) {
#pragma unroll
  for (int i = 0; i < VW; ++i) vset(a, i, nanmax(vget(a, i), vget(b, i)));
  return a;
}

// (val, idx) "a beats b" under torch.argmax's rule.
__device__ __forceinline__ bool beats(float va, int32_t ia, float vb, int32_t ib) {
  const bool na = va != va, nb = vb != vb;
  if (na || nb) return na && (!nb || ia < ib);
  return va > vb || (va == vb && ia < ib);
}

// SELF (gather form only): the wave also copies table[self_idx[m]] into self_out[m] -- the
// centre half of the SageLayer's cat[self, agg] (GraphSAGE/GraphSAGE.py:17, 47-48) written by
// the same launch as the aggregate half, its load in flight with the neighbour loads.
template <int VW, int LPR, int NCH, int MODE, bool GATHER, int U, bool SELF = false>
__global__ __launch_bounds__(kSageBlock) void sage_aggregate_kernel(
    const float* __restrict__ src, int64_t ld_row, int64_t ld_m, int64_t n_table,
    const int64_t* __restrict__ idx, int64_t ldi, int64_t M, int64_t k, int64_t feat,
    void* __restrict__ out, int64_t ldo, int32_t* __restrict__ err,
    const int64_t* __restrict__ self_idx = nullptr, float* __restrict__ self_out = nullptr,
    int64_t ld_self = 0, const int64_t* __restrict__ live = nullptr) {
  constexpr int EPI = kWave / LPR;
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t m = static_cast<int64_t>(blockIdx.x) * kSageWaves + (threadIdx.x >> 6);
  if (m >= M || (live != nullptr && m >= *live)) return;  // live: a device row count
  const int sub = lane & (LPR - 1);
  const int grp = lane / LPR;

  typename Vec<VW>::T acc[NCH];
  int32_t arg[NCH][VW];
  typename Vec<VW>::T self_v[NCH];
  if constexpr (SELF) {  // issued first, stored last: overlaps the neighbour gathers
    const int64_t rs = self_idx[m];
    const bool ok = rs >= 0 && rs < n_table;
    if (!ok && lane == 0) atomicOr(err, 1);
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      const int64_t f = static_cast<int64_t>(ch * LPR + sub) * VW;
      self_v[ch] = (ok && grp == 0 && f < feat) ? vload<VW>(src + rs * ld_row + f) : vzero<VW>();
    }
  }
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    acc[ch] = (MODE == kMean || MODE == kSum) ? vzero<VW>() : typename Vec<VW>::T(-INFINITY);
#pragma unroll
    for (int i = 0; i < VW; ++i) arg[ch][i] = 0x7fffffff;
  }

  for (int64_t k0 = 0; k0 < k; k0 += EPI * U) {
    typename Vec<VW>::T xv[U][NCH];
    int32_t kk[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t j = k0 + u * EPI + grp;
      kk[u] = static_cast<int32_t>(j);
      bool ok = j < k;
      const float* row = nullptr;
      if (ok) {
        if (GATHER) {
          const int64_t r = idx[m * ldi + j];
          if (r < 0 || r >= n_table) {
            ok = false;
            if (sub == 0) atomicOr(err, 1);
          } else {
            row = src + r * ld_row;
          }
        } else {
          row = src + m * ld_m + j * ld_row;
        }
      }
      if (!ok) kk[u] = 0x7fffffff;
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) {
        const int64_t f = static_cast<int64_t>(ch * LPR + sub) * VW;
        xv[u][ch] = (ok && f < feat) ? vload<VW>(row + f)
                                     : ((MODE == kMean || MODE == kSum) ? vzero<VW>()
                                                                        : typename Vec<VW>::T(-INFINITY));
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) {
        if (MODE == kMean || MODE == kSum) {
          acc[ch] += xv[u][ch];
        } else if (MODE == kMaxPool) {
          acc[ch] = vnanmax<VW>(acc[ch], xv[u][ch]);
        } else if (kk[u] != 0x7fffffff) {
#pragma unroll
          for (int i = 0; i < VW; ++i) {
            const float v = vget(xv[u][ch], i);
            if (beats(v, kk[u], vget(acc[ch], i), arg[ch][i])) {
              vset(acc[ch], i, v);
              arg[ch][i] = kk[u];
            }
          }
        }
      }
    }
  }
  // combine the EPI neighbour slots
#pragma unroll
  for (int mm = LPR; mm < kWave; mm <<= 1) {
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      if (MODE == kMean || MODE == kSum) {
        acc[ch] += shfl_xor_f(acc[ch], mm);
      } else if (MODE == kMaxPool) {
        acc[ch] = vnanmax<VW>(acc[ch], shfl_xor_f(acc[ch], mm));
      } else {
#pragma unroll
        for (int i = 0; i < VW; ++i) {
          const float ov = __shfl_xor(vget(acc[ch], i), mm, kWave);
          const int32_t oi = __shfl_xor(arg[ch][i], mm, kWave);
          if (beats(ov, oi, vget(acc[ch], i), arg[ch][i])) {
            vset(acc[ch], i, ov);
            arg[ch][i] = oi;
          }
        }
      }
    }
  }
  if (lane >= LPR) return;
  if constexpr (SELF) {
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      const int64_t f = static_cast<int64_t>(ch * LPR + sub) * VW;
      if (f < feat) vstore<VW>(self_out + m * ld_self + f, self_v[ch]);
    }
  }
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    const int64_t f = static_cast<int64_t>(ch * LPR + sub) * VW;
    if (f >= feat) continue;
    if (MODE == kArgmaxF) {
      typename Vec<VW>::T r;
#pragma unroll
      for (int i = 0; i < VW; ++i)
        vset(r, i, arg[ch][i] == 0x7fffffff ? 0.f : static_cast<float>(arg[ch][i]));
      vstore<VW>(static_cast<float*>(out) + m * ldo + f, r);
    } else if (MODE != kArgmax) {
      // torch.mean: sum / k;  torch.sum: the sum;  torch.max(...).values: the max
      typename Vec<VW>::T r = MODE == kMean ? acc[ch] / static_cast<float>(k) : acc[ch];
      vstore<VW>(static_cast<float*>(out) + m * ldo + f, r);
    } else {
      int64_t* o = static_cast<int64_t*>(out) + m * ldo + f;
#pragma unroll
      for (int i = 0; i < VW; ++i) o[i] = arg[ch][i] == 0x7fffffff ? 0 : arg[ch][i];
    }
  }
}

// out[i, :] = x[idx[i], :]  (torch.embedding / halo send-buffer packing)
template <int VW>
__global__ __launch_bounds__(256) void gather_rows_kernel(const float* __restrict__ x, int64_t ldx,
                                                         int64_t n_x, const int64_t* __restrict__ idx,
                                                         int64_t n, int64_t feat,
                                                         float* __restrict__ out, int64_t ldo,
                                                         int32_t* __restrict__ err) {
  const int64_t nv = feat / VW;
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int64_t total = n * nv;
  for (int64_t q = t; q < total; q += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t i = q / nv, v = q % nv;
    const int64_t r = idx[i];
    if (r < 0 || r >= n_x) {
      if (v == 0) atomicOr(err, 1);
      continue;
    }
    vstore<VW>(out + i * ldo + v * VW, vload<VW>(x + r * ldx + v * VW));
  }
}

// out[i, c] = keep(seed, key, c) ? x[r, c] / (1 - p) : x[r, c] * 0 (torch's x * mask * scale:
// NaN stays NaN) with r = idx ? idx[i] : i and key = r
// (KEY_SRC) or i: F.dropout (GAT/models/GAT.py:15,17) as a hashed element mask, fused with the
// models' relabelling gather. The mask is never stored: the backward re-derives it from the
// seed (the same launch with key = the source row through the inverse permutation).
template <int VW, bool KEY_SRC>
__global__ __launch_bounds__(256) void dropout_rows_kernel(
    const float* __restrict__ x, int64_t ldx, int64_t n_x, const int64_t* __restrict__ idx,
    int64_t n, int64_t feat, float p, float scale, uint64_t seed, float* __restrict__ out,
    int64_t ldo, int32_t* __restrict__ err) {
  const int64_t nv = feat / VW;
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int64_t total = n * nv;
  for (int64_t q = t; q < total; q += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t i = q / nv, v = q % nv;
    const int64_t r = idx ? idx[i] : i;
    if (r < 0 || r >= n_x) {
      if (v == 0) atomicOr(err, 1);
      continue;
    }
    const int64_t key = KEY_SRC ? r : i;
    typename Vec<VW>::T a = vload<VW>(x + r * ldx + v * VW);
#pragma unroll
    for (int j = 0; j < VW; ++j) {
      const int c = static_cast<int>(v * VW + j);
      vset(a, j, dropout_keep(seed, key, c, p) ? vget(a, j) * scale : vget(a, j) * 0.f);
    }
    vstore<VW>(out + i * ldo + v * VW, a);
  }
}

struct SageArgs {
  const float* src;
  int64_t ld_row, ld_m, n_table;
  const int64_t* idx;
  int64_t ldi, M, k, feat;
  void* out;
  int64_t ldo;
  int32_t* err;
  hipStream_t s;
  const int64_t* self_idx = nullptr;  // gather form: also copy table[self_idx[m]] ...
  float* self_out = nullptr;          // ... into self_out[m] (one launch for cat[self, agg])
  int64_t ld_self = 0;
  const int64_t* live = nullptr;      // rows [0, min(*live, M)) only (device row count)
};

template <int VW, int LPR, int NCH, int MODE, bool GATHER>
static int launch_sage(const SageArgs& a) {
  constexpr int U = NCH >= 2 ? 2 : GNN_SAGE_U;
  const int64_t blocks = (a.M + kSageWaves - 1) / kSageWaves;
  if (blocks > 0x7fffffffLL) return GNN_E_UNSUPPORTED;
  if (GATHER && a.self_idx != nullptr)
    hipLaunchKernelGGL((sage_aggregate_kernel<VW, LPR, NCH, MODE, GATHER, U, GATHER>),
                       dim3(static_cast<unsigned>(blocks)), dim3(kSageBlock), GNN_SAGE_LDS_PAD, a.s,
                       a.src, a.ld_row, a.ld_m, a.n_table, a.idx, a.ldi, a.M, a.k, a.feat, a.out,
                       a.ldo, a.err, a.self_idx, a.self_out, a.ld_self, a.live);
  else
    hipLaunchKernelGGL((sage_aggregate_kernel<VW, LPR, NCH, MODE, GATHER, U>),
                       dim3(static_cast<unsigned>(blocks)), dim3(kSageBlock), GNN_SAGE_LDS_PAD, a.s,
                       a.src, a.ld_row, a.ld_m, a.n_table, a.idx, a.ldi, a.M, a.k, a.feat, a.out,
                       a.ldo, a.err, nullptr, nullptr, 0, a.live);
  return launch_status();
}

template <int VW, int MODE, bool GATHER>
static int dispatch_sage(const SageArgs& a) {
  const int64_t nv = (a.feat + VW - 1) / VW;
  if (nv <= 64) {
    switch (next_pow2_le64(nv)) {
      case 1: return launch_sage<VW, 1, 1, MODE, GATHER>(a);
      case 2: return launch_sage<VW, 2, 1, MODE, GATHER>(a);
      case 4: return launch_sage<VW, 4, 1, MODE, GATHER>(a);
      case 8: return launch_sage<VW, 8, 1, MODE, GATHER>(a);
      case 16: return launch_sage<VW, 16, 1, MODE, GATHER>(a);
      case 32: return launch_sage<VW, 32, 1, MODE, GATHER>(a);
      default: return launch_sage<VW, 64, 1, MODE, GATHER>(a);
    }
  }
  if (nv <= 128) return launch_sage<VW, 64, 2, MODE, GATHER>(a);
  if (nv <= 256) return launch_sage<VW, 64, 4, MODE, GATHER>(a);
  return launch_sage<VW, 64, 8, MODE, GATHER>(a);
}

template <bool GATHER>
static int run_sage(SageArgs a, int32_t mode, bool vec4) {
  // feature blocks of at most 512 vectors per launch
  const int64_t vw = vec4 ? 4 : 1;
  const int64_t blk = 512 * vw;
  const int64_t feat = a.feat;
  const float* src0 = a.src;
  void* out0 = a.out;
  float* self0 = a.self_out;
  for (int64_t c0 = 0; c0 < feat; c0 += blk) {
    a.feat = feat - c0 < blk ? feat - c0 : blk;
    a.src = src0 + c0;
    if (self0 != nullptr) a.self_out = self0 + c0;
    a.out = mode != kArgmax ? static_cast<void*>(static_cast<float*>(out0) + c0)
                            : static_cast<void*>(static_cast<int64_t*>(out0) + c0);
    int rc;
    if (mode == kMean)
      rc = vec4 ? dispatch_sage<4, kMean, GATHER>(a) : dispatch_sage<1, kMean, GATHER>(a);
    else if (mode == kSum)
      rc = vec4 ? dispatch_sage<4, kSum, GATHER>(a) : dispatch_sage<1, kSum, GATHER>(a);
    else if (mode == kMaxPool)
      rc = vec4 ? dispatch_sage<4, kMaxPool, GATHER>(a) : dispatch_sage<1, kMaxPool, GATHER>(a);
    else if (mode == kArgmaxF)
      rc = vec4 ? dispatch_sage<4, kArgmaxF, GATHER>(a) : dispatch_sage<1, kArgmaxF, GATHER>(a);
    else
      rc = vec4 ? dispatch_sage<4, kArgmax, GATHER>(a) : dispatch_sage<1, kArgmax, GATHER>(a);
    if (rc != GNN_OK) return rc;
  }
  return GNN_OK;
}

}  // namespace gnn

using namespace gnn;

extern "C" int gnn_sage_aggregate_f32(const float* neigh, int64_t ld_k, int64_t ld_m, int64_t M,
                                      int64_t k, int64_t feat, int32_t mode, void* out,
                                      int64_t ldo, void* stream) {
  if (M < 0 || k < 0 || feat < 0 || (mode < kMean || mode > kMaxPool)) return GNN_E_ARG;
  if (M == 0 || feat == 0) return GNN_OK;
  if (!neigh || !out || ld_k < feat || ldo < feat) return GNN_E_ARG;
  if (k == 0) return GNN_E_UNSUPPORTED;  // torch: mean of nothing is NaN, argmax raises
  const bool vec4 = feat % 4 == 0 && ld_k % 4 == 0 && ld_m % 4 == 0 && ldo % 4 == 0 &&
                    aligned_to(neigh, 16) && aligned_to(out, mode != kArgmax ? 16 : 32);
  SageArgs a{neigh, ld_k, ld_m, 0, nullptr, 0, M, k, feat, out, ldo, nullptr,
             static_cast<hipStream_t>(stream)};
  return run_sage<false>(a, mode, vec4);
}

extern "C" int gnn_sage_gather_aggregate_f32(const float* table, int64_t ldt, int64_t n_table,
                                             const int64_t* idx, int64_t ldi, int64_t M, int64_t k,
                                             int64_t feat, int32_t mode, void* out, int64_t ldo,
                                             int32_t* err_flag, void* stream) {
  if (M < 0 || k < 0 || feat < 0 || n_table < 0 || (mode < kMean || mode > kMaxPool))
    return GNN_E_ARG;  // GNN_SAGE_ARGMAX_F32: the concat entries only
  if (M == 0 || feat == 0) return GNN_OK;
  if (!table || !idx || !out || !err_flag || ldt < feat || ldo < feat || ldi < k) return GNN_E_ARG;
  if (k == 0) return GNN_E_UNSUPPORTED;
  const bool vec4 = feat % 4 == 0 && ldt % 4 == 0 && ldo % 4 == 0 && aligned_to(table, 16) &&
                    aligned_to(out, mode != kArgmax ? 16 : 32);
  SageArgs a{table, ldt, 0, n_table, idx, ldi, M, k, feat, out, ldo, err_flag,
             static_cast<hipStream_t>(stream)};
  return run_sage<true>(a, mode, vec4);
}

extern "C" int gnn_gather_rows_f32(const float* x, int64_t ldx, int64_t n_x, const int64_t* idx,
                                   int64_t n, int64_t feat, float* out, int64_t ldo,
                                   int32_t* err_flag, void* stream) {
  if (n < 0 || feat < 0 || n_x < 0) return GNN_E_ARG;
  if (n == 0 || feat == 0) return GNN_OK;
  if (!x || !idx || !out || !err_flag || ldx < feat || ldo < feat) return GNN_E_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool vec4 = feat % 4 == 0 && ldx % 4 == 0 && ldo % 4 == 0 && aligned_to(x, 16) &&
                    aligned_to(out, 16);
  const int64_t total = n * (vec4 ? feat / 4 : feat);
  const int64_t blocks = total / 256 + 1 < 65536 ? total / 256 + 1 : 65536;
  if (vec4)
    hipLaunchKernelGGL(gather_rows_kernel<4>, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, s,
                       x, ldx, n_x, idx, n, feat, out, ldo, err_flag);
  else
    hipLaunchKernelGGL(gather_rows_kernel<1>, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, s,
                       x, ldx, n_x, idx, n, feat, out, ldo, err_flag);
  return launch_status();
}

extern "C" int gnn_dropout_rows_f32(const float* x, int64_t ldx, int64_t n_x, const int64_t* idx,
                                    int32_t key_by_source, int64_t n, int64_t feat, float p,
                                    uint64_t seed, float* out, int64_t ldo, int32_t* err_flag,
                                    void* stream) {
  if (n < 0 || feat < 0 || n_x < 0 || !(p >= 0.f && p < 1.f)) return GNN_E_ARG;
  if (feat > 0x7fffffff) return GNN_E_ARG;  // the hash takes the column as an int
  if (n == 0 || feat == 0) return GNN_OK;
  if (!x || !out || !err_flag || ldx < feat || ldo < feat) return GNN_E_ARG;
  if (!idx && n > n_x) return GNN_E_ARG;
  if (x == out && idx) return GNN_E_ARG;  // in place only without a gather
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool vec4 = feat % 4 == 0 && ldx % 4 == 0 && ldo % 4 == 0 && aligned_to(x, 16) &&
                    aligned_to(out, 16);
  const float scale = 1.0f / (1.0f - p);
  const int64_t total = n * (vec4 ? feat / 4 : feat);
  const int64_t blocks = total / 256 + 1 < 65536 ? total / 256 + 1 : 65536;
  const dim3 grid(static_cast<unsigned>(blocks));
  const bool ks = key_by_source != 0;
  if (vec4 && ks)
    hipLaunchKernelGGL((dropout_rows_kernel<4, true>), grid, dim3(256), 0, s, x, ldx, n_x, idx, n,
                       feat, p, scale, seed, out, ldo, err_flag);
  else if (vec4)
    hipLaunchKernelGGL((dropout_rows_kernel<4, false>), grid, dim3(256), 0, s, x, ldx, n_x, idx, n,
                       feat, p, scale, seed, out, ldo, err_flag);
  else if (ks)
    hipLaunchKernelGGL((dropout_rows_kernel<1, true>), grid, dim3(256), 0, s, x, ldx, n_x, idx, n,
                       feat, p, scale, seed, out, ldo, err_flag);
  else
    hipLaunchKernelGGL((dropout_rows_kernel<1, false>), grid, dim3(256), 0, s, x, ldx, n_x, idx, n,
                       feat, p, scale, seed, out, ldo, err_flag);
  return launch_status();
}

extern "C" int gnn_sage_gather_concat_live_f32(const float* table, int64_t ldt, int64_t n_table,
                                               const int64_t* self_idx, const int64_t* idx,
                                               int64_t ldi, int64_t M, const int64_t* live,
                                               int64_t k, int64_t feat, int32_t mode,
                                               float* self_out, int64_t ld_self, float* out,
                                               int64_t ldo, int32_t* err_flag, void* stream);

extern "C" int gnn_sage_gather_concat_f32(const float* table, int64_t ldt, int64_t n_table,
                                          const int64_t* self_idx, const int64_t* idx, int64_t ldi,
                                          int64_t M, int64_t k, int64_t feat, int32_t mode,
                                          float* self_out, int64_t ld_self, float* out, int64_t ldo,
                                          int32_t* err_flag, void* stream) {
  return gnn_sage_gather_concat_live_f32(table, ldt, n_table, self_idx, idx, ldi, M, nullptr, k,
                                         feat, mode, self_out, ld_self, out, ldo, err_flag, stream);
}

extern "C" int gnn_sage_gather_concat_live_f32(const float* table, int64_t ldt, int64_t n_table,
                                               const int64_t* self_idx, const int64_t* idx,
                                               int64_t ldi, int64_t M, const int64_t* live,
                                               int64_t k, int64_t feat, int32_t mode,
                                               float* self_out, int64_t ld_self, float* out,
                                               int64_t ldo, int32_t* err_flag, void* stream) {
  if (M < 0 || k < 0 || feat < 0 || n_table < 0 ||
      !(mode == kMean || mode == kSum || mode == kMaxPool || mode == kArgmaxF))
    return GNN_E_ARG;
  if (M == 0 || feat == 0) return GNN_OK;
  if (!table || !self_idx || !idx || !self_out || !out || !err_flag || ldt < feat ||
      ldo < feat || ld_self < feat || ldi < k)
    return GNN_E_ARG;
  if (k == 0) return GNN_E_UNSUPPORTED;
  const bool vec4 = feat % 4 == 0 && ldt % 4 == 0 && ldo % 4 == 0 && ld_self % 4 == 0 &&
                    aligned_to(table, 16) && aligned_to(out, 16) && aligned_to(self_out, 16);
  SageArgs a{table, ldt, 0, n_table, idx, ldi, M, k, feat, out, ldo, err_flag,
             static_cast<hipStream_t>(stream), self_idx, self_out, ld_self, live};
  return run_sage<true>(a, mode, vec4);
}
