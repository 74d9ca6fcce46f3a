// spmm.hip -- GCN neighbour aggregation on gfx950: Y = A_hat . X (+ bias) over CSR.
//
// Replaces torch.spmm(adj, support) + bias at GCN/GCN.py:43-45 (reference
// Graph_conv_layer.forward). The reference reduces an uncoalesced fp32 COO with
// ATen's serial CPU kernel; here the adjacency is CSR (rowptr int64, col int32,
// val fp32) and the reduction is one wavefront per output row:
//
//   * the wave splits into EPI = 64/LPR "edge slots" of LPR lanes; each slot
//     gathers one neighbour row per instruction with VW-wide (16 B for fp32x4)
//     loads, so at F = 128 one wave instruction moves two whole 512-B rows
//     (1 KiB, the widest coalesced access per instruction on CDNA4);
//   * the 64 (col, val) pairs of an edge chunk are loaded coalesced once per
//     chunk and broadcast to the slots with __shfl (ds_bpermute), never
//     re-read per feature lane;
//   * U edge-slot loads are issued before the first FMA so every wave keeps
//     U x NCH x 16 B per lane in flight (latency hiding across ~900-cycle HBM
//     misses);
//   * slot partial sums are combined with xor-shuffles in a fixed order, so
//     results are bitwise reproducible run to run (no float atomics).
//
// Power-law graphs: rows whose degree exceeds `seg_len` ("long rows", e.g. the
// 187k-degree hub of the 10M-node RMAT graph) are cut into seg_len-edge
// segments reduced by independent waves into a partial buffer, then summed in
// segment order by a fix-up kernel. Segment waves are dispatched first (low
// block ids) so the heavy work starts before the short-row tail.
#include "common.hpp"

namespace gnn {

constexpr int kBlock = 256;                 // 4 waves per workgroup
constexpr int kWavesPerBlock = kBlock / kWave;

// acc[ch] += sum_{e in [beg, end)} val[e] * x[col[e]][(ch*LPR + sub)*VW .. +VW)
template <int VW, int LPR, int NCH, int U, int LOADMODE = 0>
__device__ __forceinline__ void gather_rows(const int32_t* __restrict__ col,
                                            const float* __restrict__ val, int64_t beg,
                                            int64_t end, const float* __restrict__ x,
                                            int64_t ldx, int64_t feat, int lane,
                                            typename Vec<VW>::T (&acc)[NCH]) {
  constexpr int EPI = kWave / LPR;
  const int sub = lane & (LPR - 1);
  const int grp = lane / LPR;
  for (int64_t base = beg; base < end; base += kWave) {
    const int n = static_cast<int>(min(static_cast<int64_t>(kWave), end - base));
    int c = 0;
    float v = 0.f;
    if (lane < n) {
      c = __builtin_nontemporal_load(col + base + lane);
      v = __builtin_nontemporal_load(val + base + lane);
    }
    for (int k = 0; k < n; k += EPI * U) {
      typename Vec<VW>::T xv[U][NCH];
      float w[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = k + u * EPI + grp;
        const int src = e & (kWave - 1);
        const int craw = __shfl(c, src, kWave);
        const int ce = LOADMODE == 2 ? (craw & 0x7fffffff) : craw;
        const float we = __shfl(v, src, kWave);
        w[u] = e < n ? we : 0.f;
        const float* xr = x + static_cast<int64_t>(ce) * ldx;
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) {
          const int64_t f = static_cast<int64_t>(ch * LPR + sub) * VW;
          const bool ok = e < n && f < feat;
          if (LOADMODE == 0) {
            xv[u][ch] = ok ? vload<VW>(xr + f) : vzero<VW>();
          } else {
            const bool nt = LOADMODE == 1 || craw < 0;
            typedef typename Vec<VW>::T VT;
            const VT* pp = reinterpret_cast<const VT*>(xr + f);
            xv[u][ch] = !ok ? vzero<VW>() : (nt ? __builtin_nontemporal_load(pp) : *pp);
          }
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) acc[ch] += w[u] * xv[u][ch];
      }
    }
  }
}

// Combine the EPI edge slots of a wave (fixed xor-tree order: deterministic).
template <int VW, int LPR, int NCH>
__device__ __forceinline__ void reduce_slots(typename Vec<VW>::T (&acc)[NCH]) {
#pragma unroll
  for (int m = LPR; m < kWave; m <<= 1) {
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) acc[ch] += shfl_xor_f(acc[ch], m);
  }
}

template <int VW, int LPR, int NCH, bool NT = false>
__device__ __forceinline__ void store_row(float* __restrict__ out, const float* __restrict__ bias,
                                          int64_t feat, uint32_t flags, int lane,
                                          typename Vec<VW>::T (&acc)[NCH]) {
  if (lane >= LPR) return;  // slot 0 holds the reduced row
  const int sub = lane;
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    const int64_t f = static_cast<int64_t>(ch * LPR + sub) * VW;
    if (f >= feat) continue;
    typename Vec<VW>::T r = acc[ch];
    if (flags & GNN_EPI_ACCUMULATE) r += vload<VW>(out + f);
    if (bias != nullptr) r += vload<VW>(bias + f);
    if (flags & (GNN_EPI_RELU | GNN_EPI_ELU)) {
#pragma unroll
      for (int i = 0; i < VW; ++i) vset(r, i, act_apply(vget(r, i), flags));
    }
    if (NT)
      __builtin_nontemporal_store(r, reinterpret_cast<typename Vec<VW>::T*>(out + f));
    else
      vstore<VW>(out + f, r);
  }
}

// One launch: waves [0, seg_waves) reduce long-row segments into `partial`,
// the remaining waves reduce one short row each straight into y.
template <int VW, int LPR, int NCH, int U, bool NT = false, int LOADMODE = 0>
__global__ __launch_bounds__(kBlock) void spmm_csr_kernel(
    const int64_t* __restrict__ rowptr, const int32_t* __restrict__ col,
    const float* __restrict__ val, int64_t n_rows, const float* __restrict__ x, int64_t ldx,
    int64_t feat, const float* __restrict__ bias, float* __restrict__ y, int64_t ldy,
    int64_t seg_len, const int32_t* __restrict__ seg_row, const int64_t* __restrict__ seg_begin,
    int64_t n_seg, int64_t seg_waves, float* __restrict__ partial, int64_t ldp, uint32_t flags) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t wave = static_cast<int64_t>(blockIdx.x) * kWavesPerBlock + (threadIdx.x >> 6);
  typename Vec<VW>::T acc[NCH];
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) acc[ch] = vzero<VW>();

  if (wave < seg_waves) {
    if (wave >= n_seg) return;
    const int32_t row = seg_row[wave];
    const int64_t beg = seg_begin[wave];
    const int64_t end = min(beg + seg_len, rowptr[row + 1]);
    gather_rows<VW, LPR, NCH, U, LOADMODE>(col, val, beg, end, x, ldx, feat, lane, acc);
    reduce_slots<VW, LPR, NCH>(acc);
    store_row<VW, LPR, NCH>(partial + wave * ldp, nullptr, feat, 0u, lane, acc);
    return;
  }
  const int64_t row = wave - seg_waves;
  if (row >= n_rows) return;
  const int64_t beg = rowptr[row];
  const int64_t end = rowptr[row + 1];
  if (end - beg > seg_len) return;  // long row: reduced by segment waves + fix-up
  gather_rows<VW, LPR, NCH, U, LOADMODE>(col, val, beg, end, x, ldx, feat, lane, acc);
  reduce_slots<VW, LPR, NCH>(acc);
  store_row<VW, LPR, NCH, NT>(y + row * ldy, bias, feat, flags, lane, acc);
}

// y[long_row[i]] = act(sum_{s in segs(i)} partial[s] + bias).
// One workgroup (4 waves x EPI slots) per long row, UF partial-row loads in flight
// per slot, so a 1,460-segment hub row is not a serial tail; the slot / wave
// partials are combined in a fixed order (xor tree, then waves 0..3 via LDS):
// bitwise reproducible.
template <int VW, int LPR, int NCH, bool NT>
__global__ __launch_bounds__(kBlock) void spmm_fixup_kernel(
    const int32_t* __restrict__ long_row, const int32_t* __restrict__ long_seg_ptr, int64_t n_long,
    const float* __restrict__ partial, int64_t ldp, int64_t feat, const float* __restrict__ bias,
    float* __restrict__ y, int64_t ldy, uint32_t flags) {
  constexpr int EPI = kWave / LPR;
  constexpr int UF = 4;
  constexpr int STRIDE = kWavesPerBlock * EPI;
  __shared__ typename Vec<VW>::T red[kWavesPerBlock][NCH][LPR];
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x >> 6;
  const int64_t i = blockIdx.x;
  if (i >= n_long) return;
  const int sub = lane & (LPR - 1);
  const int grp = lane / LPR;
  typename Vec<VW>::T acc[NCH];
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) acc[ch] = vzero<VW>();
  const int32_t s1 = long_seg_ptr[i + 1];
  for (int32_t s0 = long_seg_ptr[i] + wid * EPI + grp; s0 < s1; s0 += UF * STRIDE) {
    typename Vec<VW>::T v[UF][NCH];
#pragma unroll
    for (int u = 0; u < UF; ++u) {
      const int32_t s = s0 + u * STRIDE;
      const float* pr = partial + static_cast<int64_t>(s) * ldp;
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) {
        const int64_t f = static_cast<int64_t>(ch * LPR + sub) * VW;
        v[u][ch] = (s < s1 && f < feat) ? vload<VW>(pr + f) : vzero<VW>();
      }
    }
#pragma unroll
    for (int u = 0; u < UF; ++u) {
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) acc[ch] += v[u][ch];
    }
  }
  reduce_slots<VW, LPR, NCH>(acc);
  if (lane < LPR) {
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) red[wid][ch][lane] = acc[ch];
  }
  __syncthreads();
  if (wid != 0) return;
  if (lane < LPR) {
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      typename Vec<VW>::T r = red[0][ch][lane];
#pragma unroll
      for (int w = 1; w < kWavesPerBlock; ++w) r += red[w][ch][lane];
      acc[ch] = r;
    }
  }
  store_row<VW, LPR, NCH, NT>(y + static_cast<int64_t>(long_row[i]) * ldy, bias, feat, flags, lane,
                              acc);
}

struct SpmmArgs {
  const int64_t* rowptr;
  const int32_t* col;
  const float* val;
  int64_t n_rows;
  const float* x;
  int64_t ldx;
  int64_t feat;  // width of this column block
  const float* bias;
  float* y;
  int64_t ldy;
  int64_t seg_len;
  const int32_t* seg_row;
  const int64_t* seg_begin;
  int64_t n_seg;
  const int32_t* long_row;
  const int32_t* long_seg_ptr;
  int64_t n_long;
  float* partial;
  int64_t ldp;
  uint32_t flags;
  hipStream_t stream;
};

template <int VW, int LPR, int NCH, int U_OVERRIDE = 0, bool NT = true, int LOADMODE = 0>
static int launch_spmm(const SpmmArgs& a) {
  constexpr int U = U_OVERRIDE ? U_OVERRIDE : (NCH >= 4 ? 1 : (NCH == 2 ? 2 : 4));
  const int64_t seg_blocks = (a.n_seg + kWavesPerBlock - 1) / kWavesPerBlock;
  const int64_t row_blocks = (a.n_rows + kWavesPerBlock - 1) / kWavesPerBlock;
  const int64_t blocks = seg_blocks + row_blocks;
  if (blocks > 0x7fffffffLL) return GNN_E_UNSUPPORTED;
  if (blocks > 0) {
    hipLaunchKernelGGL((spmm_csr_kernel<VW, LPR, NCH, U, NT, LOADMODE>), dim3(static_cast<unsigned>(blocks)),
                       dim3(kBlock), 0, a.stream, a.rowptr, a.col, a.val, a.n_rows, a.x, a.ldx,
                       a.feat, a.bias, a.y, a.ldy, a.seg_len, a.seg_row, a.seg_begin, a.n_seg,
                       seg_blocks * kWavesPerBlock, a.partial, a.ldp, a.flags);
  }
  if (a.n_long > 0) {
    const int64_t fb = a.n_long;
    hipLaunchKernelGGL((spmm_fixup_kernel<VW, LPR, NCH, NT>), dim3(static_cast<unsigned>(fb)),
                       dim3(kBlock), 0, a.stream, a.long_row, a.long_seg_ptr, a.n_long, a.partial,
                       a.ldp, a.feat, a.bias, a.y, a.ldy, a.flags);
  }
  return launch_status();
}

// Picks (VW, LPR, NCH) for one column block of width a.feat (<= 64*8*VW).
template <int VW>
static int dispatch_spmm(const SpmmArgs& a) {
  const int64_t nv = (a.feat + VW - 1) / VW;  // vectors per row
  if (nv <= 64) {
    switch (next_pow2_le64(nv)) {
      case 1: return launch_spmm<VW, 1, 1>(a);
      case 2: return launch_spmm<VW, 2, 1>(a);
      case 4: return launch_spmm<VW, 4, 1>(a);
      case 8: return launch_spmm<VW, 8, 1>(a);
      case 16: return launch_spmm<VW, 16, 1>(a);
      case 32: return launch_spmm<VW, 32, 1>(a);
      default: return launch_spmm<VW, 64, 1>(a);
    }
  }
  if (nv <= 128) return launch_spmm<VW, 64, 2>(a);
  if (nv <= 256) return launch_spmm<VW, 64, 4>(a);
  return launch_spmm<VW, 64, 8>(a);
}

}  // namespace gnn

using namespace gnn;

extern "C" int gnn_spmm_csr_f32(const int64_t* rowptr, const int32_t* col, const float* val,
                                int64_t n_rows, const float* x, int64_t ldx, int64_t feat,
                                const float* bias, float* y, int64_t ldy, int64_t seg_len,
                                const int32_t* seg_row, const int64_t* seg_begin, int64_t n_seg,
                                const int32_t* long_row, const int32_t* long_seg_ptr,
                                int64_t n_long, float* partial, uint32_t flags, void* stream) {
  if (n_rows < 0 || feat < 0 || n_seg < 0 || n_long < 0 || seg_len < 1) return GNN_E_ARG;
  if (n_rows == 0 || feat == 0) return GNN_OK;
  if (rowptr == nullptr || y == nullptr || x == nullptr) return GNN_E_ARG;
  if (ldx < feat || ldy < feat) return GNN_E_ARG;
  if (n_rows > 0x7fffffffLL) return GNN_E_UNSUPPORTED;  // int32 column ids
  if ((n_seg > 0 || n_long > 0) &&
      (seg_row == nullptr || seg_begin == nullptr || long_row == nullptr ||
       long_seg_ptr == nullptr || partial == nullptr || n_long == 0 || n_seg == 0))
    return GNN_E_ARG;
  if (flags & ~(GNN_EPI_RELU | GNN_EPI_ELU | GNN_EPI_ACCUMULATE)) return GNN_E_ARG;

  const bool vec4 = (feat % 4 == 0) && (ldx % 4 == 0) && (ldy % 4 == 0) && aligned_to(x, 16) &&
                    aligned_to(y, 16) && (bias == nullptr || aligned_to(bias, 16)) &&
                    (partial == nullptr || aligned_to(partial, 16));
  const int64_t vw = vec4 ? 4 : 1;
  const int64_t blk = 64 * 8 * vw;  // widest column block one launch covers
  SpmmArgs a{rowptr, col, val, n_rows, x, ldx, 0, bias, y, ldy, seg_len, seg_row, seg_begin,
             n_seg, long_row, long_seg_ptr, n_long, partial, feat, flags,
             static_cast<hipStream_t>(stream)};
  for (int64_t c0 = 0; c0 < feat; c0 += blk) {
    a.feat = feat - c0 < blk ? feat - c0 : blk;
    a.x = x + c0;
    a.y = y + c0;
    a.bias = bias ? bias + c0 : nullptr;
    a.partial = partial ? partial + c0 : nullptr;
    const int rc = vec4 ? dispatch_spmm<4>(a) : dispatch_spmm<1>(a);
    if (rc != GNN_OK) return rc;
  }
  return GNN_OK;
}

// ---- developer entry: kernel-variant A/B at one shape (tools/spmm_ab.py) ----
extern "C" int gnn_dev_spmm_variant_f32(const int64_t* rowptr, const int32_t* col, const float* val,
                                        int64_t n_rows, const float* x, int64_t ldx, int64_t feat,
                                        const float* bias, float* y, int64_t ldy, int64_t seg_len,
                                        const int32_t* seg_row, const int64_t* seg_begin,
                                        int64_t n_seg, const int32_t* long_row,
                                        const int32_t* long_seg_ptr, int64_t n_long,
                                        float* partial, int32_t variant, void* stream) {
  if (feat != 128 || ldx % 4 || ldy % 4 || !aligned_to(x, 16) || !aligned_to(y, 16))
    return GNN_E_UNSUPPORTED;
  SpmmArgs a{rowptr, col, val, n_rows, x, ldx, feat, bias, y, ldy, seg_len, seg_row, seg_begin,
             n_seg, long_row, long_seg_ptr, n_long, partial, feat, 0u,
             static_cast<hipStream_t>(stream)};
  switch (variant) {
    case 0: return launch_spmm<4, 32, 1, 4, true>(a);  // the shipped configuration
    case 7: return launch_spmm<4, 32, 1, 4, false>(a);
    case 8: return launch_spmm<4, 32, 1, 4, true, 1>(a);  // every X gather non-temporal
    case 9: return launch_spmm<4, 32, 1, 4, true, 2>(a);  // col sign bit = cold -> non-temporal
    case 1: return launch_spmm<4, 32, 1, 8, false>(a);
    case 2: return launch_spmm<4, 32, 1, 2, false>(a);
    case 3: return launch_spmm<4, 32, 1, 4, true>(a);
    case 4: return launch_spmm<2, 64, 1, 4, false>(a);
    case 5: return launch_spmm<2, 64, 1, 8, true>(a);
    case 6: return launch_spmm<4, 32, 1, 8, true>(a);
    default: return GNN_E_ARG;
  }
}
