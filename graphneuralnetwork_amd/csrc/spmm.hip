// spmm.hip -- GCN neighbour aggregation on gfx950: Y = A_hat . X (+ bias) over CSR.
//
// Replaces torch.spmm(adj, support) + bias at GCN/GCN.py:43-45 (reference
// Graph_conv_layer.forward). The reference reduces an uncoalesced fp32 COO with
// ATen's serial CPU kernel; here the adjacency is CSR (rowptr int64, col int32,
// val fp32) and rows are reduced by wavefronts according to the row-class plan
// of plan.hip:
//
//   * mid rows (1 < deg <= seg_len): one wavefront per row. The wave splits into
//     EPI = 64/LPR "edge slots" of LPR lanes; each slot gathers one neighbour row
//     per instruction with VW-wide (16 B for fp32x4) loads, so at F = 128 one wave
//     instruction moves two whole 512-B rows (1 KiB, the widest coalesced access
//     per instruction on CDNA4). The 64 (col, val) pairs of an edge chunk are
//     loaded coalesced once and broadcast to the slots with __shfl (ds_bpermute);
//     U slot loads are issued before the first FMA (U x 16 B per lane in flight).
//   * small rows (deg <= 1, 44% of the rows of the R-MAT graphs: self-loop only):
//     their (col, val) was resolved by the plan, so one wavefront packs
//     EPI x kSmallUnroll of them -- every slot gathers a different row -- instead
//     of spending a whole wave (and a rowptr -> col -> X dependency chain) per row.
//   * long rows (deg > seg_len, the power-law hubs): cut into seg_len-edge
//     segments, one wave each, written to a partial buffer and merged by a
//     fix-up workgroup per row (32 partial loads in flight, fixed order).
//   * slot partial sums are combined with xor-shuffles in a fixed order and no
//     float atomics are used anywhere: results are bitwise reproducible.
//   * the final Y rows are written with non-temporal stores (Y is not re-read by
//     this kernel; keeping it out of L2/MALL leaves room for hub rows of X:
//     +1-3 % measured, tools/spmm_ab.py).
// Segment waves are dispatched first (lowest block ids), then mid rows, then the
// packed small rows.
#include "common.hpp"

namespace gnn {

constexpr int kBlock = 256;                 // 4 waves per workgroup
constexpr int kWavesPerBlock = kBlock / kWave;
#ifndef GNN_SPMM_SMALL_UNROLL
// small rows per slot per wave at NCH = 1 (halved per doubling of NCH). The unrolled loads
// set the register budget of the WHOLE kernel (one launch for every row class): 16 took
// 134 VGPRs = 3 waves/SIMD, 4 takes 48 = 8 waves/SIMD. A/B with isolated variant libraries
// (tools/lib_ab.py, profiles/r02e_lib_ab_*): cfg2 1.574 -> 1.128 ms, the north star
// 18.73 -> 14.55 ms; 2 is the same, 32 spills (4x slower).
#define GNN_SPMM_SMALL_UNROLL 4
#endif
#ifndef GNN_SPMM_U
#define GNN_SPMM_U 4  // slot loads in flight per lane for one-chunk rows (A/B: tools/lib_ab.py)
#endif
#ifndef GNN_SPMM_SMALL_SPLIT
#define GNN_SPMM_SMALL_SPLIT 0
#endif
#ifndef GNN_SPMM_NARROW_CH
#define GNN_SPMM_NARROW_CH 8  // edges per slot chunk in packed tasks of narrow rows (1 = LPR)
#endif
#ifndef GNN_SPMM_TASK_U
#define GNN_SPMM_TASK_U 0  // neighbour rows in flight per slot in packed tasks (0: as GNN_SPMM_U)
#endif
#ifndef GNN_SPMM_SMALL_SPLIT_UNROLL
#define GNN_SPMM_SMALL_SPLIT_UNROLL 16
#endif
#ifndef GNN_SPMM_LDS_PAD
#define GNN_SPMM_LDS_PAD 0  // A/B: dynamic LDS per workgroup to cap workgroups per CU
#endif
constexpr int kSmallUnroll = GNN_SPMM_SMALL_UNROLL;  // small rows per slot per wave (NCH = 1)
// per column-chunk count: the unrolled loads stay at ~16 x 16 B per lane
template <int NCH>
constexpr int small_unroll() {
  return kSmallUnroll / NCH >= 2 ? kSmallUnroll / NCH : 2;
}
constexpr bool kSmallSplit = GNN_SPMM_SMALL_SPLIT;   // small rows in their own launch
constexpr int kSmallSplitUnroll = GNN_SPMM_SMALL_SPLIT_UNROLL;

struct SpmmParams {
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
  const int32_t* mid_row;  // NULL: mid rows are all rows 0..n_rows-1 (no plan)
  int64_t n_mid;
  const int32_t* small_row;
  const int32_t* small_col;
  const float* small_val;
  int64_t n_small;
  float* partial;
  int64_t ldp;
  uint32_t flags;
  // hub staging (HUB kernels): col < 0 names row -1-col of the staged hub table xh
  const float* xh;
  int64_t ldh;
  // packed row tasks (gnn_spmm_csr_tasks_f32): task t = rows [task_row[2t], task_row[2t+1]),
  // at most kTaskRows rows, every row of degree <= the plan's packing threshold
  const int32_t* task_row;
  int64_t n_task;
  // launch geometry (wave index boundaries)
  int64_t seg_waves;
  int64_t mid_waves;
};

// rows per packed task: the task's rowptr values (rows + 1) live in one VGPR (lane = row)
constexpr int kTaskRows = kWave - 1;

#ifndef GNN_SPMM_READLANE
#define GNN_SPMM_READLANE 0  // A/B: edge (col, val) moved to the slots by v_readlane + select
#endif
// v of lane (base + s * stride) & 63 for the calling lane's slot s = lane / LPR (base wave-
// uniform): EPI scalar lane reads and selects instead of one ds_bpermute round trip through LDS
template <int LPR>
__device__ __forceinline__ int slot_lane_i(int v, int base, int stride, int grp) {
  constexpr int EPI = kWave / LPR;
  int r = __builtin_amdgcn_readlane(v, base & (kWave - 1));
#pragma unroll
  for (int s = 1; s < EPI; ++s) {
    const int t = __builtin_amdgcn_readlane(v, (base + s * stride) & (kWave - 1));
    r = grp == s ? t : r;
  }
  return r;
}
template <int LPR>
__device__ __forceinline__ float slot_lane_f(float v, int base, int stride, int grp) {
  return __int_as_float(slot_lane_i<LPR>(__float_as_int(v), base, stride, grp));
}

// acc[ch] += sum_{e in [beg, end)} val[e] * x[col[e]][(ch*LPR + sub)*VW .. +VW)
//
// HUB: a column id c < 0 names row -1-c of the staged hub table xh (the highest-degree
// columns of X copied into one compact buffer per call, see gnn_spmm_csr_hub_f32).
template <int VW, int LPR, int NCH, int U, bool HUB = false>
__device__ __forceinline__ void gather_rows(const int32_t* __restrict__ col,
                                            const float* __restrict__ val, int64_t beg,
                                            int64_t end, const float* __restrict__ x,
                                            int64_t ldx, int64_t feat, int lane,
                                            typename Vec<VW>::T (&acc)[NCH],
                                            const float* __restrict__ xh = nullptr,
                                            int64_t ldh = 0) {
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
#if GNN_SPMM_READLANE
        const int ce = slot_lane_i<LPR>(c, k + u * EPI, 1, grp);
        const float we = slot_lane_f<LPR>(v, k + u * EPI, 1, grp);
#else
        const int src = e & (kWave - 1);
        const int ce = __shfl(c, src, kWave);
        const float we = __shfl(v, src, kWave);
#endif
        w[u] = e < n ? we : 0.f;
        const float* xr = (HUB && ce < 0) ? xh + static_cast<int64_t>(-1 - ce) * ldh
                                          : x + static_cast<int64_t>(ce) * ldx;
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) {
          const int64_t f = static_cast<int64_t>(ch * LPR + sub) * VW;
          xv[u][ch] = (e < n && f < feat) ? vload<VW>(xr + f) : vzero<VW>();
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

// A/B variant (tools/spmm_ab.py variant 3): the same gather with every neighbour row
// staged through LDS by LDS-DMA (global_load_lds_dwordx4: per-lane source address, the
// wave's 1 KiB lands lane-linear at a wave-uniform LDS base) instead of loaded into
// VGPRs -- the "LDS-staged feature tiles" alternative. Each staged row is read back once
// by the lane that requested it, so LDS adds a write + read per byte and frees no reuse;
// measured against the register path in profiles/ (DESIGN.md section 4). VW = 4, NCH = 1.
template <int LPR, int U>
__device__ __forceinline__ void gather_rows_lds(const int32_t* __restrict__ col,
                                                const float* __restrict__ val, int64_t beg,
                                                int64_t end, const float* __restrict__ x,
                                                int64_t ldx, int lane, f4& acc, f4* stage) {
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
      float w[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = k + u * EPI + grp;
        const int ce = __shfl(c, e & (kWave - 1), kWave);
        const float we = __shfl(v, e & (kWave - 1), kWave);
        w[u] = we;
        const float* src = x + static_cast<int64_t>(e < n ? ce : 0) * ldx + sub * 4;
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void*)src,
            (__attribute__((address_space(3))) void*)(stage + u * kWave), 16, 0, 0);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (k + u * EPI + grp < n) acc += w[u] * stage[u * kWave + lane];
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next DMA
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

// Epilogue for one output row held by the LPR lanes `sub` = 0..LPR-1 of a slot.
template <int VW, int LPR, int NCH, bool NT>
__device__ __forceinline__ void store_slot_row(float* __restrict__ out,
                                               const float* __restrict__ bias, int64_t feat,
                                               uint32_t flags, int sub,
                                               typename Vec<VW>::T (&acc)[NCH]) {
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

// Rows with at most one edge, pre-resolved by the plan (small_col -1 = no edge): EPI x SU
// rows per wave, one per slot and unroll step, all SU loads issued before the stores.
template <int VW, int LPR, int NCH, bool NT, int SU>
__device__ __forceinline__ void small_rows(const SpmmParams& P, int64_t swave, int lane) {
  constexpr int EPI = kWave / LPR;
  const int sub = lane & (LPR - 1);
  const int grp = lane / LPR;
  const int64_t i0 = swave * (EPI * SU);
  typename Vec<VW>::T xv[SU][NCH];
  float w[SU];
  int64_t rows[SU];
#pragma unroll
  for (int u = 0; u < SU; ++u) {
    const int64_t i = i0 + u * EPI + grp;
    const bool ok = i < P.n_small;
    const int c = ok ? P.small_col[i] : -1;
    rows[u] = ok ? P.small_row[i] : -1;
    w[u] = c >= 0 ? P.small_val[i] : 0.f;
    const float* xr = P.x + static_cast<int64_t>(c < 0 ? 0 : c) * P.ldx;
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      const int64_t f = static_cast<int64_t>(ch * LPR + sub) * VW;
      xv[u][ch] = (c >= 0 && f < P.feat) ? vload<VW>(xr + f) : vzero<VW>();
    }
  }
#pragma unroll
  for (int u = 0; u < SU; ++u) {
    if (rows[u] < 0) continue;
    typename Vec<VW>::T r[NCH];
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) r[ch] = w[u] * xv[u][ch];
    store_slot_row<VW, LPR, NCH, NT>(P.y + rows[u] * P.ldy, P.bias, P.feat, P.flags, sub, r);
  }
}

// Packed row task: rows [rb, re) of consecutive ids (at most kTaskRows, each of low degree),
// their edges contiguous in col[] / val[]. The rows are split between the EPI edge slots of
// the wave by cost (edges + rows, balanced); each slot streams ITS rows' edges in CSR order,
// U neighbour rows in flight, and writes a row as soon as the stream passes its end. The
// rowptr -> col -> X dependency chain is paid once per task instead of once per row, and the
// gathers of a row overlap the bookkeeping of the next one. Each row's sum runs in edge order
// in one slot: deterministic, no shuffle reduction.
// CPL: edges per lane per chunk (a chunk = LPR * CPL edges of the slot, lane `sub` holding edges
// sub, sub + LPR, ...): narrow rows (LPR = 2 at feat 8) take several, so that a slot keeps more
// than LPR neighbour rows in flight.
template <int VW, int LPR, int NCH, int U, bool NT, bool HUB, int CPL = 1>
__device__ __forceinline__ void packed_rows(const SpmmParams& P, int64_t t, int lane) {
  constexpr int EPI = kWave / LPR;
  constexpr int CH = LPR * CPL;  // edges per slot chunk
  static_assert(CH % U == 0, "a batch of U edges never straddles a chunk");
  const int sub = lane & (LPR - 1);
  const int grp = lane / LPR;
  const int32_t rb = P.task_row[2 * t];
  const int32_t re = P.task_row[2 * t + 1];
  // a task outside the contract (1..kTaskRows rows inside [0, n_rows)) is skipped, never read
  // out of bounds; gnn_spmm_tasks_check reports such tasks before a launch
  if (rb < 0 || re <= rb || re - rb > kTaskRows || re > P.n_rows) return;
  const int nr = re - rb;  // 1 .. kTaskRows
  const int64_t e0 = P.rowptr[rb];
  // lane l < nr: start of row rb + l relative to e0; lanes >= nr: the task's end
  const int rp = static_cast<int>(P.rowptr[rb + min(lane, nr)] - e0);
  const int E = __shfl(rp, nr, kWave);
  // slot g takes rows [sb, se): the first row whose (edges + rows) prefix reaches g/EPI of
  // the task's, found by a ballot over the row lanes
  int sb = 0, se = nr;
  if (EPI > 1) {
    const int64_t total = static_cast<int64_t>(E) + nr;
#pragma unroll
    for (int b = 1; b < EPI; ++b) {
      const int64_t target = total * b / EPI;
      const uint64_t m = __ballot(lane <= nr && static_cast<int64_t>(rp) + lane >= target);
      const int row_b = m ? (__ffsll(static_cast<unsigned long long>(m)) - 1) : nr;
      if (grp == b) sb = row_b;
      if (grp == b - 1) se = row_b;
    }
  }
  int cur = sb;                                   // the row being accumulated
  int cur_end = __shfl(rp, min(cur + 1, nr), kWave);  // its end (slot-uniform)
  const int es = __shfl(rp, sb, kWave);          // the slot's edge range [es, ee)
  const int ee = __shfl(rp, se, kWave);
  int cur_beg = es;                               // its start (slot-uniform, no shuffle later)
  const bool skip_empty = (P.flags & GNN_EPI_SKIP_EMPTY) != 0;
  const uint32_t epi = P.flags & (GNN_EPI_RELU | GNN_EPI_ELU | GNN_EPI_ACCUMULATE);
  typename Vec<VW>::T acc[NCH];
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) acc[ch] = vzero<VW>();

  // write every row of the slot that ends at or before edge position `pos` (several when
  // rows without edges follow each other). The only shuffle runs outside the divergent
  // branch, with the whole wave active: a ds_bpermute whose source lane (here a row index,
  // usually in another slot's lane group) is outside EXEC does not return its value. The
  // row's start is tracked slot-uniformly (the previous row's end), not shuffled.
  auto flush_upto = [&](int pos) {
    bool need = cur < se && pos >= cur_end;
    while (__ballot(need)) {
      if (need) {
        const bool empty = cur_beg == cur_end;
        if (!(empty && skip_empty))
          store_slot_row<VW, LPR, NCH, NT>(P.y + static_cast<int64_t>(rb + cur) * P.ldy, P.bias,
                                           P.feat, epi, sub, acc);
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) acc[ch] = vzero<VW>();
      }
      cur += need ? 1 : 0;
      const int nxt = __shfl(rp, min(cur + 1, nr), kWave);
      cur_beg = need ? cur_end : cur_beg;
      cur_end = need ? nxt : cur_end;
      need = cur < se && pos >= cur_end;
    }
  };

  // every loop below is wave-uniform (the slots' streams differ in length, so the shorter
  // ones idle with their loads masked): the shuffles read rp / c / v from any lane, and a
  // ds_bpermute from a lane outside EXEC would not return its value
  int len = ee - es;
#pragma unroll
  for (int m = 1; m < kWave; m <<= 1) len = max(len, __shfl_xor(len, m, kWave));
  flush_upto(es);  // leading rows without edges
  for (int off = 0; off < len; off += CH) {
    const int cb = es + off;  // this slot's chunk: lane `sub` holds edges cb + sub + j * LPR
    int c[CPL];
    float v[CPL];
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      c[j] = 0;
      v[j] = 0.f;
      if (cb + sub + j * LPR < ee) {
        c[j] = __builtin_nontemporal_load(P.col + e0 + cb + sub + j * LPR);
        v[j] = __builtin_nontemporal_load(P.val + e0 + cb + sub + j * LPR);
      }
    }
    const int n = min(CH, len - off);  // wave-uniform
    auto batch = [&](int k, auto kc) {  // edges k .. k + U - 1 of the chunk (kc: k when constant)
      typename Vec<VW>::T xv[U][NCH];
      float w[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        int ce;
        float we;
        if constexpr (CPL == 1) {
#if GNN_SPMM_READLANE
          ce = slot_lane_i<LPR>(c[0], (k + u) & (LPR - 1), LPR, grp);
          we = slot_lane_f<LPR>(v[0], (k + u) & (LPR - 1), LPR, grp);
#else
          const int src = grp * LPR + ((k + u) & (LPR - 1));
          ce = __shfl(c[0], src, kWave);
          we = __shfl(v[0], src, kWave);
#endif
        } else {  // k is a constant here: the register of edge k + u is known
          constexpr int K0 = decltype(kc)::value;
          const int src = grp * LPR + ((K0 + u) % LPR);
          ce = __shfl(c[(K0 + u) / LPR], src, kWave);
          we = __shfl(v[(K0 + u) / LPR], src, kWave);
        }
        const bool ok = cb + k + u < ee;
        w[u] = ok ? we : 0.f;
        const float* xr = (HUB && ce < 0) ? P.xh + static_cast<int64_t>(-1 - ce) * P.ldh
                                          : P.x + static_cast<int64_t>(ce) * P.ldx;
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) {
          const int64_t f = static_cast<int64_t>(ch * LPR + sub) * VW;
          xv[u][ch] = (ok && f < P.feat) ? vload<VW>(xr + f) : vzero<VW>();
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        flush_upto(cb + k + u);  // rows that end before this edge (all of them past ee)
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) acc[ch] += w[u] * xv[u][ch];
      }
    };
    if constexpr (CPL == 1) {
      for (int k = 0; k < n; k += U) batch(k, std::integral_constant<int, 0>{});
    } else {  // CH / U batches, unrolled (the register index of each edge is a constant)
      static_assert(CH / U <= 4, "at most 4 batches per chunk");
      batch(0, std::integral_constant<int, 0>{});
      if constexpr (CH / U > 1) {
        if (U < n) batch(U, std::integral_constant<int, U>{});
      }
      if constexpr (CH / U > 2) {
        if (2 * U < n) batch(2 * U, std::integral_constant<int, 2 * U>{});
      }
      if constexpr (CH / U > 3) {
        if (3 * U < n) batch(3 * U, std::integral_constant<int, 3 * U>{});
      }
    }
  }
  flush_upto(0x7fffffff);  // the last row and trailing rows without edges
}

template <int VW, int LPR, int NCH, int U, bool NT, bool STAGE = false, bool HUB = false,
          bool TASKS = false, int CPL = 1>
__global__ __launch_bounds__(kBlock) void spmm_csr_kernel(SpmmParams P) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t wave = static_cast<int64_t>(blockIdx.x) * kWavesPerBlock + (threadIdx.x >> 6);
  __shared__ f4 stage_all[STAGE ? kWavesPerBlock * U * kWave : 1];
  f4* stage = stage_all + (STAGE ? (threadIdx.x >> 6) * U * kWave : 0);
  const int sub = lane & (LPR - 1);
  typename Vec<VW>::T acc[NCH];
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) acc[ch] = vzero<VW>();

  if (wave < P.seg_waves) {  // ---- long-row segment -> partial row
    if (wave >= P.n_seg) return;
    const int32_t row = P.seg_row[wave];
    const int64_t beg = P.seg_begin[wave];
    const int64_t end = min(beg + P.seg_len, P.rowptr[row + 1]);
    if constexpr (STAGE)
      gather_rows_lds<LPR, U>(P.col, P.val, beg, end, P.x, P.ldx, lane, acc[0], stage);
    else
      gather_rows<VW, LPR, NCH, U, HUB>(P.col, P.val, beg, end, P.x, P.ldx, P.feat, lane, acc,
                                        P.xh, P.ldh);
    reduce_slots<VW, LPR, NCH>(acc);
    if (lane < LPR) store_slot_row<VW, LPR, NCH, false>(P.partial + wave * P.ldp, nullptr, P.feat,
                                                        0u, sub, acc);
    return;
  }
  if (wave < P.seg_waves + P.mid_waves) {  // ---- one wave per mid row
    const int64_t i = wave - P.seg_waves;
    if (i >= P.n_mid) return;
    const int64_t row = P.mid_row ? P.mid_row[i] : i;
    if constexpr (STAGE)
      gather_rows_lds<LPR, U>(P.col, P.val, P.rowptr[row], P.rowptr[row + 1], P.x, P.ldx, lane,
                              acc[0], stage);
    else
      gather_rows<VW, LPR, NCH, U, HUB>(P.col, P.val, P.rowptr[row], P.rowptr[row + 1], P.x,
                                        P.ldx, P.feat, lane, acc, P.xh, P.ldh);
    reduce_slots<VW, LPR, NCH>(acc);
    if (lane < LPR) store_slot_row<VW, LPR, NCH, NT>(P.y + row * P.ldy, P.bias, P.feat, P.flags,
                                                     sub, acc);
    return;
  }
  if constexpr (TASKS) {  // ---- packed row tasks
    const int64_t t = wave - P.seg_waves - P.mid_waves;
    if (t < P.n_task) packed_rows<VW, LPR, NCH, U, NT, HUB, CPL>(P, t, lane);
  } else if constexpr (!kSmallSplit) {
    // ---- packed small rows (unless they have their own launch, spmm_small_kernel)
    small_rows<VW, LPR, NCH, NT, small_unroll<NCH>()>(P, wave - P.seg_waves - P.mid_waves, lane);
  }
}

// Packed small rows as their own launch: their unrolled loads then do not set the
// register budget (and so the occupancy) of the segment / mid-row waves.
template <int VW, int LPR, int NCH, bool NT>
__global__ __launch_bounds__(kBlock) void spmm_small_kernel(SpmmParams P) {
  small_rows<VW, LPR, NCH, NT, kSmallSplitUnroll>(
      P, static_cast<int64_t>(blockIdx.x) * kWavesPerBlock + (threadIdx.x >> 6),
      threadIdx.x & (kWave - 1));
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
  if (wid != 0 || lane >= LPR) return;
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    typename Vec<VW>::T r = red[0][ch][lane];
#pragma unroll
    for (int w = 1; w < kWavesPerBlock; ++w) r += red[w][ch][lane];
    acc[ch] = r;
  }
  store_slot_row<VW, LPR, NCH, NT>(y + static_cast<int64_t>(long_row[i]) * ldy, bias, feat, flags,
                                   sub, acc);
}

struct SpmmLaunch {
  SpmmParams p;
  const int32_t* long_row;
  const int32_t* long_seg_ptr;
  int64_t n_long;
  hipStream_t stream;
};

template <int VW, int LPR, int NCH, int U_OVERRIDE = 0, bool NT = true, bool STAGE = false,
          bool HUB = false>
static int launch_spmm_t(const SpmmLaunch& L) {
  constexpr int U = U_OVERRIDE ? U_OVERRIDE : (NCH >= 4 ? 1 : (NCH == 2 ? 2 : GNN_SPMM_U));
  constexpr int EPI = kWave / LPR;
  SpmmParams p = L.p;
  const int64_t seg_blocks = (p.n_seg + kWavesPerBlock - 1) / kWavesPerBlock;
  const int64_t mid_blocks = (p.n_mid + kWavesPerBlock - 1) / kWavesPerBlock;
  if constexpr (VW == 4 && !STAGE) {
    if (p.task_row != nullptr) {  // packed row tasks in place of the small-row class
      // neighbour rows in flight per slot: at most LPR (a batch never straddles a chunk of LPR
      // edges), so the narrow rows (LPR = 2: feat 5-8, 32 slots per wave) take 2
      constexpr int UT0 = (GNN_SPMM_TASK_U > 0 && NCH == 1) ? GNN_SPMM_TASK_U : (U > 1 ? U : 2);
      // rows of LPR < GNN_SPMM_NARROW_CH lanes: chunks of GNN_SPMM_NARROW_CH edges per slot,
      // all in flight at once
      constexpr int CPL = LPR < GNN_SPMM_NARROW_CH ? GNN_SPMM_NARROW_CH / LPR : 1;
      constexpr int UT = CPL > 1 ? (LPR * CPL > 8 ? 8 : LPR * CPL) : (UT0 < LPR ? UT0 : LPR);
      const int64_t task_blocks = (p.n_task + kWavesPerBlock - 1) / kWavesPerBlock;
      p.seg_waves = seg_blocks * kWavesPerBlock;
      p.mid_waves = mid_blocks * kWavesPerBlock;
      const int64_t blocks = seg_blocks + mid_blocks + task_blocks;
      if (blocks > 0x7fffffffLL) return GNN_E_UNSUPPORTED;
      if (blocks > 0)
        hipLaunchKernelGGL((spmm_csr_kernel<VW, LPR, NCH, UT, NT, false, HUB, true, CPL>),
                           dim3(static_cast<unsigned>(blocks)), dim3(kBlock), 0, L.stream, p);
      if (L.n_long > 0)
        hipLaunchKernelGGL((spmm_fixup_kernel<VW, LPR, NCH, NT>), dim3(static_cast<unsigned>(L.n_long)),
                           dim3(kBlock), 0, L.stream, L.long_row, L.long_seg_ptr, L.n_long, p.partial,
                           p.ldp, p.feat, p.bias, p.y, p.ldy, p.flags & ~GNN_EPI_SKIP_EMPTY);
      return launch_status();
    }
  }
  if (p.task_row != nullptr) return GNN_E_UNSUPPORTED;
  constexpr int SU = kSmallSplit ? kSmallSplitUnroll : small_unroll<NCH>();
  const int64_t small_waves = (p.n_small + EPI * SU - 1) / (EPI * SU);
  const int64_t small_blocks = (small_waves + kWavesPerBlock - 1) / kWavesPerBlock;
  p.seg_waves = seg_blocks * kWavesPerBlock;
  p.mid_waves = mid_blocks * kWavesPerBlock;
  const int64_t blocks = seg_blocks + mid_blocks + (kSmallSplit ? 0 : small_blocks);
  if (blocks > 0x7fffffffLL || small_blocks > 0x7fffffffLL) return GNN_E_UNSUPPORTED;
  if (blocks > 0) {
    hipLaunchKernelGGL((spmm_csr_kernel<VW, LPR, NCH, U, NT, STAGE, HUB>), dim3(static_cast<unsigned>(blocks)),
                       dim3(kBlock), GNN_SPMM_LDS_PAD, L.stream, p);
  }
  if (kSmallSplit && small_blocks > 0) {
    hipLaunchKernelGGL((spmm_small_kernel<VW, LPR, NCH, NT>), dim3(static_cast<unsigned>(small_blocks)),
                       dim3(kBlock), 0, L.stream, p);
  }
  if (L.n_long > 0) {
    hipLaunchKernelGGL((spmm_fixup_kernel<VW, LPR, NCH, NT>), dim3(static_cast<unsigned>(L.n_long)),
                       dim3(kBlock), 0, L.stream, L.long_row, L.long_seg_ptr, L.n_long, p.partial,
                       p.ldp, p.feat, p.bias, p.y, p.ldy, p.flags);
  }
  return launch_status();
}

template <int VW, int LPR, int NCH, int U_OVERRIDE = 0, bool NT = true, bool STAGE = false>
static int launch_spmm(const SpmmLaunch& L) {
  return L.p.xh ? launch_spmm_t<VW, LPR, NCH, U_OVERRIDE, NT, STAGE, true>(L)
                : launch_spmm_t<VW, LPR, NCH, U_OVERRIDE, NT, STAGE, false>(L);
}

// Picks (VW, LPR, NCH) for one column block of width feat (<= 64*8*VW).
template <int VW>
static int dispatch_spmm(const SpmmLaunch& L) {
  const int64_t nv = (L.p.feat + VW - 1) / VW;  // vectors per row
  if (nv <= 64) {
    switch (next_pow2_le64(nv)) {
      case 1: return launch_spmm<VW, 1, 1>(L);
      case 2: return launch_spmm<VW, 2, 1>(L);
      case 4: return launch_spmm<VW, 4, 1>(L);
      case 8: return launch_spmm<VW, 8, 1>(L);
      case 16: return launch_spmm<VW, 16, 1>(L);
      case 32: return launch_spmm<VW, 32, 1>(L);
      default: return launch_spmm<VW, 64, 1>(L);
    }
  }
  if (nv <= 128) return launch_spmm<VW, 64, 2>(L);
  if (nv <= 256) return launch_spmm<VW, 64, 4>(L);
  return launch_spmm<VW, 64, 8>(L);
}

static int check_spmm_args(const int64_t* rowptr, int64_t n_rows, const float* x, int64_t ldx,
                           int64_t feat, float* y, int64_t ldy, int64_t seg_len, int64_t n_seg,
                           int64_t n_long, int64_t n_small, int64_t n_mid, const int32_t* seg_row,
                           const int64_t* seg_begin, const int32_t* long_row,
                           const int32_t* long_seg_ptr, const int32_t* small_row,
                           const int32_t* small_col, const float* small_val,
                           const int32_t* mid_row, const float* partial, uint32_t flags) {
  if (n_rows < 0 || feat < 0 || n_seg < 0 || n_long < 0 || n_small < 0 || seg_len < 1)
    return GNN_E_ARG;
  if (rowptr == nullptr || y == nullptr || x == nullptr) return GNN_E_ARG;
  if (ldx < feat || ldy < feat) return GNN_E_ARG;
  if (n_rows > 0x7fffffffLL) return GNN_E_UNSUPPORTED;  // int32 column ids / row lists
  if ((n_seg > 0 || n_long > 0) &&
      (seg_row == nullptr || seg_begin == nullptr || long_row == nullptr ||
       long_seg_ptr == nullptr || partial == nullptr || n_long == 0 || n_seg == 0))
    return GNN_E_ARG;
  if (n_small > 0 && (small_row == nullptr || small_col == nullptr || small_val == nullptr))
    return GNN_E_ARG;
  if (mid_row != nullptr && (n_mid < 0 || n_mid + n_small + n_long > n_rows)) return GNN_E_ARG;
  if (flags & ~(GNN_EPI_RELU | GNN_EPI_ELU | GNN_EPI_ACCUMULATE | GNN_EPI_SKIP_EMPTY))
    return GNN_E_ARG;
  return GNN_OK;
}

static int run_spmm(SpmmLaunch L, const float* x, const float* bias, float* y, float* partial,
                    int64_t feat, int variant) {
  const float* xh = L.p.xh;
  const bool vec4 = (feat % 4 == 0) && (L.p.ldx % 4 == 0) && (L.p.ldy % 4 == 0) &&
                    aligned_to(x, 16) && aligned_to(y, 16) &&
                    (xh == nullptr || (aligned_to(xh, 16) && L.p.ldh % 4 == 0)) &&
                    (bias == nullptr || aligned_to(bias, 16)) &&
                    (partial == nullptr || aligned_to(partial, 16));
  if (variant >= 0) {  // developer A/B (feat == 128, vector path only)
    if (feat != 128 || !vec4) return GNN_E_UNSUPPORTED;
    L.p.feat = feat;
    L.p.x = x;
    L.p.y = y;
    L.p.bias = bias;
    L.p.partial = partial;
    switch (variant) {
      case 0: return launch_spmm<4, 32, 1, 4, true>(L);  // the shipped configuration
      case 1: return launch_spmm<4, 32, 1, 8, true>(L);
      case 2: return launch_spmm<4, 32, 1, 2, true>(L);
      case 3: return launch_spmm<4, 32, 1, 4, true, true>(L);   // LDS-DMA staged gather
      case 4: return launch_spmm<4, 32, 1, 8, true, true>(L);   // LDS-DMA, 8 slots in flight
      case 7: return launch_spmm<4, 32, 1, 4, false>(L);
      default: return GNN_E_ARG;
    }
  }
  const int64_t vw = vec4 ? 4 : 1;
  const int64_t blk = 64 * 8 * vw;  // widest column block one launch covers
  for (int64_t c0 = 0; c0 < feat; c0 += blk) {
    L.p.feat = feat - c0 < blk ? feat - c0 : blk;
    L.p.x = x + c0;
    L.p.xh = xh ? xh + c0 : nullptr;
    L.p.y = y + c0;
    L.p.bias = bias ? bias + c0 : nullptr;
    L.p.partial = partial ? partial + c0 : nullptr;
    const int rc = vec4 ? dispatch_spmm<4>(L) : dispatch_spmm<1>(L);
    if (rc != GNN_OK) return rc;
  }
  return GNN_OK;
}

static int spmm_entry(const int64_t* rowptr, const int32_t* col, const float* val, int64_t n_rows,
                      const float* x, int64_t ldx, int64_t feat, const float* bias, float* y,
                      int64_t ldy, int64_t seg_len, const int32_t* seg_row,
                      const int64_t* seg_begin, int64_t n_seg, const int32_t* long_row,
                      const int32_t* long_seg_ptr, int64_t n_long, const int32_t* small_row,
                      const int32_t* small_col, const float* small_val, int64_t n_small,
                      const int32_t* mid_row, int64_t n_mid, float* partial, uint32_t flags,
                      void* stream, int variant, const float* xh = nullptr, int64_t ldh = 0,
                      const int32_t* task_row = nullptr, int64_t n_task = 0) {
  int rc = check_spmm_args(rowptr, n_rows, x, ldx, feat, y, ldy, seg_len, n_seg, n_long, n_small,
                           n_mid, seg_row, seg_begin, long_row, long_seg_ptr, small_row, small_col,
                           small_val, mid_row, partial, flags);
  if (rc != GNN_OK) return rc;
  if (xh != nullptr && ldh < feat) return GNN_E_ARG;
  if (n_rows == 0 || feat == 0) return GNN_OK;
  const bool plan = mid_row != nullptr;
  SpmmLaunch L{};
  L.p.rowptr = rowptr;
  L.p.col = col;
  L.p.val = val;
  L.p.n_rows = n_rows;
  L.p.ldx = ldx;
  L.p.ldy = ldy;
  L.p.seg_len = plan ? seg_len : INT64_MAX;  // no plan: every row by one wave
  L.p.seg_row = seg_row;
  L.p.seg_begin = seg_begin;
  L.p.n_seg = plan ? n_seg : 0;
  L.p.mid_row = mid_row;
  L.p.n_mid = plan ? n_mid : n_rows;
  L.p.small_row = small_row;
  L.p.small_col = small_col;
  L.p.small_val = small_val;
  L.p.n_small = plan ? n_small : 0;
  L.p.ldp = feat;
  L.p.flags = flags;
  L.p.xh = xh;
  L.p.ldh = ldh;
  L.p.task_row = task_row;
  L.p.n_task = n_task;
  L.long_row = long_row;
  L.long_seg_ptr = long_seg_ptr;
  L.n_long = plan ? n_long : 0;
  L.stream = static_cast<hipStream_t>(stream);
  return run_spmm(L, x, bias, y, partial, feat, variant);
}

// err |= 1 for a task with no row, more than kTaskRows rows or rows outside [0, n_rows);
// err |= 2 for a task that overlaps the previous one (tasks must be disjoint and ascending)
__global__ __launch_bounds__(kBlock) void spmm_tasks_check_kernel(const int32_t* __restrict__ task_row,
                                                                  int64_t n_task, int64_t n_rows,
                                                                  int32_t* __restrict__ err) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (t >= n_task) return;
  const int32_t rb = task_row[2 * t], re = task_row[2 * t + 1];
  int32_t e = 0;
  if (rb < 0 || re <= rb || re - rb > kTaskRows || re > n_rows) e |= 1;
  if (t > 0 && task_row[2 * t - 1] > rb) e |= 2;
  if (e) atomicOr(err, e);
}

}  // namespace gnn

using namespace gnn;

extern "C" int gnn_spmm_tasks_check(const int32_t* task_row, int64_t n_task, int64_t n_rows,
                                    int32_t* err, void* stream) {
  if (n_task < 0 || n_rows < 0 || err == nullptr || (n_task > 0 && task_row == nullptr))
    return GNN_E_ARG;
  if (n_task == 0) return GNN_OK;
  const int64_t blocks = (n_task + kBlock - 1) / kBlock;
  if (blocks > 0x7fffffffLL) return GNN_E_UNSUPPORTED;
  hipLaunchKernelGGL(spmm_tasks_check_kernel, dim3(static_cast<unsigned>(blocks)), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), task_row, n_task, n_rows, err);
  return launch_status();
}

extern "C" int gnn_spmm_csr_f32(const int64_t* rowptr, const int32_t* col, const float* val,
                                int64_t n_rows, const float* x, int64_t ldx, int64_t feat,
                                const float* bias, float* y, int64_t ldy, int64_t seg_len,
                                const int32_t* seg_row, const int64_t* seg_begin, int64_t n_seg,
                                const int32_t* long_row, const int32_t* long_seg_ptr,
                                int64_t n_long, const int32_t* small_row, const int32_t* small_col,
                                const float* small_val, int64_t n_small, const int32_t* mid_row,
                                int64_t n_mid, float* partial, uint32_t flags, void* stream) {
  return spmm_entry(rowptr, col, val, n_rows, x, ldx, feat, bias, y, ldy, seg_len, seg_row,
                    seg_begin, n_seg, long_row, long_seg_ptr, n_long, small_row, small_col,
                    small_val, n_small, mid_row, n_mid, partial, flags, stream, -1);
}

extern "C" int gnn_spmm_csr_hub_f32(const int64_t* rowptr, const int32_t* col_hub,
                                    const float* val, int64_t n_rows, const float* x, int64_t ldx,
                                    const float* xh, int64_t ldh, int64_t feat, const float* bias,
                                    float* y, int64_t ldy, int64_t seg_len, const int32_t* seg_row,
                                    const int64_t* seg_begin, int64_t n_seg,
                                    const int32_t* long_row, const int32_t* long_seg_ptr,
                                    int64_t n_long, const int32_t* small_row,
                                    const int32_t* small_col, const float* small_val,
                                    int64_t n_small, const int32_t* mid_row, int64_t n_mid,
                                    float* partial, uint32_t flags, void* stream) {
  if (xh == nullptr) return GNN_E_ARG;
  return spmm_entry(rowptr, col_hub, val, n_rows, x, ldx, feat, bias, y, ldy, seg_len, seg_row,
                    seg_begin, n_seg, long_row, long_seg_ptr, n_long, small_row, small_col,
                    small_val, n_small, mid_row, n_mid, partial, flags, stream, -1, xh, ldh);
}

// ---- developer entry: kernel-variant A/B at one shape (tools/spmm_ab.py) ----
extern "C" int gnn_dev_spmm_variant_f32(const int64_t* rowptr, const int32_t* col,
                                        const float* val, int64_t n_rows, const float* x,
                                        int64_t ldx, int64_t feat, const float* bias, float* y,
                                        int64_t ldy, int64_t seg_len, const int32_t* seg_row,
                                        const int64_t* seg_begin, int64_t n_seg,
                                        const int32_t* long_row, const int32_t* long_seg_ptr,
                                        int64_t n_long, const int32_t* small_row,
                                        const int32_t* small_col, const float* small_val,
                                        int64_t n_small, const int32_t* mid_row, int64_t n_mid,
                                        float* partial, int32_t variant, void* stream) {
  if (variant < 0) return GNN_E_ARG;
  return spmm_entry(rowptr, col, val, n_rows, x, ldx, feat, bias, y, ldy, seg_len, seg_row,
                    seg_begin, n_seg, long_row, long_seg_ptr, n_long, small_row, small_col,
                    small_val, n_small, mid_row, n_mid, partial, 0u, stream, variant);
}

// ---- packed row tasks (GCN/GCN.py:43-45, same aggregation): see packed_rows ----
extern "C" int gnn_spmm_csr_tasks_f32(const int64_t* rowptr, const int32_t* col, const float* val,
                                      int64_t n_rows, const float* x, int64_t ldx, const float* xh,
                                      int64_t ldh, int64_t feat, const float* bias, float* y,
                                      int64_t ldy, int64_t seg_len, const int32_t* seg_row,
                                      const int64_t* seg_begin, int64_t n_seg,
                                      const int32_t* long_row, const int32_t* long_seg_ptr,
                                      int64_t n_long, const int32_t* mid_row, int64_t n_mid,
                                      const int32_t* task_row, int64_t n_task, float* partial,
                                      uint32_t flags, void* stream) {
  if (n_task < 0 || (n_task > 0 && task_row == nullptr) || mid_row == nullptr) return GNN_E_ARG;
  if (n_task > 0x7fffffffLL) return GNN_E_UNSUPPORTED;
  if (xh == nullptr) ldh = 0;
  return spmm_entry(rowptr, col, val, n_rows, x, ldx, feat, bias, y, ldy, seg_len, seg_row,
                    seg_begin, n_seg, long_row, long_seg_ptr, n_long, nullptr, nullptr, nullptr, 0,
                    mid_row, n_mid, partial, flags, stream, -1, xh, ldh,
                    task_row != nullptr ? task_row : mid_row, n_task);
}
