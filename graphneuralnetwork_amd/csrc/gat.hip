// gat.hip -- GAT edge-softmax + neighbour aggregation on gfx950, all heads in one pass.
//
// Replaces, per attention layer, the reference's
//   dense  GraphAttentionLayer.forward   GAT/models/layers.py:22-37
//          (N x N a_input, LeakyReLU, mask adj > 0 with -9e15, softmax(dim=1), att @ Wh, ELU)
//   sparse SpGraphAttentionLayer.forward GAT/models/layers.py:94-131
//          (edge_h gather/cat, exp(-LeakyReLU(a.edge_h)), two COO spmm's, div, ELU)
// and the per-head Python loop + torch.cat of GAT/models/GAT.py:16.
//
// Inputs are the projected features Wh [N, H*Fh] (one MFMA GEMM for all heads)
// and the per-node attention logits el = a_src.Wh_i, er = a_dst.Wh_j [N, H]
// (gnn_gat_logits_f32). Per output row i the kernel streams the row's edges once:
//
//   phase A (lane = edge, 64 edges per chunk): s_ijh = LeakyReLU(el_ih + er_jh);
//     dense : online softmax -- chunk max per head by a wave reduction, running
//             max m_h, rescale of the lane-local denominators and of acc;
//     sparse: p = exp(-s) with NO max subtraction (the reference's arithmetic,
//             including its overflow to inf / NaN; v_exp_f32-based __expf, within
//             ~1e-6 relative of the correctly rounded exp and overflowing at the
//             same argument to within rounding);
//     p[e][h] goes to a 64 x HP LDS tile private to the wave.
//   phase B (lanes = features): acc[f] += p[e][head(f)] * Wh[col_e][f] with the
//     same wide-gather geometry as the SpMM (EPI edge slots x LPR lanes x VW).
//   epilogue: slot reduction, out = acc / l[head(f)] (+ ELU), one store per row.
//
// Dropout (training mode) is applied to the numerator weights only -- exactly
// where both reference layers apply it (after softmax / after the rowsum) --
// with a counter-based hash RNG keyed by (seed, edge, head).
// Power-law rows are split into segments like the SpMM; a segment emits
// (acc, l, m) and the fix-up merges segments with the standard log-sum-exp rule.
#include "common.hpp"

namespace gnn {

constexpr int kGatBlock = 256;
constexpr int kGatWaves = kGatBlock / kWave;
constexpr int kMaxHeads = 8;  // heads per launch; more heads are split by the host

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int m = 1; m < kWave; m <<= 1) v = fmaxf(v, __shfl_xor(v, m, kWave));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int m = 1; m < kWave; m <<= 1) v += __shfl_xor(v, m, kWave);
  return v;
}

__device__ __forceinline__ uint32_t hash3(uint64_t seed, int64_t edge, int head) {
  uint32_t h = static_cast<uint32_t>(seed) ^ (static_cast<uint32_t>(seed >> 32) * 0x27d4eb2fu);
  h ^= static_cast<uint32_t>(edge) * 0x9e3779b9u;
  h ^= static_cast<uint32_t>(static_cast<uint64_t>(edge) >> 32) * 0x85ebca6bu;
  h ^= static_cast<uint32_t>(head) * 0xc2b2ae35u;
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}

struct GatParams {
  const int64_t* rowptr;
  const int32_t* col;
  int64_t n_rows;
  const float* wh;
  int64_t ldw;
  int64_t feat;  // H * Fh of this head group
  int64_t fh;
  const float* el;
  const float* er;
  int64_t lde;
  int heads;
  float slope;
  const float* empty_fill;
  float drop_p;
  float drop_scale;
  uint64_t drop_seed;
  int head0;  // global index of this group's first head (dropout stream)
  float* out;
  int64_t ldo;
  int64_t seg_len;
  const int32_t* seg_row;
  const int64_t* seg_begin;
  int64_t n_seg;
  int64_t seg_waves;
  const int32_t* mid_row;  // NULL: every row is a mid row (no plan)
  int64_t n_mid;
  const int32_t* short_row;  // short rows (a few edges): lane-private softmax, LPR lanes per row
  int64_t n_short;
  int64_t short_waves;
  int64_t mid_waves;
  const int32_t* small_row;
  const int32_t* small_col;
  int64_t n_small;
  const int32_t* long_row;
  const int32_t* long_seg_ptr;
  int64_t n_long;
  float* partial;  // per segment: [feat acc][heads l][heads m]
  int64_t ldp;
  uint32_t flags;
  float* stats;    // optional [n_rows, lds]: per-head log-sum-exp of the row (backward)
  int64_t lds;
  // hub staging (gnn_gat_csr_hub_f32): a column id c < 0 names row -1-c of the staged
  // tables whh [K, ldwh] / erh [K, ldeh] (the highest-degree columns' Wh and er rows)
  const float* whh;
  int64_t ldwh;
  const float* erh;
  int64_t ldeh;
  // packed row tasks (gnn_gat_csr_tasks_f32): task t = rows [task_row[2t], task_row[2t+1]),
  // at most kGatTaskRows consecutive rows of low degree (edgeless and one-edge rows included)
  const int32_t* task_row;
  int64_t n_task;
  // er recomputed from the gathered Wh rows (gnn_gat_csr_ex_f32 with a_dst): er_j[h] =
  // a_dst[h] . Wh_j[h], the lane's VW-feature partial dot summed over the er_g lanes of its
  // head -- no er gather in the one-chunk loop, the short rows and the small rows (the er gather
  // was 0.17 of 0.78 ms at cfg3, tools/gat_tasks_ab.py --libs noer). NULL: er gathered.
  const float* a_dst;
  int er_g;
};

template <int VW>
__device__ __forceinline__ float er_partial(typename Vec<VW>::T x, typename Vec<VW>::T a) {
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < VW; ++k) s = fmaf(vget(x, k), vget(a, k), s);
  return s;
}
// sum over the er_g lanes of a head (aligned lane groups, all active)
__device__ __forceinline__ float er_reduce(float v, int g) {
  for (int o = 1; o < g; o <<= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// Wh row / er entry of column c (hub-staged when c < 0). Without staging no column id is
// negative and the select never picks the hub tables.
__device__ __forceinline__ const float* wh_row(const GatParams& P, int c) {
  return c < 0 ? P.whh + static_cast<int64_t>(-1 - c) * P.ldwh
               : P.wh + static_cast<int64_t>(c) * P.ldw;
}
__device__ __forceinline__ float er_at(const GatParams& P, int c, int h) {
  return c < 0 ? P.erh[static_cast<int64_t>(-1 - c) * P.ldeh + h]
               : P.er[static_cast<int64_t>(c) * P.lde + h];
}

#ifndef GNN_GAT_SMALL_UNROLL
// edgeless / one-edge rows per slot per wave at NCH = 1 (halved per doubling of NCH). The
// unrolled loads set the register budget of the whole gat_csr_kernel: 16 took 129 VGPRs
// (3 waves/SIMD), 4 takes 58-66 (7-8). A/B with isolated variant libraries at cfg3
// (tools/gat_ab.py, profiles/r02f_gat_ab.log): 1.295 -> 0.791 ms (with GNN_GAT_U = 4).
#define GNN_GAT_SMALL_UNROLL 4
#endif
constexpr int kGatSmallUnroll = GNN_GAT_SMALL_UNROLL;
template <int NCH>
constexpr int gat_small_unroll() {
  return kGatSmallUnroll / NCH >= 2 ? kGatSmallUnroll / NCH : 2;
}
#ifndef GNN_GAT_U
#define GNN_GAT_U 4  // feature-row gathers in flight per lane in phase B (capped at the chunk's slots)
#endif
#ifndef GNN_GAT_PIPE
#define GNN_GAT_PIPE 1  // pipelined chunk loop in gat_csr_kernel (0: plain loop; a depth-2 form,
                        // two chunks in flight, was slower: profiles/r05b_gat_tasks_ab.log)
#endif
#ifndef GNN_GAT_EH
#define GNN_GAT_EH 1  // segments and mid rows in the edge-head layout (gat_eh_kernel)
#endif
#ifndef GNN_GAT_CHUNK
#define GNN_GAT_CHUNK 8  // edges per phase-A chunk (A/B at cfg3 with the short-row path: 8 > 16 > 32 > 64)
#endif

// Rows with at most one edge (44 % of the R-MAT rows: the self-loop only), packed
// EPI x kGatSmallUnroll per wave. One edge j: dense softmax weight exp(z - z) = 1,
// so out = Wh_j exactly; sparse computes (p * Wh_j) / p with p = exp(-LeakyReLU)
// like the reference (inf/0 -> NaN preserved). No edge: dense -> empty_fill,
// sparse -> 0/0 = NaN.
template <int VW, int LPR, int NCH, bool SPARSE, bool REC>
__device__ __forceinline__ void gat_small_rows(const GatParams& P, int64_t wave, int lane) {
  constexpr int EPI = kWave / LPR;
  const int sub = lane & (LPR - 1);
  const int grp = lane / LPR;
  constexpr int SU = gat_small_unroll<NCH>();
  const int64_t i0 = wave * (EPI * SU);
  typename Vec<VW>::T xv[SU][NCH];
  int64_t rows[SU];
  int cols[SU];
#pragma unroll
  for (int u = 0; u < SU; ++u) {
    const int64_t i = i0 + u * EPI + grp;
    const bool ok = i < P.n_small;
    const int c = ok ? P.small_col[i] : -1;
    rows[u] = ok ? P.small_row[i] : -1;
    cols[u] = c;
    const float* xr = P.wh + static_cast<int64_t>(c < 0 ? 0 : c) * P.ldw;
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      const int64_t f = static_cast<int64_t>(ch * LPR + sub) * VW;
      xv[u][ch] = (c >= 0 && f < P.feat) ? vload<VW>(xr + f) : vzero<VW>();
    }
  }
  float erx[SU];  // er of (slot's column, lane's head) from the gathered row (NCH == 1)
  if constexpr (REC) {
    const int64_t f = static_cast<int64_t>(sub) * VW;
    const typename Vec<VW>::T ad = f < P.feat ? vload<VW>(P.a_dst + f) : vzero<VW>();
#pragma unroll
    for (int u = 0; u < SU; ++u) erx[u] = er_reduce(er_partial<VW>(xv[u][0], ad), P.er_g);
  }
#pragma unroll
  for (int u = 0; u < SU; ++u) {
    if (rows[u] < 0) continue;
    float* orow = P.out + rows[u] * P.ldo;
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      const int64_t f = static_cast<int64_t>(ch * LPR + sub) * VW;
      if (f >= P.feat) continue;
      typename Vec<VW>::T r;
      if (P.stats && f % P.fh == 0) {  // one lane per head records the row's log-sum-exp
        const int h = static_cast<int>(f / P.fh);
        float lse = -INFINITY;
        if (cols[u] >= 0) {
          const float erv = REC ? erx[u] : P.er[static_cast<int64_t>(cols[u]) * P.lde + h];
          const float sv = P.el[rows[u] * P.lde + h] + erv;
          const float x = sv > 0.f ? sv : P.slope * sv;
          lse = SPARSE ? -x : x;
        }
        P.stats[rows[u] * P.lds + h] = lse;
      }
      if (cols[u] < 0) {
        r = (!SPARSE && P.empty_fill) ? vload<VW>(P.empty_fill + f) : typename Vec<VW>::T(NAN);
      } else if (SPARSE) {
        const int h = static_cast<int>(f / P.fh);
        const float erv = REC ? erx[u] : P.er[static_cast<int64_t>(cols[u]) * P.lde + h];
        const float sv = P.el[rows[u] * P.lde + h] + erv;
        const float p = __expf(-(sv > 0.f ? sv : P.slope * sv));
        float wv = p;
        if (P.drop_p > 0.f) {
          const uint32_t rr = hash3(P.drop_seed, P.rowptr[rows[u]], P.head0 + h);
          wv = (static_cast<float>(rr >> 8) * (1.0f / 16777216.0f) < P.drop_p) ? 0.f
                                                                                : wv * P.drop_scale;
        }
        r = (wv * xv[u][ch]) / p;
      } else {
        float wv = 1.f;
        if (P.drop_p > 0.f) {
          const int h = static_cast<int>(f / P.fh);
          const uint32_t rr = hash3(P.drop_seed, P.rowptr[rows[u]], P.head0 + h);
          wv = (static_cast<float>(rr >> 8) * (1.0f / 16777216.0f) < P.drop_p) ? 0.f : P.drop_scale;
        }
        r = wv * xv[u][ch];
      }
#pragma unroll
      for (int k = 0; k < VW; ++k) vset(r, k, act_apply(vget(r, k), P.flags));
      vstore<VW>(orow + f, r);
    }
  }
}

#ifndef GNN_GAT_SHORT_CHUNK
#define GNN_GAT_SHORT_CHUNK 4  // A/B at cfg3 (tools/gat_ab.py, profiles/r03ai_gat_short_chunk_ab.log): 4 0.794, 8 0.803, 16 0.859 ms
#endif
constexpr int kGatShortChunk = GNN_GAT_SHORT_CHUNK;  // edges whose loads one lane issues together

// Short rows (deg 2..8 on R-MAT: 35 % of the rows, 6 % of the edges), 64/LPR rows per
// wave: each LPR-lane group owns one row and every lane runs the edge softmax for the
// head of its own VW features privately -- no cross-lane reduction, no LDS, no
// shuffles; the row's column ids, er values and feature rows are all issued at once
// (chunks of kGatShortChunk edges, online max across chunks). Same arithmetic per
// edge as gat_csr_kernel (dense: exp(z - max), sparse: exp(z)); requires fh % VW == 0
// and NCH == 1 (the launcher routes other shapes through the one-row-per-wave path).
template <int VW, int LPR, bool SPARSE, bool REC>
__device__ __forceinline__ void gat_short_rows(const GatParams& P, int64_t wave, int lane) {
  constexpr int RPW = kWave / LPR;
  constexpr int K = kGatShortChunk;
  const int64_t i = wave * RPW + lane / LPR;
  const int64_t f = static_cast<int64_t>(lane & (LPR - 1)) * VW;
  if (i >= P.n_short || f >= P.feat) return;
  const int64_t row = P.short_row[i];
  const int64_t beg = P.rowptr[row], end = P.rowptr[row + 1];
  const int h = static_cast<int>(f / P.fh);
  const float eli = P.el[row * P.lde + h];
  const typename Vec<VW>::T adst = REC ? vload<VW>(P.a_dst + f) : vzero<VW>();
  float m = SPARSE ? 0.f : -INFINITY, l = 0.f;
  typename Vec<VW>::T acc = vzero<VW>();
  for (int64_t b = beg; b < end; b += K) {
    const int n = static_cast<int>(min(static_cast<int64_t>(K), end - b));
    int c[K];
    float z[K];
    typename Vec<VW>::T xv[K];
#pragma unroll
    for (int e = 0; e < K; ++e) c[e] = e < n ? P.col[b + e] : 0;
    if constexpr (REC) {  // er from the gathered rows: one round trip, no er loads
#pragma unroll
      for (int e = 0; e < K; ++e) xv[e] = e < n ? vload<VW>(wh_row(P, c[e]) + f) : vzero<VW>();
#pragma unroll
      for (int e = 0; e < K; ++e) {
        const float erv = er_reduce(er_partial<VW>(xv[e], adst), P.er_g);
        z[e] = -INFINITY;
        if (e < n) {
          const float sv = eli + erv;
          const float x = sv > 0.f ? sv : P.slope * sv;
          z[e] = SPARSE ? -x : x;
        }
      }
    } else {
#pragma unroll
      for (int e = 0; e < K; ++e) {
        z[e] = -INFINITY;
        if (e < n) {
          const float sv = eli + er_at(P, c[e], h);
          const float x = sv > 0.f ? sv : P.slope * sv;
          z[e] = SPARSE ? -x : x;
        }
        xv[e] = e < n ? vload<VW>(wh_row(P, c[e]) + f) : vzero<VW>();
      }
    }
    if (!SPARSE) {
      float cm = z[0];
#pragma unroll
      for (int e = 1; e < K; ++e) cm = fmaxf(cm, z[e]);
      const float mn = fmaxf(m, cm);
      const float scale = __expf(m - mn);  // 0 on the first chunk (m = -inf)
      m = mn;
      l *= scale;
      acc *= scale;
    }
#pragma unroll
    for (int e = 0; e < K; ++e) {
      if (e >= n) continue;
      const float p = SPARSE ? __expf(z[e]) : (z[e] == -INFINITY ? 0.f : __expf(z[e] - m));
      l += p;
      float w = p;
      if (P.drop_p > 0.f) {
        const uint32_t r = hash3(P.drop_seed, b + e, P.head0 + h);
        w = (static_cast<float>(r >> 8) * (1.0f / 16777216.0f) < P.drop_p) ? 0.f : w * P.drop_scale;
      }
      acc += w * xv[e];
    }
  }
  if (P.stats && f % P.fh == 0) P.stats[row * P.lds + h] = (SPARSE ? 0.f : m) + __logf(l);
  typename Vec<VW>::T r = acc / l;
#pragma unroll
  for (int k = 0; k < VW; ++k) vset(r, k, act_apply(vget(r, k), P.flags));
  vstore<VW>(P.out + row * P.ldo + f, r);
}

template <int VW, int LPR, bool SPARSE, bool REC>
__global__ __launch_bounds__(kGatBlock) void gat_short_kernel(GatParams P) {
  gat_short_rows<VW, LPR, SPARSE, REC>(P, static_cast<int64_t>(blockIdx.x) * kGatWaves + (threadIdx.x >> 6),
                                  threadIdx.x & (kWave - 1));
}

#ifndef GNN_GAT_TASK_U
#define GNN_GAT_TASK_U 4  // edges whose er / Wh loads a slot issues together in a packed task
#endif
constexpr int kGatTaskRows = 63;  // a task's rowptr values fit one VGPR (lane = row)

// Packed row tasks for the low-degree rows (the SpMM's packed_rows with an edge softmax): a
// wave takes <= 63 consecutive rows of degree <= the plan's threshold, splits them between its
// EPI edge slots by cost (edges + rows), and every slot streams ITS rows' edges in CSR order --
// column ids loaded coalesced by the slot's LPR lanes and broadcast, U edges' er entries and Wh
// rows in flight -- with a lane-private online softmax for the head of the lane's VW features,
// writing a row (out = acc / l, stats) as soon as the stream passes its end. The rowptr ->
// col -> (er, Wh) chain is paid once per task instead of per row (gat_short_kernel: 4 rows per
// wave, one chain each), and the row's el values come from an LDS copy of the task's el rows.
// Edgeless rows: dense -> the column mean (empty_fill), sparse -> 0/0 = NaN; one-edge rows
// give the edge's Wh row (dense, weight exp(0) = 1) or (p Wh) / p (sparse), as the small-row
// path. Requires NCH == 1 and fh % VW == 0 (the launcher's condition).
template <int VW, int LPR, bool SPARSE, int U>
__device__ __forceinline__ void gat_packed_rows(const GatParams& P, int64_t t, int lane,
                                                float* __restrict__ el_lds) {
  constexpr int EPI = kWave / LPR;
  static_assert(LPR % U == 0, "a batch of U edges never straddles a chunk of LPR edges");
  const int sub = lane & (LPR - 1);
  const int grp = lane / LPR;
  const int32_t rb = P.task_row[2 * t];
  const int32_t re = P.task_row[2 * t + 1];
  if (rb < 0 || re <= rb || re - rb > kGatTaskRows || re > P.n_rows) return;
  const int nr = re - rb;
  const int H = P.heads;
  // the task's el rows into this wave's LDS slice (row r, head h at r * H + h)
  for (int i = lane; i < nr * H; i += kWave) {
    const int r = i / H, hh = i - r * H;
    el_lds[i] = P.el[static_cast<int64_t>(rb + r) * P.lde + hh];
  }
  const int64_t e0 = P.rowptr[rb];
  const int rp = static_cast<int>(P.rowptr[rb + min(lane, nr)] - e0);
  const int E = __shfl(rp, nr, kWave);
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
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int64_t f = static_cast<int64_t>(sub) * VW;
  const bool fok = f < P.feat;
  const int h = fok ? static_cast<int>(f / P.fh) : 0;
  int cur = sb;
  int cur_end = __shfl(rp, min(cur + 1, nr), kWave);
  const int es = __shfl(rp, sb, kWave);
  const int ee = __shfl(rp, se, kWave);
  int cur_beg = es;
  float eli = cur < se ? el_lds[cur * H + h] : 0.f;
  float m = SPARSE ? 0.f : -INFINITY, l = 0.f;
  typename Vec<VW>::T acc = vzero<VW>();

  auto flush_upto = [&](int pos) {
    bool need = cur < se && pos >= cur_end;
    while (__ballot(need)) {
      if (need) {
        const int64_t row = rb + cur;
        const bool empty = cur_beg == cur_end;
        if (P.stats && fok && f % P.fh == 0)
          P.stats[row * P.lds + h] = empty ? -INFINITY : (SPARSE ? 0.f : m) + __logf(l);
        if (fok) {
          typename Vec<VW>::T r;
          if (!SPARSE && empty)
            r = P.empty_fill ? vload<VW>(P.empty_fill + f) : typename Vec<VW>::T(NAN);
          else
            r = acc / l;  // sparse, no edge: 0/0 = NaN like the reference
#pragma unroll
          for (int k = 0; k < VW; ++k) vset(r, k, act_apply(vget(r, k), P.flags));
          vstore<VW>(P.out + row * P.ldo + f, r);
        }
        m = SPARSE ? 0.f : -INFINITY;
        l = 0.f;
        acc = vzero<VW>();
      }
      cur += need ? 1 : 0;
      const int nxt = __shfl(rp, min(cur + 1, nr), kWave);
      cur_beg = need ? cur_end : cur_beg;
      cur_end = need ? nxt : cur_end;
      if (need && cur < se) eli = el_lds[cur * H + h];
      need = cur < se && pos >= cur_end;
    }
  };

  int len = ee - es;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) len = max(len, __shfl_xor(len, o, kWave));
  flush_upto(es);  // leading rows without edges
  for (int off = 0; off < len; off += LPR) {
    const int cb = es + off;  // this slot's chunk: lane `sub` holds edge cb + sub
    const int c = cb + sub < ee ? P.col[e0 + cb + sub] : 0;
    const int n = min(LPR, len - off);  // wave-uniform
    for (int k = 0; k < n; k += U) {
      float erv[U];
      typename Vec<VW>::T xv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int ce = __shfl(c, grp * LPR + ((k + u) & (LPR - 1)), kWave);
        const bool ok = cb + k + u < ee;
        erv[u] = ok ? er_at(P, ce, h) : 0.f;
        xv[u] = (ok && fok) ? vload<VW>(wh_row(P, ce) + f) : vzero<VW>();
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        flush_upto(cb + k + u);  // rows that end before this edge
        if (cb + k + u < ee) {
          const float sv = eli + erv[u];
          const float x = sv > 0.f ? sv : P.slope * sv;
          float p;
          if (SPARSE) {
            p = __expf(-x);  // exp(-LeakyReLU), no max subtraction
          } else {
            if (x > m) {  // online softmax: rescale the row's state to the new maximum
              const float sc = __expf(m - x);  // 0 on the row's first edge (m = -inf)
              acc *= sc;
              l *= sc;
              m = x;
            }
            p = __expf(x - m);
          }
          l += p;
          float w = p;
          if (P.drop_p > 0.f) {
            const uint32_t r = hash3(P.drop_seed, e0 + cb + k + u, P.head0 + h);
            w = (static_cast<float>(r >> 8) * (1.0f / 16777216.0f) < P.drop_p) ? 0.f
                                                                                : w * P.drop_scale;
          }
          acc += w * xv[u];
        }
      }
    }
  }
  flush_upto(0x7fffffff);  // the last row and trailing rows without edges
}

template <int VW, int LPR, bool SPARSE>
__global__ __launch_bounds__(kGatBlock) void gat_task_kernel(GatParams P) {
  __shared__ float el_lds[kGatWaves][kGatTaskRows * kMaxHeads];
  const int wid = threadIdx.x >> 6;
  const int64_t t = static_cast<int64_t>(blockIdx.x) * kGatWaves + wid;
  if (t < P.n_task)
    gat_packed_rows<VW, LPR, SPARSE, (LPR < GNN_GAT_TASK_U ? LPR : GNN_GAT_TASK_U)>(
        P, t, threadIdx.x & (kWave - 1), el_lds[wid]);
}

#ifndef GNN_GAT_LDS_PAD
#define GNN_GAT_LDS_PAD 0  // A/B: dynamic LDS per workgroup to cap workgroups per CU
#endif
#ifdef GNN_GAT_WAVES_PER_EU
#define GNN_GAT_OCC __attribute__((amdgpu_waves_per_eu(GNN_GAT_WAVES_PER_EU)))
#else
#define GNN_GAT_OCC
#endif

// Edge-head layout (heads <= 8 per group, fh = 4 NF): lane (ae, ah) = (edge slot, head) holds
// head ah's fh features of edge ae's Wh row (NF float4 loads: 8 lanes read a 256-B row at fh = 8),
// so the score, the online softmax and the weighted sum all run lane-locally: no per-chunk lane
// permutes of column ids or weights (gat_csr_kernel moves both between its edge x head and
// feature layouts every chunk), one xor-butterfly over the edge slots per row at the end. With
// REC, er_j[ah] = a_dst[ah] . Wh_j[ah] comes from the lane's own slice (no er gather: 1.2 of
// the 4.1 GB the one-chunk kernel fetched at cfg3, profiles/r05r_*); U chunks of EPP edges are
// loaded before any is used. Segments and mid rows here, edgeless / one-edge rows as in
// gat_csr_kernel (gat_small_rows), short rows in gat_short_kernel.
template <int NF, int HP, bool SPARSE, bool REC, int LPR>
__global__ __launch_bounds__(kGatBlock) void gat_eh_kernel(GatParams P) {
  constexpr int EPP = kWave / HP;  // edges per chunk
  constexpr int U = 2;             // chunks loaded together
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t wave = static_cast<int64_t>(blockIdx.x) * kGatWaves + (threadIdx.x >> 6);
  const int ah = lane & (HP - 1);
  const int ae = lane / HP;
  int64_t row, beg, end;
  bool is_seg = false;
  if (wave < P.seg_waves) {
    if (wave >= P.n_seg) return;
    row = P.seg_row[wave];
    beg = P.seg_begin[wave];
    end = min(beg + P.seg_len, P.rowptr[row + 1]);
    is_seg = true;
  } else if (wave < P.seg_waves + P.mid_waves) {
    const int64_t i = wave - P.seg_waves;
    if (i >= P.n_mid) return;
    row = P.mid_row ? P.mid_row[i] : i;
    beg = P.rowptr[row];
    end = P.rowptr[row + 1];
  } else {
    gat_small_rows<4, LPR, 1, SPARSE, REC>(P, wave - P.seg_waves - P.mid_waves, lane);
    return;
  }
  const bool head_ok = ah < P.heads;
  const int64_t hoff = head_ok ? ah : 0;
  const int64_t fo = hoff * P.fh;  // the head's first feature
  const float eli = P.el[row * P.lde + hoff];
  f4 ad[NF];
#pragma unroll
  for (int v = 0; v < NF; ++v) ad[v] = REC ? vload<4>(P.a_dst + fo + 4 * v) : f4(0.f);
  float m = SPARSE ? 0.f : -INFINITY;
  float l = 0.f;
  f4 acc[NF];
#pragma unroll
  for (int v = 0; v < NF; ++v) acc[v] = f4(0.f);
  const float sgn = SPARSE ? -1.f : 1.f;
  int cn[U];
#pragma unroll
  for (int u = 0; u < U; ++u) cn[u] = beg + u * EPP + ae < end ? P.col[beg + u * EPP + ae] : 0;
  for (int64_t b = beg; b < end; b += U * EPP) {
    f4 x[U][NF];
    float erv[U];
    bool live[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      live[u] = b + u * EPP + ae < end && head_ok;
      const float* xr = wh_row(P, cn[u]) + fo;
#pragma unroll
      for (int v = 0; v < NF; ++v) x[u][v] = live[u] ? vload<4>(xr + 4 * v) : f4(0.f);
      if constexpr (!REC) erv[u] = live[u] ? er_at(P, cn[u], ah) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {  // the next U chunks' column ids while these rows land
      const int64_t e = b + (U + u) * EPP + ae;
      cn[u] = e < end ? P.col[e] : 0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (b + u * EPP >= end) break;  // uniform
      if constexpr (REC) {
        float s = 0.f;
#pragma unroll
        for (int v = 0; v < NF; ++v) {
          s = fmaf(x[u][v].x, ad[v].x, s);
          s = fmaf(x[u][v].y, ad[v].y, s);
          s = fmaf(x[u][v].z, ad[v].z, s);
          s = fmaf(x[u][v].w, ad[v].w, s);
        }
        erv[u] = s;
      }
      float z = -INFINITY;
      if (live[u]) {
        const float sv = eli + erv[u];
        z = sgn * (sv > 0.f ? sv : P.slope * sv);
      }
      float p;
      if (!SPARSE) {
        float pm = z;
#pragma unroll
        for (int o = HP; o < kWave; o <<= 1) pm = fmaxf(pm, __shfl_xor(pm, o, kWave));
        const float mn = fmaxf(m, pm);
        const float scale = __expf(m - mn);  // 0 on the first chunk (m = -inf)
        m = mn;
        p = z == -INFINITY ? 0.f : __expf(z - mn);
        l = l * scale + p;
#pragma unroll
        for (int v = 0; v < NF; ++v) acc[v] *= scale;
      } else {
        p = z == -INFINITY ? 0.f : __expf(z);  // exp(-LeakyReLU), no max subtraction
        l += p;
      }
      float w = p;
      if (P.drop_p > 0.f && live[u]) {
        const uint32_t r = hash3(P.drop_seed, b + u * EPP + ae, P.head0 + ah);
        w = (static_cast<float>(r >> 8) * (1.0f / 16777216.0f) < P.drop_p) ? 0.f : w * P.drop_scale;
      }
#pragma unroll
      for (int v = 0; v < NF; ++v) acc[v] += w * x[u][v];
    }
  }
  // the head's sums over the edge slots (every lane of the head ends with them)
#pragma unroll
  for (int o = HP; o < kWave; o <<= 1) {
    l += __shfl_xor(l, o, kWave);
#pragma unroll
    for (int v = 0; v < NF; ++v) acc[v] += shfl_xor_f(acc[v], o);
  }
  if (lane >= HP || !head_ok) return;
  if (is_seg) {
    float* pr = P.partial + wave * P.ldp;
#pragma unroll
    for (int v = 0; v < NF; ++v) vstore<4>(pr + fo + 4 * v, acc[v]);
    pr[P.feat + ah] = l;
    pr[P.feat + P.heads + ah] = m;
    return;
  }
  const bool empty = end == beg;
  if (P.stats) P.stats[row * P.lds + ah] = empty ? -INFINITY : (SPARSE ? 0.f : m) + __logf(l);
  float* orow = P.out + row * P.ldo + fo;
#pragma unroll
  for (int v = 0; v < NF; ++v) {
    f4 r;
    if (!SPARSE && empty)
      r = P.empty_fill ? vload<4>(P.empty_fill + fo + 4 * v) : f4(NAN);
    else
      r = acc[v] / l;  // sparse, no edge: 0/0 = NaN like the reference
#pragma unroll
    for (int k = 0; k < 4; ++k) r[k] = act_apply(r[k], P.flags);
    vstore<4>(orow + 4 * v, r);
  }
}

template <int VW, int LPR, int NCH, int HP, bool SPARSE, int U, int J, bool REC>
__global__ __launch_bounds__(kGatBlock) GNN_GAT_OCC void gat_csr_kernel(GatParams P) {
  constexpr int EPI = kWave / LPR;  // phase B: edges per gather instruction
  constexpr int EPP = kWave / HP;   // phase A: edges per pass (lane = edge x head)
  constexpr int C = EPP * J;        // edges per chunk
  static_assert(J == 1 || (EPI <= EPP && EPP % EPI == 0), "multi-pass chunks need EPI | EPP");
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t wave = static_cast<int64_t>(blockIdx.x) * kGatWaves + (threadIdx.x >> 6);
  const int sub = lane & (LPR - 1);
  const int grp = lane / LPR;
  const int ah = lane & (HP - 1);  // phase-A head of this lane
  const int ae = lane / HP;        // phase-A edge slot of this lane

  int64_t row, beg, end;
  bool is_seg = false;
  if (wave < P.seg_waves) {
    if (wave >= P.n_seg) return;
    row = P.seg_row[wave];
    beg = P.seg_begin[wave];
    end = min(beg + P.seg_len, P.rowptr[row + 1]);
    is_seg = true;
  } else if (wave < P.seg_waves + P.mid_waves) {
    const int64_t i = wave - P.seg_waves;
    if (i >= P.n_mid) return;
    row = P.mid_row ? P.mid_row[i] : i;
    beg = P.rowptr[row];
    end = P.rowptr[row + 1];
  } else if (NCH > 1 && wave < P.seg_waves + P.mid_waves + P.short_waves) {
    // wide rows (NCH > 1) only: short rows take the one-row-per-wave path here;
    // otherwise they have their own launch (gat_short_kernel, own register budget)
    const int64_t i = wave - P.seg_waves - P.mid_waves;
    if (i >= P.n_short) return;
    row = P.short_row[i];
    beg = P.rowptr[row];
    end = P.rowptr[row + 1];
  } else {
    gat_small_rows<VW, LPR, NCH, SPARSE, REC>(
        P, wave - P.seg_waves - P.mid_waves - P.short_waves, lane);
    return;
  }
  const bool head_ok = ah < P.heads;
  const float eli = head_ok ? P.el[row * P.lde + ah] : 0.f;
  float m = SPARSE ? 0.f : -INFINITY;  // running max of head `ah` (uniform over its lanes)
  float lsum = 0.f;                     // lane-local partial denominator of head `ah`
  int hid[NCH];
  typename Vec<VW>::T acc[NCH];
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    const int64_t f = static_cast<int64_t>(ch * LPR + sub) * VW;
    hid[ch] = f < P.feat ? static_cast<int>(f / P.fh) : 0;
    acc[ch] = vzero<VW>();
  }

  constexpr int CE = (C + EPI - 1) / EPI;  // gather slots per chunk
  if constexpr (GNN_GAT_PIPE && J == 1 && NCH == 1 && CE <= 4) {
    // Pipelined chunk loop: the next chunk's column ids are loaded while this chunk is
    // processed, and this chunk's er entries and Wh rows are issued together, before the
    // softmax arithmetic -- one memory round trip per chunk instead of col -> er -> Wh.
    // Same arithmetic in the same order as the loop below (bit-identical results).
    int c_next = ae < end - beg ? P.col[beg + ae] : 0;
    constexpr bool rec = REC;
    const int64_t f0 = static_cast<int64_t>(sub) * VW;
    const typename Vec<VW>::T adst = (rec && f0 < P.feat) ? vload<VW>(P.a_dst + f0) : vzero<VW>();
    // this chunk's Wh rows: CE gather slots, EPI edges per slot
    auto load_rows = [&](int cj, int np, typename Vec<VW>::T (&xv)[CE]) {
#pragma unroll
      for (int q = 0; q < CE; ++q) {
        const int e = q * EPI + grp;
        const int ce = __shfl(cj, (e < EPP ? e : 0) * HP, kWave);
        xv[q] = (e < np && f0 < P.feat) ? vload<VW>(wh_row(P, ce) + f0) : vzero<VW>();
      }
    };
    // softmax update and accumulation of one chunk with its gathered er values
    auto consume = [&](int64_t b, int np, float erv, const typename Vec<VW>::T (&xv)[CE]) {
      const bool live = ae < np && head_ok;
      float z = -INFINITY;
      if (live) {
        const float sv = eli + erv;
        const float x = sv > 0.f ? sv : P.slope * sv;
        z = SPARSE ? -x : x;
      }
      float pv;
      if (!SPARSE) {
        float pm = z;
#pragma unroll
        for (int o = HP; o < kWave; o <<= 1) pm = fmaxf(pm, __shfl_xor(pm, o, kWave));
        const float mn = fmaxf(m, pm);
        const float scale = __expf(m - mn);  // 0 on the first chunk (m = -inf)
        m = mn;
        pv = z == -INFINITY ? 0.f : __expf(z - mn);
        lsum = lsum * scale + pv;
        acc[0] *= __shfl(scale, hid[0], kWave);
      } else {
        pv = z == -INFINITY ? 0.f : __expf(z);  // exp(-LeakyReLU), no max subtraction
        lsum += pv;
      }
#pragma unroll
      for (int q = 0; q < CE; ++q) {
        const int e = q * EPI + grp;
        const bool ok = e < np && f0 < P.feat;
        float wv = __shfl(pv, (e < EPP ? e : 0) * HP + hid[0], kWave);
        if (P.drop_p > 0.f && ok) {
          const uint32_t r = hash3(P.drop_seed, b + e, P.head0 + hid[0]);
          wv = (static_cast<float>(r >> 8) * (1.0f / 16777216.0f) < P.drop_p) ? 0.f
                                                                               : wv * P.drop_scale;
        }
        acc[0] += (ok ? wv : 0.f) * xv[q];
      }
    };
    auto chunk_np = [&](int64_t b) {
      return b < end ? static_cast<int>(min(static_cast<int64_t>(C), end - b)) : 0;
    };
    auto next_col = [&](int64_t b) { return (b < end && b + ae < end) ? P.col[b + ae] : 0; };
    if constexpr (rec) {
      // er comes with the rows: the whole chunk runs in the feature layout -- lane (sub, grp)
      // holds edge q EPI + grp of slot q for its head hid[0]: er and z per slot from its own
      // row slice (xor-summed over the head's er_g lanes), the chunk max over the slots and
      // lane groups (xor shuffles), a lane-partial denominator. No phase-A layout, so none of
      // the per-slot column-id / weight / scale lane permutes; one permute at the end hands
      // the denominator and max to the epilogue's phase-A lanes. (4 slots per chunk: 0.93 ms,
      // the next chunk's rows kept in flight: 1.02 ms, against 0.79 for this form at cfg3 --
      // register-bound occupancy, profiles/r05p_gat_ab.log.)
      constexpr int RS = CE;
      constexpr int CR = RS * EPI;
      const float elh = P.el[row * P.lde + hid[0]];
      const bool fok = f0 < P.feat;
      float mh = SPARSE ? 0.f : -INFINITY;
      float lh = 0.f;
      auto cols = [&](int64_t b, int (&c)[RS]) {
#pragma unroll
        for (int q = 0; q < RS; ++q) {
          const int64_t e = b + q * EPI + grp;
          c[q] = e < end ? P.col[e] : 0;
        }
      };
      auto rows = [&](int64_t b, const int (&c)[RS], typename Vec<VW>::T (&xv)[RS]) {
#pragma unroll
        for (int q = 0; q < RS; ++q)
          xv[q] = (b + q * EPI + grp < end && fok) ? vload<VW>(wh_row(P, c[q]) + f0) : vzero<VW>();
      };
      auto use = [&](int64_t b, const typename Vec<VW>::T (&xv)[RS]) {
        float z[RS];
#pragma unroll
        for (int q = 0; q < RS; ++q) {
          const float sv = elh + er_reduce(er_partial<VW>(xv[q], adst), P.er_g);
          const float x = sv > 0.f ? sv : P.slope * sv;
          z[q] = b + q * EPI + grp < end ? (SPARSE ? -x : x) : -INFINITY;
        }
        if (!SPARSE) {
          float cm = z[0];
#pragma unroll
          for (int q = 1; q < RS; ++q) cm = fmaxf(cm, z[q]);
#pragma unroll
          for (int o = LPR; o < kWave; o <<= 1) cm = fmaxf(cm, __shfl_xor(cm, o, kWave));
          const float mn = fmaxf(mh, cm);
          const float scale = __expf(mh - mn);  // 0 on the first chunk (mh = -inf)
          mh = mn;
          lh *= scale;
          acc[0] *= scale;
        }
#pragma unroll
        for (int q = 0; q < RS; ++q) {
          const int64_t e = b + q * EPI + grp;
          const float p = z[q] == -INFINITY ? 0.f : (SPARSE ? __expf(z[q]) : __expf(z[q] - mh));
          lh += p;
          float wv = p;
          if (P.drop_p > 0.f && e < end) {
            const uint32_t r = hash3(P.drop_seed, e, P.head0 + hid[0]);
            wv = (static_cast<float>(r >> 8) * (1.0f / 16777216.0f) < P.drop_p) ? 0.f
                                                                                 : wv * P.drop_scale;
          }
          acc[0] += (e < end && fok ? wv : 0.f) * xv[q];
        }
      };
      int cn[RS];
      cols(beg, cn);
      for (int64_t b = beg; b < end; b += CR) {
        typename Vec<VW>::T xv[RS];
        rows(b, cn, xv);
        cols(b + CR, cn);  // the next chunk's column ids while this chunk's rows are in flight
        use(b, xv);
      }
      // the head's denominator over every lane group, then into the epilogue's layout: phase-A
      // lane (0, ah) holds it (the epilogue sums the edge slots), every lane the head's max
#pragma unroll
      for (int o = LPR; o < kWave; o <<= 1) lh += __shfl_xor(lh, o, kWave);
      const int src = (ah * P.er_g) & (kWave - 1);
      const float lA = __shfl(lh, src, kWave);
      const float mA = __shfl(mh, src, kWave);
      lsum = ae == 0 ? lA : 0.f;
      if (!SPARSE) m = mA;
    } else {
      // er runs one chunk ahead of the rows: chunk k + 1's er (and chunk k + 2's column ids)
      // load while chunk k's rows are in flight, so chunk k's softmax arithmetic needs only
      // values already in registers and runs under its rows' latency; only the weighted sum
      // waits for them. (er issued beside the rows, the softmax waited for both: a probe
      // without er loads ran 0.605 against 0.777 ms, profiles/r05j_gat_noer_ab.log.)
      int cj = c_next;
      float erv = (ae < chunk_np(beg) && head_ok) ? er_at(P, cj, ah) : 0.f;
      c_next = next_col(beg + C);
      for (int64_t b = beg; b < end; b += C) {
        const int np = chunk_np(b);
        typename Vec<VW>::T xv[CE];
        load_rows(cj, np, xv);
        const float er_n = (ae < chunk_np(b + C) && head_ok) ? er_at(P, c_next, ah) : 0.f;
        const int c_n2 = next_col(b + 2 * C);
        consume(b, np, erv, xv);
        cj = c_next;
        erv = er_n;
        c_next = c_n2;
      }
    }
  } else
  // A chunk is J phase-A passes (C = J * EPP edges): every lane issues its J column
  // and J er loads at once, then the whole chunk's feature rows are gathered in
  // C / EPI slots -- one dependent round trip per chunk instead of per pass.
  for (int64_t b = beg; b < end; b += C) {
    const int np = static_cast<int>(min(static_cast<int64_t>(C), end - b));
    // ---- phase A: lane (edge j * EPP + ae, head ah)
    int cj[J];
    float zj[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int e = j * EPP + ae;
      cj[j] = e < np ? P.col[b + e] : 0;
    }
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const bool live = j * EPP + ae < np && head_ok;
      zj[j] = -INFINITY;
      if (live) {
        const float sv = eli + er_at(P, cj[j], ah);
        const float x = sv > 0.f ? sv : P.slope * sv;
        zj[j] = SPARSE ? -x : x;
      }
    }
    float pj[J];
    if (!SPARSE) {
      float pm = zj[0];
#pragma unroll
      for (int j = 1; j < J; ++j) pm = fmaxf(pm, zj[j]);
#pragma unroll
      for (int o = HP; o < kWave; o <<= 1) pm = fmaxf(pm, __shfl_xor(pm, o, kWave));
      const float mn = fmaxf(m, pm);
      const float scale = __expf(m - mn);  // 0 on the first chunk (m = -inf)
      m = mn;
      float ps = 0.f;
#pragma unroll
      for (int j = 0; j < J; ++j) {
        pj[j] = zj[j] == -INFINITY ? 0.f : __expf(zj[j] - mn);
        ps += pj[j];
      }
      lsum = lsum * scale + ps;
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) acc[ch] *= __shfl(scale, hid[ch], kWave);
    } else {
#pragma unroll
      for (int j = 0; j < J; ++j) {
        pj[j] = zj[j] == -INFINITY ? 0.f : __expf(zj[j]);  // exp(-LeakyReLU), no max subtraction
        lsum += pj[j];
      }
    }
    // ---- phase B: lanes = features, EPI edges per gather instruction, U in flight
#pragma unroll 1
    for (int k0 = 0; k0 < C / EPI; k0 += U) {
      if (k0 * EPI >= np) break;
      typename Vec<VW>::T xv[U][NCH];
      float w[U][NCH];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = (k0 + u) * EPI + grp;                 // edge within the chunk
        const int j = J == 1 ? 0 : ((k0 + u) * EPI) / EPP;  // uniform: EPI <= EPP when J > 1
        const int es = (J == 1 ? (e < EPP ? e : 0) : (e - j * EPP)) * HP;
        int cv = cj[0];
        float pv = pj[0];
#pragma unroll
        for (int jj = 1; jj < J; ++jj)
          if (jj == j) { cv = cj[jj]; pv = pj[jj]; }
        const int ce = __shfl(cv, es, kWave);
        const float* xr = wh_row(P, ce);
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) {
          const int64_t f = static_cast<int64_t>(ch * LPR + sub) * VW;
          const bool ok = e < np && f < P.feat;
          float wv = __shfl(pv, es + hid[ch], kWave);
          xv[u][ch] = ok ? vload<VW>(xr + f) : vzero<VW>();
          if (P.drop_p > 0.f && ok) {
            const uint32_t r = hash3(P.drop_seed, b + e, P.head0 + hid[ch]);
            wv = (static_cast<float>(r >> 8) * (1.0f / 16777216.0f) < P.drop_p) ? 0.f
                                                                                 : wv * P.drop_scale;
          }
          w[u][ch] = ok ? wv : 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) acc[ch] += w[u][ch] * xv[u][ch];
      }
    }
  }

  // ---- epilogue
#pragma unroll
  for (int mm = LPR; mm < kWave; mm <<= 1) {
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) acc[ch] += shfl_xor_f(acc[ch], mm);
  }
#pragma unroll
  for (int o = HP; o < kWave; o <<= 1) lsum += __shfl_xor(lsum, o, kWave);  // per head, all lanes

  if (is_seg) {
    float* pr = P.partial + wave * P.ldp;
    if (lane < LPR) {
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) {
        const int64_t f = static_cast<int64_t>(ch * LPR + sub) * VW;
        if (f < P.feat) vstore<VW>(pr + f, acc[ch]);
      }
    }
    if (lane < HP && head_ok) {
      pr[P.feat + lane] = lsum;
      pr[P.feat + P.heads + lane] = m;
    }
    return;
  }
  if (P.stats && lane < HP && head_ok)
    P.stats[row * P.lds + lane] = end == beg ? -INFINITY : (SPARSE ? 0.f : m) + __logf(lsum);
  const bool empty = end == beg;
  float lh[NCH];
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) lh[ch] = __shfl(lsum, hid[ch], kWave);
  if (lane >= LPR) return;
  float* orow = P.out + row * P.ldo;
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    const int64_t f = static_cast<int64_t>(ch * LPR + sub) * VW;
    if (f >= P.feat) continue;
    typename Vec<VW>::T r;
    if (!SPARSE && empty) {
      r = P.empty_fill ? vload<VW>(P.empty_fill + f) : typename Vec<VW>::T(NAN);
    } else {
      r = acc[ch] / lh[ch];  // sparse, no edge: 0/0 = NaN like the reference
    }
#pragma unroll
    for (int i = 0; i < VW; ++i) vset(r, i, act_apply(vget(r, i), P.flags));
    vstore<VW>(orow + f, r);
  }
}

// Merge the (acc, l, m) partial states of each long row with the log-sum-exp rule
// (m = 0 for sparse). One workgroup per long row: pass 1 takes the max of the
// segment maxima, pass 2 sums the rescaled partials; segments are spread over
// the 4 waves x EPI slots and combined in a fixed order (xor tree, then LDS):
// no serial tail for the hub rows, bitwise reproducible.
template <int VW, int LPR, int NCH, bool SPARSE>
__global__ __launch_bounds__(kGatBlock) void gat_fixup_kernel(GatParams P) {
  constexpr int EPI = kWave / LPR;
  constexpr int STRIDE = kGatWaves * EPI;
  __shared__ typename Vec<VW>::T red_a[kGatWaves][NCH][LPR];
  __shared__ float red_s[kGatWaves][NCH][LPR];
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x >> 6;
  const int64_t i = blockIdx.x;
  if (i >= P.n_long) return;
  const int sub = lane & (LPR - 1);
  const int grp = lane / LPR;
  const int32_t s0 = P.long_seg_ptr[i], s1 = P.long_seg_ptr[i + 1];
  const int64_t row = P.long_row[i];
  int hid[NCH];
  float M[NCH];
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    const int64_t f = static_cast<int64_t>(ch * LPR + sub) * VW;
    hid[ch] = f < P.feat ? static_cast<int>(f / P.fh) : 0;
    M[ch] = SPARSE ? 0.f : -INFINITY;
  }
  if (!SPARSE) {  // pass 1: max of the segment maxima per head
    for (int32_t s = s0 + wid * EPI + grp; s < s1; s += STRIDE) {
      const float* pm = P.partial + static_cast<int64_t>(s) * P.ldp + P.feat + P.heads;
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) M[ch] = fmaxf(M[ch], pm[hid[ch]]);
    }
#pragma unroll
    for (int o = LPR; o < kWave; o <<= 1) {
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) M[ch] = fmaxf(M[ch], __shfl_xor(M[ch], o, kWave));
    }
    if (lane < LPR) {
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) red_s[wid][ch][lane] = M[ch];
    }
    __syncthreads();
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      float v = red_s[0][ch][sub];
#pragma unroll
      for (int w = 1; w < kGatWaves; ++w) v = fmaxf(v, red_s[w][ch][sub]);
      M[ch] = v;
    }
    __syncthreads();
  }
  // pass 2: rescaled sums of acc and l
  typename Vec<VW>::T a[NCH];
  float l[NCH];
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    a[ch] = vzero<VW>();
    l[ch] = 0.f;
  }
  for (int32_t s = s0 + wid * EPI + grp; s < s1; s += STRIDE) {
    const float* pr = P.partial + static_cast<int64_t>(s) * P.ldp;
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      const int64_t f = static_cast<int64_t>(ch * LPR + sub) * VW;
      if (f >= P.feat) continue;
      const float sc = SPARSE ? 1.f : __expf(pr[P.feat + P.heads + hid[ch]] - M[ch]);
      a[ch] += sc * vload<VW>(pr + f);
      l[ch] += sc * pr[P.feat + hid[ch]];
    }
  }
#pragma unroll
  for (int o = LPR; o < kWave; o <<= 1) {
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      a[ch] += shfl_xor_f(a[ch], o);
      l[ch] += __shfl_xor(l[ch], o, kWave);
    }
  }
  if (lane < LPR) {
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      red_a[wid][ch][lane] = a[ch];
      red_s[wid][ch][lane] = l[ch];
    }
  }
  __syncthreads();
  if (wid != 0 || lane >= LPR) return;
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    const int64_t f = static_cast<int64_t>(ch * LPR + sub) * VW;
    if (f >= P.feat) continue;
    typename Vec<VW>::T av = red_a[0][ch][lane];
    float lv = red_s[0][ch][lane];
#pragma unroll
    for (int w = 1; w < kGatWaves; ++w) {
      av += red_a[w][ch][lane];
      lv += red_s[w][ch][lane];
    }
    if (P.stats && f % P.fh == 0) P.stats[row * P.lds + hid[ch]] = M[ch] + __logf(lv);
    typename Vec<VW>::T r = av / lv;
#pragma unroll
    for (int k = 0; k < VW; ++k) vset(r, k, act_apply(vget(r, k), P.flags));
    vstore<VW>(P.out + row * P.ldo + f, r);
  }
}

template <int VW, int LPR, int NCH, int HP, bool SPARSE>
static void launch_gat(const GatParams& P, hipStream_t s) {
  // phase B covers a pass of 64/HP edges in ceil(EPP/EPI) gather instructions
  constexpr int EPI = kWave / LPR, EPP = kWave / HP;
  // chunk = J passes (~32 edges) when an EPI group never straddles two passes
  constexpr int J = (EPI <= EPP && EPP % EPI == 0 && EPP < GNN_GAT_CHUNK && NCH == 1)
                        ? GNN_GAT_CHUNK / EPP : 1;
  constexpr int CE = (EPP * J + EPI - 1) / EPI;  // gather slots per chunk
  constexpr int U = NCH >= 2 ? 1 : (CE < GNN_GAT_U ? CE : GNN_GAT_U);
  const int64_t seg_blocks = (P.n_seg + kGatWaves - 1) / kGatWaves;
  const int64_t mid_blocks = (P.n_mid + kGatWaves - 1) / kGatWaves;
  // NCH == 1: short rows in their own launch, EPI rows per wave; else one wave per row here
  const int64_t short_waves = NCH == 1 ? 0 : P.n_short;
  const int64_t short_blocks = (short_waves + kGatWaves - 1) / kGatWaves;
  constexpr int SU = gat_small_unroll<NCH>();
  const int64_t small_waves = (P.n_small + EPI * SU - 1) / (EPI * SU);
  const int64_t small_blocks = (small_waves + kGatWaves - 1) / kGatWaves;
  GatParams Q = P;
  Q.seg_waves = seg_blocks * kGatWaves;
  Q.mid_waves = mid_blocks * kGatWaves;
  Q.short_waves = short_blocks * kGatWaves;
  const int64_t blocks = seg_blocks + mid_blocks + short_blocks + small_blocks;
  // the edge-head layout kernel when a head's features are 1, 2 or 4 float4 (GNN_GAT_EH)
  if constexpr (VW == 4 && NCH == 1 && HP <= 8) {
    const int nf = static_cast<int>(P.fh / 4);
    if (GNN_GAT_EH && P.fh % 4 == 0 && (nf == 1 || nf == 2 || nf == 4) && blocks - short_blocks > 0 &&
        short_blocks == 0) {
      const dim3 grid(static_cast<unsigned>(blocks));
#define GNN_EH(NFV)                                                                         \
  do {                                                                                      \
    if (P.a_dst != nullptr)                                                                 \
      hipLaunchKernelGGL((gat_eh_kernel<NFV, HP, SPARSE, true, LPR>), grid, dim3(kGatBlock), \
                         0, s, Q);                                                          \
    else                                                                                    \
      hipLaunchKernelGGL((gat_eh_kernel<NFV, HP, SPARSE, false, LPR>), grid, dim3(kGatBlock),\
                         0, s, Q);                                                          \
  } while (0)
      if (nf == 1)
        GNN_EH(1);
      else if (nf == 2)
        GNN_EH(2);
      else
        GNN_EH(4);
#undef GNN_EH
      goto after_main;
    }
  }
  {
  // er recomputed from the gathered rows: separate instances (the gathering loop's registers
  // do not weigh on the recomputing one), only where the one-chunk loop runs
  constexpr bool kRec = GNN_GAT_PIPE && J == 1 && NCH == 1 && CE <= 4;
  if (blocks > 0) {
    if constexpr (kRec) {
      if (P.a_dst != nullptr) {
        hipLaunchKernelGGL((gat_csr_kernel<VW, LPR, NCH, HP, SPARSE, U, J, true>),
                           dim3(static_cast<unsigned>(blocks)), dim3(kGatBlock), GNN_GAT_LDS_PAD,
                           s, Q);
      } else {
        hipLaunchKernelGGL((gat_csr_kernel<VW, LPR, NCH, HP, SPARSE, U, J, false>),
                           dim3(static_cast<unsigned>(blocks)), dim3(kGatBlock), GNN_GAT_LDS_PAD,
                           s, Q);
      }
    } else {
      hipLaunchKernelGGL((gat_csr_kernel<VW, LPR, NCH, HP, SPARSE, U, J, false>),
                         dim3(static_cast<unsigned>(blocks)), dim3(kGatBlock), GNN_GAT_LDS_PAD, s,
                         Q);
    }
  }
  }
after_main:
  if constexpr (NCH == 1) {
    if (P.n_task > 0) {
      hipLaunchKernelGGL((gat_task_kernel<VW, LPR, SPARSE>),
                         dim3(static_cast<unsigned>((P.n_task + kGatWaves - 1) / kGatWaves)),
                         dim3(kGatBlock), 0, s, Q);
    }
    if (P.n_short > 0) {
      const int64_t sw = (P.n_short + EPI - 1) / EPI;
      const dim3 grid(static_cast<unsigned>((sw + kGatWaves - 1) / kGatWaves));
      if (P.a_dst != nullptr)
        hipLaunchKernelGGL((gat_short_kernel<VW, LPR, SPARSE, true>), grid, dim3(kGatBlock), 0, s, Q);
      else
        hipLaunchKernelGGL((gat_short_kernel<VW, LPR, SPARSE, false>), grid, dim3(kGatBlock), 0, s, Q);
    }
  }
  if (P.n_long > 0)
    hipLaunchKernelGGL((gat_fixup_kernel<VW, LPR, NCH, SPARSE>),
                       dim3(static_cast<unsigned>(P.n_long)), dim3(kGatBlock), 0, s, Q);
}

template <int VW, int HP, bool SPARSE>
static int dispatch_gat_lpr(const GatParams& P, hipStream_t s) {
  const int64_t nv = (P.feat + VW - 1) / VW;
  if (nv <= 64) {
    switch (next_pow2_le64(nv)) {
      case 1: launch_gat<VW, 1, 1, HP, SPARSE>(P, s); break;
      case 2: launch_gat<VW, 2, 1, HP, SPARSE>(P, s); break;
      case 4: launch_gat<VW, 4, 1, HP, SPARSE>(P, s); break;
      case 8: launch_gat<VW, 8, 1, HP, SPARSE>(P, s); break;
      case 16: launch_gat<VW, 16, 1, HP, SPARSE>(P, s); break;
      case 32: launch_gat<VW, 32, 1, HP, SPARSE>(P, s); break;
      default: launch_gat<VW, 64, 1, HP, SPARSE>(P, s); break;
    }
  } else if (nv <= 128) {
    launch_gat<VW, 64, 2, HP, SPARSE>(P, s);
  } else if (nv <= 256) {
    launch_gat<VW, 64, 4, HP, SPARSE>(P, s);
  } else {
    return GNN_E_UNSUPPORTED;
  }
  return launch_status();
}

template <int VW, bool SPARSE>
static int dispatch_gat(const GatParams& P, hipStream_t s) {
  if (P.heads <= 1) return dispatch_gat_lpr<VW, 1, SPARSE>(P, s);
  if (P.heads <= 2) return dispatch_gat_lpr<VW, 2, SPARSE>(P, s);
  if (P.heads <= 4) return dispatch_gat_lpr<VW, 4, SPARSE>(P, s);
  return dispatch_gat_lpr<VW, 8, SPARSE>(P, s);
}

// el[n, h] = sum_f Wh[n, h*fh + f] * a_src[h*fh + f]; er likewise with a_dst.
__global__ __launch_bounds__(256) void gat_logits_kernel(const float* __restrict__ wh, int64_t ldw,
                                                         int64_t n_rows, int64_t heads, int64_t fh,
                                                         const float* __restrict__ a_src,
                                                         const float* __restrict__ a_dst,
                                                         float* __restrict__ el,
                                                         float* __restrict__ er, int64_t lde) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= n_rows * heads) return;
  const int64_t n = t / heads, h = t % heads;
  const float* x = wh + n * ldw + h * fh;
  const float* as = a_src + h * fh;
  const float* ad = a_dst + h * fh;
  float sl = 0.f, sr = 0.f;
  for (int64_t f = 0; f < fh; ++f) {
    const float v = x[f];
    sl = fmaf(v, as[f], sl);
    sr = fmaf(v, ad[f], sr);
  }
  el[n * lde + h] = sl;
  er[n * lde + h] = sr;
}

// Vector form of gat_logits_kernel for fh % 4 == 0 and 16-B aligned rows: a lane per
// (node, head) loads its head's fh floats as float4 (a wave reads 64 contiguous head
// slices), 32-bit index math. Same fmaf order over f as the scalar kernel.
__global__ __launch_bounds__(256) void gat_logits_vec_kernel(const float* __restrict__ wh,
                                                             uint32_t ldw4, uint32_t total,
                                                             uint32_t heads, uint32_t fh4,
                                                             const float* __restrict__ a_src,
                                                             const float* __restrict__ a_dst,
                                                             float* __restrict__ el,
                                                             float* __restrict__ er, uint32_t lde) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const uint32_t n = t / heads, h = t - n * heads;
  const float4* x = reinterpret_cast<const float4*>(wh) + static_cast<uint64_t>(n) * ldw4 + h * fh4;
  const float4* as = reinterpret_cast<const float4*>(a_src) + h * fh4;
  const float4* ad = reinterpret_cast<const float4*>(a_dst) + h * fh4;
  float sl = 0.f, sr = 0.f;
  for (uint32_t k = 0; k < fh4; ++k) {
    const float4 v = x[k];
    const float4 a = as[k], d = ad[k];
    sl = fmaf(v.x, a.x, sl); sr = fmaf(v.x, d.x, sr);
    sl = fmaf(v.y, a.y, sl); sr = fmaf(v.y, d.y, sr);
    sl = fmaf(v.z, a.z, sl); sr = fmaf(v.z, d.z, sr);
    sl = fmaf(v.w, a.w, sl); sr = fmaf(v.w, d.w, sr);
  }
  el[static_cast<uint64_t>(n) * lde + h] = sl;
  er[static_cast<uint64_t>(n) * lde + h] = sr;
}

// out[f] = mean over rows of x[:, f] (double accumulation; two passes, deterministic).
constexpr int kMeanRows = 4096;
__global__ __launch_bounds__(256) void col_sum_partial_kernel(const float* __restrict__ x,
                                                              int64_t ldx, int64_t n_rows,
                                                              int64_t feat,
                                                              double* __restrict__ part) {
  const int64_t f = static_cast<int64_t>(blockIdx.y) * blockDim.x + threadIdx.x;
  if (f >= feat) return;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * kMeanRows;
  const int64_t r1 = min(r0 + kMeanRows, n_rows);
  double s = 0.0;
  for (int64_t r = r0; r < r1; ++r) s += static_cast<double>(x[r * ldx + f]);
  part[static_cast<int64_t>(blockIdx.x) * feat + f] = s;
}
__global__ __launch_bounds__(256) void col_mean_final_kernel(const double* __restrict__ part,
                                                             int64_t nblk, int64_t n_rows,
                                                             int64_t feat, float* __restrict__ out) {
  const int64_t f = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (f >= feat) return;
  double s = 0.0;
  for (int64_t b = 0; b < nblk; ++b) s += part[b * feat + f];
  out[f] = static_cast<float>(s / static_cast<double>(n_rows));
}

}  // namespace gnn

using namespace gnn;

extern "C" int gnn_gat_logits_f32(const float* wh, int64_t ldw, int64_t n_rows, int64_t heads,
                                  int64_t fh, const float* a_src, const float* a_dst, float* el,
                                  float* er, int64_t lde, void* stream) {
  if (n_rows < 0 || heads < 1 || fh < 1 || ldw < heads * fh || lde < heads) return GNN_E_ARG;
  if (n_rows == 0) return GNN_OK;
  if (!wh || !a_src || !a_dst || !el || !er) return GNN_E_ARG;
  const int64_t total = n_rows * heads;
  const bool aligned = ((reinterpret_cast<uintptr_t>(wh) | reinterpret_cast<uintptr_t>(a_src) |
                         reinterpret_cast<uintptr_t>(a_dst)) & 15) == 0;
  if (aligned && fh % 4 == 0 && ldw % 4 == 0 && total < (int64_t{1} << 31) &&
      ldw < (int64_t{1} << 31) && lde < (int64_t{1} << 31)) {
    hipLaunchKernelGGL(gat_logits_vec_kernel, dim3(static_cast<unsigned>((total + 255) / 256)),
                       dim3(256), 0, static_cast<hipStream_t>(stream), wh,
                       static_cast<uint32_t>(ldw / 4), static_cast<uint32_t>(total),
                       static_cast<uint32_t>(heads), static_cast<uint32_t>(fh / 4), a_src, a_dst,
                       el, er, static_cast<uint32_t>(lde));
    return launch_status();
  }
  hipLaunchKernelGGL(gat_logits_kernel, dim3(static_cast<unsigned>((total + 255) / 256)), dim3(256),
                     0, static_cast<hipStream_t>(stream), wh, ldw, n_rows, heads, fh, a_src, a_dst,
                     el, er, lde);
  return launch_status();
}

extern "C" int64_t gnn_col_mean_scratch_bytes(int64_t n_rows, int64_t feat) {
  if (n_rows < 0 || feat < 0) return GNN_E_ARG;
  return ((n_rows + kMeanRows - 1) / kMeanRows) * feat * static_cast<int64_t>(sizeof(double));
}

extern "C" int gnn_col_mean_f32(const float* x, int64_t ldx, int64_t n_rows, int64_t feat,
                                float* out, void* scratch, void* stream) {
  if (n_rows < 1 || feat < 1 || ldx < feat || !x || !out || !scratch) return GNN_E_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t nblk = (n_rows + kMeanRows - 1) / kMeanRows;
  if (nblk > 0x7fffffffLL || (feat + 255) / 256 > 65535) return GNN_E_UNSUPPORTED;
  double* part = static_cast<double*>(scratch);
  hipLaunchKernelGGL(col_sum_partial_kernel,
                     dim3(static_cast<unsigned>(nblk), static_cast<unsigned>((feat + 255) / 256)),
                     dim3(256), 0, s, x, ldx, n_rows, feat, part);
  hipLaunchKernelGGL(col_mean_final_kernel, dim3(static_cast<unsigned>((feat + 255) / 256)),
                     dim3(256), 0, s, part, nblk, n_rows, feat, out);
  return launch_status();
}

static int gat_entry(const int64_t* rowptr, const int32_t* col, int64_t n_rows,
                     const float* wh, int64_t ldw, int64_t heads, int64_t fh,
                     const float* el, const float* er, int64_t lde, float negative_slope,
                     int32_t mode, const float* empty_row_fill, float dropout_p,
                     uint64_t dropout_seed, float* out, int64_t ldo, int64_t seg_len,
                     const int32_t* seg_row, const int64_t* seg_begin, int64_t n_seg,
                     const int32_t* long_row, const int32_t* long_seg_ptr,
                     int64_t n_long, const int32_t* small_row, const int32_t* small_col,
                     int64_t n_small, const int32_t* mid_row, int64_t n_mid,
                     const int32_t* short_row, int64_t n_short,
                     float* partial, float* stats, uint32_t flags, void* stream,
                     const float* whh, int64_t ldwh, const float* erh, int64_t ldeh,
                     const int32_t* task_row = nullptr, int64_t n_task = 0,
                     const float* a_dst = nullptr) {
  if (n_rows < 0 || heads < 1 || fh < 1 || seg_len < 1 || n_seg < 0 || n_long < 0 || n_small < 0)
    return GNN_E_ARG;
  if (n_task < 0 || (n_task > 0 && (task_row == nullptr || mid_row == nullptr))) return GNN_E_ARG;
  if (n_task > 0x7fffffffLL) return GNN_E_UNSUPPORTED;
  const bool plan = mid_row != nullptr;
  if (plan && (n_mid < 0 || n_short < 0 || n_mid + n_short + n_small + n_long > n_rows))
    return GNN_E_ARG;
  if (plan && n_short > 0 && !short_row) return GNN_E_ARG;
  if (plan && n_small > 0 && (!small_row || !small_col)) return GNN_E_ARG;
  if (mode != 0 && mode != 1) return GNN_E_ARG;
  if (!(dropout_p >= 0.f && dropout_p < 1.f)) return GNN_E_ARG;
  if (flags & ~(GNN_EPI_RELU | GNN_EPI_ELU)) return GNN_E_ARG;
  if (n_rows == 0) return GNN_OK;
  const int64_t feat_all = heads * fh;
  if (!rowptr || !wh || !el || !er || !out || ldw < feat_all || ldo < feat_all || lde < heads)
    return GNN_E_ARG;
  if (n_rows > 0x7fffffffLL) return GNN_E_UNSUPPORTED;
  if ((n_seg > 0 || n_long > 0) &&
      (!seg_row || !seg_begin || !long_row || !long_seg_ptr || !partial || n_seg == 0 || n_long == 0))
    return GNN_E_ARG;
  if ((whh == nullptr) != (erh == nullptr)) return GNN_E_ARG;
  if (whh && (ldwh < feat_all || ldeh < heads)) return GNN_E_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  // partial row layout per segment: [heads*fh acc | heads l | heads m] of the WHOLE layer;
  // each head group writes its own slice (the host allocates ldp = heads*fh + 2*heads).
  const int64_t ldp = feat_all + 2 * heads;
  const int64_t groups = (heads + kMaxHeads - 1) / kMaxHeads;
  for (int64_t g = 0; g < groups; ++g) {
    const int64_t h0 = g * kMaxHeads;
    const int64_t hg = heads - h0 < kMaxHeads ? heads - h0 : kMaxHeads;
    GatParams P{};
    P.rowptr = rowptr;
    P.col = col;
    P.n_rows = n_rows;
    P.feat = hg * fh;
    P.fh = fh;
    P.wh = wh + h0 * fh;
    P.ldw = ldw;
    P.el = el + h0;
    P.er = er + h0;
    P.lde = lde;
    P.heads = static_cast<int>(hg);
    P.slope = negative_slope;
    P.empty_fill = empty_row_fill ? empty_row_fill + h0 * fh : nullptr;
    P.drop_p = dropout_p;
    P.drop_scale = dropout_p > 0.f ? 1.0f / (1.0f - dropout_p) : 1.0f;
    P.drop_seed = dropout_seed;
    P.head0 = static_cast<int>(h0);
    P.out = out + h0 * fh;
    P.ldo = ldo;
    P.seg_len = plan ? seg_len : INT64_MAX;  // no plan: every row by one wave
    P.seg_row = seg_row;
    P.seg_begin = seg_begin;
    P.n_seg = plan ? n_seg : 0;
    P.long_row = long_row;
    P.long_seg_ptr = long_seg_ptr;
    P.n_long = plan ? n_long : 0;
    P.mid_row = mid_row;
    P.n_mid = plan ? n_mid : n_rows;
    P.short_row = short_row;
    P.n_short = plan ? n_short : 0;
    P.small_row = small_row;
    P.small_col = small_col;
    P.n_small = plan ? n_small : 0;
    // group slice of the partial rows: acc at h0*fh, l/m stored right after the slice's feat
    P.partial = partial ? partial + g * (kMaxHeads * fh + 2 * kMaxHeads) : nullptr;
    P.ldp = ldp;  // same row stride for every group
    P.flags = flags;
    P.stats = stats ? stats + h0 : nullptr;
    P.lds = heads;
    P.whh = whh ? whh + h0 * fh : nullptr;
    P.ldwh = ldwh;
    P.erh = erh ? erh + h0 : nullptr;
    P.ldeh = ldeh;
    P.task_row = task_row;
    P.n_task = plan ? n_task : 0;
    const bool vec4 = (fh % 4 == 0) && (ldw % 4 == 0) && (ldo % 4 == 0) && aligned_to(P.wh, 16) &&
                      (P.whh == nullptr || (aligned_to(P.whh, 16) && ldwh % 4 == 0)) &&
                      aligned_to(P.out, 16) &&
                      (P.empty_fill == nullptr || aligned_to(P.empty_fill, 16)) &&
                      (P.partial == nullptr || (aligned_to(P.partial, 16) && ldp % 4 == 0)) &&
                      (a_dst == nullptr || aligned_to(a_dst + h0 * fh, 16));
    // er from the gathered rows: the lanes of a head a power of two, one lane chunk per row
    {
      const int64_t vw = vec4 ? 4 : 1, g = fh / vw;
      const bool rec = a_dst != nullptr && fh % vw == 0 && (g & (g - 1)) == 0 && P.feat <= 64 * vw;
      P.a_dst = rec ? a_dst + h0 * fh : nullptr;
      P.er_g = static_cast<int>(g);
    }
    // tasks run in the one-chunk geometry only (NCH == 1: <= 64 lanes x VW features per row)
    if (P.n_task > 0 && P.feat > 64 * (vec4 ? 4 : 1)) return GNN_E_UNSUPPORTED;
    int rc;
    if (mode == 1)
      rc = vec4 ? dispatch_gat<4, true>(P, s) : dispatch_gat<1, true>(P, s);
    else
      rc = vec4 ? dispatch_gat<4, false>(P, s) : dispatch_gat<1, false>(P, s);
    if (rc != GNN_OK) return rc;
  }
  return GNN_OK;
}

extern "C" int gnn_gat_csr_f32(const int64_t* rowptr, const int32_t* col, int64_t n_rows,
                               const float* wh, int64_t ldw, int64_t heads, int64_t fh,
                               const float* el, const float* er, int64_t lde, float negative_slope,
                               int32_t mode, const float* empty_row_fill, float dropout_p,
                               uint64_t dropout_seed, float* out, int64_t ldo, int64_t seg_len,
                               const int32_t* seg_row, const int64_t* seg_begin, int64_t n_seg,
                               const int32_t* long_row, const int32_t* long_seg_ptr,
                               int64_t n_long, const int32_t* small_row, const int32_t* small_col,
                               int64_t n_small, const int32_t* mid_row, int64_t n_mid,
                               const int32_t* short_row, int64_t n_short,
                               float* partial, float* stats, uint32_t flags, void* stream) {
  return gat_entry(rowptr, col, n_rows, wh, ldw, heads, fh, el, er, lde, negative_slope, mode,
                   empty_row_fill, dropout_p, dropout_seed, out, ldo, seg_len, seg_row, seg_begin,
                   n_seg, long_row, long_seg_ptr, n_long, small_row, small_col, n_small, mid_row,
                   n_mid, short_row, n_short, partial, stats, flags, stream, nullptr, 0, nullptr,
                   0);
}

extern "C" int gnn_gat_csr_hub_f32(const int64_t* rowptr, const int32_t* col_hub, int64_t n_rows,
                                   const float* wh, int64_t ldw, int64_t heads, int64_t fh,
                                   const float* el, const float* er, int64_t lde,
                                   float negative_slope, int32_t mode,
                                   const float* empty_row_fill, float dropout_p,
                                   uint64_t dropout_seed, float* out, int64_t ldo,
                                   int64_t seg_len, const int32_t* seg_row,
                                   const int64_t* seg_begin, int64_t n_seg,
                                   const int32_t* long_row, const int32_t* long_seg_ptr,
                                   int64_t n_long, const int32_t* small_row,
                                   const int32_t* small_col, int64_t n_small,
                                   const int32_t* mid_row, int64_t n_mid,
                                   const int32_t* short_row, int64_t n_short, float* partial,
                                   float* stats, uint32_t flags, void* stream, const float* whh,
                                   int64_t ldwh, const float* erh, int64_t ldeh) {
  if (whh == nullptr || erh == nullptr) return GNN_E_ARG;
  return gat_entry(rowptr, col_hub, n_rows, wh, ldw, heads, fh, el, er, lde, negative_slope,
                   mode, empty_row_fill, dropout_p, dropout_seed, out, ldo, seg_len, seg_row,
                   seg_begin, n_seg, long_row, long_seg_ptr, n_long, small_row, small_col,
                   n_small, mid_row, n_mid, short_row, n_short, partial, stats, flags, stream,
                   whh, ldwh, erh, ldeh);
}

// ---- packed row tasks for the low-degree rows (GAT/models/layers.py:22-37 / :94-131, the
// same softmax + aggregation): see gat_packed_rows. The small / short row classes are replaced
// by tasks (ranges of consecutive rows of degree <= the threshold, edgeless rows included); the
// plan's segments and mid rows run as in gnn_gat_csr_hub_f32. whh / erh: hub tables (c < 0) or
// NULL (ldwh / ldeh ignored). Requires fh % 4 == 0, heads * fh <= 256 per group of 8 heads,
// 16-B aligned rows (GNN_E_UNSUPPORTED otherwise).
extern "C" int gnn_gat_csr_tasks_f32(const int64_t* rowptr, const int32_t* col, int64_t n_rows,
                                     const float* wh, int64_t ldw, int64_t heads, int64_t fh,
                                     const float* el, const float* er, int64_t lde,
                                     float negative_slope, int32_t mode,
                                     const float* empty_row_fill, float dropout_p,
                                     uint64_t dropout_seed, float* out, int64_t ldo,
                                     int64_t seg_len, const int32_t* seg_row,
                                     const int64_t* seg_begin, int64_t n_seg,
                                     const int32_t* long_row, const int32_t* long_seg_ptr,
                                     int64_t n_long, const int32_t* mid_row, int64_t n_mid,
                                     const int32_t* task_row, int64_t n_task, float* partial,
                                     float* stats, uint32_t flags, void* stream,
                                     const float* whh, int64_t ldwh, const float* erh,
                                     int64_t ldeh) {
  if (mid_row == nullptr) return GNN_E_ARG;
  if ((whh == nullptr) != (erh == nullptr)) return GNN_E_ARG;
  if (whh == nullptr) ldwh = ldeh = 0;
  return gat_entry(rowptr, col, n_rows, wh, ldw, heads, fh, el, er, lde, negative_slope, mode,
                   empty_row_fill, dropout_p, dropout_seed, out, ldo, seg_len, seg_row, seg_begin,
                   n_seg, long_row, long_seg_ptr, n_long, nullptr, nullptr, 0, mid_row, n_mid,
                   nullptr, 0, partial, stats, flags, stream, whh, ldwh, erh, ldeh, task_row,
                   n_task);
}

// gnn_gat_csr_hub_f32 with optional hub tables (whh / erh both NULL: none) and optional a_dst
// [heads * fh]: the attention vector er = Wh . a_dst came from (GAT/models/layers.py:26-27 /
// :106), with which the kernels recompute er_j from the Wh_j rows they gather instead of
// loading er (the one-chunk loop, the short and the small rows; er is still read by the other
// row paths and must be given). Same values up to the rounding of er's dot products.
extern "C" int gnn_gat_csr_ex_f32(const int64_t* rowptr, const int32_t* col, int64_t n_rows,
                                  const float* wh, int64_t ldw, int64_t heads, int64_t fh,
                                  const float* el, const float* er, int64_t lde,
                                  float negative_slope, int32_t mode,
                                  const float* empty_row_fill, float dropout_p,
                                  uint64_t dropout_seed, float* out, int64_t ldo, int64_t seg_len,
                                  const int32_t* seg_row, const int64_t* seg_begin, int64_t n_seg,
                                  const int32_t* long_row, const int32_t* long_seg_ptr,
                                  int64_t n_long, const int32_t* small_row,
                                  const int32_t* small_col, int64_t n_small,
                                  const int32_t* mid_row, int64_t n_mid,
                                  const int32_t* short_row, int64_t n_short, float* partial,
                                  float* stats, uint32_t flags, void* stream, const float* whh,
                                  int64_t ldwh, const float* erh, int64_t ldeh,
                                  const float* a_dst) {
  if ((whh == nullptr) != (erh == nullptr)) return GNN_E_ARG;
  if (whh == nullptr) ldwh = ldeh = 0;
  return gat_entry(rowptr, col, n_rows, wh, ldw, heads, fh, el, er, lde, negative_slope, mode,
                   empty_row_fill, dropout_p, dropout_seed, out, ldo, seg_len, seg_row, seg_begin,
                   n_seg, long_row, long_seg_ptr, n_long, small_row, small_col, n_small, mid_row,
                   n_mid, short_row, n_short, partial, stats, flags, stream, whh, ldwh, erh, ldeh,
                   nullptr, 0, a_dst);
}
