// gat_bwd.hip -- GAT backward on gfx950 (training through the drop-in GAT layers).
//
// The reference trains through ATen autograd of GAT/models/layers.py:22-37 (dense:
// O(N^2) a_input) and through SpecialSpmmFunction.backward (layers.py:54-64, which
// materialises a dense N x N grad_output . b^T). Here, per head h, with
//   out_i = sum_j m_ij a_ij Wh_j,  a_ij = exp(z_ij - lse_i),  z_ij = +-LeakyReLU(el_i + er_j),
//   y = ELU(out) (concat layers) or y = out,  m_ij = dropout mask / (1 - p):
//
//   prep  (row):   dout_i = dy_i * ELU'(out_i) ; out_i recovered from y (log1p) ;
//                  D_i = dout_i . out_i
//   edges (CSR rows i, lanes = (edge, head)):
//                  g_ij  = dout_i . Wh_j                       (SDDMM)
//                  w_ij  = m_ij a_ij                           (aggregation weight)
//                  ds_ij = a_ij (m_ij g_ij - D_i) dz/ds        (softmax + LeakyReLU backward)
//                  del_i = sum_j ds_ij
//   nodes (transposed CSR rows j, lanes = features):
//                  dWh_j = sum_i w_ij dout_i + der_j a_dst + del_j a_src,  der_j = sum_i ds_ij
// where el = a_src . Wh, er = a_dst . Wh. d a_src / d a_dst (two N x H x Fh
// reductions) and dW, dh (GEMMs) are left to the caller (torch). All three passes
// use the row-class plans (long rows / long columns split into segments merged in
// a fixed order): deterministic, no atomics.
#include "common.hpp"

namespace gnn {

constexpr int kBw = 256;
constexpr int kBwWaves = kBw / kWave;

__device__ __forceinline__ uint32_t bwd_hash3(uint64_t seed, int64_t edge, int head) {
  // identical to gat.hip's hash3: the backward must see the forward's dropout mask
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

// ---------------------------------------------------------------- prep
__global__ __launch_bounds__(256) void gat_bwd_prep_kernel(const float* __restrict__ dy,
                                                           const float* __restrict__ y, int64_t ldo,
                                                           int64_t n_rows, int64_t heads, int64_t fh,
                                                           int elu, float* __restrict__ dout,
                                                           float* __restrict__ D) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= n_rows * heads) return;
  const int64_t r = t / heads, h = t % heads;
  const float* yr = y + r * ldo + h * fh;
  const float* dyr = dy + r * ldo + h * fh;
  float* dr = dout + r * heads * fh + h * fh;
  float acc = 0.f;
  for (int64_t f = 0; f < fh; ++f) {
    const float yv = yr[f], g = dyr[f];
    float d = g, o = yv;
    if (elu && yv <= 0.f) {
      // ELU'(x) = exp(x) = y + 1 for x <= 0, and x = log1p(y); a saturated y = -1
      // (x < -17 in fp32) has ELU' = 0: its D term is 0 * log(0) := 0, not NaN.
      const float t = yv + 1.f;
      d = g * t;
      o = t > 0.f ? log1pf(yv) : 0.f;
    }
    dr[f] = d;
    acc = fmaf(d, o, acc);
  }
  D[r * heads + h] = acc;
}

// Vector form (fh % 4 == 0, fh / 4 a power of two, 16-B rows): a thread per 4 features, the
// head's D summed over its G = fh / 4 lanes by xor shuffles. The scalar kernel above runs a
// thread per (row, head) over fh scalar loads: 0.51 ms at cfg3 (1.6 TB/s).
template <int G>
__global__ __launch_bounds__(256) void gat_bwd_prep_vec_kernel(const float* __restrict__ dy,
                                                               const float* __restrict__ y,
                                                               int64_t ldo, int64_t n_rows,
                                                               int64_t heads, int elu,
                                                               float* __restrict__ dout,
                                                               float* __restrict__ D) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int64_t per_row = heads * G;  // float4s per row
  const bool live = t < n_rows * per_row;
  const int64_t r = live ? t / per_row : 0, c = live ? t % per_row : 0;
  float4 yv = make_float4(0.f, 0.f, 0.f, 0.f), gv = yv;
  if (live) {
    yv = *reinterpret_cast<const float4*>(y + r * ldo + 4 * c);
    gv = *reinterpret_cast<const float4*>(dy + r * ldo + 4 * c);
  }
  float yy[4] = {yv.x, yv.y, yv.z, yv.w}, gg[4] = {gv.x, gv.y, gv.z, gv.w}, dd[4];
  float acc = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float d = gg[i], o = yy[i];
    if (elu && yy[i] <= 0.f) {  // ELU'(x) = y + 1 for x <= 0, x = log1p(y) (saturated: 0)
      const float tt = yy[i] + 1.f;
      d = gg[i] * tt;
      o = tt > 0.f ? log1pf(yy[i]) : 0.f;
    }
    dd[i] = d;
    acc = fmaf(d, o, acc);
  }
#pragma unroll
  for (int o = 1; o < G; o <<= 1) acc += __shfl_xor(acc, o, 64);
  if (!live) return;
  *reinterpret_cast<float4*>(dout + r * (heads * 4 * G) + 4 * c) = make_float4(dd[0], dd[1], dd[2], dd[3]);
  if (c % G == 0) D[r * heads + c / G] = acc;
}

// The same with the row pass's per-(row, head) record: nstat[r][h] = {el, lse, D, 0} (the row
// pass then reads dout and the record from HBM instead of computing them per row in LDS).
template <int G>
__global__ __launch_bounds__(256) void gat_bwd_prep_rec_kernel(const float* __restrict__ dy,
                                                               const float* __restrict__ y,
                                                               int64_t ldo, int64_t n_rows,
                                                               int64_t heads, int elu,
                                                               const float* __restrict__ el,
                                                               const float* __restrict__ lse,
                                                               float* __restrict__ dout,
                                                               float* __restrict__ nstat,
                                                               float dyp, float dyscale,
                                                               uint64_t dyseed) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int64_t per_row = heads * G;  // float4s per row
  const bool live = t < n_rows * per_row;
  const int64_t r = live ? t / per_row : 0, c = live ? t % per_row : 0;
  float4 yv = make_float4(0.f, 0.f, 0.f, 0.f), gv = yv;
  if (live) {
    yv = *reinterpret_cast<const float4*>(y + r * ldo + 4 * c);
    gv = *reinterpret_cast<const float4*>(dy + r * ldo + 4 * c);
  }
  float yy[4] = {yv.x, yv.y, yv.z, yv.w}, gg[4] = {gv.x, gv.y, gv.z, gv.w}, dd[4];
  if (dyp > 0.f) {  // dy is the gradient of dropout(y): the mask of gnn_dropout_rows_f32 (key r)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      gg[i] = dropout_keep(dyseed, r, static_cast<int>(4 * c + i), dyp) ? gg[i] * dyscale
                                                                         : gg[i] * 0.f;
  }
  float acc = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float d = gg[i], o = yy[i];
    if (elu && yy[i] <= 0.f) {  // ELU'(x) = y + 1 for x <= 0, x = log(y + 1) (saturated: 0)
      const float tt = yy[i] + 1.f;
      d = gg[i] * tt;
      o = tt > 0.f ? __logf(tt) : 0.f;
    }
    dd[i] = d;
    acc = fmaf(d, o, acc);
  }
#pragma unroll
  for (int o = 1; o < G; o <<= 1) acc += __shfl_xor(acc, o, 64);
  if (!live) return;
  *reinterpret_cast<float4*>(dout + r * (heads * 4 * G) + 4 * c) = make_float4(dd[0], dd[1], dd[2], dd[3]);
  if (c % G == 0) {
    const int64_t h = c / G;
    *reinterpret_cast<float4*>(nstat + (r * heads + h) * 4) =
        make_float4(el[r * heads + h], lse[r * heads + h], acc, 0.f);
  }
}

// ---------------------------------------------------------------- edges
struct BwdEdgeParams {
  const int64_t* rowptr;
  const int32_t* col;
  const float* wh;
  int64_t ldw;
  const float* el;
  const float* er;
  const float* lse;  // [n, H]
  const float* dout;  // [n, H*fh]
  const float* D;     // [n, H]
  int heads;          // heads of this group (<= 8)
  int64_t H;          // total heads (row stride of el/er/lse/D, edge stride of w/ds)
  int64_t fh;
  float slope;
  float drop_p, drop_scale;
  uint64_t drop_seed;
  int head0;
  float* w_edge;   // [nnz, H]
  float* ds_edge;  // [nnz, H]
  float* del;      // [n, H]
  float* del_part; // [n_seg, H]
  // plan
  int64_t seg_len;
  const int32_t* seg_row;
  const int64_t* seg_begin;
  int64_t n_seg, seg_waves;
  const int32_t* rows;  // mid + small rows (any order)
  int64_t n_rows_list;
};

template <int VW, int HP, bool SPARSE>
__global__ __launch_bounds__(kBw) void gat_bwd_edge_kernel(BwdEdgeParams P) {
  constexpr int EPP = kWave / HP;
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t wave = static_cast<int64_t>(blockIdx.x) * kBwWaves + (threadIdx.x >> 6);
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
  } else {
    const int64_t i = wave - P.seg_waves;
    if (i >= P.n_rows_list) return;
    row = P.rows[i];
    beg = P.rowptr[row];
    end = P.rowptr[row + 1];
  }
  const bool head_ok = ah < P.heads;
  const int64_t hoff = head_ok ? ah : 0;
  const float eli = P.el[row * P.H + hoff];
  const float lse = P.lse[row * P.H + hoff];
  const float Di = P.D[row * P.H + hoff];
  const float* dr = P.dout + row * (P.H * P.fh) + hoff * P.fh;
  float dsum = 0.f;
  for (int64_t b = beg; b < end; b += EPP) {
    const int64_t e = b + ae;
    if (head_ok && e < end) {
      const int c = P.col[e];
      const float sv = eli + P.er[static_cast<int64_t>(c) * P.H + ah];
      const float x = sv > 0.f ? sv : P.slope * sv;
      const float z = SPARSE ? -x : x;
      const float dzds = (sv > 0.f ? 1.f : P.slope) * (SPARSE ? -1.f : 1.f);
      const float a = __expf(z - lse);
      const float* xr = P.wh + static_cast<int64_t>(c) * P.ldw + hoff * P.fh;
      float g = 0.f;
      for (int64_t f = 0; f < P.fh; f += VW) {
        const typename Vec<VW>::T wv = vload<VW>(xr + f);
        const typename Vec<VW>::T dv = vload<VW>(dr + f);
#pragma unroll
        for (int k = 0; k < VW; ++k) g = fmaf(vget(dv, k), vget(wv, k), g);
      }
      float m = 1.f;
      if (P.drop_p > 0.f) {
        const uint32_t r = bwd_hash3(P.drop_seed, e, P.head0 + ah);
        m = (static_cast<float>(r >> 8) * (1.0f / 16777216.0f) < P.drop_p) ? 0.f : P.drop_scale;
      }
      const float ds = a * (m * g - Di) * dzds;
      P.w_edge[e * P.H + ah] = m * a;
      P.ds_edge[e * P.H + ah] = ds;
      dsum += ds;
    }
  }
#pragma unroll
  for (int o = HP; o < kWave; o <<= 1) dsum += __shfl_xor(dsum, o, kWave);
  if (lane < HP && head_ok) {
    if (is_seg)
      P.del_part[wave * P.H + ah] = dsum;
    else
      P.del[row * P.H + ah] = dsum;
  }
}

// del[long_row] = sum of its segments' partials, in segment order
__global__ __launch_bounds__(256) void gat_bwd_del_fixup_kernel(const int32_t* __restrict__ long_row,
                                                                const int32_t* __restrict__ long_seg_ptr,
                                                                int64_t n_long, int64_t heads,
                                                                int64_t H, int64_t head0,
                                                                const float* __restrict__ del_part,
                                                                float* __restrict__ del) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= n_long * heads) return;
  const int64_t i = t / heads, h = head0 + t % heads;
  float s = 0.f;
  for (int32_t k = long_seg_ptr[i]; k < long_seg_ptr[i + 1]; ++k) s += del_part[k * H + h];
  del[static_cast<int64_t>(long_row[i]) * H + h] = s;
}

// ---------------------------------------------------------------- nodes
struct BwdNodeParams {
  const int64_t* rowptr_t;  // transposed CSR: edges into node j
  const int32_t* src_t;     // source row i of each transposed edge
  const int64_t* eid_t;     // CSR edge id of each transposed edge
  int64_t n_nodes;
  const float* dout;  // [n, H*fh]
  const float* w_edge;
  const float* ds_edge;
  const float* del;  // [n, H]
  const float* a_src;
  const float* a_dst;  // [H*fh]
  int64_t H, fh, feat;
  float* dwh;  // [n, H*fh]
  float* der;  // [n, H]
  float* part;  // [n_seg, feat + H]
  int64_t ldp;
  int64_t seg_len;
  const int32_t* seg_row;
  const int64_t* seg_begin;
  int64_t n_seg, seg_waves;
  const int32_t* rows;
  int64_t n_rows_list;
};

template <int VW, int LPR, int NCH>
__device__ __forceinline__ void node_epilogue(const BwdNodeParams& P, int64_t j, int sub,
                                              const int (&hid)[NCH],
                                              typename Vec<VW>::T (&acc)[NCH],
                                              const float (&derh)[NCH]) {
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    const int64_t f = static_cast<int64_t>(ch * LPR + sub) * VW;
    if (f >= P.feat) continue;
    const float dl = P.del[j * P.H + hid[ch]];
    typename Vec<VW>::T r = acc[ch] + derh[ch] * vload<VW>(P.a_dst + f) + dl * vload<VW>(P.a_src + f);
    vstore<VW>(P.dwh + j * P.feat + f, r);
  }
}

template <int VW, int LPR, int NCH, int HP>
__global__ __launch_bounds__(kBw) void gat_bwd_node_kernel(BwdNodeParams P) {
  constexpr int EPI = kWave / LPR;
  constexpr int EPP = kWave / HP;
  constexpr int U = 2;
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t wave = static_cast<int64_t>(blockIdx.x) * kBwWaves + (threadIdx.x >> 6);
  const int sub = lane & (LPR - 1);
  const int grp = lane / LPR;
  const int ah = lane & (HP - 1);
  const int ae = lane / HP;
  int64_t j, beg, end;
  bool is_seg = false;
  if (wave < P.seg_waves) {
    if (wave >= P.n_seg) return;
    j = P.seg_row[wave];
    beg = P.seg_begin[wave];
    end = min(beg + P.seg_len, P.rowptr_t[j + 1]);
    is_seg = true;
  } else {
    const int64_t i = wave - P.seg_waves;
    if (i >= P.n_rows_list) return;
    j = P.rows[i];
    beg = P.rowptr_t[j];
    end = P.rowptr_t[j + 1];
  }
  int hid[NCH];
  typename Vec<VW>::T acc[NCH];
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    const int64_t f = static_cast<int64_t>(ch * LPR + sub) * VW;
    hid[ch] = f < P.feat ? static_cast<int>(f / P.fh) : 0;
    acc[ch] = vzero<VW>();
  }
  // sum_i w_ij dout_i: lanes = features, EPI edge slots
  for (int64_t b = beg; b < end; b += EPI * U) {
    typename Vec<VW>::T xv[U][NCH];
    float w[U][NCH];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t e = b + u * EPI + grp;
      const bool ok = e < end;
      const int64_t eid = ok ? P.eid_t[e] : 0;
      const int64_t i = ok ? P.src_t[e] : 0;
      const float* dr = P.dout + i * P.feat;
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) {
        const int64_t f = static_cast<int64_t>(ch * LPR + sub) * VW;
        const bool okf = ok && f < P.feat;
        xv[u][ch] = okf ? vload<VW>(dr + f) : vzero<VW>();
        w[u][ch] = okf ? P.w_edge[eid * P.H + hid[ch]] : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) acc[ch] += w[u][ch] * xv[u][ch];
    }
  }
#pragma unroll
  for (int o = LPR; o < kWave; o <<= 1) {
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) acc[ch] += shfl_xor_f(acc[ch], o);
  }
  // der_j = sum_i ds_ij: lanes = (edge, head), HP heads per pass (any head count)
  float* pr = is_seg ? P.part + wave * P.ldp : nullptr;
  float derh[NCH];
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) derh[ch] = 0.f;
  for (int64_t h0 = 0; h0 < P.H; h0 += HP) {
    const int64_t hh = h0 + ah;
    float dsum = 0.f;
    if (hh < P.H) {
      for (int64_t b = beg + ae; b < end; b += EPP) dsum += P.ds_edge[P.eid_t[b] * P.H + hh];
    }
#pragma unroll
    for (int o = HP; o < kWave; o <<= 1) dsum += __shfl_xor(dsum, o, kWave);
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      const int64_t rel = hid[ch] - h0;
      const float v = __shfl(dsum, static_cast<int>(rel & (HP - 1)), kWave);
      if (rel >= 0 && rel < HP) derh[ch] = v;
    }
    if (lane < HP && hh < P.H) {
      if (is_seg)
        pr[P.feat + hh] = dsum;
      else
        P.der[j * P.H + hh] = dsum;
    }
  }
  if (is_seg) {
    if (lane < LPR) {
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) {
        const int64_t f = static_cast<int64_t>(ch * LPR + sub) * VW;
        if (f < P.feat) vstore<VW>(pr + f, acc[ch]);
      }
    }
    return;
  }
  if (lane < LPR) node_epilogue<VW, LPR, NCH>(P, j, sub, hid, acc, derh);
}

// Long nodes: sum segment partials (acc and der) in order, then the a-terms.
template <int VW, int LPR, int NCH>
__global__ __launch_bounds__(kBw) void gat_bwd_node_fixup_kernel(BwdNodeParams P,
                                                                 const int32_t* long_row,
                                                                 const int32_t* long_seg_ptr,
                                                                 int64_t n_long) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kBwWaves + (threadIdx.x >> 6);
  if (i >= n_long || lane >= LPR) return;
  const int sub = lane;
  const int64_t j = long_row[i];
  const int32_t s0 = long_seg_ptr[i], s1 = long_seg_ptr[i + 1];
  int hid[NCH];
  typename Vec<VW>::T acc[NCH];
  float derh[NCH];
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    const int64_t f = static_cast<int64_t>(ch * LPR + sub) * VW;
    hid[ch] = f < P.feat ? static_cast<int>(f / P.fh) : 0;
    acc[ch] = vzero<VW>();
    derh[ch] = 0.f;
  }
  for (int32_t s = s0; s < s1; ++s) {
    const float* pr = P.part + static_cast<int64_t>(s) * P.ldp;
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      const int64_t f = static_cast<int64_t>(ch * LPR + sub) * VW;
      if (f < P.feat) {
        acc[ch] += vload<VW>(pr + f);
        derh[ch] += pr[P.feat + hid[ch]];
      }
    }
  }
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    const int64_t f = static_cast<int64_t>(ch * LPR + sub) * VW;
    if (f < P.feat && f % P.fh == 0) P.der[j * P.H + hid[ch]] = derh[ch];
  }
  node_epilogue<VW, LPR, NCH>(P, j, sub, hid, acc, derh);
}

template <int VW, int HP, bool SPARSE>
static void launch_edges(const BwdEdgeParams& P0, hipStream_t s) {
  BwdEdgeParams P = P0;
  const int64_t seg_blocks = (P.n_seg + kBwWaves - 1) / kBwWaves;
  const int64_t row_blocks = (P.n_rows_list + kBwWaves - 1) / kBwWaves;
  P.seg_waves = seg_blocks * kBwWaves;
  if (seg_blocks + row_blocks > 0)
    hipLaunchKernelGGL((gat_bwd_edge_kernel<VW, HP, SPARSE>),
                       dim3(static_cast<unsigned>(seg_blocks + row_blocks)), dim3(kBw), 0, s, P);
}

template <int VW, int LPR, int NCH, int HP>
static void launch_nodes(const BwdNodeParams& P0, const int32_t* long_row,
                         const int32_t* long_seg_ptr, int64_t n_long, hipStream_t s) {
  BwdNodeParams P = P0;
  const int64_t seg_blocks = (P.n_seg + kBwWaves - 1) / kBwWaves;
  const int64_t row_blocks = (P.n_rows_list + kBwWaves - 1) / kBwWaves;
  P.seg_waves = seg_blocks * kBwWaves;
  if (seg_blocks + row_blocks > 0)
    hipLaunchKernelGGL((gat_bwd_node_kernel<VW, LPR, NCH, HP>),
                       dim3(static_cast<unsigned>(seg_blocks + row_blocks)), dim3(kBw), 0, s, P);
  if (n_long > 0)
    hipLaunchKernelGGL((gat_bwd_node_fixup_kernel<VW, LPR, NCH>),
                       dim3(static_cast<unsigned>((n_long + kBwWaves - 1) / kBwWaves)), dim3(kBw), 0,
                       s, P, long_row, long_seg_ptr, n_long);
}

template <int VW, int HP>
static int dispatch_nodes(const BwdNodeParams& P, const int32_t* lr, const int32_t* lsp, int64_t nl,
                          hipStream_t s) {
  const int64_t nv = (P.feat + VW - 1) / VW;
  if (nv <= 64) {
    switch (next_pow2_le64(nv)) {
      case 1: launch_nodes<VW, 1, 1, HP>(P, lr, lsp, nl, s); break;
      case 2: launch_nodes<VW, 2, 1, HP>(P, lr, lsp, nl, s); break;
      case 4: launch_nodes<VW, 4, 1, HP>(P, lr, lsp, nl, s); break;
      case 8: launch_nodes<VW, 8, 1, HP>(P, lr, lsp, nl, s); break;
      case 16: launch_nodes<VW, 16, 1, HP>(P, lr, lsp, nl, s); break;
      case 32: launch_nodes<VW, 32, 1, HP>(P, lr, lsp, nl, s); break;
      default: launch_nodes<VW, 64, 1, HP>(P, lr, lsp, nl, s); break;
    }
  } else if (nv <= 128) {
    launch_nodes<VW, 64, 2, HP>(P, lr, lsp, nl, s);
  } else if (nv <= 256) {
    launch_nodes<VW, 64, 4, HP>(P, lr, lsp, nl, s);
  } else {
    return GNN_E_UNSUPPORTED;
  }
  return launch_status();
}

// ---------------------------------------------------------------- rows + recomputing nodes
// The two passes above hand 2 x 4 H bytes per (edge, head) from the edge pass to the node
// pass (w_ij, ds_ij written in CSR order, then read through eid_t: two random 4 H-byte reads per
// edge, each its own cache line) and the prep pass writes dout for the edge pass to re-read.
// Here the row pass does the prep itself and writes, besides dout and del, only a per-row
// record nstat_i = {el, lse, D, 0} per head (4 H floats: one 128-B line at H = 8); the node pass
// gathers dout_i with nstat_i and recomputes a_ij, g_ij = dout_i . Wh_j (Wh_j is the node's
// own row, held in registers), w_ij and ds_ij. Per edge the node pass reads 4 + 4 feat + 16 H
// bytes (12 + 4 feat + 2 x 2 lines before) and the row pass writes nothing.
constexpr int kRowLds = 1152;    // floats of LDS per wave (4.5 KB: 8 waves per SIMD stay)
#ifndef GNN_BWD_SPLIT_PREP
#define GNN_BWD_SPLIT_PREP 1  // prep in its own coalesced kernel (0: fused into the row pass)
#endif
constexpr int kShortRowsW = 8;   // rows per wave of the short-row class (8 lanes each)

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float bwd_keep(float p, float scale, uint64_t seed, int64_t e, int64_t h) {
  if (p <= 0.f) return 1.f;
  const uint32_t r = bwd_hash3(seed, e, static_cast<int>(h));
  return (static_cast<float>(r >> 8) * (1.0f / 16777216.0f) < p) ? 0.f : scale;
}

struct BwdRowParams {
  const int64_t* rowptr;
  const int32_t* col;
  const float* wh;
  int64_t ldw;
  const float* el;
  const float* er;
  const float* lse;
  const float* dy;
  const float* y;
  int64_t ldo;
  int elu, sparse, hp;
  int64_t H, fh, feat;
  float slope, drop_p, drop_scale;
  uint64_t drop_seed;
  float* dout;      // [n, feat]
  float* nstat;     // [n, 4 H]
  float* del;       // [n, H]
  float* del_part;  // [n_seg, H]
  int64_t seg_len;
  const int32_t* seg_row;
  const int64_t* seg_begin;
  int64_t n_seg, seg_waves;
  const int32_t* rows;  // one wave per row
  int64_t n_rows_list, row_waves;
  const int32_t* short_rows;  // kShortRowsW rows per wave
  int64_t n_short;
  const float* a_dst;  // non-NULL (and NFV > 0): er_j = a_dst . Wh_j from the gathered row
};

// Waves: [segments of long rows | rows | short rows, 8 per wave]. Prep (lanes = features):
// dout_i = dy_i ELU'(out_i) into LDS (and HBM: by a long row's first segment only), the
// products dout . out into LDS, D_i per head summed from them. Edges (lanes = (edge slot,
// head), HP heads per pass): ds_ij as gat_bwd_edge_kernel, summed into del_i (segments: partials).
// Edges in flight per lane: row pass 2 (4: 1.18 vs 0.85 ms at cfg3), node pass 2 (4 / 8:
// 1.097 / 1.397 vs 1.047 ms), profiles/r05r2_gat_bwd_u_drop_ab.log. A row-pass instance
// without the dropout-mask code took 88 instead of 78 VGPRs and was slower (0.928 vs 0.847 ms).
#ifndef GNN_BWD_ROW_U
#define GNN_BWD_ROW_U 2
#endif
#ifndef GNN_BWD_NODE_U
#define GNN_BWD_NODE_U 2
#endif
template <int VW, int NFV, bool PREP, bool REC>
__global__ __launch_bounds__(kBw) void gat_bwd_rows_kernel(BwdRowParams P) {
  constexpr int U = GNN_BWD_ROW_U;
  // PREP = false: dout and the {el, lse, D} records came from gat_bwd_prep_rec_kernel
  __shared__ float lds[kBwWaves][PREP ? kRowLds : 1];
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x >> 6;
  const int64_t wave = static_cast<int64_t>(blockIdx.x) * kBwWaves + wid;
  int mode;  // 0 segment, 1 row, 2 short rows
  int64_t row0 = -1, sbase = 0;
  if (wave < P.seg_waves) {
    if (wave >= P.n_seg) return;
    mode = 0;
    row0 = P.seg_row[wave];
  } else if (wave < P.seg_waves + P.row_waves) {
    const int64_t i = wave - P.seg_waves;
    if (i >= P.n_rows_list) return;
    mode = 1;
    row0 = P.rows[i];
  } else {
    sbase = (wave - P.seg_waves - P.row_waves) * kShortRowsW;
    if (sbase >= P.n_short) return;
    mode = 2;
  }
  const int nr = mode == 2 ? kShortRowsW : 1;
  const bool write = mode != 0 || P.seg_begin[wave] == P.rowptr[row0];
  auto row_of = [&](int r) -> int64_t {
    if (mode != 2) return row0;
    return sbase + r < P.n_short ? P.short_rows[sbase + r] : -1;
  };
  float* dbuf = lds[wid];
  float* pbuf = dbuf + nr * P.feat;
  float* Dbuf = pbuf + nr * P.feat;
  // ---- prep: the (row, feature vector) pairs of the wave's rows spread over the lanes (a
  // short-row wave's 8 rows at 64 features take 2 lane passes, not 8)
  const int nv = static_cast<int>(P.feat / VW);  // feat % VW == 0 when VW = 4
  if constexpr (PREP) {
  for (int t = lane; t < nr * nv; t += kWave) {
    const int r = t / nv;
    const int64_t f = static_cast<int64_t>(t - r * nv) * VW;
    const int64_t i = row_of(r);
    if (i < 0) continue;  // the tail slots of a short-row wave
    const typename Vec<VW>::T yv = vload<VW>(P.y + i * P.ldo + f);
    const typename Vec<VW>::T gv = vload<VW>(P.dy + i * P.ldo + f);
    typename Vec<VW>::T dv, pv;
#pragma unroll
    for (int k = 0; k < VW; ++k) {
      const float yy = vget(yv, k), g = vget(gv, k);
      float d = g, o = yy;
      if (P.elu && yy <= 0.f) {  // ELU'(x) = y + 1 for x <= 0, x = log(y + 1) (saturated: 0)
        const float tt = yy + 1.f;
        d = g * tt;
        o = tt > 0.f ? __logf(tt) : 0.f;
      }
      vset(dv, k, d);
      vset(pv, k, d * o);
    }
    vstore<VW>(dbuf + r * P.feat + f, dv);
    vstore<VW>(pbuf + r * P.feat + f, pv);
    if (write) vstore<VW>(P.dout + i * P.feat + f, dv);
  }
  wave_lds_sync();
  const int H32 = static_cast<int>(P.H), fh32 = static_cast<int>(P.fh);
  for (int t = lane; t < nr * H32; t += kWave) {
    const int r = t / H32;
    const int h = t - r * H32;
    const int64_t i = row_of(r);
    const float* pp = pbuf + r * P.feat + h * fh32;
    float s = 0.f;
    for (int k = 0; k < fh32; ++k) s += pp[k];
    Dbuf[t] = s;
    if (i >= 0 && write)
      *reinterpret_cast<float4*>(P.nstat + (i * P.H + h) * 4) =
          make_float4(P.el[i * P.H + h], P.lse[i * P.H + h], s, 0.f);
  }
  wave_lds_sync();
  }
  // ---- edges
  const int LR = kWave / nr;         // lanes of one row
  const int r = lane / LR, l = lane % LR;
  const int HP = P.hp;
  const int ah = l & (HP - 1), es = l / HP, ES = LR / HP;
  const int64_t i = row_of(r);
  int64_t beg = 0, end = 0;
  if (i >= 0) {
    if (mode == 0) {
      beg = P.seg_begin[wave];
      end = min(beg + P.seg_len, P.rowptr[i + 1]);
    } else {
      beg = P.rowptr[i];
      end = P.rowptr[i + 1];
    }
  }
  const int64_t ii = i >= 0 ? i : 0;
  const float* drow = dbuf + r * P.feat;
  const float sgn = P.sparse ? -1.f : 1.f;
  for (int64_t h0 = 0; h0 < P.H; h0 += HP) {
    const int64_t h = h0 + ah;
    const bool hk = h < P.H && i >= 0;
    const int64_t hh = h < P.H ? h : 0;
    float eli, lsei, Di;
    const float* dh;
    if constexpr (PREP) {
      eli = P.el[ii * P.H + hh];
      lsei = P.lse[ii * P.H + hh];
      Di = Dbuf[r * P.H + hh];
      dh = drow + hh * P.fh;
    } else {  // the row's own record and dout slice, from the prep kernel
      const float4 ns = *reinterpret_cast<const float4*>(P.nstat + (ii * P.H + hh) * 4);
      eli = ns.x;
      lsei = ns.y;
      Di = ns.z;
      dh = P.dout + ii * P.feat + hh * P.fh;
    }
    typename Vec<VW>::T dreg[NFV > 0 ? NFV : 1], areg[NFV > 0 ? NFV : 1];
    constexpr bool rec = NFV > 0 && REC;  // er_j from the gathered Wh_j (no er loads)
    if constexpr (NFV > 0) {
#pragma unroll
      for (int v = 0; v < NFV; ++v) {
        dreg[v] = vload<VW>(dh + v * VW);
        areg[v] = rec ? vload<VW>(P.a_dst + hh * P.fh + v * VW) : vzero<VW>();
      }
    }
    float dsum = 0.f;
    if (hk) {
      for (int64_t b = beg + es; b < end; b += static_cast<int64_t>(ES) * U) {
        int32_t c[U];
        bool ok[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int64_t e = b + static_cast<int64_t>(u) * ES;
          ok[u] = e < end;
          c[u] = ok[u] ? P.col[e] : 0;
        }
        float erv[U];
        typename Vec<VW>::T wv[U][NFV > 0 ? NFV : 1];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          erv[u] = (ok[u] && !rec) ? P.er[static_cast<int64_t>(c[u]) * P.H + h] : 0.f;
          if constexpr (NFV > 0) {
            const float* xr = P.wh + static_cast<int64_t>(c[u]) * P.ldw + h * P.fh;
#pragma unroll
            for (int v = 0; v < NFV; ++v) wv[u][v] = ok[u] ? vload<VW>(xr + v * VW) : vzero<VW>();
          }
        }
        if constexpr (NFV > 0) {
          if (rec) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
              float e = 0.f;
#pragma unroll
              for (int v = 0; v < NFV; ++v) {
#pragma unroll
                for (int k = 0; k < VW; ++k) e = fmaf(vget(wv[u][v], k), vget(areg[v], k), e);
              }
              erv[u] = e;
            }
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          float g = 0.f;
          if constexpr (NFV > 0) {
#pragma unroll
            for (int v = 0; v < NFV; ++v) {
#pragma unroll
              for (int k = 0; k < VW; ++k) g = fmaf(vget(dreg[v], k), vget(wv[u][v], k), g);
            }
          } else {
            const float* xr = P.wh + static_cast<int64_t>(c[u]) * P.ldw + h * P.fh;
            for (int64_t f = 0; f < P.fh; f += VW) {
              const typename Vec<VW>::T dv = vload<VW>(dh + f);
              const typename Vec<VW>::T xv = vload<VW>(xr + f);
#pragma unroll
              for (int k = 0; k < VW; ++k) g = fmaf(vget(dv, k), vget(xv, k), g);
            }
          }
          const float sv = eli + erv[u];
          const float x = sv > 0.f ? sv : P.slope * sv;
          const float dzds = (sv > 0.f ? 1.f : P.slope) * sgn;
          const float a = __expf(sgn * x - lsei);
          const float m = bwd_keep(P.drop_p, P.drop_scale, P.drop_seed,
                                   b + static_cast<int64_t>(u) * ES, h);
          const float ds = a * (m * g - Di) * dzds;
          if (ok[u]) dsum += ds;
        }
      }
    }
    for (int o = HP; o < LR; o <<= 1) dsum += __shfl_xor(dsum, o, kWave);
    if (hk && es == 0) {
      if (mode == 0)
        P.del_part[wave * P.H + h] = dsum;
      else
        P.del[i * P.H + h] = dsum;
    }
  }
}

struct BwdNodeRParams {
  const int64_t* rowptr_t;
  const int32_t* src_t;
  const int64_t* eid_t;  // read only with dropout (the mask hashes the CSR edge id)
  const float* dout;
  const float* nstat;
  const float* wh;
  int64_t ldw;
  const float* er;
  int sparse, G;  // G = lanes per head (fh / VW, a power of two)
  float slope, drop_p, drop_scale;
  uint64_t drop_seed;
  int64_t row_waves;
  const int32_t* short_rows;  // EPI rows per wave (one per lane group)
  int64_t n_short;
};

// Lanes = features (LPR lanes x VW, NCH chunks), EPI = 64 / LPR lane groups; a segment or row
// wave spreads its edges over the groups, a short-row wave gives each group a row of its own.
template <int VW, int LPR, int NCH, bool DROP>
__global__ __launch_bounds__(kBw) void gat_bwd_node_r_kernel(BwdNodeParams P, BwdNodeRParams R) {
  constexpr int EPI = kWave / LPR;
  constexpr int U = GNN_BWD_NODE_U;
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t wave = static_cast<int64_t>(blockIdx.x) * kBwWaves + (threadIdx.x >> 6);
  const int sub = lane & (LPR - 1);
  const int grp = lane / LPR;
  int mode;
  int64_t j = -1, beg = 0, end = 0;
  if (wave < P.seg_waves) {
    if (wave >= P.n_seg) return;
    mode = 0;
    j = P.seg_row[wave];
    beg = P.seg_begin[wave];
    end = min(beg + P.seg_len, P.rowptr_t[j + 1]);
  } else if (wave < P.seg_waves + R.row_waves) {
    const int64_t i = wave - P.seg_waves;
    if (i >= P.n_rows_list) return;
    mode = 1;
    j = P.rows[i];
    beg = P.rowptr_t[j];
    end = P.rowptr_t[j + 1];
  } else {
    const int64_t s = (wave - P.seg_waves - R.row_waves) * EPI;
    if (s >= R.n_short) return;
    mode = 2;
    if (s + grp < R.n_short) {
      j = R.short_rows[s + grp];
      beg = R.rowptr_t[j];
      end = R.rowptr_t[j + 1];
    }
  }
  const int eo = mode == 2 ? 0 : grp;
  const int ES = mode == 2 ? 1 : EPI;
  const int64_t jj = j >= 0 ? j : 0;
  int hid[NCH];
  typename Vec<VW>::T whj[NCH], acc[NCH];
  float erj[NCH], dsa[NCH];
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    const int64_t f = static_cast<int64_t>(ch * LPR + sub) * VW;
    const bool okf = f < P.feat;
    hid[ch] = okf ? static_cast<int>(f / P.fh) : 0;
    whj[ch] = okf ? vload<VW>(R.wh + jj * R.ldw + f) : vzero<VW>();
    erj[ch] = R.er[jj * P.H + hid[ch]];
    acc[ch] = vzero<VW>();
    dsa[ch] = 0.f;
  }
  const float sgn = R.sparse ? -1.f : 1.f;
  for (int64_t b = beg + eo; b < end; b += static_cast<int64_t>(ES) * U) {
    bool ok[U];
    int64_t src[U], eid[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t e = b + static_cast<int64_t>(u) * ES;
      ok[u] = e < end;
      src[u] = ok[u] ? R.src_t[e] : 0;
      eid[u] = (DROP && ok[u]) ? R.eid_t[e] : 0;  // the mask hashes the CSR edge id
    }
    typename Vec<VW>::T xv[U][NCH];
    float4 st[U][NCH];  // {el, lse, D, 0} of (source, head)
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float4* ns = reinterpret_cast<const float4*>(R.nstat) + src[u] * P.H;
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) {
        const int64_t f = static_cast<int64_t>(ch * LPR + sub) * VW;
        // masked slots (past the row's end) issue no loads
        xv[u][ch] = (ok[u] && f < P.feat) ? vload<VW>(R.dout + src[u] * P.feat + f) : vzero<VW>();
        st[u][ch] = ok[u] ? ns[hid[ch]] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) {
        float g = 0.f;
#pragma unroll
        for (int k = 0; k < VW; ++k) g = fmaf(vget(xv[u][ch], k), vget(whj[ch], k), g);
        for (int o = 1; o < R.G; o <<= 1) g += __shfl_xor(g, o, kWave);
        const float sv = st[u][ch].x + erj[ch];
        const float x = sv > 0.f ? sv : R.slope * sv;
        const float dzds = (sv > 0.f ? 1.f : R.slope) * sgn;
        const float a = __expf(sgn * x - st[u][ch].y);
        const float m = DROP ? bwd_keep(R.drop_p, R.drop_scale, R.drop_seed, eid[u], hid[ch]) : 1.f;
        const float w = ok[u] ? m * a : 0.f;
        const float ds = ok[u] ? a * (m * g - st[u][ch].z) * dzds : 0.f;
        acc[ch] += w * xv[u][ch];
        dsa[ch] += ds;
      }
    }
  }
  if (mode != 2) {
#pragma unroll
    for (int o = LPR; o < kWave; o <<= 1) {
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) {
        acc[ch] += shfl_xor_f(acc[ch], o);
        dsa[ch] += __shfl_xor(dsa[ch], o, kWave);
      }
    }
  }
  if (mode == 0) {
    if (lane < LPR) {
      float* pr = P.part + wave * P.ldp;
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) {
        const int64_t f = static_cast<int64_t>(ch * LPR + sub) * VW;
        if (f < P.feat) {
          vstore<VW>(pr + f, acc[ch]);
          if (f % P.fh == 0) pr[P.feat + hid[ch]] = dsa[ch];
        }
      }
    }
    return;
  }
  if (j < 0 || (mode == 1 && lane >= LPR)) return;
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    const int64_t f = static_cast<int64_t>(ch * LPR + sub) * VW;
    if (f < P.feat && f % P.fh == 0) P.der[j * P.H + hid[ch]] = dsa[ch];
  }
  node_epilogue<VW, LPR, NCH>(P, j, sub, hid, acc, dsa);
}

template <int VW, int LPR, int NCH>
static void launch_nodes_r(const BwdNodeParams& P0, const BwdNodeRParams& R0, const int32_t* long_row,
                           const int32_t* long_seg_ptr, int64_t n_long, hipStream_t s) {
  constexpr int EPI = kWave / LPR;
  BwdNodeParams P = P0;
  BwdNodeRParams R = R0;
  const int64_t seg_blocks = (P.n_seg + kBwWaves - 1) / kBwWaves;
  const int64_t row_blocks = (P.n_rows_list + kBwWaves - 1) / kBwWaves;
  const int64_t short_waves = (R.n_short + EPI - 1) / EPI;
  const int64_t short_blocks = (short_waves + kBwWaves - 1) / kBwWaves;
  P.seg_waves = seg_blocks * kBwWaves;
  R.row_waves = row_blocks * kBwWaves;
  const int64_t blocks = seg_blocks + row_blocks + short_blocks;
  if (blocks > 0) {  // dropout as a template flag: its edge ids stay out of the common path
    if (R.drop_p > 0.f)
      hipLaunchKernelGGL((gat_bwd_node_r_kernel<VW, LPR, NCH, true>),
                         dim3(static_cast<unsigned>(blocks)), dim3(kBw), 0, s, P, R);
    else
      hipLaunchKernelGGL((gat_bwd_node_r_kernel<VW, LPR, NCH, false>),
                         dim3(static_cast<unsigned>(blocks)), dim3(kBw), 0, s, P, R);
  }
  if (n_long > 0)
    hipLaunchKernelGGL((gat_bwd_node_fixup_kernel<VW, LPR, NCH>),
                       dim3(static_cast<unsigned>((n_long + kBwWaves - 1) / kBwWaves)), dim3(kBw), 0,
                       s, P, long_row, long_seg_ptr, n_long);
}

// lanes per row chunk for feat / VW vectors (0: feat above 256 vectors)
static int node_r_lpr(int64_t nv) { return nv <= 64 ? next_pow2_le64(nv) : nv <= 256 ? 64 : 0; }

template <int VW>
static int dispatch_nodes_r(const BwdNodeParams& P, const BwdNodeRParams& R, const int32_t* lr,
                            const int32_t* lsp, int64_t nl, hipStream_t s) {
  const int64_t nv = (P.feat + VW - 1) / VW;
  if (nv <= 64) {
    switch (next_pow2_le64(nv)) {
      case 1: launch_nodes_r<VW, 1, 1>(P, R, lr, lsp, nl, s); break;
      case 2: launch_nodes_r<VW, 2, 1>(P, R, lr, lsp, nl, s); break;
      case 4: launch_nodes_r<VW, 4, 1>(P, R, lr, lsp, nl, s); break;
      case 8: launch_nodes_r<VW, 8, 1>(P, R, lr, lsp, nl, s); break;
      case 16: launch_nodes_r<VW, 16, 1>(P, R, lr, lsp, nl, s); break;
      case 32: launch_nodes_r<VW, 32, 1>(P, R, lr, lsp, nl, s); break;
      default: launch_nodes_r<VW, 64, 1>(P, R, lr, lsp, nl, s); break;
    }
  } else if (nv <= 128) {
    launch_nodes_r<VW, 64, 2>(P, R, lr, lsp, nl, s);
  } else {
    launch_nodes_r<VW, 64, 4>(P, R, lr, lsp, nl, s);
  }
  return launch_status();
}

}  // namespace gnn

using namespace gnn;

extern "C" int gnn_gat_backward_prep_f32(const float* dy, const float* y, int64_t ldo,
                                         int64_t n_rows, int64_t heads, int64_t fh, int32_t elu,
                                         float* dout, float* D, void* stream) {
  if (n_rows < 0 || heads < 1 || fh < 1 || ldo < heads * fh) return GNN_E_ARG;
  if (n_rows == 0) return GNN_OK;
  if (!dy || !y || !dout || !D) return GNN_E_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t g = fh / 4;
  if (fh % 4 == 0 && (g & (g - 1)) == 0 && g <= 64 && ldo % 4 == 0 && aligned_to(dy, 16) &&
      aligned_to(y, 16) && aligned_to(dout, 16)) {
    const int64_t tv = n_rows * heads * g;
    const dim3 grid(static_cast<unsigned>((tv + 255) / 256));
    switch (g) {
      case 1: hipLaunchKernelGGL(gat_bwd_prep_vec_kernel<1>, grid, dim3(256), 0, s, dy, y, ldo, n_rows, heads, elu, dout, D); break;
      case 2: hipLaunchKernelGGL(gat_bwd_prep_vec_kernel<2>, grid, dim3(256), 0, s, dy, y, ldo, n_rows, heads, elu, dout, D); break;
      case 4: hipLaunchKernelGGL(gat_bwd_prep_vec_kernel<4>, grid, dim3(256), 0, s, dy, y, ldo, n_rows, heads, elu, dout, D); break;
      case 8: hipLaunchKernelGGL(gat_bwd_prep_vec_kernel<8>, grid, dim3(256), 0, s, dy, y, ldo, n_rows, heads, elu, dout, D); break;
      case 16: hipLaunchKernelGGL(gat_bwd_prep_vec_kernel<16>, grid, dim3(256), 0, s, dy, y, ldo, n_rows, heads, elu, dout, D); break;
      case 32: hipLaunchKernelGGL(gat_bwd_prep_vec_kernel<32>, grid, dim3(256), 0, s, dy, y, ldo, n_rows, heads, elu, dout, D); break;
      default: hipLaunchKernelGGL(gat_bwd_prep_vec_kernel<64>, grid, dim3(256), 0, s, dy, y, ldo, n_rows, heads, elu, dout, D); break;
    }
    return launch_status();
  }
  const int64_t t = n_rows * heads;
  hipLaunchKernelGGL(gat_bwd_prep_kernel, dim3(static_cast<unsigned>((t + 255) / 256)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), dy, y, ldo, n_rows, heads, fh, elu, dout, D);
  return launch_status();
}

extern "C" int gnn_gat_backward_edges_f32(
    const int64_t* rowptr, const int32_t* col, int64_t n_rows, const float* wh, int64_t ldw,
    int64_t heads, int64_t fh, const float* el, const float* er, const float* lse,
    const float* dout, const float* D, float negative_slope, int32_t mode, float dropout_p,
    uint64_t dropout_seed, float* w_edge, float* ds_edge, float* del, int64_t seg_len,
    const int32_t* seg_row, const int64_t* seg_begin, int64_t n_seg, const int32_t* long_row,
    const int32_t* long_seg_ptr, int64_t n_long, const int32_t* rows, int64_t n_rows_list,
    float* del_part, void* stream) {
  if (n_rows < 0 || heads < 1 || fh < 1 || ldw < heads * fh || n_seg < 0 || n_long < 0 ||
      n_rows_list < 0 || seg_len < 1 || (mode != 0 && mode != 1))
    return GNN_E_ARG;
  if (!(dropout_p >= 0.f && dropout_p < 1.f)) return GNN_E_ARG;
  if (n_rows == 0) return GNN_OK;
  if (!rowptr || !wh || !el || !er || !lse || !dout || !D || !w_edge || !ds_edge || !del)
    return GNN_E_ARG;
  if (n_seg > 0 && (!seg_row || !seg_begin || !long_row || !long_seg_ptr || !del_part))
    return GNN_E_ARG;
  if (n_rows_list > 0 && !rows) return GNN_E_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool vec4 = fh % 4 == 0 && ldw % 4 == 0 && aligned_to(wh, 16) && aligned_to(dout, 16);
  for (int64_t h0 = 0; h0 < heads; h0 += 8) {
    const int64_t hg = heads - h0 < 8 ? heads - h0 : 8;
    BwdEdgeParams P{};
    P.rowptr = rowptr;
    P.col = col;
    P.wh = wh + h0 * fh;
    P.ldw = ldw;
    P.el = el + h0;
    P.er = er + h0;
    P.lse = lse + h0;
    P.dout = dout + h0 * fh;
    P.D = D + h0;
    P.heads = static_cast<int>(hg);
    P.H = heads;
    P.fh = fh;
    P.slope = negative_slope;
    P.drop_p = dropout_p;
    P.drop_scale = dropout_p > 0.f ? 1.f / (1.f - dropout_p) : 1.f;
    P.drop_seed = dropout_seed;
    P.head0 = static_cast<int>(h0);
    P.w_edge = w_edge + h0;
    P.ds_edge = ds_edge + h0;
    P.del = del + h0;
    P.del_part = del_part ? del_part + h0 : nullptr;
    P.seg_len = seg_len;
    P.seg_row = seg_row;
    P.seg_begin = seg_begin;
    P.n_seg = n_seg;
    P.rows = rows;
    P.n_rows_list = n_rows_list;
    // dout row stride is heads*fh: P.dout rows are indexed with (H * fh) inside the kernel
    const int HPsel = hg <= 1 ? 1 : hg <= 2 ? 2 : hg <= 4 ? 4 : 8;
#define GNN_EDGES(VW, HP)                                                       \
  (mode == 1 ? launch_edges<VW, HP, true>(P, s) : launch_edges<VW, HP, false>(P, s))
    if (vec4) {
      switch (HPsel) {
        case 1: GNN_EDGES(4, 1); break;
        case 2: GNN_EDGES(4, 2); break;
        case 4: GNN_EDGES(4, 4); break;
        default: GNN_EDGES(4, 8); break;
      }
    } else {
      switch (HPsel) {
        case 1: GNN_EDGES(1, 1); break;
        case 2: GNN_EDGES(1, 2); break;
        case 4: GNN_EDGES(1, 4); break;
        default: GNN_EDGES(1, 8); break;
      }
    }
#undef GNN_EDGES
    if (n_long > 0) {
      const int64_t t = n_long * hg;
      hipLaunchKernelGGL(gat_bwd_del_fixup_kernel, dim3(static_cast<unsigned>((t + 255) / 256)),
                         dim3(256), 0, s, long_row, long_seg_ptr, n_long, hg, heads, h0, del_part,
                         del);
    }
    const int rc = launch_status();
    if (rc != GNN_OK) return rc;
  }
  return GNN_OK;
}

extern "C" int gnn_gat_backward_nodes_f32(
    const int64_t* rowptr_t, const int32_t* src_t, const int64_t* eid_t, int64_t n_nodes,
    int64_t heads, int64_t fh, const float* dout, const float* w_edge, const float* ds_edge,
    const float* del, const float* a_src, const float* a_dst, float* dwh, float* der,
    int64_t seg_len, const int32_t* seg_row, const int64_t* seg_begin, int64_t n_seg,
    const int32_t* long_row, const int32_t* long_seg_ptr, int64_t n_long, const int32_t* rows,
    int64_t n_rows_list, float* part, void* stream) {
  if (n_nodes < 0 || heads < 1 || fh < 1 || n_seg < 0 || n_long < 0 || n_rows_list < 0 ||
      seg_len < 1)
    return GNN_E_ARG;
  if (n_nodes == 0) return GNN_OK;
  if (!rowptr_t || !dout || !w_edge || !ds_edge || !del || !a_src || !a_dst || !dwh || !der)
    return GNN_E_ARG;
  if (n_seg > 0 && (!seg_row || !seg_begin || !long_row || !long_seg_ptr || !part))
    return GNN_E_ARG;
  if (n_rows_list > 0 && !rows) return GNN_E_ARG;
  BwdNodeParams P{};
  P.rowptr_t = rowptr_t;
  P.src_t = src_t;
  P.eid_t = eid_t;
  P.n_nodes = n_nodes;
  P.dout = dout;
  P.w_edge = w_edge;
  P.ds_edge = ds_edge;
  P.del = del;
  P.a_src = a_src;
  P.a_dst = a_dst;
  P.H = heads;
  P.fh = fh;
  P.feat = heads * fh;
  P.dwh = dwh;
  P.der = der;
  P.part = part;
  P.ldp = P.feat + heads;
  P.seg_len = seg_len;
  P.seg_row = seg_row;
  P.seg_begin = seg_begin;
  P.n_seg = n_seg;
  P.rows = rows;
  P.n_rows_list = n_rows_list;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool vec4 = fh % 4 == 0 && aligned_to(dout, 16) && aligned_to(dwh, 16) &&
                    aligned_to(a_src, 16) && aligned_to(a_dst, 16) &&
                    (part == nullptr || (aligned_to(part, 16) && P.ldp % 4 == 0));
  const int HPsel = heads <= 1 ? 1 : heads <= 2 ? 2 : heads <= 4 ? 4 : 8;
#define GNN_NODES(VW, HP) return dispatch_nodes<VW, HP>(P, long_row, long_seg_ptr, n_long, s)
  if (vec4) {
    switch (HPsel) {
      case 1: GNN_NODES(4, 1);
      case 2: GNN_NODES(4, 2);
      case 4: GNN_NODES(4, 4);
      default: GNN_NODES(4, 8);
    }
  }
  switch (HPsel) {
    case 1: GNN_NODES(1, 1);
    case 2: GNN_NODES(1, 2);
    case 4: GNN_NODES(1, 4);
    default: GNN_NODES(1, 8);
  }
#undef GNN_NODES
}

static int hp_for(int64_t heads) { return heads <= 1 ? 1 : heads <= 2 ? 2 : heads <= 4 ? 4 : 8; }

extern "C" int gnn_gat_backward_rows_ex_f32(
    const int64_t* rowptr, const int32_t* col, int64_t n_rows, const float* wh, int64_t ldw,
    int64_t heads, int64_t fh, const float* el, const float* er, const float* lse, const float* dy,
    const float* y, int64_t ldo, int32_t elu, float negative_slope, int32_t mode, float dropout_p,
    uint64_t dropout_seed, float* dout, float* nstat, float* del, int64_t seg_len,
    const int32_t* seg_row, const int64_t* seg_begin, int64_t n_seg, const int32_t* long_row,
    const int32_t* long_seg_ptr, int64_t n_long, const int32_t* rows, int64_t n_rows_list,
    const int32_t* short_rows, int64_t n_short, float* del_part, const float* a_dst,
    float dy_dropout_p, uint64_t dy_dropout_seed, void* stream);

extern "C" int gnn_gat_backward_rows_f32(
    const int64_t* rowptr, const int32_t* col, int64_t n_rows, const float* wh, int64_t ldw,
    int64_t heads, int64_t fh, const float* el, const float* er, const float* lse, const float* dy,
    const float* y, int64_t ldo, int32_t elu, float negative_slope, int32_t mode, float dropout_p,
    uint64_t dropout_seed, float* dout, float* nstat, float* del, int64_t seg_len,
    const int32_t* seg_row, const int64_t* seg_begin, int64_t n_seg, const int32_t* long_row,
    const int32_t* long_seg_ptr, int64_t n_long, const int32_t* rows, int64_t n_rows_list,
    const int32_t* short_rows, int64_t n_short, float* del_part, const float* a_dst,
    void* stream) {
  return gnn_gat_backward_rows_ex_f32(rowptr, col, n_rows, wh, ldw, heads, fh, el, er, lse, dy, y,
                                      ldo, elu, negative_slope, mode, dropout_p, dropout_seed,
                                      dout, nstat, del, seg_len, seg_row, seg_begin, n_seg,
                                      long_row, long_seg_ptr, n_long, rows, n_rows_list,
                                      short_rows, n_short, del_part, a_dst, 0.f, 0, stream);
}

extern "C" int gnn_gat_backward_rows_ex_f32(
    const int64_t* rowptr, const int32_t* col, int64_t n_rows, const float* wh, int64_t ldw,
    int64_t heads, int64_t fh, const float* el, const float* er, const float* lse, const float* dy,
    const float* y, int64_t ldo, int32_t elu, float negative_slope, int32_t mode, float dropout_p,
    uint64_t dropout_seed, float* dout, float* nstat, float* del, int64_t seg_len,
    const int32_t* seg_row, const int64_t* seg_begin, int64_t n_seg, const int32_t* long_row,
    const int32_t* long_seg_ptr, int64_t n_long, const int32_t* rows, int64_t n_rows_list,
    const int32_t* short_rows, int64_t n_short, float* del_part, const float* a_dst,
    float dy_dropout_p, uint64_t dy_dropout_seed, void* stream) {
  const int64_t feat = heads * fh;
  if (n_rows < 0 || heads < 1 || fh < 1 || ldw < feat || ldo < feat || n_seg < 0 || n_long < 0 ||
      n_rows_list < 0 || n_short < 0 || seg_len < 1 || (mode != 0 && mode != 1))
    return GNN_E_ARG;
  if (!(dropout_p >= 0.f && dropout_p < 1.f)) return GNN_E_ARG;
  if (!(dy_dropout_p >= 0.f && dy_dropout_p < 1.f)) return GNN_E_ARG;
  if (n_rows == 0) return GNN_OK;
  if (!rowptr || !wh || !el || !er || !lse || !dy || !y || !dout || !nstat || !del) return GNN_E_ARG;
  if (!aligned_to(nstat, 16)) return GNN_E_ALIGN;
  if (n_seg > 0 && (!seg_row || !seg_begin || !long_row || !long_seg_ptr || !del_part))
    return GNN_E_ARG;
  if ((n_rows_list > 0 && !rows) || (n_short > 0 && !short_rows)) return GNN_E_ARG;
  // the prep's LDS: dout and products of the wave's rows, D per (row, head)
  if (2 * feat + heads > kRowLds || (n_short > 0 && kShortRowsW * (2 * feat + heads) > kRowLds))
    return GNN_E_UNSUPPORTED;
  BwdRowParams P{};
  P.rowptr = rowptr;
  P.col = col;
  P.wh = wh;
  P.ldw = ldw;
  P.el = el;
  P.er = er;
  P.lse = lse;
  P.dy = dy;
  P.y = y;
  P.ldo = ldo;
  P.elu = elu != 0;
  P.sparse = mode;
  P.hp = hp_for(heads);
  P.H = heads;
  P.fh = fh;
  P.feat = feat;
  P.slope = negative_slope;
  P.drop_p = dropout_p;
  P.drop_scale = dropout_p > 0.f ? 1.f / (1.f - dropout_p) : 1.f;
  P.drop_seed = dropout_seed;
  P.dout = dout;
  P.nstat = nstat;
  P.del = del;
  P.del_part = del_part;
  P.seg_len = seg_len;
  P.seg_row = seg_row;
  P.seg_begin = seg_begin;
  P.n_seg = n_seg;
  P.rows = rows;
  P.n_rows_list = n_rows_list;
  P.short_rows = short_rows;
  P.n_short = n_short;
  const int64_t seg_blocks = (n_seg + kBwWaves - 1) / kBwWaves;
  const int64_t row_blocks = (n_rows_list + kBwWaves - 1) / kBwWaves;
  const int64_t short_waves = (n_short + kShortRowsW - 1) / kShortRowsW;
  const int64_t blocks = seg_blocks + row_blocks + (short_waves + kBwWaves - 1) / kBwWaves;
  P.seg_waves = seg_blocks * kBwWaves;
  P.row_waves = row_blocks * kBwWaves;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool vec4 = fh % 4 == 0 && ldw % 4 == 0 && ldo % 4 == 0 && aligned_to(wh, 16) &&
                    aligned_to(dy, 16) && aligned_to(y, 16) && aligned_to(dout, 16) &&
                    (a_dst == nullptr || aligned_to(a_dst, 16));
  const int64_t nfv = vec4 ? fh / 4 : fh;
  P.a_dst = a_dst;
  const dim3 grid(static_cast<unsigned>(blocks));
  // the prep as its own coalesced pass (a float4 per thread, D summed over the head's lanes)
  // when the head's features are whole float4s, 2^k of them; else fused into the row pass
  const bool rec = a_dst != nullptr;
  const int64_t g4 = fh / 4;
  const bool split = GNN_BWD_SPLIT_PREP && vec4 && (g4 & (g4 - 1)) == 0 && g4 <= 64 &&
                     aligned_to(nstat, 16);
  // the upstream dropout mask is applied by the coalesced prep only (the caller masks dy itself
  // for the shapes that fuse the prep into the row pass)
  if (dy_dropout_p > 0.f && (!split || ldo != feat)) return GNN_E_UNSUPPORTED;
  const float dy_scale = dy_dropout_p > 0.f ? 1.f / (1.f - dy_dropout_p) : 1.f;
  if (split) {
    const int64_t tv = n_rows * heads * g4;
    const dim3 pg(static_cast<unsigned>((tv + 255) / 256));
#define GNN_PREP(G) hipLaunchKernelGGL(gat_bwd_prep_rec_kernel<G>, pg, dim3(256), 0, s, dy, y, ldo, n_rows, heads, static_cast<int>(elu != 0), el, lse, dout, nstat, dy_dropout_p, dy_scale, dy_dropout_seed)
    switch (g4) {
      case 1: GNN_PREP(1); break;
      case 2: GNN_PREP(2); break;
      case 4: GNN_PREP(4); break;
      case 8: GNN_PREP(8); break;
      case 16: GNN_PREP(16); break;
      case 32: GNN_PREP(32); break;
      default: GNN_PREP(64); break;
    }
#undef GNN_PREP
  }
  if (blocks > 0) {
#define GNN_ROWS(VW, NFV)                                                                       \
  do {                                                                                          \
    if (split && rec)                                                                           \
      hipLaunchKernelGGL((gat_bwd_rows_kernel<VW, NFV, false, NFV != 0>), grid, dim3(kBw), 0, s, \
                         P);                                                                    \
    else if (split)                                                                             \
      hipLaunchKernelGGL((gat_bwd_rows_kernel<VW, NFV, false, false>), grid, dim3(kBw), 0, s, P); \
    else if (rec)                                                                               \
      hipLaunchKernelGGL((gat_bwd_rows_kernel<VW, NFV, true, NFV != 0>), grid, dim3(kBw), 0, s,  \
                         P);                                                                    \
    else                                                                                        \
      hipLaunchKernelGGL((gat_bwd_rows_kernel<VW, NFV, true, false>), grid, dim3(kBw), 0, s, P); \
  } while (0)
    if (vec4) {
      switch (nfv) {
        case 1: GNN_ROWS(4, 1); break;
        case 2: GNN_ROWS(4, 2); break;
        case 4: GNN_ROWS(4, 4); break;
        default: GNN_ROWS(4, 0); break;
      }
    } else {
      switch (nfv) {
        case 1: GNN_ROWS(1, 1); break;
        case 2: GNN_ROWS(1, 2); break;
        case 4: GNN_ROWS(1, 4); break;
        default: GNN_ROWS(1, 0); break;
      }
    }
#undef GNN_ROWS
  }
  if (n_long > 0) {
    const int64_t t = n_long * heads;
    hipLaunchKernelGGL(gat_bwd_del_fixup_kernel, dim3(static_cast<unsigned>((t + 255) / 256)),
                       dim3(256), 0, s, long_row, long_seg_ptr, n_long, heads, heads,
                       static_cast<int64_t>(0), del_part, del);
  }
  return launch_status();
}

extern "C" int gnn_gat_backward_nodes_recompute_f32(
    const int64_t* rowptr_t, const int32_t* src_t, const int64_t* eid_t, int64_t n_nodes,
    int64_t heads, int64_t fh, const float* dout, const float* nstat, const float* wh,
    int64_t ldw, const float* er, const float* del, const float* a_src, const float* a_dst,
    float negative_slope, int32_t mode, float dropout_p, uint64_t dropout_seed, float* dwh,
    float* der, int64_t seg_len, const int32_t* seg_row, const int64_t* seg_begin, int64_t n_seg,
    const int32_t* long_row, const int32_t* long_seg_ptr, int64_t n_long, const int32_t* rows,
    int64_t n_rows_list, const int32_t* short_rows, int64_t n_short, float* part, void* stream) {
  const int64_t feat = heads * fh;
  if (n_nodes < 0 || heads < 1 || fh < 1 || ldw < feat || n_seg < 0 || n_long < 0 ||
      n_rows_list < 0 || n_short < 0 || seg_len < 1 || (mode != 0 && mode != 1))
    return GNN_E_ARG;
  if (!(dropout_p >= 0.f && dropout_p < 1.f)) return GNN_E_ARG;
  if (n_nodes == 0) return GNN_OK;
  if (!rowptr_t || !dout || !nstat || !wh || !er || !del || !a_src || !a_dst || !dwh || !der)
    return GNN_E_ARG;
  if (dropout_p > 0.f && !eid_t) return GNN_E_ARG;
  if (!aligned_to(nstat, 16)) return GNN_E_ALIGN;
  if (n_seg > 0 && (!seg_row || !seg_begin || !long_row || !long_seg_ptr || !part))
    return GNN_E_ARG;
  if ((n_rows_list > 0 && !rows) || (n_short > 0 && !short_rows)) return GNN_E_ARG;
  const int64_t ldp = feat + heads;
  const bool vec4 = fh % 4 == 0 && ldw % 4 == 0 && aligned_to(dout, 16) && aligned_to(wh, 16) &&
                    aligned_to(dwh, 16) && aligned_to(a_src, 16) && aligned_to(a_dst, 16) &&
                    (part == nullptr || (aligned_to(part, 16) && ldp % 4 == 0));
  const int VW = vec4 ? 4 : 1;
  const int64_t G = fh / VW;  // lanes of one head: a power of two inside one lane row
  const int lpr = node_r_lpr((feat + VW - 1) / VW);
  if (fh % VW != 0 || (G & (G - 1)) != 0 || lpr == 0 || G > lpr) return GNN_E_UNSUPPORTED;
  BwdNodeParams P{};
  P.rowptr_t = rowptr_t;
  P.src_t = src_t;
  P.eid_t = eid_t;
  P.n_nodes = n_nodes;
  P.del = del;
  P.a_src = a_src;
  P.a_dst = a_dst;
  P.H = heads;
  P.fh = fh;
  P.feat = feat;
  P.dwh = dwh;
  P.der = der;
  P.part = part;
  P.ldp = ldp;
  P.seg_len = seg_len;
  P.seg_row = seg_row;
  P.seg_begin = seg_begin;
  P.n_seg = n_seg;
  P.rows = rows;
  P.n_rows_list = n_rows_list;
  BwdNodeRParams R{};
  R.rowptr_t = rowptr_t;
  R.src_t = src_t;
  R.eid_t = eid_t;
  R.dout = dout;
  R.nstat = nstat;
  R.wh = wh;
  R.ldw = ldw;
  R.er = er;
  R.sparse = mode;
  R.G = static_cast<int>(G);
  R.slope = negative_slope;
  R.drop_p = dropout_p;
  R.drop_scale = dropout_p > 0.f ? 1.f / (1.f - dropout_p) : 1.f;
  R.drop_seed = dropout_seed;
  R.short_rows = short_rows;
  R.n_short = n_short;
  hipStream_t s = static_cast<hipStream_t>(stream);
  return vec4 ? dispatch_nodes_r<4>(P, R, long_row, long_seg_ptr, n_long, s)
              : dispatch_nodes_r<1>(P, R, long_row, long_seg_ptr, n_long, s);
}
