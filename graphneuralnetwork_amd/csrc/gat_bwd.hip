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
