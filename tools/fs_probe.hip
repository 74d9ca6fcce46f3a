// fs_probe.hip -- feature-sliced SpMM probe (measurement harness, not the library).
//
// Question: the gathers of the CSR SpMM at cfg2 are served by L2 at ~50 G rows/s when the
// gathered set fits an XCD's 4 MiB L2 and at ~13 G rows/s from the Infinity Cache / HBM
// (profiles/r02y_workingset.log). With whole 512-B rows an XCD's L2 holds 8192 rows. Here
// XCD x gathers only a slice of the feature columns (F / SL floats, SL = 1, 2, 4, 8) for its
// share of the rows, so its L2 holds SL x more rows of the table: at SL = 4 the 32768 hottest
// columns (66 % of the cfg2 edges) in 128-B lines. Cost: each row's (col, val) list is read
// by SL XCDs.
//
// Workgroup w runs on XCD w % 8; slice = (w % 8) % SL, row half = (w % 8) / SL.
//   fs_short: rows of <= 64 edges, one lane group (F / SL / 4 lanes, a float4 each) per row
//   fs_seg:   segments ([begin, end) edge pairs) of longer rows, one wave per segment,
//             64 / LPG edge slots, partials
//   fs_fixup: sums a long row's segment partials in order
#include <hip/hip_runtime.h>
#include <cstdint>

namespace {

constexpr int kF = 128;
constexpr int kU = 8;  // gathers in flight per lane

template <int SL>
__global__ __launch_bounds__(256) void fs_short(const int64_t* __restrict__ rp,
                                                const int32_t* __restrict__ col,
                                                const float* __restrict__ val,
                                                const float* __restrict__ x,
                                                float* __restrict__ y,
                                                const int32_t* __restrict__ rows, int64_t n_rows_list,
                                                int wgs_per_class) {
  constexpr int FPS = kF / SL, LPG = FPS / 4, GPW = 64 / LPG, NH = 8 / SL;
  const int xcd = blockIdx.x & 7, slice = xcd % SL, half = xcd / SL;
  const int q = blockIdx.x >> 3;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int grp = lane / LPG, lig = lane % LPG;
  const int64_t n_tasks = (n_rows_list + GPW - 1) / GPW;
  const int64_t stride = static_cast<int64_t>(wgs_per_class) * 4;
  for (int64_t gw = static_cast<int64_t>(q) * 4 + wave;; gw += stride) {
    const int64_t t = gw * NH + half;
    if (t >= n_tasks) break;
    const int64_t li = t * GPW + grp;
    const bool live = li < n_rows_list;
    const int32_t r = live ? rows[li] : 0;
    const int64_t e0 = live ? rp[r] : 0, e1 = live ? rp[r + 1] : 0;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    const float* xs = x + slice * FPS + lig * 4;
    for (int64_t e = e0; e < e1; e += kU) {
      int32_t c[kU];
      float v[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const bool ok = e + u < e1;
        c[u] = ok ? col[e + u] : 0;
        v[u] = ok ? val[e + u] : 0.f;
      }
      float4 g[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u)
        g[u] = *reinterpret_cast<const float4*>(xs + static_cast<int64_t>(c[u]) * kF);
#pragma unroll
      for (int u = 0; u < kU; ++u)
        if (e + u < e1) {
          acc.x = fmaf(v[u], g[u].x, acc.x);
          acc.y = fmaf(v[u], g[u].y, acc.y);
          acc.z = fmaf(v[u], g[u].z, acc.z);
          acc.w = fmaf(v[u], g[u].w, acc.w);
        }
    }
    if (live)
      *reinterpret_cast<float4*>(y + static_cast<int64_t>(r) * kF + slice * FPS + lig * 4) = acc;
  }
}

template <int SL>
__global__ __launch_bounds__(256) void fs_seg(const int32_t* __restrict__ col,
                                              const float* __restrict__ val,
                                              const float* __restrict__ x,
                                              const int64_t* __restrict__ seg_e, int64_t n_seg,
                                              float* __restrict__ part, int wgs_per_class) {
  constexpr int FPS = kF / SL, LPG = FPS / 4, GPW = 64 / LPG, NH = 8 / SL, UU = 4;
  const int xcd = blockIdx.x & 7, slice = xcd % SL, half = xcd / SL;
  const int q = blockIdx.x >> 3;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int grp = lane / LPG, lig = lane % LPG;
  const int64_t stride = static_cast<int64_t>(wgs_per_class) * 4;
  for (int64_t gw = static_cast<int64_t>(q) * 4 + wave;; gw += stride) {
    const int64_t s = gw * NH + half;
    if (s >= n_seg) break;
    const int64_t e0 = seg_e[2 * s], e1 = seg_e[2 * s + 1];  // [begin, end) pairs
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    const float* xs = x + slice * FPS + lig * 4;
    for (int64_t e = e0 + grp; e < e1; e += GPW * UU) {
      int32_t c[UU];
      float v[UU];
#pragma unroll
      for (int u = 0; u < UU; ++u) {
        const bool ok = e + u * GPW < e1;
        c[u] = ok ? col[e + u * GPW] : 0;
        v[u] = ok ? val[e + u * GPW] : 0.f;
      }
      float4 g[UU];
#pragma unroll
      for (int u = 0; u < UU; ++u)
        g[u] = *reinterpret_cast<const float4*>(xs + static_cast<int64_t>(c[u]) * kF);
#pragma unroll
      for (int u = 0; u < UU; ++u)
        if (e + u * GPW < e1) {
          acc.x = fmaf(v[u], g[u].x, acc.x);
          acc.y = fmaf(v[u], g[u].y, acc.y);
          acc.z = fmaf(v[u], g[u].z, acc.z);
          acc.w = fmaf(v[u], g[u].w, acc.w);
        }
    }
#pragma unroll
    for (int o = LPG; o < 64; o <<= 1) {
      acc.x += __shfl_xor(acc.x, o, 64);
      acc.y += __shfl_xor(acc.y, o, 64);
      acc.z += __shfl_xor(acc.z, o, 64);
      acc.w += __shfl_xor(acc.w, o, 64);
    }
    if (grp == 0)
      *reinterpret_cast<float4*>(part + s * kF + slice * FPS + lig * 4) = acc;
  }
}

// Every row as work items [e0, e1, dst] of at most SEGL edges (dst >= 0: the output row;
// dst < 0: partial -1 - dst of a long row), sorted by length so that the lane groups of a
// wave walk items of about the same length. One lane group per item, software-pipelined:
// the (col, val) of the next kU edges are requested behind the current kU gathers.
template <int SL>
__global__ __launch_bounds__(256) void fs_items(const int32_t* __restrict__ col,
                                                const float* __restrict__ val,
                                                const float* __restrict__ x, float* __restrict__ y,
                                                float* __restrict__ part,
                                                const int64_t* __restrict__ items, int64_t n_items,
                                                int wgs_per_class) {
  constexpr int FPS = kF / SL, LPG = FPS / 4, GPW = 64 / LPG, NH = 8 / SL;
  const int xcd = blockIdx.x & 7, slice = xcd % SL, half = xcd / SL;
  const int q = blockIdx.x >> 3;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int grp = lane / LPG, lig = lane % LPG;
  const int64_t n_tasks = (n_items + GPW - 1) / GPW;
  const int64_t stride = static_cast<int64_t>(wgs_per_class) * 4;
  const float* xs = x + slice * FPS + lig * 4;
  for (int64_t gw = static_cast<int64_t>(q) * 4 + wave;; gw += stride) {
    const int64_t t = gw * NH + half;
    if (t >= n_tasks) break;
    const int64_t it = t * GPW + grp;
    const bool live = it < n_items;
    const int64_t e0 = live ? items[3 * it] : 0, e1 = live ? items[3 * it + 1] : 0;
    const int64_t dst = live ? items[3 * it + 2] : 0;
    int32_t c[kU];
    float v[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const bool ok = e0 + u < e1;
      c[u] = ok ? col[e0 + u] : 0;
      v[u] = ok ? val[e0 + u] : 0.f;
    }
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t e = e0; e < e1; e += kU) {
      float4 g[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u)
        g[u] = *reinterpret_cast<const float4*>(xs + static_cast<int64_t>(c[u]) * kF);
      float vv[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) vv[u] = v[u];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const bool ok = e + kU + u < e1;
        c[u] = ok ? col[e + kU + u] : 0;
        v[u] = ok ? val[e + kU + u] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {  // vv = 0 past the end: the row 0 gather adds 0 * x
        acc.x = fmaf(vv[u], g[u].x, acc.x);
        acc.y = fmaf(vv[u], g[u].y, acc.y);
        acc.z = fmaf(vv[u], g[u].z, acc.z);
        acc.w = fmaf(vv[u], g[u].w, acc.w);
      }
    }
    if (live) {
      float* o = dst >= 0 ? y + dst * kF : part + (-1 - dst) * kF;
      *reinterpret_cast<float4*>(o + slice * FPS + lig * 4) = acc;
    }
  }
}

__global__ void fs_fixup(const int32_t* __restrict__ lrow, const int64_t* __restrict__ lseg,
                         int64_t n_long, const float* __restrict__ part, float* __restrict__ y) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= n_long * (kF / 4)) return;
  const int64_t i = t / (kF / 4);
  const int f4 = static_cast<int>(t % (kF / 4));
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t s = lseg[i]; s < lseg[i + 1]; ++s) {
    const float4 p = reinterpret_cast<const float4*>(part + s * kF)[f4];
    a.x += p.x;
    a.y += p.y;
    a.z += p.z;
    a.w += p.w;
  }
  reinterpret_cast<float4*>(y + static_cast<int64_t>(lrow[i]) * kF)[f4] = a;
}

template <int SL>
int run(const int64_t* rp, const int32_t* col, const float* val, const float* x, float* y,
        const int32_t* rows, int64_t n_rows_list, const int64_t* seg_e, int64_t n_seg,
        const int32_t* lrow, const int64_t* lseg, int64_t n_long, float* part, int wgs_per_xcd,
        hipStream_t s) {
  const dim3 g(8 * wgs_per_xcd);
  const int per_class = wgs_per_xcd;  // XCD x is the one (slice, half) class x
  if (n_rows_list > 0)
    hipLaunchKernelGGL(fs_short<SL>, g, dim3(256), 0, s, rp, col, val, x, y, rows, n_rows_list,
                       per_class);
  if (n_seg > 0) {
    hipLaunchKernelGGL(fs_seg<SL>, g, dim3(256), 0, s, col, val, x, seg_e, n_seg, part, per_class);
    const int64_t th = n_long * (kF / 4);
    hipLaunchKernelGGL(fs_fixup, dim3(static_cast<unsigned>((th + 255) / 256)), dim3(256), 0, s,
                       lrow, lseg, n_long, part, y);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}


template <int SL>
int run_items(const int32_t* col, const float* val, const float* x, float* y, const int64_t* items,
              int64_t n_items, const int32_t* lrow, const int64_t* lseg, int64_t n_long, float* part,
              int wgs_per_xcd, hipStream_t s) {
  hipLaunchKernelGGL(fs_items<SL>, dim3(8 * wgs_per_xcd), dim3(256), 0, s, col, val, x, y, part,
                     items, n_items, wgs_per_xcd);
  if (n_long > 0) {
    const int64_t th = n_long * (kF / 4);
    hipLaunchKernelGGL(fs_fixup, dim3(static_cast<unsigned>((th + 255) / 256)), dim3(256), 0, s,
                       lrow, lseg, n_long, part, y);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace

extern "C" int fs_probe_items(int sl, const int32_t* col, const float* val, const float* x,
                              float* y, const int64_t* items, int64_t n_items, const int32_t* lrow,
                              const int64_t* lseg, int64_t n_long, float* part, int wgs_per_xcd,
                              void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (sl) {
    case 1: return run_items<1>(col, val, x, y, items, n_items, lrow, lseg, n_long, part, wgs_per_xcd, s);
    case 2: return run_items<2>(col, val, x, y, items, n_items, lrow, lseg, n_long, part, wgs_per_xcd, s);
    case 4: return run_items<4>(col, val, x, y, items, n_items, lrow, lseg, n_long, part, wgs_per_xcd, s);
    case 8: return run_items<8>(col, val, x, y, items, n_items, lrow, lseg, n_long, part, wgs_per_xcd, s);
    default: return -2;
  }
}

extern "C" int fs_probe_run(int sl, const int64_t* rp, const int32_t* col, const float* val,
                            const float* x, float* y, const int32_t* rows, int64_t n_rows_list,
                            const int64_t* seg_e, int64_t n_seg, const int32_t* lrow,
                            const int64_t* lseg, int64_t n_long, float* part, int wgs_per_xcd,
                            void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (sl) {
    case 1: return run<1>(rp, col, val, x, y, rows, n_rows_list, seg_e, n_seg, lrow, lseg, n_long, part, wgs_per_xcd, s);
    case 2: return run<2>(rp, col, val, x, y, rows, n_rows_list, seg_e, n_seg, lrow, lseg, n_long, part, wgs_per_xcd, s);
    case 4: return run<4>(rp, col, val, x, y, rows, n_rows_list, seg_e, n_seg, lrow, lseg, n_long, part, wgs_per_xcd, s);
    case 8: return run<8>(rp, col, val, x, y, rows, n_rows_list, seg_e, n_seg, lrow, lseg, n_long, part, wgs_per_xcd, s);
    default: return -2;
  }
}
