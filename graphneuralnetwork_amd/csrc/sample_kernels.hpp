// sample_kernels.hpp -- the per-node neighbour draw of GraphSAGE sampling (shared by
// sample.hip's gnn_sample_neighbors and frontier.hip's fused gnn_sample_layers).
//
// Restates get_layer_adj_nodes' per-node draw (GraphSAGE/data_utils.py:89-94):
//   deg >  k : random.sample(neighs, k)   -- k distinct neighbours (no replacement)
//   deg <= k : random.choices(neighs, k)  -- k draws with replacement
//   deg == 0 : the reference raises IndexError (random.choices of an empty list)
// for a whole frontier at once, one thread per frontier node, with a counter-based hash RNG
// keyed by (seed, position in `nodes`, draw) instead of CPython's Mersenne Twister (the
// reference sampler is unseeded, so only the distribution -- not the exact draw -- is
// reproducible). Keying by position, not node id, makes a node listed twice draw two
// independent neighbour lists, as the reference's sequential draws do; the host derives `seed`
// per (batch seed, layer). Without replacement uses Robert Floyd's algorithm: k iterations,
// each a uniform draw and a membership test against the <= k picks so far.
//
// Output row i is out[i * ld + 0 .. k); with SELF (the gcn flag, data_utils.py:95-96) column k
// holds the node itself. n_dev (nullable): the live row count is min(*n_dev, n) -- the fused
// batch sampler chains hops on the device without reading sizes back to the host.
#pragma once

#include "common.hpp"

namespace gnn {

// sampler error bits (*err): 1 = a node without neighbours, 2 = a node id out of range
constexpr int32_t kSampleErrEmpty = 1;
constexpr int32_t kSampleErrRange = 2;

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

// uniform integer in [0, n) (n < 2^32 on this path; Lemire's multiply-shift)
__device__ __forceinline__ int64_t uniform_below(uint64_t seed, int64_t pos, int64_t draw, int64_t n) {
  const uint64_t r = mix64(seed ^ mix64(static_cast<uint64_t>(pos) * 0x100000001b3ull +
                                        static_cast<uint64_t>(draw)));
  if (n <= 0xffffffffll) return static_cast<int64_t>(((r >> 32) * static_cast<uint64_t>(n)) >> 32);
  return static_cast<int64_t>(r % static_cast<uint64_t>(n));
}

constexpr int kMaxFanout = 256;
#ifndef GNN_SAMPLE_THREAD_SERIAL
#define GNN_SAMPLE_THREAD_SERIAL 0  // A/B: the thread-per-node kernels for every k <= 32
#endif
constexpr bool kThreadSerialSample = GNN_SAMPLE_THREAD_SERIAL;

__device__ __forceinline__ int64_t live_rows(int64_t n, const int64_t* n_dev) {
  return n_dev ? min(*n_dev, n) : n;
}

// a row of -1 (and the node itself in the SELF column) for a node that cannot be sampled
__device__ __forceinline__ void sample_fail(int64_t* o, int k, bool self, int64_t v) {
  for (int j = 0; j < k; ++j) o[j] = -1;
  if (self) o[k] = v;
}

// Fanouts up to KMAX: Floyd's picks stay in registers (both loops unrolled over KMAX with
// a k predicate, so every array index is a compile-time constant) and the k column loads
// are issued together at the end. Same draws and picks as the generic path below.
template <int KMAX>
__global__ __launch_bounds__(256) void sample_reg_kernel(const int64_t* __restrict__ rowptr,
                                                         const int32_t* __restrict__ col,
                                                         int64_t n_graph,
                                                         const int64_t* __restrict__ nodes,
                                                         int64_t n, const int64_t* n_dev, int k,
                                                         int64_t ld, bool self, uint64_t seed,
                                                         int64_t* __restrict__ out,
                                                         int32_t* __restrict__ err) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= live_rows(n, n_dev)) return;
  const int64_t v = nodes[i];
  int64_t* o = out + i * ld;
  if (v < 0 || v >= n_graph) {
    atomicOr(err, kSampleErrRange);
    sample_fail(o, k, self, v);
    return;
  }
  const int64_t b = rowptr[v];
  const int64_t deg = rowptr[v + 1] - b;
  if (deg == 0) {
    atomicOr(err, kSampleErrEmpty);
    sample_fail(o, k, self, v);
    return;
  }
  int64_t pick[KMAX];
  if (deg <= k) {  // random.choices: k independent draws
#pragma unroll
    for (int j = 0; j < KMAX; ++j)
      pick[j] = j < k ? uniform_below(seed, i, j, deg) : 0;
  } else {         // random.sample: Floyd, draw j over [0, deg - k + jj]
#pragma unroll
    for (int jj = 0; jj < KMAX; ++jj) {
      if (jj < k) {
        const int64_t j = deg - k + jj;
        const int64_t t = uniform_below(seed, i, j, j + 1);
        bool seen = false;
#pragma unroll
        for (int q = 0; q < jj; ++q) seen |= (pick[q] == t);
        pick[jj] = seen ? j : t;
      }
    }
  }
  int64_t c[KMAX];
#pragma unroll
  for (int j = 0; j < KMAX; ++j) c[j] = j < k ? col[b + pick[j]] : 0;
#pragma unroll
  for (int j = 0; j < KMAX; ++j)
    if (j < k) o[j] = c[j];
  if (self) o[k] = v;
}

template <int UNUSED = 0>  // a template: the header is included by two translation units
__global__ __launch_bounds__(256) void sample_kernel(const int64_t* __restrict__ rowptr,
                                                     const int32_t* __restrict__ col,
                                                     int64_t n_graph,
                                                     const int64_t* __restrict__ nodes, int64_t n,
                                                     const int64_t* n_dev, int k, int64_t ld,
                                                     bool self, uint64_t seed,
                                                     int64_t* __restrict__ out,
                                                     int32_t* __restrict__ err) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= live_rows(n, n_dev)) return;
  const int64_t v = nodes[i];
  int64_t* o = out + i * ld;
  if (v < 0 || v >= n_graph) {
    atomicOr(err, kSampleErrRange);
    sample_fail(o, k, self, v);
    return;
  }
  const int64_t b = rowptr[v];
  const int64_t deg = rowptr[v + 1] - b;
  if (deg == 0) {
    atomicOr(err, kSampleErrEmpty);
    sample_fail(o, k, self, v);
    return;
  }
  if (self) o[k] = v;
  if (deg <= k) {  // random.choices: k independent draws
    for (int64_t j = 0; j < k; ++j) o[j] = col[b + uniform_below(seed, i, j, deg)];
    return;
  }
  // random.sample: Floyd -- positions chosen so far live in o[] (as offsets, then mapped)
  int64_t cnt = 0;
  for (int64_t j = deg - k; j < deg; ++j) {
    const int64_t t = uniform_below(seed, i, j, j + 1);
    bool seen = false;
    for (int64_t q = 0; q < cnt; ++q) seen |= (o[q] == t);
    o[cnt++] = seen ? j : t;
  }
  for (int64_t j = 0; j < k; ++j) o[j] = col[b + o[j]];
}

// Lane-parallel form of the same draws (fanouts k <= LPN <= 64): a group of LPN lanes per node,
// lane `sub` owns draw `sub`. The draws of Floyd's algorithm do not depend on earlier picks
// (draw jj is uniform_below(seed, i, j, j + 1), j = deg - k + jj), only the resolution does
// ("already picked? then take j"), so every lane draws at once and the resolution runs as k
// group-wide steps: step jj broadcasts lane jj's draw, the lanes q < jj compare it with their
// final picks, one ballot decides. Same picks as sample_reg_kernel, bit for bit, with a whole
// wave per 64 / LPN nodes instead of one thread per node (a thread-serial Floyd over k = 25 took
// 30.6 us for the 8192 seeds of a cfg4 batch: 128 waves for 256 CUs, profiles/r03ac_cfg4_*).
// The body of the lane-parallel sampler for one wave: node groups of LPN lanes, node i of
// `nodes` = wave * (64 / LPN) + lane / LPN. err == nullptr: the caller derives the sampler's
// error bits elsewhere (the fused batch does, in the next hop's rank pass). MARK: every drawn
// neighbour id and the node itself (ids inside [0, n_graph)) get flags[id] = 1 -- the batch
// frontier's marks, fused into the draw (frontier.hip, gnn_sample_layers).
template <int LPN, bool MARK>
__device__ __forceinline__ void sample_lane_wave(const int64_t* __restrict__ rowptr,
                                                 const int32_t* __restrict__ col, int64_t n_graph,
                                                 const int64_t* __restrict__ nodes, int64_t live,
                                                 int64_t wave, int k, int64_t ld, bool self,
                                                 uint64_t seed, int64_t* __restrict__ out,
                                                 int32_t* err, uint8_t* __restrict__ flags) {
  constexpr int GPW = kWave / LPN;  // node groups per wave
  const int lane = threadIdx.x & (kWave - 1);
  const int sub = lane & (LPN - 1);
  const int gbase = lane & ~(LPN - 1);
  const int64_t i = wave * GPW + lane / LPN;
  if (wave * GPW >= live) return;  // wave-uniform: every group of the wave is past the end
  const bool act = i < live;
  int64_t v = act ? nodes[i] : -1;
  int64_t b = 0, deg = 0;
  const bool ok = act && v >= 0 && v < n_graph;
  if (ok) {
    b = rowptr[v];
    deg = rowptr[v + 1] - b;
  }
  if (err != nullptr && act && sub == 0) {
    if (!ok) atomicOr(err, kSampleErrRange);
    else if (deg == 0) atomicOr(err, kSampleErrEmpty);
  }
  const bool good = ok && deg > 0;
  const bool floyd = good && deg > k;
  int64_t pick = 0;
  if (good && sub < k) {
    if (!floyd)
      pick = uniform_below(seed, i, sub, deg);      // random.choices: independent draws
    else {
      const int64_t j = deg - k + sub;
      pick = uniform_below(seed, i, j, j + 1);       // Floyd's draw jj = sub
    }
  }
  // Floyd's resolution, in draw order: lane jj's draw stands unless a lane q < jj already
  // holds it, then lane jj takes j = deg - k + jj (never held: earlier picks are < j)
  for (int jj = 1; jj < LPN; ++jj) {
    const int64_t t = __shfl(pick, gbase + jj, kWave);
    const uint64_t hit = __ballot(floyd && sub < jj && pick == t);
    const uint64_t gmask = (LPN == 64 ? ~0ull : ((1ull << LPN) - 1)) << gbase;
    if (floyd && sub == jj && jj < k && (hit & gmask)) pick = deg - k + jj;
  }
  if (!act) return;
  int64_t* o = out + i * ld;
  if (sub < k) {
    const int64_t id = good ? static_cast<int64_t>(col[b + pick]) : -1;
    o[sub] = id;
    if (MARK && id >= 0 && id < n_graph) flags[id] = 1;
  }
  if (sub == 0) {
    if (self) o[k] = v;
    if (MARK && ok) flags[v] = 1;
  }
}

// Lane-parallel form of the same draws (fanouts k <= LPN <= 64): a group of LPN lanes per node,
// lane `sub` owns draw `sub`. The draws of Floyd's algorithm do not depend on earlier picks
// (draw jj is uniform_below(seed, i, j, j + 1), j = deg - k + jj), only the resolution does
// ("already picked? then take j"), so every lane draws at once and the resolution runs as k
// group-wide steps: step jj broadcasts lane jj's draw, the lanes q < jj compare it with their
// final picks, one ballot decides. Same picks as sample_reg_kernel, bit for bit, with a whole
// wave per 64 / LPN nodes instead of one thread per node (a thread-serial Floyd over k = 25 took
// 30.6 us for the 8192 seeds of a cfg4 batch: 128 waves for 256 CUs, profiles/r03ac_cfg4_*).
template <int LPN>
__global__ __launch_bounds__(256) void sample_lane_kernel(const int64_t* __restrict__ rowptr,
                                                          const int32_t* __restrict__ col,
                                                          int64_t n_graph,
                                                          const int64_t* __restrict__ nodes,
                                                          int64_t n, const int64_t* n_dev, int k,
                                                          int64_t ld, bool self, uint64_t seed,
                                                          int64_t* __restrict__ out,
                                                          int32_t* __restrict__ err) {
  const int64_t wave = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  sample_lane_wave<LPN, false>(rowptr, col, n_graph, nodes, live_rows(n, n_dev), wave, k, ld,
                               self, seed, out, err, nullptr);
}

// one launch of the right kernel for fanout k (k <= kMaxFanout): rows [0, min(*n_dev, n))
inline void launch_sample(const int64_t* rowptr, const int32_t* col, int64_t n_graph,
                          const int64_t* nodes, int64_t n, const int64_t* n_dev, int k,
                          int64_t ld, bool self, uint64_t seed, int64_t* out, int32_t* err,
                          hipStream_t s) {
  const dim3 g(static_cast<unsigned>((n + 255) / 256)), t(256);
  auto lane_grid = [&](int lpn) {  // 4 waves of 64 / lpn nodes per workgroup
    const int64_t per_block = 4 * (kWave / lpn);
    return dim3(static_cast<unsigned>((n + per_block - 1) / per_block));
  };
  if (k <= 16 && !kThreadSerialSample) {
    hipLaunchKernelGGL(sample_lane_kernel<16>, lane_grid(16), t, 0, s, rowptr, col, n_graph, nodes,
                       n, n_dev, k, ld, self, seed, out, err);
    return;
  }
  if (k <= 32 && !kThreadSerialSample) {
    hipLaunchKernelGGL(sample_lane_kernel<32>, lane_grid(32), t, 0, s, rowptr, col, n_graph, nodes,
                       n, n_dev, k, ld, self, seed, out, err);
    return;
  }
  if (k <= 64 && !kThreadSerialSample) {
    hipLaunchKernelGGL(sample_lane_kernel<64>, lane_grid(64), t, 0, s, rowptr, col, n_graph, nodes,
                       n, n_dev, k, ld, self, seed, out, err);
    return;
  }
  if (k <= 16)
    hipLaunchKernelGGL(sample_reg_kernel<16>, g, t, 0, s, rowptr, col, n_graph, nodes, n, n_dev,
                       k, ld, self, seed, out, err);
  else if (k <= 32)
    hipLaunchKernelGGL(sample_reg_kernel<32>, g, t, 0, s, rowptr, col, n_graph, nodes, n, n_dev,
                       k, ld, self, seed, out, err);
  else
    hipLaunchKernelGGL(sample_kernel<0>, g, t, 0, s, rowptr, col, n_graph, nodes, n, n_dev, k, ld,
                       self, seed, out, err);
}

}  // namespace gnn
