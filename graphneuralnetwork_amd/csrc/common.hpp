// common.hpp -- shared device helpers for the gfx950 aggregation kernels.
//
// Everything here is wave64-native (CDNA4): lane = threadIdx.x & 63, cross-lane
// traffic goes through __shfl / __shfl_xor (ds_bpermute / DPP), never through
// 32-lane warp idioms.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gnn_mi355x.h"

namespace gnn {

constexpr int kWave = 64;

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

// Vector of VW floats as one register group; VW in {1, 2, 4}.
template <int VW> struct Vec;
template <> struct Vec<1> { typedef float T; };
template <> struct Vec<2> { typedef f2 T; };
template <> struct Vec<4> { typedef f4 T; };

template <int VW>
__device__ __forceinline__ typename Vec<VW>::T vload(const float* p) {
  return *reinterpret_cast<const typename Vec<VW>::T*>(p);
}
template <int VW>
__device__ __forceinline__ void vstore(float* p, typename Vec<VW>::T v) {
  *reinterpret_cast<typename Vec<VW>::T*>(p) = v;
}
template <int VW>
__device__ __forceinline__ typename Vec<VW>::T vzero() {
  return typename Vec<VW>::T(0.0f);
}

__device__ __forceinline__ float shfl_xor_f(float v, int m) { return __shfl_xor(v, m, kWave); }
__device__ __forceinline__ f2 shfl_xor_f(f2 v, int m) {
  return f2{__shfl_xor(v.x, m, kWave), __shfl_xor(v.y, m, kWave)};
}
__device__ __forceinline__ f4 shfl_xor_f(f4 v, int m) {
  return f4{__shfl_xor(v.x, m, kWave), __shfl_xor(v.y, m, kWave), __shfl_xor(v.z, m, kWave),
            __shfl_xor(v.w, m, kWave)};
}

__device__ __forceinline__ float act_apply(float v, uint32_t flags) {
  if (flags & GNN_EPI_RELU) v = (v > 0.f || v != v) ? v : 0.f;  // torch.relu: NaN stays NaN
  if (flags & GNN_EPI_ELU) v = v > 0.f ? v : expm1f(v);
  return v;
}
__device__ __forceinline__ float vget(float v, int) { return v; }
__device__ __forceinline__ float vget(f2 v, int i) { return v[i]; }
__device__ __forceinline__ float vget(f4 v, int i) { return v[i]; }
__device__ __forceinline__ void vset(float& v, int, float x) { v = x; }
__device__ __forceinline__ void vset(f2& v, int i, float x) { v[i] = x; }
__device__ __forceinline__ void vset(f4& v, int i, float x) { v[i] = x; }

inline bool aligned_to(const void* p, uintptr_t a) { return (reinterpret_cast<uintptr_t>(p) % a) == 0; }

inline int next_pow2_le64(int64_t v) {
  int p = 1;
  while (p < v && p < 64) p <<= 1;
  return p;
}

inline int launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? GNN_OK : static_cast<int>(e);
}

// ---------------------------------------------------------------------------------------
// LDS image of an MFMA A tile (K floats per row; gat_project_kernel, gcn_transform_kernel): row rr of K floats at rr * 4 * L4, its float4 c4 stored at
// float4 slot c4 ^ swz(rr). Chosen (by enumerating pads and xor swizzles against the lane
// groups of ds_write_b128 -- 8 x 8 lanes, bank (a/4) mod 32 -- and ds_read_b128 -- 4 x 16
// lanes {0-3,12-15,20-27}, {4-11,16-19,28-31}, ..., bank (a/4) mod 64,
// MI355X_MICROARCH.md LDS table) so that both the coalesced tile stores and the per-lane
// fragment reads (lane l: row l & 15, float4s [q * K/16, (q + 1) * K/16)) are free of bank
// conflicts. The round-2 layout (row pad of 4 floats, no swizzle) had 2-way conflicts on the
// fragment reads at K = 16..128 (2.1 conflict cycles per LDS instruction at K = 64,
// profiles/r02zk_sq_counters_summary.txt).
#ifdef GNN_TILE_OLD_LDS  // A/B: the round-2 layout (row pad of 4 floats, no swizzle)
template <int K> struct TileLds {
  static constexpr int L4 = K / 4 + 1;
  static __device__ __forceinline__ int swz(int) { return 0; }
};
#else
template <int K> struct TileLds;
template <> struct TileLds<16> {
  static constexpr int L4 = 4;
  static __device__ __forceinline__ int swz(int rr) { return (rr >> 1) & 3; }
};
template <> struct TileLds<32> {
  static constexpr int L4 = 12;
  static __device__ __forceinline__ int swz(int rr) { return rr & 7; }
};
template <> struct TileLds<64> {
  static constexpr int L4 = 18;
  static __device__ __forceinline__ int swz(int rr) { return rr & 15; }
};
template <> struct TileLds<128> {
  static constexpr int L4 = 33;
  static __device__ __forceinline__ int swz(int rr) { return ((rr >> 3) & 3) << 3; }
};
template <> struct TileLds<256> {  // a 1-float4 row pad alone is conflict-free at K = 256
  static constexpr int L4 = 65;
  static __device__ __forceinline__ int swz(int) { return 0; }
};
#endif

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------------------
// fp32 products from bf16 MFMAs (X6 kernels). Every fp32 value is split into three bf16
// pieces, v = v0 + v1 + v2 + e with |e| <= 2^-24 |v| (v0 = bf16(v), v1 = bf16(v - v0),
// v2 = bf16(v - v0 - v1); the differences are exact in fp32), and a product x w is summed
// from the six piece products down to order 2^-16: x0w0 + x0w1 + x1w0 + x0w2 + x1w1 + x2w0.
// A bf16 x bf16 product is exact in fp32 and v_mfma_f32_16x16x32_bf16 accumulates in fp32,
// so what is left out (x1w2, x2w1, x2w2 and the pieces' residues) is ~4 * 2^-24 |x w| per
// product -- the size of fp32's own rounding -- while the six MFMAs take 6 x 16 cycles
// against 8 x 32 for the same 32-long k-step on v_mfma_f32_16x16x4_f32.
// Non-finite inputs: an inf becomes NaN (inf - inf in the split); the GCN / SAGE layers
// never feed one.
__device__ __forceinline__ void split3(float v, __bf16& a, __bf16& b, __bf16& c) {
  a = static_cast<__bf16>(v);
  const float r1 = v - static_cast<float>(a);
  b = static_cast<__bf16>(r1);
  c = static_cast<__bf16>(r1 - static_cast<float>(b));
}
// LDS image of an X6 tile: three bf16 planes (pieces 0, 1, 2), row pitch 2K + 32 bytes, the
// 16-B chunk c of row rr stored at chunk c ^ swz6(rr): enumerated against the ds_read_b128
// lane groups (4 x 16 lanes, bank (a/4) mod 64) for the fragment reads (lane (q, r): row r,
// chunk q*K/32 + s) -- conflict-free -- and the staging ds_write_b64 (16 contiguous lanes =
// one 128-B run of a row) stays conflict-free under the permutation.
template <int K> __device__ __forceinline__ int swz6(int rr) {
  return K >= 256 ? (rr >> 2) & 1 : K >= 128 ? (rr >> 1) & 1 : rr & 1;
}
template <int K> constexpr int x6_pitch() { return 2 * K + 32; }  // bytes per LDS row
// One 32-bit hash of (seed, a, b): the dropout stream of the HIP kernels (the same function as
// gat.hip's hash3 over (edge, head); restated by oracle/spmm_oracle.c oracle_hash3). An item is
// kept when (h >> 8) / 2^24 >= p.
__device__ __forceinline__ uint32_t dropout_hash(uint64_t seed, int64_t a, int b) {
  uint32_t h = static_cast<uint32_t>(seed) ^ (static_cast<uint32_t>(seed >> 32) * 0x27d4eb2fu);
  h ^= static_cast<uint32_t>(a) * 0x9e3779b9u;
  h ^= static_cast<uint32_t>(static_cast<uint64_t>(a) >> 32) * 0x85ebca6bu;
  h ^= static_cast<uint32_t>(b) * 0xc2b2ae35u;
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}
__device__ __forceinline__ bool dropout_keep(uint64_t seed, int64_t a, int b, float p) {
  return static_cast<float>(dropout_hash(seed, a, b) >> 8) * (1.0f / 16777216.0f) >= p;
}
// the transforms' arithmetic at K >= 128 and the GAT projection's at K in {64, 128}
// (gnn_transform_set_precision, defined in transform.hip): 1 = X6 split bf16, 0 = fp32 MFMA
extern int g_tf_x6;

}  // namespace gnn
