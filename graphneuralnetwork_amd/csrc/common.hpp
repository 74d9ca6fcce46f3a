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
  if (flags & GNN_EPI_RELU) v = v > 0.f ? v : 0.f;
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

}  // namespace gnn
