// kcommon.hpp -- small device helpers shared by the kernel translation units of libmarlsc
// (env_kernels.hip, alloc_kernels.hip). Not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace msc {

// Explicit global address space for hot buffers: pointers loaded from the device-resident DevEnv
// are generic, and generic (flat_*) loads also count against lgkmcnt, so any LDS wait would also
// wait for them and defeat software prefetching.
#define MSC_GLOBAL __attribute__((address_space(1)))
template <typename T>
__device__ __forceinline__ MSC_GLOBAL T* gp(T* p) {
  return (MSC_GLOBAL T*)p;
}
typedef unsigned int v4u __attribute__((ext_vector_type(4)));  // uint4 as a native vector type
__device__ __forceinline__ uint4 gload4(const MSC_GLOBAL uint4* p, int64_t i) {
  const v4u v = reinterpret_cast<const MSC_GLOBAL v4u*>(p)[i];
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void gstore4(MSC_GLOBAL uint4* p, int64_t i, uint4 x) {
  v4u v;
  v.x = x.x; v.y = x.y; v.z = x.z; v.w = x.w;
  reinterpret_cast<MSC_GLOBAL v4u*>(p)[i] = v;
}

// one order record of the per-step order buffer: 16-bit fields {region, q_0, ..., q_{K-1}}
// packed into NV uint4 words, stored [order][NV][E] (env fastest)
template <int K>
struct Rec {
  static constexpr int NV = (1 + K + 7) / 8;  // uint4 words per order record
  uint16_t h[8 * NV];
};

// a wave-uniform double kept in scalar registers
__device__ __forceinline__ double sgpr_d(double v) {
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b), hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// v as the output of an (empty) asm statement: no load of it is pending afterwards, so the compiler
// places its wait for the load here instead of at the value's first use (inside a loop, that wait
// is a vmcnt(0) that also drains every LDS-DMA and store in flight)
__device__ __forceinline__ int vsettle(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

// numpy pairwise sum (add.reduce, n <= 16): sequential below 8 elements, else 8 accumulators
// (static indices only: v stays in registers)
__device__ __forceinline__ double np_sum_f64_16(const double (&v)[16], int n) {
  if (n < 8) {
    double r = 0.0;
#pragma unroll
    for (int i = 0; i < 8; i++) r = i < n ? r + v[i] : r;
    return r;
  }
  double a[8];
#pragma unroll
  for (int j = 0; j < 8; j++) a[j] = n >= 16 ? v[j] + v[8 + j] : v[j];
  double r = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
#pragma unroll
  for (int i = 8; i < 16; i++) r = (n < 16 && i < n) ? r + v[i] : r;
  return r;
}

// Butterfly partner exchange inside a group of GW lanes with DPP (a VALU operand modifier, no LDS
// round trip): step 0 pairs lanes i ^ 1 and step 1 lanes i ^ 2 (quad_perm), step 2 the two quads
// of an 8-lane row half (row_half_mirror), step 3 the two halves of a 16-lane row (row_mirror),
// step 4 (32-lane groups, > 16 warehouses) lanes i ^ 16 across rows (DPP stays inside a row: a
// lane shuffle). Every step pairs lanes whose partial results cover disjoint halves, so min / sum
// reductions end with the group result in every lane.
template <int S>
__device__ __forceinline__ int dpp_x(int v) {
  if constexpr (S == 4) {
    return __shfl_xor(v, 16);
  } else {
    constexpr int ctrl = S == 0 ? 0xB1 : S == 1 ? 0x4E : S == 2 ? 0x141 : 0x140;
    // (every lane of these patterns has a source inside its row, so no `old` value is needed:
    // mov_dpp with bound_ctrl leaves the compiler free to skip zeroing the destination first)
    return __builtin_amdgcn_mov_dpp(v, ctrl, 0xF, 0xF, true);
  }
}
template <int S>
__device__ __forceinline__ double dpp_x(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = dpp_x<S>((int)(b & 0xffffffffLL)), hi = dpp_x<S>((int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// numpy add.reduce order (pairwise_sum, n <= 128) of the group's lane values v_0..v_{n-1} without
// materialising them: sequential below 8 (lane shuffles), else the eight strided accumulators
// r_j = v_j + v_{j+8} + ... over the whole 8-blocks (lane j < 8 gathers its column), their tree as
// 3 DPP butterfly steps over lanes 0..7 (IEEE addition is commutative, so the butterfly's pairs are
// numpy's pairs), then the tail sequentially; the result reaches every lane of the group
template <int GW>
__device__ __forceinline__ double group_np_sum(double v, int n) {
  if (n < 8) {
    double r = 0.0;
#pragma unroll
    for (int j = 0; j < (GW < 8 ? GW : 8); j++) {
      const double x = __shfl(v, j, GW);
      r = j < n ? r + x : r;
    }
    return r;
  }
  if constexpr (GW < 8) {
    return 0.0;  // unreachable: n <= GW
  } else {
    const int m = n - n % 8;  // end of the whole 8-blocks
    double a = v;
#pragma unroll
    for (int b = 8; b < GW; b += 8) {
      const double x = __shfl(v, (threadIdx.x + b) % GW, GW);  // v_{k+b} for lane k < 8
      a = b < m ? a + x : a;
    }
    a = a + dpp_x<0>(a);
    a = a + dpp_x<1>(a);
    a = a + dpp_x<2>(a);
    double r = __shfl(a, 0, GW);
#pragma unroll
    for (int i = 8; i < GW; i++) {
      const double x = __shfl(v, i, GW);
      r = (i >= m && i < n) ? r + x : r;
    }
    return r;
  }
}

}  // namespace msc
