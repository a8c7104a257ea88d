// device_common.hpp — shared gfx950 device helpers for libragmi.so
//
// Wave64 bitonic sort/merge of (score, id) pairs used by the scan's top-k and the merges,
// the canonical vector normalisation shared by upsert and query preparation, and the MFMA
// vector types. Everything here is CDNA4-only (wave = 64 lanes).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ragmi {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr float kNegInf = -__builtin_inff();
constexpr int kIdNone32 = 0x7fffffff;

// Total order used everywhere for ranking: score descending, then id ascending
// ("sorted by (score desc, row id asc)").
template <typename IdT>
__device__ __forceinline__ bool better(float as, IdT ai, float bs, IdT bi) {
  return (as > bs) || (as == bs && ai < bi);
}

template <typename IdT>
__device__ __forceinline__ IdT shfl_xor_id(IdT v, int mask) {
  if constexpr (sizeof(IdT) == 8) {
    int lo = __shfl_xor((int)(uint32_t)((uint64_t)v), mask, 64);
    int hi = __shfl_xor((int)(uint32_t)((uint64_t)v >> 32), mask, 64);
    return (IdT)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
  } else {
    return (IdT)__shfl_xor((int)v, mask, 64);
  }
}

// One compare-exchange stage across lanes (lane, lane ^ j). `asc` = this lane's block is
// sorted best-first.
template <typename IdT>
__device__ __forceinline__ void cas_stage(float& s, IdT& id, int lane, int j, bool asc) {
  const float os = __shfl_xor(s, j, 64);
  const IdT oi = shfl_xor_id(id, j);
  const bool lower = (lane & j) == 0;
  const bool take = (asc == lower) ? better(os, oi, s, id) : better(s, id, os, oi);
  s = take ? os : s;
  id = take ? oi : id;
}

// Full bitonic sort of the 64 (score, id) pairs held one per lane; lane 0 ends best.
template <typename IdT>
__device__ __forceinline__ void bitonic_sort64(float& s, IdT& id, int lane) {
#pragma unroll
  for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) cas_stage(s, id, lane, j, (lane & k) == 0);
  }
}

// Bitonic merge: lanes 0..31 sorted best-first, lanes 32..63 sorted worst-first
// -> all 64 sorted best-first.
template <typename IdT>
__device__ __forceinline__ void bitonic_merge64(float& s, IdT& id, int lane) {
#pragma unroll
  for (int j = 32; j > 0; j >>= 1) cas_stage(s, id, lane, j, true);
}

// Canonical L2 norm of a D-vector held in global memory, computed by one wave.
// Lane l accumulates the 8-element chunks c = l, l+64, ... sequentially with fp64 fma
// (acc = fma(x, x, acc)); then a xor butterfly (32,16,8,4,2,1) in fp64; lane 0's sum is
// broadcast. oracle/scan_ref.c:canon_sumsq restates exactly this order.
template <int D>
__device__ __forceinline__ double canon_sumsq(const float* __restrict__ x, int lane) {
  double acc = 0.0;
  for (int c = lane; c < D / 8; c += 64) {
    const float4 a = *reinterpret_cast<const float4*>(x + 8 * c);
    const float4 b = *reinterpret_cast<const float4*>(x + 8 * c + 4);
    acc = fma((double)a.x, (double)a.x, acc);
    acc = fma((double)a.y, (double)a.y, acc);
    acc = fma((double)a.z, (double)a.z, acc);
    acc = fma((double)a.w, (double)a.w, acc);
    acc = fma((double)b.x, (double)b.x, acc);
    acc = fma((double)b.y, (double)b.y, acc);
    acc = fma((double)b.z, (double)b.z, acc);
    acc = fma((double)b.w, (double)b.w, acc);
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) acc = acc + __shfl_xor(acc, d, 64);
  return __shfl(acc, 0, 64);
}

// fp32 -> fp16 RNE of an fp32 value. The empty asm makes `y` opaque: without it LLVM folds
// (half)(float)(double) into one direct f64->f16 rounding, which differs from the canonical
// double rounding (fp64 -> fp32 -> fp16) in ~1/8192 of the elements.
__device__ __forceinline__ _Float16 f32_to_f16(float y) {
  asm volatile("" : "+v"(y));
  return (_Float16)y;
}

// y = fp32(x / sqrt(sumsq)) with fp64 division; zero vector stays zero.
__device__ __forceinline__ float canon_scale(float x, double norm) {
  return norm > 0.0 ? (float)((double)x / norm) : 0.0f;
}

}  // namespace ragmi
