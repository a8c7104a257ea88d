// device_common.hpp — shared gfx950 device helpers for libragmi.so
//
// Wave64 bitonic sort/merge of (score, id) pairs used by the scan's top-k and the merges,
// the canonical vector normalisation shared by upsert and query preparation, and the MFMA
// vector types. Everything here is CDNA4-only (wave = 64 lanes).
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <tuple>
#include <utility>

namespace ragmi {

// Launch geometry. Every kernel whose LDS layout or wave roles assume a
// block size (the LDS-ring GEMMs and scans, attention, the tier-2 rescan) takes that size from
// ONE constexpr, which its __launch_bounds__ uses and which launch_fixed passes as the block:
// no launch site spells a block size, so a launcher cannot size the block for a different
// instance (round 3's RAG_GEMM_WS_SMALL fault: four loader waves launched for a one-loader
// ring wrote past it).
template <int BLOCK, typename... KArgs, typename... Args>
inline void launch_fixed(void (*k)(KArgs...), dim3 grid, size_t lds, hipStream_t st,
                         Args&&... args) {
  static_assert(BLOCK > 0 && BLOCK % 64 == 0 && BLOCK <= 1024, "whole waves, <= 1024 threads");
  k<<<grid, dim3(BLOCK), lds, st>>>(static_cast<Args&&>(args)...);
}

// launch_fixed with the launch timed by its own dispatch packet (hipExtLaunchKernel: ev_a /
// ev_b take the kernel's start / end timestamps). Two hipEventRecord markers around the
// launch would put a barrier packet with a cache flush on each side of it: at 1.25M rows with
// 4 batches in flight those markers cost 1.5% of throughput (profiles/r04l_*).
template <int BLOCK, typename... KArgs, typename... Args>
inline hipError_t launch_fixed_timed(void (*k)(KArgs...), dim3 grid, size_t lds, hipStream_t st,
                                     hipEvent_t ev_a, hipEvent_t ev_b, Args&&... args) {
  static_assert(BLOCK > 0 && BLOCK % 64 == 0 && BLOCK <= 1024, "whole waves, <= 1024 threads");
  static_assert(sizeof...(KArgs) == sizeof...(Args), "argument count");
  std::tuple<KArgs...> vals{static_cast<KArgs>(static_cast<Args&&>(args))...};
  return std::apply(
      [&](auto&... v) {
        void* ptrs[] = {static_cast<void*>(&v)...};
        return hipExtLaunchKernel(reinterpret_cast<const void*>(k), grid, dim3(BLOCK), ptrs, lds,
                                  st, ev_a, ev_b, 0);
      },
      vals);
}

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr float kNegInf = -__builtin_inff();
constexpr int kIdNone32 = 0x7fffffff;

// 16 B per lane global -> LDS DMA (global_load_lds_dwordx4): lane l's 16 bytes from `gsrc`
// land at LDS byte address lds_addr + 16 l (lds_addr wave-uniform).
// Issued through inline asm on purpose: hipcc (ROCm 7.2) tracks the builtin's LDS write and
// puts `s_waitcnt vmcnt(0)` before the first ds_read after it (it cannot prove the read
// misses the DMA target), which drains a multi-stage ring on every step. Hidden in asm, the
// DMA is invisible to its waitcnt bookkeeping: the caller retires it with its own counted
// `s_waitcnt vmcnt(N)` + barrier before reading the slot. M0 is compiler-reserved, so it is
// saved and restored inside the statement.
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_addr) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_addr)
      : "memory");
}

// the same with the non-temporal policy (`nt`): for streams read once per pass that are far
// larger than the Infinity Cache (MI355X_MICROARCH.md ldsdma-fill: chip 6.4 TB/s default
// policy, 6.5-6.8 nt)
__device__ __forceinline__ void glds16_nt(const void* gsrc, uint32_t lds_addr) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_addr)
      : "memory");
}

// LDS byte address of a __shared__ pointer (for glds16), made provably wave-uniform
template <typename T>
__device__ __forceinline__ uint32_t lds_addr_of(const T* p) {
  return __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) T*)p);
}

// Total order used everywhere for ranking: score descending, then id ascending
// ("sorted by (score desc, row id asc)"). Bitwise ops, no short-circuit: the
// comparator must compile to v_cmp + mask logic, not exec-masked branches.
template <typename IdT>
__device__ __forceinline__ bool better(float as, IdT ai, float bs, IdT bi) {
  return (as > bs) | ((as == bs) & (ai < bi));
}

// Lane exchange v[lane ^ J] for a compile-time J. J = 1, 2 (quad_perm), 4, 8 (two DPP mirror
// steps: i^4 = half_mirror(i^3), i^8 = mirror(half_mirror)) stay in the VALU; 16 and 32 use
// ds_bpermute.
template <int J>
__device__ __forceinline__ int xor_lane(int v) {
  if constexpr (J == 1) {
    return __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
  } else if constexpr (J == 2) {
    return __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
  } else if constexpr (J == 4) {
    const int t = __builtin_amdgcn_update_dpp(0, v, 0x1B, 0xF, 0xF, false);  // [3,2,1,0]
    return __builtin_amdgcn_update_dpp(0, t, 0x141, 0xF, 0xF, false);        // row_half_mirror
  } else if constexpr (J == 8) {
    const int t = __builtin_amdgcn_update_dpp(0, v, 0x141, 0xF, 0xF, false); // row_half_mirror
    return __builtin_amdgcn_update_dpp(0, t, 0x140, 0xF, 0xF, false);        // row_mirror
  } else {
    return __shfl_xor(v, J, 64);
  }
}

template <int J>
__device__ __forceinline__ float xor_lane_f(float v) {
  return __builtin_bit_cast(float, xor_lane<J>(__builtin_bit_cast(int, v)));
}

template <int J, typename IdT>
__device__ __forceinline__ IdT xor_lane_id(IdT v) {
  if constexpr (sizeof(IdT) == 8) {
    const uint64_t u = (uint64_t)v;
    const int lo = xor_lane<J>((int)(uint32_t)u);
    const int hi = xor_lane<J>((int)(uint32_t)(u >> 32));
    return (IdT)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
  } else {
    return (IdT)xor_lane<J>((int)v);
  }
}

// One compare-exchange stage across lanes (lane, lane ^ J). `asc` = this lane's block is
// sorted best-first.
template <int J, typename IdT>
__device__ __forceinline__ void cas_stage(float& s, IdT& id, int lane, bool asc) {
  const float os = xor_lane_f<J>(s);
  const IdT oi = xor_lane_id<J>(id);
  const bool lower = (lane & J) == 0;
  const bool ob = better(os, oi, s, id);
  const bool sb = better(s, id, os, oi);
  const bool take = (asc == lower) ? ob : sb;
  s = take ? os : s;
  id = take ? oi : id;
}

template <int K, int J, typename IdT>
__device__ __forceinline__ void bitonic_steps(float& s, IdT& id, int lane) {
  if constexpr (J > 0) {
    cas_stage<J>(s, id, lane, K == 64 ? true : (lane & K) == 0);
    bitonic_steps<K, J / 2>(s, id, lane);
  }
}

template <int K, typename IdT>
__device__ __forceinline__ void bitonic_sort_from(float& s, IdT& id, int lane) {
  if constexpr (K <= 64) {
    bitonic_steps<K, K / 2>(s, id, lane);
    bitonic_sort_from<K * 2>(s, id, lane);
  }
}

// Full bitonic sort of the 64 (score, id) pairs held one per lane; lane 0 ends best.
template <typename IdT>
__device__ __forceinline__ void bitonic_sort64(float& s, IdT& id, int lane) {
  bitonic_sort_from<2>(s, id, lane);
}

// Four independent 16-lane bitonic sorts (lanes 16b .. 16b+15 each end best-first): 10
// compare-exchange stages against the 32-lane sort's 15.
template <int K, typename IdT>
__device__ __forceinline__ void bitonic_sort16_from(float& s, IdT& id, int lane) {
  if constexpr (K <= 16) {
    if constexpr (K == 16)
      bitonic_steps<64, 8>(s, id, lane);    // final pass: every 16-lane block best-first
    else
      bitonic_steps<K, K / 2>(s, id, lane);
    bitonic_sort16_from<K * 2>(s, id, lane);
  }
}

template <typename IdT>
__device__ __forceinline__ void bitonic_sort16x4(float& s, IdT& id, int lane) {
  bitonic_sort16_from<2>(s, id, lane);
}

// Eight independent 8-lane bitonic sorts (6 stages).
template <int K, typename IdT>
__device__ __forceinline__ void bitonic_sort8_from(float& s, IdT& id, int lane) {
  if constexpr (K <= 8) {
    if constexpr (K == 8)
      bitonic_steps<64, 4>(s, id, lane);
    else
      bitonic_steps<K, K / 2>(s, id, lane);
    bitonic_sort8_from<K * 2>(s, id, lane);
  }
}

template <typename IdT>
__device__ __forceinline__ void bitonic_sort8x8(float& s, IdT& id, int lane) {
  bitonic_sort8_from<2>(s, id, lane);
}

template <int K, typename IdT>
__device__ __forceinline__ void bitonic_sort32_from(float& s, IdT& id, int lane) {
  if constexpr (K <= 32) {
    if constexpr (K == 32)
      bitonic_steps<64, 16>(s, id, lane);   // final pass: both halves best-first
    else
      bitonic_steps<K, K / 2>(s, id, lane);
    bitonic_sort32_from<K * 2>(s, id, lane);
  }
}

// Two independent 32-element bitonic sorts (lanes 0..31 and 32..63), each best-first.
template <typename IdT>
__device__ __forceinline__ void bitonic_sort32x2(float& s, IdT& id, int lane) {
  bitonic_sort32_from<2>(s, id, lane);
}

// Bitonic merge: lanes 0..31 sorted best-first, lanes 32..63 sorted worst-first
// -> all 64 sorted best-first.
template <typename IdT>
__device__ __forceinline__ void bitonic_merge64(float& s, IdT& id, int lane) {
  bitonic_steps<64, 32>(s, id, lane);
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

// max of values that are never NaN (MFMA scores, exp2 outputs, -inf masks): IEEE-754
// `maximum` lowers to v_maximum(3)_f32 on gfx950, where fmaxf's maxnum first canonicalises
// every input that is not provably canonical (one v_max_f32 x, x per MFMA result: 11 VALU
// for an 8-value max instead of 5). Equal to fmaxf for every non-NaN input.
__device__ __forceinline__ float fmax_nc(float a, float b) {
  return __builtin_elementwise_maximum(a, b);
}

// a * b + c as ONE scalar v_fma_f32 that the compiler cannot pair into v_pk_fma_f32 (SLP):
// beside MFMAs a packed fp32 op costs ~22 cycles more than two scalar ones
// (MI355X_MICROARCH.md, price of one filler beside MFMAs). Same value as fmaf.
__device__ __forceinline__ float fma_scalar(float a, float b, float c) {
  float d;
  asm("v_fma_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
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
