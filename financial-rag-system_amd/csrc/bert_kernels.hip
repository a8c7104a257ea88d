// bert_kernels.hip — BERT-small encoder forward for gfx950 (bge-small-en-v1.5 and
// ms-marco-MiniLM-L-6-v2 cross-encoder).
//
// Replaces the torch CPU forward behind sentence-transformers' SentenceTransformer.encode
// (reference main.py:80-84, 144-149, 211-213; main2.py:170-171) and CrossEncoder.predict
// (main.py:86-90, 241-247). Arithmetic follows transformers modeling_bert.py (post-LN,
// erf-GELU, softmax(QK^T/sqrt(d) + mask)V); see oracle/bert_ref.py.
//
// Numerics: GEMM operands fp16 (weights and activations), fp32 MFMA accumulation, fp32
// residual stream, fp32 LayerNorm/softmax statistics.
// Layout: sequences are PACKED (no padding): token t of sequence b sits at row cu[b] + pos.
// Right padding never changes a valid token's output (masked keys contribute exp(-inf) = 0),
// so packing is exact w.r.t. the padded reference.
#include "device_common.hpp"

namespace ragmi {
namespace bert {

// Built shapes (template parameters below): hidden H in {384, 768, 1024} with head_dim HD in
// {32, 64} (bge-small / MiniLM: 384/32; bge-base: 768/64; bge-large: 1024/64); intermediate
// size is a runtime GEMM dimension.

typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef _Float16 half2 __attribute__((ext_vector_type(2)));

// fp16x3 split: v = hi + lo with hi = fp16(v), lo = fp16(v - hi); a*b ~ ah*bh + ah*bl + al*bh
// (relative error ~2^-22) on the fp16 MFMA pipe.
// v is pinned as an fp32 register value before either conversion: under -ffp-contract=fast
// the compiler may fuse the operation that produced v into the hi conversion (one rounding of
// the unrounded product / sum straight to fp16, v_fma_mix*_f16) while lo subtracts hi from
// the fp32-rounded v — where an fp16 rounding midpoint falls between the two, hi and lo
// disagree and hi + lo is off by one fp16 ulp (measured: 1-4 of ~1e5 attention outputs, every
// error exactly one ulp; tests/test_attention_gpu.py).
__device__ __forceinline__ half2 split16(float v) {   // {hi, lo}
  asm("" : "+v"(v));
  const _Float16 hi = (_Float16)v;
  return half2{hi, (_Float16)(v - (float)hi)};
}

// The same split of two values in 3 instructions instead of 8 (round 2): the hi pair by one
// v_cvt_pk_f16_f32, each lo by v_fma_mix{lo,hi}_f16 computing -hi * 1 + v exactly and rounding
// once to fp16. v - hi is exact in fp32 (Sterbenz: hi is within a factor 2 of v, or 0), so
// this is fp16(v - hi) bit for bit, as split16 computes it (which converts hi back to fp32,
// subtracts and converts again, and converts hi twice). Inputs pinned as above.
__device__ __forceinline__ void split16x2(float v0, float v1, half2& h, half2& l) {
  asm("" : "+v"(v0), "+v"(v1));
  h = half2{(_Float16)v0, (_Float16)v1};
  const uint32_t hu = __builtin_bit_cast(uint32_t, h);
  uint32_t lu;
  asm("v_fma_mixlo_f16 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %0, -%1, 1.0, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
      : "=&v"(lu)
      : "v"(hu), "v"(v0), "v"(v1));
  l = __builtin_bit_cast(half2, lu);
}

// erf-GELU, 0.5 x (1 + erf(x / sqrt 2)), with erfc(|z|) from Abramowitz & Stegun 7.1.26
// (|error of erf| <= 1.5e-7 absolute, i.e. at fp32 rounding level for the GELU output):
// 1 + erf(z) = 2 - erfc(z) for z >= 0 and erfc(-z) for z < 0 (no cancellation for z << 0).
// Two transcendentals (rcp, exp2) and 7 FMAs instead of the libm erff's branchy polynomial.
__device__ __forceinline__ float gelu_erf(float x) {
  const float z = fabsf(x) * 0.70710678118654752440f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  float q = fmaf(1.061405429f, t, -1.453152027f);
  q = fmaf(q, t, 1.421413741f);
  q = fmaf(q, t, -0.284496736f);
  q = fmaf(q, t, 0.254829592f);
  q *= t * __builtin_amdgcn_exp2f(-z * z * 1.44269504088896341f);   // erfc(z)
  return 0.5f * x * (x >= 0.f ? 2.0f - q : q);
}

// the same on 4 values at once: every non-transcendental step as 4-wide vector arithmetic
// (gfx950 packed fp32: v_pk_fma_f32 / v_pk_mul_f32 take 2 lanes' worth per instruction), the
// rcp / exp2 per value. Per value the same operations in the same order as gelu_erf.
__device__ __forceinline__ floatx4 gelu_erf4(floatx4 x) {
  const floatx4 z = __builtin_elementwise_abs(x) * 0.70710678118654752440f;
  const floatx4 d = __builtin_elementwise_fma((floatx4)(0.3275911f), z, (floatx4)(1.0f));
  floatx4 t, e;
  const floatx4 zz = -z * z * 1.44269504088896341f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    t[r] = __builtin_amdgcn_rcpf(d[r]);
    e[r] = __builtin_amdgcn_exp2f(zz[r]);
  }
  floatx4 q = __builtin_elementwise_fma((floatx4)(1.061405429f), t, (floatx4)(-1.453152027f));
  q = __builtin_elementwise_fma(q, t, (floatx4)(1.421413741f));
  q = __builtin_elementwise_fma(q, t, (floatx4)(-0.284496736f));
  q = __builtin_elementwise_fma(q, t, (floatx4)(0.254829592f));
  q *= t * e;
  floatx4 w;
#pragma unroll
  for (int r = 0; r < 4; ++r) w[r] = x[r] >= 0.f ? 2.0f - q[r] : q[r];
  return 0.5f * x * w;
}

// ----------------------------------------------------------------------------------------
// embeddings: x = LN(word[id] + type[tt] + pos[p]); one wave per token, grid (ceil(L/4), B)
// ----------------------------------------------------------------------------------------
template <int H>
__global__ __launch_bounds__(256) void embed_ln_kernel(
    const int* __restrict__ ids, const int* __restrict__ types, const int* __restrict__ cu,
    const float* __restrict__ wemb, const float* __restrict__ pemb, const float* __restrict__ temb,
    const float* __restrict__ g, const float* __restrict__ bt, float eps, int vocab,
    int type_vocab, int max_pos, float* __restrict__ x, _Float16* __restrict__ xh,
    _Float16* __restrict__ xl) {
  const int b = blockIdx.y;
  const int pos = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int len = cu[b + 1] - cu[b];
  if (pos >= len) return;
  const int64_t t = cu[b] + pos;
  // clamp: a bad id must never become an out-of-bounds gather
  const int id = min(max(ids[t], 0), vocab - 1);
  const int ty = min(max(types[t], 0), type_vocab - 1);
  const int pp = min(pos, max_pos - 1);
  float v[H / 64];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < H / 64; ++j) {
    const int c = lane + 64 * j;
    v[j] = wemb[(int64_t)id * H + c] + temb[ty * H + c] + pemb[pp * H + c];
    s += v[j];
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) s += __shfl_xor(s, d, 64);
  const float mu = s * (1.0f / H);
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < H / 64; ++j) q += (v[j] - mu) * (v[j] - mu);
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) q += __shfl_xor(q, d, 64);
  const float rs = rsqrtf(q * (1.0f / H) + eps);
#pragma unroll
  for (int j = 0; j < H / 64; ++j) {
    const int c = lane + 64 * j;
    const float y = (v[j] - mu) * rs * g[c] + bt[c];
    if (x) x[t * H + c] = y;                 // (null: fp16x3 residual kept as xh + xl only)
    _Float16 yh, yl;
    { const half2 s16_ = split16(y); yh = s16_[0]; yl = s16_[1]; }
    xh[t * H + c] = yh;
    if (xl) xl[t * H + c] = yl;
  }
}

// ----------------------------------------------------------------------------------------
// residual + LayerNorm: x = LN(x + y) (fp32, in place), xh = fp16(x); one wave per row.
// XF (fp16x3 only): the residual stream lives in the operand planes alone, x = xh + xl
// (fp16(x - xh) keeps x to 2^-22 relative), so the fp32 copy is neither read nor written:
// 12 instead of 20 bytes per element.
// ----------------------------------------------------------------------------------------
// y may hold `parts` split-K partial products (gemm_pipe_kernel ksplit > 1), part p at
// y + p * pstride: they are summed in part order (deterministic) before the residual add.
template <int H, bool XF = false>
__global__ __launch_bounds__(256) void add_ln_kernel(float* __restrict__ x,
                                                     const float* __restrict__ y,
                                                     const float* __restrict__ g,
                                                     const float* __restrict__ bt, float eps,
                                                     _Float16* __restrict__ xh,
                                                     _Float16* __restrict__ xl, int T,
                                                     int parts = 1, int64_t pstride = 0) {
  const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (t >= T) return;
  float v[H / 64];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < H / 64; ++j) {
    const int c = lane + 64 * j;
    const float r = XF ? (float)xh[t * H + c] + (float)xl[t * H + c] : x[t * H + c];
    float yy = y[t * H + c];
    for (int p = 1; p < parts; ++p) yy += y[p * pstride + t * H + c];
    v[j] = r + yy;
    s += v[j];
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) s += __shfl_xor(s, d, 64);
  const float mu = s * (1.0f / H);
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < H / 64; ++j) q += (v[j] - mu) * (v[j] - mu);
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) q += __shfl_xor(q, d, 64);
  const float rs = rsqrtf(q * (1.0f / H) + eps);
#pragma unroll
  for (int j = 0; j < H / 64; ++j) {
    const int c = lane + 64 * j;
    const float o = (v[j] - mu) * rs * g[c] + bt[c];
    if constexpr (!XF) x[t * H + c] = o;
    _Float16 oh, ol;
    { const half2 s16_ = split16(o); oh = s16_[0]; ol = s16_[1]; }
    xh[t * H + c] = oh;
    if (xl) xl[t * H + c] = ol;
  }
}

// Sum over the 64 lanes, the same bits in every lane: DPP within each 16-lane row (xor 1,
// xor 2, half-row mirror, row mirror — each step adds a lane's value to its partner's, and
// fp32 addition commutes, so partners agree), then the row pairs and halves by
// v_permlane16_swap / v_permlane32_swap. No LDS round trips (ds_bpermute: ~12 dependent ones
// for two butterfly reductions in add_ln_kernel).
__device__ __forceinline__ float dpp_add(float v, int ctrl_sel) {
  int d;
  switch (ctrl_sel) {   // dpp_ctrl must be an immediate
    case 0: d = __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false); break;
    case 1: d = __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false); break;
    case 2: d = __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false); break;
    default: d = __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false); break;
  }
  return v + __builtin_bit_cast(float, d);
}
__device__ __forceinline__ float wave_sum64(float v) {
  v = dpp_add(v, 0);   // quad_perm [1,0,3,2]
  v = dpp_add(v, 1);   // quad_perm [2,3,0,1]: every lane holds its quad's sum
  v = dpp_add(v, 2);   // row_half_mirror: + the other quad of the 8
  v = dpp_add(v, 3);   // row_mirror: + the other 8 of the row
  const uint32_t u = __builtin_bit_cast(uint32_t, v);
  const auto r16 = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  v = __builtin_bit_cast(float, (uint32_t)r16[0]) + __builtin_bit_cast(float, (uint32_t)r16[1]);
  const uint32_t u2 = __builtin_bit_cast(uint32_t, v);
  const auto r32 = __builtin_amdgcn_permlane32_swap(u2, u2, false, false);
  return __builtin_bit_cast(float, (uint32_t)r32[0]) + __builtin_bit_cast(float, (uint32_t)r32[1]);
}

// add_ln_kernel for hidden 384 (bge-small / MiniLM; round 3): lane l < 48 owns columns
// 8l .. 8l+7 — 16-B loads of the residual planes (or 2 x 16 B of the fp32 rows) and of each
// split-K part, 16-B plane stores — and both reductions run on wave_sum64. The small-batch
// forward's residual passes (2 per layer, ~87 launches per 32-query encode) were
// latency-bound on 2-byte accesses and 12 dependent ds_bpermute round trips.
// Same formula, parts summed in part order; the reduction order differs from add_ln_kernel's.
// ln384_rows: R rows t[0..R) of one wave (t < 0: none), every row's loads issued before any
// row's reductions (add_ln384_kernel: R = 1). Round 5 also ran it with R = 4 inside the SMALL
// split-K GEMM, the last arriving workgroup of each 64-row block finishing the block behind an
// agent-scope release / acquire ticket: bit-identical forward, but the per-unit L2 write-back
// of the release made the 32-query forward 0.71 -> 1.17 ms (profiles/r05r_split_ln_ab.jsonl).
template <bool XF, int R>
__device__ __forceinline__ void ln384_rows(float* __restrict__ x, const float* __restrict__ y,
                                           const float* __restrict__ g,
                                           const float* __restrict__ bt, float eps,
                                           _Float16* __restrict__ xh, _Float16* __restrict__ xl,
                                           const int64_t (&t)[R], int lane, int parts,
                                           int64_t pstride) {
  constexpr int H = 384;
  const bool on = lane < H / 8;
  float v[R][8];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int64_t o = (t[r] < 0 ? 0 : t[r]) * H + 8 * (on ? lane : 0);
    if (on && t[r] >= 0) {
      floatx4 y0 = *reinterpret_cast<const floatx4*>(y + o);
      floatx4 y1 = *reinterpret_cast<const floatx4*>(y + o + 4);
#pragma unroll
      for (int p = 1; p < 4; ++p)
        if (p < parts) {
          y0 += *reinterpret_cast<const floatx4*>(y + p * pstride + o);
          y1 += *reinterpret_cast<const floatx4*>(y + p * pstride + o + 4);
        }
      if constexpr (XF) {
        const half8 h = *reinterpret_cast<const half8*>(xh + o);
        const half8 l = xl ? *reinterpret_cast<const half8*>(xl + o) : half8{};
#pragma unroll
        for (int e = 0; e < 8; ++e) v[r][e] = ((float)h[e] + (float)l[e]) + (e < 4 ? y0[e] : y1[e - 4]);
      } else {
        const floatx4 r0 = *reinterpret_cast<const floatx4*>(x + o);
        const floatx4 r1 = *reinterpret_cast<const floatx4*>(x + o + 4);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[r][e] = (e < 4 ? r0[e] : r1[e - 4]) + (e < 4 ? y0[e] : y1[e - 4]);
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[r][e] = 0.f;
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (t[r] < 0) continue;                     // (wave-uniform)
    const int64_t o = t[r] * H + 8 * (on ? lane : 0);
    const float s = ((v[r][0] + v[r][1]) + (v[r][2] + v[r][3])) +
                    ((v[r][4] + v[r][5]) + (v[r][6] + v[r][7]));
    const float mu = wave_sum64(s) * (1.0f / H);
    float q = 0.f;
    if (on)
#pragma unroll
      for (int e = 0; e < 8; ++e) q = fmaf(v[r][e] - mu, v[r][e] - mu, q);
    const float rs = rsqrtf(wave_sum64(q) * (1.0f / H) + eps);
    if (!on) continue;
    const floatx4 g0 = *reinterpret_cast<const floatx4*>(g + 8 * lane);
    const floatx4 g1 = *reinterpret_cast<const floatx4*>(g + 8 * lane + 4);
    const floatx4 b0 = *reinterpret_cast<const floatx4*>(bt + 8 * lane);
    const floatx4 b1 = *reinterpret_cast<const floatx4*>(bt + 8 * lane + 4);
    float out[8];
#pragma unroll
    for (int e = 0; e < 8; ++e)
      out[e] = (v[r][e] - mu) * rs * (e < 4 ? g0[e] : g1[e - 4]) + (e < 4 ? b0[e] : b1[e - 4]);
    if constexpr (!XF) {
      *reinterpret_cast<floatx4*>(x + o) = floatx4{out[0], out[1], out[2], out[3]};
      *reinterpret_cast<floatx4*>(x + o + 4) = floatx4{out[4], out[5], out[6], out[7]};
    }
    half8 hh, ll;
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      half2 h2, l2;
      split16x2(out[e], out[e + 1], h2, l2);
      hh[e] = h2[0]; hh[e + 1] = h2[1]; ll[e] = l2[0]; ll[e + 1] = l2[1];
    }
    *reinterpret_cast<half8*>(xh + o) = hh;
    if (xl) *reinterpret_cast<half8*>(xl + o) = ll;
  }
}

template <bool XF, bool L2 = false>
__global__ __launch_bounds__(256) void add_ln384_kernel(float* __restrict__ x,
                                                        const float* __restrict__ y,
                                                        const float* __restrict__ g,
                                                        const float* __restrict__ bt, float eps,
                                                        _Float16* __restrict__ xh,
                                                        _Float16* __restrict__ xl, int T,
                                                        int parts = 1, int64_t pstride = 0,
                                                        float* __restrict__ l2out = nullptr) {
  const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= T) return;
  const int64_t tr[1] = {t};
  const int lane = threadIdx.x & 63;
  ln384_rows<XF, 1>(x, y, g, bt, eps, xh, xl, tr, lane, parts, pstride);
  if constexpr (L2 && !XF) {
  // (round 6) the bge head fused into the last layer's residual + LayerNorm of the CLS rows:
  // out[t] = x[t] / max(||x[t]||, 1e-12) with cls_normalize_kernel's exact arithmetic — its
  // lane m holds columns m + 64 j, so the row just written goes through this wave's LDS
  // slice into that layout (one dispatch fewer per query-batch forward)
  __shared__ float rowbuf[4][384];
  float* rb = rowbuf[threadIdx.x >> 6];
  if (lane < 48) {
    const floatx4 a = *reinterpret_cast<const floatx4*>(x + t * 384 + 8 * lane);
    const floatx4 b = *reinterpret_cast<const floatx4*>(x + t * 384 + 8 * lane + 4);
    *reinterpret_cast<floatx4*>(rb + 8 * lane) = a;
    *reinterpret_cast<floatx4*>(rb + 8 * lane + 4) = b;
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  float v[6];
  float sq = 0.f;
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    v[j] = rb[lane + 64 * j];
    sq += v[j] * v[j];
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) sq += __shfl_xor(sq, d, 64);
  const float inv = 1.0f / fmaxf(sqrtf(sq), 1e-12f);
#pragma unroll
  for (int j = 0; j < 6; ++j) l2out[t * 384 + lane + 64 * j] = v[j] * inv;
  }
}

// ----------------------------------------------------------------------------------------
// GEMM: C[M,N] = A[M,K] . W[N,K]^T + bias[N]   (A fp16 row-major, W fp16 [N][K] = HF Linear)
// 128x128 tile, BK = 64 (fp16) / 32 (fp16x3), 256 threads = 2x2 waves of 64x64,
// v_mfma_f32_16x16x32_f16.
// Register-staged double-buffered LDS (one barrier per K step), XOR-swizzled 16-B chunks.
// ----------------------------------------------------------------------------------------
// kEpiAddLn (gemm_pipe_kernel<PipeRow> only): x = LN(x + A.W^T + bias) on whole rows
enum Epi { kEpiF16 = 0, kEpiGeluF16 = 1, kEpiF32 = 2, kEpiAddLn = 3 };

constexpr int BM = 128, BN = 128;

// K step: 64 for fp16 (2 planes: 64 KB double-buffered LDS), 32 for fp16x3 (4 planes, also
// 64 KB) so both modes fit two workgroups per CU.
template <bool SPLIT> constexpr int kBK = SPLIT ? 32 : 64;

// 16-B chunk swizzle of a row-major [rows][CPR chunks] LDS image for the MFMA fragment read
// (lane l: row l & 15 of a 16-row block, chunk c0 + (l >> 4)), conflict-free under the
// ds_read_b128 lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31}, {32-35,44-47,52-59},
// {36-43,48-51,60-63} (MI355X_MICROARCH.md §LDS): each group's 16 lanes must cover all 64
// banks. CPR 8 (128-B rows, bank = 32 (r % 2) + 4 c'): c' = c ^ (r & 7). CPR 4 (64-B rows,
// bank = 16 (r % 4) + 4 c'): c' = c ^ 3 [r & 8] — a group pairs rows {0-3, 12-15} at chunk c
// with rows {4-11} at chunk c + 1, so the flip has to separate rows 0-7 from 8-15 (the
// round-1 flip by row quad, c ^ (r / 4 % 4), left rows 0-3 and 4-7 on the same banks:
// 2-way conflicts in every fp16x3 fragment read).
template <int CPR>
__device__ __forceinline__ int swz_chunk(int row, int chunk) {
  if constexpr (CPR == 8) return chunk ^ (row & 7);
  else return chunk ^ (((row >> 3) & 1) * 3);
}
template <int CPR>
__device__ __forceinline__ int swz(int row, int chunk) {
  return row * CPR + swz_chunk<CPR>(row, chunk);
}

template <int EPI, bool SPLIT>
__global__ __launch_bounds__(256) void gemm_kernel(const _Float16* __restrict__ A,
                                                   const _Float16* __restrict__ Al,
                                                   const _Float16* __restrict__ W,
                                                   const _Float16* __restrict__ Wl,
                                                   const float* __restrict__ bias, int M, int N,
                                                   int K, void* __restrict__ Cout,
                                                   _Float16* __restrict__ Clo) {
  // SPLIT (fp16x3): tiles of A_hi, A_lo, W_hi, W_lo; 3 MFMAs per product.
  constexpr int NP = SPLIT ? 4 : 2;                     // staged planes
  constexpr int BK = kBK<SPLIT>, CPR = BK / 8, LPT = BM * CPR / 256;   // loads/thread/plane
  // [buf][plane][row][CPR chunks]; also the epilogue's 4 x 32 x 68 fp32 staging (34 KB)
  constexpr int kLdsH8 = 2 * NP * BM * CPR > 4 * 32 * 68 / 4 ? 2 * NP * BM * CPR : 4 * 32 * 68 / 4;
  __shared__ half8 lds[kLdsH8];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  // XCD-aware tile order: blocks are dealt round-robin over the 8 XCDs, so XCD x runs
  // blocks x, x+8, ...; give it the contiguous tile range [x*cpx, (x+1)*cpx) with the N
  // tiles of one M tile adjacent, so the A panel is fetched into that XCD's L2 once and
  // reused by all N/BN column tiles (instead of once per XCD).
  const int nN = N / BN, nM = (M + BM - 1) / BM;
  const int cpx = gridDim.x >> 3;
  const int tile = (blockIdx.x & 7) * cpx + (blockIdx.x >> 3);
  if (tile >= nM * nN) return;
  const int m0 = (tile / nN) * BM, n0 = (tile % nN) * BN;
  const int nk = K / BK;
  const _Float16* src[4] = {A, W, Al, Wl};

  half8 rg[NP][LPT];
  auto gload = [&](int kt) {
#pragma unroll
    for (int p = 0; p < NP; ++p)
#pragma unroll
      for (int i = 0; i < LPT; ++i) {
        const int c = tid + 256 * i;
        const int row = c / CPR, ch = c % CPR;
        const int r = (p & 1) ? (n0 + row) : min(m0 + row, M - 1);   // planes 0,2: A; 1,3: W
        rg[p][i] = *reinterpret_cast<const half8*>(src[p] + (int64_t)r * K + kt * BK + ch * 8);
      }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      half8* lp = lds + (buf * NP + p) * (BM * CPR);
#pragma unroll
      for (int i = 0; i < LPT; ++i) {
        const int c = tid + 256 * i;
        lp[swz<CPR>(c / CPR, c % CPR)] = rg[p][i];
      }
    }
  };

  floatx4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  gload(0);
  lstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
    const half8* la = lds + (buf * NP + 0) * (BM * CPR);
    const half8* lb = lds + (buf * NP + 1) * (BM * CPR);
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      half8 af[4], bf[4];
      const int ch = ks * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = la[swz<CPR>(wr * 64 + i * 16 + (lane & 15), ch)];
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = lb[swz<CPR>(wc * 64 + j * 16 + (lane & 15), ch)];
      if constexpr (SPLIT) {
        const half8* lal = lds + (buf * NP + 2) * (BM * CPR);
        const half8* lbl = lds + (buf * NP + 3) * (BM * CPR);
        half8 afl[4], bfl[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) afl[i] = lal[swz<CPR>(wr * 64 + i * 16 + (lane & 15), ch)];
#pragma unroll
        for (int j = 0; j < 4; ++j) bfl[j] = lbl[swz<CPR>(wc * 64 + j * 16 + (lane & 15), ch)];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(afl[i], bf[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bfl[j], acc[i][j], 0, 0, 0);
          }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) lstore(buf ^ 1);
    __syncthreads();
  }

  // epilogue: lane holds C[rows 16i + 4(l>>4) + r][col 16j + (l&15)] of the wave's 64x64
  // tile. Stage 32-row halves through the (now idle) LDS as fp32 [32][68] per wave (stride
  // 68 dwords: the four 16-lane row groups land on disjoint banks), then each lane takes
  // 8 consecutive columns of a row: bias + activation + conversion there, and 16-B stores
  // (full 128-B row segments per 8 lanes) instead of 2-B scattered ones.
  constexpr int ES = 68;
  float* ep = reinterpret_cast<float*>(lds) + wid * (32 * ES);
  const int rr = lane >> 3, cc = (lane & 7) * 8;       // read: row rr + 8s, cols cc..cc+7
  const int gn = n0 + wc * 64 + cc;
  float bn[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bn[e] = bias[gn + e];
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
#pragma unroll
    for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          ep[(i2 * 16 + 4 * (lane >> 4) + r) * ES + j * 16 + (lane & 15)] = acc[hf * 2 + i2][j][r];
    __builtin_amdgcn_s_waitcnt(0xc07f);                 // lgkmcnt(0): own LDS writes landed
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int s8 = 0; s8 < 4; ++s8) {
      const int lr = rr + 8 * s8;
      const int m = m0 + wr * 64 + hf * 32 + lr;
      const floatx4 lo4 = *reinterpret_cast<const floatx4*>(ep + lr * ES + cc);
      const floatx4 hi4 = *reinterpret_cast<const floatx4*>(ep + lr * ES + cc + 4);
      float v[8] = {lo4[0], lo4[1], lo4[2], lo4[3], hi4[0], hi4[1], hi4[2], hi4[3]};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        v[e] += bn[e];
        if constexpr (EPI == kEpiGeluF16) v[e] = gelu_erf(v[e]);
      }
      if (m < M) {
        if constexpr (EPI == kEpiF32) {
          float* o = static_cast<float*>(Cout) + (int64_t)m * N + gn;
          *reinterpret_cast<floatx4*>(o) = floatx4{v[0], v[1], v[2], v[3]};
          *reinterpret_cast<floatx4*>(o + 4) = floatx4{v[4], v[5], v[6], v[7]};
        } else {
          half8 h, l;
#pragma unroll
          for (int e = 0; e < 8; e += 2) {
            if constexpr (SPLIT) {
              half2 h2, l2;
              split16x2(v[e], v[e + 1], h2, l2);
              h[e] = h2[0]; h[e + 1] = h2[1]; l[e] = l2[0]; l[e + 1] = l2[1];
            } else {
              h[e] = (_Float16)v[e];
              h[e + 1] = (_Float16)v[e + 1];
            }
          }
          *reinterpret_cast<half8*>(static_cast<_Float16*>(Cout) + (int64_t)m * N + gn) = h;
          if constexpr (SPLIT) *reinterpret_cast<half8*>(Clo + (int64_t)m * N + gn) = l;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// ----------------------------------------------------------------------------------------
// Persistent pipelined GEMM for large token counts (rerank batches, chunk encode):
// C[M,N] = A[M,K] . W[N,K]^T + bias, same epilogues as gemm_kernel.
//
// One 8-wave workgroup per CU loops over 256x128 output tiles (XCD-aware: in every round of
// gridDim.x tiles, the workgroups of one XCD take a contiguous tile range, so the N tiles of
// an A panel run on the same L2). K is short here (384 / 1024 / 1536), so a tile is only
// 6-24 K steps: a per-tile load prologue would expose one HBM latency per few hundred MFMA
// cycles. Instead the loads run on a flat (tile, k-step) sequence through a 3-stage LDS ring
// filled by direct buffer->LDS DMA (buffer_load_dwordx4 ... lds), two stages in flight,
// straight across tile boundaries — the next tile's first stages land while this tile's
// epilogue runs.
// Addressing is hoisted out of the loop: a tile's A and W panels are two buffer resources
// (wave-uniform SGPRs, rebuilt once per tile; A's extent ends at row M, so rows past M read
// as zeros), every lane's byte offset inside a panel is a launch constant (the XOR swizzle of
// the LDS image is applied to it), and a K step only moves the scalar soffset. A step costs
// 6 DMAs + their M0 writes besides its 32 (fp16) / 48 (fp16x3) MFMAs and 16 ds_read_b128.
// Sync per K step: counted `s_waitcnt vmcnt` + one raw s_barrier (step g landed for every
// wave AND every wave is done reading step g-1, whose slot the next DMA reuses). Besides the
// DMAs the loop issues only the epilogue's stores, a fixed number S per tile (buffer stores
// bounded to the M x N output: rows past M are dropped by the range check, never by exec
// masking), so every vmcnt is exact.
// Operands are swapped in the MFMA (D = W . A^T): lane l holds C[m][n .. n+3] for
// m = row (l & 15) of the fragment and 4 consecutive features n, so the epilogue adds bias
// (staged in LDS once per launch), applies GELU and stores 8-B (fp16) / 16-B (fp32) vectors
// straight from registers; the LDS stays the ring's.
// ----------------------------------------------------------------------------------------
// Two shapes of the same kernel (PipeCfg): LARGE — 256x128 tiles, 8 waves of 64x64, 3-stage
// ring, one workgroup per CU, persistent (rerank / chunk-encode token counts); SMALL —
// 64x64 tiles, 4 waves of 32x32, a 4-stage ring (fp16: the whole K = 384 of a tile in
// flight after the prologue), for query batches of a few hundred to a few thousand tokens,
// where a GEMM is a handful of tiles per CU and latency, not MFMA rate, sets its time.
constexpr int kPipeBiasMax = 4096;            // floats of bias staged in LDS (N <= 4096)
template <int BM_, int BN_, int WAVES_M_, int WAVES_N_, int NS_, int BK_ = 0, int LOADERS_ = 4,
          int BIAS_ = kPipeBiasMax>
struct PipeCfg {
  static constexpr int BM = BM_, BN = BN_, WAVES_M = WAVES_M_, WAVES_N = WAVES_N_, NS = NS_;
  static constexpr int BIAS = BIAS_;   // gemm_pipe_kernel's staged-vector area (floats)
  static constexpr int BK = BK_;   // K step; 0 = kBK<SPLIT> (64 fp16 / 32 fp16x3)
  static constexpr int LOADERS = LOADERS_;   // gemm_ws_kernel's loader waves
  static constexpr int THREADS = 64 * WAVES_M * WAVES_N;
  static constexpr int FM = BM / WAVES_M / 16, FN = BN / WAVES_N / 16;   // 16x16 frags/wave
  // a K step's fragments all loaded before its MFMAs (the large tiles; see the main loop)
  static constexpr bool PRELOAD = BM * BN >= 256 * 128;
};
using PipeLarge = PipeCfg<256, 128, 4, 2, 3>;
// whole 384-wide rows per tile (bge-small / MiniLM hidden size): the output projections with
// residual + LayerNorm fused into the epilogue (kEpiAddLn); 2 x 4 waves of 64 x 96
using PipeRow = PipeCfg<128, 384, 2, 4, 2>;
// (fp16x3: a 3-stage ring, 64 KB with the staged vectors, two workgroups per CU. Round 5
// A/B builds: 4 stages (2 per CU) and 6 / 8 stages (1 per CU, for GEMMs whose units fit the
// CUs) each ran the 32-query bge-small forward slower, 0.69 -> 0.71 / 0.72 / 0.73 ms, and
// config 2 at 72.6-74.5K -> 71.0-71.2K / 64.8-65.4K / 64.1K qps: a K step's time there is not
// the ring's latency; profiles/r05b_small_ring_depth_ab.jsonl)
// (wave grid, round 5 A/B builds: 2 x 1 / 1 x 2 / 1 x 1 waves of 32 x 64 / 64 x 32 / 64 x 64
// ran the 32-query forward in 0.757 / 0.762 / 0.99 ms vs 0.675 for 2 x 2 — fewer LDS fragment
// reads per step, but fewer waves to issue them; profiles/r05i_small_wave_grid_ab.jsonl)
template <bool SPLIT> using PipeSmall = PipeCfg<64, 64, 2, 2, SPLIT ? 3 : 4>;
// (Measured and removed in round 5 — numbers in DESIGN.md §R5: 256x256 / 256x192 PIPE tiles,
// register-blocked BIG / BIG128 shapes, BK-64 and 64x128 query-batch tiles, the one-loader and
// deferred-LN query-batch WS tiles, and the 256x192 ping-pong kernel.)
// fp16x3 query-batch GEMMs with N <= 2048 (round 6): a 2-stage ring and an 8 KB staged-vector
// area, 40 KB of LDS — four workgroups per CU instead of two, room for the config-2
// pipeline's concurrent batches. Bitwise the same outputs (same tiles, K order and epilogue);
// the 32-query forward alone 0.694 -> 0.704 ms, config 2 77.4-80.6K -> 80.0-81.5K qps over
// five interleaved pairs, config 3 unchanged (profiles/r06_small_ring/). Wider N (bge-large's
// 3072 / 4096) keeps PipeSmall<true>.
using PipeSmallR2 = PipeCfg<64, 64, 2, 2, 2, 0, 4, 2048>;
constexpr int PBM = PipeLarge::BM, PBN = PipeLarge::BN;
constexpr int kPipeThreads = PipeLarge::THREADS;

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// 16 B per lane buffer -> LDS DMA: lane l's bytes at panel + soff + voff land at LDS byte
// address lds_addr + 16 l. Inline asm for the same reason as glds16 (device_common.hpp).
__device__ __forceinline__ void blds16(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff,
                                       uint32_t lds_addr) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(rs), "s"(lds_addr), "s"(soff)
      : "memory");
}

// raw buffer resource over [base, base + bytes) from wave-uniform inputs (reads past the
// end return zeros, stores past it are dropped); bytes < 2^31 (checked by the launcher)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t panel(const void* base, int64_t bytes) {
  // every input made provably wave-uniform (T20): a descriptor the compiler cannot prove
  // uniform lands in VGPRs (asm "s" operand error / waterfall loops around buffer ops)
  const uint64_t a = (uint64_t)(uintptr_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const int nb = bytes > 0 ? (int)bytes : 0;
  void* p = reinterpret_cast<void*>((uintptr_t)(((uint64_t)hi << 32) | lo));
  return __builtin_amdgcn_make_buffer_rsrc(p, 0, __builtin_amdgcn_readfirstlane(nb),
                                           0x00020000);
}

// s_waitcnt vmcnt(Y*L + (stored ? S : 0)) for a runtime Y in [0, Y_MAX] (vmcnt takes an
// immediate): Y = ring stages issued after the one being waited for
template <int L, int S, int Y>
__device__ __forceinline__ void wait_ring(int y, bool stored) {
  if (y == Y) {
    if (stored)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(Y * L + S) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(Y * L) : "memory");
    return;
  }
  if constexpr (Y > 0) wait_ring<L, S, Y - 1>(y, stored);
}

// fp16 out: fragments j, j+1 of a row pair up through one v_permlane16_swap per dword
// (lanes 16-31 of the j value <-> lanes 0-15 of the j+1 value, same for 48-63 / 32-47), after
// which every lane holds 8 consecutive columns: 16-B stores, half the store instructions of
// 8-B ones (the epilogue is store-issue-bound). Lane group g = lane >> 4 then owns columns
// 16 j + {0, 16, 8, 24}[g] .. +7 (byte offset vo).
template <int AUX = 0>
__device__ __forceinline__ void store_f16_pair(half4 xa, half4 xb, __amdgpu_buffer_rsrc_t rsc,
                                               int vo, int so = 0) {
  u32x2 a = __builtin_bit_cast(u32x2, xa), b = __builtin_bit_cast(u32x2, xb);
  const auto r0 = __builtin_amdgcn_permlane16_swap(a[0], b[0], false, false);
  const auto r1 = __builtin_amdgcn_permlane16_swap(a[1], b[1], false, false);
  const u32x4 d = {r0[0], r1[0], r0[1], r1[1]};
  __builtin_amdgcn_raw_buffer_store_b128(d, rsc, vo, so, AUX);
}

// the plain epilogues (kEpiF16 / kEpiGeluF16 / kEpiF32) of one wave's FM x FN accumulator
// fragments of the tile at column n0 (rc / rl: the output panels from the tile's row m0):
// bias (staged in LDS), GELU, then fp32 16-B stores or fp16 [+ lo plane] paired 16-B stores
// straight from registers — exactly pipe_plain_stores<EPI, SPLIT, CFG>() stores per wave (the
// ring's vmcnt accounting counts them). NO_STORE: timing probe, nothing written. AUX: the
// stores' cache policy (buffer-op aux bits; 2 = nt).
template <int EPI, bool SPLIT, typename CFG>
constexpr int pipe_plain_stores() {
  return EPI == kEpiF32 ? CFG::FM * CFG::FN : CFG::FM * CFG::FN / 2 * (SPLIT ? 2 : 1);
}

// one fragment pair (i, jp), (i, jp + 1) of it
template <int EPI, bool SPLIT, typename CFG, bool NO_STORE, int AUX = 0>
__device__ __forceinline__ void pipe_epi_pair(const floatx4& a0, const floatx4& a1, int i, int jp,
                                              const float* bias_l, __amdgpu_buffer_rsrc_t rc,
                                              __amdgpu_buffer_rsrc_t rl, int N, int n0, int wr,
                                              int wc, int lane) {
  constexpr int WTM = 16 * CFG::FM, WTN = 16 * CFG::FN;
  const int g = lane >> 4;
  const int ml = wr * WTM + i * 16 + (lane & 15);
  if constexpr (EPI == kEpiF32) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int nl = wc * WTN + (jp + h) * 16 + 4 * g;
      const floatx4 v = (h ? a1 : a0) + *reinterpret_cast<const floatx4*>(bias_l + n0 + nl);
      if (!NO_STORE || v[0] == 1234.5f)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rc,
                                               (ml * N + n0 + nl) * 4, 0, AUX);
    }
  } else {
    // fp16 out, two fragments per 16-B store (store_f16_pair)
    const int cofs = 8 * ((g & 1) * 2 + (g >> 1));
    const floatx4 b0 = *reinterpret_cast<const floatx4*>(bias_l + n0 + wc * WTN + jp * 16 + 4 * g);
    const floatx4 b1 = *reinterpret_cast<const floatx4*>(bias_l + n0 + wc * WTN + jp * 16 + 16 + 4 * g);
    const int vo = (ml * N + n0 + wc * WTN + jp * 16 + cofs) * 2;
    floatx4 va = a0 + b0, vb = a1 + b1;
    if constexpr (EPI == kEpiGeluF16) {
      va = gelu_erf4(va);
      vb = gelu_erf4(vb);
    }
    half4 ha, hb, la, lb;
#pragma unroll
    for (int r = 0; r < 4; r += 2) {
      if constexpr (SPLIT) {
        half2 h2, l2;
        split16x2(va[r], va[r + 1], h2, l2);
        ha[r] = h2[0]; ha[r + 1] = h2[1]; la[r] = l2[0]; la[r + 1] = l2[1];
        split16x2(vb[r], vb[r + 1], h2, l2);
        hb[r] = h2[0]; hb[r + 1] = h2[1]; lb[r] = l2[0]; lb[r + 1] = l2[1];
      } else {
        ha[r] = (_Float16)va[r];
        ha[r + 1] = (_Float16)va[r + 1];
        hb[r] = (_Float16)vb[r];
        hb[r + 1] = (_Float16)vb[r + 1];
      }
    }
    if (!NO_STORE || va[0] == 1234.5f) store_f16_pair<AUX>(ha, hb, rc, vo);
    if constexpr (SPLIT)
      if (!NO_STORE || vb[0] == 1234.5f) store_f16_pair<AUX>(la, lb, rl, vo);
  }
}

template <int EPI, bool SPLIT, typename CFG, bool NO_STORE, int AUX = 0>
__device__ __forceinline__ void pipe_plain_epilogue(const floatx4 (&acc)[CFG::FM][CFG::FN],
                                                    const float* bias_l,
                                                    __amdgpu_buffer_rsrc_t rc,
                                                    __amdgpu_buffer_rsrc_t rl, int N, int n0,
                                                    int wr, int wc, int lane) {
#pragma unroll
  for (int jp = 0; jp < CFG::FN; jp += 2)
#pragma unroll
    for (int i = 0; i < CFG::FM; ++i)
      pipe_epi_pair<EPI, SPLIT, CFG, NO_STORE, AUX>(acc[i][jp], acc[i][jp + 1], i, jp, bias_l, rc,
                                                   rl, N, n0, wr, wc, lane);
}

// ----------------------------------------------------------------------------------------
// Deferred LayerNorm (fp16x3, hidden 384, the WS GEMMs of large token batches). Between the
// sublayers the token rows' residual stream is kept un-normalised: z = x + sublayer output, as
// fp16 hi + lo planes, plus per row kDlParts partial statistics (mean, centred sum of squares)
// of its 64-column blocks, written by the producing GEMM's epilogue (kEpiResLn). LN(z) is never
// materialised for the token rows:
//  * the consuming GEMMs (QKV, FFN1: kEpiLnF16 / kEpiLnGeluF16) multiply z by W' = W diag(gamma)
//    and correct each row in the epilogue: LN(z) W^T + b = rs (z W'^T - mu c1) + c2, with
//    c1[n] = sum_k W'[n][k] (of the fp16x3 planes) and c2 = b + W beta, folded at encoder
//    creation;
//  * the next residual add (kEpiResLn) recomputes LN(z) per element from the planes and the row
//    statistics: x = (z - mu) rs gamma + beta (fp32), then z' = x + (A W^T + b).
// Per element of a 384-wide projection this replaces the fp32 y write, add_ln's reads of y and
// x and its write of x (16 B) with the residual read and the z write (8 B), and drops the
// add_ln launches.
// ----------------------------------------------------------------------------------------
enum EpiDl { kEpiLnF16 = 4, kEpiLnGeluF16 = 5, kEpiResLn = 6 };
constexpr int kDlH = 384, kDlParts = kDlH / 64;
struct DlArgs {
  const float* st_in = nullptr;    // [M][kDlParts] x {mean, M2}: stats of the A rows (Ln*) or of
                                   // the residual rows (ResLn; null = already normalised)
  float* st_out = nullptr;         // ResLn: stats of the rows written
  const float* gamma = nullptr;    // ResLn: the LayerNorm pending on the residual rows
  const float* beta = nullptr;
  const float* c1 = nullptr;       // Ln*: [N] column sums of W' (the bias argument is c2)
  float eps = 0.f;
};

// hi + lo fp16 planes (4 values each, as loaded) -> fp32 by v_fma_mix_f32 (hi * 1 + lo in one
// instruction; exact, as (float)hi + (float)lo). The inputs come from memory loads, never
// straight from an MFMA (no inline-asm hazard; see split16x2).
__device__ __forceinline__ floatx4 mix_f16x4(u32x2 h, u32x2 l) {
  floatx4 z;
#pragma unroll
  for (int d = 0; d < 2; ++d) {
    float lo, hi;
    asm("v_fma_mix_f32 %0, %1, 1.0, %2 op_sel_hi:[1,0,1]" : "=v"(lo) : "v"(h[d]), "v"(l[d]));
    asm("v_fma_mix_f32 %0, %1, 1.0, %2 op_sel:[1,0,1] op_sel_hi:[1,0,1]"
        : "=v"(hi) : "v"(h[d]), "v"(l[d]));
    z[2 * d] = lo;
    z[2 * d + 1] = hi;
  }
  return z;
}

// combine a row's kDlParts block statistics (s0..s2 = {mean_0, M2_0, mean_1, M2_1}, ...;
// Chan et al.'s pairwise update over equal 64-element blocks) into its mean and 1/sqrt(var+eps)
__device__ __forceinline__ void dl_row_stats(const floatx4& s0, const floatx4& s1,
                                             const floatx4& s2, float eps, float& mu, float& rs) {
  const float m[kDlParts] = {s0[0], s0[2], s1[0], s1[2], s2[0], s2[2]};
  float q = (s0[1] + s0[3]) + (s1[1] + s1[3]) + (s2[1] + s2[3]);
  mu = ((m[0] + m[1]) + (m[2] + m[3]) + (m[4] + m[5])) * (1.0f / kDlParts);
#pragma unroll
  for (int j = 0; j < kDlParts; ++j) {
    const float d = m[j] - mu;
    q += 64.f * d * d;
  }
  rs = rsqrtf(q * (1.0f / kDlH) + eps);
}

// A row's statistics as the epilogue holds them: the 4 lanes of row ml (g = lane >> 4) load
// floats 4g..4g+3 of its 12 (g < 3: blocks 2g, 2g+1; g = 3 nothing new) a whole tile before
// the epilogue needs them (4 VGPRs per row group; all 12 per lane would not
// fit beside the fragments), and the epilogue combines them across the lanes.
template <int FM>
__device__ __forceinline__ void dl_prefetch_stats(floatx4 (&dls)[FM], __amdgpu_buffer_rsrc_t rsi,
                                                  int wr, int lane) {
  const int g = lane >> 4;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int ml = wr * 16 * FM + i * 16 + (lane & 15);
    // (lane group 3 re-reads group 2's floats; dl_lane_stats ignores them)
    dls[i] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(
                                             rsi, (ml * kDlParts * 2 + 4 * min(g, 2)) * 4, 0, 0));
  }
}

// mean and 1/sqrt(var + eps) of the row from the lane-split statistics (dl_row_stats' Chan
// combination, reduced over lanes l, l^16, l^32, l^48)
__device__ __forceinline__ void dl_lane_stats(const floatx4& v, int g, float eps, float& mu,
                                              float& rs) {
  float sm = g < 3 ? v[0] + v[2] : 0.f;
  sm += __shfl_xor(sm, 16, 64);
  sm += __shfl_xor(sm, 32, 64);
  mu = sm * (1.0f / kDlParts);
  float q = 0.f;
  if (g < 3) {
    const float d0 = v[0] - mu, d2 = v[2] - mu;
    q = (v[1] + v[3]) + 64.f * (d0 * d0 + d2 * d2);
  }
  q += __shfl_xor(q, 16, 64);
  q += __shfl_xor(q, 32, 64);
  rs = rsqrtf(q * (1.0f / kDlH) + eps);
}

// the deferred-LayerNorm epilogues of one wave's FM x FN fragments (its 64 columns are one
// stats block): fp16 hi + lo planes out through paired 16-B stores (store_f16_pair), ResLn also
// the block's {mean, M2} per row. lds_f: bias | c1 (Ln*) or bias | gamma | beta (ResLn).
// dls: the rows' prefetched statistics (dl_prefetch_stats); rs_out: the output stats panel
// from the tile's row m0.
// fragments (i, jp), (i, jp + 1) of a deferred-LN epilogue -> fp16 hi / lo planes (16-B
// paired stores, store_f16_pair)
template <int AUX, int FM, int FN>
__device__ __forceinline__ void dl_store_pair(const floatx4 (&acc)[FM][FN], int i, int jp, int ml,
                                              int N, int n0, int wc, int cofs,
                                              __amdgpu_buffer_rsrc_t rc,
                                              __amdgpu_buffer_rsrc_t rl) {
  const int vo = (ml * N + n0 + wc * (16 * FN) + jp * 16 + cofs) * 2;
  half4 ha, hb, la, lb;
#pragma unroll
  for (int r = 0; r < 4; r += 2) {
    half2 h2, l2;
    split16x2(acc[i][jp][r], acc[i][jp][r + 1], h2, l2);
    ha[r] = h2[0]; ha[r + 1] = h2[1]; la[r] = l2[0]; la[r + 1] = l2[1];
    split16x2(acc[i][jp + 1][r], acc[i][jp + 1][r + 1], h2, l2);
    hb[r] = h2[0]; hb[r + 1] = h2[1]; lb[r] = l2[0]; lb[r + 1] = l2[1];
  }
  store_f16_pair<AUX>(ha, hb, rc, vo);
  store_f16_pair<AUX>(la, lb, rl, vo);
}

template <int EPI, typename CFG, int AUX>
__device__ __forceinline__ void ws_dl_epilogue(floatx4 (&acc)[CFG::FM][CFG::FN],
                                               const float* lds_f, __amdgpu_buffer_rsrc_t rc,
                                               __amdgpu_buffer_rsrc_t rl,
                                               const floatx4 (&dls)[CFG::FM],
                                               __amdgpu_buffer_rsrc_t rs_out, bool has_stats,
                                               int N, int n0, int wr, int wc, int lane,
                                               float eps) {
  constexpr int FM = CFG::FM, FN = CFG::FN, WTM = 16 * FM, WTN = 16 * FN;
  static_assert(WTN == 64 && FN % 2 == 0, "a wave's columns are one stats block");
  const int g = lane >> 4;
  const int cofs = 8 * ((g & 1) * 2 + (g >> 1));
  const float* bias_l = lds_f;
  const float* c1_l = lds_f + N;                          // Ln*
  const float *gam_l = lds_f + N, *bet_l = lds_f + 2 * N;  // ResLn
  // ResLn: residual z of row group i + 1 loaded before group i is computed (read before this
  // wave overwrites it; all four groups at once would spill)
  u32x2 zh[2][FN], zl[2][FN];
  auto load_res = [&](int i) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int vo = ((wr * WTM + i * 16 + (lane & 15)) * N + n0 + wc * WTN + j * 16 + 4 * g) * 2;
      zh[i & 1][j] = __builtin_amdgcn_raw_buffer_load_b64(rc, vo, 0, 0);
      zl[i & 1][j] = __builtin_amdgcn_raw_buffer_load_b64(rl, vo, 0, 0);
    }
  };
  if constexpr (EPI == kEpiResLn) load_res(0);
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    if constexpr (EPI == kEpiResLn)
      if (i + 1 < FM) load_res(i + 1);
    const int ml = wr * WTM + i * 16 + (lane & 15);
    float mu = 0.f, rs = 1.f;
    if (EPI != kEpiResLn || has_stats) dl_lane_stats(dls[i], g, eps, mu, rs);
    if constexpr (EPI == kEpiResLn) {
      // residual x = LN(z) = z rs gamma + (beta - mu rs gamma) from the planes; 4-wide vector
      // arithmetic throughout (gfx950 packed fp32: v_pk_fma / v_pk_add / v_pk_mul)
      const floatx4 a4 = {rs, rs, rs, rs}, b4 = {-mu * rs, -mu * rs, -mu * rs, -mu * rs};
      floatx4 s4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int nl = n0 + wc * WTN + j * 16 + 4 * g;
        const floatx4 z = mix_f16x4(zh[i & 1][j], zl[i & 1][j]);
        const floatx4 b = *reinterpret_cast<const floatx4*>(bias_l + nl);
        floatx4 xr = z;
        if (has_stats)
          xr = __builtin_elementwise_fma(__builtin_elementwise_fma(z, a4, b4),
                                         *reinterpret_cast<const floatx4*>(gam_l + nl),
                                         *reinterpret_cast<const floatx4*>(bet_l + nl));
        acc[i][j] = (acc[i][j] + b) + xr;
        s4 += acc[i][j];
      }
      // the row's 64 columns sit in lanes l, l^16, l^32, l^48
      float s = (s4[0] + s4[1]) + (s4[2] + s4[3]);
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      const float mw = s * (1.0f / 64);
      const floatx4 m4 = {mw, mw, mw, mw};
      floatx4 q4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const floatx4 d = acc[i][j] - m4;
        q4 = __builtin_elementwise_fma(d, d, q4);
      }
      float q = (q4[0] + q4[1]) + (q4[2] + q4[3]);
      q += __shfl_xor(q, 16, 64);
      q += __shfl_xor(q, 32, 64);
      if (g == 0) {
        const u32x2 d = {__builtin_bit_cast(uint32_t, mw), __builtin_bit_cast(uint32_t, q)};
        __builtin_amdgcn_raw_buffer_store_b64(d, rs_out,
                                              (ml * kDlParts + (n0 + wc * WTN) / 64) * 8, 0, 0);
      }
    } else {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int nl = n0 + wc * WTN + j * 16 + 4 * g;
        const floatx4 c1 = *reinterpret_cast<const floatx4*>(c1_l + nl);
        const floatx4 c2 = *reinterpret_cast<const floatx4*>(bias_l + nl);
        const floatx4 nm4 = {-mu, -mu, -mu, -mu}, rs4 = {rs, rs, rs, rs};
        acc[i][j] = __builtin_elementwise_fma(rs4, __builtin_elementwise_fma(nm4, c1, acc[i][j]), c2);
        if constexpr (EPI == kEpiLnGeluF16) acc[i][j] = gelu_erf4(acc[i][j]);
      }
    }
    if constexpr (EPI == kEpiResLn) {   // z planes (default policy): row group by row group
#pragma unroll
      for (int jp = 0; jp < FN; jp += 2) dl_store_pair<AUX>(acc, i, jp, ml, N, n0, wc, cofs, rc, rl);
    }
  }
  // QKV / FFN1 outputs (non-temporal): column pair outer, row group inner — the plain
  // epilogue's order. Stored row group by row group like the z planes, these nt streams
  // measured 1.37 / 1.42x their bytes in WRITE_SIZE inside the forward, 1.12 / 1.10x in this
  // order (and FETCH 1.25 -> 1.22 / 1.55 -> 1.43x); the z planes go the other way (1.00 ->
  // 1.14 / 1.20x), so they keep theirs (profiles/r02t_fwd_pmc.jsonl,
  // r02u_fwd_pmc_storeorder_all.jsonl)
  if constexpr (EPI != kEpiResLn) {
#pragma unroll
    for (int jp = 0; jp < FN; jp += 2)
#pragma unroll
      for (int i = 0; i < FM; ++i)
        dl_store_pair<AUX>(acc, i, jp, wr * WTM + i * 16 + (lane & 15), N, n0, wc, cofs, rc, rl);
  }
}

// kEpiAddLn operands besides the GEMM's (Cout = the fp32 residual rows x, read and
// overwritten; Clo = the lo plane of the fp16x3 copy)
struct LnArgs {
  const float* gamma = nullptr;
  const float* beta = nullptr;
  _Float16* xh = nullptr;       // fp16 copy of the normalised rows (the next GEMM's A)
  float eps = 0.f;
};

// block size of a gemm_pipe_kernel instance (launch_fixed; its __launch_bounds__)
template <typename CFG> constexpr int kPipeBlock = CFG::THREADS;

template <int EPI, bool SPLIT, typename CFG>
__global__ __launch_bounds__(kPipeBlock<CFG>, 1) void gemm_pipe_kernel(
    const _Float16* __restrict__ A, const _Float16* __restrict__ Al,
    const _Float16* __restrict__ W, const _Float16* __restrict__ Wl,
    const float* __restrict__ bias, int M, int N, int K, void* __restrict__ Cout,
    _Float16* __restrict__ Clo, LnArgs ln, int ksplit = 1) {
  constexpr int BM = CFG::BM, BN = CFG::BN, NS = CFG::NS, TH = CFG::THREADS;
  constexpr int FM = CFG::FM, FN = CFG::FN, WTM = 16 * FM, WTN = 16 * FN;
  constexpr int BK = CFG::BK ? CFG::BK : kBK<SPLIT>, CPR = BK / 8;
  constexpr int NPL = SPLIT ? 2 : 1;                     // planes per operand (hi[, lo])
  constexpr int A_H8 = BM * CPR, W_H8 = BN * CPR;        // half8 per plane per stage
  constexpr int STAGE_H8 = NPL * (A_H8 + W_H8);
  constexpr int LA = A_H8 / TH, LW = W_H8 / TH;          // DMAs per wave per plane
  constexpr int L = NPL * (LA + LW);                      // DMAs per wave per stage
  // epilogue stores per wave: 16 B each; fp16 outputs pair two fragments per store
  // (kEpiAddLn: the fp32 rows and the fp16 copy [+ lo plane], 8-B stores for the latter).
  // The count is capped at what vmcnt can express: waiting until fewer ops are outstanding
  // than were issued after the awaited stage is only stricter.
  constexpr int S_ISSUED = EPI == kEpiF32   ? FM * FN
                           : EPI == kEpiAddLn ? FM * FN * (SPLIT ? 3 : 2)
                                              : FM * FN / 2 * (SPLIT ? 2 : 1);
  constexpr int S = S_ISSUED < 63 - (NS - 2) * L ? S_ISSUED : 63 - (NS - 2) * L;
  constexpr int OUT_B = EPI == kEpiF32 || EPI == kEpiAddLn ? 4 : 2;   // Cout element bytes
  static_assert(A_H8 % TH == 0 && W_H8 % TH == 0 && FN % 2 == 0, "tile shape");
  static_assert((NS - 2) * L + S <= 63, "vmcnt range");
  // kEpiAddLn keeps bias | gamma | beta | two [WAVES_N][BM] row-sum tables in the bias area
  static_assert(EPI != kEpiAddLn || 3 * BN + 2 * CFG::WAVES_N * BM <= CFG::BIAS,
                "LN staging");
  // one LDS object (ring | bias): a second __shared__ object beside a DMA target can make
  // hipcc drain vmcnt before every ds_read
  __shared__ half8 lds[NS * STAGE_H8 + CFG::BIAS / 4];
  float* bias_l = reinterpret_cast<float*>(lds + NS * STAGE_H8);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid / CFG::WAVES_N, wc = wid % CFG::WAVES_N;
  const uint32_t lbase = lds_addr_of(lds);
  // split-K (kEpiF32 only; the launcher checks K / BK % ksplit == 0 and N <= CFG::BIAS / 2):
  // work unit u = (tile u % n_tiles, K part u / n_tiles) over nk = K / BK / ksplit K steps;
  // part p writes its fp32 partial product to Cout + p M N, the bias only in part 0 (the
  // other parts read zeros staged in the upper half of the bias area); add_ln_kernel sums
  // the parts in order
  const int nN = N / BN, nM = (M + BM - 1) / BM, n_tiles = nM * nN;
  const int nk = K / BK / ksplit;
  const int n_units = n_tiles * ksplit;
  const int G = gridDim.x, per_xcd = G >> 3;
  const int off = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
  const int n_mine = off < n_units ? (n_units - off + G - 1) / G : 0;
  const int steps = n_mine * nk;

  if (ksplit > 1)
    for (int i = tid * 4; i < N; i += TH * 4)
      *reinterpret_cast<floatx4*>(bias_l + CFG::BIAS / 2 + i) = floatx4{0.f, 0.f, 0.f, 0.f};
  // The staged vectors (bias [| gamma | beta]) are loaded into registers here and written to
  // LDS only after the ring prologue's DMAs are issued (below), so their load latency and the
  // first stages' run concurrently instead of back to back — a query-batch GEMM is one or two
  // tiles per workgroup, where that serial latency was a visible part of the launch.
  constexpr int NBV = CFG::BIAS / (TH * 4) > 0 ? CFG::BIAS / (TH * 4) : 1;
  constexpr int NLN = EPI == kEpiAddLn ? (BN + TH * 4 - 1) / (TH * 4) : 0;
  static_assert(NBV * TH * 4 >= CFG::BIAS, "every staged bias float has a register slot");
  floatx4 bv[NBV], gv[NLN > 0 ? NLN : 1], ev[NLN > 0 ? NLN : 1];
#pragma unroll
  for (int u = 0; u < NBV; ++u) {
    const int i = tid * 4 + u * TH * 4;
    if (i < N) bv[u] = *reinterpret_cast<const floatx4*>(bias + i);
  }
#pragma unroll
  for (int u = 0; u < NLN; ++u) {               // N == BN here (checked by the launcher)
    const int i = tid * 4 + u * TH * 4;
    if (i < N) {
      gv[u] = *reinterpret_cast<const floatx4*>(ln.gamma + i);
      ev[u] = *reinterpret_cast<const floatx4*>(ln.beta + i);
    }
  }
  auto stage_vectors = [&]() {
#pragma unroll
    for (int u = 0; u < NBV; ++u) {
      const int i = tid * 4 + u * TH * 4;
      if (i < N) *reinterpret_cast<floatx4*>(bias_l + i) = bv[u];
    }
#pragma unroll
    for (int u = 0; u < NLN; ++u) {
      const int i = tid * 4 + u * TH * 4;
      if (i < N) {
        *reinterpret_cast<floatx4*>(bias_l + BN + i) = gv[u];
        *reinterpret_cast<floatx4*>(bias_l + 2 * BN + i) = ev[u];
      }
    }
    __syncthreads();
  };

  // per-lane byte offsets inside a panel (launch constants): LDS position q of the
  // lane-linear image holds row q / CPR, 16-B chunk (q % CPR) ^ swizzle(row)
  uint32_t voA[LA], voW[LW];
#pragma unroll
  for (int i = 0; i < LA; ++i) {
    const int q = (wid * LA + i) * 64 + lane, r = q / CPR, cs = q % CPR;
    const int c = swz_chunk<CPR>(r, cs);
    voA[i] = (uint32_t)(r * K + c * 8) * 2u;
  }
#pragma unroll
  for (int i = 0; i < LW; ++i) {
    const int q = (wid * LW + i) * 64 + lane, r = q / CPR, cs = q % CPR;
    const int c = swz_chunk<CPR>(r, cs);
    voW[i] = (uint32_t)(r * K + c * 8) * 2u;
  }

  // issue side: next (tile iteration, k-step) to load, its panels and ring slot.
  // A tile's K steps run in a rotated order, starting at k-step (n-tile % nk): the nN tiles
  // that share an A panel (same XCD, same time) then touch different K slices of it at any
  // moment, so one of them takes each slice's L2 miss and the others hit, instead of all of
  // them waiting on the same HBM fetch at every step.
  int it_i = 0, kt_i = 0, kr_i = 0, slot_i = 0, kb_i = 0;
  __amdgpu_buffer_rsrc_t rA0 = panel(A, 0), rA1 = rA0, rW0 = rA0, rW1 = rA0;
  auto issue_next = [&]() {
    if (it_i >= n_mine) return;
    if (kt_i == 0) {
      const int unit = it_i * G + off;
      const int tile = unit % n_tiles;
      kb_i = (unit / n_tiles) * nk;
      const int m0 = (tile / nN) * BM, n0 = (tile % nN) * BN;
      kr_i = (tile % nN) % nk;
      const int64_t abytes = (int64_t)(M - m0) * K * 2, wbytes = (int64_t)BN * K * 2;
      rA0 = panel(A + (int64_t)m0 * K, abytes);
      rW0 = panel(W + (int64_t)n0 * K, wbytes);
      if constexpr (SPLIT) {
        rA1 = panel(Al + (int64_t)m0 * K, abytes);
        rW1 = panel(Wl + (int64_t)n0 * K, wbytes);
      }
    }
    // (wave-uniform by construction; readfirstlane keeps it an SGPR in every instance)
    const uint32_t soff = __builtin_amdgcn_readfirstlane((uint32_t)(kb_i + kr_i) * (BK * 2));
    if (++kr_i == nk) kr_i = 0;
    const uint32_t slot = lbase + (uint32_t)slot_i * (STAGE_H8 * 16);
#ifndef RAGMI_PIPE_PROBE
// build-time timing probe (ragmi/_build.py OUT.so -DRAGMI_PIPE_PROBE=n; results meaningless):
// 1 = no LDS reads / MFMAs in the query-batch tiles' K loop, 2 = no DMAs, 3 = neither
#define RAGMI_PIPE_PROBE 0
#endif
#pragma unroll
    for (int i = 0; i < ((RAGMI_PIPE_PROBE & 2) ? 0 : LA); ++i) {
      const uint32_t d = slot + (uint32_t)((wid * LA + i) * 64 * 16);
      blds16(rA0, voA[i], soff, d);
      if constexpr (SPLIT) blds16(rA1, voA[i], soff, d + A_H8 * 16);
    }
#pragma unroll
    for (int i = 0; i < ((RAGMI_PIPE_PROBE & 2) ? 0 : LW); ++i) {
      const uint32_t d = slot + (uint32_t)((NPL * A_H8 + (wid * LW + i) * 64) * 16);
      blds16(rW0, voW[i], soff, d);
      if constexpr (SPLIT) blds16(rW1, voW[i], soff, d + W_H8 * 16);
    }
    if (++kt_i == nk) { kt_i = 0; ++it_i; }
    if (++slot_i == NS) slot_i = 0;
  };

  floatx4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int p = 0; p < NS - 1; ++p) issue_next();
  stage_vectors();
  int kt_c = 0, it_c = 0, slot_c = 0;
  for (int g = 0; g < steps; ++g) {
    // stages issued after step g: min(NS - 2, steps - 1 - g); plus the last epilogue's
    // stores when it ran at the end of step g-1
    wait_ring<L, S, NS - 2>(min(NS - 2, steps - 1 - g), g > 0 && kt_c == 0);
    __builtin_amdgcn_s_barrier();     // step g landed for all waves; all are past step g-1
    asm volatile("" ::: "memory");    // no LDS read of step g may be scheduled above it
    issue_next();                     // step g+NS-1 -> slot (g-1) % NS

    const half8* sa = lds + slot_c * STAGE_H8;
    const half8* sw = sa + NPL * A_H8;
    if constexpr (CFG::PRELOAD) {
      // every fragment of the K step issued back to back, then the MFMAs (left alone, the
      // compiler loads each fragment just before its first use and waits every few MFMAs;
      // this order measured ~3% faster on the 256-row tiles)
      constexpr int KSN = BK / 32;
      half8 af[KSN][NPL][FM], wf[KSN][NPL][FN];
#pragma unroll
      for (int ks = 0; ks < KSN; ++ks) {
        const int ch = ks * 4 + (lane >> 4);
#pragma unroll
        for (int p = 0; p < NPL; ++p) {
#pragma unroll
          for (int i = 0; i < FM; ++i)
            af[ks][p][i] = sa[p * A_H8 + swz<CPR>(wr * WTM + i * 16 + (lane & 15), ch)];
#pragma unroll
          for (int j = 0; j < FN; ++j)
            wf[ks][p][j] = sw[p * W_H8 + swz<CPR>(wc * WTN + j * 16 + (lane & 15), ch)];
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ks = 0; ks < KSN; ++ks)
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            if constexpr (SPLIT) {   // small terms first: W_lo A_hi + W_hi A_lo + W_hi A_hi
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[ks][1][j], af[ks][0][i], acc[i][j], 0, 0, 0);
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[ks][0][j], af[ks][1][i], acc[i][j], 0, 0, 0);
            }
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[ks][0][j], af[ks][0][i], acc[i][j], 0, 0, 0);
          }
    }
#pragma unroll
    for (int ks = 0; ks < (CFG::PRELOAD || (RAGMI_PIPE_PROBE & 1) ? 0 : BK / 32); ++ks) {
      const int ch = ks * 4 + (lane >> 4);
      half8 af[FM], wf[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = sa[swz<CPR>(wr * WTM + i * 16 + (lane & 15), ch)];
#pragma unroll
      for (int j = 0; j < FN; ++j) wf[j] = sw[swz<CPR>(wc * WTN + j * 16 + (lane & 15), ch)];
      if constexpr (SPLIT) {
        half8 afl[FM], wfl[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) afl[i] = sa[A_H8 + swz<CPR>(wr * WTM + i * 16 + (lane & 15), ch)];
#pragma unroll
        for (int j = 0; j < FN; ++j) wfl[j] = sw[W_H8 + swz<CPR>(wc * WTN + j * 16 + (lane & 15), ch)];
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wfl[j], af[i], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[j], afl[i], acc[i][j], 0, 0, 0);
          }
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[j], af[i], acc[i][j], 0, 0, 0);
    }
    if (++slot_c == NS) slot_c = 0;

    if (++kt_c == nk) {               // tile done: epilogue from registers
      kt_c = 0;
      const int unit = it_c * G + off;
      const int tile = unit % n_tiles, kpart = unit / n_tiles;
      ++it_c;
      const int m0 = (tile / nN) * BM, n0 = (tile % nN) * BN;
      const int64_t cbytes = (int64_t)(M - m0) * N * OUT_B;
      const __amdgpu_buffer_rsrc_t rc =
          panel(static_cast<char*>(Cout) + ((int64_t)kpart * M + m0) * N * OUT_B, cbytes);
      __amdgpu_buffer_rsrc_t rl = rc;
      if constexpr (SPLIT && EPI != kEpiF32)
        rl = panel(Clo + (int64_t)m0 * N, (int64_t)(M - m0) * N * 2);
      if constexpr (EPI == kEpiAddLn) {
        // x = LN(x + acc + bias) over whole rows (BN == N, n0 = 0). Row statistics: a lane's
        // 4 FN values -> the 4 lane groups (shuffles) -> the WAVES_N waves of a row band (LDS
        // tables, one barrier each); two passes, mean then centred squares, as add_ln_kernel.
        // Every wave runs the same epilogues, so the extra barriers pair up across the
        // workgroup like the main loop's.
        const int g = lane >> 4;
        float* red = bias_l + 3 * BN;                      // [2][WAVES_N][BM]
        const float* gam = bias_l + BN;
        const float* bet = bias_l + 2 * BN;
        const __amdgpu_buffer_rsrc_t rh = panel(ln.xh + (int64_t)m0 * N, (int64_t)(M - m0) * N * 2);
        // Addressing: a per-lane byte offset per fragment row i (the row must sit in the
        // voffset: the buffer range check that drops rows past M ignores soffset) plus a
        // wave-uniform soffset per fragment column j — per-fragment lane offsets would be
        // hoisted out of the tile loop by the compiler and spilled (96 accumulators live).
        auto vf = [&](int i) { return ((wr * WTM + i * 16 + (lane & 15)) * N + 4 * g) * 4; };
        auto sf = [&](int j) { return (wc * WTN + j * 16) * 4; };
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const floatx4 bj = *reinterpret_cast<const floatx4*>(bias_l + wc * WTN + j * 16 + 4 * g);
#pragma unroll
          for (int i = 0; i < FM; ++i) {   // rows past M read as zeros (bounded panel)
            const u32x4 xr = __builtin_amdgcn_raw_buffer_load_b128(rc, vf(i), sf(j), 0);
            acc[i][j] += bj + __builtin_bit_cast(floatx4, xr);
          }
        }
        float mu[FM], rsd[FM];
#pragma unroll
        for (int i = 0; i < FM; ++i) mu[i] = rsd[i] = 0.f;
#pragma unroll
        for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
          for (int i = 0; i < FM; ++i) {
            float s = 0.f;
#pragma unroll
            for (int j = 0; j < FN; ++j)
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float d = acc[i][j][r] - mu[i];
                s = pass ? fmaf(d, d, s) : s + d;
              }
            s += __shfl_xor(s, 16, 64);
            s += __shfl_xor(s, 32, 64);
            if (g == 0) red[(pass * CFG::WAVES_N + wc) * BM + wr * WTM + i * 16 + lane] = s;
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_s_barrier();
          asm volatile("" ::: "memory");
#pragma unroll
          for (int i = 0; i < FM; ++i) {
            const int row = wr * WTM + i * 16 + (lane & 15);
            float s = 0.f;
#pragma unroll
            for (int w = 0; w < CFG::WAVES_N; ++w) s += red[(pass * CFG::WAVES_N + w) * BM + row];
            if (pass == 0) mu[i] = s * (1.0f / BN);
            else rsd[i] = rsqrtf(s * (1.0f / BN) + ln.eps);
          }
        }
        // fp16 copy [+ lo plane]: 8-B stores straight from the fragment layout. (Paired 16-B
        // stores issue fewer stores than the 8-B count S; with S unchanged the next tile's
        // first ring stage was read before it landed: wrong dwords — round 2.)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const floatx4 gj = *reinterpret_cast<const floatx4*>(gam + wc * WTN + j * 16 + 4 * g);
          const floatx4 ej = *reinterpret_cast<const floatx4*>(bet + wc * WTN + j * 16 + 4 * g);
#pragma unroll
          for (int i = 0; i < FM; ++i) {
            floatx4 v;
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = (acc[i][j][r] - mu[i]) * rsd[i] * gj[r] + ej[r];
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rc, vf(i),
                                                   sf(j), 0);
            half4 h, l;
#pragma unroll
            for (int r = 0; r < 4; r += 2) {
              if constexpr (SPLIT) {
                half2 h2, l2;
                split16x2(v[r], v[r + 1], h2, l2);
                h[r] = h2[0]; h[r + 1] = h2[1]; l[r] = l2[0]; l[r + 1] = l2[1];
              } else {
                h[r] = (_Float16)v[r];
                h[r + 1] = (_Float16)v[r + 1];
              }
            }
            const int vh = vf(i) / 2;                  // same element offsets in fp16
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, h), rh, vh,
                                                  sf(j) / 2, 0);
            if constexpr (SPLIT)
              __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, l), rl, vh,
                                                    sf(j) / 2, 0);
          }
        }
      } else {
        pipe_plain_epilogue<EPI, SPLIT, CFG, false>(
            acc, kpart ? bias_l + CFG::BIAS / 2 : bias_l, rc, rl, N, n0, wr, wc, lane);
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
  }
}

// ----------------------------------------------------------------------------------------
// GEMM, loader-specialised pipe (gemm_ws_kernel; round 2): gemm_pipe_kernel's tiles and ring
// with the DMAs moved to 4 loader waves (one per SIMD), beside the 8 MFMA waves.
// Probes of gemm_pipe_kernel at 117K x 1152 x 384 fp16x3 (rag_bert_gemm variants 13-15):
// MFMAs + LDS reads + barriers 0.206 ms, DMAs alone 0.163 ms (~28 B/clk/CU of LDS-DMA intake),
// both 0.260 ms, + the epilogue stores 0.373 ms — the parts add instead of overlapping. Two
// couplings cause it: an LDS-DMA issue holds its wave for ~60-185 cycles (MI355X_MICROARCH
// price list), so the 6 DMAs every wave issued per step stalled the MFMA issue of both waves of
// a SIMD together (they leave the barrier in lockstep); and loads and stores share one
// in-order vmcnt, so a tile's stores had to complete before the next-but-one ring wait passed.
// Here the loader waves issue every DMA and wait only for DMAs (exact counts, no stores), and
// the MFMA waves issue only LDS reads, MFMAs and the epilogue's stores and never wait on
// vmcnt. One s_barrier per K step is the hand-off: the loaders pass it once stage g has
// landed, the MFMA waves once they are done reading stage g-1 (whose slot the loaders refill
// right after it). 12 waves: 3 per SIMD, <= 168 VGPRs each (the MFMA path needs ~145).
// ----------------------------------------------------------------------------------------
// block size of a gemm_ws_kernel instance: the MFMA waves plus one wave per loader
// (launch_fixed; its __launch_bounds__)
template <typename CFG> constexpr int kWsBlock = CFG::THREADS + 64 * CFG::LOADERS;

// PROBE (diagnostic timing probes of the forward's large-batch GEMM, rag_bert_gemm variants
// RAG_GEMM_WS_NO_STORE / _MFMA_ONLY / _DMA_ONLY; results meaningless): 6 = the epilogue without
// its stores, 7 = no DMAs and no stores (MFMAs, LDS reads and barriers only), 8 = no MFMAs and
// no stores (the DMA ring alone). The other round 2-4 probes and A/B forms of this kernel are
// gone (round 5); their measurements are in DESIGN.md.
template <int EPI, bool SPLIT, typename CFG, int PROBE = 0, int AUX = 0>
__global__ __launch_bounds__(kWsBlock<CFG>, 1) void gemm_ws_kernel(
    const _Float16* __restrict__ A, const _Float16* __restrict__ Al,
    const _Float16* __restrict__ W, const _Float16* __restrict__ Wl,
    const float* __restrict__ bias, int M, int N, int K, void* __restrict__ Cout,
    _Float16* __restrict__ Clo, DlArgs dl) {
  static_assert(EPI != kEpiAddLn && CFG::PRELOAD, "plain / deferred-LN epilogues, large tiles");
  static_assert(PROBE == 0 || PROBE == 6 || PROBE == 7 || PROBE == 8, "probe");
  constexpr bool DL = EPI == kEpiLnF16 || EPI == kEpiLnGeluF16 || EPI == kEpiResLn;
  static_assert(!DL || SPLIT, "deferred LayerNorm: fp16x3 only");
  constexpr int BM = CFG::BM, BN = CFG::BN, NS = CFG::NS, TH = CFG::THREADS;
  constexpr int LTH = 64 * CFG::LOADERS;            // loader threads
  constexpr int FM = CFG::FM, FN = CFG::FN, WTM = 16 * FM, WTN = 16 * FN;
  constexpr int BK = CFG::BK ? CFG::BK : kBK<SPLIT>, CPR = BK / 8, KSN = BK / 32;
  constexpr int NPL = SPLIT ? 2 : 1;
  constexpr int A_H8 = BM * CPR, W_H8 = BN * CPR;
  constexpr int STAGE_H8 = NPL * (A_H8 + W_H8);
  constexpr int LA = A_H8 / LTH, LW = W_H8 / LTH;  // DMAs per loader wave per plane
  constexpr int L = NPL * (LA + LW);               // DMAs per loader wave per stage
  constexpr bool P_NO_MFMA = PROBE == 8;
  constexpr bool P_NO_DMA = PROBE == 7;
  constexpr bool P_NO_STORE = PROBE == 6 || PROBE == 7 || PROBE == 8;
  constexpr int OUT_B = EPI == kEpiF32 ? 4 : 2;
  static_assert(A_H8 % LTH == 0 && W_H8 % LTH == 0 && FN % 2 == 0, "tile shape");
  static_assert((NS - 2) * (L + 1) <= 63, "vmcnt range");
  __shared__ half8 lds[NS * STAGE_H8 + kPipeBiasMax / 4];
  float* bias_l = reinterpret_cast<float*>(lds + NS * STAGE_H8);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t lbase = lds_addr_of(lds);
  const int nN = N / BN, nM = (M + BM - 1) / BM;
  const int nk = K / BK;
  // Panel-aligned XCD placement (from 64 row panels up): workgroups b and b + 8 share an XCD
  // (round-robin dealing), so XCD x = b & 7 owns the A row panels x, x + 8, x + 16, ... and its
  // G / 8 workgroups walk those panels' tiles n-fastest with the K steps in the same order:
  // every n-tile of a panel runs on one XCD at about the same time and takes each K slice from
  // its L2 while the first reader's fetch is still there. FETCH_SIZE at 117K tokens fp16x3, per
  // algorithmic byte, QKV / FFN1 / O / FFN2: 2.15 / 2.94 / 1.46 / 1.25 with 32 consecutive
  // tiles per XCD (panels straddling two XCDs) and the rotated K order, 1.55 / 1.76 / 1.19 /
  // 1.22 aligned (time unchanged: the DMA intake per CU, not HBM, bounds these). Below 64
  // panels the XCDs' panel counts differ by up to 1/8, so the tiles are dealt evenly instead
  // (32 consecutive per XCD per round, rotated K order: 14.8K tokens 0.190 vs 0.244 ms).
  const int G = gridDim.x, per_xcd = G >> 3;    // G: a multiple of 8 (launcher)
  const int xcd = blockIdx.x & 7, lx = blockIdx.x >> 3;
  const bool aligned = nM >= 64;
  const int t_x = aligned ? (nM > xcd ? (nM - xcd + 7) >> 3 : 0) * nN : nM * nN;
  const int l0 = aligned ? lx : xcd * per_xcd + lx, stride = aligned ? per_xcd : G;
  // Split last round (aligned mode): when the XCD's last round of tiles would leave more
  // than half of its workgroups idle (r_x <= stride / 2 tiles), each of those r_x tiles runs
  // as two 128-row halves on two workgroups, so the round ends after a half tile instead of a
  // full one. A half tile keeps the 256-row ring image (rows past its 128 read as zeros
  // through the A panel's extent, so no bytes move for them); the MFMA waves of the upper
  // rows skip their MFMAs and stores (round 2: one layer at 117K tokens 1.252 / 1.247 vs
  // 1.263 / 1.273 ms without).
  const int r_x = aligned ? t_x % stride : 0;
  const bool halves = aligned && r_x > 0 && 2 * r_x <= stride;
  const int n_full = halves ? t_x / stride : l0 < t_x ? (t_x - l0 + stride - 1) / stride : 0;
  const int n_mine = n_full + (halves && lx < 2 * r_x ? 1 : 0);
  const int steps = n_mine * nk;
  // tile `it`: rows [m0, m_end) (m_end <= M) and n-tile nt
  auto tile_mn = [&](int it, int& m0, int& nt, int& m_end) __attribute__((always_inline)) {
    if (it < n_full) {
      const int t = it * stride + l0;
      m0 = (aligned ? xcd + 8 * (t / nN) : t / nN) * BM;
      nt = t % nN;
      m_end = min(M, m0 + BM);
    } else {                                  // the half tile of the split last round
      const int t = n_full * stride + (lx >> 1);
      m0 = (xcd + 8 * (t / nN)) * BM + (lx & 1) * (BM / 2);
      nt = t % nN;
      m_end = min(M, m0 + BM / 2);
    }
  };

  for (int i = tid * 4; i < N; i += (TH + LTH) * 4) {
    *reinterpret_cast<floatx4*>(bias_l + i) = *reinterpret_cast<const floatx4*>(bias + i);
    if constexpr (EPI == kEpiLnF16 || EPI == kEpiLnGeluF16)
      *reinterpret_cast<floatx4*>(bias_l + N + i) = *reinterpret_cast<const floatx4*>(dl.c1 + i);
    if constexpr (EPI == kEpiResLn)
      if (dl.st_in) {
        *reinterpret_cast<floatx4*>(bias_l + N + i) = *reinterpret_cast<const floatx4*>(dl.gamma + i);
        *reinterpret_cast<floatx4*>(bias_l + 2 * N + i) = *reinterpret_cast<const floatx4*>(dl.beta + i);
      }
  }
  __syncthreads();

  if (wid >= TH / 64) {
    // ---- loader waves: stage g+NS-1 issued after the barrier of step g ----
    const int lw = wid - TH / 64;
    uint32_t voA[LA], voW[LW];
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int q = (lw * LA + i) * 64 + lane, r = q / CPR, cs = q % CPR;
      voA[i] = (uint32_t)(r * K + swz_chunk<CPR>(r, cs) * 8) * 2u;
    }
#pragma unroll
    for (int i = 0; i < LW; ++i) {
      const int q = (lw * LW + i) * 64 + lane, r = q / CPR, cs = q % CPR;
      voW[i] = (uint32_t)(r * K + swz_chunk<CPR>(r, cs) * 8) * 2u;
    }
    int it_i = 0, kt_i = 0, kr_i = 0, slot_i = 0;
    __amdgpu_buffer_rsrc_t rA0 = panel(A, 0), rA1 = rA0, rW0 = rA0, rW1 = rA0;
    auto issue_next = [&]() __attribute__((always_inline)) {
      if (it_i >= n_mine) return;
      if constexpr (P_NO_DMA) {
        if (++kt_i == nk) { kt_i = 0; ++it_i; }
        return;
      }
      if (kt_i == 0) {
        int m0, nt, m_end;
        tile_mn(it_i, m0, nt, m_end);
        const int n0 = nt * BN;
        kr_i = aligned ? 0 : nt % nk;   // rotated K order unless aligned
        const int64_t abytes = (int64_t)(m_end - m0) * K * 2, wbytes = (int64_t)BN * K * 2;
        rA0 = panel(A + (int64_t)m0 * K, abytes);
        rW0 = panel(W + (int64_t)n0 * K, wbytes);
        if constexpr (SPLIT) {
          rA1 = panel(Al + (int64_t)m0 * K, abytes);
          rW1 = panel(Wl + (int64_t)n0 * K, wbytes);
        }
      }
      const uint32_t soff = __builtin_amdgcn_readfirstlane((uint32_t)kr_i * (BK * 2));
      if (++kr_i == nk) kr_i = 0;
      const uint32_t slot = lbase + (uint32_t)slot_i * (STAGE_H8 * 16);
#pragma unroll
      for (int i = 0; i < LA; ++i) {
        const uint32_t d = slot + (uint32_t)((lw * LA + i) * 64 * 16);
        blds16(rA0, voA[i], soff, d);
        if constexpr (SPLIT) blds16(rA1, voA[i], soff, d + A_H8 * 16);
      }
#pragma unroll
      for (int i = 0; i < LW; ++i) {
        const uint32_t d = slot + (uint32_t)((NPL * A_H8 + (lw * LW + i) * 64) * 16);
        blds16(rW0, voW[i], soff, d);
        if constexpr (SPLIT) blds16(rW1, voW[i], soff, d + W_H8 * 16);
      }
      if (++kt_i == nk) { kt_i = 0; ++it_i; }
      if (++slot_i == NS) slot_i = 0;
    };
#pragma unroll
    for (int p = 0; p < NS - 1; ++p) issue_next();
    for (int g = 0; g < steps; ++g) {
      wait_ring<L, 0, NS - 2>(min(NS - 2, steps - 1 - g), false);   // stage g landed
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      issue_next();                     // stage g+NS-1 -> slot (g-1) % NS
    }
    return;
  }

  // ---- MFMA waves ----
  const int wr = wid / CFG::WAVES_N, wc = wid % CFG::WAVES_N;
  // (round 6 A/B builds, removed: static s_setprio 1 on MFMA waves 4-7, and s_setprio 1
  // around each step's MFMA chain — rerank forward 9.01-9.06 / 9.00-9.07 vs 8.98-9.04 ms,
  // chunk encode 3.16-3.17 / 3.16-3.18 vs 3.15-3.18: neutral; profiles/r06_ws_prio/. A
  // stagger — the odd workgroups owning a half tile ran it first, so their epilogue bursts
  // alternated with the others' MFMA phases — gave bitwise the same forward but 9.06-9.11 vs
  // 8.91-8.97 ms, chunk encode unchanged: a panel's n-tiles no longer ran on one XCD at the
  // same time to share its A slices in L2; profiles/r06_ws_stagger/)
  floatx4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  int kt_c = 0, it_c = 0, slot_c = 0;
  half8 af[KSN][NPL][FM], wf[KSN][NPL][FN];
  // deferred LN: the current tile's row statistics, loaded right after the previous tile's
  // epilogue (a whole tile before they are used; loaded at the tile's first K step instead, the
  // compiler's waitcnt model put a vmcnt(0) there — a wait for the previous tile's stores)
  floatx4 dls[FM];
  auto prefetch = [&](int it) __attribute__((always_inline)) {
    if constexpr (DL) {
      if (dl.st_in && it < n_mine) {
        int m0, nt, m_end;
        tile_mn(it, m0, nt, m_end);
        const __amdgpu_buffer_rsrc_t rsi =
            panel(dl.st_in + (int64_t)m0 * kDlParts * 2, (int64_t)(m_end - m0) * kDlParts * 8);
        dl_prefetch_stats<FM>(dls, rsi, wr, lane);
      }
    }
  };
  prefetch(0);
  for (int g = 0; g < steps; ++g) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // done reading stage g-1
    __builtin_amdgcn_s_barrier();                        // stage g landed
    asm volatile("" ::: "memory");
    const half8* sa = lds + slot_c * STAGE_H8;
    const half8* sw = sa + NPL * A_H8;
    auto read_a = [&](int i) __attribute__((always_inline)) {
#pragma unroll
      for (int ks = 0; ks < KSN; ++ks)
#pragma unroll
        for (int p = 0; p < NPL; ++p)
          af[ks][p][i] = sa[p * A_H8 + swz<CPR>(wr * WTM + i * 16 + (lane & 15), ks * 4 + (lane >> 4))];
    };
    // the upper-row MFMA waves of a half tile (split last round) have no rows: no reads,
    // MFMAs or stores (they still keep the ring's barriers)
    const bool idle = halves && it_c == n_full && wr >= CFG::WAVES_M / 2;
    if (!idle && !P_NO_MFMA) {
      // interleaved order: A_0, W_0..W_{FN-1}, A_1, ... read in the order the i-major MFMAs
      // consume them, with no barrier between the reads and the MFMAs, so the first MFMA
      // waits for 4 reads instead of 13 (all 8 waves issue their reads together after the
      // barrier; the LDS serves them interleaved). Round 2: 117K-token layer fp16x3 1.274 ->
      // 1.264 ms against all reads first (profiles/r02e_gemm_ilv.jsonl).
      read_a(0);
#pragma unroll
      for (int j = 0; j < FN; ++j)    // W_j's planes together: MFMA (0, j) needs 2 + 2j reads
#pragma unroll
        for (int ks = 0; ks < KSN; ++ks)
#pragma unroll
          for (int p = 0; p < NPL; ++p)
            wf[ks][p][j] = sw[p * W_H8 + swz<CPR>(wc * WTN + j * 16 + (lane & 15), ks * 4 + (lane >> 4))];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        if (i + 1 < FM) read_a(i + 1);
#pragma unroll
        for (int ks = 0; ks < KSN; ++ks)
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            if constexpr (SPLIT) {   // small terms first: W_lo A_hi + W_hi A_lo + W_hi A_hi
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[ks][1][j], af[ks][0][i], acc[i][j], 0, 0, 0);
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[ks][0][j], af[ks][1][i], acc[i][j], 0, 0, 0);
            }
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[ks][0][j], af[ks][0][i], acc[i][j], 0, 0, 0);
          }
      }
    }
    if (++slot_c == NS) slot_c = 0;
    if (++kt_c == nk) {               // tile done (stores never waited on)
      kt_c = 0;
      int m0, nt, m_end;
      tile_mn(it_c, m0, nt, m_end);
      ++it_c;
      const int n0 = nt * BN;
      const __amdgpu_buffer_rsrc_t rc = panel(static_cast<char*>(Cout) + (int64_t)m0 * N * OUT_B,
                                              (int64_t)(m_end - m0) * N * OUT_B);
      __amdgpu_buffer_rsrc_t rl = rc;
      if constexpr (SPLIT && EPI != kEpiF32)
        rl = panel(Clo + (int64_t)m0 * N, (int64_t)(m_end - m0) * N * 2);
      if (idle) {
        // no rows of this wave in the half tile
      } else if constexpr (DL) {
        const int64_t sb = (int64_t)(m_end - m0) * kDlParts * 8;
        const __amdgpu_buffer_rsrc_t rso = panel(dl.st_out + (int64_t)m0 * kDlParts * 2, dl.st_out ? sb : 0);
        ws_dl_epilogue<EPI, CFG, AUX>(acc, bias_l, rc, rl, dls, rso, dl.st_in != nullptr, N, n0,
                                      wr, wc, lane, dl.eps);
      } else {
        pipe_plain_epilogue<EPI, SPLIT, CFG, P_NO_STORE, AUX>(acc, bias_l, rc, rl, N, n0, wr, wc,
                                                              lane);
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
      prefetch(it_c);
    }
  }
}

#ifdef RAGMI_DIAG_BUILD
// ----------------------------------------------------------------------------------------
// Fused FFN of the deferred-LayerNorm forward (round 6): one launch for
//   H  = GELU(LN1(z) W1^T + b1)        (FFN1, kEpiLnGeluF16 with LN1 folded: W1' = W1 diag(g1))
//   z' = LN1(z) + (H W2^T + b2)        (FFN2, kEpiResLn; row statistics of z' out)
// (modeling_bert.py BertIntermediate + BertOutput) over 128-row tiles of the token rows,
// with the 1536-wide intermediate H never leaving the CU: per tile, for each 128-column chunk
// c of H, (1) 12 K-steps of z x W1'[c]^T into H_c (128 x 128 accumulators), (2) the LnGelu
// epilogue in registers, split into fp16 hi + lo, re-laid lane to lane into MFMA operand
// fragments (v_permlane32/16_swap, no LDS), (3) 4 K-steps of H_c x W2[:, c]^T accumulated into
// the tile's 128 x 384 output; after the 12 chunks, the ResLn epilogue writes z' in place.
// The two-kernel path writes H (T x 1536, hi + lo: 725 MB at 118K tokens) to HBM and reads it
// back (1.19x, FFN2's A streamed from HBM); its FFN1 epilogue's store bursts stall the MFMA
// waves. Arithmetic: every output element is computed by the same MFMA sequence
// (K steps in natural order, the three fp16x3 terms W_lo A_hi, W_hi A_lo, W_hi A_hi), the same
// epilogue operations and the same operand-to-lane mapping as gemm_ws_kernel's FFN1 / FFN2 at
// aligned (>= 64 row panels) token counts, so the forward's outputs are bitwise those of the
// two-kernel path there (tests/test_ffn_fused_gpu.py).
// MEASURED SLOWER: 1.08 ms per launch against 0.90 ms for the two WS GEMMs at
// 118K tokens (rerank forward 9.2-9.9 vs 8.9-9.1 ms over five shapes), MFMA busy 0.35, waves
// waiting 43% — so it is compiled into the diagnostic build only (-DRAGMI_DIAG_BUILD).
// Layout: 8 waves, wave w owns rows 16w .. 16w+15 of the tile and ALL columns (H_c: 8 16x16
// fragments = 32 VGPRs; the output: 24 fragments = 96), so a wave's H_c rows are exactly the
// A operand rows its phase (3) needs. The waves issue their own LDS-DMA (no loader waves: the
// register budget needs two waves per SIMD); a 3-slot ring of 48 KB stages (phase 1: z hi/lo
// 128 rows x 32 K + W1'[c] hi/lo 128 rows x 32 K = 32 KB; phase 3: W2[:, c] hi/lo 384 rows x
// 32 K = 48 KB), one barrier per K step; c1 | c2 (LN1 fold vectors) staged in LDS.
// ----------------------------------------------------------------------------------------
constexpr int kFfnBM = 128, kFfnFF = 1536;
constexpr int kFfnWaves = 8, kFfnThreads = 64 * kFfnWaves;
constexpr int kFfnS1 = kDlH / 32;                       // phase-1 K steps per chunk (12)
// timing probes of a diagnostic build (-DRAGMI_FFN_PROBE=n; results meaningless): 1 no MFMAs,
// 2 no DMAs, 3 no W fragment LDS reads (A fragments stand in), 4 no LnGelu epilogue math
#ifndef RAGMI_FFN_PROBE
#define RAGMI_FFN_PROBE 0
#endif
constexpr int kFfnProbe = RAGMI_FFN_PROBE;

// chunk width CH of the intermediate per pass (V): 0 -> 128 (12 chunks; a phase-1 stage is
// 32 KB in a 48 KB slot), 1 -> 256 (6 chunks: every stage 48 KB, half the z re-reads, 24 MFMAs
// -> 48 per wave in a phase-1 K step). A 3-slot ring of 48 KB slots either way.
template <int V> struct FfnRing {
  static constexpr int CH = (V & 1) ? 256 : 128;
  static constexpr bool LATE_DMA = (V & 2) != 0;          // next stage issued mid-step
  static constexpr bool PRIO = (V & 4) != 0;              // s_setprio 1 on waves 4-7
  static constexpr int CHUNKS = kFfnFF / CH;
  static constexpr int S3 = CH / 32;                      // phase-3 K steps per chunk
  static constexpr int PER_CHUNK = kFfnS1 + S3;
  static constexpr int PER_TILE = CHUNKS * PER_CHUNK;
  static constexpr int SLOTS = 3, SLOT_H8 = 3072;         // 48 KB in 16-B units
  static constexpr int P1 = (kFfnBM + CH) * 2 / 16 / kFfnWaves;  // phase-1 pieces per wave
  static constexpr int P3 = 6;                            // phase-3 pieces per wave
  static constexpr int FN1 = CH / 16;                     // H_c fragments per wave
  static constexpr int AHEAD = SLOTS - 1;
};

struct FfnArgs {
  const _Float16 *w1, *w1l;     // W1' = W1 diag(g_prev) [1536][384] (folded), hi / lo
  const float *c1, *c2;         // [1536]: column sums of W1' and b1 + W1 beta_prev
  const _Float16 *w2, *w2l;     // [384][1536]
  const float *b2, *gamma, *beta;   // FFN2 bias; the LayerNorm pending on z (LN1)
  const float* st_in;           // [M][6] x {mean, M2} of z (the attention block's ResLn)
  float* st_out;                // [M][6] of z'
  float eps;
};

// lane-to-lane re-lay of two adjacent 16-column accumulator fragments (f0 = columns 0..15, f1
// = 16..31 of a 32-deep K step; lane group g holds columns 4g..4g+3 of each, one dword per two
// fp16) into the MFMA A-operand fragment of that K step (lane group g: columns 8g .. 8g+7):
// permlane32_swap then permlane16_swap (derivation in DESIGN §R6.1)
__device__ __forceinline__ half8 ffn_relay(u32x2 f0, u32x2 f1) {
  u32x4 o;
#pragma unroll
  for (int d = 0; d < 2; ++d) {
    const auto x = __builtin_amdgcn_permlane32_swap(f0[d], f1[d], false, false);
    const auto y = __builtin_amdgcn_permlane16_swap(x[0], x[1], false, false);
    o[d] = y[0];         // columns 8g + 2d, +1
    o[2 + d] = y[1];     // columns 8g + 4 + 2d, +1
  }
  return __builtin_bit_cast(half8, o);
}

// s_waitcnt vmcnt(n) for a runtime n in [0, N] (the immediate is compile-time)
template <int N>
__device__ __forceinline__ void wait_vm(int n) {
  if (n >= N) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
    return;
  }
  if constexpr (N > 0) wait_vm<N - 1>(n);
}

template <int V = 0>
__global__ __launch_bounds__(kFfnThreads, 1) void ffn_fused_kernel(
    _Float16* __restrict__ zh, _Float16* __restrict__ zl, int M, FfnArgs a) {
  using R = FfnRing<V>;
  constexpr int H = kDlH, FF = kFfnFF, CPR = 4, CH = R::CH;
  constexpr int A_H8 = kFfnBM * CPR;                    // 512: one plane of a 128-row stage
  constexpr int W1_H8 = CH * CPR;                       // one plane of W1'[c] in a stage
  constexpr int W3_H8 = H * CPR;                        // one plane of a phase-3 stage
  __shared__ half8 lds[R::SLOTS * R::SLOT_H8];
  __shared__ float cvec[2 * FF];                        // c1 | c2
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t lbase = lds_addr_of(lds);
  const int nT = (M + kFfnBM - 1) / kFfnBM;
  const int G = gridDim.x, b = blockIdx.x;
  const int n_mine = b < nT ? (nT - b + G - 1) / G : 0;
  const int steps = n_mine * R::PER_TILE;

  for (int i = tid * 4; i < FF; i += kFfnThreads * 4) {
    *reinterpret_cast<floatx4*>(cvec + i) = *reinterpret_cast<const floatx4*>(a.c1 + i);
    *reinterpret_cast<floatx4*>(cvec + FF + i) = *reinterpret_cast<const floatx4*>(a.c2 + i);
  }

  // ---- this wave's share of each stage's DMA pieces (1 KB = 64 lanes x 16 B) ----
  // phase 1: the stage's pieces in image order — z hi (8), z lo (8), W1'[c] hi (CH / 16),
  // W1'[c] lo — wave w takes pieces P1 w .. P1 w + P1 - 1; every operand row is 384 K long, so
  // a piece's lane offsets depend only on its index inside its region
  uint32_t vo1[R::P1], vo3[R::P3];
  int reg1[R::P1];
#pragma unroll
  for (int i = 0; i < R::P1; ++i) {
    const int p = R::P1 * w + i;
    const int region = p < 8 ? 0 : p < 16 ? 1 : p < 16 + CH / 16 ? 2 : 3;
    const int q = region < 2 ? p - 8 * region : p - 16 - (region - 2) * (CH / 16);
    const int r = q * 16 + (lane >> 2), cs = lane & 3;
    reg1[i] = region;
    vo1[i] = (uint32_t)(r * H + swz_chunk<CPR>(r, cs) * 8) * 2u;
  }
  // phase 3: region w / 4 (0 W2 hi, 1 W2 lo), pieces (w & 3) * P3 + i of the stage's rows
#pragma unroll
  for (int i = 0; i < R::P3; ++i) {
    const int q = (w & 3) * R::P3 + i, r = q * 16 + (lane >> 2), cs = lane & 3;
    vo3[i] = (uint32_t)(r * FF + swz_chunk<CPR>(r, cs) * 8) * 2u;
  }
  const __amdgpu_buffer_rsrc_t rW2 = panel((w >> 2) ? a.w2l : a.w2, (int64_t)H * FF * 2);
  // stage gi of this workgroup's sequence -> slot gi % SLOTS
  auto issue = [&](int gi) __attribute__((always_inline)) {
    if (gi >= steps || kFfnProbe == 2) return;
    const int it = gi / R::PER_TILE, loc = gi % R::PER_TILE;
    const int c = loc / R::PER_CHUNK, s = loc % R::PER_CHUNK;
    const uint32_t slot = lbase + (uint32_t)(gi % R::SLOTS) * (R::SLOT_H8 * 16);
    if (s < kFfnS1) {
      const int m0 = (it * G + b) * kFfnBM, rows = min(M - m0, kFfnBM);
      const __amdgpu_buffer_rsrc_t rz0 = panel(zh + (int64_t)m0 * H, (int64_t)rows * H * 2);
      const __amdgpu_buffer_rsrc_t rz1 = panel(zl + (int64_t)m0 * H, (int64_t)rows * H * 2);
      const __amdgpu_buffer_rsrc_t rw0 = panel(a.w1 + (int64_t)c * CH * H, (int64_t)CH * H * 2);
      const __amdgpu_buffer_rsrc_t rw1 = panel(a.w1l + (int64_t)c * CH * H, (int64_t)CH * H * 2);
      const uint32_t soff = __builtin_amdgcn_readfirstlane((uint32_t)(s * 64));
#pragma unroll
      for (int i = 0; i < R::P1; ++i) {
        // (image position of piece P1 w + i: pieces are laid out in their global order)
        const uint32_t d = slot + (uint32_t)((R::P1 * w + i) * 64 * 16);
        const int rg = reg1[i];
        blds16(rg == 0 ? rz0 : rg == 1 ? rz1 : rg == 2 ? rw0 : rw1, vo1[i], soff, d);
      }
    } else {
      const int k = s - kFfnS1;
      const uint32_t soff = __builtin_amdgcn_readfirstlane((uint32_t)((c * CH + k * 32) * 2));
#pragma unroll
      for (int i = 0; i < R::P3; ++i)
        blds16(rW2, vo3[i], soff,
               slot + (uint32_t)(((w >> 2) * W3_H8 + ((w & 3) * R::P3 + i) * 64) * 16));
    }
  };
  auto pieces = [&](int gi) -> int {
    if (gi >= steps || kFfnProbe == 2) return 0;
    return (gi % R::PER_TILE) % R::PER_CHUNK < kFfnS1 ? R::P1 : R::P3;
  };

  // the tile's row statistics (one 16-row group per wave), loaded a tile ahead of use
  floatx4 dls[1];
  auto prefetch = [&](int it) __attribute__((always_inline)) {
    if (it < n_mine) {
      const int m0 = (it * G + b) * kFfnBM, rows = min(M - m0, kFfnBM);
      dl_prefetch_stats<1>(dls, panel(a.st_in + (int64_t)m0 * kDlParts * 2,
                                      (int64_t)rows * kDlParts * 8), w, lane);
    }
  };
  prefetch(0);
#pragma unroll
  for (int p = 0; p < R::AHEAD; ++p) issue(p);
  __syncthreads();                                       // cvec staged

  // one ring step: stage gi landed (this wave's pieces: everything older than the AHEAD - 1
  // stages issued after it), every wave done reading stage gi - 1 (its slot is refilled next)
  auto step_begin = [&](int gi) __attribute__((always_inline)) -> const half8* {
    int younger = 0;
#pragma unroll
    for (int p = 1; p < R::AHEAD; ++p) younger += pieces(gi + p);
    wait_vm<(R::AHEAD - 1) * 6>(younger);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if constexpr (!R::LATE_DMA) issue(gi + R::AHEAD);
    return lds + (gi % R::SLOTS) * R::SLOT_H8;
  };
  if constexpr (R::PRIO)
    if (w >= 4) __builtin_amdgcn_s_setprio(1);

  int gi = 0;
  for (int it = 0; it < n_mine; ++it) {
    floatx4 y[24];
#pragma unroll
    for (int j = 0; j < 24; ++j) y[j] = floatx4{0.f, 0.f, 0.f, 0.f};
    float mu, rs;
    dl_lane_stats(dls[0], g, a.eps, mu, rs);             // the tile's rows
    for (int c = 0; c < R::CHUNKS; ++c) {
      // ---- phase 1: H_c = z W1'[c]^T, 12 K steps ----
      floatx4 hacc[R::FN1];
#pragma unroll
      for (int j = 0; j < R::FN1; ++j) hacc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
      for (int s = 0; s < kFfnS1; ++s, ++gi) {
        const half8* sl = step_begin(gi);
        const int ar = swz<CPR>(16 * w + (lane & 15), g);
        const half8 a0 = sl[ar], a1 = sl[A_H8 + ar];
#pragma unroll
        for (int j = 0; j < R::FN1; ++j) {
          if constexpr (R::LATE_DMA)
            if (j == R::FN1 / 2) issue(gi + R::AHEAD);
          const int wrw = swz<CPR>(16 * j + (lane & 15), g);
          half8 w0, w1;
          if constexpr (kFfnProbe == 3) {
            w0 = a1;
            w1 = a0;
          } else {
            w0 = sl[2 * A_H8 + wrw];
            w1 = sl[2 * A_H8 + W1_H8 + wrw];
          }
          if constexpr (kFfnProbe == 1) {
            hacc[j][0] += (float)w0[0] + (float)w1[1];
            continue;
          }
          hacc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1, a0, hacc[j], 0, 0, 0);
          hacc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w0, a1, hacc[j], 0, 0, 0);
          hacc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w0, a0, hacc[j], 0, 0, 0);
        }
      }
      // ---- phase 2: the LnGelu epilogue of H_c in registers (ws_dl_epilogue's arithmetic)
      // -> fp16 hi / lo -> the A operand fragments of phase 3's four K steps ----
      half8 ah[R::S3], al[R::S3];
      {
        const floatx4 nm4 = {-mu, -mu, -mu, -mu}, rs4 = {rs, rs, rs, rs};
        u32x2 hh[R::FN1], hl[R::FN1];
#pragma unroll
        for (int j = 0; j < R::FN1; ++j) {
          const int nl = c * CH + 16 * j + 4 * g;
          const floatx4 c1 = *reinterpret_cast<const floatx4*>(cvec + nl);
          const floatx4 c2 = *reinterpret_cast<const floatx4*>(cvec + FF + nl);
          floatx4 v = hacc[j];
          if constexpr (kFfnProbe != 4) {
            v = __builtin_elementwise_fma(rs4, __builtin_elementwise_fma(nm4, c1, hacc[j]), c2);
            v = gelu_erf4(v);
          }
          half2 h0, l0, h1, l1;
          split16x2(v[0], v[1], h0, l0);
          split16x2(v[2], v[3], h1, l1);
          hh[j] = u32x2{__builtin_bit_cast(uint32_t, h0), __builtin_bit_cast(uint32_t, h1)};
          hl[j] = u32x2{__builtin_bit_cast(uint32_t, l0), __builtin_bit_cast(uint32_t, l1)};
        }
#pragma unroll
        for (int k = 0; k < R::S3; ++k) {
          ah[k] = ffn_relay(hh[2 * k], hh[2 * k + 1]);
          al[k] = ffn_relay(hl[2 * k], hl[2 * k + 1]);
        }
      }
      // ---- phase 3: out += H_c W2[:, c]^T, CH / 32 K steps ----
#pragma unroll
      for (int k = 0; k < R::S3; ++k, ++gi) {
        const half8* sl = step_begin(gi);
        constexpr int NJ = H / 16;
        const int j0 = 0;
#pragma unroll
        for (int jj = 0; jj < NJ; ++jj) {
          if constexpr (R::LATE_DMA)
            if (jj == NJ / 4) issue(gi + R::AHEAD);
          const int wrw = swz<CPR>(16 * jj + (lane & 15), g);
          half8 w0, w1;
          if constexpr (kFfnProbe == 3) {
            w0 = al[k];
            w1 = ah[k];
          } else {
            w0 = sl[wrw];
            w1 = sl[W3_H8 + wrw];
          }
          floatx4& yy = y[j0 + jj];
          if constexpr (kFfnProbe == 1) {
            yy[0] += (float)w0[0] + (float)w1[1];
            continue;
          }
          yy = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1, ah[k], yy, 0, 0, 0);
          yy = __builtin_amdgcn_mfma_f32_16x16x32_f16(w0, al[k], yy, 0, 0, 0);
          yy = __builtin_amdgcn_mfma_f32_16x16x32_f16(w0, ah[k], yy, 0, 0, 0);
        }
      }
    }
    // ---- the tile's ResLn epilogue (ws_dl_epilogue<kEpiResLn>'s arithmetic): x = LN1(z)
    // from the planes + statistics, z' = x + (out + b2) in place, z' row statistics ----
    const int m0 = (it * G + b) * kFfnBM, rows = min(M - m0, kFfnBM);
    const __amdgpu_buffer_rsrc_t rc = panel(zh + (int64_t)m0 * H, (int64_t)rows * H * 2);
    const __amdgpu_buffer_rsrc_t rl = panel(zl + (int64_t)m0 * H, (int64_t)rows * H * 2);
    const __amdgpu_buffer_rsrc_t rso =
        panel(a.st_out + (int64_t)m0 * kDlParts * 2, (int64_t)rows * kDlParts * 8);
    const int ml = 16 * w + (lane & 15);
    const int cofs = 8 * ((g & 1) * 2 + (g >> 1));
    const floatx4 a4 = {rs, rs, rs, rs}, b4 = {-mu * rs, -mu * rs, -mu * rs, -mu * rs};
#pragma unroll
    for (int blk = 0; blk < kDlParts; ++blk) {
      u32x2 zhv[4], zlv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int vo = (ml * H + 64 * blk + 16 * j + 4 * g) * 2;
        zhv[j] = __builtin_amdgcn_raw_buffer_load_b64(rc, vo, 0, 0);
        zlv[j] = __builtin_amdgcn_raw_buffer_load_b64(rl, vo, 0, 0);
      }
      floatx4 s4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int nl = 64 * blk + 16 * j + 4 * g;
        const floatx4 z = mix_f16x4(zhv[j], zlv[j]);
        const floatx4 bv = *reinterpret_cast<const floatx4*>(a.b2 + nl);
        const floatx4 xr = __builtin_elementwise_fma(
            __builtin_elementwise_fma(z, a4, b4), *reinterpret_cast<const floatx4*>(a.gamma + nl),
            *reinterpret_cast<const floatx4*>(a.beta + nl));
        y[4 * blk + j] = (y[4 * blk + j] + bv) + xr;
        s4 += y[4 * blk + j];
      }
      float sm = (s4[0] + s4[1]) + (s4[2] + s4[3]);
      sm += __shfl_xor(sm, 16, 64);
      sm += __shfl_xor(sm, 32, 64);
      const float mw = sm * (1.0f / 64);
      const floatx4 m4 = {mw, mw, mw, mw};
      floatx4 q4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const floatx4 d = y[4 * blk + j] - m4;
        q4 = __builtin_elementwise_fma(d, d, q4);
      }
      float q = (q4[0] + q4[1]) + (q4[2] + q4[3]);
      q += __shfl_xor(q, 16, 64);
      q += __shfl_xor(q, 32, 64);
      if (g == 0) {
        const u32x2 d = {__builtin_bit_cast(uint32_t, mw), __builtin_bit_cast(uint32_t, q)};
        __builtin_amdgcn_raw_buffer_store_b64(d, rso, (ml * kDlParts + blk) * 8, 0, 0);
      }
#pragma unroll
      for (int jp = 0; jp < 4; jp += 2) {
        const int vo = (ml * H + 64 * blk + 16 * jp + cofs) * 2;
        half4 ha, hb, la, lb;
#pragma unroll
        for (int r = 0; r < 4; r += 2) {
          half2 h2, l2;
          split16x2(y[4 * blk + jp][r], y[4 * blk + jp][r + 1], h2, l2);
          ha[r] = h2[0]; ha[r + 1] = h2[1]; la[r] = l2[0]; la[r + 1] = l2[1];
          split16x2(y[4 * blk + jp + 1][r], y[4 * blk + jp + 1][r + 1], h2, l2);
          hb[r] = h2[0]; hb[r + 1] = h2[1]; lb[r] = l2[0]; lb[r + 1] = l2[1];
        }
        store_f16_pair<0>(ha, hb, rc, vo);
        store_f16_pair<0>(la, lb, rl, vo);
      }
    }
    // this tile's stores and the DMAs in flight drained before the next tile's first ring
    // wait (its vmcnt counts assume no stores in between), then the next tile's statistics
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    prefetch(it + 1);
  }
}

#endif  // RAGMI_DIAG_BUILD

// ----------------------------------------------------------------------------------------
// attention (varlen, one workgroup per (head, sequence), 8 waves (fp16) / 16 (fp16x3)).
// K and V of the sequence's keys are staged into LDS (all of them when they fit — always for
// head_dim 32, and for head_dim 64 up to ~288 keys in fp16x3 — else in chunks of kc keys),
// then every wave walks its own 16-query blocks over all key blocks of 32 with no further
// barriers.
// Transposed formulation keeps P in registers:
//   S^T[key][q] = K . Q^T   (A = K rows from LDS, B = Q^T fragments held for the block)
//   O^T[d][q]  += V^T . P^T (A = V^T rows from LDS, B = P^T = the lane's own S^T values)
// The MFMA C layout puts query q = lane&15 in every lane's column, so the softmax running
// max / sum and the O rescale are per-lane scalars; the P^T fragment slot 8g+j (g = lane>>4)
// holds key 4g+j (j<4) or 16+4g+(j-4) (j>=4) of the block, i.e. exactly the lane's two S^T
// accumulators. V stays row-major in LDS ([key][HD], 16-B copies from the Q|K|V rows) and
// the V^T fragment is gathered by two ds_read_b64_tr_b16 (gfx950 transposed LDS read: per
// 16-lane group, 4 rows x 16 columns delivered column-major): rows 4g..4g+3 and 16+4g..
// 16+4g+3 of the block — the P^T slot order, so no key permutation is stored anywhere.
// (Round 1 staged V^T with eight 2-byte LDS stores per 16-B chunk: SQ_LDS_BANK_CONFLICT
// 1.9e7 cycles per launch against 1.24e7 active LDS cycles at rerank size.)
// qkv: fp16 [T][3H] (Q | K | V; head h = columns h*HD .. +HD-1 of each); ctx: fp16 [T][H].
// LDS (dynamic) per plane: K [cap][HD] (16-B chunks swizzled as the GEMM images, swz_chunk)
// + V [cap][HD] (16-B chunk c of row r at c ^ attn_vsw(r), which spreads the 8 rows a 32-lane
// half reads over all 64 banks), cap = keys staged at once. Two fp16x3 workgroups share a CU
// up to ~300 keys.
// ----------------------------------------------------------------------------------------
template <bool SPLIT> constexpr int kAttnThreads = 512;   // 2 waves per SIMD per workgroup
constexpr int kAttnLdsMax = 160 * 1024;
// occupancy: head_dim 32 fp16 fits 64 VGPRs (8 waves per SIMD: four 8-wave workgroups per
// CU, LDS permitting) without spilling; head_dim 32 fp16x3 fits 128 (two workgroups per CU,
// so one stages its K/V while the other computes: rerank 10.33 -> 10.08 ms against 16-wave
// workgroups, one per CU); head_dim 64 is left unconstrained
template <int HD, bool SPLIT> constexpr int kAttnWavesPerEU = HD == 32 ? (SPLIT ? 4 : 8) : 1;

template <int HD>
__host__ __device__ constexpr int attn_lds_bytes(int cap, int planes) {
  return planes * 2 * cap * HD * 2;
}
// keys staged per chunk (multiple of 32): all of them if they fit, else the most that fit
template <int HD>
__host__ __device__ constexpr int attn_chunk_keys(int max_len, int planes) {
  const int sp = (max_len + 31) & ~31;
  int kc = sp;
  while (kc > 32 && attn_lds_bytes<HD>(kc, planes) > kAttnLdsMax) kc -= 32;
  return kc;
}

// V image chunk swizzle: a transposed read takes 32 B (16 columns) of each of 8 rows per
// 32-lane half (rows 4g + q, g = two groups); rows 128 / HD apart share a bank window, so the
// chunk pair is XORed by the row's window index
template <int HD>
__device__ __forceinline__ int attn_vsw(int r) {
  return ((r / (128 / HD)) & (HD / 16 - 1)) << 1;
}

typedef short short4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ half4 lds_read_tr16(const _Float16* p) {
  return __builtin_bit_cast(half4, __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) short4v*)(p)));
}

template <int HD, bool SPLIT>
struct AttnState {
  static constexpr int DT = HD / 16, KS = HD / 32, NP = SPLIT ? 2 : 1;
  half8 qf[KS][NP];
  floatx4 o[DT];
  // row sums of P: fp16x3 by MFMA against a ones fragment (every element = l(q)); fp16 by
  // v_dot2 into l[0] (lane-partial, reduced across the lane groups at the end)
  floatx4 l;
  float m;
};

// VAR bit 512 (round 6, diagnostic build): the P scalings as scalar v_fma_f32 (fma_scalar)
// instead of the packed v_pk_fma_f32 of VPRE; bitwise the same values, measured neutral at the
// rerank shape (554: 0.2427-0.2436 ms vs 42: 0.2414-0.2428, profiles/r06_attn/): the loop is
// not bound by its vector issue.
// VAR (bit mask; rag_bert_attention A/Bs them): 1 = rolling Q prefetch, 2 = fp16x3 row sums
// by MFMA (else v_dot2), 4 = software-pipelined scores (block kb+1's K.Q^T MFMAs issued
// before block kb's softmax, so they run in the matrix pipe under its vector work), 8 = lean
// block (round 2): the block max by IEEE maximum (fmax_nc: no canonicalising v_max per MFMA
// result), the cross-lane max by v_permlane16/32_swap instead of two ds_bpermute
// round trips, P and O split by split16x2 (3 instead of 8 VALU per pair), and a block's V^T
// fragments read in one batch before its P.V MFMAs (one LDS wait instead of DT). Bitwise the
// same results as without it.
// Measured at the rerank shape (scripts/bench_attn.py, profiles/r02_attn_variants.jsonl):
// fp16x3 0.270-0.283 ms over all eight, 2 the fastest; fp16 0.140 ms without 4, 0.19-0.21
// with it (64-VGPR budget). The kernel's time is not in these (staging / latency bound).
// Bit 8 (profiles/r02e_lean_split.jsonl, same process): fp16x3 2 -> 10 0.281 -> 0.272 ms
// (the default since), fp16 unchanged (0.148 / 0.149: no split there).
// Bit 16 (two query blocks per wave side by side, bitwise the same; 114 VGPRs, no spill,
// same 4 waves per SIMD) measured slower at the rerank shape (profiles/r02q_attn_pairs.jsonl,
// same process, 7 rounds): 10 -> 26 0.254 -> 0.282 ms, 2 -> 18 0.268 -> 0.303: a diagnostic.
constexpr int kAttnVar = 42;
// rag_bert_attention's A/B slot in the production library: VAR 10 = 42 without the peeled,
// prefetched block loop (bitwise the same outputs, tests/test_attention_gpu.py)
constexpr int kAttnVarAB = 10;
// THREADS (round 6): 512 (8 waves) in general; 128 (2 waves) for query batches whose
// sequences are at most 32 tokens (2 query blocks, so 6 of 8 waves would only stage), which
// leaves the CUs' wave slots to the other batches in flight. A query block's arithmetic does
// not depend on which wave runs it: the outputs are bitwise the same.
template <int H, int HD, bool SPLIT, int VAR = kAttnVar, int THREADS = kAttnThreads<SPLIT>>
__global__ __launch_bounds__(THREADS, (kAttnWavesPerEU<HD, SPLIT>)) void attn_kernel(
    const _Float16* __restrict__ qkv, const _Float16* __restrict__ qkv_lo,
    const int* __restrict__ cu, int max_len, int kc, float scale, _Float16* __restrict__ ctx,
    _Float16* __restrict__ ctx_lo, int max_qb) {
  using St = AttnState<HD, SPLIT>;
  constexpr int NP = St::NP, KS = St::KS, DT = St::DT, KROW = HD, KCPR = HD / 8;
  constexpr int NW = THREADS / 64;
  extern __shared__ _Float16 alds[];
  // XCD-aware (sequence, head) order: blocks are dealt round-robin over the 8 XCDs, so give
  // XCD x a contiguous range of (sequence, head) pairs: the heads of one sequence run on one
  // XCD back to back and share the 128-B lines of the Q|K|V rows (64 B per head) in its L2
  // instead of each line being fetched once per head by different XCDs.
  constexpr int NH = H / HD;
  const int n_pairs = NH * (gridDim.x / NH);            // gridDim.x = NH * B rounded up to 8
  const int per_xcd = gridDim.x >> 3;
  const int pair = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
  if (pair >= n_pairs) return;
  const int b = pair / NH, h = pair % NH;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // LDS was sized for max_len on the host: a longer sequence (a caller breaking the
  // max_len contract of rag_encoder_forward) is truncated rather than overrunning LDS
  const int base = cu[b], len = min(cu[b + 1] - cu[b], max_len);
  if (len <= 0) return;
  const int sp = (len + 31) & ~31;
  const int cap = min(sp, kc);                      // keys per staged chunk
  const int nch = (sp + cap - 1) / cap;
  _Float16* kls[2] = {alds, alds + 2 * cap * KROW};
  _Float16* vls[2] = {alds + cap * KROW, alds + 3 * cap * KROW};
  const _Float16* planes[2] = {qkv, qkv_lo};
  const int g = lane >> 4, ql = lane & 15;
  const float c2 = scale * 1.44269504088896341f;
  const float rescale_gap = 8.0f / c2;             // deferred-max threshold (score units)

  // ---- stage keys [k0, k0 + n) (n multiple of 32; zeros past len): K and V row-major,
  // 16-B chunks (swizzled: swz_chunk for K's row reads, attn_vsw for V's transposed reads)
  auto stage = [&](int k0, int n) {
    // timing probes (diagnostic build, round 6; results meaningless): VAR bit 256 = no staging
    // at all (LDS left as it is), bit 128 = zeros stored instead of the loaded K / V
    if constexpr ((VAR & 256) != 0) return;
    if constexpr ((VAR & 2048) != 0) {
      // VAR bit 2048 (round 6): the K / V images filled by LDS-DMA (buffer_load ... lds): one
      // wave-instruction writes 1 KB = 64 / KCPR whole rows, lane l to LDS chunk position
      // (row l / KCPR, chunk l % KCPR); the swizzles are XORs, so that position's source chunk
      // is the swizzle of the position. Rows past len read as zeros through the sequence's
      // buffer extent. No VGPR round trip, no ds_write; same bytes in the same LDS places.
      // Diagnostic build: bitwise 42's outputs but 0.342 vs 0.242 ms per rerank-shape launch
      // (profiles/r06_attn/r06n3_*) — each piece gathers 16 rows' 64-B segments 2,304 B apart.
      constexpr int RPP = 64 / KCPR;
      const int pieces = n / RPP, tot = NP * 2 * pieces;
      const int rl = lane / KCPR, q = lane % KCPR;
      __amdgpu_buffer_rsrc_t rs[NP];
#pragma unroll
      for (int p = 0; p < NP; ++p)
        rs[p] = panel(planes[p] + (int64_t)base * (3 * H), (int64_t)len * (3 * H) * 2);
      const int wu = __builtin_amdgcn_readfirstlane(wid);   // piece indices wave-uniform
      for (int j = wu; j < tot; j += NW) {
        const int p = j / (2 * pieces), kv = (j / pieces) & 1, pc = j % pieces;
        const int r = pc * RPP + rl;
        const int ch = kv ? (q ^ attn_vsw<HD>(r)) : swz_chunk<KCPR>(r, q);
        const uint32_t voff =
            (uint32_t)((k0 + r) * (3 * H) + (kv ? 2 * H : H) + h * HD + 8 * ch) * 2u;
        const _Float16* dst = (kv ? vls[p] : kls[p]) + pc * RPP * KROW;
        blds16(p ? rs[NP - 1] : rs[0], voff, 0u,
               __builtin_amdgcn_readfirstlane(lds_addr_of(dst)));
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      return;
    }
    if constexpr ((VAR & 128) != 0) {
      for (int c = tid; c < n * (HD / 8); c += THREADS) {
        const int kl = c / (HD / 8), ch = c % (HD / 8);
#pragma unroll
        for (int p = 0; p < NP; ++p) {
          *reinterpret_cast<half8*>(kls[p] + kl * KROW + 8 * swz_chunk<KCPR>(kl, ch)) = half8{};
          *reinterpret_cast<half8*>(vls[p] + kl * HD + 8 * (ch ^ attn_vsw<HD>(kl))) = half8{};
        }
      }
      return;
    }
    if constexpr ((VAR & 64) != 0) {
      // VAR bit 64 (round 4): every staging load of up to SU passes issued before any LDS
      // store (one memory round trip per SU passes instead of one per pass); same bytes to
      // the same LDS places
      constexpr int SU = 2;
      constexpr int T = THREADS;
      const int total = n * (HD / 8);
      for (int c0 = tid; c0 < total; c0 += SU * T) {
        half8 kv[SU][NP], vv[SU][NP];
#pragma unroll
        for (int u = 0; u < SU; ++u) {
          const int c = c0 + u * T, kl = c / (HD / 8), ch = c % (HD / 8), key = k0 + kl;
#pragma unroll
          for (int p = 0; p < NP; ++p) {
            kv[u][p] = half8{};
            vv[u][p] = half8{};
            if (c < total && key < len) {
              const _Float16* src = planes[p] + (int64_t)(base + key) * (3 * H) + h * HD + 8 * ch;
              kv[u][p] = *reinterpret_cast<const half8*>(src + H);
              vv[u][p] = *reinterpret_cast<const half8*>(src + 2 * H);
            }
          }
        }
#pragma unroll
        for (int u = 0; u < SU; ++u) {
          const int c = c0 + u * T, kl = c / (HD / 8), ch = c % (HD / 8);
          if (c < total) {
#pragma unroll
            for (int p = 0; p < NP; ++p) {
              *reinterpret_cast<half8*>(kls[p] + kl * KROW + 8 * swz_chunk<KCPR>(kl, ch)) = kv[u][p];
              *reinterpret_cast<half8*>(vls[p] + kl * HD + 8 * (ch ^ attn_vsw<HD>(kl))) = vv[u][p];
            }
          }
        }
      }
      return;
    }
    for (int c = tid; c < n * (HD / 8); c += THREADS) {
      const int kl = c / (HD / 8), ch = c % (HD / 8), key = k0 + kl;
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        half8 kv = {}, vv = {};
        if (key < len) {
          const _Float16* src = planes[p] + (int64_t)(base + key) * (3 * H) + h * HD + 8 * ch;
          kv = *reinterpret_cast<const half8*>(src + H);
          vv = *reinterpret_cast<const half8*>(src + 2 * H);
        }
        *reinterpret_cast<half8*>(kls[p] + kl * KROW + 8 * swz_chunk<KCPR>(kl, ch)) = kv;
        *reinterpret_cast<half8*>(vls[p] + kl * HD + 8 * (ch ^ attn_vsw<HD>(kl))) = vv;
      }
    }
  };
  // this lane's transposed-read offset (halves) for V^T fragment dt of a 32-key block at
  // row 0: lane 4q + pp of 16-lane group g supplies row 4g + q, columns 16 dt + 4 pp .. + 3
  // (the second read: rows + 16; the swizzle is the same for both and for every block)
  const int vq = (lane & 15) >> 2, vpp = lane & 3;
  auto voff = [&](int dt) {
    const int r = 4 * g + vq;
    return r * HD + 8 * ((2 * dt + (vpp >> 1)) ^ attn_vsw<HD>(r)) + 4 * (vpp & 1);
  };
  auto load_q = [&](half8 (&qf)[KS][NP], int qb) {
    const int r = min(qb * 16 + ql, len - 1);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int p = 0; p < NP; ++p)
        qf[ks][p] = *reinterpret_cast<const half8*>(
            planes[p] + (int64_t)(base + r) * (3 * H) + h * HD + 32 * ks + 8 * g);
  };
  auto reset = [&](St& st) {
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) st.o[dt] = floatx4{0.f, 0.f, 0.f, 0.f};
    st.l = floatx4{0.f, 0.f, 0.f, 0.f};
    st.m = kNegInf;
  };
  auto init = [&](St& st, int qb) {
    load_q(st.qf, qb);
    reset(st);
  };
  half8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (_Float16)1.0f;
  // S^T of the 32-key block at LDS position kb
  auto qk = [&](const St& st, int kb, floatx4 (&sc)[2]) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        sc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const int krow = kb + 16 * j + ql;
          const int kr = krow * KROW + 8 * swz_chunk<KCPR>(krow, 4 * ks + g);
          const half8 kf = *reinterpret_cast<const half8*>(kls[0] + kr);
          sc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf, st.qf[ks][0], sc[j], 0, 0, 0);
          if constexpr (SPLIT) {
            const half8 kfl = *reinterpret_cast<const half8*>(kls[1] + kr);
            sc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kfl, st.qf[ks][0], sc[j], 0, 0, 0);
            sc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf, st.qf[ks][1], sc[j], 0, 0, 0);
          }
        }
      }
  };
  // softmax update and P.V for the block at LDS position kb (keys k0 + kb ..). mode (VAR bit
  // 32's peeled loop): 0 = is the block full? checked here; 1 = known full; 2 = known partial.
  // Bit 32 also issues the block's V^T fragment reads first, so their LDS latency runs under
  // the max / exp / split work instead of between the P.V MFMAs.
  auto softmax_pv_m = [&](St& st, int k0, int kb, floatx4 (&sc)[2], auto mode) {
      constexpr int MODE = decltype(mode)::value;
      constexpr bool VPRE = (VAR & 40) == 40;
      half8 vh[DT], vlo[DT];
      if constexpr (VPRE) {
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          const int vr = kb * HD + voff(dt);
          vh[dt] = __builtin_shufflevector(lds_read_tr16(vls[0] + vr),
                                           lds_read_tr16(vls[0] + vr + 16 * HD),
                                           0, 1, 2, 3, 4, 5, 6, 7);
          if constexpr (SPLIT)
            vlo[dt] = __builtin_shufflevector(lds_read_tr16(vls[1] + vr),
                                              lds_read_tr16(vls[1] + vr + 16 * HD),
                                              0, 1, 2, 3, 4, 5, 6, 7);
        }
        __builtin_amdgcn_sched_barrier(0);   // keep the reads ahead of the softmax
      }
      // lane: S^T[key k0 + kb + 16j + 4g + r][q]. Softmax in base 2 with the 1/sqrt(d) scale
      // folded into one FMA: p = 2^(s*c - m*c), c = scale*log2(e) > 0 (max commutes).
      float mx;
      if (MODE == 1 || (MODE == 0 && k0 + kb + 32 <= len)) {
        if constexpr ((VAR & 8) != 0)   // IEEE maximum: no per-input canonicalisation
          mx = fmax_nc(fmax_nc(fmax_nc(sc[0][0], sc[0][1]), fmax_nc(sc[0][2], sc[0][3])),
                       fmax_nc(fmax_nc(sc[1][0], sc[1][1]), fmax_nc(sc[1][2], sc[1][3])));
        else
          mx = fmaxf(fmaxf(fmaxf(sc[0][0], sc[0][1]), fmaxf(sc[0][2], sc[0][3])),
                     fmaxf(fmaxf(sc[1][0], sc[1][1]), fmaxf(sc[1][2], sc[1][3])));
      } else {
        mx = kNegInf;
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            if (k0 + kb + 16 * j + 4 * g + r >= len) sc[j][r] = kNegInf;
            mx = (VAR & 8) != 0 ? fmax_nc(mx, sc[j][r]) : fmaxf(mx, sc[j][r]);
          }
      }
      if constexpr ((VAR & 8) != 0) {
        // lanes l, l^16, l^32, l^48 hold the same query's other keys
        const uint32_t mu = __builtin_bit_cast(uint32_t, mx);
        const auto r16 = __builtin_amdgcn_permlane16_swap(mu, mu, false, false);
        mx = fmax_nc(__builtin_bit_cast(float, (uint32_t)r16[0]),
                     __builtin_bit_cast(float, (uint32_t)r16[1]));
        const uint32_t mu2 = __builtin_bit_cast(uint32_t, mx);
        const auto r32 = __builtin_amdgcn_permlane32_swap(mu2, mu2, false, false);
        mx = fmax_nc(__builtin_bit_cast(float, (uint32_t)r32[0]),
                     __builtin_bit_cast(float, (uint32_t)r32[1]));
      } else {
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      }
      // Deferred rescale: the running max only moves when some query's block max exceeds it
      // by more than 8 / c2 (P = 2^(s c2 - m c2) then stays <= 2^8, exact in the fp16 MFMA
      // operand and far from its range limit); otherwise the old max is kept and the
      // rescale of l and O (an exp2 and DT*4 + 1 multiplies per block) is skipped. The
      // normalisation divides by l summed from the same P, so the result is unchanged up to
      // rounding. Wave-uniform branch (ballot).
      if (__builtin_amdgcn_ballot_w64(mx > st.m + rescale_gap)) {
        const float mnew = fmaxf(st.m, mx);
        const float corr = __builtin_amdgcn_exp2f((st.m - mnew) * c2);
#pragma unroll
        for (int r = 0; r < 4; ++r) st.l[r] *= corr;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt)
#pragma unroll
          for (int r = 0; r < 4; ++r) st.o[dt][r] *= corr;
        st.m = mnew;
      }
      const float nm = -st.m * c2;
      half8 ph, pl;
      if constexpr (SPLIT && (VAR & 8) != 0) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 4; r += 2) {
            float e0, e1;
            if constexpr ((VAR & 512) != 0) {   // two scalar FMAs, never paired into a
              e0 = __builtin_amdgcn_exp2f(fma_scalar(sc[j][r], c2, nm));   // v_pk_fma_f32
              e1 = __builtin_amdgcn_exp2f(fma_scalar(sc[j][r + 1], c2, nm));
            } else if constexpr (VPRE) {   // the two scalings as one packed fp32 FMA (v_pk_fma_f32)
              typedef float f2 __attribute__((ext_vector_type(2)));
              const f2 t = __builtin_elementwise_fma(f2{sc[j][r], sc[j][r + 1]}, f2{c2, c2},
                                                     f2{nm, nm});
              e0 = __builtin_amdgcn_exp2f(t[0]);
              e1 = __builtin_amdgcn_exp2f(t[1]);
            } else {
              e0 = __builtin_amdgcn_exp2f(fmaf(sc[j][r], c2, nm));
              e1 = __builtin_amdgcn_exp2f(fmaf(sc[j][r + 1], c2, nm));
            }
            half2 h2, l2;
            split16x2(e0, e1, h2, l2);
            ph[4 * j + r] = h2[0]; ph[4 * j + r + 1] = h2[1];
            pl[4 * j + r] = l2[0]; pl[4 * j + r + 1] = l2[1];
          }
      } else {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float e = __builtin_amdgcn_exp2f(fmaf(sc[j][r], c2, nm));
            if constexpr (SPLIT) { const half2 s16_ = split16(e); ph[4 * j + r] = s16_[0]; pl[4 * j + r] = s16_[1]; }
            else ph[4 * j + r] = (_Float16)e;
          }
      }
      // row sum of P exactly as the MFMA sees it (hi [+ lo]). fp16x3: the same MFMA against
      // a ones fragment (the MFMA pipe has the slack there, the vector ALU does not: 2 MFMAs
      // for 8 v_dot2, and every lane ends up with its query's whole sum); fp16: v_dot2 (the
      // 64-VGPR budget of 8 waves per SIMD has no room for the fragment and accumulator)
      if constexpr (SPLIT && (VAR & 2)) {
        st.l = __builtin_amdgcn_mfma_f32_16x16x32_f16(ones, pl, st.l, 0, 0, 0);
        st.l = __builtin_amdgcn_mfma_f32_16x16x32_f16(ones, ph, st.l, 0, 0, 0);
      } else {
        const half2 one2 = {(_Float16)1.0f, (_Float16)1.0f};
#pragma unroll
        for (int e2 = 0; e2 < 4; ++e2) {
          st.l[0] = __builtin_amdgcn_fdot2(half2{ph[2 * e2], ph[2 * e2 + 1]}, one2, st.l[0], false);
          if constexpr (SPLIT)
            st.l[0] = __builtin_amdgcn_fdot2(half2{pl[2 * e2], pl[2 * e2 + 1]}, one2, st.l[0], false);
        }
      }
      if constexpr ((VAR & 8) != 0) {
        if constexpr (!VPRE) {
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) {
            const int vr = kb * HD + voff(dt);
            vh[dt] = __builtin_shufflevector(lds_read_tr16(vls[0] + vr),
                                             lds_read_tr16(vls[0] + vr + 16 * HD),
                                             0, 1, 2, 3, 4, 5, 6, 7);
            if constexpr (SPLIT)
              vlo[dt] = __builtin_shufflevector(lds_read_tr16(vls[1] + vr),
                                                lds_read_tr16(vls[1] + vr + 16 * HD),
                                                0, 1, 2, 3, 4, 5, 6, 7);
          }
        }
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          if constexpr (SPLIT) {
            st.o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vlo[dt], ph, st.o[dt], 0, 0, 0);
            st.o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vh[dt], pl, st.o[dt], 0, 0, 0);
          }
          st.o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vh[dt], ph, st.o[dt], 0, 0, 0);
        }
        return;
      }
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const int vr = kb * HD + voff(dt);
        const half8 v = __builtin_shufflevector(lds_read_tr16(vls[0] + vr),
                                                lds_read_tr16(vls[0] + vr + 16 * HD),
                                                0, 1, 2, 3, 4, 5, 6, 7);
        if constexpr (SPLIT) {
          const half8 vl = __builtin_shufflevector(lds_read_tr16(vls[1] + vr),
                                                   lds_read_tr16(vls[1] + vr + 16 * HD),
                                                   0, 1, 2, 3, 4, 5, 6, 7);
          st.o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vl, ph, st.o[dt], 0, 0, 0);
          st.o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(v, pl, st.o[dt], 0, 0, 0);
        }
        st.o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(v, ph, st.o[dt], 0, 0, 0);
      }
  };
  auto softmax_pv = [&](St& st, int k0, int kb, floatx4 (&sc)[2]) {
    softmax_pv_m(st, k0, kb, sc, std::integral_constant<int, 0>{});
  };
  // VAR bit 32: the K fragments of a block (read one block ahead) and their S^T MFMAs
  auto kread = [&](int kb, half8 (&kf)[2][KS][NP]) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int krow = kb + 16 * j + ql;
        const int kr = krow * KROW + 8 * swz_chunk<KCPR>(krow, 4 * ks + g);
#pragma unroll
        for (int p = 0; p < NP; ++p) kf[j][ks][p] = *reinterpret_cast<const half8*>(kls[p] + kr);
      }
  };
  auto kmma = [&](const St& st, const half8 (&kf)[2][KS][NP], floatx4 (&sc)[2]) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      sc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {   // the term order of qk()
        sc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf[j][ks][0], st.qf[ks][0], sc[j], 0, 0, 0);
        if constexpr (SPLIT) {
          sc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf[j][ks][1], st.qf[ks][0], sc[j], 0, 0, 0);
          sc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf[j][ks][0], st.qf[ks][1], sc[j], 0, 0, 0);
        }
      }
    }
  };
  // keys [k0, k0 + n) of the staged chunk (LDS positions 0 .. n-1)
  auto attend = [&](St& st, int k0, int n) {
    if constexpr ((VAR & 32) != 0) {
      // Peeled loop: the blocks wholly inside the sequence run without the key mask (no
      // per-block branch, and no register copies between a masked and an unmasked version of
      // the scores); the last, partial block (if any) after them. Block kb + 32's K fragments
      // are read while block kb's softmax runs. Same arithmetic, same order: bitwise the
      // outputs of the variant without bit 32.
      const int nf = min(n, len - k0) & ~31;
      half8 kf[2][KS][NP];
      if (n > 0) kread(0, kf);
      if constexpr ((VAR & 4) != 0) {
        // + bit 4: block kb + 32's S^T MFMAs issued before block kb's softmax (they run in
        // the matrix pipe under its vector work), block kb + 64's K read behind them
        floatx4 sn[2];
        if (n > 0) {
          kmma(st, kf, sn);
          if (32 < n) kread(32, kf);
        }
        int kb = 0;
        for (; kb < nf; kb += 32) {
          floatx4 sc[2] = {sn[0], sn[1]};
          if (kb + 32 < n) {
            kmma(st, kf, sn);
            if (kb + 64 < n) kread(kb + 64, kf);
          }
          softmax_pv_m(st, k0, kb, sc, std::integral_constant<int, 1>{});
        }
        if (kb < n) softmax_pv_m(st, k0, kb, sn, std::integral_constant<int, 2>{});
        return;
      }
      for (int kb = 0; kb < nf; kb += 32) {
        floatx4 sc[2];
        kmma(st, kf, sc);
        if (kb + 32 < n) kread(kb + 32, kf);
        softmax_pv_m(st, k0, kb, sc, std::integral_constant<int, 1>{});
      }
      if (nf < n) {
        floatx4 sc[2];
        kmma(st, kf, sc);
        softmax_pv_m(st, k0, nf, sc, std::integral_constant<int, 2>{});
      }
    } else if constexpr ((VAR & 4) != 0) {
      floatx4 sn[2];
      qk(st, 0, sn);
      for (int kb = 0; kb < n; kb += 32) {
        floatx4 sc[2] = {sn[0], sn[1]};
        if (kb + 32 < n) qk(st, kb + 32, sn);
        softmax_pv(st, k0, kb, sc);
      }
    } else {
      for (int kb = 0; kb < n; kb += 32) {
        floatx4 sc[2];
        qk(st, kb, sc);
        softmax_pv(st, k0, kb, sc);
      }
    }
  };
  auto finish = [&](St& st, int qb) {
    float l = st.l[0];
    if constexpr (!(SPLIT && (VAR & 2))) {
      l += __shfl_xor(l, 16, 64);
      l += __shfl_xor(l, 32, 64);
    }
    const int q = qb * 16 + ql;
    if (q < len) {
      // lane: O^T[d = 16dt + 4g + r][q]
      const float inv = 1.0f / l;
      const int64_t off = (int64_t)(base + q) * H + h * HD + 4 * g;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        half4 a, al;
        if constexpr (SPLIT && (VAR & 8) != 0) {
#pragma unroll
          for (int r = 0; r < 4; r += 2) {
            half2 h2, l2;
            split16x2(st.o[dt][r] * inv, st.o[dt][r + 1] * inv, h2, l2);
            a[r] = h2[0]; a[r + 1] = h2[1]; al[r] = l2[0]; al[r + 1] = l2[1];
          }
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float x = st.o[dt][r] * inv;
            if constexpr (SPLIT) { const half2 s16_ = split16(x); a[r] = s16_[0]; al[r] = s16_[1]; }
            else a[r] = (_Float16)x;
          }
        }
        *reinterpret_cast<half4*>(ctx + off + 16 * dt) = a;
        if constexpr (SPLIT) *reinterpret_cast<half4*>(ctx_lo + off + 16 * dt) = al;
      }
    }
  };

  const int nqb = min((len + 15) >> 4, max_qb);     // max_qb = 1: the CLS query block only
  if ((VAR & 16) != 0 && nch == 1) {
    // paired query blocks: a wave carries blocks qb and qb + NW through the key blocks side
    // by side (two independent score -> softmax -> P.V chains for the scheduler to interleave;
    // a rerank sequence of 200-288 tokens has 13-18 blocks, i.e. about one pair per wave of
    // the 8). A wave left with one block runs it twice and stores it once. Per block the
    // arithmetic is the single-block path's, so the outputs are bitwise the same.
    for (int qb = wid; qb < nqb; qb += 2 * NW) {
      const bool two = qb + NW < nqb;
      const int qb2 = two ? qb + NW : qb;
      St s0, s1;
      init(s0, qb);
      init(s1, qb2);
      if (qb == wid) {                  // first round: the Q loads ride under the staging
        stage(0, sp);
        __syncthreads();
      }
      for (int kb = 0; kb < sp; kb += 32) {
        floatx4 sc0[2], sc1[2];
        qk(s0, kb, sc0);
        qk(s1, kb, sc1);
        softmax_pv(s0, 0, kb, sc0);
        softmax_pv(s1, 0, kb, sc1);
      }
      finish(s0, qb);
      if (two) finish(s1, qb2);
    }
    if (wid >= nqb) {                   // a wave without a block still joins the staging
      stage(0, sp);
      __syncthreads();
    }
  } else if (nch == 1) {
    // rolling Q prefetch: a wave's first QPF query blocks are loaded before the K/V staging
    // (their latency hides behind it), and each later one while the block QPF ahead computes
    // (fp16 at head_dim 32 runs 8 waves per SIMD in 64 VGPRs: one block ahead fits)
    // (VAR bit 1024, round 6, diagnostic build: one block ahead in fp16x3 too — 8 VGPRs instead
    // of bit 1's 24, still 112 in all; bitwise 42's outputs, timing neutral: 1066 0.2486-0.2519
    // vs 42 0.2485-0.2507 ms, profiles/r06_attn/r06n2_*: the Q loads' latency is not exposed)
    constexpr int QPF = (VAR & 1) == 0 ? ((VAR & 1024) != 0 ? 1 : 0) : SPLIT || HD > 32 ? 3 : 1;
    half8 qpre[QPF > 0 ? QPF : 1][KS][NP];
#pragma unroll
    for (int i = 0; i < QPF; ++i)
      if (wid + i * NW < nqb) load_q(qpre[i], wid + i * NW);
    stage(0, sp);
    __syncthreads();
    for (int qb = wid; qb < nqb; qb += NW) {
      St st;
      if constexpr (QPF > 0) {
        reset(st);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
#pragma unroll
          for (int p = 0; p < NP; ++p) {
            st.qf[ks][p] = qpre[0][ks][p];
#pragma unroll
            for (int i = 0; i + 1 < QPF; ++i) qpre[i][ks][p] = qpre[i + 1][ks][p];
          }
        if (qb + QPF * NW < nqb) load_q(qpre[QPF - 1], qb + QPF * NW);
      } else {
        init(st, qb);
      }
      attend(st, 0, sp);
      finish(st, qb);
    }
  } else {
    // keys do not fit at once: for each round of query blocks, stream the key chunks
    // (every wave joins every barrier; waves without a block this round only stage)
    for (int q0 = 0; q0 < nqb; q0 += NW) {
      const int qb = q0 + wid;
      St st;
      if (qb < nqb) init(st, qb);
      for (int ch = 0; ch < nch; ++ch) {
        const int k0 = ch * cap, n = min(cap, sp - k0);
        __syncthreads();
        stage(k0, n);
        __syncthreads();
        if (qb < nqb) attend(st, k0, n);
      }
      if (qb < nqb) finish(st, qb);
    }
  }
}

// ----------------------------------------------------------------------------------------
// last layer, CLS rows only: both heads read only the CLS token's final hidden state
// (sentence-transformers Pooling(cls); BertPooler takes hidden_states[:, 0]), and a token's
// row after the last attention depends on the other tokens only through that attention. So
// the last layer computes Q|K|V for every token (K, V are needed), attention for the first
// query block of each sequence, and everything after it — O-proj, residual + LN, FFN,
// residual + LN — on the B gathered CLS rows instead of all T tokens.
// gather: x_cls[b] = x[cu[b]], ctx_cls[b] = ctx[cu[b]] (+ lo plane); one wave per sequence.
// Deferred LayerNorm (st non-null, H = kDlH): the token rows hold z = xh + xl and its block
// statistics, and x_cls = LN(z) with (gamma, beta) = (g, bt).
// ----------------------------------------------------------------------------------------
template <int H>
__global__ __launch_bounds__(64) void gather_cls_kernel(
    const float* __restrict__ x, const _Float16* __restrict__ xh,
    const _Float16* __restrict__ xl, const _Float16* __restrict__ ctx,
    const _Float16* __restrict__ ctx_lo, const int* __restrict__ cu, float* __restrict__ x_cls,
    _Float16* __restrict__ ctx_cls, _Float16* __restrict__ ctx_cls_lo,
    const float* __restrict__ st = nullptr, const float* __restrict__ g = nullptr,
    const float* __restrict__ bt = nullptr, float eps = 0.f,
    _Float16* __restrict__ xh_cls = nullptr, _Float16* __restrict__ xl_cls = nullptr) {
  // (ctx null: the CLS rows only, before a CLS-only attention, attn_cls_kernel; xh_cls /
  // xl_cls: also their hi / lo fp16 planes, the Q projection's operands)
  const int b = blockIdx.x, lane = threadIdx.x;
  const int64_t r = cu[b];
  float mu = 0.f, rs = 1.f;
  if (H == kDlH && st) {
    const floatx4* sr = reinterpret_cast<const floatx4*>(st + r * kDlParts * 2);
    dl_row_stats(sr[0], sr[1], sr[2], eps, mu, rs);
  }
#pragma unroll
  for (int j = 0; j < H / 64; ++j) {
    const int c = lane + 64 * j;
    // (x null: the residual stream is xh + xl, add_ln_kernel<XF> / deferred LayerNorm)
    float v = x ? x[r * H + c] : (float)xh[r * H + c] + (float)xl[r * H + c];
    if (st) v = (v - mu) * rs * g[c] + bt[c];
    x_cls[(int64_t)b * H + c] = v;
    if (xh_cls) {
      const _Float16 hv = (_Float16)v;
      xh_cls[(int64_t)b * H + c] = hv;
      if (xl_cls) xl_cls[(int64_t)b * H + c] = (_Float16)(v - (float)hv);
    }
    if (ctx) {
      ctx_cls[(int64_t)b * H + c] = ctx[r * H + c];
      if (ctx_lo) ctx_cls_lo[(int64_t)b * H + c] = ctx_lo[r * H + c];
    }
  }
}

// ----------------------------------------------------------------------------------------
// CLS-only attention of the last encoder layer (round 4): the cross-encoder / bge heads read
// only the [CLS] row, so the last layer needs the attention output of one query per
// (sequence, head). One wave per (sequence, head), 4 heads per workgroup: lane j takes keys
// j, j + 64, ... of the sequence; scores from the fp16x3 planes in fp32 (the MFMA path's
// three products: k_hi q_hi + k_lo q_hi + k_hi q_lo), softmax in base 2 with the 1/sqrt(d)
// scale folded in, P . V against v_hi + v_lo, then one cross-lane combine (max, rescale, sum).
// kv: [T][2H] planes (K | V of every token: the last layer's K|V-only projection); q: [B][H]
// planes of the CLS rows' Q; out: [B][H] planes of the CLS rows' context.
// ----------------------------------------------------------------------------------------
constexpr int kAttnClsHeads = 4;
constexpr int kAttnClsBlock = 64 * kAttnClsHeads;   // launch_fixed / __launch_bounds__
template <int H, int HD>
__global__ __launch_bounds__(kAttnClsBlock) void attn_cls_kernel(
    const _Float16* __restrict__ kv, const _Float16* __restrict__ kv_lo,
    const _Float16* __restrict__ q, const _Float16* __restrict__ q_lo,
    const int* __restrict__ cu, int B, int max_len, float scale, _Float16* __restrict__ out,
    _Float16* __restrict__ out_lo) {
  static_assert(HD % 8 == 0 && (H / HD) % kAttnClsHeads == 0, "head groups");
  constexpr int NH = H / HD;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int b = blockIdx.x / (NH / kAttnClsHeads);
  const int h = (blockIdx.x % (NH / kAttnClsHeads)) * kAttnClsHeads + wv;
  if (b >= B) return;
  const int base = cu[b], len = min(cu[b + 1] - cu[b], max_len);
  float qh[HD], ql[HD];
#pragma unroll
  for (int c = 0; c < HD / 8; ++c) {
    const half8 a = *reinterpret_cast<const half8*>(q + (int64_t)b * H + h * HD + 8 * c);
    const half8 l = *reinterpret_cast<const half8*>(q_lo + (int64_t)b * H + h * HD + 8 * c);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      qh[8 * c + e] = (float)a[e];
      ql[8 * c + e] = (float)l[e];
    }
  }
  const float c2 = scale * 1.44269504088896341f;
  float m = kNegInf, l = 0.f, o[HD];
#pragma unroll
  for (int d = 0; d < HD; ++d) o[d] = 0.f;
  for (int j = lane; j < len; j += 64) {
    const _Float16* kr = kv + (int64_t)(base + j) * (2 * H) + h * HD;
    const _Float16* krl = kv_lo + (int64_t)(base + j) * (2 * H) + h * HD;
    half8 k8[HD / 8], kl8[HD / 8], v8[HD / 8], vl8[HD / 8];
#pragma unroll
    for (int c = 0; c < HD / 8; ++c) {
      k8[c] = *reinterpret_cast<const half8*>(kr + 8 * c);
      kl8[c] = *reinterpret_cast<const half8*>(krl + 8 * c);
      v8[c] = *reinterpret_cast<const half8*>(kr + H + 8 * c);
      vl8[c] = *reinterpret_cast<const half8*>(krl + H + 8 * c);
    }
    float s0 = 0.f, s1 = 0.f;   // k_hi q_hi and the two correction products
#pragma unroll
    for (int c = 0; c < HD / 8; ++c)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float kh = (float)k8[c][e], klo = (float)kl8[c][e];
        s0 = fmaf(kh, qh[8 * c + e], s0);
        s1 = fmaf(klo, qh[8 * c + e], fmaf(kh, ql[8 * c + e], s1));
      }
    const float sc = (s0 + s1) * c2;
    const float mn = fmaxf(m, sc);
    const float corr = __builtin_amdgcn_exp2f(m - mn);   // m = -inf: 0
    const float p = __builtin_amdgcn_exp2f(sc - mn);
    l = l * corr + p;
#pragma unroll
    for (int c = 0; c < HD / 8; ++c)
#pragma unroll
      for (int e = 0; e < 8; ++e)
        o[8 * c + e] = fmaf(p, (float)v8[c][e] + (float)vl8[c][e], o[8 * c + e] * corr);
    m = mn;
  }
  // combine the 64 lanes: common max, rescale, sums
  float mw = m;
#pragma unroll
  for (int sh = 32; sh >= 1; sh >>= 1) mw = fmaxf(mw, __shfl_xor(mw, sh, 64));
  const float f = m == kNegInf ? 0.f : __builtin_amdgcn_exp2f(m - mw);
  l *= f;
#pragma unroll
  for (int sh = 32; sh >= 1; sh >>= 1) l += __shfl_xor(l, sh, 64);
#pragma unroll
  for (int d = 0; d < HD; ++d) {
    float x = o[d] * f;
#pragma unroll
    for (int sh = 32; sh >= 1; sh >>= 1) x += __shfl_xor(x, sh, 64);
    o[d] = x;
  }
  if (lane < HD) {
    float v = 0.f;
#pragma unroll
    for (int d = 0; d < HD; ++d) v = lane == d ? o[d] : v;
    v = v / l;
    const _Float16 hv = (_Float16)v;
    out[(int64_t)b * H + h * HD + lane] = hv;
    out_lo[(int64_t)b * H + h * HD + lane] = (_Float16)(v - (float)hv);
  }
}

// ----------------------------------------------------------------------------------------
// cross-encoder batch assembly from cached chunk tokens (rag_build_pairs; the torch
// restatement ragmi.pairs.build_pairs is its CPU-tested twin): pair p = b K + k is
//   [CLS] q_b [SEP] c_{rows[b][k]} [SEP], token types 0 .. 0 1 .. 1,
// the chunk cut so the pair fits max_len (longest_first truncation removes chunk tokens for
// the reference's short queries). pairs_len_kernel: one workgroup, pair lengths -> cu (block
// scan) + stats {T, longest}; pairs_fill_kernel: one workgroup per pair writes its tokens.
// ----------------------------------------------------------------------------------------
constexpr int kPairsMax = 1024;   // B * K per call

__device__ __forceinline__ void pair_parts(const int* __restrict__ q_cu, const int64_t* rows,
                                           const int* __restrict__ c_lens, int K, int p,
                                           int max_len, int& ql, int& cl, int64_t& r) {
  const int b = p / K;
  ql = q_cu[b + 1] - q_cu[b] - 2;                 // query tokens without its [CLS] / [SEP]
  r = rows[p] < 0 ? 0 : rows[p];                  // -1 (no hit): row 0, caller masks
  cl = min(c_lens[r], max_len - 3 - ql);
}

__global__ __launch_bounds__(kPairsMax) void pairs_len_kernel(
    const int* __restrict__ q_cu, const int64_t* __restrict__ rows,
    const int* __restrict__ c_lens, int P, int K, int max_len, int* __restrict__ cu,
    int* __restrict__ stats) {
  __shared__ int wsum[kPairsMax / 64];
  __shared__ int wmax[kPairsMax / 64];
  const int p = threadIdx.x, lane = p & 63, w = p >> 6;
  int len = 0;
  if (p < P) {
    int ql, cl;
    int64_t r;
    pair_parts(q_cu, rows, c_lens, K, p, max_len, ql, cl, r);
    len = ql + cl + 3;
  }
  // inclusive wave scan, then across waves
  int incl = len, mx = len;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int v = __shfl_up(incl, d, 64);
    if (lane >= d) incl += v;
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) mx = max(mx, __shfl_xor(mx, d, 64));
  if (lane == 63) wsum[w] = incl;
  if (lane == 0) wmax[w] = mx;
  __syncthreads();
  int base = 0, gmax = 0;
  for (int i = 0; i < kPairsMax / 64; ++i) {
    if (i < w) base += wsum[i];
    gmax = max(gmax, wmax[i]);
  }
  if (p < P) cu[p + 1] = base + incl;
  if (p == 0) cu[0] = 0;
  if (p == P - 1) {
    stats[0] = base + incl;                       // T
    stats[1] = gmax;                              // longest pair
  }
}

__global__ __launch_bounds__(256) void pairs_fill_kernel(
    const int* __restrict__ q_ids, const int* __restrict__ q_cu,
    const int64_t* __restrict__ rows, const int16_t* __restrict__ c_toks, int lmax,
    const int* __restrict__ c_lens, const int* __restrict__ cu, int K, int max_len,
    int* __restrict__ ids, int* __restrict__ types) {
  const int p = blockIdx.x;
  int ql, cl;
  int64_t r;
  pair_parts(q_cu, rows, c_lens, K, p, max_len, ql, cl, r);
  const int n = ql + cl + 3, o = cu[p], qs = q_cu[p / K] + 1;
  for (int t = threadIdx.x; t < n; t += 256) {
    int id;
    if (t == 0) id = 101;                                        // [CLS]
    else if (t <= ql) id = q_ids[qs + t - 1];
    else if (t == ql + 1 || t == n - 1) id = 102;                // [SEP]
    else id = (int)(uint16_t)c_toks[r * lmax + (t - ql - 2)];
    ids[o + t] = id;
    types[o + t] = t > ql + 1 ? 1 : 0;
  }
}

// ----------------------------------------------------------------------------------------
// heads
// ----------------------------------------------------------------------------------------
// bge (sentence-transformers Pooling(cls) + Normalize): out[b] = x[cls] / max(||x[cls]||, 1e-12)
template <int H>
__global__ __launch_bounds__(64) void cls_normalize_kernel(const float* __restrict__ x,
                                                           const int* __restrict__ cu,
                                                           float* __restrict__ out) {
  const int b = blockIdx.x, lane = threadIdx.x;
  const float* r = x + (cu ? (int64_t)cu[b] : (int64_t)b) * H;   // cu null: x holds CLS rows
  float v[H / 64];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < H / 64; ++j) {
    v[j] = r[lane + 64 * j];
    s += v[j] * v[j];
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) s += __shfl_xor(s, d, 64);
  const float inv = 1.0f / fmaxf(sqrtf(s), 1e-12f);
#pragma unroll
  for (int j = 0; j < H / 64; ++j) out[(int64_t)b * H + lane + 64 * j] = v[j] * inv;
}

// cross-encoder: pooled = tanh(Wp x[cls] + bp); logit = Wc pooled + bc (num_labels = 1)
template <int H>
__global__ __launch_bounds__(256) void ce_head_kernel(const float* __restrict__ x,
                                                      const int* __restrict__ cu,
                                                      const float* __restrict__ wp,
                                                      const float* __restrict__ bp,
                                                      const float* __restrict__ wc,
                                                      const float* __restrict__ bc,
                                                      float* __restrict__ out) {
  __shared__ float cls[H];
  __shared__ float part[4];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t row = cu ? (int64_t)cu[b] : (int64_t)b;   // cu null: x holds CLS rows
  for (int c = tid; c < H; c += 256) cls[c] = x[row * H + c];
  __syncthreads();
  float acc = 0.f;
  for (int o = tid; o < H; o += 256) {
    const float* wr = wp + (int64_t)o * H;
    float d = 0.f;
    for (int c = 0; c < H; c += 4) {
      const float4 w4 = *reinterpret_cast<const float4*>(wr + c);
      d += w4.x * cls[c] + w4.y * cls[c + 1] + w4.z * cls[c + 2] + w4.w * cls[c + 3];
    }
    acc += tanhf(d + bp[o]) * wc[o];
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) acc += __shfl_xor(acc, d, 64);
  if (lane == 0) part[wid] = acc;
  __syncthreads();
  if (tid == 0) out[b] = part[0] + part[1] + part[2] + part[3] + bc[0];
}

}  // namespace bert
}  // namespace ragmi
