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

constexpr int H = 384;      // hidden
constexpr int NH = 12;      // heads
constexpr int HD = 32;      // head dim
constexpr int FF = 1536;    // intermediate

typedef _Float16 half4 __attribute__((ext_vector_type(4)));

// fp16x3 split: v = hi + lo with hi = fp16(v), lo = fp16(v - hi); a*b ~ ah*bh + ah*bl + al*bh
// (relative error ~2^-22) on the fp16 MFMA pipe.
__device__ __forceinline__ _Float16 lo_part(float v, _Float16 hi) { return (_Float16)(v - (float)hi); }

__device__ __forceinline__ float gelu_erf(float x) {
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752440f));
}

// ----------------------------------------------------------------------------------------
// embeddings: x = LN(word[id] + type[tt] + pos[p]); one wave per token, grid (ceil(L/4), B)
// ----------------------------------------------------------------------------------------
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
    x[t * H + c] = y;
    const _Float16 yh = (_Float16)y;
    xh[t * H + c] = yh;
    if (xl) xl[t * H + c] = lo_part(y, yh);
  }
}

// ----------------------------------------------------------------------------------------
// residual + LayerNorm: x = LN(x + y) (fp32, in place), xh = fp16(x); one wave per row
// ----------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void add_ln_kernel(float* __restrict__ x,
                                                     const float* __restrict__ y,
                                                     const float* __restrict__ g,
                                                     const float* __restrict__ bt, float eps,
                                                     _Float16* __restrict__ xh,
                                                     _Float16* __restrict__ xl, int T) {
  const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (t >= T) return;
  float v[H / 64];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < H / 64; ++j) {
    const int c = lane + 64 * j;
    v[j] = x[t * H + c] + y[t * H + c];
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
    x[t * H + c] = o;
    const _Float16 oh = (_Float16)o;
    xh[t * H + c] = oh;
    if (xl) xl[t * H + c] = lo_part(o, oh);
  }
}

// ----------------------------------------------------------------------------------------
// GEMM: C[M,N] = A[M,K] . W[N,K]^T + bias[N]   (A fp16 row-major, W fp16 [N][K] = HF Linear)
// 128x128 tile, BK = 64, 256 threads = 2x2 waves of 64x64, v_mfma_f32_16x16x32_f16.
// Register-staged double-buffered LDS (one barrier per K step), XOR-swizzled 16-B chunks.
// ----------------------------------------------------------------------------------------
enum Epi { kEpiF16 = 0, kEpiGeluF16 = 1, kEpiF32 = 2 };

constexpr int BM = 128, BN = 128, BK = 64;

__device__ __forceinline__ int swz(int row, int chunk) { return row * 8 + (chunk ^ (row & 7)); }

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
  __shared__ half8 lds[2 * NP * BM * (BK / 8)];         // [buf][plane][row][8 chunks]
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

  half8 rg[NP][4];
  auto gload = [&](int kt) {
#pragma unroll
    for (int p = 0; p < NP; ++p)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = tid + 256 * i;
        const int row = c >> 3, ch = c & 7;
        const int r = (p & 1) ? (n0 + row) : min(m0 + row, M - 1);   // planes 0,2: A; 1,3: W
        rg[p][i] = *reinterpret_cast<const half8*>(src[p] + (int64_t)r * K + kt * BK + ch * 8);
      }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      half8* lp = lds + (buf * NP + p) * (BM * 8);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = tid + 256 * i;
        lp[swz(c >> 3, c & 7)] = rg[p][i];
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
    const half8* la = lds + (buf * NP + 0) * (BM * 8);
    const half8* lb = lds + (buf * NP + 1) * (BM * 8);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      half8 af[4], bf[4];
      const int ch = ks * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = la[swz(wr * 64 + i * 16 + (lane & 15), ch)];
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = lb[swz(wc * 64 + j * 16 + (lane & 15), ch)];
      if constexpr (SPLIT) {
        const half8* lal = lds + (buf * NP + 2) * (BM * 8);
        const half8* lbl = lds + (buf * NP + 3) * (BM * 8);
        half8 afl[4], bfl[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) afl[i] = lal[swz(wr * 64 + i * 16 + (lane & 15), ch)];
#pragma unroll
        for (int j = 0; j < 4; ++j) bfl[j] = lbl[swz(wc * 64 + j * 16 + (lane & 15), ch)];
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
          for (int e = 0; e < 8; ++e) {
            h[e] = (_Float16)v[e];
            if constexpr (SPLIT) l[e] = lo_part(v[e], h[e]);
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
// attention (flash style, varlen): grid (ceil(maxlen/64), NH, B), 256 threads; wave w owns
// query rows qb*64 + 16w .. +15 of sequence b, head h. Key blocks of 32 staged in LDS
// (K as [key][dim], V transposed as [dim][key]); S = Q K^T and O += P V on
// v_mfma_f32_16x16x32_f16 (head_dim 32 = one K step); online softmax in fp32.
// qkv: fp16 [T][3H] (Q | K | V, head h = columns h*32 .. +31 of each); ctx: fp16 [T][H].
// ----------------------------------------------------------------------------------------
template <bool SPLIT>
__global__ __launch_bounds__(256) void attn_kernel(const _Float16* __restrict__ qkv,
                                                   const _Float16* __restrict__ qkv_lo,
                                                   const int* __restrict__ cu, float scale,
                                                   _Float16* __restrict__ ctx,
                                                   _Float16* __restrict__ ctx_lo) {
  constexpr int NP = SPLIT ? 2 : 1;
  __shared__ _Float16 kl[NP][32][HD + 8];     // [plane][key][dim] (+8 pad: 80-B rows)
  __shared__ _Float16 vt[NP][HD][32 + 8];     // [plane][dim][key]
  __shared__ _Float16 pl[NP][4][16][32 + 8];  // [plane][wave] P tile [row][key]
  const int b = blockIdx.z, h = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int base = cu[b], len = cu[b + 1] - cu[b];
  const int q0 = blockIdx.x * 64 + wid * 16;
  if (blockIdx.x * 64 >= len) return;
  const int qrow = q0 + (lane & 15);
  const _Float16* planes[2] = {qkv, qkv_lo};

  half8 qf[NP];
  {
    const int r = min(qrow, len - 1);
#pragma unroll
    for (int p = 0; p < NP; ++p)
      qf[p] = *reinterpret_cast<const half8*>(planes[p] + (int64_t)(base + r) * (3 * H) +
                                              h * HD + 8 * (lane >> 4));
  }
  floatx4 o0 = {0.f, 0.f, 0.f, 0.f}, o1 = {0.f, 0.f, 0.f, 0.f};
  float mrow[4], lrow[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    mrow[i] = kNegInf;
    lrow[i] = 0.f;
  }

  for (int kb = 0; kb < len; kb += 32) {
    // stage K and V^T of keys kb .. kb+31 (zeros past the end)
    {
      const int key = tid >> 3, dc = (tid & 7) * 4;
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        half4 kv = {0, 0, 0, 0}, vv = {0, 0, 0, 0};
        if (kb + key < len) {
          const _Float16* src = planes[p] + (int64_t)(base + kb + key) * (3 * H) + h * HD + dc;
          kv = *reinterpret_cast<const half4*>(src + H);
          vv = *reinterpret_cast<const half4*>(src + 2 * H);
        }
        *reinterpret_cast<half4*>(&kl[p][key][dc]) = kv;
#pragma unroll
        for (int e = 0; e < 4; ++e) vt[p][dc + e][key] = vv[e];
      }
    }
    __syncthreads();
    // S = Q K^T for two 16-key tiles
    floatx4 s[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const half8 kf = *reinterpret_cast<const half8*>(&kl[0][16 * j + (lane & 15)][8 * (lane >> 4)]);
      s[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(qf[0], kf, floatx4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      if constexpr (SPLIT) {
        const half8 kfl =
            *reinterpret_cast<const half8*>(&kl[1][16 * j + (lane & 15)][8 * (lane >> 4)]);
        s[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(qf[1], kf, s[j], 0, 0, 0);
        s[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(qf[0], kfl, s[j], 0, 0, 0);
      }
    }
    // lane: rows 4(l>>4)+i, keys kb + 16j + (l&15)
    float p[2][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float mx = kNegInf;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const bool ok = kb + 16 * j + (lane & 15) < len;
        s[j][i] = ok ? s[j][i] * scale : kNegInf;
        mx = fmaxf(mx, s[j][i]);
      }
      mx = fmaxf(mx, xor_lane_f<1>(mx));
      mx = fmaxf(mx, xor_lane_f<2>(mx));
      mx = fmaxf(mx, xor_lane_f<4>(mx));
      mx = fmaxf(mx, xor_lane_f<8>(mx));
      const float mnew = fmaxf(mrow[i], mx);
      const float corr = __expf(mrow[i] - mnew);
      float rsum = 0.f;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        float e = __expf(s[j][i] - mnew);
        if constexpr (!SPLIT) e = (float)(_Float16)e;   // P exactly as the MFMA sees it
        p[j][i] = e;
        rsum += e;
      }
      rsum += xor_lane_f<1>(rsum);
      rsum += xor_lane_f<2>(rsum);
      rsum += xor_lane_f<4>(rsum);
      rsum += xor_lane_f<8>(rsum);
      lrow[i] = lrow[i] * corr + rsum;
      mrow[i] = mnew;
      o0[i] *= corr;
      o1[i] *= corr;
    }
    // P -> LDS (this wave's tile) -> A fragment
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const _Float16 ph = (_Float16)p[j][i];
        pl[0][wid][4 * (lane >> 4) + i][16 * j + (lane & 15)] = ph;
        if constexpr (SPLIT) pl[1][wid][4 * (lane >> 4) + i][16 * j + (lane & 15)] = lo_part(p[j][i], ph);
      }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const half8 pf = *reinterpret_cast<const half8*>(&pl[0][wid][lane & 15][8 * (lane >> 4)]);
    const half8 v0 = *reinterpret_cast<const half8*>(&vt[0][lane & 15][8 * (lane >> 4)]);
    const half8 v1 = *reinterpret_cast<const half8*>(&vt[0][16 + (lane & 15)][8 * (lane >> 4)]);
    if constexpr (SPLIT) {
      const half8 pfl = *reinterpret_cast<const half8*>(&pl[1][wid][lane & 15][8 * (lane >> 4)]);
      const half8 v0l = *reinterpret_cast<const half8*>(&vt[1][lane & 15][8 * (lane >> 4)]);
      const half8 v1l = *reinterpret_cast<const half8*>(&vt[1][16 + (lane & 15)][8 * (lane >> 4)]);
      o0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(pfl, v0, o0, 0, 0, 0);
      o1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(pfl, v1, o1, 0, 0, 0);
      o0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(pf, v0l, o0, 0, 0, 0);
      o1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(pf, v1l, o1, 0, 0, 0);
    }
    o0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(pf, v0, o0, 0, 0, 0);
    o1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(pf, v1, o1, 0, 0, 0);
    __syncthreads();
  }
  // O: lane rows 4(l>>4)+i, dims (l&15) and 16 + (l&15)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = q0 + 4 * (lane >> 4) + i;
    if (r < len) {
      const float inv = 1.0f / lrow[i];
      const int64_t off = (int64_t)(base + r) * H + h * HD;
      const float a = o0[i] * inv, c = o1[i] * inv;
      const _Float16 ah = (_Float16)a, ch = (_Float16)c;
      ctx[off + (lane & 15)] = ah;
      ctx[off + 16 + (lane & 15)] = ch;
      if constexpr (SPLIT) {
        ctx_lo[off + (lane & 15)] = lo_part(a, ah);
        ctx_lo[off + 16 + (lane & 15)] = lo_part(c, ch);
      }
    }
  }
}

// ----------------------------------------------------------------------------------------
// heads
// ----------------------------------------------------------------------------------------
// bge (sentence-transformers Pooling(cls) + Normalize): out[b] = x[cls] / max(||x[cls]||, 1e-12)
__global__ __launch_bounds__(64) void cls_normalize_kernel(const float* __restrict__ x,
                                                           const int* __restrict__ cu,
                                                           float* __restrict__ out) {
  const int b = blockIdx.x, lane = threadIdx.x;
  const float* r = x + (int64_t)cu[b] * H;
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
  for (int c = tid; c < H; c += 256) cls[c] = x[(int64_t)cu[b] * H + c];
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
