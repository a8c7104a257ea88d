// scan_kernels.hip — in-HBM flat cosine index for gfx950 (MI355X): upsert, query prep,
// brute-force MFMA scan with a per-wave top-k, and the exact-rescoring merges.
//
// Replaces the Qdrant server's COSINE collection behind QdrantClient.query_points / upsert
// (reference main.py:215-239, ingest.py:148-175).
//
// Storage layout in HBM ("tile16"): rows are grouped in tiles of 16; a tile is stored in the
// exact order the v_mfma_f32_16x16x32_f16 A-operand wants it, so every wave-wide load of the
// scan is one perfectly coalesced 1 KiB dwordx4 (16 B/lane x 64 lanes):
//     tile t, k-step s (32 dims), lane l = h*16 + r  ->  8 halves  row 16t+r, dims 32s+8h..+7
//     half8 index = t*(D/32)*64 + s*64 + l
// The query batch (32 queries = two 16-wide MFMA column tiles) is prepared into the matching
// B-operand order and kept in VGPRs for the whole scan.
#include "device_common.hpp"

namespace ragmi {

constexpr int kTileRows = 16;
constexpr int kQ = 32;            // queries per pass
constexpr int kKS = 32;           // candidates kept per (wave, query)
constexpr int kP = 8;             // pending slots per (lane, query tile)
constexpr int kWavesPerWG = 4;
constexpr int kLdsPerWave = 4096; // dwords: keep_s[32][32] keep_i[32][32] pend_s[2][8][64] pend_i[2][8][64]

template <int D>
__host__ __device__ constexpr int steps() { return D / 32; }

// ----------------------------------------------------------------------------------------
// upsert: one wave per vector. Canonical normalisation -> fp16 (RNE) -> tile16 slot.
// ----------------------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(64) void upsert_kernel(const float* __restrict__ vecs,
                                                    const int64_t* __restrict__ rows,
                                                    const uint32_t* __restrict__ tags_in,
                                                    half8* __restrict__ corpus,
                                                    uint32_t* __restrict__ tags, int64_t n,
                                                    int64_t cap_rows) {
  const int64_t i = blockIdx.x;
  if (i >= n) return;
  const int lane = threadIdx.x;
  const int64_t row = rows[i];
  if (row < 0 || row >= cap_rows) return;  // host validates; never write out of bounds
  const float* x = vecs + i * D;
  const double norm = sqrt(canon_sumsq<D>(x, lane));
  const int64_t t = row >> 4;
  const int r = (int)(row & 15);
  for (int c = lane; c < D / 8; c += 64) {
    half8 h;
#pragma unroll
    for (int j = 0; j < 8; ++j) h[j] = (_Float16)canon_scale(x[8 * c + j], norm);
    const int s = c >> 2, hh = c & 3;
    corpus[t * (steps<D>() * 64) + s * 64 + hh * 16 + r] = h;
  }
  if (lane == 0) tags[row] = tags_in ? tags_in[i] : 0u;
}

// ----------------------------------------------------------------------------------------
// query prep: one wave per query slot (32 slots; slots >= B are zero).
//   qn    [32][D] fp32 canonical-normalised queries (exact rescoring operand)
//   qfrag [2][D/32][64] half8: B-operand fragments, lane l -> query 16*qt + (l&15),
//         dims 32s + 8(l>>4) .. +7
//   filt  [32][2] (tag mask, tag value) per query slot
// ----------------------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(64) void qprep_kernel(const float* __restrict__ q, int B,
                                                   const uint32_t* __restrict__ filt_in,
                                                   float* __restrict__ qn,
                                                   half8* __restrict__ qfrag,
                                                   uint32_t* __restrict__ filt) {
  const int b = blockIdx.x;
  const int lane = threadIdx.x;
  const bool live = b < B;
  if (lane == 0) {
    // per-query payload filter (mask, value); padding / unfiltered queries match every row
    filt[2 * b] = (live && filt_in) ? filt_in[2 * b] : 0u;
    filt[2 * b + 1] = (live && filt_in) ? filt_in[2 * b + 1] : 0u;
  }
  double norm = 0.0;
  if (live) norm = sqrt(canon_sumsq<D>(q + (int64_t)b * D, lane));
  const int qt = b >> 4, c16 = b & 15;
  for (int c = lane; c < D / 8; c += 64) {
    half8 h;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float y = live ? canon_scale(q[(int64_t)b * D + 8 * c + j], norm) : 0.0f;
      qn[b * D + 8 * c + j] = y;
      h[j] = (_Float16)y;
    }
    const int s = c >> 2, hh = c & 3;
    qfrag[(qt * steps<D>() + s) * 64 + hh * 16 + c16] = h;
  }
}

// ----------------------------------------------------------------------------------------
// scan: each wave streams a contiguous range of tiles, MFMA-scores them against the 32
// queries, and keeps its own top-32 per query.
//
// Per tile and query tile qt the accumulator gives lane l the scores of query 16qt+(l&15)
// for rows 16t + 4(l>>4) + {0..3}. Top-k bookkeeping per wave:
//   thr_qt (VGPR)  current 32nd-best score of the lane's query (-inf until 32 are known)
//   pending        lane-private LDS slots [qt][slot][lane] for scores > thr
//   keep           LDS [32 queries][32] sorted best-first
// A query whose lanes hold > kP-4 pending entries is flushed: its 32 kept + 4x8 pending
// entries are bitonic-sorted across the wave and the best 32 kept (thr := 32nd). Rows are
// visited in increasing order per wave, so a later row never beats an equal-scored earlier
// one and the strict `> thr` filter is exact for the (score desc, row asc) order.
// ----------------------------------------------------------------------------------------
struct WaveTopK {
  float* keep_s;
  int* keep_i;
  float* pend_s;
  int* pend_i;
};

__device__ __forceinline__ void lds_fence() {
  // LDS ops of one wave complete in order; this stops the compiler from reordering
  // the cross-lane LDS traffic around the flush.
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

__device__ __forceinline__ void flush_query(const WaveTopK& w, int q, int lane, float& thr0,
                                            int& cnt0, float& thr1, int& cnt1) {
  const int qt = q >> 4, c = q & 15;
  float s;
  int id;
  int pidx = 0;
  if (lane < 32) {
    s = w.keep_s[q * kKS + lane];
    id = w.keep_i[q * kKS + lane];
  } else {
    const int pl = lane - 32;
    const int src = c + 16 * (pl >> 3);
    const int slot = pl & 7;
    pidx = (qt * kP + slot) * 64 + src;
    s = w.pend_s[pidx];
    id = w.pend_i[pidx];
  }
  lds_fence();
  bitonic_sort64(s, id, lane);
  if (lane < 32) {
    w.keep_s[q * kKS + lane] = s;
    w.keep_i[q * kKS + lane] = id;
  } else {
    w.pend_s[pidx] = kNegInf;
    w.pend_i[pidx] = kIdNone32;
  }
  lds_fence();
  const float nt = __shfl(s, 31, 64);
  if ((lane & 15) == c) {
    if (qt == 0) {
      thr0 = nt;
      cnt0 = 0;
    } else {
      thr1 = nt;
      cnt1 = 0;
    }
  }
}

__device__ __forceinline__ void flush_mask(const WaveTopK& w, uint64_t b, int qt, int lane,
                                           float& thr0, int& cnt0, float& thr1, int& cnt1) {
  uint32_t m = (uint32_t)((b | (b >> 16) | (b >> 32) | (b >> 48)) & 0xffffu);
  while (m) {
    const int c = __builtin_ctz(m);
    m &= m - 1;
    flush_query(w, qt * 16 + c, lane, thr0, cnt0, thr1, cnt1);
  }
}

template <int D, bool FILTER>
__global__ __launch_bounds__(256, 2) void scan_kernel(
    const half8* __restrict__ corpus, const uint32_t* __restrict__ tags,
    const uint32_t* __restrict__ filt, const half8* __restrict__ qfrag, int n_rows, int n_tiles,
    float* __restrict__ part_s, int* __restrict__ part_i) {
  constexpr int S = steps<D>();
  __shared__ int lds[kWavesPerWG * kLdsPerWave];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  WaveTopK w;
  w.keep_s = reinterpret_cast<float*>(lds + wid * kLdsPerWave);
  w.keep_i = lds + wid * kLdsPerWave + 1024;
  w.pend_s = reinterpret_cast<float*>(lds + wid * kLdsPerWave + 2048);
  w.pend_i = lds + wid * kLdsPerWave + 3072;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    w.keep_s[lane + 64 * j] = kNegInf;
    w.keep_i[lane + 64 * j] = kIdNone32;
    w.pend_s[lane + 64 * j] = kNegInf;
    w.pend_i[lane + 64 * j] = kIdNone32;
  }
  lds_fence();

  const int gw = blockIdx.x * kWavesPerWG + wid;
  const int nw = gridDim.x * kWavesPerWG;
  const int t_begin = (int)((int64_t)n_tiles * gw / nw);
  const int t_end = (int)((int64_t)n_tiles * (gw + 1) / nw);

  half8 q0[S], q1[S];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    q0[s] = qfrag[s * 64 + lane];
    q1[s] = qfrag[(S + s) * 64 + lane];
  }

  float thr0 = kNegInf, thr1 = kNegInf;
  int cnt0 = 0, cnt1 = 0;
  const int rsub = 4 * (lane >> 4);
  uint32_t fm0 = 0, fv0 = 0, fm1 = 0, fv1 = 0;
  if constexpr (FILTER) {
    fm0 = filt[2 * (lane & 15)];
    fv0 = filt[2 * (lane & 15) + 1];
    fm1 = filt[2 * (16 + (lane & 15))];
    fv1 = filt[2 * (16 + (lane & 15)) + 1];
  }

  auto process = [&](const half8(&a)[S], int t) {
    floatx4 acc0 = {0.f, 0.f, 0.f, 0.f};
    floatx4 acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < S; ++s) {
      acc0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[s], q0[s], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[s], q1[s], acc1, 0, 0, 0);
    }
    const int rbase = t * kTileRows + rsub;
    uint4 tg = {0u, 0u, 0u, 0u};
    if constexpr (FILTER) tg = *reinterpret_cast<const uint4*>(tags + rbase);
    float v0[4], v1[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool ok = (rbase + r) < n_rows;
      bool ok0 = ok, ok1 = ok;
      if constexpr (FILTER) {
        const uint32_t tr = r == 0 ? tg.x : r == 1 ? tg.y : r == 2 ? tg.z : tg.w;
        ok0 = ok0 && ((tr & fm0) == fv0);
        ok1 = ok1 && ((tr & fm1) == fv1);
      }
      v0[r] = ok0 ? acc0[r] : kNegInf;
      v1[r] = ok1 ? acc1[r] : kNegInf;
    }
    const float m0 = fmaxf(fmaxf(v0[0], v0[1]), fmaxf(v0[2], v0[3]));
    const float m1 = fmaxf(fmaxf(v1[0], v1[1]), fmaxf(v1[2], v1[3]));
    if (__ballot((m0 > thr0) || (m1 > thr1))) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (v0[r] > thr0) {
          w.pend_s[cnt0 * 64 + lane] = v0[r];
          w.pend_i[cnt0 * 64 + lane] = rbase + r;
          ++cnt0;
        }
        if (v1[r] > thr1) {
          w.pend_s[(kP + cnt1) * 64 + lane] = v1[r];
          w.pend_i[(kP + cnt1) * 64 + lane] = rbase + r;
          ++cnt1;
        }
      }
      lds_fence();
      const uint64_t b0 = __ballot(cnt0 > kP - 4);
      const uint64_t b1 = __ballot(cnt1 > kP - 4);
      if (b0) flush_mask(w, b0, 0, lane, thr0, cnt0, thr1, cnt1);
      if (b1) flush_mask(w, b1, 1, lane, thr0, cnt0, thr1, cnt1);
    }
  };

  if (t_begin < t_end) {
    half8 a0[S], a1[S];
    const half8* base = corpus + lane;
    auto load = [&](half8(&a)[S], int t) {
      const half8* p = base + (int64_t)t * (S * 64);
#pragma unroll
      for (int s = 0; s < S; ++s) a[s] = p[s * 64];
    };
    load(a0, t_begin);
    int t = t_begin;
    while (true) {
      load(a1, min(t + 1, t_end - 1));
      process(a0, t);
      if (++t >= t_end) break;
      load(a0, min(t + 1, t_end - 1));
      process(a1, t);
      if (++t >= t_end) break;
    }
  }

  // final flush of every query with pending entries
  {
    const uint64_t b0 = __ballot(cnt0 > 0);
    const uint64_t b1 = __ballot(cnt1 > 0);
    if (b0) flush_mask(w, b0, 0, lane, thr0, cnt0, thr1, cnt1);
    if (b1) flush_mask(w, b1, 1, lane, thr0, cnt0, thr1, cnt1);
  }
  float* ps = part_s + (int64_t)gw * (kQ * kKS);
  int* pi = part_i + (int64_t)gw * (kQ * kKS);
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    ps[lane + 64 * j] = w.keep_s[lane + 64 * j];
    pi[lane + 64 * j] = w.keep_i[lane + 64 * j];
  }
}

// ----------------------------------------------------------------------------------------
// merge stage 1: grid (groups, Bq); one wave merges up to `per_group` sorted wave lists of
// one query into its top-32 (approximate MFMA scores).
// ----------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void merge1_kernel(const float* __restrict__ part_s,
                                                    const int* __restrict__ part_i,
                                                    int n_lists, int per_group,
                                                    float* __restrict__ mid_s,
                                                    int* __restrict__ mid_i) {
  const int g = blockIdx.x, b = blockIdx.y, lane = threadIdx.x;
  const int l0 = g * per_group;
  const int l1 = min(l0 + per_group, n_lists);
  float s = kNegInf;
  int id = kIdNone32;
  if (lane < 32 && l0 < n_lists) {
    s = part_s[((int64_t)l0 * kQ + b) * kKS + lane];
    id = part_i[((int64_t)l0 * kQ + b) * kKS + lane];
  }
  for (int l = l0 + 1; l < l1; ++l) {
    if (lane >= 32) {
      s = part_s[((int64_t)l * kQ + b) * kKS + (63 - lane)];
      id = part_i[((int64_t)l * kQ + b) * kKS + (63 - lane)];
    }
    bitonic_merge64(s, id, lane);
  }
  if (lane < 32) {
    mid_s[((int64_t)g * kQ + b) * kKS + lane] = s;
    mid_i[((int64_t)g * kQ + b) * kKS + lane] = id;
  }
}

// ----------------------------------------------------------------------------------------
// merge stage 2: one wave per query. Merge the group lists -> approximate top-32, then
// rescore each candidate exactly: fp32( sequential fp64 fma over k of fp16 row x fp32
// normalised query ), sort by (exact score desc, row asc) and emit the top k.
// ----------------------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(64) void merge2_kernel(const float* __restrict__ mid_s,
                                                    const int* __restrict__ mid_i,
                                                    int n_groups,
                                                    const half8* __restrict__ corpus,
                                                    const float* __restrict__ qn, int k,
                                                    int64_t id_offset,
                                                    float* __restrict__ out_s,
                                                    int64_t* __restrict__ out_i) {
  constexpr int S = steps<D>();
  const int b = blockIdx.x, lane = threadIdx.x;
  float s = kNegInf;
  int id = kIdNone32;
  if (lane < 32) {
    s = mid_s[(int64_t)b * kKS + lane];
    id = mid_i[(int64_t)b * kKS + lane];
  }
  for (int g = 1; g < n_groups; ++g) {
    if (lane >= 32) {
      s = mid_s[((int64_t)g * kQ + b) * kKS + (63 - lane)];
      id = mid_i[((int64_t)g * kQ + b) * kKS + (63 - lane)];
    }
    bitonic_merge64(s, id, lane);
  }
  // exact rescoring of the approximate top-32
  float es = kNegInf;
  int eid = kIdNone32;
  if (lane < 32 && s != kNegInf) {
    const int64_t t = id >> 4;
    const int r = id & 15;
    const half8* row = corpus + t * (S * 64) + r;
    const float* qq = qn + b * D;
    double acc = 0.0;
    for (int c = 0; c < D / 8; ++c) {
      const half8 h = row[(c >> 2) * 64 + (c & 3) * 16];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc = fma((double)h[j], (double)qq[8 * c + j], acc);
    }
    es = (float)acc;
    eid = id;
  }
  bitonic_sort64(es, eid, lane);
  if (lane < k) {
    const bool ok = es != kNegInf;
    out_s[(int64_t)b * k + lane] = es;
    out_i[(int64_t)b * k + lane] = ok ? (int64_t)eid + id_offset : (int64_t)-1;
  }
}

// ----------------------------------------------------------------------------------------
// merge of exact per-shard lists (after the RCCL all-gather): [n_lists][B][k] -> [B][k]
// ----------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void merge_exact_kernel(const float* __restrict__ in_s,
                                                         const int64_t* __restrict__ in_i,
                                                         int n_lists, int B, int k,
                                                         float* __restrict__ out_s,
                                                         int64_t* __restrict__ out_i) {
  const int b = blockIdx.x, lane = threadIdx.x;
  auto fetch = [&](int l, int pos, float& s, int64_t& id) {
    s = kNegInf;
    id = INT64_MAX;
    if (l < n_lists && pos < k) {
      const int64_t off = ((int64_t)l * B + b) * k + pos;
      const int64_t v = in_i[off];
      if (v >= 0) {
        s = in_s[off];
        id = v;
      }
    }
  };
  float s;
  int64_t id;
  if (lane < 32)
    fetch(0, lane, s, id);
  else {
    s = kNegInf;
    id = INT64_MAX;
  }
  for (int l = 1; l < n_lists; ++l) {
    if (lane >= 32) fetch(l, 63 - lane, s, id);
    bitonic_merge64(s, id, lane);
  }
  if (lane < k) {
    const bool ok = s != kNegInf;
    out_s[(int64_t)b * k + lane] = s;
    out_i[(int64_t)b * k + lane] = ok ? id : (int64_t)-1;
  }
}

// ----------------------------------------------------------------------------------------
// export: tile16 -> row-major fp16 (one thread per 8-half chunk)
// ----------------------------------------------------------------------------------------
template <int D>
__global__ void export_kernel(const half8* __restrict__ corpus, int64_t row0, int64_t n,
                              half8* __restrict__ out) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n * (D / 8)) return;
  const int64_t i = idx / (D / 8);
  const int c = (int)(idx % (D / 8));
  const int64_t row = row0 + i;
  const int64_t t = row >> 4;
  const int r = (int)(row & 15);
  out[idx] = corpus[t * (steps<D>() * 64) + (c >> 2) * 64 + (c & 3) * 16 + r];
}

}  // namespace ragmi
