/*
 * oracle/scan_ref.c — CPU restatement of the reference's COSINE search path.
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker. The product path
 * (libragmi.so) never links, loads or falls back to it.
 *
 * What it restates (reference pythonmailer/financial-rag-system, /root/reference):
 *   - database.py:111-143 / ingest.py:86-96: collection of 384-d vectors, Distance.COSINE.
 *   - ingest.py:148-175: PointStruct upsert; same id => overwrite (handled by the host layer).
 *   - main.py:215-239: query_points(query=vec, limit=15, query_filter=Filter(must=[ticker ==
 *     T.upper(), (document_type == D.upper())])) -> points sorted by score desc.
 *   - Qdrant COSINE semantics [external, qdrant/qdrant:latest, docker-compose.yml:22; not in
 *     the container]: vectors are L2-normalised at insert, the query is normalised, and the
 *     score is the dot product. The reference pins no numbers for this path (tests.py runs
 *     TESTING stubs only, main.py:216), so this restatement is "parity unpinned" against the
 *     reference itself; it is pinned against an independent numpy float64 formulation in
 *     tests/test_oracle_scan.py and the committed fixtures in tests/golden/.
 *
 * Canonical arithmetic (shared bit-for-bit with the HIP path):
 *   sumsq   : 64 lane partials, lane l sums chunks c = l, l+64, ... (8 elems each) with
 *             fp64 fma in order; xor-butterfly d = 32..1 (v[i] += v[i^d]); take v[0].
 *   norm    : sqrt(sumsq) (fp64, correctly rounded)
 *   y_k     : fp32(fp64(x_k) / norm), 0 if norm == 0
 *   stored  : fp16_rne(y_k)            (fp16 storage; fp32 storage keeps y_k itself:
 *                                        Qdrant's default Float32 vectors, database.py:124-130)
 *   score   : fp32( canonical fp64 sum of fp64(c_k) * fp64(qn_k) ), c = the stored row (fp16
 *             or fp32): 64 lane partials
 *             (chunks of 8, fp64 fma in order) + xor-butterfly, exactly as for sumsq
 *   order   : score desc, row asc; rows with (tag & mask) != value are excluded when filtering.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_API __attribute__((visibility("default")))

/* IEEE binary32 -> binary16, round to nearest even, with subnormals, inf and nan. */
ORC_API uint16_t orc_f32_to_f16(float f) {
  uint32_t x;
  memcpy(&x, &f, 4);
  const uint32_t sign = (x >> 16) & 0x8000u;
  const uint32_t exp = (x >> 23) & 0xffu;
  uint32_t man = x & 0x7fffffu;
  if (exp == 0xffu) return (uint16_t)(sign | 0x7c00u | (man ? 0x200u | (man >> 13) : 0u));
  int e = (int)exp - 127 + 15;
  if (e >= 31) return (uint16_t)(sign | 0x7c00u);
  if (e <= 0) {
    if (e < -10) return (uint16_t)sign;
    man |= 0x800000u;
    const int shift = 14 - e; /* 24-bit mantissa -> subnormal 10-bit field */
    uint32_t h = man >> shift;
    const uint32_t rem = man & ((1u << shift) - 1u);
    const uint32_t half = 1u << (shift - 1);
    if (rem > half || (rem == half && (h & 1u))) ++h;
    return (uint16_t)(sign | h);
  }
  uint32_t h = ((uint32_t)e << 10) | (man >> 13);
  const uint32_t rem = man & 0x1fffu;
  if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) ++h; /* may carry into exponent: ok */
  return (uint16_t)(sign | h);
}

ORC_API float orc_f16_to_f32(uint16_t h) {
  const uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
  const uint32_t exp = (h >> 10) & 0x1fu;
  uint32_t man = h & 0x3ffu;
  uint32_t x;
  if (exp == 0) {
    if (man == 0) {
      x = sign;
    } else {
      int e = -1;
      do {
        ++e;
        man <<= 1;
      } while (!(man & 0x400u));
      x = sign | ((uint32_t)(127 - 15 - e) << 23) | ((man & 0x3ffu) << 13);
    }
  } else if (exp == 31) {
    x = sign | 0x7f800000u | (man << 13);
  } else {
    x = sign | ((exp - 15 + 127) << 23) | (man << 13);
  }
  float f;
  memcpy(&f, &x, 4);
  return f;
}

ORC_API double orc_canon_sumsq(const float* x, int D) {
  double v[64];
  for (int l = 0; l < 64; ++l) {
    double acc = 0.0;
    for (int c = l; c < D / 8; c += 64)
      for (int j = 0; j < 8; ++j) {
        const double a = (double)x[8 * c + j];
        acc = fma(a, a, acc);
      }
    v[l] = acc;
  }
  for (int d = 32; d > 0; d >>= 1) {
    double w[64];
    for (int i = 0; i < 64; ++i) w[i] = v[i] + v[i ^ d];
    memcpy(v, w, sizeof(v));
  }
  return v[0];
}

/* y = canonical normalised fp32 vector; h (optional) = its fp16 bits. */
ORC_API void orc_normalize(const float* x, int D, float* y, uint16_t* h) {
  const double norm = sqrt(orc_canon_sumsq(x, D));
  for (int k = 0; k < D; ++k) {
    const float v = norm > 0.0 ? (float)((double)x[k] / norm) : 0.0f;
    y[k] = v;
    if (h) h[k] = orc_f32_to_f16(v);
  }
}

/* Stored rows for n input vectors: out16 [n][D]. */
ORC_API void orc_encode_rows(const float* x, int64_t n, int D, uint16_t* out16) {
  float* y = (float*)malloc(sizeof(float) * (size_t)D);
  for (int64_t i = 0; i < n; ++i) orc_normalize(x + i * D, D, y, out16 + i * D);
  free(y);
}

/* fp32 storage: the canonical normalised fp32 rows [n][D]. */
ORC_API void orc_encode_rows32(const float* x, int64_t n, int D, float* out32) {
  for (int64_t i = 0; i < n; ++i) orc_normalize(x + i * D, D, out32 + i * D, NULL);
}

/* Canonical exact score: 64 lane partials (lane l: chunks c = l, l+64, ... of 8 elements,
 * fp64 fma in order), xor-butterfly d = 32..1, v[0] rounded to fp32 — the order of the HIP
 * select kernel's exact_score_wave. Row = fp16 bits (c16) or, when c16 is NULL, fp32 (c32). */
static float exact_score_any(const uint16_t* c16, const float* c32, const float* qn, int D) {
  double v[64];
  for (int l = 0; l < 64; ++l) {
    double acc = 0.0;
    for (int c = l; c < D / 8; c += 64)
      for (int j = 0; j < 8; ++j) {
        const double r = c16 ? (double)orc_f16_to_f32(c16[8 * c + j]) : (double)c32[8 * c + j];
        acc = fma(r, (double)qn[8 * c + j], acc);
      }
    v[l] = acc;
  }
  for (int d = 32; d > 0; d >>= 1) {
    double w[64];
    for (int i = 0; i < 64; ++i) w[i] = v[i] + v[i ^ d];
    memcpy(v, w, sizeof(v));
  }
  return (float)v[0];
}

ORC_API float orc_exact_score(const uint16_t* c16, const float* qn, int D) {
  return exact_score_any(c16, NULL, qn, D);
}

ORC_API float orc_exact_score32(const float* c32, const float* qn, int D) {
  return exact_score_any(NULL, c32, qn, D);
}

static int better(float as, int64_t ai, float bs, int64_t bi) {
  return (as > bs) || (as == bs && ai < bi);
}

/* Exact top-k over a row-major fp16 (corpus16) or, when corpus16 is NULL, fp32 (corpus32)
 * corpus. queries [B][D] fp32 (raw, normalised here). out_s [B][k], out_i [B][k] (-1 / -inf
 * when fewer than k rows qualify). */
static void search_any(const uint16_t* corpus16, const float* corpus32, const uint32_t* tags,
                       int64_t n_rows, int D, const float* queries, int B, int k,
                       int use_filter, uint32_t mask, uint32_t value, float* out_s,
                       int64_t* out_i) {
  float* qn = (float*)malloc(sizeof(float) * (size_t)D);
  float* bs = (float*)malloc(sizeof(float) * (size_t)k);
  int64_t* bi = (int64_t*)malloc(sizeof(int64_t) * (size_t)k);
  for (int b = 0; b < B; ++b) {
    orc_normalize(queries + (int64_t)b * D, D, qn, NULL);
    for (int j = 0; j < k; ++j) {
      bs[j] = -INFINITY;
      bi[j] = -1;
    }
    for (int64_t r = 0; r < n_rows; ++r) {
      if (use_filter && (tags[r] & mask) != value) continue;
      const float s = exact_score_any(corpus16 ? corpus16 + r * D : NULL,
                                      corpus16 ? NULL : corpus32 + r * D, qn, D);
      if (bi[k - 1] >= 0 && !better(s, r, bs[k - 1], bi[k - 1])) continue;
      int p = k - 1;
      while (p > 0 && (bi[p - 1] < 0 || better(s, r, bs[p - 1], bi[p - 1]))) {
        bs[p] = bs[p - 1];
        bi[p] = bi[p - 1];
        --p;
      }
      bs[p] = s;
      bi[p] = r;
    }
    for (int j = 0; j < k; ++j) {
      out_s[(int64_t)b * k + j] = bs[j];
      out_i[(int64_t)b * k + j] = bi[j];
    }
  }
  free(qn);
  free(bs);
  free(bi);
}

ORC_API void orc_search(const uint16_t* corpus16, const uint32_t* tags, int64_t n_rows, int D,
                        const float* queries, int B, int k, int use_filter, uint32_t mask,
                        uint32_t value, float* out_s, int64_t* out_i) {
  search_any(corpus16, NULL, tags, n_rows, D, queries, B, k, use_filter, mask, value, out_s,
             out_i);
}

ORC_API void orc_search32(const float* corpus32, const uint32_t* tags, int64_t n_rows, int D,
                          const float* queries, int B, int k, int use_filter, uint32_t mask,
                          uint32_t value, float* out_s, int64_t* out_i) {
  search_any(NULL, corpus32, tags, n_rows, D, queries, B, k, use_filter, mask, value, out_s,
             out_i);
}

/* Exact rescoring of given candidate rows (used by the fast numpy oracle):
 * cand [B][m] row ids (-1 = none) -> sc [B][m]. qn is already normalised [B][D].
 * corpus16 NULL: fp32 rows corpus32. */
static void rescore_any(const uint16_t* corpus16, const float* corpus32, int D, const float* qn,
                        int B, const int64_t* cand, int m, float* sc) {
  for (int b = 0; b < B; ++b)
    for (int j = 0; j < m; ++j) {
      const int64_t r = cand[(int64_t)b * m + j];
      sc[(int64_t)b * m + j] =
          r < 0 ? -INFINITY
                : exact_score_any(corpus16 ? corpus16 + r * D : NULL,
                                  corpus16 ? NULL : corpus32 + r * D, qn + (int64_t)b * D, D);
    }
}

ORC_API void orc_rescore(const uint16_t* corpus16, int D, const float* qn, int B,
                         const int64_t* cand, int m, float* sc) {
  rescore_any(corpus16, NULL, D, qn, B, cand, m, sc);
}

ORC_API void orc_rescore32(const float* corpus32, int D, const float* qn, int B,
                           const int64_t* cand, int m, float* sc) {
  rescore_any(NULL, corpus32, D, qn, B, cand, m, sc);
}
