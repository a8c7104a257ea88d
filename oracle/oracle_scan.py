"""oracle/oracle_scan.py — numpy + ctypes front end of the CPU search restatement.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the checker. The product path (ragmi / libragmi.so) never imports it.

Restates the reference's COSINE search (reference main.py:215-239 query_points with
limit=15 and the ticker/document_type `must` filter; ingest.py:86-96,148-175 collection +
upsert; Qdrant COSINE = normalise at insert, dot product) with the canonical arithmetic of
oracle/scan_ref.c (see its header). Parity against the reference itself is UNPINNED: the
reference's only test file (tests.py) runs TESTING stubs (main.py:216) and pins no numbers,
and neither Qdrant nor sentence-transformers is installed here.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "liboracle_scan.so")
_lib = None


def build() -> str:
    """Compile scan_ref.c -> liboracle_scan.so (gcc; no reference sources involved)."""
    src = os.path.join(_HERE, "scan_ref.c")
    if not os.path.exists(_SO) or os.path.getmtime(_SO) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", _HERE, "liboracle_scan.so"])
    return _SO


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_SO)
        f32p = ctypes.POINTER(ctypes.c_float)
        u16p = ctypes.POINTER(ctypes.c_uint16)
        u32p = ctypes.POINTER(ctypes.c_uint32)
        i64p = ctypes.POINTER(ctypes.c_int64)
        L.orc_canon_sumsq.restype = ctypes.c_double
        L.orc_canon_sumsq.argtypes = [f32p, ctypes.c_int]
        L.orc_encode_rows.argtypes = [f32p, ctypes.c_int64, ctypes.c_int, u16p]
        L.orc_normalize.argtypes = [f32p, ctypes.c_int, f32p, u16p]
        L.orc_search.argtypes = [u16p, u32p, ctypes.c_int64, ctypes.c_int, f32p, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32,
                                 f32p, i64p]
        L.orc_rescore.argtypes = [u16p, ctypes.c_int, f32p, ctypes.c_int, i64p, ctypes.c_int,
                                  f32p]
        L.orc_encode_rows32.argtypes = [f32p, ctypes.c_int64, ctypes.c_int, f32p]
        L.orc_search32.argtypes = [f32p, u32p, ctypes.c_int64, ctypes.c_int, f32p, ctypes.c_int,
                                   ctypes.c_int, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32,
                                   f32p, i64p]
        L.orc_rescore32.argtypes = [f32p, ctypes.c_int, f32p, ctypes.c_int, i64p, ctypes.c_int,
                                    f32p]
        L.orc_f32_to_f16.restype = ctypes.c_uint16
        L.orc_f32_to_f16.argtypes = [ctypes.c_float]
        _lib = L
    return _lib


def _p(a, ct):
    return a.ctypes.data_as(ctypes.POINTER(ct))


def encode_rows(x: np.ndarray) -> np.ndarray:
    """fp32 [n, D] input vectors -> stored fp16 rows (as uint16 bits), canonical normalise."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    n, d = x.shape
    out = np.empty((n, d), dtype=np.uint16)
    lib().orc_encode_rows(_p(x, ctypes.c_float), n, d, _p(out, ctypes.c_uint16))
    return out


def encode_rows32(x: np.ndarray) -> np.ndarray:
    """fp32 storage: the canonical normalised fp32 rows [n, D] (Qdrant's Float32 vectors)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    n, d = x.shape
    out = np.empty((n, d), dtype=np.float32)
    lib().orc_encode_rows32(_p(x, ctypes.c_float), n, d, _p(out, ctypes.c_float))
    return out


def _rows_f32(corpus: np.ndarray, r0: int, n: int) -> np.ndarray:
    """Rows [r0, r0+n) of a stored corpus as fp32: fp16 bits (uint16) or fp32 storage."""
    c = corpus[r0:r0 + n]
    return c.view(np.float16).astype(np.float32) if c.dtype == np.uint16 else c


def normalize(x: np.ndarray) -> np.ndarray:
    """Canonical fp32 normalisation of each row of x [n, D]."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.empty_like(x)
    for i in range(x.shape[0]):
        lib().orc_normalize(_p(x[i], ctypes.c_float), x.shape[1], _p(out[i], ctypes.c_float),
                            None)
    return out


def search(corpus16: np.ndarray, queries: np.ndarray, k: int, tags: np.ndarray | None = None,
           mask: int = 0, value: int = 0, use_filter: bool = False):
    """Exact top-k by (score desc, row asc). corpus16: uint16 fp16 bits [N, D] (fp16 storage)
    or float32 [N, D] (fp32 storage, encode_rows32)."""
    if corpus16.dtype == np.float32:
        return _search32(corpus16, queries, k, tags, mask, value, use_filter)
    corpus16 = np.ascontiguousarray(corpus16, dtype=np.uint16)
    queries = np.ascontiguousarray(queries, dtype=np.float32)
    n, d = corpus16.shape
    b = queries.shape[0]
    if tags is None:
        tags = np.zeros(max(n, 1), dtype=np.uint32)
    tags = np.ascontiguousarray(tags, dtype=np.uint32)
    out_s = np.empty((b, k), dtype=np.float32)
    out_i = np.empty((b, k), dtype=np.int64)
    lib().orc_search(_p(corpus16, ctypes.c_uint16), _p(tags, ctypes.c_uint32), n, d,
                     _p(queries, ctypes.c_float), b, k, int(use_filter), mask, value,
                     _p(out_s, ctypes.c_float), _p(out_i, ctypes.c_int64))
    return out_s, out_i


def _search32(corpus32, queries, k, tags, mask, value, use_filter):
    corpus32 = np.ascontiguousarray(corpus32, dtype=np.float32)
    queries = np.ascontiguousarray(queries, dtype=np.float32)
    n, d = corpus32.shape
    b = queries.shape[0]
    if tags is None:
        tags = np.zeros(max(n, 1), dtype=np.uint32)
    tags = np.ascontiguousarray(tags, dtype=np.uint32)
    out_s = np.empty((b, k), dtype=np.float32)
    out_i = np.empty((b, k), dtype=np.int64)
    lib().orc_search32(_p(corpus32, ctypes.c_float), _p(tags, ctypes.c_uint32), n, d,
                       _p(queries, ctypes.c_float), b, k, int(use_filter), mask, value,
                       _p(out_s, ctypes.c_float), _p(out_i, ctypes.c_int64))
    return out_s, out_i


def rescore(corpus16: np.ndarray, qn: np.ndarray, cand: np.ndarray) -> np.ndarray:
    if corpus16.dtype == np.float32:
        c32 = np.ascontiguousarray(corpus16)
        qn = np.ascontiguousarray(qn, dtype=np.float32)
        cand = np.ascontiguousarray(cand, dtype=np.int64)
        b, m = cand.shape
        sc = np.empty((b, m), dtype=np.float32)
        lib().orc_rescore32(_p(c32, ctypes.c_float), c32.shape[1], _p(qn, ctypes.c_float), b,
                            _p(cand, ctypes.c_int64), m, _p(sc, ctypes.c_float))
        return sc
    corpus16 = np.ascontiguousarray(corpus16, dtype=np.uint16)
    qn = np.ascontiguousarray(qn, dtype=np.float32)
    cand = np.ascontiguousarray(cand, dtype=np.int64)
    b, m = cand.shape
    sc = np.empty((b, m), dtype=np.float32)
    lib().orc_rescore(_p(corpus16, ctypes.c_uint16), corpus16.shape[1], _p(qn, ctypes.c_float),
                      b, _p(cand, ctypes.c_int64), m, _p(sc, ctypes.c_float))
    return sc


def _blas_scores(corpus16, qn, r0, chunk, tags, mask, value, use_filter):
    c = _rows_f32(corpus16, r0, chunk)
    s = qn @ c.T  # [b, chunk]
    if use_filter:
        t = tags[r0:r0 + chunk]
        s[:, (t & mask) != value] = -np.inf
    return s


def search_fast(corpus16: np.ndarray, queries: np.ndarray, k: int, margin: int = 64,
                chunk: int = 1 << 20, tags: np.ndarray | None = None, mask: int = 0,
                value: int = 0, use_filter: bool = False, stats: dict | None = None):
    """Same result as search() for large corpora, with a certificate: numpy fp32 BLAS
    shortlist of k+margin candidates per query (chunked), canonical exact rescoring, (score
    desc, row asc) ordering. |BLAS - exact| <= delta (fp32 accumulation over D terms of
    unit-norm operands), so the result is certified when the k-th exact score exceeds the
    last shortlisted BLAS score + delta; otherwise every row with BLAS score >= (k-th exact
    - delta) is rescored exactly (the oracle's own exactness fallback, counted in
    stats["widened"])."""
    queries = np.ascontiguousarray(queries, dtype=np.float32)
    qn = normalize(queries)
    n, d = corpus16.shape
    b = qn.shape[0]
    m = min(k + margin, n)
    delta = np.float32(2.0 * d * 2.0 ** -24 * 1.01 + 2.0 ** -20)
    best_s = np.full((b, 0), -np.inf, dtype=np.float32)
    best_i = np.zeros((b, 0), dtype=np.int64)
    for r0 in range(0, n, chunk):
        s = _blas_scores(corpus16, qn, r0, chunk, tags, mask, value, use_filter)
        mm = min(m, s.shape[1])
        part = np.argpartition(-s, mm - 1, axis=1)[:, :mm]
        ps = np.take_along_axis(s, part, axis=1)
        best_s = np.concatenate([best_s, ps], axis=1)
        best_i = np.concatenate([best_i, part + r0], axis=1)
        if best_s.shape[1] > m:
            sel = np.argpartition(-best_s, m - 1, axis=1)[:, :m]
            best_s = np.take_along_axis(best_s, sel, axis=1)
            best_i = np.take_along_axis(best_i, sel, axis=1)
    cand = np.where(np.isfinite(best_s), best_i, -1)
    ex = rescore(corpus16, qn, cand)
    out_s = np.full((b, k), -np.inf, dtype=np.float32)
    out_i = np.full((b, k), -1, dtype=np.int64)
    widen = []
    for q in range(b):
        valid = cand[q] >= 0
        ids, sc = cand[q][valid], ex[q][valid]
        order = np.lexsort((ids, -sc.astype(np.float64)))[:k]
        out_s[q, :len(order)] = sc[order]
        out_i[q, :len(order)] = ids[order]
        # certificate: rows outside the shortlist have BLAS score <= its last one
        if valid.sum() >= m and len(order) == k:
            s_m = best_s[q][valid].min()
            if not sc[order[-1]] > s_m + delta:
                widen.append(q)
    for q in widen:
        floor = np.float32(out_s[q, k - 1] - delta)
        ids = []
        for r0 in range(0, n, chunk):
            s = _blas_scores(corpus16, qn[q:q + 1], r0, chunk, tags, mask, value, use_filter)[0]
            ids.append(np.nonzero(s >= floor)[0] + r0)
        ids = np.concatenate(ids)
        sc = rescore(corpus16, qn[q:q + 1], ids[None, :])[0]
        order = np.lexsort((ids, -sc.astype(np.float64)))[:k]
        out_s[q] = sc[order]
        out_i[q] = ids[order]
    if stats is not None:
        stats["widened"] = stats.get("widened", 0) + len(widen)
    return out_s, out_i


def blas_delta(d: int) -> np.float32:
    """Bound on |numpy fp32 BLAS score - canonical exact score| for unit-norm operands."""
    return np.float32(2.0 * d * 2.0 ** -24 * 1.01 + 2.0 ** -20)


def candidates_above(corpus16: np.ndarray, qn: np.ndarray, floor: np.ndarray,
                     chunk: int = 1 << 17, row_offset: int = 0):
    """Every row whose canonical exact score against normalised query q is >= floor[q]:
    a BLAS pass keeps rows with fp32 score >= floor - delta (a superset), which are then
    rescored exactly. Returns per query (ids + row_offset, exact scores), unordered. Used to
    CERTIFY a top-k: with floor = the k-th best exact score among any k returned rows (a
    lower bound of the true k-th score), the true top-k is inside the result."""
    qn = np.ascontiguousarray(qn, dtype=np.float32)
    n, d = corpus16.shape
    b = qn.shape[0]
    thr = (np.asarray(floor, np.float32) - blas_delta(d))[:, None]
    hits = [[] for _ in range(b)]
    for r0 in range(0, n, chunk):
        c = _rows_f32(corpus16, r0, chunk)
        s = qn @ c.T
        qq, rr = np.nonzero(s >= thr)
        for q in np.unique(qq):
            hits[q].append(rr[qq == q] + r0)
    out = []
    for q in range(b):
        ids = np.concatenate(hits[q]) if hits[q] else np.zeros(0, np.int64)
        sc = rescore(corpus16, qn[q:q + 1], ids[None, :].astype(np.int64))[0] if len(ids) \
            else np.zeros(0, np.float32)
        keep = sc >= floor[q]
        out.append((ids[keep].astype(np.int64) + row_offset, sc[keep]))
    return out


def search_f64_reference(corpus16: np.ndarray, queries: np.ndarray, k: int):
    """Independent numpy formulation used to pin the C oracle in tests: float64 matmul on
    the fp16 corpus against canonically normalised queries, rounded to fp32, full lexsort.
    (Summation order differs from the canonical one; equal to it whenever no fp32 rounding
    boundary is straddled, which the tests check on fixtures.)"""
    qn = normalize(queries).astype(np.float64)
    c = corpus16.view(np.float16).astype(np.float64)
    s = (qn @ c.T).astype(np.float32)
    out_s = np.empty((qn.shape[0], k), dtype=np.float32)
    out_i = np.empty((qn.shape[0], k), dtype=np.int64)
    ids = np.arange(c.shape[0])
    for q in range(qn.shape[0]):
        order = np.lexsort((ids, -s[q].astype(np.float64)))[:k]
        out_s[q] = s[q][order]
        out_i[q] = order
    return out_s, out_i
