"""FlatIndex — Python handle over the in-HBM flat cosine index of libragmi.so.

This is the storage + search engine that replaces the Qdrant server's COSINE collection
(reference main.py:92-95 get_qdrant, main.py:215-239 retrieve_from_qdrant, ingest.py:86-96
ensure_collection, ingest.py:148-175 upsert). Vectors live in HBM as fp16 in the MFMA
"tile16" layout; search runs the HIP scan + top-k + exact-rescoring merge on
the caller's current torch stream. Inputs may be numpy arrays (copied to the device) or cuda
torch tensors (used in place).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import check

MAX_K = 32          # RAG_MAX_K in include/ragmi.h: the scan's certified top-k path
MAX_K_LARGE = 4096  # RAG_MAX_K_LARGE: k in (32, 4096] takes the exact large-k pass; larger k
                    # the full exact pass (and the packed exchange form stops here)
QUERY_TILE = 32     # RAG_QUERY_TILE
STORAGE = {"fp16": 0, "fp32": 1}   # RAG_STORE_FP16 / RAG_STORE_FP32
CREATE_DIAGNOSTIC = 0x100          # RAG_CREATE_DIAGNOSTIC: honour the RAGMI_* A/B knobs


def _stream_ptr(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _as_dev(x, dtype, device) -> torch.Tensor:
    if isinstance(x, torch.Tensor):
        t = x.to(device=device, dtype=dtype)
    else:
        t = torch.from_numpy(np.ascontiguousarray(np.asarray(x))).to(dtype=dtype)
        t = t.to(device=device, non_blocking=False)
    return t.contiguous()


class FlatIndex:
    """In-HBM flat index with exact (score desc, row asc) top-k search. storage "fp16": the
    fp16 rows only (what the scan streams); "fp32": the normalised fp32 rows too, which the
    exact scores read (Qdrant's default Float32 vectors; rag_index_create_ex).
    diagnostic=True (bench / profiling scripts only) lets the process honour the RAGMI_*
    kernel A/B environment knobs (RAG_CREATE_DIAGNOSTIC); serving code leaves it off, and
    the library then ignores (and reports) any such variable."""

    def __init__(self, dim: int = 384, capacity: int = 0, device=None, storage: str = "fp16",
                 diagnostic: bool = False):
        dev = _lib.resolve_device(device)        # "cpu" refused before any HIP call
        _lib.require_gpu()
        self._L = _lib.load()
        self.device = torch.device("cuda", _lib.device_index(dev))
        self.dim = int(dim)
        if storage not in STORAGE:
            raise ValueError(f"storage must be one of {sorted(STORAGE)}")
        self.storage = storage
        h = ctypes.c_void_p()
        flags = STORAGE[storage] | (CREATE_DIAGNOSTIC if diagnostic else 0)
        check(self._L.rag_index_create_ex(self.dim, int(capacity), self.device.index, flags,
                                          ctypes.byref(h)))
        self._h = h

    # ---------------------------------------------------------------- lifetime
    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            self._L.rag_index_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------------- properties
    @property
    def capacity(self) -> int:
        return int(self._L.rag_index_capacity(self._h))

    @property
    def count(self) -> int:
        return int(self._L.rag_index_count(self._h))

    def reserve(self, capacity: int) -> None:
        check(self._L.rag_index_reserve(self._h, int(capacity)))

    # ---------------------------------------------------------------- writes
    def upsert(self, vectors, rows, tags=None, new_count: int | None = None) -> None:
        """Normalise + store vectors [n, dim] at row slots `rows` [n] (overwrite allowed)."""
        v = _as_dev(vectors, torch.float32, self.device)
        if v.dim() != 2 or v.shape[1] != self.dim:
            raise ValueError(f"vectors must be [n, {self.dim}]")
        r = _as_dev(rows, torch.int64, self.device)
        n = v.shape[0]
        if r.shape != (n,):
            raise ValueError("rows must be [n]")
        if n and (int(r.min()) < 0 or int(r.max()) >= self.capacity):
            raise IndexError("row slot outside capacity; reserve() first")
        t = None
        if tags is not None:
            t = _as_dev(np.asarray(tags, dtype=np.uint32).view(np.int32)
                        if not isinstance(tags, torch.Tensor) else tags, torch.int32,
                        self.device)
        if new_count is None:
            new_count = max(self.count, int(r.max()) + 1 if n else 0)
        check(self._L.rag_index_upsert(self._h, v.data_ptr(), r.data_ptr(),
                                       t.data_ptr() if t is not None else None, n,
                                       int(new_count), _stream_ptr(self.device)))
        # staging tensors are released to the stream-ordered caching allocator (safe reuse).

    def set_count(self, new_count: int) -> None:
        check(self._L.rag_index_upsert(self._h, None, None, None, 0, int(new_count),
                                       _stream_ptr(self.device)))

    # ---------------------------------------------------------------- search
    def _search_args(self, queries, k, filters, k_max=None):
        if k < 1 or (k_max is not None and k > k_max):
            raise ValueError(f"k must be in [1, {k_max}]" if k_max else "k must be >= 1")
        q = _as_dev(queries, torch.float32, self.device)
        if q.dim() == 1:
            q = q.unsqueeze(0)
        if q.shape[-1] != self.dim:
            raise ValueError(f"query dim {q.shape[-1]} != index dim {self.dim}")
        B = q.shape[0]
        f = None
        if filters is not None:
            if isinstance(filters, torch.Tensor):
                f = filters.to(device=self.device, dtype=torch.int32).contiguous()
            else:
                f = torch.from_numpy(np.ascontiguousarray(
                    np.asarray(filters, dtype=np.uint32).reshape(B, 2)).view(np.int32))
                f = f.to(self.device)
            if f.shape != (B, 2):
                raise ValueError("filters must be [B, 2] (tag_mask, tag_value)")
        return q, B, f

    def search_packed(self, queries, k: int, filters=None, id_offset: int = 0) -> torch.Tensor:
        """Top-k in the multi-GPU exchange form: int32 [B, k, 2] = (fp32 score bits, global
        row; -1 = none), enqueued on the current stream (rag_index_search_packed)."""
        q, B, f = self._search_args(queries, k, filters, k_max=MAX_K_LARGE)
        out = torch.empty((B, k, 2), dtype=torch.int32, device=self.device)
        check(self._L.rag_index_search_packed(self._h, q.data_ptr(), B, int(k),
                                              f.data_ptr() if f is not None else None,
                                              int(id_offset), out.data_ptr(),
                                              _stream_ptr(self.device)))
        return out

    def search(self, queries, k: int, filters=None, id_offset: int = 0,
               out: tuple[torch.Tensor, torch.Tensor] | None = None, full: bool = False):
        """Top-k of each query row. Returns (scores fp32 [B,k], ids int64 [B,k]) as cuda
        tensors, enqueued on the current stream (ids -1 where fewer than k rows match).
        `filters`: None, or per-query (tag_mask, tag_value) pairs [B, 2] (uint32).
        Any k >= 1: k <= 32 on the scan, k <= 4096 on the large-k pass, beyond on the full
        exact pass (every row scored exactly, then sorted); full=True forces the full pass
        (rag_index_search_full) — the same result, the path for queries a large-k pass left
        unanswered."""
        q, B, f = self._search_args(queries, k, filters)
        if out is None:
            out_s = torch.empty((B, k), dtype=torch.float32, device=self.device)
            out_i = torch.empty((B, k), dtype=torch.int64, device=self.device)
        else:
            out_s, out_i = out
        fn = self._L.rag_index_search_full if full else self._L.rag_index_search
        check(fn(self._h, q.data_ptr(), B, int(k),
                 f.data_ptr() if f is not None else None,
                 int(id_offset), out_s.data_ptr(), out_i.data_ptr(),
                 _stream_ptr(self.device)))
        # staging tensors (q, f) go back to torch's stream-ordered caching allocator: any
        # reuse is enqueued on this same stream after our kernels, so no sync is needed.
        return out_s, out_i

    # ---------------------------------------------------------------- introspection
    def export_rows(self, row0: int = 0, n: int | None = None) -> np.ndarray:
        """Stored fp16 rows (uint16 bits) [n, dim], row-major."""
        if n is None:
            n = self.count - row0
        out = np.empty((n, self.dim), dtype=np.uint16)
        torch.cuda.current_stream(self.device).synchronize()
        check(self._L.rag_index_export_rows(self._h, int(row0), int(n),
                                            out.ctypes.data_as(_lib.c_u16p)))
        return out

    def import_rows(self, rows_f16, row0: int = 0, tags=None,
                    new_count: int | None = None) -> None:
        """Write already-stored fp16 rows [n, dim] (float16 or uint16 bits, host) back into
        rows [row0, row0+n) unchanged — the load side of persistence (no renormalisation)."""
        a = np.ascontiguousarray(rows_f16)
        if a.dtype == np.float16:
            a = a.view(np.uint16)
        if a.dtype != np.uint16 or a.ndim != 2 or a.shape[1] != self.dim:
            raise ValueError(f"rows must be float16/uint16 [n, {self.dim}]")
        n = a.shape[0]
        t = None
        if tags is not None:
            t = np.ascontiguousarray(tags, dtype=np.uint32)
            if t.shape != (n,):
                raise ValueError("tags must be [n]")
        if new_count is None:
            new_count = max(self.count, row0 + n)
        torch.cuda.current_stream(self.device).synchronize()
        check(self._L.rag_index_import_rows(
            self._h, int(row0), int(n), a.ctypes.data_as(_lib.c_u16p),
            t.ctypes.data_as(_lib.c_u32p) if t is not None else None, int(new_count)))

    def export_rows32(self, row0: int = 0, n: int | None = None) -> np.ndarray:
        """fp32 storage: the stored normalised fp32 rows [n, dim]."""
        if n is None:
            n = self.count - row0
        out = np.empty((n, self.dim), dtype=np.float32)
        torch.cuda.current_stream(self.device).synchronize()
        check(self._L.rag_index_export_rows32(self._h, int(row0), int(n),
                                              out.ctypes.data_as(_lib.c_f32p)))
        return out

    def import_rows32(self, rows_f32, row0: int = 0, tags=None,
                      new_count: int | None = None) -> None:
        """fp32 storage: write saved fp32 rows [n, dim] back unchanged (their fp16 scan copy
        is re-derived by the same rounding as upsert)."""
        a = np.ascontiguousarray(rows_f32, dtype=np.float32)
        if a.ndim != 2 or a.shape[1] != self.dim:
            raise ValueError(f"rows must be float32 [n, {self.dim}]")
        n = a.shape[0]
        t = None
        if tags is not None:
            t = np.ascontiguousarray(tags, dtype=np.uint32)
            if t.shape != (n,):
                raise ValueError("tags must be [n]")
        if new_count is None:
            new_count = max(self.count, row0 + n)
        torch.cuda.current_stream(self.device).synchronize()
        check(self._L.rag_index_import_rows32(
            self._h, int(row0), int(n), a.ctypes.data_as(_lib.c_f32p),
            t.ctypes.data_as(_lib.c_u32p) if t is not None else None, int(new_count)))

    def export_tags(self, row0: int = 0, n: int | None = None) -> np.ndarray:
        if n is None:
            n = self.count - row0
        out = np.empty((n,), dtype=np.uint32)
        torch.cuda.current_stream(self.device).synchronize()
        check(self._L.rag_index_export_tags(self._h, int(row0), int(n),
                                            out.ctypes.data_as(_lib.c_u32p)))
        return out

    def set_scan_order(self, serial: bool) -> None:
        """serial=True: each pass's scan waits for the previous pass's scan on any stream
        (rag_index_set_scan_order); prep / seeding / select still overlap across streams."""
        mode = serial if isinstance(serial, int) and not isinstance(serial, bool) else int(bool(serial))
        check(self._L.rag_index_set_scan_order(self._h, mode))

    def exactness_stats(self, n_last: int = 0):
        """(tier1 total, tier2 total, tiers of the last pass's first n_last queries): which
        path certified each top-k (0 error-bound check, 1 list re-scoring, 2 second pass);
        rag_index_exactness_stats. The totals count every query since creation; the per-query
        tiers cover only the most recent PASS (<= 32 queries, <= 128 on the D = 1024 wide
        scan) of this handle on any stream — not the whole last search when it had more
        queries, and not a search of this thread when other threads search concurrently.
        Synchronises the device."""
        t1 = ctypes.c_int64()
        t2 = ctypes.c_int64()
        last = np.empty((max(n_last, 0),), dtype=np.int32)
        check(self._L.rag_index_exactness_stats(
            self._h, ctypes.byref(t1), ctypes.byref(t2),
            last.ctypes.data_as(_lib.c_i32p) if n_last > 0 else None, int(n_last)))
        return int(t1.value), int(t2.value), last

    def unanswered(self) -> int:
        """Queries since creation that got NO result (their tier reads 3, their ids -1):
        k <= 32 passes whose second pass was skipped (RAGMI_RESCAN_WG=0, diagnostic handles
        only), and 32 < k <= 4096 passes where more than 16384 rows tie within the MFMA error
        band of a query's k-th best score after the last collection round (possible in
        production, e.g. thousands of identical boilerplate chunks). Collection.search re-runs
        such queries on the full exact pass (search(full=True)). rag_index_unanswered;
        synchronises the device."""
        n = ctypes.c_int64()
        check(self._L.rag_index_unanswered(self._h, ctypes.byref(n)))
        return int(n.value)

    # ---------------------------------------------------------------- profiling
    def profile(self, every: int | bool) -> None:
        """Time every `every`-th scan launch with HIP events (0/False: off, True: every one)."""
        check(self._L.rag_profile_enable(self._h, int(every)))

    def bench_scan(self, queries: torch.Tensor, variant: int, reps: int = 10) -> float:
        """Diagnostic: avg device ms per launch of scan variant `variant` (rag_bench_scan)."""
        q = _as_dev(queries, torch.float32, self.device)
        ms = ctypes.c_double()
        torch.cuda.synchronize(self.device)
        check(self._L.rag_bench_scan(self._h, q.data_ptr(), q.shape[0], int(variant),
                                     int(reps), ctypes.byref(ms)))
        return float(ms.value)

    def profile_scan_ms(self) -> tuple[float, int]:
        tot = ctypes.c_double()
        n = ctypes.c_int64()
        check(self._L.rag_profile_scan_ms(self._h, ctypes.byref(tot), ctypes.byref(n)))
        return float(tot.value), int(n.value)

    def profile_scan_intervals(self, cap: int = 1 << 16) -> tuple[np.ndarray, np.ndarray]:
        """(start_ms, end_ms) of every recorded scan launch, relative to the first one's start
        (rag_profile_scan_intervals); clears the record."""
        a = np.zeros(cap, np.float64)
        b = np.zeros(cap, np.float64)
        n = ctypes.c_int64()
        dp = ctypes.POINTER(ctypes.c_double)
        check(self._L.rag_profile_scan_intervals(self._h, a.ctypes.data_as(dp),
                                                 b.ctypes.data_as(dp), cap, ctypes.byref(n)))
        m = min(int(n.value), cap)
        return a[:m], b[:m]


class PartitionStreams:
    """`parts` HIP streams on disjoint shares of the device's CUs
    (rag_stream_create_cu_partition) as torch streams, for `parts` batches in flight: a search
    issued on one sizes its scan to that share, so the batches scan side by side instead of
    interleaving over every CU. Results are the same on any stream. close() (or the end of
    the process) destroys them; call it only after their work has finished."""

    def __init__(self, device, parts: int, whole: bool = False):
        """whole=True: `parts` streams that each may use EVERY CU (a full CU mask): still one
        dedicated hardware queue per stream (a CU-masked queue is never shared), so batches in
        flight cannot land on one queue whatever streams the process created before (the
        serving-shape fix of DESIGN §R6.4)."""
        dev = _lib.resolve_device(device)
        self.device = torch.device("cuda", _lib.device_index(dev))
        self._L = _lib.load()
        self._raw, self.streams = [], []
        for p in range(parts):
            h = ctypes.c_void_p()
            check(self._L.rag_stream_create_cu_partition(self.device.index,
                                                         0 if whole else p, 1 if whole else parts,
                                                         ctypes.byref(h)))
            self._raw.append(h)
            self.streams.append(torch.cuda.ExternalStream(h.value, device=self.device))

    def __len__(self):
        return len(self.streams)

    def __getitem__(self, i):
        return self.streams[i]

    def close(self) -> None:
        if self._raw:
            torch.cuda.synchronize(self.device)
            for h in self._raw:
                self._L.rag_stream_destroy(h)
            self._raw, self.streams = [], []


def busy_union_ms(start_ms, end_ms) -> float:
    """Length of the union of [start, end) intervals: the time at least one of the launches
    was running (overlapping launches counted once)."""
    order = np.argsort(start_ms, kind="stable")
    busy, cur_a, cur_b = 0.0, None, None
    for i in order:
        a, b = float(start_ms[i]), float(end_ms[i])
        if cur_b is None or a > cur_b:
            if cur_b is not None:
                busy += cur_b - cur_a
            cur_a, cur_b = a, b
        else:
            cur_b = max(cur_b, b)
    if cur_b is not None:
        busy += cur_b - cur_a
    return busy


def merge_topk(scores: torch.Tensor, ids: torch.Tensor, k: int):
    """Merge per-shard exact lists [n_lists, B, k] -> global [B, k] on the GPU."""
    L = _lib.load()
    n_lists, B, kk = scores.shape
    if kk != k:
        raise ValueError("list length must equal k")
    scores = scores.contiguous()
    ids = ids.contiguous()
    out_s = torch.empty((B, k), dtype=torch.float32, device=scores.device)
    out_i = torch.empty((B, k), dtype=torch.int64, device=scores.device)
    check(L.rag_merge_topk(scores.data_ptr(), ids.data_ptr(), n_lists, B, k, out_s.data_ptr(),
                           out_i.data_ptr(), _stream_ptr(scores.device)))
    return out_s, out_i


def merge_topk_packed(packed: torch.Tensor, k: int):
    """Merge all-gathered packed lists int32 [n_lists, B, k, 2] -> (scores [B,k], ids [B,k])."""
    L = _lib.load()
    n_lists, B, kk, two = packed.shape
    if kk != k or two != 2 or packed.dtype != torch.int32:
        raise ValueError("packed lists must be int32 [n_lists, B, k, 2]")
    packed = packed.contiguous()
    out_s = torch.empty((B, k), dtype=torch.float32, device=packed.device)
    out_i = torch.empty((B, k), dtype=torch.int64, device=packed.device)
    check(L.rag_merge_topk_packed(packed.data_ptr(), n_lists, B, k, out_s.data_ptr(),
                                  out_i.data_ptr(), _stream_ptr(packed.device)))
    return out_s, out_i
