"""QdrantClient-shaped front end of the in-HBM flat index.

Drop-in for the calls the reference makes on `qdrant_client.QdrantClient`:
  get_collections()                       main.py:135, main2.py:337 (/ready)
  collection_exists(name)                 ingest.py:87, database.py:121
  create_collection(name, vectors_config) ingest.py:89-95, database.py:122-128
  upsert(name, points=[PointStruct])      ingest.py:171-175
  query_points(name, query, limit, query_filter) -> .points[i].{id,score,payload}
                                          main.py:232-237, main2.py:163
plus query_batch_points (one GPU scan for a whole micro-batch; main2.py:281-295 stage 2),
count, retrieve and delete_collection.

`url` is accepted and ignored: the collection lives in this process's GPU memory (the
Qdrant service of docker-compose.yml:22 is replaced, not contacted). `path=` plays the role
of Qdrant's local mode / storage volume: existing collections under it are loaded at
construction and `save()` / `close()` write them back (ragmi.store shard format). Payloads stay host-side
keyed by row; the keyword payload fields used by the reference's `must` filter (`ticker`,
`document_type`, main.py:218-230) are dictionary-coded into a per-row uint32 tag in HBM
(16 bits per field) so filtering runs inside the scan kernel.
"""
from __future__ import annotations

import os
import shutil
import threading
import time
import uuid
from typing import Any, Iterable

import numpy as np
import torch

from . import qdrant_models as models
from .index import MAX_K, FlatIndex

DEFAULT_TAG_FIELDS = ("ticker", "document_type")


def _norm_id(pid):
    """Qdrant point ids are unsigned ints or UUIDs; 32-hex md5 digests (ingest.py:151-154)
    are accepted as UUIDs and reported back in canonical dashed form."""
    if isinstance(pid, bool):
        raise ValueError("point id must be int or UUID string")
    if isinstance(pid, (int, np.integer)):
        if pid < 0:
            raise ValueError("integer point ids must be unsigned")
        return int(pid)
    if isinstance(pid, uuid.UUID):
        return str(pid)
    if isinstance(pid, str):
        return str(uuid.UUID(pid))
    raise ValueError(f"unsupported point id type {type(pid)!r}")


class UnsupportedFilter(NotImplementedError):
    pass


class PayloadTags:
    """Dictionary-codes up to two keyword payload fields into a per-row uint32 tag
    (16 bits per field, code 0 = field absent) and compiles Qdrant `must` filters on those
    fields into (mask, value) so the GPU scan filters with (tag & mask) == value.
    Host-only logic (no device code)."""

    def __init__(self, fields=DEFAULT_TAG_FIELDS):
        if len(fields) > 2:
            raise ValueError("at most two indexed keyword payload fields (16 bits each)")
        self.fields = tuple(fields)
        self.codes: list[dict[Any, int]] = [dict() for _ in self.fields]

    def code(self, f: int, value, create: bool) -> int | None:
        if isinstance(value, (list, dict)) or value is None:
            return None
        table = self.codes[f]
        c = table.get(value)
        if c is None and create:
            if len(table) >= 0xFFFF:
                raise OverflowError(f"more than 65535 distinct values for {self.fields[f]}")
            c = len(table) + 1          # 0 = field absent
            table[value] = c
        return c

    def tag(self, payload: dict | None) -> int:
        tag = 0
        if payload:
            for f, key in enumerate(self.fields):
                if key in payload:
                    c = self.code(f, payload[key], create=True)
                    if c:
                        tag |= c << (16 * f)
        return tag

    def compile(self, flt: models.Filter | None):
        """Filter(must=[FieldCondition(key, MatchValue(v))...]) -> (mask, value); None when
        nothing can match (a value never ingested); (0, 0) for no filter."""
        if flt is None:
            return (0, 0)
        if flt.should or flt.must_not:
            raise UnsupportedFilter("only `must` conditions are supported (main.py:218-236)")
        mask = value = 0
        for cond in flt.must or []:
            if not isinstance(cond, models.FieldCondition) or cond.range is not None:
                raise UnsupportedFilter("only FieldCondition(key, match=MatchValue) is supported")
            if cond.key not in self.fields:
                raise UnsupportedFilter(
                    f"payload key {cond.key!r} is not an indexed keyword field "
                    f"{self.fields}; create the collection with payload_tag_fields")
            if not isinstance(cond.match, models.MatchValue):
                raise UnsupportedFilter("only MatchValue matches are supported")
            f = self.fields.index(cond.key)
            c = self.code(f, cond.match.value, create=False)
            if c is None:
                return None
            m = 0xFFFF << (16 * f)
            if mask & m and (value & m) != (c << (16 * f)):
                return None             # two different values for one field
            mask |= m
            value |= c << (16 * f)
        return (mask, value)


class _Req:
    __slots__ = ("q", "limit", "filt", "result", "exc", "wake", "lead")

    def __init__(self, q, limit, filt):
        self.q, self.limit, self.filt = q, limit, filt
        self.result = self.exc = None
        self.wake = threading.Event()
        self.lead = False


class Coalescer:
    """Rides concurrent single-query searches on one GPU scan.

    The reference's batched service still searches per request: main2.py's batch_processor
    fans a micro-batch out to process_independently tasks that each call
    retrieve_from_qdrant -> query_points from an asyncio.to_thread worker (<= 25 at once,
    main2.py:52-53,218,228). Unchanged, that is one full-corpus scan per query. Here the
    first caller becomes the LEADER and searches; callers arriving while a search runs queue
    up, and the next leader (the oldest queued request) searches all of them in ONE batched
    scan (per-query payload filters ride inside the kernel). With no concurrency a request
    runs at once (no added latency); `window_s` > 0 additionally holds a leader back for up
    to that long to gather more callers. Results are bit-identical to individual calls: every
    query's top-k is exact, independent of its batch-mates (tests/test_qdrant_gpu.py)."""

    def __init__(self, col: "Collection", window_s: float = 0.0, max_batch: int = 32):
        self.col = col
        self.window = float(window_s)
        self.max_batch = int(max_batch)
        self.lock = threading.Lock()
        self.pending: list[_Req] = []
        self.leader_active = False
        self.batches = 0            # scans issued (stats)
        self.requests = 0

    def search(self, q: np.ndarray, limit: int, filt):
        req = _Req(q, int(limit), filt)
        with self.lock:
            self.pending.append(req)
            self.requests += 1
            if not self.leader_active:
                self.leader_active = True
                req.lead = True
        if not req.lead:
            req.wake.wait()
            if not req.lead:                       # served by another leader
                if req.exc is not None:
                    raise req.exc
                return req.result
        batch: list[_Req] = []
        fatal = None
        try:
            if self.window > 0:
                t_end = time.perf_counter() + self.window
                while time.perf_counter() < t_end:
                    with self.lock:
                        if len(self.pending) >= self.max_batch:
                            break
                    time.sleep(min(5e-5, self.window / 4))
            with self.lock:
                batch = self.pending[:self.max_batch]
                del self.pending[:self.max_batch]
                self.batches += 1
            hits = self.col.search(np.stack([r.q for r in batch]),
                                   max(r.limit for r in batch), [r.filt for r in batch])
            for r, h in zip(batch, hits):
                r.result = h[:r.limit]
        except BaseException as e:                 # every rider sees the failure
            for r in batch:
                r.exc = e
            if not isinstance(e, Exception):       # KeyboardInterrupt, SystemExit: re-raise
                fatal = e                          # after the hand-off below
        finally:
            # whatever was raised: hand leadership on and wake every rider, so no caller of
            # this collection can block forever behind a leader that is gone
            with self.lock:
                if req in self.pending:            # interrupted before taking the batch
                    self.pending.remove(req)
                if self.pending:                   # hand leadership to the oldest waiter
                    nxt = self.pending[0]
                    nxt.lead = True
                    nxt.wake.set()
                else:
                    self.leader_active = False
            for r in batch:
                if r is not req:
                    r.wake.set()
        if fatal is not None:
            raise fatal
        if req.exc is not None:
            raise req.exc
        return req.result


def _storage_of(vectors_config) -> str:
    """VectorParams.datatype -> FlatIndex storage. Qdrant stores Float32 unless told otherwise
    (the reference never sets a datatype, database.py:124-130, ingest.py:89-95), so the
    default is fp32 storage: exact scores on the fp32 rows, the scan on their fp16 copy."""
    dt = getattr(vectors_config, "datatype", None)
    dt = getattr(dt, "value", dt)
    if dt is None or str(dt).lower() == "float32":
        return "fp32"
    if str(dt).lower() == "float16":
        return "fp16"
    raise NotImplementedError(f"vector datatype {dt!r} (float32 and float16 are supported)")


class Collection:
    """One COSINE collection: FlatIndex in HBM + host-side id/payload maps."""

    def __init__(self, name: str, dim: int, device, tag_fields=DEFAULT_TAG_FIELDS,
                 capacity: int = 1024, storage: str = "fp32"):
        self.name = name
        self.dim = dim
        self.tags = PayloadTags(tag_fields)
        self.index = FlatIndex(dim=dim, capacity=capacity, device=device, storage=storage)
        self.id_to_row: dict[Any, int] = {}
        self.row_ids: list[Any] = []
        self.payloads: list[dict | None] = []
        self.versions: list[int] = []
        self.op = 0
        self._unanswered = 0     # index.unanswered() as last read (Collection.search)
        self.rescued = 0         # queries re-answered on the full exact pass (stats)
        self.lock = threading.RLock()
        # 32 queries per scan pass at D = 384, 4 groups of 32 at D = 1024 (ragmi.h)
        self.coalescer = Coalescer(self, 0.0, 32 if dim <= 384 else 128)

    def compile_filter(self, flt):
        return self.tags.compile(flt)

    # ---------------------------------------------------------------- writes
    def upsert(self, ids: list, vectors, payloads: list) -> int:
        with self.lock:
            self.op += 1
            vec = np.asarray(vectors, dtype=np.float32) if not isinstance(
                vectors, torch.Tensor) else vectors
            if vec.ndim != 2 or vec.shape[1] != self.dim:
                raise ValueError(f"vectors must be [n, {self.dim}]")
            # last write wins for duplicate ids inside one batch (Qdrant semantics)
            last: dict[Any, int] = {}
            for i, pid in enumerate(ids):
                last[_norm_id(pid)] = i
            rows, sel, tags = [], [], []
            new_count = len(self.row_ids)
            for pid, i in last.items():
                r = self.id_to_row.get(pid)
                if r is None:
                    r = new_count
                    new_count += 1
                    self.id_to_row[pid] = r
                    self.row_ids.append(pid)
                    self.payloads.append(None)
                    self.versions.append(0)
                p = payloads[i] if payloads is not None else None
                self.payloads[r] = dict(p) if p is not None else None
                self.versions[r] = self.op
                rows.append(r)
                sel.append(i)
                tags.append(self.tags.tag(p))
            if new_count > self.index.capacity:
                self.index.reserve(max(new_count, 2 * self.index.capacity))
            if rows:
                sel_t = vec[sel] if isinstance(vec, torch.Tensor) else vec[np.asarray(sel)]
                self.index.upsert(sel_t, np.asarray(rows, dtype=np.int64),
                                  np.asarray(tags, dtype=np.uint32), new_count=new_count)
            return self.op

    # ---------------------------------------------------------------- reads
    def search(self, queries, limit: int, filters: list):
        """queries [B, dim]; filters: per query compiled filter ((mask, value) or None)."""
        with self.lock:
            B = len(filters)
            if limit < 1:
                return [[] for _ in range(B)]
            # Qdrant answers any limit with at most the collection's points (main.py:215,
            # 232-237): k <= 32 on the scan, <= 4096 on the large-k pass, beyond that on the
            # full exact pass (rag_index_search)
            k = min(limit, max(1, self.index.count))
            live = [i for i, f in enumerate(filters) if f is not None]
            out = [[] for _ in range(B)]
            if not live or self.index.count == 0:
                return out
            q = queries if isinstance(queries, torch.Tensor) else np.asarray(queries, np.float32)
            q = q[live] if len(live) != B else q
            fl = np.asarray([filters[i] for i in live], dtype=np.uint32).reshape(-1, 2)
            use = fl if fl.any() else None
            s, ids = self.index.search(q, k, filters=use)
            s = s.cpu().numpy()
            ids = ids.cpu().numpy()
            if (ids < 0).any():
                # a -1 is padding (fewer matching points than k) unless the pass left the
                # query unanswered (tier 3: more than 16384 rows tied within the error band
                # of its k-th best on the large-k pass). Only then, re-run those queries on
                # the full exact pass: an unanswered query must never read as "no documents"
                # (ADVICE r5).
                n_un = self.index.unanswered()
                if n_un > self._unanswered:
                    redo = np.nonzero((ids < 0).any(axis=1))[0].tolist()
                    s2, i2 = self.index.search(q[redo], k, filters=use[redo] if use is not None
                                               else None, full=True)
                    s[redo] = s2.cpu().numpy()
                    ids[redo] = i2.cpu().numpy()
                    self.rescued += len(redo)
                self._unanswered = n_un
            for j, i in enumerate(live):
                out[i] = [(int(r), float(sc)) for r, sc in zip(ids[j], s[j]) if r >= 0]
            return out

    def point(self, row: int, score: float, with_payload=True, with_vectors=False):
        payload = self.payloads[row] if with_payload else None
        vec = None
        if with_vectors:
            vec = (self.index.export_rows32(row, 1)[0] if self.index.storage == "fp32" else
                   self.index.export_rows(row, 1)[0].view(np.float16).astype(np.float32)).tolist()
        return models.ScoredPoint(id=self.row_ids[row], version=self.versions[row],
                                  score=score, payload=payload, vector=vec)


class QdrantClient:
    """In-process, GPU-resident replacement for qdrant_client.QdrantClient."""

    def __init__(self, url: str | None = None, *args, device=None, path: str | None = None,
                 coalesce: bool = True, coalesce_window_s: float = 0.0, **kwargs):
        self.url = url
        self.device = device
        self.path = path
        # concurrent query_points calls share GPU scans (Coalescer); coalesce=False searches
        # every call on its own
        self.coalesce = bool(coalesce)
        self.coalesce_window_s = float(coalesce_window_s)
        self._collections: dict[str, Collection] = {}
        self._lock = threading.Lock()
        if path is not None and os.path.isdir(path):
            from .store import load_collection
            for name in sorted(os.listdir(path)):
                d = os.path.join(path, name)
                if os.path.isfile(os.path.join(d, "collection.json")):
                    col = load_collection(d, device)
                    col.coalescer.window = self.coalesce_window_s
                    self._collections[col.name] = col

    def save(self, path: str | None = None) -> None:
        """Persist every collection under `path` (default: the client's path); collection
        directories of deleted collections are removed."""
        from .store import save_collection
        path = path or self.path
        if path is None:
            raise ValueError("no storage path: pass path= here or to QdrantClient(...)")
        os.makedirs(path, exist_ok=True)
        with self._lock:
            cols = dict(self._collections)
        for name, col in cols.items():
            save_collection(col, os.path.join(path, name))
        for name in os.listdir(path):
            d = os.path.join(path, name)
            if name not in cols and os.path.isfile(os.path.join(d, "collection.json")):
                shutil.rmtree(d)

    # ---------------------------------------------------------------- collections
    def get_collections(self) -> models.CollectionsResponse:
        with self._lock:
            return models.CollectionsResponse(
                collections=[models.CollectionDescription(name=n) for n in self._collections])

    def collection_exists(self, collection_name: str) -> bool:
        with self._lock:
            return collection_name in self._collections

    def create_collection(self, collection_name: str, vectors_config: models.VectorParams,
                          payload_tag_fields: Iterable[str] = DEFAULT_TAG_FIELDS,
                          capacity: int = 1024, **kwargs) -> bool:
        if vectors_config.distance != models.Distance.COSINE:
            raise NotImplementedError("only Distance.COSINE collections (database.py:126)")
        storage = _storage_of(vectors_config)
        with self._lock:
            if collection_name in self._collections:
                raise ValueError(f"collection {collection_name!r} already exists")
            col = Collection(collection_name, int(vectors_config.size), self.device,
                             tuple(payload_tag_fields), capacity, storage)
            col.coalescer.window = self.coalesce_window_s
            self._collections[collection_name] = col
        return True

    def recreate_collection(self, collection_name: str, vectors_config, **kwargs) -> bool:
        self.delete_collection(collection_name)
        return self.create_collection(collection_name, vectors_config, **kwargs)

    def delete_collection(self, collection_name: str, **kwargs) -> bool:
        with self._lock:
            col = self._collections.pop(collection_name, None)
        if col is not None:
            col.index.close()
        return col is not None

    def _col(self, name: str) -> Collection:
        with self._lock:
            col = self._collections.get(name)
        if col is None:
            raise ValueError(f"Collection `{name}` doesn't exist!")
        return col

    # ---------------------------------------------------------------- points
    def upsert(self, collection_name: str, points, wait: bool = True, **kwargs):
        col = self._col(collection_name)
        if isinstance(points, models.Batch):
            ids, vecs, pls = points.ids, points.vectors, points.payloads
        else:
            points = list(points)
            ids = [p.id for p in points]
            vecs = [p.vector for p in points]
            pls = [p.payload for p in points]
        if not ids:
            return models.UpdateResult(operation_id=col.op, status=models.UpdateStatus.COMPLETED)
        op = col.upsert(ids, vecs, pls)
        return models.UpdateResult(operation_id=op, status=models.UpdateStatus.COMPLETED)

    def count(self, collection_name: str, **kwargs) -> models.CountResult:
        return models.CountResult(count=len(self._col(collection_name).row_ids))

    def retrieve(self, collection_name: str, ids, with_payload=True, with_vectors=False,
                 **kwargs):
        col = self._col(collection_name)
        out = []
        for pid in ids:
            r = col.id_to_row.get(_norm_id(pid))
            if r is not None:
                p = col.point(r, 0.0, with_payload, with_vectors)
                out.append(models.Record(id=p.id, payload=p.payload, vector=p.vector))
        return out

    def query_points(self, collection_name: str, query=None, limit: int = 10,
                     query_filter: models.Filter | None = None, with_payload=True,
                     with_vectors=False, **kwargs) -> models.QueryResponse:
        col = self._col(collection_name)
        flt = col.compile_filter(query_filter)
        if self.coalesce and 1 <= int(limit) <= MAX_K:
            q = (query.detach().float().cpu().numpy() if isinstance(query, torch.Tensor)
                 else np.asarray(query, dtype=np.float32))
            if q.shape != (col.dim,):
                q = q.reshape(-1)
                if q.shape != (col.dim,):
                    raise ValueError(f"query must be one {col.dim}-dim vector")
            hits = col.coalescer.search(q, int(limit), flt)
        else:
            q = query if isinstance(query, torch.Tensor) else np.asarray(query, dtype=np.float32)
            q = q.reshape(1, -1)
            hits = col.search(q, int(limit), [flt])[0]
        return models.QueryResponse(points=[col.point(r, s, with_payload, with_vectors)
                                            for r, s in hits])

    def query_batch_points(self, collection_name: str, requests: list,
                           **kwargs) -> list[models.QueryResponse]:
        """One GPU scan for the whole batch (per-query filters ride along in the kernel)."""
        col = self._col(collection_name)
        if not requests:
            return []
        limit = max(int(r.limit) for r in requests)
        qs = [r.query for r in requests]
        Q = torch.stack([x if isinstance(x, torch.Tensor) else
                         torch.as_tensor(np.asarray(x, np.float32)) for x in qs]) \
            if any(isinstance(x, torch.Tensor) for x in qs) else np.asarray(qs, np.float32)
        hits = col.search(Q, limit, [col.compile_filter(r.filter) for r in requests])
        return [models.QueryResponse(points=[col.point(i, s, r.with_payload)
                                             for i, s in h[:int(r.limit)]])
                for r, h in zip(requests, hits)]

    def search(self, collection_name: str, query_vector, limit: int = 10,
               query_filter=None, with_payload=True, **kwargs):
        """Legacy qdrant_client.search: list[ScoredPoint]."""
        return self.query_points(collection_name, query_vector, limit, query_filter,
                                 with_payload).points

    def close(self) -> None:
        if self.path is not None and self._collections:
            self.save()
        with self._lock:
            cols = list(self._collections.values())
            self._collections.clear()
        for c in cols:
            c.index.close()
