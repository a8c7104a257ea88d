"""On-disk shard format: the persistence that replaces the Qdrant volume (SURVEY §8f row 3;
docker-compose.yml's `qdrant_storage` volume, database.py:111-143 recreating the collection
at start-up).

A shard directory holds exactly what the GPU index stores, so loading is a byte copy:

  meta.json          {"format": "ragmi-shard", "version": 1, "dim": D, "count": N,
                      "storage": "fp16" | "fp32"}  (no "storage": fp16)
  vectors.f16.npy    [N, D] float16 — the stored (normalised, fp16-rounded) rows, row-major
  vectors.f32.npy    [N, D] float32 — instead, for fp32 storage: the normalised fp32 rows
                     (their fp16 scan copy is re-derived on load by the same rounding)
  tags.u32.npy       [N] uint32     — per-row payload tags (PayloadTags codes)

A collection directory adds the host-side state of `qdrant.Collection`:

  collection.json    name, dim, distance, tag fields + codebooks, op counter
  points.jsonl       one line per row, in row order: {"id": ..., "version": v, "payload": {...}}
  shard/             the shard above

Rows move host<->HBM in chunks (`chunk_rows`, default 1M rows = 768 MB at D=384) through
memory-mapped .npy files, so a 10M-row shard never needs the whole corpus in host RAM.
Saved rows are written back with rag_index_import_rows: no renormalisation, so a loaded
index returns bit-identical scores and ids to the one that was saved.
"""
from __future__ import annotations

import json
import os

import numpy as np

FORMAT = "ragmi-shard"
VERSION = 1
CHUNK_ROWS = 1 << 20


def _write_json(path, obj):
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(obj, f)
    os.replace(tmp, path)


def _vec_file(storage: str) -> tuple[str, type]:
    return ("vectors.f32.npy", np.float32) if storage == "fp32" else ("vectors.f16.npy", np.float16)


def _export(index, r0: int, m: int) -> np.ndarray:
    return (index.export_rows32(r0, m) if getattr(index, "storage", "fp16") == "fp32"
            else index.export_rows(r0, m).view(np.float16))


def save_index(index, path: str, chunk_rows: int = CHUNK_ROWS) -> None:
    """Write FlatIndex `index` (rows [0, count)) to shard directory `path`."""
    os.makedirs(path, exist_ok=True)
    n, d = index.count, index.dim
    storage = getattr(index, "storage", "fp16")
    vname, vdt = _vec_file(storage)
    # meta.json marks a complete save: drop it before the arrays are rewritten in place, so a
    # crash mid-save leaves an incomplete directory (load refuses it), never a stale meta.json
    # over partially written rows
    meta = os.path.join(path, "meta.json")
    if os.path.exists(meta):
        os.remove(meta)
    for old in ("vectors.f16.npy", "vectors.f32.npy"):   # a re-save may change storage
        if old != vname and os.path.exists(os.path.join(path, old)):
            os.remove(os.path.join(path, old))
    vec = np.lib.format.open_memmap(os.path.join(path, vname), mode="w+", dtype=vdt,
                                    shape=(n, d))
    tags = np.lib.format.open_memmap(os.path.join(path, "tags.u32.npy"), mode="w+",
                                     dtype=np.uint32, shape=(n,))
    for r0 in range(0, n, chunk_rows):
        m = min(chunk_rows, n - r0)
        vec[r0:r0 + m] = _export(index, r0, m)
        tags[r0:r0 + m] = index.export_tags(r0, m)
    vec.flush()
    tags.flush()
    del vec, tags
    # meta last: a directory without meta.json is an incomplete save
    _write_json(os.path.join(path, "meta.json"),
                {"format": FORMAT, "version": VERSION, "dim": d, "count": n,
                 "storage": storage})


def read_meta(path: str) -> dict:
    with open(os.path.join(path, "meta.json")) as f:
        meta = json.load(f)
    if meta.get("format") != FORMAT or meta.get("version") != VERSION:
        raise ValueError(f"{path}: not a {FORMAT} v{VERSION} directory")
    return meta


# Row-norm bounds the exact top-k certificate assumes (scan_kernels.hip kRowNorm, index_capi.hip
# store_eps): a stored fp16 row is the RNE rounding of a unit vector, ||c|| - 1 within
# 2^-11 + sqrt(D) 2^-25 (<= 1e-3 for D <= 1024); a stored fp32 row is fp32(x / ||x||),
# ||y|| - 1 within 2^-20. Zero rows (never-filled slots, zero vectors) are allowed.
NORM_TOL = {"fp16": 1e-3, "fp32": 2.0 ** -20}


def check_row_norms(v: np.ndarray, storage: str, first_row: int = 0) -> None:
    """Refuse rows a ragmi index could not have stored: the scan's per-query error bound (and
    with it the certified exact top-k) holds only for normalised rows, so a hand-built or
    corrupted shard must not load silently."""
    if v.size == 0:
        return
    x = np.asarray(v, dtype=np.float64 if storage == "fp32" else np.float32)
    nrm = np.sqrt(np.einsum("ij,ij->i", x, x, dtype=np.float64))
    bad = ~((nrm == 0.0) | (np.abs(nrm - 1.0) <= NORM_TOL[storage]))
    if bad.any():
        r = int(np.argmax(bad))
        raise ValueError(f"shard row {first_row + r} has norm {nrm[r]!r}: not a normalised "
                         f"{storage} row (shards must come from save_index / save_sharded)")


def load_into(index, path: str, row0: int = 0, chunk_rows: int = CHUNK_ROWS,
              rows: tuple[int, int] | None = None, check_norms: bool = True) -> int:
    """Copy a saved shard (or its row range `rows` = (start, stop)) into `index` at row0.
    Returns the number of rows loaded. The index must have capacity for them. Every row's
    norm is checked first (check_row_norms) unless check_norms=False."""
    meta = read_meta(path)
    if meta["dim"] != index.dim:
        raise ValueError(f"shard dim {meta['dim']} != index dim {index.dim}")
    saved = meta.get("storage", "fp16")
    into = getattr(index, "storage", "fp16")
    if saved == "fp16" and into == "fp32":
        raise ValueError(f"{path}: fp16 shard cannot fill an fp32-storage index (the fp32 "
                         "rows were not saved)")
    vec = np.load(os.path.join(path, _vec_file(saved)[0]), mmap_mode="r")
    tags = np.load(os.path.join(path, "tags.u32.npy"), mmap_mode="r")
    if vec.shape != (meta["count"], meta["dim"]) or tags.shape != (meta["count"],):
        raise ValueError(f"{path}: array shapes disagree with meta.json")
    a, b = rows if rows is not None else (0, meta["count"])
    if not 0 <= a <= b <= meta["count"]:
        raise ValueError("row range outside the shard")
    n = b - a
    if row0 + n > index.capacity:
        index.reserve(row0 + n)
    for c0 in range(0, n, chunk_rows):
        m = min(chunk_rows, n - c0)
        v = np.asarray(vec[a + c0:a + c0 + m])
        t = np.asarray(tags[a + c0:a + c0 + m])
        if check_norms:
            check_row_norms(v, saved, a + c0)
        nc = max(index.count, row0 + c0 + m)
        if into == "fp32":
            index.import_rows32(v, row0 + c0, t, new_count=nc)
        else:   # an fp32 shard into an fp16 index: upsert's RNE rounding of the fp32 rows
            index.import_rows(v.astype(np.float16), row0 + c0, t, new_count=nc)
    return n


def load_index(path: str, device=None, capacity: int | None = None):
    """A new FlatIndex holding the saved shard."""
    from .index import FlatIndex
    meta = read_meta(path)
    idx = FlatIndex(dim=meta["dim"], capacity=max(capacity or 0, meta["count"], 16),
                    device=device, storage=meta.get("storage", "fp16"))
    try:
        load_into(idx, path)
    except BaseException:
        idx.close()
        raise
    return idx


def save_sharded(sharded, path: str, chunk_rows: int = CHUNK_ROWS) -> None:
    """Collective: every rank of a ragmi.dist.ShardedIndex writes its rows [lo, hi) into ONE
    world-size-independent shard directory (rank 0 creates the files; ranks write disjoint
    row slices of the memory-mapped arrays; rank 0 writes meta.json last). Needs a
    filesystem all ranks see (one node). Rows a rank never filled are saved as zeros."""
    import torch.distributed as dist
    n, d = sharded.n_total, sharded.local.dim
    multi = sharded.world > 1
    storage = getattr(sharded.local, "storage", "fp16")
    vname, vdt = _vec_file(storage)
    vp, tp = os.path.join(path, vname), os.path.join(path, "tags.u32.npy")
    if sharded.rank == 0:
        os.makedirs(path, exist_ok=True)
        if os.path.exists(os.path.join(path, "meta.json")):
            os.remove(os.path.join(path, "meta.json"))
        np.lib.format.open_memmap(vp, mode="w+", dtype=vdt, shape=(n, d)).flush()
        np.lib.format.open_memmap(tp, mode="w+", dtype=np.uint32, shape=(n,)).flush()
    if multi:
        dist.barrier(group=sharded.group)
    vec = np.load(vp, mmap_mode="r+")
    tags = np.load(tp, mmap_mode="r+")
    have = min(sharded.local.count, sharded.rows)
    for c0 in range(0, have, chunk_rows):
        m = min(chunk_rows, have - c0)
        g = sharded.lo + c0
        vec[g:g + m] = _export(sharded.local, c0, m)
        tags[g:g + m] = sharded.local.export_tags(c0, m)
    vec.flush()
    tags.flush()
    del vec, tags
    if multi:
        dist.barrier(group=sharded.group)
    if sharded.rank == 0:
        _write_json(os.path.join(path, "meta.json"),
                    {"format": FORMAT, "version": VERSION, "dim": d, "count": n,
                     "storage": storage})
    if multi:
        dist.barrier(group=sharded.group)


def load_sharded(sharded, path: str, chunk_rows: int = CHUNK_ROWS) -> int:
    """Each rank loads its own rows [lo, hi) of a saved shard directory (any world size)."""
    meta = read_meta(path)
    if meta["count"] != sharded.n_total:
        raise ValueError(f"saved shard has {meta['count']} rows, index expects "
                         f"{sharded.n_total}")
    return load_into(sharded.local, path, 0, chunk_rows, rows=(sharded.lo, sharded.hi))


# ---------------------------------------------------------------- collections
def save_collection(col, path: str) -> None:
    """qdrant.Collection -> collection directory."""
    os.makedirs(path, exist_ok=True)
    with col.lock:
        save_index(col.index, os.path.join(path, "shard"))
        tmp = os.path.join(path, "points.jsonl.tmp")
        with open(tmp, "w") as f:
            for pid, ver, pl in zip(col.row_ids, col.versions, col.payloads):
                f.write(json.dumps({"id": pid, "version": ver, "payload": pl}) + "\n")
        os.replace(tmp, os.path.join(path, "points.jsonl"))
        _write_json(os.path.join(path, "collection.json"), {
            "name": col.name, "dim": col.dim, "distance": "Cosine", "op": col.op,
            "storage": col.index.storage,
            "tag_fields": list(col.tags.fields),
            "codebooks": [[[v, c] for v, c in t.items()] for t in col.tags.codes]})


def load_collection(path: str, device=None):
    """collection directory -> qdrant.Collection (rows, tags, ids, payloads, versions)."""
    from .qdrant import Collection
    with open(os.path.join(path, "collection.json")) as f:
        cj = json.load(f)
    meta = read_meta(os.path.join(path, "shard"))
    col = Collection(cj["name"], int(cj["dim"]), device, tuple(cj["tag_fields"]),
                     capacity=max(meta["count"], 1024),
                     storage=cj.get("storage", meta.get("storage", "fp16")))
    for f_i, book in enumerate(cj["codebooks"]):
        col.tags.codes[f_i] = {v: int(c) for v, c in book}
    with open(os.path.join(path, "points.jsonl")) as f:
        for line in f:
            rec = json.loads(line)
            col.id_to_row[rec["id"]] = len(col.row_ids)
            col.row_ids.append(rec["id"])
            col.versions.append(int(rec["version"]))
            col.payloads.append(rec["payload"])
    if len(col.row_ids) != meta["count"]:
        col.index.close()
        raise ValueError(f"{path}: {len(col.row_ids)} points but {meta['count']} shard rows")
    col.op = int(cj["op"])
    load_into(col.index, os.path.join(path, "shard"))
    return col
