"""CPU tests of the persistence layer (ragmi.store): shard directory
format, chunked save/load, row-range loads, the collective sharded save at world size 2 and
reload at world size 3 (gloo on 127.0.0.1). The index here is a numpy stand-in with the
FlatIndex row I/O surface (export_rows/export_tags/import_rows/reserve); the GPU round trip
through libragmi is tests/test_store_gpu.py."""
import json
import os
import socket
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _paths():
    for p in (ROOT, os.path.join(ROOT, "financial-rag-system_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)


class HostIndex:
    """numpy stand-in for FlatIndex's row I/O (stored rows as uint16 fp16 bits)."""

    def __init__(self, dim, capacity=16):
        self.dim = dim
        self.rows = np.zeros((capacity, dim), np.uint16)
        self.tags = np.zeros(capacity, np.uint32)
        self.count = 0

    @property
    def capacity(self):
        return self.rows.shape[0]

    def reserve(self, cap):
        if cap > self.capacity:
            r = np.zeros((cap, self.dim), np.uint16)
            t = np.zeros(cap, np.uint32)
            r[:self.capacity], t[:self.capacity] = self.rows, self.tags
            self.rows, self.tags = r, t

    def export_rows(self, row0=0, n=None):
        n = self.count - row0 if n is None else n
        return self.rows[row0:row0 + n].copy()

    def export_tags(self, row0=0, n=None):
        n = self.count - row0 if n is None else n
        return self.tags[row0:row0 + n].copy()

    def import_rows(self, a, row0=0, tags=None, new_count=None):
        a = np.asarray(a)
        a = a.view(np.uint16) if a.dtype == np.float16 else a
        assert row0 + len(a) <= self.capacity
        self.rows[row0:row0 + len(a)] = a
        if tags is not None:
            self.tags[row0:row0 + len(a)] = tags
        self.count = new_count if new_count is not None else max(self.count, row0 + len(a))


def _filled(n, dim, seed):
    rng = np.random.default_rng(seed)
    h = HostIndex(dim, n)
    x = rng.standard_normal((n, dim))
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    x[::97] = 0.0                                    # never-filled slots are zero rows
    h.import_rows(x.astype(np.float16), 0,
                  rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32), n)
    return h


def test_save_load_roundtrip_chunked(tmp_path):
    _paths()
    from ragmi import store
    src = _filled(1000, 384, 0)
    store.save_index(src, str(tmp_path / "s"), chunk_rows=97)
    meta = json.loads((tmp_path / "s" / "meta.json").read_text())
    assert meta == {"format": "ragmi-shard", "version": 1, "dim": 384, "count": 1000,
                    "storage": "fp16"}
    v = np.load(tmp_path / "s" / "vectors.f16.npy")
    assert v.dtype == np.float16 and v.shape == (1000, 384)
    dst = HostIndex(384)
    assert store.load_into(dst, str(tmp_path / "s"), chunk_rows=128) == 1000
    assert dst.count == 1000
    np.testing.assert_array_equal(dst.export_rows(), src.export_rows())
    np.testing.assert_array_equal(dst.export_tags(), src.export_tags())
    part = HostIndex(384)
    store.load_into(part, str(tmp_path / "s"), rows=(300, 650), chunk_rows=64)
    np.testing.assert_array_equal(part.export_rows(), src.export_rows(300, 350))


def test_incomplete_or_foreign_directories_refused(tmp_path):
    _paths()
    from ragmi import store
    src = _filled(10, 32, 1)
    store.save_index(src, str(tmp_path / "s"))
    os.remove(tmp_path / "s" / "meta.json")             # incomplete save
    with pytest.raises(FileNotFoundError):
        store.load_into(HostIndex(32), str(tmp_path / "s"))
    store.save_index(src, str(tmp_path / "s"))
    with pytest.raises(ValueError):
        store.load_into(HostIndex(64), str(tmp_path / "s"))      # dim mismatch
    (tmp_path / "s" / "meta.json").write_text(json.dumps({"format": "x", "version": 1}))
    with pytest.raises(ValueError):
        store.load_into(HostIndex(32), str(tmp_path / "s"))
    with pytest.raises(ValueError):
        store.save_index(src, str(tmp_path / "t"))
        store.load_into(HostIndex(32), str(tmp_path / "t"), rows=(5, 11))


def test_empty_index(tmp_path):
    _paths()
    from ragmi import store
    store.save_index(HostIndex(384), str(tmp_path / "e"))
    dst = HostIndex(384)
    assert store.load_into(dst, str(tmp_path / "e")) == 0 and dst.count == 0


def _worker(rank, world, port, n, path, mode, q):
    _paths()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ragmi.dist import ShardedIndex
        full = _filled(n, 64, 7)
        if mode == "save":
            sh = ShardedIndex(n, local=HostIndex(64))
            sh.local.reserve(sh.rows)
            sh.local.import_rows(full.rows[sh.lo:sh.hi], 0, full.tags[sh.lo:sh.hi], sh.rows)
            sh.save(path)
        else:
            sh = ShardedIndex(n, local=HostIndex(64))
            got = sh.load(path)
            ok = (got == sh.rows and sh.local.count == sh.rows and
                  np.array_equal(sh.local.export_rows(), full.rows[sh.lo:sh.hi]) and
                  np.array_equal(sh.local.export_tags(), full.tags[sh.lo:sh.hi]))
            q.put((rank, ok))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_sharded_save_world2_load_world3(tmp_path):
    n, path = 1001, str(tmp_path / "g")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.start_processes(_worker, args=(2, _free_port(), n, path, "save", q), nprocs=2,
                       start_method="spawn")
    meta = json.loads(open(os.path.join(path, "meta.json")).read())
    assert meta["count"] == n
    full = _filled(n, 64, 7)
    np.testing.assert_array_equal(np.load(os.path.join(path, "vectors.f16.npy")).view(np.uint16),
                                  full.rows)
    mp.start_processes(_worker, args=(3, _free_port(), n, path, "load", q), nprocs=3,
                       start_method="spawn")
    res = sorted(q.get(timeout=60) for _ in range(3))
    assert res == [(0, True), (1, True), (2, True)]


def test_save_drops_stale_meta_before_rewriting(tmp_path):
    """A save over an existing shard removes meta.json first: if the rewrite dies midway the
    directory is refused by load instead of pairing the old meta with partial rows."""
    _paths()
    from ragmi import store
    idx = HostIndex(8, 64)
    idx.import_rows(np.arange(40 * 8, dtype=np.uint16).reshape(40, 8), 0, None, 40)
    d = str(tmp_path / "s")
    store.save_index(idx, d)
    assert os.path.exists(os.path.join(d, "meta.json"))

    class Boom(HostIndex):
        def export_rows(self, r0, n):
            raise RuntimeError("crash mid-save")

    bad = Boom(8, 64)
    bad.count = 40
    with pytest.raises(RuntimeError):
        store.save_index(bad, d)
    assert not os.path.exists(os.path.join(d, "meta.json"))
    with pytest.raises(FileNotFoundError):
        store.read_meta(d)


class HostIndex32(HostIndex):
    """fp32-storage stand-in: fp32 rows kept, the fp16 copy derived by RNE rounding."""
    storage = "fp32"

    def __init__(self, dim, capacity=16):
        super().__init__(dim, capacity)
        self.rows32 = np.zeros((capacity, dim), np.float32)

    def reserve(self, cap):
        old = self.capacity
        super().reserve(cap)
        if self.rows32.shape[0] < self.capacity:
            r = np.zeros((self.capacity, self.dim), np.float32)
            r[:old] = self.rows32[:old]
            self.rows32 = r

    def export_rows32(self, row0=0, n=None):
        n = self.count - row0 if n is None else n
        return self.rows32[row0:row0 + n].copy()

    def import_rows32(self, a, row0=0, tags=None, new_count=None):
        a = np.asarray(a, np.float32)
        self.rows32[row0:row0 + len(a)] = a
        self.import_rows(a.astype(np.float16), row0, tags, new_count)


def test_fp32_storage_roundtrip_and_downcast(tmp_path):
    """fp32 storage saves vectors.f32.npy (meta storage fp32) and reloads bit for bit; the
    same shard loads into an fp16 index as the RNE rounding of its rows; an fp16 shard is
    refused by an fp32 index (its fp32 rows were never saved)."""
    _paths()
    from ragmi import store
    rng = np.random.default_rng(4)
    n, d = 700, 384
    src = HostIndex32(d, 1024)
    v = rng.standard_normal((n, d)).astype(np.float32)
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    src.import_rows32(v, 0, rng.integers(0, 9, n).astype(np.uint32), new_count=n)
    p = str(tmp_path / "s32")
    store.save_index(src, p, chunk_rows=256)
    assert store.read_meta(p)["storage"] == "fp32"
    assert os.path.exists(os.path.join(p, "vectors.f32.npy"))
    assert not os.path.exists(os.path.join(p, "vectors.f16.npy"))
    dst = HostIndex32(d)
    assert store.load_into(dst, p, chunk_rows=300) == n
    assert np.array_equal(dst.rows32[:n], v) and np.array_equal(dst.rows[:n], src.rows[:n])
    assert np.array_equal(dst.tags[:n], src.tags[:n])
    d16 = HostIndex(d)
    store.load_into(d16, p)
    assert np.array_equal(d16.rows[:n], v.astype(np.float16).view(np.uint16))
    p16 = str(tmp_path / "s16")
    store.save_index(d16, p16)
    with pytest.raises(ValueError, match="fp16 shard"):
        store.load_into(HostIndex32(d), p16)


def test_unnormalised_rows_refused(tmp_path):
    """A hand-built or corrupted shard (rows not unit-norm) would void the exact top-k
    certificate (its error bound assumes ||c|| <= 1.001): load refuses it, naming the row."""
    _paths()
    from ragmi import store
    src = _filled(300, 64, 9)
    bad = src.rows[123].view(np.float16).astype(np.float32) * 1.01
    src.rows[123] = bad.astype(np.float16).view(np.uint16)
    p = str(tmp_path / "bad")
    store.save_index(src, p)
    with pytest.raises(ValueError, match="shard row 123"):
        store.load_into(HostIndex(64), p, chunk_rows=100)
    assert store.load_into(HostIndex(64), p, check_norms=False) == 300
    rng = np.random.default_rng(1)
    v = rng.standard_normal((50, 64)).astype(np.float32)
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    store.check_row_norms(v, "fp32")
    v[7] *= 1.0 + 1e-5
    with pytest.raises(ValueError, match="shard row 107"):
        store.check_row_norms(v, "fp32", first_row=100)
