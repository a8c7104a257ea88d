"""Host logic of bench.py's measurement helpers on CPU tensors (no GPU): recall@5 against
the unrounded fp32 corpus, including a corpus split over two shards whose per-shard lists
are merged the way rank 0 merges them; the certified per-batch exactness check against the
oracle (unsharded and over two shards), which must flag a wrong answer."""
import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


@pytest.fixture
def small_chunks(monkeypatch):
    monkeypatch.setattr(bench, "CHUNK", 1000)

    def gen_chunk(c, dev, rows=1000):
        g = torch.Generator()
        g.manual_seed(1000 + c)
        return torch.randn((rows, bench.D), generator=g)

    monkeypatch.setattr(bench, "gen_chunk", gen_chunk)
    return gen_chunk


def _corpus(gen_chunk, n):
    return torch.cat([gen_chunk(c, None, bench.chunk_rows(c, n))
                      for c in range((n + bench.CHUNK - 1) // bench.CHUNK)])


def test_recall_fp32_exact_and_reversed(small_chunks):
    n = 2500
    x = _corpus(small_chunks, n)
    q = x[[5, 1200, 2400, 77]] + 0.01 * torch.randn(4, bench.D)
    qn = torch.nn.functional.normalize(q, dim=1)
    xn = torch.nn.functional.normalize(x, dim=1)
    ref = torch.topk(qn @ xn.T, 15, dim=1).indices.numpy()
    dev = torch.device("cpu")
    assert bench.recall_fp32(q, ref, 0, n, n, 0, 1, dev).mean() == 1.0
    # the best 5 replaced by ranks 11..15: no overlap
    assert bench.recall_fp32(q, ref[:, ::-1].copy(), 0, n, n, 0, 1, dev).mean() == 0.0


def test_recall_fp32_shard_merge_matches_unsharded(small_chunks, monkeypatch):
    """Two shards [0, 1300) and [1300, 2500): each computes its own top-15 with global row ids;
    merging them as rank 0 does gives the unsharded top-5."""
    n, cut = 2500, 1300
    x = _corpus(small_chunks, n)
    q = x[[10, 1290, 1310, 2499]] + 0.01 * torch.randn(4, bench.D)
    dev = torch.device("cpu")
    qn = torch.nn.functional.normalize(q, dim=1)
    xn = torch.nn.functional.normalize(x, dim=1)
    ref = torch.topk(qn @ xn.T, 15, dim=1).indices.numpy()
    # capture each shard's partial result through a fake all_gather_object
    shard_parts = []
    for lo, hi in ((0, cut), (cut, n)):
        got = {}

        def fake_gather(out, obj, _got=got):
            _got["mine"] = obj
            for i in range(len(out)):
                out[i] = obj
        monkeypatch.setattr(bench.dist, "all_gather_object", fake_gather)
        bench.recall_fp32(q, ref, lo, hi, n, 1, 2, dev)   # rank 1: returns None
        shard_parts.append(got["mine"])

    def merged_gather(out, obj):
        out[0], out[1] = shard_parts
    monkeypatch.setattr(bench.dist, "all_gather_object", merged_gather)
    assert bench.recall_fp32(q, ref, 0, cut, n, 0, 2, dev).mean() == 1.0
    S = np.concatenate([p[0] for p in shard_parts], axis=1)
    I = np.concatenate([p[1] for p in shard_parts], axis=1)
    top5 = np.take_along_axis(I, np.argsort(-S, axis=1, kind="stable")[:, :5], axis=1)
    assert all(set(top5[b]) == set(ref[b, :5]) for b in range(4))


class _Shard:
    """export_rows surface of FlatIndex over oracle-encoded rows."""

    def __init__(self, enc):
        self.enc = enc

    def export_rows(self):
        return self.enc


def _oracle():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_scan as O
    return O


def test_verify_exact_unsharded_flags_wrong_answers():
    O = _oracle()
    rng = np.random.default_rng(4)
    n = 3000
    x = rng.standard_normal((n, bench.D)).astype(np.float32)
    enc = O.encode_rows(x)
    q = np.concatenate([x[[3, 900]] + 0.05 * rng.standard_normal((2, bench.D)).astype(np.float32),
                        rng.standard_normal((2, bench.D)).astype(np.float32)])
    s, i = O.search(enc, q, bench.K_TOP)
    r5, ok = bench.verify_exact(_Shard(enc), q, s, i, 0, 0, 1, torch.device("cpu"))
    assert ok.all() and (r5 == 1.0).all()
    bad_i = i.copy()
    bad_i[1, 0], bad_i[1, 14] = bad_i[1, 14], bad_i[1, 0]      # order swapped
    bad_i[2, 3] = (bad_i[2, 3] + 1) % n                         # a wrong row
    r5, ok = bench.verify_exact(_Shard(enc), q, s, bad_i, 0, 0, 1, torch.device("cpu"))
    assert list(ok) == [True, False, False, True]
    assert r5[2] < 1.0


def test_verify_exact_two_shards(monkeypatch):
    O = _oracle()
    rng = np.random.default_rng(5)
    n, cut = 3000, 1700
    x = rng.standard_normal((n, bench.D)).astype(np.float32)
    enc = O.encode_rows(x)
    q = x[[10, 1650, 1800, 2999]] + 0.05 * rng.standard_normal((4, bench.D)).astype(np.float32)
    s, i = O.search(enc, q, bench.K_TOP)
    shards = [(0, enc[:cut]), (cut, enc[cut:])]
    qn = O.normalize(q)
    # the all-reduce MAX of the per-rank exact scores of the returned rows
    e_all = np.maximum(*[O.rescore(e, qn, np.where((i >= lo) & (i < lo + len(e)), i - lo, -1))
                         for lo, e in shards])
    parts = []
    for rank, (lo, e) in enumerate(shards):
        def fake_reduce(t, op=None):
            t.copy_(torch.from_numpy(e_all))

        def fake_gather(out, obj):
            parts.append(obj)
            for j in range(len(out)):
                out[j] = obj
        monkeypatch.setattr(bench.dist, "all_reduce", fake_reduce)
        monkeypatch.setattr(bench.dist, "all_gather_object", fake_gather)
        bench.verify_exact(_Shard(e), q, s, i, lo, 1, 2, torch.device("cpu"))

    def merged(out, obj):
        out[0], out[1] = parts
    monkeypatch.setattr(bench.dist, "all_gather_object", merged)
    r5, ok = bench.verify_exact(_Shard(shards[0][1]), q, s, i, 0, 0, 2, torch.device("cpu"))
    assert ok.all() and (r5 == 1.0).all()


def test_busy_union_counts_overlap_once():
    """bench.py's device time for overlapped scan launches: the union of their intervals."""
    import numpy as np
    from ragmi.index import busy_union_ms
    assert busy_union_ms(np.array([]), np.array([])) == 0.0
    # disjoint: the plain sum of durations (== the average launch duration x launches)
    assert busy_union_ms(np.array([0.0, 2.0, 5.0]), np.array([1.0, 3.0, 6.5])) == 3.5
    # nested / overlapping / unsorted, negative starts (launches recorded before the first)
    a = np.array([4.0, 0.0, 0.5, -1.0, 10.0])
    b = np.array([6.0, 2.0, 1.0, 0.25, 10.5])
    assert busy_union_ms(a, b) == (2.0 - (-1.0)) + 2.0 + 0.5


# ------------------------------------------------------------------ N-rank launcher (bench.py)
_RANK_BODY = ("import json, os, sys\n"
              "keys = ['RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'LOCAL_WORLD_SIZE', 'MASTER_ADDR',"
              " 'MASTER_PORT', 'HSA_ENABLE_IPC_MODE_LEGACY']\n"
              "open(os.path.join(os.environ['OUT'], os.environ['RANK']), 'w')"
              ".write(json.dumps({k: os.environ.get(k) for k in keys}))\n")


def test_launch_ranks_starts_n_children_with_the_env_contract(tmp_path):
    env = dict(os.environ, OUT=str(tmp_path))
    env.pop("WORLD_SIZE", None)
    rc = bench.launch_ranks(4, [], cmd=[sys.executable, "-c", _RANK_BODY], env=env)
    assert rc == 0
    import json
    got = {int(p.name): json.loads(p.read_text()) for p in tmp_path.iterdir()}
    assert sorted(got) == [0, 1, 2, 3]
    ports = {g["MASTER_PORT"] for g in got.values()}
    assert len(ports) == 1 and int(ports.pop()) > 0
    for r, g in got.items():
        assert g["RANK"] == g["LOCAL_RANK"] == str(r)
        assert g["WORLD_SIZE"] == g["LOCAL_WORLD_SIZE"] == "4"
        assert g["MASTER_ADDR"] == "127.0.0.1"
        assert g["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_launch_ranks_failure_stops_the_others(tmp_path):
    """rank 1 fails at once; the others would sleep for a minute: the launcher must return
    rank 1's status and terminate them."""
    body = ("import os, sys, time\n"
            "if os.environ['RANK'] == '1': sys.exit(3)\n"
            "time.sleep(60)\n")
    import time as _t
    t0 = _t.time()
    rc = bench.launch_ranks(3, [], cmd=[sys.executable, "-c", body], env=dict(os.environ))
    assert rc == 3
    assert _t.time() - t0 < 30


def test_check_world_mismatch_and_default():
    assert bench.check_world(1, {}) == 1
    assert bench.check_world(8, {}) == 8                    # launch_ranks will start 8
    assert bench.check_world(2, {"WORLD_SIZE": "2"}) == 2   # under torch.distributed.run
    with pytest.raises(SystemExit) as e:
        bench.check_world(8, {"WORLD_SIZE": "1"})
    assert e.value.code == 2
    with pytest.raises(SystemExit):
        bench.check_world(0, {})


def test_bench_py_refuses_world_size_mismatch_before_gpu():
    """`WORLD_SIZE=3 python bench.py --gpus 2` exits 2 before any GPU or data work."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 2
    assert "WORLD_SIZE=3" in r.stderr


def test_scan_traffic_table(tmp_path):
    import json
    p = tmp_path / "pmc.json"
    p.write_text(json.dumps({"hbm_bytes_per_launch": 7.7e9, "source": "a.csv", "commit": "x",
                             "by_rows_per_gpu": {"1250000": {"hbm_bytes_per_launch": 9.7e8,
                                                             "source": "b.csv"}}}))
    b, src = bench.scan_traffic(10_000_000, path=str(p))
    assert b == 7.7e9 and "a.csv" in src and "10000000 rows" in src
    b, src = bench.scan_traffic(1_250_000, path=str(p))
    assert b == 9.7e8 and "b.csv" in src
    assert bench.scan_traffic(2_500_000, path=str(p)) == (None, None)
    assert bench.scan_traffic(10_000_000, "fp32", path=str(p)) == (None, None)
    assert bench.scan_traffic(10_000_000, path=str(tmp_path / "missing.json")) == (None, None)


def test_bench_py_help_renders():
    """every option's help text formats (argparse %-expands help strings)"""
    import subprocess
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--help"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "--legs" in r.stdout and "--certify" in r.stdout
