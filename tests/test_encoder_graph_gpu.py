"""hipGraph replay of small-batch encoder forwards (rag_encoder_set_graphs; round 3).

A replay stages the call's ids / types / cu into the stream's workspace, replays the graph
captured for the padded shape (T to a multiple of 64, max_len to a multiple of 32) and copies
the output rows out (a call on the null stream replays on the encoder's own stream between
two events). Checked here:
  * the replayed outputs match the eager forward of the same batch (within 1e-6: the padded
    T may pick a different GEMM tiling, never a different arithmetic) and the oracle within
    the encoders' bars (bge 5e-5, CE 1e-3);
  * a graph reused for a different batch of the same padded shape reads the NEW inputs;
  * more shapes than the per-workspace cache holds (LRU eviction) stay correct;
  * the CE head (one logit per row), graphs on two streams at once, and null-stream calls
    whose inputs are produced and outputs consumed by null-stream work.
"""
import numpy as np
import pytest
import torch

import bert_ref as R

pytestmark = pytest.mark.gpu


def _batch(rng, B, lo, hi, pair=False):
    lens = rng.integers(lo, hi + 1, B)
    ids = np.zeros((B, int(lens.max())), np.int64)
    tt, m = np.zeros_like(ids), np.zeros_like(ids)
    for b, L in enumerate(lens):
        t = rng.integers(1000, 30522, L)
        t[0], t[L - 1] = 101, 102
        if pair:
            cut = int(rng.integers(4, max(5, L // 3)))
            t[cut] = 102
            tt[b, cut + 1:L] = 1
        ids[b, :L] = t
        m[b, :L] = 1
    return ids, tt, m


def _packed(ids, tt, m):
    lens = m.sum(1)
    cu = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    fi = np.concatenate([ids[b, :L] for b, L in enumerate(lens)]).astype(np.int32)
    ft = np.concatenate([tt[b, :L] for b, L in enumerate(lens)]).astype(np.int32)
    return fi, ft, cu


@pytest.fixture(scope="module")
def encs(gpu):
    from ragmi.encoders import HEAD_CLS_L2, HEAD_POOLER_CLS, BertEncoder
    wb = R.make_weights(R.BGE_SMALL, 11)
    wc = R.make_weights(R.MINILM_CE, 12)
    eb = BertEncoder(R.BGE_SMALL, wb, HEAD_CLS_L2, gpu, "fp16x3")
    ec = BertEncoder(R.MINILM_CE, wc, HEAD_POOLER_CLS, gpu, "fp16x3")
    yield (eb, wb), (ec, wc)
    eb.close()
    ec.close()


def _run(enc, packed, mode, stream):
    enc.set_graphs(mode)
    with torch.cuda.stream(stream):
        out = enc.forward_packed(*packed)
    stream.synchronize()
    return out.cpu().numpy()


def test_graph_matches_eager_and_oracle(encs, gpu):
    (eb, wb), (ec, wc) = encs
    rng = np.random.default_rng(5)
    st = torch.cuda.Stream(gpu)
    try:
        for B, lo, hi in ((32, 12, 30), (1, 5, 9), (7, 30, 70), (32, 16, 27)):
            ids, tt, m = _batch(rng, B, lo, hi)
            p = _packed(ids, tt, m)
            ge = _run(eb, p, 1, st)
            ee = _run(eb, p, 0, st)
            ref = R.bge_embed(wb, R.BGE_SMALL, ids, tt, m)
            assert np.abs(ge - ee).max() <= 1e-6
            assert np.abs(ge - ref).max() <= 5e-5
            ids, tt, m = _batch(rng, B, lo + 10, hi + 40, pair=True)
            p = _packed(ids, tt, m)
            gc = _run(ec, p, 1, st)
            ecv = _run(ec, p, 0, st)
            refc = R.ce_logits(wc, R.MINILM_CE, ids, tt, m)
            assert np.abs(gc - ecv).max() <= 1e-6
            assert np.abs(gc - refc).max() <= 1e-3
    finally:
        eb.set_graphs(-1)
        ec.set_graphs(-1)


def test_graph_reuse_reads_new_inputs_and_evicts(encs, gpu):
    (eb, wb), _ = encs
    rng = np.random.default_rng(9)
    st = torch.cuda.Stream(gpu)
    try:
        # two batches of the same padded shape (same B, T and max_len buckets), then more
        # shapes than the cache holds, then the first shape again
        a = _batch(rng, 32, 16, 24)
        ids_b = np.where(a[2] > 0, rng.integers(1000, 30522, a[0].shape), 0)
        ids_b[:, 0] = 101
        b = (ids_b, a[1], a[2])                         # same lengths, new tokens
        pa, pb = _packed(*a), _packed(*b)
        ga = _run(eb, pa, 1, st)
        gb = _run(eb, pb, 1, st)
        assert np.abs(ga - R.bge_embed(wb, R.BGE_SMALL, *a)).max() <= 5e-5
        assert np.abs(gb - R.bge_embed(wb, R.BGE_SMALL, *b)).max() <= 5e-5
        assert np.abs(ga - gb).max() > 1e-2            # different inputs, different rows
        for B in range(2, 22):                          # 20 more shapes: LRU eviction
            c = _batch(rng, B, 8, 16)
            gc = _run(eb, _packed(*c), 1, st)
            assert np.abs(gc - R.bge_embed(wb, R.BGE_SMALL, *c)).max() <= 5e-5
        assert np.abs(_run(eb, pa, 1, st) - ga).max() == 0.0
    finally:
        eb.set_graphs(-1)


def test_graphs_on_two_streams(encs, gpu):
    (eb, wb), _ = encs
    rng = np.random.default_rng(13)
    s1, s2 = torch.cuda.Stream(gpu), torch.cuda.Stream(gpu)
    batches = [_batch(rng, 32, 14, 28) for _ in range(6)]
    eb.set_graphs(1)
    try:
        outs = []
        for i, bt in enumerate(batches):
            st = s1 if i % 2 == 0 else s2
            with torch.cuda.stream(st):
                outs.append(eb.forward_packed(*_packed(*bt)))
        torch.cuda.synchronize(gpu)
        for bt, o in zip(batches, outs):
            assert np.abs(o.cpu().numpy() - R.bge_embed(wb, R.BGE_SMALL, *bt)).max() <= 5e-5
    finally:
        eb.set_graphs(-1)


def test_graph_on_null_stream_is_ordered(encs, gpu):
    """Default (null) stream: the replay runs on the encoder's stream, after the H2D copy of
    the inputs and before the null-stream ops that read the output."""
    (eb, wb), _ = encs
    rng = np.random.default_rng(21)
    eb.set_graphs(1)
    try:
        assert torch.cuda.current_stream(gpu).cuda_stream == 0
        for _ in range(4):
            bt = _batch(rng, 32, 12, 30)
            out = eb.forward_packed(*_packed(bt[0], bt[1], bt[2]))
            y = (out * 2.0).cpu().numpy() / 2.0          # consumed on the null stream
            assert np.abs(y - R.bge_embed(wb, R.BGE_SMALL, *bt)).max() <= 5e-5
    finally:
        eb.set_graphs(-1)
