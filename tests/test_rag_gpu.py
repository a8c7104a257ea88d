"""GPU end-to-end test of the drop-in function layer (ragmi.rag): ingest -> embed_query ->
retrieve_from_qdrant (ticker / document_type filters) -> rerank_documents, and the batched
forms, checked against the oracles. Models are 2-layer synthetic bge / cross-encoder
checkpoints with a synthetic vocab written to disk in the HF layout (the real ones are not
available offline)."""
import importlib
import json

import numpy as np
import pytest
import torch

import bert_ref as R
import oracle_scan as O

pytestmark = pytest.mark.gpu

WORDS = ("apple iphone revenue services margin risk supply chain china tariffs cash flow "
         "dividend buyback microsoft azure cloud gaming licence windows office growth "
         "operating income net sales fiscal quarter guidance inflation currency debt").split()


def _write_model(d, cfg, w, vocab, kind):
    """A local checkpoint in the real models' layout (ragmi.synth.write_checkpoint: bge with its
    Transformer -> Pooling(cls) -> Normalize stack, the cross-encoder with its configured
    Identity activation)."""
    from ragmi.synth import write_checkpoint
    write_checkpoint(str(d), cfg, w, vocab, kind)


@pytest.fixture(scope="module")
def rag(gpu, tmp_path_factory):
    vocab = ["[PAD]"] + [f"[unused{i}]" for i in range(99)] + ["[UNK]", "[CLS]", "[SEP]",
                                                               "[MASK]"]
    vocab += sorted(set(WORDS)) + [chr(c) for c in range(97, 123)] + list("0123456789")
    root = tmp_path_factory.mktemp("models")
    cb = dict(R.BGE_SMALL, vocab=len(vocab), layers=2)
    cc = dict(R.MINILM_CE, vocab=len(vocab), layers=2)
    wb, wc = R.make_weights(cb, 21), R.make_weights(cc, 22)
    _write_model(root / "bge", cb, wb, vocab, "bge")
    _write_model(root / "ce", cc, wc, vocab, "ce")
    mp = pytest.MonkeyPatch()
    mp.setenv("TESTING", "False")
    mp.setenv("USE_GPU", "true")                   # main.py:23,83: device = "cuda"
    mp.setenv("RAGMI_BGE_DIR", str(root / "bge"))
    mp.setenv("RAGMI_CE_DIR", str(root / "ce"))
    import ragmi.rag as rag
    rag = importlib.reload(rag)
    for f in (rag.get_embedder, rag.get_reranker, rag.get_qdrant):
        f.cache_clear()
    yield rag, (cb, wb), (cc, wc)
    mp.undo()


def _sentences(rng, n):
    return [" ".join(rng.choice(WORDS, rng.integers(6, 40))) for _ in range(n)]


def test_end_to_end_retrieval_and_rerank(rag):
    rag, (cb, wb), (cc, wc) = rag
    rng = np.random.default_rng(0)
    q = rag.get_qdrant()
    rag.ensure_collection(q)
    rag.ensure_collection(q)                       # idempotent
    docs = {}
    for ticker, ftype in (("aapl", "10-k"), ("aapl", "10-q"), ("msft", "10-k")):
        chunks = _sentences(rng, 120)
        emb = rag.embed_chunks(chunks)
        assert len(emb) == 120 and len(emb[0]) == 384
        pts = rag.chunk_points(ticker, ftype, "primary_document.html", chunks, emb)
        rag.upsert_points(q, pts)
        docs[(ticker, ftype)] = chunks
    n = q.count(rag.COLLECTION_NAME).count
    assert n == 360
    # re-ingest is idempotent (md5 ids overwrite)
    rag.upsert_points(q, rag.chunk_points("aapl", "10-k", "primary_document.html",
                                          docs[("aapl", "10-k")],
                                          rag.embed_chunks(docs[("aapl", "10-k")])))
    assert q.count(rag.COLLECTION_NAME).count == n

    col = q._col(rag.COLLECTION_NAME)
    # the collection stores fp32 rows (Qdrant's default Float32 datatype; ensure_collection
    # sets none, ingest.py:89-95): the oracle searches the stored fp32 rows
    assert col.index.storage == "fp32"
    enc16, tags = col.index.export_rows32(), col.index.export_tags()
    query = "what was apple iphone revenue growth in fiscal quarter"
    vec = rag.embed_query(query)
    assert len(vec) == 384 and abs(np.linalg.norm(vec) - 1) < 1e-5
    # stage 1 vs oracle embedding (fp16x3 encoder)
    tok = rag.get_embedder().tokenizer
    ids, tt, cu = tok.encode_packed([query])
    ref = R.bge_embed(wb, cb, ids[None], tt[None], np.ones((1, len(ids)), np.int64))
    np.testing.assert_allclose(vec, ref[0], atol=5e-5)

    res = rag.retrieve_from_qdrant(vec, "aapl")
    got = [p.id for p in res.points]
    assert len(got) == 15 and all(p.payload["ticker"] == "AAPL" for p in res.points)
    # stage 2 bit-exact vs the oracle on the stored rows with the same filter
    mask, val = col.compile_filter(rag._filter("aapl"))
    s2, i2 = O.search(enc16, np.asarray([vec], np.float32), 15, tags=tags, mask=mask,
                      value=val, use_filter=True)
    assert got == [col.row_ids[r] for r in i2[0]]
    assert [p.score for p in res.points] == [float(x) for x in s2[0]]
    res_d = rag.retrieve_from_qdrant(vec, "AAPL", document_type="10-q")
    assert all(p.payload["document_type"] == "10-Q" for p in res_d.points)
    assert rag.retrieve_from_qdrant(vec, "tsla").points == []

    # stage 3: rerank the retrieved texts (main.py:380-385)
    texts = [p.payload.get("text", "") for p in res.points]
    idx, scores = rag.rerank_documents(query, texts, 5)
    ids, tt, cu = rag.get_reranker().tokenizer.encode_packed([query] * len(texts), texts)
    L = np.diff(cu)
    S = int(L.max())
    pid = np.zeros((len(texts), S), np.int64)
    ptt = np.zeros_like(pid)
    pm = np.zeros_like(pid)
    for b in range(len(texts)):
        pid[b, :L[b]], ptt[b, :L[b]], pm[b, :L[b]] = ids[cu[b]:cu[b + 1]], tt[cu[b]:cu[b + 1]], 1
    ref = R.ce_logits(wc, cc, pid, ptt, pm)
    np.testing.assert_allclose(scores, ref, atol=1e-3)
    srt = np.sort(ref)[::-1]
    if np.min(np.abs(np.diff(srt[:6]))) > 2e-3:
        np.testing.assert_array_equal(idx, np.argsort(ref)[::-1][:5])

    # batched forms equal the per-request ones
    queries = [query, "microsoft azure cloud growth", "apple risk supply chain china"]
    tick = ["aapl", "msft", "aapl"]
    vecs = rag.embed_query_batch(queries)
    for i, qq in enumerate(queries):
        np.testing.assert_array_equal(vecs[i], rag.embed_query(qq))
    batch = rag.retrieve_batch(vecs, tick)
    for v, t, r in zip(vecs, tick, batch):
        one = rag.retrieve_from_qdrant(v, t)
        assert [p.id for p in r.points] == [p.id for p in one.points]
        assert [p.score for p in r.points] == [p.score for p in one.points]
    tl = [[p.payload["text"] for p in r.points] for r in batch]
    rb = rag.rerank_batch(queries, tl, 5)
    for qq, t, (bi, bs) in zip(queries, tl, rb):
        si, ss = rag.rerank_documents(qq, t, 5)
        np.testing.assert_array_equal(bs, ss)
        np.testing.assert_array_equal(bi, si)


def test_build_pairs_gpu_matches_torch(gpu):
    """rag_build_pairs (HIP) == ragmi.pairs.build_pairs (torch, itself CPU-tested against a
    per-pair loop), bit for bit, incl. truncation to max_len and -1 rows."""
    import torch
    from ragmi.pairs import build_pairs, build_pairs_gpu, build_pairs_gpu_async
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    rows_n, lmax = 5000, 300
    c_toks = torch.randint(0, 65535, (rows_n, lmax), generator=g, device="cuda",
                           dtype=torch.int32).to(torch.int16)
    c_lens = torch.randint(1, lmax + 1, (rows_n,), generator=g, device="cuda",
                           dtype=torch.int32)
    for B, K, max_len in ((32, 15, 512), (3, 7, 64), (1, 1, 512), (64, 16, 256)):
        ql = torch.randint(3, 40, (B,), generator=g, device="cuda")
        q_cu = torch.zeros(B + 1, dtype=torch.int32, device="cuda")
        q_cu[1:] = torch.cumsum(ql, 0)
        q_ids = torch.randint(1000, 30000, (int(q_cu[-1]),), generator=g, device="cuda",
                              dtype=torch.int32)
        rows = torch.randint(-1, rows_n, (B, K), generator=g, device="cuda")
        a = build_pairs(q_ids, q_cu, rows, c_toks, c_lens, max_len)
        b = build_pairs_gpu(q_ids, q_cu, rows, c_toks, c_lens, max_len)
        # the pipelined form: enqueue on a side stream, collect after more work was queued
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            pend = build_pairs_gpu_async(q_ids, q_cu, rows, c_toks, c_lens, max_len)
            _ = torch.randn(1 << 20, device="cuda").sum()
            c = pend.result()
        torch.cuda.synchronize()
        for x, y, z in zip(a[:3], b[:3], c[:3]):
            assert torch.equal(x.cpu(), y.cpu())
            assert torch.equal(x.cpu(), z.cpu())
        assert a[3] == b[3] == c[3]
