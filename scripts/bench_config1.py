"""BASELINE config 1 as a latency: one query -> bge-small encode -> cosine top-5
over a 1k-chunk collection with the ticker filter, through the drop-in function layer
(ragmi.rag.embed_query + retrieve_from_qdrant, main.py:211-239) after a corpus built by the
ingest path (ensure_collection / embed_chunks / chunk_points / upsert_points, ingest.py:52-175).

Model: a 12-layer bge-small-shaped checkpoint with seeded synthetic weights and a synthetic
WordPiece vocab written in the HF layout (the real checkpoint and vocab are not on disk, no hub
access). Chunks are synthetic financial-word sentences of ~150-220 tokens, 4 tickers.

CPU leg (reported baseline, not the target): the same query through transformers' BertModel
(fp32, torch CPU threads) + CLS L2-normalise + numpy fp32 cosine top-5 over the stored rows with
the same ticker mask — the reference's CPU path minus Qdrant's HTTP hop. Its top-5 ids are
compared with the GPU path's.

Prints one JSON line.
"""
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "financial-rag-system_amd"))

from ragmi import synth as R  # noqa: E402  (model shapes, seeded weights)

WORDS = ("apple iphone revenue services margin risk supply chain china tariffs cash flow "
         "dividend buyback microsoft azure cloud gaming licence windows office growth "
         "operating income net sales fiscal quarter guidance inflation currency debt "
         "segment americas europe greater wearables mac ipad research development "
         "liquidity capital expenditure repurchase share outstanding diluted earnings").split()
TICKERS = ("AAPL", "MSFT", "NVDA", "AMZN")
N_CHUNKS = int(os.environ.get("N_CHUNKS", 1000))
N_QUERIES = int(os.environ.get("N_QUERIES", 200))


def write_model(d, cfg, w, vocab):
    from ragmi.synth import write_checkpoint
    write_checkpoint(d, cfg, w, vocab, "bge")


def hf_bge(cfg, w):
    from transformers import BertConfig, BertModel
    c = BertConfig(vocab_size=cfg["vocab"], hidden_size=384, num_hidden_layers=cfg["layers"],
                   num_attention_heads=12, intermediate_size=1536, max_position_embeddings=512,
                   type_vocab_size=2, layer_norm_eps=1e-12, hidden_act="gelu",
                   hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    m = BertModel(c, add_pooling_layer=False)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in w.items()}, strict=False)
    return m.eval()


def main():
    vocab = ["[PAD]"] + [f"[unused{i}]" for i in range(99)] + ["[UNK]", "[CLS]", "[SEP]",
                                                               "[MASK]"]
    vocab += sorted(set(WORDS)) + [chr(c) for c in range(97, 123)] + list("0123456789")
    cfg = dict(R.BGE_SMALL, vocab=len(vocab))
    w = R.make_weights(cfg, 31)
    tmp = tempfile.mkdtemp(prefix="cfg1_")
    write_model(os.path.join(tmp, "bge"), cfg, w, vocab)
    os.environ["TESTING"] = "False"
    os.environ["USE_GPU"] = "true"
    os.environ["RAGMI_BGE_DIR"] = os.path.join(tmp, "bge")
    import ragmi.rag as rag

    rng = np.random.default_rng(0)

    def sentence(lo, hi):
        return " ".join(rng.choice(WORDS, rng.integers(lo, hi)))

    # ---- corpus build through the ingest path
    q = rag.get_qdrant()
    rag.ensure_collection(q)
    t0 = time.perf_counter()
    per = N_CHUNKS // len(TICKERS)
    for t in TICKERS:
        chunks = [sentence(150, 220) for _ in range(per)]
        emb = rag.embed_chunks(chunks)
        rag.upsert_points(q, rag.chunk_points(t, "10-K", "primary_document.html", chunks, emb))
    ingest_s = time.perf_counter() - t0
    n = q.count(rag.COLLECTION_NAME).count
    col = q._col(rag.COLLECTION_NAME)
    rows16 = col.index.export_rows().view(np.float16).astype(np.float32)[:n]

    queries = [sentence(6, 24) for _ in range(N_QUERIES)]
    tick = [TICKERS[i % len(TICKERS)] for i in range(N_QUERIES)]

    # ---- GPU path: per-request latency, as main.py serves one request
    for i in range(10):
        rag.retrieve_from_qdrant(rag.embed_query(queries[i]), tick[i], limit=5)
    torch.cuda.synchronize()
    lat, gpu_top = [], []
    for qq, t in zip(queries, tick):
        s = time.perf_counter()
        vec = rag.embed_query(qq)
        res = rag.retrieve_from_qdrant(vec, t, limit=5)
        lat.append(time.perf_counter() - s)
        gpu_top.append([p.id for p in res.points])
    lat = np.asarray(lat) * 1e3

    # ---- CPU leg: transformers BertModel + numpy cosine top-5, bounded sample
    m = hf_bge(cfg, w)
    tok = rag.get_embedder().tokenizer
    tags = [col.payloads[r]["ticker"] for r in range(n)]
    ids_by_row = [col.row_ids[r] for r in range(n)]
    cpu_lat, agree = [], 0
    n_cpu = min(N_QUERIES, int(os.environ.get("N_CPU", 50)))
    with torch.no_grad():
        for i in range(n_cpu):
            s = time.perf_counter()
            ids, tt, cu = tok.encode_packed([queries[i]])
            h = m(input_ids=torch.from_numpy(ids[None].astype(np.int64)),
                  token_type_ids=torch.from_numpy(tt[None].astype(np.int64))).last_hidden_state
            v = torch.nn.functional.normalize(h[:, 0], p=2, dim=1).numpy()[0]
            sc = rows16 @ v
            mask = np.fromiter((x == tick[i] for x in tags), bool, n)
            sc = np.where(mask, sc, -np.inf)
            top = np.argsort(-sc, kind="stable")[:5]
            cpu_lat.append(time.perf_counter() - s)
            agree += [ids_by_row[r] for r in top] == gpu_top[i]
    cpu_lat = np.asarray(cpu_lat) * 1e3
    print(json.dumps({
        "config": "1: single query, bge-small (12 layers) encode + cosine top-5 over "
                  f"{n} chunks, ticker filter",
        "gpu_ms_p50": round(float(np.median(lat)), 3),
        "gpu_ms_p99": round(float(np.percentile(lat, 99)), 3),
        "gpu_qps_serial": round(1e3 / float(np.median(lat)), 1),
        "cpu_ms_p50": round(float(np.median(cpu_lat)), 3),
        "cpu_threads": torch.get_num_threads(),
        "cpu_kind": "transformers BertModel fp32 + numpy cosine top-5",
        "top5_agree_vs_cpu": f"{agree}/{n_cpu}",
        "ingest_s": round(ingest_s, 2),
        "data": "synthetic (seeded weights, synthetic vocab and chunks)",
    }))


if __name__ == "__main__":
    main()
