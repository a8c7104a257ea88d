"""The reference's RAG-core function layer on the MI355X path (drop-in for main.py / main2.py /
ingest.py's hot-path functions, same names, arguments, return shapes and TESTING stubs).

  get_embedder / get_reranker / get_qdrant   main.py:80-95, main2.py:88-108 (lazy singletons)
  embed_query(query) -> list[float] (384)    main.py:211-213 (TESTING: zeros)
  embed_query_batch(queries) -> list[list]   main2.py:170-171
  embed(texts) -> {"embeddings": ...}        main.py:144-149 /embed (TESTING: zeros)
  retrieve_from_qdrant(vec, ticker, document_type=None, limit=15)
                                             main.py:215-239 (exception -> empty .points)
  rerank_documents(query, texts, top_k) -> (idx, scores)
                                             main.py:241-247 (TESTING: range / zeros)
  ensure_collection, embed_chunks, chunk_points, upsert_points
                                             ingest.py:52-66, 86-96, 148-175
plus the batched forms a rewritten main2.batch_processor uses:
  retrieve_batch  -> one GPU scan for all requests of a micro-batch (per-query filters)
  rerank_batch    -> one cross-encoder forward for all (query, chunk) pairs of a micro-batch

Models come from local directories (env RAGMI_BGE_DIR, RAGMI_CE_DIR: config.json +
model.safetensors + vocab.txt) — the reference's hub names cannot be fetched here. Env
RAGMI_STORAGE (optional) points the in-HBM collection at an on-disk shard directory
(ragmi.store), the role of the reference's Qdrant storage volume.
"""
from __future__ import annotations

import hashlib
import os
from datetime import datetime, timezone
from functools import lru_cache

import numpy as np

from . import qdrant_models as models

TESTING = os.getenv("TESTING", "False") == "True"
QDRANT_URL = os.getenv("QDRANT_URL", "http://qdrant:6333")
COLLECTION_NAME = "financial_documents"          # main.py:25
VECTOR_SIZE = 384                                # database.py:31
EMBED_BATCH = 64                                 # ingest.py:27
UPSERT_BATCH = 256                               # ingest.py:28
RETRIEVE_LIMIT = 15                              # main.py:215
PRECISION = os.getenv("RAGMI_PRECISION", "fp16x3")
# main.py:23 — the loaders pass device = "cuda" if USE_GPU else "cpu" (main.py:83,89), read per
# call here so tests can set it; "cpu" makes the encoders raise RagmiDeviceError (this build
# has no CPU path): set USE_GPU=true, as the reference needs on a GPU host.


def _device() -> str:
    return "cuda" if os.getenv("USE_GPU", "false").lower() == "true" else "cpu"


def _testing() -> bool:
    return os.getenv("TESTING", "False") == "True"


# ------------------------------------------------------------------ lazy loaders
@lru_cache()
def get_embedder():
    if _testing():
        return None
    from .encoders import SentenceTransformer
    d = os.environ.get("RAGMI_BGE_DIR")
    if not d:
        raise RuntimeError("set RAGMI_BGE_DIR to a local bge-small-en-v1.5 directory "
                           "(config.json, model.safetensors, vocab.txt)")
    return SentenceTransformer(d, device=_device(), precision=PRECISION)


@lru_cache()
def get_reranker():
    if _testing():
        return None
    from .encoders import CrossEncoder
    d = os.environ.get("RAGMI_CE_DIR")
    if not d:
        raise RuntimeError("set RAGMI_CE_DIR to a local ms-marco-MiniLM-L-6-v2 directory")
    return CrossEncoder(d, device=_device(), precision=PRECISION)


@lru_cache()
def get_qdrant():
    if _testing():
        return None
    from .qdrant import QdrantClient
    # RAGMI_STORAGE: directory of saved collections (the Qdrant volume's role); loaded here,
    # written back by QdrantClient.save()/close()
    return QdrantClient(url=QDRANT_URL, path=os.environ.get("RAGMI_STORAGE") or None)


# ------------------------------------------------------------------ stage 1: embed
def embed_query(query: str):
    if _testing():
        return [0.0] * VECTOR_SIZE
    return get_embedder().encode(query).tolist()


def embed_query_batch(queries):
    if _testing():
        return [[0.0] * VECTOR_SIZE for _ in queries]
    return get_embedder().encode(list(queries)).tolist()


def embed(texts):
    """/embed endpoint body (main.py:144-149)."""
    if _testing():
        return {"embeddings": [[0.0] * VECTOR_SIZE for _ in texts]}
    return {"embeddings": get_embedder().encode(list(texts)).tolist()}


# ------------------------------------------------------------------ stage 2: search
class _Empty:
    points: list = []


def _filter(ticker, document_type=None):
    must = [models.FieldCondition(key="ticker", match=models.MatchValue(value=ticker.upper()))]
    if document_type:
        must.append(models.FieldCondition(key="document_type",
                                          match=models.MatchValue(value=document_type.upper())))
    return models.Filter(must=must)


def retrieve_from_qdrant(query_vector, ticker, document_type=None, limit=RETRIEVE_LIMIT):
    if _testing():
        return type("obj", (object,), {"points": []})
    # the reference's swallow-to-empty (main.py:232-239) unchanged: query_points answers any
    # limit exactly (large limits on the full exact pass), so an exception here is a real
    # failure, as it is for the reference's Qdrant call
    try:
        return get_qdrant().query_points(collection_name=COLLECTION_NAME, query=query_vector,
                                         limit=limit,
                                         query_filter=_filter(ticker, document_type))
    except Exception:
        return type("obj", (object,), {"points": []})


def retrieve_batch(query_vectors, tickers, document_types=None, limit=RETRIEVE_LIMIT):
    """One GPU scan for a whole micro-batch (main2.py:281-295 + 228), per-request filters."""
    if _testing():
        return [type("obj", (object,), {"points": []}) for _ in tickers]
    document_types = document_types or [None] * len(tickers)
    reqs = [models.QueryRequest(query=v, limit=limit, filter=_filter(t, d))
            for v, t, d in zip(query_vectors, tickers, document_types)]
    return get_qdrant().query_batch_points(COLLECTION_NAME, reqs)


# ------------------------------------------------------------------ stage 3: rerank
def rerank_documents(query, texts, top_k):
    if _testing() or not texts:
        return list(range(min(top_k, len(texts)))), np.zeros(len(texts))
    scores = get_reranker().predict([[query, t] for t in texts])
    idx = np.argsort(scores)[::-1][:top_k]
    return idx, scores


def rerank_batch(queries, texts_lists, top_k):
    """All (query, chunk) pairs of a micro-batch in ONE cross-encoder forward; per request
    the same (idx, scores) as rerank_documents."""
    if _testing():
        return [rerank_documents(q, t, top_k) for q, t in zip(queries, texts_lists)]
    pairs, owner = [], []
    for i, (q, texts) in enumerate(zip(queries, texts_lists)):
        pairs += [[q, t] for t in texts]
        owner += [i] * len(texts)
    # batch_size = all pairs: ONE packed forward (CrossEncoder.predict's default of 32 would
    # split a 32 x 15 micro-batch into 15 forwards)
    scores = (get_reranker().predict(pairs, batch_size=len(pairs)) if pairs
              else np.zeros(0, np.float32))
    out, pos = [], 0
    for i, texts in enumerate(texts_lists):
        s = scores[pos:pos + len(texts)]
        pos += len(texts)
        if len(texts) == 0:
            out.append(([], np.zeros(0)))
        else:
            out.append((np.argsort(s)[::-1][:top_k], s))
    return out


# ------------------------------------------------------------------ ingest
def ensure_collection(qdrant, collection_name=COLLECTION_NAME):
    """ingest.py:86-96 / database.py:111-143."""
    if not qdrant.collection_exists(collection_name):
        qdrant.create_collection(collection_name=collection_name,
                                 vectors_config=models.VectorParams(size=VECTOR_SIZE,
                                                                    distance=models.Distance.COSINE))


def embed_chunks(chunks, batch=EMBED_BATCH):
    """ingest.py:52-66 without the HTTP hop: same batching, local GPU embedder."""
    out = []
    for i in range(0, len(chunks), batch):
        out.extend(embed(chunks[i:i + batch])["embeddings"])
    return out


def chunk_points(ticker, f_type, file, chunks, embeddings, ingested_at=None):
    """ingest.py:148-168: md5 point ids (idempotent re-ingest) + payloads."""
    ts = ingested_at or datetime.now(timezone.utc).isoformat()
    pts = []
    for chunk, vector in zip(chunks, embeddings):
        h = hashlib.md5(f"{ticker}_{f_type}_{file}_{chunk}".encode()).hexdigest()
        pts.append(models.PointStruct(id=h, vector=vector, payload={
            "ticker": ticker.upper(), "document_type": f_type.upper(), "text": chunk,
            "source_file": file, "ingested_at": ts}))
    return pts


def upsert_points(qdrant, points, collection_name=COLLECTION_NAME, batch=UPSERT_BATCH):
    """ingest.py:171-175: memory-safe batched upsert."""
    for i in range(0, len(points), batch):
        qdrant.upsert(collection_name=collection_name, points=points[i:i + batch])
