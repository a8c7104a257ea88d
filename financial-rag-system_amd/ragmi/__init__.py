"""ragmi — MI355X-native (gfx950) two-stage retrieval hot path of
pythonmailer/financial-rag-system: in-HBM flat cosine index (Qdrant replacement) and the
bge-small / MiniLM cross-encoder forwards, behind the reference's own call shapes.

Layout:
  ragmi.index      FlatIndex over libragmi.so (HIP scan + top-k + exact merge)
  ragmi.qdrant     QdrantClient-shaped client (create_collection / upsert / query_points)
  ragmi.qdrant_models  Filter, FieldCondition, MatchValue, PointStruct, VectorParams, ...
  ragmi.dist       corpus sharded over GPUs, per-shard top-k + RCCL all-gather merge
"""
__version__ = "0.1.0"
