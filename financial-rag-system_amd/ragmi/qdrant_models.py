"""Qdrant model types used by the reference, restated for the in-HBM index.

The reference imports `from qdrant_client.http import models` (main.py:36) and
`from qdrant_client.http.models import PointStruct, Distance, VectorParams` (ingest.py:11),
and uses: Distance.COSINE, VectorParams(size, distance), PointStruct(id, vector, payload),
Filter(must=[...]), FieldCondition(key, match=MatchValue(value)) (main.py:218-236), and
reads QueryResponse.points[i].id / .score / .payload (main.py:380, main2.py:230).
These dataclasses keep the same constructor keywords and attribute names.
"""
from __future__ import annotations

import enum
from dataclasses import dataclass, field
from typing import Any, Optional, Union

ExtendedPointId = Union[int, str]


class Distance(str, enum.Enum):
    COSINE = "Cosine"
    EUCLID = "Euclid"
    DOT = "Dot"
    MANHATTAN = "Manhattan"


class Datatype(str, enum.Enum):
    FLOAT32 = "float32"
    FLOAT16 = "float16"
    UINT8 = "uint8"


@dataclass
class VectorParams:
    size: int
    distance: Distance = Distance.COSINE
    on_disk: Optional[bool] = None
    # None = Qdrant's default, Float32 (the reference sets none: database.py:124-130,
    # ingest.py:89-95) -> fp32 storage; FLOAT16 -> fp16 storage (ragmi FlatIndex storage)
    datatype: Optional[str] = None


@dataclass
class PointStruct:
    id: ExtendedPointId
    vector: Any
    payload: Optional[dict] = None


@dataclass
class Batch:
    ids: list
    vectors: Any
    payloads: Optional[list] = None


@dataclass
class MatchValue:
    value: Any


@dataclass
class MatchAny:
    any: list


@dataclass
class FieldCondition:
    key: str
    match: Any = None
    range: Any = None


@dataclass
class Filter:
    must: Optional[list] = None
    should: Optional[list] = None
    must_not: Optional[list] = None
    min_should: Any = None


@dataclass
class ScoredPoint:
    id: ExtendedPointId
    version: int
    score: float
    payload: Optional[dict] = None
    vector: Any = None
    shard_key: Any = None
    order_value: Any = None


@dataclass
class Record:
    id: ExtendedPointId
    payload: Optional[dict] = None
    vector: Any = None
    shard_key: Any = None
    order_value: Any = None


@dataclass
class QueryResponse:
    points: list = field(default_factory=list)


@dataclass
class CollectionDescription:
    name: str


@dataclass
class CollectionsResponse:
    collections: list = field(default_factory=list)


class UpdateStatus(str, enum.Enum):
    ACKNOWLEDGED = "acknowledged"
    COMPLETED = "completed"


@dataclass
class UpdateResult:
    operation_id: Optional[int]
    status: UpdateStatus


@dataclass
class CountResult:
    count: int


@dataclass
class QueryRequest:
    """Batched query entry for query_batch_points (one per request of a micro-batch)."""
    query: Any
    filter: Optional[Filter] = None
    limit: int = 10
    with_payload: Any = True
