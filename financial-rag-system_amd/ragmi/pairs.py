"""GPU-side assembly of cross-encoder batches from cached token ids (SURVEY §8f rows 1-2:
the batched rerank stage without a host round trip).

At ingest every chunk is tokenised once; its WordPiece ids can stay in HBM next to its vector
(a row-indexed [rows, Lmax] table + lengths). After the search returns the top-k rows of each
query, the packed cross-encoder input for all (query, chunk) pairs is built on the device:

    [CLS] q [SEP] c [SEP]      token types 0 ... 0 1 ... 1     (BertTokenizer pair encoding)

with the chunk truncated so a pair fits max_len (`longest_first` truncation removes tokens from
the longer side — the chunk, for the reference's short queries; main.py:241-247 via
CrossEncoder.predict). Output: packed ids / types (int32 [T]), cu_seqlens (int32 [P+1]) and the
longest pair, ready for BertEncoder.forward_device.

build_pairs_gpu: the production form — two HIP kernels (rag_build_pairs: lengths + scan,
then one workgroup per pair) and one 8-byte read-back of {T, longest} (the forward's launch
grids need T on the host). build_pairs_gpu_async moves that read-back off the critical path:
the 8 bytes go to pinned memory behind an event and the caller collects them after it has
enqueued the next batch. build_pairs: the same assembly in pure torch ops
(works on CPU tensors too, which is how tests/test_pairs_cpu.py checks it against a per-pair
loop; the GPU test checks build_pairs_gpu against it bit for bit).
"""
from __future__ import annotations

import torch

CLS, SEP = 101, 102


def build_pairs(q_ids, q_cu, rows, c_toks, c_lens, max_len: int = 512):
    """q_ids int32 [Tq] / q_cu [B+1]: the packed query tokens (each [CLS] ... [SEP]);
    rows int64 [B, K]: search result rows (-1 = none: treated as row 0, caller masks);
    c_toks [rows, Lmax] (int16/int32 ids, < 32768 for int16), c_lens [rows].
    Returns (ids int32 [T], types int32 [T], cu int32 [B*K+1], longest pair)."""
    dev = rows.device
    Bq, Kq = rows.shape
    # query tokens without their own [CLS]/[SEP]: the pair adds them back
    q_len = (q_cu[1:] - q_cu[:-1]).long() - 2                      # [B]
    ql = q_len.repeat_interleave(Kq)                                # [P]
    r = rows.reshape(-1).clamp_min(0)
    cl = torch.minimum(c_lens[r].long(), max_len - 3 - ql)
    plen = ql + cl + 3
    cu = torch.zeros(plen.numel() + 1, dtype=torch.int64, device=dev)
    cu[1:] = torch.cumsum(plen, 0)
    T = int(cu[-1])                                                 # one host sync per batch
    t = torch.arange(T, device=dev)
    p = torch.searchsorted(cu[1:], t, right=True)
    off = t - cu[p]
    qlp, clp = ql[p], cl[p]
    qstart = q_cu[:-1].long().repeat_interleave(Kq)[p] + 1       # skip the query's [CLS]
    qi = q_ids[(qstart + (off - 1).clamp(0, None)).clamp(max=q_ids.numel() - 1)]
    ci = c_toks[r[p], (off - qlp - 2).clamp(0, c_toks.shape[1] - 1)].to(torch.int32) & 0xFFFF
    ids = torch.where(off == 0, CLS,
                      torch.where(off <= qlp, qi,
                                  torch.where(off == qlp + 1, SEP,
                                              torch.where(off < qlp + clp + 2, ci, SEP))))
    types = (off > qlp + 1).to(torch.int32)
    return ids.to(torch.int32).contiguous(), types.contiguous(), cu.to(torch.int32), \
        int(plen.max())


class PendingPairs:
    """build_pairs_gpu_async's result: the packed pair tensors are enqueued on the stream; the
    8-byte {T, longest} travels to pinned host memory behind an event. result() waits for
    that event only — by the time a pipelined caller asks (after enqueueing the next batch's
    encode + search), the assembly has long finished and the wait costs nothing."""

    def __init__(self, ids, types, cu, stats_host, event):
        self._ids, self._types, self.cu = ids, types, cu
        self._stats, self._event = stats_host, event

    def ready(self) -> bool:
        return self._event.query()

    def result(self):
        self._event.synchronize()
        T, longest = (int(v) for v in self._stats)
        return self._ids[:T], self._types[:T], self.cu, longest


def _launch_pairs(q_ids, q_cu, rows, c_toks, c_lens, max_len):
    from . import _lib
    dev = rows.device
    Bq, Kq = rows.shape
    for t, dt in ((q_ids, torch.int32), (q_cu, torch.int32), (c_toks, torch.int16),
                  (c_lens, torch.int32), (rows, torch.int64)):
        if t.dtype != dt or not t.is_cuda or not t.is_contiguous():
            raise ValueError("q_ids/q_cu int32, rows int64, c_toks int16, c_lens int32: "
                             "contiguous cuda tensors")
    P = Bq * Kq
    ids = torch.empty(P * max_len, dtype=torch.int32, device=dev)
    types = torch.empty_like(ids)
    cu = torch.empty(P + 1, dtype=torch.int32, device=dev)
    stats = torch.empty(2, dtype=torch.int32, device=dev)
    _lib.check(_lib.load().rag_build_pairs(
        q_ids.data_ptr(), q_cu.data_ptr(), Bq, rows.data_ptr(), Kq, c_toks.data_ptr(),
        c_toks.shape[1], c_lens.data_ptr(), max_len, ids.data_ptr(), types.data_ptr(),
        cu.data_ptr(), stats.data_ptr(), torch.cuda.current_stream(dev).cuda_stream))
    return ids, types, cu, stats


def build_pairs_gpu(q_ids, q_cu, rows, c_toks, c_lens, max_len: int = 512):
    """Same contract as build_pairs for cuda tensors (c_toks int16, c_lens int32), through the
    rag_build_pairs kernels. Reads {T, longest} back at once (one host sync per call); a
    pipelined caller uses build_pairs_gpu_async instead."""
    ids, types, cu, stats = _launch_pairs(q_ids, q_cu, rows, c_toks, c_lens, max_len)
    T, longest = (int(v) for v in stats.cpu())
    return ids[:T], types[:T], cu, longest


def build_pairs_gpu_async(q_ids, q_cu, rows, c_toks, c_lens, max_len: int = 512):
    """build_pairs_gpu without the blocking read: returns a PendingPairs whose result() is the
    same tuple. The host can enqueue batch i+1's encode and search before it asks for batch
    i's pair count, so the GPU queue never drains behind the read-back."""
    ids, types, cu, stats = _launch_pairs(q_ids, q_cu, rows, c_toks, c_lens, max_len)
    host = torch.empty(2, dtype=torch.int32, pin_memory=True)
    host.copy_(stats, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(rows.device))
    return PendingPairs(ids, types, cu, host, ev)
