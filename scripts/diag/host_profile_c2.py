"""Host-side cost of one config-2 batch (encode 32 pre-tokenised queries + top-15 over 1M
rows), 4 batches in flight: cProfile of the issuing thread over 200 batches, top entries by
own time (the ctypes entry points' own time is the C ABI's host work: graph replay, kernel
launches). Usage (GPU box): python scripts/diag/host_profile_c2.py > gpurun_out/host_c2.txt"""
import cProfile
import io
import os
import pstats
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "financial-rag-system_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import bench_modes as BM  # noqa: E402
from ragmi import synth as R  # noqa: E402
from ragmi.encoders import HEAD_CLS_L2, BertEncoder, WordPiece  # noqa: E402
from ragmi.index import FlatIndex  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n = 1_000_000
    idx = FlatIndex(384, n, dev)
    BM.build_shard(idx, 0, n, n, 384, 1000, dev)
    import tempfile
    vocab = R.make_vocab(30522, seed=5)
    vdir = tempfile.mkdtemp(prefix="ragmi_vocab_")
    with open(os.path.join(vdir, "vocab.txt"), "w") as f:
        f.write("\n".join(vocab) + "\n")
    tok = WordPiece(os.path.join(vdir, "vocab.txt"), 512)
    rng = np.random.default_rng(3)
    nb = 220
    texts = [R.query_texts(rng, vocab, 32) for _ in range(nb)]
    batches = [tok.encode_packed(t) for t in texts]
    bge = BertEncoder(R.BGE_SMALL, R.make_weights(R.BGE_SMALL, 1), HEAD_CLS_L2, dev, "fp16x3")
    streams = [torch.cuda.Stream(dev) for _ in range(4)]

    def one(i, text=False):
        ids, tt, cu = tok.encode_packed(texts[i]) if text else batches[i]
        with torch.cuda.stream(streams[i % 4]):
            q = bge.forward_packed(ids, tt, cu)
            idx.search(q, 15)

    for i in range(20):
        one(i)
    torch.cuda.synchronize()
    for mode in (False, True):
        pr = cProfile.Profile()
        t0 = time.perf_counter()
        pr.enable()
        for i in range(20, nb):
            one(i, mode)
        pr.disable()
        t_enq = time.perf_counter() - t0
        torch.cuda.synchronize()
        t_all = time.perf_counter() - t0
        print(f"== {'text (inline tokenise)' if mode else 'ids'}: {nb - 20} batches, host enqueue "
              f"{t_enq / (nb - 20) * 1e3:.4f} ms/batch, wall {t_all / (nb - 20) * 1e3:.4f} ms/batch")
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(18)
        print(s.getvalue())
    idx.close()


if __name__ == "__main__":
    main()
