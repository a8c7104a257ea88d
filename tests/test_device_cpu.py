"""Device selection: the reference's loaders pass
device = "cuda" if USE_GPU else "cpu" (/root/reference/main.py:23,83,89). This build has no CPU
path, so "cpu" must be refused with an error naming the HIP-only build — before any HIP call,
never by silently running on the GPU — and "cuda:N" must mean device N. All of it runs on the
CPU container: the refusal happens before the GPU is touched."""
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)),
                                "financial-rag-system_amd"))

from ragmi import _lib  # noqa: E402


@pytest.mark.parametrize("dev", ["cpu", torch.device("cpu"), "meta"])
def test_resolve_device_refuses_non_hip(dev):
    with pytest.raises(_lib.RagmiDeviceError, match="HIP-only"):
        _lib.resolve_device(dev)


def test_resolve_device_keeps_the_index():
    assert _lib.resolve_device(None) is None
    assert _lib.resolve_device("cuda") == torch.device("cuda")
    assert _lib.resolve_device("cuda:3") == torch.device("cuda", 3)
    assert _lib.resolve_device(2) == torch.device("cuda", 2)
    assert _lib.resolve_device(torch.device("cuda", 1)).index == 1
    with pytest.raises(_lib.RagmiDeviceError):
        _lib.resolve_device("not-a-device")


def test_encoders_and_index_refuse_cpu():
    from ragmi.encoders import BertEncoder, CrossEncoder, SentenceTransformer
    from ragmi.index import FlatIndex
    # (the refusal precedes the checkpoint load and the GPU check: no files, no GPU needed)
    with pytest.raises(_lib.RagmiDeviceError, match="USE_GPU=false"):
        SentenceTransformer("/nonexistent/bge-small-en-v1.5", device="cpu")
    with pytest.raises(_lib.RagmiDeviceError, match="USE_GPU=false"):
        CrossEncoder("/nonexistent/ms-marco-MiniLM-L-6-v2", device="cpu")
    with pytest.raises(_lib.RagmiDeviceError):
        BertEncoder({}, {}, 0, device="cpu")
    with pytest.raises(_lib.RagmiDeviceError):
        FlatIndex(384, 16, device="cpu")


def test_rag_loaders_follow_use_gpu(monkeypatch):
    """ragmi.rag.get_embedder / get_reranker restate main.py:80-90: USE_GPU unset or false ->
    device "cpu" -> RagmiDeviceError; the reference's TESTING stubs still return None."""
    import importlib

    import ragmi.rag as rag
    monkeypatch.setenv("TESTING", "False")
    monkeypatch.setenv("RAGMI_BGE_DIR", "/nonexistent/bge")
    monkeypatch.setenv("RAGMI_CE_DIR", "/nonexistent/ce")
    monkeypatch.delenv("USE_GPU", raising=False)
    rag = importlib.reload(rag)
    for f in (rag.get_embedder, rag.get_reranker):
        f.cache_clear()
        with pytest.raises(_lib.RagmiDeviceError):
            f()
    monkeypatch.setenv("USE_GPU", "false")
    rag.get_embedder.cache_clear()
    with pytest.raises(_lib.RagmiDeviceError):
        rag.get_embedder()
    assert rag._device() == "cpu"
    monkeypatch.setenv("USE_GPU", "TRUE")
    assert rag._device() == "cuda"
    monkeypatch.setenv("TESTING", "True")
    rag = importlib.reload(rag)
    rag.get_embedder.cache_clear()
    assert rag.get_embedder() is None
    importlib.reload(rag)


@pytest.mark.gpu
def test_cuda_n_picks_device_n(gpu):
    """'cuda:N' -> device N; an index past the visible devices is refused, not remapped."""
    from ragmi.index import FlatIndex
    n = torch.cuda.device_count()
    idx = FlatIndex(384, 16, device=f"cuda:{n - 1}")
    assert idx.device == torch.device("cuda", n - 1)
    idx.close()
    assert FlatIndex(384, 16, device="cuda").device.index == torch.cuda.current_device()
    with pytest.raises(_lib.RagmiDeviceError, match="visible"):
        FlatIndex(384, 16, device=f"cuda:{n}")
