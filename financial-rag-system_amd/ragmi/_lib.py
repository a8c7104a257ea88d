"""ctypes binding of libragmi.so (the C ABI declared in include/ragmi.h).

torch is imported first on purpose: libragmi.so links libamdhip64.so.7, and loading torch
first makes the dynamic loader reuse torch's HIP runtime (same SONAME) so tensors, streams
and our kernels share one runtime in the process.

There is no fallback: if libragmi.so is missing or fails to load, every product entry point
raises RagmiUnavailable.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

from ._build import LIB_PATH as _BUILT_LIB

# RAGMI_LIB_AB: diagnostic A/B timing of two builds of the same tree (scripts/gpu_ab.sh); the
# default is the in-tree build
LIB_PATH = os.environ.get("RAGMI_LIB_AB") or _BUILT_LIB

_lock = threading.Lock()
_lib = None


class RagmiUnavailable(RuntimeError):
    """libragmi.so is not built or cannot be loaded (no CPU fallback exists)."""


class RagmiDeviceError(ValueError):
    """A device the HIP-only build cannot run on — notably the reference's USE_GPU=false
    "cpu" (main.py:83,89) — or a HIP device index that does not exist."""


def resolve_device(device) -> torch.device | None:
    """The HIP device behind a reference-style `device` argument (main.py:83,89:
    ``device = "cuda" if USE_GPU else "cpu"``; sentence-transformers takes a str, an int or a
    torch.device). None -> None (the caller takes the current HIP device); "cuda" / "cuda:N" /
    N / torch.device("cuda", N) -> that device. Any other type — "cpu" above all — raises
    RagmiDeviceError instead of silently running on the GPU: this build has no CPU path.
    Checked before any HIP call, so the refusal is the same with or without a GPU."""
    if device is None:
        return None
    try:
        d = device if isinstance(device, torch.device) else torch.device(device)
    except (RuntimeError, TypeError) as e:
        raise RagmiDeviceError(f"device {device!r}: {e}") from e
    if d.type != "cuda":
        raise RagmiDeviceError(
            f"device {str(d)!r}: ragmi is a HIP-only build (MI355X, gfx950) with no CPU path; "
            "the reference's USE_GPU=false / device='cpu' cannot be honoured — pass "
            "device='cuda' or 'cuda:N' (or None for the current HIP device)")
    return d


def device_index(d: torch.device | None) -> int:
    """Index of a resolved HIP device (resolve_device), the current one for None / 'cuda'."""
    if d is None or d.index is None:
        return torch.cuda.current_device()
    n = torch.cuda.device_count()
    if not 0 <= d.index < n:
        raise RagmiDeviceError(f"device {str(d)!r}: {n} HIP device(s) visible")
    return d.index


class RagmiError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"libragmi error {code}: {msg}")
        self.code = code


c_f32p = ctypes.POINTER(ctypes.c_float)
c_i64p = ctypes.POINTER(ctypes.c_int64)
c_u32p = ctypes.POINTER(ctypes.c_uint32)
c_u16p = ctypes.POINTER(ctypes.c_uint16)
c_i32p = ctypes.POINTER(ctypes.c_int32)
c_vp = ctypes.c_void_p

# name -> (restype, argtypes); the single source of truth for the exported C ABI.
INDEX_API = {
    "rag_last_error": (ctypes.c_char_p, []),
    "rag_version": (ctypes.c_char_p, []),
    "rag_index_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_int64, ctypes.c_int,
                                        ctypes.POINTER(c_vp)]),
    "rag_index_create_ex": (ctypes.c_int, [ctypes.c_int, ctypes.c_int64, ctypes.c_int,
                                           ctypes.c_int, ctypes.POINTER(c_vp)]),
    "rag_index_storage": (ctypes.c_int, [c_vp]),
    "rag_index_export_rows32": (ctypes.c_int, [c_vp, ctypes.c_int64, ctypes.c_int64, c_f32p]),
    "rag_index_import_rows32": (ctypes.c_int, [c_vp, ctypes.c_int64, ctypes.c_int64, c_f32p,
                                               c_u32p, ctypes.c_int64]),
    "rag_index_destroy": (ctypes.c_int, [c_vp]),
    "rag_index_reserve": (ctypes.c_int, [c_vp, ctypes.c_int64]),
    "rag_index_capacity": (ctypes.c_int64, [c_vp]),
    "rag_index_count": (ctypes.c_int64, [c_vp]),
    "rag_index_dim": (ctypes.c_int, [c_vp]),
    "rag_index_upsert": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, ctypes.c_int64, ctypes.c_int64,
                                        c_vp]),
    "rag_index_upsert_host": (ctypes.c_int, [c_vp, c_f32p, c_i64p, c_u32p, ctypes.c_int64,
                                             ctypes.c_int64]),
    "rag_index_search": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int, ctypes.c_int, c_vp,
                                        ctypes.c_int64, c_vp, c_vp, c_vp]),
    "rag_index_search_full": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int, ctypes.c_int, c_vp,
                                             ctypes.c_int64, c_vp, c_vp, c_vp]),
    "rag_index_search_packed": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int, ctypes.c_int, c_vp,
                                               ctypes.c_int64, c_vp, c_vp]),
    "rag_index_search_host": (ctypes.c_int, [c_vp, c_f32p, ctypes.c_int, ctypes.c_int, c_u32p,
                                             ctypes.c_int64, c_f32p, c_i64p]),
    "rag_index_export_rows": (ctypes.c_int, [c_vp, ctypes.c_int64, ctypes.c_int64, c_u16p]),
    "rag_index_export_tags": (ctypes.c_int, [c_vp, ctypes.c_int64, ctypes.c_int64, c_u32p]),
    "rag_index_import_rows": (ctypes.c_int, [c_vp, ctypes.c_int64, ctypes.c_int64, c_u16p,
                                             c_u32p, ctypes.c_int64]),
    "rag_merge_topk": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      c_vp, c_vp, c_vp]),
    "rag_merge_topk_packed": (ctypes.c_int, [c_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                             c_vp, c_vp, c_vp]),
    "rag_bench_scan": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.POINTER(ctypes.c_double)]),
    "rag_index_set_scan_order": (ctypes.c_int, [c_vp, ctypes.c_int]),
    "rag_stream_create_cu_partition": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                      ctypes.POINTER(c_vp)]),
    "rag_stream_create_cu_mask": (ctypes.c_int, [ctypes.c_int, c_u32p, ctypes.c_int,
                                                 ctypes.POINTER(c_vp)]),
    "rag_diag_cu_probe": (ctypes.c_int, [c_vp, ctypes.c_int, c_vp]),
    "rag_stream_destroy": (ctypes.c_int, [c_vp]),
    "rag_index_exactness_stats": (ctypes.c_int, [c_vp, c_i64p, c_i64p, c_i32p, ctypes.c_int]),
    "rag_index_unanswered": (ctypes.c_int, [c_vp, c_i64p]),
    "rag_knob_probe": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int]),
    "rag_diagnostic_build": (ctypes.c_int, []),
    "rag_profile_enable": (ctypes.c_int, [c_vp, ctypes.c_int]),
    "rag_profile_scan_ms": (ctypes.c_int, [c_vp, ctypes.POINTER(ctypes.c_double), c_i64p]),
    "rag_profile_scan_intervals": (ctypes.c_int, [c_vp, ctypes.POINTER(ctypes.c_double),
                                                  ctypes.POINTER(ctypes.c_double),
                                                  ctypes.c_int64, c_i64p]),
}

class RagBertConfig(ctypes.Structure):
    """rag_bert_config (include/ragmi_bert.h)."""
    _fields_ = [("vocab", ctypes.c_int), ("hidden", ctypes.c_int), ("layers", ctypes.c_int),
                ("heads", ctypes.c_int), ("intermediate", ctypes.c_int),
                ("max_position", ctypes.c_int), ("type_vocab", ctypes.c_int),
                ("layer_norm_eps", ctypes.c_float), ("head", ctypes.c_int),
                ("precision", ctypes.c_int)]


c_i32p_ = ctypes.POINTER(ctypes.c_int32)
BERT_API = {
    "rag_encoder_num_weights": (ctypes.c_int, [ctypes.POINTER(RagBertConfig)]),
    "rag_encoder_create": (ctypes.c_int, [ctypes.POINTER(RagBertConfig),
                                          ctypes.POINTER(ctypes.POINTER(ctypes.c_float)),
                                          ctypes.c_int, ctypes.c_int, ctypes.POINTER(c_vp)]),
    "rag_encoder_create_ex": (ctypes.c_int, [ctypes.POINTER(RagBertConfig),
                                             ctypes.POINTER(ctypes.POINTER(ctypes.c_float)),
                                             ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                             ctypes.POINTER(c_vp)]),
    "rag_encoder_destroy": (ctypes.c_int, [c_vp]),
    "rag_encoder_forward": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_int, c_vp, c_vp]),
    "rag_encoder_forward_host": (ctypes.c_int, [c_vp, c_i32p_, c_i32p_, c_i32p_, ctypes.c_int,
                                                ctypes.c_int, c_f32p]),
    "rag_wordpiece_create": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int64, ctypes.c_int,
                                            ctypes.c_int, ctypes.POINTER(c_vp)]),
    "rag_wordpiece_destroy": (ctypes.c_int, [c_vp]),
    "rag_wordpiece_encode": (ctypes.c_int, [c_vp, ctypes.c_char_p, c_i64p, ctypes.c_char_p,
                                            c_i64p, ctypes.c_int, c_i32p_, c_i32p_, c_i32p_,
                                            ctypes.c_int64, ctypes.POINTER(ctypes.c_uint8)]),
    "rag_build_pairs": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int, c_vp, ctypes.c_int, c_vp,
                                       ctypes.c_int, c_vp, ctypes.c_int, c_vp, c_vp, c_vp, c_vp,
                                       c_vp]),
    "rag_bert_gemm": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_vp, c_vp, c_vp, c_vp, c_vp,
                                     ctypes.c_int, ctypes.c_int, ctypes.c_int, c_vp, c_vp, c_vp]),
    "rag_bert_gemm_splitk": (ctypes.c_int, [ctypes.c_int, c_vp, c_vp, c_vp, c_vp, c_vp,
                                            ctypes.c_int, ctypes.c_int, ctypes.c_int, c_vp,
                                            ctypes.c_int, ctypes.POINTER(ctypes.c_int), c_vp]),
    "rag_bert_gemm_add_ln": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                            ctypes.c_float, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_int, c_vp, c_vp, c_vp, c_vp]),
    "rag_encoder_set_fusion": (ctypes.c_int, [c_vp, ctypes.c_int]),
    "rag_encoder_set_graphs": (ctypes.c_int, [c_vp, ctypes.c_int]),
    "rag_encoder_set_defer_ln": (ctypes.c_int, [c_vp, ctypes.c_int]),
    "rag_encoder_set_ffn_fused": (ctypes.c_int, [c_vp, ctypes.c_int]),
    "rag_encoder_range_bounds": (ctypes.c_int, [c_vp, ctypes.POINTER(ctypes.c_double),
                                                ctypes.POINTER(ctypes.c_double)]),
    "rag_encoder_weight_bounds": (ctypes.c_int, [ctypes.POINTER(RagBertConfig),
                                                 ctypes.POINTER(ctypes.POINTER(ctypes.c_float)),
                                                 ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                                 ctypes.POINTER(ctypes.c_double)]),
    "rag_bert_gemm_dl": (ctypes.c_int, [ctypes.c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                        c_vp, c_vp, ctypes.c_float, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_int, c_vp, c_vp, c_vp, c_vp]),
    "rag_bert_attention": (ctypes.c_int, [ctypes.c_int, c_vp, c_vp, c_vp, ctypes.c_int,
                                          ctypes.c_int, c_vp, c_vp, c_vp]),
}


def load():
    """Load libragmi.so (raises RagmiUnavailable; never falls back)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise RagmiUnavailable(
                f"{LIB_PATH} is not built; run `python -c 'import __graft_entry__ as g; "
                f"g.build()'` (hipcc --offload-arch=gfx950)")
        try:
            L = ctypes.CDLL(LIB_PATH)
        except OSError as e:
            raise RagmiUnavailable(f"cannot load {LIB_PATH}: {e}") from e
        for name, (res, args) in {**INDEX_API, **BERT_API}.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
        return L


def check(rc: int) -> None:
    if rc != 0:
        msg = load().rag_last_error()
        raise RagmiError(rc, msg.decode() if msg else "")


def require_gpu() -> None:
    if not torch.cuda.is_available():
        raise RagmiUnavailable("no HIP device visible: the ragmi hot path runs only on MI355X "
                               "(gfx950); there is no CPU fallback")
