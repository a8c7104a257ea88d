"""The library's diagnostic surface is the short documented list: the GEMM
variant ids include/ragmi_bert.h exports, and the RAGMI_* A/B knobs the product sources read
(all through ragmi::Knob, honoured only for RAG_CREATE_DIAGNOSTIC handles). The lists below
are the ones DESIGN.md "Diagnostic surface" documents; a new variant or knob must be added
there and here, a measured loser removed from both. CPU only: parses the header and sources,
and calls rag_bert_gemm with removed ids (refused during argument checks, before any HIP call).
"""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "financial-rag-system_amd", "csrc")

# rag_bert_gemm variants: production forms, then the WS kernel's three timing probes
GEMM_VARIANTS = {"RAG_GEMM_AUTO": 0, "RAG_GEMM_TILE": 1, "RAG_GEMM_SMALL": 5, "RAG_GEMM_WS": 19,
                 "RAG_GEMM_WS_MFMA_ONLY": 20, "RAG_GEMM_WS_NO_STORE": 21,
                 "RAG_GEMM_WS_DMA_ONLY": 22}
# RAGMI_* knobs: index (scan grid sizes, fused query prep) and encoder (GEMM pick, split-K,
# deferred / fused LayerNorm, graph replay, CLS-only last layer)
KNOBS = {"RAGMI_SCAN_WGS", "RAGMI_RESCAN_WG", "RAGMI_SAMPLE_DIV", "RAGMI_WIDE_WGS",
         "RAGMI_FUSED_PREP", "RAGMI_GEMM", "RAGMI_KSPLIT", "RAGMI_DEFER_LN", "RAGMI_FUSE_LN",
         "RAGMI_ENC_GRAPH", "RAGMI_CLS_ATTN", "RAGMI_SMALL_RING",
         "RAGMI_ATTN_SHORT"}
# removed in round 5 (measured losers / retired probes): must not come back silently
REMOVED_KNOBS = {"RAGMI_WS_PHASE", "RAGMI_WS_BIG128", "RAGMI_GEMM_PP", "RAGMI_PP_STAGGER",
                 "RAGMI_DL_SMALL", "RAGMI_CE_ROWS", "RAGMI_ATTN_VAR", "RAGMI_SMALL_BK",
                 "RAGMI_SMALL_WIDE", "RAGMI_SMALL_WS", "RAGMI_WIDE_HALF", "RAGMI_ADDLN_VEC",
                 "RAGMI_RESIDUAL_F32"}
REMOVED_IDS = [2, 3, 4, 8, 9, 10, 11, 12, 13, 14, 15] + list(range(23, 50))


@pytest.fixture(scope="module")
def libpath():
    from ragmi import _build
    return _build.build()


def _src(name):
    return open(os.path.join(CSRC, name)).read()


def test_exported_gemm_variants_are_the_documented_list():
    hdr = open(os.path.join(ROOT, "include", "ragmi_bert.h")).read()
    ids = {m.group(1): int(m.group(2))
           for m in re.finditer(r"\b(RAG_GEMM_[A-Z0-9_]+)\s*=\s*(\d+)", hdr)}
    assert ids == GEMM_VARIANTS


def test_knobs_read_by_the_sources_are_the_documented_list():
    found = set()
    for f in os.listdir(CSRC):
        if f.endswith((".hip", ".hpp", ".cpp")):
            found |= set(re.findall(r'Knob\s+\w+\("(RAGMI_[A-Z0-9_]+)"\)', _src(f)))
    assert found == KNOBS
    text = "".join(_src(f) for f in os.listdir(CSRC) if f.endswith((".hip", ".hpp", ".cpp")))
    for k in REMOVED_KNOBS:
        assert f'"{k}"' not in text, k


def test_design_documents_the_surface():
    design = open(os.path.join(ROOT, "DESIGN.md")).read()
    sec = design[design.index("### Diagnostic surface"):]
    sec = sec[:sec.index("\n## ", 1)] if "\n## " in sec[1:] else sec
    for k in KNOBS | set(GEMM_VARIANTS):
        assert k in sec, f"{k} not documented in DESIGN.md 'Diagnostic surface'"


def test_removed_variant_ids_are_refused(libpath):
    L = ctypes.CDLL(libpath)
    L.rag_bert_gemm.restype = ctypes.c_int
    L.rag_bert_gemm.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 5 + \
        [ctypes.c_int] * 3 + [ctypes.c_void_p] * 3
    fake = ctypes.c_void_p(16)          # never dereferenced: refused before any launch
    for v in REMOVED_IDS:
        rc = L.rag_bert_gemm(v, 2, fake, None, fake, None, fake, 64, 128, 128, fake, None, None)
        assert rc != 0, f"variant {v} accepted"


@pytest.mark.parametrize("v", sorted(GEMM_VARIANTS.values()))
def test_python_constants_match(v):
    from ragmi import encoders as E
    names = {n: getattr(E, n) for n in dir(E) if n.startswith("GEMM_")}
    assert v in names.values()


# round 6: the scan's MODE / DYN / VALU probes and the attention VAR
# family are compiled into the diagnostic build only (-DRAGMI_DIAG_BUILD); the production
# library exports these ids and refuses the rest during argument checks
PROD_SCAN_VARIANTS = [0, 7]
PROD_ATTN_VARIANTS = [-1, 42, 10]


def test_production_build_is_not_diagnostic(libpath):
    L = ctypes.CDLL(libpath)
    assert L.rag_diagnostic_build() == 0


def test_scan_and_attention_probes_are_refused(libpath):
    L = ctypes.CDLL(libpath)
    L.rag_last_error.restype = ctypes.c_char_p
    ms = ctypes.c_double()
    fake = ctypes.c_void_p(16)          # never dereferenced: refused before any HIP call
    for v in range(17):
        if v in PROD_SCAN_VARIANTS:
            continue
        rc = L.rag_bench_scan(None, fake, 1, v, 1, ctypes.byref(ms))
        assert rc != 0 and b"diagnostic build" in L.rag_last_error(), v
    for v in list(range(16)) + [18, 26, 40, 43, 44, 46, 106, 107]:
        if v in PROD_ATTN_VARIANTS:
            continue
        rc = L.rag_bert_attention(v, fake, None, fake, 1, 32, fake, None, None)
        assert rc != 0 and b"diagnostic build" in L.rag_last_error(), v


def _inside_diag(src, pos):
    """True when offset pos of src sits inside the diagnostic side of a RAGMI_DIAG_BUILD
    conditional (#ifdef's body or #ifndef's #else), nested conditionals tracked."""
    stack = []
    for line in src[:pos].splitlines():
        t = line.strip()
        if t.startswith("#if"):
            stack.append("diag" if t.startswith("#ifdef RAGMI_DIAG_BUILD") else
                         "prod" if t.startswith("#ifndef RAGMI_DIAG_BUILD") else "other")
        elif t.startswith("#else") and stack:
            stack[-1] = {"diag": "prod", "prod": "diag"}.get(stack[-1], stack[-1])
        elif t.startswith("#endif") and stack:
            stack.pop()
    return "diag" in stack


def test_diagnostic_instances_are_gated_in_the_sources():
    """Every non-production scan / attention instantiation sits under RAGMI_DIAG_BUILD."""
    idx = _src("index_capi.hip")
    for probe in ("scan_valu_kernel<D><<<", "launch_variant<D, 3>", "launch_variant<D, 9>",
                  "RAG_WIDE(4)"):
        assert _inside_diag(idx, idx.index(probe)), probe
    assert not _inside_diag(idx, idx.index("launch_variant<D, 0>(h, w, grid, nullptr);"))
    bert = _src("bert_capi.hip")
    assert _inside_diag(bert, bert.index("integral_constant<int, 106>"))
    # round 6: the fused FFN (measured slower) is diagnostic-build only, kernel and launch
    kern = _src("bert_kernels.hip")
    for src, probe in ((kern, "void ffn_fused_kernel("), (bert, "launch_ffn_fused(w->xh")):
        assert _inside_diag(src, src.index(probe)), probe
