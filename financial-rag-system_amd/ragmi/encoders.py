"""Encoders on MI355X: bge-small-en-v1.5 embedder and ms-marco-MiniLM-L-6-v2 cross-encoder.

Drop-ins for the two sentence-transformers objects the reference builds in its lazy loaders:
  get_embedder() -> SentenceTransformer("BAAI/bge-small-en-v1.5")       main.py:80-84, main2.py:88-96
      .encode(str) -> float32 [384]; .encode(list[str]) -> float32 [n, 384]
      (main.py:144-149 /embed, 211-213 embed_query; main2.py:170-171 embed_query_batch)
  get_reranker() -> CrossEncoder("cross-encoder/ms-marco-MiniLM-L-6-v2")  main.py:86-90
      .predict([[query, text], ...]) -> float32 [n]   (main.py:241-247 rerank_documents)
The transformer forward runs in libragmi.so (csrc/bert_kernels.hip); tokenisation is host-side
WordPiece (`tokenizers`) from the checkpoint's own vocab.txt. Models load from LOCAL
directories in the HF layout (config.json + model.safetensors + vocab.txt): there is no hub
access, and no CPU forward to fall back to.
"""
from __future__ import annotations

import ctypes
import itertools
import json
import os

import numpy as np
import torch

from . import _lib
from ._lib import check

HEAD_CLS_L2 = 0        # sentence-transformers: Pooling(cls) + Normalize  (bge)
HEAD_POOLER_CLS = 1    # BertForSequenceClassification, num_labels = 1   (cross-encoder)
PREC_FP16 = 0          # fp16 GEMM / attention operands, fp32 accumulation
PREC_FP16X3 = 1        # split fp16 products (a_hi b_hi + a_hi b_lo + a_lo b_hi): ~fp32 accuracy
PRECISIONS = {"fp16": PREC_FP16, "fp16x3": PREC_FP16X3}


# ------------------------------------------------------------------ weights
def weight_order(layers: int, head: int) -> list[str]:
    """HF state-dict names in the order rag_encoder_create expects (include/ragmi_bert.h)."""
    names = ["embeddings.word_embeddings.weight", "embeddings.position_embeddings.weight",
             "embeddings.token_type_embeddings.weight", "embeddings.LayerNorm.weight",
             "embeddings.LayerNorm.bias"]
    for l in range(layers):
        p = f"encoder.layer.{l}."
        for n in ("attention.self.query", "attention.self.key", "attention.self.value",
                  "attention.output.dense"):
            names += [p + n + ".weight", p + n + ".bias"]
        names += [p + "attention.output.LayerNorm.weight", p + "attention.output.LayerNorm.bias",
                  p + "intermediate.dense.weight", p + "intermediate.dense.bias",
                  p + "output.dense.weight", p + "output.dense.bias",
                  p + "output.LayerNorm.weight", p + "output.LayerNorm.bias"]
    if head == HEAD_POOLER_CLS:
        names += ["pooler.dense.weight", "pooler.dense.bias", "classifier.weight",
                  "classifier.bias"]
    return names


def _lookup(w: dict, name: str):
    for k in (name, "bert." + name, "model." + name):
        if k in w:
            return w[k]
    raise KeyError(f"weight {name!r} not found")


def load_safetensors(path: str) -> dict:
    """Tensors of a local .safetensors file as fp32 numpy (safe loader: executes nothing)."""
    from safetensors.numpy import load_file
    return {k: np.asarray(v, dtype=np.float32) for k, v in load_file(path).items()}


def config_from_hf(cfg: dict) -> dict:
    """HF BertConfig dict -> encoder shape. Refuses what the kernels do not implement (they
    hard-code erf-GELU, absolute positions and post-LN BERT, modeling_bert.py:96-107,325-351)
    instead of running a different function silently."""
    act = cfg.get("hidden_act", "gelu")
    if act != "gelu":
        raise NotImplementedError(f"hidden_act {act!r}: only erf-GELU ('gelu') is implemented")
    pos = cfg.get("position_embedding_type", "absolute")
    if pos != "absolute":
        raise NotImplementedError(f"position_embedding_type {pos!r}: only 'absolute'")
    mt = cfg.get("model_type", "bert")
    if mt != "bert":
        raise NotImplementedError(f"model_type {mt!r}: only 'bert'")
    out = dict(vocab=cfg["vocab_size"], hidden=cfg["hidden_size"],
               layers=cfg["num_hidden_layers"], heads=cfg["num_attention_heads"],
               inter=cfg["intermediate_size"], max_pos=cfg["max_position_embeddings"],
               type_vocab=cfg.get("type_vocab_size", 2), eps=cfg.get("layer_norm_eps", 1e-12))
    out["num_labels"] = hf_num_labels(cfg)
    return out


def hf_num_labels(cfg: dict) -> int:
    """PretrainedConfig.num_labels: len(id2label) when present, else num_labels, else 2 (the
    transformers default)."""
    if cfg.get("id2label"):
        return len(cfg["id2label"])
    return int(cfg.get("num_labels", 2))


# sentence-transformers' activation names (CrossEncoder: config.json
# "sentence_transformers": {"activation_fn": ...} (v4+) or "sbert_ce_default_activation_function"
# (v2/v3)) -> the activations this head implements
_ACTIVATIONS = {
    "torch.nn.modules.linear.Identity": "identity", "torch.nn.Identity": "identity",
    "torch.nn.modules.activation.Sigmoid": "sigmoid", "torch.nn.Sigmoid": "sigmoid",
}


def ce_activation(hf_cfg: dict | None, override=None) -> str:
    """The activation sentence-transformers' CrossEncoder applies to the logits in predict()
    (reference main.py:245 returns these scores to users as sources[].score):
      1. an explicit override (CrossEncoder(..., activation_fn=...));
      2. config.json "sentence_transformers"."activation_fn" (sentence-transformers >= 4);
      3. config.json "sbert_ce_default_activation_function" (2.x / 3.x; the
         ms-marco-MiniLM-L-6-v2 checkpoint sets torch.nn.modules.linear.Identity);
      4. otherwise Sigmoid when num_labels == 1 (Identity for more labels, which this head
         does not implement).
    Returns "identity" or "sigmoid"; anything else raises NotImplementedError."""
    hf_cfg = hf_cfg or {}
    name = override
    if name is None:
        name = (hf_cfg.get("sentence_transformers") or {}).get("activation_fn")
    if name is None:
        name = hf_cfg.get("sbert_ce_default_activation_function")
    if name is None:
        return "sigmoid" if hf_num_labels(hf_cfg) == 1 else "identity"
    if isinstance(name, torch.nn.Module):
        name = type(name).__module__ + "." + type(name).__name__
    if name in ("identity", "sigmoid"):
        return name
    if name not in _ACTIVATIONS:
        raise NotImplementedError(f"cross-encoder activation {name!r}: only Identity and "
                                  "Sigmoid are implemented")
    return _ACTIVATIONS[name]


_POOL_MODES = ("pooling_mode_cls_token", "pooling_mode_mean_tokens", "pooling_mode_max_tokens",
               "pooling_mode_mean_sqrt_len_tokens", "pooling_mode_weightedmean_tokens",
               "pooling_mode_lasttoken")


def st_head_from_dir(model_dir: str) -> int:
    """The sentence-transformers module stack of a local checkpoint (modules.json +
    <pooling>/config.json) -> the encoder head. Implemented: Transformer -> Pooling(cls) ->
    Normalize (bge-small-en-v1.5's stack: HEAD_CLS_L2). Everything else raises — including a
    directory without modules.json, for which sentence-transformers would build MEAN pooling
    (a different embedding), so it must not silently get the CLS head."""
    mj = os.path.join(model_dir, "modules.json")
    if not os.path.exists(mj):
        raise NotImplementedError(
            f"{model_dir}: no modules.json (sentence-transformers would use mean pooling; "
            "only Transformer -> Pooling(cls) -> Normalize is implemented)")
    with open(mj) as f:
        mods = json.load(f)
    types = [m.get("type", "").rsplit(".", 1)[-1] for m in mods]
    if types != ["Transformer", "Pooling", "Normalize"]:
        raise NotImplementedError(f"{model_dir}: module stack {types}; only "
                                  "[Transformer, Pooling, Normalize] is implemented")
    with open(os.path.join(model_dir, mods[1].get("path", ""), "config.json")) as f:
        pc = json.load(f)
    on = [m for m in _POOL_MODES if pc.get(m)]
    if on != ["pooling_mode_cls_token"]:
        raise NotImplementedError(f"{model_dir}: pooling {on or 'none'}; only CLS pooling is "
                                  "implemented")
    return HEAD_CLS_L2


# ------------------------------------------------------------------ one encoder GEMM
# rag_bert_gemm variants (ragmi_bert.h): production forms, then the WS timing probes
GEMM_AUTO, GEMM_TILE, GEMM_SMALL, GEMM_WS = 0, 1, 5, 19
GEMM_WS_MFMA_ONLY, GEMM_WS_NO_STORE, GEMM_WS_DMA_ONLY = 20, 21, 22
EPI_F16, EPI_GELU_F16, EPI_F32 = 0, 1, 2            # epilogues


def linear(a: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, epilogue: int = EPI_F32,
           a_lo: torch.Tensor | None = None, w_lo: torch.Tensor | None = None,
           variant: int = GEMM_AUTO):
    """nn.Linear of the encoder layers (modeling_bert.py BertSelfAttention / BertIntermediate /
    BertOutput dense) through the forward's own GEMM kernels: a fp16 [M,K], w fp16 [N,K],
    bias fp32 [N] -> fp32 [M,N] (EPI_F32) or fp16 [M,N] (+ lo plane when a_lo/w_lo are
    given, the fp16x3 mode). Diagnostic entry for parity tests and the GEMM benchmark."""
    M, K = a.shape
    N = w.shape[0]
    for t, dt in ((a, torch.float16), (w, torch.float16), (bias, torch.float32)):
        if t.dtype != dt or not t.is_cuda or not t.is_contiguous():
            raise ValueError("a, w: contiguous fp16 cuda; bias: contiguous fp32 cuda")
    split = a_lo is not None
    odt = torch.float32 if epilogue == EPI_F32 else torch.float16
    c = torch.empty((M, N), dtype=odt, device=a.device)
    c_lo = torch.empty((M, N), dtype=torch.float16, device=a.device) \
        if split and epilogue != EPI_F32 else None
    L = _lib.load()
    check(L.rag_bert_gemm(variant, epilogue, a.data_ptr(), a_lo.data_ptr() if split else None,
                          w.data_ptr(), w_lo.data_ptr() if w_lo is not None else None,
                          bias.data_ptr(), M, N, K, c.data_ptr(),
                          c_lo.data_ptr() if c_lo is not None else None,
                          torch.cuda.current_stream(a.device).cuda_stream))
    return (c, c_lo) if c_lo is not None else c


def attention(qkv: torch.Tensor, cu: torch.Tensor, max_len: int,
              qkv_lo: torch.Tensor | None = None, variant: int | None = None):
    """The forward's attention kernel alone (hidden 384, head_dim 32: bge-small / MiniLM-L6;
    modeling_bert.py eager attention, no mask beyond the packed sequence bounds): qkv fp16
    [T, 1152] (Q | K | V) [+ lo plane], cu int32 [B+1] packed row offsets -> ctx fp16 [T, 384]
    [+ lo plane]. variant: the kernel's VAR bit mask (None = the forward's). Diagnostic entry
    for parity tests and A/B timing."""
    if qkv.dtype != torch.float16 or qkv.dim() != 2 or qkv.shape[1] != 1152 or not qkv.is_cuda:
        raise ValueError("qkv: fp16 cuda [T, 1152]")
    if cu.dtype != torch.int32 or not cu.is_cuda:
        raise ValueError("cu: int32 cuda [B+1]")
    split = qkv_lo is not None
    T = qkv.shape[0]
    ctx = torch.empty((T, 384), dtype=torch.float16, device=qkv.device)
    ctx_lo = torch.empty_like(ctx) if split else None
    check(_lib.load().rag_bert_attention(
        -1 if variant is None else int(variant), qkv.data_ptr(),
        qkv_lo.data_ptr() if split else None, cu.data_ptr(), cu.numel() - 1, int(max_len),
        ctx.data_ptr(), ctx_lo.data_ptr() if split else None,
        torch.cuda.current_stream(qkv.device).cuda_stream))
    return (ctx, ctx_lo) if split else ctx


def linear_add_ln(a: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, gamma: torch.Tensor,
                  beta: torch.Tensor, eps: float, x: torch.Tensor,
                  a_lo: torch.Tensor | None = None, w_lo: torch.Tensor | None = None):
    """BertSelfOutput / BertOutput (modeling_bert.py: LayerNorm(dense(h) + x)) through the
    forward's fused kernel: x fp32 [M, 384] is updated in place to LN(x + a.w^T + bias); returns
    (x, xh) or (x, xh, xl) with the fp16 copy [+ lo plane] the next GEMM reads."""
    M, K = a.shape
    N = w.shape[0]
    for t, dt in ((a, torch.float16), (w, torch.float16), (bias, torch.float32),
                  (gamma, torch.float32), (beta, torch.float32), (x, torch.float32)):
        if t.dtype != dt or not t.is_cuda or not t.is_contiguous():
            raise ValueError("a, w: contiguous fp16 cuda; bias, gamma, beta, x: fp32 cuda")
    if x.shape != (M, N):
        raise ValueError("x must be [M, N]")
    split = a_lo is not None
    xh = torch.empty((M, N), dtype=torch.float16, device=a.device)
    xl = torch.empty_like(xh) if split else None
    check(_lib.load().rag_bert_gemm_add_ln(
        a.data_ptr(), a_lo.data_ptr() if split else None, w.data_ptr(),
        w_lo.data_ptr() if w_lo is not None else None, bias.data_ptr(), gamma.data_ptr(),
        beta.data_ptr(), float(eps), M, N, K, x.data_ptr(), xh.data_ptr(),
        xl.data_ptr() if split else None, torch.cuda.current_stream(a.device).cuda_stream))
    return (x, xh, xl) if split else (x, xh)


EPI_LN_F16, EPI_LN_GELU_F16, EPI_RES_LN = 4, 5, 6   # deferred-LayerNorm epilogues


def linear_dl(epilogue: int, a: torch.Tensor, a_lo: torch.Tensor, w: torch.Tensor,
              w_lo: torch.Tensor, bias: torch.Tensor, c: torch.Tensor, c_lo: torch.Tensor,
              c1: torch.Tensor | None = None, st_in: torch.Tensor | None = None,
              gamma: torch.Tensor | None = None, beta: torch.Tensor | None = None,
              eps: float = 1e-12, st_out: torch.Tensor | None = None) -> None:
    """The deferred-LayerNorm GEMM epilogues (ragmi_bert.h rag_bert_gemm_dl; fp16x3 operand
    planes): EPI_LN_F16 / EPI_LN_GELU_F16 write [gelu](rstd (a.w^T - mean c1) + bias) to the
    planes c / c_lo; EPI_RES_LN reads the residual z from c / c_lo, applies the pending LN
    (st_in, gamma, beta; st_in None: z is already normalised), adds a.w^T + bias and writes the
    sum back with its block statistics to st_out ([M, 6, 2] fp32)."""
    M, K = a.shape
    N = w.shape[0]
    for t in (a, a_lo, w, w_lo, c, c_lo):
        if t.dtype != torch.float16 or not t.is_cuda or not t.is_contiguous():
            raise ValueError("a, a_lo, w, w_lo, c, c_lo: contiguous fp16 cuda")
    if c.shape != (M, N) or c_lo.shape != (M, N):
        raise ValueError("c, c_lo must be [M, N]")
    ptr = lambda t: None if t is None else t.data_ptr()   # noqa: E731
    check(_lib.load().rag_bert_gemm_dl(
        int(epilogue), a.data_ptr(), a_lo.data_ptr(), w.data_ptr(), w_lo.data_ptr(),
        bias.data_ptr(), ptr(c1), ptr(st_in), ptr(gamma), ptr(beta), float(eps), M, N, K,
        c.data_ptr(), c_lo.data_ptr(), ptr(st_out),
        torch.cuda.current_stream(a.device).cuda_stream))


def _weight_ptrs(cfg: dict, weights: dict, head: int, precision: str):
    c = _lib.RagBertConfig(cfg["vocab"], cfg["hidden"], cfg["layers"], cfg["heads"],
                           cfg["inter"], cfg["max_pos"], cfg["type_vocab"], cfg["eps"], head,
                           PRECISIONS[precision])
    names = weight_order(cfg["layers"], head)
    if _lib.load().rag_encoder_num_weights(ctypes.byref(c)) != len(names):
        raise RuntimeError("weight order / ABI mismatch")
    arrs = [np.ascontiguousarray(_lookup(weights, n), dtype=np.float32) for n in names]
    ptrs = (ctypes.POINTER(ctypes.c_float) * len(arrs))(
        *[a.ctypes.data_as(ctypes.POINTER(ctypes.c_float)) for a in arrs])
    return c, arrs, ptrs


def weight_bounds(cfg: dict, weights: dict, head: int = None) -> tuple[float, float]:
    """Static fp16 range bounds of a model's weights (rag_encoder_weight_bounds, host only):
    (plain, deferred) = the largest |value| any fp16 activation plane of the forward can hold
    for any input, without / with the deferred LayerNorm. create refuses plain > 60000; the
    deferred LayerNorm is not used above 60000."""
    head = HEAD_CLS_L2 if head is None else head
    c, arrs, ptrs = _weight_ptrs(cfg, weights, head, "fp16x3")
    p, d = ctypes.c_double(), ctypes.c_double()
    check(_lib.load().rag_encoder_weight_bounds(ctypes.byref(c), ptrs, len(arrs),
                                                ctypes.byref(p), ctypes.byref(d)))
    return p.value, d.value


# ------------------------------------------------------------------ device encoder
class BertEncoder:
    """One encoder instance in HBM (fp16 GEMM weights, fp32 norms/embeddings)."""

    def __init__(self, cfg: dict, weights: dict, head: int, device=None,
                 precision: str = "fp16x3", diagnostic: bool = False):
        # the reference's device argument (main.py:83,89): "cuda[:N]" / None run on that HIP
        # device; "cpu" (USE_GPU=false) is refused, never remapped (_lib.resolve_device)
        dev = _lib.resolve_device(device)
        _lib.require_gpu()
        self._L = _lib.load()
        self.device = torch.device("cuda", _lib.device_index(dev))
        self.cfg, self.head = dict(cfg), head
        self.precision = precision
        c, arrs, ptrs = _weight_ptrs(cfg, weights, head, precision)
        h = ctypes.c_void_p()
        # diagnostic=True (bench / profiling scripts): the process honours the RAGMI_* kernel
        # A/B knobs (RAG_CREATE_DIAGNOSTIC, rag_encoder_create_ex); off in serving code
        check(self._L.rag_encoder_create_ex(ctypes.byref(c), ptrs, len(arrs), self.device.index,
                                            0x100 if diagnostic else 0, ctypes.byref(h)))
        self._h = h
        self.out_dim = cfg["hidden"] if head == HEAD_CLS_L2 else 1

    def set_fusion(self, mode: int) -> None:
        """Residual + LayerNorm fused into the output projections: -1 auto, 0 off, 1 on."""
        check(self._L.rag_encoder_set_fusion(self._h, int(mode)))

    def set_graphs(self, mode: int) -> None:
        """hipGraph replay of small-batch forwards (rag_encoder_set_graphs): -1 auto (T <= 8192
        tokens), 0 off, 1 on."""
        check(self._L.rag_encoder_set_graphs(self._h, int(mode)))

    def set_defer_ln(self, mode: int) -> None:
        """Deferred LayerNorm on the token rows (fp16x3, hidden 384; ragmi_bert.h
        rag_encoder_set_defer_ln): -1 auto, 0 off, 1 on where the model allows."""
        check(self._L.rag_encoder_set_defer_ln(self._h, int(mode)))

    def set_ffn_fused(self, mode: int) -> None:
        """The deferred-LayerNorm forward's FFN as one fused launch per layer (intermediate
        kept on the CU; rag_encoder_set_ffn_fused): -1 auto, 0 off, 1 on."""
        check(self._L.rag_encoder_set_ffn_fused(self._h, int(mode)))

    def range_bounds(self) -> tuple[float, float]:
        """(plain, deferred) static fp16 range bounds of this model (rag_encoder_range_bounds)."""
        p, d = ctypes.c_double(), ctypes.c_double()
        check(self._L.rag_encoder_range_bounds(self._h, ctypes.byref(p), ctypes.byref(d)))
        return p.value, d.value

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._L.rag_encoder_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def forward_packed(self, ids: np.ndarray, types: np.ndarray, cu: np.ndarray,
                       out: torch.Tensor | None = None) -> torch.Tensor:
        """ids/types int32 [T], cu int32 [B+1] (host) -> cuda fp32 [B, out_dim] (or [B])."""
        ids = np.ascontiguousarray(ids, np.int32)
        types = np.ascontiguousarray(types, np.int32)
        cu = np.ascontiguousarray(cu, np.int32)
        B = len(cu) - 1
        T = int(cu[-1])
        lens = np.diff(cu)
        if B < 1 or cu[0] != 0 or (lens < 1).any() or ids.shape != (T,) or types.shape != (T,):
            raise ValueError("bad packed batch")
        if int(lens.max()) > self.cfg["max_pos"]:
            raise ValueError("sequence longer than max_position_embeddings")
        if ids.min() < 0 or ids.max() >= self.cfg["vocab"] or types.min() < 0 or \
                types.max() >= self.cfg["type_vocab"]:
            raise ValueError("token id / type out of range")
        dev = self.device
        # one asynchronous copy from pinned memory (ids | types | cu) instead of three
        # synchronous pageable ones; torch's caching host allocator keeps the pinned block
        # until the copy has run
        staging = torch.empty(2 * T + B + 1, dtype=torch.int32, pin_memory=True)
        sv = staging.numpy()
        sv[:T] = ids
        sv[T:2 * T] = types
        sv[2 * T:] = cu
        dbuf = staging.to(dev, non_blocking=True)
        t_ids, t_ty, t_cu = dbuf[:T], dbuf[T:2 * T], dbuf[2 * T:]
        if out is None:
            shape = (B, self.out_dim) if self.head == HEAD_CLS_L2 else (B,)
            out = torch.empty(shape, dtype=torch.float32, device=dev)
        check(self._L.rag_encoder_forward(self._h, t_ids.data_ptr(), t_ty.data_ptr(),
                                          t_cu.data_ptr(), B, T, int(lens.max()),
                                          out.data_ptr(),
                                          torch.cuda.current_stream(dev).cuda_stream))
        return out

    def forward_device(self, ids: torch.Tensor, types: torch.Tensor, cu: torch.Tensor,
                       max_len: int, out: torch.Tensor | None = None) -> torch.Tensor:
        """Packed batch already in HBM (int32 ids/types [T], cu [B+1]; e.g. assembled on the
        GPU from cached chunk tokens): no host round trip. `max_len` must bound every
        sequence (<= max_position); out-of-range ids are clamped by the embedding kernel."""
        B = cu.numel() - 1
        T = ids.numel()
        if B < 1 or types.numel() != T or not 1 <= max_len <= self.cfg["max_pos"]:
            raise ValueError("bad device batch")
        for t in (ids, types, cu):
            if t.dtype != torch.int32 or not t.is_cuda or not t.is_contiguous():
                raise ValueError("ids/types/cu must be contiguous int32 cuda tensors")
        if out is None:
            shape = (B, self.out_dim) if self.head == HEAD_CLS_L2 else (B,)
            out = torch.empty(shape, dtype=torch.float32, device=self.device)
        check(self._L.rag_encoder_forward(self._h, ids.data_ptr(), types.data_ptr(),
                                          cu.data_ptr(), B, T, int(max_len), out.data_ptr(),
                                          torch.cuda.current_stream(self.device).cuda_stream))
        return out

    def forward_padded(self, ids: np.ndarray, types: np.ndarray, mask: np.ndarray):
        """HF-style right-padded [B, S] batch -> same outputs as the padded reference."""
        lens = mask.sum(1).astype(np.int32)
        cu = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
        sel = mask.astype(bool)
        return self.forward_packed(ids[sel], types[sel], cu)


# ------------------------------------------------------------------ tokenisation
class WordPiece:
    """BERT WordPiece from a local vocab.txt ([CLS] a [SEP] (b [SEP]); truncation
    'longest_first' to max_length; token types 0/1) — what sentence-transformers' tokenizer
    does for both reference models (transformers BertTokenizer: BertNormalizer(clean_text,
    handle_chinese_chars, strip_accents, lowercase) + BertPreTokenizer + WordPiece('##',
    100-char words)). The normaliser flags come from the checkpoint's tokenizer_config.json
    (`from_model_dir`; bge-small-en-v1.5 and ms-marco-MiniLM-L-6-v2: do_lower_case true,
    strip_accents unset = follow lowercasing, tokenize_chinese_chars true). Parity: tests/
    test_tokenizer_cpu.py, against transformers.BertTokenizer and a pure-Python restatement
    (oracle/wordpiece_ref.py)."""

    def __init__(self, vocab_file: str, max_length: int = 512, lowercase: bool = True,
                 strip_accents: bool | None = None, tokenize_chinese_chars: bool = True):
        from tokenizers import BertWordPieceTokenizer
        self.tok = BertWordPieceTokenizer(vocab_file, lowercase=lowercase,
                                          strip_accents=strip_accents,
                                          handle_chinese_chars=tokenize_chinese_chars,
                                          clean_text=True, wordpieces_prefix="##")
        self.tok.enable_truncation(max_length=max_length, strategy="longest_first")
        self.max_length = max_length
        # host-native ASCII path (rag_wordpiece_*, csrc/wordpiece_capi.cpp): same ids, no GIL;
        # texts with non-ASCII bytes go through the Rust tokenizer above
        self._native = None
        try:
            with open(vocab_file, "rb") as f:
                vb = f.read()
            L = _lib.load()
            h = ctypes.c_void_p()
            check(L.rag_wordpiece_create(vb, len(vb), int(max_length), int(bool(lowercase)),
                                         ctypes.byref(h)))
            self._native = (L, h)
        except _lib.RagmiUnavailable:
            self._native = None

    def __del__(self):
        nat = getattr(self, "_native", None)
        if nat is not None:
            try:
                nat[0].rag_wordpiece_destroy(nat[1])
            except Exception:
                pass

    @classmethod
    def from_model_dir(cls, model_dir: str, max_length: int | None = None) -> "WordPiece":
        """vocab.txt + tokenizer_config.json (+ sentence_bert_config.json's max_seq_length)
        of a local checkpoint; max_length: explicit > sentence_bert_config > model_max_length
        > 512."""
        def _json(name):
            f = os.path.join(model_dir, name)
            if not os.path.exists(f):
                return {}
            with open(f) as fh:
                return json.load(fh)
        tc, sb = _json("tokenizer_config.json"), _json("sentence_bert_config.json")
        if max_length is None:
            max_length = sb.get("max_seq_length") or tc.get("model_max_length") or 512
            max_length = min(int(max_length), 512)
        return cls(os.path.join(model_dir, "vocab.txt"), int(max_length),
                   lowercase=bool(tc.get("do_lower_case", True)),
                   strip_accents=tc.get("strip_accents"),
                   tokenize_chinese_chars=bool(tc.get("tokenize_chinese_chars", True)))

    def encode_packed(self, texts, pairs=None):
        """Packed WordPiece ids / token types (int32 [T]) and cu_seqlens (int32 [B+1]) of a
        batch of texts (or (text, pair) pairs). ASCII texts: the host-native encoder
        (rag_wordpiece_encode; releases the GIL); anything else: the Rust tokenizer, spliced
        in place. Same ids either way (tests/test_tokenizer_cpu.py)."""
        texts = list(texts)
        pairs = None if pairs is None else list(pairs)
        if self._native is not None and texts:
            return self._encode_native(texts, pairs)
        return self._encode_rust(texts, pairs)

    def _encode_native(self, texts, pairs):
        L, h = self._native
        n = len(texts)

        def blob(strs):
            bs = [t.encode("utf-8") for t in strs]
            off = np.zeros(n + 1, np.int64)
            np.cumsum([len(b) for b in bs], out=off[1:])
            return b"".join(bs), off
        tb, to = blob(texts)
        pb, po = blob(pairs) if pairs is not None else (None, None)
        cap = n * self.max_length
        ids = np.empty(cap, np.int32)
        types = np.empty(cap, np.int32)
        cu = np.empty(n + 1, np.int32)
        fb = np.zeros(n, np.uint8)
        check(L.rag_wordpiece_encode(
            h, tb, to.ctypes.data_as(_lib.c_i64p), pb,
            po.ctypes.data_as(_lib.c_i64p) if po is not None else None, n,
            ids.ctypes.data_as(_lib.c_i32p), types.ctypes.data_as(_lib.c_i32p),
            cu.ctypes.data_as(_lib.c_i32p), cap,
            fb.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))))
        if not fb.any():
            T = int(cu[-1])
            return ids[:T].copy(), types[:T].copy(), cu
        # splice the Rust tokenizer's encodings of the non-ASCII entries into place
        js = np.nonzero(fb)[0]
        r_ids, r_types, r_cu = self._encode_rust([texts[j] for j in js],
                                                 None if pairs is None else [pairs[j] for j in js])
        parts_i, parts_t, lens = [], [], np.diff(cu).astype(np.int64)
        k = 0
        for j in range(n):
            if fb[j]:
                a, b = r_cu[k], r_cu[k + 1]
                parts_i.append(r_ids[a:b])
                parts_t.append(r_types[a:b])
                lens[j] = b - a
                k += 1
            else:
                parts_i.append(ids[cu[j]:cu[j + 1]])
                parts_t.append(types[cu[j]:cu[j + 1]])
        out_cu = np.zeros(n + 1, np.int32)
        np.cumsum(lens, out=out_cu[1:])
        return np.concatenate(parts_i), np.concatenate(parts_t), out_cu

    def _encode_rust(self, texts, pairs=None):
        inp = list(texts) if pairs is None else list(zip(texts, pairs))
        raw = getattr(self.tok, "_tokenizer", None)
        encs = (raw.encode_batch_fast(inp) if raw is not None and
                hasattr(raw, "encode_batch_fast") else self.tok.encode_batch(inp))
        id_lists = [e.ids for e in encs]
        lens = np.fromiter((len(x) for x in id_lists), np.int32, len(id_lists))
        T = int(lens.sum())
        ids = np.fromiter(itertools.chain.from_iterable(id_lists), np.int32, T)
        if pairs is None:
            types = np.zeros(T, np.int32)
        else:
            types = np.fromiter(itertools.chain.from_iterable(e.type_ids for e in encs),
                                np.int32, T)
        cu = np.zeros(len(id_lists) + 1, np.int32)
        np.cumsum(lens, out=cu[1:])
        return ids, types, cu


def _load_dir(model_dir: str):
    with open(os.path.join(model_dir, "config.json")) as f:
        hf = json.load(f)
    st = os.path.join(model_dir, "model.safetensors")
    if not os.path.exists(st):
        raise FileNotFoundError(f"{st}: only safetensors checkpoints are loaded")
    return config_from_hf(hf), load_safetensors(st), os.path.join(model_dir, "vocab.txt"), hf


# ------------------------------------------------------------------ reference-shaped APIs
class SentenceTransformer:
    """`SentenceTransformer(model_dir).encode(...)` for bge-small-en-v1.5 (CLS + L2 norm)."""

    def __init__(self, model_dir: str | None = None, device=None, *, cfg=None, weights=None,
                 vocab_file=None, max_seq_length: int | None = None, precision: str = "fp16x3"):
        _lib.resolve_device(device)                # "cpu" refused before the checkpoint loads
        if model_dir is not None:
            st_head_from_dir(model_dir)            # refuses any head but CLS + Normalize
            cfg, weights, vocab_file, _ = _load_dir(model_dir)
        if cfg is None or weights is None:
            raise ValueError("need a local model_dir or cfg + weights (no hub access)")
        self.encoder = BertEncoder(cfg, weights, HEAD_CLS_L2, device, precision)
        self.tokenizer = (WordPiece.from_model_dir(model_dir, max_seq_length) if model_dir
                          else WordPiece(vocab_file, max_seq_length or 512) if vocab_file
                          else None)
        self.max_seq_length = self.tokenizer.max_length if self.tokenizer else max_seq_length

    def encode(self, sentences, batch_size: int = 32, convert_to_numpy: bool = True,
               show_progress_bar=None, **kwargs):
        single = isinstance(sentences, str)
        texts = [sentences] if single else list(sentences)
        if not texts:
            return np.zeros((0, self.encoder.out_dim), np.float32)
        if self.tokenizer is None:
            raise RuntimeError("no vocab.txt: use encode_ids with token ids")
        outs = []
        for i in range(0, len(texts), max(batch_size, 1)):
            ids, types, cu = self.tokenizer.encode_packed(texts[i:i + batch_size])
            outs.append(self.encoder.forward_packed(ids, types, cu))
        emb = torch.cat(outs)
        if not convert_to_numpy:
            return emb[0] if single else emb
        emb = emb.cpu().numpy()
        return emb[0] if single else emb

    def encode_ids(self, ids, types, cu) -> np.ndarray:
        return self.encoder.forward_packed(ids, types, cu).cpu().numpy()


class CrossEncoder:
    """`CrossEncoder(model_dir).predict([[q, t], ...])` for ms-marco-MiniLM-L-6-v2
    (BertForSequenceClassification, num_labels = 1). The activation applied to the logits is
    sentence-transformers' (`ce_activation`): the checkpoint's configured one — Identity for
    ms-marco-MiniLM-L-6-v2, i.e. raw logits, which frontend.py:112-117 then squashes itself —
    or Sigmoid when num_labels == 1 and the config names none. `activation_fn` overrides it
    (sentence-transformers' CrossEncoder(default_activation_function=...) /
    (activation_fn=...)); predict(activation_fct=...) overrides it per call."""

    def __init__(self, model_dir: str | None = None, device=None, *, cfg=None, weights=None,
                 vocab_file=None, max_length: int | None = None, precision: str = "fp16x3",
                 activation_fn=None, default_activation_function=None):
        _lib.resolve_device(device)                # "cpu" refused before the checkpoint loads
        hf = None
        if model_dir is not None:
            cfg, weights, vocab_file, hf = _load_dir(model_dir)
        if cfg is None or weights is None:
            raise ValueError("need a local model_dir or cfg + weights (no hub access)")
        nl = hf_num_labels(hf) if hf is not None else int(cfg.get("num_labels", 1))
        if nl != 1:
            raise NotImplementedError(f"num_labels {nl}: only the 1-logit head is implemented")
        self.activation = ce_activation(
            hf if hf is not None else {"num_labels": 1, **{k: cfg[k] for k in (
                "sbert_ce_default_activation_function", "sentence_transformers") if k in cfg}},
            activation_fn if activation_fn is not None else default_activation_function)
        self.encoder = BertEncoder(cfg, weights, HEAD_POOLER_CLS, device, precision)
        self.tokenizer = (WordPiece.from_model_dir(model_dir, max_length) if model_dir
                          else WordPiece(vocab_file, max_length or 512) if vocab_file else None)

    def _activate(self, logits: torch.Tensor, activation_fct=None) -> torch.Tensor:
        if activation_fct is not None and not isinstance(activation_fct, (str, torch.nn.Module)):
            return activation_fct(logits)              # a caller's own callable
        act = self.activation if activation_fct is None else ce_activation(None, activation_fct)
        return torch.sigmoid(logits) if act == "sigmoid" else logits

    def predict(self, sentences, batch_size: int = 32, convert_to_numpy: bool = True,
                activation_fct=None, **kwargs):
        pairs = [list(p) for p in sentences]
        if not pairs:
            return np.zeros((0,), np.float32)
        if self.tokenizer is None:
            raise RuntimeError("no vocab.txt: use predict_ids with token ids")
        outs = []
        for i in range(0, len(pairs), max(batch_size, 1)):
            chunk = pairs[i:i + batch_size]
            ids, types, cu = self.tokenizer.encode_packed([p[0] for p in chunk],
                                                          [p[1] for p in chunk])
            outs.append(self.encoder.forward_packed(ids, types, cu))
        s = self._activate(torch.cat(outs), activation_fct)
        return s.cpu().numpy() if convert_to_numpy else s

    def predict_ids(self, ids, types, cu, activation_fct=None) -> np.ndarray:
        return self._activate(self.encoder.forward_packed(ids, types, cu),
                              activation_fct).cpu().numpy()
