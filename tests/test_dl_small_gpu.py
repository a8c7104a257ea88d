"""The query-batch deferred-LayerNorm tiles (PipeDlSmall, diagnostic A/B RAGMI_DL_SMALL=1;
csrc/bert_capi.hip launch_dl): the same parity bounds as tests/test_deferred_ln_gpu.py, run in
a fresh process where the variable is set and a diagnostic handle is created first, so the
knob is honoured (common_host.hpp ragmi::Knob). Round 4 measured this path slower than the
split-K + add_ln forward at 32 queries; it stays tested as an A/B."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

SCRIPT = r"""
import sys, torch
sys.path[:0] = [{pkg!r}, {tests!r}, {oracle!r}]
from ragmi.index import FlatIndex
h = FlatIndex(384, 16, torch.device("cuda", 0), diagnostic=True)   # honour RAGMI_DL_SMALL
import test_deferred_ln_gpu as T
from ragmi import _lib
dev = torch.device("cuda", 0)
assert _lib.load().rag_knob_probe(b"RAGMI_DL_SMALL", 0) == 1
for M in (777, 3000):
    for N, gelu in ((1152, False), (1536, True)):
        T.test_ln_consumer_matches_fp64(dev, M, N, gelu)
    for K in (384, 1536):
        for pending in (True, False):
            T.test_residual_ln_matches_fp64(dev, M, K, pending)
for model in ("ce", "bge"):
    T.test_encoder_deferred_forced_vs_oracle(dev, model)
print("dl-small parity ok")
"""


def test_dl_small_tiles_match_fp64(gpu):
    code = SCRIPT.format(pkg=os.path.join(ROOT, "financial-rag-system_amd"), tests=HERE,
                         oracle=os.path.join(ROOT, "oracle"))
    env = dict(os.environ, RAGMI_DL_SMALL="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "dl-small parity ok" in r.stdout
