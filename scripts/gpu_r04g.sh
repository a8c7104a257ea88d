#!/bin/bash
# round 4: WS GEMM probe decomposition, 8 x 64x64 MFMA waves (WS) vs 4 x 128x64 (BIG128)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; O=gpurun_out
GEMM_M=117000 GEMM_VARIANTS=19,20,21,22,35,36,38,37 timeout -k 10 300 python3 -u scripts/bench_gemm.py > $O/gemm_probes_b128.jsonl 2> $O/gemm.err || { tail -20 $O/gemm.err; exit 1; }
grep layer_ms $O/gemm_probes_b128.jsonl
