#!/bin/bash
# round 4: rescan v3 (prefetched final merge) parity + tier-2 latency; WS GEMM probes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; O=gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_exactness_gpu.py tests/test_storage32_gpu.py > $O/t_exact.log 2>&1 \
  || { tail -40 $O/t_exact.log; exit 1; }
tail -2 $O/t_exact.log
timeout -k 10 300 python3 -u scripts/bench_tier2.py --marked 4 16 32 > $O/tier2.jsonl 2> $O/tier2.err \
  || { tail -20 $O/tier2.err; exit 1; }
cat $O/tier2.jsonl
GEMM_M=117000 GEMM_VARIANTS=19,20,21,22 timeout -k 10 300 python3 -u scripts/bench_gemm.py > $O/gemm_probes.jsonl 2> $O/gemm.err || { tail -20 $O/gemm.err; exit 1; }
cat $O/gemm_probes.jsonl
