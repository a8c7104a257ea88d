#!/bin/bash
# WS GEMM: what the MFMA waves' LDS fragment reads cost (probes 28/29) next to production (19),
# MFMA-only (20: no DMA, no stores) and no-store (21)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
GEMM_M=117000 GEMM_VARIANTS=19,28,29,20,21 ROUNDS=5 timeout -k 10 300 python -u scripts/bench_gemm.py > gpurun_out/probe_rd.jsonl 2> gpurun_out/probe_rd.err \
    || { rc=$?; tail -20 gpurun_out/probe_rd.err; exit $rc; }
grep '^{' gpurun_out/probe_rd.jsonl | cut -c1-250
