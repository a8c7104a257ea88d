#!/bin/bash
# Exactness fallback: parity tests (near-duplicate clusters, saturated waves) + scan tests +
# a short bench for the cost of the always-launched fallback kernels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_exactness_gpu.py tests/test_scan_gpu.py -m gpu -x -v \
    -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/exact_tests.log 2>&1
rc=$?
tail -3 gpurun_out/exact_tests.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|E  )" gpurun_out/exact_tests.log | head -30; exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu > gpurun_out/bench_exact.log 2>&1 \
    || { rc=$?; tail -20 gpurun_out/bench_exact.log; exit $rc; }
tail -1 gpurun_out/bench_exact.log
