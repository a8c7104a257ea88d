#!/bin/bash
# config-3 full-size parity tests + the headline bench with per-batch certified checks
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_config3_gpu.py -m gpu -x -v -s \
    -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/config3_tests.log 2>&1
rc=$?
grep -E "max\|d\||passed|failed" gpurun_out/config3_tests.log | tail -12
if [ $rc -ne 0 ]; then grep -E "^(FAILED|E  )" gpurun_out/config3_tests.log | head -30; exit $rc; fi
/usr/bin/time -v timeout -k 10 500 python -u bench.py > gpurun_out/bench_r02b.log 2> gpurun_out/bench_r02b.err \
    || { rc=$?; tail -20 gpurun_out/bench_r02b.err; exit $rc; }
tail -1 gpurun_out/bench_r02b.log
grep -E "Elapsed|Maximum resident" gpurun_out/bench_r02b.err
