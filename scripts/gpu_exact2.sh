#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_exactness_gpu.py tests/test_scan_gpu.py -m gpu -x -q \
    -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/exact2_tests.log 2>&1
rc=$?; tail -3 gpurun_out/exact2_tests.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|E  )" gpurun_out/exact2_tests.log | head -30; exit $rc; fi
for s in 2 4; do timeout -k 10 200 python -u bench.py --rows 1250000 --steps 300 --warmup 10 --no-cpu --no-recall --streams $s > gpurun_out/small2_$s.log 2>&1 || exit 1; python3 -c "import json; d=json.loads(open(\"gpurun_out/small2_$s.log\").read().strip().splitlines()[-1]); r=d[\"roofline\"]; print($s, d[\"value\"], d[\"ms_per_step\"], r[\"avg_ms\"], r[\"standalone_avg_ms\"], r[\"standalone_frac\"])"; done
