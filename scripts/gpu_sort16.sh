#!/bin/bash
# end-of-scan sort of pending-only queries, 4 per 16-lane pass: parity + A/B vs the 32-lane sort
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/sort16.jsonl
: > $out
timeout -k 10 600 python -u -m pytest tests/test_scan_gpu.py tests/test_exactness_gpu.py tests/test_storage32_gpu.py \
    -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/sort16_tests.log 2>&1
rc=$?; tail -2 gpurun_out/sort16_tests.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|E  )" gpurun_out/sort16_tests.log | head -30; exit $rc; fi
for rows in 1250000 2500000 10000000; do
  echo "# rows=$rows" >> $out
  ROWS=$rows VARIANTS=0,16,15,7,4 ROUNDS=7 timeout -k 10 300 python -u scripts/scan_variants.py >> $out 2> gpurun_out/sort16.err || { rc=$?; tail -20 gpurun_out/sort16.err; exit $rc; }
done
timeout -k 10 300 python -u bench.py --rows 1250000 --steps 300 --warmup 10 --no-cpu >> $out 2>> gpurun_out/sort16.err || { rc=$?; tail -20 gpurun_out/sort16.err; exit $rc; }
cut -c1-260 $out
