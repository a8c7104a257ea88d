#!/bin/bash
# IEEE-maximum tile/block maxima: parity (scan, exactness, attention) + timing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/maxnc.jsonl
: > $out
timeout -k 10 600 python -u -m pytest tests/test_scan_gpu.py tests/test_exactness_gpu.py tests/test_attention_gpu.py \
    tests/test_storage32_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/maxnc_tests.log 2>&1
rc=$?; tail -2 gpurun_out/maxnc_tests.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|E  )" gpurun_out/maxnc_tests.log | head -30; exit $rc; fi
for rows in 10000000 1250000; do
  echo "# rows=$rows" >> $out
  ROWS=$rows VARIANTS=0,4,7 ROUNDS=5 timeout -k 10 300 python -u scripts/scan_variants.py >> $out 2> gpurun_out/maxnc.err || { rc=$?; tail -20 gpurun_out/maxnc.err; exit $rc; }
done
VARIANTS=2,10 PRECS=fp16x3 timeout -k 10 200 python -u scripts/bench_attn.py >> $out 2>> gpurun_out/maxnc.err || { rc=$?; tail -20 gpurun_out/maxnc.err; exit $rc; }
timeout -k 10 300 python -u bench.py --no-cpu >> $out 2>> gpurun_out/maxnc.err || { rc=$?; tail -20 gpurun_out/maxnc.err; exit $rc; }
cut -c1-300 $out
