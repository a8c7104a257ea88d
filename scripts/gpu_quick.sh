#!/bin/bash
# parity tests + 10M bench + 1.25M bench + variants at both sizes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then grep -E "^(FAILED|E  )" gpurun_out/pytest_gpu.log | head -30; exit $rc; fi
for R in 10000000 1250000; do
  timeout -k 10 300 python bench.py --rows $R --steps 100 --warmup 5 --no-cpu > gpurun_out/bench_$R.log 2>&1 || { rc=$?; tail -20 gpurun_out/bench_$R.log; exit $rc; }
  grep '^{' gpurun_out/bench_$R.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($R, d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_ms'], d['recall_at_5'], d['top15_exact_vs_oracle'])"
done
for R in 10000000 1250000; do
  ROWS=$R VARIANTS=${VARIANTS:-0,3} ROUNDS=5 timeout -k 10 300 python scripts/scan_variants.py > gpurun_out/variants_$R.log 2>&1 || exit $?
  grep variant gpurun_out/variants_$R.log
done
