#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for R in 2500000 5000000 10000000; do
for S in 1 2 4; do
  timeout -k 10 200 python bench.py --rows $R --steps 100 --warmup 10 --no-cpu --no-recall --streams $S > gpurun_out/bench_r${R}_s$S.log 2>&1 || { rc=$?; tail -20 gpurun_out/bench_r${R}_s$S.log; exit $rc; }
  grep '^{' gpurun_out/bench_r${R}_s$S.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rows', $R, 'streams', $S, d['value'], d['ms_per_step'], d['roofline']['avg_ms'], d['roofline']['frac'], d['roofline']['step_frac'])"
done
done
