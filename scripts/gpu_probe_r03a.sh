#!/bin/bash
# round-3 probes: (1) kernel trace of the 32-query bge-small forward (config 2's encoder),
# (2) FETCH_SIZE of one scan launch at the N = 2 / 4 / 8 shard sizes for bench.py's traffic
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out/profiles
export TMPDIR=/tmp
rm -rf gpurun_out/prof_encq
STAGES=encode_q PRECS=fp16x3 CPU=0 REPS=30 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv \
  -d "$R/gpurun_out/prof_encq" -o encq -- python3 "$R/scripts/bench_stages.py" > gpurun_out/prof_encq.log 2>&1 || { rc=$?; tail -20 gpurun_out/prof_encq.log; exit $rc; }
grep '^{' gpurun_out/prof_encq.log
python3 scripts/trace_forward.py gpurun_out/prof_encq 87 > gpurun_out/encq_forward.txt && tail -25 gpurun_out/encq_forward.txt
for rows in 1250000 2500000 5000000; do
  rm -rf gpurun_out/prof_pmc_$rows
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/prof_pmc_$rows" -o pmc \
    -- python3 "$R/bench.py" --rows $rows --steps 10 --warmup 2 --no-recall --no-cpu > gpurun_out/prof_pmc_$rows.log 2>&1 || { rc=$?; tail -20 gpurun_out/prof_pmc_$rows.log; exit $rc; }
  COMMIT=${COMMIT:-} python3 scripts/pmc_by_rows.py gpurun_out/prof_pmc_$rows $rows r03a_rows$rows || exit 1
done
