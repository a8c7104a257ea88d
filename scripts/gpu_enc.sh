#!/bin/bash
# Encoder iteration on the GPU box: encoder/rag/store parity tests, stage bench, kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest ${TESTS:-tests/test_encoders_gpu.py tests/test_rag_gpu.py tests/test_store_gpu.py} \
    -q -p no:cacheprovider --timeout 500 > gpurun_out/pytest_enc.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_enc.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then grep -E "^(FAILED|E  )" gpurun_out/pytest_enc.log | head -30; exit $rc; fi
CPU=${CPU:-0} timeout -k 10 400 python scripts/bench_stages.py > gpurun_out/stages.log 2>&1 || { rc=$?; tail -20 gpurun_out/stages.log; exit $rc; }
grep '^{' gpurun_out/stages.log
if [ "${PROF:-1}" = "1" ]; then
  export TMPDIR=/tmp
  REPS=5 CPU=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_stages" -o st \
      -- python3 "$R/scripts/bench_stages.py" > gpurun_out/prof_stages.log 2>&1 || { rc=$?; tail -20 gpurun_out/prof_stages.log; exit $rc; }
  python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof_stages/**/st_kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:14]:
    print(f"{r['Name'][:60]:60s} {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:9.1f} us  max {float(r['MaxNs'])/1e3:9.1f} us  {r['Percentage'][:5]}%")
PY
fi
exit 0
