#!/bin/bash
# full GPU suite, pipeline bench, encoder stage kernel trace (rocprof) -> gpurun_out
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 \
    --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then grep -E "^(FAILED|E  )" gpurun_out/pytest_gpu.log | head -30; exit $rc; fi
STEPS=40 timeout -k 10 400 python -u scripts/bench_pipeline.py > gpurun_out/pipeline.log 2>&1 || { rc=$?; tail -20 gpurun_out/pipeline.log; exit $rc; }
grep '^{' gpurun_out/pipeline.log | cut -c1-200
export TMPDIR=/tmp
rm -rf gpurun_out/prof_stages
REPS=5 CPU=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_stages" -o st \
    -- python3 "$R/scripts/bench_stages.py" > gpurun_out/prof_stages.log 2>&1 || { rc=$?; tail -20 gpurun_out/prof_stages.log; exit $rc; }
python3 scripts/stage_breakdown.py gpurun_out/prof_stages > gpurun_out/stage_breakdown.txt
cp "$(find gpurun_out/prof_stages -name 'st_kernel_stats.csv' | head -1)" gpurun_out/stages_kernel_stats.csv
echo done
