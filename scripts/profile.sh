#!/bin/bash
# rocprofv3 evidence for the bench: (1) kernel trace + stats, (2) a separate PMC pass for
# HBM bytes (FETCH_SIZE), then summaries into profiles/ (copied back via gpurun_out/).
# Usage on the GPU box: TAG=r01 bash scripts/profile.sh; then locally: cp gpurun_out/profiles/* profiles/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
TAG=${TAG:-r01}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > gpurun_out/bench_full.log 2>&1 || { rc=$?; tail -20 gpurun_out/bench_full.log; exit $rc; }
tail -1 gpurun_out/bench_full.log
rm -rf gpurun_out/prof_trace gpurun_out/prof_pmc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_trace" -o trace \
    -- python3 "$R/bench.py" --steps 50 --warmup 20 --no-recall --no-cpu --no-configs > gpurun_out/prof_trace.log 2>&1 || { rc=$?; tail -20 gpurun_out/prof_trace.log; exit $rc; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/prof_pmc" -o pmc \
    -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-recall --no-cpu --no-configs > gpurun_out/prof_pmc.log 2>&1 || { rc=$?; tail -20 gpurun_out/prof_pmc.log; exit $rc; }
# summaries land in gpurun_out/profiles (merged back by gpurun); copy them into profiles/ locally
PROFILES_DIR=gpurun_out/profiles python scripts/summarize_prof.py "$TAG" gpurun_out/prof_trace gpurun_out/prof_pmc gpurun_out/bench_full.log
