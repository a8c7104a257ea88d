#!/bin/bash
# Fused residual+LayerNorm check: its parity tests, then the stage bench with the fusion on
# (auto) and off (RAGMI_FUSE_LN=0), then a kernel trace of the stages with it on.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
[ "${SKIP_TESTS:-0}" = 1 ] || timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -k "add_ln" -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > gpurun_out/pytest_fuse.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_fuse.log; echo "pytest gemm rc=$rc"
if [ $rc -ne 0 ]; then grep -E "^(FAILED|E  )" gpurun_out/pytest_fuse.log | head -30; exit $rc; fi
timeout -k 10 500 python -u -m pytest tests/test_encoders_gpu.py tests/test_rag_gpu.py -q -p no:cacheprovider \
    --timeout 200 --timeout-method thread > gpurun_out/pytest_fuse_enc.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_fuse_enc.log; echo "pytest enc rc=$rc"
if [ $rc -ne 0 ]; then grep -E "^(FAILED|E  )" gpurun_out/pytest_fuse_enc.log | head -30; exit $rc; fi
for F in -1 0; do
  RAGMI_FUSE_LN=$F CPU=0 timeout -k 10 300 python scripts/bench_stages.py > gpurun_out/stages_fuse$F.log 2>&1 || { rc=$?; tail -20 gpurun_out/stages_fuse$F.log; exit $rc; }
  echo "fuse=$F"; grep '^{' gpurun_out/stages_fuse$F.log
done
export TMPDIR=/tmp
REPS=5 CPU=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_fuse" -o st \
    -- python3 "$R/scripts/bench_stages.py" > gpurun_out/prof_fuse.log 2>&1 || { rc=$?; tail -20 gpurun_out/prof_fuse.log; exit $rc; }
python3 scripts/stage_breakdown.py gpurun_out/prof_fuse > gpurun_out/fuse_breakdown.txt && head -60 gpurun_out/fuse_breakdown.txt
