#!/bin/bash
# HBM traffic of each encoder GEMM inside the rerank forward (deferred-LN WS kernels, 117K
# tokens fp16x3): one FETCH_SIZE pass, one WRITE_SIZE pass, one MFMA-busy pass
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/fpmc_*
j=0
for ctrs in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  j=$((j+1))
  STAGES=rerank PRECS=fp16x3 CPU=0 REPS=2 timeout -s KILL 240 rocprofv3 --pmc $ctrs --output-format csv \
      -d "$R/gpurun_out/fpmc_$j" -o p -- python3 "$R/scripts/bench_stages.py" > gpurun_out/fpmc_$j.log 2>&1 \
      || { rc=$?; echo "pass $j rc=$rc"; tail -5 gpurun_out/fpmc_$j.log; exit $rc; }
done
T=$(grep '^{' gpurun_out/fpmc_1.log | head -1 | python3 -c "import json,sys; print(json.loads(sys.stdin.readline())['tokens'])")
python3 scripts/fwd_pmc_summary.py gpurun_out/fpmc_1 $T FETCH_SIZE | tee gpurun_out/fwd_pmc.jsonl
python3 scripts/fwd_pmc_summary.py gpurun_out/fpmc_2 $T WRITE_SIZE | tee -a gpurun_out/fwd_pmc.jsonl
python3 scripts/fwd_pmc_summary.py gpurun_out/fpmc_3 $T MFMA | tee -a gpurun_out/fwd_pmc.jsonl
