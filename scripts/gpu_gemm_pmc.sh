#!/bin/bash
# PMC passes over one GEMM shape (TILE and PIPE): MFMA busy, wave states, LDS, clock.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out/gemm_pmc
export TMPDIR=/tmp
timeout -k 5 60 rocprofv3 -L > gpurun_out/gemm_pmc/counters.txt 2>&1 || true
SHAPE=${SHAPE:-"117000 1152 384 0 fp16"}
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM"
for V in 1 2; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d "$R/gpurun_out/gemm_pmc/v${V}_p$i" -o pmc \
      -- python3 "$R/scripts/gemm_one.py" $SHAPE $V 20 > gpurun_out/gemm_pmc/v${V}_p$i.log 2>&1 || { echo "pass v$V p$i failed"; tail -5 gpurun_out/gemm_pmc/v${V}_p$i.log; }
  done
done
ls -R gpurun_out/gemm_pmc | head -40
