#!/bin/bash
# Memory-side PMC passes over one GEMM shape: L2 hit rate, TCP->TCC latency, TA busy, TLB.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out/gemm_pmc2
export TMPDIR=/tmp
SHAPE=${SHAPE:-"117000 1152 384 0 fp16"}
P1="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE"
P2="FETCH_SIZE GRBM_GUI_ACTIVE"
P3="TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCC_EA0_RDREQ_DRAM_sum TCC_TAG_STALL_sum"
P4="WRITE_SIZE TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum"
for V in 1 2; do
  i=0
  for P in "$P1" "$P2" "$P3" "$P4"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d "$R/gpurun_out/gemm_pmc2/v${V}_p$i" -o pmc \
      -- python3 "$R/scripts/gemm_one.py" $SHAPE $V 20 > gpurun_out/gemm_pmc2/v${V}_p$i.log 2>&1 || { echo "pass v$V p$i failed"; tail -5 gpurun_out/gemm_pmc2/v${V}_p$i.log; }
  done
done
