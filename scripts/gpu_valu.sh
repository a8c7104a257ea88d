#!/bin/bash
# VALU (v_dot2) vs MFMA scan ablation at 10M x 384: kernel times (interleaved rounds), then a
# rocprofv3 kernel-trace pass and a PMC pass (MFMA / VALU busy) of variants 0 and 8.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
VARIANTS=0,3,4,8 ROUNDS=4 timeout -k 10 300 python -u scripts/scan_variants.py > gpurun_out/valu_variants.jsonl 2> gpurun_out/valu_variants.err \
    || { rc=$?; tail -20 gpurun_out/valu_variants.err; exit $rc; }
cat gpurun_out/valu_variants.jsonl
rm -rf gpurun_out/valu_trace gpurun_out/valu_pmc
VARIANTS=0,8 ROUNDS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/valu_trace" -o trace \
    -- python3 "$R/scripts/scan_variants.py" > gpurun_out/valu_trace.log 2>&1 || { rc=$?; tail -20 gpurun_out/valu_trace.log; exit $rc; }
VARIANTS=0,8 ROUNDS=1 timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d "$R/gpurun_out/valu_pmc" -o pmc \
    -- python3 "$R/scripts/scan_variants.py" > gpurun_out/valu_pmc.log 2>&1 || { rc=$?; tail -20 gpurun_out/valu_pmc.log; exit $rc; }
find gpurun_out/valu_trace gpurun_out/valu_pmc -name "*.csv" | head
