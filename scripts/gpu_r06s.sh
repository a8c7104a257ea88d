#!/bin/bash
# round 6: CU-mask bit -> XCD / SE / CU mapping (diagnostic probe kernel)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
RAGMI_LIB_AB=$PWD/ab/diag.so timeout -k 10 120 python -u scripts/diag/cu_mask_probe.py > gpurun_out/r06s_cu_mask.jsonl 2> gpurun_out/r06s.err \
  || { rc=$?; tail -5 gpurun_out/r06s.err; exit $rc; }
cat gpurun_out/r06s_cu_mask.jsonl
