#!/bin/bash
# HBM traffic of one encoder forward: FETCH_SIZE and WRITE_SIZE passes
# (separate rocprofv3 runs) over scripts/bench_stages.py for the config-3 rerank forward and
# the config-2 query forward, summarised by scripts/encoder_traffic.py into
# gpurun_out/encoder_pmc.json (copied to profiles/ and read by the bench line's legs).
# Graph replay off (RAGMI_ENC_GRAPH=0 on the diagnostic handle): the same kernels, dispatched
# eagerly so every one is counted.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/epmc_* gpurun_out/encoder_pmc.json
for st in rerank encode_q; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    RAGMI_ENC_GRAPH=0 STAGES=$st PRECS=fp16x3 CPU=0 REPS=3 timeout -s KILL 240 rocprofv3 --pmc $ctr \
        --output-format csv -d "$R/gpurun_out/epmc_${st}_$ctr" -o p -- python3 "$R/scripts/bench_stages.py" \
        > gpurun_out/epmc_${st}_$ctr.log 2>&1 \
        || { rc=$?; echo "pass $st $ctr rc=$rc"; tail -5 gpurun_out/epmc_${st}_$ctr.log; exit $rc; }
  done
  python3 scripts/encoder_traffic.py $st gpurun_out/epmc_${st}_FETCH_SIZE gpurun_out/epmc_${st}_WRITE_SIZE \
      gpurun_out/epmc_${st}_FETCH_SIZE.log gpurun_out/encoder_pmc.json || exit 1
done
