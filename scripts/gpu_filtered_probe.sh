#!/bin/bash
# filtered line (10M x 384, per-query ticker filter) at 192 vs 512 scan workgroups, then kernel
# traces of the filtered and headline commands: the scan launches' true durations and overlap
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp
mkdir -p gpurun_out
VAR=RAGMI_SCAN_WGS VALS="192 512" ARGS="--config filtered --no-cpu --no-recall" OUT=gpurun_out/filtered_wgs.jsonl TMO=300 bash scripts/gpu_env_sweep.sh || exit 1
for m in filtered 4; do
  rm -rf gpurun_out/prof_$m
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/prof_$m" -o tr \
      -- python3 "$R/bench.py" --config $m --no-cpu --no-recall --steps 30 > gpurun_out/prof_$m.log 2>&1 || { tail -20 gpurun_out/prof_$m.log; exit 1; }
  python3 scripts/scan_overlap.py gpurun_out/prof_$m config_$m
done
