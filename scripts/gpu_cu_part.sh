#!/bin/bash
# CU-partitioned batches in flight at the 8-GPU shard size (scripts/diag/cu_partition.py):
# baseline (4 torch streams, default grid) vs 4 CU-masked streams at several scan grids
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; out=gpurun_out/cu_part.jsonl; : > $out
for rep in 1 2; do
  for cfg in "1 0" "4 48" "4 64" "4 96" "4 128" "2 96"; do
    set -- $cfg
    if [ "$2" = "0" ]; then env_wgs=""; else env_wgs="RAGMI_SCAN_WGS=$2"; fi
    env $env_wgs timeout -k 10 200 python3 -u scripts/diag/cu_partition.py $1 2> gpurun_out/cu_part.err >> $out || { tail -20 gpurun_out/cu_part.err; exit 1; }
  done
done
cat $out
