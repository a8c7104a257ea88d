#!/bin/bash
# PMC FETCH_SIZE of the partitioned small-shard scan launches (1.25M / 2.5M rows per GPU) into
# profiles/scan_pmc.json's by_rows table, and a kernel-trace --stats run at 1.25M rows
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp; mkdir -p gpurun_out/profiles
cp profiles/scan_pmc.json gpurun_out/profiles/scan_pmc.json
for rows in 1250000 2500000; do
  rm -rf gpurun_out/pmc_$rows
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_$rows" -o p \
    -- python3 "$R/bench.py" --rows $rows --steps 20 --warmup 5 --no-recall --no-cpu --no-configs > gpurun_out/pmc_$rows.log 2>&1 || { tail -20 gpurun_out/pmc_$rows.log; exit 1; }
  python3 scripts/pmc_by_rows.py gpurun_out/pmc_$rows $rows r05n_rows$rows || exit 1
done
rm -rf gpurun_out/tr125
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/tr125" -o t \
  -- python3 "$R/bench.py" --rows 1250000 --steps 200 --warmup 10 --no-recall --no-cpu --no-configs > gpurun_out/tr125.log 2>&1 || { tail -20 gpurun_out/tr125.log; exit 1; }
grep '^{' gpurun_out/tr125.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); r=d['roofline']; print('bench', d['value'], r['avg_ms'], r['busy_ms_per_launch'], r['frac'])"
grep -i "scan_kernel" gpurun_out/tr125/*kernel_stats.csv | head -3
