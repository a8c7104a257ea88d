#!/bin/bash
# CU-partitioned batches in flight, productized: parity tests, then bench lines at the N = 8 /
# N = 4 shard sizes with the partition on / off, and the per-rank RCCL rehearsal at 1.25M
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_partition_gpu.py tests/test_scan_gpu.py tests/test_dist_rccl_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_part.log 2>&1 || { tail -30 gpurun_out/t_part.log; exit 1; }
tail -1 gpurun_out/t_part.log
out=gpurun_out/part_lines.jsonl; : > $out
for rep in 1 2; do
  for a in "--rows 1250000 --partition on" "--rows 1250000 --partition off" "--rows 2500000 --partition on" "--rows 2500000 --partition off"; do
    timeout -k 10 300 python3 -u bench.py $a --steps 200 --warmup 10 --no-cpu --no-configs 2> gpurun_out/pl.err | grep '^{' | sed "s/^{/{\"args\": \"$a\", /" >> $out || { tail -20 gpurun_out/pl.err; exit 1; }
  done
done
RAGMI_DIST_REHEARSAL=1 timeout -k 10 300 python3 -u bench.py --rows 1250000 --steps 200 --warmup 10 --no-configs 2> gpurun_out/pl.err | grep '^{' | sed 's/^{/{"args": "rehearsal 1.25M", /' >> $out || { tail -20 gpurun_out/pl.err; exit 1; }
python3 -c "
import json
for l in open('$out'):
    d=json.loads(l); r=d['roofline']; print(d['args'], d['value'], d['exact_batches'], d['config'].get('cu_partition'), r['frac'], d.get('backend'))"
