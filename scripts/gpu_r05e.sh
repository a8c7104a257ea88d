#!/bin/bash
# CU partition at the larger shards: 5M (N = 2) and 10M (N = 1 headline) rows, serial order
# with 2 in flight (the default there) vs free order on 2 / 4 partition streams
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/part_big.jsonl; : > $out
for rep in 1 2; do
  for a in "--rows 10000000" "--rows 10000000 --scan-order free --streams 4 --partition on" "--rows 10000000 --scan-order free --streams 2 --partition on" "--rows 5000000" "--rows 5000000 --scan-order free --streams 4 --partition on"; do
    timeout -k 10 300 python3 -u bench.py $a --steps 50 --warmup 5 --no-cpu --no-configs 2> gpurun_out/pb.err | grep '^{' | sed "s/^{/{\"args\": \"$a\", /" >> $out || { tail -20 gpurun_out/pb.err; exit 1; }
  done
done
python3 -c "
import json
for l in open('$out'):
    d=json.loads(l); r=d['roofline']; print(d['args'], d['value'], d['exact_batches'], d['config'].get('cu_partition'), r['frac'])"
