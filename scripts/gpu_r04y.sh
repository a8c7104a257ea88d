#!/bin/bash
# round 4: filter tags loaded with the tile's vectors — parity (filtered tests) + filtered line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_scan_gpu.py tests/test_exactness_gpu.py tests/test_rag_gpu.py -k "filt or tag" -x -q --timeout 200 --timeout-method thread > $O/t_filt.log 2>&1 || { tail -30 $O/t_filt.log; exit 1; }
tail -2 $O/t_filt.log
out=$O/filt_ab.jsonl; : > $out
for rep in 1 2; do
  timeout -k 10 400 python3 -u bench.py --config filtered --no-cpu 2>> $O/filt.err | grep '^{' >> $out || { tail $O/filt.err; exit 1; }
done
python3 -c "
import json
for l in open('$out'):
    d=json.loads(l); r=d['roofline']; print(d['value'], r['frac'], r.get('avg_ms'), d.get('exact_batches'))"
