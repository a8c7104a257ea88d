#!/bin/bash
# round 4: wide-scan half-tile ring (MODE 5) — bitwise test, DL-small test, config-5 A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_wide_half_gpu.py tests/test_dl_small_gpu.py -x -q --timeout 500 --timeout-method thread > $O/t_half.log 2>&1 || { tail -30 $O/t_half.log; exit 1; }
tail -2 $O/t_half.log
out=$O/wide_half_ab.jsonl; : > $out
run() { timeout -k 10 400 python3 -u bench.py --config 5 --no-cpu --diagnostic "$@" 2>> $O/wh.err | grep '^{' | python3 -c "
import json,sys,os
d=json.loads(sys.stdin.read()); r=d.get('roofline') or {}
print(json.dumps({'args':'$*','half':os.environ.get('RAGMI_WIDE_HALF'),'value':d['value'],'ms':d['ms_per_step'],'frac':r.get('frac'),'avg_ms':r.get('avg_ms')}))" >> $out; }
for rep in 1 2; do
  run --rows 12500000 || exit 1
  RAGMI_WIDE_HALF=1 run --rows 12500000 || exit 1
done
run || exit 1
RAGMI_WIDE_HALF=1 run || exit 1
cat $out
