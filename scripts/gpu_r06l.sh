#!/bin/bash
# round 6: batches in flight for the config-2 / config-3 pipelines now that every batch stream
# has a dedicated hardware queue (whole-CU-mask streams)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/r06l_streams.jsonl
rm -f $out
for spec in "2 4" "2 6" "2 8" "3 3" "3 4" "3 6" "2 4" "3 3"; do
  set -- $spec
  timeout -k 10 240 python -u bench.py --config $1 --streams $2 --no-cpu > gpurun_out/r06l_c$1_s$2.json 2> gpurun_out/r06l.err \
      || { rc=$?; tail -5 gpurun_out/r06l.err; exit $rc; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r06l_c$1_s$2.json').read().strip().splitlines()[-1])
print(json.dumps({'config':$1,'streams':$2,'value':d['value'],'ms_per_step':d['ms_per_step'],'checks':{k:v for k,v in d.items() if 'exact' in k or 'recall' in k or 'max' in k}}))" | tee -a $out
done
