#!/bin/bash
# round 6: default bench with in-process legs (dedicated-queue pipeline streams) vs child legs,
# and the headline on whole-CU-mask streams
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rm -f gpurun_out/r06i_legs.jsonl
for legs in inproc child; do
  timeout -k 10 420 python -u bench.py --legs $legs --no-cpu > gpurun_out/r06i_$legs.json 2> gpurun_out/r06i_$legs.err \
      || { rc=$?; tail -5 gpurun_out/r06i_$legs.err; exit $rc; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r06i_$legs.json').read().strip().splitlines()[-1])
print(json.dumps({'legs':'$legs','headline':d['value'],'config2':d['config2'].get('value'),'config3':d['config3'].get('value'),
 'c2_traffic':(d['config2'].get('roofline') or {}).get('traffic'),'c3_traffic':(d['config3'].get('roofline') or {}).get('traffic'),
 'c2_err':d['config2'].get('error'),'c3_err':d['config3'].get('error')}))" | tee -a gpurun_out/r06i_legs.jsonl
done
timeout -k 10 300 python -u bench.py --no-configs --no-cpu --partition whole > gpurun_out/r06i_whole.json 2> gpurun_out/r06i_whole.err \
    || { rc=$?; tail -5 gpurun_out/r06i_whole.err; exit $rc; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r06i_whole.json').read().strip().splitlines()[-1]); print('whole headline', d['value'], d['roofline']['frac'], d['exact_batches'])"
# attention staging probes (diagnostic build): 42 vs 42+128 (zeros stored, no loads) vs 42+256
RAGMI_LIB_AB=$PWD/ab/diag.so VARIANTS=42,170,298 PRECS=fp16x3 ROUNDS=3 REPS=10 timeout -k 10 200 \
    python -u scripts/bench_attn.py > gpurun_out/r06i_attn_probes.jsonl 2> gpurun_out/r06i_attn.err \
    || { rc=$?; tail -5 gpurun_out/r06i_attn.err; exit $rc; }
cat gpurun_out/r06i_attn_probes.jsonl
