#!/bin/bash
# round 6: 2-wave attention workgroups for <= 32-token query batches (RAGMI_ATTN_SHORT):
# encode_q stage time + output digest, config-2 pipeline, alternating (diagnostic handles)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/r06x_attn_short.jsonl
rm -f $out
for a in ${SPECS:-1 0 1 0 1 0}; do
  RAGMI_ATTN_SHORT=$a STAGES=encode_q PRECS=fp16x3 CPU=0 REPS=50 SAVE_OUT=1 \
    timeout -k 10 200 python -u scripts/bench_stages.py > gpurun_out/r06x_st.jsonl 2> gpurun_out/r06x.err \
    || { rc=$?; tail -5 gpurun_out/r06x.err; exit $rc; }
  RAGMI_ATTN_SHORT=$a timeout -k 10 300 python -u bench.py --config 2 --diagnostic --no-cpu \
    > gpurun_out/r06x_c2.json 2>> gpurun_out/r06x.err || { rc=$?; tail -5 gpurun_out/r06x.err; exit $rc; }
  python3 -c "
import json
st=[json.loads(l) for l in open('gpurun_out/r06x_st.jsonl') if l.startswith('{')][0]
c2=json.loads(open('gpurun_out/r06x_c2.json').read().strip().splitlines()[-1])
print(json.dumps({'attn_short': $a, 'encode_q_ms': st['ms'], 'out_sha1': st.get('out_sha1'), 'config2_qps': c2['value'], 'encode_diff': c2.get('encode_max_abs_diff_vs_oracle'), 'exact': c2.get('search_top15_exact_queries')}))" | tee -a $out
done
