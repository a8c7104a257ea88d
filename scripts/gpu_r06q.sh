#!/bin/bash
# round 6: small-GEMM ring A/B (diagnostic build, RAGMI_SMALL_RING=2: 2-stage ring + 8 KB
# vector area = 40 KB LDS, 4 workgroups per CU) — encode_q stage time + output digest, and
# the config-2 pipeline, alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export RAGMI_LIB_AB=$PWD/ab/diag.so
out=gpurun_out/r06q_small_ring.jsonl
rm -f $out
for r in ${RINGS:-0 2 0 2}; do
  RAGMI_SMALL_RING=$r STAGES=encode_q PRECS=fp16x3 CPU=0 REPS=50 SAVE_OUT=1 \
    timeout -k 10 200 python -u scripts/bench_stages.py > gpurun_out/r06q_st.jsonl 2> gpurun_out/r06q.err \
    || { rc=$?; tail -5 gpurun_out/r06q.err; exit $rc; }
  RAGMI_SMALL_RING=$r timeout -k 10 300 python -u bench.py --config 2 --diagnostic --no-cpu \
    > gpurun_out/r06q_c2.json 2>> gpurun_out/r06q.err || { rc=$?; tail -5 gpurun_out/r06q.err; exit $rc; }
  c3=null
  if [ -n "$C3" ]; then
    RAGMI_SMALL_RING=$r timeout -k 10 300 python -u bench.py --config 3 --diagnostic --no-cpu \
      > gpurun_out/r06q_c3.json 2>> gpurun_out/r06q.err || { rc=$?; tail -5 gpurun_out/r06q.err; exit $rc; }
    c3=$(python3 -c "import json; print(json.loads(open('gpurun_out/r06q_c3.json').read().strip().splitlines()[-1])['value'])")
  fi
  python3 -c "
import json
st=[json.loads(l) for l in open('gpurun_out/r06q_st.jsonl') if l.startswith('{')][0]
c2=json.loads(open('gpurun_out/r06q_c2.json').read().strip().splitlines()[-1])
print(json.dumps({'small_ring': $r, 'encode_q_ms': st['ms'], 'out_sha1': st.get('out_sha1'), 'config2_qps': c2['value'], 'config2_encode_max_abs_diff': c2.get('encode_max_abs_diff_vs_oracle'), 'exact': c2.get('search_top15_exact_queries'), 'config3_qps': $c3}))" | tee -a $out
done
