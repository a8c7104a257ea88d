#!/bin/bash
# round 6: (1) the bge head fused into the last LayerNorm (new in-tree build) vs the previous
# build (ab/prev.so): encode_q output digest + time, config 2 alternating; (2) dispatch-cost
# probe: n empty kernels per forward (diagnostic build, RAGMI_PROBE_EXTRA)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/r06ab.jsonl
rm -f $out
one() {   # label lib extra
  RAGMI_LIB_AB=$2 RAGMI_PROBE_EXTRA=$3 STAGES=encode_q PRECS=fp16x3 CPU=0 REPS=50 SAVE_OUT=1 \
    timeout -k 10 200 python -u scripts/bench_stages.py > gpurun_out/r06ab_st.jsonl 2> gpurun_out/r06ab.err || return $?
  RAGMI_LIB_AB=$2 RAGMI_PROBE_EXTRA=$3 timeout -k 10 300 python -u bench.py --config 2 --no-cpu \
    > gpurun_out/r06ab_c2.json 2>> gpurun_out/r06ab.err || return $?
  python3 -c "
import json
st=[json.loads(l) for l in open('gpurun_out/r06ab_st.jsonl') if l.startswith('{')][0]
c2=json.loads(open('gpurun_out/r06ab_c2.json').read().strip().splitlines()[-1])
print(json.dumps({'label': '$1', 'extra': $3, 'encode_q_ms': st['ms'], 'out_sha1': st.get('out_sha1'), 'config2_qps': c2['value'], 'encode_diff': c2.get('encode_max_abs_diff_vs_oracle'), 'exact': c2.get('search_top15_exact_queries')}))" | tee -a $out
}
P=$PWD
for r in 1 2; do
  one fused "" 0 || { rc=$?; tail -5 gpurun_out/r06ab.err; exit $rc; }
  one prev $P/ab/prev.so 0 || { rc=$?; tail -5 gpurun_out/r06ab.err; exit $rc; }
done
for n in 0 24 0 24; do
  one diag_extra $P/ab/diag.so $n || { rc=$?; tail -5 gpurun_out/r06ab.err; exit $rc; }
done
