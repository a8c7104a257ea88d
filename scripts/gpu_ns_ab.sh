#!/bin/bash
# Build-time A/B of the query-batch GEMM ring depth (RAGMI_SMALL_NS, ab/libragmi_ns*.so built
# on the CPU side by ragmi/_build.py): SMALL GEMM parity per build, then encode_q and the
# config-2 line per build, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; out=gpurun_out/ns_ab.jsonl; : > $out
for v in ${BUILDS:-ns3 ns4 deep6 deep8}; do
  RAGMI_LIB_AB=$PWD/ab/libragmi_$v.so timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_gemm_exact_gpu.py -k "small or auto" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ns_t_$v.log 2>&1 || { tail -20 gpurun_out/ns_t_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/ns_t_$v.log)"
done
for rep in 1 2; do for v in ${BUILDS:-ns3 ns4 deep6 deep8}; do
  RAGMI_LIB_AB=$PWD/ab/libragmi_$v.so STAGES=encode_q PRECS=fp16x3 CPU=0 REPS=50 timeout -k 10 200 python -u scripts/bench_stages.py 2> gpurun_out/ns_st.err | grep '^{' | sed "s/^{/{\"build\": \"$v\", \"rep\": $rep, /" >> $out || { tail -20 gpurun_out/ns_st.err; exit 1; }
  RAGMI_LIB_AB=$PWD/ab/libragmi_$v.so timeout -k 10 300 python -u bench.py --config 2 --no-cpu --steps 50 2> gpurun_out/ns_c2.err | grep '^{' | sed "s/^{/{\"build\": \"$v\", \"rep\": $rep, \"line\": \"config2\", /" >> $out || { tail -20 gpurun_out/ns_c2.err; exit 1; }
done; done
python3 -c "
import json
for l in open('$out'):
    d=json.loads(l); print(d['build'], d['rep'], d.get('line', d.get('stage')), d.get('ms'), d.get('value'))"
