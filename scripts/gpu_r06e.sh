#!/bin/bash
# round 6: fused FFN timing probes (diagnostic builds under ab/), a kernel trace of the fused
# forward, then the in-process config-2 leg diagnosis
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/r06e_probes.jsonl
timeout -k 10 300 python -u -m pytest -x -v -p no:cacheprovider --timeout 240 --timeout-method thread \
    tests/test_ffn_fused_gpu.py -m gpu > gpurun_out/r06e_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r06e_pytest.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|E  )" gpurun_out/r06e_pytest.log | head -20; exit $rc; fi
for lib in prod; do
  if [ "$lib" = prod ]; then unset RAGMI_LIB_AB; else export RAGMI_LIB_AB=$PWD/$lib; fi
  STAGES=rerank PRECS=fp16x3 CPU=0 REPS=10 FFNS=0,2,3,4,5 timeout -k 10 200 python -u scripts/bench_stages.py \
      > gpurun_out/r06e_tmp.jsonl 2> gpurun_out/r06e_probes.err || { rc=$?; tail -5 gpurun_out/r06e_probes.err; exit $rc; }
  sed "s|^{|{\"lib\": \"$lib\", |" gpurun_out/r06e_tmp.jsonl >> gpurun_out/r06e_probes.jsonl
done
unset RAGMI_LIB_AB
cat gpurun_out/r06e_probes.jsonl | cut -c1-200
STAGES=rerank PRECS=fp16x3 CPU=0 REPS=3 FFNS=2 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/r06e_trace -o t -- python3 scripts/bench_stages.py > gpurun_out/r06e_trace.log 2>&1 \
    || { rc=$?; tail -5 gpurun_out/r06e_trace.log; exit $rc; }
f=$(find gpurun_out/r06e_trace -name "*kernel_stats.csv" | head -1); head -12 "$f" | cut -c1-160
exit 0
    || { rc=$?; tail -5 gpurun_out/r06e_inproc.err; exit $rc; }
cat gpurun_out/r06e_inproc.jsonl
