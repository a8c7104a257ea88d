#!/bin/bash
# round 6: fused FFN parity (bitwise vs the two-kernel forward) then its timing A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -p no:cacheprovider --timeout 240 --timeout-method thread \
    tests/test_ffn_fused_gpu.py -m gpu > gpurun_out/r06d_pytest.log 2>&1
rc=$?
tail -4 gpurun_out/r06d_pytest.log; echo "pytest rc=$rc"
grep -E "max \|" gpurun_out/r06d_pytest.log | head -20
if [ $rc -ne 0 ]; then grep -E "^(FAILED|E  )" gpurun_out/r06d_pytest.log | head -30; exit $rc; fi
for rep in 1 2; do
  STAGES=rerank PRECS=fp16x3 CPU=0 REPS=10 FFNS=0,1 timeout -k 10 200 python -u scripts/bench_stages.py \
      >> gpurun_out/r06d_stages.jsonl 2> gpurun_out/r06d_stages.err || { rc=$?; tail -5 gpurun_out/r06d_stages.err; exit $rc; }
done
cat gpurun_out/r06d_stages.jsonl
