#!/bin/bash
# round 6: fused FFN A/B shapes (chunk 256, mid-step DMA, setprio) against the two-kernel FFN
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rm -f gpurun_out/r06g_ab.jsonl
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 240 --timeout-method thread \
    tests/test_ffn_fused_gpu.py -m gpu > gpurun_out/r06g_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r06g_pytest.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|E  )" gpurun_out/r06g_pytest.log | head -20; exit $rc; fi
for rep in 1 2; do
  STAGES=rerank PRECS=fp16x3 CPU=0 REPS=10 FFNS=0,2,3,4,5 timeout -k 10 200 python -u scripts/bench_stages.py \
      >> gpurun_out/r06g_ab.jsonl 2> gpurun_out/r06g_ab.err || { rc=$?; tail -5 gpurun_out/r06g_ab.err; exit $rc; }
done
python3 -c "
import json
for l in open('gpurun_out/r06g_ab.jsonl'):
    d=json.loads(l); print(d['ffn_fused'], d['ms'])"
