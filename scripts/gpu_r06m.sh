#!/bin/bash
# round 6: gemm_ws_kernel stagger A/B (RAGMI_WS_STAGGER, odd workgroups run their half tile
# first): rerank + chunk encode forward times and output digests, alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/r06m_stagger_ab.jsonl
rm -f $out
for s in 0 1 0 1 0 1; do
  RAGMI_WS_STAGGER=$s STAGES=rerank,encode_c PRECS=fp16x3 CPU=0 REPS=30 SAVE_OUT=1 \
    timeout -k 10 300 python -u scripts/bench_stages.py > gpurun_out/r06m_s$s.jsonl 2> gpurun_out/r06m.err \
    || { rc=$?; tail -5 gpurun_out/r06m.err; exit $rc; }
  python3 -c "
import json
for l in open('gpurun_out/r06m_s$s.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); d['stagger']=$s; print(json.dumps(d))" | tee -a $out
done
