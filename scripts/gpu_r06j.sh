#!/bin/bash
# round 6: WS GEMM priority A/B (rerank forward + chunk encode), interleaved, 3 rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rm -f gpurun_out/r06j_prio.jsonl
for rep in 1 2 3; do
  for lib in prod ab/wsprio1.so ab/wsprio2.so; do
    if [ "$lib" = prod ]; then unset RAGMI_LIB_AB; else export RAGMI_LIB_AB=$PWD/$lib; fi
    STAGES=rerank,encode_c PRECS=fp16x3 CPU=0 REPS=10 timeout -k 10 200 python -u scripts/bench_stages.py \
        > gpurun_out/r06j_tmp.jsonl 2> gpurun_out/r06j.err || { rc=$?; tail -5 gpurun_out/r06j.err; exit $rc; }
    sed "s|^{|{\"lib\": \"$lib\", \"rep\": $rep, |" gpurun_out/r06j_tmp.jsonl >> gpurun_out/r06j_prio.jsonl
  done
done
unset RAGMI_LIB_AB
python3 -c "
import json
for l in open('gpurun_out/r06j_prio.jsonl'):
    d=json.loads(l); print(d['lib'], d['rep'], d['stage'], d['ms'])"
