#!/bin/bash
# A/B of an environment knob on the encoder stage bench, interleaved runs in separate
# processes: ENVS="RAGMI_KSPLIT=1 RAGMI_KSPLIT=0" STAGES=encode_q PRECS=fp16x3 bash scripts/gpu_ab_env.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/ab_env.jsonl
: > $out
for rep in 1 2; do
  for e in $ENVS; do
    env $e CPU=0 REPS=${REPS:-50} timeout -k 10 300 python3 scripts/bench_stages.py 2> gpurun_out/ab_env.err \
      | sed "s/^{/{\"env\": \"$e\", \"rep\": $rep, /" >> $out || { tail -20 gpurun_out/ab_env.err; exit 1; }
  done
done
cat $out
