#!/bin/bash
# deferred LayerNorm forward A/B: off, auto, and the A-stream nt probes (RAGMI_DL_PROBE)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/profiles; TAG=${TAG:-r02n}
out=gpurun_out/profiles/${TAG}_defer_probe.jsonl; : > $out
for p in 0 1 2 3; do
  RAGMI_DL_PROBE=$p STAGES=rerank PRECS=fp16x3 DEFERS=0,-1,0,-1 CPU=0 REPS=20 timeout -k 10 200 \
      python -u scripts/bench_stages.py | sed "s/^{/{\"dl_probe\": $p, /" >> $out || exit $?
done
cut -c1-20,90-140 $out
