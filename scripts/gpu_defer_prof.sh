#!/bin/bash
# per-kernel rerank breakdown (fp16x3, 117K tokens) with the deferred LayerNorm on and off
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; TAG=${TAG:-r02l}
mkdir -p gpurun_out/profiles
cd /tmp && export TMPDIR=/tmp
for d in ${DEFERS:--1 0}; do
  STAGES=rerank PRECS=fp16x3 DEFERS=$d CPU=0 REPS=10 timeout -k 10 300 rocprofv3 --kernel-trace --stats \
      --output-format csv -d $R/gpurun_out/prof_dl$d -o st -- python3 $R/scripts/bench_stages.py \
      > $R/gpurun_out/prof_dl$d.log 2>&1 || exit $?
  f=$(find $R/gpurun_out/prof_dl$d -name "*kernel_stats.csv" | head -1)
  cp "$f" $R/gpurun_out/profiles/${TAG}_rerank_defer${d}_kernel_stats.csv
  echo "== defer $d"; grep stage $R/gpurun_out/prof_dl$d.log
  cut -d, -f1-5 "$f" | cut -c1-160 | head -16
done
