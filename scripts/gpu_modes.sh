#!/bin/bash
# bench.py --config lines (configs 3, filtered, 5, 2); MODES / STEPS override
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for m in ${MODES:-3 filtered 5}; do
  T0=$(date +%s)
  timeout -k 10 400 python -u bench.py --config $m --steps ${STEPS:-20} --warmup 3 \
      > gpurun_out/mode_${m}.log 2> gpurun_out/mode_${m}.err \
      || { rc=$?; echo "config $m rc=$rc"; tail -20 gpurun_out/mode_${m}.err; exit $rc; }
  echo "config $m wall $(( $(date +%s) - T0 )) s"
  tail -1 gpurun_out/mode_${m}.log
done
