#!/bin/bash
# round 6: headline vs the tier-2 rescan grid (RAGMI_RESCAN_WG on a diagnostic handle): the
# idle rescan launch after every select waits for CUs beside the other batch's scan
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/r06af_rescan_grid.jsonl
rm -f $out
for g in ${SPECS:-256 64 128 256 64 128}; do
  RAGMI_RESCAN_WG=$g timeout -k 10 300 python -u bench.py --no-configs --no-cpu --diagnostic > gpurun_out/r06af_b.json 2> gpurun_out/r06af.err \
    || { rc=$?; tail -5 gpurun_out/r06af.err; exit $rc; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r06af_b.json').read().strip().splitlines()[-1])
print(json.dumps({'rescan_wg': $g, 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'frac': d['roofline']['frac'], 'exact': d['exact_batches']}))" | tee -a $out
done
