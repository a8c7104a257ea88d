#!/bin/bash
# round 6: is config 2 bound by its dispatch count? n empty kernels added per encoder forward
# (diagnostic build, RAGMI_PROBE_EXTRA=n) against the config-2 rate
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export RAGMI_LIB_AB=$PWD/ab/diag.so
out=gpurun_out/r06aa_extra_launches.jsonl
rm -f $out
for n in ${SPECS:-0 10 0 10 20 0}; do
  RAGMI_PROBE_EXTRA=$n timeout -k 10 300 python -u bench.py --config 2 --no-cpu > gpurun_out/r06aa_c2.json 2> gpurun_out/r06aa.err \
    || { rc=$?; tail -5 gpurun_out/r06aa.err; exit $rc; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r06aa_c2.json').read().strip().splitlines()[-1])
print(json.dumps({'extra_launches': $n, 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'enc_ms': d['roofline']['avg_ms']}))" | tee -a $out
done
