#!/bin/bash
# where a query-batch GEMM K step goes: the SMALL kernel with its MFMAs / DMAs removed
# (A/B builds ab/libragmi_p{0..3}.so, RAGMI_PIPE_PROBE), device time over K at M = 782
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; out=gpurun_out/small_probe.jsonl; : > $out
for rep in 1 2; do for p in 0 1 2 3; do
  RAGMI_LIB_AB=$PWD/ab/libragmi_p$p.so SWEEP_K=64,384,768,1536 timeout -k 10 200 python3 -u scripts/diag/small_gemm_sweep.py >> $out 2> gpurun_out/sp.err || { tail -20 gpurun_out/sp.err; exit 1; }
done; done
python3 -c "
import json,collections
d=collections.defaultdict(list)
for l in open('$out'):
    r=json.loads(l); d[(r['kind'],r['N'],r['K'],r['lib'])].append(r['us'])
for k,v in sorted(d.items()): print(k, v)"
