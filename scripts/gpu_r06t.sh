#!/bin/bash
# (the --front-cus option was removed after this A/B: negative)
# round 6: config 3 with a front / back CU split (--front-cus; CU-mask bit i is on XCD i % 8,
# profiles/r06_cu_mask/r06s_cu_mask_probe.jsonl, so "interleaved" takes an equal share of
# every XCD)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/r06t_front_back.jsonl
rm -f $out
for spec in ${SPECS:-"0 interleaved" "16 interleaved" "32 interleaved" "0 interleaved"}; do
  set -- $spec
  timeout -k 10 300 python -u bench.py --config 3 --front-cus $1 --cu-layout $2 --no-cpu > gpurun_out/r06t_c3.json 2> gpurun_out/r06t.err \
    || { rc=$?; tail -5 gpurun_out/r06t.err; exit $rc; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r06t_c3.json').read().strip().splitlines()[-1])
print(json.dumps({'front_cus': $1, 'layout': '$2', 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'split': d['config'].get('front_back_cus'), 'rerank_diff': d.get('rerank_max_abs_diff_vs_oracle'), 'top5': d.get('rerank_top5_order_matches'), 'exact': d.get('search_top15_exact_queries'), 'fwd_ms': d['roofline'].get('standalone_avg_ms')}))" | tee -a $out
done
