#!/bin/bash
# Small-shard (8-GPU shard size) bench at 1-4 batches in flight, plus the 2-rank gloo rehearsal.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for S in 1 2 3 4; do
  timeout -k 10 200 python bench.py --rows 1250000 --steps 200 --warmup 10 --no-cpu --streams $S > gpurun_out/bench_s$S.log 2>&1 || { rc=$?; tail -20 gpurun_out/bench_s$S.log; exit $rc; }
  grep '^{' gpurun_out/bench_s$S.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('streams', $S, d['value'], d['ms_per_step'], d['roofline']['avg_ms'], d['roofline']['step_frac'], d['recall_at_5'], d['top15_exact_vs_oracle'])"
done
RAGMI_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
   --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 3 --no-cpu \
   > gpurun_out/bench_2rank_gloo.log 2>&1 || { rc=$?; tail -30 gpurun_out/bench_2rank_gloo.log; exit $rc; }
grep '^{' gpurun_out/bench_2rank_gloo.log | cut -c1-400
