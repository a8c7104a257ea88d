#!/bin/bash
# round 6: encoder forward PMC (item 5), config 5 per-rank shard certified (item 2), full-pass cost
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_encoder_pmc.sh || exit $?
timeout -k 10 300 python -u scripts/diag/full_pass_timing.py > gpurun_out/r06b_full_pass.jsonl 2> gpurun_out/r06b_full_pass.err \
    || { rc=$?; tail -5 gpurun_out/r06b_full_pass.err; exit $rc; }
cat gpurun_out/r06b_full_pass.jsonl
timeout -k 10 600 python -u bench.py --config 5 --rows 6250000 --certify > gpurun_out/r06b_config5_rank.jsonl 2> gpurun_out/r06b_config5_rank.err \
    || { rc=$?; tail -5 gpurun_out/r06b_config5_rank.err; exit $rc; }
cat gpurun_out/r06b_config5_rank.jsonl
