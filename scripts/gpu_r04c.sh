#!/bin/bash
# round 4: FETCH_SIZE passes for the config-5 wide scan (N = 8 shard 6.25M x 1024 and the
# 1-GPU 50M x 1024) and the filtered 10M scan, merged into scan_pmc.json (bench `traffic`)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp; mkdir -p gpurun_out/profiles
export PROFILES_DIR=gpurun_out/profiles COMMIT=${COMMIT:-r04}
cp profiles/scan_pmc.json gpurun_out/profiles/scan_pmc.json
pass() {  # tag kind rows kernel algo -- bench args
  local tag=$1 kind=$2 rows=$3 kern=$4 algo=$5; shift 5
  rm -rf gpurun_out/pmc_$tag
  timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_$tag" -o pmc \
    -- python3 "$R/bench.py" "$@" > gpurun_out/pmc_$tag.log 2>&1 || { tail -20 gpurun_out/pmc_$tag.log; return 1; }
  python3 scripts/pmc_table.py $kind $rows gpurun_out/pmc_$tag "$kern" $tag $algo
}
pass r04c_wide6p25M wide_1024 6250000 scan_wide_kernel 12800000000 --config 5 --rows 6250000 --steps 4 --warmup 1 --no-cpu --no-recall \
&& pass r04c_filtered10M filtered_384 10000000 scan_kernel 7720000000 --config filtered --steps 4 --warmup 1 --no-cpu --no-recall \
&& pass r04c_wide50M wide_1024 50000000 scan_wide_kernel 102400000000 --config 5 --steps 3 --warmup 1 --no-cpu --no-recall
