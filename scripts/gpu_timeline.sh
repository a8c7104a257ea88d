cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$PWD/gpurun_out/tl" -o tl -- python3 bench.py --rows 1250000 --steps 30 --warmup 3 --no-recall --no-cpu > gpurun_out/tl.log 2>&1 || { tail -5 gpurun_out/tl.log; exit 1; }
tail -1 gpurun_out/tl.log
python3 scripts/timeline.py $(find gpurun_out/tl -name "*kernel_trace.csv" | head -1)
