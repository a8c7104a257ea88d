#!/bin/bash
# round 6: the new / changed GPU tests (full exact pass, 1M x 1024 B=128, production attention
# variants, partition streams), then smoke
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 240 --timeout-method thread \
    tests/test_large_k_gpu.py tests/test_attention_gpu.py tests/test_partition_gpu.py \
    "tests/test_scan_gpu.py::test_d1024_million_rows_batch128" tests/test_rag_gpu.py \
    -m gpu > gpurun_out/r06a_pytest.log 2>&1
rc=$?
tail -4 gpurun_out/r06a_pytest.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then grep -E "^(FAILED|E  )" gpurun_out/r06a_pytest.log | head -30; exit $rc; fi
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
