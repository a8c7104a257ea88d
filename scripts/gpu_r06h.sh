#!/bin/bash
# round 6: the fused FFN's bitwise suite against the diagnostic build, then the in-process
# config-2 leg diagnosis with whole-CU-mask (dedicated queue) streams
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
RAGMI_LIB_AB=$PWD/ab/diag.so RAGMI_TEST_DIAG_BUILD=1 timeout -k 10 300 python -u -m pytest -x -v -p no:cacheprovider \
    --timeout 240 --timeout-method thread tests/test_ffn_fused_gpu.py tests/test_attention_gpu.py -m gpu \
    > gpurun_out/r06h_diag_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r06h_diag_pytest.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|E  )" gpurun_out/r06h_diag_pytest.log | head -20; exit $rc; fi
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 240 --timeout-method thread \
    tests/test_ffn_fused_gpu.py tests/test_attention_gpu.py -m gpu > gpurun_out/r06h_prod_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r06h_prod_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u scripts/diag/inproc_legs.py > gpurun_out/r06h_inproc.jsonl 2> gpurun_out/r06h_inproc.err \
    || { rc=$?; tail -5 gpurun_out/r06h_inproc.err; exit $rc; }
cat gpurun_out/r06h_inproc.jsonl
