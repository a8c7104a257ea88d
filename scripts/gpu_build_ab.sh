#!/bin/bash
# same-box A/B of two builds (ab/libragmi_old.so / _new.so via RAGMI_LIB_AB): GEMM + encoder
# suites on the in-tree build, encoder stages, then the config-2 line per build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gemm_gpu.py tests/test_gemm_exact_gpu.py tests/test_encoders_gpu.py} -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
STAGES=${STAGES:-encode_q,encode_c} TAG=${TAG:-build} bash scripts/gpu_ab.sh || exit 1
out=gpurun_out/build_ab_c2.jsonl; : > $out
for rep in 1 2; do for v in old new; do
  RAGMI_LIB_AB=$PWD/ab/libragmi_$v.so timeout -k 10 300 python -u bench.py --config ${CONFIG:-2} --no-cpu 2> gpurun_out/c2.err | grep '^{' | sed "s/^{/{\"build\": \"$v\", \"rep\": $rep, /" >> $out || { tail -20 gpurun_out/c2.err; exit 1; }
done; done
python3 -c "
import json
for l in open('$out'):
    d=json.loads(l); print(d['build'], d['rep'], d['value'], d.get('id_input_qps'))"
