#!/bin/bash
# wave grid of the query-batch GEMM tiles (A/B builds ab/libragmi_w{22,21,12,11}.so): SMALL
# parity per build, then the K sweep, encode_q and the config-2 line per build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B="${BUILDS:-w22 w21 w12 w11}"
for v in $B; do
  RAGMI_LIB_AB=$PWD/ab/libragmi_$v.so timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_gemm_exact_gpu.py -k "small or auto" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/w_t_$v.log 2>&1 || { tail -30 gpurun_out/w_t_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/w_t_$v.log)"
done
out=gpurun_out/wave_ab.jsonl; : > $out
for rep in 1 2; do for v in $B; do
  RAGMI_LIB_AB=$PWD/ab/libragmi_$v.so SWEEP_K=384,1536 timeout -k 10 200 python3 -u scripts/diag/small_gemm_sweep.py >> $out 2> gpurun_out/wa.err || { tail -20 gpurun_out/wa.err; exit 1; }
  RAGMI_LIB_AB=$PWD/ab/libragmi_$v.so STAGES=encode_q PRECS=fp16x3 CPU=0 REPS=50 timeout -k 10 200 python -u scripts/bench_stages.py 2> gpurun_out/wa.err | grep '^{' | sed "s/^{/{\"lib\": \"$v\", /" >> $out || { tail -20 gpurun_out/wa.err; exit 1; }
  RAGMI_LIB_AB=$PWD/ab/libragmi_$v.so timeout -k 10 300 python -u bench.py --config 2 --no-cpu 2> gpurun_out/wa.err | grep '^{' | sed "s/^{/{\"lib\": \"$v\", \"line\": \"config2\", /" >> $out || { tail -20 gpurun_out/wa.err; exit 1; }
done; done
python3 -c "
import json
for l in open('$out'):
    d=json.loads(l); print(d.get('lib'), d.get('kind', d.get('line', d.get('stage'))), d.get('N'), d.get('K'), d.get('us', d.get('ms')), d.get('value'), d.get('id_input_qps'))"
