#!/bin/bash
# PMC passes over the 117K-token fp16x3 encoder GEMMs (PIPE / WIDE variants)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/gpmc*
i=0
for ctrs in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
            "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE" \
            "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  GEMM_M=117000 GEMM_VARIANTS=2 timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d "$R/gpurun_out/gpmc$i" -o p \
      -- python3 "$R/scripts/bench_gemm.py" > gpurun_out/gpmc$i.log 2>&1 || { rc=$?; echo "pass $i rc=$rc"; tail -5 gpurun_out/gpmc$i.log; }
done
python3 - <<'PY'
import csv, glob, collections, json
out = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/gpmc*/**/p_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "gemm_pipe" not in k: continue
        key = k.split("(")[0][25:110] + " grid=" + r["Grid_Size"]
        out[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in out.items()}
json.dump(res, open("gpurun_out/gemm_pmc3.json", "w"), indent=1)
for k, d in res.items():
    print(k)
    print("   ", {c: f"{v:.3g}" for c, v in sorted(d.items())})
PY
