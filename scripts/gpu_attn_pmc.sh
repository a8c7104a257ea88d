#!/bin/bash
# PMC passes over the encoder attention kernel in the config-3 rerank forward (480 pairs,
# ~117K tokens, fp16x3 unless PREC is set): wave time split, instruction mix, LDS conflicts.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/apmc*
j=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
            "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE" \
            "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE GRBM_GUI_ACTIVE"; do
  j=$((j+1))
  PREC=${PREC:-fp16x3} REPS=2 timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d "$R/gpurun_out/apmc$j" -o p \
      -- python3 "$R/scripts/enc_probe.py" > gpurun_out/apmc$j.log 2>&1 \
      || { rc=$?; echo "pass $j rc=$rc"; tail -5 gpurun_out/apmc$j.log; exit $rc; }
done
python3 - <<'PY'
import csv, glob, collections, json
acc = collections.defaultdict(list)
for f in glob.glob("gpurun_out/apmc*/**/p_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "attn_kernel" not in r["Kernel_Name"]: continue
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {c: sum(v) / len(v) for c, v in acc.items()}
json.dump(res, open("gpurun_out/attn_pmc.json", "w"), indent=1, sort_keys=True)
print({c: f"{v:.4g}" for c, v in sorted(res.items())})
PY
