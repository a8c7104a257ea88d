#!/bin/bash
# PMC passes over the 117K-token fp16x3 encoder GEMMs as the forward runs them (AUTO = the
# loader-specialised WS kernel): HBM bytes (FETCH_SIZE, WRITE_SIZE) and MFMA busy cycles,
# one process per shape, each counter group in its own pass (MI355X_MICROARCH.md HBM section).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/wpmc*
# name M N K epi
SHAPES="qkv:117000:1152:384:0 o:117000:384:384:2 ffn1:117000:1536:384:1 ffn2:117000:384:1536:2"
for sh in $SHAPES; do
  IFS=: read name M N K epi <<< "$sh"
  j=0
  for ctrs in "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE GRBM_GUI_ACTIVE" \
              "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAVES GRBM_GUI_ACTIVE"; do
    j=$((j+1))
    timeout -s KILL 90 rocprofv3 --pmc $ctrs --output-format csv -d "$R/gpurun_out/wpmc_${name}_$j" -o p \
        -- python3 "$R/scripts/gemm_one.py" $M $N $K $epi fp16x3 ${VARIANT:-0} 10 > gpurun_out/wpmc_${name}_$j.log 2>&1 \
        || { rc=$?; echo "$name pass $j rc=$rc"; tail -5 gpurun_out/wpmc_${name}_$j.log; exit $rc; }
  done
done
python3 - <<'PY'
import csv, glob, collections, json
res = {}
for d in sorted(glob.glob("gpurun_out/wpmc_*")):
    if not d.endswith(tuple("123")) or "." in d.split("/")[-1]: continue
    name = d.split("wpmc_")[1].rsplit("_", 1)[0]
    for f in glob.glob(d + "/**/p_counter_collection.csv", recursive=True):
        acc = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            if "gemm_ws_kernel" not in r["Kernel_Name"]: continue
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
        for c, v in acc.items():
            res.setdefault(name, {})[c] = sum(v) / len(v)
json.dump(res, open("gpurun_out/gemm_ws_pmc.json", "w"), indent=1, sort_keys=True)
for k, d in res.items():
    print(k, {c: f"{v:.4g}" for c, v in sorted(d.items())})
PY
