#!/bin/bash
# round 6: PMC of the fused FFN vs the WS GEMMs (one rerank stage process with FFNS=0,2)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/r06f_*
j=0
for ctrs in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" \
            "SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE" \
            "FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE"; do
  j=$((j+1))
  STAGES=rerank PRECS=fp16x3 CPU=0 REPS=2 FFNS=0,2 timeout -s KILL 240 rocprofv3 --pmc $ctrs --output-format csv \
      -d "$PWD/gpurun_out/r06f_$j" -o p -- python3 scripts/bench_stages.py > gpurun_out/r06f_$j.log 2>&1 \
      || { rc=$?; echo "pass $j rc=$rc"; tail -5 gpurun_out/r06f_$j.log; exit $rc; }
done
python3 - <<'PY'
import csv, glob, collections, json
for j in (1, 2, 3):
    f = glob.glob(f"gpurun_out/r06f_{j}/**/*counter_collection.csv", recursive=True)[0]
    disp = collections.OrderedDict()
    for r in csv.DictReader(open(f)):
        k = int(r["Dispatch_Id"]); e = disp.setdefault(k, {"name": r["Kernel_Name"]})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for e in disp.values():
        n = e["name"]
        key = ("ffn_fused" if "ffn_fused" in n else "ws_epi" + n.split("gemm_ws_kernelILi")[1][0]
               if "gemm_ws_kernel" in n else "attn" if "attn_kernel" in n else None)
        if key:
            for c, v in e.items():
                if c != "name": agg[key][c].append(v)
    out = {k: {c: sorted(v)[len(v) // 2] for c, v in d.items()} for k, d in agg.items()}
    print(json.dumps({"pass": j, **out}))
PY
