#!/bin/bash
# Counter passes over the encoder kernels (config-3 rerank forward): SQ issue/stall breakdown,
# MFMA busy, LDS bank conflicts; then HBM bytes (FETCH_SIZE / WRITE_SIZE in separate passes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/enc_pmc*
PREC=${PREC:-fp16} timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES \
   --output-format csv -d "$R/gpurun_out/enc_pmc1" -o p -- python3 "$R/scripts/enc_probe.py" > gpurun_out/enc_pmc1.log 2>&1 || { tail -20 gpurun_out/enc_pmc1.log; exit 1; }
PREC=${PREC:-fp16} timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/enc_pmc2" -o p -- python3 "$R/scripts/enc_probe.py" > gpurun_out/enc_pmc2.log 2>&1 || { tail -20 gpurun_out/enc_pmc2.log; exit 1; }
PREC=${PREC:-fp16} timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/enc_pmc3" -o p -- python3 "$R/scripts/enc_probe.py" > gpurun_out/enc_pmc3.log 2>&1 || { tail -20 gpurun_out/enc_pmc3.log; exit 1; }
PREC=${PREC:-fp16} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/enc_pmc4" -o p -- python3 "$R/scripts/enc_probe.py" > gpurun_out/enc_pmc4.log 2>&1 || { tail -20 gpurun_out/enc_pmc4.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(int)
for d in ("enc_pmc1", "enc_pmc2", "enc_pmc3"):
    f = glob.glob(f"gpurun_out/{d}/**/*counter_collection.csv", recursive=True)[0]
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][:60]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        if d == "enc_pmc1" and r["Counter_Name"] == "SQ_WAVE_CYCLES":
            cnt[k] += 1
f = glob.glob("gpurun_out/enc_pmc4/**/*kernel_stats.csv", recursive=True)[0]
dur = {r["Name"].split("(")[0][:60]: (float(r["TotalDurationNs"]), int(r["Calls"])) for r in csv.DictReader(open(f))}
for k, v in sorted(agg.items(), key=lambda kv: -dur.get(kv[0], (0, 1))[0])[:8]:
    w = v["SQ_WAVE_CYCLES"] or 1
    tot, n = dur.get(k, (0, 1))
    print(f"{k:60s} n={n:4d} avg_us={tot/n/1e3:8.1f} waitany={v['SQ_WAIT_ANY']/w:.2f} "
          f"waitinst={v['SQ_WAIT_INST_ANY']/w:.2f} active={v['SQ_ACTIVE_INST_ANY']/w:.2f} "
          f"ldswait={v['SQ_WAIT_INST_LDS']/w:.2f} mfma_busy/busy={v['SQ_VALU_MFMA_BUSY_CYCLES']/max(v['SQ_BUSY_CYCLES'],1):.3f} "
          f"ldsconf={v['SQ_LDS_BANK_CONFLICT']:.3g} fetchMB/call={v['FETCH_SIZE']*2/1024/max(n,1):.1f} "
          f"writeMB/call={v['WRITE_SIZE']/1024/max(n,1):.1f}")
PY
