#!/bin/bash
# same-box A/B of two builds (ab/libragmi_old.so vs ab/libragmi_new.so, RAGMI_LIB_AB) on the
# encoder stages, alternating, so box-to-box clock differences cancel
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/profiles; out=gpurun_out/profiles/${TAG:-ab}_ab.jsonl; : > $out
for rep in 1 2; do for v in old new; do
  RAGMI_LIB_AB=$PWD/ab/libragmi_$v.so STAGES=${STAGES:-rerank,encode_c} PRECS=${PRECS:-fp16x3} CPU=0 REPS=20 \
      timeout -k 10 200 python -u scripts/bench_stages.py | sed "s/^{/{\"build\": \"$v\", /" >> $out || exit $?
done; done
python3 -c "
import json,collections
d=collections.defaultdict(list)
for l in open('$out'):
    r=json.loads(l); d[(r['stage'],r['precision'],r['build'])].append(r['ms'])
for k,v in sorted(d.items()): print(k, v)
"
