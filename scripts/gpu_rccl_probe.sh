#!/bin/bash
# what slows the 1.25M-row search once an RCCL communicator exists (scripts/rccl_exchange_probe.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; o=gpurun_out/rccl_probe3.jsonl; : > $o
P="timeout -k 10 300 python3 -u scripts/rccl_exchange_probe.py"
NO_PG=1 MODES=plain $P 2>/dev/null | grep '^{' >> $o || exit 1
MODES=plain,pg $P 2>/dev/null | grep '^{' >> $o || exit 1
PG_MODE=lazy MODES=plain,pg $P 2>/dev/null | grep '^{' >> $o || exit 1
PG_MODE=late MODES=plain,pg $P 2>/dev/null | grep '^{' >> $o || exit 1
PROBE_ENV_LABEL=msccl_off RCCL_MSCCL_ENABLE=0 RCCL_MSCCLPP_ENABLE=0 MODES=plain,pg $P 2>/dev/null | grep '^{' >> $o || exit 1
PROBE_ENV_LABEL=no_watchdog TORCH_NCCL_ENABLE_MONITORING=0 TORCH_NCCL_ASYNC_ERROR_HANDLING=0 MODES=plain,pg $P 2>/dev/null | grep '^{' >> $o || exit 1
python3 -c "
import json
for l in open('$o'):
    d=json.loads(l); print(d['mode'], d['rep'], d['pg'], d['env'], d['qps'], d['host_enqueue_us_per_step'])"
