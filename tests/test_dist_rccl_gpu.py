"""The multi-GPU exchange over RCCL itself on a one-GPU box: ragmi.dist's packed
all-gather through a world-1 torch.distributed "nccl" (= RCCL) process group, replayed over
S logical shards and merged on the GPU, equals the unsharded search bit for bit
(tests/_rccl_exchange.py; the gloo tests cover world 2 and 3 on CPU). Run in a child process so
the RCCL communicator lives and dies outside the pytest process."""
import json
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.gpu
@pytest.mark.parametrize("n,shards,k", [(200_000, 8, 15), (100_003, 3, 32), (40, 8, 15)])
def test_rccl_packed_exchange_equals_unsharded(gpu, n, shards, k):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, os.path.join(HERE, "_rccl_exchange.py"), str(n),
                        str(shards), str(k), "7"], capture_output=True, text=True, timeout=180,
                       env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["backend"] == "nccl" and out["world"] == 1
    assert out["ids_equal"] and out["scores_bitwise_equal"], out
