"""The PH step's rank sums through the library's own RCCL communicator (include/phgpu.h
phgpu_comm_init / phgpu_allreduce_sum, csrc/comm_rccl.inc) against the same sums through
torch.distributed's nccl backend: the engine's multi-rank path (x̄ reduce -> all-reduce ->
update, the conv all-reduce on the side stream) on the 8,192-scenario share with a loopback
communicator that reports 8 ranks over a one-rank RCCL group (tools/fake_ranks.py
``rccl-state``, in a subprocess so that this process's torch.distributed stays untouched).
The two runs issue the same collectives on the same streams, so the PH state after 8
iterations must agree bit for bit; the library's run must have used its communicator."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_rccl_matches_torch_distributed(gpu):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29541", HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "fake_ranks.py"), "8", "8", "rccl-state"],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("STATE ")][-1]
    out = json.loads(line[len("STATE "):])
    a, b = out["library"], out["torch"]
    assert a["native_rccl"] and not b["native_rccl"]
    assert a["calls"]["allreduce_xbar"] > 0 and a["calls"]["allreduce_conv_side"] > 0, a["calls"]
    assert a["conv"] == b["conv"], (a["conv"], b["conv"])
    assert np.array_equal(np.array(a["W"]), np.array(b["W"]))
    assert np.array_equal(np.array(a["xbar"]), np.array(b["xbar"]))
