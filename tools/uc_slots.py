"""Config 5 (UC, path 4): per-PH-iteration solve time under different slot layouts of the
queue kernel, on one warm PH trajectory, plus the per-scenario PDHG iteration counts (for a
list-scheduling study of how many resident slots pay).

    python tools/uc_slots.py '<json list of {"PER_CU": k, "SPLIT": T, "SLOTS": B}>'

Iter0 is a cold solve (cap 100,000) and one warm continuation solve; PH iteration k then
runs with layout k mod len(list).  Writes gpurun_out/uc_slots.npz (iters [K, S], times).  UC_K: PH iterations (default: one per layout)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy-1_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from mpisppy_amd import _lib  # noqa: E402
from mpisppy_amd.engine import PHEngine  # noqa: E402
from mpisppy_amd.examples import uc  # noqa: E402

layouts = json.loads(sys.argv[1]) if len(sys.argv) > 1 else [{}]
S = int(os.environ.get("UC_S", "1000"))
b = uc.batch_creator(uc.scenario_names_creator(S), num_scens=1000)
e = PHEngine(b, device="cuda:0")


def env(lay):
    for k in ("PER_CU", "SPLIT", "SLOTS", "PAIR"):
        v = lay.get(k)
        name = "PHGPU_STREAM_" + k
        if v is None:
            os.environ.pop(name, None)
        else:
            os.environ[name] = str(v)


def solve(o, warm):
    torch.cuda.synchronize()
    t = time.time()
    e.solve(o, warm=warm)
    torch.cuda.synchronize()
    return time.time() - t


env({})
o = _lib.default_options(eps_rel=1e-6, max_iter=100000)
t0 = solve(o, False)
capped = int((e.host("status") != 0).sum())
print(json.dumps({"iter0_s": round(t0, 1), "capped": capped}), flush=True)
if capped:
    t1 = solve(_lib.default_options(eps_rel=1e-6, max_iter=100000, split_longest=min(capped, 16)), True)
    print(json.dumps({"continuation_s": round(t1, 1), "capped": int((e.host("status") != 0).sum())}), flush=True)
e.set_rho(1.0)
e.set_terms(1, 1)
K = int(os.environ.get("UC_K", str(len(layouts))))
its, times = [], []
for k in range(K):
    lay = layouts[k % len(layouts)]
    env(lay)
    e.compute_xbar()
    e.update(True)
    dt = solve(o, True)
    it = e.host("iters").copy()
    its.append(it)
    times.append(dt)
    st = e.host("status")
    print(json.dumps({"k": k + 1, "layout": lay, "solve_s": round(dt, 2), "mean": float(it.mean()), "max": int(it.max()),
                      "p99": float(np.percentile(it, 99)), "not_optimal": int((st != 0).sum())}), flush=True)
os.makedirs("gpurun_out", exist_ok=True)
np.savez("gpurun_out/uc_slots.npz", iters=np.array(its, dtype=np.int32), times=np.array(times),
         layouts=json.dumps(layouts))
e.close()
