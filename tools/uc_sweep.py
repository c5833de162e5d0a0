"""PDHG option sweep on UC scenarios (path 4): iterations / time of a cold solve."""
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

S = int(sys.argv[1]) if len(sys.argv) > 1 else 64
configs = [json.loads(a) for a in sys.argv[2:]] or [{}]
b = uc.batch_creator(uc.scenario_names_creator(S), num_scens=1000)
e = PHEngine(b, device="cuda:0")
for cfg in configs:
    o = {"eps_rel": 1e-6, "max_iter": 100000}
    o.update(cfg)
    torch.cuda.synchronize()
    t = time.time()
    e.solve(_lib.default_options(**o), warm=False)
    torch.cuda.synchronize()
    dt = time.time() - t
    it = e.host("iters")
    st = e.host("status")
    print(json.dumps({"cfg": cfg, "time_s": round(dt, 2), "iters_mean": float(it.mean()), "iters_max": int(it.max()),
                      "iters_p90": float(np.percentile(it, 90)), "not_optimal": int((st != 0).sum())}), flush=True)
