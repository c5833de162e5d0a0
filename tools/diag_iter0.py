"""GPU diagnostic: Iter0 PDHG iteration distribution on farmer scenarios."""
import sys, os, json
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-sppy-1_amd"))
import numpy as np, torch
from mpisppy_amd.examples import farmer
from mpisppy_amd.engine import PHEngine
from mpisppy_amd import _lib
S = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
names = farmer.scenario_names_creator(S)
b = farmer.batch_creator(names, num_scens=S)
e = PHEngine(b, device="cuda:0")
for mi in [20000]:
    o = _lib.default_options(max_iter=mi)
    e.solve(o, warm=False)
    it = e.host("iters"); st = e.host("status")
    print("max", it.max(), "mean", it.mean(), "p99", np.percentile(it, 99), "fail", (st != 0).sum(),
          "fail idx", np.nonzero(st != 0)[0][:20].tolist(), flush=True)
    x = e.host("x")
    for s in np.nonzero(st != 0)[0][:3]:
        print(names[s], x[s, :3], e.host("obj")[s], e.host("bound")[s])
