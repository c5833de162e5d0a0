"""Per-scenario PDHG iteration counts of consecutive PH iterations (farmer, cm=1), for
the queue-order study: gpurun_out/iters_S<S>.npy [iterations, S]."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-sppy-1_amd"))
import numpy as np, torch
from mpisppy_amd.examples import farmer
from mpisppy_amd.engine import PHEngine
from mpisppy_amd import _lib

S = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
K = int(sys.argv[2]) if len(sys.argv) > 2 else 40
b = farmer.batch_creator(farmer.scenario_names_creator(S), crops_multiplier=1, num_scens=S)
e = PHEngine(b, device="cuda:0")
e.solve(_lib.default_options(eps_rel=1e-10), warm=False)
e.set_rho(1.0); e.set_terms(1, 1)
o = _lib.default_options()
out = []
for k in range(K):
    e.compute_xbar(); e.update(True)
    e.solve(o, warm=True)
    out.append(e.host("iters").copy())
os.makedirs("gpurun_out", exist_ok=True)
np.save(f"gpurun_out/iters_S{S}.npy", np.array(out, dtype=np.int32))
print("saved", len(out), "iterations; mean per iteration", [int(a.mean()) for a in out])
