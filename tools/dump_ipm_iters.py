"""Per-scenario interior-point iteration counts of consecutive PH iterations on path 6
(farmer cm = 1 by default; aircond with --aircond): gpurun_out/<out>.npz, iters [K, S].
For the wave-tail study of DESIGN.md 3.7 (a wave of 64 one-lane scenarios runs to its
slowest lane)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-sppy-1_amd"))
import numpy as np  # noqa: E402

from mpisppy_amd.examples import farmer  # noqa: E402
from mpisppy_amd.engine import PHEngine  # noqa: E402
from mpisppy_amd import _lib  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
K = int(sys.argv[2]) if len(sys.argv) > 2 else 30
out = sys.argv[3] if len(sys.argv) > 3 else f"ipm_iters_S{S}"
b = farmer.batch_creator(farmer.scenario_names_creator(S), crops_multiplier=1, num_scens=S)
e = PHEngine(b, device="cuda:0")
e.solve(_lib.default_options(eps_rel=1e-10), warm=False)
assert e.kernel_info()["path"] == 6, e.kernel_info()
e.set_rho(1.0)
e.set_terms(1, 1)
o = _lib.default_options()
its = []
for k in range(K):
    e.compute_xbar()
    e.update(True)
    e.solve(o, warm=True)
    its.append(e.host("iters").copy())
e.close()
its = np.array(its, dtype=np.int16)
os.makedirs("gpurun_out", exist_ok=True)
np.savez_compressed(f"gpurun_out/{out}.npz", iters=its)
w = its.reshape(K, -1, 64)
print("mean", its.mean(1).round(2).tolist())
print("max", its.max(1).tolist())
print("mean of wave max", w.max(2).mean(1).round(2).tolist())
