"""Host-side timeline of the PH loop (farmer 65,536, config 3): where the time outside
the solve kernel goes.  Mirrors PHBase.iterk_loop's calls with timestamps."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy-1_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from mpisppy_amd.opt.ph import PH  # noqa: E402
from mpisppy_amd.examples import farmer  # noqa: E402

S = 65536
opts = {"solver_name": "mi355x_pdhg", "PHIterLimit": 5, "defaultPHrho": 1.0, "convthresh": -1.0,
        "verbose": False, "display_progress": False, "toc": False, "device": "cuda:0",
        "batch_creator": farmer.batch_creator, "iterk_solver_options": {"eps_rel": 1e-9}}
ph = PH(opts, farmer.scenario_names_creator(S), farmer.scenario_creator,
        scenario_creator_kwargs={"crops_multiplier": 1, "num_scens": S})
ph.PH_Prep()
ph.Iter0()
ph.iterk_loop()
torch.cuda.synchronize()
rows = []
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for it in range(20):
    t0 = time.perf_counter()
    ph.Compute_Xbar()
    t1 = time.perf_counter()
    ph.Update_W()
    t2 = time.perf_counter()
    conv = ph.convergence_diff()
    t3 = time.perf_counter()
    ph.gripe_report()
    t4 = time.perf_counter()
    e0.record()
    ph.solve_loop(solver_options=ph.current_solver_options, gripe="deferred")
    e1.record()
    t5 = time.perf_counter()
    rows.append([t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4])
torch.cuda.synchronize()
r = np.median(np.array(rows[2:]), axis=0) * 1e6
print("median us: compute_xbar %.1f  update_w %.1f  conv (incl. wait) %.1f  gripe %.1f  solve_loop call %.1f"
      % tuple(r), flush=True)
# GPU time of the non-solve kernels of one iteration, alone
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(20):
    ph.Compute_Xbar()
    ph.Update_W()
b.record()
torch.cuda.synchronize()
print("x̄ + W kernels back to back: %.1f us per iteration" % (a.elapsed_time(b) * 1e3 / 20), flush=True)
t = time.perf_counter()
for _ in range(20):
    ph.convergence_diff()
print("conv readback with nothing queued: %.1f us" % ((time.perf_counter() - t) * 1e6 / 20), flush=True)
