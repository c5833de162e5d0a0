"""Per PH iteration of config 2 (farmer 1,024 scenarios, cm = 10) on the subtree interior
point: solve time, jam hand-overs and re-centrings (phgpu_ipm_info of that solve), the IPM /
fallback iteration maximum (TOOL ONLY; the non-speculative loop, synchronising per step).

    python tools/diag_jams.py [iterations] [scenarios] [cm]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy-1_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mpisppy_amd.opt.ph import PH  # noqa: E402
from mpisppy_amd.examples import farmer  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 60
S = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
cm = int(sys.argv[3]) if len(sys.argv) > 3 else 10
opts = {"solver_name": "mi355x_pdhg", "PHIterLimit": K, "defaultPHrho": 1.0, "convthresh": -1.0, "verbose": False,
        "display_progress": False, "toc": False, "device": "cuda:0", "batch_creator": farmer.batch_creator,
        "iterk_solver_options": dict(farmer.PDHG_ITERK_OPTIONS)}
ph = PH(opts, farmer.scenario_names_creator(S), farmer.scenario_creator,
        scenario_creator_kwargs={"crops_multiplier": cm, "num_scens": S})
ph.PH_Prep()
ph.Iter0()
e = ph.engine
rows = []
for k in range(K):
    ph.Compute_Xbar()
    ph.Update_W()
    ph.convergence_diff()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ph.solve_loop(solver_options=ph.iterk_solver_options)
    torch.cuda.synchronize()
    dt = 1e3 * (time.perf_counter() - t0)
    ii = e.ipm_info()
    it = e.host("iters")
    rows.append((dt, ii["jam_handovers"], ii["recentrings"], int(it.max())))
    print(f"ph{k + 1} {dt:8.3f} ms jams {int(ii['jam_handovers'])} recentrings {int(ii['recentrings'])} "
          f"iters max {int(it.max())} status!=0 {int((e.host('status') != 0).sum())}", flush=True)
r = np.array(rows)
print("median ms", np.median(r[:, 0]), "mean ms", r[:, 0].mean(), "steps with jams", int((r[:, 1] > 0).sum()),
      "jams", int(r[:, 1].sum()))
