"""cm = 64 PH accuracy vs the exact oracle fixtures for several iterk eps_rel values:
max |W - W_oracle| on the fixture sample, PDHG iterations and solve time (GPU)."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy-1_amd")); sys.path.insert(0, ROOT)
import numpy as np, torch
from mpisppy_amd.opt.ph import PH
from mpisppy_amd.examples import farmer
g = json.load(open(os.path.join(ROOT, "tests", "golden", "farmer_scale.json")))["farmer2048_cm64"]
names = g["names"]
smp = np.array(g["sample"])
eps0s = [float(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "1e-9").split(",")]
for eps, eps0 in [(float(v), e0) for v in (sys.argv[1] if len(sys.argv) > 1 else "1e-9").split(",") for e0 in eps0s]:
    opts = {"solver_name": "mi355x_pdhg", "PHIterLimit": 5, "defaultPHrho": 1.0, "convthresh": -1.0,
            "verbose": False, "display_progress": False, "toc": False, "device": "cuda:0",
            "batch_creator": farmer.batch_creator, "iterk_solver_options": {"eps_rel": eps},
            "iter0_solver_options": {"eps_rel": eps0}}
    ph = PH(opts, names, farmer.scenario_creator, scenario_creator_kwargs={"crops_multiplier": 64, "num_scens": len(names)})
    ph.PH_Prep(); torch.cuda.synchronize(); t0 = time.perf_counter(); ph.Iter0(); torch.cuda.synchronize()
    t_iter0 = time.perf_counter() - t0; i0 = ph.engine.host("iters")
    x0err = None
    its, ts, xe = [], [], []
    for it in range(5):
        ph.Compute_Xbar(); ph.Update_W(); ph.convergence_diff()
        xe.append(np.abs(ph.xbar_by_node()["ROOT"][:192] - np.array(g["xbar"][it])).max())
        torch.cuda.synchronize(); t0 = time.perf_counter()
        ph.solve_loop(solver_options=ph.iterk_solver_options)
        torch.cuda.synchronize(); ts.append(time.perf_counter() - t0)
        i = ph.engine.host("iters"); its.append((int(i.max()), float(i.mean())))
    err = np.abs(ph.W_array()[smp] - np.array(g["W"]))
    print(f"iter0 eps {eps0:g} ({1e3 * t_iter0:.1f} ms, iters max {i0.max()} mean {i0.mean():.0f}) iterk eps {eps:g}: max W err {err.max():.2e} (99.9% {np.quantile(err, 0.999):.2e}) max xbar err {max(xe):.2e} "
          f"iters {its} solve ms {[round(1e3 * t, 2) for t in ts]} nonopt {(ph.engine.host('status') != 0).sum()}", flush=True)
    ph.engine.close()
