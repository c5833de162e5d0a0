"""Diagnostic (TEST INFRASTRUCTURE, not collected): PH on the cm = 64 fixture scenarios with
the automatic path-6 kernel, and every PH subproblem's nonants against the oracle's exact
proximal solve (oracle/farmer_vec.py prox) with the same W / x̄ / rho.  Prints per PH
iteration the worst scenarios, their IPM iteration counts and statuses, and the launch time.

    python tests/diag_ipm_cm64.py [iterations] [scenarios] [fixture|first] [crops_multiplier]
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "mpi-sppy-1_amd"))
sys.path.insert(0, os.path.join(HERE, ".."))


def main():
    import torch
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.examples import farmer
    from oracle import farmer_vec as fv
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    g = json.load(open(os.path.join(HERE, "golden", "farmer_scale.json")))["farmer2048_cm64"]
    names = g["names"][:int(sys.argv[2])] if len(sys.argv) > 2 else g["names"]
    if len(sys.argv) > 3 and sys.argv[3] == "first":  # scen0.. (ties at scen0..2, near-ties)
        names = [f"scen{i}" for i in range(len(names))]
    cm = int(sys.argv[4]) if len(sys.argv) > 4 else 64
    opts = {"solver_name": "mi355x_pdhg", "PHIterLimit": iters, "defaultPHrho": 1.0, "convthresh": -1.0,
            "verbose": False, "display_progress": False, "toc": False, "device": "cuda:0",
            "batch_creator": farmer.batch_creator}
    ph = PH(opts, names, farmer.scenario_creator,
            scenario_creator_kwargs={"crops_multiplier": cm, "num_scens": len(names)})
    ph.PH_Prep()
    e = ph.engine
    e.want_duals = True
    t0 = time.perf_counter()
    ph.Iter0()
    torch.cuda.synchronize()
    print("iter0 %.3f s" % (time.perf_counter() - t0), e.kernel_info()["path"], e.ipm_info(), flush=True)
    bp, sl, f0 = fv.pieces(fv.yields(names, cm), cm)
    nc = e.batch.nonant_col if hasattr(e, "batch") else ph.batch.nonant_col
    for it in range(iters):
        ph.Compute_Xbar()
        ph.Update_W()
        K = 3 * cm
        W = e.host("W")[:, :K].copy()
        xb = e.host("xbar")[:, :K].copy()
        rho = e.host("rho")[:, :K].copy()
        x_in, y_in = e.host("x").copy(), e.host("y").copy()
        t0 = time.perf_counter()
        ph.solve_loop(solver_options=ph.iterk_solver_options, gripe=False)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        x = e.host("x")[:, nc]
        st, its = e.host("status"), e.host("iters")
        xv, ov = fv.prox(bp, sl, f0, W, xb, rho, 500.0 * cm)
        err = np.abs(x - xv).max(1)
        worst = np.argsort(-err)[:5]
        print(f"PH it {it + 1}: solve {dt * 1e3:.2f} ms, max err {err.max():.3e}, mean err {err.mean():.3e}, "
              f"iters max {its.max()} mean {its.mean():.1f}, status {np.bincount(st, minlength=4)[:4]}, "
              f"x̄ err {np.abs(x.T @ np.full(len(names), 1.0 / len(names)) - xv.mean(0)).max():.3e}", flush=True)
        dump = os.environ.get("DIAG_DUMP")
        if dump:  # the worst scenarios' subproblem inputs, for a host-emulation replay
            np.savez(f"{dump}_it{it + 1}.npz", names=np.array([names[s] for s in worst]), W=W[worst], xbar=xb[worst],
                     rho=rho[worst], x_in=x_in[worst], y_in=y_in[worst], x=x[worst], xv=xv[worst])
        for s in worst:
            print(f"    scen {names[s]}: err {err[s]:.3e} iters {its[s]} status {st[s]} obj {e.host('obj')[s]:.10g} "
                  f"oracle {ov[s]:.10g}", flush=True)


if __name__ == "__main__":
    main()
