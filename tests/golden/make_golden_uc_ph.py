"""Generate tests/golden/uc_ph.npz: three PH iterations of config 5 (the UC LP relaxation,
examples/uc.py) on Scenario1..8, solved by the CPU interior-point oracle oracle/uc_qp.py.

Run:  python tests/golden/make_golden_uc_ph.py      (~5 minutes on 8 cores)

PH over the 8 scenarios as one batch (probability 1/8 each), uc_funcs.py's rho
(examples/uc.py rho_vector), the loop of PHBase (phbase.py:758-979):

  Iter0       LP of every scenario (W = 0, no prox) -> x0
  x̄0 = mean x0_N,  W1 = rho (x0_N - x̄0),  conv1 = mean |x0_N - x̄0|
  k = 1..3:   QP  min c'x + W_k'x_N + rho/2 ||x_N - x̄_{k-1}||^2  -> x_k
              x̄_k = mean x_k,N,  W_{k+1} = W_k + rho (x_k,N - x̄_k),  conv_{k+1}

The Iter0 LPs have optimal faces (several optimal UnitOn vectors), so their x -- the
interior point's centre of the face here, a vertex for a simplex code, another face point for
the engine's PDHG -- is not solver-independent; the fixture therefore records x̄0 and W1 as the
PH state the GPU test installs, and pins the three PH iterations from there, whose QPs are
strongly convex in the nonants (unique x_N).  Parity stays UNPINNED against the reference (no
UC output ships with it): this checks the GPU's PH trajectory against an independent
second-order solve of the same QPs.
"""
import os
import sys
import time
from multiprocessing import Pool

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy-1_amd"))

NAMES = [f"Scenario{k}" for k in range(1, 9)]
ITERS = 3
TOL = 1e-10


def _solve(args):
    k, W, xbar, rho = args
    from mpisppy_amd.examples import uc
    from oracle import uc as ouc
    from oracle.uc_qp import solve_qp
    b = uc.batch_creator([NAMES[k]], num_scens=len(NAMES))
    A = ouc.scenario_matrix(b, 0)
    c, q = b.c[0].copy(), np.zeros(b.n)
    nc = np.asarray(b.nonant_col)
    if W is not None:
        c[nc] += W - rho * xbar
        q[nc] += rho
    t = time.time()
    r = solve_qp(A, b.rl[0], b.ru[0], b.lb[0], b.ub[0], c, q, tol=TOL)
    const = float(b.obj_const[0]) + (0.5 * float(np.sum(rho * xbar * xbar)) if W is not None else 0.0)
    return r["x"][nc], r["obj"] + const, r["status"], r["iters"], [float(v) for v in r["kkt"]], time.time() - t


def main():
    from mpisppy_amd.examples import uc
    S = len(NAMES)
    rho = uc.rho_vector(uc.scenario_creator(NAMES[0], num_scens=S))
    out = {"names": np.array(NAMES), "rho": rho}
    with Pool(min(8, S)) as pool:
        res = pool.map(_solve, [(k, None, None, rho) for k in range(S)])
        x = np.array([r[0] for r in res])
        out["iter0_obj"] = np.array([r[1] for r in res])
        out["iter0_kkt"] = np.array([r[4] for r in res])
        print("Iter0", [r[2] for r in res], [r[3] for r in res], f"{max(r[5] for r in res):.0f}s", flush=True)
        xbar = x.mean(0)
        W = rho * (x - xbar)
        out["xbar0"], out["W1"] = xbar, W.copy()
        out["conv1"] = np.abs(x - xbar).mean()
        xbars, convs, objs, kkts, Ws = [], [], [], [], []
        for it in range(ITERS):
            res = pool.map(_solve, [(k, W[k], xbar, rho) for k in range(S)])
            x = np.array([r[0] for r in res])
            objs.append([r[1] for r in res])
            kkts.append([r[4] for r in res])
            print(f"PH {it + 1}", [r[2] for r in res], [r[3] for r in res], f"{max(r[5] for r in res):.0f}s",
                  "kkt max", np.max([r[4] for r in res]), flush=True)
            xbar = x.mean(0)
            W = W + rho * (x - xbar)
            xbars.append(xbar)
            convs.append(np.abs(x - xbar).mean())
            Ws.append(W.copy())
    out["xbar"] = np.array(xbars)            # x̄_k, k = 1..ITERS
    out["conv"] = np.array(convs)            # conv after the update of iteration k
    out["W"] = np.array(Ws)                  # W_{k+1}
    out["obj"] = np.array(objs)              # augmented PH objective of each QP
    out["kkt"] = np.array(kkts)
    out["tol"] = TOL
    np.savez_compressed(os.path.join(HERE, "uc_ph.npz"), **out)
    print("wrote uc_ph.npz")


if __name__ == "__main__":
    main()
