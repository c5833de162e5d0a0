"""Generate the config-4 scale fixture (tests/golden/aircond_scale.json).

Run:  python tests/golden/make_golden_aircond.py [workers]     (~5 minutes on 8 cores)
      python tests/golden/make_golden_aircond.py --conv [workers]
            (aircond_conv.json: the same run continued until conv < CONV_THRESH, the
             PH iteration count of iterk_loop's break, phbase.py:925-934)

Config 4 as bench.py times it: aircond, branching factors 32 x 32 x 64 (65,536 scenarios,
1,057 non-leaf nodes), straight_tests.py:36 parameters (Capacity 200, QuadShortCoeff 0.3,
BeginInventory 50, mu_dev 0, sigma_dev 40, start_seed 0), rho = 1.  Source: the oracle's
restatement of aircond.py:37-330 (oracle/models.py aircond_scenario) solved scenario by
scenario with the dense IPM (oracle/lpqp.py solve_qp_ipm; Iter0 is already a QP here), and
PHBase.Iter0 / iterk_loop (phbase.py:758-979) as oracle/ph.py states them, with the
solve loop spread over worker processes (contiguous chunks; every reduction is done in
scenario order in the parent, so the result does not depend on the worker count).

Contents: the trivial bound (all 65,536 Iter0 solves), the Iter0 objective of every 64th
scenario, and for PH_ITERS iterations the x̄ of every non-leaf node and conv; W of every
64th scenario after the last iteration; E[obj] after it.
"""
import json
import math
import os
import sys
import time
import warnings
from multiprocessing import get_context

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

BF = [32, 32, 64]
KW = dict(Capacity=200, QuadShortCoeff=0.3, BeginInventory=50, mu_dev=0, sigma_dev=40, start_seed=0)
RHO = 1.0
PH_ITERS = 3
STRIDE = 64


def _solve_chunk(args):
    """Solve scenarios [a, b) with the PH terms given (phbase.py:617-699): returns their
    nonant x and (augmented) objectives."""
    a, b, W, xbar, terms = args
    warnings.simplefilter("ignore")
    from oracle.models import aircond_scenario
    from oracle.lpqp import solve_qp_ipm, kkt_certify
    xs, objs, loose = [], [], {}
    for k, s in enumerate(range(a, b)):
        sc = aircond_scenario(f"scen{s}", BF, **KW)
        A, rl, ru, lb, ub, c, q = sc.arrays()
        idx = sc.nonant_indices()
        c = c.copy()
        q = q.copy()
        const = 0.0
        if terms:
            c[idx] += W[k] - RHO * xbar[k]
            q[idx] += RHO
            const = 0.5 * float(np.sum(RHO * xbar[k] ** 2))
        x, obj, st = solve_qp_ipm(A, rl, ru, lb, ub, c, q)
        if st != 0:
            # a QP that stops short of the IPM's 1e-11 tolerance is re-solved with a longer
            # run, then looser tolerances; its answer is kept only with an independent KKT
            # certificate (lpqp.kkt_certify), and the tolerance used is recorded
            for tol in (1e-11, 1e-10, 1e-9, 1e-8):
                x, obj, st = solve_qp_ipm(A, rl, ru, lb, ub, c, q, tol=tol, max_iter=1000)
                if st == 0:
                    break
            pv, sv = kkt_certify(A, rl, ru, lb, ub, c, q, x)
            if st != 0 or pv > 1e-9 or sv > 1e-9:
                raise RuntimeError(f"scen{s}: IPM status {st}, KKT violation {pv:.2e} / {sv:.2e}")
            print(f"  scen{s}: IPM tolerance {tol:g}, KKT {pv:.1e} / {sv:.1e}", flush=True)
            loose[s] = tol
        xs.append(x[idx])
        objs.append(obj + const)
    return np.array(xs), np.array(objs), loose


CONV_THRESH = 1e-2     # the coarse threshold of the convergence-count fixture
CONV_LIMIT = 80


def main():
    from oracle.models import aircond_scenario
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    to_conv = "--conv" in sys.argv
    workers = int(args[0]) if args else max(1, (os.cpu_count() or 2) - 1)
    S = int(np.prod(BF))
    t0 = time.time()
    # tree bookkeeping (spbase.py:378-391): nonant k of scenario s belongs to node
    # node_of[s, k // 2]; prob_coeff = pi_s / pi_node
    node_names, node_of = [], np.empty((S, len(BF)), dtype=np.int64)
    nid = {}
    for s in range(S):
        sc = aircond_scenario(f"scen{s}", BF, **KW)
        for d, (ndn, _cond, _stage, _idx) in enumerate(sc.nodes):
            if ndn not in nid:
                nid[ndn] = len(node_names)
                node_names.append(ndn)
            node_of[s, d] = nid[ndn]
    prob = 1.0 / S
    uncond = np.array([1.0] + [1.0 / np.prod(BF[:d]) for d in range(1, len(BF))])
    pcoef = prob / uncond                                  # [depth]
    nn = 2 * len(BF)
    depth_of = np.repeat(np.arange(len(BF)), 2)
    chunks = [(int(i * S / (8 * workers)), int((i + 1) * S / (8 * workers))) for i in range(8 * workers)]
    W = np.zeros((S, nn))
    xbar = np.zeros((S, nn))
    ctx = get_context("spawn")
    loose_all = {}
    with ctx.Pool(workers) as pool:
        def solve(terms):
            res = pool.map(_solve_chunk, [(a, b, W[a:b], xbar[a:b], terms) for a, b in chunks])
            for r in res:
                loose_all.update({f"scen{k}": v for k, v in r[2].items()})
            return np.concatenate([r[0] for r in res]), np.concatenate([r[1] for r in res])
        x, obj = solve(False)                                        # Iter0 (phbase.py:802)
        tb = math.fsum(prob * obj)                                   # Ebound (spopt.py:346-391)
        print(f"Iter0: trivial bound {tb:.10f} ({time.time() - t0:.0f}s)", flush=True)
        sample = list(range(0, S, STRIDE))
        out = {"branching_factors": BF, "kwargs": KW, "rho": RHO, "S": S, "trivial_bound": tb,
               "sample": sample, "iter0_obj": obj[sample].tolist(), "node_names": node_names,
               "xbar": [], "conv": []}
        n_iters = CONV_LIMIT if to_conv else PH_ITERS
        for it in range(n_iters):
            # _Compute_Xbar (phbase.py:27-107): per node sum of prob_coeff * x, in scenario order
            nx = np.zeros((len(node_names), 2))
            for k in range(nn):
                d = depth_of[k]
                np.add.at(nx[:, k % 2], node_of[:, d], pcoef[d] * x[:, k])
            for k in range(nn):
                xbar[:, k] = nx[node_of[:, depth_of[k]], k % 2]
            W += RHO * (x - xbar)                                    # Update_W (:293-318)
            conv = float(np.abs(x - xbar).sum() / (S * nn))          # convergence_diff (:321-343)
            out["xbar"].append(nx.tolist())
            out["conv"].append(conv)
            print(f"PH iteration {it + 1}: conv {conv:.10f} ({time.time() - t0:.0f}s)", flush=True)
            if to_conv and conv < CONV_THRESH:
                # iterk_loop breaks here, before the solve (phbase.py:925-934)
                out["conv_thresh"] = CONV_THRESH
                out["break_iteration"] = it + 1
                break
            x, obj = solve(True)                                     # solve_loop (:941)
    if to_conv:
        # aircond_conv.json: the PH iteration count to conv < CONV_THRESH, the conv
        # trajectory, and x̄ of every node at the last two iterations (a run that breaks one
        # iteration off is compared against its own iteration)
        if "break_iteration" not in out:
            raise RuntimeError(f"conv >= {CONV_THRESH} after {CONV_LIMIT} PH iterations")
        conv_out = {k: out[k] for k in ("branching_factors", "kwargs", "rho", "S", "trivial_bound", "node_names",
                                        "conv", "conv_thresh", "break_iteration")}
        conv_out["xbar_last"] = {str(len(out["xbar"]) - k): out["xbar"][-1 - k] for k in range(min(2, len(out["xbar"])))}
        conv_out["W_sample"] = sample
        conv_out["W_break"] = W[sample].tolist()
        conv_out["ipm_loose_tolerance"] = loose_all
        with open(os.path.join(HERE, "aircond_conv.json"), "w") as f:
            json.dump(conv_out, f)
        print(f"done: break at {out['break_iteration']} ({time.time() - t0:.0f}s)", flush=True)
        return
    out["ph_iters"] = PH_ITERS
    out["W"] = W[sample].tolist()
    out["Eobj"] = math.fsum(prob * obj)
    out["ipm_loose_tolerance"] = loose_all
    with open(os.path.join(HERE, "aircond_scale.json"), "w") as f:
        json.dump(out, f)
    print(f"done ({time.time() - t0:.0f}s)", flush=True)


if __name__ == "__main__":
    main()
