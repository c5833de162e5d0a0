"""GPU diagnostic: the aircond 32x32x64 Iter0 QPs that reach the PDHG iteration cap.

Solves every scenario's Iter0 problem (W_on = prox_on = 0) at eps_rel 1e-10 and 1e-9
(100,000 iterations), prints the iteration distribution and the scenarios at the cap,
then re-solves those alone with a 1,000,000 cap and prints their objective against the
oracle IPM (nonant x too)."""
import os
import sys
import warnings

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy-1_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
from mpisppy_amd.examples import aircond  # noqa: E402
from mpisppy_amd.engine import PHEngine  # noqa: E402
from mpisppy_amd.sputils import create_nodenames_from_branching_factors  # noqa: E402
from mpisppy_amd import _lib  # noqa: E402

KW = {"Capacity": 200, "QuadShortCoeff": 0.3, "BeginInventory": 50, "mu_dev": 0, "sigma_dev": 40, "start_seed": 0}
BF = [32, 32, 64]
S = int(np.prod(BF))
names = aircond.scenario_names_creator(S)
b = aircond.batch_creator(names, branching_factors=BF, **KW)
e = PHEngine(b, device="cuda:0", node_names=[nd for nd in create_nodenames_from_branching_factors(BF)
                                            if nd.count("_") < len(BF)])
bad = set()
for eps in (1e-10, 1e-9):
    e.solve(_lib.default_options(eps_rel=eps), warm=False)
    it, st = e.host("iters"), e.host("status")
    print(f"eps {eps:g}: max {it.max()} mean {it.mean():.1f} p99.99 {np.percentile(it, 99.99):.0f} "
          f"not optimal {(st != 0).sum()} {np.nonzero(st != 0)[0][:10].tolist()}", flush=True)
    bad |= set(np.nonzero(st != 0)[0].tolist())
warnings.simplefilter("ignore")
from oracle.models import aircond_scenario  # noqa: E402
from oracle.lpqp import solve_qp_ipm  # noqa: E402
for s in sorted(bad)[:5]:
    one = aircond.batch_creator([names[s]], branching_factors=BF, **KW)
    e1 = PHEngine(one, device="cuda:0", node_names=e.node_names)
    sc = aircond_scenario(names[s], BF, **KW)
    A, rl, ru, lb, ub, c, q = sc.arrays()
    xo, oo, so = solve_qp_ipm(A, rl, ru, lb, ub, c, q)
    for eps in (1e-10, 1e-9, 1e-8):
        e1.solve(_lib.default_options(eps_rel=eps, max_iter=1000000), warm=False)
        print(f"{names[s]} eps {eps:g}: status {e1.host('status')[0]} iters {e1.host('iters')[0]} "
              f"obj {e1.host('obj')[0]:.10f} bound {e1.host('bound')[0]:.10f} ipm {oo:.10f} "
              f"|x-x_ipm|max {np.abs(e1.host('x')[0] - xo).max():.3e}", flush=True)
    print("  demands", [round(d, 3) for d in sc.demands] if hasattr(sc, "demands") else "", "x_ipm", np.round(xo, 4).tolist(),
          flush=True)
