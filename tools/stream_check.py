"""GPU check of the shared-matrix streaming path (path 4) -- development driver.
aircond (same matrix in every scenario) on path 4 vs the default path; UC scenarios vs HiGHS."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy-1_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from mpisppy_amd import _lib  # noqa: E402
from mpisppy_amd.engine import PHEngine  # noqa: E402
from mpisppy_amd.examples import aircond, uc  # noqa: E402


def aircond_check():
    bf = [4, 3, 2]
    kw = {"branching_factors": bf, "start_seed": 0, "QuadShortCoeff": 0.3}
    names = aircond.scenario_names_creator(24)
    b = aircond.batch_creator(names, **kw)
    e0 = PHEngine(b, device="cuda:0", shared=False)
    e0.solve(_lib.default_options(), warm=False)
    o0 = e0.host("obj").copy()
    e4 = PHEngine(b, device="cuda:0", shared=True)
    print("path", e4.kernel_info()["path"], "ws", e4.workspace_bytes(), flush=True)
    t = time.time()
    e4.solve(_lib.default_options(), warm=False)
    torch.cuda.synchronize()
    print("solve", time.time() - t, flush=True)
    o4 = e4.host("obj")
    st = e4.host("status")
    print("aircond status", np.bincount(st), "max rel obj diff", np.max(np.abs(o4 - o0) / np.maximum(1, np.abs(o0))),
          "iters", e4.host("iters").max(), e0.host("iters").max(), flush=True)
    x0, x4 = e0.host("x"), e4.host("x")
    print("max |x diff|", np.abs(x0 - x4).max(), flush=True)
    e0.close()
    e4.close()


def uc_check(S=4, eps=1e-6):
    from oracle import uc as ouc
    names = uc.scenario_names_creator(S)
    t = time.time()
    b = uc.batch_creator(names, num_scens=1000)
    print(f"uc batch n {b.n} m {b.m} nnz {b.nnz} ({time.time() - t:.1f}s)", flush=True)
    e = PHEngine(b, device="cuda:0")
    print("path", e.kernel_info()["path"], "ws GB", e.workspace_bytes() / 1e9, flush=True)
    t = time.time()
    e.solve(_lib.default_options(eps_rel=eps, max_iter=200000), warm=False)
    torch.cuda.synchronize()
    dt = time.time() - t
    obj, st, it = e.host("obj"), e.host("status"), e.host("iters")
    print(f"uc solve {dt:.2f}s status {st} iters {it} obj {obj}", flush=True)
    for s in range(min(S, 2)):
        x, ob, rc = ouc.solve_lp(b, s)
        print(f"  scen {s}: HiGHS {ob:.8g} gpu {obj[s]:.8g} rel {abs(obj[s] - ob) / abs(ob):.2e}", flush=True)
    e.close()


if __name__ == "__main__":
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    if what in ("all", "aircond"):
        aircond_check()
    if what in ("all", "uc"):
        uc_check(int(sys.argv[2]) if len(sys.argv) > 2 else 4)
