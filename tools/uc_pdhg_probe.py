"""How many PDHG iterations does a UC LP relaxation need?  (development probe)

Runs tools/pdhg_proto.py's restarted reflected-Halpern PDHG -- the algorithm the HIP
kernels implement -- on one UC scenario with scipy.sparse mat-vecs, and reports the
iteration count / objective against HiGHS at a few tolerances.
usage: python tools/uc_pdhg_probe.py [scen] [eps ...]
"""
import os
import sys
import time

import numpy as np
import scipy.sparse as sp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy-1_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import pdhg_proto  # noqa: E402
from mpisppy_amd.examples import uc  # noqa: E402
from oracle import uc as ouc  # noqa: E402

_MATS = {}


def _mat(rp, ci, Av):
    key = (id(Av), Av.shape)
    if key not in _MATS:
        rows = np.repeat(np.arange(len(rp) - 1), np.diff(rp))
        n = int(ci.max()) + 1 if _N is None else _N
        _MATS[key] = sp.csr_matrix((Av[0], (rows, ci)), shape=(len(rp) - 1, n))
    return _MATS[key]


_N = None


def spmv(rp, ci, Av, x):
    return (_mat(rp, ci, Av) @ x[0])[None, :]


def spmvT(rp, ci, Av, y, n):
    return (_mat(rp, ci, Av).T @ y[0])[None, :]


def main():
    global _N
    scen = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    epss = [float(e) for e in sys.argv[2:]] or [1e-4, 1e-6, 1e-8]
    b = uc.batch_creator([f"Scenario{scen}"], num_scens=1000)
    _N = b.n
    pdhg_proto.spmv, pdhg_proto.spmvT = spmv, spmvT
    t = time.time()
    x_ref, obj_ref, st = ouc.solve_lp(b, 0)
    print(f"HiGHS obj {obj_ref:.10g} ({time.time() - t:.1f}s)", flush=True)
    t = time.time()
    pr = pdhg_proto.Proto(b)
    print(f"setup {time.time() - t:.1f}s  normA {pr.normA[0]:.4g}", flush=True)
    for eps in epss:
        pr.x[:] = 0
        pr.y[:] = 0
        t = time.time()
        x, y, iters, done, restarts = pr.solve(b.c, b.q, eps=eps, max_iter=200000, check=64, restart_every=16,
                                               kernel_mode=True)
        obj = float(b.c[0] @ x[0])
        print(f"eps {eps:g}: iters {iters[0]} done {done[0]} restarts {restarts[0]} obj {obj:.10g} "
              f"rel.err {abs(obj - obj_ref) / abs(obj_ref):.2e}  max|x-x*|_nonant "
              f"{np.max(np.abs(x[0][b.nonant_col] - x_ref[b.nonant_col])):.2e} ({time.time() - t:.1f}s)", flush=True)


if __name__ == "__main__":
    main()
