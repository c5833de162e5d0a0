"""UC LP-relaxation oracle (TEST INFRASTRUCTURE ONLY -- tests/, smoke() and bench.py's
cpu_baseline leg may use it; the product path never does).

Solves one UC scenario's LP relaxation (mpisppy_amd/examples/uc.py, a restatement of
paperruns/larger_uc/ReferenceModel_OK.py) exactly with scipy's HiGHS, from the same
ScenarioBatch arrays the engine receives.  This stands in for the external solver the
reference reaches through Pyomo (spopt.py:85-223).  Parity for UC is UNPINNED: the
reference holds no UC outputs, so this checks the GPU solve of our restated LP, not
the restatement itself.
"""
import numpy as np
import scipy.sparse as sp
from scipy.optimize import linprog


def scenario_matrix(b, s):
    rows = np.repeat(np.arange(b.m), np.diff(b.row_ptr))
    return sp.csr_matrix((b.A_val[s], (rows, b.col_idx)), shape=(b.m, b.n))


def solve_lp(b, s, c=None, method="highs-ds", tol=1e-9):
    """min c'x s.t. rl <= A x <= ru, lb <= x <= ub for scenario ``s`` of batch ``b``.
    Returns (x, obj, status) with obj including obj_const."""
    A = scenario_matrix(b, s)
    rl, ru = b.rl[s], b.ru[s]
    c = b.c[s] if c is None else c
    eq = np.isfinite(rl) & np.isfinite(ru) & (rl == ru)
    ub_rows = (~eq) & np.isfinite(ru)
    lb_rows = (~eq) & np.isfinite(rl)
    A_ub = sp.vstack([A[ub_rows], -A[lb_rows]]).tocsr()
    b_ub = np.concatenate([ru[ub_rows], -rl[lb_rows]])
    bounds = np.column_stack([np.where(np.isfinite(b.lb[s]), b.lb[s], -np.inf),
                              np.where(np.isfinite(b.ub[s]), b.ub[s], np.inf)])
    res = linprog(c, A_ub=A_ub, b_ub=b_ub, A_eq=A[eq], b_eq=rl[eq], bounds=bounds, method=method,
                  options={"primal_feasibility_tolerance": tol, "dual_feasibility_tolerance": tol})
    if res.status != 0:
        return None, None, res.status
    return res.x, float(res.fun) + float(b.obj_const[s]), 0
