"""Path 6 for medium scenarios: the workgroup interior points -- the subtree kernel
(jit_ipm_blk.hip.in) for block-angular patterns and the workgroup kernel
(jit_ipm_wave.hip.in, 3.9) otherwise; one workgroup of 64 WPS threads per scenario, the normal equations
factored with the elimination tree split into per-thread subtrees and a dense root block
(tools/ipm_wave_proto.py states the plan and checks it on the CPU).

Checked against the same oracle as the other paths:
  * random block-arrow LP / QP batches (per-scenario data of every kind, long rows, one and
    two waves per scenario) against HiGHS / the oracle's QP IPM;
  * farmer cm = 10 (config 2's size, 30-entry acreage row as a long row) Iter0 against the
    exact vectorised oracle, objective and x (the cm copies of scen0..2 tie: symmetric point);
  * the fallback: scenarios the IPM does not finish go to the global-memory PDHG over the
    list (PHGPU_IPM_MAXIT), with the same answers; an infeasible scenario is certified there.
(Config 2 to 5 PH iterations and to convergence, and cm = 64 on 2,048 scenarios, run on this
kernel in test_gpu_scale.py / test_gpu_wg.py.)
Tolerances (north_star): objectives 1e-5 relative, x 1e-5 of its scale.
"""
import os

import numpy as np
import pytest

from test_gpu_parity import OBJ_REL

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _workgroup_ipms_on():
    """Multi-wave subtree plans and the workgroup kernel are opt-in (PHGPU_IPM_WAVE=1,
    solve_ipm.inc ipm_wg_bound); these tests check them against the oracle."""
    keep = os.environ.get("PHGPU_IPM_WAVE")
    os.environ["PHGPU_IPM_WAVE"] = "1"
    yield
    if keep is None:
        os.environ.pop("PHGPU_IPM_WAVE", None)
    else:
        os.environ["PHGPU_IPM_WAVE"] = keep


def arrow_batch(S, blocks, seed, with_q=False, link=2, bad=None, shapes="random"):
    """S scenarios sharing a block-arrow pattern: per block 3 columns and 2 rows (random
    entries; ``shapes`` "full": every block dense, one shape; "two": odd blocks lack one
    entry, two shapes), plus ``link`` rows each over every third column (long rows when
    blocks > 12), like farmer's crops and acreage row.  Feasible and bounded by
    construction; scenario ``bad`` (if given) gets every column bounded by 10 and a
    first-block row that needs 1e6: primal infeasible."""
    from mpisppy_amd.batch import ScenarioBatch
    rng = np.random.default_rng(seed)
    n, m = 3 * blocks, 2 * blocks + link
    mask = np.zeros((m, n), bool)
    for bk in range(blocks):
        for r in (2 * bk, 2 * bk + 1):
            mask[r, 3 * bk:3 * bk + 3] = rng.random(3) < 0.8 if shapes == "random" else True
            if not mask[r].any():
                mask[r, 3 * bk + rng.integers(3)] = True
        if shapes == "two" and bk % 2:
            mask[2 * bk, 3 * bk + 2] = False
    for l in range(link):
        mask[2 * blocks + l, l::3] = True
    rows, cols = np.nonzero(mask)
    row_ptr = np.concatenate([[0], np.cumsum(mask.sum(1))]).astype(np.int32)
    nnz = rows.size
    A = rng.normal(size=(S, nnz))
    x_feas = rng.uniform(0.0, 5.0, size=(S, n))
    Ax = np.zeros((S, m))
    for k in range(nnz):
        Ax[:, rows[k]] += A[:, k] * x_feas[:, cols[k]]
    kind = rng.integers(0, 3, size=m)
    rl = np.where(kind == 1, -np.inf, Ax - rng.uniform(0.1, 2.0, size=(S, m)))
    ru = np.where(kind == 0, np.inf, Ax + rng.uniform(0.1, 2.0, size=(S, m)))
    eqr = kind == 2
    rl[:, eqr] = Ax[:, eqr]
    ru[:, eqr] = Ax[:, eqr]
    lb = np.zeros((S, n))
    ub = np.full((S, n), 10.0)
    ub[:, ::3] = np.inf
    c = rng.normal(size=(S, n))
    c[:, ::3] = np.abs(c[:, ::3]) + 0.1
    q = rng.uniform(0.0, 1.0, size=(S, n)) if with_q else np.zeros((S, n))
    if bad is not None:
        ub[bad] = 10.0
        rl[bad, 0], ru[bad, 0] = 1e6, np.inf
    nn = 2
    return ScenarioBatch([f"s{i}" for i in range(S)], row_ptr, cols.astype(np.int32), A, c, lb, ub, rl, ru,
                         q, np.zeros(S), np.arange(nn, dtype=np.int32), np.zeros(nn, np.int32),
                         np.arange(nn, dtype=np.int32), np.zeros((S, 1), np.int32), ["ROOT"],
                         np.full(S, 1.0 / S), np.full((S, 1), 1.0 / S))


def _assert_wave(e, lanes=None):
    info, ii = e.kernel_info(), e.ipm_info()
    assert info["path"] == 6 and ii["compiled"] == 1 and ii["lanes"] >= 64, (info, ii)
    assert ii["scratch_bytes"] == 0, ii
    if lanes is not None:
        assert int(ii["lanes"]) == lanes, ii


@pytest.mark.parametrize("blocks,S,with_q,lanes", [(15, 24, False, 64), (30, 40, True, 64), (100, 16, False, 128)])
def test_wave_random_arrow_batches(gpu, blocks, S, with_q, lanes):
    from mpisppy_amd.engine import PHEngine
    from mpisppy_amd import _lib
    from oracle.lpqp import solve_lp_highs, solve_qp_ipm
    b = arrow_batch(S, blocks, seed=blocks + S, with_q=with_q)
    e = PHEngine(b, device="cuda:0")
    e.solve(_lib.default_options(eps_rel=1e-9), warm=False)
    _assert_wave(e, lanes)
    st, obj, bnd, x, it = e.host("status"), e.host("obj"), e.host("bound"), e.host("x"), e.host("iters")
    assert (st == _lib.OPTIMAL).all(), st
    assert it.max() <= 80, it                      # interior-point iterations: no fallback
    for s in range(S):
        A = b.dense_A(s)
        if with_q:
            xr, ob, rc = solve_qp_ipm(A, b.rl[s], b.ru[s], b.lb[s], b.ub[s], b.c[s], b.q[s])
        else:
            xr, ob, rc = solve_lp_highs(A, b.rl[s], b.ru[s], b.lb[s], b.ub[s], b.c[s])
        assert rc == 0
        tol = OBJ_REL * max(1.0, abs(ob))
        assert abs(obj[s] - ob) <= tol and abs(bnd[s] - ob) <= tol, (s, obj[s], bnd[s], ob)
        ax = A @ x[s]
        assert np.all(ax >= b.rl[s] - 1e-6 * (1 + np.abs(b.rl[s])))
        assert np.all(ax <= b.ru[s] + 1e-6 * (1 + np.abs(b.ru[s])))
        assert np.all(x[s] >= b.lb[s] - 1e-9) and np.all(x[s] <= b.ub[s] + 1e-9)
    # a warm-started re-solve with PH terms: still the oracle's answers
    rng = np.random.default_rng(1)
    W = rng.normal(size=(S, 2))
    xb = rng.uniform(0.0, 3.0, size=(S, 2))
    e.set_rho(1.0)
    e.set_W(W)
    e.set_xbar(xb)
    e.set_terms(1, 1)
    e.solve(_lib.default_options(eps_rel=1e-9), warm=True)
    obj2, st2 = e.host("obj"), e.host("status")
    assert (st2 == 0).all()
    for s in range(0, S, 3):
        A = b.dense_A(s)
        c = b.c[s].copy()
        q = b.q[s].copy()
        c[:2] += W[s] - xb[s]
        q[:2] += 1.0
        xr, ob, rc = solve_qp_ipm(A, b.rl[s], b.ru[s], b.lb[s], b.ub[s], c, q)
        ob += 0.5 * float(np.sum(xb[s] ** 2))
        assert rc == 0 and abs(obj2[s] - ob) <= OBJ_REL * max(1.0, abs(ob)), (s, obj2[s], ob)
    e.close()


def test_wave_farmer_cm10_iter0_vs_oracle(gpu):
    """Config 2's size (cm = 10): Iter0 LP objectives and x of 256 scenarios vs the exact
    vectorised oracle (scen0..2: the cm copies tie, the oracle takes the symmetric point,
    which the interior point converges to as well)."""
    from mpisppy_amd.engine import PHEngine
    from mpisppy_amd.examples import farmer
    from mpisppy_amd import _lib
    from oracle import farmer_vec as fv
    S, cm = 256, 10
    names = farmer.scenario_names_creator(S)
    b = farmer.batch_creator(names, crops_multiplier=cm, num_scens=S)
    e = PHEngine(b, device="cuda:0")
    e.solve(_lib.default_options(eps_rel=1e-10), warm=False)
    _assert_wave(e, 64)
    assert (e.host("status") == 0).all()
    bp, sl, f0 = fv.pieces(fv.yields(names, cm), cm)
    x_ref, obj_ref = fv.iter0_lp(bp, sl, f0, 500.0 * cm)
    obj = e.host("obj")
    assert np.abs(obj - obj_ref).max() <= OBJ_REL * np.abs(obj_ref).max(), np.abs(obj - obj_ref).max()
    xn = e.host("x")[:, b.nonant_col]
    err = np.abs(xn - x_ref)
    assert err.max() <= 1e-5 * 500 * cm, (err.max(), int(err.max(1).argmax()))
    e.close()


def test_wave_fallback_list_and_certificate(gpu):
    """PHGPU_IPM_MAXIT=3 sends every scenario to the fallback (the global-memory PDHG over
    the list): the objectives are still the oracle's; an infeasible scenario is certified
    (status 2) by the fallback while the others stay OPTIMAL; the statistics count both."""
    import torch
    from mpisppy_amd.engine import PHEngine
    from mpisppy_amd import _lib
    from oracle.lpqp import solve_lp_highs
    S, bad = 20, 7
    b = arrow_batch(S, 15, seed=5, bad=bad)
    e = PHEngine(b, device="cuda:0")
    e.solve(_lib.default_options(eps_rel=1e-9), warm=False)
    _assert_wave(e)
    st = e.host("status")
    assert st[bad] == _lib.PRIMAL_INFEASIBLE, st
    others = np.delete(np.arange(S), bad)
    assert (st[others] == 0).all(), st
    ref = {}
    for s in others[:6]:
        A = b.dense_A(s)
        _, ob, rc = solve_lp_highs(A, b.rl[s], b.ru[s], b.lb[s], b.ub[s], b.c[s])
        ref[s] = ob
    stats = torch.zeros(6, dtype=torch.int64).pin_memory()
    _lib.check(e.lib.phgpu_solve_stats(e.h, stats.data_ptr(), e._stream()), "stats")
    torch.cuda.synchronize()
    assert int(stats[0]) == S - 1 and int(stats[2]) == 1, stats.tolist()
    keep = os.environ.get("PHGPU_IPM_MAXIT")
    os.environ["PHGPU_IPM_MAXIT"] = "3"
    try:
        e.solve(_lib.default_options(eps_rel=1e-9), warm=False)
    finally:
        if keep is None:
            os.environ.pop("PHGPU_IPM_MAXIT", None)
        else:
            os.environ["PHGPU_IPM_MAXIT"] = keep
    st, obj, it = e.host("status"), e.host("obj"), e.host("iters")
    assert st[bad] == _lib.PRIMAL_INFEASIBLE and (st[others] == 0).all(), st
    assert it[others].min() > 3                     # PDHG iteration counts: the fallback solved them
    for s, ob in ref.items():
        assert abs(obj[s] - ob) <= OBJ_REL * max(1.0, abs(ob)), (s, obj[s], ob)
    e.close()
