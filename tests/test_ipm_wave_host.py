"""The two workgroup interior points -- the subtree kernel (jit_ipm_blk.hip.in, the automatic
choice for block-angular patterns) and the workgroup kernel (jit_ipm_wave.hip.in,
PHGPU_IPM_BLK=0) -- run on the CPU by tests/ipm_wave_host.py (one std::thread per GPU
thread, barriers for the workgroup syncs and sums): their generated code and arithmetic
against HiGHS / the oracle's QP IPM / the exact farmer oracle, without a GPU.
test_gpu_ipm_wave.py checks the real kernels."""
import os

import numpy as np
import pytest

import ipm_wave_host
from test_gpu_ipm_wave import arrow_batch

OBJ_REL = 1e-5
KERNELS = {"blk": "k_solve_ipm_blk", "wave": "k_solve_ipm_wave"}


@pytest.fixture(params=["blk", "wave"])
def kernel(request):
    keep = os.environ.get("PHGPU_IPM_BLK")
    os.environ["PHGPU_IPM_BLK"] = "1" if request.param == "blk" else "0"
    yield request.param
    if keep is None:
        os.environ.pop("PHGPU_IPM_BLK", None)
    else:
        os.environ["PHGPU_IPM_BLK"] = keep


def _src_kernel(b, lanes):
    import mpisppy_amd._lib as L
    src, _ = L.ipm_source(b, lanes)
    return src


@pytest.mark.parametrize("blocks,S,with_q,lanes,shapes", [(15, 3, False, 64, "random"), (30, 2, True, 64, "full"),
                                                          (100, 1, False, 128, "two"), (40, 2, True, 64, "two")])
def test_host_arrow_vs_oracle(kernel, blocks, S, with_q, lanes, shapes):
    """Block-arrow LPs / QPs: random block shapes (many classes: the workgroup kernel either
    way), one shape, two shapes (two class layers of the subtree kernel)."""
    from oracle.lpqp import solve_lp_highs, solve_qp_ipm
    b = arrow_batch(S, blocks, seed=blocks + S, with_q=with_q, shapes=shapes)
    want = KERNELS[kernel] if shapes != "random" else "k_solve_ipm_wave"
    assert want in _src_kernel(b, lanes)
    x, y, obj, bound, st, it = ipm_wave_host.solve(b, lanes=lanes)
    assert (st == 0).all(), (st, it)
    for s in range(S):
        A = b.dense_A(s)
        if with_q:
            xr, ob, rc = solve_qp_ipm(A, b.rl[s], b.ru[s], b.lb[s], b.ub[s], b.c[s], b.q[s])
        else:
            xr, ob, rc = solve_lp_highs(A, b.rl[s], b.ru[s], b.lb[s], b.ub[s], b.c[s])
        assert rc == 0
        tol = OBJ_REL * max(1.0, abs(ob))
        assert abs(obj[s] - ob) <= tol and abs(bound[s] - ob) <= tol, (s, obj[s], bound[s], ob, it[s])
        ax = A @ x[s]
        assert np.all(ax >= b.rl[s] - 1e-6 * (1 + np.abs(b.rl[s])))
        assert np.all(ax <= b.ru[s] + 1e-6 * (1 + np.abs(b.ru[s])))


def test_host_farmer_cm10_vs_oracle(kernel):
    from mpisppy_amd.examples import farmer
    from oracle import farmer_vec as fv
    names = ["scen0", "scen5", "scen17", "scen600"]
    b = farmer.batch_creator(names, crops_multiplier=10, num_scens=1024)
    assert KERNELS[kernel] in _src_kernel(b, 64)
    x, y, obj, bound, st, it = ipm_wave_host.solve(b, lanes=64, eps_rel=1e-10)
    assert (st == 0).all(), (st, it)
    bp, sl, f0 = fv.pieces(fv.yields(names, 10), 10)
    x_ref, obj_ref = fv.iter0_lp(bp, sl, f0, 5000.0)
    assert np.abs(obj - obj_ref).max() <= OBJ_REL * np.abs(obj_ref).max(), (obj, obj_ref)
    err = np.abs(x[:, b.nonant_col] - x_ref).max()
    assert err <= 1e-5 * 5000, err


def test_host_farmer_cm10_ph_terms_vs_oracle():
    """A PH subproblem (W, rho, x̄ on the acreage nonants) warm-started from the Iter0 answer
    on the subtree kernel, against the oracle's exact proximal farmer solve."""
    from mpisppy_amd.examples import farmer
    from oracle import farmer_vec as fv
    names = ["scen3", "scen40", "scen777"]
    b = farmer.batch_creator(names, crops_multiplier=10, num_scens=1024)
    assert "k_solve_ipm_blk" in _src_kernel(b, 64)
    x0, y0, obj0, _, st0, _ = ipm_wave_host.solve(b, lanes=64, eps_rel=1e-10)
    assert (st0 == 0).all()
    rng = np.random.default_rng(7)
    K = b.nn
    W = rng.normal(0, 40, (len(names), K))
    xbar = np.broadcast_to(5000.0 / K * rng.uniform(0.3, 1.7, K), W.shape).copy()
    rho = np.full((len(names), K), 1.0)
    x, y, obj, bound, st, it = ipm_wave_host.solve(b, lanes=64, W=W, rho=rho, xbar=xbar, eps_rel=1e-10, x_in=x0,
                                                   y_in=y0)
    assert (st == 0).all(), (st, it)
    bp, sl, f0 = fv.pieces(fv.yields(names, 10), 10)
    xv, ov = fv.prox(bp, sl, f0, W, xbar, rho, 5000.0)
    assert np.abs(obj - ov).max() <= OBJ_REL * np.abs(ov).max(), (obj, ov)
    assert np.abs(x[:, b.nonant_col] - xv).max() <= 1e-5 * 5000


def test_host_farmer_cm64_vs_oracle(kernel):
    """cm = 64 (n 768, m 385): 191 two-row subtrees on 192 threads (subtree kernel), or four
    waves per scenario (workgroup kernel)."""
    from mpisppy_amd.examples import farmer
    from oracle import farmer_vec as fv
    names = ["scen7"]
    b = farmer.batch_creator(names, crops_multiplier=64, num_scens=2048)
    lanes = 192 if kernel == "blk" else 256
    assert KERNELS[kernel] in _src_kernel(b, lanes)
    x, y, obj, bound, st, it = ipm_wave_host.solve(b, lanes=lanes, eps_rel=1e-10)
    assert (st == 0).all(), (st, it)
    bp, sl, f0 = fv.pieces(fv.yields(names, 64), 64)
    x_ref, obj_ref = fv.iter0_lp(bp, sl, f0, 500.0 * 64)
    assert abs(obj[0] - obj_ref[0]) <= OBJ_REL * abs(obj_ref[0]), (obj, obj_ref)
    assert np.abs(x[:, b.nonant_col] - x_ref).max() <= 1e-5 * 500 * 64


def test_host_blk_fallback_hands_over():
    """max_ipm = 2: every scenario goes to the fallback list with its warm state."""
    b = arrow_batch(3, 15, seed=11, shapes="full")
    assert "k_solve_ipm_blk" in _src_kernel(b, 64)
    x, y, obj, bound, st, it = ipm_wave_host.solve(b, lanes=64, max_ipm=2)
    assert (st == -1).all(), st


def test_blk_plan_shapes():
    """The subtree plan: farmer cm = 10 / 64 are block-angular (one class of crop subtrees;
    64 / 192 threads); a pattern whose rows all share one column is not (workgroup kernel)."""
    import mpisppy_amd._lib as L
    from mpisppy_amd.batch import ScenarioBatch
    from mpisppy_amd.examples import farmer
    for cm, lanes in ((10, 64), (64, 192)):
        b = farmer.batch_creator(farmer.scenario_names_creator(2), crops_multiplier=cm, num_scens=2)
        src = _src_kernel(b, lanes)
        assert "k_solve_ipm_blk" in src and f"#define WT {lanes}\n" in src
        # the ordering's tie-break leaves the acreage row alone at the root: one root row,
        # every crop a two-row subtree of four columns, no free columns
        assert "#define NRT 1\n" in src and "#define NLC 4\n" in src and "#define NLRW 2\n" in src
    # 40 rows in a chain (row i on columns i and i + 1): the elimination tree is a path, one
    # subtree of 40 rows -- too big for a thread, and no small root set splits it
    m, n = 40, 41
    rows, cols = [], []
    for i in range(m):
        for j in (i, i + 1):
            rows.append(i)
            cols.append(j)
    rp = np.searchsorted(np.array(rows), np.arange(m + 1)).astype(np.int32)
    S = 2
    nnz = len(cols)
    A = np.ones((S, nnz))
    b = ScenarioBatch(["a", "b"], rp, np.array(cols, np.int32), A, np.ones((S, n)), np.zeros((S, n)),
                      np.full((S, n), 5.0), np.ones((S, m)), np.full((S, m), 3.0), np.zeros((S, n)), np.zeros(S),
                      np.arange(1, dtype=np.int32), np.zeros(1, np.int32), np.arange(1, dtype=np.int32),
                      np.zeros((S, 1), np.int32), ["ROOT"], np.full(S, 0.5), np.full((S, 1), 0.5))
    assert "k_solve_ipm_wave" in _src_kernel(b, 64)
