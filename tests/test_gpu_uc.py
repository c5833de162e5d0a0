"""The shared-matrix streaming path (path 4, include/phgpu.h PHGPU_SHARED_MATRIX) on the
GPU: config 5 (UC LP relaxation) against HiGHS (tests/golden/uc.json -- parity UNPINNED,
see make_golden_uc.py), and path 4 against the other paths and the oracle on models
whose matrix is the same in every scenario (aircond, the tiny infeasibility batch)."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "uc.json")))
GOLDEN = json.load(open(os.path.join(HERE, "golden", "golden.json")))
UC_EPS = 1e-6          # the tolerance config 5 runs at (bench.py --model uc)
UC_OBJ_REL = 1e-5


def test_uc_lp_relaxation_vs_highs(gpu):
    from mpisppy_amd import _lib
    from mpisppy_amd.engine import PHEngine
    from mpisppy_amd.examples import uc
    names = GOLD["names"]
    b = uc.batch_creator(names, num_scens=GOLD["num_scens"])
    e = PHEngine(b, device="cuda:0")
    info = e.kernel_info()
    assert e.shared and info["path"] == 4, info
    e.solve(_lib.default_options(eps_rel=UC_EPS), warm=False)
    st, obj, bnd = e.host("status"), e.host("obj"), e.host("bound")
    assert (st == _lib.OPTIMAL).all(), (st, e.host("iters"))
    want = np.array(GOLD["lp_obj"])
    assert np.all(np.abs(obj - want) <= UC_OBJ_REL * np.abs(want)), (obj, want)
    assert np.all(np.abs(bnd - want) <= UC_OBJ_REL * np.abs(want)), (bnd, want)
    # the returned x is (nearly) feasible in the original units
    x = e.host("x")
    for s in range(2):
        A = b.dense_A(s) if b.n * b.m < 1e8 else None
        if A is None:
            from oracle import uc as ouc
            ax = ouc.scenario_matrix(b, s) @ x[s]
        else:
            ax = A @ x[s]
        scale = 1 + np.abs(np.where(np.isfinite(b.rl[s]), b.rl[s], 0)) + \
            np.abs(np.where(np.isfinite(b.ru[s]), b.ru[s], 0))
        viol = np.maximum(b.rl[s] - ax, 0) + np.maximum(ax - b.ru[s], 0)
        assert np.linalg.norm(viol) <= 1e-4 * np.linalg.norm(scale)
        assert np.all(x[s] >= b.lb[s] - 1e-7) and np.all(x[s] <= b.ub[s] + 1e-7)
    # warm start: the same answer, fewer iterations
    it0 = e.host("iters").copy()
    e.solve(_lib.default_options(eps_rel=UC_EPS), warm=True)
    assert np.all(np.abs(e.host("obj") - want) <= UC_OBJ_REL * np.abs(want))
    assert e.host("iters").max() < it0.max()
    e.close()


@pytest.mark.parametrize("tuned", [False, True])
def test_uc_ph_iterations(gpu, tuned):
    """Three PH iterations of config 5 on 8 scenarios (uc_funcs.py rho setter): every
    subproblem solved, W moves, the PH objective terms reach the kernel -- with the library's
    options and with the example's recommended PH-solve options (the bench's)."""
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.examples import uc
    names = GOLD["names"]
    rho = uc.rho_vector(uc.scenario_creator(names[0], num_scens=GOLD["num_scens"]))
    iterk = {"eps_rel": UC_EPS}
    if tuned:
        iterk.update(uc.PDHG_ITERK_OPTIONS)
    opts = {"solver_name": "mi355x_pdhg", "PHIterLimit": 3, "defaultPHrho": 1.0, "convthresh": -1.0,
            "verbose": False, "display_progress": False, "toc": False, "device": "cuda:0",
            "batch_creator": uc.batch_creator, "rho_array": rho,
            "iter0_solver_options": {"eps_rel": UC_EPS}, "iterk_solver_options": iterk}
    ph = PH(opts, names, uc.scenario_creator, scenario_creator_kwargs={"num_scens": len(names)})
    conv, eobj, tb = ph.ph_main()
    e = ph.engine
    assert e.kernel_info()["path"] == 4
    assert e.count_not_optimal() == 0
    # trivial bound = probability-weighted Iter0 LP bounds (8 scenarios, p = 1/8)
    want = np.mean(GOLD["lp_obj"])
    assert abs(tb - want) <= UC_OBJ_REL * abs(want), (tb, want)
    W = ph.W_array()
    assert np.abs(W).max() > 0 and np.isfinite(conv)
    # sum_s p_s W_s = 0 at every nonant (PH keeps the probability-weighted W at zero)
    assert np.abs(W.sum(axis=0)).max() <= 1e-6 * max(1.0, np.abs(W).max())


def test_path4_matches_default_path_on_aircond(gpu):
    """aircond has the same matrix in every scenario: solve it on path 4 and on the
    default path; then 5 PH iterations on path 4 against the oracle's W trajectory."""
    from mpisppy_amd import _lib
    from mpisppy_amd.engine import PHEngine
    from mpisppy_amd.examples import aircond
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.sputils import create_nodenames_from_branching_factors
    g = GOLDEN["aircond432_rho1"]
    kw = dict(g["kwargs"])
    kw["branching_factors"] = g["branching_factors"]
    names = g["names"]
    b = aircond.batch_creator(names, **kw)
    e2 = PHEngine(b, device="cuda:0", shared=False)
    e4 = PHEngine(b, device="cuda:0", shared=True)
    assert e4.kernel_info()["path"] == 4 and e2.kernel_info()["path"] != 4
    for e in (e2, e4):
        e.solve(_lib.default_options(), warm=False)
    assert (e4.host("status") == 0).all()
    o2, o4 = e2.host("obj"), e4.host("obj")
    assert np.all(np.abs(o2 - o4) <= 1e-7 * np.maximum(1.0, np.abs(o2)))
    assert np.abs(e2.host("x") - e4.host("x")).max() <= 1e-5
    with pytest.raises(_lib.PhgpuError, match="path 4 only"):
        e4.solve(_lib.default_options(kernel=2), warm=False)
    with pytest.raises(_lib.PhgpuError, match="path 4 only"):
        e2.solve(_lib.default_options(kernel=4), warm=False)
    e2.close()
    e4.close()
    opts = {"solver_name": "mi355x_pdhg", "PHIterLimit": 5, "defaultPHrho": 1.0, "convthresh": 1e-10,
            "verbose": False, "display_progress": False, "toc": False, "device": "cuda:0",
            "shared_matrix": True, "batch_creator": aircond.batch_creator}
    ph = PH(opts, names, aircond.scenario_creator, scenario_creator_kwargs=kw,
            all_nodenames=create_nodenames_from_branching_factors(g["branching_factors"]))
    conv, eobj, tb = ph.ph_main()
    assert ph.engine.kernel_info()["path"] == 4
    assert abs(tb - g["trivial_bound"]) <= 1e-5 * abs(g["trivial_bound"])
    assert np.abs(ph.W_array() - np.array(g["traj5"][4]["W"])).max() <= 1e-5


@pytest.mark.parametrize("kind,code", [("primal", 2), ("dual", 3)])
def test_path4_certifies_infeasibility(gpu, kind, code):
    """The tiny batch of test_gpu_scale.py (one matrix for all scenarios): the bad
    scenario's row range (primal) / cost (dual) is per-scenario data on path 4."""
    from mpisppy_amd import _lib
    from mpisppy_amd.engine import PHEngine
    from test_gpu_scale import _tiny_batch
    S, bad = 70, 37
    e = PHEngine(_tiny_batch(S, bad, kind), device="cuda:0", shared=True)
    assert e.kernel_info()["path"] == 4
    e.solve(_lib.default_options(), warm=False)
    st, it, obj = e.host("status"), e.host("iters"), e.host("obj")
    assert st[bad] == code and it[bad] <= 4096, (st[bad], it[bad])
    others = np.delete(np.arange(S), bad)
    assert (st[others] == _lib.OPTIMAL).all()
    assert np.isinf(obj[bad]) and (obj[bad] > 0) == (code == 2)
    assert np.abs(obj[others] + 8.0).max() <= 1e-6
    e.close()


def test_path4_fix_nonants(gpu):
    """phgpu_fix_nonants on a shared-matrix handle (the xhat evaluation of the
    spokes): fixing every nonant at a feasible point's values reproduces its objective
    through the per-scenario bound records; NULL restores the model bounds."""
    import torch
    from mpisppy_amd import _lib
    from mpisppy_amd.engine import PHEngine
    from mpisppy_amd.examples import aircond
    g = GOLDEN["aircond432_rho1"]
    kw = dict(g["kwargs"])
    kw["branching_factors"] = g["branching_factors"]
    b = aircond.batch_creator(g["names"], **kw)
    e = PHEngine(b, device="cuda:0", shared=True)
    e.solve(_lib.default_options(), warm=False)
    o_free = e.host("obj").copy()
    xfix = e.nonant_x_dev().clone()
    e.fix_nonants(0.5 * xfix)                      # another (feasible: overtime covers) first stage
    e.solve(_lib.default_options(), warm=True)
    assert (e.host("status") == 0).all()
    xn = e.nonant_x_dev()
    assert torch.allclose(xn, 0.5 * xfix, atol=1e-9)
    assert np.all(e.host("obj") >= o_free - 1e-7 * np.abs(o_free))
    e.fix_nonants(None)
    e.solve(_lib.default_options(), warm=True)
    assert np.all(np.abs(e.host("obj") - o_free) <= 1e-7 * np.maximum(1.0, np.abs(o_free)))
    e.close()


@pytest.mark.parametrize("split", [1, 3])
def test_uc_split_stragglers_vs_highs(gpu, split):
    """PHGPU_STREAM_SPLIT=T: the T longest scenarios of the previous solve (the first T of
    the queue order on a cold solve) run over the whole GPU in the split form of the
    streaming kernel (cooperative launch, grid barriers and grid sums), the rest on the
    queue: the same objectives as HiGHS, cold and warm."""
    from mpisppy_amd import _lib
    from mpisppy_amd.engine import PHEngine
    from mpisppy_amd.examples import uc
    keep = os.environ.get("PHGPU_STREAM_SPLIT")
    os.environ["PHGPU_STREAM_SPLIT"] = str(split)
    try:
        names = GOLD["names"]
        b = uc.batch_creator(names, num_scens=GOLD["num_scens"])
        e = PHEngine(b, device="cuda:0")
        assert e.shared and e.kernel_info()["path"] == 4
        want = np.array(GOLD["lp_obj"])
        for warm in (False, True):
            e.solve(_lib.default_options(eps_rel=UC_EPS), warm=warm)
            st, obj, bnd = e.host("status"), e.host("obj"), e.host("bound")
            assert (st == _lib.OPTIMAL).all(), (warm, st, e.host("iters"))
            assert np.all(np.abs(obj - want) <= UC_OBJ_REL * np.abs(want)), (warm, obj, want)
            assert np.all(np.abs(bnd - want) <= UC_OBJ_REL * np.abs(want)), (warm, bnd, want)
        e.close()
    finally:
        if keep is None:
            os.environ.pop("PHGPU_STREAM_SPLIT", None)
        else:
            os.environ["PHGPU_STREAM_SPLIT"] = keep


def test_path4_split_matches_queue_on_aircond(gpu):
    """The split form against the queue form on aircond (path 4 forced): statuses and
    objectives agree to the solve tolerance -- also with the grid barrier's counter started
    4,096 below 2^32 (PHGPU_SPLIT_BAR_BASE), so that it wraps within the first scenario
    (the barrier compares the signed distance to its target)."""
    from mpisppy_amd import _lib
    from mpisppy_amd.engine import PHEngine
    from mpisppy_amd.examples import aircond
    g = GOLDEN["aircond432_rho1"]
    kw = dict(g["kwargs"])
    kw["branching_factors"] = g["branching_factors"]
    b = aircond.batch_creator(g["names"], **kw)
    res = []
    for split, base in ((None, None), ("5", None), ("5", hex(2**32 - 4096))):
        if split:
            os.environ["PHGPU_STREAM_SPLIT"] = split
        if base:
            os.environ["PHGPU_SPLIT_BAR_BASE"] = base
        try:
            e = PHEngine(b, device="cuda:0", shared=True)
            assert e.kernel_info()["path"] == 4
            e.solve(_lib.default_options(eps_rel=1e-8), warm=False)
            res.append((e.host("status").copy(), e.host("obj").copy()))
            e.close()
        finally:
            os.environ.pop("PHGPU_STREAM_SPLIT", None)
            os.environ.pop("PHGPU_SPLIT_BAR_BASE", None)
    for st, ob in res[1:]:
        assert (res[0][0] == _lib.OPTIMAL).all() and (st == _lib.OPTIMAL).all()
        assert np.allclose(res[0][1], ob, rtol=1e-6, atol=1e-6), (res[0][1], ob)
    # the wrapped-counter run takes the same branches: bit-identical to the plain split run
    assert np.array_equal(res[1][1], res[2][1])


@pytest.mark.timeout(900)
@pytest.mark.parametrize("eps,obj_rel", [(UC_EPS, 5e-5), (2e-7, UC_OBJ_REL)])
def test_uc_ph_subproblems_vs_cpu_interior_point(gpu, eps, obj_rel):
    """Config 5's PH subproblems against an independent second-order solve:
    tests/golden/uc_ph.npz holds three PH iterations on Scenario1..8 solved by the sparse
    Mehrotra interior point of oracle/uc_qp.py (make_golden_uc_ph.py).  Each iteration installs
    the oracle's PH state (W_k, x̄_{k-1}) on the GPU engine, solves all 8 QPs on path 4 at
    config 5's eps_rel 1e-6, and compares:

      * the augmented PH objective of every QP: north_star's 1e-5 relative with the QPs
        solved to eps_rel 2e-7; at config 5's own eps_rel 1e-6 within 5e-5 (the relative KKT
        test bounds the primal residual by eps (1 + ||b||), and UC's loads put ||b|| at
        ~1e4: 3.4e-5 measured on Scenario5 of the first PH iteration);
      * the nonants in the rho-weighted norm the proximal term makes the QP strongly convex
        in: within twice sqrt(2 (objective gap)).  A per-nonant comparison is not well posed:
        uc_funcs.py's rho spans 1e-4 .. 11.6 and a nonant's distance to the optimum is only
        bounded by sqrt(2 gap / rho) -- at rho = 1e-4 a gap of 1e-6 of the objective leaves
        it free across [0, 1] (the oracle's own nonants move by 2.3e-2 between its KKT
        tolerances 1e-8 and 1e-10; x̄ of the GPU differed from the oracle's by 0.12 at eps 1e-6).

    Parity stays UNPINNED against the reference (it ships no UC output)."""
    from mpisppy_amd import _lib
    from mpisppy_amd.engine import PHEngine
    from mpisppy_amd.examples import uc
    d = np.load(os.path.join(HERE, "golden", "uc_ph.npz"))
    names = [str(v) for v in d["names"]]
    S = len(names)
    b = uc.batch_creator(names, num_scens=S)
    e = PHEngine(b, device="cuda:0")
    assert e.shared and e.kernel_info()["path"] == 4
    e.set_rho(d["rho"])
    e.set_terms(1, 1)
    Ws = [d["W1"], d["W"][0], d["W"][1]]
    xbs = [d["xbar0"], d["xbar"][0], d["xbar"][1]]
    nc = np.asarray(b.nonant_col)
    opts = dict(uc.PDHG_ITERK_OPTIONS)
    opts["eps_rel"] = eps
    for k in range(3):
        e.set_W(Ws[k])
        e.set_xbar(np.tile(xbs[k], (S, 1)))
        e.solve(_lib.default_options(**opts), warm=k > 0)
        st = e.host("status")
        assert (st == _lib.OPTIMAL).all(), (k, st)
        obj = e.host("obj")
        want = d["obj"][k]
        rel = np.abs(obj - want) / np.abs(want)
        assert rel.max() <= obj_rel, (k, rel.max(), obj, want)
        # the oracle's nonants of this iteration from its PH state: x_k = (W_{k+1} - W_k) / rho + x̄_k
        x = e.host("x")[:, nc]
        xo = (d["W"][k] - Ws[k]) / d["rho"] + d["xbar"][k]
        # strong convexity in the rho-norm: f(x) - f(x*) >= 1/2 ||x_N - x*_N||_rho^2, so two
        # solutions whose objectives agree to dobj sit within sqrt(2 (dobj_gpu + dobj_oracle))
        # of the optimum's nonants; dobj from the measured objective gap plus the oracle's
        # own 2e-6 relative (its LP objectives against HiGHS, test_uc.py)
        dist = np.sqrt((d["rho"] * (x - xo) ** 2).sum(1))
        bound = np.sqrt(2.0 * (np.abs(obj - want) + 2e-6 * np.abs(want))) * 2.0
        assert (dist <= bound).all(), (k, dist, bound)
    e.close()


def test_uc_cluster_form_matches_queue(gpu):
    """A batch smaller than the GPU (a rank's share of a strong-scaling run) runs in the
    cluster form of the streaming kernel: every scenario over K = capacity / S co-resident
    workgroups with cluster barriers and cluster sums (phgpu_stream_info).  Against the
    queue form (PHGPU_STREAM_CLUSTER=0, one workgroup per scenario slot) and HiGHS: the
    same objectives, cold and warm; the run with the clusters' barrier counters started
    4,096 below 2^32 (wrapping within the first scenario) is bit-identical to the plain one."""
    from mpisppy_amd import _lib
    from mpisppy_amd.engine import PHEngine
    from mpisppy_amd.examples import uc
    names = GOLD["names"]
    b = uc.batch_creator(names, num_scens=GOLD["num_scens"])
    want = np.array(GOLD["lp_obj"])
    res = {}
    for mode, env in (("queue", {"PHGPU_STREAM_CLUSTER": "0"}), ("cluster", {}),
                      ("cluster_wrap", {"PHGPU_SPLIT_BAR_BASE": hex(2**32 - 4096)})):
        keep = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            e = PHEngine(b, device="cuda:0")
            assert e.shared and e.kernel_info()["path"] == 4
            out = []
            for warm in (False, True):
                e.solve(_lib.default_options(eps_rel=UC_EPS), warm=warm)
                info = e.stream_info()
                assert info["path4"] == 1
                assert (info["cluster"] >= 2) == (mode != "queue"), (mode, info)
                st, obj, bnd = e.host("status"), e.host("obj"), e.host("bound")
                assert (st == _lib.OPTIMAL).all(), (mode, warm, st, e.host("iters"))
                assert np.all(np.abs(obj - want) <= UC_OBJ_REL * np.abs(want)), (mode, warm, obj, want)
                assert np.all(np.abs(bnd - want) <= UC_OBJ_REL * np.abs(want)), (mode, warm, bnd, want)
                out.append((obj.copy(), e.host("x").copy(), e.host("iters").copy()))
            res[mode] = out
            e.close()
        finally:
            for k, v in keep.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
    for (o1, x1, i1), (o2, x2, i2) in zip(res["cluster"], res["cluster_wrap"]):
        assert np.array_equal(o1, o2) and np.array_equal(x1, x2) and np.array_equal(i1, i2)
