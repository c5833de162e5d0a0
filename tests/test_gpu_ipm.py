"""Path 6: the batched interior-point solve (csrc/solve_ipm.inc, jit_ipm.hip.in), compiled
at run time with hipRTC for the handle's pattern and data, and the automatic path for
farmer cm = 1 (the headline, config 3).  Checked against the same oracle and fixtures as
the PDHG paths:

  * the reference's farmer fixtures (w_test_data: W and x̄ after 5 PH iterations);
  * config 3's headline fixture on the full 65,536 scenarios with the bench's options
    (trivial bound, 1,024 Iter0 objectives, x̄ and conv of 5 iterations, sampled W,
    E[obj]) -- the instance bench.py times;
  * aircond bf 4-3-2 (multistage, equality rows, a diagonal quadratic in the model);
  * random LP / QP batches with ranged, equality, one-sided and free rows and infinite
    bounds against HiGHS / the oracle's IPM (per-scenario data of every kind);
  * infeasible / unbounded scenarios: the IPM hands them to the path-5 PDHG fallback,
    which certifies them; the IPM iteration cap routes every scenario through the
    fallback and the answers stay the oracle's;
  * nonant fixing (Xhat evaluation) against the register path.
Tolerances (north_star): objectives 1e-5 relative, x̄ / W 1e-5 absolute, iterations +-1.
"""
import os

import numpy as np
import pytest

from test_gpu_parity import _ph, _random_lp_batch, GOLD, OBJ_REL, ABS
from test_gpu_scale import SCALE, _farmer_ph, _run_and_compare, _tiny_batch

pytestmark = pytest.mark.gpu
K6 = {"kernel": 6}


def _assert_path6(engine, scratch_free=True):
    info, ii = engine.kernel_info(), engine.ipm_info()
    assert ii["compiled"] == 1, ii
    if scratch_free:
        assert info["path"] == 6 and ii["scratch_bytes"] == 0 and ii["off"] == 0, (info, ii)


def test_farmer3_reference_fixtures_on_path6(gpu):
    from mpisppy_amd.examples import farmer
    names = farmer.scenario_names_creator(3)
    ph = _ph(names, farmer.scenario_creator, {"num_scens": 3})
    conv, eobj, tb = ph.ph_main()
    _assert_path6(ph.engine)
    g = GOLD["farmer3_rho1"]
    assert abs(tb - g["trivial_bound"]) <= OBJ_REL * abs(g["trivial_bound"])
    assert np.abs(ph.W_array() - np.array(g["traj"][4]["W"])).max() <= ABS
    assert np.abs(ph.xbar_by_node()["ROOT"][:3] - np.array(g["traj"][4]["xbar"])).max() <= ABS


def test_headline_farmer65536_on_path6(gpu):
    """Config 3 exactly as bench.py runs it (automatic path = 6, the example's options)."""
    from mpisppy_amd.examples import farmer
    g = SCALE["farmer65536_cm1"]
    names = [f"scen{i}" for i in range(65536)]
    ph = _farmer_ph(names, 1, 65536, iterk_solver_options=dict(farmer.PDHG_ITERK_OPTIONS))
    _run_and_compare(ph, g)
    _assert_path6(ph.engine)
    it = ph.engine.host("iters")
    assert it.max() <= 60, it.max()  # interior-point iterations, not PDHG ones


def test_aircond432_on_path6(gpu):
    from mpisppy_amd.examples import aircond
    from mpisppy_amd.sputils import create_nodenames_from_branching_factors
    g = GOLD["aircond432_rho1"]
    kw = dict(g["kwargs"])
    kw["branching_factors"] = g["branching_factors"]
    nodes = create_nodenames_from_branching_factors(g["branching_factors"])
    ph = _ph(g["names"], aircond.scenario_creator, kw, iters=5, all_nodenames=nodes,
             batch_creator=aircond.batch_creator, iter0_solver_options=dict(K6), iterk_solver_options=dict(K6))
    conv, eobj, tb = ph.ph_main()
    _assert_path6(ph.engine, scratch_free=False)
    assert abs(tb - g["trivial_bound"]) <= OBJ_REL * abs(g["trivial_bound"])
    assert np.abs(ph.W_array() - np.array(g["traj5"][4]["W"])).max() <= ABS
    ph2 = _ph(g["names"], aircond.scenario_creator, kw, iters=300, thresh=1e-4, all_nodenames=nodes,
              batch_creator=aircond.batch_creator, iter0_solver_options=dict(K6), iterk_solver_options=dict(K6))
    ph2.ph_main()
    assert ph2.converged and abs(ph2._PHIter - g["conv_1e-4_iter"]) <= 1, (ph2._PHIter, g["conv_1e-4_iter"])


@pytest.mark.parametrize("S,with_q", [(1, False), (67, False), (130, True), (300, True)])
def test_random_batches_on_path6(gpu, S, with_q):
    from mpisppy_amd.engine import PHEngine
    from mpisppy_amd import _lib
    from oracle.lpqp import solve_lp_highs, solve_qp_ipm
    b = _random_lp_batch(S, 9, 6, 0.5, seed=S + 7, with_q=with_q)
    e = PHEngine(b, device="cuda:0")
    e.solve(_lib.default_options(kernel=6), warm=False)
    st, obj, bnd, x = e.host("status"), e.host("obj"), e.host("bound"), e.host("x")
    assert (st == _lib.OPTIMAL).all(), st
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
    # the same problems on the runtime-pattern PDHG kernel agree
    e.solve(_lib.default_options(kernel=1), warm=False)
    o1 = e.host("obj")
    assert np.all(np.abs(o1 - obj) <= OBJ_REL * np.maximum(1.0, np.abs(o1)))
    e.close()


@pytest.mark.parametrize("kind,code", [("primal", 2), ("dual", 3)])
def test_path6_hands_infeasible_scenarios_to_the_pdhg(gpu, kind, code):
    from mpisppy_amd.engine import PHEngine
    from mpisppy_amd import _lib
    S, bad = 70, 37
    e = PHEngine(_tiny_batch(S, bad, kind), device="cuda:0")
    e.solve(_lib.default_options(kernel=6), warm=False)
    st, it, obj = e.host("status"), e.host("iters"), e.host("obj")
    assert st[bad] == code, (st[bad], it[bad])
    others = np.delete(np.arange(S), bad)
    assert (st[others] == _lib.OPTIMAL).all()
    assert np.isinf(obj[bad]) and (obj[bad] > 0) == (code == 2)
    assert np.abs(obj[others] + 8.0).max() <= 1e-6
    assert it[others].max() <= 60  # the IPM solved the others
    e.close()


def test_path6_fallback_for_every_scenario(gpu):
    """PHGPU_IPM_MAXIT=2: every scenario leaves the IPM unfinished and the path-5 PDHG
    solves the whole list (warm-started from the IPM's iterate); the answers are the
    oracle's (config 3's fixture on a 4,096-scenario slice)."""
    g = SCALE["farmer65536_cm1"]
    os.environ["PHGPU_IPM_MAXIT"] = "2"
    try:
        names = [f"scen{i}" for i in range(0, 65536, 16)]
        ph = _farmer_ph(names, 1, len(names))
        ph.PH_Prep()
        ph.Iter0()
        st, it, obj = ph.engine.host("status"), ph.engine.host("iters"), ph.engine.host("obj")
    finally:
        del os.environ["PHGPU_IPM_MAXIT"]
    assert (st == 0).all()
    assert it.min() > 2  # PDHG iteration counts: every scenario went through the fallback
    idx = [k for k, s in enumerate(range(0, 65536, 16)) if s in set(g["sample"])]
    want = np.array([g["iter0_obj"][g["sample"].index(s)] for s in range(0, 65536, 16) if s in set(g["sample"])])
    assert np.abs(obj[idx] - want).max() <= OBJ_REL * np.abs(want).max()


def test_path6_compile_failure_falls_back_to_the_pdhg_path(gpu):
    """A path-6 module that does not compile (here a broken macro definition injected by
    PHGPU_IPM_DEFS): the automatic choice turns path 6 off for the handle and solves on
    the handle's PDHG path with the same answers; kernel 6 asked for explicitly raises."""
    from mpisppy_amd.engine import PHEngine
    from mpisppy_amd.examples import farmer
    from mpisppy_amd import _lib
    S = 256
    b = farmer.batch_creator(farmer.scenario_names_creator(S), crops_multiplier=1, num_scens=S)
    ref = PHEngine(b, device="cuda:0")
    ref.solve(_lib.default_options(kernel=2, eps_rel=1e-10), warm=False)
    want = ref.host("obj").copy()
    ref.close()
    keep = os.environ.get("PHGPU_IPM_DEFS")
    os.environ["PHGPU_IPM_DEFS"] = "IPM_SIG_MAX=(0.05"   # unbalanced parenthesis: hipRTC fails
    try:
        e = PHEngine(b, device="cuda:0")
        with pytest.raises(_lib.PhgpuError):
            e.solve(_lib.default_options(kernel=6, eps_rel=1e-10), warm=False)
        e.solve(_lib.default_options(eps_rel=1e-10), warm=False)
        assert (e.host("status") == 0).all()
        assert e.ipm_info()["off"] == 2 and e.kernel_info()["path"] in (2, 5), (e.ipm_info(), e.kernel_info())
        assert np.abs(e.host("obj") - want).max() <= OBJ_REL * np.abs(want).max()
        e.close()
    finally:
        if keep is None:
            os.environ.pop("PHGPU_IPM_DEFS", None)
        else:
            os.environ["PHGPU_IPM_DEFS"] = keep


def test_path6_fixed_nonants_match_register_path(gpu):
    """Xhat-style evaluation: nonants fixed per scenario (phgpu_fix_nonants) on path 6 and
    on the register path give the same objectives; restoring the bounds restores the LP."""
    import torch
    from mpisppy_amd.engine import PHEngine
    from mpisppy_amd.examples import farmer
    from mpisppy_amd import _lib
    S = 512
    b = farmer.batch_creator(farmer.scenario_names_creator(S), crops_multiplier=1, num_scens=S)
    e = PHEngine(b, device="cuda:0")
    e.solve(_lib.default_options(kernel=6, eps_rel=1e-10), warm=False)
    base = e.host("obj").copy()
    rng = np.random.default_rng(3)
    xf = rng.uniform(20.0, 160.0, size=(b.nn, S))  # total acreage <= 480 < 500: always feasible
    xfix = torch.as_tensor(xf, device=e.device)
    _lib.check(e.lib.phgpu_fix_nonants(e.h, xfix.data_ptr(), None), "fix")
    got = {}
    for k in (6, 2):
        e.solve(_lib.default_options(kernel=k, eps_rel=1e-10), warm=False)
        assert (e.host("status") == 0).all()
        got[k] = e.host("obj").copy()
        assert np.abs(e.host("x")[:, b.nonant_col] - xf.T).max() <= 1e-7
    assert np.abs(got[6] - got[2]).max() <= OBJ_REL * np.abs(got[2]).max()
    _lib.check(e.lib.phgpu_fix_nonants(e.h, None, None), "restore")
    e.solve(_lib.default_options(kernel=6, eps_rel=1e-10), warm=False)
    assert np.abs(e.host("obj") - base).max() <= 1e-7 * np.abs(base).max()
    e.close()


@pytest.mark.parametrize("kernel,maxit", [(6, None), (6, "3"), (2, None)])
def test_solve_stats_match_the_outputs(gpu, kernel, maxit):
    """phgpu_solve_stats: path 6 accumulates the statistics in its kernels (IPM and
    fallback), the other paths reduce the outputs; both equal the host counts."""
    import torch
    from mpisppy_amd.engine import PHEngine
    from mpisppy_amd.examples import farmer
    from mpisppy_amd import _lib
    S = 3000
    b = farmer.batch_creator(farmer.scenario_names_creator(S), crops_multiplier=1, num_scens=S)
    e = PHEngine(b, device="cuda:0")
    if maxit:
        os.environ["PHGPU_IPM_MAXIT"] = maxit
    try:
        for warm in (False, True):
            e.solve(_lib.default_options(kernel=kernel), warm=warm)
            out = torch.zeros(6, dtype=torch.int64, device=e.device)
            _lib.check(e.lib.phgpu_solve_stats(e.h, out.data_ptr(), None), "stats")
            got = out.cpu().numpy()
            st, it = e.host("status"), e.host("iters")
            want = [int((st == k).sum()) for k in range(4)] + [int(it.sum()), int(it.max())]
            assert list(got) == want, (list(got), want)
    finally:
        os.environ.pop("PHGPU_IPM_MAXIT", None)
    e.close()


# ---------------------------------------------------------------- lane groups (ML_L > 1)
@pytest.fixture
def ipm_lanes(request):
    keep = os.environ.get("PHGPU_IPM_LANES")
    os.environ["PHGPU_IPM_LANES"] = str(request.param)
    yield request.param
    if keep is None:
        os.environ.pop("PHGPU_IPM_LANES", None)
    else:
        os.environ["PHGPU_IPM_LANES"] = keep


@pytest.mark.parametrize("ipm_lanes", [2, 4, 8, 16], indirect=True)
def test_lane_groups_farmer_slice_vs_fixture(gpu, ipm_lanes):
    """The multi-lane kernel (k_solve_ipm_ml) on config 3's fixture slice: Iter0 objectives,
    then 5 PH iterations against the same run on one lane per scenario (x̄ / W 1e-5)."""
    g = SCALE["farmer65536_cm1"]
    names = [f"scen{i}" for i in range(0, 65536, 16)]
    ph = _farmer_ph(names, 1, len(names))
    ph.PH_Prep()
    ph.Iter0()
    ii = ph.engine.ipm_info()
    assert ii["lanes"] == ipm_lanes and ii["compiled"] == 1, ii
    st, obj = ph.engine.host("status"), ph.engine.host("obj")
    assert (st == 0).all()
    idx = [k for k, s in enumerate(range(0, 65536, 16)) if s in set(g["sample"])]
    want = np.array([g["iter0_obj"][g["sample"].index(s)] for s in range(0, 65536, 16) if s in set(g["sample"])])
    assert np.abs(obj[idx] - want).max() <= OBJ_REL * np.abs(want).max()
    got = _five_iters(ph)
    os.environ["PHGPU_IPM_LANES"] = "1"
    ph1 = _farmer_ph(names, 1, len(names))
    ph1.PH_Prep()
    ph1.Iter0()
    assert ph1.engine.ipm_info()["lanes"] == 1
    ref = _five_iters(ph1)
    for k in ("xbar", "W"):
        assert np.abs(got[k] - ref[k]).max() <= ABS, (k, np.abs(got[k] - ref[k]).max())
    assert np.abs(got["conv"] - ref["conv"]).max() <= ABS


def _five_iters(ph):
    convs = []
    for _ in range(5):
        ph.Compute_Xbar()
        ph.Update_W()
        convs.append(ph.convergence_diff())
        ph.solve_loop(solver_options=ph.iterk_solver_options, gripe=True)
        assert (ph.engine.host("status") == 0).all()
    return {"xbar": ph.xbar_by_node()["ROOT"][:3].copy(), "W": ph.W_array().copy(), "conv": np.array(convs)}


@pytest.mark.parametrize("ipm_lanes", [4, 8], indirect=True)
def test_lane_groups_aircond432(gpu, ipm_lanes):
    from mpisppy_amd.examples import aircond
    from mpisppy_amd.sputils import create_nodenames_from_branching_factors
    g = GOLD["aircond432_rho1"]
    kw = dict(g["kwargs"])
    kw["branching_factors"] = g["branching_factors"]
    nodes = create_nodenames_from_branching_factors(g["branching_factors"])
    ph = _ph(g["names"], aircond.scenario_creator, kw, iters=5, all_nodenames=nodes,
             batch_creator=aircond.batch_creator, iter0_solver_options=dict(K6), iterk_solver_options=dict(K6))
    conv, eobj, tb = ph.ph_main()
    assert ph.engine.ipm_info()["lanes"] == ipm_lanes
    assert abs(tb - g["trivial_bound"]) <= OBJ_REL * abs(g["trivial_bound"])
    assert np.abs(ph.W_array() - np.array(g["traj5"][4]["W"])).max() <= ABS


@pytest.mark.parametrize("ipm_lanes", [4], indirect=True)
@pytest.mark.parametrize("S,with_q", [(67, False), (130, True)])
def test_lane_groups_random_batches(gpu, ipm_lanes, S, with_q):
    test_random_batches_on_path6(gpu, S, with_q)


@pytest.mark.parametrize("ipm_lanes", [8], indirect=True)
@pytest.mark.parametrize("kind,code", [("primal", 2), ("dual", 3)])
def test_lane_groups_hand_infeasible_scenarios_to_the_pdhg(gpu, ipm_lanes, kind, code):
    test_path6_hands_infeasible_scenarios_to_the_pdhg(gpu, kind, code)


@pytest.mark.parametrize("model,S,lanes", [("farmer", 8192, 8), ("farmer", 16384, 4), ("farmer", 32768, 1),
                                           ("aircond", 16384, 4), ("aircond", 32768, 1)])
def test_lane_policy_by_share(gpu, model, S, lanes):
    """ipm_lanes (solve_ipm.inc): lane groups of 8 for <= 8,192 local scenarios, of 4 for
    <= 16,384, one lane above -- also for aircond, whose one-lane module spills 524 B per
    lane (below IPM_SPILL_MAX: 0.315 ms per solve at 65,536 against 0.426 on lane groups of
    4); the lane-group modules stay scratch-free."""
    from mpisppy_amd import _lib
    from mpisppy_amd.engine import PHEngine
    from mpisppy_amd.examples import aircond, farmer
    if model == "farmer":
        b = farmer.batch_creator(farmer.scenario_names_creator(S), crops_multiplier=1, num_scens=S)
    else:
        kw = {"Capacity": 200, "QuadShortCoeff": 0.3, "BeginInventory": 50, "mu_dev": 0, "sigma_dev": 40,
              "start_seed": 0}
        b = aircond.batch_creator(aircond.scenario_names_creator(S), branching_factors=[S // 2048, 32, 64], **kw)
    e = PHEngine(b, device="cuda:0")
    e.solve(_lib.default_options(eps_rel=1e-9), warm=False)
    ii = e.ipm_info()
    assert e.kernel_info()["path"] == 6 and ii["lanes"] == lanes and ii["off"] == 0, ii
    assert ii["scratch_bytes"] == 0 if (lanes > 1 or model == "farmer") else 0 < ii["scratch_bytes"] <= 1024, ii
    assert (e.host("status") == 0).all()
    e.close()


def test_warm_start_cuts_iterations_same_answers(gpu):
    """The warm start (jit_ipm.hip.in IPM_WARM): a PH solve from the previous x / y needs
    fewer IPM iterations than from the cold start and reaches the same solutions (1e-5
    absolute on x, 1e-9 relative on the objectives, both against the exact oracle)."""
    from mpisppy_amd import _lib
    from mpisppy_amd.engine import PHEngine
    from mpisppy_amd.examples import farmer
    from oracle import farmer_vec as FV
    S = 4096
    names = farmer.scenario_names_creator(S)
    ph = FV.FarmerVecPH(names, 1)
    ph.iter0()
    ph.iterk_loop(2)
    b = farmer.batch_creator(names, crops_multiplier=1, num_scens=S)
    runs = {}
    for warm in (False, True):
        e = PHEngine(b, device="cuda:0")
        e.set_rho(ph.rho)
        e.solve(_lib.default_options(eps_rel=1e-9), warm=False)      # the state a PH solve starts from
        e.set_W(ph.W)
        e.set_xbar(ph.xbar)
        e.set_terms(1, 1)
        e.solve(_lib.default_options(eps_rel=1e-9), warm=warm)
        runs[warm] = (e.host("x")[:, b.nonant_col].copy(), e.host("obj").copy(), e.host("iters").copy(),
                      e.host("status").copy())
        e.close()
    xo, oo = FV.prox(ph.bp, ph.sl, ph.f0, ph.W, ph.xbar, ph.rho, ph.total)
    for warm, (x, obj, it, st) in runs.items():
        assert (st == 0).all()
        assert np.abs(x - xo).max() <= 1e-5, (warm, np.abs(x - xo).max())
        assert (np.abs(obj - oo) / np.abs(oo)).max() <= 1e-9
    assert runs[True][2].mean() < 0.8 * runs[False][2].mean(), (runs[True][2].mean(), runs[False][2].mean())


@pytest.mark.parametrize("ipm_lanes", [1, 4], indirect=True)
@pytest.mark.parametrize("S,with_q", [(67, False), (130, True)])
def test_warm_started_ph_terms_on_random_batches(gpu, ipm_lanes, S, with_q):
    """A PH-like warm-started solve (W and the prox term on the nonant columns, the start
    from the previous solve's x / y) on random batches with ranged, equality, one-sided and
    free rows and infinite bounds, one lane and lane groups: the same optima as the oracle's
    QP IPM on the W- and prox-augmented problems."""
    from mpisppy_amd.engine import PHEngine
    from mpisppy_amd import _lib
    from oracle.lpqp import solve_qp_ipm
    b = _random_lp_batch(S, 9, 6, 0.5, seed=S + 11, with_q=with_q)
    e = PHEngine(b, device="cuda:0")
    e.solve(_lib.default_options(kernel=6), warm=False)                 # Iter0
    rng = np.random.default_rng(S)
    nc = np.asarray(b.nonant_col)
    x0 = e.host("x")[:, nc]
    xbar = np.broadcast_to(x0.mean(0), x0.shape).copy()
    W = rng.normal(scale=0.3, size=x0.shape)
    rho = np.full(x0.shape, 0.7)
    e.set_rho(rho)
    e.set_W(W)
    e.set_xbar(xbar)
    e.set_terms(1, 1)
    e.solve(_lib.default_options(kernel=6), warm=True)                  # warm: from Iter0's x / y
    st, obj, x = e.host("status"), e.host("obj"), e.host("x")
    assert (st == _lib.OPTIMAL).all(), st
    assert e.ipm_info()["lanes"] == ipm_lanes
    for s in range(S):
        c = b.c[s].copy()
        q = b.q[s].copy()
        c[nc] += W[s] - rho[s] * xbar[s]
        q[nc] += rho[s]
        xr, ob, rc = solve_qp_ipm(b.dense_A(s), b.rl[s], b.ru[s], b.lb[s], b.ub[s], c, q)
        assert rc == 0
        ob += 0.5 * float(np.sum(rho[s] * xbar[s] ** 2))                 # the prox constant
        assert abs(obj[s] - ob) <= OBJ_REL * max(1.0, abs(ob)), (s, obj[s], ob)
        assert np.abs(x[s][nc] - xr[nc]).max() <= 1e-5 * (1 + np.abs(xr[nc]).max()), (s, x[s][nc], xr[nc])
    e.close()
