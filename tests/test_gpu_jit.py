"""Path 5: the pattern-specialised kernel compiled at run time with hipRTC (csrc/solve_jit.inc,
jit_kernel.hip.in).  It runs solve_reg.inc's algorithm with one lane per scenario and the
pattern baked in, so it is checked against the same oracle and fixtures as the other paths:

  * the reference's farmer fixtures (w_test_data: W and x̄ after 5 PH iterations);
  * config 3's headline fixture on the full 65,536 scenarios (trivial bound, 1,024 Iter0
    objectives, x̄ and conv of 5 iterations, sampled W, E[obj]);
  * aircond bf 4-3-2 (multistage, a diagonal quadratic in the model, equality rows):
    trivial bound, W after 5 iterations, iterations to 1e-4 within +-1;
  * random LP / QP batches with ranged, equality, one-sided and free rows and infinite
    bounds against HiGHS / the IPM, and a warm restart;
  * PDLP-style infeasibility / unboundedness certificates;
  * the speculative solve's warm-state slots (bit-identical PH with and without it).
Tolerances (north_star): objectives 1e-5 relative, x̄ / W 1e-5 absolute, iterations +-1.
"""
import numpy as np
import pytest

from test_gpu_parity import _ph, _random_lp_batch, GOLD, OBJ_REL, ABS
from test_gpu_scale import SCALE, _farmer_ph, _run_and_compare, _tiny_batch

pytestmark = pytest.mark.gpu
K5 = {"kernel": 5}


def test_farmer3_reference_fixtures_on_path5(gpu):
    from mpisppy_amd.examples import farmer
    names = farmer.scenario_names_creator(3)
    ph = _ph(names, farmer.scenario_creator, {"num_scens": 3}, iter0_solver_options=dict(K5),
             iterk_solver_options=dict(K5))
    conv, eobj, tb = ph.ph_main()
    assert ph.engine.kernel_info()["jit_wpe"] >= 1
    g = GOLD["farmer3_rho1"]
    assert abs(tb - g["trivial_bound"]) <= OBJ_REL * abs(g["trivial_bound"])
    assert np.abs(ph.W_array() - np.array(g["traj"][4]["W"])).max() <= ABS
    assert np.abs(ph.xbar_by_node()["ROOT"][:3] - np.array(g["traj"][4]["xbar"])).max() <= ABS


def test_headline_farmer65536_on_path5(gpu):
    from mpisppy_amd.examples import farmer
    g = SCALE["farmer65536_cm1"]
    names = [f"scen{i}" for i in range(65536)]
    ph = _farmer_ph(names, 1, 65536, iter0_solver_options=dict(K5),
                    iterk_solver_options={**farmer.PDHG_ITERK_OPTIONS, **K5})
    _run_and_compare(ph, g)
    assert ph.engine.kernel_info()["jit_wpe"] >= 1


def test_aircond432_on_path5(gpu):
    from mpisppy_amd.examples import aircond
    from mpisppy_amd.sputils import create_nodenames_from_branching_factors
    g = GOLD["aircond432_rho1"]
    kw = dict(g["kwargs"])
    kw["branching_factors"] = g["branching_factors"]
    nodes = create_nodenames_from_branching_factors(g["branching_factors"])
    ph = _ph(g["names"], aircond.scenario_creator, kw, iters=5, all_nodenames=nodes,
             batch_creator=aircond.batch_creator, iter0_solver_options=dict(K5), iterk_solver_options=dict(K5))
    conv, eobj, tb = ph.ph_main()
    assert abs(tb - g["trivial_bound"]) <= OBJ_REL * abs(g["trivial_bound"])
    assert np.abs(ph.W_array() - np.array(g["traj5"][4]["W"])).max() <= ABS
    ph2 = _ph(g["names"], aircond.scenario_creator, kw, iters=300, thresh=1e-4, all_nodenames=nodes,
              batch_creator=aircond.batch_creator, iter0_solver_options=dict(K5), iterk_solver_options=dict(K5))
    ph2.ph_main()
    assert ph2.converged and abs(ph2._PHIter - g["conv_1e-4_iter"]) <= 1, (ph2._PHIter, g["conv_1e-4_iter"])


@pytest.mark.parametrize("S,with_q", [(1, False), (67, False), (130, True), (300, True)])
def test_random_batches_on_path5(gpu, S, with_q):
    from mpisppy_amd.engine import PHEngine
    from mpisppy_amd import _lib
    from oracle.lpqp import solve_lp_highs, solve_qp_ipm
    b = _random_lp_batch(S, 9, 6, 0.5, seed=S + 7, with_q=with_q)
    e = PHEngine(b, device="cuda:0")
    e.solve(_lib.default_options(kernel=5), warm=False)
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
    # the same problems on the runtime-pattern kernels agree
    e.solve(_lib.default_options(kernel=1), warm=False)
    o1 = e.host("obj")
    assert np.all(np.abs(o1 - obj) <= OBJ_REL * np.maximum(1.0, np.abs(o1)))
    # warm restart on path 5 from path 1's answer
    e.solve(_lib.default_options(kernel=5), warm=True)
    assert np.abs(e.host("obj") - obj).max() <= 1e-6 * max(1.0, np.abs(obj).max())
    e.close()


@pytest.mark.parametrize("kind,code", [("primal", 2), ("dual", 3)])
def test_path5_certifies_infeasibility(gpu, kind, code):
    from mpisppy_amd.engine import PHEngine
    from mpisppy_amd import _lib
    S, bad = 70, 37
    e = PHEngine(_tiny_batch(S, bad, kind), device="cuda:0")
    e.solve(_lib.default_options(kernel=5), warm=False)
    st, it, obj = e.host("status"), e.host("iters"), e.host("obj")
    assert st[bad] == code and it[bad] <= 4096, (st[bad], it[bad])
    others = np.delete(np.arange(S), bad)
    assert (st[others] == _lib.OPTIMAL).all()
    assert np.isinf(obj[bad]) and (obj[bad] > 0) == (code == 2)
    assert np.abs(obj[others] + 8.0).max() <= 1e-6
    e.close()


def test_path5_speculative_solve_is_invisible(gpu):
    from test_gpu_speculative import _farmer, _run

    def make(spec):
        ph = _farmer(4096, spec, 3e-2)
        ph.options["iter0_solver_options"] = dict(K5)
        ph.options["iterk_solver_options"] = dict(K5)
        ph.iter0_solver_options.update(K5)
        ph.iterk_solver_options = dict(K5)
        return ph
    a, b = _run(make, True), _run(make, False)
    assert a["iter"] == b["iter"] and a["conv"] == b["conv"]
    for k in ("W", "xbar", "node_buf", "x", "x_after", "iters_after"):
        assert np.array_equal(a[k], b[k]), (k, np.abs(a[k] - b[k]).max())
