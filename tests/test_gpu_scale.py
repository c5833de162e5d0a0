"""GPU parity at configuration scale, against the committed fixtures of
tests/golden/farmer_scale.json (oracle/farmer_vec.py, pinned in test_oracle_scale.py).

Tolerances (BASELINE.json north_star): objectives 1e-5 relative, x̄ / W 1e-5 absolute.
The headline test runs exactly the instance bench.py times: farmer, 65,536 scenarios,
cm = 1, the L = 4 register kernel <3,3,2,4>.
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
SCALE = json.load(open(os.path.join(HERE, "golden", "farmer_scale.json")))
OBJ_REL = 1e-5
ABS = 1e-5


def _farmer_ph(names, cm, num_scens, iters=5, **extra):
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.examples import farmer
    opts = {"solver_name": "mi355x_pdhg", "PHIterLimit": iters, "defaultPHrho": 1.0,
            "convthresh": -1.0, "verbose": False, "display_progress": False, "toc": False,
            "device": "cuda:0", "batch_creator": farmer.batch_creator}
    opts.update(extra)
    return PH(opts, names, farmer.scenario_creator,
              scenario_creator_kwargs={"crops_multiplier": cm, "num_scens": num_scens})


def _run_and_compare(ph, g):
    """Iter0 + g['ph_iters'] PH iterations of iterk_loop's body, compared per step."""
    ph.PH_Prep()
    tb = ph.Iter0()
    assert (ph.engine.host("status") == 0).all()
    smp = np.array(g["sample"])
    assert abs(tb - g["trivial_bound"]) <= OBJ_REL * abs(g["trivial_bound"]), (tb, g["trivial_bound"])
    obj0 = ph.engine.host("obj")[smp]
    want0 = np.array(g["iter0_obj"])
    rel0 = np.abs(obj0 - want0) / np.abs(want0)
    assert rel0.max() <= OBJ_REL, (rel0.max(), int(smp[rel0.argmax()]))
    for it in range(g.get("ph_iters", 0)):
        ph.Compute_Xbar()
        ph.Update_W()
        conv = ph.convergence_diff()
        xb = ph.xbar_by_node()["ROOT"][:len(g["xbar"][it])]
        assert np.abs(xb - np.array(g["xbar"][it])).max() <= ABS, (it, np.abs(xb - g["xbar"][it]).max())
        assert abs(conv - g["conv"][it]) <= ABS, (it, conv, g["conv"][it])
        ph.solve_loop(solver_options=ph.iterk_solver_options, gripe=True)
        assert (ph.engine.host("status") == 0).all()
    if g.get("ph_iters"):
        W = ph.W_array()[smp]
        err = np.abs(W - np.array(g["W"]))
        assert err.max() <= ABS, (err.max(), int(smp[err.max(1).argmax()]))
        eobj = ph.Eobjective()
        assert abs(eobj - g["Eobj"]) <= OBJ_REL * abs(g["Eobj"]), (eobj, g["Eobj"])
    return tb


def test_headline_farmer65536_cm1_register_path(gpu, register_path):
    """Config 3 on one GPU on the register path (the bench instance until round 3; path 6,
    the interior point, is tested on the same fixture in test_gpu_ipm.py), checked end to
    end (trivial bound, sampled Iter0 objectives, x̄ and conv of 5 PH iterations, sampled
    W, E[obj])."""
    g = SCALE["farmer65536_cm1"]
    names = [f"scen{i}" for i in range(65536)]
    from mpisppy_amd.examples import farmer
    # the bench's solver options too (examples/farmer.py PDHG_ITERK_OPTIONS)
    ph = _farmer_ph(names, 1, 65536, iterk_solver_options=dict(farmer.PDHG_ITERK_OPTIONS))
    ph._create_solvers()
    info = ph.engine.kernel_info()
    assert info["lanes"] == 4 and (info["KC"], info["ZC"], info["KR"], info["ZR"]) == (3, 3, 2, 4), info
    _run_and_compare(ph, g)
    # the bench's queue mode: scenario-major records, longest-first queue
    assert ph.engine.kernel_info()["rec"] == 1


def _bench_path(ph):
    """The kernel path of the handle's last solve (phgpu_kernel_info)."""
    return ph.engine.kernel_info()["path"]


def _group_sums(v, cm):
    """Per base crop, the sum over its cm copies (nonant order: crops sorted by name)."""
    from oracle.farmer_vec import crops_sorted
    bases = [c.rstrip("0123456789") for c in crops_sorted(cm)]
    return np.array([sum(v[k] for k, b in enumerate(bases) if b == g) for g in ("CORN", "SUGAR_BEETS", "WHEAT")])


def test_config2_farmer1024_cm10_bound(gpu):
    """Config 2 on the path bench.py times (the automatic choice): trivial bound, sampled
    Iter0 objectives, x̄ and conv of 5 PH iterations, every 8th scenario's W and E[obj]
    after them, for scen0..scen1023 at cm = 10.  scen0..2's Iter0 optimum is a face (tied
    crop copies): the first x̄'s per-crop group sums are the solver-independent check
    (test_oracle_scale.py::test_tied_face_group_sums_are_solver_independent); the per-copy
    values and the later iterates are pinned to the symmetric point of that face, the one
    an interior point converges to (a simplex solver, the reference's, returns a vertex)."""
    g = SCALE["farmer1024_cm10"]
    assert g["ph_iters"] == 5
    names = [f"scen{i}" for i in range(1024)]
    from mpisppy_amd.examples import farmer
    ph = _farmer_ph(names, 10, 1024, iterk_solver_options=dict(farmer.PDHG_ITERK_OPTIONS))
    first = []
    conv_diff = ph.convergence_diff

    def keep_first():
        v = conv_diff()
        if not first:
            first.append(ph.xbar_by_node()["ROOT"][:30].copy())
        return v
    ph.convergence_diff = keep_first
    _run_and_compare(ph, g)
    assert np.abs(_group_sums(first[0], 10) - _group_sums(np.array(g["xbar"][0]), 10)).max() <= ABS
    # the bench's kernel: path 6, the subtree interior point (k_solve_ipm_blk), no scratch
    ii = ph.engine.ipm_info()
    assert _bench_path(ph) == 6 and ii["kernel"] == 4 and ii["scratch_bytes"] == 0, (ph.engine.kernel_info(), ii)


@pytest.mark.parametrize("thr", ["0.01"])
def test_config2_ph_iterations_to_convergence(gpu, thr):
    """Config 2 run by ph_main to conv < thr: iterk_loop breaks at the oracle's PH
    iteration +-1 (phbase.py:925-934), with x̄ at that iteration within 1e-5."""
    g = SCALE["farmer1024_cm10"]
    want = g["breaks"][thr]
    names = [f"scen{i}" for i in range(1024)]
    from mpisppy_amd.examples import farmer
    ph = _farmer_ph(names, 10, 1024, iters=want["iteration"] + 20,
                    iterk_solver_options=dict(farmer.PDHG_ITERK_OPTIONS))
    ph.options["convthresh"] = float(thr)
    ph.ph_main()
    assert ph.converged
    assert abs(ph._PHIter - want["iteration"]) <= 1, (ph._PHIter, want["iteration"])
    xb = ph.xbar_by_node()["ROOT"][:30]
    ref = np.array(want["xbar"][str(ph._PHIter)])
    assert np.abs(xb - ref).max() <= ABS, np.abs(xb - ref).max()


def test_headline_instance_on_a_slice(gpu, register_path):
    """The same L = 4 <3,3,2,4> instance pinned on a 4,096-scenario slice
    (PHGPU_LANES=4): Iter0 objectives of every scenario in the slice."""
    g = SCALE["farmer65536_cm1"]
    os.environ["PHGPU_LANES"] = "4"
    try:
        names = [f"scen{i}" for i in range(0, 65536, 16)]
        ph = _farmer_ph(names, 1, len(names))
        ph._create_solvers()
        info = ph.engine.kernel_info()
    finally:
        del os.environ["PHGPU_LANES"]
    assert info["lanes"] == 4 and (info["KC"], info["KR"]) == (3, 2), info
    ph.PH_Prep()
    ph.Iter0()
    obj = ph.engine.host("obj")
    idx = [k for k, s in enumerate(range(0, 65536, 16)) if s in set(g["sample"])]
    want = np.array([g["iter0_obj"][g["sample"].index(s)] for s in range(0, 65536, 16) if s in set(g["sample"])])
    assert np.abs(obj[idx] - want).max() <= OBJ_REL * np.abs(want).max()


# ---------------------------------------------------------------- infeasibility
def _tiny_batch(S, bad, kind):
    """S copies of  min -x0 - 2 x1 + x2/2  s.t.  x0 + x1 <= 4 (row 0),  x0 - x2 <= 1
    (row 1),  x in [0, 10] x [0, 10] x [0, inf)  (optimum -8 at x = (0, 4, 0)).
    Scenario ``bad`` is made primal infeasible (x0 + x1 >= 25 > 20, the most the bounds
    allow) or unbounded (cost -1 on x2, which only row 1 bounds, and from below)."""
    from mpisppy_amd.batch import ScenarioBatch
    row_ptr = np.array([0, 2, 4], dtype=np.int32)
    col_idx = np.array([0, 1, 0, 2], dtype=np.int32)
    A = np.tile([1.0, 1.0, 1.0, -1.0], (S, 1))
    c = np.tile([-1.0, -2.0, 0.5], (S, 1))
    lb = np.zeros((S, 3))
    ub = np.tile([10.0, 10.0, np.inf], (S, 1))
    rl = np.tile([-np.inf, -np.inf], (S, 1))
    ru = np.tile([4.0, 1.0], (S, 1))
    if kind == "primal":
        rl[bad, 0], ru[bad, 0] = 25.0, np.inf
    else:
        c[bad, 2] = -1.0
    return ScenarioBatch([f"s{i}" for i in range(S)], row_ptr, col_idx, A, c, lb, ub, rl, ru,
                         np.zeros((S, 3)), np.zeros(S), np.array([0, 1], np.int32), np.zeros(2, np.int32),
                         np.array([0, 1], np.int32), np.zeros((S, 1), np.int32), ["ROOT"],
                         np.full(S, 1.0 / S), np.full((S, 1), 1.0 / S))


@pytest.mark.parametrize("kernel", [1, 2])
@pytest.mark.parametrize("kind,code", [("primal", 2), ("dual", 3)])
def test_infeasible_and_unbounded_scenarios_are_certified(gpu, kernel, kind, code):
    from mpisppy_amd.engine import PHEngine
    from mpisppy_amd import _lib
    S, bad = 70, 37
    e = PHEngine(_tiny_batch(S, bad, kind), device="cuda:0")
    e.solve(_lib.default_options(kernel=kernel), warm=False)
    st = e.host("status")
    it = e.host("iters")
    assert st[bad] == code, (st[bad], it[bad])
    assert it[bad] <= 4096, it[bad]            # certified within bounded iterations
    others = np.delete(np.arange(S), bad)
    assert (st[others] == _lib.OPTIMAL).all()
    obj = e.host("obj")
    assert np.isinf(obj[bad]) and (obj[bad] > 0) == (code == 2)
    assert np.abs(obj[others] + 8.0).max() <= 1e-6      # x = (0, 4, 0)
    e.close()


def test_iter0_raises_on_an_infeasible_scenario(gpu):
    """phbase.py:818-823: Iter0 stops when a scenario is infeasible."""
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.examples import farmer

    def creator(name, **kw):
        mdl = farmer.scenario_creator(name, **kw)
        if name == "scen2":
            # ConstrainTotalAcreage becomes sum x >= 2000, above 3 x 500 (the acreage bounds)
            r = mdl.rows[0]
            mdl.rows[0] = (r[0], 2000.0, float("inf"), r[3])
        return mdl

    opts = {"solver_name": "mi355x_pdhg", "PHIterLimit": 2, "defaultPHrho": 1.0, "convthresh": -1.0,
            "verbose": False, "display_progress": False, "toc": False, "device": "cuda:0"}
    ph = PH(opts, farmer.scenario_names_creator(3), creator, scenario_creator_kwargs={"num_scens": 3})
    with pytest.raises(RuntimeError, match="Infeasibility detected"):
        ph.ph_main()
    assert int(ph.engine.host("status")[2]) == 2


def test_max_iter_must_be_a_multiple_of_restart_every(gpu):
    from mpisppy_amd.engine import PHEngine
    from mpisppy_amd import _lib
    e = PHEngine(_tiny_batch(8, 0, "dual"), device="cuda:0")
    with pytest.raises(_lib.PhgpuError, match="multiples of restart_every"):
        e.solve(_lib.default_options(max_iter=1000, restart_every=16 * 3), warm=False)
    e.close()
