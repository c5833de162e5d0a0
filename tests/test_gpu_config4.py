"""Config 4 (aircond multistage) on the exact kernel instances bench.py times.

bench.py --model aircond runs bf 32 x 32 x 64 (65,536 scenarios, 1,057 non-leaf nodes) on
path 6, the batched interior point (the automatic choice; since round 5 the one-lane
k_solve_ipm, whose 524 B of spills per lane cost less than lane groups of 4, DESIGN.md
3.7).  The register PDHG kernel <3,3,1,4> at L = 8
in record mode (path 2, PHGPU_IPM=0) was the round-2 bench instance and stays tested.
Checks, all against the oracle's restatement of aircond.py:37-330
(tests/examples/aircond.py in the reference) with straight_tests.py:36 parameters and
rho = 1:

  * the path-2 instance pinned (PHGPU_LANES=8, PHGPU_REG_REC=1) on bf 4 x 3 x 2, against
    golden.json aircond432_rho1: trivial bound, W after 5 PH iterations, PH iterations to
    conv < 1e-4 within +-1 and the final per-node x̄;
  * the full 32 x 32 x 64 instance on path 6 and on path 2 against
    tests/golden/aircond_scale.json (make_golden_aircond.py): trivial bound over all
    65,536 Iter0 QPs, every 64th Iter0 objective, x̄ of all 1,057 nodes and conv for 3 PH
    iterations, every 64th scenario's W and E[obj] after them; each solve asserts the
    kernel that ran;
  * the full instance on path 6 run by ph_main to conv < 1e-2: the PH iteration count of
    iterk_loop's break (phbase.py:925-934) within +-1 of the oracle's
    (tests/golden/aircond_conv.json, make_golden_aircond.py --conv) and x̄ of every node at
    the break.

Tolerances (north_star): objectives 1e-5 relative, x̄ / W 1e-5 absolute, iterations +-1.
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "golden.json")))
SCALE_FILE = os.path.join(HERE, "golden", "aircond_scale.json")
CONV_FILE = os.path.join(HERE, "golden", "aircond_conv.json")
OBJ_REL = 1e-5
ABS = 1e-5
# bench.py AIRCOND_KW (straight_tests.py:36)
KW = {"Capacity": 200, "QuadShortCoeff": 0.3, "BeginInventory": 50, "mu_dev": 0, "sigma_dev": 40, "start_seed": 0}


def _aircond_ph(bf, iters, thresh, **extra):
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.examples import aircond
    from mpisppy_amd.sputils import create_nodenames_from_branching_factors
    S = int(np.prod(bf))
    opts = {"solver_name": "mi355x_pdhg", "PHIterLimit": iters, "defaultPHrho": 1.0, "convthresh": thresh,
            "verbose": False, "display_progress": False, "toc": False, "device": "cuda:0",
            "batch_creator": aircond.batch_creator}
    opts.update(extra)
    return PH(opts, aircond.scenario_names_creator(S), aircond.scenario_creator,
              scenario_creator_kwargs={"branching_factors": list(bf), **KW},
              all_nodenames=create_nodenames_from_branching_factors(list(bf)))


def _assert_path2_instance(ph):
    info = ph.engine.kernel_info()
    assert info["path"] == 2 and info["lanes"] == 8, info
    assert (info["KC"], info["ZC"], info["KR"], info["ZR"]) == (3, 3, 1, 4), info
    assert info["rec"] == 1, info


@pytest.fixture
def pinned_l8_record_mode():
    keep = {k: os.environ.get(k) for k in ("PHGPU_LANES", "PHGPU_REG_REC", "PHGPU_IPM")}
    os.environ["PHGPU_LANES"] = "8"
    os.environ["PHGPU_REG_REC"] = "1"
    os.environ["PHGPU_IPM"] = "0"
    yield
    for k, v in keep.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


def test_aircond432_on_the_path2_instance(gpu, pinned_l8_record_mode):
    g = GOLD["aircond432_rho1"]
    assert g["kwargs"] == KW and g["branching_factors"] == [4, 3, 2]
    ph = _aircond_ph([4, 3, 2], 5, 1e-10)
    conv, eobj, tb = ph.ph_main()
    _assert_path2_instance(ph)
    assert abs(tb - g["trivial_bound"]) <= OBJ_REL * abs(g["trivial_bound"]), (tb, g["trivial_bound"])
    err = np.abs(ph.W_array() - np.array(g["traj5"][4]["W"]))
    assert err.max() <= ABS, err.max()
    ph2 = _aircond_ph([4, 3, 2], 300, 1e-4)
    ph2.ph_main()
    _assert_path2_instance(ph2)
    assert ph2.converged and abs(ph2._PHIter - g["conv_1e-4_iter"]) <= 1, (ph2._PHIter, g["conv_1e-4_iter"])
    nx = ph2.xbar_by_node()
    for nd, v in g["node_xbar_final"].items():
        assert np.abs(nx[nd][:2] - np.array(v)).max() <= 1e-4, nd


def _assert_path6(ph, lds=True):
    """The bench's config-4 instance: path 6 (interior point), one lane per scenario at
    65,536 scenarios.  Its register-only module spills 516 B per lane (below IPM_SPILL_MAX:
    faster than lane groups of 4); with the slack reciprocals in LDS (the
    automatic choice for a module that spills, solve_ipm.inc ipm_prepare) 132 B."""
    info = ph.engine.kernel_info()
    assert info["path"] == 6, info
    ipm = ph.engine.ipm_info()
    assert ipm["compiled"] == 1 and ipm["off"] == 0 and ipm["scratch_bytes"] <= 1024, ipm
    assert int(ipm["lanes"]) == 1, ipm
    assert int(ipm["lds_slacks"]) == int(lds), ipm
    if lds:
        assert ipm["scratch_bytes"] <= 256, ipm


def _assert_path6_regs(ph):
    _assert_path6(ph, lds=False)


@pytest.fixture(params=["path6", "path6_regs", "path2"])
def config4_path(request):
    """path6: the automatic choice (what bench.py runs); path6_regs: PHGPU_IPM_LDS=0, the
    register-only module (slack reciprocals in registers and scratch); path2: PHGPU_IPM=0,
    the register PDHG kernel <3,3,1,4>, L = 8, record mode."""
    keep = {k: os.environ.get(k) for k in ("PHGPU_IPM", "PHGPU_IPM_LDS")}
    os.environ.pop("PHGPU_IPM_LDS", None)
    if request.param == "path2":
        os.environ["PHGPU_IPM"] = "0"
    else:
        os.environ.pop("PHGPU_IPM", None)
    if request.param == "path6_regs":
        os.environ["PHGPU_IPM_LDS"] = "0"
    yield request.param
    for k, v in keep.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


@pytest.mark.skipif(not os.path.exists(SCALE_FILE), reason="aircond_scale.json not generated")
def test_config4_aircond65536_vs_oracle(gpu, config4_path):
    check = {"path6": _assert_path6, "path6_regs": _assert_path6_regs}.get(config4_path, _assert_path2_instance)
    g = json.load(open(SCALE_FILE))
    assert g["kwargs"] == KW and g["rho"] == 1.0
    ph = _aircond_ph(g["branching_factors"], g["ph_iters"], -1.0)
    ph.PH_Prep()
    tb = ph.Iter0()
    assert (ph.engine.host("status") == 0).all()
    check(ph)
    assert abs(tb - g["trivial_bound"]) <= OBJ_REL * abs(g["trivial_bound"]), (tb, g["trivial_bound"])
    smp = np.array(g["sample"])
    obj0 = ph.engine.host("obj")[smp]
    rel = np.abs(obj0 - np.array(g["iter0_obj"])) / np.abs(np.array(g["iter0_obj"]))
    assert rel.max() <= OBJ_REL, (rel.max(), int(smp[rel.argmax()]))
    names = g["node_names"]
    for it in range(g["ph_iters"]):
        ph.Compute_Xbar()
        ph.Update_W()
        conv = ph.convergence_diff()
        nx = ph.xbar_by_node()
        got = np.array([nx[nd][:2] for nd in names])
        err = np.abs(got - np.array(g["xbar"][it]))
        assert err.max() <= ABS, (it, err.max(), names[int(err.max(1).argmax())])
        assert abs(conv - g["conv"][it]) <= ABS, (it, conv, g["conv"][it])
        ph.solve_loop(solver_options=ph.iterk_solver_options, gripe=True)
        assert (ph.engine.host("status") == 0).all()
        check(ph)
    W = ph.W_array()[smp]
    err = np.abs(W - np.array(g["W"]))
    assert err.max() <= ABS, (err.max(), int(smp[err.max(1).argmax()]))
    eobj = ph.Eobjective()
    assert abs(eobj - g["Eobj"]) <= OBJ_REL * abs(g["Eobj"]), (eobj, g["Eobj"])


@pytest.mark.skipif(not os.path.exists(CONV_FILE), reason="aircond_conv.json not generated")
def test_config4_aircond65536_iterations_to_convergence(gpu):
    """Config 4 on path 6 (the bench's kernel and interior-point constants) by ph_main to
    conv < 1e-2: the oracle's PH iteration count +-1 and x̄ of all 1,057 nodes at the break
    within 1e-5."""
    g = json.load(open(CONV_FILE))
    assert g["kwargs"] == KW and g["rho"] == 1.0
    want = g["break_iteration"]
    from mpisppy_amd.examples import aircond
    # (with the model's interior-point constants, as the bench runs config 4)
    ph = _aircond_ph(g["branching_factors"], want + 10, g["conv_thresh"], ipm_tuning=aircond.IPM_TUNING)
    ph.ph_main()
    _assert_path6(ph)
    assert ph.converged and abs(ph._PHIter - want) <= 1, (ph._PHIter, want, g["conv"][-3:])
    key = str(ph._PHIter)
    if key in g["xbar_last"]:
        nx = ph.xbar_by_node()
        got = np.array([nx[nd][:2] for nd in g["node_names"]])
        err = np.abs(got - np.array(g["xbar_last"][key]))
        assert err.max() <= ABS, (err.max(), g["node_names"][int(err.max(1).argmax())])
    if ph._PHIter == want:
        # W accumulates 14 iterations of rho (x - x̄): per-iteration x errors at the solves'
        # 1e-9 KKT tolerance add up to ~1e-5 on entries of size ~10 (|W| <= 9.4 here), so
        # this one is checked relative to max(1, |W|)
        W = ph.W_array()[np.array(g["W_sample"])]
        ref = np.array(g["W_break"])
        err = np.abs(W - ref) / np.maximum(1.0, np.abs(ref))
        assert err.max() <= ABS, (err.max(), np.abs(W - ref).max())


def test_ipm_tuning_reaches_the_module_and_is_checked(gpu):
    """phgpu_set_ipm_tuning: the definitions go into the handle's generated module (the
    config-4 constants change the iteration counts), bad names / values and a call after
    the module is built are refused."""
    from mpisppy_amd import _lib
    from mpisppy_amd.engine import PHEngine
    from mpisppy_amd.examples import aircond
    bf = [4, 8, 16]
    b = aircond.batch_creator(aircond.scenario_names_creator(int(np.prod(bf))), branching_factors=bf, **KW)
    its = []
    for tun in (None, aircond.IPM_TUNING):
        e = PHEngine(b, device="cuda:0")
        if tun:
            with pytest.raises(_lib.PhgpuError, match="not an IPM_ constant"):
                e.set_ipm_tuning({"NC": 3})
            with pytest.raises(_lib.PhgpuError, match="not a number"):
                _lib.check(e.lib.phgpu_set_ipm_tuning(e.h, b"IPM_WARM_T=abc"), "phgpu_set_ipm_tuning")
            e.set_ipm_tuning(tun)
        e.solve(_lib.default_options(eps_rel=1e-9), warm=False)
        assert e.kernel_info()["path"] == 6
        its.append(e.host("iters").copy())
        with pytest.raises(_lib.PhgpuError, match="already built"):
            e.set_ipm_tuning(aircond.IPM_TUNING)
        e.close()
    assert not np.array_equal(its[0], its[1])
