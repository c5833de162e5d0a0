"""Config 4 (aircond multistage) on the exact kernel instance bench.py times.

bench.py --model aircond runs bf 32 x 32 x 64 (65,536 scenarios, 1,057 non-leaf nodes) on
the register kernel <3,3,1,4> at L = 8 lanes per scenario in record mode (scenario-major
records, longest-first queue).  Two checks, both against the oracle's restatement of
aircond.py:37-330 (tests/examples/aircond.py in the reference) with straight_tests.py:36
parameters and rho = 1:

  * the same instance pinned (PHGPU_LANES=8, PHGPU_REG_REC=1) on bf 4 x 3 x 2, against
    golden.json aircond432_rho1: trivial bound, W after 5 PH iterations, PH iterations to
    conv < 1e-4 within +-1 and the final per-node x̄;
  * the full 32 x 32 x 64 instance against tests/golden/aircond_scale.json
    (make_golden_aircond.py): trivial bound over all 65,536 Iter0 QPs, every 64th Iter0
    objective, x̄ of all 1,057 nodes and conv for 3 PH iterations, every 64th scenario's W
    and E[obj] after them.

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


def _assert_bench_instance(ph):
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


def test_aircond432_on_the_bench_instance(gpu, pinned_l8_record_mode):
    g = GOLD["aircond432_rho1"]
    assert g["kwargs"] == KW and g["branching_factors"] == [4, 3, 2]
    ph = _aircond_ph([4, 3, 2], 5, 1e-10)
    conv, eobj, tb = ph.ph_main()
    _assert_bench_instance(ph)
    assert abs(tb - g["trivial_bound"]) <= OBJ_REL * abs(g["trivial_bound"]), (tb, g["trivial_bound"])
    err = np.abs(ph.W_array() - np.array(g["traj5"][4]["W"]))
    assert err.max() <= ABS, err.max()
    ph2 = _aircond_ph([4, 3, 2], 300, 1e-4)
    ph2.ph_main()
    _assert_bench_instance(ph2)
    assert ph2.converged and abs(ph2._PHIter - g["conv_1e-4_iter"]) <= 1, (ph2._PHIter, g["conv_1e-4_iter"])
    nx = ph2.xbar_by_node()
    for nd, v in g["node_xbar_final"].items():
        assert np.abs(nx[nd][:2] - np.array(v)).max() <= 1e-4, nd


@pytest.mark.skipif(not os.path.exists(SCALE_FILE), reason="aircond_scale.json not generated")
def test_config4_aircond65536_vs_oracle(gpu, register_path):
    g = json.load(open(SCALE_FILE))
    assert g["kwargs"] == KW and g["rho"] == 1.0
    ph = _aircond_ph(g["branching_factors"], g["ph_iters"], -1.0)
    ph.PH_Prep()
    tb = ph.Iter0()
    assert (ph.engine.host("status") == 0).all()
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
        _assert_bench_instance(ph)
    W = ph.W_array()[smp]
    err = np.abs(W - np.array(g["W"]))
    assert err.max() <= ABS, (err.max(), int(smp[err.max(1).argmax()]))
    eobj = ph.Eobjective()
    assert abs(eobj - g["Eobj"]) <= OBJ_REL * abs(g["Eobj"]), (eobj, g["Eobj"])
