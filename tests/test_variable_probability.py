"""Variable probabilities (spbase.py:394-497, phbase.py:54-79 and 315-318): per-nonant
probability coefficients replace the node's prob_coeff in the x̄ sums, W is masked where a
coefficient is 0, and every nonant's coefficients must sum to 1 over its node.

CPU: the setter on the reference's callable interface ((id(vardata), prob) pairs, as
examples/sizes/special_sizes.py:61-80), the batch_creator array form, the sum check, and the
oracle restatement (with the node coefficients it reproduces the plain oracle).  GPU: PH on
farmer and on aircond 4-3-2 (a stage-2 nonant) through the engine's reduce / update path
(phgpu_set_nonant_probs) against the oracle, W exactly 0 where the probability is 0.
"""
import numpy as np
import pytest

from oracle.models import aircond_scenario, farmer_scenario, farmer_yields
from oracle.ph import OraclePH

OBJ_REL = 1e-5
ABS = 1e-5


def _farmer_varprob(mdl):
    """scen0 carries no probability on the first nonant (DevotedAcreage of the first crop in
    nonant order), scen1 / scen2 half each -- the sizes example's pattern."""
    v = mdl._mpisppy_node_list[0].nonant_vardata_list[0]
    return [(id(v), 0.0 if mdl.name == "scen0" else 0.5)]


def _farmer_ph(iters=5, vp=_farmer_varprob, **extra):
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.examples import farmer
    opts = {"solver_name": "mi355x_pdhg", "PHIterLimit": iters, "defaultPHrho": 1.0, "convthresh": -1.0,
            "verbose": False, "display_progress": False, "toc": False, "device": "cuda:0"}
    opts.update(extra)
    return PH(opts, farmer.scenario_names_creator(3), farmer.scenario_creator,
              scenario_creator_kwargs={"num_scens": 3}, variable_probability=vp)


def _farmer_expected_vp():
    vp = np.full((3, 3), 1.0 / 3.0)
    vp[:, 0] = [0.0, 0.5, 0.5]
    return vp


def test_setter_builds_coefficients_and_mask():
    ph = _farmer_ph()
    np.testing.assert_allclose(ph.var_prob, _farmer_expected_vp(), rtol=0, atol=1e-15)
    assert ph.prob0_mask.tolist() == (_farmer_expected_vp() != 0).astype(float).tolist()


def test_probability_sum_is_checked():
    def bad(mdl):
        v = mdl._mpisppy_node_list[0].nonant_vardata_list[1]
        return [(id(v), 0.5)]                    # 1.5 over the three scenarios
    with pytest.raises(RuntimeError, match="conditional probability sum"):
        _farmer_ph(vp=bad)
    ph = _farmer_ph(vp=bad, do_not_check_variable_probabilities=True)
    assert ph.var_prob[0, 1] == 0.5


def test_batch_creator_takes_the_array():
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.examples import farmer
    opts = {"solver_name": "mi355x_pdhg", "PHIterLimit": 1, "defaultPHrho": 1.0, "convthresh": -1.0,
            "verbose": False, "display_progress": False, "toc": False, "batch_creator": farmer.batch_creator,
            "variable_probability_array": _farmer_expected_vp()}
    ph = PH(opts, farmer.scenario_names_creator(3), farmer.scenario_creator, scenario_creator_kwargs={"num_scens": 3})
    np.testing.assert_array_equal(ph.var_prob, _farmer_expected_vp())
    with pytest.raises(RuntimeError, match="per-scenario models"):
        PH(dict(opts, variable_probability_array=None), farmer.scenario_names_creator(3), farmer.scenario_creator,
           scenario_creator_kwargs={"num_scens": 3}, variable_probability=_farmer_varprob)


def _farmer_oracle(var_prob):
    names = ["scen0", "scen1", "scen2"]
    scens = [farmer_scenario(n, 1, num_scens=3) for n in names]
    crops_sorted = sorted(farmer_yields("scen0", 1)[0])
    return OraclePH(scens, 1.0, solver="farmer", var_prob=var_prob,
                    farmer_info=(crops_sorted, [farmer_yields(n, 1)[1] for n in names], 1))


def test_oracle_with_node_coefficients_is_the_plain_oracle():
    a = _farmer_oracle(None)
    b = _farmer_oracle(np.full((3, 3), 1.0 / 3.0))
    for o in (a, b):
        o.iter0()
        o.iterk_loop(5, -1.0)
    np.testing.assert_array_equal(a.W, b.W)
    np.testing.assert_array_equal(a.xbar, b.xbar)


def test_oracle_weights_and_masks():
    o = _farmer_oracle(_farmer_expected_vp())
    o.iter0()
    o.compute_xbar()
    assert o.xbar[0, 0] == 0.5 * o.x[1, 0] + 0.5 * o.x[2, 0]      # scen0's weight is 0
    assert abs(o.xbar[0, 1] - o.x[:, 1].mean()) <= 1e-12 * abs(o.xbar[0, 1])
    o.iterk_loop(5, -1.0)
    assert o.W[0, 0] == 0.0 and np.abs(o.W[1:, 0]).max() > 0


@pytest.mark.gpu
def test_farmer_variable_probability_on_the_gpu(gpu):
    ph = _farmer_ph()
    conv, eobj, tb = ph.ph_main()
    o = _farmer_oracle(_farmer_expected_vp())
    otb = o.iter0()
    o.iterk_loop(5, -1.0)
    assert abs(tb - otb) <= OBJ_REL * abs(otb)
    W = ph.W_array()
    assert W[0, 0] == 0.0                                   # prob0_mask
    assert np.abs(W - o.W).max() <= ABS, (W, o.W)
    xb = ph.xbar_by_node()["ROOT"][:3]
    assert np.abs(xb - o.node_xbar["ROOT"]).max() <= ABS, (xb, o.node_xbar["ROOT"])
    assert abs(conv - o.conv) <= ABS, (conv, o.conv)


AIR_BF = [4, 3, 2]
AIR_KW = dict(Capacity=200, QuadShortCoeff=0.3, BeginInventory=50, mu_dev=0, sigma_dev=40, start_seed=0)


def _air_varprob(mdl):
    """A stage-2 nonant (the first of the scenario's second node, ROOT_i, which has 3 x 2 = 6
    scenarios below it): the first scenario of each such node carries none, the other five a
    fifth each."""
    v = mdl._mpisppy_node_list[1].nonant_vardata_list[0]
    k = int(mdl.name[4:])
    return [(id(v), 0.0 if k % 6 == 0 else 0.2)]


@pytest.mark.gpu
def test_aircond_stage2_variable_probability_on_the_gpu(gpu):
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.examples import aircond
    from mpisppy_amd.sputils import create_nodenames_from_branching_factors
    opts = {"solver_name": "mi355x_pdhg", "PHIterLimit": 5, "defaultPHrho": 1.0, "convthresh": -1.0,
            "verbose": False, "display_progress": False, "toc": False, "device": "cuda:0"}
    ph = PH(opts, aircond.scenario_names_creator(24), aircond.scenario_creator,
            scenario_creator_kwargs=dict(AIR_KW, branching_factors=AIR_BF),
            all_nodenames=create_nodenames_from_branching_factors(AIR_BF), variable_probability=_air_varprob)
    conv, eobj, tb = ph.ph_main()
    sc = [aircond_scenario(f"scen{i}", AIR_BF, **AIR_KW) for i in range(24)]
    o = OraclePH(sc, 1.0, var_prob=ph.var_prob)
    otb = o.iter0()
    o.iterk_loop(5, -1.0)
    assert abs(tb - otb) <= OBJ_REL * abs(otb)
    W = ph.W_array()
    assert (W[ph.var_prob == 0.0] == 0.0).all()
    assert np.abs(W - o.W).max() <= ABS, np.abs(W - o.W).max()
    nx = ph.xbar_by_node()
    for nd, v in o.node_xbar.items():
        assert np.abs(nx[nd][:len(v)] - v).max() <= ABS, nd


def test_aircond_stage2_setter_and_sum_check():
    """The multistage setter: a stage-2 nonant's coefficients sum to 1 over each ROOT_i's six
    scenarios (checked in the constructor); the other nonants keep their node coefficients."""
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.examples import aircond
    from mpisppy_amd.sputils import create_nodenames_from_branching_factors
    opts = {"solver_name": "mi355x_pdhg", "PHIterLimit": 1, "defaultPHrho": 1.0, "convthresh": -1.0,
            "verbose": False, "display_progress": False, "toc": False}
    ph = PH(opts, aircond.scenario_names_creator(24), aircond.scenario_creator,
            scenario_creator_kwargs=dict(AIR_KW, branching_factors=AIR_BF),
            all_nodenames=create_nodenames_from_branching_factors(AIR_BF), variable_probability=_air_varprob)
    b = ph.batch
    k2 = [k for k in range(b.nn) if b.nonant_depth[k] == 1]
    assert ph.var_prob[:, k2[0]].tolist() == [0.0 if s % 6 == 0 else 0.2 for s in range(24)]
    for k in range(b.nn):
        if k != k2[0]:
            np.testing.assert_allclose(ph.var_prob[:, k], b.prob_coeff[:, b.nonant_depth[k]])


@pytest.mark.gpu
def test_probabilities_set_after_a_path6_solve_drop_its_partials(gpu):
    """the path-6 epilogue x̄ partials of a solve are weighted with the node's
    prob_coeff; probabilities installed after that solve must not be reduced from them.
    Iter0 on 256 farmer scenarios (path 6 writes the partials), then per-nonant weights,
    then phgpu_ph_reduce: x̄ equals sum_s p_ks x_ks of the solved x."""
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.examples import farmer
    S = 256
    opts = {"solver_name": "mi355x_pdhg", "PHIterLimit": 1, "defaultPHrho": 1.0, "convthresh": -1.0,
            "verbose": False, "display_progress": False, "toc": False, "device": "cuda:0",
            "batch_creator": farmer.batch_creator}
    ph = PH(opts, farmer.scenario_names_creator(S), farmer.scenario_creator,
            scenario_creator_kwargs={"num_scens": S})
    ph.PH_Prep()
    ph.Iter0()
    e = ph.engine
    assert e.kernel_info()["path"] == 6
    x = e.nonant_x()                                   # [S, nn]
    rng = np.random.default_rng(3)
    vp = rng.random((S, x.shape[1]))
    vp[5, :] = 0.0
    vp /= vp.sum(0, keepdims=True)
    e.set_nonant_probs(vp)
    e.compute_xbar()
    xb = e.node_xbar()["ROOT"][:x.shape[1]]
    want = (vp * x).sum(0)
    assert np.abs(xb - want).max() <= 1e-9 * np.abs(want).max(), (xb, want)
    plain = x.mean(0)
    assert np.abs(xb - plain).max() > 1e-3            # the weights changed x̄ (not the stale partials)
