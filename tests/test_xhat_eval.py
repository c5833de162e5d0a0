"""Xhat_Eval.evaluate / evaluate_one / fix_nonants_upto_stage (mpisppy/utils/xhat_eval.py).

Pinned by the reference's own tests (2 significant digits, round_pos_sig of
mpisppy/tests/utils.py):
  test_conf_int_farmer.py:168-202   farmer, names scen0..99, num_scens=10 (prob 1/10),
                                    xhat ROOT = (74, 245, 181): E = -1.3e6, scen0 = -4.8e4
  test_conf_int_aircond.py:216-240  aircond bf 4-3-2, start_seed 0, every node (200, 0):
                                    E = 1000, scen0 = 1100
CPU tests check the oracle against those numbers; GPU tests check the engine against
the oracle at 1e-5 relative (BASELINE.json north_star) and against the same numbers."""
import math

import numpy as np
import pytest

from oracle.models import aircond_scenario, create_nodenames_from_branching_factors, farmer_scenario
from oracle.wheel import xhat_objective

REL = 1e-5
FARMER_XHAT = {"ROOT": np.array([74.0, 245.0, 181.0])}
BFS = [4, 3, 2]


def round_pos_sig(x, sig=1):
    return round(x, sig - int(math.floor(math.log10(abs(x)))) - 1)


def _farmer_scens():
    return [farmer_scenario(f"scen{i}", 1, num_scens=10) for i in range(100)]


def _aircond():
    an = create_nodenames_from_branching_factors(BFS)
    scens = [aircond_scenario(f"scen{i}", BFS, start_seed=0) for i in range(24)]
    xhat = {nd: [200.0, 0.0] for nd in an}
    return an, scens, xhat


def test_oracle_farmer_evaluate_pinned():
    scens = _farmer_scens()
    assert round_pos_sig(xhat_objective(scens, FARMER_XHAT), 2) == -1300000.0
    assert round_pos_sig(xhat_objective(scens[:1], FARMER_XHAT) / scens[0].prob, 2) == -48000.0


def test_oracle_aircond_evaluate_pinned():
    an, scens, xhat = _aircond()
    assert round_pos_sig(xhat_objective(scens, xhat), 2) == 1000.0
    assert round_pos_sig(xhat_objective(scens[:1], xhat) / scens[0].prob, 2) == 1100.0


# ---------------------------------------------------------------- GPU
def _xe(creator, names, kw, an=None, solver_options=None):
    from mpisppy_amd.utils.xhat_eval import Xhat_Eval
    opts = {"iter0_solver_options": None, "iterk_solver_options": solver_options, "display_timing": False,
            "solver_name": "mi355x_pdhg", "verbose": False, "solver_options": solver_options, "toc": False,
            "device": "cuda:0"}
    return Xhat_Eval(opts, names, creator, scenario_denouement=None, all_nodenames=an,
                     scenario_creator_kwargs=kw)


@pytest.mark.gpu
@pytest.mark.parametrize("so", [None, {"kernel": 1}, {"gamma": 0.5}, {"kernel": 2}])
def test_xhat_eval_farmer(gpu, so):
    """Fixed nonants on every solve kernel: the register kernel (default / 2), the
    global-memory kernel (1) and another Halpern gamma (which runs on kernel 1); the
    global-memory kernel's KKT test must use the fixed working bounds."""
    from mpisppy_amd.examples import farmer
    names = farmer.scenario_names_creator(100)
    ev = _xe(farmer.scenario_creator, names, {"crops_multiplier": 1, "num_scens": 10}, solver_options=so)
    scens = _farmer_scens()
    E = ev.evaluate(FARMER_XHAT)
    oE = xhat_objective(scens, FARMER_XHAT)
    assert abs(E - oE) <= REL * abs(oE), (E, oE)
    assert round_pos_sig(E, 2) == -1300000.0
    o1 = ev.evaluate_one(FARMER_XHAT, names[0], None)
    oo1 = xhat_objective(scens[:1], FARMER_XHAT) / scens[0].prob
    assert abs(o1 - oo1) <= REL * abs(oo1), (o1, oo1)
    assert round_pos_sig(o1, 2) == -48000.0
    # calculate_incumbent fixes at the last solve's values: same point, same E
    assert (ev.engine.host("status") == 0).all()
    inc = ev.calculate_incumbent()
    assert inc is not None and abs(inc - E) <= REL * abs(E)


@pytest.mark.gpu
def test_xhat_eval_aircond(gpu):
    from mpisppy_amd.examples import aircond
    an, scens, xhat = _aircond()
    names = aircond.scenario_names_creator(24)
    ev = _xe(aircond.scenario_creator, names, {"branching_factors": BFS, "start_seed": 0}, an)
    E = ev.evaluate(xhat)
    oE = xhat_objective(scens, xhat)
    assert abs(E - oE) <= REL * abs(oE), (E, oE)
    assert round_pos_sig(E, 2) == 1000.0
    o1 = ev.evaluate_one(xhat, names[0], None)
    assert round_pos_sig(o1, 2) == 1100.0
    # stage-1 nonants only: the later stages are re-optimised per scenario
    ev.fix_nonants_upto_stage(1, {"ROOT": [200.0, 0.0]})
    ev.solve_loop(gripe=True)
    E1 = ev.Eobjective()
    oE1 = xhat_objective(scens, {"ROOT": [200.0, 0.0]})
    assert abs(E1 - oE1) <= REL * abs(oE1), (E1, oE1)
    assert E1 <= E + 1e-9 * abs(E)
    with pytest.raises(RuntimeError, match="Could not find"):
        ev.fix_nonants_upto_stage(2, {"ROOT": [200.0, 0.0]})
