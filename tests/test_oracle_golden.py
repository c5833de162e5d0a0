"""The CPU oracle pinned against the reference's own fixtures and known answers."""
import csv
import json
import os
import warnings

import numpy as np
import pytest

from oracle.models import farmer_scenario, farmer_yields, aircond_scenario, extract_num
from oracle.ph import OraclePH, rank_slices
from oracle.lpqp import solve_lp_highs, solve_qp_ipm, farmer_prox_exact

warnings.simplefilter("ignore")
HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "golden.json")))


def _farmer_ph(names, cm=1, rho=1.0, num_scens=None, solver="farmer"):
    scens = [farmer_scenario(n, cm, num_scens=num_scens) for n in names]
    cs = sorted(farmer_yields(names[0], cm)[0])
    return OraclePH(scens, rho, solver=solver, farmer_info=(cs, [farmer_yields(n, cm)[1] for n in names], cm))


@pytest.mark.parametrize("solver", ["farmer", "ipm"])
def test_oracle_reproduces_reference_w_xbar_fixtures(solver):
    """mpisppy/tests/test_w_writer.py:85-117 + w_test_data/*.csv (5 places there;
    the oracle is within 1e-6 of every entry)."""
    names = [f"scen{i}" for i in range(3)]
    ph = _farmer_ph(names, num_scens=3, solver=solver)
    ph.iter0()
    ph.iterk_loop(5, 1e-10)
    nonants = ["DevotedAcreage[CORN0]", "DevotedAcreage[SUGAR_BEETS0]", "DevotedAcreage[WHEAT0]"]
    with open(os.path.join(HERE, "golden", "ref_w_file.csv")) as f:
        for row in csv.reader(f):
            s = names.index(row[0])
            k = nonants.index(row[1])
            assert abs(ph.W[s, k] - float(row[2])) <= 1e-6
    with open(os.path.join(HERE, "golden", "ref_xbar_file.csv")) as f:
        for row in csv.reader(f):
            assert abs(ph.xbar[0, nonants.index(row[0])] - float(row[1])) <= 1e-6
    # the asserted values of the reference test itself
    assert round(ph.W[0, 1], 5) == round(70.84705093609978, 5)
    assert round(ph.W[1, 0], 5) == round(-41.104251445950844, 5)


def test_trivial_bounds():
    names = [f"scen{i}" for i in range(3)]
    assert abs(_farmer_ph(names, num_scens=3).iter0() - (-115405.5555555)) < 1e-4
    # test_aph.py:230-253: Scenario1..30 -> 137846 to 3 significant digits
    names30 = [f"Scenario{i + 1}" for i in range(30)]
    tb = _farmer_ph(names30).iter0()
    assert round(-tb, -3) == 138000 and abs(tb - (-137846.178)) < 1e-2


def test_ph_converges_to_ef_optimum():
    """test_sc.py:30-38: EF optimum x = (CORN 80, SUGAR_BEETS 250, WHEAT 170)."""
    names = [f"scen{i}" for i in range(3)]
    ph = _farmer_ph(names, num_scens=3)
    ph.iter0()
    ph.iterk_loop(2000, 1e-9)
    assert np.allclose(ph.xbar[0], [80, 250, 170], atol=1e-3)


def test_golden_json_matches_oracle():
    g = GOLD["farmer3_rho1"]
    names = g["names"]
    ph = _farmer_ph(names, num_scens=3)
    assert abs(ph.iter0() - g["trivial_bound"]) < 1e-9
    ph.iterk_loop(10, 1e-12)
    for h, ref in zip(ph.history, g["traj"][:10]):
        assert np.abs(h["W"] - np.array(ref["W"])).max() < 1e-9
    assert g["conv_1e-4_iter"] == 94 and g["conv_1e-3_iter"] == 49


def test_ipm_matches_highs_on_lps_and_closed_form_on_qps():
    s = farmer_scenario("scen7", 2, num_scens=10)
    A, rl, ru, lb, ub, c, q = s.arrays()
    x1, o1, _ = solve_lp_highs(A, rl, ru, lb, ub, c)
    x2, o2, _ = solve_qp_ipm(A, rl, ru, lb, ub, c, q)
    assert abs(o1 - o2) <= 1e-8 * abs(o1)
    crops, Y = farmer_yields("scen7", 2)
    cs = sorted(crops)
    idx = s.nonant_indices()
    rng = np.random.default_rng(0)
    W = rng.normal(0, 50, 6)
    xb = rng.uniform(50, 200, 6)
    rho = np.full(6, 2.0)
    c2 = c.copy()
    q2 = q.copy()
    c2[idx] += W - rho * xb
    q2[idx] += rho
    x3, o3, _ = solve_qp_ipm(A, rl, ru, lb, ub, c2, q2)
    xf, of = farmer_prox_exact(cs, Y, W, xb, rho, 2)
    assert np.abs(x3[idx] - xf).max() < 1e-7
    assert abs(o3 + 0.5 * np.sum(rho * xb ** 2) - of) < 1e-6 * abs(of)


def test_aircond_golden_and_demands():
    g = GOLD["aircond432_rho1"]
    kw = g["kwargs"]
    sc = aircond_scenario("scen5", g["branching_factors"], **kw)
    assert [nd[0] for nd in sc.nodes] == ["ROOT", "ROOT_0", "ROOT_0_2"]
    assert sc.demands[0] == 200.0
    assert g["conv_1e-4_iter"] == 20


def test_rank_slices_match_reference_formula():
    assert rank_slices(3, 1) == [[0, 1, 2]]
    assert rank_slices(10, 3) == [[0, 1, 2], [3, 4, 5], [6, 7, 8, 9]]
    assert extract_num("scen0012") == 12


def test_ipm_does_not_cycle_on_ph_augmented_aircond_qp():
    """A PH subproblem of config 4 (aircond scen5371, PH iteration 3) on which Mehrotra's
    corrector cycled; with the centring safeguard the IPM converges, and lpqp.kkt_certify
    confirms the answer independently (feasible, signed multipliers, stationarity)."""
    import json
    from oracle.lpqp import solve_qp_ipm, kkt_certify
    g = json.load(open(os.path.join(HERE, "golden", "aircond_qp_cycling.json")))
    f = lambda k: np.where(np.abs(np.array(g[k])) >= g["inf_as"], np.sign(g[k]) * np.inf, g[k])  # noqa: E731
    A, rl, ru, lb, ub, c, q = (f(k) for k in ("A", "rl", "ru", "lb", "ub", "c", "q"))
    x, obj, st = solve_qp_ipm(A, rl, ru, lb, ub, c, q)
    assert st == 0
    pv, sv = kkt_certify(A, rl, ru, lb, ub, c, q, x)
    assert pv <= 1e-12 and sv <= 1e-12, (pv, sv)
    xb = x.copy()
    xb[0] += 1.0
    xb[2] += 1.0                      # still feasible (material balance), not optimal
    assert kkt_certify(A, rl, ru, lb, ub, c, q, xb)[1] > 1e-3
