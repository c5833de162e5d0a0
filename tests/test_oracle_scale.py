"""Pin the vectorised farmer oracle (oracle/farmer_vec.py) and the configuration-scale
fixtures it produced (tests/golden/farmer_scale.json, make_golden_scale.py).

  * Iter0 LP objectives and x against scipy's HiGHS on the explicit row model
    (oracle.models.farmer_scenario, a restatement of farmer.py:85-224 with no presolve);
  * PH subproblems against lpqp.farmer_prox_exact, the closed form that reproduces the
    reference's w_test_data fixtures (test_oracle_golden.py);
  * the committed fixtures against a fresh recomputation on their sampled scenarios.
"""
import json
import os
import warnings

import numpy as np
import pytest

from oracle import farmer_vec as fv
from oracle.lpqp import solve_lp_highs, farmer_prox_exact
from oracle.models import farmer_scenario, farmer_yields

HERE = os.path.dirname(os.path.abspath(__file__))
SCALE = json.load(open(os.path.join(HERE, "golden", "farmer_scale.json")))


@pytest.mark.parametrize("cm,names", [(1, [f"scen{i}" for i in list(range(0, 40)) + [65535, 40001]]),
                                      (10, [f"scen{i}" for i in range(0, 12)] + ["scen1023"]),
                                      (64, [f"scen{i}" for i in (3, 4, 5, 700, 2050)])])
def test_vec_lp_matches_highs(cm, names):
    warnings.simplefilter("ignore")
    bp, sl, f0 = fv.pieces(fv.yields(names, cm), cm)
    x, obj = fv.iter0_lp(bp, sl, f0, 500.0 * cm)
    for s, nm in enumerate(names):
        sc = farmer_scenario(nm, cm, num_scens=len(names))
        A, rl, ru, lb, ub, c, q = sc.arrays()
        xr, ob, st = solve_lp_highs(A, rl, ru, lb, ub, c)
        assert st == 0
        assert abs(ob - obj[s]) <= 1e-12 * abs(ob), (nm, ob, obj[s])
        if cm == 1 or extract_group(nm) > 0:   # scen0..2 at cm > 1: tied crop copies
            assert np.abs(xr[sc.nonant_indices()] - x[s]).max() <= 1e-8 * 500 * cm


def extract_group(nm):
    return int(nm[4:]) // 3


@pytest.mark.parametrize("cm", [2, 10])
def test_vec_lp_tied_copies_take_the_symmetric_point(cm):
    """scen0..2 at cm > 1: every copy of a crop has the same yields, the Iter0 optimum is a
    face; the oracle takes its symmetric point (equal acreage per copy), which is feasible
    and optimal (HiGHS objective) and equals cm copies of the cm = 1 solution scaled."""
    warnings.simplefilter("ignore")
    names = ["scen0", "scen1", "scen2"]
    bp, sl, f0 = fv.pieces(fv.yields(names, cm), cm)
    x, obj = fv.iter0_lp(bp, sl, f0, 500.0 * cm)
    bp1, sl1, f01 = fv.pieces(fv.yields(names, 1), 1)
    x1, obj1 = fv.iter0_lp(bp1, sl1, f01, 500.0)
    bases = [c.rstrip("0123456789") for c in fv.crops_sorted(cm)]
    for s in range(3):
        for k, b in enumerate(bases):
            assert abs(x[s, k] - x1[s, fv.crops_sorted(1).index(b + "0")]) <= 1e-9, (s, k)
        assert abs(obj[s] - cm * obj1[s]) <= 1e-9 * abs(obj[s])
        assert x[s].sum() <= 500.0 * cm + 1e-9


def _group_sums(x, cm):
    """Per base crop, the sum over its cm copies (the face-invariant part of a tied x)."""
    bases = [c.rstrip("0123456789") for c in fv.crops_sorted(cm)]
    return np.stack([x[..., [k for k, b in enumerate(bases) if b == g]].sum(-1) for g in ("CORN", "SUGAR_BEETS",
                                                                                          "WHEAT")], -1)


def test_tied_face_group_sums_are_solver_independent():
    """Config 2's scen0..2 (cm = 10, identical crop copies): a simplex basis (ties="vertex",
    what the reference's solvers return) and the symmetric point (ties="symmetric", the
    fixtures' and the interior point's) have the same objective and the same acreage per
    base crop, but different per-copy acreage -- so x̄ per copy after Iter0 is pinned only
    up to the face, and its per-crop group sums are the solver-independent comparison
    (tests/test_gpu_scale.py config 2 checks both).  Every later PH iterate depends on the
    choice (W per copy), which is why farmer_scale.json records the symmetric one."""
    warnings.simplefilter("ignore")
    names = [f"scen{i}" for i in range(1024)]
    bp, sl, f0 = fv.pieces(fv.yields(names, 10), 10)
    xs, os_ = fv.iter0_lp(bp, sl, f0, 5000.0, ties="symmetric")
    xv, ov = fv.iter0_lp(bp, sl, f0, 5000.0, ties="vertex")
    assert np.array_equal(xs[3:], xv[3:])               # no ties beyond scen0..2
    assert np.abs(os_ - ov).max() <= 1e-9 * np.abs(os_).max()
    assert np.abs(_group_sums(xs, 10) - _group_sums(xv, 10)).max() <= 1e-9
    assert np.abs(xs[:3] - xv[:3]).max() > 1.0           # the face is real
    xbar_s, xbar_v = xs.mean(0), xv.mean(0)
    assert np.abs(_group_sums(xbar_s, 10) - _group_sums(xbar_v, 10)).max() <= 1e-12 * 5000
    # the fixture's first x̄ is the symmetric choice
    g = SCALE["farmer1024_cm10"]
    assert np.abs(np.array(g["xbar"][0]) - xbar_s).max() <= 1e-9


@pytest.mark.parametrize("cm", [1, 10])
def test_vec_prox_matches_exact(cm):
    names = [f"scen{i}" for i in range(3, 23)]
    bp, sl, f0 = fv.pieces(fv.yields(names, cm), cm)
    rng = np.random.default_rng(cm)
    K = 3 * cm
    W = rng.normal(0, 40, (len(names), K))
    xbar = np.broadcast_to(500.0 * cm / K * rng.uniform(0.3, 1.7, K), W.shape)
    rho = rng.uniform(0.5, 2.0, (len(names), K))
    xv, ov = fv.prox(bp, sl, f0, W, xbar, rho, 500.0 * cm)
    cs = fv.crops_sorted(cm)
    for s, nm in enumerate(names):
        _, Y = farmer_yields(nm, cm)
        xe, oe = farmer_prox_exact(cs, Y, W[s], xbar[s], rho[s], cm)
        assert np.abs(xe - xv[s]).max() <= 1e-9, nm
        assert abs(oe - ov[s]) <= 1e-10 * abs(oe), nm


def test_fixture_iter0_samples_recompute():
    """Fixture Iter0 values are what the oracle gives for those scenarios (spot check)."""
    for key, names_of in (("farmer65536_cm1", lambda i: f"scen{i}"),
                          ("farmer1024_cm10", lambda i: f"scen{i}"),
                          ("farmer2048_cm64", lambda i: SCALE["farmer2048_cm64"]["names"][i])):
        g = SCALE[key]
        cm = g["crops_multiplier"]
        idx = g["sample"][::max(1, len(g["sample"]) // 8)]
        names = [names_of(i) for i in idx]
        bp, sl, f0 = fv.pieces(fv.yields(names, cm), cm)
        x, obj = fv.iter0_lp(bp, sl, f0, 500.0 * cm)
        want = np.array(g["iter0_obj"])[[g["sample"].index(i) for i in idx]]
        assert np.allclose(obj, want, rtol=1e-14, atol=0.0), key


def test_fixture_headline_bound_is_the_30_scenario_model():
    """The config-3 trivial bound sits where the pinned small-case bounds put it: the
    same model and solver reproduce test_aph.py's -137846 on Scenario1..30."""
    names = [f"Scenario{i + 1}" for i in range(30)]
    ph = fv.FarmerVecPH(names, 1)
    assert round(ph.iter0()) == -137846
    g = SCALE["farmer65536_cm1"]
    assert g["S"] == 65536 and len(g["xbar"]) == 5 and len(g["W"]) == len(g["sample"]) == 1024
    assert -140000 < g["trivial_bound"] < -137000


def test_cm64_fixture_set_is_well_conditioned():
    g = SCALE["farmer2048_cm64"]
    bp, sl, _ = fv.pieces(fv.yields(g["names"], 64), 64)
    assert fv.lp_margin(bp, sl, 32000.0).min() >= 1e-2
    t = SCALE["farmer_cm64_neartie"]
    assert "scen411" in t["names"] and max(t["margin"]) < 1e-3
