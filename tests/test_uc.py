"""Config 5 (UC LP relaxation) on the CPU: the .dat reader, the packed wind data, the
restated model's structure and its HiGHS optimum (tests/golden/uc.json; parity
UNPINNED -- the reference holds no UC results, see make_golden_uc.py)."""
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "uc.json")))
REF = "/root/reference/paperruns/larger_uc"


def test_dat_reader_forms():
    from mpisppy_amd.utils.datfile import parse_dat
    p, s = parse_dat("""# comment
param N := 3 ;
set G := a b c ;
set L[a] := 1 2 ;
set E[b] := ;
param: X Y :=
 a 1.5 -2
 b 2 3.25
;
param Z :=
W 1 0.5
W 2 7
;""")
    assert p["N"] == 3 and s["G"] == ["a", "b", "c"] and s["L[a]"] == [1, 2] and s["E[b]"] == []
    assert p["X"] == {"a": 1.5, "b": 2} and p["Y"] == {"a": -2, "b": 3.25}
    assert p["Z"] == {("W", 1): 0.5, ("W", 2): 7}


def test_root_node_data():
    from mpisppy_amd.examples import uc
    d, p = uc.load_data(1)
    assert len(d.gens) == 85 and d.T == 48 and d.buses == ["SingleBus"] and d.nd_gens == ["WIND"]
    assert d.pmin["BRIDGER_20_6333_C"] == 7.4025 and d.pmax["BRIDGER_20_6333_C"] == 29.61
    assert d.lags["BRIDGER_20_6333_C"] == [12, 14, 18] and d.lmp == 1e6
    assert all(d.reserve[t] == 20 for t in d.times)
    # MinimumProductionCost = first piecewise value x fuel cost (ReferenceModel_OK.py:603-611)
    g = "BRIDGER_20_6333_C"
    assert d.min_prod_cost[g] == pytest.approx(7709.70375 * 0.00227)


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference data not present")
def test_packed_root_data_matches_root_node_file():
    from mpisppy_amd.examples import uc
    assert uc._root_data(None) == uc._root_data(REF)


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference data not present")
def test_packed_wind_matches_node_files():
    from mpisppy_amd.examples import uc
    for k in (1, 17, 500, 1000):
        packed = uc.wind_bounds(k)
        files = uc.wind_bounds(k, path=os.path.join(REF, "1000scenarios_wind"))
        for i in (0, 1):
            assert packed[i] == {key: float(v) for key, v in files[i].items()}


def test_model_structure():
    from mpisppy_amd.examples import uc
    from collections import Counter
    b = uc.batch_creator(uc.scenario_names_creator(2), num_scens=1000)
    mdl = b.template
    assert (b.n, b.m, b.nnz, b.nn) == (GOLD["n"], GOLD["m"], GOLD["nnz"], GOLD["nn"])
    assert dict(Counter(v.name.split("[")[0] for v in mdl.vars)) == GOLD["var_families"]
    assert dict(Counter(r[3].split("[")[0] for r in mdl.rows)) == GOLD["row_families"]
    G, T = 85, 48
    fam = GOLD["var_families"]
    assert fam["UnitOn"] == G * T and fam["PowerGeneratedAboveMinimum"] == G * T
    # nonants: UnitOn[*,*] in sorted key order (uc_funcs.py:78-83, scenario_tree.py:39)
    names = [b.var_names[j] for j in b.nonant_col]
    keys = [(nm[7:-1].rsplit(",", 1)[0], int(nm[7:-1].rsplit(",", 1)[1])) for nm in names]
    assert keys == sorted(keys) and len(keys) == G * T
    # scenarios differ only in the wind bounds
    diff_c = np.nonzero((b.lb[0] != b.lb[1]) | (b.ub[0] != b.ub[1]))[0]
    assert set(b.var_names[j].split("[")[0] for j in diff_c) == {"NondispatchablePowerUsed"}
    assert np.array_equal(b.A_val[0], b.A_val[1]) and np.array_equal(b.c[0], b.c[1])
    # the production-cost rows of ReferenceModel_OK.py:1466-1470 repeat per segment: the
    # presolve keeps one copy
    assert b.m < GOLD["model_rows"]


def test_rho_setter():
    from mpisppy_amd.examples import uc
    mdl = uc.scenario_creator("Scenario1", num_scens=1000)
    rho = uc.rho_vector(mdl)
    assert np.all(rho >= 0) and rho.shape == (85 * 48,)
    assert np.allclose(rho[:50], GOLD["rho_first"]) and rho.sum() == pytest.approx(GOLD["rho_sum"])
    # uc_funcs.py:99-116 for one generator by hand: 0.1 x (cost at the midpoint output)
    d = mdl.uc
    g = "BRIDGER_20_6333_C"
    mid = d.pmin[g] + (d.pmax[g] - d.pmin[g]) / 2
    pts = d.pw_pts[g]                       # [0, 22.2075]: mid (absolute) is inside
    slope = d.slopes(g)[0]
    assert rho[0] == pytest.approx(0.1 * (slope * (mid - pts[0]) + d.min_prod_cost[g]))


def test_lp_optimum_vs_fixture():
    from mpisppy_amd.examples import uc
    from oracle import uc as ouc
    b = uc.batch_creator(["Scenario1", "Scenario2"], num_scens=1000)
    for s in range(2):
        x, obj, st = ouc.solve_lp(b, s)
        assert st == 0
        assert obj == pytest.approx(GOLD["lp_obj"][s], rel=1e-9)
        # the relaxation's commitment is mostly integral
        on = x[b.nonant_col]
        assert np.mean((on > 1e-6) & (on < 1 - 1e-6)) < 0.05


def test_uc_ph_oracle_fixture_consistent():
    """tests/golden/uc_ph.npz (oracle/uc_qp.py's three PH iterations on Scenario1..8): its
    Iter0 LP objectives agree with HiGHS (uc.json) to north_star's 1e-5 relative (1.8e-6 at
    worst: the two solvers' answers on these degenerate LPs), every solve reached a relative KKT
    error of 2e-8, and its PH state follows the PH updates
    (phbase.py:293-318): W_{k+1} - W_k = rho (x_k - x̄_k) sums to 0 over the scenarios."""
    import json
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "uc_ph.npz"))
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "uc.json")))
    assert list(d["names"]) == g["names"]
    rel = np.abs(d["iter0_obj"] - np.array(g["lp_obj"])) / np.abs(g["lp_obj"])
    assert rel.max() <= 1e-5, rel
    assert d["kkt"].max() <= 2e-8 and d["iter0_kkt"].max() <= 2e-8
    Ws = np.concatenate([d["W1"][None], d["W"]])
    for k in range(3):
        dW = Ws[k + 1] - Ws[k]
        assert np.abs(dW.sum(0)).max() <= 1e-9 * max(1.0, np.abs(dW).max())
    assert np.abs(d["W1"].sum(0)).max() <= 1e-9 * max(1.0, np.abs(d["W1"]).max())


def test_uc_qp_oracle_matches_dense_ipm_on_random_qps():
    """oracle/uc_qp.py (sparse Mehrotra IPM) against oracle/lpqp.py's dense IPM on small
    random LP / QP batches with every row and bound kind."""
    from oracle.lpqp import solve_qp_ipm
    from oracle.uc_qp import solve_qp
    rng = np.random.default_rng(0)
    for trial in range(5):
        m, n = 8, 12
        A = rng.standard_normal((m, n)) * (rng.random((m, n)) < 0.5)
        x0 = rng.random(n)
        ax = A @ x0
        rl, ru = ax - rng.random(m), ax + rng.random(m)
        rl[:2] = ru[:2] = ax[:2]
        rl[2] = -np.inf
        lb, ub = np.zeros(n), np.full(n, 2.0)
        ub[3], lb[4] = np.inf, -np.inf
        c = rng.standard_normal(n)
        q = np.where(rng.random(n) < 0.5, rng.random(n), 0.0)
        r = solve_qp(A, rl, ru, lb, ub, c, q)
        xr, ob, st = solve_qp_ipm(A, rl, ru, lb, ub, c, q)
        assert r["status"] == 0 and st == 0
        assert abs(r["obj"] - ob) <= 1e-8 * (1 + abs(ob)), (trial, r["obj"], ob)
        assert np.abs(r["x"] - xr).max() <= 1e-6, trial
