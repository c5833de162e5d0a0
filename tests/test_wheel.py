"""Hub-and-spoke cylinders: Lagrangian outer bound, xhat
shuffle inner bound, PHHub termination.

CPU tests: the scenario tree ranges and the xhat candidate walk against the oracle's
independent restatement of xhatshufflelooper_bounder.py:90-300.
GPU tests: the spokes' bounds through libphgpu.so against the oracle's exact solvers,
and a whole farmer wheel (hub + Lagrangian + xhatshuffle) against the oracle wheel.
Tolerance: objectives / bounds 1e-5 relative (BASELINE.json north_star)."""
import numpy as np
import pytest

from oracle.models import (aircond_scenario, create_nodenames_from_branching_factors, farmer_scenario,
                           farmer_yields)
from oracle.ph import OraclePH
from oracle.wheel import OracleWheel, candidate_sequence, lagrangian_bound, tree_ranges, xhat_objective

REL = 1e-5
FARMER_EF_OBJ = -108390.0     # farmer 3 scenarios EF optimum (test_sc.py:30-38: x* = 80/250/170)


def _cycler_seq(names, all_nodenames, count):
    import random
    from mpisppy_amd.cylinders.xhatshufflelooper_bounder import ScenarioCycler
    from mpisppy_amd.sputils import scenario_tree
    rng = random.Random()
    rng.seed(42)
    shuffled = rng.sample(list(enumerate(names)), len(names))
    tree = scenario_tree(all_nodenames, len(names))
    nonleaves = {nd: t for nd, t in tree.items() if not t.is_leaf or nd == "ROOT"}
    cyc = ScenarioCycler(shuffled, nonleaves, True, None)
    out = []
    while len(out) < count:
        d = cyc.get_next()
        if d is None:
            out.append(None)
            cyc.begin_epoch()
        else:
            out.append(dict(d))
    return out


def test_tree_ranges_match_oracle():
    from mpisppy_amd.sputils import scenario_tree
    for bfs in ([4, 3, 2], [3, 2], [2, 2, 2, 2]):
        an = create_nodenames_from_branching_factors(bfs)
        S = int(np.prod(bfs))
        t = scenario_tree(an, S)
        o = tree_ranges(an, S)
        nl = {nd: (v.scenfirst, v.scenlast) for nd, v in t.items() if not v.is_leaf}
        assert nl == {nd: (a, b) for nd, (a, b, _) in o.items()}
        assert list(nl)[0] == "ROOT"


@pytest.mark.parametrize("S", [3, 30, 257])
def test_xhat_candidate_walk_two_stage(S):
    names = [f"scen{i}" for i in range(S)]
    assert _cycler_seq(names, None, 3 * S + 3) == candidate_sequence(names, None, 3 * S + 3)


@pytest.mark.parametrize("bfs", [[4, 3, 2], [3, 3], [2, 2, 2, 2]])
def test_xhat_candidate_walk_multistage(bfs):
    an = create_nodenames_from_branching_factors(bfs)
    S = int(np.prod(bfs))
    names = [f"scen{i}" for i in range(S)]
    got = _cycler_seq(names, an, 3 * S)
    exp = candidate_sequence(names, an, 3 * S)
    assert got == exp


# ---------------------------------------------------------------- GPU
def _farmer_oracle(names, rho=1.0):
    scens = [farmer_scenario(n, 1, num_scens=len(names)) for n in names]
    crops = sorted(farmer_yields("scen0", 1)[0])
    return scens, OraclePH(scens, rho, solver="farmer",
                           farmer_info=(crops, [farmer_yields(n, 1)[1] for n in names], 1))


@pytest.mark.gpu
def test_lagrangian_bound_vs_oracle(gpu):
    """LagrangianOuterBound.lagrangian with a given W = sum_s p_s min (c_s + W_s) x (HiGHS)."""
    from mpisppy_amd.examples import farmer
    from mpisppy_amd.phbase import PHBase
    from mpisppy_amd.cylinders.lagrangian_bounder import LagrangianOuterBound
    names = farmer.scenario_names_creator(30)
    opts = {"solver_name": "mi355x_pdhg", "PHIterLimit": 1, "defaultPHrho": 1.0, "convthresh": 0.0,
            "verbose": False, "display_progress": False, "toc": False, "device": "cuda:0"}
    opt = PHBase(opts, names, farmer.scenario_creator, scenario_creator_kwargs={"num_scens": 30})
    sp = LagrangianOuterBound(opt)
    sp.main()
    scens = [farmer_scenario(n, 1, num_scens=30) for n in names]
    assert abs(sp.trivial_bound - lagrangian_bound(scens, np.zeros((30, 3)))) <= REL * abs(sp.trivial_bound)
    rng = np.random.default_rng(5)
    for trial in range(3):
        W = rng.normal(0.0, 30.0, (30, 3))
        W -= W.mean(0)                      # sum_s p_s W_s = 0, as PH keeps it
        opt.engine.set_W(W)
        b = sp.lagrangian()
        ob = lagrangian_bound(scens, W)
        assert abs(b - ob) <= REL * abs(ob), (trial, b, ob)


@pytest.mark.gpu
def test_xhat_eval_multistage_vs_oracle(gpu):
    """Xhat_Eval with per-node fixed values on aircond 4-3-2 (QP second stages)."""
    from mpisppy_amd.examples import aircond
    from mpisppy_amd.utils.xhat_eval import Xhat_Eval
    from mpisppy_amd.extensions.xhatbase import XhatBase
    import json
    import os
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))["aircond432_rho1"]
    bfs = g["branching_factors"]
    kw = dict(g["kwargs"])
    kw["branching_factors"] = bfs
    an = create_nodenames_from_branching_factors(bfs)
    names = g["names"]
    opts = {"solver_name": "mi355x_pdhg", "verbose": False, "toc": False, "device": "cuda:0"}
    xe = Xhat_Eval(opts, names, aircond.scenario_creator, all_nodenames=an, scenario_creator_kwargs=kw)
    xe._lazy_create_solvers()
    # candidate values: the Iter0 LP solution's nonants of the scenarios the walk picks
    xe.solve_loop(warm_start=False)
    xb = XhatBase(xe)
    cache = xe.engine.nonant_x_dev().clone()
    scens = [aircond_scenario(n, bfs, **{k: v for k, v in kw.items() if k != "branching_factors"}) for n in names]
    for cand in candidate_sequence(names, an, 4):
        if cand is None:
            continue
        obj = xb._try_one(cand, nonant_cache=cache)
        tab = xb.last_table.cpu().numpy()
        values = {nd: tab[g] for g, nd in enumerate(xe.engine.node_names)}
        oobj = xhat_objective(scens, values)
        assert oobj is not None and obj is not None
        assert abs(obj - oobj) <= REL * abs(oobj), (cand, obj, oobj)


@pytest.mark.gpu
def test_wheel_farmer3_vs_oracle_wheel(gpu):
    """WheelSpinner(ph_hub, [lagrangian, xhatshuffle]) on farmer 3 scenarios: per-iteration
    best bounds equal the oracle wheel's, same terminating iteration, and the inner bound
    reaches the EF optimum."""
    from types import SimpleNamespace
    from mpisppy_amd.examples import farmer
    from mpisppy_amd.spin_the_wheel import WheelSpinner
    from mpisppy_amd.utils import cfg_vanilla as vanilla
    names = farmer.scenario_names_creator(3)
    cfg = SimpleNamespace(solver_name="mi355x_pdhg", default_rho=1.0, max_iterations=200, rel_gap=1e-4,
                          intra_hub_conv_thresh=1e-10, device="cuda:0", toc=False)
    kw = {"num_scens": 3}
    hub = vanilla.ph_hub(cfg, farmer.scenario_creator, None, names, scenario_creator_kwargs=kw)
    spokes = [vanilla.lagrangian_spoke(cfg, farmer.scenario_creator, None, names, scenario_creator_kwargs=kw),
              vanilla.xhatshuffle_spoke(cfg, farmer.scenario_creator, None, names, scenario_creator_kwargs=kw)]
    trace = []
    ws = WheelSpinner(hub, spokes)
    from mpisppy_amd.cylinders import hub as hubmod
    orig = hubmod.PHHub.is_converged

    def spy(self):
        r = orig(self)
        trace.append((self.opt._PHIter, self.BestOuterBound, self.BestInnerBound))
        return r
    hubmod.PHHub.is_converged = spy
    try:
        ws.spin()
    finally:
        hubmod.PHHub.is_converged = orig
    scens, oph = _farmer_oracle(names)
    ow = OracleWheel(oph, names, rel_gap=1e-4)
    oo, oi = ow.run(200)
    assert len(trace) == len(ow.trace), (len(trace), len(ow.trace))
    for (it, ob, ib), r in zip(trace, ow.trace):
        assert it == r["iter"]
        assert abs(ob - r["outer"]) <= REL * abs(r["outer"]), (it, ob, r["outer"])
        assert abs(ib - r["inner"]) <= REL * abs(r["inner"]), (it, ib, r["inner"])
    assert abs(ws.BestInnerBound - oi) <= REL * abs(oi)
    assert abs(ws.BestOuterBound - oo) <= REL * abs(oo)
    assert ws.BestOuterBound <= ws.BestInnerBound + REL * abs(ws.BestInnerBound)
    assert abs(ws.BestInnerBound - FARMER_EF_OBJ) <= 1e-4 * abs(FARMER_EF_OBJ)
