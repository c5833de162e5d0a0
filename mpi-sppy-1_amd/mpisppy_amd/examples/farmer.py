"""Scalable farmer model (mirrors examples/farmer/farmer.py of the reference).

``scenario_creator`` builds one scenario as a :class:`LinearModel` with exactly the
variables, rows, objective, node list and seeded yields of farmer.py:25-224.
``batch_creator`` builds the same scenarios for a whole rank at once as a
:class:`ScenarioBatch` (vectorised; what the 65,536-scenario runs use) -- tests check
the two agree bit for bit.
"""
import numpy as np

from ..model import LinearModel, INF
from ..sputils import extract_num, attach_root_node
from ..batch import ScenarioBatch, batch_from_models

# PDHG options recommended for farmer's warm-started PH solves (iterk_solver_options, the
# way a reference user passes solver options per example): restart the Halpern scheme once
# the fixed-point residual has decayed to 0.6 of its value at the last restart instead of
# PDLP's 0.2.  The prox QPs start next to their optimum, and restarting at the anchor
# sooner cuts the mean PDHG iterations per PH iteration from 224 to 199 and the max from
# 448 to 384 (config 3 2267 vs 2028 PH it/s; config 2 +8%; profiles/r02/s2/beta/).
# Model-specific: aircond is slower with it (1371 vs 1455 at 0.5), so it is not a
# library default.
PDHG_ITERK_OPTIONS = {"beta_sufficient": 0.6}

# farmer.py:127-150
PRICE_QUOTA = {"WHEAT": 100000.0, "CORN": 100000.0, "SUGAR_BEETS": 6000.0}
SUB_PRICE = {"WHEAT": 170.0, "CORN": 150.0, "SUGAR_BEETS": 36.0}
SUPER_PRICE = {"WHEAT": 0.0, "CORN": 0.0, "SUGAR_BEETS": 10.0}
FEED = {"WHEAT": 200.0, "CORN": 240.0, "SUGAR_BEETS": 0.0}
PURCHASE = {"WHEAT": 238.0, "CORN": 210.0, "SUGAR_BEETS": 100000.0}
PLANT = {"WHEAT": 150.0, "CORN": 230.0, "SUGAR_BEETS": 260.0}
YIELD = {
    "BelowAverageScenario": {"WHEAT": 2.0, "CORN": 2.4, "SUGAR_BEETS": 16.0},
    "AverageScenario": {"WHEAT": 2.5, "CORN": 3.0, "SUGAR_BEETS": 20.0},
    "AboveAverageScenario": {"WHEAT": 3.0, "CORN": 3.6, "SUGAR_BEETS": 24.0},
}
BASENAMES = ["BelowAverageScenario", "AverageScenario", "AboveAverageScenario"]
BASE_CROPS = ["WHEAT", "CORN", "SUGAR_BEETS"]


def crops(crops_multiplier):
    """CROPS insertion order (farmer.py:99-105)."""
    out = []
    for i in range(crops_multiplier):
        out += ["WHEAT" + str(i), "CORN" + str(i), "SUGAR_BEETS" + str(i)]
    return out


def yields_for(scennum, crops_multiplier=1, seedoffset=0):
    """Yield vector in CROPS order: base[scennum % 3] + rand() per crop unless the
    group scennum // 3 is 0 (farmer.py:52-60, 151-157; RandomState seeded with
    scennum + seedoffset)."""
    base = YIELD[BASENAMES[scennum % 3]]
    y = np.array([base[b] for b in BASE_CROPS] * crops_multiplier, dtype=np.float64)
    if scennum // 3 != 0:
        rs = np.random.RandomState(scennum + seedoffset)
        y = y + rs.rand(3 * crops_multiplier)
    return y


def scenario_creator(scenario_name, use_integer=False, sense=1, crops_multiplier=1,
                     num_scens=None, seedoffset=0):
    """farmer.py:25-83 (sense=1 minimise, -1 maximise).  Integer farmer is not on the
    PH LP/QP path this engine accelerates."""
    if use_integer:
        raise NotImplementedError("farmer_with_integers is outside the LP/QP hot path")
    scennum = extract_num(scenario_name)
    Y = yields_for(scennum, crops_multiplier, seedoffset)
    cl = crops(crops_multiplier)
    total = 500.0 * crops_multiplier
    mdl = LinearModel(scenario_name)
    sgn = 1.0 if sense == 1 else -1.0
    b = lambda c: c.rstrip("0123456789")  # noqa: E731
    DevotedAcreage = {c: mdl.var(f"DevotedAcreage[{c}]", 0.0, total, sgn * PLANT[b(c)]) for c in cl}
    Sub = {c: mdl.var(f"QuantitySubQuotaSold[{c}]", 0.0, INF, -sgn * SUB_PRICE[b(c)]) for c in cl}
    Sup = {c: mdl.var(f"QuantitySuperQuotaSold[{c}]", 0.0, INF, -sgn * SUPER_PRICE[b(c)]) for c in cl}
    Pur = {c: mdl.var(f"QuantityPurchased[{c}]", 0.0, INF, sgn * PURCHASE[b(c)]) for c in cl}
    mdl.set_objective_sense(sense == 1)
    mdl.row([(DevotedAcreage[c], 1.0) for c in cl], -INF, total, "ConstrainTotalAcreage")
    for k, c in enumerate(cl):
        mdl.row([(DevotedAcreage[c], Y[k]), (Pur[c], 1.0), (Sub[c], -1.0), (Sup[c], -1.0)],
                FEED[b(c)], INF, f"EnforceCattleFeedRequirement[{c}]")
    for k, c in enumerate(cl):
        mdl.row([(Sub[c], 1.0), (Sup[c], 1.0), (DevotedAcreage[c], -Y[k])], -INF, 0.0,
                f"LimitAmountSold[{c}]")
    for c in cl:
        mdl.row([(Sub[c], 1.0)], 0.0, PRICE_QUOTA[b(c)], f"EnforceQuotas[{c}]")
    mdl.DevotedAcreage = DevotedAcreage
    mdl.Yield = dict(zip(cl, Y))
    attach_root_node(mdl, None, [DevotedAcreage])
    if num_scens is not None:
        mdl._mpisppy_probability = 1 / num_scens
    return mdl


def scenario_names_creator(num_scens, start=None):
    """farmer.py:229-234."""
    if start is None:
        start = 0
    return [f"scen{i}" for i in range(start, start + num_scens)]


def kw_creator(cfg):
    """farmer.py:254-260."""
    return {"use_integer": cfg.get("farmer_with_integers", False),
            "crops_multiplier": cfg.get("crops_multiplier", 1),
            "num_scens": cfg.get("num_scens", None)}


def scenario_denouement(rank, scenario_name, scenario):
    pass


def batch_creator(scenario_names, use_integer=False, sense=1, crops_multiplier=1,
                  num_scens=None, seedoffset=0, num_all_scens=None):
    """All of ``scenario_names`` as one ScenarioBatch, vectorised.

    Same result as ``batch_from_models([scenario_creator(n, ...) for n in names])``
    (checked in tests/test_batch.py): the template scenario fixes the pattern, and
    only the 2 * 3cm yield entries (feed and limit rows) change per scenario.
    """
    if use_integer:
        raise NotImplementedError("farmer_with_integers is outside the LP/QP hot path")
    names = list(scenario_names)
    S = len(names)
    cm = crops_multiplier
    tmpl = scenario_creator("scen0", sense=sense, crops_multiplier=cm, num_scens=num_scens)
    tb = batch_from_models(["scen0"], [tmpl], num_all_scens=num_all_scens or S)
    nc = 3 * cm
    # locate the yield entries: feed rows 1..nc (entry of column k), limit rows nc+1..2nc
    y_pos_feed = np.empty(nc, dtype=np.int64)
    y_pos_lim = np.empty(nc, dtype=np.int64)
    for k in range(nc):
        for which, r in ((0, 1 + k), (1, 1 + nc + k)):
            lo, hi = tb.row_ptr[r], tb.row_ptr[r + 1]
            pos = lo + int(np.nonzero(tb.col_idx[lo:hi] == k)[0][0])
            (y_pos_feed if which == 0 else y_pos_lim)[k] = pos
    Y = np.empty((S, nc))
    for s, nm in enumerate(names):
        Y[s] = yields_for(extract_num(nm), cm, seedoffset)
    A_val = np.repeat(tb.A_val, S, axis=0)
    A_val[:, y_pos_feed] = Y
    A_val[:, y_pos_lim] = -Y
    rep = lambda a: np.repeat(a, S, axis=0)  # noqa: E731
    if num_scens is not None:
        prob = np.full(S, 1.0 / num_scens)
    else:
        prob = np.full(S, 1.0 / (num_all_scens or S))
    return ScenarioBatch(names, tb.row_ptr, tb.col_idx, A_val, rep(tb.c), rep(tb.lb),
                         rep(tb.ub), rep(tb.rl), rep(tb.ru), rep(tb.q), rep(tb.obj_const),
                         tb.nonant_col, tb.nonant_depth, tb.nonant_off,
                         np.zeros((S, 1), dtype=np.int32), ["ROOT"], prob,
                         prob[:, None].copy(), tb.sense, tb.var_names, tb.nonant_names)
