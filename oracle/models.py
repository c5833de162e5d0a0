"""Oracle restatement of the reference scenario models (TEST INFRASTRUCTURE ONLY).

Each scenario is an explicit LP/QP in the exact variable / row order in which the
reference declares its Pyomo components, with no presolve (the product builder in
mpisppy_amd folds singleton rows into bounds; keeping the rows here makes the
oracle an independent check of that presolve).

    min  c'x + 1/2 sum_j q_j x_j^2   s.t.  rl <= A x <= ru,  lb <= x <= ub
"""
import re
import numpy as np

INF = float("inf")


class ScenLP:
    """One scenario subproblem (what one Pyomo ConcreteModel holds)."""

    def __init__(self, name):
        self.name = name
        self.var_names = []
        self.lb = []
        self.ub = []
        self.c = []
        self.q = []
        self.rows = []          # list of (dict{var index: coef}, rl, ru, name)
        self.nodes = []         # list of (node name, cond_prob, stage, [var indices])
        self.prob = None

    def add_var(self, name, lb=-INF, ub=INF, cost=0.0, quad=0.0):
        self.var_names.append(name)
        self.lb.append(lb)
        self.ub.append(ub)
        self.c.append(cost)
        self.q.append(quad)
        return len(self.var_names) - 1

    def add_row(self, coefs, rl, ru, name=""):
        self.rows.append((dict(coefs), rl, ru, name))

    def arrays(self):
        n = len(self.var_names)
        m = len(self.rows)
        A = np.zeros((m, n))
        rl = np.empty(m)
        ru = np.empty(m)
        for i, (co, lo, hi, _) in enumerate(self.rows):
            for j, a in co.items():
                A[i, j] += a
            rl[i] = lo
            ru[i] = hi
        return (A, rl, ru, np.array(self.lb, float), np.array(self.ub, float),
                np.array(self.c, float), np.array(self.q, float))

    def nonant_indices(self):
        """Flat nonant order: node list order, then index (spbase.py:293-302)."""
        out = []
        for (_, _, _, idx) in self.nodes:
            out.extend(idx)
        return out


def extract_num(string):
    """sputils.py:481-490: longest run of digits at the right end."""
    return int(re.compile(r"(\d+)$").search(string).group(1))


# ----------------------------------------------------------------- farmer
# examples/farmer/farmer.py:85-224 (and mpisppy/tests/examples/farmer.py, identical
# model); data tables at farmer.py:127-150.
_F_PRICE_QUOTA = {"WHEAT": 100000.0, "CORN": 100000.0, "SUGAR_BEETS": 6000.0}
_F_SUB_PRICE = {"WHEAT": 170.0, "CORN": 150.0, "SUGAR_BEETS": 36.0}
_F_SUPER_PRICE = {"WHEAT": 0.0, "CORN": 0.0, "SUGAR_BEETS": 10.0}
_F_FEED = {"WHEAT": 200.0, "CORN": 240.0, "SUGAR_BEETS": 0.0}
_F_PURCHASE = {"WHEAT": 238.0, "CORN": 210.0, "SUGAR_BEETS": 100000.0}
_F_PLANT = {"WHEAT": 150.0, "CORN": 230.0, "SUGAR_BEETS": 260.0}
_F_YIELD = {
    "BelowAverageScenario": {"WHEAT": 2.0, "CORN": 2.4, "SUGAR_BEETS": 16.0},
    "AverageScenario": {"WHEAT": 2.5, "CORN": 3.0, "SUGAR_BEETS": 20.0},
    "AboveAverageScenario": {"WHEAT": 3.0, "CORN": 3.6, "SUGAR_BEETS": 24.0},
}


def farmer_yields(scenario_name, crops_multiplier=1, seedoffset=0):
    """Yield[crop] for one scenario, crops in CROPS insertion order.

    farmer.py:52-60 (scennum, basenum, groupnum, farmerstream.seed(scennum+seedoffset)),
    farmer.py:99-105 (CROPS order WHEATi, CORNi, SUGAR_BEETSi) and
    farmer.py:151-157 (Yield_init: base + rand() unless group 0).
    """
    scennum = extract_num(scenario_name)
    basenames = ["BelowAverageScenario", "AverageScenario", "AboveAverageScenario"]
    base = basenames[scennum % 3]
    groupnum = scennum // 3
    stream = np.random.RandomState()
    stream.seed(scennum + seedoffset)
    crops = []
    for i in range(crops_multiplier):
        crops += ["WHEAT" + str(i), "CORN" + str(i), "SUGAR_BEETS" + str(i)]
    y = {}
    for cname in crops:
        b = _F_YIELD[base][cname.rstrip("0123456789")]
        y[cname] = b + stream.rand() if groupnum != 0 else b
    return crops, y


def farmer_scenario(scenario_name, crops_multiplier=1, num_scens=None, seedoffset=0):
    """Restates farmer.scenario_creator (farmer.py:25-83) for sense=minimize."""
    crops, Y = farmer_yields(scenario_name, crops_multiplier, seedoffset)
    cm = crops_multiplier
    total = 500.0 * cm
    s = ScenLP(scenario_name)
    base = lambda c: c.rstrip("0123456789")  # noqa: E731
    # Vars in declaration order (farmer.py:163-175).
    xa = {c: s.add_var(f"DevotedAcreage[{c}]", 0.0, total, _F_PLANT[base(c)]) for c in crops}
    sub = {c: s.add_var(f"QuantitySubQuotaSold[{c}]", 0.0, INF, -_F_SUB_PRICE[base(c)]) for c in crops}
    sup = {c: s.add_var(f"QuantitySuperQuotaSold[{c}]", 0.0, INF, -_F_SUPER_PRICE[base(c)]) for c in crops}
    pur = {c: s.add_var(f"QuantityPurchased[{c}]", 0.0, INF, _F_PURCHASE[base(c)]) for c in crops}
    # Rows (farmer.py:181-202).
    s.add_row({xa[c]: 1.0 for c in crops}, -INF, total, "ConstrainTotalAcreage")
    for c in crops:
        s.add_row({xa[c]: Y[c], pur[c]: 1.0, sub[c]: -1.0, sup[c]: -1.0},
                  _F_FEED[base(c)], INF, f"EnforceCattleFeedRequirement[{c}]")
    for c in crops:
        s.add_row({sub[c]: 1.0, sup[c]: 1.0, xa[c]: -Y[c]}, -INF, 0.0, f"LimitAmountSold[{c}]")
    for c in crops:
        s.add_row({sub[c]: 1.0}, 0.0, _F_PRICE_QUOTA[base(c)], f"EnforceQuotas[{c}]")
    # Root node: DevotedAcreage expanded in sorted key order (scenario_tree.py:39).
    s.nodes = [("ROOT", 1.0, 1, [xa[c] for c in sorted(crops)])]
    s.prob = 1.0 / num_scens if num_scens is not None else None
    return s


# ----------------------------------------------------------------- aircond
# mpisppy/tests/examples/aircond.py:19-35 default parameters.
AIRCOND_PARMS = {
    "mu_dev": 0.0, "sigma_dev": 40.0, "start_ups": False, "StartUpCost": 300.0,
    "start_seed": 1134, "min_d": 0.0, "max_d": 400.0, "starting_d": 200.0,
    "BeginInventory": 200.0, "InventoryCost": 0.5, "LastInventoryCost": -0.8,
    "Capacity": 200.0, "RegularProdCost": 1.0, "OvertimeProdCost": 3.0,
    "NegInventoryCost": 5.0, "QuadShortCoeff": 0.0,
}


def _nodenum_before_stage(t, bfs):
    """sputils.py:654-657."""
    return int(sum(np.prod(bfs[0:i]) for i in range(t)))


def node_idx(node_path, bfs):
    """sputils.py:494-519."""
    if node_path == []:
        return 0
    stage_id = 0
    for t in range(len(node_path)):
        stage_id = node_path[t] + bfs[t] * stage_id
    return _nodenum_before_stage(len(node_path), bfs) + stage_id


def aircond_demands(sname, bfs, **kw):
    """aircond.py:37-67 (_demands_creator)."""
    start_seed = kw["start_seed"]
    max_d = kw.get("max_d", 400)
    min_d = kw.get("min_d", 0)
    mu_dev = kw.get("mu_dev", None)
    sigma_dev = kw.get("sigma_dev", None)
    scennum = extract_num(sname)
    prod = int(np.prod(bfs))
    s = int(scennum % prod)
    d = kw.get("starting_d", 200)
    demands = [d]
    nodenames = ["ROOT"]
    for bf in bfs:
        prod = prod // bf
        nodenames.append(str(s // prod))
        s = s % prod
    stagelist = [int(x) for x in nodenames[1:]]
    stream = np.random.RandomState()
    for t in range(1, len(nodenames)):
        stream.seed(start_seed + node_idx(stagelist[:t], bfs))
        d = min(max_d, max(min_d, d + stream.normal(mu_dev, sigma_dev)))
        demands.append(d)
    return demands, nodenames


def aircond_scenario(sname, branching_factors, **kwargs):
    """aircond.py:88-330 (stage models, material balance, nodes) for start_ups=False."""
    kw = dict(AIRCOND_PARMS)
    kw.update(kwargs)
    bfs = list(branching_factors)
    demands, nodenames = aircond_demands(sname, bfs, **kw)
    T = len(demands)
    bigM = kw["Capacity"] * 25
    s = ScenLP(sname)
    v = {}
    for t in range(1, T + 1):
        last = t == T
        # Vars in declaration order of _StageModel_creator (aircond.py:126-149).
        v["Reg", t] = s.add_var(f"stage_model_{t}.RegularProd", 0.0, bigM, kw["RegularProdCost"])
        v["Over", t] = s.add_var(f"stage_model_{t}.OvertimeProd", 0.0, bigM, kw["OvertimeProdCost"])
        v["Inv", t] = s.add_var(f"stage_model_{t}.Inventory", -bigM, bigM, 0.0)
        quad = 2.0 * kw["QuadShortCoeff"] if (kw["QuadShortCoeff"] > 0 and not last) else 0.0
        v["neg", t] = s.add_var(f"stage_model_{t}.negInventory", 0.0, bigM,
                                kw["NegInventoryCost"], quad)
        v["pos", t] = s.add_var(f"stage_model_{t}.posInventory", 0.0, bigM,
                                kw["LastInventoryCost"] if last else kw["InventoryCost"])
        # MaximumCapacity (aircond.py:137-139), doleInventory (:149).
        s.add_row({v["Reg", t]: 1.0}, -INF, kw["Capacity"], f"stage_model_{t}.MaximumCapacity")
        s.add_row({v["Inv", t]: 1.0, v["pos", t]: -1.0, v["neg", t]: 1.0}, 0.0, 0.0,
                  f"stage_model_{t}.doleInventory")
    # MaterialBalance (aircond.py:212-222).
    for t in range(1, T + 1):
        co = {v["Reg", t]: 1.0, v["Over", t]: 1.0, v["Inv", t]: -1.0}
        rhs = demands[t - 1]
        if t == 1:
            rhs -= kw["BeginInventory"]
        else:
            co[v["Inv", t - 1]] = 1.0
        s.add_row(co, rhs, rhs, f"MaterialBalance[{t}]")
    # Nodes (aircond.py:251-302, starting_stage=1): ROOT, then ROOT_i, ... for t < T.
    ndn = "ROOT"
    s.nodes.append(("ROOT", 1.0, 1, [v["Reg", 1], v["Over", 1]]))
    for t in range(2, T):
        ndn = ndn + "_" + nodenames[t - 1]
        s.nodes.append((ndn, 1.0 / bfs[t - 2], t, [v["Reg", t], v["Over", t]]))
    s.prob = 1.0 / np.prod(bfs)
    s.demands = demands
    return s


def aircond_rho_setter(s, rho_scale_factor=0.01, **kw):
    """aircond.py:69-85 general_rho_setter / primal_rho_setter: rho = cost * factor."""
    p = dict(AIRCOND_PARMS)
    p.update(kw)
    out = []
    for (_, _, _, idx) in s.nodes:
        out.append((idx[0], p["RegularProdCost"] * rho_scale_factor))
        out.append((idx[1], p["OvertimeProdCost"] * rho_scale_factor))
    return out


def create_nodenames_from_branching_factors(bfs):
    """sputils.py:934-959."""
    stage_nodes = ["ROOT"]
    nodenames = ["ROOT"]
    if len(bfs) == 1:
        return nodenames
    for bf in bfs:
        old = stage_nodes
        stage_nodes = []
        for k in range(len(old)):
            stage_nodes += ["%s_%i" % (old[k], b) for b in range(bf)]
        nodenames += stage_nodes
    return nodenames
