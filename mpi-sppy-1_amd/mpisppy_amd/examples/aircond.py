"""Multistage aircond inventory model (mirrors mpisppy/tests/examples/aircond.py).

``scenario_creator`` restates aircond.py:88-330 for ``start_ups=False`` (the LP/QP
case; start-up binaries are outside this engine's hot path) as a LinearModel;
``batch_creator`` builds a rank's scenarios at once.
"""
import numpy as np

from ..model import LinearModel, INF
from ..sputils import extract_num, node_idx, create_nodenames_from_branching_factors
from ..scenario_tree import ScenarioNode
from ..batch import batch_from_models, ScenarioBatch

# Interior-point constants measured for this model (PH option "ipm_tuning" ->
# phgpu_set_ipm_tuning): a lower centring floor and a deeper warm-start push.  Config 4
# (65,536 scenarios, one lane per scenario): 2,759-2,791 PH it/s against 2,556-2,576 with the
# library's 0.01 / 0.1, max / mean IPM iterations per PH solve 18 / 7.7 against 20 / 7.9
# (profiles/r05/x); farmer gains nothing from them (8,906-8,919 against 8,971-8,975).
IPM_TUNING = {"IPM_SIG_MIN": 0.003, "IPM_WARM_T": 0.3}

# aircond.py:19-35 ("Do not edit these defaults!")
PARMS = {
    "mu_dev": 0.0, "sigma_dev": 40.0, "start_ups": False, "StartUpCost": 300.0,
    "start_seed": 1134, "min_d": 0.0, "max_d": 400.0, "starting_d": 200.0,
    "BeginInventory": 200.0, "InventoryCost": 0.5, "LastInventoryCost": -0.8,
    "Capacity": 200.0, "RegularProdCost": 1.0, "OvertimeProdCost": 3.0,
    "NegInventoryCost": 5.0, "QuadShortCoeff": 0.0,
}


def _kw(kwargs, p):
    return kwargs.get(p, PARMS[p])


def demands_creator(sname, sample_branching_factors, root_name="ROOT", **kwargs):
    """aircond.py:37-67: demand path from per-node seeds start_seed + node_idx."""
    if "start_seed" not in kwargs:
        raise RuntimeError(f"start_seed not in kwargs={kwargs}")
    start_seed = kwargs["start_seed"]
    max_d = kwargs.get("max_d", 400)
    min_d = kwargs.get("min_d", 0)
    mu_dev = kwargs.get("mu_dev", None)
    sigma_dev = kwargs.get("sigma_dev", None)
    scennum = extract_num(sname)
    prod = int(np.prod(sample_branching_factors))
    s = int(scennum % prod)
    d = kwargs.get("starting_d", 200)
    demands = [d]
    nodenames = [root_name]
    for bf in sample_branching_factors:
        assert prod % bf == 0
        prod = prod // bf
        nodenames.append(str(s // prod))
        s = s % prod
    stagelist = [int(x) for x in nodenames[1:]]
    rs = np.random.RandomState()
    for t in range(1, len(nodenames)):
        rs.seed(start_seed + node_idx(stagelist[:t], sample_branching_factors))
        d = min(max_d, max(min_d, d + rs.normal(mu_dev, sigma_dev)))
        demands.append(d)
    return demands, nodenames


def scenario_creator(sname, **kwargs):
    """aircond.py:304-330 (+ the stage models 88-182 and material balance 212-222)."""
    if "start_seed" not in kwargs:
        raise RuntimeError("start_seed not in kwargs")
    if "branching_factors" not in kwargs:
        raise RuntimeError("scenario_creator for aircond needs branching_factors in kwargs")
    if _kw(kwargs, "start_ups"):
        raise NotImplementedError("start_ups (binaries) is outside the LP/QP hot path")
    # parameters the caller leaves out take the module defaults (what kw_creator does
    # in the reference, aircond.py:19-35 / 441-460)
    kwargs = {**{k: v for k, v in PARMS.items() if k != "start_seed"}, **kwargs}
    bfs = list(kwargs["branching_factors"])
    demands, nodenames = demands_creator(sname, bfs, **kwargs)
    T = len(demands)
    cap = _kw(kwargs, "Capacity")
    bigM = cap * 25
    qsc = _kw(kwargs, "QuadShortCoeff")
    mdl = LinearModel(sname)
    st = {}
    for t in range(1, T + 1):
        last = t == T
        Reg = mdl.var(f"stage_model_{t}.RegularProd", 0.0, bigM, _kw(kwargs, "RegularProdCost"))
        Over = mdl.var(f"stage_model_{t}.OvertimeProd", 0.0, bigM, _kw(kwargs, "OvertimeProdCost"))
        Inv = mdl.var(f"stage_model_{t}.Inventory", -bigM, bigM, 0.0)
        neg = mdl.var(f"stage_model_{t}.negInventory", 0.0, bigM, _kw(kwargs, "NegInventoryCost"),
                      2.0 * qsc if (qsc > 0 and not last) else 0.0)
        pos = mdl.var(f"stage_model_{t}.posInventory", 0.0, bigM,
                      _kw(kwargs, "LastInventoryCost") if last else _kw(kwargs, "InventoryCost"))
        mdl.row([(Reg, 1.0)], -INF, cap, f"stage_model_{t}.MaximumCapacity")
        mdl.row([(Inv, 1.0), (pos, -1.0), (neg, 1.0)], 0.0, 0.0, f"stage_model_{t}.doleInventory")
        st[t] = (Reg, Over, Inv, neg, pos)
    for t in range(1, T + 1):
        Reg, Over, Inv, _, _ = st[t]
        terms = [(Reg, 1.0), (Over, 1.0), (Inv, -1.0)]
        rhs = demands[t - 1]
        if t == 1:
            rhs -= _kw(kwargs, "BeginInventory")
        else:
            terms.append((st[t - 1][2], 1.0))
        mdl.row(terms, rhs, rhs, f"MaterialBalance[{t}]")
    # MakeNodesforScen, aircond.py:251-302 (starting_stage=1)
    nodes = [ScenarioNode("ROOT", 1.0, 1, None, [st[1][0], st[1][1]], mdl)]
    ndn = "ROOT"
    for t in range(2, T):
        parent = ndn
        ndn = parent + "_" + nodenames[t - 1]
        nodes.append(ScenarioNode(ndn, 1.0 / bfs[t - 2], t, None, [st[t][0], st[t][1]], mdl,
                                  parent_name=parent))
    mdl._mpisppy_node_list = nodes
    mdl._mpisppy_probability = 1 / np.prod(bfs)
    mdl.demands = demands
    mdl.stage_vars = st
    return mdl


def scenario_names_creator(num_scens, start=None):
    if start is None:
        start = 0
    return [f"scen{i}" for i in range(start, start + num_scens)]


def general_rho_setter(scenario_instance, rho_scale_factor=1.0):
    """aircond.py:69-79: rho = production cost * factor on each stage's nonants."""
    out = []
    for nd in scenario_instance._mpisppy_node_list:
        reg, over = nd.nonant_vardata_list
        out.append((id(reg), scenario_instance.cost[reg.index] * rho_scale_factor))
        out.append((id(over), scenario_instance.cost[over.index] * rho_scale_factor))
    return out


def dual_rho_setter(scenario_instance):
    return general_rho_setter(scenario_instance, rho_scale_factor=0.0001)


def primal_rho_setter(scenario_instance):
    return general_rho_setter(scenario_instance, rho_scale_factor=0.01)


def batch_creator(scenario_names, **kwargs):
    """Vectorised ScenarioBatch for ``scenario_names``: the pattern comes from one
    template scenario; per scenario only the material-balance right-hand sides
    (demands) and tree node ids change."""
    names = list(scenario_names)
    kwargs = {**{k: v for k, v in PARMS.items() if k != "start_seed"}, **kwargs}
    bfs = list(kwargs["branching_factors"])
    tmpl = scenario_creator(names[0], **kwargs)
    all_nodes = create_nodenames_from_branching_factors(bfs)
    nonleaf = [nd for nd in all_nodes if nd.count("_") < len(bfs)]
    tb = batch_from_models([names[0]], [tmpl], node_names=nonleaf)
    S = len(names)
    T = len(bfs) + 1
    # material balance rows are the last T kept rows (singleton capacity rows folded)
    mb = np.arange(tb.m - T, tb.m)
    rl = np.repeat(tb.rl, S, axis=0)
    ru = np.repeat(tb.ru, S, axis=0)
    node_of = np.empty((S, T - 1), dtype=np.int32)
    nid = {nd: i for i, nd in enumerate(nonleaf)}
    begin = _kw(kwargs, "BeginInventory")
    for s, nm in enumerate(names):
        dem, nodenames = demands_creator(nm, bfs, **kwargs)
        rhs = np.array(dem, dtype=np.float64)
        rhs[0] -= begin
        rl[s, mb] = rhs
        ru[s, mb] = rhs
        ndn = "ROOT"
        node_of[s, 0] = 0
        for t in range(2, T):
            ndn = ndn + "_" + nodenames[t - 1]
            node_of[s, t - 1] = nid[ndn]
    rep = lambda a: np.repeat(a, S, axis=0)  # noqa: E731
    prob = np.full(S, 1.0 / np.prod(bfs))
    uncond = np.array([1.0] + [1.0 / np.prod(bfs[:d]) for d in range(1, T - 1)])
    prob_coeff = prob[:, None] / uncond[None, :]
    return ScenarioBatch(names, tb.row_ptr, tb.col_idx, rep(tb.A_val), rep(tb.c), rep(tb.lb),
                         rep(tb.ub), rl, ru, rep(tb.q), rep(tb.obj_const), tb.nonant_col,
                         tb.nonant_depth, tb.nonant_off, node_of, nonleaf, prob, prob_coeff,
                         tb.sense, tb.var_names, tb.nonant_names)
