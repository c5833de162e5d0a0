"""Pyomo -> LinearModel extraction (guarded import: Pyomo is not installed in this image).

The reference's scenario creators return Pyomo ``ConcreteModel`` objects
(spbase.py:255-291 calls them per local scenario) that a solver plugin reads through
Pyomo's standard representation.  This bridge turns such a model -- with its
``_mpisppy_node_list`` and ``_mpisppy_probability`` attributes -- into this engine's
``LinearModel``, once per scenario, so an unmodified mpi-sppy scenario creator can feed
the batched GPU solve (north_star: "the shared sparsity pattern, extracted once from the
Pyomo model"):

    from mpisppy_amd.pyomo_bridge import wrap_creator
    ph = PH(options, names, wrap_creator(farmer.scenario_creator), ...)

What it keeps (spopt.py:129-142 builds the same pieces for a persistent solver):

* variables in component order, bounds (``None`` -> +-inf), fixed variables as lb = ub =
  value; integer / binary domains are relaxed (the PH subproblems here are LP / QP);
* one active objective: linear part, constant, and a *diagonal* quadratic part
  (``x_j**2`` terms -> q_j = 2 coef); sense ``maximize`` -> ``sense_min = False``;
* every active constraint as ``lower - const <= linear(x) <= upper - const``;
* the scenario tree: each node's ``nonant_vardata_list`` (already in the reference's
  sorted-key order, scenario_tree.py:39) mapped onto the extracted columns.

Nonlinear terms and off-diagonal quadratic terms raise: they have no place in the
batched LP / QP.  Parity: UNPINNED here (no Pyomo to run against); the logic is tested
with a stand-in of the small Pyomo API surface it uses (tests/test_pyomo_bridge.py).
"""
from .model import LinearModel, INF
from .scenario_tree import ScenarioNode


def _pyomo():
    try:
        import pyomo.environ as pyo
        from pyomo.repn import generate_standard_repn
    except ImportError as e:  # pragma: no cover - exercised by the no-Pyomo test
        raise ImportError("mpisppy_amd.pyomo_bridge needs Pyomo, which is not installed; scenario "
                          "creators for this engine can return mpisppy_amd.model.LinearModel "
                          "directly") from e
    return pyo, generate_standard_repn


def _num(v, default):
    return default if v is None else float(v)


def extract(model, name=None):
    """LinearModel with the variables, objective, rows and tree of Pyomo ``model``."""
    pyo, gsr = _pyomo()
    lm = LinearModel(name if name is not None else getattr(model, "name", ""))
    col = {}
    for v in model.component_data_objects(pyo.Var, descend_into=True):
        if v.fixed:
            lb = ub = float(pyo.value(v))
        else:
            lb, ub = _num(v.lb, -INF), _num(v.ub, INF)
        col[id(v)] = lm.var(v.name, lb, ub)
    objs = list(model.component_data_objects(pyo.Objective, active=True, descend_into=True))
    if len(objs) != 1:
        raise RuntimeError(f"{lm.name}: expected one active objective, found {len(objs)}")
    obj = objs[0]
    repn = gsr(obj.expr, quadratic=True, compute_values=True)
    if repn.nonlinear_expr is not None:
        raise ValueError(f"{lm.name}: nonlinear objective terms are not supported")
    for v, a in zip(repn.linear_vars, repn.linear_coefs):
        lm.cost[col[id(v)].index] += float(a)
    for (v1, v2), a in zip(repn.quadratic_vars, repn.quadratic_coefs):
        if v1 is not v2:
            raise ValueError(f"{lm.name}: off-diagonal quadratic objective term {v1.name}*{v2.name}")
        lm.quad[col[id(v1)].index] += 2.0 * float(a)
    lm.obj_const = float(repn.constant)
    lm.set_objective_sense(obj.sense == pyo.minimize)
    for c in model.component_data_objects(pyo.Constraint, active=True, descend_into=True):
        r = gsr(c.body, quadratic=False, compute_values=True)
        if r.nonlinear_expr is not None or len(getattr(r, "quadratic_vars", ()) or ()) > 0:
            raise ValueError(f"{lm.name}: constraint {c.name} is not linear")
        k = float(r.constant)
        lo = float(pyo.value(c.lower)) - k if c.has_lb() else -INF
        hi = float(pyo.value(c.upper)) - k if c.has_ub() else INF
        terms = {}
        for v, a in zip(r.linear_vars, r.linear_coefs):
            j = col[id(v)]
            terms[j] = terms.get(j, 0.0) + float(a)
        lm.row(list(terms.items()), lo, hi, c.name)
    nodes = []
    for nd in getattr(model, "_mpisppy_node_list", None) or []:
        nodes.append(ScenarioNode(nd.name, nd.cond_prob, nd.stage, None,
                                  [col[id(v)] for v in nd.nonant_vardata_list], lm,
                                  parent_name=getattr(nd, "parent_name", None)))
    if not nodes:
        raise RuntimeError(f"{lm.name}: the model has no _mpisppy_node_list (sputils.attach_root_node)")
    lm._mpisppy_node_list = nodes
    lm._mpisppy_probability = getattr(model, "_mpisppy_probability", None)
    return lm


def wrap_creator(pyomo_creator):
    """A scenario creator for this engine from a reference (Pyomo) scenario creator."""
    def creator(scenario_name, **kwargs):
        return extract(pyomo_creator(scenario_name, **kwargs), scenario_name)
    creator.__name__ = getattr(pyomo_creator, "__name__", "creator") + "_linear"
    return creator
