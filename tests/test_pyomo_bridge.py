"""The Pyomo -> LinearModel bridge (mpisppy_amd/pyomo_bridge.py) against a stand-in for
the small Pyomo API it uses (Pyomo is not installed, so parity with real Pyomo models is
unpinned): a farmer / aircond LinearModel is written out as stand-in Pyomo components
(constant offsets in constraint bodies, duplicated terms, a fixed variable, a
maximisation) and read back; the batch built from the round trip equals the original's."""
import sys
import types

import numpy as np
import pytest

INF = float("inf")


class _Expr:
    def __init__(self, lin=(), quad=(), const=0.0, nonlinear=None):
        self.lin, self.quad, self.const, self.nonlinear = list(lin), list(quad), const, nonlinear


class _Repn:
    def __init__(self, e):
        self.linear_vars = [v for v, _ in e.lin]
        self.linear_coefs = [a for _, a in e.lin]
        self.quadratic_vars = [vv for vv, _ in e.quad]
        self.quadratic_coefs = [a for _, a in e.quad]
        self.constant = e.const
        self.nonlinear_expr = e.nonlinear


class _VarData:
    def __init__(self, name, lb, ub, fixed=False, value=None):
        self.name, self.lb, self.ub, self.fixed, self.value = name, lb, ub, fixed, value


class _ConData:
    def __init__(self, name, body, lower, upper):
        self.name, self.body, self.lower, self.upper = name, body, lower, upper

    def has_lb(self):
        return self.lower is not None

    def has_ub(self):
        return self.upper is not None


class _ObjData:
    def __init__(self, expr, sense):
        self.expr, self.sense = expr, sense


class _Model:
    def __init__(self, name):
        self.name = name
        self.vars, self.cons, self.objs = [], [], []

    def component_data_objects(self, kind, active=True, descend_into=True):
        return {"Var": self.vars, "Constraint": self.cons, "Objective": self.objs}[kind]


@pytest.fixture
def fake_pyomo(monkeypatch):
    env = types.ModuleType("pyomo.environ")
    env.Var, env.Constraint, env.Objective = "Var", "Constraint", "Objective"
    env.minimize, env.maximize = 1, -1
    env.value = lambda x: x.value if isinstance(x, _VarData) else x
    repn = types.ModuleType("pyomo.repn")
    repn.generate_standard_repn = lambda e, quadratic=True, compute_values=True: _Repn(e)
    pkg = types.ModuleType("pyomo")
    pkg.environ, pkg.repn = env, repn
    monkeypatch.setitem(sys.modules, "pyomo", pkg)
    monkeypatch.setitem(sys.modules, "pyomo.environ", env)
    monkeypatch.setitem(sys.modules, "pyomo.repn", repn)
    return env


def _to_fake(lm, maximize=False):
    """Write a LinearModel as stand-in Pyomo components (the reference's shape)."""
    fm = _Model(lm.name)
    vd = []
    for j, v in enumerate(lm.vars):
        lb = None if lm.lb[j] == -INF else lm.lb[j]
        ub = None if lm.ub[j] == INF else lm.ub[j]
        vd.append(_VarData(v.name, lb, ub))
    fm.vars = vd
    sgn = -1.0 if maximize else 1.0
    lin = [(vd[j], sgn * c) for j, c in enumerate(lm.cost) if c != 0.0]
    quad = [((vd[j], vd[j]), sgn * 0.5 * q) for j, q in enumerate(lm.quad) if q != 0.0]
    fm.objs = [_ObjData(_Expr(lin, quad, sgn * lm.obj_const), -1 if maximize else 1)]
    for r, (terms, lo, hi, name) in enumerate(lm.rows):
        k = 3.0 * (r % 2)                      # a constant inside the body
        ts = []
        for (j, a) in terms:                   # every coefficient split in two terms
            ts += [(vd[j], 0.25 * a), (vd[j], 0.75 * a)]
        fm.cons.append(_ConData(name, _Expr(ts, (), k), None if lo == -INF else lo + k,
                                None if hi == INF else hi + k))
    fm._mpisppy_node_list = [types.SimpleNamespace(name=nd.name, cond_prob=nd.cond_prob, stage=nd.stage,
                                                   parent_name=nd.parent_name,
                                                   nonant_vardata_list=[vd[v.index] for v in nd.nonant_vardata_list])
                             for nd in lm._mpisppy_node_list]
    fm._mpisppy_probability = lm._mpisppy_probability
    return fm


def _same_batch(b1, b2):
    for f in ("row_ptr", "col_idx", "A_val", "c", "lb", "ub", "rl", "ru", "q", "obj_const", "nonant_col",
              "nonant_depth", "nonant_off", "node_of", "prob", "prob_coeff"):
        assert np.array_equal(getattr(b1, f), getattr(b2, f)), f
    assert b1.sense == b2.sense


def test_round_trip_farmer(fake_pyomo):
    from mpisppy_amd.examples import farmer
    from mpisppy_amd.batch import batch_from_models
    from mpisppy_amd.pyomo_bridge import wrap_creator
    names = farmer.scenario_names_creator(3)
    kw = {"num_scens": 3, "crops_multiplier": 2}
    mods = [farmer.scenario_creator(nm, **kw) for nm in names]
    creator = wrap_creator(lambda nm, **k: _to_fake(farmer.scenario_creator(nm, **k)))
    back = [creator(nm, **kw) for nm in names]
    _same_batch(batch_from_models(names, mods), batch_from_models(names, back))


def test_round_trip_aircond_multistage_with_quadratic(fake_pyomo):
    from mpisppy_amd.examples import aircond
    from mpisppy_amd.batch import batch_from_models
    from mpisppy_amd.pyomo_bridge import extract
    from mpisppy_amd.sputils import create_nodenames_from_branching_factors
    bf = [2, 2]
    kw = {"branching_factors": bf, "start_seed": 0, "QuadShortCoeff": 0.3}
    names = aircond.scenario_names_creator(4)
    mods = [aircond.scenario_creator(nm, **kw) for nm in names]
    back = [extract(_to_fake(m), m.name) for m in mods]
    nodes = create_nodenames_from_branching_factors(bf)
    _same_batch(batch_from_models(names, mods, all_nodenames=nodes),
                batch_from_models(names, back, all_nodenames=nodes))


def test_maximize_fixed_and_errors(fake_pyomo):
    from mpisppy_amd.examples import farmer
    from mpisppy_amd.pyomo_bridge import extract
    m = farmer.scenario_creator("scen0", num_scens=3)
    fm = _to_fake(m, maximize=True)
    fm.vars[0].fixed, fm.vars[0].value = True, 123.0
    lm = extract(fm)
    assert not lm.sense_min and lm.lb[0] == lm.ub[0] == 123.0
    assert np.allclose(lm.cost, [-c for c in m.cost])
    fm.objs[0].expr.quad.append(((fm.vars[0], fm.vars[1]), 1.0))
    with pytest.raises(ValueError, match="off-diagonal"):
        extract(fm)
    fm = _to_fake(m)
    fm.cons[0].body.nonlinear = "x*y"
    with pytest.raises(ValueError, match="not linear"):
        extract(fm)
    fm = _to_fake(m)
    fm._mpisppy_node_list = None
    with pytest.raises(RuntimeError, match="_mpisppy_node_list"):
        extract(fm)


def test_without_pyomo_the_error_says_so(monkeypatch):
    monkeypatch.setitem(sys.modules, "pyomo", None)
    monkeypatch.setitem(sys.modules, "pyomo.environ", None)
    from mpisppy_amd.pyomo_bridge import extract
    with pytest.raises(ImportError, match="Pyomo"):
        extract(object())
