"""Minimal algebraic scenario model (the Pyomo ConcreteModel stand-in).

The reference's ``scenario_creator`` returns a Pyomo ``ConcreteModel`` whose
objective the PH layer augments (phbase.py:617-699) and whose variables a solver
plugin fills (spopt.py:197-200).  Pyomo is not part of this image, so scenario
creators for this engine return a :class:`LinearModel`: the same information as an
LP/QP with a diagonal quadratic term, recorded row by row.  ``mpisppy_amd.batch``
turns a list of them (or a vectorised batch creator) into the shared CSR pattern +
per-scenario coefficient arrays the HIP kernels consume.

Attributes that mirror the Pyomo model the PH code reads:
  ``_mpisppy_node_list``   list of ScenarioNode (scenario_tree.py:44-96)
  ``_mpisppy_probability`` scenario probability, or None / "uniform"
"""
import math

INF = math.inf


class Var:
    """One scalar decision variable; ``_value`` is filled after a solve, as a Pyomo
    VarData's ``_value`` is (phbase.py reads ``nonant._value``)."""

    __slots__ = ("model", "index", "name", "_value")

    def __init__(self, model, index, name):
        self.model = model
        self.index = index
        self.name = name
        self._value = None

    @property
    def value(self):
        return self._value

    @property
    def lb(self):
        return self.model.lb[self.index]

    @property
    def ub(self):
        return self.model.ub[self.index]

    def __repr__(self):
        return f"Var({self.name})"


class LinearModel:
    """min / max  c'x + 1/2 sum q_j x_j^2 + const  s.t.  rl <= A x <= ru,  lb <= x <= ub."""

    def __init__(self, name=""):
        self.name = name
        self.vars = []
        self.lb = []
        self.ub = []
        self.cost = []
        self.quad = []
        self.rows = []            # (list of (var index, coef), rl, ru, name)
        self.obj_const = 0.0
        self.sense_min = True
        self._mpisppy_node_list = None
        self._mpisppy_probability = None
        self._by_name = {}

    # -- construction
    def var(self, name, lb=-INF, ub=INF, cost=0.0, quad=0.0):
        """Add a variable with objective coefficient ``cost`` and diagonal quadratic
        coefficient ``quad`` (the objective term is quad/2 * x^2)."""
        v = Var(self, len(self.vars), name)
        self.vars.append(v)
        self.lb.append(float(lb))
        self.ub.append(float(ub))
        self.cost.append(float(cost))
        self.quad.append(float(quad))
        self._by_name[name] = v
        return v

    def row(self, terms, rl=-INF, ru=INF, name=""):
        """Add rl <= sum(coef * var) <= ru; ``terms`` is an iterable of (Var, coef)."""
        t = [(v.index, float(a)) for (v, a) in terms]
        self.rows.append((t, float(rl), float(ru), name))

    def set_objective_sense(self, minimize=True):
        self.sense_min = bool(minimize)

    def find_var(self, name):
        return self._by_name[name]

    # -- evaluation helpers
    def objective_value(self, x=None):
        if x is None:
            x = [v._value for v in self.vars]
        s = self.obj_const
        for j, xv in enumerate(x):
            s += self.cost[j] * xv + 0.5 * self.quad[j] * xv * xv
        return s

    @property
    def n(self):
        return len(self.vars)

    @property
    def m(self):
        return len(self.rows)
