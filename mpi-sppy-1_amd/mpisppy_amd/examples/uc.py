"""Unit commitment (config 5): the LP relaxation of the reference's WECC-240 UC model.

The reference builds its UC scenarios with egret (paperruns/larger_uc/uc_funcs.py:18-84:
``RootNode.dat`` + ``NodeN.dat`` -> egret's tight UC model).  egret is not part of this
image, so this module restates the Pyomo model that ships with the same data,
paperruns/larger_uc/ReferenceModel_OK.py (the Knueven-Ostrowski-Watson matching
formulation, flags at :59-69: t=1 ramp rates enforced, no regulation / reserve
products, storage enabled but no storage in the data), with every binary relaxed to
[0, 1].  Parity is **unpinned**: no reference output exists for this model; tests pin
it against HiGHS on the same LP (oracle/uc.py).

Scenarios differ only in the wind bounds ``MinNondispatchablePower`` /
``MaxNondispatchablePower`` (NodeN.dat).  The nonants are ``UnitOn[g,t]`` in sorted key
order (uc_funcs.py:78-83 -> sputils.attach_root_node -> scenario_tree.py:39); the
probability is uniform (ScenarioStructure.dat: 0.001 each for 1000 scenarios).

``path`` (the reference's kwarg) names a directory holding ``RootNode.dat`` and
``NodeN.dat``; without it the packaged form of the 1000-scenario data is used
(``uc_data/``: RootNode.dat's parsed parameters and sets, and the wind bounds of
Node1..1000.dat, packed by tools/make_uc_data.py).
"""
import json
import os

import numpy as np

from ..model import LinearModel, INF
from ..sputils import extract_num, attach_root_node
from ..batch import ScenarioBatch, batch_from_models
from ..utils.datfile import load_dat, load_data as load_packed

DATA_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "uc_data")
BIG_PENALTY = 1e6              # ReferenceModel_OK.py:995-999
MODERATELY_BIG_PENALTY = 1e5
INITIAL_TIME = 1               # :133

# Recommended options of the warm-started PH solves (path 4): restart once the fixed-point
# residual fell to 0.7 of its value at the last restart (library default 0.2).  Config 5,
# two timed PH iterations on one trajectory: mean PDHG iterations 15,836 (0.2) / 15,063
# (0.4) / 13,718 (0.6) / 13,203 (0.7) / 13,973 (0.8), mean PH iteration 39.4 / 36.8 / 34.3
# / 32.7 / 36.8 s (profiles/r05/s, t); and the KKT test every 128 iterations instead of 64
# (its two passes cost ~3% of the iterations; 13,439 mean iterations, 31.4 s; a restart test
# every 32, an artificial restart at 0.5, a KKT test every 256 or a step fraction of 0.999
# did not help, profiles/r05/v, cc).
PDHG_ITERK_OPTIONS = {"beta_sufficient": 0.7, "check_every": 128}


# ---------------------------------------------------------------- data
_ROOT_CACHE = {}


def _root_data(path):
    key = os.path.abspath(path) if path else None
    if key not in _ROOT_CACHE:
        if key is None:
            with open(os.path.join(DATA_DIR, "rootnode.json")) as f:
                _ROOT_CACHE[key] = load_packed(json.load(f))
        else:
            _ROOT_CACHE[key] = load_dat(os.path.join(key, "RootNode.dat"))
    p, s = _ROOT_CACHE[key]
    return dict(p), dict(s)


_WIND = {}


def wind_bounds(scennum, path=None):
    """(MinNondispatchablePower, MaxNondispatchablePower) of NodeN.dat as {(n, t): v}."""
    if path is not None:
        p, _ = load_dat(os.path.join(path, f"Node{scennum}.dat"))
        return p.get("MinNondispatchablePower", {}), p.get("MaxNondispatchablePower", {})
    if "packed" not in _WIND:
        with np.load(os.path.join(DATA_DIR, "wind_1000scen.npz")) as z:
            _WIND["packed"] = (z["node"].copy(), z["lo"].copy(), z["hi"].copy(), [str(g) for g in z["gens"]])
    node, lo, hi, gens = _WIND["packed"]
    k = int(np.searchsorted(node, scennum))
    if k >= len(node) or node[k] != scennum:
        raise ValueError(f"no packed wind data for Node{scennum} (have Node{node[0]}..Node{node[-1]})")
    T = lo.shape[2]
    mn = {(g, t + 1): float(lo[k, i, t]) for i, g in enumerate(gens) for t in range(T)}
    mx = {(g, t + 1): float(hi[k, i, t]) for i, g in enumerate(gens) for t in range(T)}
    return mn, mx


class UCData:
    """The derived parameters of ReferenceModel_OK.py for one scenario's data."""

    def __init__(self, p, s):
        self.T = int(p["NumTimePeriods"])
        self.TPL = p.get("TimePeriodLength", 1.0)                       # :130
        self.times = list(range(INITIAL_TIME, self.T + 1))              # :134
        self.buses = list(s["Buses"])
        self.gens = list(s["ThermalGenerators"])
        self.gens_at = {b: list(s.get(f"ThermalGeneratorsAtBus[{b}]", [])) for b in self.buses}
        self.nd_at = {b: list(s.get(f"NondispatchableGeneratorsAtBus[{b}]", [])) for b in self.buses}
        nd = set()
        for b in self.buses:
            nd.update(self.nd_at[b])
        self.nd_gens = sorted(nd)                                        # :208-214
        self.must_run = [g for g in self.gens if p.get("MustRun", {}).get(g, 0)]
        if s.get("Storage"):
            raise NotImplementedError("storage units (ReferenceModel_OK.py:885-1437) are not in the UC data")
        if p.get("NumTransmissionLines", 0):
            raise NotImplementedError("transmission lines: the UC data is a single bus")
        self.demand = {(b, t): float(p["Demand"].get((b, t), 0.0)) for b in self.buses for t in self.times}
        self.total_demand = {t: sum(self.demand[b, t] for b in self.buses) for t in self.times}  # :250-252
        rf = p.get("ReserveFactor", -1.0)                                # :276-287
        rr = p.get("ReserveRequirement", {})
        self.reserve = {t: (rf * self.total_demand[t] if rf > 0 else float(rr.get(t, 0.0))) for t in self.times}
        self.lmp = float(p.get("LoadMismatchPenalty", BIG_PENALTY))
        self.rsp = float(p.get("ReserveShortfallPenalty", MODERATELY_BIG_PENALTY))
        g_ = self.gens
        P = lambda nm, d=0.0: {g: float(p.get(nm, {}).get(g, d)) for g in g_}  # noqa: E731
        self.pmin, self.pmax = P("MinimumPowerOutput"), P("MaximumPowerOutput")
        self.fuel = P("FuelCost", 1.0)                                   # :598
        self.shutdown_fixed = P("ShutdownFixedCost")                     # :812
        self.t0state = P("UnitOnT0State")
        self.pt0 = P("PowerGeneratedT0")
        self.mut = {g: int(p.get("MinimumUpTime", {}).get(g, 0)) for g in g_}
        self.mdt = {g: int(p.get("MinimumDownTime", {}).get(g, 0)) for g in g_}
        cap = lambda v, g: self.pmax[g] if v > self.pmax[g] else v       # noqa: E731
        self.ru = {g: cap(float(p["NominalRampUpLimit"][g]) * self.TPL, g) for g in g_}    # :357-363
        self.rd = {g: cap(float(p["NominalRampDownLimit"][g]) * self.TPL, g) for g in g_}  # :365-371
        self.su = {g: cap(float(p["StartupRampLimit"][g]), g) for g in g_}                 # :373-379
        self.sd = {g: cap(float(p["ShutdownRampLimit"][g]), g) for g in g_}                # :381-387
        self.smut = {g: min(int(round(self.mut[g] / self.TPL)), self.T) for g in g_}       # :397-400
        self.smdt = {g: min(int(round(self.mdt[g] / self.TPL)), self.T) for g in g_}       # :402-405
        self.on_t0 = {g: int(self.t0state[g] >= 1) for g in g_}                            # :420-423
        self.init_on = {g: (0 if not self.on_t0[g] else int(min(self.T, round(
            max(0, self.mut[g] - self.t0state[g]) / self.TPL)))) for g in g_}              # :445-452
        self.init_off = {g: (0 if self.on_t0[g] else int(min(self.T, round(
            max(0, self.mdt[g] + self.t0state[g]) / self.TPL)))) for g in g_}              # :454-461
        for g in g_:                                                      # :467-472
            lo, hi = self.pmin[g] * self.on_t0[g], self.pmax[g] * self.on_t0[g]
            if not (lo <= self.pt0[g] <= hi):
                raise ValueError(f"PowerGeneratedT0 of {g} outside its limits")
        # piecewise cost data (:498-611, 643-746); PiecewiseType is "Absolute" unless a
        # quadratic cost is given (:501-510)
        if any(p.get(nm, {}).get(g, 0.0) for nm in ("ProductionCostA0", "ProductionCostA1",
                                                    "ProductionCostA2") for g in g_):
            raise NotImplementedError("quadratic production costs (PiecewiseType NoPiecewise)")
        self.pw_pts, self.pw_vals, self.min_prod_cost = {}, {}, {}
        for g in g_:
            pts, vals = _validated_piecewise(s.get(f"CostPiecewisePoints[{g}]", []),
                                             s.get(f"CostPiecewiseValues[{g}]", []),
                                             self.pmin[g], self.pmax[g], g)
            mpc = vals[0] * self.fuel[g] if len(pts) > 1 else 0.0        # :603-611
            self.min_prod_cost[g] = mpc
            base = mpc / self.fuel[g]
            rel = [x - self.pmin[g] for x in pts]                        # :654-663
            if any(x < 0.0 for x in rel):
                raise ValueError(f"negative piecewise level for {g}")
            self.pw_pts[g] = rel
            self.pw_vals[g] = {x: v - base for x, v in zip(rel, vals)}
        # startup lags / costs (:755-806)
        self.lags, self.scosts = {}, {}
        for g in g_:
            lags = [int(x) for x in _ordered_set(s.get(f"StartupLags[{g}]", [self.mdt[g]]))]
            costs = [float(x) for x in _ordered_set(s.get(f"StartupCosts[{g}]", [0.0]))]
            if not lags or lags[0] != self.mdt[g] or any(a >= b for a, b in zip(lags, lags[1:])):
                raise ValueError(f"startup lags of {g} invalid (:765-781)")
            if len(lags) != len(costs):
                raise ValueError(f"startup lag / cost cardinality of {g} (:793-798)")
            self.lags[g], self.scosts[g] = lags, costs
        # ValidShutdownTimePeriods / ShutdownHotStartupPairs (:1020-1027)
        self.vstp, self.pairs = {}, {}
        for g in g_:
            v = list(self.times) + ([] if self.t0state[g] >= 0 else [INITIAL_TIME + int(self.t0state[g])])
            self.vstp[g] = v
            f, l = self.lags[g][0], self.lags[g][-1]
            self.pairs[g] = [(tp, t) for tp in v for t in self.times if f <= t - tp < l]

    def production_cost(self, g, x):
        """production_cost_function (:1444-1445)."""
        return self.TPL * self.pw_vals[g][x] * self.fuel[g]

    def slopes(self, g):
        pts = self.pw_pts[g]
        return [(self.production_cost(g, pts[i + 1]) - self.production_cost(g, pts[i])) / (pts[i + 1] - pts[i])
                for i in range(len(pts) - 1)]

    def compute_production_costs(self, g, avg_power):
        """ComputeProductionCosts (:1483-1501), the rho helper."""
        pts = self.pw_pts[g]
        ev = [0.0] * (len(pts) - 1)
        for l in range(len(ev)):
            if avg_power >= pts[l + 1]:
                ev[l] = pts[l + 1] - pts[l]
            elif avg_power < pts[l + 1]:
                ev[l] = avg_power - pts[l]
                break
        return sum(sl * e for sl, e in zip(self.slopes(g), ev))


def _ordered_set(seq):
    """A Pyomo ordered Set keeps the first occurrence of each element."""
    out, seen = [], set()
    for x in seq:
        if x not in seen:
            seen.add(x)
            out.append(x)
    return out


def _validated_piecewise(points, values, pmin, pmax, g):
    """validate_cost_piecewise_points_and_values_rule (:530-593)."""
    points, values = _ordered_set(points), _ordered_set(values)
    if len(points) == 0:
        raise ValueError(f"no piecewise cost points for {g}")
    new_points = sorted(points)
    new_values = sorted(values)
    if pmin not in new_points:
        new_points.insert(0, pmin)
    if pmax not in new_points:
        new_points.append(pmax)
    new_points = [x for x in new_points if pmin <= x <= pmax]
    if len(new_points) < len(new_values):
        new_values = new_values[:len(new_points)]
    i = 1
    while len(new_points) > len(new_values):
        new_values.append(new_values[-1] + i)
        i += 1
    return [float(x) for x in new_points], [float(v) for v in new_values]


def load_data(scennum, path=None):
    p, s = _root_data(path)
    mn, mx = wind_bounds(scennum, path)
    p["MinNondispatchablePower"] = {**p.get("MinNondispatchablePower", {}), **mn}
    p["MaxNondispatchablePower"] = {**p.get("MaxNondispatchablePower", {}), **mx}
    return UCData(p, s), p


# ---------------------------------------------------------------- model
def _build(d, p, name):
    """The LP relaxation of ReferenceModel_OK.py as a LinearModel (rows in the order
    the reference declares its constraints)."""
    mdl = LinearModel(name)
    T, G, times = d.T, d.gens, d.times
    keys = sorted((g, t) for g in G for t in times)
    V = {}

    def add(fam, key, lb, ub, cost=0.0):
        V[fam, key] = mdl.var(f"{fam}[{','.join(str(k) for k in (key if isinstance(key, tuple) else (key,)))}]",
                              lb, ub, cost)

    # UnitOn first: the nonants, sorted by key (scenario_tree.py:39)
    for g, t in keys:
        add("UnitOn", (g, t), 0.0, 1.0, d.min_prod_cost[g] * d.TPL)     # :1768 (commitment cost)
    for g, t in keys:
        add("UnitStart", (g, t), 0.0, 1.0)                               # :1014
    for g, t in keys:
        add("UnitStop", (g, t), 0.0, 1.0)                                # :1017
    for g in G:
        for tp, t in d.pairs[g]:
            add("StartupIndicator", (g, tp, t), 0.0, 1.0)                # :1034
    for g, t in keys:
        add("PowerGeneratedAboveMinimum", (g, t), 0.0, d.pmax[g] - d.pmin[g])         # :1037-1039
    for g, t in keys:
        add("MaximumPowerAvailableAboveMinimum", (g, t), 0.0, d.pmax[g] - d.pmin[g])  # :1056
    mn, mx = p["MinNondispatchablePower"], p["MaxNondispatchablePower"]
    for n in d.nd_gens:
        for t in times:
            add("NondispatchablePowerUsed", (n, t), float(mn.get((n, t), 0.0)),
                float(mx.get((n, t), 0.0)))                              # :1051-1053
    for b in d.buses:
        for t in times:
            add("Angle", (b, t), -3.14159265, 3.14159265)                # :1063
    for g, t in keys:
        add("ProductionCost", (g, t), 0.0, INF, 1.0)                     # :1126, :1776
    for g, t in keys:
        add("StartupCost", (g, t), 0.0, INF, 1.0)                        # :1129, :1768
    for g, t in keys:
        add("ShutdownCost", (g, t), 0.0, INF, 1.0)                       # :1130, :1768
    for t in times:
        add("TotalProductionCost", t, 0.0, INF)                          # :1133
    for t in times:
        add("TotalNoLoadCost", t, 0.0, INF)                              # :1136
    for b in d.buses:
        for t in times:
            add("LoadGenerateMismatch", (b, t), -INF, INF)               # :1141
    for b in d.buses:
        for t in times:
            add("posLoadGenerateMismatch", (b, t), 0.0, INF, d.lmp)      # :1142, :1777
    for b in d.buses:
        for t in times:
            add("negLoadGenerateMismatch", (b, t), 0.0, INF, d.lmp)      # :1143, :1777
    for t in times:
        add("ReserveShortfall", t, 0.0, INF, d.rsp)                      # :1145, :1778
    for g, t in keys:
        pts = d.pw_pts[g]
        for i in range(len(pts) - 1):
            add("PiecewiseProduction", (g, t, i), 0.0, pts[i + 1] - pts[i])  # :1448-1455

    On = lambda g, t: V["UnitOn", (g, t)]                # noqa: E731
    St = lambda g, t: V["UnitStart", (g, t)]             # noqa: E731
    Sp = lambda g, t: V["UnitStop", (g, t)]              # noqa: E731
    SI = lambda g, tp, t: V["StartupIndicator", (g, tp, t)]  # noqa: E731
    PGA = lambda g, t: V["PowerGeneratedAboveMinimum", (g, t)]  # noqa: E731
    MPA = lambda g, t: V["MaximumPowerAvailableAboveMinimum", (g, t)]  # noqa: E731
    row = mdl.row

    def terms(*parts):
        return [(v, a) for (v, a) in parts if a != 0.0]

    for b in d.buses:                                                    # :1154-1160
        row([(V["posLoadGenerateMismatch", (b, t)], 1.0) for t in times], 0.0, INF,
            f"PosLoadGenerateMismatchTolerance[{b}]")
    for b in d.buses:
        row([(V["negLoadGenerateMismatch", (b, t)], 1.0) for t in times], 0.0, INF,
            f"NegLoadGenerateMismatchTolerance[{b}]")
    for t in times:                                                      # :1065-1068
        row([(V["Angle", (d.buses[0], t)], 1.0)], 0.0, 0.0, f"FixFirstAngle[{t}]")
    for b in d.buses:                                                    # :1176-1195
        for t in times:
            tt = []
            for g in d.gens_at[b]:
                tt += [(PGA(g, t), 1.0), (On(g, t), d.pmin[g])]
            tt += [(V["NondispatchablePowerUsed", (n, t)], 1.0) for n in d.nd_at[b]]
            tt.append((V["LoadGenerateMismatch", (b, t)], 1.0))
            row(terms(*tt), d.demand[b, t], d.demand[b, t], f"PowerBalance[{b},{t}]")
    for b in d.buses:                                                    # :1198-1200
        for t in times:
            row([(V["posLoadGenerateMismatch", (b, t)], 1.0), (V["negLoadGenerateMismatch", (b, t)], -1.0),
                 (V["LoadGenerateMismatch", (b, t)], -1.0)], 0.0, 0.0,
                f"DefinePosNegLoadGenerateMismatch[{b},{t}]")
    for t in times:                                                      # :1203-1205
        row([(V["ReserveShortfall", t], 1.0)], -INF, d.reserve[t], f"BoundReserveShortfall[{t}]")
    for t in times:                                                      # :1214-1232
        tt = []
        for g in G:
            tt += [(MPA(g, t), 1.0), (On(g, t), d.pmin[g])]
        tt += [(V["NondispatchablePowerUsed", (n, t)], 1.0) for n in d.nd_gens]
        tt += [(V["LoadGenerateMismatch", (b, t)], 1.0) for b in d.buses]
        tt.append((V["ReserveShortfall", t], 1.0))
        row(terms(*tt), d.total_demand[t] + d.reserve[t], INF, f"EnforceReserveRequirements[{t}]")
    for g, t in keys:                                                    # :1266-1269
        row([(PGA(g, t), 1.0), (MPA(g, t), -1.0)], -INF, 0.0, f"EnforceGeneratorOutputLimitsPartB[{g},{t}]")
    for g in d.must_run:                                                 # :1272-1275
        for t in times:
            row([(On(g, t), 1.0)], 1.0, 1.0, f"EnforceMustRun[{g},{t}]")
    span = {g: d.pmax[g] - d.pmin[g] for g in G}
    for g, t in keys:                                                    # :1287-1293
        if d.mut[g] != 1:
            continue
        row(terms((MPA(g, t), 1.0), (On(g, t), -span[g]), (St(g, t), d.pmax[g] - d.su[g])), -INF, 0.0,
            f"power_limit_from_start[{g},{t}]")
    for g, t in keys:                                                    # :1295-1303
        if d.mut[g] != 1:
            continue
        tt = [(MPA(g, t), 1.0), (On(g, t), -span[g])]
        if t != T:
            tt.append((Sp(g, t + 1), d.pmax[g] - d.sd[g]))
        row(terms(*tt), -INF, 0.0, f"power_limit_from_stop[{g},{t}]")
    for g, t in keys:                                                    # :1305-1315
        if d.mut[g] == 1:
            continue
        tt = [(MPA(g, t), 1.0), (On(g, t), -span[g]), (St(g, t), d.pmax[g] - d.su[g])]
        if t != T:
            tt.append((Sp(g, t + 1), d.pmax[g] - d.sd[g]))
        row(terms(*tt), -INF, 0.0, f"power_limit_from_start_stop[{g},{t}]")
    for g, t in keys:                                                    # :1325-1334
        if t == INITIAL_TIME:
            row([(MPA(g, t), 1.0)], -INF, (d.pt0[g] - d.pmin[g]) * d.on_t0[g] + d.ru[g],
                f"EnforceMaxAvailableRampUpRates[{g},{t}]")
        else:
            row([(MPA(g, t), 1.0), (PGA(g, t - 1), -1.0)], -INF, d.ru[g],
                f"EnforceMaxAvailableRampUpRates[{g},{t}]")
    for g, t in keys:                                                    # :1338-1349 (enforce_t1_ramp_rates)
        if t == INITIAL_TIME:
            row([(PGA(g, t), -1.0)], -INF, d.rd[g] - (d.pt0[g] - d.pmin[g]) * d.on_t0[g],
                f"EnforceScaledNominalRampDownLimits[{g},{t}]")
        else:
            row([(PGA(g, t - 1), 1.0), (PGA(g, t), -1.0)], -INF, d.rd[g],
                f"EnforceScaledNominalRampDownLimits[{g},{t}]")
    for g, t in keys:                                                    # :1457-1459
        npc = len(d.pw_pts[g]) - 1
        row([(V["PiecewiseProduction", (g, t, i)], 1.0) for i in range(npc)] + [(PGA(g, t), -1.0)],
            0.0, 0.0, f"PiecewiseProductionSum[{g},{t}]")
    for g, t in keys:                                                    # :1461-1463
        pts = d.pw_pts[g]
        for i in range(len(pts) - 1):
            row(terms((V["PiecewiseProduction", (g, t, i)], 1.0), (On(g, t), -(pts[i + 1] - pts[i]))),
                -INF, 0.0, f"PiecewiseProductionLimtis[{g},{t},{i}]")
    for g, t in keys:                                                    # :1466-1470: one copy per
        sl = d.slopes(g)                                                 # index i, as the reference
        for i in range(len(sl)):                                         # declares it
            row([(V["ProductionCost", (g, t)], 1.0)] +
                terms(*[(V["PiecewiseProduction", (g, t, k)], -sl[k]) for k in range(len(sl))]),
                0.0, 0.0, f"PiecewiseProductionCostsConstr[{g},{t},{i}]")
    for t in times:                                                      # :1505-1508
        row([(V["TotalProductionCost", t], 1.0)] + [(V["ProductionCost", (g, t)], -1.0) for g in G],
            0.0, 0.0, f"ComputeTotalProductionCost[{t}]")
    for t in times:                                                      # :1510-1513
        row([(V["TotalNoLoadCost", t], 1.0)] + terms(*[(On(g, t), -d.min_prod_cost[g]) for g in G]),
            0.0, 0.0, f"ComputeTotalNoLoadCost[{t}]")
    for g, t in keys:                                                    # :1519-1521
        row([(SI(g, tp, s), 1.0) for (tp, s) in d.pairs[g] if s == t] + [(St(g, t), -1.0)], -INF, 0.0,
            f"StartupMatch[{g},{t}]")
    for g in G:                                                          # :1523-1536
        for t in d.vstp[g]:
            first = [(tp, s) for (tp, s) in d.pairs[g] if tp == t]
            if t < INITIAL_TIME:
                if first:
                    row([(SI(g, tp, s), 1.0) for (tp, s) in first], -INF, 1.0, f"ShutdownMatch[{g},{t}]")
            else:
                row([(SI(g, tp, s), 1.0) for (tp, s) in first] + [(Sp(g, t), -1.0)], -INF, 0.0,
                    f"ShutdownMatch[{g},{t}]")
    for g, t in keys:                                                    # :1538-1545
        lags, costs = d.lags[g], d.scosts[g]
        tt = [(V["StartupCost", (g, t)], 1.0), (St(g, t), -costs[-1])]
        for s in range(1, len(lags)):
            coef = costs[s - 1] - costs[-1]
            for tp in d.vstp[g]:
                if lags[s - 1] <= t - tp < lags[s]:
                    tt.append((SI(g, tp, t), -coef))
        row(terms(*tt), 0.0, 0.0, f"ComputeStartupCost2[{g},{t}]")
    for g, t in keys:                                                    # :1552-1555
        row(terms((V["ShutdownCost", (g, t)], 1.0), (Sp(g, t), -d.shutdown_fixed[g])), 0.0, 0.0,
            f"ComputeShutdownCosts[{g},{t}]")
    for g in G:                                                          # :1562-1567
        if d.init_on[g] == 0:
            continue
        ts = [t for t in times if t <= d.init_on[g]]
        row([(On(g, t), 1.0) for t in ts], float(len(ts)), float(len(ts)), f"EnforceUpTimeConstraintsInitial[{g}]")
    for g, t in keys:                                                    # :1569-1575
        if t < d.smut[g]:
            continue
        row([(St(g, i), 1.0) for i in times if t - d.smut[g] + 1 <= i <= t] + [(On(g, t), -1.0)], -INF, 0.0,
            f"unit_start[{g},{t}]")
    for g in G:                                                          # :1583-1588
        if d.init_off[g] == 0:
            continue
        row([(On(g, t), 1.0) for t in times if t <= d.init_off[g]], 0.0, 0.0,
            f"EnforceDownTimeConstraintsInitial[{g}]")
    for g, t in keys:                                                    # :1590-1596
        if t < d.smdt[g]:
            continue
        row([(Sp(g, i), 1.0) for i in times if t - d.smdt[g] + 1 <= i <= t] + [(On(g, t), 1.0)], -INF, 1.0,
            f"unit_stop[{g},{t}]")
    for g, t in keys:                                                    # :1603-1608
        if t == 1:
            row([(On(g, t), 1.0), (St(g, t), -1.0), (Sp(g, t), 1.0)], float(d.on_t0[g]), float(d.on_t0[g]),
                f"start_stop[{g},{t}]")
        else:
            row([(On(g, t), 1.0), (On(g, t - 1), -1.0), (St(g, t), -1.0), (Sp(g, t), 1.0)], 0.0, 0.0,
                f"start_stop[{g},{t}]")
    mdl.uc = d
    mdl.uc_vars = V
    mdl.uc_wind_cols = [V["NondispatchablePowerUsed", (n, t)].index for n in d.nd_gens for t in times]
    return mdl, keys


def scenario_creator(scenario_name, path=None, scenario_count=None, num_scens=None):
    """uc_funcs.py:53-84: one scenario, nonants UnitOn[*,*] on the ROOT node."""
    scennum = extract_num(scenario_name)
    d, p = load_data(scennum, path)
    mdl, keys = _build(d, p, scenario_name)
    attach_root_node(mdl, None, [mdl.uc_vars["UnitOn", k] for k in keys])
    mdl._mpisppy_probability = (1.0 / num_scens) if num_scens else "uniform"
    return mdl


def scenario_names_creator(num_scens, start=None):
    """Scenario1..ScenarioN map to Node1..NodeN (extract_num, uc_funcs.py:28)."""
    start = 1 if start is None else start
    return [f"Scenario{i}" for i in range(start, start + num_scens)]


def scenario_denouement(rank, scenario_name, scenario):
    pass


def scenario_rhos(scenario_instance, rho_scale_factor=0.1):
    """uc_funcs.py:99-116: rho = 0.1 * cost at the midpoint output, per UnitOn[g,t]."""
    d = scenario_instance.uc
    out = []
    for t in d.times:
        for g in d.gens:
            avg_power = d.pmin[g] + (d.pmax[g] - d.pmin[g]) / 2.0
            avg_cost = d.compute_production_costs(g, avg_power) + d.min_prod_cost[g]
            out.append((id(scenario_instance.uc_vars["UnitOn", (g, t)]), rho_scale_factor * avg_cost))
    return out


def _rho_setter(scenario_instance):
    return scenario_rhos(scenario_instance)


def rho_vector(tmpl, rho_scale_factor=0.1):
    """The same rhos in nonant order, as an array (what the PH engine consumes)."""
    by_id = dict(scenario_rhos(tmpl, rho_scale_factor))
    nl = tmpl._mpisppy_node_list[0].nonant_vardata_list
    return np.array([by_id[id(v)] for v in nl])


def batch_creator(scenario_names, path=None, num_scens=None, **kwargs):
    """ScenarioBatch for ``scenario_names``: pattern, costs and rows from the first
    scenario; per scenario only the wind bounds change."""
    names = list(scenario_names)
    S = len(names)
    tmpl = scenario_creator(names[0], path=path, num_scens=num_scens)
    tb = batch_from_models([names[0]], [tmpl], num_all_scens=num_scens or S)
    wc = np.array(tmpl.uc_wind_cols, dtype=np.int64)
    d = tmpl.uc
    lb = np.repeat(tb.lb, S, axis=0)
    ub = np.repeat(tb.ub, S, axis=0)
    for s, nm in enumerate(names):
        mn, mx = wind_bounds(extract_num(nm), path)
        lb[s, wc] = [float(mn.get((n, t), 0.0)) for n in d.nd_gens for t in d.times]
        ub[s, wc] = [float(mx.get((n, t), 0.0)) for n in d.nd_gens for t in d.times]
    rep = lambda a: np.repeat(a, S, axis=0)  # noqa: E731
    prob = np.full(S, 1.0 / (num_scens or S))
    b = ScenarioBatch(names, tb.row_ptr, tb.col_idx, rep(tb.A_val), rep(tb.c), lb, ub, rep(tb.rl),
                      rep(tb.ru), rep(tb.q), rep(tb.obj_const), tb.nonant_col, tb.nonant_depth,
                      tb.nonant_off, np.zeros((S, 1), dtype=np.int32), ["ROOT"], prob, prob[:, None],
                      tb.sense, tb.var_names, tb.nonant_names)
    b.template = tmpl
    return b
