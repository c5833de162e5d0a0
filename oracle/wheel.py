"""Oracle restatement of the hub-and-spoke bounds (TEST INFRASTRUCTURE ONLY).

What the engine's co-located wheel computes, restated on the CPU with exact solvers:
  * Lagrangian outer bound   cylinders/lagrangian_bounder.py:19-60: W on, prox off,
                             bound = sum_s p_s min_x (f_s(x) + W_s x_N)   (spopt.py:346-391)
  * xhat inner bound         extensions/xhatbase.py:38-216: nonants of every scenario
                             fixed at the candidate's per-node values, E[f] over all
                             scenarios, None if one is infeasible
  * candidate order          cylinders/xhatshufflelooper_bounder.py:90-300:
                             random.Random(42).sample of the enumerated names, walked by
                             the scenario cycler (restated here independently)
  * hub bookkeeping          cylinders/hub.py:77-161, 202-226, 519-547 (trivial bound at
                             PH iteration 1, best bounds, rel/abs gap termination)
and the synchronous schedule of the engine's WheelSpinner (every sync: deliver W and
nonants, one Lagrangian solve, one xhat candidate, then receive the bounds).
"""
import math
import random

import numpy as np

from .lpqp import solve_lp_highs, solve_qp_ipm


def _solve(A, rl, ru, lb, ub, c, q):
    if not np.any(q):
        return solve_lp_highs(A, rl, ru, lb, ub, c)
    return solve_qp_ipm(A, rl, ru, lb, ub, c, q)


def lagrangian_bound(scens, W):
    """sum_s p_s min_x f_s(x) + W_s . x_nonant  (W: [S, nn])."""
    tot = []
    for k, s in enumerate(scens):
        A, rl, ru, lb, ub, c, q = s.arrays()
        c = c.copy()
        c[s.nonant_indices()] += W[k]
        x, obj, st = _solve(A, rl, ru, lb, ub, c, q)
        if st != 0:
            raise RuntimeError(f"oracle Lagrangian solve failed for {s.name}")
        tot.append(s.prob * obj)
    return math.fsum(tot)


def xhat_objective(scens, node_values):
    """E[f] with every scenario's nonants fixed at node_values[node] (None if infeasible)."""
    tot = []
    for s in scens:
        A, rl, ru, lb, ub, c, q = s.arrays()
        xf = np.full(len(c), np.nan)
        for (ndn, _cond, _stage, idx) in s.nodes:
            if ndn not in node_values:          # partial fix (fix_nonants_upto_stage)
                continue
            v = np.asarray(node_values[ndn], dtype=float)
            for o, j in enumerate(idx):
                xf[j] = min(max(v[o], lb[j]), ub[j])
        # eliminate the fixed columns (the IPM needs lb < ub): shift the row ranges and
        # add their objective contribution as a constant
        fx = ~np.isnan(xf)
        shift = A[:, fx] @ xf[fx]
        const = float(c[fx] @ xf[fx] + 0.5 * np.sum(q[fx] * xf[fx] ** 2))
        fr = ~fx
        rl, ru = rl - shift, ru - shift
        # rows left without a free column are pure feasibility checks: drop them
        live = np.any(A[:, fr] != 0.0, axis=1)
        tol = 1e-9 * (1.0 + np.abs(shift[~live]))
        if np.any(rl[~live] > tol) or np.any(ru[~live] < -tol):
            return None
        x, obj, st = _solve(A[live][:, fr], rl[live], ru[live], lb[fr], ub[fr], c[fr], q[fr])
        if st != 0:
            return None
        tot.append(s.prob * (obj + const))
    return math.fsum(tot)


def tree_ranges(all_nodenames, num_scens):
    """{non-leaf node: (first, last scenario index, has non-leaf kids)} of a balanced tree
    given by its node names (sputils._ScenTree, 672-772)."""
    if all_nodenames is None or list(all_nodenames) == ["ROOT"]:
        return {"ROOT": (0, num_scens - 1, False)}
    names = set(all_nodenames)
    out = {}
    counter = [0]

    def walk(nd):
        kids = []
        i = 0
        while f"{nd}_{i}" in names:
            kids.append(f"{nd}_{i}")
            i += 1
        if not kids:
            counter[0] += 1
            return False
        first = counter[0]
        leafy = [walk(k) for k in kids]
        out[nd] = (first, counter[0] - 1, any(leafy) or any(f"{k}_0" in names for k in kids))
        return True

    walk("ROOT")
    return out


def candidate_sequence(all_scenario_names, all_nodenames, count, reverse=True, iter_step=None, seed=42):
    """The first ``count`` results of the shuffle looper's candidate walk: dicts
    {node: scenario name} or None (end of an epoch).  Independent restatement of
    xhatshufflelooper_bounder.py:99-106 and 158-300."""
    rng = random.Random()
    rng.seed(seed)
    order = rng.sample(list(enumerate(all_scenario_names)), len(all_scenario_names))
    tree = tree_ranges(all_nodenames, len(all_scenario_names))
    multi = tree["ROOT"][2]
    nodes = list(tree.keys())
    step = (1 if iter_step is None else iter_step)
    if multi:
        bf0 = sum(1 for nd in all_nodenames if nd.count("_") == 1)
        step = bf0 if iter_step is None else iter_step
    use_rev = multi and (True if reverse is None else reverse)
    N = len(order)
    res = []
    rev = False
    seq = order
    cur = 0
    used = set()
    assign = {}

    def fill(empty):
        i = cur
        empty = list(empty)
        while empty:
            nm, ix = seq[i][1], seq[i][0]
            empty = [nd for nd in empty if not (tree[nd][0] <= ix <= tree[nd][1] and assign.__setitem__(nd, nm) is None)]
            i = (i + 1) % N

    def start(reversed_order):
        nonlocal seq, cur, used, assign, rev
        rev = reversed_order
        seq = list(reversed(order)) if reversed_order else order
        cur = 0
        used = set()
        assign = {}
        if multi:
            fill(nodes)
        else:
            assign["ROOT"] = seq[0][1]

    start(False)
    while len(res) < count:
        root = seq[cur][1]
        if root in used:
            res.append(None)
            start(use_rev and not rev)
            continue
        used.add(root)
        old = cur
        tgt = (old + step) % N
        c = tgt
        while seq[c][1] in used and (c + 1) % N != tgt:
            c = (c + 1) % N
        cur = c
        passed = [seq[i % N][1] for i in range(old, old + ((c - old) % N or N))]
        if multi:
            stale = [nd for nd in nodes if assign[nd] in passed]
            for nd in stale:
                assign[nd] = None
            fill(stale)
            res.append(dict(assign))          # live dict: already advanced (see product docstring)
        else:
            res.append({"ROOT": root})
            assign = {"ROOT": seq[cur][1]}
    return res


class OracleWheel:
    """PH hub + Lagrangian spoke + xhat shuffle spoke, synchronous schedule."""

    def __init__(self, oracle_ph, all_scenario_names, all_nodenames=None, rel_gap=None, abs_gap=None,
                 minimizing=True):
        self.ph = oracle_ph
        self.names = list(all_scenario_names)
        self.all_nodenames = all_nodenames
        self.rel_gap = rel_gap
        self.abs_gap = abs_gap
        self.minimizing = minimizing
        self.best_inner = math.inf
        self.best_outer = -math.inf
        self.best_xhat_bound = math.inf
        self.trace = []
        self._cands = candidate_sequence(self.names, all_nodenames, 10 * len(self.names) + 10)
        self._ci = 0

    def _sync(self):
        ph = self.ph
        # Lagrangian spoke with the hub's current W
        lb = lagrangian_bound(ph.scens, ph.W)
        if lb > self.best_outer:
            self.best_outer = lb
        # xhat spoke: next candidate from the hub's nonants
        cand = self._cands[self._ci]
        self._ci += 1
        if cand is None:
            cand = self._cands[self._ci]
            self._ci += 1
        idx = {nm: k for k, nm in enumerate(self.names)}
        values = {}
        for ndn, sname in cand.items():
            k = idx[sname]
            for (nd, a, b) in ph.node_slices[k]:
                if nd == ndn:
                    values[ndn] = ph.x[k, a:b].copy()
        obj = xhat_objective(ph.scens, values)
        if obj is not None and obj < self.best_inner:
            self.best_inner = obj
        return lb, obj, cand

    def gaps(self):
        abs_gap = self.best_inner - self.best_outer
        rel_gap = abs_gap / abs(self.best_outer) if (math.isfinite(abs_gap) and self.best_outer != 0) else math.inf
        return abs_gap, rel_gap

    def run(self, max_iterations, convthresh=0.0):
        ph = self.ph
        self.spoke_trivial = lagrangian_bound(ph.scens, np.zeros_like(ph.W))
        self.best_outer = self.spoke_trivial
        ph.iter0()
        self._sync()
        for it in range(1, max_iterations + 1):
            ph.compute_xbar()
            ph.update_W()
            ph.conv = ph.convergence_diff()
            if ph.conv < convthresh:
                break
            ph.solve_loop()
            lb, obj, cand = self._sync()
            if it == 1 and ph.trivial_bound > self.best_outer:
                self.best_outer = ph.trivial_bound
            a, r = self.gaps()
            self.trace.append({"iter": it, "outer": self.best_outer, "inner": self.best_inner,
                               "lagrangian": lb, "xhat": obj, "cand": dict(cand)})
            if (self.rel_gap is not None and r <= self.rel_gap) or (self.abs_gap is not None and a <= self.abs_gap):
                break
        # final Lagrangian pass with the last W (the engine's send_terminate delivery)
        lb = lagrangian_bound(ph.scens, ph.W)
        if lb > self.best_outer:
            self.best_outer = lb
        return self.best_outer, self.best_inner
