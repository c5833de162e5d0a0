"""Oracle restatement of the PH hot path (TEST INFRASTRUCTURE ONLY).

Follows, step for step:
  * PHBase.Iter0            phbase.py:758-872  (LP solves with W_on = prox_on = 0,
                                                E1 / feasibility checks, rho_setter
                                                after the solve, trivial bound = Ebound)
  * PHBase.iterk_loop       phbase.py:875-979  (x̄ -> W -> conv -> break? -> solve)
  * _Compute_Xbar           phbase.py:27-107   (prob_coeff = pi_s / pi_node, spbase.py:384-391)
  * Update_W                phbase.py:293-318
  * convergence_diff        phbase.py:321-343  (mean of per-rank means)
  * attach_PH_to_objective  phbase.py:617-699  (f + W x + rho/2 (x - x̄)^2, minimise)
  * SPOpt.Ebound/Eobjective spopt.py:310-391
  * _ScenTree.scen_names_to_ranks sputils.py:774-840 (contiguous slices)
"""
import math
import numpy as np

from .lpqp import solve_lp_highs, solve_qp_ipm, farmer_prox_exact


def rank_slices(num_scens, n_proc):
    """sputils.py:798-810."""
    if n_proc == 1:
        return [list(range(num_scens))]
    avg = num_scens / n_proc
    return [list(range(int(i * avg), int((i + 1) * avg))) for i in range(n_proc)]


class OraclePH:
    """Single-process restatement of PH over a list of oracle ScenLP scenarios."""

    def __init__(self, scens, default_rho, n_proc=1, rho_setter=None, solver="ipm",
                 farmer_info=None, var_prob=None):
        self.scens = scens
        S = len(scens)
        for s in scens:
            if s.prob is None:           # spbase.py:515-520 uniform default
                s.prob = 1.0 / S
        self.n_proc = n_proc
        self.slices = rank_slices(S, n_proc)
        self.solver = solver
        self.farmer_info = farmer_info  # (crops_sorted, [Y dicts], cm) for the closed form
        self.arr = [s.arrays() for s in scens]
        self.nonant_idx = [s.nonant_indices() for s in scens]
        self.nn = len(self.nonant_idx[0])
        # node bookkeeping: per scenario the list of (node name, slice into the nonant vector)
        self.node_slices = []
        self.prob_coeff = []
        for s in scens:
            sl = []
            pc = []
            off = 0
            uncond = 1.0
            for (ndn, cond, _stage, idx) in s.nodes:
                uncond = uncond * cond if ndn != "ROOT" else 1.0
                sl.append((ndn, off, off + len(idx)))
                pc.append(s.prob / uncond)        # spbase.py:390
                off += len(idx)
            self.node_slices.append(sl)
            self.prob_coeff.append(pc)
        # variable probabilities (spbase.py:394-437): per-nonant coefficients [S, nn] replacing
        # the node's prob_coeff in the x̄ sums, and W masked where they are 0 (phbase.py:315-318)
        self.var_prob = None if var_prob is None else np.asarray(var_prob, dtype=np.float64)
        self.rho = np.full((S, self.nn), float(default_rho))
        self.rho_setter = rho_setter
        self.W = np.zeros((S, self.nn))
        self.xbar = np.zeros((S, self.nn))
        self.x = np.zeros((S, self.nn))
        self.obj = np.zeros(S)
        self.outer = np.zeros(S)
        self.W_on = 0
        self.prox_on = 0
        self.history = []

    # -- one scenario solve (spopt.py:85-223 with the objective of phbase.py:617-699)
    def _solve_one(self, k):
        A, rl, ru, lb, ub, c, q = self.arr[k]
        idx = self.nonant_idx[k]
        c = c.copy()
        q = q.copy()
        const = 0.0
        if self.W_on:
            c[idx] += self.W[k]
        if self.prox_on:
            c[idx] -= self.rho[k] * self.xbar[k]
            q[idx] += self.rho[k]
            const = 0.5 * float(np.sum(self.rho[k] * self.xbar[k] ** 2))
        if self.solver == "farmer" and self.prox_on:
            crops_sorted, Ys, cm = self.farmer_info
            xn, obj = farmer_prox_exact(crops_sorted, Ys[k], self.W[k] if self.W_on else 0 * self.W[k],
                                        self.xbar[k], self.rho[k], cm)
            self.x[k] = xn
            self.obj[k] = obj
            self.outer[k] = obj
            return
        if (not self.prox_on) and not np.any(q):
            x, obj, st = solve_lp_highs(A, rl, ru, lb, ub, c)
        else:
            x, obj, st = solve_qp_ipm(A, rl, ru, lb, ub, c, q)
        if st != 0:
            raise RuntimeError(f"oracle solve failed for {self.scens[k].name}: status {st}")
        self.x[k] = x[idx]
        self.obj[k] = obj + const
        self.outer[k] = obj + const   # exact solver: bound == objective

    def solve_loop(self):
        for k in range(len(self.scens)):
            self._solve_one(k)

    # -- phbase.py:27-107
    def compute_xbar(self):
        acc = {}
        for k in range(len(self.scens)):
            for (ndn, a, b), pc in zip(self.node_slices[k], self.prob_coeff[k]):
                xs = self.x[k, a:b]
                if self.var_prob is not None:
                    pc = self.var_prob[k, a:b]
                if ndn not in acc:
                    acc[ndn] = [np.zeros(b - a), np.zeros(b - a)]
                acc[ndn][0] += pc * xs
                acc[ndn][1] += pc * xs ** 2
        for k in range(len(self.scens)):
            for (ndn, a, b) in self.node_slices[k]:
                self.xbar[k, a:b] = acc[ndn][0]
        self.node_xbar = {nd: v[0] for nd, v in acc.items()}
        self.node_xsqbar = {nd: v[1] for nd, v in acc.items()}

    # -- phbase.py:293-318
    def update_W(self):
        self.W += self.rho * (self.x - self.xbar)
        if self.var_prob is not None:
            self.W *= (self.var_prob != 0.0)                       # prob0_mask

    # -- phbase.py:321-343
    def convergence_diff(self):
        tot = 0.0
        for sl in self.slices:
            d = np.abs(self.x[sl] - self.xbar[sl]).sum()
            tot += d / (len(sl) * self.nn)
        return tot / self.n_proc

    # -- spopt.py:346-391 / 310-343
    def Ebound(self):
        return sum(math.fsum(self.scens[k].prob * self.outer[k] for k in sl) for sl in self.slices)

    def Eobjective(self):
        return sum(math.fsum(self.scens[k].prob * self.obj[k] for k in sl) for sl in self.slices)

    # -- phbase.py:758-872
    def iter0(self):
        self.W_on = 0
        self.prox_on = 0
        self.solve_loop()
        E1 = sum(s.prob for s in self.scens)
        if abs(1 - E1) > 1e-5:
            raise RuntimeError(f"Total probability of scenarios was {E1}")
        if self.rho_setter is not None:
            for k, s in enumerate(self.scens):
                for (vi, r) in self.rho_setter(s):
                    self.rho[k, self.nonant_idx[k].index(vi)] = r
        self.trivial_bound = self.Ebound()
        self.iter0_x = self.x.copy()
        self.iter0_obj = self.obj.copy()
        self.W_on = 1
        self.prox_on = 1
        return self.trivial_bound

    # -- phbase.py:875-979
    def iterk_loop(self, max_iterations, convthresh, record=True):
        self.conv = None
        self.iters_done = 0
        for it in range(1, max_iterations + 1):
            self.compute_xbar()
            self.update_W()
            self.conv = self.convergence_diff()
            if record:
                self.history.append({"iter": it, "conv": self.conv, "xbar": self.xbar.copy(),
                                     "W": self.W.copy()})
            self.iters_done = it
            if self.conv < convthresh:
                self.converged_at = it
                return it
            self.solve_loop()
            if record:
                self.history[-1]["x"] = self.x.copy()
                self.history[-1]["obj"] = self.obj.copy()
        self.converged_at = None
        return max_iterations

    def ph_main(self, max_iterations, convthresh):
        """opt/ph.py:25-71: (conv, Eobj, trivial_bound)."""
        tb = self.iter0()
        self.iterk_loop(max_iterations, convthresh)
        return self.conv, self.Eobjective(), tb
