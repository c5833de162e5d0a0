"""Xhat_Eval: evaluate a candidate first-stage (or per-node) solution on the batched engine
(mirrors mpisppy/utils/xhat_eval.py:29-434).

The reference fixes the nonants of every local Pyomo model (spopt.py:557-592), solves
each scenario with its solver plugin (xhat_eval.py:141-209) and takes the expected
objective (xhat_eval.py:212-291).  Here the fix is one kernel over all local scenarios
(``phgpu_fix_nonants``), the solve is one batched PDHG launch, and the expectation is
the engine's deterministic tree sum.  The objective has no PH terms (W and prox are
never attached to an Xhat_Eval, xhat_eval.py:29-60).

A candidate is accepted only when every scenario solve is certified OPTIMAL: the
engine has no infeasibility certificate yet, so ITER_LIMIT counts as infeasible here
(stricter than feas_prob, which the hub uses for Iter0).
"""
import numpy as np
import torch

from ..spopt import SPOpt


class Xhat_Eval(SPOpt):
    def __init__(self, options, all_scenario_names, scenario_creator, scenario_denouement=None,
                 all_nodenames=None, mpicomm=None, scenario_creator_kwargs=None,
                 variable_probability=None):
        super().__init__(options, all_scenario_names, scenario_creator,
                         scenario_denouement=scenario_denouement, all_nodenames=all_nodenames,
                         mpicomm=mpicomm, scenario_creator_kwargs=scenario_creator_kwargs,
                         variable_probability=variable_probability)
        self.verbose = options.get("verbose", False)
        self._fixed = False

    # xhat_eval.py:113-139
    def _lazy_create_solvers(self):
        if self.engine is None:
            self._create_solvers()
            self.engine.set_terms(0, 0)

    def _node_table(self, cache):
        """dict node name -> values (spopt.py:557-592 cache) -> device [num_nodes, nlen_max]."""
        e = self.engine
        tab = np.zeros((e.num_nodes, e.nlen_max))
        for g, nd in enumerate(e.node_names):
            if nd in cache and cache[nd] is not None:
                v = np.asarray(cache[nd], dtype=np.float64).reshape(-1)
                tab[g, :len(v)] = v
        return torch.from_numpy(tab).to(e.device)

    # spopt.py:557-592
    def _fix_nonants(self, cache):
        """Fix the nonants of all local scenarios: ``cache`` is {node name: values} or a
        device [num_nodes, nlen_max] tensor (global node order)."""
        self._lazy_create_solvers()
        tab = cache if torch.is_tensor(cache) else self._node_table(cache)
        self.engine.fix_nonants_by_node(tab)
        self._fixed = True

    # spopt.py:638-660
    def _restore_nonants(self):
        if self.engine is not None and self._fixed:
            self.engine.fix_nonants(None)
        self._fixed = False

    # xhat_eval.py:141-209
    def solve_loop(self, solver_options=None, use_scenarios_not_subproblems=False, dtiming=False,
                   gripe=False, disable_pyomo_signal_handling=False, tee=False, verbose=False,
                   compute_val_at_nonant=False, warm_start=True):
        self._lazy_create_solvers()
        super().solve_loop(solver_options, use_scenarios_not_subproblems, dtiming, gripe=False,
                           disable_pyomo_signal_handling=disable_pyomo_signal_handling, tee=tee,
                           verbose=verbose, warm_start=warm_start)

    # xhatbase.py:210-216 acceptance: every scenario certified
    def infeas_prob(self):
        e = self.engine.expectations()
        return e[2] - e[4]

    # xhat_eval.py:212-291 (fct=None case)
    def Eobjective(self, verbose=False, fct=None):
        if fct is not None:
            raise NotImplementedError("Eobjective(fct=...) is outside the batched hot path")
        self._lazy_create_solvers()
        return super().Eobjective(verbose)

    # xhat_eval.py:293-322
    def evaluate(self, nonant_cache, fct=None):
        """Fix at ``nonant_cache`` ({node: values}), solve all scenarios, return E[obj]
        (None if some scenario is not certified optimal)."""
        self._lazy_create_solvers()
        self._fix_nonants(nonant_cache)
        self.solve_loop(solver_options=self.options.get("solver_options"), gripe=True)
        if self.infeas_prob() > 1e-12:
            return None
        return self.Eobjective(self.verbose, fct=fct)

    # xhat_eval.py:402-434 (fix at the current values, solve, E[obj] or None)
    def calculate_incumbent(self, fix_nonants=True, verbose=False):
        self._lazy_create_solvers()
        if fix_nonants:
            self.engine.fix_nonants(self.engine.nonant_x_dev())
            self._fixed = True
        self.solve_loop(solver_options=self.options.get("iterk_solver_options"), verbose=verbose)
        if self.infeas_prob() > 1e-12:
            return None
        return self.Eobjective(verbose)
