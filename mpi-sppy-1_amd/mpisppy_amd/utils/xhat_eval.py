"""Xhat_Eval: evaluate a candidate first-stage (or per-node) solution on the batched engine
(mirrors mpisppy/utils/xhat_eval.py:29-434).

The reference fixes the nonants of every local Pyomo model (spopt.py:557-592), solves
each scenario with its solver plugin (xhat_eval.py:141-209) and takes the expected
objective (xhat_eval.py:212-291).  Here the fix is one kernel over all local scenarios
(``phgpu_fix_nonants``), the solve is one batched PDHG launch, and the expectation is
the engine's deterministic tree sum.  The objective has no PH terms (W and prox are
never attached to an Xhat_Eval, xhat_eval.py:29-60).

A candidate is accepted only when every scenario solve is certified OPTIMAL: a fixing
that makes a scenario infeasible is certified PRIMAL_INFEASIBLE by the engine, and a
solve left at ITER_LIMIT counts as not accepted too (stricter than feas_prob, which
counts ITER_LIMIT as a loaded solution).
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

    # xhat_eval.py:261-291
    def evaluate_one(self, nonant_cache, scenario_name, s=None):
        """Objective of one scenario with its nonants fixed at ``nonant_cache`` (None if
        that solve is not certified optimal).  The batched engine solves every local
        scenario in the one launch; the others' results are simply not read."""
        self._lazy_create_solvers()
        self._fix_nonants(nonant_cache)
        self.solve_loop(solver_options=self.options.get("solver_options"), gripe=True)
        k = self.local_scenario_names.index(scenario_name)
        if int(self.engine.status[k].item()) != 0:
            return None
        obj = float(self.engine.obj[k].item())
        if not hasattr(self, "objs_dict"):
            self.objs_dict = {}
        self.objs_dict[scenario_name] = obj
        return obj

    # xhat_eval.py:326-362
    def fix_nonants_upto_stage(self, t, cache):
        """Fix the nonants of the nodes of stages 1..t at ``cache`` ({node: values});
        later stages keep their model bounds (NaN entries of the device fix table)."""
        self._lazy_create_solvers()
        e = self.engine
        depth = np.asarray(self.batch.nonant_depth)
        need = {nd for nd, st in zip(e.node_names, self._node_stages()) if st <= t}
        for nd in need:
            if nd not in cache:
                raise RuntimeError(f"Could not find {nd} in {cache}")
            if cache[nd] is None:
                raise RuntimeError(f"Empty cache for node={nd}")
            want = self._node_len(nd)
            if len(cache[nd]) != want:
                raise RuntimeError(f"Needed {want} nonant Vars for {nd}, got {len(cache[nd])}")
        tab = self._node_table({nd: cache[nd] for nd in need})
        if not hasattr(e, "_fix_index"):
            e.fix_nonants_by_node(tab)          # builds the index once
        xfix = tab.reshape(-1)[e._fix_index].clone()
        late = torch.as_tensor(depth + 1 > t, device=e.device)
        xfix[late] = float("nan")
        e.fix_nonants(xfix)
        self._fixed = True

    def _node_stages(self):
        """Stage (1 + tree depth) of each engine node held by a local scenario; nodes
        no local scenario passes through get a stage past the tree (never fixed here)."""
        node_of = self.engine.node_of.cpu().numpy()          # [depth, S] global node ids
        stages = [10 ** 9] * self.engine.num_nodes
        for d in range(node_of.shape[0]):
            for g in np.unique(node_of[d]):
                stages[int(g)] = d + 1
        return stages

    def _node_len(self, nd):
        d = self._node_stages()[self.engine.node_names.index(nd)] - 1
        return int(np.sum(np.asarray(self.batch.nonant_depth) == d))

    # xhat_eval.py:368-400
    def _fix_nonants_at_value(self):
        """Fix every nonant at its current (last-solve) value."""
        self._lazy_create_solvers()
        self.engine.fix_nonants(self.engine.nonant_x_dev())
        self._fixed = True

    # xhat_eval.py:402-434 (fix at the current values, solve, E[obj] or None)
    def calculate_incumbent(self, fix_nonants=True, verbose=False):
        self._lazy_create_solvers()
        if fix_nonants:
            self._fix_nonants_at_value()
        self.solve_loop(solver_options=self.options.get("iterk_solver_options"), verbose=verbose)
        if self.infeas_prob() > 1e-12:
            return None
        return self.Eobjective(verbose)
