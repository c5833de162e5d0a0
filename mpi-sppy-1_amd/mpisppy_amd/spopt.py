"""SPOpt: the batched solve loop and expectations (mirrors mpisppy/spopt.py).

``solve_loop`` keeps the reference's signature (spopt.py:226-233) but replaces the
per-scenario ``solve_one`` + SolverFactory plugin call (spopt.py:85-223) with ONE
``phgpu_solve`` over all local scenarios.  Solver selection is by ``solver_name``
(cfg_vanilla.py:43 -> spopt.py:844): this engine answers to ``"mi355x_pdhg"``
(aliases below).  ``iter0_solver_options`` / ``iterk_solver_options`` keys are the
fields of ``phgpu_options`` (include/phgpu.h).

Per-scenario extension hooks ``pre_solve`` / ``post_solve`` (spopt.py:146-147, 220-221)
bracket the batched solve: all local scenarios' ``pre_solve`` before the launch, all
``post_solve`` after it (solutions loaded, one ``ScenarioResults`` each).
"""
import time
import numpy as np

from . import _lib
from .spbase import SPBase
from .engine import PHEngine
from .extensions.extension import overrides

_TERMINATION = {_lib.OPTIMAL: "optimal", _lib.ITER_LIMIT: "maxIterations",
                _lib.PRIMAL_INFEASIBLE: "infeasible", _lib.DUAL_INFEASIBLE: "unbounded"}


class ScenarioResults:
    """What ``post_solve`` gets for one scenario, in the shape of the Pyomo results the
    reference passes (spopt.py:165-206): ``solver.termination_condition`` /
    ``solver.status``, ``Problem[0].Lower_bound`` / ``Upper_bound`` (the Lagrangian bound
    and the objective of the solve, swapped for a maximisation), plus the engine's own
    ``status`` code and ``iterations``."""

    class _Solver:
        def __init__(self, tc):
            self.termination_condition = tc
            self.status = "ok" if tc in ("optimal", "maxIterations") else "warning"

    class _Problem:
        def __init__(self, lo, up):
            self.Lower_bound = lo
            self.Upper_bound = up

    def __init__(self, status, obj, bound, iterations, sense=1):
        self.status = int(status)
        self.iterations = int(iterations)
        self.solver = self._Solver(_TERMINATION.get(self.status, "error"))
        lo, up = (bound, obj) if sense > 0 else (obj, bound)
        self.Problem = [self._Problem(float(lo), float(up))]
        self.solution = _SolutionSet([self] if self.status in (_lib.OPTIMAL, _lib.ITER_LIMIT) else [])


class _SolutionSet(list):
    """``results.solution`` of a Pyomo results object: indexable and callable
    (``results.solution(0)``); empty for an infeasible / unbounded solve."""

    def __call__(self, i=0):
        return self[i]


class ScenarioView:
    """The subproblem handed to ``pre_solve`` / ``post_solve`` when the scenarios were
    built by a ``batch_creator`` (no per-scenario models): its name, its index in the local
    batch and, after the solve, its x."""

    def __init__(self, opt, k, name):
        self._opt, self.index, self.name = opt, k, name
        self._name = name

    @property
    def x(self):
        return self._opt.engine.host("x")[self.index]

SOLVER_NAMES = ("mi355x_pdhg", "phgpu", "mi355x")


# phgpu_options structs by their settings (built once: the PH loop solves with the same
# options every iteration)
_OPTIONS_CACHE = {}

class SPOpt(SPBase):
    def __init__(self, options, all_scenario_names, scenario_creator, scenario_denouement=None,
                 all_nodenames=None, mpicomm=None, extensions=None, extension_kwargs=None,
                 scenario_creator_kwargs=None, variable_probability=None, E1_tolerance=1e-5):
        super().__init__(options, all_scenario_names, scenario_creator, scenario_denouement,
                         all_nodenames, mpicomm, scenario_creator_kwargs, variable_probability,
                         E1_tolerance)
        self.extensions = extensions
        self.extension_kwargs = extension_kwargs
        if extensions is not None:
            self.extobject = extensions(self) if extension_kwargs is None else extensions(self, **extension_kwargs)
        self.spcomm = None
        self.engine = None
        self.solve_times = []
        self.pdhg_iters = []

    # spopt.py:839-868
    def _create_solvers(self):
        sname = self.options.get("solver_name")
        if sname not in SOLVER_NAMES:
            raise RuntimeError(f"solver_name {sname!r} is not served by this engine; use one of {SOLVER_NAMES}")
        if self.engine is None:
            self.engine = PHEngine(self.batch, device=self.options.get("device"), comm=self.mpicomm,
                                   node_names=self.node_names, shared=self.options.get("shared_matrix"))
            if getattr(self, "var_prob", None) is not None:
                self.engine.set_nonant_probs(self.var_prob)
            if self.options.get("ipm_tuning"):
                # a model's interior-point constants (e.g. examples/aircond.py IPM_TUNING)
                self.engine.set_ipm_tuning(self.options["ipm_tuning"])

    # options the reference's cfg_vanilla.shared_options passes to MIP/LP plugins
    # (threads, mipgap; cfg_vanilla.py:41-62) or that only drive plugin output (Tee):
    # meaningless for PDHG, accepted and ignored; any other unknown key raises
    FOREIGN_SOLVER_OPTIONS = ("threads", "mipgap", "Tee", "tee", "timelimit", "time_limit")

    @staticmethod
    def _to_phgpu_options(solver_options):
        so = {k: v for k, v in (solver_options or {}).items() if k not in SPOpt.FOREIGN_SOLVER_OPTIONS}
        key = tuple(sorted(so.items()))
        o = _OPTIONS_CACHE.get(key)
        if o is None:
            o = _OPTIONS_CACHE[key] = _lib.default_options(**so)
        return o

    # spopt.py:226-307
    def solve_loop(self, solver_options=None, use_scenarios_not_subproblems=False, dtiming=False,
                   gripe=False, disable_pyomo_signal_handling=False, tee=False, verbose=False,
                   warm_start=True, speculative=False):
        if self.extensions is not None and hasattr(self.extobject, "pre_solve_loop"):
            self.extobject.pre_solve_loop()
        ext = self.extobject if self.extensions is not None else None
        pre, post = overrides(ext, "pre_solve"), overrides(ext, "post_solve")
        if pre:
            for sp in self._subproblems():
                ext.pre_solve(sp)
        t0 = time.perf_counter()
        self.engine.solve(self._to_phgpu_options(solver_options), warm=warm_start, speculative=speculative)
        if dtiming or self.options.get("record_pdhg_iters", False):
            import torch
            torch.cuda.synchronize()
            it = self.engine.iters.cpu().numpy()
            self.pdhg_iters.append((int(it.max()), float(it.mean())))
        self.solve_times.append(time.perf_counter() - t0)
        if post:
            self._post_solve_hooks(ext)
        if self.extensions is not None and hasattr(self.extobject, "post_solve_loop"):
            self.extobject.post_solve_loop()
        if dtiming and self.cylinder_rank == 0:
            print("Batched solve time (seconds): %4.4f  PDHG iters max/mean %d/%.1f"
                  % (self.solve_times[-1], *self.pdhg_iters[-1]))
        if gripe == "deferred":
            # iterk_loop: the count is read at the next host synchronisation (the conv
            # readback of the next PH iteration, or the end of the loop), not here
            self.engine.count_not_optimal_async()
            self._gripe_pending = True
        elif gripe and self.engine.count_not_optimal() > 0:
            self._gripe_print()

    def _subproblems(self):
        """Per-scenario models when the creator built them, else ScenarioViews."""
        if self.local_scenarios:
            return [self.local_scenarios[nm] for nm in self.local_scenario_names]
        return [ScenarioView(self, k, nm) for k, nm in enumerate(self.local_scenario_names)]

    def _post_solve_hooks(self, ext):
        # (a speculative solve is never bracketed: PHBase._speculate is off with these hooks)
        self.load_solutions_to_models()
        st, obj, bd, it = (self.engine.host(k) for k in ("status", "obj", "bound", "iters"))
        sense = self.batch.sense
        # spopt.py:165-221: the results object with termination 'infeasible' / 'unbounded'
        # (and no solution) for a certified failure; None only where the solver raised,
        # which a batched launch does not do per scenario
        for k, sp in enumerate(self._subproblems()):
            ext.post_solve(sp, ScenarioResults(st[k], sense * obj[k], sense * bd[k], it[k], sense))

    def gripe_report(self):
        """The gripe of a solve_loop(gripe="deferred") (spopt.py:284-294 prints it right
        after the solves; here it comes at the next synchronisation)."""
        if getattr(self, "_gripe_pending", False):
            self._gripe_pending = False
            if self.engine.pending_not_optimal() > 0:
                self._gripe_print()

    def _gripe_print(self):
        st = self.engine.status.cpu().numpy()
        bad = np.nonzero((st != _lib.OPTIMAL) & (st != _lib.ITER_LIMIT))[0]
        for k in bad[:10]:
            print(f"Solve failed for scenario {self.batch.names[k]} (status {st[k]})")
        lim = np.nonzero(st == _lib.ITER_LIMIT)[0]
        if len(lim) and self.cylinder_rank == 0:
            print(f"WARNING: {len(lim)} scenario(s) hit the PDHG iteration limit "
                  f"(e.g. {self.batch.names[lim[0]]}); their solutions are approximate")

    # spopt.py:310-343 ("weighted, proxed" objective, phbase.py:991)
    def Eobjective(self, verbose=False):
        e = self.engine.expectations()
        return self.batch.sense * e[0]

    # spopt.py:346-391
    def Ebound(self, verbose=False, extra_sum_terms=None):
        e = self.engine.expectations()
        b = self.batch.sense * e[1]
        if extra_sum_terms is not None:
            import torch
            t = torch.tensor(list(extra_sum_terms), dtype=torch.float64, device=self.engine.device)
            self.mpicomm.allreduce_sum_(t)
            return b, t.cpu().numpy()
        return b

    # spopt.py:394-408
    def _update_E1(self):
        self.E1 = self.engine.expectations()[2]

    # spopt.py:411-439
    def feas_prob(self):
        return self.engine.expectations()[3]

    def infeas_prob(self):
        e = self.engine.expectations()
        return e[2] - e[3]

    # -- values back into the LinearModels (for denouement / writers)
    def load_solutions_to_models(self):
        if not self.local_scenarios:
            return
        x = self.engine.host("x")  # [S, n]
        for s, nm in enumerate(self.local_scenario_names):
            mdl = self.local_scenarios[nm]
            for j, v in enumerate(mdl.vars):
                v._value = float(x[s, j])
