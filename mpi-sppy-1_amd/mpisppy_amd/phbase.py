"""PHBase: the progressive-hedging algorithm on the batched engine (mirrors mpisppy/phbase.py).

Same constructor (phbase.py:235-249), required options (phbase.py:732-752), method
names and loop order (Iter0 758-872; iterk_loop 875-979: x̄ -> W -> conv -> break? ->
solve -> sync).  The per-scenario Python loops become device kernels:

  Compute_Xbar      -> phgpu_ph_reduce + one all-reduce of the node buffer
  Update_W + conv   -> phgpu_ph_update (one fused kernel) + one scalar all-reduce
  solve_loop        -> phgpu_solve over all local scenarios
"""
import time
import numpy as np

from . import _lib, global_toc
from .spopt import SPOpt
from .extensions.extension import overrides


LP_EPS_REL = 1e-10
PH_EPS_REL = 1e-9      # the library default (phgpu_default_options), used by the PH QPs


class PHBase(SPOpt):
    def __init__(self, options, all_scenario_names, scenario_creator, scenario_denouement=None,
                 all_nodenames=None, mpicomm=None, scenario_creator_kwargs=None, extensions=None,
                 extension_kwargs=None, ph_converger=None, rho_setter=None,
                 variable_probability=None):
        self.start_time = time.perf_counter()
        super().__init__(options, all_scenario_names, scenario_creator,
                         scenario_denouement=scenario_denouement, all_nodenames=all_nodenames,
                         mpicomm=mpicomm, extensions=extensions, extension_kwargs=extension_kwargs,
                         scenario_creator_kwargs=scenario_creator_kwargs,
                         variable_probability=variable_probability)
        global_toc("Initializing PHBase", self.cylinder_rank == 0 and options.get("toc", True))
        self.options = options
        self.options_check()
        self.ph_converger = ph_converger
        self.rho_setter = rho_setter
        # Iter0 solves pure LPs (W_on = prox_on = 0, phbase.py:594-597).  A first-order LP
        # solution's x is only as accurate as the LP's sharpness allows (the KKT residuals
        # bound the objective, not x), and that x seeds x̄ and W; so the LP default is one
        # decade tighter than the prox QPs' (farmer cm = 64 needs it
        # for W within 1e-5).  An explicit eps_rel in iter0_solver_options wins.
        self.iter0_solver_options = dict(options.get("iter0_solver_options") or {})
        self._iter0_eps_default = "eps_rel" not in self.iter0_solver_options
        self.iter0_solver_options.setdefault("eps_rel", LP_EPS_REL)
        self.iterk_solver_options = options.get("iterk_solver_options") or {}
        self.current_solver_options = self.iter0_solver_options
        self.convobject = None
        self.conv = None
        self._PHIter = 0
        self.iter_times = []

    # phbase.py:732-752
    def options_check(self):
        required = ["solver_name", "PHIterLimit", "defaultPHrho", "convthresh", "verbose",
                    "display_progress"]
        self._options_check(required, self.options)
        self.options.setdefault("display_timing", False)
        self.options.setdefault("display_convergence_detail", False)

    # phbase.py:585-602 + 1040-1050 (W = 0, rho = defaultPHrho, x̄ = 0, terms off)
    def attach_Ws_and_prox(self):
        self._create_solvers()
        e = self.engine
        e.W.zero_()
        e.xbar.zero_()
        e.set_rho(float(self.options["defaultPHrho"]))
        e.set_terms(0, 0)

    def PH_Prep(self, attach_duals=True, attach_prox=True):
        """phbase.py:702-716."""
        self._attach_duals = attach_duals
        self._attach_prox = attach_prox
        self.attach_Ws_and_prox()

    # W_on / prox_on toggles (phbase.py:408-437)
    @property
    def W_disabled(self):
        return not bool(self.engine.W_on)

    @property
    def prox_disabled(self):
        return not bool(self.engine.prox_on)

    def _disable_W(self):
        self.engine.set_terms(0, self.engine.prox_on)

    def _disable_prox(self):
        self.engine.set_terms(self.engine.W_on, 0)

    def _reenable_W(self):
        self.engine.set_terms(1 if getattr(self, "_attach_duals", True) else 0, self.engine.prox_on)

    def _reenable_prox(self):
        self.engine.set_terms(self.engine.W_on, 1 if getattr(self, "_attach_prox", True) else 0)

    def disable_W_and_prox(self):
        self.engine.set_terms(0, 0)

    def reenable_W_and_prox(self):
        self._reenable_W()
        self._reenable_prox()

    # phbase.py:494-568 (dis_W / dis_prox wrappers around SPOpt.solve_loop)
    def solve_loop(self, solver_options=None, use_scenarios_not_subproblems=False, dtiming=False,
                   dis_W=False, dis_prox=False, gripe=False, disable_pyomo_signal_handling=False,
                   tee=False, verbose=False, warm_start=True, speculative=False):
        wo, po = self.engine.W_on, self.engine.prox_on
        if dis_W or dis_prox:
            self.engine.set_terms(0 if dis_W else wo, 0 if dis_prox else po)
        super().solve_loop(solver_options, use_scenarios_not_subproblems, dtiming, gripe,
                           disable_pyomo_signal_handling, tee, verbose, warm_start=warm_start,
                           speculative=speculative)
        if dis_W or dis_prox:
            self.engine.set_terms(wo, po)

    # phbase.py:27-107 / 265-291
    def Compute_Xbar(self, verbose=False):
        # with one rank the engine folds x̄ into the Update_W launch (engine.compute_xbar)
        self.engine.compute_xbar(lazy=True)

    # phbase.py:293-318 (fused with the x̄ scatter and the conv partial sum; in the
    # speculative loop deferred into the next solve launch, engine.update(defer=True))
    def Update_W(self, verbose=False):
        self.engine.update(update_W=True, defer=getattr(self, "_defer_update", False))

    # phbase.py:321-343
    def convergence_diff(self):
        return self.engine.convergence_diff()

    # phbase.py:346-385 -- "ci" order = local scenarios x nonant order
    def _populate_W_cache(self, cache, padding):
        W = self.engine.host("W")[:, :self.batch.nn]
        flat = W.reshape(-1)
        if len(flat) + padding != len(cache):
            raise RuntimeError("W cache length mismatch")
        cache[:len(flat)] = flat

    def W_from_flat_list(self, flat_list):
        S, nn = self.batch.S, self.batch.nn
        self.engine.set_W(np.asarray(flat_list[:S * nn], dtype=np.float64).reshape(S, nn))

    # phbase.py:387-406
    def _use_rho_setter(self, verbose):
        if self.rho_setter is None:
            return
        if not self.local_scenarios:
            raise RuntimeError("rho_setter needs per-scenario models; pass options['rho_array'] with a batch_creator")
        kw = self.options.get("rho_setter_kwargs", {})
        rho = self.engine.host("rho")[:, :self.batch.nn].copy()
        for s, nm in enumerate(self.local_scenario_names):
            mdl = self.local_scenarios[nm]
            id2k = {}
            k = 0
            for nd in mdl._mpisppy_node_list:
                for v in nd.nonant_vardata_list:
                    id2k[id(v)] = k
                    k += 1
            for (vid, r) in self.rho_setter(mdl, **kw):
                rho[s, id2k[vid]] = r
        self.engine.set_rho(rho)

    # phbase.py:758-872
    def Iter0(self):
        if self.extensions is not None and hasattr(self.extobject, "pre_iter0"):
            self.extobject.pre_iter0()
        verbose = self.options["verbose"]
        dprogress = self.options["display_progress"]
        dtiming = self.options["display_timing"]
        self._PHIter = 0
        global_toc("Creating solvers", self.cylinder_rank == 0 and self.options.get("toc", True))
        self._create_solvers()
        global_toc("Entering solve loop in PHBase.Iter0", self.cylinder_rank == 0 and self.options.get("toc", True))
        self.solve_loop(solver_options=self.current_solver_options, dtiming=dtiming,
                        gripe=not self._iter0_eps_default, verbose=verbose, warm_start=False)
        # local scenarios whose Iter0 LP needed the relaxed re-solve below (reported by
        # bench.py next to iter0_not_optimal, and by a warning on the ranks that have any)
        self.iter0_relaxed = self.engine.count_not_optimal() if self._iter0_eps_default else 0
        if self.iter0_relaxed > 0:
            print(f"WARNING (rank {self.cylinder_rank}): {self.iter0_relaxed} Iter0 LP(s) missed eps_rel "
                  f"{LP_EPS_REL:g}; every scenario is re-solved at {PH_EPS_REL:g} from its warm start",
                  flush=True)
            # the tighter LP default is out of reach for a scenario whose dual is nearly
            # degenerate (aircond 32x32x64 scen982: x exact to 5e-12 but the gap stalls at
            # 7e-8 relative for 1e6 iterations): finish every
            # scenario at the PH subproblems' 1e-9 from this warm start (the converged ones
            # stop at their first KKT check)
            relaxed = dict(self.current_solver_options)
            relaxed["eps_rel"] = PH_EPS_REL
            self.solve_loop(solver_options=relaxed, dtiming=dtiming, gripe=True, verbose=verbose,
                            warm_start=True)
        self.iter0_continued = self._iter0_continue(dtiming, verbose)
        self._update_E1()
        if abs(1 - self.E1) > self.E1_tolerance:
            # the reference prints ERROR and calls quit() (phbase.py:812-817)
            raise RuntimeError(f"Total probability of scenarios was {self.E1} "
                               f"(E1_tolerance = {self.E1_tolerance})")
        _, _, _, feasP, optP = self.engine.expectations()
        if abs(feasP - self.E1) > 1e-12 * max(1.0, abs(self.E1)):
            # a PDHG infeasibility / unboundedness certificate (status 2 / 3); the reference
            # prints the same message and quit()s (phbase.py:818-823)
            raise RuntimeError(f"Infeasibility detected; E_feas, E1= {feasP} {self.E1}")
        # scenarios at the PDHG iteration cap carry an approximate x and an uncertified
        # bound: say so on every rank, and keep the trivial bound out of the hub's
        # BestOuterBound (trivial_bound_converged)
        self.trivial_bound_converged = abs(optP - self.E1) <= 1e-12 * max(1.0, abs(self.E1))
        if not self.trivial_bound_converged:
            print(f"WARNING (rank {self.cylinder_rank}): Iter0 solves at the PDHG iteration limit "
                  f"carry probability {self.E1 - optP:.3g}; their x enters x̄ unconverged and the "
                  f"trivial bound is not certified", flush=True)
        if self.extensions is not None and hasattr(self.extobject, "post_iter0"):
            self.extobject.post_iter0()
        if self.spcomm is not None:
            self.spcomm.sync()
        if self.extensions is not None and hasattr(self.extobject, "post_iter0_after_sync"):
            self.extobject.post_iter0_after_sync()
        if self.rho_setter is not None:
            self._use_rho_setter(verbose and self.cylinder_rank == 0)
        if "rho_array" in self.options:
            self.engine.set_rho(self.options["rho_array"])
        if self.ph_converger is not None:
            self.convobject = self.ph_converger(self)
        self.conv = None
        self.trivial_bound = self.Ebound(verbose)
        if dprogress and self.cylinder_rank == 0:
            print("")
            print("After PH Iteration", self._PHIter)
            print("Trivial bound =", self.trivial_bound)
            print("PHBase Convergence Metric =", self.conv)
            print("Elapsed time: %6.2f" % (time.perf_counter() - self.start_time))
        self.reenable_W_and_prox()
        self.current_solver_options = self.iterk_solver_options
        return self.trivial_bound

    ITER0_CONTINUATIONS = 3

    def _iter0_continue(self, dtiming, verbose):
        """Iter0 LPs left at the PDHG iteration cap on the streaming path (path 4: large
        scenarios sharing one matrix, config 5) are continued, not accepted: a warm re-solve
        of every local scenario (the converged ones stop at their first KKT check) in which
        the longest ones -- those at the cap -- run first, each over the whole GPU (the split
        form, phgpu_options.split_longest), up to ITER0_CONTINUATIONS times.  The reference
        takes Iter0's x and Lower_bound from a solver that finished (spopt.py:175-206); a
        larger iteration cap on the queue would leave the stragglers in one slot each.
        Returns the continuation solves run."""
        n = 0
        if not self.engine.shared or self.options.get("iter0_continue", True) is False:
            return 0
        while n < self.ITER0_CONTINUATIONS:
            st = self.engine.host("status")
            lim = int((st == _lib.ITER_LIMIT).sum())
            if self.n_proc > 1:
                # every rank runs the same number of continuation solve_loops (an extension's
                # pre / post_solve_loop may hold a collective)
                import torch
                t = torch.tensor([float(lim)], dtype=torch.float64, device=self.engine.device)
                self.mpicomm.allreduce_max_(t)
                lim = int(t.item())
            if lim == 0:
                break
            opts = dict(self.current_solver_options)
            opts["split_longest"] = min(16, lim)
            self.solve_loop(solver_options=opts, dtiming=dtiming, gripe=False, verbose=verbose, warm_start=True)
            n += 1
        return n

    # phbase.py:875-979
    def _speculate(self, have_ext):
        if not self.options.get("speculative_solve", True):
            return False
        if self.options.get("display_timing") or self.options.get("record_pdhg_iters"):
            return False
        if self.ph_converger is not None:
            return False
        if self.engine.shared:
            # path 4 keeps one warm-start slot (phgpu_solve_deferred is rejected), and its
            # solves take seconds, against the ~0.05 ms a speculative launch hides
            return False
        if have_ext and any(overrides(self.extobject, h) for h in ("miditer", "pre_solve_loop", "post_solve_loop",
                                                                    "pre_solve", "post_solve")):
            return False
        return True

    def _fused_loop(self, have_ext):
        """The whole loop in one launch (engine.ph_loop) when nothing but the
        convergence test decides between the iterations: one rank, no extension, converger or
        spoke, no progress / timing display -- the state the speculative solve needs plus
        those.  Opt-in (options["fused_ph_loop"] = True): on config 3 its PH iteration takes
        what the step-by-step loop's does (0.1169 against 0.1163 ms, the launch overhead
        being hidden already by the speculative solve), and its fixed cost per call is ~0.1 ms
        (DESIGN.md 3.11)."""
        if not self.options.get("fused_ph_loop", False) or self.n_proc > 1 or self.spcomm is not None:
            return False
        if have_ext or self.options.get("display_progress") or self.options.get("display_convergence_detail"):
            return False
        return self._speculate(have_ext)

    def iterk_loop(self):
        verbose = self.options["verbose"]
        have_ext = self.extensions is not None
        dprogress = self.options["display_progress"]
        dtiming = self.options["display_timing"]
        self.conv = None
        max_iterations = int(self.options["PHIterLimit"])
        self.converged = False
        first = 1
        if max_iterations >= 1 and self._fused_loop(have_ext):
            t0 = time.perf_counter()
            r = self.engine.ph_loop(self._to_phgpu_options(self.current_solver_options), max_iterations,
                                    float(self.options["convthresh"]))
            if r is not None:
                steps = r["steps"]
                self.fused_loops = getattr(self, "fused_loops", []) + [r]
                dt = (time.perf_counter() - t0) / max(1, steps)
                self.iter_times.extend([dt] * steps)
                self._PHIter = steps
                self.conv = r["conv"][-1] if steps else None
                if r["end"] == 1:
                    self.converged = True
                    global_toc("Convergence metric=%f dropped below user-supplied threshold=%f"
                               % (self.conv, self.options["convthresh"]), self.cylinder_rank == 0)
                    self.gripe_report()
                    return
                if r["end"] == 0:
                    if self.engine.count_not_optimal() > 0:
                        self._gripe_print()
                    self.mpicomm.Barrier()
                    global_toc("Reached user-specified limit=%d on number of PH iterations" % max_iterations,
                               self.cylinder_rank == 0)
                    return
                # a solve handed scenarios to the PDHG fallback (solved after the launch): the
                # remaining iterations run one by one
                if self.engine.count_not_optimal() > 0:
                    self._gripe_print()
                first = steps + 1
        for self._PHIter in range(first, max_iterations + 1):
            t0 = time.perf_counter()
            if dprogress:
                global_toc(f"\nInitiating PH Iteration {self._PHIter}\n", self.cylinder_rank == 0)
            # Speculative solve: the next solve_loop only depends on W and x̄, which are
            # final here, so it is launched before the convergence readback and committed
            # after the test (discarded when the loop stops) -- the GPU does not idle
            # while the host reads conv and returns to launch the solve.  Off when an
            # extension could change the problem between the test and the solve.  With it,
            # one rank's x̄ / W / conv step runs in the solve launch itself.
            spec = self._speculate(have_ext)
            self.Compute_Xbar(verbose)
            self._defer_update = spec
            try:
                self.Update_W(verbose)
            finally:
                self._defer_update = False
            if spec:
                # (several ranks: the update is marked, the solve launched, then the conv
                # all-reduce issued on the side stream behind the mark)
                self.engine.convergence_mark()
                self.solve_loop(solver_options=self.current_solver_options, dtiming=dtiming,
                                gripe=False, verbose=verbose, speculative=True)
                self.engine.convergence_diff_async()
                if self.options.get("xbar_ahead", True):
                    self.engine.xbar_ahead()
                self.conv = self.engine.convergence_wait()
            else:
                self.conv = self.convergence_diff()
            self.gripe_report()                        # the previous iteration's solves
            if have_ext and hasattr(self.extobject, "miditer"):
                self.extobject.miditer()
            if self.ph_converger is not None:
                if self.convobject.is_converged():
                    self.converged = True
                    global_toc("User-supplied converger determined termination criterion reached",
                               self.cylinder_rank == 0)
                    break
            elif self.conv is not None and self.conv < self.options["convthresh"]:
                self.converged = True
                global_toc("Convergence metric=%f dropped below user-supplied threshold=%f"
                           % (self.conv, self.options["convthresh"]), self.cylinder_rank == 0)
                break
            if spec:
                self.engine.commit()
                self.engine.count_not_optimal_async()  # its gripe, read at the next sync
                self._gripe_pending = True
            else:
                self.solve_loop(solver_options=self.current_solver_options, dtiming=dtiming,
                                gripe="deferred", verbose=verbose)
            if have_ext and hasattr(self.extobject, "enditer"):
                self.extobject.enditer()
            if self.spcomm is not None:
                self.spcomm.sync()
                if self.spcomm.is_converged():
                    global_toc("Cylinder convergence", self.cylinder_rank == 0)
                    break
            if have_ext and hasattr(self.extobject, "enditer_after_sync"):
                self.extobject.enditer_after_sync()
            self.iter_times.append(time.perf_counter() - t0)
            if dprogress and self.cylinder_rank == 0:
                print("")
                print("After PH Iteration", self._PHIter)
                print("Scaled PHBase Convergence Metric=", self.conv)
                print("Iteration time: %6.2f" % (time.perf_counter() - t0))
                print("Elapsed time:   %6.2f" % (time.perf_counter() - self.start_time))
        else:
            self.gripe_report()
            self.mpicomm.Barrier()
            global_toc("Reached user-specified limit=%d on number of PH iterations" % max_iterations,
                       self.cylinder_rank == 0)
        self.gripe_report()

    # phbase.py:982-1037
    def post_loops(self, extensions=None):
        dprogress = self.options["display_progress"]
        self.mpicomm.Barrier()
        if self.scenario_denouement is not None and self.local_scenarios:
            self.load_solutions_to_models()
            for sname, s in self.local_scenarios.items():
                self.scenario_denouement(self.cylinder_rank, sname, s)
        self.mpicomm.Barrier()
        if extensions is not None and hasattr(self.extobject, "post_everything"):
            self.extobject.post_everything()
        Eobj = self.Eobjective()
        self.mpicomm.Barrier()
        if dprogress and self.cylinder_rank == 0:
            print("")
            print("Current ***weighted*** E[objective] =", Eobj)
            print("")
        return Eobj

    # -- host views used by tests / writers
    def xbar_by_node(self):
        return self.engine.node_xbar()

    def W_array(self):
        return self.engine.host("W")[:, :self.batch.nn]

    def nonants_array(self):
        return self.engine.nonant_x()
