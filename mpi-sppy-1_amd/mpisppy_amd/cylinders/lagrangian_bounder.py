"""Lagrangian outer bound spoke (mirrors mpisppy/cylinders/lagrangian_bounder.py:5-95).

Same scenarios as the hub, W on, prox off: every delivery of the hub's W is one batched
LP solve over all local scenarios (warm-started from the previous one) and the bound
is E[dual bound] = sum_s pi_s * bound_s (spopt.py:346-391).  The per-scenario bound is
the PDHG Lagrangian dual objective with projected reduced costs, i.e. a valid lower
bound up to the solve tolerance, like the solver's Lower_bound the reference reads
(spopt.py:201-206).
"""
from .spoke import OuterBoundWSpoke


class LagrangianOuterBound(OuterBoundWSpoke):
    converger_spoke_char = "L"

    # lagrangian_bounder.py:9-17
    def lagrangian_prep(self):
        self.opt.PH_Prep(attach_prox=False)
        self.opt._reenable_W()
        self.opt._create_solvers()
        self.opt.engine.set_terms(1, 0)

    # lagrangian_bounder.py:19-56
    def lagrangian(self):
        verbose = self.opt.options["verbose"]
        self.opt.solve_loop(solver_options=self.opt.current_solver_options, dtiming=False, gripe=True,
                            verbose=verbose)
        # only a fully certified solve gives a valid Lagrangian bound: a scenario at the
        # iteration cap reports a dual objective that is not a bound, an infeasible one
        # +-inf.  None keeps the previous bound (do_work), as a failed solve does in the
        # reference (lagrangian_bounder.py:36-47)
        Eobj, Ebound, E1, Efeas, Eopt = self.opt.engine.expectations()
        if abs(Eopt - E1) > 1e-12 * max(1.0, abs(E1)):
            return None
        return self.opt.batch.sense * Ebound

    # lagrangian_bounder.py:58-60 (W_from_flat_list with the hub's W, device to device)
    def _set_weights_and_solve(self):
        self.opt.engine.W[: self.localWs.shape[0]].copy_(self.localWs)
        return self.lagrangian()

    # lagrangian_bounder.py:62-80, split into main (prep + trivial bound) and do_work
    def main(self):
        self.lagrangian_prep()
        self.dk_iter = 1
        self.trivial_bound = self.lagrangian()
        self.opt.current_solver_options = self.opt.iterk_solver_options
        if self.trivial_bound is not None:
            self.bound = self.trivial_bound

    def do_work(self):
        if self.new_Ws:
            bound = self._set_weights_and_solve()
            if bound is not None:
                self.bound = bound
            self.dk_iter += 1

    # lagrangian_bounder.py:82-95: one final pass with the final PH weights (the hub
    # delivers them with the kill signal; without a new W the last bound stands)
    def finalize(self):
        self.got_kill_signal()
        final = self._set_weights_and_solve() if self.new_Ws else None
        if final is not None:
            self.final_bound = final
            self.bound = final
        else:
            self.final_bound = self.bound
        if self.opt.extensions is not None and hasattr(self.opt.extobject, "post_everything"):
            self.opt.extobject.post_everything()
        return self.final_bound
