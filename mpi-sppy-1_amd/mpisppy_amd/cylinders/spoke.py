"""Spokes (mirrors mpisppy/cylinders/spoke.py:20-400).

Transport: the hub hands a spoke a device tensor plus a write id (``_deliver``); the
spoke copies it into its own buffer when it next calls ``got_kill_signal`` (the
``spoke_from_hub`` window Get + write-id test of spoke.py:80-118).  A spoke's bound goes
back the same way (``bound`` setter -> ``local_write_id`` bump, spoke.py:60-78).

Scheduling: the reference spoke ``main`` spins on its own ranks until the kill
signal.  Co-located on the hub's GPU, a spoke instead splits into ``main`` (its
preparation and first bound, run once by the hub's ``setup_hub``) and ``do_work``
(one pass of its loop body, run by the hub after each ``sync`` delivery).
"""
import enum
import math
import os
import time

import torch

from .spcommunicator import SPCommunicator


class ConvergerSpokeType(enum.Enum):
    OUTER_BOUND = 1
    INNER_BOUND = 2
    W_GETTER = 3
    NONANT_GETTER = 4


class Spoke(SPCommunicator):
    def __init__(self, spbase_object, fullcomm=None, strata_comm=None, cylinder_comm=None, options=None):
        super().__init__(spbase_object, fullcomm, strata_comm, cylinder_comm, options)
        self.local_write_id = 0
        self.remote_write_id = 0
        self._inbox = None        # (write_id, device tensor) delivered by the hub
        self._killed = False
        self._new_locals = False
        self._locals = None
        self._remote = False      # True when the spoke runs on its own ranks (run_remote)

    # hub -> spoke (hub.py:370-395 Put; here a reference to the hub's snapshot)
    def _deliver(self, write_id, tensor):
        self._inbox = (write_id, tensor)

    def _terminate(self):
        self._killed = True

    # spoke.py:80-118: take a new buffer only when its write id advanced
    def spoke_from_hub(self):
        if self._inbox is None:
            return False
        wid, t = self._inbox
        if wid > self.remote_write_id:
            if self._locals is None or self._locals.shape != t.shape:
                self._locals = torch.empty_like(t)
            self._locals.copy_(t)
            self.remote_write_id = wid
            return True
        return False

    def got_kill_signal(self):
        if self._remote:          # the Get of run_remote already took the window
            return self._killed
        self._new_locals = self.spoke_from_hub()
        return self._killed

    # spoke.py:186-214 (the spoke's own loop when it has ranks of its own): prepare, then
    # alternate a Get of the hub's window with one pass of the loop body until the kill
    # signal; ``port`` is a transport.SpokePort.  After finalize the final bound goes to
    # the hub (its hub_finalize waits for it, as the reference's Barrier makes the hub wait
    # for the spokes' finalize, spin_the_wheel.py:126-139); if anything raises, the hub is
    # told instead of being left waiting.
    def run_remote(self, port):
        self._remote = True
        try:
            result = self._run_remote(port)
        except BaseException:
            port.post_failure()
            raise
        port.post_final(getattr(self, "_bound", float("nan")), self.local_write_id)
        return result

    def _run_remote(self, port):
        from . import transport as tp
        self.main()
        nn, S = max(self.opt.batch.nn, 1), self.opt.batch.S
        device = self.opt.engine.device if self.opt.engine is not None else None
        while True:
            bound = getattr(self, "_bound", float("nan"))
            vals, outer, inner, wid = port.get(bound, self.local_write_id, self.remote_write_id)
            if device is None and self.opt.engine is not None:
                device = self.opt.engine.device
            t = tp.from_ci_order(vals, nn, S, device)
            if self._locals is None or self._locals.shape != t.shape:
                self._locals = t
            else:
                self._locals.copy_(t)
            self.hub_outer_bound, self.hub_inner_bound = outer, inner
            self._new_locals = True
            if wid == tp.KILL:
                self._killed = True
                break
            self.remote_write_id = int(wid)
            self.do_work()
        return self.finalize()

    def get_serial_number(self):
        return self.remote_write_id

    def main(self):
        """Preparation and first bound (run once by the hub's setup_hub)."""
        raise NotImplementedError

    def do_work(self):
        """One pass of the spoke's loop body (run by the hub after each sync)."""
        raise NotImplementedError


class _BoundSpoke(Spoke):
    """spoke.py:145-214: a spoke that sends one bound to the hub."""

    def __init__(self, spbase_object, fullcomm=None, strata_comm=None, cylinder_comm=None, options=None):
        super().__init__(spbase_object, fullcomm, strata_comm, cylinder_comm, options)
        self._bound = math.nan
        self.trace_filen = None
        tp = spbase_object.options.get("trace_prefix")
        if self.cylinder_rank == 0 and tp is not None:
            filen = tp + self.__class__.__name__ + ".csv"
            if os.path.exists(filen):
                raise RuntimeError(f"Spoke trace file {filen} already exists!")
            with open(filen, "w") as f:
                f.write("time,bound\n")
            self.trace_filen = filen
        self.start_time = getattr(spbase_object, "start_time", time.perf_counter())

    @property
    def bound(self):
        return self._bound

    @bound.setter
    def bound(self, value):
        self._append_trace(value)
        self._bound = value
        self.local_write_id += 1      # spoke_to_hub (spoke.py:60-78)

    def _append_trace(self, value):
        if self.cylinder_rank != 0 or self.trace_filen is None:
            return
        with open(self.trace_filen, "a") as f:
            f.write(f"{time.perf_counter() - self.start_time},{value}\n")


class InnerBoundSpoke(_BoundSpoke):
    converger_spoke_types = (ConvergerSpokeType.INNER_BOUND,)
    converger_spoke_char = "I"


class OuterBoundSpoke(_BoundSpoke):
    converger_spoke_types = (ConvergerSpokeType.OUTER_BOUND,)
    converger_spoke_char = "O"


class _BoundWSpoke(_BoundSpoke):
    """spoke.py:270-292: receives the hub's W ([nn, S_local] device tensor, 'ci' order)."""

    @property
    def localWs(self):
        return self._locals

    @property
    def new_Ws(self):
        return self._new_locals


class OuterBoundWSpoke(_BoundWSpoke):
    converger_spoke_types = (ConvergerSpokeType.OUTER_BOUND, ConvergerSpokeType.W_GETTER)
    converger_spoke_char = "O"


class _BoundNonantSpoke(_BoundSpoke):
    """spoke.py:308-325: receives the hub's nonants ([nn, S_local] device tensor)."""

    @property
    def localnonants(self):
        return self._locals

    @property
    def new_nonants(self):
        return self._new_locals


class InnerBoundNonantSpoke(_BoundNonantSpoke):
    """spoke.py:328-384: keeps the best inner bound and its solution."""
    converger_spoke_types = (ConvergerSpokeType.INNER_BOUND, ConvergerSpokeType.NONANT_GETTER)
    converger_spoke_char = "I"

    def __init__(self, spbase_object, fullcomm=None, strata_comm=None, cylinder_comm=None, options=None):
        super().__init__(spbase_object, fullcomm, strata_comm, cylinder_comm, options)
        self.is_minimizing = self.opt.is_minimizing
        self.best_inner_bound = math.inf if self.is_minimizing else -math.inf
        self.solver_options = None
        self.best_solution_cache = None   # device copy of x of the best xhat evaluation
        self.best_xhat = None             # {node name: values} of the best xhat

    def update_if_improving(self, candidate_inner_bound):
        if candidate_inner_bound is None:
            return False
        update = (candidate_inner_bound < self.best_inner_bound) if self.is_minimizing \
            else (self.best_inner_bound < candidate_inner_bound)
        if not update:
            return False
        self.best_inner_bound = candidate_inner_bound
        self.bound = candidate_inner_bound
        self._cache_best_solution()
        return True

    def _cache_best_solution(self):
        e = self.opt.engine
        if self.best_solution_cache is None:
            self.best_solution_cache = torch.empty_like(e.x)
        self.best_solution_cache.copy_(e.x)

    def finalize(self):
        if self.best_solution_cache is None:
            return None
        self.opt.engine.x.copy_(self.best_solution_cache)
        self.opt.first_stage_solution_available = True
        self.opt.tree_solution_available = True
        self.final_bound = self.bound
        return self.final_bound


class OuterBoundNonantSpoke(_BoundNonantSpoke):
    converger_spoke_types = (ConvergerSpokeType.OUTER_BOUND, ConvergerSpokeType.NONANT_GETTER)
    converger_spoke_char = "A"
