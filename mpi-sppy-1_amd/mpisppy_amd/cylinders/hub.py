"""Hub and PHHub (mirrors mpisppy/cylinders/hub.py:24-600).

Bound bookkeeping, gap computation, termination tests and the screen trace follow
hub.py:24-240 line for line in behaviour.  What changes is the transport (see
spcommunicator.py): ``send_ws`` / ``send_nonants`` publish a device snapshot of the
hub engine's W / nonant values ([nn, S_local], the 'ci' order of phbase.py:355-365)
with a new write id; ``sync`` then lets every spoke take it and do one pass of its
loop, and reads back the bounds whose write id advanced (hub_from_spoke, hub.py:396-436).
"""
import logging
import math

import torch

from .. import global_toc
from .spcommunicator import SPCommunicator
from .spoke import ConvergerSpokeType
from . import transport as tp

logger = logging.getLogger("mpisppy_amd.cylinders.hub")


class Hub(SPCommunicator):
    def __init__(self, spbase_object, fullcomm=None, strata_comm=None, cylinder_comm=None, spokes=None,
                 options=None, layout=None):
        super().__init__(spbase_object, fullcomm, strata_comm, cylinder_comm, options)
        # co-located: spoke OBJECTS driven from sync(); on their own ranks (``layout``, a
        # transport.CylinderLayout): spoke CLASSES, reached through transport ports
        self.spokes = list(spokes or [])
        self.layout = layout
        self.ports = {}
        self._remote = {}
        self.n_spokes = len(self.spokes)
        self.latest_ib_char = None
        self.latest_ob_char = None
        self.last_ib_idx = None
        self.last_ob_idx = None
        self.stalled_iter_cnt = 0
        self.last_gap = float("inf")
        self.print_init = True
        self._spoke_seen = {}
        self._hub_write_id = 0

    # hub.py:297-343
    def initialize_spoke_indices(self):
        self.outerbound_spoke_indices = set()
        self.innerbound_spoke_indices = set()
        self.nonant_spoke_indices = set()
        self.w_spoke_indices = set()
        self.outerbound_spoke_chars = dict()
        self.innerbound_spoke_chars = dict()
        for i, spoke in enumerate(self.spokes):
            cls = spoke if isinstance(spoke, type) else type(spoke)
            for cst in getattr(cls, "converger_spoke_types", ()):
                if cst == ConvergerSpokeType.OUTER_BOUND:
                    self.outerbound_spoke_indices.add(i + 1)
                    self.outerbound_spoke_chars[i + 1] = cls.converger_spoke_char
                elif cst == ConvergerSpokeType.INNER_BOUND:
                    self.innerbound_spoke_indices.add(i + 1)
                    self.innerbound_spoke_chars[i + 1] = cls.converger_spoke_char
                elif cst == ConvergerSpokeType.W_GETTER:
                    self.w_spoke_indices.add(i + 1)
                elif cst == ConvergerSpokeType.NONANT_GETTER:
                    self.nonant_spoke_indices.add(i + 1)
                else:
                    raise RuntimeError(f"Unrecognized converger_spoke_type {cst}")
        self.bounds_only_indices = (self.outerbound_spoke_indices | self.innerbound_spoke_indices) - \
            (self.w_spoke_indices | self.nonant_spoke_indices)
        self.has_outerbound_spokes = len(self.outerbound_spoke_indices) > 0
        self.has_innerbound_spokes = len(self.innerbound_spoke_indices) > 0
        self.has_nonant_spokes = len(self.nonant_spoke_indices) > 0
        self.has_w_spokes = len(self.w_spoke_indices) > 0
        self.has_bounds_only_spokes = len(self.bounds_only_indices) > 0

    # hub.py:228-238
    def initialize_bound_values(self):
        if self.opt.is_minimizing:
            self.BestInnerBound = math.inf
            self.BestOuterBound = -math.inf
            self._inner_bound_update = lambda new, old: (new < old)
            self._outer_bound_update = lambda new, old: (new > old)
        else:
            self.BestInnerBound = -math.inf
            self.BestOuterBound = math.inf
            self._inner_bound_update = lambda new, old: (new > old)
            self._outer_bound_update = lambda new, old: (new < old)

    def clear_latest_chars(self):
        self.latest_ib_char = None
        self.latest_ob_char = None

    # hub.py:77-98
    def compute_gaps(self):
        if self.opt.is_minimizing:
            abs_gap = self.BestInnerBound - self.BestOuterBound
        else:
            abs_gap = self.BestOuterBound - self.BestInnerBound
        if abs_gap != float("nan") and abs_gap != float("inf") and abs_gap != float("-inf") \
                and self.BestOuterBound != 0:
            rel_gap = abs_gap / abs(self.BestOuterBound)
        else:
            rel_gap = float("inf")
        return abs_gap, rel_gap

    def get_update_string(self):
        if self.latest_ib_char is None and self.latest_ob_char is None:
            return "   "
        if self.latest_ib_char is None:
            return self.latest_ob_char + "  "
        if self.latest_ob_char is None:
            return "  " + self.latest_ib_char
        return self.latest_ob_char + " " + self.latest_ib_char

    # hub.py:111-123
    def screen_trace(self):
        current_iteration = self.current_iteration()
        abs_gap, rel_gap = self.compute_gaps()
        update_source = self.get_update_string()
        if self.print_init:
            row = (f'{"Iter.":>5s}  {"   "}  {"Best Bound":>14s}  {"Best Incumbent":>14s}  '
                   f'{"Rel. Gap":>12s}  {"Abs. Gap":>14s}')
            global_toc(row, True)
            self.print_init = False
        row = (f"{current_iteration:5d}  {update_source}  {self.BestOuterBound:14.4f}  "
               f"{self.BestInnerBound:14.4f}  {rel_gap * 100:12.3f}%  {abs_gap:14.4f}")
        global_toc(row, True)
        self.clear_latest_chars()

    # hub.py:125-161
    def determine_termination(self):
        if ("rel_gap" not in self.options and "abs_gap" not in self.options
                and "max_stalled_iters" not in self.options):
            return False
        abs_gap, rel_gap = self.compute_gaps()
        abs_gap_satisfied = False
        rel_gap_satisfied = False
        max_stalled_satisfied = False
        if self.options.get("rel_gap") is not None and rel_gap <= self.options["rel_gap"]:
            rel_gap_satisfied = True
        if self.options.get("abs_gap") is not None and abs_gap <= self.options["abs_gap"]:
            abs_gap_satisfied = True
        if self.options.get("max_stalled_iters") is not None:
            if abs_gap < self.last_gap:
                self.last_gap = abs_gap
                self.stalled_iter_cnt = 0
            else:
                self.stalled_iter_cnt += 1
                if self.stalled_iter_cnt >= self.options["max_stalled_iters"]:
                    max_stalled_satisfied = True
        if abs_gap_satisfied:
            global_toc(f"Terminating based on inter-cylinder absolute gap {abs_gap:12.4f}", self.global_rank == 0)
        if rel_gap_satisfied:
            global_toc(f"Terminating based on inter-cylinder relative gap {rel_gap * 100:12.3f}%",
                       self.global_rank == 0)
        if max_stalled_satisfied:
            global_toc(f"Terminating based on max-stalled-iters {self.stalled_iter_cnt}", self.global_rank == 0)
        return abs_gap_satisfied or rel_gap_satisfied or max_stalled_satisfied

    # hub.py:202-226
    def OuterBoundUpdate(self, new_bound, idx=None, char="*"):
        current_bound = self.BestOuterBound
        if self._outer_bound_update(new_bound, current_bound):
            if idx is None:
                self.latest_ob_char = char
                self.last_ob_idx = 0
            else:
                self.latest_ob_char = self.outerbound_spoke_chars[idx]
                self.last_ob_idx = idx
            return new_bound
        return current_bound

    def InnerBoundUpdate(self, new_bound, idx=None, char="*"):
        current_bound = self.BestInnerBound
        if self._inner_bound_update(new_bound, current_bound):
            if idx is None:
                self.latest_ib_char = char
                self.last_ib_idx = 0
            else:
                self.latest_ib_char = self.innerbound_spoke_chars[idx]
                self.last_ib_idx = idx
            return new_bound
        return current_bound

    # hub.py:396-436: a bound is new when the spoke's write id advanced
    def hub_from_spoke(self, idx):
        if self.layout is not None:
            bound, wid = self._remote.get(idx, (math.nan, 0))
            if wid > self._spoke_seen.get(idx, 0):
                self._spoke_seen[idx] = wid
                return True, bound
            return False, None
        spoke = self.spokes[idx - 1]
        wid = spoke.local_write_id
        if wid > self._spoke_seen.get(idx, 0):
            self._spoke_seen[idx] = wid
            return True, spoke.bound
        return False, None

    def receive_innerbounds(self):
        for idx in sorted(self.innerbound_spoke_indices):
            is_new, bound = self.hub_from_spoke(idx)
            if is_new:
                self.BestInnerBound = self.InnerBoundUpdate(bound, idx)

    def receive_outerbounds(self):
        for idx in sorted(self.outerbound_spoke_indices):
            is_new, bound = self.hub_from_spoke(idx)
            if is_new:
                self.BestOuterBound = self.OuterBoundUpdate(bound, idx)

    def hub_to_spoke(self, tensor, idx):
        self.spokes[idx - 1]._deliver(self._hub_write_id, tensor)

    def run_spokes(self):
        """Co-located scheduling: each spoke takes what was delivered and does one pass."""
        for spoke in self.spokes:
            if not spoke.got_kill_signal():
                spoke.do_work()

    # hub.py:438-452
    def send_terminate(self):
        if self.layout is not None:
            for idx in sorted(self.ports):
                self._answer(idx, tp.KILL)
            return
        for spoke in self.spokes:
            spoke._terminate()

    # spokes on their own ranks: answer a spoke's pending Get with the window it reads
    def _window_values(self, idx):
        return None

    def _answer(self, idx, write_id):
        vals = self._window_values(idx)
        bound, wid = self.ports[idx].answer(None if vals is None else tp.ci_order(vals), self.BestOuterBound,
                                            self.BestInnerBound, write_id)
        if wid > self._remote.get(idx, (math.nan, 0))[1]:
            self._remote[idx] = (bound, wid)

    def serve_spokes(self):
        """One pass over the spokes' Gets (the reference's hub_to_spoke Puts, hub.py:369-395):
        answered only when every hub rank has its peer's request (MIN agreement)."""
        idxs = sorted(self.ports)
        ok = tp.agree_ready(self.layout, [self.ports[i].ready() for i in idxs])
        for i, go in zip(idxs, ok):
            if go:
                self._answer(i, float(self._hub_write_id))

    # hub.py:163-172
    def hub_finalize(self):
        if self.layout is not None:
            # the spokes' bounds after their finalize (the Lagrangian's final pass with
            # the final W): the reference's hub_finalize runs after the spokes' finalize
            # and a Barrier (spin_the_wheel.py:126-139)
            for idx in sorted(self.ports):
                bound, wid = self.ports[idx].final()
                if wid > self._remote.get(idx, (math.nan, 0))[1]:
                    self._remote[idx] = (bound, wid)
        if self.has_outerbound_spokes:
            self.receive_outerbounds()
        if self.has_innerbound_spokes:
            self.receive_innerbounds()
        if self.global_rank == 0:
            self.print_init = True
            global_toc("Statistics at termination", True)
            self.screen_trace()


class PHHub(Hub):
    # hub.py:454-499
    def setup_hub(self):
        self.initialize_spoke_indices()
        self.initialize_bound_values()
        if self.has_outerbound_spokes and not self.has_innerbound_spokes:
            logger.warning("No InnerBound Spokes defined, this converger will not cause the hub to terminate")
        self._w_snapshot = None
        self._nonant_snapshot = None
        if self.layout is not None:
            nn, S = max(self.opt.batch.nn, 1), self.opt.batch.S
            for idx in sorted(self.w_spoke_indices | self.nonant_spoke_indices | self.bounds_only_indices):
                self.ports[idx] = tp.HubPort(self.layout, idx, nn * S)
            return
        # spokes prepare (their own Iter0-equivalent work) before the hub's Iter0
        for spoke in self.spokes:
            spoke.main()

    # hub.py:501-514
    def sync(self):
        self._hub_write_id += 1
        if self.layout is not None:
            self.serve_spokes()
            if self.has_outerbound_spokes:
                self.receive_outerbounds()
            if self.has_innerbound_spokes:
                self.receive_innerbounds()
            return
        if self.has_w_spokes:
            self.send_ws()
        if self.has_nonant_spokes:
            self.send_nonants()
        self.run_spokes()
        if self.has_outerbound_spokes:
            self.receive_outerbounds()
        if self.has_innerbound_spokes:
            self.receive_innerbounds()

    def sync_with_spokes(self):
        self.sync()

    # hub.py:519-547
    def is_converged(self):
        # the trivial bound is a valid outer bound only when every Iter0 solve was certified
        # optimal (an ITER_LIMIT dual bound may overstate it; see PHBase.Iter0)
        if self.opt._PHIter == 1 and getattr(self.opt, "trivial_bound_converged", True):
            self.BestOuterBound = self.OuterBoundUpdate(self.opt.trivial_bound)
        if not self.has_innerbound_spokes:
            if self.opt._PHIter == 1:
                logger.warning("PHHub cannot compute convergence without inner bound spokes.")
            if self.global_rank == 0:
                self.screen_trace()
            return False
        if not self.has_outerbound_spokes and self.opt._PHIter == 1:
            global_toc("Without outer bound spokes, no progress will be made on the Best Bound",
                       self.global_rank == 0)
        if self.global_rank == 0:
            self.screen_trace()
        return self.determine_termination()

    def current_iteration(self):
        return self.opt._PHIter

    def main(self):
        self.opt.ph_main(finalize=False)

    def _window_values(self, idx):
        if idx in self.w_spoke_indices:
            return self.opt.engine.W[: max(self.opt.batch.nn, 1)]
        if idx in self.nonant_spoke_indices:
            return self.opt.engine.nonant_x_dev()
        return None

    def send_terminate(self):
        # the final W (updated at the top of the last PH iteration) goes out with the
        # kill signal so W spokes can do their final pass (lagrangian_bounder.py:82-95)
        if self.layout is not None:
            self._hub_write_id += 1
            return super().send_terminate()
        if self.has_w_spokes:
            self._hub_write_id += 1
            self.send_ws()
        super().send_terminate()

    def finalize(self):
        return self.opt.post_loops(self.opt.extensions)

    # hub.py:562-577 (nonant values in 'ci' order, device snapshot)
    def send_nonants(self):
        x = self.opt.engine.nonant_x_dev()
        if self._nonant_snapshot is None:
            self._nonant_snapshot = torch.empty_like(x)
        self._nonant_snapshot.copy_(x)
        for idx in self.nonant_spoke_indices:
            self.hub_to_spoke(self._nonant_snapshot, idx)

    # hub.py:590-598 (_populate_W_cache, phbase.py:346-366)
    def send_ws(self):
        W = self.opt.engine.W[: max(self.opt.batch.nn, 1)]
        if self._w_snapshot is None:
            self._w_snapshot = torch.empty_like(W)
        self._w_snapshot.copy_(W)
        for idx in self.w_spoke_indices:
            self.hub_to_spoke(self._w_snapshot, idx)
