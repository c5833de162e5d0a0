"""Xhat shuffle inner bound spoke (mirrors mpisppy/cylinders/xhatshufflelooper_bounder.py:20-300).

The candidate order is the reference's exactly: ``random.Random()`` seeded 42 samples
the enumerated scenario names without replacement (:99-106) and ``ScenarioCycler``
(:158-300, restated below) walks it, filling every non-leaf node of a multistage tree
from the scenarios below it and alternating normal / reversed epochs.  Each candidate
is one batched fixed-nonant solve over all local scenarios (extensions/xhatbase.py).
Co-located with the hub, the spoke tries ``xhat_looper_options["tries_per_sync"]``
candidates (default 1) per hub sync instead of spinning on ranks of its own.
"""
import random

from .spoke import InnerBoundNonantSpoke
from ..extensions.xhatbase import XhatBase
from ..sputils import scenario_tree
from ..utils.xhat_eval import Xhat_Eval


class XhatShuffleInnerBound(InnerBoundNonantSpoke):
    converger_spoke_char = "X"

    # :24-60
    def xhatbase_prep(self):
        if self.opt.options.get("bundles_per_rank", 0):
            raise RuntimeError("xhat spokes cannot have bundles (yet)")
        if not isinstance(self.opt, Xhat_Eval):
            raise RuntimeError("XhatShuffleInnerBound must be used with Xhat_Eval.")
        self.verbose = self.opt.options["verbose"]
        lo = self.opt.options.get("xhat_looper_options", {})
        self.solver_options = lo.get("xhat_solver_options")
        self.tries_per_sync = int(lo.get("tries_per_sync", 1))
        self.xhatter = XhatBase(self.opt)
        self.xhatter.pre_iter0()
        self.opt._lazy_create_solvers()
        self.opt._update_E1()
        if abs(1 - self.opt.E1) > self.opt.E1_tolerance:
            raise ValueError(f"Total probability of scenarios was {self.opt.E1} "
                             f"(E1_tolerance is {self.opt.E1_tolerance})")
        self.xhatter.post_iter0()
        self.random_seed = 42
        self.random_stream = random.Random()

    # :63-88
    def try_scenario_dict(self, xhat_scenario_dict):
        obj = self.xhatter._try_one(xhat_scenario_dict, solver_options=self.solver_options, verbose=False,
                                    restore_nonants=False, nonant_cache=self.localnonants)
        if obj is None:
            if self.verbose and self.opt.cylinder_rank == 0:
                print(f"(rank0)     Infeasible {xhat_scenario_dict}")
            return False
        if self.verbose and self.opt.cylinder_rank == 0:
            print(f"(rank0)     Feasible {xhat_scenario_dict}, obj: {obj}")
        update = self.update_if_improving(obj)
        if update:
            self.best_xhat = {nd: v for nd, v in zip(self.opt.engine.node_names,
                                                     self.xhatter.last_table.cpu().numpy())}
        return update

    # :90-117 (set-up part of main)
    def main(self):
        self.xhatbase_prep()
        lo = self.opt.options.get("xhat_looper_options", {})
        self.reverse = lo.get("reverse", True)
        self.iter_step = lo.get("iter_step", None)
        self.random_stream.seed(self.random_seed)
        scen_names = list(enumerate(self.opt.all_scenario_names))
        shuffled_scenarios = self.random_stream.sample(scen_names, len(scen_names))
        nonleaves = {nd: t for nd, t in scenario_tree(
            self.opt.all_nodenames, len(self.opt.all_scenario_names)).items() if not t.is_leaf or nd == "ROOT"}
        self.scenario_cycler = ScenarioCycler(shuffled_scenarios, nonleaves, self.reverse, self.iter_step)
        self.tried = []

    # :119-156 (loop body); the cache update of :134-141 is the delivery itself
    def do_work(self):
        if self.get_serial_number() == 0:
            return
        tries = 0
        idle = 0
        while tries < self.tries_per_sync and idle < 2:
            next_scendict = self.scenario_cycler.get_next()
            if next_scendict is not None:
                idle = 0
                tries += 1
                self.tried.append(dict(next_scendict))
                update = self.try_scenario_dict(next_scendict)
                if update:
                    self.scenario_cycler.best = next_scendict
            else:
                # an epoch boundary costs the reference's spinning loop one cheap pass;
                # it does not use up one of this sync's candidate evaluations
                idle += 1
                self.scenario_cycler.begin_epoch()


class ScenarioCycler:
    """Candidate walk of xhatshufflelooper_bounder.py:158-300, restated.

    An epoch walks the shuffled list (or, on every other epoch of a multistage tree,
    the reversed list) from its start; after each candidate the cursor jumps by
    ``iter_step`` (default 1, or the root's branching factor for a multistage tree) and
    then forward past scenarios already used as ROOT this epoch.  Each non-leaf node is
    assigned the first scenario at or after the cursor that lies below it; nodes whose
    scenario was skipped over get a new one.  The epoch ends when the ROOT candidate
    repeats (``get_next`` returns None once, then ``begin_epoch``).

    Behavioural detail kept from the reference: for a multistage tree the dict
    returned by ``get_next`` is the cycler's live assignment, which the advance that
    follows has already updated (two-stage returns a fresh dict each time).
    """

    def __init__(self, shuffled_scenarios, nonleaves, reverse, iter_step):
        kids = nonleaves["ROOT"].kids if "ROOT" in nonleaves else None
        self._multi = bool(kids) and not kids[0].is_leaf
        if self._multi:
            self._nodes = nonleaves
            self.BF0 = len(kids)
            self._step = self.BF0 if iter_step is None else iter_step
            self._alternate = True if reverse is None else reverse
        else:
            self._nodes = None
            self._step = 1 if iter_step is None else iter_step
            self._alternate = False
        self._reversed = False
        self._shuffled = list(shuffled_scenarios)
        self._n = len(self._shuffled)
        self.best = None
        self._start_epoch(reversed_order=False)

    # -- epochs
    def _start_epoch(self, reversed_order):
        self._reversed = reversed_order
        seq = list(reversed(self._shuffled)) if reversed_order else self._shuffled
        self._names = [nm for _, nm in seq]
        self._index = [ix for ix, _ in seq]
        self._pos = 0
        self._used = set()
        if self._multi:
            self.nodescen_dict = {}
            self._assign(list(self._nodes.keys()))
        else:
            self.nodescen_dict = {"ROOT": self._names[0]}

    def begin_epoch(self):
        self._start_epoch(reversed_order=self._multi and self._alternate and not self._reversed)

    # -- node assignment (multistage)
    def _assign(self, nodes):
        """Give every node in ``nodes`` the first scenario at/after the cursor below it."""
        p = self._pos
        pending = list(nodes)
        while pending:
            if p == self._pos and self.nodescen_dict.get("ROOT") is not None:
                raise RuntimeError("_fill_nodescen_dict looped over every scenario but was not able "
                                   "to find a scen for every nonleaf node.")
            nm, ix = self._names[p], self._index[p]
            still = []
            for nd in pending:
                t = self._nodes[nd]
                if t.scenfirst <= ix <= t.scenlast:
                    self.nodescen_dict[nd] = nm
                else:
                    still.append(nd)
            pending = still
            p = (p + 1) % self._n

    # -- walk
    def get_next(self):
        root = self._names[self._pos]
        if root in self._used:
            return None
        self._used.add(root)
        out = self.nodescen_dict
        self._advance()
        return out

    def _advance(self):
        old = self._pos
        new = (old + self._step) % self._n
        p = new
        while self._names[p] in self._used and (p + 1) % self._n != new:
            p = (p + 1) % self._n
        self._pos = p
        passed = self._names[old:p] if old < p else self._names[old:] + self._names[:p]
        if self._multi:
            gone = set(passed)
            stale = [nd for nd in self._nodes if self.nodescen_dict[nd] in gone]
            for nd in stale:
                self.nodescen_dict[nd] = None
            self._assign(stale)
        else:
            self.nodescen_dict = {"ROOT": self._names[p]}
