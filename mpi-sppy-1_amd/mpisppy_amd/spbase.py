"""SPBase: scenario creation, rank partition, tree bookkeeping (mirrors mpisppy/spbase.py).

Constructor signature and attribute names follow spbase.py:44-120.  What changes is
the storage: instead of one Pyomo model per local scenario, the local scenarios are
one :class:`ScenarioBatch` (shared CSR pattern + per-scenario arrays), built either

  * from ``options["batch_creator"](local_names, **scenario_creator_kwargs)``
    (vectorised; used for the 65,536-scenario configurations), or
  * from ``scenario_creator(name, **kwargs)`` per local name, exactly like
    SPBase._create_scenarios (spbase.py:255-291); those LinearModels are kept in
    ``local_scenarios`` so values can be loaded back into them.
"""
import numpy as np

from . import global_toc
from .batch import batch_from_models
from .comm import Comm
from .sputils import rank_slices


def nonleaf_nodenames(all_nodenames):
    """Non-leaf nodes in all_nodenames order (a node is a leaf when it has no child
    '<name>_0', sputils.find_leaves 659-670); two-stage = ['ROOT']."""
    if all_nodenames is None or all_nodenames == ["ROOT"]:
        return ["ROOT"]
    s = set(all_nodenames)
    return [nd for nd in all_nodenames if nd + "_0" in s]


class SPBase:
    def __init__(self, options, all_scenario_names, scenario_creator, scenario_denouement=None,
                 all_nodenames=None, mpicomm=None, scenario_creator_kwargs=None,
                 variable_probability=None, E1_tolerance=1e-5):
        self.options = options
        self.all_scenario_names = list(all_scenario_names)
        self.scenario_creator = scenario_creator
        self.scenario_denouement = scenario_denouement
        self.E1_tolerance = E1_tolerance
        if all_nodenames is None:
            self.all_nodenames = ["ROOT"]
        elif "ROOT" in all_nodenames:
            self.all_nodenames = list(all_nodenames)
        else:
            raise RuntimeError("'ROOT' must be in the list of node names")
        self.variable_probability = variable_probability
        self.multistage = len(self.all_nodenames) > 1
        self.mpicomm = mpicomm if mpicomm is not None else Comm()
        self.cylinder_rank = self.mpicomm.Get_rank()
        self.n_proc = self.mpicomm.Get_size()
        self.global_rank = self.cylinder_rank
        if options.get("toc", True):
            global_toc("Initializing SPBase", self.cylinder_rank == 0)
        if self.n_proc > len(self.all_scenario_names):
            raise RuntimeError("More ranks than scenarios")                 # spbase.py:94-95
        if options.get("bundles_per_rank", 0):
            raise NotImplementedError("bundles are outside the batched PH hot path")
        self.bundling = False
        # rank slices (sputils.py:798-810 via spbase.py:184-216)
        self._rank_slices = rank_slices(len(self.all_scenario_names), self.n_proc)
        self.local_scenario_names = [self.all_scenario_names[i]
                                     for i in self._rank_slices[self.cylinder_rank]]
        self.node_names = nonleaf_nodenames(self.all_nodenames)
        self.scenario_creator_kwargs = scenario_creator_kwargs or {}
        self._create_scenarios()
        self._use_variable_probability_setter()

    def _create_scenarios(self):
        kw = self.scenario_creator_kwargs
        bc = self.options.get("batch_creator")
        num_all = len(self.all_scenario_names)
        if bc is not None:
            self.local_scenarios = {}
            self.batch = bc(self.local_scenario_names, **kw)
            # uniform default probability when the creator gives none (spbase.py:515-520)
            if np.any(~np.isfinite(self.batch.prob)):
                self.batch.prob[:] = 1.0 / num_all
        else:
            models = [self.scenario_creator(nm, **kw) for nm in self.local_scenario_names]
            self.local_scenarios = dict(zip(self.local_scenario_names, models))
            for nm, mdl in self.local_scenarios.items():
                if mdl._mpisppy_node_list is None:
                    raise RuntimeError(f"_mpisppy_node_list not found on scenario {nm}")
                if mdl._mpisppy_probability is None and self.cylinder_rank == 0 and nm == self.local_scenario_names[0]:
                    print(f"Did not find _mpisppy_probability, assuming uniform probability {1.0 / num_all}")
            self.batch = batch_from_models(self.local_scenario_names, models,
                                           all_nodenames=self.all_nodenames, num_all_scens=num_all,
                                           node_names=self.node_names if self.multistage else None)
        for nd in self.batch.node_names:
            if nd not in self.node_names:
                raise RuntimeError(f"Tree node '{nd}' not in all_nodenames list {self.all_nodenames}")
        self.is_minimizing = self.batch.sense > 0
        self.nonant_length = self.batch.nn
        self.scenarios_constructed = True

    @property
    def local_subproblems(self):
        return self.local_scenarios

    def _options_check(self, required_options, given_options):
        missing = [o for o in required_options if o not in given_options]
        if missing:
            raise ValueError(f"Missing option(s) {missing}")

    # spbase.py:394-437
    def _use_variable_probability_setter(self, verbose=False):
        """Per-nonant probability coefficients (``variable_probability(model, **kwargs)`` ->
        [(id(vardata), prob)]; spbase.py:394-437): ``self.var_prob`` [S_local, nn], each
        nonant's node coefficient (prob_coeff) unless the function names it, and
        ``self.prob0_mask`` (prob != 0) -- the x̄ weights of _Compute_Xbar and the W mask of
        Update_W (phbase.py:54-79, 315-318), on the device through phgpu_set_nonant_probs.
        With a batch_creator there are no per-scenario models: pass the [S_local, nn] array
        as ``options["variable_probability_array"]``."""
        self.var_prob = None
        self.prob0_mask = None
        arr = self.options.get("variable_probability_array")
        if self.variable_probability is None and arr is None:
            return
        b = self.batch
        dep = np.asarray(b.nonant_depth, dtype=np.int64)
        vp = np.asarray(b.prob_coeff, dtype=np.float64)[:, dep].copy()
        if arr is not None:
            arr = np.asarray(arr, dtype=np.float64)
            if arr.shape != vp.shape:
                raise ValueError(f"variable_probability_array has shape {arr.shape}, expected {vp.shape}")
            vp[:] = arr
        else:
            if not self.local_scenarios:
                raise RuntimeError("variable_probability needs per-scenario models; with a batch_creator pass "
                                   "options['variable_probability_array']")
            kw = self.options.get("variable_probability_kwargs", {})
            for s, nm in enumerate(self.local_scenario_names):
                mdl = self.local_scenarios[nm]
                id2k = {}
                k = 0
                for nd in mdl._mpisppy_node_list:
                    for v in nd.nonant_vardata_list:
                        id2k[id(v)] = k
                        k += 1
                for vid, prob in self.variable_probability(mdl, **kw):
                    vp[s, id2k[vid]] = prob
        self.var_prob = vp
        self.prob0_mask = (vp != 0.0).astype(np.float64)
        if not self.options.get("do_not_check_variable_probabilities", False):
            self._check_variable_probabilities_sum(verbose)

    # spbase.py:456-497
    def _check_variable_probabilities_sum(self, verbose=False):
        """Every nonant's coefficients sum to 1 over its node's scenarios (all ranks)."""
        import torch
        b = self.batch
        gid = {nd: i for i, nd in enumerate(self.node_names)}
        node_of = np.array([[gid[b.node_names[g]] for g in row] for row in np.asarray(b.node_of)], dtype=np.int64)
        nl = max(1, int(b.nlen_max))
        acc = np.zeros((len(self.node_names), nl))
        seen = np.zeros((len(self.node_names), nl))
        dep = np.asarray(b.nonant_depth, dtype=np.int64)
        off = np.asarray(b.nonant_off, dtype=np.int64)
        for k in range(b.nn):
            np.add.at(acc, (node_of[:, dep[k]], off[k]), self.var_prob[:, k])
            seen[node_of[:, dep[k]], off[k]] = 1.0
        t = torch.from_numpy(np.concatenate([acc.ravel(), seen.ravel()]))
        import torch.distributed as dist
        if self.n_proc > 1 and dist.get_backend() == "nccl":
            t = t.to(self.options.get("device") or "cuda")  # (RCCL reduces device tensors only)
        self.mpicomm.allreduce_sum_(t)
        t = t.cpu()
        acc = t[:acc.size].numpy().reshape(acc.shape)
        seen = t[acc.size:].numpy().reshape(acc.shape) > 0
        bad = seen & ~np.isclose(acc, 1.0, atol=self.E1_tolerance)
        if bad.any():
            g, i = np.argwhere(bad)[0]
            raise RuntimeError(f"Node {self.node_names[g]}, nonant {i} has conditional probability sum {acc[g, i]}")

