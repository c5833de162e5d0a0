"""XhatBase._try_one on the batched engine (mirrors mpisppy/extensions/xhatbase.py:38-231).

A candidate xhat is named by ``snamedict`` {non-leaf node: scenario name}: node nd's
nonants are taken from scenario snamedict[nd]'s cached nonant values (the hub's x,
delivered to the spoke).  The reference broadcasts each node's values from the rank
that owns that scenario over the node communicator (xhatbase.py:72-123); here the
owner writes its values into a node-indexed device table [num_nodes, nlen_max] and one
SUM all-reduce over the ranks plays the broadcast.  Then every local scenario's
nonants are fixed by one kernel, all scenarios are solved in one launch, and
E[objective] is the candidate's inner bound if every scenario was certified optimal
(xhatbase.py:199-216).
"""
import torch

from ..sputils import rank_slices


class XhatBase:
    def __init__(self, opt):
        self.opt = opt
        self.cylinder_rank = opt.cylinder_rank
        self.n_proc = opt.n_proc
        names = opt.all_scenario_names
        self._slices = rank_slices(len(names), self.n_proc)
        self._where = {}
        for r, sl in enumerate(self._slices):
            for li, gi in enumerate(sl):
                self._where[names[gi]] = (r, li)

    def pre_iter0(self):
        pass

    def post_iter0(self):
        pass

    def _node_depth(self, ndn):
        return ndn.count("_")

    def xhat_table(self, snamedict, nonant_cache):
        """Device [num_nodes, nlen_max] table of the candidate's per-node values.
        nonant_cache: device [nn, S_local] ('ci' order) of the values to draw from."""
        e = self.opt.engine
        b = self.opt.batch
        tab = torch.zeros(e.num_nodes, e.nlen_max, dtype=torch.float64, device=e.device)
        dep = torch.as_tensor(b.nonant_depth, device=e.device)
        off = torch.as_tensor(b.nonant_off, dtype=torch.long, device=e.device)
        for g, ndn in enumerate(e.node_names):
            sname = snamedict.get(ndn)
            if sname is None:
                continue
            if sname not in self._where:
                raise RuntimeError(f"Bad scenario selection for xhat: {sname} for node {ndn}")
            r, li = self._where[sname]
            if r != self.cylinder_rank:
                continue
            sel = torch.nonzero(dep == self._node_depth(ndn)).reshape(-1)
            tab[g].index_copy_(0, off[sel], nonant_cache[sel, li])
        self.opt.mpicomm.allreduce_sum_(tab)
        return tab

    # xhatbase.py:38-216
    def _try_one(self, snamedict, solver_options=None, verbose=False, restore_nonants=True,
                 stage2EFsolvern=None, branching_factors=None, nonant_cache=None):
        if stage2EFsolvern is not None:
            raise NotImplementedError("stage2EFsolvern (EF sub-solves) is outside the batched hot path")
        if nonant_cache is None:
            nonant_cache = self.opt.engine.nonant_x_dev()
        tab = self.xhat_table(snamedict, nonant_cache)
        self.opt._fix_nonants(tab)
        self.opt.solve_loop(solver_options=solver_options, verbose=verbose)
        infeasP = self.opt.infeas_prob()
        if infeasP > 1e-12:
            self.opt._restore_nonants()
            return None
        obj = self.opt.Eobjective(verbose=verbose)
        self.last_table = tab
        if restore_nonants:
            self.opt._restore_nonants()
        return obj
