"""The multi-rank step path in one process (GPU): a loopback communicator that reports N
ranks and whose all-reduce multiplies by N stands for N ranks holding the same scenarios,
so rank 0's x̄, W and conv must equal those of a one-rank run on the same share.  The
loopback run takes every multi-rank branch of the loop -- ``phgpu_ph_reduce`` (one-node
stores, no clear), the x̄ all-reduce, ``phgpu_ph_update_ex``, the conv all-reduce and its
copy on the side stream behind ``convergence_mark``, the next x̄ reduced ahead of the
convergence test on the speculative solve's x (``xbar_ahead``, into a second buffer) -- the
one-rank run the folded step.  tools/fake_ranks.py times the same pair."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


class LoopbackComm:
    def __init__(self, size):
        self.rank, self.size, self.group = 0, size, None

    def Get_rank(self):
        return 0

    def Get_size(self):
        return self.size

    def allreduce_sum_(self, t):
        t.mul_(self.size)
        return t

    def allreduce_max_(self, t):
        return t

    def Barrier(self):
        pass

    def bcast_object(self, obj, root=0):
        return obj

    def allgather_object(self, obj):
        return [obj] * self.size

    def gather_object(self, obj, root=0):
        return [obj] * self.size


def _run(share, size, comm, iters, convthresh=-1.0):
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.examples import farmer
    names = farmer.scenario_names_creator(share * size)
    if comm is None:
        names = names[:share]
    opts = {"solver_name": "mi355x_pdhg", "PHIterLimit": iters, "defaultPHrho": 1.0, "convthresh": convthresh,
            "verbose": False, "display_progress": False, "toc": False, "device": "cuda:0",
            "batch_creator": farmer.batch_creator, "iter0_solver_options": {"eps_rel": 1e-9},
            "fused_ph_loop": False,  # (the step-by-step one-rank loop is the comparison)
            "iterk_solver_options": {"eps_rel": 1e-9}}
    kw = {"crops_multiplier": 1, "num_scens": share * size if comm is not None else share}
    ph = PH(opts, names, farmer.scenario_creator, scenario_creator_kwargs=kw, mpicomm=comm)
    conv, eobj, tb = ph.ph_main()
    e = ph.engine
    out = dict(conv=conv, tb=tb, W=ph.W_array().copy(), xbar=e.host("xbar").copy(), it=ph._PHIter,
               calls=dict(e.calls), spec=ph._speculate(False))
    e.close()
    return out


@pytest.mark.parametrize("share,size", [(4096, 2), (8192, 8)])
def test_loopback_ranks_match_one_rank(gpu, share, size):
    a = _run(share, size, None, 6)
    b = _run(share, size, LoopbackComm(size), 6)
    assert a["spec"] and b["spec"]
    ca, cb = a["calls"], b["calls"]
    assert ca["ph_step_defer"] >= 6 and ca["ph_update_ex"] == 0, ca
    assert cb["ph_update_ex"] == 6 and cb["allreduce_conv_side"] == 6 and cb["ph_step_defer"] == 0, cb
    assert cb["xbar_ahead_used"] >= 5, cb
    assert abs(a["tb"] - b["tb"]) <= 1e-9 * abs(a["tb"])
    assert abs(a["conv"] - b["conv"]) <= 1e-8 * max(1.0, abs(a["conv"])), (a["conv"], b["conv"])
    # (the two x̄ differ in their last bits -- different summation orders -- and a degenerate
    # prox subproblem can turn that into ~1e-7 in one W entry; the parity bar is 1e-5)
    np.testing.assert_allclose(b["W"], a["W"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(b["xbar"], a["xbar"], rtol=0, atol=1e-8)


def test_loopback_break_matches_one_rank(gpu):
    """To convergence: the same PH iteration at the break, the x̄ at the break (node_buf
    still holds the last update's sums although x̄ was reduced ahead on the discarded
    speculative solve)."""
    a = _run(4096, 2, None, 400, convthresh=1e-2)
    b = _run(4096, 2, LoopbackComm(2), 400, convthresh=1e-2)
    assert a["it"] == b["it"] and a["it"] < 400, (a["it"], b["it"])
    assert abs(a["conv"] - b["conv"]) <= 1e-8, (a["conv"], b["conv"])
    np.testing.assert_allclose(b["xbar"], a["xbar"], rtol=0, atol=1e-8)
