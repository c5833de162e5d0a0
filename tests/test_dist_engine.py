"""Engine-level multi-rank PH: 2 ranks (gloo, sharing cuda:0) run ``PH.ph_main`` through
the engine's own reduction path -- phgpu_ph_reduce partials, the Comm all-reduce of the
node buffer (phbase.py:83-87, spbase.py:349-359), phgpu_ph_update, the conv all-reduce
and /n_proc (phbase.py:330-343), the expectation sums (spopt.py:310-391) -- on aircond
4-3-2, whose tree nodes straddle the rank boundary.  Compared with the single-process
oracle restatement run with n_proc = 2 (rank partition of sputils.py:798-810)."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

BF = [4, 3, 2]
KW = dict(Capacity=200, QuadShortCoeff=0.3, BeginInventory=50, mu_dev=0, sigma_dev=40, start_seed=0)
ITERS = 5


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "mpi-sppy-1_amd"))
    sys.path.insert(0, root)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mpisppy_amd.comm import Comm
        from mpisppy_amd.opt.ph import PH
        from mpisppy_amd.examples import aircond
        from mpisppy_amd.sputils import create_nodenames_from_branching_factors
        kw = dict(KW, branching_factors=BF)
        opts = {"solver_name": "mi355x_pdhg", "PHIterLimit": ITERS, "defaultPHrho": 1.0, "convthresh": -1.0,
                "verbose": False, "display_progress": False, "toc": False, "device": "cuda:0"}
        ph = PH(opts, aircond.scenario_names_creator(24), aircond.scenario_creator, mpicomm=Comm(),
                scenario_creator_kwargs=kw, all_nodenames=create_nodenames_from_branching_factors(BF))
        conv, eobj, tb = ph.ph_main()
        nx = ph.xbar_by_node()
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), W=ph.W_array(), conv=conv, eobj=eobj, tb=tb,
                 names=np.array(ph.local_scenario_names),
                 nodes=np.array(list(nx.keys())), xbar=np.array([v[:2] for v in nx.values()]))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_engine_ph_matches_oracle(gpu, tmp_path):
    import torch.multiprocessing as mp
    from oracle.models import aircond_scenario
    from oracle.ph import OraclePH
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    r = [np.load(tmp_path / f"r{k}.npz") for k in range(2)]
    names = list(r[0]["names"]) + list(r[1]["names"])
    assert names == [f"scen{i}" for i in range(24)] and len(r[0]["names"]) == 12
    sc = [aircond_scenario(f"scen{i}", BF, **KW) for i in range(24)]
    oph = OraclePH(sc, 1.0, n_proc=2)
    otb = oph.iter0()
    oph.iterk_loop(ITERS, -1.0)
    for k in range(2):
        assert abs(float(r[k]["tb"]) - otb) <= 1e-5 * abs(otb)
        assert abs(float(r[k]["conv"]) - oph.conv) <= 1e-5, (float(r[k]["conv"]), oph.conv)
        assert abs(float(r[k]["eobj"]) - oph.Eobjective()) <= 1e-5 * abs(oph.Eobjective())
        # every rank holds the global x̄ of every node
        for nd, v in zip(r[k]["nodes"], r[k]["xbar"]):
            if str(nd) in oph.node_xbar:
                assert np.abs(v - oph.node_xbar[str(nd)]).max() <= 1e-5, (k, nd)
    W = np.concatenate([r[0]["W"], r[1]["W"]])
    assert np.abs(W - oph.W).max() <= 1e-5
