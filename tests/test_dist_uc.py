"""Config 5 on two ranks: 8 UC scenarios split over 2 gloo ranks sharing cuda:0, each rank
on the shared-matrix streaming path (path 4), two PH iterations through the engine's
reductions (node-buffer and conv all-reduces, phbase.py:83-87 / 330-343).  The same
8 scenarios in one process are the reference for the 2-rank run: trivial bound, W, x̄
and conv agree to the PDHG tolerance of config 5 (parity against the reference itself is
unpinned, see test_gpu_uc.py)."""
import json
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "uc.json")))
ITERS = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(comm=None):
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.examples import uc
    names = GOLD["names"]
    rho = uc.rho_vector(uc.scenario_creator(names[0], num_scens=len(names)))
    opts = {"solver_name": "mi355x_pdhg", "PHIterLimit": ITERS, "defaultPHrho": 1.0, "convthresh": -1.0,
            "verbose": False, "display_progress": False, "toc": False, "device": "cuda:0",
            "batch_creator": uc.batch_creator, "rho_array": rho,
            "iter0_solver_options": {"eps_rel": 1e-6}, "iterk_solver_options": {"eps_rel": 1e-6}}
    ph = PH(opts, names, uc.scenario_creator, mpicomm=comm, scenario_creator_kwargs={"num_scens": len(names)})
    conv, eobj, tb = ph.ph_main()
    assert ph.engine.kernel_info()["path"] == 4
    return ph, conv, eobj, tb


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
        ph, conv, eobj, tb = _run(Comm())
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), W=ph.W_array(), conv=conv, eobj=eobj, tb=tb,
                 xbar=ph.xbar_by_node()["ROOT"], names=np.array(ph.local_scenario_names))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_uc_two_ranks_match_one(gpu, tmp_path):
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    r = [np.load(tmp_path / f"r{k}.npz") for k in range(2)]
    assert list(r[0]["names"]) + list(r[1]["names"]) == GOLD["names"]
    ph, conv, eobj, tb = _run()
    W1 = ph.W_array()
    W2 = np.concatenate([r[0]["W"], r[1]["W"]])
    scale = max(1.0, np.abs(W1).max())
    for k in range(2):
        assert abs(float(r[k]["tb"]) - tb) <= 1e-6 * abs(tb)
        assert abs(float(r[k]["conv"]) - conv) <= 1e-4 * max(1.0, abs(conv))
        assert np.abs(r[k]["xbar"] - ph.xbar_by_node()["ROOT"]).max() <= 1e-4
    assert np.abs(W2 - W1).max() <= 1e-4 * scale
