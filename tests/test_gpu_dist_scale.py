"""The N > 1 product path at configuration scale: 2 ranks (gloo, sharing cuda:0), each
holding its contiguous half of the scenarios (sputils.py:803-810), run PHBase.iterk_loop
-- the loop bench.py times -- through the engine's multi-rank step:

    phgpu_ph_reduce (x̄ partials)  ->  all-reduce of the node buffer (phbase.py:83-87)
    ->  phgpu_ph_update_ex (x̄ scatter, W, local conv)  ->  conv all-reduce on the side
    stream, / n_proc (phbase.py:339-343)  ->  the speculative next solve (path 6)

which is exactly what the driver's 8-GPU run executes (RCCL instead of gloo).  No fused
one-rank step may run (asserted from the engine's call counters and ipm_info's
folded_steps).  Against the single-process fixtures (the partition does not change the
PH iterates: conv is the mean of two equal slices' means):

  * farmer 65,536 (config 3, 32,768 per rank, the one-lane interior point): trivial bound,
    x̄ and conv of 5 PH iterations, sampled W and E[obj] (farmer_scale.json); then ph_main
    to conv < 1e-2 breaking at the oracle's PH iteration 331 +-1, x̄ and sampled W there
    (farmer_conv.json);
  * aircond 32 x 32 x 64 (config 4, 1,057 nodes; the root node straddles the ranks):
    trivial bound, x̄ of every node and conv of 3 PH iterations, sampled W and E[obj]
    (aircond_scale.json).

Tolerances (north_star): objectives 1e-5 relative, x̄ / W 1e-5 absolute, iterations +-1.
"""
import json
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
SCALE = json.load(open(os.path.join(HERE, "golden", "farmer_scale.json")))
CONV = json.load(open(os.path.join(HERE, "golden", "farmer_conv.json")))
AIR_FILE = os.path.join(HERE, "golden", "aircond_scale.json")
OBJ_REL = 1e-5
ABS = 1e-5
WORLD = 2
AIR_KW = {"Capacity": 200, "QuadShortCoeff": 0.3, "BeginInventory": 50, "mu_dev": 0, "sigma_dev": 40,
          "start_seed": 0}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _record(ph, names=None):
    """Wrap the engine's conv readback to keep the trajectory and the x̄ of each
    iteration (node_xbar synchronises the stream; the values are unaffected)."""
    e = ph.engine
    seen, xbars = [], []
    wait, diff = e.convergence_wait, e.convergence_diff

    def snap(v):
        seen.append(v)
        nx = e.node_xbar()
        if names is None:
            xbars.append(np.array(nx["ROOT"][:3]))
        else:
            xbars.append(np.array([nx[nd][:2] for nd in names]))
        return v

    e.convergence_wait = lambda: snap(wait())
    e.convergence_diff = lambda: snap(diff())
    return seen, xbars


def _path_record(ph):
    e = ph.engine
    k = e.kernel_info()
    i = e.ipm_info()
    return dict(path=k["path"], lanes=int(i["lanes"]), compiled=int(i["compiled"]), scratch=int(i["scratch_bytes"]),
                folded=int(i["folded_steps"]), calls=dict(e.calls))


def _worker(rank, world, port, out_dir, case):
    import sys
    root = os.path.dirname(HERE)
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
        res = {}
        if case == "farmer":
            from mpisppy_amd.examples import farmer
            S = 65536
            names = farmer.scenario_names_creator(S)

            def make(iters, thresh):
                opts = {"solver_name": "mi355x_pdhg", "PHIterLimit": iters, "defaultPHrho": 1.0,
                        "convthresh": thresh, "verbose": False, "display_progress": False, "toc": False,
                        "device": "cuda:0", "batch_creator": farmer.batch_creator,
                        "iterk_solver_options": dict(farmer.PDHG_ITERK_OPTIONS)}
                return PH(opts, names, farmer.scenario_creator, mpicomm=Comm(),
                          scenario_creator_kwargs={"crops_multiplier": 1, "num_scens": S})

            # (a) 5 PH iterations of the product loop against farmer_scale.json
            ph = make(5, -1.0)
            ph.PH_Prep()
            res["tb"] = ph.Iter0()
            res["spec"] = ph._speculate(False)
            seen, xbars = _record(ph)
            ph.iterk_loop()
            res["conv5"] = np.array(seen)
            res["xbar5"] = np.array(xbars)
            res["W5"] = ph.W_array()
            res["eobj5"] = ph.Eobjective()
            res["names"] = np.array(ph.local_scenario_names)
            res["rec5"] = _path_record(ph)
            res["all_optimal5"] = bool((ph.engine.host("status") == 0).all())
            ph.engine.close()
            # (b) ph_main to conv < 1e-2
            want = CONV["breaks"]["0.01"]["iteration"]
            ph = make(want + 20, 1e-2)
            ph._create_solvers()       # the engine ph_main will use, so that _record can wrap it
            seen, _ = _record(ph)
            ph.ph_main()
            res["converged"] = bool(ph.converged)
            res["break"] = int(ph._PHIter)
            res["conv_b"] = np.array(seen)
            res["xbar_b"] = ph.xbar_by_node()["ROOT"][:3]
            res["W_b"] = ph.W_array()
            res["rec_b"] = _path_record(ph)
            ph.engine.close()
        else:
            from mpisppy_amd.examples import aircond
            from mpisppy_amd.sputils import create_nodenames_from_branching_factors
            g = json.load(open(AIR_FILE))
            bf = list(g["branching_factors"])
            S = int(np.prod(bf))
            opts = {"solver_name": "mi355x_pdhg", "PHIterLimit": g["ph_iters"], "defaultPHrho": 1.0,
                    "convthresh": -1.0, "verbose": False, "display_progress": False, "toc": False,
                    "device": "cuda:0", "batch_creator": aircond.batch_creator}
            ph = PH(opts, aircond.scenario_names_creator(S), aircond.scenario_creator, mpicomm=Comm(),
                    scenario_creator_kwargs={"branching_factors": bf, **AIR_KW},
                    all_nodenames=create_nodenames_from_branching_factors(bf))
            ph.PH_Prep()
            res["tb"] = ph.Iter0()
            res["spec"] = ph._speculate(False)
            seen, xbars = _record(ph, g["node_names"])
            ph.iterk_loop()
            res["conv"] = np.array(seen)
            res["xbar"] = np.array(xbars)
            res["W"] = ph.W_array()
            res["eobj"] = ph.Eobjective()
            res["names"] = np.array(ph.local_scenario_names)
            res["rec"] = _path_record(ph)
            res["all_optimal"] = bool((ph.engine.host("status") == 0).all())
            ph.engine.close()
        with open(os.path.join(out_dir, f"{case}_r{rank}.json"), "w") as f:
            json.dump({k: (v.tolist() if isinstance(v, np.ndarray) else v) for k, v in res.items()}, f)
    finally:
        dist.destroy_process_group()


def _spawn(case, tmp_path):
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(WORLD, _free_port(), str(tmp_path), case), nprocs=WORLD, join=True)
    return [json.load(open(tmp_path / f"{case}_r{k}.json")) for k in range(WORLD)]


def _assert_multirank_step(rec, iters, lanes):
    """Path 6 on its expected lane count, every PH step through reduce -> all-reduce ->
    update_ex with the conv all-reduce on the side stream, nothing folded or fused, the next
    x̄ reduced ahead of each convergence test."""
    assert rec["path"] == 6 and rec["compiled"] == 1 and rec["scratch"] <= 1024, rec
    assert rec["lanes"] == lanes, rec
    c = rec["calls"]
    assert c["ph_reduce"] >= iters and c["allreduce_xbar"] == c["ph_reduce"], c
    assert c["ph_update_ex"] == iters and c["allreduce_conv_side"] == iters, c
    assert c["ph_step_local"] == 0 and c["ph_step_defer"] == 0 and rec["folded"] == 0, (c, rec)
    # from the second PH iteration on, x̄ was reduced ahead of the convergence test
    # (engine.xbar_ahead on the speculative solve's x, used once that solve is committed)
    assert c["xbar_ahead_used"] >= iters - 1, c


def _global_rows(r, sample):
    """Rows of the sampled global scenarios from the ranks' local W arrays."""
    names = r[0]["names"] + r[1]["names"]
    assert names == [f"scen{i}" for i in range(len(names))]
    W = np.concatenate([np.array(r[0]["W" if "W" in r[0] else "W5"]), np.array(r[1]["W" if "W" in r[1] else "W5"])])
    return W[np.array(sample)]


@pytest.mark.timeout(600)
def test_two_rank_farmer65536_headline_path(gpu, tmp_path):
    r = _spawn("farmer", tmp_path)
    g = SCALE["farmer65536_cm1"]
    assert len(r[0]["names"]) == 32768 and r[0]["names"][0] == "scen0" and r[1]["names"][0] == "scen32768"
    for k in range(WORLD):
        assert r[k]["spec"], "the bench's loop variant (speculative solve) must be the one tested"
        assert abs(r[k]["tb"] - g["trivial_bound"]) <= OBJ_REL * abs(g["trivial_bound"]), (k, r[k]["tb"])
        _assert_multirank_step(r[k]["rec5"], 5, lanes=1)
        assert r[k]["all_optimal5"]
        conv = np.array(r[k]["conv5"])
        assert np.abs(conv - np.array(g["conv"])).max() <= ABS, (k, conv, g["conv"])
        xb = np.array(r[k]["xbar5"])
        assert np.abs(xb - np.array(g["xbar"])[:, :3]).max() <= ABS, (k, xb)
        assert abs(r[k]["eobj5"] - g["Eobj"]) <= OBJ_REL * abs(g["Eobj"]), (k, r[k]["eobj5"], g["Eobj"])
    W = np.concatenate([np.array(r[0]["W5"]), np.array(r[1]["W5"])])[np.array(g["sample"])]
    err = np.abs(W - np.array(g["W"]))
    assert err.max() <= ABS, (err.max(), g["sample"][int(err.max(1).argmax())])
    # (b) ph_main to conv < 1e-2: the break iteration +-1, x̄ and W there
    want = CONV["breaks"]["0.01"]
    for k in range(WORLD):
        assert r[k]["converged"] and abs(r[k]["break"] - want["iteration"]) <= 1, (k, r[k]["break"])
        it = r[k]["break"]
        _assert_multirank_step(r[k]["rec_b"], it, lanes=1)
        dev = np.abs(np.array(r[k]["conv_b"]) - np.array(CONV["conv"][:it]))
        assert dev.max() <= 1e-6, (k, dev.max(), int(dev.argmax()) + 1)
        assert np.abs(np.array(r[k]["xbar_b"]) - np.array(want["xbar"][str(it)])).max() <= ABS
    assert r[0]["break"] == r[1]["break"]
    it = r[0]["break"]
    W = np.concatenate([np.array(r[0]["W_b"]), np.array(r[1]["W_b"])])[np.array(CONV["sample"])]
    err = np.abs(W - np.array(want["W"][str(it)]))
    assert err.max() <= ABS, (err.max(), CONV["sample"][int(err.max(1).argmax())])


@pytest.mark.timeout(600)
@pytest.mark.skipif(not os.path.exists(AIR_FILE), reason="aircond_scale.json not generated")
def test_two_rank_aircond65536_node_reductions(gpu, tmp_path):
    r = _spawn("aircond", tmp_path)
    g = json.load(open(AIR_FILE))
    assert g["kwargs"] == AIR_KW and g["rho"] == 1.0
    assert len(r[0]["names"]) == 32768
    for k in range(WORLD):
        assert r[k]["spec"]
        assert abs(r[k]["tb"] - g["trivial_bound"]) <= OBJ_REL * abs(g["trivial_bound"]), (k, r[k]["tb"])
        rec = r[k]["rec"]
        # one lane above 16,384 local scenarios (aircond's module spills 524 B per lane)
        _assert_multirank_step(rec, g["ph_iters"], lanes=1)
        assert r[k]["all_optimal"]
        conv = np.array(r[k]["conv"])
        assert np.abs(conv - np.array(g["conv"])).max() <= ABS, (k, conv, g["conv"])
        xb = np.array(r[k]["xbar"])                         # [iters, 1057 nodes, 2]
        err = np.abs(xb - np.array(g["xbar"]))
        assert err.max() <= ABS, (k, err.max(), g["node_names"][int(err.max(axis=(0, 2)).argmax())])
        assert abs(r[k]["eobj"] - g["Eobj"]) <= OBJ_REL * abs(g["Eobj"]), (k, r[k]["eobj"], g["Eobj"])
    W = _global_rows(r, g["sample"])
    err = np.abs(W - np.array(g["W"]))
    assert err.max() <= ABS, (err.max(), g["sample"][int(err.max(1).argmax())])
