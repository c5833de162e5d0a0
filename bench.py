"""PH throughput benchmark (BASELINE.json metric): farmer, 65,536 scenarios, 1-8 GPUs.

One "step" = one PH iteration of PHBase.iterk_loop (phbase.py:901-957):
Compute_Xbar (kernel + RCCL all-reduce) -> Update_W + convergence_diff (kernel +
all-reduce) -> solve_loop (one batched PDHG solve over the rank's scenarios).
Model generation, Iter0 and the warmup iterations are outside the timed region.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scens S] [--cm CM]
    python bench.py --model aircond --bf 32,32,64     # config 4 (multistage), not the headline

N > 1 is launched by torch.distributed.run (one rank per GPU, RCCL); scenarios are
sharded contiguously (sputils.py:798-810); total scenarios are fixed (strong scaling).
Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy-1_amd"))
sys.path.insert(0, ROOT)

METRIC = "PH iterations/sec + scenario subproblem solves/sec, farmer 64K scen, 1–8 GPUs"
# config 4 parameters (straight_tests.py:36)
AIRCOND_KW = {"Capacity": 200, "QuadShortCoeff": 0.3, "BeginInventory": 50, "mu_dev": 0, "sigma_dev": 40,
              "start_seed": 0}
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--scens", type=int, default=65536)
    p.add_argument("--cm", type=int, default=1)
    p.add_argument("--model", choices=["farmer", "aircond"], default="farmer",
                   help="farmer (config 3, the headline) or aircond (config 4, multistage)")
    p.add_argument("--bf", type=str, default="32,32,64",
                   help="aircond branching factors (scenarios = their product)")
    p.add_argument("--rho", type=float, default=1.0)
    p.add_argument("--eps", type=float, default=1e-9)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-sample", type=int, default=0, help="scenarios in the CPU sample (0 = auto)")
    return p.parse_args()


# ---------------------------------------------------------------- CPU baseline
def _cpu_worker(args):
    """One worker = one rank of the reference's loop: its scenarios solved one at a time
    by the oracle's exact per-scenario QP solver (spopt.py:284-294 structure)."""
    names, cm, W, xbar, rho, S_total = args
    import warnings
    warnings.simplefilter("ignore")
    import numpy as np
    from oracle.models import farmer_scenario
    from oracle.lpqp import solve_qp_ipm
    xs = []
    for k, nm in enumerate(names):
        s = farmer_scenario(nm, cm, num_scens=S_total)
        A, rl, ru, lb, ub, c, q = s.arrays()
        idx = s.nonant_indices()
        c = c.copy()
        q = q.copy()
        c[idx] += W[k] - rho * xbar
        q[idx] += rho
        x, obj, st = solve_qp_ipm(A, rl, ru, lb, ub, c, q)
        xs.append(x[idx])
    return np.array(xs)


def cpu_baseline(S_total, cm, rho, sample):
    """Time PH iterations of the CPU restatement on a bounded sample of the same farmer
    workload, P = min(16, available cores) worker processes (spawned, no GPU state),
    contiguous slices; extrapolate linearly in scenarios to S_total."""
    import multiprocessing as mp
    import numpy as np
    cores = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    P = max(1, min(16, cores))
    names = [f"scen{i}" for i in range(sample)]
    nn = 3 * cm
    rng = np.random.default_rng(0)
    xbar = np.full(nn, 500.0 * cm / (3 * cm)) * rng.uniform(0.5, 1.0, nn)
    W = rng.normal(0.0, 20.0, (sample, nn))
    avg = sample / P
    slices = [list(range(int(i * avg), int((i + 1) * avg))) for i in range(P)]
    jobs = [([names[i] for i in sl], cm, W[sl], xbar, rho, S_total) for sl in slices if sl]
    ctx = mp.get_context("spawn")
    times = []
    with ctx.Pool(len(jobs)) as pool:
        pool.map(_cpu_worker, [(j[0][:1],) + j[1:] for j in jobs])  # warm the workers
        for _ in range(2):
            t0 = time.perf_counter()
            out = pool.map(_cpu_worker, jobs)
            x = np.concatenate(out)
            xb = x.mean(0)                         # Compute_Xbar + Update_W + conv
            W = W + rho * (x - xb)
            _ = np.abs(x - xb).mean()
            times.append(time.perf_counter() - t0)
    t_it = float(np.median(times))
    it_s_full = 1.0 / (t_it * (S_total / sample))
    return {"value": it_s_full, "unit": "PH iterations/s", "cores": len(jobs), "kind": "port",
            "sample": (f"farmer cm={cm}: {sample} of {S_total} scenarios, 2 PH iterations (QP solves "
                       f"by the oracle's dense IPM, one scenario at a time per worker, {len(jobs)} "
                       f"spawned workers); per-iteration time {t_it:.3f}s scaled x{S_total / sample:.0f} "
                       f"to {S_total} scenarios"),
            "sample_seconds_per_iteration": t_it}


# ---------------------------------------------------------------- GPU run
def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if a.gpus > 1 and world == 1:
            raise SystemExit("for --gpus N > 1 launch with: python -m torch.distributed.run "
                             "--nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N")
    cpu = None
    if a.model == "aircond":
        a.bf = [int(v) for v in a.bf.split(",")]
        a.scens = int(np.prod(a.bf))
    if rank == 0 and world == 1 and not a.no_cpu_baseline and a.model == "farmer":
        sample = a.cpu_sample or min(a.scens, 1024)
        cpu = cpu_baseline(a.scens, a.cm, a.rho, sample)

    import torch
    import torch.distributed as dist
    ndev = torch.cuda.device_count()
    # several ranks may share one GPU in the gloo rehearsal (PHGPU_DIST_BACKEND=gloo)
    local_rank = local_rank % max(1, ndev)
    torch.cuda.set_device(local_rank)
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        # RCCL ("nccl") by default; PHGPU_DIST_BACKEND=gloo lets several ranks share one
        # GPU (functional rehearsal of the multi-rank path on a 1-GPU box)
        backend = os.environ.get("PHGPU_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(backend)
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.examples import farmer
    from mpisppy_amd.comm import Comm

    comm = Comm()
    opts = {"solver_name": "mi355x_pdhg", "PHIterLimit": 1, "defaultPHrho": a.rho, "convthresh": -1.0,
            "verbose": False, "display_progress": False, "toc": False,
            "device": f"cuda:{local_rank}",
            "iter0_solver_options": {"eps_rel": a.eps}, "iterk_solver_options": {"eps_rel": a.eps}}
    t_setup = time.perf_counter()
    if a.model == "farmer":
        names = farmer.scenario_names_creator(a.scens)
        opts["batch_creator"] = farmer.batch_creator
        ph = PH(opts, names, farmer.scenario_creator, mpicomm=comm,
                scenario_creator_kwargs={"crops_multiplier": a.cm, "num_scens": a.scens})
        tag = f"farmer{a.scens}_cm{a.cm}"
        workload = {(65536, 1): "farmer PH (config 3)",
                    (1024, 10): "farmer PH (config 2)"}.get((a.scens, a.cm), f"farmer PH, cm={a.cm}")
    else:
        # config 4: aircond multistage (aircond.py:37-330), default parameters, one
        # scenario per leaf of the bf tree; per-node x̄ over all non-leaf nodes
        from mpisppy_amd.examples import aircond
        from mpisppy_amd.sputils import create_nodenames_from_branching_factors
        names = aircond.scenario_names_creator(a.scens)
        opts["batch_creator"] = aircond.batch_creator
        ph = PH(opts, names, aircond.scenario_creator, mpicomm=comm,
                scenario_creator_kwargs={"branching_factors": a.bf, **AIRCOND_KW},
                all_nodenames=create_nodenames_from_branching_factors(a.bf))
        tag = f"aircond{a.scens}"
        workload = f"aircond multistage PH (config 4), bf {'x'.join(map(str, a.bf))}"
    ph.PH_Prep()
    trivial_bound = ph.Iter0()
    e = ph.engine
    b = ph.batch
    torch.cuda.synchronize()
    t_setup = time.perf_counter() - t_setup

    solve_ms = []
    pdhg_iters = []
    red_ms = []

    # per-launch scenario-iterations for the roofline: a D2D snapshot of the iteration
    # counts per step (one copy, no reduction kernel inside the timed region)
    it_snap = torch.empty((a.warmup + a.steps, b.S), dtype=e.iters.dtype, device=e.device)

    def step(k):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        ev[0].record()
        ph.Compute_Xbar()
        ph.Update_W()
        conv = ph.convergence_diff()          # host sync (the reference's break test)
        ev[1].record()
        ph.solve_loop(solver_options=ph.current_solver_options)
        ev[2].record()
        it_snap[k].copy_(ph.engine.iters)
        return ev, conv

    for k in range(a.warmup):
        step(k)
    torch.cuda.synchronize()
    comm.Barrier()
    t0 = time.perf_counter()
    evs = []
    for k in range(a.steps):
        evs.append(step(a.warmup + k))
    torch.cuda.synchronize()
    comm.Barrier()
    elapsed = time.perf_counter() - t0
    units_per_step = it_snap[a.warmup:].sum(dim=1, dtype=torch.int64).cpu().tolist()
    for (ev, conv) in evs:
        red_ms.append(ev[0].elapsed_time(ev[1]))
        solve_ms.append(ev[1].elapsed_time(ev[2]))
    it_host = e.iters.cpu().numpy()
    pdhg_iters = (int(it_host.max()), float(it_host.mean()))
    t = torch.tensor([elapsed], dtype=torch.float64, device=e.device)
    comm.allreduce_max_(t)
    elapsed = float(t.item())
    # roofline of the dominant kernel (the batched solve): algorithmic bytes per launch
    n, m, nnz, nn = b.n, b.m, b.nnz, b.nn
    kinfo = e.kernel_info()
    if kinfo["instance"] >= 0:
        kname = f"k_solve_reg<{kinfo['KC']}, {kinfo['ZC']}, {kinfo['KR']}, {kinfo['ZR']}>"
    else:
        kname = "k_solve"
    traffic, traffic_src = None, None
    pmc = os.path.join(ROOT, "profiles", "r01", f"pmc_summary_{tag}.json")
    if world == 1 and os.path.exists(pmc):
        try:
            d = json.load(open(pmc))
            tr = d.get("solve_traffic_bytes_per_launch", {}).get("void " + kname)
            if tr is not None:
                traffic = tr["total_upper"]
                traffic_src = os.path.relpath(pmc, ROOT)
        except Exception:
            traffic = None
    # issue-side counters of the same kernel (rocprofv3 SQ_* passes, profiles/r01): what
    # actually bounds it, since the iterate never streams through HBM
    issue = None
    sq = os.path.join(ROOT, "profiles", "r01", f"pmc_sq_summary_{tag}.json")
    if world == 1 and os.path.exists(sq):
        try:
            d = json.load(open(sq))
            if d.get("kernel") == "void " + kname:
                dv = d["derived"]
                issue = {"valu_busy": dv["valu_busy"], "lds_issue_busy": dv["lds_issue_busy"],
                         "mean_waves_per_simd": dv["mean_waves_per_simd"],
                         "fp64_tflops": dv["fp64_tflops"], "fp64_frac_of_vector_peak": dv["fp64_frac_of_peak"],
                         "source": os.path.relpath(sq, ROOT)}
        except Exception:
            issue = None
    B = 8 * (nnz + 5 * n + 4 * m + 3 * nn)           # SURVEY.md 8(d), per PDHG iter per scenario
    # average over the K timed launches (HIP events on the launch stream); the rocprofv3
    # kernel trace of the same command gives the per-dispatch durations (profiles/)
    units = float(np.mean(units_per_step))           # scenario-iterations per launch
    solve_s = float(np.mean(solve_ms)) / 1e3
    achieved = B * units / solve_s / 1e9
    ph_its = a.steps / elapsed
    status_ok = bool((e.status.cpu().numpy() == 0).all())
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": ph_its,
            "unit": "PH iterations/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": 1e3 * elapsed / a.steps,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": (f"synthetic ({a.model} scenario generator, seeded as "
                     f"{'farmer.py:52-60' if a.model == 'farmer' else 'aircond.py:37-67'})"),
            "config": {"workload": workload, "scenarios": a.scens,
                       "crops_multiplier": a.cm if a.model == "farmer" else None,
                       "tree_nodes": len(b.node_names),
                       "rho": a.rho, "eps_rel": a.eps, "scenarios_per_gpu": b.S,
                       "n": n, "m": m, "nnz": nnz, "parallelism": f"scenario-sharded x{world} (RCCL x̄ all-reduce)"},
            "solves_per_sec": ph_its * a.scens,
            "pdhg_iters_per_ph_iter": {"max": pdhg_iters[0], "mean": pdhg_iters[1]},
            "time_split_ms": {"solve": float(np.mean(solve_ms)), "xbar_W_conv": float(np.mean(red_ms))},
            "all_optimal": status_ok,
            "trivial_bound": trivial_bound,
            "setup_s": t_setup,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_source": traffic_src, "issue": issue,
                         "kernel": kname, "lanes_per_scenario": kinfo["lanes"],
                         "bytes_per_scenario_iter": B,
                         "scenario_iters_per_launch": units, "launch_ms": solve_s * 1e3,
                         "note": ("achieved = algorithmic PDHG bytes (SURVEY.md 8(d): 8*(nnz+5n+4m+3nn) per "
                                  "scenario-iteration) / launch time; the register-resident kernel keeps the "
                                  "iterates in VGPRs/LDS, so measured HBM traffic per launch (PMC FETCH_SIZE*2 + "
                                  "WRITE_SIZE) is far below it")},
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
