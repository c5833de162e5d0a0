"""PH throughput benchmark (BASELINE.json metric): farmer, 65,536 scenarios, 1-8 GPUs.

One "step" = one PH iteration of the product loop PHBase.iterk_loop (phbase.py:901-957):
Compute_Xbar (kernels + all-reduce of the node buffer) -> Update_W + convergence_diff
(kernel + scalar all-reduce, host readback of conv) -> solve_loop (one batched PDHG solve
over the rank's scenarios, gripe status check).  The timed region is ``iterk_loop``
itself, run for exactly K iterations.  Model generation, Iter0 and the W warmup
iterations are outside it.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scens S] [--cm CM]
    python bench.py --model aircond --bf 32,32,64     # config 4 (multistage)
    python bench.py --model uc [--scens 1000]          # config 5 (UC LP relaxation, path 4)

--gpus N > 1 started without torch.distributed.run launches itself with N local ranks
(one per GPU, RCCL).  ``--backend gloo`` lets several ranks share one GPU (a functional
rehearsal on a 1-GPU box; the x̄ all-reduce then goes through host memory).  Scenarios
are sharded contiguously (sputils.py:798-810); the total is fixed (strong scaling).
Rank 0 prints ONE JSON line on stdout (everything else goes to stderr).
"""
import argparse
import contextlib
import json
import os
import socket
import subprocess
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
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
FP64_PEAK_TFLOPS = 78.6   # MI355X spec: fp64 vector = 1/2 of the 157.3 TF fp32 vector peak
INFINITY_CACHE = 256 << 20
INSTRUMENT_EVERY = 4      # one timed solve in 4 carries HIP timing events (engine.instrument)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--scens", type=int, default=65536)
    p.add_argument("--cm", type=int, default=1)
    p.add_argument("--model", choices=["farmer", "aircond", "uc"], default="farmer",
                   help="farmer (config 3, the headline), aircond (config 4, multistage) or uc "
                        "(config 5: the UC LP relaxation, 1,000 wind scenarios)")
    p.add_argument("--bf", type=str, default="32,32,64",
                   help="aircond branching factors (scenarios = their product)")
    p.add_argument("--rho", type=float, default=1.0)
    p.add_argument("--eps", type=float, default=None,
                   help="PDHG eps_rel of the PH solves (default 1e-9; uc: 1e-6 for Iter0 and PH)")
    p.add_argument("--no-conv-overlap", action="store_true",
                   help="N > 1: the conv all-reduce on the launch stream ahead of the next solve "
                        "instead of on a side stream under it (the comparison for the overlap)")
    p.add_argument("--backend", choices=["auto", "nccl", "gloo"], default="auto",
                   help="torch.distributed backend for N > 1 (auto: RCCL when every rank has its own GPU)")
    p.add_argument("--solver-opt", action="append", default=[], metavar="KEY=VALUE",
                   help="extra phgpu_options for the PH solves (tuning), e.g. check_every=32")
    p.add_argument("--default-solver-options", action="store_true",
                   help="farmer: ignore the example's recommended PH-solve options (library defaults)")
    p.add_argument("--check", choices=["auto", "on", "off"], default="auto",
                   help="compare the warmup with the oracle fixture of the workload (farmer 65,536 cm=1, "
                        "farmer 1,024 cm=10, aircond 32x32x64) and exit non-zero on a mismatch; auto: when "
                        "the workload and rho match a fixture, on: whenever the workload has one (a "
                        "different --rho then fails by design)")
    p.add_argument("--fused-loop", action="store_true",
                   help="one rank: PHBase.iterk_loop's K iterations in one cooperative launch (phgpu_ph_loop, "
                        "opt-in: measured no faster than the step-by-step loop, DESIGN.md 3.11)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-sample", type=int, default=0, help="scenarios in the CPU sample (0 = auto)")
    p.add_argument("--profile-dir", default=None,
                   help="profiles/<round> directory holding the PMC summaries (default: newest)")
    return p.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# ---------------------------------------------------------------- self-launch
def launch_ranks(a):
    """--gpus N without a torch.distributed.run parent: start one (127.0.0.1 rendezvous)
    as a child process -- nothing here has touched the GPU -- and exit with its code."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    log("launching:", " ".join(cmd))
    return subprocess.run(cmd, env=env).returncode


# ---------------------------------------------------------------- CPU baseline
_MODELS = {}


def _cpu_worker(args):
    """One worker = one rank of the reference's solve loop (spopt.py:284-294): its
    scenarios solved one at a time, Iter0 LPs by HiGHS, PH QPs by the oracle's dense IPM
    (stand-ins for the external LP/QP solver the reference calls per scenario)."""
    names, cm, S_total, W, xbar, rho, iter0, qp = args
    import warnings
    warnings.simplefilter("ignore")
    from oracle.models import farmer_scenario
    from oracle.lpqp import solve_qp_ipm, solve_lp_highs, solve_qp_highs
    xs = []
    for k, nm in enumerate(names):
        if nm not in _MODELS:
            s = farmer_scenario(nm, cm, num_scens=S_total)
            _MODELS[nm] = (s.arrays(), s.nonant_indices())
        (A, rl, ru, lb, ub, c, q), idx = _MODELS[nm]
        if iter0:
            x, obj, st = solve_lp_highs(A, rl, ru, lb, ub, c)
        else:
            c = c.copy()
            q = q.copy()
            c[idx] += W[k] - rho * xbar
            q[idx] += rho
            if qp == "highs":
                x, obj, st = solve_qp_highs(A, rl, ru, lb, ub, c, q)
            else:
                x, obj, st = solve_qp_ipm(A, rl, ru, lb, ub, c, q)
        xs.append(x[idx])
    return np.array(xs)


def _cgroup_cpus():
    """CPUs this process may use by its cgroup's CPU quota: (count or None, evidence).
    cgroup v2 /sys/fs/cgroup/cpu.max ("QUOTA PERIOD" or "max PERIOD"), else v1
    cpu.cfs_quota_us / cpu.cfs_period_us."""
    try:
        raw = open("/sys/fs/cgroup/cpu.max").read().strip()
        q, per = raw.split()[:2]
        return (None if q == "max" else max(1, int(int(q) // int(per)))), f"/sys/fs/cgroup/cpu.max = {raw!r}"
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        ev = f"cpu.cfs_quota_us = {q}, cpu.cfs_period_us = {per}"
        return (None if q <= 0 else max(1, q // per)), ev
    except (OSError, ValueError):
        return None, "no cgroup CPU quota file"


def cpu_share():
    """Worker count of the CPU baseline and its evidence: the cgroup quota when there is
    one, capped by the affinity set; without a quota, the affinity set capped by
    OMP_NUM_THREADS (which the GPU box sets to its per-GPU CPU share)."""
    _, ncpu, aff = _host_cpu()
    quota, ev = _cgroup_cpus()
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if quota is not None:
        return min(aff, quota), {"cgroup": ev, "cores_source": "cgroup CPU quota"}
    if omp > 0:
        return min(aff, omp), {"cgroup": ev, "cores_source": f"no quota; OMP_NUM_THREADS={omp} (the box's CPU share)"}
    return aff, {"cgroup": ev, "cores_source": "no quota; sched_getaffinity"}


def _host_cpu():
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    return model, os.cpu_count(), aff


def cpu_baseline(S_total, cm, rho, sample, iters=4):
    """PH iterations of the CPU restatement on a bounded sample of the same workload.

    P worker processes (spawned, no GPU state), one per host core this process may use
    (the affinity set, capped by OMP_NUM_THREADS -- the box's CPU share); contiguous
    slices (sputils.py:798-810); Iter0 (LP) then ``iters`` PH iterations with the real PH
    state of the sample (x̄ -> W -> solve); per-iteration time = median of iterations
    2..iters, scaled linearly to S_total scenarios."""
    import multiprocessing as mp
    model, ncpu, aff = _host_cpu()
    P, cores_ev = cpu_share()
    names = [f"scen{i}" for i in range(sample)]
    nn = 3 * cm
    avg = sample / P
    slices = [list(range(int(i * avg), int((i + 1) * avg))) for i in range(P)]
    slices = [sl for sl in slices if sl]
    W = np.zeros((sample, nn))
    xbar = np.zeros(nn)
    ctx = mp.get_context("spawn")
    t_start = time.perf_counter()
    with ctx.Pool(len(slices)) as pool:
        def run(iter0, W, xbar, qp="ipm"):
            out = pool.map(_cpu_worker, [([names[i] for i in sl], cm, S_total, W[sl], xbar, rho, iter0, qp)
                                         for sl in slices])
            return np.concatenate(out)

        def ph_loop(x, qp):
            W, times = np.zeros((sample, nn)), []
            for _ in range(iters):
                t0 = time.perf_counter()
                xbar = x.mean(0)                       # Compute_Xbar (uniform p on the sample)
                W = W + rho * (x - xbar)               # Update_W
                _ = np.abs(x - xbar).mean()            # convergence_diff
                x = run(False, W, xbar, qp)            # solve_loop
                times.append(time.perf_counter() - t0)
            return float(np.median(times[1:]))
        x0 = run(True, W, xbar)                        # Iter0 (builds and caches the models)
        t_it = ph_loop(x0, "ipm")
        # the stock HiGHS QP solver timed separately (its x is only
        # ~4e-3 accurate on these QPs, SURVEY.md 8c, so it is not the headline baseline)
        t_hq = ph_loop(x0, "highs")
    return {"value": 1.0 / (t_it * (S_total / sample)), "unit": "PH iterations/s", "cores": len(slices),
            "kind": "port", "host_cpus": ncpu, "affinity_cpus": aff, "cpu_model": model, **cores_ev,
            "sample": (f"farmer cm={cm}: {sample} of {S_total} scenarios; Iter0 (HiGHS LP) + {iters} PH "
                       f"iterations (QPs by the oracle's dense IPM, one scenario at a time per worker, "
                       f"{len(slices)} spawned workers, {cores_ev['cores_source']}); median per-iteration "
                       f"time of iterations 2..{iters} = {t_it:.3f}s, scaled x{S_total / sample:g} to "
                       f"{S_total} scenarios"),
            "sample_seconds_per_iteration": t_it, "wall_seconds": time.perf_counter() - t_start,
            "stock_highs_qp": {"value": 1.0 / (t_hq * (S_total / sample)), "unit": "PH iterations/s",
                               "cores": len(slices), "sample_seconds_per_iteration": t_hq,
                               "note": ("same loop and sample with the PH QPs solved by the HiGHS 1.8.0 QP "
                                        "solver bundled in scipy (default options; x accurate to ~4e-3 on "
                                        "these QPs, SURVEY.md 8c)")}}


# ---------------------------------------------------------------- roofline
def _latest_profile_file(name, pdir=None):
    dirs = [pdir] if pdir else sorted((d for d in os.listdir(os.path.join(ROOT, "profiles"))
                                       if d.startswith("r")), reverse=True)
    for d in dirs:
        p = os.path.join(ROOT, "profiles", d, name)
        if os.path.exists(p):
            return p
    return None


def ipm_flops_per_iter(b, ipm):
    """Algorithmic fp64 flops of one path-6 iteration of one scenario (one Newton solve,
    DESIGN.md 3.7): A x and A'y (4 nnz), the KKT test (12 n + 6 m), slacks, reciprocals
    and mu (7 per finite bound side), D and E (5 per column / row), the normal-equation
    assembly (k(k+1) + k per column of k entries), the LDL' factorisation and one forward
    + backward solve (counted by the library from the symbolic factor), the right-hand
    side (2 nnz + 14 n + 8 m), dx and dw (4 nnz + 3 n + m), step lengths (8 per side) and
    the update (6 per side + 2 n + 4 m)."""
    n, m, nnz = b.n, b.m, b.nnz
    k = np.bincount(np.asarray(b.col_idx), minlength=n)
    eq = (b.rl[0] == b.ru[0])
    sides = int(np.isfinite(b.lb[0]).sum() + np.isfinite(b.ub[0]).sum()
                + (np.isfinite(b.rl[0]) & ~eq).sum() + (np.isfinite(b.ru[0]) & ~eq).sum())
    return (4 * nnz + 12 * n + 6 * m + 7 * sides + 5 * (n + m) + int((k * (k + 1) + k).sum())
            + ipm["factor_flops"] + ipm["solve_flops"] + 2 * nnz + 14 * n + 8 * m + 4 * nnz + 3 * n + m
            + 8 * sides + 6 * sides + 2 * n + 4 * m)


def roofline_ipm(b, ipm, launches, ws_bytes, tag, pdir):
    """Roofline of the interior-point kernel (path 6): fp64 issue-bound like the other
    register-resident paths (each lane holds its scenario's whole IPM state), achieved =
    ipm_flops_per_iter x IPM iterations per launch / mean HIP-event launch time."""
    launch_ms = float(np.mean([t for t, _ in launches]))
    units = float(np.mean([u for _, u in launches]))
    F = ipm_flops_per_iter(b, ipm)
    tflops = F * units / (launch_ms * 1e-3) / 1e12
    lanes = int(ipm.get("lanes", 1))
    kname = {1: "k_solve_ipm", 2: "k_solve_ipm_ml", 3: "k_solve_ipm_wave", 4: "k_solve_ipm_blk"}.get(
        int(ipm.get("kernel", 0)), "k_solve_ipm" if lanes <= 1 else ("k_solve_ipm_ml" if lanes < 64 else "k_solve_ipm_wave"))
    traffic, src = None, None
    pmc = _latest_profile_file(f"pmc_summary_{tag}.json", pdir)
    if pmc:
        try:
            tr = json.load(open(pmc)).get("solve_traffic_bytes_per_launch", {}).get(kname)
            if tr is not None:
                traffic, src = tr["total_upper"], os.path.relpath(pmc, ROOT)
        except Exception:
            traffic = None
    hbm_gbs = traffic / (launch_ms * 1e-3) / 1e9 if traffic else None
    return {"bound": "fp64", "achieved": tflops, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": tflops / FP64_PEAK_TFLOPS, "traffic": traffic, "traffic_source": src,
            "hbm": {"achieved_GBs": hbm_gbs, "peak_GBs": HBM_PEAK_GBS,
                    "frac": (hbm_gbs / HBM_PEAK_GBS) if hbm_gbs else None,
                    "note": "measured PMC bytes per launch (profiles/) / HIP-event launch time"},
            "cache_resident": ws_bytes < INFINITY_CACHE, "working_set_bytes": ws_bytes,
            "kernel": kname + " (hipRTC, pattern-specialised)", "lanes_per_scenario": int(ipm.get("lanes", 1)),
            "launch_ms": launch_ms, "scenario_iters_per_launch": units, "flops_per_scenario_iter": F,
            "ipm": {k: ipm[k] for k in ("rows", "factor_entries", "scratch_bytes", "compile_s")},
            "note": ("achieved = F x IPM scenario-iterations per launch / mean HIP-event launch time (the "
                     "launch includes the PDHG fallback kernel over the IPM's fallback list); F = "
                     "ipm_flops_per_iter (bench.py)")}


def roofline(b, kinfo, launches, ws_bytes, tag, pdir, ipm=None):
    """Roofline of the solve kernel.

    The register-resident kernels keep each scenario's iterate in VGPRs / LDS for the
    whole solve, so the binding resource is fp64 issue / latency: ``achieved`` =
    algorithmic fp64 flops per launch (F = 4 nnz + 10 n + 6 m per scenario-iteration,
    SURVEY.md 8(d)) / mean launch time, against the 78.6 TF fp64 vector peak.  The HBM
    side is reported from measured PMC bytes (FETCH_SIZE x 2 + WRITE_SIZE, gfx950
    correction of MI355X_MICROARCH.md) of the same kernel, not from the per-iteration
    byte model, which would exceed the 8 TB/s peak for an on-chip iterate."""
    n, m, nnz, nn = b.n, b.m, b.nnz, b.nn
    path = kinfo["path"]
    if path == 2:
        rec = "true" if kinfo.get("rec") == 1 else "false"
        kname = f"k_solve_reg<{kinfo['KC']}, {kinfo['ZC']}, {kinfo['KR']}, {kinfo['ZR']}, {rec}>"
        lanes = kinfo["lanes"]
    elif path == 3:
        kname = f"k_solve_wg<{kinfo['wKC']}, {kinfo['wZC']}, {kinfo['wKR']}, {kinfo['wZR']}, {kinfo['wps']}>"
        lanes = 64 * kinfo["wps"]
    elif path == 4:
        return roofline_stream(b, launches, ws_bytes, tag, pdir, kinfo.get("cluster", 0))
    elif path == 6:
        return roofline_ipm(b, ipm, launches, ws_bytes, tag, pdir)
    else:
        kname, lanes = "k_solve", 1
    launch_ms = float(np.mean([t for t, _ in launches]))
    units = float(np.mean([u for _, u in launches]))
    F = 4 * nnz + 10 * n + 6 * m
    B = 8 * (nnz + 5 * n + 4 * m + 3 * nn)
    tflops = F * units / (launch_ms * 1e-3) / 1e12
    traffic, src = None, None
    pmc = _latest_profile_file(f"pmc_summary_{tag}.json", pdir)
    if pmc:
        try:
            d = json.load(open(pmc))
            tr = d.get("solve_traffic_bytes_per_launch", {}).get("void " + kname)
            if tr is not None:
                traffic = tr["total_upper"]
                src = os.path.relpath(pmc, ROOT)
        except Exception:
            traffic = None
    hbm_gbs = traffic / (launch_ms * 1e-3) / 1e9 if traffic else None
    out = {"bound": "fp64", "achieved": tflops, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
           "frac": tflops / FP64_PEAK_TFLOPS, "traffic": traffic, "traffic_source": src,
           "hbm": {"achieved_GBs": hbm_gbs, "peak_GBs": HBM_PEAK_GBS,
                   "frac": (hbm_gbs / HBM_PEAK_GBS) if hbm_gbs else None,
                   "note": "measured PMC bytes per launch (profiles/) / HIP-event launch time"},
           "cache_resident": ws_bytes < INFINITY_CACHE, "working_set_bytes": ws_bytes,
           "kernel": kname, "lanes_per_scenario": lanes, "launch_ms": launch_ms,
           "scenario_iters_per_launch": units, "flops_per_scenario_iter": F,
           "model_bytes_per_scenario_iter": B,
           "model_GBs_if_streamed": B * units / (launch_ms * 1e-3) / 1e9,
           "note": ("achieved = F x scenario-iterations per launch / mean HIP-event launch time over the "
                    "timed steps; F = 4nnz + 10n + 6m; bound fp64 because the iterate never leaves "
                    "VGPRs/LDS (model_GBs_if_streamed, the SURVEY 8(d) byte model, exceeds HBM peak)")}
    return out


def roofline_stream(b, launches, ws_bytes, tag, pdir, cluster=0):
    """Roofline of the shared-matrix streaming kernel (path 4): HBM-bound.
    Algorithmic bytes per scenario-iteration = 8 (5n + 4m): X, X0 read and X, U written,
    U read once by the row-pass gathers (n each); Y, Y0 read, Y written and Y read once
    by the column-pass gathers (m each).  The shared matrix and the shared column / row
    data are L2 / MALL-resident and not counted.  Measured HBM bytes (PMC) alongside.
    cluster = K >= 2: a batch smaller than the GPU ran in the cluster form (K workgroups
    per scenario, k_solve_stream<1, true>)."""
    n, m, nnz = b.n, b.m, b.nnz
    slots = 1 if os.environ.get("PHGPU_STREAM_SLOTS") == "1" else 2      # phgpu_solve's choice
    kname = f"k_solve_stream<{slots}>" if cluster < 2 else "k_solve_stream<1, true>"
    launch_ms = float(np.mean([t for t, _ in launches]))
    units = float(np.mean([u for _, u in launches]))
    B = 8 * (5 * n + 4 * m)
    gbs = B * units / (launch_ms * 1e-3) / 1e9
    traffic, src = None, None
    pmc = _latest_profile_file(f"pmc_summary_{tag}.json", pdir)
    if pmc:
        try:
            d = json.load(open(pmc))
            if d.get("kernel", "").replace(", false>", ">") == "void " + kname:
                traffic = d["bytes_per_scenario_iter"]["total_upper"] * units
                src = os.path.relpath(pmc, ROOT)
        except Exception:
            traffic = None
    return {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
            "traffic": traffic, "traffic_source": src, "algorithmic_bytes_per_launch": B * units,
            "cache_resident": ws_bytes < INFINITY_CACHE, "working_set_bytes": ws_bytes,
            "kernel": kname, "lanes_per_scenario": 1024 // slots if cluster < 2 else 1024 * cluster,
            "workgroups_per_scenario": cluster if cluster >= 2 else None, "launch_ms": launch_ms,
            "scenario_iters_per_launch": units, "bytes_per_scenario_iter": B,
            "flops_per_scenario_iter": 4 * nnz + 10 * n + 6 * m,
            "note": ("achieved = 8 (5n + 4m) bytes x scenario-iterations per launch / mean HIP-event launch "
                     "time; one workgroup streams one scenario's iterates (X X0 U / Y Y0) per PDHG "
                     "iteration, the shared scaled matrix stays in L2 / MALL")}


def uc_cpu_baseline(S_total, sample, rho_vec):
    """CPU proxy of one PH iteration of config 5 on a bounded sample: per scenario one
    HiGHS dual-simplex solve (scipy) of the W-augmented LP -- the prox term dropped, since
    no sparse QP solver is in this image; a QP solve costs at least as much, so this
    over-states the CPU rate -- with a W from one PH update of the sample, one process
    per core of the process's CPU share."""
    import multiprocessing as mp
    model, ncpu, aff = _host_cpu()
    share, cores_ev = cpu_share()
    P = max(1, min(share, sample))
    ctx = mp.get_context("spawn")
    t0 = time.perf_counter()
    with ctx.Pool(P) as pool:
        res = pool.map(_uc_cpu_worker, [(k, S_total, rho_vec) for k in range(1, sample + 1)])
    wall = time.perf_counter() - t0
    per_scen = float(np.median([r for r in res]))
    t_it = per_scen * S_total / P
    return {"value": 1.0 / t_it, "unit": "PH iterations/s", "cores": P, "kind": "port",
            "host_cpus": ncpu, "affinity_cpus": aff, "cpu_model": model, **cores_ev,
            "sample": (f"uc: {sample} of {S_total} scenarios, one HiGHS dual-simplex LP each (the W-augmented "
                       f"PH subproblem without its prox term: no sparse QP solver here, so this is an upper "
                       f"bound on the CPU rate); median {per_scen:.2f}s per solve, {P} workers -> "
                       f"{S_total} solves per PH iteration"),
            "wall_seconds": wall}


def _uc_cpu_worker(args):
    k, S_total, rho_vec = args
    import warnings
    warnings.simplefilter("ignore")
    from mpisppy_amd.examples import uc
    from oracle import uc as ouc
    b = uc.batch_creator([f"Scenario{k}"], num_scens=S_total)
    x, _, _ = ouc.solve_lp(b, 0)
    on = x[b.nonant_col]
    W = rho_vec * (on - 0.5)                     # one PH update away from x̄ = 0.5
    c = b.c[0].copy()
    c[b.nonant_col] += W
    t = time.perf_counter()
    ouc.solve_lp(b, 0, c=c)
    return time.perf_counter() - t


# ---------------------------------------------------------------- self-check
# The warmup iterations of a fixture workload are exactly the PH iterations the committed
# oracle fixtures pin (tests/golden/make_golden_scale.py, make_golden_aircond.py): the
# bench compares them on every rank before timing, so an N > 1 run (RCCL all-reduces of
# the node buffer and of conv, phbase.py:83-87, 339-343) that computes a wrong x̄, W or
# conv says so in its JSON line and exits non-zero.  Tolerances are north_star's.
CHECK_REL = 1e-5
CHECK_ABS = 1e-5
CHECK_FIXTURES = {("farmer", 65536, 1): ("farmer_scale.json", "farmer65536_cm1"),
                  ("farmer", 1024, 10): ("farmer_scale.json", "farmer1024_cm10"),
                  ("aircond", 65536, None): ("aircond_scale.json", None)}


def load_check_fixture(model, scens, cm, bf=None):
    """The oracle fixture of this workload, or None (the bench then runs unchecked)."""
    key = (model, scens, cm if model == "farmer" else None)
    if key not in CHECK_FIXTURES:
        return None
    fname, sub = CHECK_FIXTURES[key]
    path = os.path.join(ROOT, "tests", "golden", fname)
    if not os.path.exists(path):
        return None
    g = json.load(open(path))
    g = g[sub] if sub else g
    if model == "aircond" and (bf is None or list(g["branching_factors"]) != list(bf)):
        return None
    return g


def parity_checks(g, obs, rho):
    """Compare one rank's view of the warmup with the oracle fixture ``g``.

    ``obs``: trivial_bound; conv (the conv of each warmup PH iteration); xbar_last (the x̄
    of the last warmup iteration, farmer: the ROOT vector, aircond: {node: vector});
    w_rows ({global scenario index: W row} for this rank's scenarios); eobj (E[obj] after
    the warmup); warmup.  Returns a dict of booleans and the largest errors.  A check the
    warmup length does not reach (fewer iterations than the fixture pins) is None."""
    k = int(obs["warmup"])
    pinned = int(g["ph_iters"])
    out = {"fixture_rho_ok": abs(float(rho) - float(g["rho"])) == 0.0}
    tb, tb_ref = float(obs["trivial_bound"]), float(g["trivial_bound"])
    out["trivial_bound_err_rel"] = abs(tb - tb_ref) / abs(tb_ref)
    out["trivial_bound_ok"] = bool(out["trivial_bound_err_rel"] <= CHECK_REL)
    n = min(k, pinned)
    conv = np.asarray(obs["conv"][:n], dtype=float)
    if n and len(conv) == n:
        err = float(np.abs(conv - np.asarray(g["conv"][:n])).max())
        out["conv_err"], out["conv_ok"] = err, bool(err <= CHECK_ABS)
    else:
        out["conv_err"], out["conv_ok"] = None, (None if n == 0 else False)
    if k == pinned:
        if isinstance(obs["xbar_last"], dict):            # multistage: every node of the fixture
            got = np.array([np.asarray(obs["xbar_last"][nd])[:2] for nd in g["node_names"]])
            ref = np.asarray(g["xbar"][pinned - 1])
        else:
            ref = np.asarray(g["xbar"][pinned - 1])
            got = np.asarray(obs["xbar_last"])[:len(ref)]
        err = float(np.abs(got - ref).max())
        out["xbar_err"], out["xbar_ok"] = err, bool(err <= CHECK_ABS)
        smp = list(g["sample"])
        pos = {s: j for j, s in enumerate(smp)}
        mine = [s for s in obs["w_rows"] if s in pos]
        if mine:
            got = np.array([np.asarray(obs["w_rows"][s]) for s in mine])
            ref = np.array([g["W"][pos[s]] for s in mine])[:, :got.shape[1]]
            err = float(np.abs(got[:, :ref.shape[1]] - ref).max())
            out["W_err"], out["W_ok"], out["W_rows"] = err, bool(err <= CHECK_ABS), len(mine)
        else:
            out["W_err"], out["W_ok"], out["W_rows"] = 0.0, True, 0
        err = abs(float(obs["eobj"]) - float(g["Eobj"])) / abs(float(g["Eobj"]))
        out["eobj_err_rel"], out["eobj_ok"] = err, bool(err <= CHECK_REL)
    else:
        for key in ("xbar", "W", "eobj"):
            out[key + "_ok"] = None
    return out


def combine_checks(per_rank, world_size, backend):
    """Fold the ranks' parity_checks dicts into the JSON line's ``checks``: every boolean
    must hold on every rank (None = not reached by this warmup), errors are maxima, and
    the ranks must agree on conv bit for bit (they read the same all-reduced value)."""
    keys = [k for k in per_rank[0] if k.endswith("_ok")]
    out = {"world_size": world_size, "backend": backend, "ranks_seen": len(per_rank)}
    for key in keys:
        vals = [r[key] for r in per_rank]
        out[key] = None if all(v is None for v in vals) else all(bool(v) for v in vals if v is not None) \
            and not any(v is None for v in vals)
    for key in per_rank[0]:
        if key.endswith("_err") or key.endswith("_err_rel"):
            vals = [r[key] for r in per_rank if r[key] is not None]
            out[key] = max(vals) if vals else None
    out["W_rows_checked"] = sum(int(r.get("W_rows", 0) or 0) for r in per_rank)
    convs = [tuple(r.get("conv_seen", ())) for r in per_rank]
    out["ranks_agree_on_conv"] = all(c == convs[0] for c in convs)
    out["ranks_seen_ok"] = out["ranks_seen"] == world_size
    verdict = [v for k, v in out.items() if k.endswith("_ok") and k != "fixture_rho_ok"]
    out["all_ok"] = bool(all(v is not False for v in verdict) and out["ranks_agree_on_conv"])
    return out


# ---------------------------------------------------------------- GPU run
def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(a))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    if a.model == "aircond":
        a.bf = [int(v) for v in a.bf.split(",")]
        a.scens = int(np.prod(a.bf))
    if a.model == "uc" and a.scens == 65536:
        a.scens = 1000
    if a.eps is None:
        a.eps = 1e-6 if a.model == "uc" else 1e-9
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline and a.model == "farmer":
        sample = a.cpu_sample or min(a.scens, 4096 if a.cm == 1 else 256)
        cpu = cpu_baseline(a.scens, a.cm, a.rho, sample)
        log("cpu baseline:", json.dumps(cpu))

    import torch
    import torch.distributed as dist
    ndev = torch.cuda.device_count()
    backend = a.backend
    if world > 1:
        if backend == "auto":
            backend = os.environ.get("PHGPU_DIST_BACKEND", "nccl" if ndev >= world else "")
            if not backend:
                raise SystemExit(f"{world} ranks but {ndev} visible GPU(s): use --backend gloo to "
                                 f"rehearse with ranks sharing a GPU")
        if backend == "nccl" and ndev < world:
            raise SystemExit(f"RCCL needs one GPU per rank ({world} ranks, {ndev} GPUs)")
    dev_index = local_rank % max(1, ndev)
    torch.cuda.set_device(dev_index)
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
        else:
            dist.init_process_group("gloo")
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.examples import farmer
    from mpisppy_amd.comm import Comm

    comm = Comm()
    opts = {"solver_name": "mi355x_pdhg", "PHIterLimit": a.warmup, "defaultPHrho": a.rho,
            "convthresh": -1.0, "verbose": False, "display_progress": False, "toc": False,
            "device": f"cuda:{dev_index}", "fused_ph_loop": a.fused_loop,
            "iterk_solver_options": {"eps_rel": a.eps}}
    if a.model == "farmer" and not a.default_solver_options:
        # the example's recommended PH-solve options (examples/farmer.py PDHG_ITERK_OPTIONS)
        opts["iterk_solver_options"].update(farmer.PDHG_ITERK_OPTIONS)
    if a.model == "aircond" and not a.default_solver_options:
        from mpisppy_amd.examples import aircond as _air
        opts["ipm_tuning"] = dict(_air.IPM_TUNING)    # the model's interior-point constants
    if a.model == "uc" and not a.default_solver_options:
        from mpisppy_amd.examples import uc as _uc
        opts["iterk_solver_options"].update(_uc.PDHG_ITERK_OPTIONS)
    for kv in a.solver_opt:
        k, v = kv.split("=", 1)
        opts["iterk_solver_options"][k] = float(v) if any(ch in v for ch in ".e") else int(v)
    t_setup = time.perf_counter()
    if a.model == "farmer":
        names = farmer.scenario_names_creator(a.scens)
        opts["batch_creator"] = farmer.batch_creator
        ph = PH(opts, names, farmer.scenario_creator, mpicomm=comm,
                scenario_creator_kwargs={"crops_multiplier": a.cm, "num_scens": a.scens})
        workload = {(65536, 1): "farmer PH (config 3)",
                    (1024, 10): "farmer PH (config 2)"}.get((a.scens, a.cm), f"farmer PH, cm={a.cm}")
    elif a.model == "uc":
        # config 5: UC LP relaxation (examples/uc.py restating ReferenceModel_OK.py), the
        # wind scenarios of 1000scenarios_wind; rho = uc_funcs.py:99-116 (0.1 x midpoint cost)
        from mpisppy_amd.examples import uc
        names = uc.scenario_names_creator(a.scens)
        opts["batch_creator"] = uc.batch_creator
        opts["iter0_solver_options"] = {"eps_rel": a.eps}
        rho_vec = uc.rho_vector(uc.scenario_creator(names[0], num_scens=a.scens))
        opts["rho_array"] = rho_vec
        ph = PH(opts, names, uc.scenario_creator, mpicomm=comm, scenario_creator_kwargs={"num_scens": a.scens})
        workload = "UC LP relaxation PH (config 5)"
        if rank == 0 and world == 1 and not a.no_cpu_baseline:
            cpu = uc_cpu_baseline(a.scens, a.cpu_sample or 16, rho_vec)
            log("cpu baseline:", json.dumps(cpu))
    else:
        # config 4: aircond multistage (aircond.py:37-330), one scenario per leaf of the bf
        # tree; per-node x̄ over all non-leaf nodes
        from mpisppy_amd.examples import aircond
        from mpisppy_amd.sputils import create_nodenames_from_branching_factors
        names = aircond.scenario_names_creator(a.scens)
        opts["batch_creator"] = aircond.batch_creator
        ph = PH(opts, names, aircond.scenario_creator, mpicomm=comm,
                scenario_creator_kwargs={"branching_factors": a.bf, **AIRCOND_KW},
                all_nodenames=create_nodenames_from_branching_factors(a.bf))
        workload = f"aircond multistage PH (config 4), bf {'x'.join(map(str, a.bf))}"
    log(f"[bench] model built ({time.perf_counter() - t_setup:.1f} s)")
    with contextlib.redirect_stdout(sys.stderr):
        ph.PH_Prep()
        ph.engine.overlap_conv = not a.no_conv_overlap
        log(f"[bench] PH_Prep done ({time.perf_counter() - t_setup:.1f} s)")
        trivial_bound = ph.Iter0()
        log(f"[bench] Iter0 done ({time.perf_counter() - t_setup:.1f} s)")
        e = ph.engine
        b = ph.batch
        # Iter0's certification, summed over ranks: scenarios whose LP / QP stopped at the
        # PDHG iteration cap (their x enters x̄ unconverged, the trivial bound is not a bound)
        iter0_bad = torch.tensor([e.count_not_optimal()], dtype=torch.float64, device=e.device)
        comm.allreduce_sum_(iter0_bad)
        iter0_bad = int(iter0_bad.item())
        iter0_relaxed = torch.tensor([getattr(ph, "iter0_relaxed", 0)], dtype=torch.float64, device=e.device)
        comm.allreduce_sum_(iter0_relaxed)
        iter0_relaxed = int(iter0_relaxed.item())
        # the PMC summaries under profiles/ are per GPU instance: keyed by the scenarios
        # one rank holds (its kernel instance / lane count depend on it)
        tag = {"farmer": f"farmer{b.S}_cm{a.cm}", "uc": f"uc{b.S}", "aircond": f"aircond{b.S}"}[a.model]
        fixture = None
        if a.check != "off" and a.warmup > 0:
            fixture = load_check_fixture(a.model, a.scens, a.cm, a.bf if a.model == "aircond" else None)
            if fixture is not None and a.check == "auto" and float(fixture["rho"]) != a.rho:
                fixture = None
        conv_seen = []
        if fixture is not None:
            # keep each warmup iteration's conv (the engine's readback, both loop variants)
            _wait, _diff = e.convergence_wait, e.convergence_diff
            e.convergence_wait = lambda: conv_seen.append(_wait()) or conv_seen[-1]
            e.convergence_diff = lambda: conv_seen.append(_diff()) or conv_seen[-1]
        nf0 = len(getattr(ph, "fused_loops", []))
        ph.iterk_loop()                                # W warmup iterations (untimed)
        torch.cuda.synchronize()
        if len(getattr(ph, "fused_loops", [])) > nf0:
            conv_seen = list(ph.fused_loops[-1]["conv"])   # the fused loop's conv of every step
        checks = None
        if fixture is not None:
            del e.convergence_wait, e.convergence_diff     # back to the class methods
            nx = ph.xbar_by_node()
            first = names.index(ph.local_scenario_names[0])      # contiguous slices (sputils.py:803-810)
            Wl = ph.W_array()
            obs = {"trivial_bound": trivial_bound, "conv": conv_seen, "warmup": a.warmup,
                   "xbar_last": (nx["ROOT"] if a.model == "farmer" else nx),
                   "w_rows": {first + i: Wl[i] for i in range(Wl.shape[0])},
                   "eobj": ph.Eobjective()}
            mine = parity_checks(fixture, obs, a.rho)
            mine["conv_seen"] = [float(v) for v in conv_seen]
            checks = combine_checks(comm.allgather_object(mine),
                                    dist.get_world_size() if world > 1 else 1,
                                    backend if world > 1 else "none (one rank)")
            checks["fixture"] = " / ".join(x for x in CHECK_FIXTURES[(a.model, a.scens, a.cm if a.model == "farmer"
                                                                     else None)] if x)
            checks["tolerance"] = {"rel": CHECK_REL, "abs": CHECK_ABS}
            log("[bench] checks:", json.dumps(checks))
            # the readbacks above flushed the deferred step: one more untimed iteration puts the
            # loop back in the state the warmup leaves it in (speculative solve, folded step)
            ph.options["PHIterLimit"] = 1
            ph.iterk_loop()
            torch.cuda.synchronize()
        log(f"[bench] warmup done ({time.perf_counter() - t_setup:.1f} s)")
        t_setup = time.perf_counter() - t_setup
        # HIP events around one solve launch in INSTRUMENT_EVERY (each event is a marker
        # packet that idles the GPU ~5.6 us; the other steps run exactly as the product loop)
        e.instrument(a.steps, every=INSTRUMENT_EVERY)
        ph.options["PHIterLimit"] = a.steps
        comm.Barrier()
        torch.cuda.synchronize()
        nf0 = len(getattr(ph, "fused_loops", []))
        t0 = time.perf_counter()
        ph.iterk_loop()                                # the product loop, K iterations
        torch.cuda.synchronize()
        comm.Barrier()
        elapsed = time.perf_counter() - t0
    fused = getattr(ph, "fused_loops", [])[nf0:]
    if fused:
        # the fused PH loop (one launch for the K iterations): its HIP-event
        # time per PH iteration and its IPM iterations per PH iteration
        r = fused[-1]
        launches = [(r["ms"] / max(1, r["steps"]), r["ipm_iters"] / max(1, r["steps"]))]
        n_ins = 1
        bad_timed = torch.tensor([e.count_not_optimal()], dtype=torch.float64, device=e.device)
    else:
        launches = e.instrumented()
        n_ins = (a.steps + INSTRUMENT_EVERY - 1) // INSTRUMENT_EVERY
        assert len(launches) == n_ins, (len(launches), n_ins)
        bad_timed = torch.tensor(e.instrumented_not_optimal(), dtype=torch.float64, device=e.device)
    comm.allreduce_sum_(bad_timed)
    ar_ms = torch.tensor([e.instrumented_allreduce_ms("critical") / a.steps,
                          e.instrumented_allreduce_ms("overlapped") / a.steps], dtype=torch.float64, device=e.device)
    comm.allreduce_max_(ar_ms)
    it_host = e.iters.cpu().numpy()
    # per-iteration wall times of the timed loop (PHBase.iterk_loop's iter_times); BASELINE.md
    # section 2 takes the median over iterations 2..K, max over ranks
    its = ph.iter_times[-a.steps:]
    med = float(np.median(its[1:] if len(its) > 1 else its))
    t = torch.tensor([elapsed, med], dtype=torch.float64, device=e.device)
    comm.allreduce_max_(t)
    elapsed, med = float(t[0].item()), float(t[1].item())
    n_bad = torch.tensor([e.count_not_optimal()], dtype=torch.float64, device=e.device)
    comm.allreduce_sum_(n_bad)
    kinfo = e.kernel_info()
    if kinfo["path"] == 4:
        kinfo["cluster"] = e.stream_info()["cluster"]
    ws = e.workspace_bytes() + 8 * (b.S * (b.n + b.m + 3 * max(b.nn, 1) + 4))
    ipm_diag = e.ipm_info()
    rl = roofline(b, kinfo, launches, ws, tag, a.profile_dir, ipm=ipm_diag)
    # value: K timed PH iterations / the synchronised wall time of the whole timed region
    # (barrier + synchronize on both sides, max over ranks) -- every GPU iteration counted,
    # including the speculative solve's overlap; the median of the host's per-iteration
    # times (BASELINE.md section 2's definition) is kept beside it
    ph_its = a.steps / elapsed
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": ph_its,
            "unit": "PH iterations/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": 1e3 * elapsed / a.steps,
            "ms_per_step_definition": "synchronised wall time of the K timed PH iterations / K (barrier + "
                                      "device synchronize on both sides), max over ranks",
            "ms_per_step_median": 1e3 * med,
            "iter_ms": [round(1e3 * v, 4) for v in its],
            "value_from_median": 1.0 / med,
            "checks": checks,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": ("reference data (paperruns/larger_uc RootNode.dat + 1000scenarios_wind/Node*.dat)"
                     if a.model == "uc" else
                     f"synthetic ({a.model} scenario generator, seeded as "
                     f"{'farmer.py:52-60' if a.model == 'farmer' else 'aircond.py:37-67'})"),
            "config": {"workload": workload, "scenarios": a.scens,
                       "crops_multiplier": a.cm if a.model == "farmer" else None,
                       "tree_nodes": len(b.node_names),
                       "rho": a.rho, "eps_rel": a.eps,
                       "iterk_solver_options": {k: v for k, v in opts["iterk_solver_options"].items()
                                                if k != "eps_rel"},
                       "ipm_tuning": opts.get("ipm_tuning"),
                       "scenarios_per_gpu": b.S,
                       "n": b.n, "m": b.m, "nnz": b.nnz,
                       "conv_allreduce": (("launch stream, ahead of the next solve" if a.no_conv_overlap
                                           else "side stream, under the next solve") if world > 1 else None),
                       "parallelism": (f"scenario-sharded x{world}" +
                                       (f" ({'RCCL' if backend == 'nccl' else 'gloo, ranks sharing a GPU'}"
                                        f" x̄ all-reduce)" if world > 1 else ""))},
            "solves_per_sec": ph_its * a.scens,
            "solver": "ipm" if kinfo["path"] == 6 else "pdhg",
            "solver_iters_per_ph_iter": {"max": int(it_host.max()), "mean": float(it_host.mean())},
            "time_split_ms": {"solve_launch": rl["launch_ms"],
                              # the x̄ all-reduce, ahead of the next solve on the launch stream
                              "allreduce": float(ar_ms[0].item()),
                              # the conv all-reduce, on a side stream under the next solve
                              "allreduce_overlapped": float(ar_ms[1].item()),
                              "rest_of_step": 1e3 * elapsed / a.steps - rl["launch_ms"] - float(ar_ms[0].item())},
            "fused_ph_loop": ({"launches": len(fused), "ph_steps": fused[-1]["steps"], "end": fused[-1]["end"],
                               "loop_ms": fused[-1]["ms"], "ipm_iters": fused[-1]["ipm_iters"],
                               "note": "PHBase.iterk_loop's K iterations in one cooperative launch "
                                       "(phgpu_ph_loop); launch_ms = loop ms / K"} if fused else None),
            "instrumented_solves": {"count": n_ins, "every": INSTRUMENT_EVERY,
                                    "note": "HIP events around every INSTRUMENT_EVERY-th timed solve launch "
                                            "(roofline launch_ms); the other timed steps carry no markers"},
            "timed_region": "PHBase.iterk_loop (x̄, W, conv readback, solve_loop with gripe)",
            # every timed solve: scenarios not OPTIMAL (summed over ranks), and the last one
            "not_optimal_per_timed_solve_max": int(bad_timed.max().item()),
            "all_optimal": bool(n_bad.item() == 0 and bad_timed.max().item() == 0),
            # the subtree kernel (config 2): scenarios of the last timed solve found still
            # jammed after their re-centrings -- handed to the PDHG fallback, not reported
            # OPTIMAL -- and its re-centrings
            "path6_last_solve_jam_handovers": int(ipm_diag.get("jam_handovers", 0)),
            "path6_last_solve_recentrings": int(ipm_diag.get("recentrings", 0)),
            "iter0_not_optimal": iter0_bad,
            "iter0_relaxed_resolve": iter0_relaxed,
            # path 4 (config 5): warm continuation solves of Iter0 LPs left at the PDHG cap
            # (PHBase._iter0_continue: the stragglers over the whole GPU), before the bound
            "iter0_continuation_solves": int(getattr(ph, "iter0_continued", 0)),
            # every Iter0 solve met the KKT tolerance: the trivial bound is the Lagrangian dual
            # bound with projected reduced costs (PDLP convention), accurate to that
            # tolerance -- not an exact certificate; an Iter0 solve at the
            # iteration cap gives no bound at all
            "trivial_bound_kkt_accurate": iter0_bad == 0,
            "trivial_bound": trivial_bound if iter0_bad == 0 else None,
            "trivial_bound_unconverged": None if iter0_bad == 0 else trivial_bound,
            "setup_s": t_setup,
            "roofline": rl,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    # release the handle while the HIP runtime (and a profiler's tool) is still up, not in
    # PHEngine.__del__ at interpreter teardown (profiles/r04/ac/uc_1.log: SIGSEGV there)
    e.close()
    if world > 1:
        dist.destroy_process_group()
    if checks is not None and not checks["all_ok"]:
        log("[bench] PARITY CHECK FAILED:", json.dumps(checks))
        sys.exit(3)


if __name__ == "__main__":
    main()
