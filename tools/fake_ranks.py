"""The N > 1 step path on one GPU without communication (TOOL ONLY): PH on rank 0's share
of farmer 65,536 with a loopback communicator that reports ``size`` ranks and whose
all-reduce multiplies by ``size`` (as if every rank held the same scenarios: x̄, W and conv
stay those of a real run on this share), against the one-rank run on the same share (the
folded step).  The difference is the multi-rank path's own cost on the GPU and the host
(the reduce / update launches, the side-stream conv copy and its event, the Python
wrappers), i.e. what an 8-GPU run pays before RCCL's latency.

    python tools/fake_ranks.py [size = 8] [steps = 40]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy-1_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402


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


def run(size, steps, comm):
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.examples import farmer
    S = 65536
    names = farmer.scenario_names_creator(S)
    if comm is None:
        names = names[:S // size]
    opts = {"solver_name": "mi355x_pdhg", "PHIterLimit": 5, "defaultPHrho": 1.0, "convthresh": -1.0,
            "verbose": False, "display_progress": False, "toc": False, "device": "cuda:0",
            "batch_creator": farmer.batch_creator, "fused_ph_loop": False, "iterk_solver_options": {"beta_sufficient": 0.6},
            "iter0_solver_options": {"eps_rel": 1e-9}}
    # (the one-rank run on the share: probabilities 1/share, the same scenario data)
    kw = {"crops_multiplier": 1, "num_scens": S if comm is not None else S // size}
    ph = PH(opts, names, farmer.scenario_creator, scenario_creator_kwargs=kw, mpicomm=comm)
    ph.PH_Prep()
    ph.Iter0()
    ph.iterk_loop()
    torch.cuda.synchronize()
    ph.options["PHIterLimit"] = steps
    prof = None
    if os.environ.get("FAKE_PROF") and comm is not None:  # (cProfile of the timed loop)
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    t0 = time.perf_counter()
    ph.iterk_loop()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if prof is not None:
        import pstats
        prof.disable()
        pstats.Stats(prof).sort_stats("tottime").print_stats(30)
    its = ph.iter_times[-steps:]
    e = ph.engine
    out = {"local_scenarios": e.S, "median_ms": 1e3 * float(np.median(its[1:])), "mean_ms": 1e3 * el / steps,
           "calls": dict(e.calls), "path": e.kernel_info()["path"], "lanes": e.ipm_info().get("lanes")}
    e.close()
    return out


def main():
    size = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    if len(sys.argv) > 3 and sys.argv[3] == "loopback":  # (under a profiler: that run alone)
        print(f"loopback {size} ranks:", run(size, steps, LoopbackComm(size)), flush=True)
        return
    print("one rank (folded step):", run(size, steps, None), flush=True)
    print(f"loopback {size} ranks (reduce / all-reduce / update, side-stream conv):",
          run(size, steps, LoopbackComm(size)), flush=True)
    print("one rank again:", run(size, steps, None), flush=True)


if __name__ == "__main__":
    main()
