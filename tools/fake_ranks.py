"""The N > 1 step path on one GPU without communication (TOOL ONLY): PH on rank 0's share
of farmer 65,536 with a loopback communicator that reports ``size`` ranks and whose
all-reduce multiplies by ``size`` (as if every rank held the same scenarios: x̄, W and conv
stay those of a real run on this share), against the one-rank run on the same share (the
folded step).  The difference is the multi-rank path's own cost on the GPU and the host
(the reduce / update launches, the side-stream conv copy and its event, the Python
wrappers), i.e. what an 8-GPU run pays before RCCL's latency.

    python tools/fake_ranks.py [size = 8] [steps = 40] [loopback | rccl]

``rccl``: the same loopback with a real RCCL all-reduce (a one-rank nccl group) underneath.
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


class RcclLoopbackComm(LoopbackComm):
    """The loopback with a real RCCL all-reduce underneath (a one-rank nccl process group on
    the same GPU): the engine's multi-rank path then issues RCCL collectives on its launch
    and side streams exactly as an N-GPU run does; the sum is then scaled by ``size``."""

    def __init__(self, size):
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if not dist.is_initialized():
            dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        self.dist = dist
        super().__init__(size)

    def allreduce_sum_(self, t):
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        t.mul_(self.size)
        return t

    def rccl_plan(self):
        # the library's own communicator over the one real rank (PHGPU_NATIVE_RCCL=0: torch)
        return (1, 0) if os.environ.get("PHGPU_NATIVE_RCCL", "1") != "0" else None

    def after_native_(self, t):
        t.mul_(self.size)
        return t


def run(size, steps, comm, state=False):
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
           "calls": dict(e.calls), "path": e.kernel_info()["path"], "lanes": e.ipm_info().get("lanes"),
           "native_rccl": bool(getattr(e, "_native", False))}
    if state:  # (tests: the PH state after the loop)
        out["conv"] = float(ph.conv)
        out["W"] = e.host("W").tolist()
        out["xbar"] = e.host("node_buf").tolist()
    e.close()
    return out


def main():
    size = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    if len(sys.argv) > 3 and sys.argv[3] == "rccl":  # RCCL collectives under the loopback
        print(f"rccl (library) loopback {size} ranks:", run(size, steps, RcclLoopbackComm(size)), flush=True)
        os.environ["PHGPU_NATIVE_RCCL"] = "0"
        print(f"rccl (torch.distributed) loopback {size} ranks:", run(size, steps, RcclLoopbackComm(size)), flush=True)
        os.environ.pop("PHGPU_NATIVE_RCCL")
        print(f"loopback {size} ranks:", run(size, steps, LoopbackComm(size)), flush=True)
        return
    if len(sys.argv) > 3 and sys.argv[3] == "rccl-state":  # (tests/test_gpu_native_rccl.py)
        import json
        out = {}
        for mode in ("library", "torch"):
            if mode == "torch":
                os.environ["PHGPU_NATIVE_RCCL"] = "0"
            out[mode] = run(size, steps, RcclLoopbackComm(size), state=True)
        print("STATE " + json.dumps(out), flush=True)
        return
    if len(sys.argv) > 3 and sys.argv[3] == "loopback":  # (under a profiler: that run alone)
        print(f"loopback {size} ranks:", run(size, steps, LoopbackComm(size)), flush=True)
        return
    print("one rank (folded step):", run(size, steps, None), flush=True)
    print(f"loopback {size} ranks (reduce / all-reduce / update, side-stream conv):",
          run(size, steps, LoopbackComm(size)), flush=True)
    print("one rank again:", run(size, steps, None), flush=True)


if __name__ == "__main__":
    main()
