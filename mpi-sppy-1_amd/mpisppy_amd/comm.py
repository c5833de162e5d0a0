"""Rank communicator over torch.distributed (RCCL on MI355X, gloo on CPU).

Stands in for the mpi4py communicator of mpisppy/MPI.py:3-82 on the hot path: the
per-node ``Allreduce`` of _Compute_Xbar (phbase.py:83-87) becomes ONE all-reduce of a
node-indexed fp64 buffer over all ranks (ranks that do not own a node contribute
zeros, so the sum per node equals the node-communicator sum of spbase.py:349-359);
the ROOT-comm Allreduce of convergence_diff (phbase.py:341) and the Ebound /
Eobjective / E1 / feas_prob sums (spopt.py:341, 386, 404, 435) are all-reduces of
tiny buffers.  With one rank every call is a no-op.
"""
import os

import torch
import torch.distributed as dist


class Comm:
    def __init__(self, group=None):
        self.group = group
        if dist.is_available() and dist.is_initialized():
            self.rank = dist.get_rank(group)
            self.size = dist.get_world_size(group)
        else:
            self.rank = 0
            self.size = 1

    def Get_rank(self):
        return self.rank

    def Get_size(self):
        return self.size

    def allreduce_sum_(self, t):
        """In-place SUM all-reduce of a tensor (device tensor with RCCL)."""
        if self.size > 1:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t

    def rccl_plan(self):
        """(nranks, rank) of the RCCL communicator the engine's library opens over these ranks
        for the PH step's sums (include/phgpu.h phgpu_comm_init), or None to keep them on
        torch.distributed: the world group on the nccl backend only (PHGPU_NATIVE_RCCL=0
        turns it off)."""
        if (self.size > 1 and self.group is None and dist.is_initialized() and dist.get_backend() == "nccl"
                and os.environ.get("PHGPU_NATIVE_RCCL", "1") != "0"):
            return self.size, self.rank
        return None

    def after_native_(self, t):
        """Hook after a library-issued sum (a loopback communicator scales here)."""
        return t

    def allreduce_max_(self, t):
        if self.size > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return t

    def Barrier(self):
        if self.size > 1:
            dist.barrier(group=self.group)

    def bcast_object(self, obj, root=0):
        if self.size == 1:
            return obj
        lst = [obj]
        dist.broadcast_object_list(lst, src=root, group=self.group)
        return lst[0]

    def allgather_object(self, obj):
        if self.size == 1:
            return [obj]
        out = [None] * self.size
        dist.all_gather_object(out, obj, group=self.group)
        return out

    def gather_object(self, obj, root=0):
        if self.size == 1:
            return [obj]
        out = [None] * self.size
        dist.all_gather_object(out, obj, group=self.group)
        return out if self.rank == root else None


def world_comm():
    return Comm(None)
