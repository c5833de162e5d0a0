"""SPCommunicator: base of hub and spokes (mirrors mpisppy/cylinders/spcommunicator.py:18-120).

The reference gives every cylinder its own MPI ranks and moves W / nonants / bounds
through one-sided MPI windows carrying a trailing write id (spcommunicator.py:93-120,
hub.py:345-450, spoke.py:34-118).  Here every cylinder is co-located on every rank's
GPU (one process per GPU): a window is a device buffer owned by the writer plus a
host-side write id, and the hub drives the spokes cooperatively from its ``sync``.
The rank communicator of each cylinder is the same ``Comm`` (torch.distributed), so a
spoke's reductions go over the same ranks that hold its scenario slice.
"""


class SPCommunicator:
    def __init__(self, spbase_object, fullcomm=None, strata_comm=None, cylinder_comm=None, options=None):
        self.opt = spbase_object
        self.fullcomm = fullcomm if fullcomm is not None else spbase_object.mpicomm
        self.strata_comm = strata_comm if strata_comm is not None else self.fullcomm
        self.cylinder_comm = cylinder_comm if cylinder_comm is not None else spbase_object.mpicomm
        self.global_rank = self.fullcomm.Get_rank()
        self.cylinder_rank = self.cylinder_comm.Get_rank()
        self.n_proc = self.cylinder_comm.Get_size()
        self.options = dict(options) if options is not None else {}
        self.opt.spcomm = self

    def main(self):
        raise NotImplementedError

    def sync(self):
        pass

    def is_converged(self):
        return False

    def finalize(self):
        pass

    def hub_finalize(self):
        pass

    def free_windows(self):
        pass
