"""SPCommunicator: base of hub and spokes (mirrors mpisppy/cylinders/spcommunicator.py:18-120).

The reference gives every cylinder its own MPI ranks and moves W / nonants / bounds
through one-sided MPI windows carrying a trailing write id (spcommunicator.py:93-120,
hub.py:345-450, spoke.py:34-118).  WheelSpinner places the cylinders in one of two ways
(spin_the_wheel.py):

  * "ranks" (the reference's placement): the world splits into n_spokes + 1 cylinders of
    P ranks each (``fullcomm`` / ``strata_comm`` / ``cylinder_comm`` as in
    spin_the_wheel.py:219-237); windows are keys of the job's rendezvous store carrying
    'ci'-ordered W or nonants plus the three trailing slots [outer bound, inner bound,
    write id] (cylinders/transport.py);
  * "colocated": every cylinder on every rank's GPU, a window a device buffer plus a
    host-side write id, the hub driving the spokes from its ``sync``; each cylinder's
    rank communicator is then the same ``Comm``.

This base class holds the communicators and the hooks the hub and spokes override.
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
