"""WheelSpinner: hub-and-spoke driver (mirrors mpisppy/spin_the_wheel.py:9-160).

Same dict contract as the reference: ``hub_dict`` with hub_class / hub_kwargs /
opt_class / opt_kwargs and one dict per spoke with spoke_class / spoke_kwargs /
opt_class / opt_kwargs; ``WheelSpinner(hub_dict, list_of_spoke_dict).spin()`` and then
``BestInnerBound`` / ``BestOuterBound`` / ``write_first_stage_solution``.

Placement differs: the reference splits the MPI world into one strata per
cylinder (spin_the_wheel.py:176-206), so each cylinder owns its own ranks.  Here every
rank (one per GPU) holds its scenario slice for EVERY cylinder -- hub and spoke engines
share the GPU and the rank communicator -- and the hub runs the spokes' loop bodies
right after each sync.  No bound is computed from a stale W, and no GPU idles while
another cylinder works.
"""
import csv

from .comm import Comm
from . import global_toc


class WheelSpinner:
    def __init__(self, hub_dict, list_of_spoke_dict):
        self.hub_dict = hub_dict
        self.list_of_spoke_dict = list(list_of_spoke_dict)
        self._ran = False

    def spin(self, comm_world=None):
        return self.run(comm_world=comm_world)

    def run(self, comm_world=None):
        if self._ran:
            raise RuntimeError("WheelSpinner can only be run once")
        hub_dict = self.hub_dict
        if "hub_class" not in hub_dict:
            raise RuntimeError("The hub_dict must contain a 'hub_class' key specifying the hub class to use")
        if "opt_class" not in hub_dict:
            raise RuntimeError("The hub_dict must contain an 'opt_class' key specifying the SPBase class "
                               "to use (e.g. PHBase, etc.)")
        hub_dict.setdefault("hub_kwargs", dict())
        hub_dict.setdefault("opt_kwargs", dict())
        for spoke_dict in self.list_of_spoke_dict:
            if "spoke_class" not in spoke_dict:
                raise RuntimeError("Each spoke_dict must contain a 'spoke_class' key specifying the spoke class to use")
            if "opt_class" not in spoke_dict:
                raise RuntimeError("Each spoke_dict must contain an 'opt_class' key specifying the SPBase class "
                                   "to use (e.g. PHBase, etc.)")
            spoke_dict.setdefault("spoke_kwargs", dict())
            spoke_dict.setdefault("opt_kwargs", dict())

        comm = comm_world if comm_world is not None else Comm()
        spokes = []
        for spoke_dict in self.list_of_spoke_dict:
            kw = dict(spoke_dict["opt_kwargs"])
            kw["mpicomm"] = comm
            sopt = spoke_dict["opt_class"](**kw)
            spokes.append(spoke_dict["spoke_class"](sopt, comm, comm, comm, **spoke_dict["spoke_kwargs"]))
        kw = dict(hub_dict["opt_kwargs"])
        kw["mpicomm"] = comm
        hopt = hub_dict["opt_class"](**kw)
        hub = hub_dict["hub_class"](hopt, comm, comm, comm, spokes, **hub_dict["hub_kwargs"])
        hub.setup_hub()
        global_toc("Starting spcomm.main()", comm.Get_rank() == 0 and hopt.options.get("toc", True))
        hub.main()
        hub.send_terminate()
        hub.finalize()
        for spoke in spokes:
            spoke.finalize()
        comm.Barrier()
        hub.hub_finalize()
        self.spcomm = hub
        self.spokes = spokes
        self.opt_dict = hub_dict
        self.global_rank = comm.Get_rank()
        self.strata_rank = 0
        self.cylinder_rank = comm.Get_rank()
        self.BestInnerBound = hub.BestInnerBound
        self.BestOuterBound = hub.BestOuterBound
        self._ran = True

    def on_hub(self):
        if not self._ran:
            raise RuntimeError("Need to call WheelSpinner.run() before finding out.")
        return True

    # spin_the_wheel.py:_determine_innerbound_winner
    def _determine_innerbound_winner(self):
        idx = self.spcomm.last_ib_idx
        if idx is None or idx == 0:
            return None
        return self.spokes[idx - 1]

    def write_first_stage_solution(self, solution_file_name, first_stage_solution_writer=None):
        """Write the ROOT nonants of the best inner-bound solution as 'name,value' lines
        (sputils.first_stage_nonant_writer); nothing when no xhat was found."""
        if not self._ran:
            raise RuntimeError("Need to call WheelSpinner.run() before querying solutions.")
        winner = self._determine_innerbound_winner()
        if winner is None or getattr(winner, "best_xhat", None) is None or self.global_rank != 0:
            return
        b = winner.opt.batch
        root = winner.best_xhat["ROOT"]
        names = b.nonant_names or [f"nonant[{k}]" for k in range(b.nn)]
        with open(solution_file_name, "w", newline="") as f:
            w = csv.writer(f)
            for k in range(b.nn):
                if b.nonant_depth[k] == 0:
                    w.writerow([names[k], float(root[b.nonant_off[k]])])

    def local_nonant_cache(self):
        winner = self._determine_innerbound_winner()
        return None if winner is None else winner.best_xhat
