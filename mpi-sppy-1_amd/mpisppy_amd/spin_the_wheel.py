"""WheelSpinner: hub-and-spoke driver (mirrors mpisppy/spin_the_wheel.py:9-160).

Same dict contract as the reference: ``hub_dict`` with hub_class / hub_kwargs /
opt_class / opt_kwargs and one dict per spoke with spoke_class / spoke_kwargs /
opt_class / opt_kwargs; ``WheelSpinner(hub_dict, list_of_spoke_dict).spin()`` and then
``BestInnerBound`` / ``BestOuterBound`` / ``write_first_stage_solution``.

Two placements, chosen by ``placement`` ("auto" by default):

* "ranks" -- the reference's (spin_the_wheel.py:219-237): the world is split into
  n_spokes + 1 cylinders of P ranks each (one GPU per rank); every cylinder solves its
  own copy of the scenarios sliced over its P ranks, and the hub and the spokes talk
  through cylinders/transport.py (write-id windows, kill signal).  "auto" picks it when
  torch.distributed is initialised with a world size that is a multiple of the number of
  cylinders (the reference's requirement, spin_the_wheel.py:228-230) and above 1.
* "colocated" -- every rank holds its scenario slice for EVERY cylinder; hub and spoke
  engines share the GPU and the rank communicator, and the hub runs the spokes' loop
  bodies right after each sync (one process, or a world the cylinders do not divide).
"""
import csv
import math

import torch
import torch.distributed as dist

from .comm import Comm
from . import global_toc


class WheelSpinner:
    def __init__(self, hub_dict, list_of_spoke_dict):
        self.hub_dict = hub_dict
        self.list_of_spoke_dict = list(list_of_spoke_dict)
        self._ran = False

    def spin(self, comm_world=None, placement="auto"):
        return self.run(comm_world=comm_world, placement=placement)

    @staticmethod
    def _placement(placement, n_cyl):
        if placement != "auto":
            return placement
        if n_cyl > 1 and dist.is_available() and dist.is_initialized():
            w = dist.get_world_size()
            if w > 1 and w % n_cyl == 0:
                return "ranks"
        return "colocated"

    def run(self, comm_world=None, placement="auto"):
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

        self.placement = self._placement(placement, 1 + len(self.list_of_spoke_dict))
        if self.placement == "ranks":
            return self._run_on_ranks()
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

    # spin_the_wheel.py:37-159 with the reference's rank placement
    def _run_on_ranks(self):
        from .cylinders import transport as tp
        hub_dict = self.hub_dict
        layout = tp.CylinderLayout(1 + len(self.list_of_spoke_dict))
        strata = tp.StrataComm(layout)
        cyl = layout.cylinder_comm
        if layout.cylinder == 0:
            kw = dict(hub_dict["opt_kwargs"])
            kw["mpicomm"] = cyl
            hopt = hub_dict["opt_class"](**kw)
            spoke_classes = [d["spoke_class"] for d in self.list_of_spoke_dict]
            hub = hub_dict["hub_class"](hopt, layout.fullcomm, strata, cyl, spoke_classes,
                                        layout=layout, **hub_dict["hub_kwargs"])
            hub.setup_hub()
            global_toc("Starting spcomm.main()", layout.rank == 0 and hopt.options.get("toc", True))
            hub.main()
            hub.send_terminate()
            hub.finalize()
            hub.hub_finalize()
            self.spcomm = hub
            self.spokes = []
            ib = hub.last_ib_idx
            bounds = [hub.BestInnerBound, hub.BestOuterBound, -1.0 if ib is None else float(ib)]
        else:
            d = self.list_of_spoke_dict[layout.cylinder - 1]
            kw = dict(d["opt_kwargs"])
            kw["mpicomm"] = cyl
            sopt = d["opt_class"](**kw)
            spoke = d["spoke_class"](sopt, layout.fullcomm, strata, cyl, **d["spoke_kwargs"])
            port = tp.SpokePort(layout, max(sopt.batch.nn, 1) * sopt.batch.S)
            spoke.run_remote(port)
            self.spcomm = spoke
            self.spokes = [spoke]
            bounds = [math.nan, math.nan, -1.0]
        # every rank learns the hub's final bounds (global rank 0 is hub rank 0)
        t = torch.tensor(bounds, dtype=torch.float64)
        dist.broadcast(t, src=0, group=layout.xgroup)
        self.BestInnerBound, self.BestOuterBound = float(t[0]), float(t[1])
        self._winner_idx = int(t[2])
        dist.barrier(group=layout.xgroup)
        self.layout = layout
        self.opt_dict = hub_dict if layout.cylinder == 0 else self.list_of_spoke_dict[layout.cylinder - 1]
        self.global_rank = layout.rank
        self.strata_rank = layout.cylinder
        self.cylinder_rank = layout.cyl_rank
        self._ran = True

    def on_hub(self):
        if not self._ran:
            raise RuntimeError("Need to call WheelSpinner.run() before finding out.")
        return self.placement != "ranks" or self.strata_rank == 0

    # spin_the_wheel.py:_determine_innerbound_winner
    def _determine_innerbound_winner(self):
        if self.placement == "ranks":
            # the winning spoke's own ranks hold its solution (spin_the_wheel.py:166-177)
            return self.spokes[0] if self._winner_idx > 0 and self.strata_rank == self._winner_idx else None
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
        writer = self.cylinder_rank == 0 if self.placement == "ranks" else self.global_rank == 0
        if winner is None or getattr(winner, "best_xhat", None) is None or not writer:
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
