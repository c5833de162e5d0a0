"""Hub <-> spoke transport for cylinders placed on their own ranks.

The reference gives every cylinder its own MPI ranks (spin_the_wheel.py:219-237: the
world is split into ``n_spokes + 1`` cylinders of P ranks; strata s holds the s-th rank
of every cylinder, and rank s of the hub talks only to rank s of each spoke) and moves
W / nonants / bounds through one-sided MPI windows: the hub Puts its buffer -- the
values in 'ci' order (local scenarios x nonants, phbase.py:355-366) plus three trailing
slots [BestOuterBound, BestInnerBound, write id] (hub.py:281-285, 369-395) -- and the
spoke Gets it when it wants and takes it only if the write id advanced (spoke.py:84-118);
the spoke's bound goes back the same way (spoke.py:60-82, hub.py:396-436), and write id
-1 is the kill signal (hub.py:438-450).

Here a window is a key of the job's TCP rendezvous store (torch.distributed's
key-value store: set / get / check / delete_key -- one-sided, like the RMA window), used
in pull mode:

  spoke rank:  set its request key (= [bound, bound write id, last hub write id seen]),
               wait for its window key, get it, delete it -- one Get, issued when the
               spoke is ready for new data (its loop body is done);
  hub rank:    at each PH sync, ``check`` (non-blocking) which spokes have a request
               waiting -- agreed over the hub's ranks by one MIN all-reduce, so every rank
               of a spoke gets the W of the same hub iteration -- take the request and
               set the window: the current W / nonants in 'ci' order, the bounds and a
               new write id; at termination, answer every spoke once more with write id
               -1 (and the final W, for the Lagrangian's last pass).

The hub never waits for a spoke inside the PH loop (a check costs ~25 us, a 196 KB
window ~85 us on one node), and a spoke always receives the hub's current values.

Termination (spin_the_wheel.py:126-139 runs the spokes' finalize, a Barrier, then
hub_finalize, so a spoke's last bound -- the Lagrangian's final pass with the final W --
counts): after its finalize a spoke sets one more key, ``fin``, holding its final bound
and write id, and the hub's ``hub_finalize`` waits for it before the last bound update.
A spoke whose loop raises sets its request / ``fin`` keys with the failure flag, and
every hub wait has a time limit (``timeout``); either ends the hub with an error that
names the spoke's cylinder instead of a hang.
"""
import datetime
import itertools
import struct

import numpy as np
import torch
import torch.distributed as dist

from ..comm import Comm

KILL = -1.0
FAILED = 1.0
_REQ = struct.Struct("<4d")   # [bound, bound write id, last hub write id seen, failure flag]
WAIT_TIMEOUT = datetime.timedelta(seconds=1800)   # longest a hub waits on one spoke key


class SpokeFailure(RuntimeError):
    """A spoke on its own ranks stopped with an error, or never answered in time."""
_serial = itertools.count()   # one key prefix per wheel (every rank creates layouts in order)


class CylinderLayout:
    """Rank placement of spin_the_wheel.py:219-237: cylinder c owns global ranks
    [c P, (c+1) P); this rank is rank ``cyl_rank`` of cylinder ``cylinder``."""

    def __init__(self, n_cylinders):
        if not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError("cylinders on their own ranks need torch.distributed to be initialised")
        world = dist.get_world_size()
        if world % n_cylinders != 0:
            # spin_the_wheel.py:228-230
            raise RuntimeError(f"world size {world} is not a multiple of the number of cylinders {n_cylinders}")
        self.n_cylinders = n_cylinders
        self.P = world // n_cylinders
        self.rank = dist.get_rank()
        self.cylinder = self.rank // self.P
        self.cyl_rank = self.rank % self.P
        # every rank creates every group, in the same order
        groups = [dist.new_group(list(range(c * self.P, (c + 1) * self.P))) for c in range(n_cylinders)]
        self.cylinder_comm = Comm(groups[self.cylinder])
        self.fullcomm = Comm(None)
        # host-side transport group (gloo) over the whole world, and per cylinder (the
        # hub's ready-flag agreement)
        self.xgroup = dist.new_group(list(range(world)), backend="gloo")
        xcyl = [dist.new_group(list(range(c * self.P, (c + 1) * self.P)), backend="gloo")
                for c in range(n_cylinders)]
        self.cyl_xgroup = xcyl[self.cylinder]
        self.store = dist.distributed_c10d._get_default_store()
        self.prefix = f"phx{next(_serial)}/"

    def peer(self, cylinder):
        """Global rank of ``cylinder`` in this rank's strata."""
        return cylinder * self.P + self.cyl_rank


def agree_ready(layout, flags):
    """MIN over the hub's ranks of per-spoke request flags (host ints): a spoke is
    answered only when every hub rank has its strata peer's request."""
    t = torch.tensor([1 if f else 0 for f in flags], dtype=torch.int32)
    if layout.P > 1 and len(flags):
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=layout.cyl_xgroup)
    return [bool(v) for v in t.tolist()]


class StrataComm:
    """strata_comm stand-in: rank = cylinder index within the strata (0 = hub); the
    strata's traffic goes through the ports below."""

    def __init__(self, layout):
        self.layout = layout

    def Get_rank(self):
        return self.layout.cylinder

    def Get_size(self):
        return self.layout.n_cylinders

    def Barrier(self):
        pass


class HubPort:
    """Hub side of one spoke's window pair (this hub rank <-> its strata peer)."""

    def __init__(self, layout, spoke_cylinder, payload_len, timeout=WAIT_TIMEOUT):
        self.store = layout.store
        self.spoke = spoke_cylinder
        self.rank = layout.cyl_rank
        self.req_key = f"{layout.prefix}req/{spoke_cylinder}/{layout.cyl_rank}"
        self.win_key = f"{layout.prefix}win/{spoke_cylinder}/{layout.cyl_rank}"
        self.fin_key = f"{layout.prefix}fin/{spoke_cylinder}/{layout.cyl_rank}"
        self.n = payload_len
        self.buf = np.empty(payload_len + 3)
        self.timeout = timeout

    def ready(self):
        return self.store.check([self.req_key])

    def _take(self, key, what):
        try:
            self.store.wait([key], self.timeout)
        except Exception as e:  # the store raises on its deadline
            raise SpokeFailure(f"spoke cylinder {self.spoke} (rank {self.rank} of its cylinder) did not post "
                               f"its {what} within {self.timeout}: {e}") from e
        bound, bound_wid, _, failed = _REQ.unpack(self.store.get(key))
        self.store.delete_key(key)
        if failed == FAILED:
            raise SpokeFailure(f"spoke cylinder {self.spoke} (rank {self.rank} of its cylinder) stopped with an "
                               f"error (see that rank's output)")
        return bound, bound_wid

    def answer(self, values, outer, inner, write_id):
        """Take the waiting request (blocks until there is one, at most ``timeout``) and
        set the window; returns the (bound, bound write id) that came with the request."""
        bound, bound_wid = self._take(self.req_key, "request")
        if values is not None:
            self.buf[:self.n] = values.numpy().reshape(-1)[:self.n]
        self.buf[self.n:] = (outer, inner, write_id)
        self.store.set(self.win_key, self.buf.tobytes())
        return bound, bound_wid

    def final(self):
        """The spoke's bound after its finalize (spoke.py finalize -> spin_the_wheel.py:132
        Barrier -> hub_finalize): (bound, bound write id)."""
        return self._take(self.fin_key, "final bound")


class SpokePort:
    """Spoke side: one Get = request + wait for the hub's answer."""

    def __init__(self, layout, payload_len, timeout=WAIT_TIMEOUT):
        self.store = layout.store
        self.req_key = f"{layout.prefix}req/{layout.cylinder}/{layout.cyl_rank}"
        self.win_key = f"{layout.prefix}win/{layout.cylinder}/{layout.cyl_rank}"
        self.fin_key = f"{layout.prefix}fin/{layout.cylinder}/{layout.cyl_rank}"
        self.n = payload_len
        self.timeout = timeout
        self.requested = False   # a request is posted and not yet answered

    def get(self, bound, bound_wid, seen_wid):
        self.store.set(self.req_key, _REQ.pack(float(bound), float(bound_wid), float(seen_wid), 0.0))
        self.requested = True
        self.store.wait([self.win_key], self.timeout)
        self.requested = False
        buf = np.frombuffer(self.store.get(self.win_key), dtype=np.float64)
        self.store.delete_key(self.win_key)
        vals = torch.from_numpy(buf[:self.n].copy())
        return vals, float(buf[self.n]), float(buf[self.n + 1]), float(buf[self.n + 2])

    def post_final(self, bound, bound_wid):
        """The bound after finalize, for the hub's hub_finalize."""
        self.store.set(self.fin_key, _REQ.pack(float(bound), float(bound_wid), 0.0, 0.0))

    def post_failure(self):
        """Tell the hub this spoke has stopped: whichever key it waits on next -- a
        request (unless one is already posted) or the final bound -- carries the flag."""
        msg = _REQ.pack(float("nan"), 0.0, 0.0, FAILED)
        if not self.requested:
            self.store.set(self.req_key, msg)
        self.store.set(self.fin_key, msg)


def ci_order(t_nn_S):
    """Device [nn, S] -> host flat 'ci' order (local scenarios x nonants, phbase.py:355-366)."""
    return t_nn_S.t().contiguous().reshape(-1).to("cpu")


def from_ci_order(flat, nn, S, device):
    """Host flat 'ci' order -> device [nn, S]."""
    return flat.reshape(S, nn).t().contiguous().to(device)
