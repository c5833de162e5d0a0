"""Device engine: one rank's ScenarioBatch resident in HBM + the libphgpu calls.

Owns the caller-side device buffers of include/phgpu.h (torch tensors on the rank's
GPU, scenario-fastest ``[k, S]``) and sequences the per-PH-iteration work:

    solve_loop      -> phgpu_solve                     (spopt.py:226-307)
    Compute_Xbar    -> phgpu_ph_reduce + all-reduce    (phbase.py:27-107)
    Update_W + conv -> phgpu_ph_update + all-reduce    (phbase.py:293-343)
    Ebound/Eobj/E1  -> phgpu_expectations + all-reduce (spopt.py:310-439)

All launches go to torch's current stream; host synchronisation happens only where
the reference needs a host scalar (the convergence test, bounds).
"""
import atexit
import ctypes
import weakref

import numpy as np
import torch

from . import _lib
from .comm import Comm


def _dev_T(a, device, dtype=torch.float64):
    """host [S, k] -> device [k, S] contiguous."""
    a = np.asarray(a)
    if a.ndim == 1:
        return torch.from_numpy(np.ascontiguousarray(a)).to(device=device, dtype=dtype)
    return torch.from_numpy(np.ascontiguousarray(a.T)).to(device=device, dtype=dtype)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def combine_node_partials(comm, node_buf):
    """Cross-rank sum of the node-indexed x̄ / x̄² partial buffer (phbase.py:83-87)."""
    return comm.allreduce_sum_(node_buf)


# scenarios at least this large (n + m) whose matrix values are the same in every
# scenario run on the shared-matrix streaming path (path 4, include/phgpu.h
# PHGPU_SHARED_MATRIX); smaller ones fit the register / workgroup-resident paths
SHARED_MIN_SIZE = 8192


# Engines still open at interpreter exit are closed by an atexit hook registered when the
# first engine is made -- after torch's own hooks, so it runs before them (LIFO), while the
# HIP runtime (and a profiler's tool library) is still up.  PHEngine.__del__ at interpreter
# teardown could run after them: a rocprofv3 run of bench.py died in it (SIGSEGV after the
# tool's finalisation, profiles/r04/ac/uc_1.log).
_LIVE = weakref.WeakSet()
_ATEXIT = []


def close_all():
    """Close every engine still open (phgpu_destroy after a device synchronise)."""
    for e in list(_LIVE):
        try:
            e.close()
        except Exception:
            pass


def _track(engine):
    if not _ATEXIT:
        atexit.register(close_all)
        _ATEXIT.append(True)
    _LIVE.add(engine)


def matrix_is_shared(batch):
    """True if every scenario of the batch has the same constraint-matrix values."""
    A = batch.A_val
    return A.shape[0] <= 1 or (A.strides[0] == 0) or bool(np.all(A == A[:1]))


class PHEngine:
    def __init__(self, batch, device=None, comm=None, node_names=None, shared=None):
        """``shared``: None = the shared-matrix path when the matrix is the same in every
        scenario and the scenarios are large (SHARED_MIN_SIZE); True / False force it
        (True requires the same matrix)."""
        if not torch.cuda.is_available():
            raise _lib.PhgpuError("PHEngine needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.lib = _lib.load()
        self.batch = batch
        self.comm = comm or Comm()
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        self.dev_index = self.device.index if self.device.index is not None else torch.cuda.current_device()
        self._stream_cache = {}
        b = batch
        S, n, m, nn = b.S, b.n, b.m, b.nn
        self.S, self.n, self.m, self.nn = S, n, m, nn
        # global node numbering (identical on all ranks): node_names of the PH object
        names = node_names if node_names is not None else b.node_names
        gid = {nd: i for i, nd in enumerate(names)}
        remap = np.array([gid[nd] for nd in b.node_names], dtype=np.int32)
        node_of = remap[b.node_of]
        self.node_names = list(names)
        self.num_nodes = len(names)
        self.nlen_max = max(1, b.nlen_max)
        h = ctypes.c_void_p()
        rp = np.ascontiguousarray(b.row_ptr, dtype=np.int32)
        ci = np.ascontiguousarray(b.col_idx, dtype=np.int32)
        nc = np.ascontiguousarray(b.nonant_col, dtype=np.int32)
        nd = np.ascontiguousarray(b.nonant_depth, dtype=np.int32)
        no = np.ascontiguousarray(b.nonant_off, dtype=np.int32)
        P = lambda a: a.ctypes.data_as(_lib.P_i32)  # noqa: E731
        if shared is None:
            shared = (n + m) >= SHARED_MIN_SIZE and matrix_is_shared(b)
        elif shared and not matrix_is_shared(b):
            raise ValueError("shared=True needs the same matrix values in every scenario")
        self.shared = bool(shared)
        torch.cuda.set_device(self.dev_index)
        _lib.check(self.lib.phgpu_create2(ctypes.byref(h), self.dev_index, S, n, m, b.nnz, P(rp), P(ci),
                                          nn, P(nc), P(nd), P(no), b.depth, self.num_nodes,
                                          self.nlen_max, _lib.SHARED_MATRIX if self.shared else 0),
                   "phgpu_create2")
        self.h = h
        _track(self)
        # library calls of the PH step, by kind (tests assert which path a loop took)
        self.calls = {"ph_reduce": 0, "ph_update_ex": 0, "ph_step_local": 0, "ph_step_defer": 0,
                      "allreduce_xbar": 0, "allreduce_conv_side": 0, "allreduce_conv_main": 0, "xbar_ahead_used": 0,
                      "ph_loop": 0}
        # several ranks: the conv all-reduce on a side stream under the next solve (False: on
        # the launch stream ahead of it -- bench.py --no-conv-overlap, the comparison case)
        self.overlap_conv = True
        dev = self.device
        self.A_val = _dev_T(b.A_val[0] if self.shared else b.A_val, dev)
        self.c = _dev_T(b.c, dev)
        self.lb = _dev_T(b.lb, dev)
        self.ub = _dev_T(b.ub, dev)
        self.rl = _dev_T(b.rl, dev)
        self.ru = _dev_T(b.ru, dev)
        self.q = _dev_T(b.q, dev)
        self.obj_const = _dev_T(b.obj_const, dev)
        self.prob = _dev_T(b.prob, dev)
        self.node_of = _dev_T(node_of, dev, torch.int32)
        self.prob_coeff = _dev_T(b.prob_coeff, dev)
        # caller-owned I/O buffers
        z = lambda *s: torch.zeros(*s, dtype=torch.float64, device=dev)  # noqa: E731
        self.x = z(n, S)
        self.y = z(max(m, 1), S)
        self.obj = z(S)
        self.bound = z(S)
        self.status = torch.zeros(S, dtype=torch.int32, device=dev)
        self.iters = torch.zeros(S, dtype=torch.int32, device=dev)
        self.W = z(max(nn, 1), S)
        self.rho = z(max(nn, 1), S)
        self.xbar = z(max(nn, 1), S)
        self.node_buf = z(2 * self.num_nodes * self.nlen_max)
        self.conv_buf = z(1)
        self.exp_buf = z(5)
        self.xfix = None
        self.pvar = None          # per-nonant probability coefficients (set_nonant_probs)
        self.W_on = 0
        self.prox_on = 0
        # row duals are an optional phgpu_solve output: PH never reads them, so the hot
        # loop leaves them on the device side (set True to have ``y`` filled by solves)
        self.want_duals = False
        # Host-mapped readbacks (phgpu_ph_update_ex writes conv and the last solve's
        # statistics straight into pinned host memory, no copy launches): launch ids of the
        # last solve launch, of the solve whose outputs are current and of a pending
        # speculative one; row_of maps a launch id to the stats row an update wrote for it.
        self._xbar_pending = False   # compute_xbar(lazy=True) left x̄ to the next update
        self._launch_id = self._cur_id = self._spec_id = 0
        self._gripe_id = 0
        self._row_of = {}
        self._stats_rows = torch.zeros((1, 6), dtype=torch.int64).pin_memory()
        self._stats_tmp = torch.zeros(6, dtype=torch.int64).pin_memory()
        # conv readback: the update kernel (one rank) or the copy behind the conv all-reduce
        # (several ranks) stores conv into this pinned word, which the host set to NaN before
        # the update was queued; the host polls it -- no event marker in the PH step (each
        # marker is a barrier packet that idles the GPU ~5.6 us)
        self._conv_host = torch.full((1,), float("nan"), dtype=torch.float64).pin_memory()
        self._conv_np = self._conv_host.numpy()
        self._conv_zero_copy = False
        self._conv_seq = 0        # the update whose conv the pending readback returns
        self._conv_seen = 0       # the last update whose conv (and statistics) the host has seen
        self._side = None         # side stream of the conv all-reduce (several ranks)
        self._ahead_id = 0        # launch whose x xbar_ahead reduced into node_buf (0: none)
        self._conv_ev = None      # the event behind its copy to pinned memory
        self._wait_stats = None   # the pinned statistics row the pending update writes (one rank)
        # markers: the event behind an update (by update number), recorded lazily, only when
        # the host needs an update's statistics before its conv arrived
        self._upd_seq = 0
        self._upd_marks = {}
        self._upload()
        self._native = False
        self._native_comm()

    # -------------------------------------------------------------- plumbing
    def _native_comm(self):
        """The PH step's rank sums through the library's own RCCL communicator (include/phgpu.h
        phgpu_comm_init): ncclAllReduce straight on the engine's stream instead of a
        torch.distributed call (~15 us of host time each in c10d, twice per PH iteration on
        the host's critical path)."""
        plan = getattr(self.comm, "rccl_plan", lambda: None)()
        if plan is None:
            return
        nranks, rank = plan
        # two communicators: the launch stream's x̄ sums (slot 0) and the side stream's conv
        # sums (slot 1), so that neither alternates between streams
        ids = [ctypes.create_string_buffer(128) for _ in range(2)]
        if rank == 0:
            for u in ids:
                _lib.check(self.lib.phgpu_comm_unique_id(u), "phgpu_comm_unique_id")
        raw = [u.raw for u in ids]
        if nranks > 1:
            raw = self.comm.bcast_object(raw if rank == 0 else None, root=0)
        for slot in (0, 1):
            u = ctypes.create_string_buffer(bytes(raw[slot]), 128)
            _lib.check(self.lib.phgpu_comm_init(self.h, u, int(nranks), int(rank), slot), "phgpu_comm_init")
        self._native = True

    def _ar(self, t, tag="critical"):
        """In-place sum of a device fp64 tensor over the ranks (tag "overlapped": the side
        stream's conv sum, on the library's second communicator)."""
        if self._native and t.is_cuda and t.dtype == torch.float64 and t.is_contiguous():
            _lib.check(self.lib.phgpu_allreduce_sum(self.h, 1 if tag == "overlapped" else 0, _ptr(t),
                                                    int(t.numel()), self._stream()), "phgpu_allreduce_sum")
            return self.comm.after_native_(t)
        return self.comm.allreduce_sum_(t)

    def _stream(self):
        # the current stream's handle, cached by the stream's identity (torch's
        # current_stream builds a Stream object per call: ~5 us, twice per PH iteration on
        # the host's critical path)
        key = torch._C._cuda_getCurrentStream(self.dev_index)
        h = self._stream_cache.get(key)
        if h is None:
            h = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
            self._stream_cache[key] = h
        return h

    def _upload(self):
        _lib.check(self.lib.phgpu_set_scenarios(
            self.h, _ptr(self.A_val), _ptr(self.c), _ptr(self.lb), _ptr(self.ub), _ptr(self.rl),
            _ptr(self.ru), _ptr(self.q), _ptr(self.obj_const), _ptr(self.prob), _ptr(self.node_of),
            _ptr(self.prob_coeff), self._stream()), "phgpu_set_scenarios")
        self._bind()

    def _bind(self):
        _lib.check(self.lib.phgpu_set_ph_state(self.h, _ptr(self.W), _ptr(self.rho), _ptr(self.xbar),
                                               self.W_on, self.prox_on), "phgpu_set_ph_state")

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            self._flush_step()
            torch.cuda.synchronize(self.device)
            if getattr(self, "_side", None) is not None:
                self._side.synchronize()
            self.lib.phgpu_destroy(self.h)
            self.h = None
        _LIVE.discard(self)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def workspace_bytes(self):
        return int(self.lib.phgpu_workspace_bytes(self.h))

    def kernel_info(self):
        """Which solve kernel the handle uses (phgpu_kernel_info)."""
        info = (ctypes.c_int32 * 20)()
        _lib.check(self.lib.phgpu_kernel_info(self.h, info), "phgpu_kernel_info")
        keys = ["instance", "lanes", "kc", "zc", "kr", "zr", "KC", "ZC", "KR", "ZR",
                "wg_instance", "wps", "wKC", "wZC", "wKR", "wZR", "path", "rec", "jit_eligible", "jit_wpe"]
        return dict(zip(keys, list(info)))

    def stream_info(self):
        """Path 4 of the last solve (phgpu_stream_info): workgroups per scenario of its
        cluster form (0: the queue), whether the last solve took path 4."""
        info = (ctypes.c_int32 * 2)()
        _lib.check(self.lib.phgpu_stream_info(self.h, info), "phgpu_stream_info")
        return {"cluster": int(info[0]), "path4": int(info[1])}

    def ipm_info(self):
        """Path 6 (interior point) of the handle (phgpu_ipm_info)."""
        info = (ctypes.c_double * 16)()
        _lib.check(self.lib.phgpu_ipm_info(self.h, info), "phgpu_ipm_info")
        keys = ["eligible", "nf_bound", "off", "compiled", "rows", "factor_entries", "scratch_bytes", "compile_s",
                "factor_flops", "solve_flops", "lanes", "folded_steps", "kernel", "jam_handovers", "recentrings",
                "lds_slacks"]
        return dict(zip(keys, list(info)))

    def ipm_prof(self):
        """Per-wave timelines of the last path-6 launch (diagnostics; modules built with
        IPM_PROF in PHGPU_IPM_DEFS on a handle created with PHGPU_IPM_PROF=1): an
        [waves, 16] uint64 array (phgpu_ipm_prof), or None without the buffer."""
        n = int(self.lib.phgpu_ipm_prof(self.h, None, 0))
        if n < 0:
            _lib.check(-1, "phgpu_ipm_prof")
        if n == 0:
            return None
        out = np.zeros(n, dtype=np.uint64)
        rc = int(self.lib.phgpu_ipm_prof(self.h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)), n))
        if rc < 0:
            _lib.check(rc, "phgpu_ipm_prof")
        return out.reshape(-1, 16)

    # -------------------------------------------------------------- PH state
    def set_rho(self, rho):
        """rho: scalar, host [nn] array (the same per-nonant rho in every scenario) or host
        [S, nn] array (the rho Params of phbase.py:598-602)."""
        self._flush_step()
        if np.isscalar(rho):
            self.rho.fill_(float(rho))
        elif np.ndim(rho) == 1:
            r = torch.as_tensor(np.asarray(rho, dtype=np.float64), device=self.device)
            assert r.shape[0] == self.nn, (r.shape, self.nn)
            self.rho[:self.nn].copy_(r[:, None].expand(self.nn, self.S))
        else:
            self.rho.copy_(_dev_T(np.asarray(rho, dtype=np.float64), self.device))

    def set_W(self, W):
        self._flush_step()
        self.W.copy_(_dev_T(np.asarray(W, dtype=np.float64), self.device))

    def set_ipm_tuning(self, tuning):
        """Interior-point constants for this handle's modules ({"IPM_SIG_MIN": 0.003, ...};
        phgpu_set_ipm_tuning, before the first solve): a model's measured values."""
        defs = ";".join(f"{k}={v if isinstance(v, int) else repr(float(v))}" for k, v in (tuning or {}).items())
        _lib.check(self.lib.phgpu_set_ipm_tuning(self.h, defs.encode()), "phgpu_set_ipm_tuning")

    def set_nonant_probs(self, var_prob):
        """Per-nonant probability coefficients, host [S, nn] (SPBase.var_prob), or None:
        the x̄ weights and the Update_W mask of variable probabilities (phgpu_set_nonant_probs,
        spbase.py:394-437, phbase.py:315-318)."""
        self._flush_step()
        if var_prob is None:
            self.pvar = None
        else:
            self.pvar = _dev_T(np.asarray(var_prob, dtype=np.float64), self.device)
            assert tuple(self.pvar.shape) == (self.nn, self.S), self.pvar.shape
        _lib.check(self.lib.phgpu_set_nonant_probs(self.h, _ptr(self.pvar)), "phgpu_set_nonant_probs")

    def set_xbar(self, xbar):
        self._flush_step()
        self.xbar.copy_(_dev_T(np.asarray(xbar, dtype=np.float64), self.device))

    def set_terms(self, W_on, prox_on):
        self.W_on = 1 if W_on else 0
        self.prox_on = 1 if prox_on else 0
        self._bind()

    # -------------------------------------------------------------- instrumentation
    _AR_TIMED = 8

    def instrument(self, max_solves, every=1):
        """Record every ``every``-th of the next ``max_solves`` phgpu_solve launches: HIP
        events on the launch stream around the launch and its statistics (status counts,
        iteration sum and maximum; written to pinned memory by the next update kernel, the
        last launch's by phgpu_solve_stats).  Used by bench.py for the per-launch roofline
        inside its timed region; each event is a marker packet that idles the GPU ~5.6 us,
        so the bench samples one step in ``every``."""
        self._ins = {"events": [], "ids": [], "max": int(max_solves), "every": max(1, int(every)), "seen": 0,
                     "ar_events": [], "ar_count": 0,
                     "rows": torch.zeros((max_solves + 4, 6), dtype=torch.int64).pin_memory(), "next": 0}

    def instrumented(self):
        """[(launch ms, scenario-iterations)] of the recorded launches (syncs)."""
        return [(a.elapsed_time(b), int(st[4])) for (a, b), st in self._ins_stats()]

    def instrumented_not_optimal(self):
        """Scenarios not OPTIMAL in each recorded launch."""
        return [int(st[1:4].sum()) for _, st in self._ins_stats()]

    def _ins_stats(self):
        """[(event pair, stats[6])] of the recorded launches whose statistics are known: the
        update after a launch wrote them (phgpu_ph_update_ex), or the launch is the last
        one (phgpu_solve_stats).  Synchronises."""
        ins = getattr(self, "_ins", None)
        if not ins:
            return []
        torch.cuda.synchronize(self.device)
        out = []
        for ev, lid in zip(ins["events"], ins["ids"]):
            st = self._stats_of(lid)
            if st is not None:
                out.append((ev, st))
        return out

    def _recording(self):
        """True while instrumenting (the next ``max_solves`` solves)."""
        ins = getattr(self, "_ins", None)
        return ins is not None and ins["seen"] < ins["max"]

    def _marker(self, seq=None):
        """The event behind update ``seq`` (default: the last one), recorded now if it has
        none yet (then it also covers whatever was queued since)."""
        seq = self._upd_seq if seq is None else seq
        ev = self._upd_marks.get(seq)
        if ev is None:
            ev = torch.cuda.Event()
            ev.record()
            self._upd_marks[seq] = ev
        return ev

    def _stats_of(self, lid):
        """Statistics of launch ``lid`` (host int64[6] copy) or None if no longer known."""
        where = self._row_of.get(lid)
        if where is not None:
            rows, r, seq = where
            if seq > self._conv_seen:   # the update's conv (written after them) not seen yet
                self._marker(seq).synchronize()
            return rows[r].clone()
        if lid == self._launch_id and lid:
            _lib.check(self.lib.phgpu_solve_stats(self.h, _ptr(self._stats_tmp), self._stream()), "phgpu_solve_stats")
            torch.cuda.current_stream(self.device).synchronize()
            return self._stats_tmp.clone()
        return None

    def instrumented_allreduce_ms(self, tag=None):
        """Total ms of the x̄ / conv all-reduces issued while instrumenting (HIP events on
        the issuing stream around each collective; 0 with one rank, where they are no-ops);
        ``tag`` "critical" / "overlapped" selects the x̄ or the conv ones."""
        ins = getattr(self, "_ins", None)
        if not ins:
            return 0.0
        torch.cuda.synchronize(self.device)
        evs = [(ev, t) for ev, t in ins["ar_events"] if tag is None or t == tag]
        if not evs or not ins["ar_events"]:
            return 0.0
        mean = sum(a.elapsed_time(b) for (a, b), _ in evs) / len(evs)
        return float(mean * ins["ar_count"] * len(evs) / len(ins["ar_events"]))

    def _allreduce_sum_(self, t, tag="critical"):
        """comm.allreduce_sum_ with HIP events around it while instrumenting (``tag``:
        "critical", ahead of the next solve on the launch stream, or "overlapped", the conv
        all-reduce on the side stream)."""
        ins = getattr(self, "_ins", None)
        if ins is None or self.comm.size == 1 or not self._recording():
            return self._ar(t, tag)
        # the first _AR_TIMED all-reduces are timed (each event record is a marker packet
        # that idles the GPU ~5.6 us); the rest are counted and the mean extrapolated
        ins["ar_count"] += 1
        if len(ins["ar_events"]) >= self._AR_TIMED:
            return self._ar(t, tag)
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
        self._ar(t, tag)
        ev[1].record()
        ins["ar_events"].append((ev, tag))
        return t

    # -------------------------------------------------------------- hot path
    _OUTS = ("x", "y", "obj", "bound", "status", "iters")

    def solve(self, options=None, warm=True, speculative=False):
        """phgpu_solve into the output tensors (x, y, obj, bound, status, iters), or with
        ``speculative`` (phgpu_solve_deferred) into a second set that ``commit()`` swaps in
        (PHBase.iterk_loop launches the next solve before it knows whether the convergence
        test stops the loop).  An uncommitted speculative solve changes nothing: its
        outputs stay in the spare set and the library keeps its warm-start state in a
        second slot that only phgpu_commit makes current (include/phgpu.h)."""
        # a pending lazy x̄ is computed now; a deferred PH step stays with the library, which
        # folds it into this launch or runs it ahead of it (phgpu_ph_step_defer)
        if getattr(self, "_xbar_pending", False):
            self.compute_xbar()
        o = options if options is not None else _lib.default_options()
        if speculative:
            if not hasattr(self, "_spec"):
                self._spec = {k: torch.empty_like(getattr(self, k)) for k in self._OUTS}
            out = self._spec
        else:
            out = {k: getattr(self, k) for k in self._OUTS}
        ins = getattr(self, "_ins", None)
        rec = False
        if self._recording():
            rec = ins["seen"] % ins["every"] == 0
            ins["seen"] += 1
        if rec:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
            if self._upd_seq and self._upd_marks.get(self._upd_seq) is None:
                self._upd_marks[self._upd_seq] = ev[0]   # the update's marker, shared
        self._launch_id += 1
        if speculative:
            self._spec_id = self._launch_id
        else:
            self._cur_id = self._launch_id
        self._step_deferred = False   # the library folds a deferred step into this launch or runs it first
        fn = self.lib.phgpu_solve_deferred if speculative else self.lib.phgpu_solve
        _lib.check(fn(self.h, ctypes.byref(o), 1 if warm else 0, _ptr(out["x"]),
                      _ptr(out["y"] if self.want_duals else None), _ptr(out["obj"]), _ptr(out["bound"]),
                      _ptr(out["status"]), _ptr(out["iters"]), self._stream()),
                   "phgpu_solve_deferred" if speculative else "phgpu_solve")
        if rec:
            ev[1].record()
            # the launch's statistics come with the next update (phgpu_ph_update_ex), the
            # last launch's from phgpu_solve_stats after the loop: no copy per launch
            ins["events"].append(ev)
            ins["ids"].append(self._launch_id)

    def commit(self):
        """Make the last speculative solve's outputs and warm-start state the current ones."""
        for k in self._OUTS:
            cur = getattr(self, k)
            setattr(self, k, self._spec[k])
            self._spec[k] = cur
        _lib.check(self.lib.phgpu_commit(self.h), "phgpu_commit")
        self._cur_id = self._spec_id

    def _status_counts(self):
        if not hasattr(self, "_counts_dev"):
            self._counts_dev = torch.zeros(4, dtype=torch.int32, device=self.device)
            self._counts_host = torch.zeros(4, dtype=torch.int32).pin_memory()
            self._counts_ev = torch.cuda.Event()
        _lib.check(self.lib.phgpu_status_counts(self.h, _ptr(self.status), _ptr(self._counts_dev), self._stream()),
                   "phgpu_status_counts")

    def count_not_optimal(self):
        """Number of local scenarios whose last solve is not OPTIMAL (phgpu_status_counts,
        one small read back)."""
        self._status_counts()
        c = self._counts_dev.cpu()
        return int(c[1:].sum())

    def count_not_optimal_async(self):
        """The same count for the current solve, without device work now: the next
        ``update`` writes its statistics (accumulated in the path-6 kernels) to pinned host
        memory with the convergence value, so ``pending_not_optimal`` after the next
        convergence readback costs nothing; without an update in between it asks
        phgpu_solve_stats (one small copy and a wait)."""
        self._gripe_id = self._cur_id

    def pending_not_optimal(self):
        st = self._stats_of(self._gripe_id)
        if st is None:  # a later launch replaced the library's statistics: count statuses
            return self.count_not_optimal()
        return int(st[1:4].sum())

    def ph_loop(self, options, max_iters, convthresh):
        """PHBase.iterk_loop of one rank in one launch (phgpu_ph_loop): up to ``max_iters``
        iterations of x̄ -> W -> conv -> (conv < convthresh: stop) -> solve, on the current
        output set, W, x̄ and node_buf.  Returns {"steps", "end", "ipm_iters", "conv",
        "ms"} -- end 0: the iteration limit, 1: converged, 2: a solve handed scenarios to the
        PDHG fallback (solved; the caller goes on step by step) -- or None when the handle's
        state is not one the loop runs (nothing launched)."""
        if self.comm.size != 1:
            return None
        self._flush_step()
        self._xbar_pending = False          # the loop computes x̄ from x itself
        self._ahead_id = 0
        conv = np.zeros(max(1, int(max_iters)), dtype=np.float64)
        out = np.zeros(4, dtype=np.int64)
        self._launch_id += 1
        self._cur_id = self._launch_id
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
        rc = self.lib.phgpu_ph_loop(self.h, ctypes.byref(options), int(max_iters), float(convthresh), _ptr(self.x),
                                    _ptr(self.y if self.want_duals else None), _ptr(self.obj), _ptr(self.bound),
                                    _ptr(self.status), _ptr(self.iters), _ptr(self.node_buf),
                                    conv.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                    out.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), self._stream())
        if rc == -3:
            self.ph_loop_declined = _lib.last_error()     # why the state is not one the loop runs
            return None
        _lib.check(rc, "phgpu_ph_loop")
        ev[1].record()
        ev[1].synchronize()
        self.calls["ph_loop"] += 1
        steps = int(out[0])
        return {"steps": steps, "end": int(out[1]), "ipm_iters": int(out[2]), "conv": conv[:steps].tolist(),
                "ms": ev[0].elapsed_time(ev[1])}

    def compute_xbar_partials(self):
        self.calls["ph_reduce"] += 1
        _lib.check(self.lib.phgpu_ph_reduce(self.h, _ptr(self.x), _ptr(self.node_buf), self._stream()),
                   "phgpu_ph_reduce")
        return self.node_buf

    def compute_xbar(self, lazy=False):
        """Local partials + cross-rank sum (phbase.py:27-87); result left in node_buf.
        ``lazy`` (PHBase.Compute_Xbar with one rank): nothing is launched yet -- the next
        ``update`` does x̄ and the update together (phgpu_ph_step_local: one launch fewer
        for two-stage problems); anything that reads node_buf first computes it.  Several
        ranks: nothing to do when ``xbar_ahead`` already reduced the current solve's x."""
        if lazy and self.comm.size == 1:
            self._xbar_pending = True
            return None
        self._xbar_pending = False
        if self._ahead_id and self._ahead_id == self._cur_id:
            self._ahead_id = 0
            self.node_buf, self._node_ahead = self._node_ahead, self.node_buf
            self.calls["xbar_ahead_used"] += 1
            return self.node_buf
        self._ahead_id = 0
        self.compute_xbar_partials()
        if self.comm.size > 1:
            self.calls["allreduce_xbar"] += 1
        self._allreduce_sum_(self.node_buf)
        return self.node_buf

    def xbar_ahead(self):
        """Several ranks (PHBase.iterk_loop): reduce the speculative solve's x and start the x̄
        all-reduce before the convergence test of the current iteration is known, so the next
        iteration's x̄ is on its way when the host returns from the test.  Used by the next
        ``compute_xbar`` if that solve is committed (its buffer then becomes node_buf), dropped
        otherwise; node_buf keeps the x̄ of the last update meanwhile (xbar_by_node after the
        loop), and every rank issues the same collectives in the same order."""
        if self.comm.size == 1 or not hasattr(self, "_spec"):
            return
        if getattr(self, "_node_ahead", None) is None:
            self._node_ahead = torch.zeros_like(self.node_buf)
        self.calls["ph_reduce"] += 1
        _lib.check(self.lib.phgpu_ph_reduce(self.h, _ptr(self._spec["x"]), _ptr(self._node_ahead), self._stream()),
                   "phgpu_ph_reduce")
        self.calls["allreduce_xbar"] += 1
        self._allreduce_sum_(self._node_ahead)
        self._ahead_id = self._spec_id

    def _flush_xbar(self):
        self._flush_step()
        if getattr(self, "_xbar_pending", False):
            self.compute_xbar()

    def _flush_step(self):
        """Run a step phgpu_ph_step_defer still holds (no solve has folded it yet)."""
        if getattr(self, "_step_deferred", False):
            self._step_deferred = False
            _lib.check(self.lib.phgpu_ph_step_flush(self.h), "phgpu_ph_step_flush")

    def update(self, update_W=True, defer=False):
        """Scatter x̄, W += rho (x - x̄), local conv (phbase.py:90-103, 293-339).  One rank:
        conv goes straight to pinned host memory (no copy launch; with several ranks it
        stays on the device for the all-reduce).  The last launch's statistics go to
        pinned host memory in the same kernel (the gripe and the instrumentation read
        them there).  ``defer`` (one rank, x̄ pending: PHBase.iterk_loop's speculative
        step) hands the step to phgpu_ph_step_defer, which folds it into the next solve
        launch when it can; the solve must follow before anything reads W."""
        if self._upd_seq > self._conv_seen and self._conv_zero_copy:
            # the previous update's conv / statistics were never read back: its kernel may
            # still store into the pinned words after the sentinels below are set
            torch.cuda.current_stream(self.device).synchronize()
        self._conv_zero_copy = self.comm.size == 1
        conv = self._conv_host if self._conv_zero_copy else self.conv_buf
        self._conv_np[0] = float("nan")     # the readback's sentinel (before the launch)
        self._upd_seq += 1
        self._upd_marks = {k: v for k, v in self._upd_marks.items() if k > self._upd_seq - 4}
        self._upd_marks[self._upd_seq] = None
        stats = None
        if self._launch_id:
            ins = getattr(self, "_ins", None)
            if ins is not None and ins["next"] < ins["rows"].shape[0]:
                rows, r = ins["rows"], ins["next"]
                ins["next"] += 1
            else:
                rows, r = self._stats_rows, 0
                self._row_of = {k: v for k, v in self._row_of.items() if v[0] is not rows}
            self._row_of[self._launch_id] = (rows, r, self._upd_seq)
            stats = rows[r]
            rows.numpy()[r] = -1            # the statistics' sentinels (convergence_wait)
        self._wait_stats = stats.numpy() if (stats is not None and self._conv_zero_copy) else None
        if getattr(self, "_xbar_pending", False):
            self._xbar_pending = False
            fn = self.lib.phgpu_ph_step_defer if defer else self.lib.phgpu_ph_step_local
            self.calls["ph_step_defer" if defer else "ph_step_local"] += 1
            _lib.check(fn(self.h, _ptr(self.x), _ptr(self.node_buf), _ptr(self.xbar),
                          _ptr(self.W), _ptr(self.rho), 1 if update_W else 0,
                          _ptr(conv), _ptr(stats), self._stream()), "phgpu_ph_step")
            self._step_deferred = bool(defer)
            return
        self.calls["ph_update_ex"] += 1
        _lib.check(self.lib.phgpu_ph_update_ex(self.h, _ptr(self.x), _ptr(self.node_buf), _ptr(self.xbar),
                                               _ptr(self.W), _ptr(self.rho), 1 if update_W else 0,
                                               _ptr(conv), _ptr(stats), self._stream()), "phgpu_ph_update_ex")

    def convergence_diff(self):
        """phbase.py:330-343: sum over ranks of per-rank means, / n_proc (host float)."""
        self.convergence_diff_async()
        return self.convergence_wait()

    def convergence_mark(self):
        """Mark the update on the launch stream (several ranks): a following
        ``convergence_diff_async`` waits for this point rather than for whatever was queued
        in between, so PHBase.iterk_loop launches the speculative solve right after the mark
        and issues the side-stream conv work behind it -- the host's side-stream calls (event,
        stream switch, all-reduce, copy) no longer delay the solve's launch (a 35 us idle gap
        per PH iteration in the loopback trace)."""
        if self._conv_zero_copy or self.comm.size == 1:
            return
        if not self.overlap_conv:
            # (the comparison case: the conv all-reduce stays ahead of the solve)
            self.convergence_diff_async()
            self._conv_issued = self._upd_seq
            return
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self._mark = (self._upd_seq, ev)

    def convergence_diff_async(self):
        """Start the same readback without waiting; ``convergence_wait`` returns it and work
        queued after this call does not delay it.  One rank: the update kernel stores conv
        into pinned memory itself.  Several ranks: the conv all-reduce (phbase.py:341) and
        its copy into pinned memory run on a side stream behind the update (or behind
        ``convergence_mark``), so the next solve launches at once and only the x̄ all-reduce
        stays ahead of it."""
        self._conv_seq = self._upd_seq
        if self._conv_zero_copy or getattr(self, "_conv_issued", 0) == self._upd_seq:
            return
        main = torch.cuda.current_stream(self.device)
        if self._conv_ev is None:
            self._conv_ev = torch.cuda.Event()
        mark = getattr(self, "_mark", None)
        self._mark = None
        if not self.overlap_conv:
            # (the comparison case of the bench: the conv all-reduce ahead of the next solve on
            # the launch stream, as the reference's Allreduce sits in the loop)
            self.calls["allreduce_conv_main"] += 1
            self._allreduce_sum_(self.conv_buf, tag="critical")
            self._conv_host.copy_(self.conv_buf, non_blocking=True)
            self._conv_ev.record(main)
            self._upd_marks[self._upd_seq] = self._conv_ev
            return
        if mark is not None and mark[0] == self._upd_seq:
            ev = mark[1]                           # recorded right after the update
        else:
            ev = torch.cuda.Event()
            ev.record(main)
        self._upd_marks[self._upd_seq] = ev        # (also the update's marker for its stats)
        if self._side is None:
            self._side = torch.cuda.Stream(device=self.device)
        self._side.wait_event(ev)
        self.calls["allreduce_conv_side"] += 1
        with torch.cuda.stream(self._side):
            self._allreduce_sum_(self.conv_buf, tag="overlapped")
            self._conv_host.copy_(self.conv_buf, non_blocking=True)
            # the host waits for this event, not for the word to change: the copy engine may
            # write the 8 bytes piecewise, and a poll caught a half-written value (its top
            # byte still the NaN sentinel's: 9.4e306 as conv on one rank, round-5 2-rank
            # test), which could make ranks disagree on the break and deadlock
            self._conv_ev.record(self._side)

    _SPIN = 200000

    def convergence_wait(self):
        """The pending conv (polls the pinned word; after a long wait it synchronises the
        streams, which also surfaces a device error)."""
        self._flush_step()          # a deferred step no solve has taken yet: run it now
        a = self._conv_np
        if not self._conv_zero_copy:
            # several ranks: the side stream's copy is complete once its event is -- polled
            # (hipEventQuery), not waited on: the blocking wait returned 15-20 us after the
            # copy had finished, on the host's critical path (loopback trace)
            ev, n = self._conv_ev, 0
            while not ev.query():
                n += 1
                if n > self._SPIN:
                    ev.synchronize()
                    break
            self._conv_seen = max(self._conv_seen, self._conv_seq)
            return float(a[0]) / self.comm.size
        st = self._wait_stats
        n = 0
        while a[0] != a[0] or (st is not None and (st == -1).any()):
            n += 1
            if n > self._SPIN:
                torch.cuda.current_stream(self.device).synchronize()
                if self._side is not None:
                    self._side.synchronize()
                break
        self._conv_seen = max(self._conv_seen, self._conv_seq)
        return float(a[0]) / self.comm.size

    def expectations(self):
        """(Eobj, Ebound, E1, Efeas, Eoptimal) summed over ranks (spopt.py:310-439)."""
        _lib.check(self.lib.phgpu_expectations(self.h, _ptr(self.obj), _ptr(self.bound), _ptr(self.status),
                                               _ptr(self.exp_buf), self._stream()), "phgpu_expectations")
        self.comm.allreduce_sum_(self.exp_buf)
        v = self.exp_buf.cpu().numpy()
        return float(v[0]), float(v[1]), float(v[2]), float(v[3]), float(v[4])

    def fix_nonants(self, xfix):
        """lb = ub = xfix on the nonant columns of every local scenario (device [nn, S]
        tensor, original units) for the next solves; None restores the model bounds
        (spopt.py:557-660 _fix_nonants / _restore_nonants)."""
        if xfix is not None:
            self.xfix = xfix.to(device=self.device, dtype=torch.float64).contiguous()
            assert tuple(self.xfix.shape) == (max(self.nn, 1), self.S), self.xfix.shape
        else:
            self.xfix = None
        _lib.check(self.lib.phgpu_fix_nonants(self.h, _ptr(self.xfix), self._stream()), "phgpu_fix_nonants")

    def fix_nonants_by_node(self, table):
        """Fix every local scenario's nonants at per-node values: ``table`` is a device
        [num_nodes, nlen_max] tensor (global node order of ``node_names``); nonant k of
        scenario s gets table[node_of[depth_k, s], off_k] (the per-node cache of
        spopt.py:557-592)."""
        if not hasattr(self, "_fix_index"):
            d = torch.as_tensor(self.batch.nonant_depth, dtype=torch.long, device=self.device)
            o = torch.as_tensor(self.batch.nonant_off, dtype=torch.long, device=self.device)
            self._fix_index = self.node_of.long().index_select(0, d) * self.nlen_max + o[:, None]
        t = table.reshape(-1).to(device=self.device, dtype=torch.float64)
        self.fix_nonants(t[self._fix_index])

    def nonant_x_dev(self):
        """[nn, S] device tensor of the nonant values of the last solve."""
        idx = torch.as_tensor(self.batch.nonant_col, dtype=torch.long, device=self.device)
        return self.x.index_select(0, idx)

    # -------------------------------------------------------------- host views
    def nonant_x(self):
        """[S, nn] host array of the nonant values (W cache 'ci' order, phbase.py:355-365)."""
        idx = torch.as_tensor(self.batch.nonant_col, dtype=torch.long, device=self.device)
        return self.x.index_select(0, idx).T.cpu().numpy()

    def host(self, name):
        self._flush_step()
        if name == "node_buf":
            self._flush_xbar()
        t = getattr(self, name)
        a = t.cpu().numpy()
        return a.T if a.ndim == 2 else a

    def node_xbar(self):
        """{node name: x̄ vector} from the (reduced) node buffer."""
        self._flush_xbar()
        buf = self.node_buf.cpu().numpy()
        nl = self.nlen_max
        return {nd: buf[g * nl:(g + 1) * nl] for g, nd in enumerate(self.node_names)}
