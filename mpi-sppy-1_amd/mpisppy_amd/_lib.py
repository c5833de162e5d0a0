"""ctypes binding of libphgpu.so (C-ABI declared in include/phgpu.h).

The library is the product path: if it is missing or fails to load, every engine
call raises -- there is no CPU fallback.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PHGPU_LIB", os.path.join(_HERE, "libphgpu.so"))

c_int = ctypes.c_int
c_i32 = ctypes.c_int32
c_i64 = ctypes.c_int64
c_dbl = ctypes.c_double
c_vp = ctypes.c_void_p
P_i32 = ctypes.POINTER(ctypes.c_int32)


class PhgpuOptions(ctypes.Structure):
    """phgpu_options (include/phgpu.h)."""
    _fields_ = [
        ("eps_rel", c_dbl),
        ("eps_abs", c_dbl),
        ("max_iter", c_i32),
        ("check_every", c_i32),
        ("gamma", c_dbl),
        ("beta_sufficient", c_dbl),
        ("beta_necessary", c_dbl),
        ("eta_frac", c_dbl),
        ("omega0", c_dbl),
        ("keep_omega", c_i32),
        ("restart_every", c_i32),
        ("beta_artificial", c_dbl),
        ("omega_clamp", c_dbl),
        ("kernel", c_i32),
        ("infeas_start", c_i32),
        ("eps_infeas", c_dbl),
        ("split_longest", c_i32),
    ]


OPTIMAL, ITER_LIMIT, PRIMAL_INFEASIBLE, DUAL_INFEASIBLE = 0, 1, 2, 3
SHARED_MATRIX = 1          # phgpu_create2 flag (include/phgpu.h)

# every symbol include/phgpu.h declares (tests check the library exports them all)
EXPORTS = ["phgpu_default_options", "phgpu_create", "phgpu_create2", "phgpu_set_scenarios", "phgpu_set_ph_state",
           "phgpu_solve", "phgpu_solve_deferred", "phgpu_commit", "phgpu_ph_reduce", "phgpu_ph_update",
           "phgpu_expectations",
           "phgpu_fix_nonants", "phgpu_status_counts", "phgpu_destroy", "phgpu_last_error", "phgpu_workspace_bytes",
           "phgpu_kernel_info", "phgpu_ipm_info", "phgpu_ipm_source", "phgpu_solve_stats",
           "phgpu_ph_update_ex", "phgpu_ph_step_local", "phgpu_ph_step_defer", "phgpu_ph_step_flush",
           "phgpu_set_nonant_probs", "phgpu_set_ipm_tuning", "phgpu_ipm_prof",
           "phgpu_ph_loop", "phgpu_stream_info", "phgpu_comm_unique_id", "phgpu_comm_init",
           "phgpu_allreduce_sum"]

_lib = None


class PhgpuError(RuntimeError):
    pass


def load(path=None):
    """Load (once) and type the library; raise PhgpuError if it is not there."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise PhgpuError(f"libphgpu.so not found at {p}: build it with "
                         f"`python -c 'import __graft_entry__ as g; g.build()'`")
    lib = ctypes.CDLL(p)
    lib.phgpu_default_options.argtypes = [ctypes.POINTER(PhgpuOptions)]
    lib.phgpu_create.argtypes = [ctypes.POINTER(c_vp), c_int, c_i64, c_i32, c_i32, c_i32, P_i32,
                                 P_i32, c_i32, P_i32, P_i32, P_i32, c_i32, c_i32, c_i32]
    lib.phgpu_create2.argtypes = lib.phgpu_create.argtypes + [ctypes.c_uint32]
    lib.phgpu_set_scenarios.argtypes = [c_vp] + [c_vp] * 11 + [c_vp]
    lib.phgpu_set_nonant_probs.argtypes = [c_vp, c_vp]
    lib.phgpu_set_ipm_tuning.argtypes = [c_vp, ctypes.c_char_p]
    lib.phgpu_set_ph_state.argtypes = [c_vp, c_vp, c_vp, c_vp, c_int, c_int]
    lib.phgpu_solve.argtypes = [c_vp, ctypes.POINTER(PhgpuOptions), c_int, c_vp, c_vp, c_vp, c_vp,
                                c_vp, c_vp, c_vp]
    lib.phgpu_solve_deferred.argtypes = lib.phgpu_solve.argtypes
    lib.phgpu_commit.argtypes = [c_vp]
    lib.phgpu_ph_reduce.argtypes = [c_vp, c_vp, c_vp, c_vp]
    lib.phgpu_ph_update.argtypes = [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_vp]
    lib.phgpu_ph_update_ex.argtypes = [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_vp]
    lib.phgpu_ph_step_local.argtypes = [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_vp]
    lib.phgpu_ph_step_defer.argtypes = lib.phgpu_ph_step_local.argtypes
    lib.phgpu_ph_step_flush.argtypes = [c_vp]
    lib.phgpu_expectations.argtypes = [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]
    lib.phgpu_fix_nonants.argtypes = [c_vp, c_vp, c_vp]
    lib.phgpu_status_counts.argtypes = [c_vp, c_vp, c_vp, c_vp]
    lib.phgpu_destroy.argtypes = [c_vp]
    lib.phgpu_last_error.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
    lib.phgpu_workspace_bytes.argtypes = [c_vp]
    lib.phgpu_workspace_bytes.restype = c_i64
    lib.phgpu_kernel_info.argtypes = [c_vp, P_i32]
    lib.phgpu_stream_info.argtypes = [c_vp, P_i32]
    lib.phgpu_comm_unique_id.argtypes = [ctypes.c_char_p]
    lib.phgpu_comm_init.argtypes = [c_vp, ctypes.c_char_p, c_int, c_int, c_int]
    lib.phgpu_allreduce_sum.argtypes = [c_vp, c_int, c_vp, c_i64, c_vp]
    lib.phgpu_ipm_info.argtypes = [c_vp, ctypes.POINTER(c_dbl)]
    lib.phgpu_ipm_prof.argtypes = [c_vp, ctypes.POINTER(ctypes.c_ulonglong), c_i64]
    lib.phgpu_ipm_prof.restype = c_i64
    lib.phgpu_solve_stats.argtypes = [c_vp, c_vp, c_vp]
    lib.phgpu_ph_loop.argtypes = [c_vp, ctypes.POINTER(PhgpuOptions), c_int, c_dbl, c_vp, c_vp, c_vp, c_vp, c_vp,
                                  c_vp, c_vp, ctypes.POINTER(c_dbl), ctypes.POINTER(c_i64), c_vp]
    lib.phgpu_ipm_source.argtypes = [c_i32, c_i32, c_i32, P_i32, P_i32, P_i32, P_i32, ctypes.POINTER(c_dbl), c_i32,
                                     ctypes.c_char_p, ctypes.c_size_t, P_i32]
    for name in EXPORTS:
        if name not in ("phgpu_workspace_bytes", "phgpu_ipm_prof"):
            getattr(lib, name).restype = c_int
    if path is None:
        _lib = lib
    return lib


def last_error():
    lib = load()
    buf = ctypes.create_string_buffer(512)
    lib.phgpu_last_error(buf, 512)
    return buf.value.decode(errors="replace")


def check(rc, what):
    if rc != 0:
        raise PhgpuError(f"{what} failed (rc={rc}): {last_error()}")


# element flags of phgpu_ipm_source (include/phgpu.h)
IPMF_UNI, IPMF_FIN_ANY, IPMF_FIN_ALL, IPMF_EQ = 1, 2, 4, 8


def ipm_flags(batch):
    """Host restatement of the library's k_ipm_flags over a ScenarioBatch (for
    phgpu_ipm_source in tests / tools): flags and first-scenario values per element of
    [A nnz | c n | q n | lb n | ub n | rl m | ru m]."""
    import numpy as np
    parts = [batch.A_val, batch.c, batch.q, batch.lb, batch.ub, batch.rl, batch.ru]
    flags, v0 = [], []
    for pi, arr in enumerate(parts):
        a = np.asarray(arr, dtype=np.float64)
        bits = a.view(np.int64)
        uni = (bits == bits[:1]).all(0)
        fin = np.isfinite(a)
        f = uni * IPMF_UNI + fin.any(0) * IPMF_FIN_ANY + fin.all(0) * IPMF_FIN_ALL
        if pi == 5:
            f = f + (fin & (np.asarray(batch.ru) == a)).all(0) * IPMF_EQ
        flags.append(f.astype(np.int32))
        v0.append(a[0])
    return np.concatenate(flags).astype(np.int32), np.concatenate(v0).astype(np.float64)


def ipm_source(batch, lanes=1):
    """The path-6 source the library generates for a batch (no GPU): (text, (rows, factor
    entries, factorisation flops, solve flops))."""
    import numpy as np
    lib = load()
    flags, v0 = ipm_flags(batch)
    slot = np.full(batch.n, -1, dtype=np.int32)
    slot[batch.nonant_col] = np.arange(batch.nn, dtype=np.int32)
    rp = np.ascontiguousarray(batch.row_ptr, dtype=np.int32)
    ci = np.ascontiguousarray(batch.col_idx, dtype=np.int32)
    ip = lambda a: a.ctypes.data_as(P_i32)  # noqa: E731
    info = np.zeros(4, dtype=np.int32)
    args = (batch.n, batch.m, batch.nnz, ip(rp), ip(ci), ip(slot), ip(flags),
            v0.ctypes.data_as(ctypes.POINTER(c_dbl)), lanes)
    need = lib.phgpu_ipm_source(*args, None, 0, ip(info))
    if need < 0:
        raise PhgpuError(f"phgpu_ipm_source failed: {last_error()}")
    buf = ctypes.create_string_buffer(need + 1)
    lib.phgpu_ipm_source(*args, buf, need + 1, ip(info))
    return buf.value.decode(), tuple(int(v) for v in info)


def default_options(**overrides):
    o = PhgpuOptions()
    check(load().phgpu_default_options(ctypes.byref(o)), "phgpu_default_options")
    for k, v in overrides.items():
        if not hasattr(o, k):
            raise KeyError(f"unknown solver option {k!r}; valid: {[f[0] for f in o._fields_]}")
        setattr(o, k, v)
    return o
