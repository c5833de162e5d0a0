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
    ]


OPTIMAL, ITER_LIMIT, PRIMAL_INFEASIBLE, DUAL_INFEASIBLE = 0, 1, 2, 3
SHARED_MATRIX = 1          # phgpu_create2 flag (include/phgpu.h)

# every symbol include/phgpu.h declares (tests check the library exports them all)
EXPORTS = ["phgpu_default_options", "phgpu_create", "phgpu_create2", "phgpu_set_scenarios", "phgpu_set_ph_state",
           "phgpu_solve", "phgpu_solve_deferred", "phgpu_commit", "phgpu_ph_reduce", "phgpu_ph_update",
           "phgpu_expectations",
           "phgpu_fix_nonants", "phgpu_status_counts", "phgpu_destroy", "phgpu_last_error", "phgpu_workspace_bytes",
           "phgpu_kernel_info"]

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
    lib.phgpu_set_ph_state.argtypes = [c_vp, c_vp, c_vp, c_vp, c_int, c_int]
    lib.phgpu_solve.argtypes = [c_vp, ctypes.POINTER(PhgpuOptions), c_int, c_vp, c_vp, c_vp, c_vp,
                                c_vp, c_vp, c_vp]
    lib.phgpu_solve_deferred.argtypes = lib.phgpu_solve.argtypes
    lib.phgpu_commit.argtypes = [c_vp]
    lib.phgpu_ph_reduce.argtypes = [c_vp, c_vp, c_vp, c_vp]
    lib.phgpu_ph_update.argtypes = [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_vp]
    lib.phgpu_expectations.argtypes = [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]
    lib.phgpu_fix_nonants.argtypes = [c_vp, c_vp, c_vp]
    lib.phgpu_status_counts.argtypes = [c_vp, c_vp, c_vp, c_vp]
    lib.phgpu_destroy.argtypes = [c_vp]
    lib.phgpu_last_error.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
    lib.phgpu_workspace_bytes.argtypes = [c_vp]
    lib.phgpu_workspace_bytes.restype = c_i64
    lib.phgpu_kernel_info.argtypes = [c_vp, P_i32]
    for name in EXPORTS:
        if name != "phgpu_workspace_bytes":
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


def default_options(**overrides):
    o = PhgpuOptions()
    check(load().phgpu_default_options(ctypes.byref(o)), "phgpu_default_options")
    for k, v in overrides.items():
        if not hasattr(o, k):
            raise KeyError(f"unknown solver option {k!r}; valid: {[f[0] for f in o._fields_]}")
        setattr(o, k, v)
    return o
