"""Run the generated path-6 kernel source on the CPU (TEST / TOOL INFRASTRUCTURE ONLY).

The library's generator (phgpu_ipm_source) emits the same text the handle compiles with
hipRTC; here the IPM part is compiled with g++ behind a small shim (HIP qualifiers
dropped, one "lane" per call, the hardware reciprocal as a division) and run scenario by
scenario, so the kernel's arithmetic can be checked against the oracle without a GPU.
The GPU tests (test_gpu_ipm.py) check the real thing; test_ipm_codegen.py uses this.
"""
import ctypes
import hashlib
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy-1_amd"))

SHIM = r"""
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#define __global__
#define __device__
#define __forceinline__ inline
#define __launch_bounds__(x)
struct ipm_dim3 { unsigned x, y, z; };
static ipm_dim3 blockIdx, threadIdx, blockDim;
#define __builtin_amdgcn_rcp(x) (1.0 / (x))
static inline int atomicAdd(int* p, int v) { int o = *p; *p += v; return o; }
static inline unsigned long long atomicAdd(unsigned long long* p, unsigned long long v) { unsigned long long o = *p; *p += v; return o; }
static inline unsigned long long atomicMax(unsigned long long* p, unsigned long long v) { unsigned long long o = *p; if (v > o) *p = v; return o; }
static inline unsigned long long __ballot(bool b) { return b ? 1ull : 0ull; }
static inline int __popcll(unsigned long long v) { return __builtin_popcountll(v); }
template <class T> static inline T __shfl_xor(T, int, int) { return T(0); }  // one lane: the others contribute 0
template <class T> static inline T __shfl_down(T, int, int) { return T(0); }
template <class T> static inline T __shfl(T v, int, int) { return v; }
static inline bool __any(bool b) { return b; }
#define __shared__ static
static inline void __syncthreads() {}
static ipm_dim3 gridDim;
#define __HIP_MEMORY_SCOPE_AGENT 0
#define __HIP_MEMORY_SCOPE_SYSTEM 0
template <class T> static inline T __hip_atomic_exchange(T* p, T v, int, int) { T o = *p; *p = v; return o; }
template <class T> static inline T __hip_atomic_fetch_add(T* p, T v, int, int) { T o = *p; *p += v; return o; }
template <class T> static inline void __hip_atomic_store(T* p, T v, int, int) { *p = v; }
#define PHS_ORDER(v) (void)(v)
"""

DRIVER = r"""
extern "C" void ipm_run(ipm_params* p, long long S) {
    blockDim.x = 256;
    for (long long s = 0; s < S; ++s) {
        blockIdx.x = (unsigned)(s / 256);
        threadIdx.x = (unsigned)(s % 256);
        k_solve_ipm(*p);
    }
}
"""

_cache = {}


def build(src, workdir="/tmp"):
    """Compile the IPM part of a generated path-6 source for the host; returns the CDLL."""
    part = src[src.index("#define IPM_GAM"):]
    text = SHIM + part + DRIVER
    key = hashlib.sha1(text.encode()).hexdigest()[:16]
    if key in _cache:
        return _cache[key]
    cpp = os.path.join(workdir, f"ipm_host_{key}.cpp")
    so = cpp[:-4] + ".so"
    if not os.path.exists(so):
        with open(cpp, "w") as f:
            f.write(text)
        subprocess.run(["g++", "-O1", "-std=c++17", "-w", "-shared", "-fPIC", "-o", so, cpp], check=True)
    lib = ctypes.CDLL(so)
    lib.ipm_run.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
    _cache[key] = lib
    return lib


_VP = ctypes.c_void_p


class _Params(ctypes.Structure):
    _fields_ = ([(f, _VP) for f in ("A", "c", "q", "lb", "ub", "rl", "ru", "objc", "lbh", "ubh", "Dc", "Dr", "W", "rho",
                                  "xbar", "omega_in", "omega_out", "x_w", "y_w", "xout", "yout", "obj", "bound",
                                  "status", "iters", "fail_list", "fail_n", "zero3")]
                + [("S", ctypes.c_longlong), ("W_on", ctypes.c_int), ("prox_on", ctypes.c_int),
                   ("eps_rel", ctypes.c_double), ("eps_abs", ctypes.c_double), ("eps_tight", ctypes.c_double),
                   ("max_ipm", ctypes.c_int), ("x_in", _VP), ("y_in", _VP), ("stats", _VP), ("stats_zero", _VP),
                   # x̄ partials of the epilogue (null here: the host run skips them)
                   ("xp", _VP), ("xp_node", _VP), ("xp_dirty", _VP), ("pcoef", _VP), ("node_of", _VP),
                   # the folded PH step (jit_ph_step.hip.in ph_step; on = 0 here)
                   ("ph_on", ctypes.c_int), ("ph_update_W", ctypes.c_int)]
                + [(f"ph_{f}", _VP) for f in ("xprev", "xp", "xp_dirty")] + [("ph_xp_n", ctypes.c_longlong),
                   ("ph_C", ctypes.c_int)] + [(f"ph_{f}", _VP) for f in ("node_buf", "nb_idx")]
                + [("ph_nb_half", ctypes.c_longlong)] + [(f"ph_{f}", _VP) for f in ("W", "xbar", "rho", "conv", "stats_dst")]
                + [("ph_scale", ctypes.c_double), ("ph_cpart", _VP), ("ph_cnt", _VP)])


def solve(batch, W=None, rho=None, xbar=None, eps_rel=1e-9, eps_abs=1e-12, max_ipm=80, eps_tight=1e-13,
          x_in=None, y_in=None):
    """Solve every scenario of a ScenarioBatch with the host-compiled kernel.  W / rho /
    xbar: [S, nn] (None = that PH term off); x_in / y_in [S, n] / [S, m]: the warm state
    (the previous solve's x and y).  Returns x [S, n], y [S, m], obj, bound,
    status (-1 = left for the PDHG fallback), iters."""
    import mpisppy_amd._lib as L
    src, _ = L.ipm_source(batch)
    lib = build(src)
    S, n, m, nn = batch.S, batch.n, batch.m, batch.nn
    T = lambda a: np.ascontiguousarray(np.asarray(a, dtype=np.float64).T)  # noqa: E731  [S, k] -> [k][S]
    keep = []

    def ptr(a):
        keep.append(a)
        return a.ctypes.data

    A, c, q, lb, ub, rl, ru = (T(batch.A_val), T(batch.c), T(batch.q), T(batch.lb), T(batch.ub), T(batch.rl),
                               T(batch.ru))
    ones_n = np.ones((n, S))
    ones_m = np.ones((m, S))
    out = {k: np.zeros((d, S)) for k, d in (("x", n), ("y", m), ("xw", n), ("yw", m))}
    obj, bound, omo = np.zeros(S), np.zeros(S), np.zeros(S)
    status = np.full(S, 7, dtype=np.int32)
    iters = np.zeros(S, dtype=np.int32)
    fl = np.zeros(S, dtype=np.int32)
    cnt = np.zeros(4, dtype=np.int32)
    p = _Params()
    p.A, p.c, p.q, p.lb, p.ub, p.rl, p.ru = map(ptr, (A, c, q, lb, ub, rl, ru))
    p.objc = ptr(np.ascontiguousarray(batch.obj_const, dtype=np.float64))
    p.lbh, p.ubh, p.Dc, p.Dr = ptr(lb.copy()), ptr(ub.copy()), ptr(ones_n), ptr(ones_m)
    zero = np.zeros((max(nn, 1), S))
    p.W = ptr(T(W) if W is not None else zero)
    p.rho = ptr(T(rho) if rho is not None else zero)
    p.xbar = ptr(T(xbar) if xbar is not None else zero)
    p.omega_in, p.omega_out = ptr(np.ones(S)), ptr(omo)
    p.x_w, p.y_w, p.xout, p.yout = ptr(out["xw"]), ptr(out["yw"]), ptr(out["x"]), ptr(out["y"])
    p.obj, p.bound, p.status, p.iters = ptr(obj), ptr(bound), ptr(status), ptr(iters)
    p.fail_list, p.fail_n, p.zero3 = ptr(fl), cnt[0:].ctypes.data, cnt[1:].ctypes.data
    keep.append(cnt)
    p.S, p.W_on, p.prox_on = S, int(W is not None), int(rho is not None)
    p.eps_rel, p.eps_abs, p.max_ipm, p.eps_tight = eps_rel, eps_abs, max_ipm, eps_tight
    p.x_in = ptr(T(x_in)) if x_in is not None else None
    p.y_in = ptr(T(y_in)) if y_in is not None else None
    st16 = np.zeros(16, dtype=np.uint64)
    keep.append(st16)
    p.stats, p.stats_zero = st16.ctypes.data, st16[8:].ctypes.data
    lib.ipm_run(ctypes.byref(p), S)
    st = status.copy()
    st[fl[:cnt[0]]] = -1
    return out["x"].T.copy(), out["y"].T.copy(), obj, bound, st, iters
