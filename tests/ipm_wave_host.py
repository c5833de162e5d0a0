"""Run the generated workgroup IPMs (jit_ipm_wave.hip.in, jit_ipm_blk.hip.in) on the CPU (TEST
INFRASTRUCTURE ONLY).

The library's generator (phgpu_ipm_source, lanes = 64 WPS) emits the text the handle
compiles with hipRTC; here it is compiled with g++ behind a shim: one std::thread per GPU
thread of the workgroup, a std::barrier for every workgroup synchronisation point (BSYNC,
__syncthreads) and for the workgroup sums (each thread posts its value, all sum the posts in
thread order), the hardware reciprocal as a division.  One scenario at a time.  The GPU
tests (test_gpu_ipm_wave.py) check the real kernel; test_ipm_wave_host.py uses this one to
check the kernel's arithmetic and its generated tables against the oracle on the CPU.
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
#include <barrier>
#include <mutex>
#include <thread>
#include <vector>
#define IPM_HOST_EMU 1
#define __global__
#define __device__
#define __forceinline__ inline
#define __launch_bounds__(x)
#define __shared__ static
struct wdim3 { unsigned x, y, z; };
static thread_local wdim3 threadIdx;
static wdim3 blockIdx, blockDim;
static std::barrier<>* g_bar = nullptr;
static std::mutex g_mu;
static inline void __syncthreads() { g_bar->arrive_and_wait(); }
#define VSYNC() __syncthreads()
#define BSYNC() __syncthreads()
#define __builtin_amdgcn_rcp(x) (1.0 / (x))
static inline int atomicAdd(int* p, int v) { std::lock_guard<std::mutex> l(g_mu); int o = *p; *p += v; return o; }
static inline unsigned long long atomicAdd(unsigned long long* p, unsigned long long v) { std::lock_guard<std::mutex> l(g_mu); unsigned long long o = *p; *p += v; return o; }
static inline unsigned long long atomicMax(unsigned long long* p, unsigned long long v) { std::lock_guard<std::mutex> l(g_mu); unsigned long long o = *p; if (v > o) *p = v; return o; }
template <class T> static inline T __shfl_xor(T, int, int) { return T(0); }  // (ipm_stats_roll without dst only)
static double g_post[4096];
template <int NV> static inline void w_bmax(double (&v)[NV], double*);
template <int NV> static inline void w_bsum(double (&v)[NV], double*) {
    for (int k = 0; k < NV; ++k) {
        g_bar->arrive_and_wait();
        g_post[threadIdx.x] = v[k];
        g_bar->arrive_and_wait();
        double a = 0.0;
        for (unsigned u = 0; u < blockDim.x; ++u) a += g_post[u];
        v[k] = a;
    }
    g_bar->arrive_and_wait();
}
template <int NS, int NM> static inline void w_bsum_max(double (&v)[NS], double (&u)[NM], double* r) {
    w_bsum(v, r);
    w_bmax(u, r);
}
template <int NV> static inline void w_bmax(double (&v)[NV], double*) {
    for (int k = 0; k < NV; ++k) {
        g_bar->arrive_and_wait();
        g_post[threadIdx.x] = v[k];
        g_bar->arrive_and_wait();
        double a = g_post[0];
        for (unsigned u = 1; u < blockDim.x; ++u) a = fmax(a, g_post[u]);
        v[k] = a;
    }
    g_bar->arrive_and_wait();
}
"""

DRIVER = r"""
extern "C" void wave_run(ipmw_params* p, long long S) {
    blockDim.x = WT;
    for (long long s = 0; s < S; ++s) {
        blockIdx.x = (unsigned)s;
        std::barrier<> bar(WT);
        g_bar = &bar;
        std::vector<std::thread> th;
        for (int t = 0; t < WT; ++t)
            th.emplace_back([p, t]() { threadIdx.x = (unsigned)t; KNAME(*p); });
        for (auto& x : th) x.join();
    }
}
"""

_cache = {}


def build(src, workdir="/tmp"):
    kname = "k_solve_ipm_blk" if "k_solve_ipm_blk" in src else "k_solve_ipm_wave"
    text = SHIM + src + f"#define KNAME {kname}\n" + DRIVER
    key = hashlib.sha1(text.encode()).hexdigest()[:16]
    if key in _cache:
        return _cache[key]
    cpp = os.path.join(workdir, f"ipm_wave_host_{key}.cpp")
    so = cpp[:-4] + ".so"
    if not os.path.exists(so):
        with open(cpp, "w") as f:
            f.write(text)
        subprocess.run(["g++", "-O1", "-std=c++20", "-w", "-shared", "-fPIC", "-pthread", "-o", so, cpp], check=True)
    lib = ctypes.CDLL(so)
    lib.wave_run.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
    _cache[key] = lib
    return lib


_VP = ctypes.c_void_p


class _Params(ctypes.Structure):
    _fields_ = ([(f, _VP) for f in ("A", "c", "q", "lb", "ub", "rl", "ru", "objc", "lbh", "ubh", "Dc", "Dr", "W", "rho",
                                  "xbar", "omega_in", "omega_out", "x_w", "y_w", "xout", "yout", "obj", "bound",
                                  "status", "iters", "fail_list", "fail_n", "zero3")]
                + [("S", ctypes.c_longlong), ("W_on", ctypes.c_int), ("prox_on", ctypes.c_int),
                   ("eps_rel", ctypes.c_double), ("eps_abs", ctypes.c_double), ("eps_tight", ctypes.c_double),
                   ("max_ipm", ctypes.c_int), ("x_in", _VP), ("y_in", _VP), ("stats", _VP), ("stats_zero", _VP)])


def solve(batch, lanes=64, W=None, rho=None, xbar=None, eps_rel=1e-9, eps_abs=1e-12, max_ipm=80, eps_tight=1e-13,
          x_in=None, y_in=None, stats=None):
    """Solve every scenario of a ScenarioBatch with the host-run workgroup kernel (lanes =
    its threads per scenario, 64 WPS).  Returns x [S, n], y [S, m], obj, bound, status
    (-1 = left for the fallback), iters.  ``stats`` (a list): the kernel's 8 statistics
    words are appended to it."""
    import mpisppy_amd._lib as L
    src, _ = L.ipm_source(batch, lanes)
    assert "#define WT " + str(lanes) in src, "the generator chose another workgroup size"
    lib = build(src)
    S, n, m, nn = batch.S, batch.n, batch.m, batch.nn
    T = lambda a: np.ascontiguousarray(np.asarray(a, dtype=np.float64).T)  # noqa: E731
    keep = []

    def ptr(a):
        keep.append(a)
        return a.ctypes.data

    A, c, q, lb, ub, rl, ru = (T(batch.A_val), T(batch.c), T(batch.q), T(batch.lb), T(batch.ub), T(batch.rl),
                               T(batch.ru))
    out = {k: np.zeros((d, S)) for k, d in (("x", n), ("y", m), ("xw", n), ("yw", m))}
    obj, bound, omo = np.zeros(S), np.zeros(S), np.zeros(S)
    status = np.full(S, 7, dtype=np.int32)
    iters = np.zeros(S, dtype=np.int32)
    fl = np.zeros(S, dtype=np.int32)
    cnt = np.zeros(4, dtype=np.int32)
    p = _Params()
    p.A, p.c, p.q, p.lb, p.ub, p.rl, p.ru = map(ptr, (A, c, q, lb, ub, rl, ru))
    p.objc = ptr(np.ascontiguousarray(batch.obj_const, dtype=np.float64))
    p.lbh, p.ubh, p.Dc, p.Dr = ptr(lb.copy()), ptr(ub.copy()), ptr(np.ones((n, S))), ptr(np.ones((m, S)))
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
    # two parities of the generated IPM_SC copies of IPM_SS words (phgpu.hip stats_word)
    sc = int(src.split("#define IPM_SC ", 1)[1].split()[0])
    ss = int(src.split("#define IPM_SS ", 1)[1].split()[0])
    stb = np.zeros(2 * sc * ss, dtype=np.uint64)
    keep.append(stb)
    p.stats, p.stats_zero = stb.ctypes.data, stb[sc * ss:].ctypes.data
    lib.wave_run(ctypes.byref(p), S)
    if stats is not None:
        cp = stb[:sc * ss].reshape(sc, ss)[:, :8]
        words = cp.sum(0)
        words[5] = cp[:, 5].max()
        stats.append(words)
    st = status.copy()
    st[fl[:cnt[0]]] = -1
    return out["x"].T.copy(), out["y"].T.copy(), obj, bound, st, iters
