// phgpu.hip -- MI355X (gfx950) kernels + C-ABI for the batched PH hot path.
//
// Design: every local scenario is one LP/QP that shares the CSR
// pattern of the rank; per-scenario arrays are stored scenario-fastest ([k][S]) so
// that the 64 lanes of a wavefront process 64 scenarios and every load/store of a
// pattern position is one coalesced 512-byte access, while the pattern itself
// (row_ptr, col_idx, col_ptr, row_idx, perm) is wave-uniform and goes through the
// scalar cache.  One lane runs its scenario's whole restarted-Halpern PDHG solve in a
// single launch (no grid-wide synchronisation: scenarios are independent), with its
// own primal weight, restart state and KKT termination test.
//
// Reference behaviour replaced (mpi-sppy, /root/reference):
//   SPOpt.solve_loop / solve_one        spopt.py:226-307 / 85-223
//   PH objective terms                  phbase.py:617-699
//   _Compute_Xbar / Update_W / conv     phbase.py:27-107, 293-343
//   Ebound / Eobjective / E1 / feas     spopt.py:310-439
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdarg.h>
#include <string.h>
#include <new>
#include <stdlib.h>
#include <algorithm>
#include <chrono>
#include <vector>
#include <mutex>
#include <map>
#include <string>
#include <cctype>

#include "phgpu.h"

#define WAVE 64
#define BLOCK 64
#define ORDER_BINS 256  // counting-sort bins of the longest-first work queue (solve_reg.inc)
#define XL_T 1024        // threads per block of k_ph_update_local at most
#define XL_NN_MAX 16     // nonants per scenario at most for the folded x̄ paths (k_ph_update_local, IPM epilogues)
#define XL_PF 4          // k_ph_update_local: nonants whose operands are loaded ahead of the x̄ sums
#define XP_CHUNK_MIN 16  // smallest x̄-partial chunk of the IPM epilogues (256 / 16 lanes)

// ------------------------------------------------------------------ errors
static thread_local char g_err[512] = {0};

static int set_err(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

#define HIPCHK(call)                                                                 \
    do {                                                                             \
        hipError_t e_ = (call);                                                      \
        if (e_ != hipSuccess)                                                        \
            return set_err(-2, "%s failed: %s (%s:%d)", #call, hipGetErrorString(e_), \
                           __FILE__, __LINE__);                                      \
    } while (0)

// ------------------------------------------------------------------ state
struct jit_module;  // solve_jit.inc: the hipRTC-compiled path-5 kernel of a handle
struct ipm_module;  // solve_ipm.inc: the hipRTC-compiled path-6 module of a handle

struct phgpu_state {
    int device;
    void* rccl[2];                 // the library's RCCL communicators over the ranks (comm_rccl.inc), or null
    int64_t S;
    int n, m, nnz, nn, depth, num_nodes, nlen_max;
    // shared pattern
    int32_t *row_ptr, *col_idx, *col_ptr, *row_idx, *perm, *row_of;
    int32_t *nonant_col, *nonant_depth, *nonant_off, *nonant_slot;
    // per-scenario problem data (library copies)
    double *A, *c, *lb, *ub, *rl, *ru, *q, *objc, *prob, *pcoef;
    // per-nonant probability coefficients ([nn][S], caller-owned; null: the per-node pcoef),
    // the variable probabilities of spbase.py:394-424 (phgpu_set_nonant_probs)
    const double* pvar;
    int32_t* node_of;
    // scaling
    double *Ah_csr, *Ah_csc, *Dr, *Dc, *normA;
    double *lbh, *ubh, *rlh, *ruh;
    // per-solve effective objective (scaled) + iterates (scaled)
    double *ch, *qh;
    double *x, *x0, *xe, *xt, *aty, *aty0, *y, *y0, *yt;
    double* omega;
    // reductions
    double* part;       // [nwaves * max(2*nn, 5)]
    int32_t* part_node; // [nwaves * nn]
    int64_t nwaves;
    int64_t ws_bytes;
    // register-resident path (solve_reg.inc): lane plan, -1 instance = unavailable
    int reg_inst;
    int reg_L, reg_kc, reg_zc, reg_kr, reg_zr;
    int32_t *pl_col_k, *pl_col_r, *pl_row_k, *pl_row_c;
    // workgroup-per-scenario path (solve_wg.inc): -1 instance = unavailable
    int wg_inst, wg_long;
    int32_t *wg_col_id, *wg_row_id, *wg_col_long, *wg_row_long, *wg_col_k, *wg_col_r, *wg_row_k, *wg_row_c;
    int default_kernel;  // 1 global, 2 register (L <= 64), 3 workgroup per scenario
    // scenario-major records of the workgroup path: one contiguous record
    // per scenario, so a workgroup loads / writes back its scenario in full lines
    double* pk;
    int64_t pk_stride;
    int pk_A, pk_C, pk_Q, pk_DC, pk_LB, pk_UB, pk_RL, pk_RU, pk_DR, pk_RLH, pk_RUH, pk_X, pk_Y, pk_W, pk_RHO,
        pk_XB;
    int last_path;       // path of the last solve (whose layout holds the warm start)
    int scen_set;
    // 1 if some wave of local scenarios spans two nodes at a nonant's depth (its x̄
    // contributions go to node_buf by atomics, so node_buf is cleared by a memset first);
    // 0 if none does (k_xbar_partial clears node_buf itself); -1 not yet known
    int xbar_mixed;
    // 1 if every nonant's local scenarios share one node (two-stage problems): a single
    // rank's x̄ final sum can then be folded into the update kernel (phgpu_ph_step_local)
    int xbar_single;
    int* qhead;  // work-queue head of the persistent solve kernel
    int num_cus;
    int occ_cache[8];  // workgroups per CU of each solve kernel (0 = not queried yet)
    // shared-matrix handle (PHGPU_SHARED_MATRIX, path 4: solve_stream.inc): one scaled A
    // (A / Ah_csr / Ah_csc [nnz], Dr [m], Dc [n]) for all scenarios; the shared base of
    // the column / row data (sh_col: ch qh lbh ubh, sh_row: rlh ruh rl ru, scenario 0);
    // per-scenario columns P (cmap[j] = index or -1, pcol) and rows R (rmap, prow)
    int shared;
    int np, nr;
    int32_t *cmap, *rmap, *pcol, *prow;
    double *sh_col, *sh_row, *sh_norm, *sh_v, *sh_u, *sh_w, *sh_part;
    // sliced-ELL copies of the scaled matrix for the two streaming passes: slice = 64
    // consecutive columns (rows), padded to its longest; entry k of slice member l at
    // off[slice] + 64 k + l (coalesced); *_src = CSC / CSR position of the entry, -1 = pad
    int nsl_c, nsl_r, nent_c, nent_r;
    int32_t *cs_off, *cs_len, *cs_idx, *cs_src, *rs_off, *rs_len, *rs_idx, *rs_src;
    double *cs_val, *rs_val;
    // slices of each pass per wave of the streaming workgroup (balanced by entries):
    // wave w takes cw_slc[cw_ptr[w] .. cw_ptr[w+1]) (rw_* for rows)
    int32_t *cw_ptr, *cw_slc, *rw_ptr, *rw_slc;
    int32_t *sk_iters, *sk_order;  // PDHG iterations of the last solve / longest-first queue order
    double* split_part;            // grid-sum partials of the split streaming form ([ncl][2][K][8]) + barriers
    size_t split_need;             // its size in doubles
    int last_cluster;              // path 4: workgroups per scenario of the last solve's cluster form (0: none)
    int32_t* sk_bins;              // [2 parities][2][ORDER_BINS] counting-sort histogram / fill counters (path 2)
    int order_parity;              // which half of sk_bins the next register-path solve uses
    int warm_rec;                  // the warm start lives in the records pk (paths 2r, 3), else in x / y
    int last_rec;                  // queue mode of the last register-path solve (-1 none yet)
    double* sk;  // stream records: X X0 U XT | Y Y0 YT | PC (8 per P column) | PR (4 per R row)
    int64_t sk_stride, sk_X, sk_X0, sk_U, sk_XT, sk_Y, sk_Y0, sk_YT, sk_PC, sk_PR, sk_cap;
    // PH state (caller-owned)
    const double *W, *rho, *xbar;
    int W_on, prox_on;
    int have_solution;
    // Warm-start slots (include/phgpu.h phgpu_solve_deferred / phgpu_commit).  The warm
    // state a solve starts from -- the iterate x / y ([k][S] arrays or the records' x^ / y^
    // fields), the primal weight omega and the queue predictor sk_iters -- lives in slot
    // wslot; the fields above (x, y, omega, sk_iters, pk_X, pk_Y, have_solution, warm_rec)
    // are bound to it at the start of every solve.  A solve writes its warm state to the
    // *_w targets below: the same slot, or the other one for a deferred (speculative)
    // solve, which becomes current only at phgpu_commit.
    double *xs[2], *ys[2], *oms[2];
    int32_t* its_s[2];
    int pkXs[2], pkYs[2];
    int have_s[2], warm_rec_s[2];
    int wslot, wq;       // read slot / write slot of the current solve
    int pending;         // slot of an uncommitted deferred solve, -1 none
    double *xw, *yw, *omega_w;
    int32_t* its_w;
    int pk_XW, pk_YW;
    // path 5 (solve_jit.inc): the pattern-specialised module, and whether the column /
    // row kinds it was built for still describe the data (reset by phgpu_set_scenarios)
    jit_module* jit;
    int jit_kinds_valid;
    // path 6 (solve_ipm.inc): the interior-point module; whether the data flags it was
    // built for still hold (reset by phgpu_set_scenarios); factor entries of the pattern
    // (0: not eligible); 1 once a compiled module spilled (path 6 is then not the
    // default); the fallback list [S] and its counters {fail_n[2], qhead[2]} by parity
    ipm_module* ipm;
    // phgpu_ph_loop: the IPM_LOOP module (built on first use from the one-lane source) and its
    // buffers {gpart [blocks * 16], gpub [16], conv_hist [cap] | gsync [2], loop_out [2],
    // loop_its [PHGPU_STATS_WORDS]}
    ipm_module* ipm_loop;
    double* loop_dbl;
    int64_t loop_dbl_n;
    unsigned long long* loop_cnt;
    int ipm_flags_valid, ipm_nf, ipm_off, ipm_parity, ipm_spill1;
    // the one-lane module's slack reciprocals in LDS (IPM_LDS_ISL, solve_ipm.inc ipm_prepare):
    // 0 not tried, 1 on (its module spills less), -1 tried and not kept; with the spill
    // bytes of the register-only module it was compared with
    int ipm_lds, ipm_lds_ref;
    int ipm_wave;  // waves per scenario of the workgroup IPMs for medium scenarios (0: not eligible;
                   // jit_ipm_blk.hip.in for block-angular patterns, else jit_ipm_wave.hip.in)
    int32_t *ipm_list, *ipm_cnt;
    // solve statistics (phgpu_solve_stats): path 6 accumulates them in its kernels (by
    // parity, [2][8]); other paths get them from k_solve_stats over the last solve's
    // status / iters outputs into stats_gen[8].  last_stats: where the last solve's are
    // (null: compute on request)
    // ipm_stats: two parities of PHGPU_STATS_COPIES copies of the 8 statistics words (the
    // path-6 kernels spread their per-wave atomics over the copies, stats_word sums them)
    unsigned long long *ipm_stats, *stats_gen, *last_stats;
    unsigned long long* ipm_prof;  // PHGPU_IPM_PROF: per-wave timelines of IPM_PROF modules
    long long ipm_prof_n;
    const int32_t *last_status, *last_iters;
    // x̄ partial sums written by the path-6 kernels' epilogue, per warm slot:
    // [chunks * nn * 2] sums of pcoef x and pcoef x^2, node tags [chunks * nn], fallback
    // flags [chunks]; valid for the x buffer xp_x[slot] when xp_C[slot] (the chunk size) > 0
    double* xp[2];
    int32_t *xp_node[2], *xp_dirty[2];
    const double* xp_x[2];
    int xp_C[2];
    int64_t xp_n[2];
    // the update kernels' last-block reduction of conv: per-block partials and a counter
    double* cpart_blk;
    int32_t* blk_cnt;
    // a one-rank PH step deferred by phgpu_ph_step_defer: folded into the next path-6
    // deferred solve's prologue (jit_ph_step.hip.in) when it can be, else run by
    // phgpu_ph_step_local before that solve or before any other call
    struct ph_pending {
        int active = 0;
        const double* x = nullptr;
        double *node_buf = nullptr, *xbar = nullptr, *W = nullptr;
        const double* rho = nullptr;
        int update_W = 0;
        double* conv = nullptr;
        int64_t* stats = nullptr;
        hipStream_t stream = nullptr;
    } pend;
    int fuse_now;      // ipm_launch folds pend into this launch
    int64_t folded;    // PH steps folded into solve launches so far (phgpu_ipm_info)
    int32_t* nb_idx;   // [nn] node_buf index (node of the local scenarios, offset) of nonant k (two-stage)
};

#define IX(k) ((size_t)(k) * (size_t)S + (size_t)s)

// ------------------------------------------------------------------ device helpers
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, WAVE);
    return v;
}

__device__ __forceinline__ double clampd(double v, double lo, double hi) {
    return fmin(fmax(v, lo), hi);
}

// y-part of the PDHG dual step for a ranged row rl <= a'x <= ru:
// maximise -y*ax + (rl y+ - ru y-) - (y - yk)^2/(2 sig)
__device__ __forceinline__ double dual_prox(double v, double sig, double rlh, double ruh) {
    double a = v + sig * rlh;
    double b = v + sig * ruh;
    return a > 0.0 ? a : (b < 0.0 ? b : 0.0);
}

// contribution of row i to the Lagrangian dual objective: min_{s in [rl,ru]} y s,
// projected (an infinite side with the wrong-sign multiplier contributes 0)
__device__ __forceinline__ double row_dual_term(double y, double rl, double ru) {
    if (y > 0.0) return isfinite(rl) ? rl * y : 0.0;
    if (y < 0.0) return isfinite(ru) ? ru * y : 0.0;
    return 0.0;
}

// min over x in [lb,ub] of r x + q/2 x^2 (projected for infinite sides when q == 0)
__device__ __forceinline__ double col_dual_term(double r, double qq, double lb, double ub) {
    if (qq > 0.0) {
        double xm = clampd(-r / qq, lb, ub);
        return r * xm + 0.5 * qq * xm * xm;
    }
    if (r > 0.0) return isfinite(lb) ? r * lb : 0.0;
    if (r < 0.0) return isfinite(ub) ? r * ub : 0.0;
    return 0.0;
}

// ---------------------------------------------------------- infeasibility certificates
// PDLP-style tests on the fixed-point residual d = T(z) - z, which for an infeasible or
// unbounded problem converges to the minimal displacement of the PDHG operator (its dual
// part is a Farkas ray, its primal part a ray of descent).  All quantities are in the
// original space.  The reference marks such a scenario infeasible (spopt.py:175-194) and
// Iter0 stops on it (phbase.py:818-823).
//
// Primal infeasibility: dual ray d (rows), ray reduced cost r = -(A^T d) (columns).  The
// ray objective sum_i min_{s in [rl,ru]} s d_i + sum_j min_{x in [lb,ub]} r_j x_j must be
// > 0 while every component that points at an infinite side (where the min is -inf) is
// ~0: certificate if sqrt(viol2) <= eps * obj.
__device__ __forceinline__ void ray_row_terms(double d, double rl, double ru, double& obj, double& viol2) {
    if (d > 0.0) {
        if (isfinite(rl)) obj += rl * d;
        else viol2 += d * d;
    } else if (d < 0.0) {
        if (isfinite(ru)) obj += ru * d;
        else viol2 += d * d;
    }
}
__device__ __forceinline__ void ray_col_terms(double r, double lb, double ub, double& obj, double& viol2) {
    if (r > 0.0) {
        if (isfinite(lb)) obj += lb * r;
        else viol2 += r * r;
    } else if (r < 0.0) {
        if (isfinite(ub)) obj += ub * r;
        else viol2 += r * r;
    }
}
// Dual infeasibility (unbounded primal): primal ray dx with c'dx < 0, Q dx = 0, A dx in
// the recession cone of [rl, ru] and dx in that of [lb, ub]; squared distance to the cone.
__device__ __forceinline__ double recession_viol2(double a, double lo, double hi) {
    double v = 0.0;
    if (isfinite(lo) && a < 0.0) v += a * a;
    if (isfinite(hi) && a > 0.0) v += a * a;
    return v;
}
__device__ __forceinline__ bool is_certificate(double obj, double viol2, double eps) {
    return obj > 0.0 && viol2 <= (eps * obj) * (eps * obj);
}

// ------------------------------------------------------------------ setup kernel
// Per scenario: copy A, Ruiz (iters) + Pock-Chambolle(alpha=1) scaling, scaled
// bounds, CSC copy of the scaled values and ||A_scaled||_2 by power iteration.
__global__ void __launch_bounds__(BLOCK) k_setup(phgpu_state st, int ruiz_iters, int power_iters) {
    const int64_t S = st.S;
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S) return;
    const int n = st.n, m = st.m, nnz = st.nnz;
    double* Ah = st.Ah_csr;
    for (int k = 0; k < nnz; ++k) Ah[IX(k)] = st.A[IX(k)];
    for (int i = 0; i < m; ++i) st.Dr[IX(i)] = 1.0;
    for (int j = 0; j < n; ++j) st.Dc[IX(j)] = 1.0;
    // temporaries: row factors in yt, column factors in xt
    for (int pass = 0; pass <= ruiz_iters; ++pass) {
        const bool pc = (pass == ruiz_iters);  // last pass: Pock-Chambolle alpha = 1
        for (int i = 0; i < m; ++i) {
            double a = 0.0;
            for (int k = st.row_ptr[i]; k < st.row_ptr[i + 1]; ++k) {
                double v = fabs(Ah[IX(k)]);
                a = pc ? a + v : fmax(a, v);
            }
            st.yt[IX(i)] = a > 0.0 ? 1.0 / sqrt(a) : 1.0;
        }
        for (int j = 0; j < n; ++j) {
            double a = 0.0;
            for (int kc = st.col_ptr[j]; kc < st.col_ptr[j + 1]; ++kc) {
                double v = fabs(Ah[IX(st.perm[kc])]);
                a = pc ? a + v : fmax(a, v);
            }
            st.xt[IX(j)] = a > 0.0 ? 1.0 / sqrt(a) : 1.0;
        }
        for (int i = 0; i < m; ++i) {
            const double ri = st.yt[IX(i)];
            st.Dr[IX(i)] *= ri;
            for (int k = st.row_ptr[i]; k < st.row_ptr[i + 1]; ++k)
                Ah[IX(k)] *= ri * st.xt[IX(st.col_idx[k])];
        }
        for (int j = 0; j < n; ++j) st.Dc[IX(j)] *= st.xt[IX(j)];
    }
    for (int kc = 0; kc < nnz; ++kc) st.Ah_csc[IX(kc)] = Ah[IX(st.perm[kc])];
    for (int j = 0; j < n; ++j) {
        const double d = st.Dc[IX(j)];
        st.lbh[IX(j)] = st.lb[IX(j)] / d;
        st.ubh[IX(j)] = st.ub[IX(j)] / d;
        st.x[IX(j)] = 0.0;
    }
    for (int i = 0; i < m; ++i) {
        const double d = st.Dr[IX(i)];
        st.rlh[IX(i)] = st.rl[IX(i)] * d;
        st.ruh[IX(i)] = st.ru[IX(i)] * d;
        st.y[IX(i)] = 0.0;
    }
    // power iteration on A^T A (v in xe, A v in yt, A^T A v in xt)
    for (int j = 0; j < n; ++j) st.xe[IX(j)] = 1.0 + 0.5 * sin(1.7 * j);
    double lam = 0.0;
    for (int it = 0; it < power_iters; ++it) {
        for (int i = 0; i < m; ++i) {
            double a = 0.0;
            for (int k = st.row_ptr[i]; k < st.row_ptr[i + 1]; ++k)
                a += Ah[IX(k)] * st.xe[IX(st.col_idx[k])];
            st.yt[IX(i)] = a;
        }
        double nv = 0.0;
        for (int j = 0; j < n; ++j) {
            double a = 0.0;
            for (int kc = st.col_ptr[j]; kc < st.col_ptr[j + 1]; ++kc)
                a += st.Ah_csc[IX(kc)] * st.yt[IX(st.row_idx[kc])];
            st.xt[IX(j)] = a;
            nv += a * a;
        }
        nv = sqrt(nv);
        lam = nv;  // ||A^T A v|| with ||v|| = 1 (after the first pass)
        const double inv = nv > 0.0 ? 1.0 / nv : 0.0;
        for (int j = 0; j < n; ++j) st.xe[IX(j)] = st.xt[IX(j)] * inv;
    }
    // power iteration under-estimates ||A||_2 (slowly when the top singular values are
    // close); 1% margin keeps tau * sigma * ||A||^2 < 1 (a violated step condition makes
    // the reflected Halpern iteration diverge)
    st.normA[s] = lam > 0.0 ? 1.01 * sqrt(lam) : 1.0;
    st.omega[s] = 1.0;
}

// ------------------------------------------------------------------ parallel setup
// k_setup's algorithm with (row | column | nonzero, scenario) pairs over threads, the
// scenario fastest (coalesced [k][S] accesses): for patterns with many nonzeros, where
// one lane per scenario walking 2 nnz x 200 power steps serially is the bottleneck
// (farmer cm=64: 439 ms).  Same operations in the same order per scenario, so the
// scaled problem and ||A|| are bit-identical to k_setup's.
#define SU_T 256
__global__ void __launch_bounds__(SU_T) k_su_init(phgpu_state st) {
    const int64_t S = st.S;
    const int64_t t = (int64_t)blockIdx.x * SU_T + threadIdx.x;
    const int64_t K = (int64_t)(st.nnz > st.n ? (st.nnz > st.m ? st.nnz : st.m) : (st.n > st.m ? st.n : st.m));
    if (t >= K * S) return;
    const int64_t k = t / S, s = t - k * S;
    if (k < st.nnz) st.Ah_csr[IX(k)] = st.A[IX(k)];
    if (k < st.m) st.Dr[IX(k)] = 1.0;
    if (k < st.n) st.Dc[IX(k)] = 1.0;
}

// row factors into yt (pc: Pock-Chambolle sum, else Ruiz max)
__global__ void __launch_bounds__(SU_T) k_su_rowfac(phgpu_state st, int pc) {
    const int64_t S = st.S;
    const int64_t t = (int64_t)blockIdx.x * SU_T + threadIdx.x;
    if (t >= (int64_t)st.m * S) return;
    const int i = (int)(t / S);
    const int64_t s = t - (int64_t)i * S;
    double a = 0.0;
    for (int k = st.row_ptr[i]; k < st.row_ptr[i + 1]; ++k) {
        const double v = fabs(st.Ah_csr[IX(k)]);
        a = pc ? a + v : fmax(a, v);
    }
    st.yt[IX(i)] = a > 0.0 ? 1.0 / sqrt(a) : 1.0;
}

__global__ void __launch_bounds__(SU_T) k_su_colfac(phgpu_state st, int pc) {
    const int64_t S = st.S;
    const int64_t t = (int64_t)blockIdx.x * SU_T + threadIdx.x;
    if (t >= (int64_t)st.n * S) return;
    const int j = (int)(t / S);
    const int64_t s = t - (int64_t)j * S;
    double a = 0.0;
    for (int kc = st.col_ptr[j]; kc < st.col_ptr[j + 1]; ++kc) {
        const double v = fabs(st.Ah_csr[IX(st.perm[kc])]);
        a = pc ? a + v : fmax(a, v);
    }
    st.xt[IX(j)] = a > 0.0 ? 1.0 / sqrt(a) : 1.0;
}

__global__ void __launch_bounds__(SU_T) k_su_apply(phgpu_state st) {
    const int64_t S = st.S;
    const int64_t t = (int64_t)blockIdx.x * SU_T + threadIdx.x;
    const int64_t K = (int64_t)(st.nnz > st.n ? (st.nnz > st.m ? st.nnz : st.m) : (st.n > st.m ? st.n : st.m));
    if (t >= K * S) return;
    const int64_t k = t / S, s = t - k * S;
    if (k < st.nnz) st.Ah_csr[IX(k)] *= st.yt[IX(st.row_of[k])] * st.xt[IX(st.col_idx[k])];
    if (k < st.m) st.Dr[IX(k)] *= st.yt[IX(k)];
    if (k < st.n) st.Dc[IX(k)] *= st.xt[IX(k)];
}

// CSC copy, scaled bounds, zero iterates, power-iteration start vector
__global__ void __launch_bounds__(SU_T) k_su_finish(phgpu_state st) {
    const int64_t S = st.S;
    const int64_t t = (int64_t)blockIdx.x * SU_T + threadIdx.x;
    const int64_t K = (int64_t)(st.nnz > st.n ? (st.nnz > st.m ? st.nnz : st.m) : (st.n > st.m ? st.n : st.m));
    if (t >= K * S) return;
    const int64_t k = t / S, s = t - k * S;
    if (k < st.nnz) st.Ah_csc[IX(k)] = st.Ah_csr[IX(st.perm[k])];
    if (k < st.n) {
        const double d = st.Dc[IX(k)];
        st.lbh[IX(k)] = st.lb[IX(k)] / d;
        st.ubh[IX(k)] = st.ub[IX(k)] / d;
        st.x[IX(k)] = 0.0;
        st.xe[IX(k)] = 1.0 + 0.5 * sin(1.7 * (int)k);
    }
    if (k < st.m) {
        const double d = st.Dr[IX(k)];
        st.rlh[IX(k)] = st.rl[IX(k)] * d;
        st.ruh[IX(k)] = st.ru[IX(k)] * d;
        st.y[IX(k)] = 0.0;
    }
}

__global__ void __launch_bounds__(SU_T) k_su_rowmv(phgpu_state st) {
    const int64_t S = st.S;
    const int64_t t = (int64_t)blockIdx.x * SU_T + threadIdx.x;
    if (t >= (int64_t)st.m * S) return;
    const int i = (int)(t / S);
    const int64_t s = t - (int64_t)i * S;
    double a = 0.0;
    for (int k = st.row_ptr[i]; k < st.row_ptr[i + 1]; ++k) a += st.Ah_csr[IX(k)] * st.xe[IX(st.col_idx[k])];
    st.yt[IX(i)] = a;
}

__global__ void __launch_bounds__(SU_T) k_su_colmv(phgpu_state st) {
    const int64_t S = st.S;
    const int64_t t = (int64_t)blockIdx.x * SU_T + threadIdx.x;
    if (t >= (int64_t)st.n * S) return;
    const int j = (int)(t / S);
    const int64_t s = t - (int64_t)j * S;
    double a = 0.0;
    for (int kc = st.col_ptr[j]; kc < st.col_ptr[j + 1]; ++kc) a += st.Ah_csc[IX(kc)] * st.yt[IX(st.row_idx[kc])];
    st.xt[IX(j)] = a;
}

// per scenario: lam = ||A^T A v||, v = A^T A v / lam (normA holds lam until the end);
// a block holds 32 scenarios x 8 column chunks (chunk c: columns c, c+8, ...), partial
// sums of squares added in chunk order
#define SU_CH 8
__global__ void __launch_bounds__(SU_T) k_su_norm(phgpu_state st) {
    __shared__ double part[SU_CH][SU_T / SU_CH];
    const int64_t S = st.S;
    const int c = threadIdx.x / (SU_T / SU_CH), l = threadIdx.x % (SU_T / SU_CH);
    const int64_t s = (int64_t)blockIdx.x * (SU_T / SU_CH) + l;
    double a2 = 0.0;
    if (s < S)
        for (int j = c; j < st.n; j += SU_CH) {
            const double a = st.xt[IX(j)];
            a2 += a * a;
        }
    part[c][l] = a2;
    __syncthreads();
    double nv = 0.0;
    for (int k = 0; k < SU_CH; ++k) nv += part[k][l];
    nv = sqrt(nv);
    if (s >= S) return;
    if (c == 0) st.normA[s] = nv;
    const double inv = nv > 0.0 ? 1.0 / nv : 0.0;
    for (int j = c; j < st.n; j += SU_CH) st.xe[IX(j)] = st.xt[IX(j)] * inv;
}

__global__ void __launch_bounds__(SU_T) k_su_done(phgpu_state st) {
    const int64_t s = (int64_t)blockIdx.x * SU_T + threadIdx.x;
    if (s >= st.S) return;
    const double lam = st.normA[s];
    st.normA[s] = lam > 0.0 ? 1.01 * sqrt(lam) : 1.0;
    st.omega[s] = 1.0;
}

// setup of a non-shared handle: k_setup (lane per scenario) for small patterns, the
// parallel kernels above for patterns with more than SETUP_PAR_NNZ nonzeros
#define SETUP_PAR_NNZ 128
static hipError_t run_setup(phgpu_state* h, hipStream_t st) {
    if (h->nnz <= SETUP_PAR_NNZ) {
        hipLaunchKernelGGL(k_setup, dim3((unsigned)((h->S + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, st, *h, 10, 200);
        return hipGetLastError();
    }
    const int64_t S = h->S;
    const int64_t K = std::max<int64_t>(h->nnz, std::max(h->n, h->m));
    auto g = [&](int64_t cnt) { return dim3((unsigned)((cnt + SU_T - 1) / SU_T)); };
    hipLaunchKernelGGL(k_su_init, g(K * S), dim3(SU_T), 0, st, *h);
    for (int pass = 0; pass <= 10; ++pass) {
        const int pc = pass == 10;
        if (h->m) hipLaunchKernelGGL(k_su_rowfac, g((int64_t)h->m * S), dim3(SU_T), 0, st, *h, pc);
        hipLaunchKernelGGL(k_su_colfac, g((int64_t)h->n * S), dim3(SU_T), 0, st, *h, pc);
        hipLaunchKernelGGL(k_su_apply, g(K * S), dim3(SU_T), 0, st, *h);
    }
    hipLaunchKernelGGL(k_su_finish, g(K * S), dim3(SU_T), 0, st, *h);
    for (int it = 0; it < 200; ++it) {
        if (h->m) hipLaunchKernelGGL(k_su_rowmv, g((int64_t)h->m * S), dim3(SU_T), 0, st, *h);
        hipLaunchKernelGGL(k_su_colmv, g((int64_t)h->n * S), dim3(SU_T), 0, st, *h);
        hipLaunchKernelGGL(k_su_norm, dim3((unsigned)((S + SU_T / SU_CH - 1) / (SU_T / SU_CH))), dim3(SU_T), 0, st,
                           *h);
    }
    hipLaunchKernelGGL(k_su_done, g(S), dim3(SU_T), 0, st, *h);
    return hipGetLastError();
}

// ------------------------------------------------------------------ record transposes
// [K][S] (scenario-fastest, the C-ABI layout) <-> scenario-major records pk[s * stride +
// off + k], through a 32 x 33 LDS tile so both sides are full-line accesses.
#define TT 32
__global__ void __launch_bounds__(256) k_to_records(const double* __restrict__ in, int K, int64_t S,
                                                    double* __restrict__ pk, int64_t stride, int off) {
    __shared__ double tile[TT][TT + 1];
    const int64_t s0 = (int64_t)blockIdx.x * TT;
    const int k0 = blockIdx.y * TT;
    const int tx = threadIdx.x % TT, ty = threadIdx.x / TT;
    for (int r = ty; r < TT; r += 256 / TT) {
        const int k = k0 + r;
        const int64_t s = s0 + tx;
        tile[r][tx] = (k < K && s < S) ? in[(size_t)k * (size_t)S + (size_t)s] : 0.0;
    }
    __syncthreads();
    for (int r = ty; r < TT; r += 256 / TT) {
        const int64_t s = s0 + r;
        const int k = k0 + tx;
        if (s < S && k < K) pk[(size_t)s * (size_t)stride + off + k] = tile[tx][r];
    }
}

// the PH state of a solve into the records in one launch: W | rho | xbar are consecutive
// record fields of nn entries each (pk_W, pk_RHO, pk_XB); a null source is skipped
__device__ __forceinline__ void to_records_ph_tile(double (*tile)[TT + 1], int bx, int by, const double* __restrict__ W,
                                                   const double* __restrict__ rho, const double* __restrict__ xbar,
                                                   int nn, int64_t S, double* __restrict__ pk, int64_t stride,
                                                   int off) {
    const int64_t s0 = (int64_t)bx * TT;
    const int k0 = by * TT;
    const int K = 3 * nn;
    const int tx = threadIdx.x % TT, ty = threadIdx.x / TT;
    for (int r = ty; r < TT; r += 256 / TT) {
        const int k = k0 + r;
        const int64_t s = s0 + tx;
        const int part = k < nn ? 0 : (k < 2 * nn ? 1 : 2);
        const double* a = part == 0 ? W : (part == 1 ? rho : xbar);
        double v = 0.0;
        if (k < K && a && s < S) v = a[(size_t)(k - part * nn) * (size_t)S + (size_t)s];
        tile[r][tx] = v;
    }
    __syncthreads();
    for (int r = ty; r < TT; r += 256 / TT) {
        const int64_t s = s0 + r;
        const int k = k0 + tx;
        const int part = k < nn ? 0 : (k < 2 * nn ? 1 : 2);
        const bool have = part == 0 ? W != nullptr : (part == 1 ? rho != nullptr : xbar != nullptr);
        if (s < S && k < K && have) pk[(size_t)s * (size_t)stride + off + k] = tile[tx][r];
    }
}

__global__ void __launch_bounds__(256) k_to_records_ph(const double* __restrict__ W, const double* __restrict__ rho,
                                                       const double* __restrict__ xbar, int nn, int64_t S,
                                                       double* __restrict__ pk, int64_t stride, int off) {
    __shared__ double tile[TT][TT + 1];
    to_records_ph_tile(tile, blockIdx.x, blockIdx.y, W, rho, xbar, nn, S, pk, stride, off);
}

// out[k][s] = pk[s][off + k] * (moff >= 0 ? pk[s][moff + k] : 1)
__global__ void __launch_bounds__(256) k_from_records(const double* __restrict__ pk, int64_t stride, int off,
                                                      int moff, int K, int64_t S, double* __restrict__ out) {
    __shared__ double tile[TT][TT + 1];
    const int64_t s0 = (int64_t)blockIdx.x * TT;
    const int k0 = blockIdx.y * TT;
    const int tx = threadIdx.x % TT, ty = threadIdx.x / TT;
    for (int r = ty; r < TT; r += 256 / TT) {
        const int64_t s = s0 + r;
        const int k = k0 + tx;
        double v = 0.0;
        if (s < S && k < K) {
            const size_t b = (size_t)s * (size_t)stride;
            v = pk[b + off + k];
            if (moff >= 0) v *= pk[b + moff + k];
        }
        tile[tx][r] = v;
    }
    __syncthreads();
    for (int r = ty; r < TT; r += 256 / TT) {
        const int k = k0 + r;
        const int64_t s = s0 + tx;
        if (k < K && s < S) out[(size_t)k * (size_t)S + (size_t)s] = tile[r][tx];
    }
}

// ------------------------------------------------------------------ solve kernel
struct solve_params {
    double eps_rel, eps_abs, gamma, bsuff, bnec, bart, eta_frac, omega0, wmin, wmax, eps_inf;
    int max_iter, check_every, restart_every, warm, keep_omega, infeas_start;
};

__global__ void __launch_bounds__(BLOCK)
k_solve(phgpu_state st, solve_params P, double* __restrict__ xout, double* __restrict__ yout,
        double* __restrict__ obj, double* __restrict__ bound, int32_t* __restrict__ status,
        int32_t* __restrict__ iters, const int32_t* __restrict__ list = nullptr,
        const int32_t* __restrict__ list_n = nullptr, unsigned long long* __restrict__ stats = nullptr) {
    const int64_t S = st.S;
    int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    // list mode (the fallback of path 6's workgroup IPM): lane q solves list[q]
    if (list) {
        if (s >= *list_n) return;
        s = list[s];
    } else if (s >= S) {
        return;
    }
    const int n = st.n, m = st.m;
    const int32_t* __restrict__ row_ptr = st.row_ptr;
    const int32_t* __restrict__ col_idx = st.col_idx;
    const int32_t* __restrict__ col_ptr = st.col_ptr;
    const int32_t* __restrict__ row_idx = st.row_idx;
    const double* __restrict__ Ahr = st.Ah_csr;
    const double* __restrict__ Ahc = st.Ah_csc;
    // the iterate lives in the write slot (the read slot for an ordinary solve); the
    // warm start is read from st.x / st.y
    double* __restrict__ x = st.xw;
    double* __restrict__ x0 = st.x0;
    double* __restrict__ xe = st.xe;
    double* __restrict__ xt = st.xt;
    double* __restrict__ aty = st.aty;
    double* __restrict__ aty0 = st.aty0;
    double* __restrict__ y = st.yw;
    double* __restrict__ y0 = st.y0;
    double* __restrict__ yt = st.yt;
    const double* __restrict__ ch = st.ch;
    const double* __restrict__ qh = st.qh;

    // ---- effective objective of this solve (phbase.py:617-699), scaled
    double cnorm2 = 0.0, const_term = st.objc ? st.objc[s] : 0.0;
    for (int j = 0; j < n; ++j) {
        double cj = st.c[IX(j)];
        double qj = st.q ? st.q[IX(j)] : 0.0;
        const int k = st.nonant_slot[j];
        if (k >= 0) {
            if (st.W_on) cj += st.W[IX(k)];
            if (st.prox_on) {
                const double r = st.rho[IX(k)], xb = st.xbar[IX(k)];
                cj -= r * xb;
                qj += r;
                const_term += 0.5 * r * xb * xb;
            }
        }
        const double d = st.Dc[IX(j)];
        st.ch[IX(j)] = d * cj;
        st.qh[IX(j)] = d * d * qj;
        cnorm2 += cj * cj;
    }
    double bnorm2 = 0.0;
    for (int i = 0; i < m; ++i) {
        const double a = st.rl[IX(i)], b = st.ru[IX(i)];
        if (isfinite(a)) bnorm2 += a * a;
        if (isfinite(b) && b != a) bnorm2 += b * b;
    }
    const double cnorm = sqrt(cnorm2), bnorm = sqrt(bnorm2);

    // ---- start point
    for (int j = 0; j < n; ++j) {
        double v = P.warm ? st.x[IX(j)] : 0.0;
        v = clampd(v, st.lbh[IX(j)], st.ubh[IX(j)]);
        x[IX(j)] = v;
        x0[IX(j)] = v;
    }
    for (int i = 0; i < m; ++i) {
        const double v = P.warm ? st.y[IX(i)] : 0.0;
        y[IX(i)] = v;
        y0[IX(i)] = v;
    }
    for (int j = 0; j < n; ++j) {
        double a = 0.0;
        for (int kc = col_ptr[j]; kc < col_ptr[j + 1]; ++kc) a += Ahc[IX(kc)] * y[IX(row_idx[kc])];
        aty[IX(j)] = a;
        aty0[IX(j)] = a;
    }
    double omega = st.omega[s];
    if (!(P.keep_omega && P.warm) && P.omega0 > 0.0) omega = P.omega0;
    const double eta = P.eta_frac / st.normA[s];
    const double g = P.gamma;

    double r0 = -1.0, rlast = INFINITY;
    double pobj = 0.0, dobj = 0.0;
    int hk = 0;  // Halpern counter since the last restart
    int it = 0;
    int stat = PHGPU_ITER_LIMIT;
    bool final_is_t = false;  // true: solution is T(z) (in xt/yt/xe)
    for (; it < P.max_iter; ++it) {
        const double tau = eta / omega, sig = eta * omega;
        const bool kkt = (it % P.check_every) == 0;
        // non-fused iteration (T(z) kept in xt / yt / xe) at restart-test points and on
        // the last iteration (the iteration-limit answer is T(z), which is box-feasible)
        const bool check = kkt || (it % P.restart_every) == 0 || it == P.max_iter - 1;
        const double a1 = (hk + 1.0) / (hk + 2.0), a0 = 1.0 / (hk + 2.0);
        double dx2 = 0.0, dy2 = 0.0;
        // --- primal step: xt = prox(x - tau (c - A^T y)); xe = 2 xt - x
        for (int j = 0; j < n; ++j) {
            const double xj = x[IX(j)];
            const double qj = qh[IX(j)];
            const double num = xj - tau * (ch[IX(j)] - aty[IX(j)]);
            const double xtj = clampd(qj != 0.0 ? num / (1.0 + tau * qj) : num, st.lbh[IX(j)], st.ubh[IX(j)]);
            xe[IX(j)] = 2.0 * xtj - xj;
            const double d = xj - xtj;
            dx2 += d * d;
            if (check) xt[IX(j)] = xtj;
            else x[IX(j)] = a1 * ((1.0 + g) * xtj - g * xj) + a0 * x0[IX(j)];
        }
        // --- dual step: yt = prox(y - sig A xe)
        for (int i = 0; i < m; ++i) {
            double ax = 0.0;
            for (int k = row_ptr[i]; k < row_ptr[i + 1]; ++k) ax += Ahr[IX(k)] * xe[IX(col_idx[k])];
            const double yi = y[IX(i)];
            const double yti = dual_prox(yi - sig * ax, sig, st.rlh[IX(i)], st.ruh[IX(i)]);
            yt[IX(i)] = yti;
            const double d = yi - yti;
            dy2 += d * d;
            if (!check) y[IX(i)] = a1 * ((1.0 + g) * yti - g * yi) + a0 * y0[IX(i)];
        }
        // --- A^T yt (Halpern-combined in place, or kept in xe at checks)
        for (int j = 0; j < n; ++j) {
            double a = 0.0;
            for (int kc = col_ptr[j]; kc < col_ptr[j + 1]; ++kc) a += Ahc[IX(kc)] * yt[IX(row_idx[kc])];
            if (check) xe[IX(j)] = a;
            else aty[IX(j)] = a1 * ((1.0 + g) * a - g * aty[IX(j)]) + a0 * aty0[IX(j)];
        }
        const double r = sqrt(omega * dx2 + dy2 / omega);
        if (r0 < 0.0) r0 = r;
        if (!check) {
            ++hk;
            continue;
        }
        // ---- KKT test on T(z) = (xt, yt), original space
        if (kkt) {
        double pres2 = 0.0, dres2 = 0.0;
        pobj = const_term;
        dobj = const_term;
        for (int i = 0; i < m; ++i) {
            double ax = 0.0;
            for (int k = row_ptr[i]; k < row_ptr[i + 1]; ++k) ax += Ahr[IX(k)] * xt[IX(col_idx[k])];
            const double dr = st.Dr[IX(i)];
            ax /= dr;
            const double rl = st.rl[IX(i)], ru = st.ru[IX(i)];
            const double v = ax - clampd(ax, rl, ru);
            pres2 += v * v;
            dobj += row_dual_term(yt[IX(i)] * dr, rl, ru);
        }
        for (int j = 0; j < n; ++j) {
            const double d = st.Dc[IX(j)];
            const double xo = d * xt[IX(j)];
            const double ce = ch[IX(j)] / d, qe = qh[IX(j)] / (d * d);
            const double at = xe[IX(j)] / d;
            // working bounds (phgpu_fix_nonants may have fixed this column)
            const double lbj = st.lbh[IX(j)] * d, ubj = st.ubh[IX(j)] * d;
            const double rc = ce + qe * xo - at;
            double lam;
            if (isfinite(lbj) && isfinite(ubj)) lam = rc;
            else if (isfinite(lbj)) lam = fmax(rc, 0.0);
            else if (isfinite(ubj)) lam = fmin(rc, 0.0);
            else lam = 0.0;
            const double dr = rc - lam;
            dres2 += dr * dr;
            pobj += ce * xo + 0.5 * qe * xo * xo;
            dobj += col_dual_term(ce - at, qe, lbj, ubj);
        }
        const bool conv = sqrt(pres2) <= P.eps_abs + P.eps_rel * (1.0 + bnorm) &&
                          sqrt(dres2) <= P.eps_abs + P.eps_rel * (1.0 + cnorm) &&
                          fabs(pobj - dobj) <= P.eps_abs + P.eps_rel * (1.0 + fabs(pobj) + fabs(dobj));
        if (conv) {
            stat = PHGPU_OPTIMAL;
            final_is_t = true;
            break;
        }
        if (P.infeas_start >= 0 && it >= P.infeas_start) {
            // certificates from d = T(z) - z (x, y: the iterate; xt, yt: T(z); aty = A^T y,
            // xe = A^T yt)
            double pobj_r = 0.0, pviol = 0.0, cdx = 0.0, dviol = 0.0;
            for (int i = 0; i < m; ++i) {
                const double dr = st.Dr[IX(i)];
                const double rl = st.rl[IX(i)], ru = st.ru[IX(i)];
                ray_row_terms(dr * (yt[IX(i)] - y[IX(i)]), rl, ru, pobj_r, pviol);
                double adx = 0.0;
                for (int k = row_ptr[i]; k < row_ptr[i + 1]; ++k)
                    adx += Ahr[IX(k)] * (xt[IX(col_idx[k])] - x[IX(col_idx[k])]);
                dviol += recession_viol2(adx / dr, rl, ru);
            }
            for (int j = 0; j < n; ++j) {
                const double d = st.Dc[IX(j)];
                const double lbj = st.lbh[IX(j)] * d, ubj = st.ubh[IX(j)] * d;
                ray_col_terms(-(xe[IX(j)] - aty[IX(j)]) / d, lbj, ubj, pobj_r, pviol);
                const double dxo = d * (xt[IX(j)] - x[IX(j)]);
                const double qe = qh[IX(j)] / (d * d);
                cdx += (ch[IX(j)] / d) * dxo;
                dviol += recession_viol2(dxo, lbj, ubj) + (qe * dxo) * (qe * dxo);
            }
            if (is_certificate(pobj_r, pviol, P.eps_inf)) {
                stat = PHGPU_PRIMAL_INFEASIBLE;
                break;
            }
            if (is_certificate(-cdx, dviol, P.eps_inf)) {
                stat = PHGPU_DUAL_INFEASIBLE;
                break;
            }
        }
        }
        // ---- restart test (cuPDLP+-style: sufficient decay / necessary decay without
        // progress / artificial: the Halpern run is a fixed fraction of the solve)
        const bool restart = (r <= P.bsuff * r0) || (r <= P.bnec * r0 && r > rlast) ||
                             (it > 0 && hk >= P.bart * it);
        rlast = r;
        if (restart) {
            double ddx = 0.0, ddy = 0.0;
            for (int j = 0; j < n; ++j) {
                const double v = xt[IX(j)];
                const double d = v - x0[IX(j)];
                ddx += d * d;
                x[IX(j)] = v;
                x0[IX(j)] = v;
                aty[IX(j)] = xe[IX(j)];
                aty0[IX(j)] = xe[IX(j)];
            }
            for (int i = 0; i < m; ++i) {
                const double v = yt[IX(i)];
                const double d = v - y0[IX(i)];
                ddy += d * d;
                y[IX(i)] = v;
                y0[IX(i)] = v;
            }
            ddx = sqrt(ddx);
            ddy = sqrt(ddy);
            if (ddx > 1e-10 && ddy > 1e-10)
                // geometric mean of omega and ||dy|| / ||dx||: exp(0.5 log(ddy/ddx) + 0.5 log(omega))
                // as one sqrt (fp64 exp / log are long software sequences)
                omega = clampd(sqrt(omega * (ddy / ddx)), P.wmin, P.wmax);
            hk = 0;
            r0 = -1.0;
            rlast = INFINITY;
        } else {
            for (int j = 0; j < n; ++j) {
                x[IX(j)] = a1 * ((1.0 + g) * xt[IX(j)] - g * x[IX(j)]) + a0 * x0[IX(j)];
                aty[IX(j)] = a1 * ((1.0 + g) * xe[IX(j)] - g * aty[IX(j)]) + a0 * aty0[IX(j)];
            }
            for (int i = 0; i < m; ++i)
                y[IX(i)] = a1 * ((1.0 + g) * yt[IX(i)] - g * y[IX(i)]) + a0 * y0[IX(i)];
            ++hk;
        }
    }
    // ---- write back: converged -> T(z); iteration limit -> current z
    if (final_is_t) {
        for (int j = 0; j < n; ++j) x[IX(j)] = xt[IX(j)];
        for (int i = 0; i < m; ++i) y[IX(i)] = yt[IX(i)];
    } else {
        // iteration limit: answer T(z) of the last iteration (xt, yt, A^T yt in xe)
        for (int j = 0; j < n; ++j) {
            x[IX(j)] = xt[IX(j)];
            aty[IX(j)] = xe[IX(j)];
        }
        for (int i = 0; i < m; ++i) y[IX(i)] = yt[IX(i)];
        pobj = const_term;
        dobj = const_term;
        for (int i = 0; i < m; ++i) dobj += row_dual_term(y[IX(i)] * st.Dr[IX(i)], st.rl[IX(i)], st.ru[IX(i)]);
        for (int j = 0; j < n; ++j) {
            const double d = st.Dc[IX(j)];
            const double xo = d * x[IX(j)];
            const double ce = ch[IX(j)] / d, qe = qh[IX(j)] / (d * d);
            pobj += ce * xo + 0.5 * qe * xo * xo;
            dobj += col_dual_term(ce - aty[IX(j)] / d, qe, st.lbh[IX(j)] * d, st.ubh[IX(j)] * d);
        }
    }
    if (stat == PHGPU_PRIMAL_INFEASIBLE) pobj = dobj = INFINITY;
    if (stat == PHGPU_DUAL_INFEASIBLE) pobj = dobj = -INFINITY;
    for (int j = 0; j < n; ++j) xout[IX(j)] = st.Dc[IX(j)] * x[IX(j)];
    if (yout)
        for (int i = 0; i < m; ++i) yout[IX(i)] = st.Dr[IX(i)] * y[IX(i)];
    st.omega_w[s] = omega;
    obj[s] = pobj;
    bound[s] = dobj;
    status[s] = stat;
    if (iters) iters[s] = (stat == PHGPU_ITER_LIMIT) ? P.max_iter : it;
    if (stats) {  // list mode: this solve's statistics (the IPM counted the others)
        const unsigned long long its = (unsigned long long)((stat == PHGPU_ITER_LIMIT) ? P.max_iter : it);
        atomicAdd(&stats[stat], 1ull);
        atomicAdd(&stats[4], its);
        atomicMax(&stats[5], its);
    }
}

// The path-6 statistics {OPTIMAL, ITER_LIMIT, PRIMAL_INF, DUAL_INF, iteration sum, iteration
// maximum, jam hand-overs, re-centrings} are PHGPU_STATS_COPIES copies, one 128-B line each:
// wave w of a path-6 kernel adds to copy w % copies.  One copy took every wave's atomics,
// thousands on one L2 line, serialised there for ~20 us at the end of the 8,192-share launch
// (the stores and epilogue queued behind them; tools/ipm_prof.py).  Readers sum
// the copies (the maximum for word 5); stats_gen (paths without in-kernel statistics) is one
// copy.
#define PHGPU_STATS_COPIES 32
#define PHGPU_STATS_STRIDE 16
#define PHGPU_STATS_WORDS (PHGPU_STATS_COPIES * PHGPU_STATS_STRIDE)
inline unsigned long long stats_word(const unsigned long long* s, int copies, int k) {
    unsigned long long a = 0;
    for (int c = 0; c < copies; ++c) {
        const unsigned long long v = s[c * PHGPU_STATS_STRIDE + k];
        a = (k == 5) ? (v > a ? v : a) : a + v;
    }
    return a;
}

// the six statistics summed over the copies by a whole wave: lane t < copies reads copy t (one
// load latency; a thread reading the 32 copies in turn took 8 us), the wave reduces, every
// lane returns them
__device__ __forceinline__ void stats_wave(const unsigned long long* __restrict__ s, int copies,
                                           unsigned long long v[6]) {
    const int t = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < 6; ++k) v[k] = t < copies ? s[t * PHGPU_STATS_STRIDE + k] : 0ull;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            const unsigned long long u = __shfl_xor(v[k], o, 64);
            v[k] = k == 5 ? (u > v[k] ? u : v[k]) : v[k] + u;
        }
}

// the six statistics of a solve into out (int64): one wave
__global__ void k_stats_copy(const unsigned long long* __restrict__ src, int copies, int64_t* __restrict__ out) {
    unsigned long long v[6];
    stats_wave(src, copies, v);
    if (threadIdx.x < 6) {
        unsigned long long w = v[0];
#pragma unroll
        for (int k = 1; k < 6; ++k) w = (int)threadIdx.x == k ? v[k] : w;
        out[threadIdx.x] = (int64_t)w;
    }
}

#include "solve_reg.inc"
#include "solve_wg.inc"
#include "solve_stream.inc"
#include "solve_jit.inc"
#include "solve_ipm.inc"

// ------------------------------------------------------------------ PH reductions
// phbase.py:54-79: per-wave partial sums of prob_coeff * x and prob_coeff * x^2 for
// each nonant; a wave whose scenarios share one node at that depth writes one
// partial (deterministic); a mixed wave adds per lane with fp64 atomics.
__global__ void __launch_bounds__(BLOCK)
k_xbar_partial(phgpu_state st, const double* __restrict__ x, double* __restrict__ node_buf, int clear) {
    const int64_t S = st.S;
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t wave = s / WAVE;
    const bool act = s < S;
    const int half = st.num_nodes * st.nlen_max;
    // no wave spans two nodes (st.xbar_mixed == 0): this kernel does not touch node_buf
    // below, so it clears it for k_xbar_final (one launch less than a memset)
    if (clear && blockIdx.y == 0)
        for (int64_t i = s; i < 2 * (int64_t)half; i += (int64_t)gridDim.x * blockDim.x) node_buf[i] = 0.0;
    // one nonant per grid row (blockIdx.y; see k_ph_update)
    if ((int)blockIdx.y < st.nn) {
        const int k = blockIdx.y;
        const int d = st.nonant_depth[k];
        const int gnode = act ? st.node_of[IX(d)] : -1;
        const double w = act ? (st.pvar ? st.pvar[IX(k)] : st.pcoef[IX(d)]) : 0.0;
        const double v = act ? x[IX(st.nonant_col[k])] : 0.0;
        const int g0 = __shfl(gnode, 0, WAVE);
        const bool uniform = !__any(act && gnode != g0);
        if (uniform) {
            const double a = wave_sum(w * v);
            const double b = wave_sum(w * v * v);
            if ((threadIdx.x & (WAVE - 1)) == 0) {
                st.part[(wave * st.nn + k) * 2 + 0] = a;
                st.part[(wave * st.nn + k) * 2 + 1] = b;
                st.part_node[wave * st.nn + k] = g0;
            }
        } else {
            if (act) {
                const int o = gnode * st.nlen_max + st.nonant_off[k];
                atomicAdd(&node_buf[o], w * v);
                atomicAdd(&node_buf[half + o], w * v * v);
            }
            if ((threadIdx.x & (WAVE - 1)) == 0) st.part_node[wave * st.nn + k] = -1;
        }
    }
}

// out[0] |= 1 if some wave of local scenarios spans two nodes at a nonant's depth (the
// test k_xbar_partial makes per wave)
// out[1] |= 1 if some local scenario's node at a nonant's depth differs from scenario 0's
__global__ void __launch_bounds__(BLOCK) k_xbar_mixed(phgpu_state st, int32_t* __restrict__ out) {
    const int64_t S = st.S;
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool act = s < S;
    bool mixed = false, multi = false;
    for (int k = 0; k < st.nn; ++k) {
        const int d = st.nonant_depth[k];
        const int gnode = act ? st.node_of[IX(d)] : -1;
        const int g0 = __shfl(gnode, 0, WAVE);
        mixed |= __any(act && gnode != g0) != 0;
        multi |= __any(act && gnode != st.node_of[(int64_t)d * S]) != 0;
    }
    if (mixed && (threadIdx.x & (WAVE - 1)) == 0) atomicOr(out, 1);
    if (multi && (threadIdx.x & (WAVE - 1)) == 0) atomicOr(out + 1, 1);
}

// Ordered segmented sum of the per-wave partials, one block per nonant.  The local
// scenarios are in tree order, so each node's waves form ONE contiguous run: a run
// that lies inside one thread's chunk of waves is complete and is flushed directly;
// the first / last run of every chunk go through shared memory and thread 0 merges
// them in chunk order (deterministic for every wave-uniform node).
// x̄ partial of nonant k over chunk w recomputed from x (a chunk of the path-6 epilogue
// partials with a scenario the fallback solved), in scenario order
__device__ __forceinline__ void xp_recompute(const phgpu_state& st, const double* __restrict__ x, int64_t w, int C,
                                             int k, double& a, double& b) {
    const int64_t S = st.S;
    const int d = st.nonant_depth[k], j = st.nonant_col[k];
    const int64_t s1 = (w + 1) * C < S ? (w + 1) * C : S;
    a = b = 0.0;
    for (int64_t s = w * C; s < s1; ++s) {
        const double p = st.pvar ? st.pvar[IX(k)] : st.pcoef[IX(d)], v = x[IX(j)];
        a += p * v;
        b += p * v * v;
    }
}

#define XF_THREADS 256
// assign: node_buf was not cleared (one tree node, every entry is some nonant's): the fast
// path stores its sums instead of adding them (phgpu_ph_reduce: one launch less per step)
__global__ void __launch_bounds__(XF_THREADS) k_xbar_final(phgpu_state st, double* __restrict__ node_buf,
                                                           const int32_t* __restrict__ dirty = nullptr,
                                                           int xpC = 0, const double* __restrict__ x = nullptr,
                                                           int assign = 0) {
    __shared__ int fnode[XF_THREADS], lnode[XF_THREADS];
    __shared__ double fa[XF_THREADS], fb[XF_THREADS], la[XF_THREADS], lb[XF_THREADS];
    const int k = blockIdx.x;
    const int t = threadIdx.x;
    const int half = st.num_nodes * st.nlen_max;
    const int off = st.nonant_off[k];
    const int64_t nw = st.nwaves;
    const int64_t C = (nw + XF_THREADS - 1) / XF_THREADS;
    const int64_t w0 = (int64_t)t * C, w1 = (w0 + C < nw) ? w0 + C : nw;
    int cur = -1, first = -1;
    double a = 0.0, b = 0.0, a_first = 0.0, b_first = 0.0;
    for (int64_t w = w0; w < w1; ++w) {
        // the chunk's node, dirty flag and partials in flight together (none gates another
        // load: one memory round trip per chunk instead of three on the x̄ critical path)
        const int gnode = st.part_node[w * st.nn + k];
        const int dw = dirty ? dirty[w] : 0;
        const double pa = st.part[(w * st.nn + k) * 2 + 0], pb = st.part[(w * st.nn + k) * 2 + 1];
        if (gnode < 0) continue;
        if (gnode != cur) {
            if (cur >= 0) {
                if (first < 0) {  // close the chunk's first run
                    first = cur;
                    a_first = a;
                    b_first = b;
                } else {          // a complete middle run
                    atomicAdd(&node_buf[cur * st.nlen_max + off], a);
                    atomicAdd(&node_buf[half + cur * st.nlen_max + off], b);
                }
            }
            cur = gnode;
            a = 0.0;
            b = 0.0;
        }
        if (dw) {
            double ra, rb;
            xp_recompute(st, x, w, xpC, k, ra, rb);
            a += ra;
            b += rb;
        } else {
            a += pa;
            b += pb;
        }
    }
    if (first < 0) {  // zero or one run in this chunk: it is the first (and last) run
        fnode[t] = cur;
        fa[t] = a;
        fb[t] = b;
        lnode[t] = -1;
        la[t] = lb[t] = 0.0;
    } else {
        fnode[t] = first;
        fa[t] = a_first;
        fb[t] = b_first;
        lnode[t] = cur;
        la[t] = a;
        lb[t] = b;
    }
    __syncthreads();
    // fast path (every two-stage problem, and any nonant whose local scenarios share one
    // node): all runs belong to thread 0's node -> fixed-order tree sum
    __shared__ int single;
    if (t == 0) single = 1;
    __syncthreads();
    {
        const int g0 = fnode[0] >= 0 ? fnode[0] : lnode[0];
        if ((fnode[t] >= 0 && fnode[t] != g0) || (lnode[t] >= 0 && lnode[t] != g0)) single = 0;
    }
    __syncthreads();
    if (single) {
        fa[t] += la[t];
        fb[t] += lb[t];
        __syncthreads();
        for (int off = XF_THREADS / 2; off > 0; off >>= 1) {
            if (t < off) {
                fa[t] += fa[t + off];
                fb[t] += fb[t + off];
            }
            __syncthreads();
        }
        if (t == 0) {
            int g0 = -1;
            for (int u = 0; u < XF_THREADS && g0 < 0; ++u) g0 = fnode[u] >= 0 ? fnode[u] : lnode[u];
            if (g0 >= 0 && assign) {
                node_buf[g0 * st.nlen_max + off] = fa[0];
                node_buf[half + g0 * st.nlen_max + off] = fb[0];
            } else if (g0 >= 0) {
                node_buf[g0 * st.nlen_max + off] += fa[0];
                node_buf[half + g0 * st.nlen_max + off] += fb[0];
            }
        }
        return;
    }
    // several nodes: every run is flushed once, by the thread where it starts (its owner),
    // which adds the continuation pieces of the following threads in thread order.  All
    // runs flush in parallel (a serial merge by one thread cost ~0.2 ms per launch on
    // 1,057 aircond nodes); one flush per node keeps tree-ordered sums deterministic.
    // (lnode[u] >= 0 implies fnode[u] >= 0: a chunk's runs are maximal and distinct.)
    for (int side = 0; side < 2; ++side) {
        const int g = side ? lnode[t] : fnode[t];
        if (g < 0) continue;
        if (side == 0) {  // does the first run continue the previous non-empty chunk's tail?
            int p = t - 1;
            while (p >= 0 && fnode[p] < 0) --p;
            if (p >= 0 && (lnode[p] >= 0 ? lnode[p] : fnode[p]) == g) continue;
        }
        double sa = side ? la[t] : fa[t];
        double sb = side ? lb[t] : fb[t];
        if (side == 1 || lnode[t] < 0) {  // this run reaches the end of the chunk
            for (int u = t + 1; u < XF_THREADS; ++u) {
                if (fnode[u] < 0) continue;  // empty chunk
                if (fnode[u] != g) break;
                sa += fa[u];
                sb += fb[u];
                if (lnode[u] >= 0) break;    // the run ends inside chunk u
            }
        }
        atomicAdd(&node_buf[g * st.nlen_max + off], sa);
        atomicAdd(&node_buf[half + g * st.nlen_max + off], sb);
    }
}

// Where the update kernels leave conv (phbase.py:330-339) and the last solve's statistics
struct conv_sink {
    double* conv;                          // conv_local (pinned host or device memory)
    const unsigned long long* stats_src;   // the last solve's statistics (device), or null
    int stats_copies;                      // copies of them at stats_src (stats_word)
    int64_t* stats_dst;                    // where they go (pinned host or device), or null
    double scale;                          // 1 / (S nn)
    double* cpart;                         // [gridDim.x] block partials
    int32_t* cnt;                          // last-block counter (0 between launches)
};

// conv = scale x (sum over the grid of every thread's acc), without a second launch: each
// block reduces its threads in a fixed order and swaps its partial into cpart[block], then
// takes a ticket; the block with the last ticket sums cpart in block order (deterministic)
// and stores the statistics, then conv.  Every cross-block exchange is an agent-scope atomic
// read-modify-write, performed at the device's coherence point, so no block needs a release
// fence (an L2 writeback on gfx950); the ticket is taken only after the swap
// has returned.  The host reads stats after it sees conv (phgpu_ph_update_ex).
__device__ __forceinline__ void conv_last_block(double acc, const conv_sink& o) {
    __shared__ double red[XL_T / WAVE];
    __shared__ int last;
    const int wv = threadIdx.x / WAVE, nwb = (int)(blockDim.x / WAVE);
    // the solve's statistics copies, loaded now by every block's first wave (the previous
    // launch wrote them: stream order) and reduced only by the last block -- their load is
    // off the exchange / ticket chain
    unsigned long long sv[6];
    {
        const int t = threadIdx.x;
#pragma unroll
        for (int k = 0; k < 6; ++k)
            sv[k] = (o.stats_dst && t < o.stats_copies) ? o.stats_src[t * PHGPU_STATS_STRIDE + k] : 0ull;
    }
    const int nblk = (int)(gridDim.x * gridDim.y), bid = (int)(blockIdx.y * gridDim.x + blockIdx.x);
    acc = wave_sum(acc);
    if ((threadIdx.x & (WAVE - 1)) == 0) red[wv] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int u = 0; u < nwb; ++u) t += red[u];
        const double old = __hip_atomic_exchange(&o.cpart[bid], t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // The swap has returned before the ticket is taken (the empty asm consumes its result,
        // so the compiler waits for it).  Ordering rests on the hardware, not on the HIP memory
        // model (both RMWs are relaxed): a returning agent-scope atomic has been performed at
        // the device's coherence point when its value is back, so the last block's reads of
        // cpart (agent-scope RMWs as well) see every partial whose ticket precedes its own.
        // Release / acquire would make it formal at the price of an L2 writeback on every XCD
        // (15-29 us per launch).  tests/test_gpu_readback.py compares this conv
        // bit for bit with the ordered device reduction and would catch a reordering.
        asm volatile("" ::"v"(old) : "memory");
        const int tk = __hip_atomic_fetch_add(o.cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = tk == nblk - 1;
    }
    __syncthreads();
    if (!last) return;
    double a = 0.0;
    for (int b = threadIdx.x; b < nblk; b += blockDim.x)
        a += __hip_atomic_fetch_add(&o.cpart[b], 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    a = wave_sum(a);
    __syncthreads();
    if ((threadIdx.x & (WAVE - 1)) == 0) red[wv] = a;
    __syncthreads();
    // lanes 0..5 store the statistics and lane 6 conv in one store instruction (no wait for
    // the host-memory acknowledgements: the host polls conv and the statistics' sentinels,
    // engine.convergence_wait)
    if (threadIdx.x < WAVE) {
        double t = 0.0;
        for (int u = 0; u < nwb; ++u) t += red[u];
        if (o.stats_dst) {
            unsigned long long v[6];
#pragma unroll
            for (int k = 0; k < 6; ++k) v[k] = sv[k];
#pragma unroll
            for (int o2 = 32; o2 > 0; o2 >>= 1)
#pragma unroll
                for (int k = 0; k < 6; ++k) {
                    const unsigned long long u = __shfl_xor(v[k], o2, 64);
                    v[k] = k == 5 ? (u > v[k] ? u : v[k]) : v[k] + u;
                }
            unsigned long long w = v[0];
#pragma unroll
            for (int k = 1; k < 6; ++k) w = (int)threadIdx.x == k ? v[k] : w;
            if (threadIdx.x < 6) o.stats_dst[threadIdx.x] = (int64_t)w;
        }
        if (threadIdx.x == 6) *o.conv = t * o.scale;
        if (threadIdx.x == 0) __hip_atomic_store(o.cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// phbase.py:90-103 (scatter x̄), 293-318 (W update), 330-339 (local |x - x̄| sum, reduced
// by the last block into conv_local).
#define UPD_T 256
#define UPD_BLOCKS 256  // at most about this many blocks: each takes a ticket on one counter
#define UPD_U 4         // scenarios per thread in flight per trip
__global__ void __launch_bounds__(UPD_T)
k_ph_update(phgpu_state st, const double* __restrict__ x, const double* __restrict__ node_buf,
            double* __restrict__ xbar, double* __restrict__ W, const double* __restrict__ rho,
            int update_W, conv_sink o) {
    // one nonant per grid row (blockIdx.y): the per-nonant index loads of a scenario's
    // thread run in parallel instead of one dependent chain per nonant (config 2, 30
    // nonants: 27 us -> a few).  A row's blocks stride over the scenarios (UPD_U loads in
    // flight per thread), so that the grid stays near UPD_BLOCKS blocks: the last-block
    // ticket is one atomic counter, and config 4's 1,536 blocks (65,536 scenarios x 6
    // nonants) queued on it for about 20 us of a 27 us launch
    const int64_t S = st.S;
    const int k = blockIdx.y;
    double acc = 0.0;
    if (k < st.nn) {
        const int d = st.nonant_depth[k];
        const int off = st.nonant_off[k], col = st.nonant_col[k], nl = st.nlen_max;
        const int64_t stride = (int64_t)gridDim.x * blockDim.x;
        for (int64_t s0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s0 < S; s0 += UPD_U * stride) {
            double xb[UPD_U], xv[UPD_U], wo[UPD_U], rv[UPD_U];
            bool pz[UPD_U];
#pragma unroll
            for (int u = 0; u < UPD_U; ++u) {
                const int64_t s = s0 + u * stride;
                xb[u] = xv[u] = wo[u] = rv[u] = 0.0;
                pz[u] = false;
                if (s < S) {  // (a wave past S skips its loads: a small batch has one trip of one)
                    const int gnode = st.node_of[(int64_t)d * S + s];
                    xb[u] = node_buf[gnode * nl + off];
                    xv[u] = x[(int64_t)col * S + s];
                    wo[u] = update_W ? W[(int64_t)k * S + s] : 0.0;
                    rv[u] = update_W ? rho[(int64_t)k * S + s] : 0.0;
                    // (variable probabilities: W masked where the probability is 0, phbase.py:315-318)
                    pz[u] = update_W && st.pvar && st.pvar[(int64_t)k * S + s] == 0.0;
                }
            }
#pragma unroll
            for (int u = 0; u < UPD_U; ++u) {
                const int64_t s = s0 + u * stride;
                if (s < S) {
                    xbar[(int64_t)k * S + s] = xb[u];
                    if (update_W) W[(int64_t)k * S + s] = pz[u] ? 0.0 : wo[u] + rv[u] * (xv[u] - xb[u]);
                    acc += fabs(xv[u] - xb[u]);
                }
            }
        }
    }
    conv_last_block(acc, o);
}

// phgpu_ph_step_local (one rank, every nonant's scenarios on one node, nn <= XL_NN_MAX):
// k_xbar_final and k_ph_update in one launch.  Every block sums the per-wave x̄ partials
// itself, in one fixed order (so every block gets the same bits), block 0 stores them in
// node_buf; then the scatter / W update / conv of k_ph_update (last-block reduction).  The
// partials are per wave (k_xbar_partial) or per chunk of the path-6 epilogue (st.part /
// st.nwaves then point at those; dirty chunks are recomputed from x).  Few, large blocks for
// a large batch (every block re-sums the partials), 256 threads for a small one.
__global__ void __launch_bounds__(XL_T)
k_ph_update_local(phgpu_state st, const double* __restrict__ x, double* __restrict__ node_buf,
                  double* __restrict__ xbar, double* __restrict__ W, const double* __restrict__ rho,
                  int update_W, conv_sink o, const int32_t* __restrict__ dirty, int C) {
    __shared__ double sa[XL_T / WAVE][XL_NN_MAX], sb[XL_T / WAVE][XL_NN_MAX];
    __shared__ double xbs[XL_NN_MAX];
    const int64_t S = st.S;
    const int nn = st.nn;
    const int half = st.num_nodes * st.nlen_max;
    // every nonant at once: strided loads of the contiguous per-wave partials, wave sums,
    // then the block's waves in order (one barrier)
    // the scenario's own operands of the first XL_PF nonants, loaded ahead of the x̄ sums
    // (independent of them; the barrier below would keep them behind)
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t sc = s < S ? s : S - 1;
    double xv[XL_PF], wo[XL_PF], rv[XL_PF];
#pragma unroll
    for (int k = 0; k < XL_PF; ++k) {
        const int kk = k < nn ? k : 0;
        xv[k] = x[(int64_t)st.nonant_col[kk] * S + sc];
        wo[k] = update_W ? W[(int64_t)kk * S + sc] : 0.0;
        rv[k] = update_W ? rho[(int64_t)kk * S + sc] : 0.0;
    }
    double a[XL_NN_MAX], b[XL_NN_MAX];
#pragma unroll
    for (int k = 0; k < XL_NN_MAX; ++k) a[k] = b[k] = 0.0;
    for (int64_t w = threadIdx.x; w < st.nwaves; w += blockDim.x) {
        const double* pw = st.part + w * nn * 2;
        // the chunk's flag and partials in flight together (the flag gates the use only)
        const int dw = dirty ? dirty[w] : 0;
        double pa[XL_PF], pb[XL_PF];
#pragma unroll
        for (int k = 0; k < XL_PF; ++k) {
            pa[k] = k < nn ? pw[2 * k] : 0.0;
            pb[k] = k < nn ? pw[2 * k + 1] : 0.0;
        }
        if (dw) {  // a chunk with a fallback scenario (path-6 partials)
            for (int k = 0; k < nn; ++k) {
                double ra, rb;
                xp_recompute(st, x, w, C, k, ra, rb);
#pragma unroll
                for (int u = 0; u < XL_NN_MAX; ++u)
                    if (u == k) a[u] += ra, b[u] += rb;
            }
            continue;
        }
#pragma unroll
        for (int k = 0; k < XL_NN_MAX; ++k)
            if (k < nn) {
                a[k] += k < XL_PF ? pa[k < XL_PF ? k : 0] : pw[2 * k];
                b[k] += k < XL_PF ? pb[k < XL_PF ? k : 0] : pw[2 * k + 1];
            }
    }
    const int wv = threadIdx.x / WAVE;
#pragma unroll
    for (int k = 0; k < XL_NN_MAX; ++k)
        if (k < nn) {
            const double ta = wave_sum(a[k]), tb = wave_sum(b[k]);
            if ((threadIdx.x & (WAVE - 1)) == 0) {
                sa[wv][k] = ta;
                sb[wv][k] = tb;
            }
        }
    __syncthreads();
    if (threadIdx.x < nn) {
        const int k = threadIdx.x;
        double ta = 0.0, tb = 0.0;
        const int nwb = (int)(blockDim.x / WAVE);
        for (int u = 0; u < nwb; ++u) {
            ta += sa[u][k];
            tb += sb[u][k];
        }
        xbs[k] = ta;
        if (blockIdx.x == 0) {
            const int g0 = st.node_of[(int64_t)st.nonant_depth[k] * S];
            node_buf[g0 * st.nlen_max + st.nonant_off[k]] = ta;
            node_buf[half + g0 * st.nlen_max + st.nonant_off[k]] = tb;
        }
    }
    __syncthreads();
    double acc = 0.0;
    if (s < S) {
#pragma unroll
        for (int k = 0; k < XL_PF; ++k)
            if (k < nn) {
                const double xb = xbs[k];
                xbar[IX(k)] = xb;
                if (update_W) W[IX(k)] = wo[k] + rv[k] * (xv[k] - xb);
                acc += fabs(xv[k] - xb);
            }
        for (int k = XL_PF; k < nn; ++k) {
            const double xb = xbs[k];
            const double xw = x[IX(st.nonant_col[k])];
            xbar[IX(k)] = xb;
            if (update_W) W[IX(k)] += rho[IX(k)] * (xw - xb);
            acc += fabs(xw - xb);
        }
    }
    conv_last_block(acc, o);
}

// spopt.py:310-439 local sums: prob*obj, prob*bound, prob, prob*feasible, prob*optimal.
__global__ void __launch_bounds__(BLOCK)
k_expect_partial(phgpu_state st, const double* __restrict__ obj, const double* __restrict__ bound,
                 const int32_t* __restrict__ status) {
    const int64_t S = st.S;
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    double v[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
    if (s < S) {
        const double p = st.prob[s];
        v[0] = p * obj[s];
        v[1] = p * bound[s];
        v[2] = p;
        v[3] = (status[s] == PHGPU_OPTIMAL || status[s] == PHGPU_ITER_LIMIT) ? p : 0.0;
        v[4] = (status[s] == PHGPU_OPTIMAL) ? p : 0.0;
    }
#pragma unroll
    for (int t = 0; t < 5; ++t) {
        const double a = wave_sum(v[t]);
        if ((threadIdx.x & (WAVE - 1)) == 0) st.part[(s / WAVE) * 5 + t] = a;
    }
}

// Xhat_Eval._fix_nonants (utils/xhat_eval.py; spopt.py _fix_nonants): nonant columns of
// every scenario get lb = ub = xfix[k, s] (scaled); xfix == NULL restores the model bounds.
__global__ void __launch_bounds__(BLOCK)
k_fix_nonants(phgpu_state st, const double* __restrict__ xfix) {
    const int64_t S = st.S;
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S) return;
    for (int k = 0; k < st.nn; ++k) {
        const int j = st.nonant_col[k];
        const double d = st.Dc[IX(j)];
        const double xv = xfix ? xfix[IX(k)] : NAN;
        if (!isnan(xv)) {
            const double v = fmin(fmax(xv, st.lb[IX(j)]), st.ub[IX(j)]);
            st.lbh[IX(j)] = v / d;
            st.ubh[IX(j)] = v / d;
        } else {
            st.lbh[IX(j)] = st.lb[IX(j)] / d;
            st.ubh[IX(j)] = st.ub[IX(j)] / d;
        }
    }
}

// Deterministic ordered sum of K interleaved per-wave partials: out[k] = sum_w part[w*K+k].
// With stats_src / stats_dst (phgpu_ph_update_ex) block 0 also copies a solve's six
// statistics (a store to host memory here saves a copy launch per PH iteration).
__global__ void __launch_bounds__(256) k_sum_partials(const double* __restrict__ part, int64_t nw, int K,
                                                     double scale, double* __restrict__ out,
                                                     const unsigned long long* __restrict__ stats_src = nullptr,
                                                     int64_t* __restrict__ stats_dst = nullptr) {
    __shared__ double sh[256];
    const int k = blockIdx.x;
    if (stats_dst && k == 0 && threadIdx.x < 6) stats_dst[threadIdx.x] = (int64_t)stats_src[threadIdx.x];  // (one copy)
    double a = 0.0;
    for (int64_t w = threadIdx.x; w < nw; w += 256) a += part[w * K + k];
    sh[threadIdx.x] = a;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if (threadIdx.x < off) sh[threadIdx.x] += sh[threadIdx.x + off];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[k] = sh[0] * scale;
}

// ------------------------------------------------------------------ lane plan (host)
#include <vector>
#include <algorithm>

// Build the per-lane plan of solve_reg.inc for L lanes per scenario: lane l owns
// columns j = l + q L and rows i = l + r L; each column's CSC entries and each row's
// CSR entries are padded to the instance's ZC / ZR slots.  Returns false if no
// compiled instance fits (then the global-memory kernel is used).
// register-cost estimate of an instance, in doubles per lane
static inline long reg_cost(const reg_instance& r) {
    return (long)r.KC * (13 + r.ZC) + (long)r.KR * (7 + r.ZR);
}

// an instance that spills more than REG_SPILL_MAX bytes of scratch per lane at 2 waves /
// SIMD is skipped by the lane search (L doubles past it).  Both variants are checked --
// scenario order (fn) and record mode (fn_rec), whichever phgpu_solve will launch.
// Measured on farmer 65,536 cm=1 (profiles/r01): <8,4,4,4> at L=2 spills 1.5 KB -> 14.4 ms
// per solve; <2,3,1,4> at L=8, no spill -> 0.77 ms.  <3,3,2,4> (the headline instance)
// spills 28 B (fn) / 268 B (fn_rec), all of it outside the PDHG step loop: the scratch
// operations of its code object sit in the prologue, the scenario load / refill, the check
// iteration and the write-back, none in the R-1 plain steps (tools/scratch_regions.py,
// profiles/r03/scratch_regions.txt) -- so the cap sits above 268 B.  The first instance
// whose step loop spills is <6,4,2,4> (568 / 940 B, 43 / 37 scratch ops in the loop);
// <4,4,2,4> (216 / 508 B) keeps its loop clean but spills 98 / 174 times in the check and
// refill paths, and stays excluded as before.
#ifndef REG_SPILL_MAX
#define REG_SPILL_MAX 320
#endif
static bool reg_spills(const reg_instance& r) {
    for (reg_kernel_t f : {r.fn, r.fn_rec}) {
        hipFuncAttributes a;
        if (hipFuncGetAttributes(&a, (const void*)f) != hipSuccess) continue;
        if (a.localSizeBytes > REG_SPILL_MAX) return true;
    }
    return false;
}

static bool build_plan(int L, int n, int m, const int32_t* row_ptr, const int32_t* col_idx,
                       int* inst_out, int* kc_out, int* zc_out, int* kr_out, int* zr_out,
                       std::vector<int32_t>& col_k, std::vector<int32_t>& col_r,
                       std::vector<int32_t>& row_k, std::vector<int32_t>& row_c) {
    if (m < 1 || n < 1) return false;
    const int kc = (n + L - 1) / L;
    const int kr = (m + L - 1) / L;
    std::vector<std::vector<std::pair<int, int>>> cols(n);  // (csr k, row)
    for (int i = 0; i < m; ++i)
        for (int k = row_ptr[i]; k < row_ptr[i + 1]; ++k) cols[col_idx[k]].push_back({k, i});
    int zc = 1, zr = 1;
    for (int j = 0; j < n; ++j) zc = std::max(zc, (int)cols[j].size());
    for (int i = 0; i < m; ++i) zr = std::max(zr, (int)(row_ptr[i + 1] - row_ptr[i]));
    int inst = -1;
    long best = 0;
    const int ninst = (int)(sizeof(g_reg_instances) / sizeof(g_reg_instances[0]));
    for (int a = 0; a < ninst; ++a) {
        const reg_instance& r = g_reg_instances[a];
        if (r.KC >= kc && r.ZC >= zc && r.KR >= kr && r.ZR >= zr) {
            const long cost = reg_cost(r);
            if (inst < 0 || cost < best) {
                inst = a;
                best = cost;
            }
        }
    }
    if (inst < 0) return false;
    col_k.assign((size_t)L * kc * zc, -1);
    col_r.assign((size_t)L * kc * zc, 0);
    for (int u = 0; u < L; ++u)
        for (int q = 0; q < kc; ++q) {
            const int j = u + q * L;
            if (j >= n) continue;
            for (int z = 0; z < (int)cols[j].size(); ++z) {
                col_k[((size_t)u * kc + q) * zc + z] = cols[j][z].first;
                col_r[((size_t)u * kc + q) * zc + z] = cols[j][z].second;
            }
        }
    row_k.assign((size_t)L * kr * zr, -1);
    row_c.assign((size_t)L * kr * zr, 0);
    for (int u = 0; u < L; ++u)
        for (int r = 0; r < kr; ++r) {
            const int i = u + r * L;
            if (i >= m) continue;
            for (int k = row_ptr[i], z = 0; k < row_ptr[i + 1]; ++k, ++z) {
                row_k[((size_t)u * kr + r) * zr + z] = k;
                row_c[((size_t)u * kr + r) * zr + z] = col_idx[k];
            }
        }
    *inst_out = inst;
    *kc_out = kc;
    *zc_out = zc;
    *kr_out = kr;
    *zr_out = zr;
    return true;
}

// per-lane VALU estimate of one PDHG iteration of a slot layout, shared by the path
// choice: a column slot ~ 10 + 2 ZC instructions, a row slot ~ 8 + 2 ZR, each long slot's
// wave reduction ~ 20.  A scenario costs (lanes / 64) times that.
static inline long slot_cost(int KC, int ZC, int KR, int ZR, int nlong) {
    return (long)KC * (10 + 2 * ZC) + (long)KR * (8 + 2 * ZR) + 20L * nlong;
}

// The workgroup kernels spill only around a scenario's load and write-back (the solve
// loops of every instance are scratch-free: objdump of the code object), once per
// several hundred PDHG iterations, so their cap is looser than the register path's.
#define WG_SPILL_MAX 512
static bool wg_spills(const wg_instance& g) {
    hipFuncAttributes a;
    if (hipFuncGetAttributes(&a, (const void*)g.fn) != hipSuccess) return false;
    return a.localSizeBytes > WG_SPILL_MAX;
}

struct wg_plan_host {
    int nlong = 0, long_per_wave = 0;
    std::vector<int32_t> col_id, row_id, col_long, row_long, col_k, col_r, row_k, row_c;
};

// Assign K slots x L lanes to N items (rows or columns) with entry lists ``items``
// (pairs CSR position, partner index), padded to Z entries per slot.  An item with more
// than Z entries is long: it takes a whole wave slot (from the last slot / wave
// backwards), its entries split evenly over the wave's 64 lanes; the short items fill the
// remaining (slot, lane) positions in order.  False if they do not fit.
static bool wg_assign(int K, int Z, int W, const std::vector<std::vector<std::pair<int, int>>>& items,
                      std::vector<int32_t>& id, std::vector<int32_t>& lng, std::vector<int32_t>& ek,
                      std::vector<int32_t>& eo, int& nlong, std::vector<int>& per_wave) {
    const int L = WAVE * W;
    const int N = (int)items.size();
    id.assign((size_t)K * L, -1);
    lng.assign((size_t)K * W, 0);
    ek.assign((size_t)K * L * Z, -1);
    eo.assign((size_t)K * L * Z, 0);
    std::vector<char> taken((size_t)K * W, 0);
    int ws = K * W - 1;
    for (int a = 0; a < N; ++a) {
        const int d = (int)items[a].size();
        if (d <= Z) continue;
        if (d > WAVE * Z || ws < 0) return false;
        const int q = ws / W, w = ws % W;
        --ws;
        taken[(size_t)q * W + w] = 1;
        lng[(size_t)q * W + w] = 1;
        ++nlong;
        ++per_wave[w];
        const int per = (d + WAVE - 1) / WAVE;
        for (int l = 0; l < WAVE; ++l) {
            const size_t slot = (size_t)q * L + w * WAVE + l;
            id[slot] = a;
            for (int z = 0; z < per; ++z) {
                const int e = l * per + z;
                if (e >= d) break;
                ek[slot * Z + z] = items[a][e].first;
                eo[slot * Z + z] = items[a][e].second;
            }
        }
    }
    long pos = 0;  // q-major over (slot, lane)
    for (int a = 0; a < N; ++a) {
        const int d = (int)items[a].size();
        if (d > Z) continue;
        while (pos < (long)K * L && taken[(size_t)(pos / L) * W + (pos % L) / WAVE])
            pos = (pos / WAVE + 1) * WAVE;     // skip the rest of a long-item wave slot
        if (pos >= (long)K * L) return false;
        const size_t slot = (size_t)pos;
        id[slot] = a;
        for (int z = 0; z < d; ++z) {
            ek[slot * Z + z] = items[a][z].first;
            eo[slot * Z + z] = items[a][z].second;
        }
        ++pos;
    }
    return true;
}

// Plan of solve_wg.inc for one instance.
static bool build_wg_plan(const wg_instance& g, int n, int m, const int32_t* row_ptr, const int32_t* col_idx,
                          wg_plan_host& out) {
    if (m < 1 || n < 1) return false;
    std::vector<std::vector<std::pair<int, int>>> cols(n), rows(m);
    for (int i = 0; i < m; ++i)
        for (int k = row_ptr[i]; k < row_ptr[i + 1]; ++k) {
            cols[col_idx[k]].push_back({k, i});
            rows[i].push_back({k, col_idx[k]});
        }
    std::vector<int> pwc(g.WPS, 0), pwr(g.WPS, 0);
    int nl = 0;
    if (!wg_assign(g.KC, g.ZC, g.WPS, cols, out.col_id, out.col_long, out.col_k, out.col_r, nl, pwc)) return false;
    if (!wg_assign(g.KR, g.ZR, g.WPS, rows, out.row_id, out.row_long, out.row_k, out.row_c, nl, pwr)) return false;
    out.nlong = nl;
    out.long_per_wave = 0;
    for (int w = 0; w < g.WPS; ++w) out.long_per_wave = std::max(out.long_per_wave, pwc[w] + pwr[w]);
    return true;
}

// ------------------------------------------------------------------ C-ABI
template <typename T>
static int dalloc(phgpu_state* h, T** p, size_t count) {
    *p = nullptr;
    if (count == 0) count = 1;
    hipError_t e = hipMalloc((void**)p, count * sizeof(T));
    if (e != hipSuccess) return set_err(-3, "hipMalloc(%zu bytes) failed: %s", count * sizeof(T), hipGetErrorString(e));
    h->ws_bytes += (int64_t)(count * sizeof(T));
    return 0;
}

#define ALLOC(ptr, cnt)                         \
    do {                                        \
        int rc_ = dalloc(h, &(ptr), (size_t)(cnt)); \
        if (rc_) { phgpu_destroy(h); return rc_; } \
    } while (0)

// ---------------------------------------------------------- scenario-major records
static hipError_t to_records(phgpu_state* h, const double* in, int K, int off, hipStream_t st) {
    if (K <= 0) return hipSuccess;
    const dim3 g((unsigned)((h->S + TT - 1) / TT), (unsigned)((K + TT - 1) / TT));
    hipLaunchKernelGGL(k_to_records, g, dim3(256), 0, st, in, K, h->S, h->pk, h->pk_stride, off);
    return hipGetLastError();
}

// this solve's PH state (W if on, rho and xbar if the prox term is on) into the records
static hipError_t ph_to_records(phgpu_state* h, hipStream_t st) {
    if (h->nn <= 0 || (!h->W_on && !h->prox_on)) return hipSuccess;
    const dim3 g((unsigned)((h->S + TT - 1) / TT), (unsigned)((3 * h->nn + TT - 1) / TT));
    hipLaunchKernelGGL(k_to_records_ph, g, dim3(256), 0, st, h->W_on ? h->W : nullptr,
                       h->prox_on ? h->rho : nullptr, h->prox_on ? h->xbar : nullptr, h->nn, h->S, h->pk,
                       h->pk_stride, h->pk_W);
    return hipGetLastError();
}

static hipError_t from_records(phgpu_state* h, int off, int moff, int K, double* out, hipStream_t st) {
    if (K <= 0 || !out) return hipSuccess;
    const dim3 g((unsigned)((h->S + TT - 1) / TT), (unsigned)((K + TT - 1) / TT));
    hipLaunchKernelGGL(k_from_records, g, dim3(256), 0, st, (const double*)h->pk, h->pk_stride, off, moff, K,
                       h->S, out);
    return hipGetLastError();
}

// Point the warm-state fields at slot wslot (read) and slot ``wq`` (write; == wslot except
// during a deferred solve) -- see the slot fields of phgpu_state.
static void bind_slots(phgpu_state* h) {
    const int p = h->wslot, wq = h->wq;
    h->x = h->xs[p];
    h->y = h->ys[p];
    h->omega = h->oms[p];
    h->sk_iters = h->its_s[p];
    h->pk_X = h->pkXs[p];
    h->pk_Y = h->pkYs[p];
    h->have_solution = h->have_s[p];
    h->warm_rec = h->warm_rec_s[p];
    h->xw = h->xs[wq];
    h->yw = h->ys[wq];
    h->omega_w = h->oms[wq];
    h->its_w = h->its_s[wq];
    h->pk_XW = h->pkXs[wq];
    h->pk_YW = h->pkYs[wq];
}

// record layout: A (CSR order) | c q Dc lb^ ub^ (n) | rl ru Dr rl^ ru^ (m) | x^ (n) y^ (m)
// warm start of slot 0 | W rho xbar (nn) PH state of the current solve | x^ (n) y^ (m) warm
// start of slot 1; stride rounded to 16 doubles
static int pack_alloc(phgpu_state* h) {
    if (h->pk) return 0;
    const int n = h->n, m = h->m, nnz = h->nnz, nn = h->nn;
    int o = 0;
    h->pk_A = o; o += nnz;
    h->pk_C = o; o += n;
    h->pk_Q = o; o += n;
    h->pk_DC = o; o += n;
    h->pk_LB = o; o += n;
    h->pk_UB = o; o += n;
    h->pk_RL = o; o += m;
    h->pk_RU = o; o += m;
    h->pk_DR = o; o += m;
    h->pk_RLH = o; o += m;
    h->pk_RUH = o; o += m;
    h->pk_X = o; o += n;
    h->pk_Y = o; o += m;
    h->pk_W = o; o += nn;
    h->pk_RHO = o; o += nn;
    h->pk_XB = o; o += nn;
    h->pkXs[0] = h->pk_X;
    h->pkYs[0] = h->pk_Y;
    h->pkXs[1] = o; o += n;
    h->pkYs[1] = o; o += m;
    h->pk_stride = (o + 15) / 16 * 16;
    bind_slots(h);
    return dalloc(h, &h->pk, (size_t)h->pk_stride * (size_t)h->S);
}

// copy the scaled problem (k_setup's output) into the records
static hipError_t pack_fill(phgpu_state* h, hipStream_t st) {
    struct { const double* a; int K, off; } f[] = {
        {h->Ah_csr, h->nnz, h->pk_A}, {h->c, h->n, h->pk_C}, {h->q, h->n, h->pk_Q}, {h->Dc, h->n, h->pk_DC},
        {h->lbh, h->n, h->pk_LB}, {h->ubh, h->n, h->pk_UB}, {h->rl, h->m, h->pk_RL}, {h->ru, h->m, h->pk_RU},
        {h->Dr, h->m, h->pk_DR}, {h->rlh, h->m, h->pk_RLH}, {h->ruh, h->m, h->pk_RUH}, {h->x, h->n, h->pk_X},
        {h->y, h->m, h->pk_Y}};
    for (auto& e : f) {
        const hipError_t r = to_records(h, e.a, e.K, e.off, st);
        if (r != hipSuccess) return r;
    }
    return hipSuccess;
}

// sliced-ELL layout of the shared pattern (rows and columns in slices of 64); values are
// filled from the scaled CSR / CSC copies by k_sh_sell_vals
static int sell_one(phgpu_state* h, int K, const std::vector<int32_t>& ptr, const std::vector<int32_t>& idx,
                    const std::vector<int32_t>& src, int& nsl, int& nent, int32_t** d_off, int32_t** d_len, int32_t** d_idx,
                    int32_t** d_src, double** d_val, int32_t** d_wptr, int32_t** d_wslc) {
    nsl = (K + WAVE - 1) / WAVE;
    std::vector<int32_t> off((size_t)nsl + 1), len((size_t)nsl);
    int64_t tot = 0;
    for (int sl = 0; sl < nsl; ++sl) {
        int L = 0;
        for (int l = 0; l < WAVE; ++l) {
            const int r = sl * WAVE + l;
            if (r < K) L = std::max(L, ptr[r + 1] - ptr[r]);
        }
        off[sl] = (int32_t)tot;
        len[sl] = L;
        tot += (int64_t)L * WAVE;
        if (tot >= (1LL << 31)) return set_err(-1, "sliced-ELL copy too large");
    }
    off[nsl] = (int32_t)tot;
    nent = (int)tot;
    std::vector<int32_t> e_idx((size_t)std::max<int64_t>(tot, 1), 0), e_src((size_t)std::max<int64_t>(tot, 1), -1);
    for (int sl = 0; sl < nsl; ++sl)
        for (int l = 0; l < WAVE; ++l) {
            const int r = sl * WAVE + l;
            if (r >= K) continue;
            for (int k = 0; k < ptr[r + 1] - ptr[r]; ++k) {
                const size_t e = (size_t)off[sl] + (size_t)k * WAVE + l;
                e_idx[e] = idx[ptr[r] + k];
                e_src[e] = src[ptr[r] + k];
            }
        }
    // slices -> waves of the streaming workgroup: longest first onto the least loaded wave
    // (cost = entries per lane + a fixed per-slice overhead), each wave's list in slice order
    std::vector<int32_t> bysz((size_t)nsl);
    for (int sl = 0; sl < nsl; ++sl) bysz[sl] = sl;
    std::stable_sort(bysz.begin(), bysz.end(), [&](int a, int b) { return len[a] > len[b]; });
    std::vector<int64_t> load(SWAVES, 0);
    std::vector<std::vector<int32_t>> lists(SWAVES);
    for (int sl : bysz) {
        int w = 0;
        for (int v = 1; v < SWAVES; ++v)
            if (load[v] < load[w]) w = v;
        load[w] += len[sl] + 4;
        lists[w].push_back(sl);
    }
    std::vector<int32_t> wptr(SWAVES + 1, 0), wslc;
    for (int w = 0; w < SWAVES; ++w) {
        std::sort(lists[w].begin(), lists[w].end());
        wslc.insert(wslc.end(), lists[w].begin(), lists[w].end());
        wptr[w + 1] = (int32_t)wslc.size();
    }
    if (dalloc(h, d_off, off.size()) || dalloc(h, d_len, len.size()) || dalloc(h, d_idx, e_idx.size()) ||
        dalloc(h, d_src, e_src.size()) || dalloc(h, d_val, e_idx.size()) || dalloc(h, d_wptr, wptr.size()) ||
        dalloc(h, d_wslc, std::max<size_t>(wslc.size(), 1)))
        return -3;
    hipError_t e = hipMemcpy(*d_off, off.data(), off.size() * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(*d_len, len.data(), std::max<size_t>(len.size(), 1) * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(*d_idx, e_idx.data(), e_idx.size() * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(*d_src, e_src.data(), e_src.size() * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(*d_wptr, wptr.data(), wptr.size() * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess && !wslc.empty()) e = hipMemcpy(*d_wslc, wslc.data(), wslc.size() * 4, hipMemcpyHostToDevice);
    if (e != hipSuccess) return set_err(-2, "sliced-ELL upload failed: %s", hipGetErrorString(e));
    return 0;
}

static int build_sell(phgpu_state* h, const int32_t* row_ptr, const int32_t* col_idx) {
    const int n = h->n, m = h->m, nnz = h->nnz;
    // rows: CSR as given, source = CSR position
    std::vector<int32_t> rp(row_ptr, row_ptr + m + 1), ci(col_idx, col_idx + nnz), rsrc((size_t)nnz);
    for (int k = 0; k < nnz; ++k) rsrc[k] = k;
    int rc = sell_one(h, m, rp, ci, rsrc, h->nsl_r, h->nent_r, &h->rs_off, &h->rs_len, &h->rs_idx, &h->rs_src, &h->rs_val,
                      &h->rw_ptr, &h->rw_slc);
    if (rc) return rc;
    // columns: the CSC order of phgpu_create (rows ascending within a column), source =
    // CSC position
    std::vector<int32_t> cp((size_t)n + 1, 0), ri((size_t)nnz), csrc((size_t)nnz);
    for (int k = 0; k < nnz; ++k) cp[col_idx[k] + 1]++;
    for (int j = 0; j < n; ++j) cp[j + 1] += cp[j];
    std::vector<int32_t> fill(cp.begin(), cp.end() - 1);
    for (int i = 0; i < m; ++i)
        for (int k = row_ptr[i]; k < row_ptr[i + 1]; ++k) {
            const int p = fill[col_idx[k]]++;
            ri[p] = i;
            csrc[p] = p;
        }
    return sell_one(h, n, cp, ri, csrc, h->nsl_c, h->nent_c, &h->cs_off, &h->cs_len, &h->cs_idx, &h->cs_src, &h->cs_val,
                    &h->cw_ptr, &h->cw_slc);
}

static int step_local_impl(phgpu_state* h, const double* x, double* node_buf, double* xbar, double* W,
                           const double* rho, int update_W, double* conv_local, int64_t* stats_out, hipStream_t st);

static bool xp_valid(const phgpu_state* h, const double* x);

// run a deferred PH step now (its recorded stream), if one is pending
static int flush_step(phgpu_state* h) {
    if (!h || !h->pend.active) return 0;
    phgpu_state::ph_pending q = h->pend;
    h->pend.active = 0;
    return step_local_impl(h, q.x, q.node_buf, q.xbar, q.W, q.rho, q.update_W, q.conv, q.stats, q.stream);
}
#define FLUSH_STEP(h)                      \
    do {                                   \
        const int frc_ = flush_step(h);    \
        if (frc_) return frc_;             \
    } while (0)

extern "C" int phgpu_default_options(phgpu_options* o) {
    if (!o) return set_err(-1, "null options");
    o->eps_rel = 1e-9;
    o->eps_abs = 1e-12;
    o->max_iter = 100000;
    o->check_every = 64;
    o->gamma = 1.0;
    o->beta_sufficient = 0.2;
    o->beta_necessary = 0.8;
    o->eta_frac = 0.998;
    o->omega0 = 1.0;
    o->keep_omega = 1;
    o->restart_every = 16;
    o->beta_artificial = 0.36;
    o->omega_clamp = 1e4;
    o->kernel = 0;
    o->infeas_start = 512;
    o->eps_infeas = 1e-8;
    o->split_longest = 0;
    return 0;
}

extern "C" int phgpu_create(phgpu_handle* out, int device, int64_t S, int32_t n, int32_t m,
                            int32_t nnz, const int32_t* row_ptr, const int32_t* col_idx,
                            int32_t nn, const int32_t* nonant_col, const int32_t* nonant_depth,
                            const int32_t* nonant_off, int32_t depth, int32_t num_nodes,
                            int32_t nlen_max) {
    return phgpu_create2(out, device, S, n, m, nnz, row_ptr, col_idx, nn, nonant_col, nonant_depth, nonant_off,
                         depth, num_nodes, nlen_max, 0u);
}

extern "C" int phgpu_create2(phgpu_handle* out, int device, int64_t S, int32_t n, int32_t m,
                             int32_t nnz, const int32_t* row_ptr, const int32_t* col_idx,
                             int32_t nn, const int32_t* nonant_col, const int32_t* nonant_depth,
                             const int32_t* nonant_off, int32_t depth, int32_t num_nodes,
                             int32_t nlen_max, uint32_t flags) {
    if (flags & ~(uint32_t)PHGPU_SHARED_MATRIX) return set_err(-1, "unknown flags 0x%x", flags);
    if (!out) return set_err(-1, "null handle pointer");
    *out = nullptr;
    if (S <= 0 || S >= (1LL << 31) || n <= 0 || m < 0 || nnz < 0 || nn < 0 || depth < 1 || num_nodes < 1 ||
        nlen_max < 0)
        return set_err(-1, "bad sizes S=%lld n=%d m=%d nnz=%d nn=%d depth=%d nodes=%d",
                       (long long)S, n, m, nnz, nn, depth, num_nodes);
    if (!row_ptr || (nnz > 0 && !col_idx) || (nn > 0 && (!nonant_col || !nonant_depth || !nonant_off)))
        return set_err(-1, "null pattern pointer");
    // host-side validation of the shared pattern
    if (row_ptr[0] != 0 || row_ptr[m] != nnz) return set_err(-1, "row_ptr must start at 0 and end at nnz");
    for (int i = 0; i < m; ++i)
        if (row_ptr[i + 1] < row_ptr[i]) return set_err(-1, "row_ptr not monotone at row %d", i);
    for (int k = 0; k < nnz; ++k)
        if (col_idx[k] < 0 || col_idx[k] >= n) return set_err(-1, "col_idx[%d]=%d out of range", k, col_idx[k]);
    int32_t* slot = new int32_t[n];
    for (int j = 0; j < n; ++j) slot[j] = -1;
    for (int k = 0; k < nn; ++k) {
        if (nonant_col[k] < 0 || nonant_col[k] >= n || slot[nonant_col[k]] >= 0 ||
            nonant_depth[k] < 0 || nonant_depth[k] >= depth || nonant_off[k] < 0 ||
            nonant_off[k] >= nlen_max) {
            delete[] slot;
            return set_err(-1, "bad nonant map at %d", k);
        }
        slot[nonant_col[k]] = k;
    }
    HIPCHK(hipSetDevice(device));
    phgpu_state* h = new (std::nothrow) phgpu_state();
    if (!h) {
        delete[] slot;
        return set_err(-3, "out of host memory");
    }
    memset(h, 0, sizeof(*h));
    h->last_rec = -1;
    h->device = device;
    h->S = S;
    h->n = n;
    h->m = m;
    h->nnz = nnz;
    h->nn = nn;
    h->depth = depth;
    h->num_nodes = num_nodes;
    h->nlen_max = nlen_max;
    h->nwaves = (S + WAVE - 1) / WAVE;
    h->xbar_mixed = -1;
    // transposed pattern (host)
    int32_t* cptr = new int32_t[n + 1]();
    int32_t* ridx = new int32_t[nnz > 0 ? nnz : 1];
    int32_t* perm = new int32_t[nnz > 0 ? nnz : 1];
    int32_t* rowof = new int32_t[nnz > 0 ? nnz : 1];
    for (int k = 0; k < nnz; ++k) cptr[col_idx[k] + 1]++;
    for (int j = 0; j < n; ++j) cptr[j + 1] += cptr[j];
    {
        int32_t* fill = new int32_t[n];
        for (int j = 0; j < n; ++j) fill[j] = cptr[j];
        for (int i = 0; i < m; ++i)
            for (int k = row_ptr[i]; k < row_ptr[i + 1]; ++k) {
                const int p = fill[col_idx[k]]++;
                ridx[p] = i;
                perm[p] = k;
                rowof[k] = i;
            }
        delete[] fill;
    }
    const size_t Sz = (size_t)S;
    int rc = 0;
    ALLOC(h->row_ptr, m + 1);
    ALLOC(h->col_idx, nnz);
    ALLOC(h->col_ptr, n + 1);
    ALLOC(h->row_idx, nnz);
    ALLOC(h->perm, nnz);
    ALLOC(h->row_of, nnz);
    ALLOC(h->nonant_col, nn);
    ALLOC(h->nonant_depth, nn);
    ALLOC(h->nonant_off, nn);
    ALLOC(h->nonant_slot, n);
    ALLOC(h->objc, Sz);
    ALLOC(h->prob, Sz);
    ALLOC(h->pcoef, (size_t)depth * Sz);
    ALLOC(h->node_of, (size_t)depth * Sz);
    ALLOC(h->omega, Sz);
    h->shared = (flags & PHGPU_SHARED_MATRIX) ? 1 : 0;
    // longest-first work queue (paths 2 and 4): iteration counts of the last solve, the
    // queue order and the counting-sort bins
    ALLOC(h->sk_iters, Sz);
    ALLOC(h->sk_order, Sz);
    ALLOC(h->sk_bins, 4 * ORDER_BINS);
    if (hipMemset(h->sk_bins, 0, 4 * ORDER_BINS * sizeof(int32_t)) != hipSuccess) {
        phgpu_destroy(h);
        return set_err(-2, "hipMemset failed");
    }
    if (h->shared) {
        // one scaled matrix; iterates and per-scenario data live in the stream records
        // (allocated by phgpu_set_scenarios once the per-scenario column set is known)
        ALLOC(h->A, nnz);
        ALLOC(h->Ah_csr, nnz);
        ALLOC(h->Ah_csc, nnz);
        ALLOC(h->Dr, m);
        ALLOC(h->Dc, n);
        ALLOC(h->cmap, n);
        ALLOC(h->rmap, m);
        ALLOC(h->sh_col, 4 * (size_t)n);
        ALLOC(h->sh_row, 4 * (size_t)m);
        ALLOC(h->sh_norm, 4);
        ALLOC(h->sh_v, n);
        ALLOC(h->sh_u, n);
        ALLOC(h->sh_w, m);
        ALLOC(h->sh_part, (size_t)(n + 255) / 256 + 1);
    } else {
        ALLOC(h->A, (size_t)nnz * Sz);
        ALLOC(h->c, (size_t)n * Sz);
        ALLOC(h->lb, (size_t)n * Sz);
        ALLOC(h->ub, (size_t)n * Sz);
        ALLOC(h->q, (size_t)n * Sz);
        ALLOC(h->rl, (size_t)m * Sz);
        ALLOC(h->ru, (size_t)m * Sz);
        ALLOC(h->Ah_csr, (size_t)nnz * Sz);
        ALLOC(h->Ah_csc, (size_t)nnz * Sz);
        ALLOC(h->Dr, (size_t)m * Sz);
        ALLOC(h->Dc, (size_t)n * Sz);
        ALLOC(h->normA, Sz);
        ALLOC(h->lbh, (size_t)n * Sz);
        ALLOC(h->ubh, (size_t)n * Sz);
        ALLOC(h->rlh, (size_t)m * Sz);
        ALLOC(h->ruh, (size_t)m * Sz);
        ALLOC(h->ch, (size_t)n * Sz);
        ALLOC(h->qh, (size_t)n * Sz);
        ALLOC(h->x, (size_t)n * Sz);
        ALLOC(h->x0, (size_t)n * Sz);
        ALLOC(h->xe, (size_t)n * Sz);
        ALLOC(h->xt, (size_t)n * Sz);
        ALLOC(h->aty, (size_t)n * Sz);
        ALLOC(h->aty0, (size_t)n * Sz);
        ALLOC(h->y, (size_t)m * Sz);
        ALLOC(h->y0, (size_t)m * Sz);
        ALLOC(h->yt, (size_t)m * Sz);
    }
    ALLOC(h->qhead, 1);
    ALLOC(h->stats_gen, 8);
    if (!h->shared) {  // path 6: the pattern's factor size, the fallback list and its counters
        h->ipm_nf = ipm_nf_bound(n, m, row_ptr, col_idx);
        if (!(h->ipm_nf > 0 && h->ipm_nf <= IPM_MAX_NF && n <= JIT_MAX_N && m <= JIT_MAX_M && nnz <= JIT_MAX_NNZ))
            h->ipm_wave = ipm_wg_bound(n, m, nnz, row_ptr, col_idx);
        if (h->ipm_nf > 0 || h->ipm_wave > 0) {
            ALLOC(h->ipm_list, Sz);
            ALLOC(h->ipm_cnt, 6);
            ALLOC(h->ipm_stats, 2 * PHGPU_STATS_WORDS);
            if (getenv("PHGPU_IPM_PROF")) {  // diagnostics: 16 words per wave of the widest plan
                h->ipm_prof_n = 16 * ((Sz * 64 + 63) / 64 + 64);
                ALLOC(h->ipm_prof, h->ipm_prof_n);
            }
            if (hipMemset(h->ipm_cnt, 0, 6 * sizeof(int32_t)) != hipSuccess ||
                hipMemset(h->ipm_stats, 0, 2 * PHGPU_STATS_WORDS * sizeof(unsigned long long)) != hipSuccess) {
                phgpu_destroy(h);
                return set_err(-2, "hipMemset failed");
            }
        }
    }
    // warm-start slots: slot 0 is the arrays above; slot 1 (deferred solves, paths 1-3)
    h->xs[0] = h->x;
    h->ys[0] = h->y;
    h->oms[0] = h->omega;
    h->its_s[0] = h->sk_iters;
    if (h->shared) {  // path 4 solves are never deferred: both slots are slot 0
        h->xs[1] = h->x;
        h->ys[1] = h->y;
        h->oms[1] = h->omega;
        h->its_s[1] = h->sk_iters;
    } else {
        ALLOC(h->xs[1], (size_t)n * Sz);
        ALLOC(h->ys[1], (size_t)m * Sz);
        ALLOC(h->oms[1], Sz);
        ALLOC(h->its_s[1], Sz);
    }
    h->pending = -1;
    bind_slots(h);
    {
        int ncu = 0;
        if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || ncu < 1)
            ncu = 256;
        h->num_cus = ncu;
    }
    {
        // per-wave partials [nwaves * K] + the conv partials of phgpu_ph_step_local [nwaves]
        size_t K = (size_t)(2 * nn > 5 ? 2 * nn : 5);
        ALLOC(h->part, (size_t)h->nwaves * (K + 1));
        ALLOC(h->part_node, (size_t)h->nwaves * (nn > 0 ? nn : 1));
        // path-6 epilogue partials (two slots) and the update kernels' conv partials (one
        // per block of the widest update grid: 64 lanes per block at least)
        if (!h->shared && h->ipm_nf > 0 && nn > 0 && nn <= XL_NN_MAX) {
            const size_t nch = (Sz + XP_CHUNK_MIN - 1) / XP_CHUNK_MIN;
            for (int k = 0; k < 2; ++k) {
                ALLOC(h->xp[k], nch * 2 * (size_t)nn);
                ALLOC(h->xp_node[k], nch * (size_t)nn);
                ALLOC(h->xp_dirty[k], nch);
            }
        }
        // one per block of the widest grid (path-6 lane groups of 16; k_ph_update's nonant x
        // scenario-block grid)
        ALLOC(h->cpart_blk, std::max<size_t>((Sz + 15) / 16 + 1, (size_t)std::max(nn, 1) * ((Sz + UPD_T - 1) / UPD_T) + 1));
        ALLOC(h->blk_cnt, 4);
        if (hipMemset(h->blk_cnt, 0, 4 * sizeof(int32_t)) != hipSuccess) {
            phgpu_destroy(h);
            return set_err(-2, "hipMemset failed");
        }
    }
    (void)rc;
    hipError_t e = hipSuccess;
    e = hipMemcpy(h->row_ptr, row_ptr, (m + 1) * sizeof(int32_t), hipMemcpyHostToDevice);
    if (e == hipSuccess && nnz) e = hipMemcpy(h->col_idx, col_idx, nnz * sizeof(int32_t), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(h->col_ptr, cptr, (n + 1) * sizeof(int32_t), hipMemcpyHostToDevice);
    if (e == hipSuccess && nnz) e = hipMemcpy(h->row_idx, ridx, nnz * sizeof(int32_t), hipMemcpyHostToDevice);
    if (e == hipSuccess && nnz) e = hipMemcpy(h->perm, perm, nnz * sizeof(int32_t), hipMemcpyHostToDevice);
    if (e == hipSuccess && nnz) e = hipMemcpy(h->row_of, rowof, nnz * sizeof(int32_t), hipMemcpyHostToDevice);
    if (e == hipSuccess && nn) e = hipMemcpy(h->nonant_col, nonant_col, nn * sizeof(int32_t), hipMemcpyHostToDevice);
    if (e == hipSuccess && nn) e = hipMemcpy(h->nonant_depth, nonant_depth, nn * sizeof(int32_t), hipMemcpyHostToDevice);
    if (e == hipSuccess && nn) e = hipMemcpy(h->nonant_off, nonant_off, nn * sizeof(int32_t), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(h->nonant_slot, slot, n * sizeof(int32_t), hipMemcpyHostToDevice);
    delete[] cptr;
    delete[] ridx;
    delete[] perm;
    delete[] rowof;
    delete[] slot;
    if (e != hipSuccess) {
        phgpu_destroy(h);
        return set_err(-2, "pattern upload failed: %s", hipGetErrorString(e));
    }
    // register-resident path: lanes per scenario L (power of two <= 64): the smallest L
    // with a fitting instance, doubled while S * L lanes would not fill REG_WAVES_PER_EU
    // waves on every SIMD of the chip and a scenario still has columns to spread
    // (measured on farmer cm=1: L=4 at S >= 32768, 8 at 16384, 16 at 8192 -- profiles/r01),
    // and past any L whose instance spills (reg_spills);
    // PHGPU_LANES=<L> pins it (tuning / tests)
    h->reg_inst = -1;
    h->wg_inst = -1;
    if (h->shared) {
        const int rcs = build_sell(h, row_ptr, col_idx);
        if (rcs) {
            phgpu_destroy(h);
            return rcs;
        }
        h->default_kernel = 4;
        *out = h;
        return 0;
    }
    {
        const int64_t target = (int64_t)h->num_cus * 4 * WAVE * REG_WAVES_PER_EU;
        const char* env = getenv("PHGPU_LANES");
        const int pinned = env ? atoi(env) : 0;
        int chosen = -1;
        bool chosen_spills = false;
        std::vector<int32_t> ck, cr, rk, rc;
        int inst = -1, kc = 0, zc = 0, kr = 0, zr = 0;
        for (int L = 1; L <= WAVE; L *= 2) {
            if (pinned > 0 && L != pinned) continue;
            std::vector<int32_t> a1, a2, a3, a4;
            int i1, i2, i3, i4, i5;
            if (!build_plan(L, n, m, row_ptr, col_idx, &i1, &i2, &i3, &i4, &i5, a1, a2, a3, a4)) continue;
            if (pinned <= 0 && chosen >= 0 && (S * (int64_t)chosen >= target || chosen >= n) &&
                !chosen_spills)
                break;
            chosen = L;
            chosen_spills = reg_spills(g_reg_instances[i1]);
            inst = i1; kc = i2; zc = i3; kr = i4; zr = i5;
            ck.swap(a1); cr.swap(a2); rk.swap(a3); rc.swap(a4);
        }
        if (chosen > 0) {
            int rc2 = 0;
            rc2 |= dalloc(h, &h->pl_col_k, ck.size());
            rc2 |= dalloc(h, &h->pl_col_r, cr.size());
            rc2 |= dalloc(h, &h->pl_row_k, rk.size());
            rc2 |= dalloc(h, &h->pl_row_c, rc.size());
            if (rc2) {
                phgpu_destroy(h);
                return set_err(-3, "plan allocation failed");
            }
            e = hipMemcpy(h->pl_col_k, ck.data(), ck.size() * 4, hipMemcpyHostToDevice);
            if (e == hipSuccess) e = hipMemcpy(h->pl_col_r, cr.data(), cr.size() * 4, hipMemcpyHostToDevice);
            if (e == hipSuccess) e = hipMemcpy(h->pl_row_k, rk.data(), rk.size() * 4, hipMemcpyHostToDevice);
            if (e == hipSuccess) e = hipMemcpy(h->pl_row_c, rc.data(), rc.size() * 4, hipMemcpyHostToDevice);
            if (e != hipSuccess) {
                phgpu_destroy(h);
                return set_err(-2, "plan upload failed: %s", hipGetErrorString(e));
            }
            h->reg_inst = inst;
            h->reg_L = chosen;
            h->reg_kc = kc;
            h->reg_zc = zc;
            h->reg_kr = kr;
            h->reg_zr = zr;
        }
    }
    // workgroup-per-scenario path: the cheapest non-spilling instance by slot_cost x waves
    // per scenario (PHGPU_WPS=<waves> pins the waves per scenario)
    h->wg_inst = -1;
    {
        const char* env = getenv("PHGPU_WPS");
        const int pinned = env ? atoi(env) : 0;
        const int ninst = (int)(sizeof(g_wg_instances) / sizeof(g_wg_instances[0]));
        long best = 0;
        wg_plan_host bp;
        for (int a = 0; a < ninst; ++a) {
            const wg_instance& g = g_wg_instances[a];
            if (pinned > 0 && g.WPS != pinned) continue;
            wg_plan_host p;
            if (!build_wg_plan(g, n, m, row_ptr, col_idx, p)) continue;
            if (wg_spills(g)) continue;
            const long cost = (long)g.WPS * slot_cost(g.KC, g.ZC, g.KR, g.ZR, p.long_per_wave);
            if (h->wg_inst < 0 || cost < best) {
                h->wg_inst = a;
                best = cost;
                bp = std::move(p);
            }
        }
        if (h->wg_inst >= 0) {
            int rc2 = 0;
            rc2 |= dalloc(h, &h->wg_col_id, bp.col_id.size());
            rc2 |= dalloc(h, &h->wg_row_id, bp.row_id.size());
            rc2 |= dalloc(h, &h->wg_col_long, bp.col_long.size());
            rc2 |= dalloc(h, &h->wg_row_long, bp.row_long.size());
            rc2 |= dalloc(h, &h->wg_col_k, bp.col_k.size());
            rc2 |= dalloc(h, &h->wg_col_r, bp.col_r.size());
            rc2 |= dalloc(h, &h->wg_row_k, bp.row_k.size());
            rc2 |= dalloc(h, &h->wg_row_c, bp.row_c.size());
            if (rc2) {
                phgpu_destroy(h);
                return set_err(-3, "workgroup plan allocation failed");
            }
            struct { int32_t* d; std::vector<int32_t>* v; } up[] = {
                {h->wg_col_id, &bp.col_id}, {h->wg_row_id, &bp.row_id}, {h->wg_col_long, &bp.col_long},
                {h->wg_row_long, &bp.row_long}, {h->wg_col_k, &bp.col_k}, {h->wg_col_r, &bp.col_r},
                {h->wg_row_k, &bp.row_k}, {h->wg_row_c, &bp.row_c}};
            for (auto& u : up)
                if (e == hipSuccess) e = hipMemcpy(u.d, u.v->data(), u.v->size() * 4, hipMemcpyHostToDevice);
            if (e != hipSuccess) {
                phgpu_destroy(h);
                return set_err(-2, "workgroup plan upload failed: %s", hipGetErrorString(e));
            }
            h->wg_long = bp.nlong;
        }
        // default path: the cheaper per scenario (register path at its chosen L)
        long reg_cost_s = -1;
        if (h->reg_inst >= 0) {
            const reg_instance& r = g_reg_instances[h->reg_inst];
            reg_cost_s = (long)h->reg_L * slot_cost(r.KC, r.ZC, r.KR, r.ZR, 0) / WAVE;
        }
        if (h->reg_inst >= 0 && (h->wg_inst < 0 || reg_cost_s <= best)) h->default_kernel = 2;
        else if (h->wg_inst >= 0) h->default_kernel = 3;
        else h->default_kernel = 1;
        if (h->default_kernel == 3) {
            const int rc3 = pack_alloc(h);
            if (rc3) {
                phgpu_destroy(h);
                return rc3;
            }
        }
    }
    *out = h;
    return 0;
}

static inline dim3 grid_for(int64_t S) { return dim3((unsigned)((S + BLOCK - 1) / BLOCK)); }

// phgpu_set_scenarios on a shared-matrix handle: A_val holds nnz values (one copy for
// all scenarios).  Scales A once, finds the columns / rows whose data differ between
// scenarios (plus every nonant column), sizes the stream records and fills them.  Sizing
// the records needs those counts on the host: this call synchronises the stream once.
static int set_scenarios_shared(phgpu_state* h, const double* A_val, const double* c, const double* lb,
                                const double* ub, const double* rl, const double* ru, const double* q,
                                const double* obj_const, const double* prob, const int32_t* node_of,
                                const double* prob_coeff, hipStream_t st) {
    const size_t Sz = (size_t)h->S;
    const int n = h->n, m = h->m, nnz = h->nnz;
    auto cp = [&](double* dst, const double* src, size_t cnt) -> hipError_t {
        if (cnt == 0) return hipSuccess;
        return hipMemcpyAsync(dst, src, cnt * sizeof(double), hipMemcpyDeviceToDevice, st);
    };
    HIPCHK(cp(h->A, A_val, (size_t)nnz));
    if (obj_const) HIPCHK(cp(h->objc, obj_const, Sz));
    else HIPCHK(hipMemsetAsync(h->objc, 0, Sz * sizeof(double), st));
    HIPCHK(cp(h->prob, prob, Sz));
    HIPCHK(cp(h->pcoef, prob_coeff, (size_t)h->depth * Sz));
    HIPCHK(hipMemcpyAsync(h->node_of, node_of, (size_t)h->depth * Sz * sizeof(int32_t), hipMemcpyDeviceToDevice, st));
    h->xbar_mixed = -1;
    if (h->nb_idx) (void)hipFree(h->nb_idx);
    h->nb_idx = nullptr;
    const int big = std::max(nnz, std::max(n, m));
    const dim3 gb((unsigned)((big + 255) / 256)), gn((unsigned)((n + 255) / 256)), gm((unsigned)((m + 255) / 256));
    const dim3 gz((unsigned)((nnz + 255) / 256 > 0 ? (nnz + 255) / 256 : 1));
    // Ruiz (10 max passes) + Pock-Chambolle (sum) pass, as k_setup
    hipLaunchKernelGGL(k_sh_init, gb, dim3(256), 0, st, *h);
    for (int pass = 0; pass <= 10; ++pass) {
        const int pc = pass == 10;
        if (m) hipLaunchKernelGGL(k_sh_rowfac, gm, dim3(256), 0, st, *h, pc, h->sh_w);
        hipLaunchKernelGGL(k_sh_colfac, gn, dim3(256), 0, st, *h, pc, h->sh_u);
        hipLaunchKernelGGL(k_sh_apply, gb, dim3(256), 0, st, *h, (const double*)h->sh_w, (const double*)h->sh_u);
    }
    hipLaunchKernelGGL(k_sh_csc, gz, dim3(256), 0, st, *h);
    {
        const int tot_c = h->nent_c, tot_r = h->nent_r;
        if (tot_c) hipLaunchKernelGGL(k_sh_sell_vals, dim3((unsigned)((tot_c + 255) / 256)), dim3(256), 0, st,
                                      (const int32_t*)h->cs_src, (const double*)h->Ah_csc, tot_c, h->cs_val);
        if (tot_r) hipLaunchKernelGGL(k_sh_sell_vals, dim3((unsigned)((tot_r + 255) / 256)), dim3(256), 0, st,
                                      (const int32_t*)h->rs_src, (const double*)h->Ah_csr, tot_r, h->rs_val);
    }
    // ||A_scaled||_2: 200 power iterations on A^T A
    hipLaunchKernelGGL(k_sh_vinit, gn, dim3(256), 0, st, *h, h->sh_v);
    for (int it = 0; it < 200; ++it) {
        if (m) hipLaunchKernelGGL(k_sh_rowmv, gm, dim3(256), 0, st, *h, (const double*)h->sh_v, h->sh_w);
        hipLaunchKernelGGL(k_sh_colmv, gn, dim3(256), 0, st, *h, (const double*)h->sh_w, h->sh_u, h->sh_part);
        hipLaunchKernelGGL(k_sh_norm, dim3(1), dim3(256), 0, st, (const double*)h->sh_part, (int)gn.x, h->sh_norm + 3);
        hipLaunchKernelGGL(k_sh_normalize, gn, dim3(256), 0, st, *h, (const double*)h->sh_u,
                           (const double*)(h->sh_norm + 3), h->sh_v);
    }
    hipLaunchKernelGGL(k_sh_finish_norm, dim3(1), dim3(1), 0, st, *h);
    hipLaunchKernelGGL(k_sh_base, gb, dim3(256), 0, st, *h, c, q, lb, ub, rl, ru);
    HIPCHK(hipGetLastError());
    // which columns / rows differ between scenarios (one wave per entry)
    int32_t* flags = nullptr;
    HIPCHK(hipMalloc((void**)&flags, (size_t)(n + m + 1) * sizeof(int32_t)));
    hipLaunchKernelGGL(k_sh_vary, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, c, q, lb, ub, n, h->S, flags);
    if (m) hipLaunchKernelGGL(k_sh_vary, dim3((unsigned)((m + 3) / 4)), dim3(256), 0, st, rl, ru, (const double*)nullptr,
                              (const double*)nullptr, m, h->S, flags + n);
    HIPCHK(hipGetLastError());
    std::vector<int32_t> fl((size_t)n + m + 1, 0), slot((size_t)n, -1);
    HIPCHK(hipMemcpyAsync(fl.data(), flags, (size_t)(n + m) * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(slot.data(), h->nonant_slot, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    HIPCHK(hipFree(flags));
    std::vector<int32_t> cmap((size_t)n, -1), rmap((size_t)m + 1, -1), pcol, prow;
    for (int j = 0; j < n; ++j)
        if (fl[j] || slot[j] >= 0) {
            cmap[j] = (int32_t)pcol.size();
            pcol.push_back(j);
        }
    for (int i = 0; i < m; ++i)
        if (fl[(size_t)n + i]) {
            rmap[i] = (int32_t)prow.size();
            prow.push_back(i);
        }
    h->np = (int)pcol.size();
    h->nr = (int)prow.size();
    if (h->pcol) HIPCHK(hipFree(h->pcol));
    if (h->prow) HIPCHK(hipFree(h->prow));
    h->pcol = h->prow = nullptr;
    if (dalloc(h, &h->pcol, pcol.size()) || dalloc(h, &h->prow, prow.size())) return -3;
    HIPCHK(hipMemcpy(h->cmap, cmap.data(), (size_t)n * sizeof(int32_t), hipMemcpyHostToDevice));
    if (m) HIPCHK(hipMemcpy(h->rmap, rmap.data(), (size_t)m * sizeof(int32_t), hipMemcpyHostToDevice));
    if (!pcol.empty()) HIPCHK(hipMemcpy(h->pcol, pcol.data(), pcol.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    if (!prow.empty()) HIPCHK(hipMemcpy(h->prow, prow.data(), prow.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    // record layout, every part aligned to 16 doubles (128 B)
    auto al = [](int64_t v) { return (v + 15) / 16 * 16; };
    int64_t o = 0;
    h->sk_X = o; o += al(n);
    h->sk_X0 = o; o += al(n);
    h->sk_U = o; o += al(n);
    h->sk_XT = o; o += al(n);
    h->sk_Y = o; o += al(m);
    h->sk_Y0 = o; o += al(m);
    h->sk_YT = o; o += al(m);
    h->sk_PC = o; o += al(8 * (int64_t)h->np);
    h->sk_PR = o; o += al(4 * (int64_t)h->nr);
    h->sk_stride = o;
    const int64_t need = o * h->S;
    if (need > h->sk_cap) {
        if (h->sk) {
            HIPCHK(hipFree(h->sk));
            h->ws_bytes -= h->sk_cap * (int64_t)sizeof(double);
            h->sk = nullptr;
        }
        const int rc = dalloc(h, &h->sk, (size_t)need);
        if (rc) return rc;
        h->sk_cap = need;
    }
    const int64_t per = (int64_t)h->np + h->nr;
    if (per > 0) {
        const int64_t tot = per * h->S;
        hipLaunchKernelGGL(k_sh_fill, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, *h, c, q, lb, ub, rl, ru);
    }
    hipLaunchKernelGGL(k_sh_normbase, dim3(1), dim3(256), 0, st, *h, c, rl, ru);
    hipLaunchKernelGGL(k_sh_fill_omega, dim3((unsigned)((h->S + 255) / 256)), dim3(256), 0, st, *h);
    HIPCHK(hipGetLastError());
    h->wslot = h->wq = 0;
    h->pending = -1;
    h->have_s[0] = h->have_s[1] = 0;
    h->warm_rec_s[0] = h->warm_rec_s[1] = 0;
    bind_slots(h);
    h->scen_set = 1;
    h->last_path = 0;
    return 0;
}

extern "C" int phgpu_set_scenarios(phgpu_handle h, const double* A_val, const double* c,
                                   const double* lb, const double* ub, const double* rl,
                                   const double* ru, const double* q, const double* obj_const,
                                   const double* prob, const int32_t* node_of,
                                   const double* prob_coeff, void* stream) {
    FLUSH_STEP(h);
    if (!h) return set_err(-1, "null handle");
    if ((h->nnz && !A_val) || !c || !lb || !ub || (h->m && (!rl || !ru)) || !prob || !node_of || !prob_coeff)
        return set_err(-1, "null scenario array");
    hipStream_t st = (hipStream_t)stream;
    if (h->shared) return set_scenarios_shared(h, A_val, c, lb, ub, rl, ru, q, obj_const, prob, node_of, prob_coeff, st);
    const size_t Sz = (size_t)h->S;
    auto cp = [&](double* dst, const double* src, size_t cnt) -> hipError_t {
        if (cnt == 0) return hipSuccess;
        return hipMemcpyAsync(dst, src, cnt * sizeof(double), hipMemcpyDeviceToDevice, st);
    };
    HIPCHK(cp(h->A, A_val, (size_t)h->nnz * Sz));
    HIPCHK(cp(h->c, c, (size_t)h->n * Sz));
    HIPCHK(cp(h->lb, lb, (size_t)h->n * Sz));
    HIPCHK(cp(h->ub, ub, (size_t)h->n * Sz));
    HIPCHK(cp(h->rl, rl, (size_t)h->m * Sz));
    HIPCHK(cp(h->ru, ru, (size_t)h->m * Sz));
    if (q) HIPCHK(cp(h->q, q, (size_t)h->n * Sz));
    else HIPCHK(hipMemsetAsync(h->q, 0, (size_t)h->n * Sz * sizeof(double), st));
    if (obj_const) HIPCHK(cp(h->objc, obj_const, Sz));
    else HIPCHK(hipMemsetAsync(h->objc, 0, Sz * sizeof(double), st));
    HIPCHK(cp(h->prob, prob, Sz));
    HIPCHK(cp(h->pcoef, prob_coeff, (size_t)h->depth * Sz));
    HIPCHK(hipMemcpyAsync(h->node_of, node_of, (size_t)h->depth * Sz * sizeof(int32_t), hipMemcpyDeviceToDevice, st));
    h->xbar_mixed = -1;
    if (h->nb_idx) (void)hipFree(h->nb_idx);
    h->nb_idx = nullptr;
    h->wslot = h->wq = 0;
    h->pending = -1;
    h->have_s[0] = h->have_s[1] = 0;
    h->warm_rec_s[0] = h->warm_rec_s[1] = 0;
    h->jit_kinds_valid = 0;
    // new data: the path-6 module is specialised again at the next solve (and a spill or a
    // failed compile of the previous data no longer decides the path)
    h->ipm_flags_valid = 0;
    h->ipm_off = 0;
    h->ipm_spill1 = 0;
    h->ipm_lds = 0;
    bind_slots(h);
    HIPCHK(run_setup(h, st));
    // the setup's start omega (slot 0) for slot 1 too
    HIPCHK(hipMemcpyAsync(h->oms[1], h->oms[0], (size_t)h->S * sizeof(double), hipMemcpyDeviceToDevice, st));
    if (h->pk) HIPCHK(pack_fill(h, st));
    h->scen_set = 1;
    h->last_path = 0;
    return 0;
}

extern "C" int phgpu_set_nonant_probs(phgpu_handle h, const double* pvar) {
    FLUSH_STEP(h);
    if (!h) return set_err(-1, "null handle");
    const double* nv = h->nn > 0 ? pvar : nullptr;
    // the path-6 epilogue partials of both slots were weighted with the per-node prob_coeff
    // (or the previous pvar, whose values the caller may have rewritten in place): a later
    // phgpu_ph_reduce must not take them for this x
    h->xp_C[0] = h->xp_C[1] = 0;
    h->pvar = nv;
    return 0;
}

extern "C" int phgpu_set_ph_state(phgpu_handle h, const double* W, const double* rho,
                                  const double* xbar, int W_on, int prox_on) {
    FLUSH_STEP(h);
    if (!h) return set_err(-1, "null handle");
    if (h->nn > 0 && ((W_on && !W) || (prox_on && (!rho || !xbar))))
        return set_err(-1, "W / rho / xbar pointer missing for the requested terms");
    h->W = W;
    h->rho = rho;
    h->xbar = xbar;
    h->W_on = W_on ? 1 : 0;
    h->prox_on = prox_on ? 1 : 0;
    return 0;
}

static int solve_impl(phgpu_handle h, const phgpu_options* opt, int warm_start, int defer, double* x, double* y,
                      double* obj, double* bound, int32_t* status, int32_t* iters, void* stream);

extern "C" int phgpu_solve(phgpu_handle h, const phgpu_options* opt, int warm_start, double* x,
                           double* y, double* obj, double* bound, int32_t* status,
                           int32_t* iters, void* stream) {
    return solve_impl(h, opt, warm_start, 0, x, y, obj, bound, status, iters, stream);
}

extern "C" int phgpu_solve_deferred(phgpu_handle h, const phgpu_options* opt, int warm_start, double* x,
                                    double* y, double* obj, double* bound, int32_t* status,
                                    int32_t* iters, void* stream) {
    return solve_impl(h, opt, warm_start, 1, x, y, obj, bound, status, iters, stream);
}

extern "C" int phgpu_commit(phgpu_handle h) {
    if (!h) return set_err(-1, "null handle");
    if (h->pending >= 0) {
        h->wslot = h->wq = h->pending;
        h->pending = -1;
        bind_slots(h);
    }
    return 0;
}

// the path phgpu_solve takes for kernel 0 (gamma = 1): the interior-point kernel (path 6)
// where it applies (PHGPU_IPM=0 turns it off, a module that spills takes it out), then
// the pattern-specialised PDHG kernel (path 5) when PHGPU_JIT asks for it, else the path
// chosen at phgpu_create
static int default_path(const phgpu_state* h) {
    const char* ie = getenv("PHGPU_IPM");
    if (ipm_eligible(h) && !h->ipm_off && !(ie && atoi(ie) == 0)) return 6;
    const char* env = getenv("PHGPU_JIT");
    if (env && atoi(env) == 0) return h->default_kernel;
    if (jit_eligible(h) && (env || h->S >= JIT_MIN_S)) return 5;
    return h->default_kernel;
}

static int solve_impl(phgpu_handle h, const phgpu_options* opt, int warm_start, int defer, double* x, double* y,
                      double* obj, double* bound, int32_t* status, int32_t* iters, void* stream) {
    if (!h) return set_err(-1, "null handle");
    if (!x || !obj || !bound || !status) return set_err(-1, "null output pointer");
    if (defer && h->shared)
        return set_err(-1, "phgpu_solve_deferred: a shared-matrix handle (path 4) keeps one warm-start slot");
    // read the committed slot; write it in place, or the other slot for a deferred solve
    // (an uncommitted deferred solve is dropped by this one)
    h->pending = -1;
    h->wq = defer ? 1 - h->wslot : h->wslot;
    bind_slots(h);
    const int wq = h->wq;
    phgpu_options o;
    if (opt) o = *opt;
    else phgpu_default_options(&o);
    if (o.check_every < 1 || o.max_iter < 1 || !(o.eta_frac > 0.0 && o.eta_frac < 1.0) ||
        o.gamma < 0.0 || o.gamma > 1.0 || o.restart_every < 1 || o.check_every % o.restart_every != 0 ||
        o.max_iter % o.restart_every != 0 || !(o.eps_infeas > 0.0))
        return set_err(-1, "bad options (check_every=%d restart_every=%d max_iter=%d eta_frac=%g gamma=%g "
                       "eps_infeas=%g; check_every and max_iter must be multiples of restart_every)",
                       o.check_every, o.restart_every, o.max_iter, o.eta_frac, o.gamma, o.eps_infeas);
    solve_params P;
    P.eps_rel = o.eps_rel;
    P.eps_abs = o.eps_abs;
    P.gamma = o.gamma;
    P.bsuff = o.beta_sufficient;
    P.bnec = o.beta_necessary;
    P.bart = o.beta_artificial > 0.0 ? o.beta_artificial : 1e300;
    P.restart_every = o.restart_every;
    P.eta_frac = o.eta_frac;
    P.omega0 = o.omega0;
    P.max_iter = o.max_iter;
    P.check_every = o.check_every;
    P.warm = (warm_start && h->have_solution) ? 1 : 0;
    P.keep_omega = o.keep_omega;
    P.infeas_start = o.infeas_start;
    P.eps_inf = o.eps_infeas;
    P.wmax = o.omega_clamp > 1.0 ? o.omega_clamp : 1e300;
    P.wmin = 1.0 / P.wmax;
    hipStream_t st = (hipStream_t)stream;
    // the register-resident kernels are specialised for the reflected step (gamma = 1, the
    // default); another gamma runs on the global-memory kernel
    if (o.kernel < 0 || o.kernel > 6) return set_err(-1, "bad kernel option %d", o.kernel);
    if (h->shared != (o.kernel == 4 || (o.kernel == 0 && h->shared)))
        return set_err(-1, "kernel option %d: a shared-matrix handle solves with path 4 only (kernel 0 or 4), "
                       "other handles with paths 1-3, 5 and 6", o.kernel);
    if (h->shared) {
        if (!h->scen_set) return set_err(-1, "phgpu_set_scenarios has not been called");
        int per_cu = 0;
        // B scenario slots per workgroup (PHGPU_STREAM_SLOTS=1|2, default 2)
        const char* env = getenv("PHGPU_STREAM_SLOTS");
        const int B = (env && atoi(env) == 1) ? 1 : 2;
        const void* fn = B == 1 ? (const void*)k_solve_stream<1> : (const void*)k_solve_stream<2>;
        int& oc = h->occ_cache[B == 1 ? 4 : 5];
        if (!oc) HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&oc, fn, SBLK, 0));
        per_cu = oc;
        // PHGPU_STREAM_PER_CU=k: launch k workgroups per CU whatever the occupancy query says
        // (the ones that do not fit wait for a free CU; the queue has no other dependency)
        const char* pce = getenv("PHGPU_STREAM_PER_CU");
        if (pce && atoi(pce) > 0) per_cu = std::min(atoi(pce), 8);
        if (per_cu < 1) per_cu = 1;
        int64_t nblk = (int64_t)per_cu * h->num_cus;
        if (nblk > (h->S + B - 1) / B) nblk = (h->S + B - 1) / B;
        // PHGPU_STREAM_SPLIT=T: the T longest scenarios of the previous solve run first, each
        // over the whole GPU (the split form of k_solve_stream, cooperative launch), then the
        // rest on the queue
        const char* spe = getenv("PHGPU_STREAM_SPLIT");
        int T = o.split_longest > 0 ? o.split_longest : (spe ? atoi(spe) : 0);
        if (T < 0) T = 0;
        if (T > 16) T = 16;
        if (T > h->S) T = (int)h->S;
        HIPCHK(hipMemsetAsync(h->qhead, 0, sizeof(int), st));
        // queue order: longest first by the previous solve's iteration counts (the launch
        // ends with its slowest scenario; starting it first shortens the tail)
        if (!h->have_solution) HIPCHK(hipMemsetAsync(h->sk_iters, 0, (size_t)h->S * sizeof(int32_t), st));
        if (h->S <= STREAM_ORDER_MAX)
            hipLaunchKernelGGL(k_stream_order, dim3((unsigned)((h->S + 255) / 256)), dim3(256), 0, st, *h);
        else
            hipLaunchKernelGGL(k_stream_order_identity, dim3((unsigned)((h->S + 255) / 256)), dim3(256), 0, st, *h);
        int occ = 0;
        HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)k_solve_stream<1, true>, SBLK, 0));
        const int64_t cap = (int64_t)std::max(occ, 1) * h->num_cus;
        // enough waves for one slice each in the longer pass: no more workgroups per scenario
        const int kmax = std::max((std::max(h->nsl_c, h->nsl_r) + SWAVES - 1) / SWAVES, 1);
        // the cluster form for a batch smaller than the GPU (a rank's share of a strong-
        // scaling run): every scenario over K = capacity / S workgroups at once instead of
        // one scenario per workgroup on a few CUs (PHGPU_STREAM_CLUSTER=0: off, =K: that K)
        int Kc = 0;
        {
            const char* ce = getenv("PHGPU_STREAM_CLUSTER");
            const int ask = ce ? atoi(ce) : -1;
            if (ask != 0 && T == 0) {
                int64_t k = cap / std::max<int64_t>(h->S, 1);
                if (ask > 1) k = std::min<int64_t>(ask, k);
                k = std::min<int64_t>(k, kmax);
                if (k >= 2) Kc = (int)k;
            }
        }
        if (T > 0 || Kc >= 2) {
            // the split form: T stragglers over the whole grid (one cluster), or S clusters of Kc
            const int ncl = Kc >= 2 ? (int)h->S : 1;
            int G = Kc >= 2 ? (int)h->S * Kc : (int)std::min<int64_t>(kmax, cap);
            G = std::max(G, 1);
            const size_t need = (size_t)2 * G * 8 + (size_t)16 * ncl;  // partials, then 128-B barrier counters
            if (h->split_need < need) {
                if (h->split_part) HIPCHK(hipFree(h->split_part));
                h->split_part = nullptr;
                HIPCHK(hipMalloc((void**)&h->split_part, need * sizeof(double)));
                h->split_need = need;
            }
            // the barrier counters start at gbase (PHGPU_SPLIT_BAR_BASE: a test starts them just
            // below 2^32 so that they wrap during the launch; the barrier compares wrap-safe)
            const char* bbe = getenv("PHGPU_SPLIT_BAR_BASE");
            unsigned gbase = bbe ? (unsigned)strtoul(bbe, nullptr, 0) : 0u;
            HIPCHK(hipMemsetD32Async((hipDeviceptr_t)(h->split_part + (size_t)2 * G * 8), (int)gbase, (size_t)32 * ncl, st));
            phgpu_state hv = *h;
            int32_t* qh = h->qhead;
            double* gp = h->split_part;
            int q0 = Kc >= 2 ? (int)h->S : T;
            int nc = ncl;
            void* args[] = {&hv, &P, &qh, &x, &y, &obj, &bound, &status, &iters, &q0, &gp, &gbase, &nc};
            HIPCHK(hipLaunchCooperativeKernel((const void*)k_solve_stream<1, true>, dim3((unsigned)G), dim3(SBLK), args,
                                              0, st));
            h->last_cluster = Kc >= 2 ? Kc : 0;
        } else {
            h->last_cluster = 0;
        }
        if (Kc < 2) {
            nblk = std::min<int64_t>(nblk, std::max<int64_t>((h->S - T + B - 1) / B, 1));
            if (B == 1)
                hipLaunchKernelGGL(k_solve_stream<1>, dim3((unsigned)nblk), dim3(SBLK), 0, st, *h, P, h->qhead, x, y, obj,
                                   bound, status, iters, T, (double*)nullptr, 0u, 1);
            else
                hipLaunchKernelGGL(k_solve_stream<2>, dim3((unsigned)nblk), dim3(SBLK), 0, st, *h, P, h->qhead, x, y, obj,
                                   bound, status, iters, T, (double*)nullptr, 0u, 1);
        }
        HIPCHK(hipGetLastError());
        h->last_stats = nullptr;
        h->last_status = status;
        h->last_iters = iters;
        h->have_s[wq] = 1;
        h->last_path = 4;
        bind_slots(h);
        return 0;
    }
    if (o.kernel == 2 && h->reg_inst < 0)
        return set_err(-1, "register-resident kernel requested but no compiled instance fits this pattern");
    if (o.kernel == 3 && h->wg_inst < 0)
        return set_err(-1, "workgroup-per-scenario kernel requested but no compiled instance fits this pattern");
    if ((o.kernel == 2 || o.kernel == 3 || o.kernel == 5) && o.gamma != 1.0)
        return set_err(-1, "register-resident kernels require gamma = 1 (got %g)", o.gamma);
    if (o.kernel == 5 && !jit_eligible(h))
        return set_err(-1, "kernel 5 (pattern-specialised) needs n <= %d, m <= %d, nnz <= %d (got %d, %d, %d)",
                       JIT_MAX_N, JIT_MAX_M, JIT_MAX_NNZ, h->n, h->m, h->nnz);
    if (o.kernel == 6 && !ipm_eligible(h))
        return set_err(-1, "kernel 6 (interior point) needs n <= %d, m <= %d, nnz <= %d and <= %d factor entries "
                       "(got %d, %d, %d, %d)", IPM_MAX_N, IPM_MAX_M, IPM_MAX_NNZ, IPM_MAX_NF, h->n, h->m, h->nnz,
                       h->ipm_nf);
    int path = o.kernel != 0 ? o.kernel : (o.gamma == 1.0 ? default_path(h) : 1);
    // the statistics / status buffers phgpu_solve_stats and phgpu_ph_update_ex read: this
    // solve's, once it is launched (a rejected solve leaves the previous ones)
    unsigned long long* stats_keep = h->last_stats;
    h->last_stats = nullptr;  // path 6 sets it when its kernels produce the statistics
    if (path == 6) {
        const int rc6 = ipm_prepare(h, st);
        if (rc6) {
            h->last_stats = stats_keep;
            if (o.kernel != 0) return rc6;
            // the automatic choice: a module that does not compile or load (a hipRTC runtime
            // problem, an unusual pattern) turns path 6 off for this handle's data and the
            // solve runs on the handle's PDHG path; phgpu_last_error keeps the reason and
            // phgpu_ipm_info reports it (off = 2)
            h->ipm_off = 2;
            fprintf(stderr, "phgpu: path 6 unavailable (%s); solving on the PDHG path\n", g_err);
            path = default_path(h);
        } else if (o.kernel == 0 && h->ipm->private_bytes > ipm_spill_max()) {
            h->ipm_off = 1;  // the automatic choice falls back to the handle's PDHG path
            path = default_path(h);
        }
    }
    // a deferred one-rank PH step (phgpu_ph_step_defer): folded into this launch's prologue
    // when it is a path-6 deferred solve that writes other buffers than the step reads and
    // the previous solve's partials / statistics are path 6's; else run now
    h->fuse_now = 0;
    if (h->pend.active) {
        const phgpu_state::ph_pending& q = h->pend;
        const char* fe = getenv("PHGPU_FUSE_STEP");
        // (the one-lane kernel only: folded into the lane-group kernel the step measured
        // slower, 8,192 scenarios 0.095 ms per PH iteration against 0.079 as its own launch,
        // profiles/r04/o/; PHGPU_FUSE_STEP=1 folds there too)
        const bool fuse = path == 6 && defer && !(fe && atoi(fe) == 0) && q.stream == st && q.x != x &&
                          // (the workgroup kernels, L >= 64, carry no folded step at all)
                          (h->ipm && (h->ipm->L == 1 || (fe && atoi(fe) == 1 && h->ipm->L < 64))) &&
                          h->nb_idx && h->xbar_single && h->xbar_mixed == 0 && h->nn > 0 && h->nn <= XL_NN_MAX &&
                          xp_valid(h, q.x) && q.W == h->W && q.xbar == h->xbar && q.rho == h->rho &&
                          (!q.stats || (stats_keep && stats_keep == h->ipm_stats + PHGPU_STATS_WORDS * (1 - h->ipm_parity)));
        if (fuse) {
            h->fuse_now = 1;
            ++h->folded;
        }
        else {
            // (the step's statistics are the previous solve's: its in-kernel ones if any)
            h->last_stats = stats_keep;
            const int frc = flush_step(h);
            h->last_stats = nullptr;
            if (frc) return frc;
        }
    }
    const bool use_reg = path == 2;
    int out_rec = 0;  // the warm state this solve writes lives in the records
    if (path == 3 && !h->pk) {
        const int rc3 = pack_alloc(h);
        if (rc3) return rc3;
        if (h->scen_set) HIPCHK(pack_fill(h, st));
    }
    if (path == 3) {
        // this solve's PH state into the records; a warm start left by another path too
        HIPCHK(ph_to_records(h, st));
        if (P.warm && !h->warm_rec) {
            HIPCHK(to_records(h, h->x, h->n, h->pk_X, st));
            HIPCHK(to_records(h, h->y, h->m, h->pk_Y, st));
        }
    }
    if (path == 3) {
        const wg_instance& gi = g_wg_instances[h->wg_inst];
        wg_plan pl;
        pl.L = WAVE * gi.WPS;
        pl.kc = gi.KC;
        pl.zc = gi.ZC;
        pl.kr = gi.KR;
        pl.zr = gi.ZR;
        pl.col_id = h->wg_col_id;
        pl.row_id = h->wg_row_id;
        pl.col_long = h->wg_col_long;
        pl.row_long = h->wg_row_long;
        pl.col_k = h->wg_col_k;
        pl.col_r = h->wg_col_r;
        pl.row_k = h->wg_row_k;
        pl.row_c = h->wg_row_c;
        const size_t lds = wg_lds_doubles(h->n, h->m, gi.KC, gi.KR, gi.WPS) * sizeof(double);
        int per_cu = 0;
        int& oc = h->occ_cache[3];
        if (!oc) HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&oc, (const void*)gi.fn, pl.L, lds));
        per_cu = oc;
        if (per_cu < 1) per_cu = 1;
        int64_t nblk = (int64_t)per_cu * h->num_cus;
        if (nblk > h->S) nblk = h->S;
        HIPCHK(hipMemsetAsync(h->qhead, 0, sizeof(int), st));
        hipLaunchKernelGGL(gi.fn, dim3((unsigned)nblk), dim3(pl.L), lds, st, *h, P, pl, h->qhead, x, y, obj, bound,
                           status, iters);
        HIPCHK(hipGetLastError());
        // outputs in the caller's scenario-fastest layout, unscaled
        HIPCHK(from_records(h, h->pk_XW, h->pk_DC, h->n, x, st));
        if (y) HIPCHK(from_records(h, h->pk_YW, h->pk_DR, h->m, y, st));
        out_rec = 1;
    } else if (use_reg) {
        const int G = WAVE / h->reg_L;
        const reg_instance& ri = g_reg_instances[h->reg_inst];
        const size_t lds = (size_t)REG_WPB * reg_wave_lds(h->n, h->m, G, ri.KC, ri.KR) * sizeof(double);
        // persistent grid: co-resident workgroups of REG_WPB independent waves (occupancy
        // x CUs), never more than there are scenario groups
        const int64_t need = (h->S + (int64_t)G * REG_WPB - 1) / ((int64_t)G * REG_WPB);
        auto grid_of = [&](reg_kernel_t f, int& oc, int64_t& nb) -> hipError_t {
            if (!oc) {
                const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&oc, (const void*)f,
                                                                                  WAVE * REG_WPB, lds);
                if (e != hipSuccess) return e;
            }
            nb = (int64_t)(oc < 1 ? 1 : oc) * h->num_cus;
            if (nb > need) nb = need;
            return hipSuccess;
        };
        int64_t nblk = 0;
        HIPCHK(grid_of(ri.fn, h->occ_cache[2], nblk));
        // record mode (solve_reg.inc, template REC) when groups take more than one scenario
        // each: then the queue order matters (PHGPU_REG_REC=0|1 pins it)
        const char* env = getenv("PHGPU_REG_REC");
        const bool rec = env ? atoi(env) != 0 : nblk * REG_WPB * G < h->S;
        const reg_kernel_t fn = rec ? ri.fn_rec : ri.fn;
        if (rec) HIPCHK(grid_of(ri.fn_rec, h->occ_cache[6], nblk));
        const int64_t first_dyn = nblk * REG_WPB * G;
        if (rec) {
            if (!h->pk) {
                const int rc3 = pack_alloc(h);
                if (rc3) return rc3;
                if (h->scen_set) HIPCHK(pack_fill(h, st));
            }
            if (P.warm && !h->warm_rec) {
                HIPCHK(to_records(h, h->x, h->n, h->pk_X, st));
                HIPCHK(to_records(h, h->y, h->m, h->pk_Y, st));
            }
            if (!h->have_solution) HIPCHK(hipMemsetAsync(h->sk_iters, 0, (size_t)h->S * sizeof(int32_t), st));
            const dim3 ob((unsigned)((h->S + ORDER_BINS - 1) / ORDER_BINS));
            int32_t* bins = h->sk_bins + 2 * ORDER_BINS * h->order_parity;
            int32_t* other = h->sk_bins + 2 * ORDER_BINS * (1 - h->order_parity);
            h->order_parity ^= 1;
            // histogram + this solve's PH state into the records, one launch (k_reg_prep)
            const bool ph = h->nn > 0 && (h->W_on || h->prox_on);
            const int nh = (int)ob.x;
            const int gx = (int)((h->S + TT - 1) / TT), gy = ph ? (3 * h->nn + TT - 1) / TT : 0;
            hipLaunchKernelGGL(k_reg_prep, dim3((unsigned)(nh + gx * gy)), dim3(256), 0, st, h->sk_iters, h->S,
                               P.restart_every, bins, nh, gx, h->W_on ? h->W : nullptr,
                               h->prox_on ? h->rho : nullptr, h->prox_on ? h->xbar : nullptr, h->nn, h->pk,
                               h->pk_stride, h->pk_W);
            hipLaunchKernelGGL(k_reg_order, ob, dim3(ORDER_BINS), 0, st, h->sk_iters, h->S, P.restart_every, bins,
                               other, h->sk_order, h->qhead);
        } else if (P.warm && h->warm_rec) {
            HIPCHK(from_records(h, h->pk_X, -1, h->n, h->x, st));
            HIPCHK(from_records(h, h->pk_Y, -1, h->m, h->y, st));
        }
        reg_plan pl;
        pl.L = h->reg_L;
        pl.kc = h->reg_kc;
        pl.zc = h->reg_zc;
        pl.kr = h->reg_kr;
        pl.zr = h->reg_zr;
        pl.col_k = h->pl_col_k;
        pl.col_r = h->pl_col_r;
        pl.row_k = h->pl_row_k;
        pl.row_c = h->pl_row_c;
        pl.order = h->sk_order;
        pl.last_iters = h->sk_iters;
        pl.last_iters_w = h->its_w;
        pl.ema = h->have_solution ? 1 : 0;
        if (!rec) HIPCHK(hipMemsetAsync(h->qhead, 0, sizeof(int), st));  // record mode: k_reg_order did
        hipLaunchKernelGGL(fn, dim3((unsigned)nblk), dim3(WAVE * REG_WPB), lds, st, *h, P, pl, h->qhead, first_dyn,
                           x, y, obj, bound, status, iters);
        HIPCHK(hipGetLastError());
        if (rec) {
            // outputs in the caller's scenario-fastest layout, unscaled
            HIPCHK(from_records(h, h->pk_XW, h->pk_DC, h->n, x, st));
            if (y) HIPCHK(from_records(h, h->pk_YW, h->pk_DR, h->m, y, st));
        }
        out_rec = rec ? 1 : 0;
        h->last_rec = rec ? 1 : 0;
    } else {
        if (P.warm && h->warm_rec) {
            HIPCHK(from_records(h, h->pk_X, -1, h->n, h->x, st));
            HIPCHK(from_records(h, h->pk_Y, -1, h->m, h->y, st));
        }
        if (path == 5) {
            const int rc5 = jit_prepare(h, st);
            if (rc5) return rc5;
            const int rc6 = jit_launch(h, P, x, y, obj, bound, status, iters, st);
            if (rc6) return rc6;
        } else if (path == 6) {
            const int rc6 = ipm_launch(h, P, x, y, obj, bound, status, iters, st);
            if (rc6) return rc6;
        } else {
            hipLaunchKernelGGL(k_solve, grid_for(h->S), dim3(BLOCK), 0, st, *h, P, x, y, obj, bound, status, iters);
        }
        out_rec = 0;
    }
    HIPCHK(hipGetLastError());
    h->last_status = status;
    h->last_iters = iters;
    if (path != 6) h->xp_C[wq] = 0;  // only path 6 writes x̄ partials with its outputs
    // the warm state written by this solve; current now, or at phgpu_commit if deferred
    h->have_s[wq] = 1;
    h->warm_rec_s[wq] = out_rec;
    h->last_path = path;
    if (defer) h->pending = wq;
    else h->wslot = wq;
    h->wq = h->wslot;
    bind_slots(h);
    return 0;
}

// Once per scenario data: does any wave span two nodes (xbar_mixed), is every nonant on one
// node (xbar_single), and the node_buf index of each nonant for the folded PH step (nb_idx)
static int xbar_layout(phgpu_state* h, hipStream_t st) {
    if (h->xbar_mixed >= 0) return 0;
    int32_t* d = nullptr;
    int32_t v[2] = {0, 0};
    HIPCHK(hipMalloc((void**)&d, 2 * sizeof(int32_t)));
    HIPCHK(hipMemsetAsync(d, 0, 2 * sizeof(int32_t), st));
    hipLaunchKernelGGL(k_xbar_mixed, grid_for(h->S), dim3(BLOCK), 0, st, *h, d);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(v, d, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    HIPCHK(hipFree(d));
    h->xbar_mixed = v[0] ? 1 : 0;
    h->xbar_single = v[1] ? 0 : 1;
    if (h->xbar_single && h->nn > 0 && h->nn <= XL_NN_MAX && !h->nb_idx) {
        // node_buf index of each nonant (its one node, offset) for the folded PH step
        std::vector<int32_t> dep(h->nn), off(h->nn), idx(h->nn);
        HIPCHK(hipMemcpy(dep.data(), h->nonant_depth, h->nn * sizeof(int32_t), hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(off.data(), h->nonant_off, h->nn * sizeof(int32_t), hipMemcpyDeviceToHost));
        for (int k = 0; k < h->nn; ++k) {
            int32_t g = 0;
            HIPCHK(hipMemcpy(&g, h->node_of + (size_t)dep[k] * h->S, sizeof(int32_t), hipMemcpyDeviceToHost));
            idx[k] = g * h->nlen_max + off[k];
        }
        int32_t* di = nullptr;
        HIPCHK(hipMalloc((void**)&di, h->nn * sizeof(int32_t)));
        HIPCHK(hipMemcpy(di, idx.data(), h->nn * sizeof(int32_t), hipMemcpyHostToDevice));
        h->nb_idx = di;
    }
    return 0;
}

// The PH loop of one rank in one cooperative launch (include/phgpu.h, solve_ipm.inc's
// IPM_LOOP module)
extern "C" int phgpu_ph_loop(phgpu_handle h, const phgpu_options* opt, int max_iters, double convthresh,
                             double* x, double* y, double* obj, double* bound, int32_t* status, int32_t* iters,
                             double* node_buf, double* conv_hist, int64_t* out, void* stream) {
    if (!h || !x || !obj || !bound || !status || !node_buf || !conv_hist || !out) return set_err(-1, "null argument");
    if (max_iters < 1) return set_err(-1, "phgpu_ph_loop: max_iters must be >= 1");
    FLUSH_STEP(h);
    hipStream_t st = (hipStream_t)stream;
    {
        const int rc = xbar_layout(h, st);  // (known after the first phgpu_ph_reduce otherwise)
        if (rc) return rc;
    }
    const int why = ph_loop_eligible(h);
    if (why) return set_err(-3, "phgpu_ph_loop: not eligible (reason %d); run the PH steps one by one", why);
    phgpu_options o;
    if (opt) o = *opt;
    else phgpu_default_options(&o);
    if (o.kernel != 0 && o.kernel != 6) return set_err(-3, "phgpu_ph_loop: path 6 only");
    {
        const int rc = ipm_prepare(h, st);
        if (rc) return rc;
    }
    if (h->ipm->L != 1 || h->ipm->private_bytes > ipm_spill_max()) return set_err(-3, "phgpu_ph_loop: no one-lane module");
    {
        const int rc = ipm_loop_prepare(h);
        if (rc) return rc;
    }
    ipm_module* im = h->ipm_loop;
    const int64_t nblk = (h->S + 255) / 256;
    if ((int64_t)std::max(im->per_cu_ipm, 0) * h->num_cus < nblk)
        return set_err(-3, "phgpu_ph_loop: %lld workgroups do not fit the GPU at once", (long long)nblk);
    // buffers
    const int64_t nd = nblk * 16 + 16 + max_iters;
    if (h->loop_dbl_n < nd) {
        if (h->loop_dbl) HIPCHK(hipFree(h->loop_dbl));
        h->loop_dbl = nullptr;
        HIPCHK(hipMalloc((void**)&h->loop_dbl, (size_t)nd * sizeof(double)));
        h->loop_dbl_n = nd;
    }
    if (!h->loop_cnt) HIPCHK(hipMalloc((void**)&h->loop_cnt, (size_t)(2 + PHGPU_STATS_WORDS) * sizeof(unsigned long long)));
    HIPCHK(hipMemsetAsync(h->loop_cnt, 0, (size_t)(2 + PHGPU_STATS_WORDS) * sizeof(unsigned long long), st));
    // a plain (non-deferred) solve's slot bookkeeping (solve_impl)
    h->pending = -1;
    h->wq = h->wslot;
    bind_slots(h);
    const int wq = h->wq;
    solve_params P;
    P.eps_rel = o.eps_rel;
    P.eps_abs = o.eps_abs;
    P.gamma = o.gamma;
    P.bsuff = o.beta_sufficient;
    P.bnec = o.beta_necessary;
    P.bart = o.beta_artificial > 0.0 ? o.beta_artificial : 1e300;
    P.restart_every = o.restart_every;
    P.eta_frac = o.eta_frac;
    P.omega0 = o.omega0;
    P.max_iter = o.max_iter;
    P.check_every = o.check_every;
    P.warm = h->have_solution ? 1 : 0;
    P.keep_omega = o.keep_omega;
    P.infeas_start = o.infeas_start;
    P.eps_inf = o.eps_infeas;
    P.wmax = o.omega_clamp > 1.0 ? o.omega_clamp : 1e300;
    P.wmin = 1.0 / P.wmax;
    const int par = h->ipm_parity;
    h->ipm_parity ^= 1;
    int32_t* fail_n = h->ipm_cnt + 3 * par;
    int32_t* qhead = h->ipm_cnt + 3 * par + 1;
    ipm_params_host a;
    a.A = h->A; a.c = h->c; a.q = h->q; a.lb = h->lb; a.ub = h->ub; a.rl = h->rl; a.ru = h->ru; a.objc = h->objc;
    a.lbh = h->lbh; a.ubh = h->ubh; a.Dc = h->Dc; a.Dr = h->Dr;
    a.W = h->W; a.rho = h->rho; a.xbar = h->xbar;
    a.omega_in = h->omega;
    a.omega_out = h->omega_w; a.x_w = h->xw; a.y_w = h->yw;
    a.xout = x; a.yout = y; a.obj = obj; a.bound = bound;
    a.status = status; a.iters = iters;
    a.fail_list = h->ipm_list; a.fail_n = fail_n;
    a.zero3 = h->ipm_cnt + 3 * (1 - par);
    a.stats = h->ipm_stats + PHGPU_STATS_WORDS * par; a.stats_zero = h->ipm_stats + PHGPU_STATS_WORDS * (1 - par);
    a.prof = nullptr;
    a.S = h->S;
    a.W_on = h->W_on; a.prox_on = h->prox_on;
    a.eps_rel = P.eps_rel; a.eps_abs = P.eps_abs;
    const char* et = getenv("PHGPU_IPM_EPS");
    a.eps_tight = (et && atof(et) > 0.0) ? atof(et) : IPM_EPS_TIGHT;
    a.x_in = P.warm ? h->x : nullptr;
    a.y_in = P.warm ? h->y : nullptr;
    const char* env = getenv("PHGPU_IPM_MAXIT");
    a.max_ipm = (env && atoi(env) >= 0) ? atoi(env) : IPM_MAXIT;
    a.xp = nullptr;  // (no epilogue partials: the loop ends on its own PH state)
    a.xp_node = h->xp_node[wq];
    a.xp_dirty = h->xp_dirty[wq];
    a.pcoef = h->pcoef;
    a.node_of = h->node_of;
    a.xprev = x;
    a.W_w = const_cast<double*>(h->W);
    a.xbar_w = const_cast<double*>(h->xbar);
    a.node_buf = node_buf;
    a.nb_idx = h->nb_idx;
    a.nb_half = (long long)h->num_nodes * h->nlen_max;
    a.gpart = h->loop_dbl;
    a.gpub = h->loop_dbl + nblk * 16;
    a.conv_hist = h->loop_dbl + nblk * 16 + 16;
    a.gsync = (unsigned*)h->loop_cnt;
    a.loop_out = (int*)(h->loop_cnt + 1);
    a.loop_its = h->loop_cnt + 2;
    a.conv_scale = 1.0 / ((double)h->S * (double)h->nn);
    a.convthresh = convthresh;
    a.loop_K = max_iters;
    h->xp_C[wq] = 0;
    h->last_stats = a.stats;
    void* args[] = {&a};
    HIPCHK(hipModuleLaunchCooperativeKernel(im->fn_ipm, (unsigned)nblk, 1, 1, 256, 1, 1, 0, st, args));
    {
        const int rc = ipm_fallback_launch(h, im, P, x, y, obj, bound, status, iters, qhead, fail_n, a.stats, st);
        if (rc) return rc;
    }
    HIPCHK(hipGetLastError());
    h->last_status = status;
    h->last_iters = iters;
    h->have_s[wq] = 1;
    h->warm_rec_s[wq] = 0;
    h->last_path = 6;
    h->wslot = wq;
    h->wq = h->wslot;
    bind_slots(h);
    // the loop's record (one synchronisation: the loop is one call of the host's PH loop)
    std::vector<unsigned long long> cnt((size_t)(2 + PHGPU_STATS_WORDS));
    HIPCHK(hipMemcpyAsync(cnt.data(), h->loop_cnt, cnt.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(conv_hist, a.conv_hist, (size_t)max_iters * sizeof(double), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    const int* lo = (const int*)(cnt.data() + 1);
    out[0] = lo[0];
    out[1] = lo[1];
    out[2] = (int64_t)stats_word(cnt.data() + 2, PHGPU_STATS_COPIES, 0);
    out[3] = 0;
    if (lo[1] == 3) return set_err(-2, "phgpu_ph_loop: a grid step timed out (the launch was not co-resident)");
    return 0;
}

// counts[c] = number of local scenarios with status c (c = 0..3), one block
// counts[k] = #{s : status[s] == k}: one block, four statuses per load, several loads in
// flight per thread (a device-wide "last block" reduction needs a release fence, i.e. an
// L2 writeback of every XCD, which costs more than the whole count)
#define SC_T 1024
__global__ void __launch_bounds__(SC_T) k_status_counts(const int32_t* __restrict__ status, int64_t S,
                                                        int32_t* __restrict__ counts) {
    __shared__ int32_t c[4];
    if (threadIdx.x < 4) c[threadIdx.x] = 0;
    __syncthreads();
    int32_t loc[4] = {0, 0, 0, 0};
    // (a macro, not a lambda: a by-reference capture of loc[] would put it in scratch)
#define SC_ADD(v) loc[0] += (v) == 0, loc[1] += (v) == 1, loc[2] += (v) == 2, loc[3] += (v) == 3
    const int64_t S4 = ((uintptr_t)status % 16 == 0) ? S / 4 : 0;  // int4 part
    const int4* s4 = (const int4*)status;
    int64_t i = threadIdx.x;
    for (; i + 3 * SC_T < S4; i += 4 * SC_T) {
        const int4 a = s4[i], b = s4[i + SC_T], d = s4[i + 2 * SC_T], e = s4[i + 3 * SC_T];
        SC_ADD(a.x); SC_ADD(a.y); SC_ADD(a.z); SC_ADD(a.w);
        SC_ADD(b.x); SC_ADD(b.y); SC_ADD(b.z); SC_ADD(b.w);
        SC_ADD(d.x); SC_ADD(d.y); SC_ADD(d.z); SC_ADD(d.w);
        SC_ADD(e.x); SC_ADD(e.y); SC_ADD(e.z); SC_ADD(e.w);
    }
    for (; i < S4; i += SC_T) {
        const int4 a = s4[i];
        SC_ADD(a.x); SC_ADD(a.y); SC_ADD(a.z); SC_ADD(a.w);
    }
    for (int64_t t = 4 * S4 + threadIdx.x; t < S; t += SC_T) SC_ADD(status[t]);
#undef SC_ADD
    for (int k = 0; k < 4; ++k)
        if (loc[k]) atomicAdd(&c[k], loc[k]);
    __syncthreads();
    if (threadIdx.x < 4) counts[threadIdx.x] = c[threadIdx.x];
}

extern "C" int phgpu_status_counts(phgpu_handle h, const int32_t* status, int32_t* counts, void* stream) {
    if (!h || !status || !counts) return set_err(-1, "null argument");
    FLUSH_STEP(h);
    hipLaunchKernelGGL(k_status_counts, dim3(1), dim3(SC_T), 0, (hipStream_t)stream, status, h->S, counts);
    HIPCHK(hipGetLastError());
    return 0;
}

// statistics of a solve from its outputs: counts by status, iteration sum and maximum
__global__ void __launch_bounds__(SC_T) k_solve_stats(const int32_t* __restrict__ status,
                                                     const int32_t* __restrict__ iters, int64_t S,
                                                     unsigned long long* __restrict__ out) {
    __shared__ unsigned long long c[6];
    if (threadIdx.x < 6) c[threadIdx.x] = 0;
    __syncthreads();
    unsigned long long loc[4] = {0, 0, 0, 0}, isum = 0, imax = 0;
    for (int64_t t = threadIdx.x; t < S; t += SC_T) {
        const int v = status[t];
        loc[0] += v == 0, loc[1] += v == 1, loc[2] += v == 2, loc[3] += v == 3;
        if (iters) {
            const unsigned long long i = (unsigned long long)iters[t];
            isum += i;
            imax = i > imax ? i : imax;
        }
    }
    for (int k = 0; k < 4; ++k)
        if (loc[k]) atomicAdd(&c[k], loc[k]);
    if (isum) atomicAdd(&c[4], isum);
    if (imax) atomicMax(&c[5], imax);
    __syncthreads();
    if (threadIdx.x < 6) out[threadIdx.x] = c[threadIdx.x];
}

extern "C" int phgpu_solve_stats(phgpu_handle h, int64_t* out, void* stream) {
    if (!h || !out) return set_err(-1, "null argument");
    FLUSH_STEP(h);
    if (!h->last_status) return set_err(-1, "phgpu_solve_stats: no solve yet");
    hipStream_t st = (hipStream_t)stream;
    const unsigned long long* src = h->last_stats;
    if (!src) {
        hipLaunchKernelGGL(k_solve_stats, dim3(1), dim3(SC_T), 0, st, h->last_status, h->last_iters, h->S,
                           h->stats_gen);
        HIPCHK(hipGetLastError());
        src = h->stats_gen;
    } else {  // the path-6 copies, summed into stats_gen (out may be pageable host memory)
        hipLaunchKernelGGL(k_stats_copy, dim3(1), dim3(64), 0, st, src, PHGPU_STATS_COPIES, (int64_t*)h->stats_gen);
        HIPCHK(hipGetLastError());
        src = h->stats_gen;
    }
    HIPCHK(hipMemcpyAsync(out, src, 6 * sizeof(int64_t), hipMemcpyDefault, st));
    return 0;
}

// the x̄ partial sums of phgpu_ph_reduce (node_buf cleared, per-wave partials in part)
static int xbar_partials(phgpu_state* h, const double* x, double* node_buf, hipStream_t st) {
    const size_t nb = (size_t)2 * h->num_nodes * h->nlen_max;
    {
        const int rc = xbar_layout(h, st);
        if (rc) return rc;
    }
    if (h->xbar_mixed) HIPCHK(hipMemsetAsync(node_buf, 0, nb * sizeof(double), st));
    {
        dim3 g = grid_for(h->S);
        g.y = (unsigned)std::max(h->nn, 1);
        hipLaunchKernelGGL(k_xbar_partial, g, dim3(BLOCK), 0, st, *h, x, node_buf, h->xbar_mixed ? 0 : 1);
    }
    HIPCHK(hipGetLastError());
    return 0;
}

// the path-6 epilogue partials of x when the last solve writing the current slot produced
// them for this x buffer, else null
static bool xp_valid(const phgpu_state* h, const double* x, int k) {
    return k >= 0 && h->xp[k] && h->xp_C[k] > 0 && h->xp_x[k] == x && h->xbar_mixed == 0;
}
static bool xp_valid(const phgpu_state* h, const double* x) { return xp_valid(h, x, h->wslot); }
static phgpu_state xp_view(const phgpu_state* h, int k) {  // the state with part = the epilogue partials
    phgpu_state v = *h;
    v.part = h->xp[k];
    v.part_node = h->xp_node[k];
    v.nwaves = h->xp_n[k];
    return v;
}
static phgpu_state xp_view(const phgpu_state* h) { return xp_view(h, h->wslot); }

extern "C" int phgpu_ph_reduce(phgpu_handle h, const double* x, double* node_buf, void* stream) {
    if (!h || !x || !node_buf) return set_err(-1, "null argument");
    FLUSH_STEP(h);
    hipStream_t st = (hipStream_t)stream;
    const size_t nb = (size_t)2 * h->num_nodes * h->nlen_max;
    if (h->nn == 0) return hipMemsetAsync(node_buf, 0, nb * sizeof(double), st) == hipSuccess
                               ? 0 : set_err(-2, "hipMemsetAsync failed");
    // the current slot's solve, or a deferred solve not yet committed (x its output: the PH
    // loop reduces a speculative solve's x ahead of its convergence test, engine.xbar_ahead)
    const int k = xp_valid(h, x) ? h->wslot : (xp_valid(h, x, h->pending) ? h->pending : -1);
    if (k >= 0) {
        // the solve's epilogue wrote the per-chunk partials: final sums.  With one tree node
        // every node_buf entry is a nonant's (its block stores it); else clear it first
        const int assign = (h->num_nodes == 1 && h->nlen_max == h->nn) ? 1 : 0;
        if (!assign) HIPCHK(hipMemsetAsync(node_buf, 0, nb * sizeof(double), st));
        hipLaunchKernelGGL(k_xbar_final, dim3(h->nn), dim3(XF_THREADS), 0, st, xp_view(h, k), node_buf,
                           (const int32_t*)h->xp_dirty[k], h->xp_C[k], x, assign);
        HIPCHK(hipGetLastError());
        return 0;
    }
    const int rc = xbar_partials(h, x, node_buf, st);
    if (rc) return rc;
    hipLaunchKernelGGL(k_xbar_final, dim3(h->nn), dim3(XF_THREADS), 0, st, *h, node_buf, nullptr, 0, nullptr);
    HIPCHK(hipGetLastError());
    return 0;
}

// the conv / statistics sink of the update kernels; launches k_solve_stats first when the
// last solve's path has no in-kernel statistics
static int make_sink(phgpu_state* h, double* conv_local, int64_t* stats_out, hipStream_t st, conv_sink& o) {
    o.conv = conv_local;
    o.stats_dst = stats_out;
    o.stats_src = stats_out ? h->last_stats : nullptr;
    o.stats_copies = PHGPU_STATS_COPIES;  // last_stats: the path-6 statistics
    if (stats_out && !o.stats_src) {  // a path without in-kernel statistics
        hipLaunchKernelGGL(k_solve_stats, dim3(1), dim3(SC_T), 0, st, h->last_status, h->last_iters, h->S,
                           h->stats_gen);
        HIPCHK(hipGetLastError());
        o.stats_src = h->stats_gen;
        o.stats_copies = 1;
    }
    o.scale = (h->nn > 0) ? 1.0 / ((double)h->S * (double)h->nn) : 0.0;
    o.cpart = h->cpart_blk;
    o.cnt = h->blk_cnt;
    return 0;
}

extern "C" int phgpu_ph_update_ex(phgpu_handle h, const double* x, const double* node_buf,
                                  double* xbar, double* W, const double* rho, int update_W,
                                  double* conv_local, int64_t* stats_out, void* stream) {
    if (!h || !x || !node_buf || !xbar || !conv_local || (update_W && (!W || !rho)))
        return set_err(-1, "null argument");
    if (stats_out && !h->last_status) return set_err(-1, "phgpu_ph_update_ex: stats_out before any solve");
    FLUSH_STEP(h);
    hipStream_t st = (hipStream_t)stream;
    conv_sink o;
    const int rc = make_sink(h, conv_local, stats_out, st, o);
    if (rc) return rc;
    // one launch: x̄ scatter, W update, conv (last-block reduction) and the statistics
    // (grid bound measured on config 4, k_ph_update us by kernel trace: 64 blocks 21.1, 128
    // 14.6, 256 12.9, 512 14.8, unbounded (1,536) 28.2; profiles/r06/ll/)
    const int64_t bx = std::min<int64_t>((h->S + UPD_T - 1) / UPD_T, std::max<int64_t>(1, UPD_BLOCKS / std::max(h->nn, 1)));
    hipLaunchKernelGGL(k_ph_update, dim3((unsigned)bx, (unsigned)std::max(h->nn, 1)), dim3(UPD_T), 0, st, *h, x,
                       node_buf, xbar, W, rho, update_W ? 1 : 0, o);
    HIPCHK(hipGetLastError());
    return 0;
}

extern "C" int phgpu_ph_update(phgpu_handle h, const double* x, const double* node_buf,
                               double* xbar, double* W, const double* rho, int update_W,
                               double* conv_local, void* stream) {
    return phgpu_ph_update_ex(h, x, node_buf, xbar, W, rho, update_W, conv_local, nullptr, stream);
}

extern "C" int phgpu_ph_step_local(phgpu_handle h, const double* x, double* node_buf, double* xbar, double* W,
                                   const double* rho, int update_W, double* conv_local, int64_t* stats_out,
                                   void* stream) {
    if (!h || !x || !node_buf || !xbar || !conv_local || (update_W && (!W || !rho)))
        return set_err(-1, "null argument");
    if (stats_out && !h->last_status) return set_err(-1, "phgpu_ph_step_local: stats_out before any solve");
    FLUSH_STEP(h);
    if (h->pvar) {
        // variable probabilities: the generic reduce + update (per-nonant weights, W mask)
        const int rc = phgpu_ph_reduce(h, x, node_buf, stream);
        if (rc) return rc;
        return phgpu_ph_update_ex(h, x, node_buf, xbar, W, rho, update_W, conv_local, stats_out, stream);
    }
    return step_local_impl(h, x, node_buf, xbar, W, rho, update_W, conv_local, stats_out, (hipStream_t)stream);
}

extern "C" int phgpu_ph_step_defer(phgpu_handle h, const double* x, double* node_buf, double* xbar, double* W,
                                   const double* rho, int update_W, double* conv_local, int64_t* stats_out,
                                   void* stream) {
    if (!h || !x || !node_buf || !xbar || !conv_local || (update_W && (!W || !rho)))
        return set_err(-1, "null argument");
    if (stats_out && !h->last_status) return set_err(-1, "phgpu_ph_step_defer: stats_out before any solve");
    FLUSH_STEP(h);
    // (variable probabilities: no folded step, the step runs now)
    if (h->pvar) return phgpu_ph_step_local(h, x, node_buf, xbar, W, rho, update_W, conv_local, stats_out, stream);
    phgpu_state::ph_pending& q = h->pend;
    q.active = 1;
    q.x = x;
    q.node_buf = node_buf;
    q.xbar = xbar;
    q.W = W;
    q.rho = rho;
    q.update_W = update_W ? 1 : 0;
    q.conv = conv_local;
    q.stats = stats_out;
    q.stream = (hipStream_t)stream;
    return 0;
}

extern "C" int phgpu_ph_step_flush(phgpu_handle h) {
    if (!h) return set_err(-1, "null handle");
    return flush_step(h);
}

static int step_local_impl(phgpu_state* h, const double* x, double* node_buf, double* xbar, double* W,
                           const double* rho, int update_W, double* conv_local, int64_t* stats_out, hipStream_t st) {
    void* stream = (void*)st;
    if (h->nn == 0 || h->nn > XL_NN_MAX || h->xbar_mixed != 0 || !h->xbar_single) {
        // the general route (also the first call, which finds out xbar_mixed / _single)
        const int rc = phgpu_ph_reduce(h, x, node_buf, stream);
        if (rc) return rc;
        return phgpu_ph_update_ex(h, x, node_buf, xbar, W, rho, update_W, conv_local, stats_out, stream);
    }
    // the per-chunk x̄ partials: from the path-6 epilogue when it wrote them for this x,
    // else from k_xbar_partial
    const bool xp = xp_valid(h, x);
    if (!xp) {
        const int rc = xbar_partials(h, x, node_buf, st);
        if (rc) return rc;
    }
    conv_sink o;
    const int rc = make_sink(h, conv_local, stats_out, st, o);
    if (rc) return rc;
    // 1,024-thread blocks for a large batch (fewer re-sums of the partials: 10.5 us at
    // 65,536 scenarios vs 14 us with 64-thread blocks), 256 for a small one (8,192: the update
    // part spread over 32 blocks; profiles/r03/x/)
    const unsigned T = h->S > 16384 ? XL_T : 256;
    hipLaunchKernelGGL(k_ph_update_local, dim3((unsigned)((h->S + T - 1) / T)), dim3(T), 0, st,
                       xp ? xp_view(h) : *h, x, node_buf, xbar, W, rho, update_W ? 1 : 0, o,
                       xp ? (const int32_t*)h->xp_dirty[h->wslot] : nullptr, xp ? h->xp_C[h->wslot] : 0);
    HIPCHK(hipGetLastError());
    return 0;
}

extern "C" int phgpu_expectations(phgpu_handle h, const double* obj, const double* bound,
                                  const int32_t* status, double* out, void* stream) {
    if (!h || !obj || !bound || !status || !out) return set_err(-1, "null argument");
    FLUSH_STEP(h);
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(k_expect_partial, grid_for(h->S), dim3(BLOCK), 0, st, *h, obj, bound, status);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(k_sum_partials, dim3(5), dim3(256), 0, st, (const double*)h->part, h->nwaves, 5, 1.0,
                       out);
    HIPCHK(hipGetLastError());
    return 0;
}

extern "C" int phgpu_fix_nonants(phgpu_handle h, const double* xfix, void* stream) {
    if (!h) return set_err(-1, "null handle");
    FLUSH_STEP(h);
    if (h->nn == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    if (h->shared) {
        const int64_t tot = (int64_t)h->nn * h->S;
        hipLaunchKernelGGL(k_fix_nonants_sh, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, *h, xfix);
        HIPCHK(hipGetLastError());
        return 0;
    }
    hipLaunchKernelGGL(k_fix_nonants, grid_for(h->S), dim3(BLOCK), 0, st, *h, xfix);
    HIPCHK(hipGetLastError());
    if (h->pk) {
        HIPCHK(to_records(h, h->lbh, h->n, h->pk_LB, st));
        HIPCHK(to_records(h, h->ubh, h->n, h->pk_UB, st));
    }
    return 0;
}

#include "comm_rccl.inc"

extern "C" int phgpu_destroy(phgpu_handle h) {
    if (!h) return 0;
    rccl_release(h);
    g_ipm_tuning_of.erase(h);
    h->pend.active = 0;  // a deferred step that never ran is dropped with the handle
    if (h->oms[0]) {  // the x / y / omega / sk_iters fields may be bound to slot 1: free by slot
        h->x = h->xs[0];
        h->y = h->ys[0];
        h->omega = h->oms[0];
        h->sk_iters = h->its_s[0];
    }
    void* ptrs[] = {h->row_ptr, h->col_idx, h->col_ptr, h->row_idx, h->perm, h->row_of,
                    h->nonant_col, h->nonant_depth, h->nonant_off, h->nonant_slot,
                    h->A, h->c, h->lb, h->ub, h->q, h->rl, h->ru, h->objc, h->prob, h->pcoef,
                    h->node_of, h->Ah_csr, h->Ah_csc, h->Dr, h->Dc, h->normA, h->lbh, h->ubh,
                    h->rlh, h->ruh, h->ch, h->qh, h->x, h->x0, h->xe, h->xt, h->aty, h->aty0,
                    h->y, h->y0, h->yt, h->omega, h->part, h->part_node, h->pl_col_k,
                    h->pl_col_r, h->pl_row_k, h->pl_row_c, h->qhead, h->wg_col_id, h->wg_row_id,
                    h->wg_col_long, h->wg_row_long, h->wg_col_k, h->wg_col_r, h->wg_row_k, h->wg_row_c,
                    h->pk, h->cmap, h->rmap, h->pcol, h->prow, h->sh_col, h->sh_row, h->sh_norm, h->sh_v,
                    h->sh_u, h->sh_w, h->sh_part, h->sk, h->cs_off, h->cs_len, h->cs_idx, h->cs_src,
                    h->rs_off, h->rs_len, h->rs_idx, h->rs_src, h->cs_val, h->rs_val, h->sk_iters, h->sk_order,
                    h->sk_bins, h->cw_ptr, h->cw_slc, h->rw_ptr, h->rw_slc};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    if (h->split_part) (void)hipFree(h->split_part);
    if (h->jit) {
        if (h->jit->mod) (void)hipModuleUnload(h->jit->mod);
        delete h->jit;
    }
    if (h->ipm) {
        if (h->ipm->mod) (void)hipModuleUnload(h->ipm->mod);
        delete h->ipm;
    }
    if (h->ipm_loop) {
        if (h->ipm_loop->mod) (void)hipModuleUnload(h->ipm_loop->mod);
        delete h->ipm_loop;
    }
    if (h->loop_dbl) (void)hipFree(h->loop_dbl);
    if (h->loop_cnt) (void)hipFree(h->loop_cnt);
    if (h->ipm_list) (void)hipFree(h->ipm_list);
    if (h->ipm_cnt) (void)hipFree(h->ipm_cnt);
    if (h->ipm_stats) (void)hipFree(h->ipm_stats);
    if (h->ipm_prof) (void)hipFree(h->ipm_prof);
    if (h->stats_gen) (void)hipFree(h->stats_gen);
    {
        void* more[] = {h->xp[0], h->xp[1], h->xp_node[0], h->xp_node[1], h->xp_dirty[0], h->xp_dirty[1],
                        h->cpart_blk, h->blk_cnt, h->nb_idx};
        for (void* p : more)
            if (p) (void)hipFree(p);
    }
    if (!h->shared) {  // warm-start slot 1 (slot 0 is x / y / omega / sk_iters above)
        void* slot1[] = {h->xs[1], h->ys[1], h->oms[1], h->its_s[1]};
        for (void* p : slot1)
            if (p) (void)hipFree(p);
    }
    delete h;
    return 0;
}

extern "C" int phgpu_last_error(char* buf, size_t len) {
    if (!buf || len == 0) return -1;
    strncpy(buf, g_err, len - 1);
    buf[len - 1] = 0;
    return 0;
}

extern "C" int64_t phgpu_workspace_bytes(phgpu_handle h) { return h ? h->ws_bytes : -1; }

// path 4 of the last solve (include/phgpu.h)
extern "C" int phgpu_stream_info(phgpu_handle h, int32_t* info) {
    if (!h || !info) return set_err(-1, "null argument");
    info[0] = h->last_path == 4 ? h->last_cluster : 0;
    info[1] = h->last_path == 4 ? 1 : 0;
    return 0;
}

extern "C" int phgpu_kernel_info(phgpu_handle h, int32_t* info) {
    if (!h || !info) return set_err(-1, "null argument");
    // info[0..9]: the register path (L <= 64); info[10..15]: the workgroup path; info[16]:
    // the path phgpu_solve takes by default (1 global, 2 register, 3 workgroup); info[17]:
    // queue mode of the last register-path solve (1 record mode, 0 scenario order, -1 none)
    for (int k = 0; k < 20; ++k) info[k] = 0;
    info[18] = jit_eligible(h) ? 1 : 0;
    info[19] = h->jit ? h->jit->wpe : 0;
    info[17] = h->last_rec;
    info[0] = h->reg_inst;
    info[1] = h->reg_inst >= 0 ? h->reg_L : 0;
    info[2] = h->reg_kc;
    info[3] = h->reg_zc;
    info[4] = h->reg_kr;
    info[5] = h->reg_zr;
    if (h->reg_inst >= 0) {
        const reg_instance& r = g_reg_instances[h->reg_inst];
        info[6] = r.KC;
        info[7] = r.ZC;
        info[8] = r.KR;
        info[9] = r.ZR;
    }
    info[10] = h->wg_inst;
    if (h->wg_inst >= 0) {
        const wg_instance& g = g_wg_instances[h->wg_inst];
        info[11] = g.WPS;
        info[12] = g.KC;
        info[13] = g.ZC;
        info[14] = g.KR;
        info[15] = g.ZR;
    }
    info[16] = h->scen_set && !h->shared ? default_path(h) : h->default_kernel;
    return 0;
}

extern "C" int64_t phgpu_ipm_prof(phgpu_handle h, unsigned long long* out, int64_t n) {
    if (!h) return set_err(-1, "null handle");
    if (!h->ipm_prof) return 0;
    const int64_t k = n < h->ipm_prof_n ? n : h->ipm_prof_n;
    if (out && k > 0 &&
        (hipDeviceSynchronize() != hipSuccess ||
         hipMemcpy(out, h->ipm_prof, k * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess))
        return set_err(-2, "phgpu_ipm_prof: copy failed");
    return h->ipm_prof_n;
}

extern "C" int phgpu_ipm_info(phgpu_handle h, double* info) {
    if (!h || !info) return set_err(-1, "null argument");
    for (int k = 0; k < 16; ++k) info[k] = 0.0;
    info[0] = ipm_eligible(h) ? 1.0 : 0.0;
    info[11] = (double)h->folded;
    info[1] = h->ipm_nf;
    info[2] = h->ipm_off;
    if (h->ipm) {
        info[3] = 1.0;
        info[4] = h->ipm->mr;
        info[5] = h->ipm->nf;
        info[6] = h->ipm->private_bytes;
        info[7] = h->ipm->compile_s;
        info[8] = h->ipm->fac_flops;
        info[9] = h->ipm->sol_flops;
        info[10] = h->ipm->L;
        info[12] = h->ipm->L == 1 ? 1 : (h->ipm->L < 64 ? 2 : (h->ipm->blk ? 4 : 3));
        info[15] = h->ipm->L == 1 && h->ipm_lds == 1 ? 1.0 : 0.0;
    }
    // the subtree kernel's jam statistics of the last path-6 solve (synchronous read)
    if (h->last_stats && h->ipm_stats && h->last_path == 6) {
        std::vector<unsigned long long> st(PHGPU_STATS_WORDS);
        // the solve may still run on a non-blocking stream (a torch side stream, the
        // speculative launch), which hipMemcpy does not wait for: finish it first
        if (hipDeviceSynchronize() == hipSuccess &&
            hipMemcpy(st.data(), h->last_stats, PHGPU_STATS_WORDS * sizeof(unsigned long long),
                      hipMemcpyDeviceToHost) == hipSuccess) {
            info[13] = (double)stats_word(st.data(), PHGPU_STATS_COPIES, 6);
            info[14] = (double)stats_word(st.data(), PHGPU_STATS_COPIES, 7);
        }
    }
    return 0;
}
