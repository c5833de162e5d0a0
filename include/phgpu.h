/*
 * phgpu.h -- C-ABI of the MI355X-native progressive-hedging hot path.
 *
 * One handle holds one rank's local scenarios: a CSR sparsity pattern shared by all
 * of them and per-scenario coefficient / bound / objective arrays.  The library
 * replaces, for all local scenarios at once:
 *
 *   - SPOpt.solve_loop / solve_one        mpisppy/spopt.py:226-307 / 85-223
 *       (one LP/QP per scenario through Pyomo's SolverFactory plugin .solve(),
 *        spopt.py:165-172; results fields spopt.py:175-206)      -> phgpu_solve
 *   - PHBase.attach_PH_to_objective terms  mpisppy/phbase.py:617-699
 *       (W_on * W.x + prox_on * rho/2 (x - xbar)^2)                -> phgpu_set_ph_state
 *   - _Compute_Xbar local sums             mpisppy/phbase.py:27-87  -> phgpu_ph_reduce
 *   - Update_W + convergence_diff          mpisppy/phbase.py:293-343 -> phgpu_ph_update
 *   - SPOpt.Ebound / Eobjective / _update_E1 / feas_prob local sums
 *                                          mpisppy/spopt.py:310-439 -> phgpu_expectations
 *
 * The cross-rank sums (the per-node MPI Allreduce of phbase.py:83-87 and the
 * ROOT-comm Allreduce of phbase.py:341) are done by the caller (RCCL all-reduce of
 * the node buffer) between phgpu_ph_reduce and phgpu_ph_update.
 *
 * Conventions
 *   - Every function returns 0 on success and a negative code on error; the text of
 *     the last error of the calling thread is available from phgpu_last_error.
 *   - "host" pointers are read during the call only.  "device" pointers are HIP
 *     device pointers (e.g. torch.Tensor.data_ptr() of a cuda tensor) owned by the
 *     caller; the library owns only the workspace it allocates in phgpu_create and
 *     frees in phgpu_destroy.
 *   - Per-scenario arrays are scenario-fastest: element (k, s) of a k-indexed
 *     quantity lives at [k * S + s]  (coalesced: 64 lanes = 64 scenarios).
 *   - All work is ordered on the given hipStream_t (NULL = default stream); no call
 *     synchronises the device except phgpu_create / phgpu_destroy and
 *     phgpu_set_scenarios on a shared-matrix handle (it sizes its records from the data).
 *   - A handle is used by one host thread; it is not re-entrant; one process per GPU.
 *   - The problem is stored as a minimisation; a maximise model is negated by the
 *     caller (phbase.py:696-699 subtracts the PH term for max, which is the same).
 */
#ifndef PHGPU_H
#define PHGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct phgpu_state* phgpu_handle;

/* Per-scenario solve status (mapped to _mpisppy_data.scenario_feasible and the
 * termination_condition checks of spopt.py:175-194).  PRIMAL_INFEASIBLE: a dual ray
 * (Farkas certificate) was found, obj = bound = +inf; DUAL_INFEASIBLE: a primal ray of
 * descent was found (the subproblem is unbounded), obj = bound = -inf. */
enum {
    PHGPU_OPTIMAL = 0,
    PHGPU_ITER_LIMIT = 1,
    PHGPU_PRIMAL_INFEASIBLE = 2,
    PHGPU_DUAL_INFEASIBLE = 3
};

/* Solver options (the iter0_solver_options / iterk_solver_options dicts of
 * phbase.py:273-274 become these fields). */
typedef struct {
    double eps_rel;        /* relative KKT tolerance (primal, dual, gap)      [1e-9] */
    double eps_abs;        /* absolute KKT tolerance                          [1e-12] */
    int32_t max_iter;      /* PDHG iteration cap per scenario                 [100000] */
    int32_t check_every;   /* KKT / restart check period (iterations)         [64] */
    double gamma;          /* Halpern reflection coefficient in [0, 1]         [1.0]
                              (kernel 2 requires 1.0; kernel 0 uses kernel 1 otherwise) */
    double beta_sufficient;/* restart if r <= beta_suff * r_restart           [0.2] */
    double beta_necessary; /* ... or r <= beta_nec * r_restart and no progress [0.8] */
    double eta_frac;       /* step = eta_frac / ||A_scaled||_2                [0.998] */
    double omega0;         /* initial primal weight (<= 0: keep previous)     [1.0] */
    int32_t keep_omega;    /* 1: carry the primal weight across solves         [1] */
    int32_t restart_every; /* restart test period (iterations; divides check_every) [16] */
    double beta_artificial;/* restart when the Halpern run exceeds this fraction
                              of all iterations of the solve                  [0.36] */
    double omega_clamp;    /* primal weight kept in [1/clamp, clamp] (scaled) [1e4] */
    int32_t kernel;        /* 0 auto, 1 global-memory kernel, 2 register-resident
                              kernel (error if no compiled instance fits),
                              3 workgroup-per-scenario kernel (large scenarios),
                              4 shared-matrix streaming kernel (the only path, and
                              the automatic one, of a PHGPU_SHARED_MATRIX handle),
                              5 pattern-specialised kernel: one lane per scenario,
                              compiled with hipRTC for this handle's pattern at its
                              first path-5 solve (n, m <= 48, nnz <= 128; that solve
                              synchronises the stream once),
                              6 interior-point kernel (Mehrotra predictor-corrector,
                              one lane per scenario, compiled with hipRTC for this
                              handle's pattern and data at its first path-6 solve, which
                              synchronises once; n <= 40, m <= 32, nnz <= 128; the
                              automatic path wherever it applies, PHGPU_IPM=0 turns that
                              off; scenarios it does not finish go to the path-5 PDHG,
                              which certifies infeasibility)              [0] */
    int32_t infeas_start;  /* infeasibility certificates are tested at the KKT
                              checks from this iteration on (< 0: never)      [512] */
    double eps_infeas;     /* certificate tolerance: ray violation <= eps * |ray
                              objective| (PDLP-style)      [1e-8] */
    int32_t split_longest; /* path 4: the split_longest (<= 16) scenarios with the most
                              iterations in the previous solve run first, each over the
                              whole GPU (the split form); 0: the
                              PHGPU_STREAM_SPLIT environment variable, else none  [0] */
} phgpu_options;
/* max_iter must be a multiple of restart_every: the register-resident kernel counts
 * iterations in chunks of restart_every and stops exactly at max_iter (both kernels then
 * report iters == max_iter on ITER_LIMIT). */

/* Fill *opt with the defaults shown above. */
int phgpu_default_options(phgpu_options* opt);

/* Create a handle for S local scenarios sharing one CSR pattern.
 * Replaces: SPOpt._create_solvers / set_instance (spopt.py:839-903) and the
 * nonant index bookkeeping of SPBase._attach_nlens / _attach_nonant_indices
 * (spbase.py:293-320).
 *   row_ptr[m+1], col_idx[nnz]          host, the shared pattern
 *   nonant_col[nn]                      host, column of flat nonant k (node-list
 *                                       order then sorted index, scenario_tree.py:39)
 *   nonant_depth[nn], nonant_off[nn]    host, tree depth of k's node / offset in it
 *   depth                               number of non-leaf nodes per scenario
 *   num_nodes, nlen_max                 size of the node-indexed x̄ buffer
 *                                       (num_nodes * nlen_max entries per half) */
int phgpu_create(phgpu_handle* h, int device, int64_t S, int32_t n, int32_t m, int32_t nnz,
                 const int32_t* row_ptr, const int32_t* col_idx, int32_t nn,
                 const int32_t* nonant_col, const int32_t* nonant_depth,
                 const int32_t* nonant_off, int32_t depth, int32_t num_nodes,
                 int32_t nlen_max);

/* Flags of phgpu_create2.
 * PHGPU_SHARED_MATRIX: every scenario has the same constraint-matrix values (the UC
 *   relaxation: scenarios differ in bounds only).  phgpu_set_scenarios then takes
 *   A_val[nnz] (one copy), scales it once, and keeps per scenario only the iterates and
 *   the columns / rows whose data differ between scenarios (plus the nonant columns);
 *   solves run on path 4 (one workgroup streams one scenario).  Meant for
 *   scenarios too large for the register / workgroup-resident paths. */
#define PHGPU_SHARED_MATRIX 1u

/* phgpu_create with flags (phgpu_create(...) == phgpu_create2(..., 0)). */
int phgpu_create2(phgpu_handle* h, int device, int64_t S, int32_t n, int32_t m, int32_t nnz,
                  const int32_t* row_ptr, const int32_t* col_idx, int32_t nn,
                  const int32_t* nonant_col, const int32_t* nonant_depth,
                  const int32_t* nonant_off, int32_t depth, int32_t num_nodes,
                  int32_t nlen_max, uint32_t flags);

/* Upload per-scenario data (device pointers, scenario-fastest):
 *   A_val[nnz*S] (A_val[nnz] on a PHGPU_SHARED_MATRIX handle), c/lb/ub/q[n*S]
 *   (q may be NULL = 0), rl/ru[m*S] (+-inf allowed),
 *   obj_const[S] (may be NULL), prob[S], node_of[depth*S] (int32 global node id),
 *   prob_coeff[depth*S] (pi_s / pi_node, spbase.py:384-391).
 * Computes the diagonal (Ruiz + Pock-Chambolle) scaling and ||A_scaled||_2 per
 * scenario; replaces the per-scenario Pyomo model construction of
 * SPBase._create_scenarios (spbase.py:255-291). */
int phgpu_set_scenarios(phgpu_handle h, const double* A_val, const double* c,
                        const double* lb, const double* ub, const double* rl,
                        const double* ru, const double* q, const double* obj_const,
                        const double* prob, const int32_t* node_of,
                        const double* prob_coeff, void* stream);

/* Variable probabilities (spbase.py:394-424, phbase.py:54-79 and 315-318): pvar, device
 * [nn*S] (k-major like W), the probability coefficient of nonant k of scenario s in the x̄
 * sums in place of the per-node prob_coeff; Update_W then sets W[k,s] = 0 where pvar[k,s]
 * is 0 (prob0_mask).  Read at every reduce / update (not copied); NULL restores the per-node
 * coefficients.  While set, the PH step always runs as phgpu_ph_reduce + phgpu_ph_update
 * (no epilogue partials, no folded or fused step); partials of earlier solves are dropped. */
int phgpu_set_nonant_probs(phgpu_handle h, const double* pvar);

/* Interior-point tuning of this handle (path 6): defs = "IPM_NAME=number;..." -- the
 * compile-time constants of the generated interior-point modules (jit_ipm*.hip.in:
 * IPM_SIG_MIN, IPM_WARM_T, ...) for the modules this handle builds; a model's measured
 * values (examples/aircond.py IPM_TUNING).  Only IPM_ names and numeric values; NULL or ""
 * clears.  Call before the first solve (-1 once the module is built).  The PHGPU_IPM_DEFS
 * environment variable (experiments) overrides it name by name. */
int phgpu_set_ipm_tuning(phgpu_handle h, const char* defs);

/* Bind the PH objective terms for the next solves (phbase.py:585-699):
 *   objective = f(x) + W_on * sum_k W[k,s] x_k + prox_on * sum_k rho[k,s]/2 (x_k - xbar[k,s])^2
 * W, rho, xbar: device [nn*S]; they are read at solve time (not copied). */
int phgpu_set_ph_state(phgpu_handle h, const double* W, const double* rho,
                       const double* xbar, int W_on, int prox_on);

/* Solve all local scenarios (SPOpt.solve_loop, spopt.py:226-307).
 *   warm_start   1: start from the previous solution (x, y) of this handle
 *   x[n*S]       device out: primal solution (all columns)
 *   y[m*S]       device out (may be NULL): row duals (positive = lower bound active)
 *   obj[S]       device out: augmented objective incl. PH terms (what
 *                Eobjective sums, spopt.py:332-333)
 *   bound[S]     device out: Lagrangian dual bound (results.Problem[0].Lower_bound,
 *                spopt.py:201-206)
 *   status[S]    device out: PHGPU_* code
 *   iters[S]     device out (may be NULL): iterations used (PDHG iterations; interior-
 *                point iterations for scenarios path 6 solved)
 * phgpu_solve_stats and phgpu_ph_update_ex(stats_out) read the status / iters outputs of
 * the last solve launched on the handle (paths without in-kernel statistics): those
 * buffers must stay alive until the next solve when statistics are requested.  A solve
 * rejected by validation leaves the previous solve's buffers in place.
 * Kernel 0 (automatic) on a pattern path 6 applies to: if its module cannot be compiled
 * or loaded, path 6 is turned off for the handle's data (phgpu_ipm_info off = 2), the
 * reason stays in phgpu_last_error and the solve runs on the handle's PDHG path;
 * kernel 6 asked for explicitly returns the error instead. */
int phgpu_solve(phgpu_handle h, const phgpu_options* opt, int warm_start, double* x,
                double* y, double* obj, double* bound, int32_t* status, int32_t* iters,
                void* stream);

/* Speculative solves.  PHBase.iterk_loop (phbase.py:909-957) decides after x̄ / W /
 * conv whether the next solve_loop runs; the engine launches it before that decision
 * and keeps it only if the loop goes on.  phgpu_solve_deferred is phgpu_solve except
 * that the warm-start state it leaves (the iterate the next warm solve starts from,
 * the primal weight, the work-queue predictor) goes to a second slot, which becomes the
 * handle's state only at phgpu_commit; any other solve before that drops it, so a
 * discarded speculative solve leaves the handle exactly as the last committed solve
 * did.  Its outputs (x, y, obj, bound, status, iters) are written as by phgpu_solve.
 * A PHGPU_SHARED_MATRIX handle (path 4) has one slot and rejects deferred solves. */
int phgpu_solve_deferred(phgpu_handle h, const phgpu_options* opt, int warm_start, double* x,
                         double* y, double* obj, double* bound, int32_t* status, int32_t* iters,
                         void* stream);

/* Make the warm-start state of the last phgpu_solve_deferred current (no-op if there is
 * none pending).  Host-side bookkeeping only: no device work, no synchronisation. */
int phgpu_commit(phgpu_handle h);

/* Local x̄ partial sums (phbase.py:54-79): node_buf[2*num_nodes*nlen_max] gets
 *   [g*nlen_max + o]                        sum_s prob_coeff * x
 *   [num_nodes*nlen_max + g*nlen_max + o]   sum_s prob_coeff * x^2
 * over the local scenarios whose depth-d node is g.  node_buf is overwritten. */
int phgpu_ph_reduce(phgpu_handle h, const double* x, double* node_buf, void* stream);

/* After the cross-rank sum of node_buf: scatter x̄ to every local scenario
 * (phbase.py:90-103), W += rho (x - x̄) if update_W (phbase.py:293-318), and
 * conv_local[0] = sum_{s,k} |x - x̄| / (S * nn)  (phbase.py:330-339; the caller
 * sums over ranks and divides by n_proc, phbase.py:341-343).
 *   xbar, W: device [nn*S] (xbar written, W updated in place). */
int phgpu_ph_update(phgpu_handle h, const double* x, const double* node_buf, double* xbar,
                    double* W, const double* rho, int update_W, double* conv_local,
                    void* stream);

/* phgpu_ph_update, plus: stats_out (int64[6], may be NULL) receives the statistics of
 * the handle's last solve launch as phgpu_solve_stats reports them, written by the same
 * kernel that writes conv_local.  conv_local and stats_out may be host-mapped pinned
 * memory (zero-copy), which saves the copy launches of the PH loop's convergence and gripe
 * readbacks (phbase.py:330-343, spopt.py:284-294): the host may read them after an event
 * recorded behind this call, or poll them -- they are written last, by one store
 * instruction, so a caller that set conv_local to NaN and stats_out to -1 before the call
 * has all seven values once none of them is a sentinel (the engine does that: no event
 * marker in the PH step).  The conv reduction over the grid is done by the kernel's last
 * block.  Clears no other state. */
int phgpu_ph_update_ex(phgpu_handle h, const double* x, const double* node_buf, double* xbar,
                       double* W, const double* rho, int update_W, double* conv_local,
                       int64_t* stats_out, void* stream);

/* phgpu_ph_reduce + phgpu_ph_update_ex for a single rank (no cross-rank sum of node_buf
 * between them), in fewer launches when every nonant's local scenarios share one node (a
 * two-stage problem) and nn <= 16: the x̄ final sum is folded into the update kernel.
 * Same outputs: node_buf (the local sums), xbar, W, conv_local, stats_out. */
int phgpu_ph_step_local(phgpu_handle h, const double* x, double* node_buf, double* xbar, double* W,
                        const double* rho, int update_W, double* conv_local, int64_t* stats_out,
                        void* stream);

/* phgpu_ph_step_local, deferred: the step is recorded and runs at the handle's next call.
 * If that call is a phgpu_solve_deferred that takes path 6 (the batched interior point),
 * writes other output buffers than x, and the previous solve was path 6 with its x̄
 * partials for x, the step is folded into the solve launch's prologue:
 * every block sums the previous solve's partials to x̄, each scenario updates its x̄ / W,
 * and the grid's last block stores conv_local; stats_out (the previous solve's statistics)
 * is stored by the same launch.  conv_local and stats_out are written a few microseconds
 * into the solve: a caller polling them (NaN / -1 sentinels, as phgpu_ph_update_ex
 * describes) learns the convergence metric while the solve runs.  Any other call on the
 * handle (or a solve that cannot fold it) first runs the step as phgpu_ph_step_local on
 * the stream given here.  PHGPU_FUSE_STEP=0 never folds (experiments). */
int phgpu_ph_step_defer(phgpu_handle h, const double* x, double* node_buf, double* xbar, double* W,
                        const double* rho, int update_W, double* conv_local, int64_t* stats_out,
                        void* stream);

/* Run a step deferred by phgpu_ph_step_defer now (no-op if none is pending). */
int phgpu_ph_step_flush(phgpu_handle h);

/* Local probability-weighted sums (spopt.py:310-439) into out[5]:
 *   out[0] = sum_s prob_s * obj_s    out[1] = sum_s prob_s * bound_s
 *   out[2] = sum_s prob_s (E1)       out[3] = sum_{s feasible} prob_s, where feasible
 *   means status is OPTIMAL or ITER_LIMIT (a solution was loaded; spopt.py:175-194
 *   marks only infeasible / unbounded / no-solution results infeasible)
 *   out[4] = sum_{s OPTIMAL} prob_s (certified solves: the xhat inner bound,
 *   xhatbase.py:210-216, is only taken when this equals E1) */
int phgpu_expectations(phgpu_handle h, const double* obj, const double* bound,
                       const int32_t* status, double* out, void* stream);

/* counts[c] = number of local scenarios whose status[s] == c, c = 0..3 (OPTIMAL,
 * ITER_LIMIT, PRIMAL_INFEASIBLE, DUAL_INFEASIBLE): the check behind SPOpt.solve_loop's
 * gripe (spopt.py:284-294) as one device reduction.  status: device [S] (phgpu_solve's
 * output), counts: device int32[4]. */
int phgpu_status_counts(phgpu_handle h, const int32_t* status, int32_t* counts, void* stream);

/* Statistics of the last solve (phgpu_solve / phgpu_solve_deferred on this handle),
 * enqueued on stream into out[6] (device or pinned host memory): the number of local
 * scenarios with status 0..3 (what phgpu_status_counts gives for its status output), the
 * sum and the maximum of its iters output.  Path 6 accumulates them inside its kernels
 * (then this is one 48-byte copy); for the other paths a one-block reduction over the
 * last solve's outputs computes them (iters may have been NULL: sum = max = 0). */
int phgpu_solve_stats(phgpu_handle h, int64_t* out, void* stream);

/* Fix the nonants of every local scenario (lb = ub = xfix[k*S + s], original units,
 * clipped to the model bounds) for the following solves, or restore the model bounds
 * when xfix is NULL.  A NaN entry leaves that nonant at its model bounds (partial
 * fixing: Xhat_Eval.fix_nonants_upto_stage, xhat_eval.py:326-362).  Replaces
 * SPOpt._fix_nonants / _restore_nonants as used by Xhat_Eval and XhatBase._try_one
 * (spopt.py:557-660, xhatbase.py:199-216).
 *   xfix: device [nn*S] (read during the call only) or NULL */
int phgpu_fix_nonants(phgpu_handle h, const double* xfix, void* stream);

/* Free the workspace and the handle. */
int phgpu_destroy(phgpu_handle h);

/* Copy the calling thread's last error message (NUL-terminated) into buf. */
int phgpu_last_error(char* buf, size_t len);

/* Workspace bytes held by the handle (diagnostics / memory planning). */
int64_t phgpu_workspace_bytes(phgpu_handle h);

/* Solve-kernel selection of the handle (diagnostics): info[20] =
 * {register path (L <= 64 lanes per scenario): instance or -1, L, column slots / CSC
 *  entries per column / row slots / CSR entries per row needed, the instance's KC, ZC, KR,
 *  ZR;  workgroup path (one workgroup per scenario): instance or -1, waves per scenario,
 *  KC, ZC, KR, ZR;  the default path of phgpu_solve: 1 global, 2 register, 3 workgroup,
 *  4 shared-matrix streaming, 5 pattern-specialised, 6 interior point;  the queue mode of the last
 *  register-path solve: 1 record mode (longest-first queue, scenario-major records), 0
 *  scenario order, -1 none yet;  1 if path 5 applies to the pattern;  the waves per SIMD
 *  of the compiled path-5 kernel, 0 if none is compiled yet}. */
int phgpu_kernel_info(phgpu_handle h, int32_t* info);

/* The ranks' sums of the PH step through the library's own RCCL communicator
 * (comm_rccl.inc), in place of the node-communicator Allreduce of _Compute_Xbar and the
 * Allreduce of convergence_diff (phbase.py:83-87, 339-343; mpisppy/MPI.py's Allreduce over
 * mpi4py).  phgpu_comm_unique_id writes a 128-byte RCCL unique id (call it on one rank and
 * broadcast it); phgpu_comm_init joins the handle's communicator slot (0: the sums issued on
 * the launch stream, 1: those on a side stream -- one user stream per communicator) to the
 * communicator of nranks ranks as rank (collective: every rank calls it, one id per slot);
 * phgpu_allreduce_sum sums n doubles in place over the ranks on stream with the slot's
 * communicator.  RCCL is loaded at run time (the process's librccl.so.1 or the system's);
 * -2 when it is absent. */
int phgpu_comm_unique_id(char* id);
int phgpu_comm_init(phgpu_handle h, const char* id, int nranks, int rank, int slot);
int phgpu_allreduce_sum(phgpu_handle h, int slot, double* buf, int64_t n, void* stream);

/* Path 4 (shared matrix, PDHG) of the last solve: info[2] = {workgroups per scenario of its
 * cluster form (0: one workgroup per scenario slot on the queue; K >= 2: a batch smaller
 * than the GPU, every scenario over K co-resident workgroups with cluster barriers), 1 if
 * the last solve took path 4}.  No reference counterpart (diagnostics). */
int phgpu_stream_info(phgpu_handle h, int32_t* info);

/* Path-6 (interior point) diagnostics: info[16] = {1 if path 6 applies to the pattern,
 * factor entries of the pattern with every row active, 1 if a compiled module spilled
 * and 2 if the module failed to compile or load (path 6 is then not the automatic path
 * until new data arrives by phgpu_set_scenarios), 1 if a module is compiled, rows in its normal
 * equations, its factor entries, its scratch bytes per lane, its hipRTC compile seconds,
 * flops of one LDL' factorisation, flops of one forward + backward solve, lanes per
 * scenario of its IPM kernel (1, or a lane group of 2..16: more lanes for fewer local
 * scenarios, PHGPU_IPM_LANES pins it; 64..256: threads of a workgroup per scenario), PH
 * steps folded into solve launches so far (phgpu_ph_step_defer), the IPM kernel (0 none
 * compiled, 1 one lane, 2 lane groups, 3 workgroup, 4 subtree), and of the last path-6 solve
 * (synchronises): scenarios the subtree kernel found still jammed after its re-centrings
 * (handed to the PDHG fallback, never reported OPTIMAL), re-centrings, and 1 when the
 * one-lane module keeps its slack reciprocals in LDS (a module that spilled otherwise,
 * PHGPU_IPM_LDS=0 turns it off)}: 16 doubles. */
int phgpu_ipm_info(phgpu_handle h, double* info);

/* PHBase.iterk_loop (phbase.py:875-979) of one rank in one cooperative launch (no
 * extension, converger or spoke: the loop's only decision is conv < convthresh):
 *   for it = 1..max_iters: x̄ = the node's pcoef-weighted mean of the last solve's nonants,
 *   W += rho (x - x̄), conv = mean |x - x̄| (phbase.py:27-107, 293-343); stop if conv <
 *   convthresh; solve every local scenario's PH subproblem (path 6, warm-started)
 * with every scenario's data and iterate in registers and x̄ / conv by grid-wide steps.
 * x / y / obj / bound / status / iters as phgpu_solve (x also gives the nonants of the solve
 * before the loop); W and x̄ are the handle's PH state (phgpu_set_ph_state, updated in place);
 * node_buf receives the last step's node sums.  conv_hist (host, max_iters) gets each step's
 * conv; out (host, 4): [0] PH steps taken, [1] 0 limit / 1 conv < convthresh / 2 a solve
 * handed scenarios to the PDHG fallback (solved after the loop; the caller continues step by
 * step), [2] IPM iterations summed over the loop's solves.  Synchronises the stream.
 * Returns -3 (nothing launched) when the handle's state is not one it runs: several nodes
 * per nonant depth, variable probabilities, no prox term, a path other than the one-lane
 * interior point, or more workgroups than fit the GPU at once. */
int phgpu_ph_loop(phgpu_handle h, const phgpu_options* opt, int max_iters, double convthresh, double* x,
                  double* y, double* obj, double* bound, int32_t* status, int32_t* iters, double* node_buf,
                  double* conv_hist, int64_t* out, void* stream);

/* Diagnostics (no reference counterpart): the per-wave timelines of the last path-6 launch,
 * stored by modules compiled with IPM_PROF=1 (PHGPU_IPM_DEFS) on a handle created with
 * PHGPU_IPM_PROF=1 in the environment: 16 words per wave (wave = block * 4 + wave in block):
 * 100 MHz real-time stamps at entry, loop start, loop end, stores done, statistics done and
 * exit, the loop trips, and with IPM_PROF=2 (lane groups) words 8..15 the shader-clock
 * cycles of the loop's phases.  Copies min(n, available) words to out (synchronising the
 * device) and returns the words available (0: no buffer), < 0 on error. */
int64_t phgpu_ipm_prof(phgpu_handle h, unsigned long long* out, int64_t n);

/* The path-6 source the library generates for a pattern and its data flags (host code
 * only; tests and tools).  flags / v0 are per element of [A nnz | c n | q n | lb n | ub n |
 * rl m | ru m]: bit 0 the same value in every scenario, bit 1 finite in some scenario,
 * bit 2 finite in every scenario, bit 3 (rl elements) rl == ru in every scenario; v0 the
 * first scenario's value.  nonant_slot[n]: nonant index of each column or -1; lanes: lanes
 * per scenario of the IPM kernel (1, 2, 4, 8 or 16), or threads of a workgroup per scenario
 * (64, 128, 192 or 256: the subtree kernel for a block-angular pattern unless
 * PHGPU_IPM_BLK=0, else the workgroup kernel).  Writes the
 * NUL-terminated source to buf when len exceeds its length; returns the length + 1 (or a
 * negative error); info[4] (may be NULL) = {rows in the normal equations, factor entries,
 * factorisation flops, solve flops}. */
int phgpu_ipm_source(int32_t n, int32_t m, int32_t nnz, const int32_t* row_ptr, const int32_t* col_idx,
                     const int32_t* nonant_slot, const int32_t* flags, const double* v0, int32_t lanes, char* buf,
                     size_t len, int32_t* info);

#ifdef __cplusplus
}
#endif
#endif /* PHGPU_H */
