/*
 * hmpc.h -- C ABI of the MI355X batched MPC/QP solve path.
 *
 * Drop-in boundary for the per-timestep QP of bbokser/hopper-mpc-inertial:
 * every entry point below replaces one piece of the reference's
 * ``Mpc`` class (src/mpc_cvx_euler_3f.py, src/mpc_cvx_euler_2f.py):
 *
 *   hmpc_create          <- Mpc.__init__(t, N, m, g, mu, Jinv, rh)
 *                           (src/mpc_cvx_euler_3f.py:12-39, 2f :12-38)
 *   hmpc_solve_batch     <- Mpc.gen_dt_dynamics + Mpc.build_qp + Mpc.solve_qp
 *                           (3f :71-160, 2f :70-158), one QP per instance,
 *                           B instances per call, device pointers
 *   hmpc_solve_batch_host  same, host pointers (staged through the context's
 *                           device buffers; synchronous)
 *   hmpc_mpcontrol_batch <- Mpc.mpcontrol(x_in, x_ref_in, pf, C, init)
 *                           (3f :41-69): builds the linearisation x_hat
 *                           (init: [x_in; x_ref], else the time shift of the
 *                           previous x*) on device, runs 1 or 2 solves
 *   hmpc_mpcontrol_plan_batch <- the Runner's call (src/robotrunner.py:98-107):
 *                           Mpc.mpcontrol on path_plan_grab(x_ref, k) /
 *                           path_plan_grab(pf_ref, k) read in place from a
 *                           device-resident plan (:228-230), no staging
 *   hmpc_plant_batch     <- Runner.rk4_normalized / dynamics_ct
 *                           (src/robotrunner.py:126-164) for n_steps
 *                           low-level steps, then convert (:19-28)
 *   hmpc_convert_batch   <- convert(X) (src/robotrunner.py:19-28)
 *   hmpc_plan_batch      <- Runner.path_plan_init (src/robotrunner.py:182-226)
 *                           + gait_map (:174-180), one plan per robot
 *   hmpc_gait_batch      <- the Runner loop's gait_scheduler / gait_map calls
 *                           (src/robotrunner.py:92-101)
 *   hmpc_destroy         <- object lifetime
 *
 * Conventions: every array is row-major, contiguous, float64, batch-major
 * (instance b's x_ref is x_ref[b*N*12 .. (b+1)*N*12)).  C holds the contact
 * schedule as 0.0/1.0 like the reference's gait_map.  Errors are returned as
 * negative int codes and never thrown across the ABI; per-instance solver
 * outcomes are written to ``status`` (HMPC_SOLVED, ...).  A status other than
 * HMPC_SOLVED corresponds to the reference raising
 * Exception("\n *** QP FAILED *** \n") (src/mpc_cvx_euler_3f.py:158-159).
 */
#ifndef HMPC_H
#define HMPC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* return codes (API level) */
#define HMPC_OK 0
#define HMPC_ERR_ARG -1           /* bad argument / null pointer / misaligned */
#define HMPC_ERR_UNSUPPORTED -2   /* (variant, N) without a compiled kernel   */
#define HMPC_ERR_HIP -3           /* HIP runtime error (see hmpc_last_error)  */
#define HMPC_ERR_NOMEM -4

/* per-instance status codes */
#define HMPC_SOLVED 0
#define HMPC_MAX_ITER 1
#define HMPC_PRIMAL_INFEASIBLE 2
#define HMPC_NUMERICAL 3          /* condensed Hessian not positive definite */

/* variants: the two dynamics formulations of the reference */
#define HMPC_VARIANT_3F 3         /* src/mpc_cvx_euler_3f.py: world-frame force */
#define HMPC_VARIANT_2F 2         /* src/mpc_cvx_euler_2f.py: body-frame, fy = 0 */
#define HMPC_VARIANT_CAS 4        /* src/mpc_cas_euler_3f.py: the CasADi/qpOASES
                                     variant's QP as the reference builds it
                                     (second-order discretisation at the yaw of
                                     x_in, one-sided dynamics rows, scalar u_ref;
                                     x_lin and pf are ignored, rf is fixed);
                                     1 <= N <= 11, fp64 only */

/* u_ref semantics */
#define HMPC_UREF_ALIASED 0       /* what cvxpy actually solves: every stage sees
                                     the last stage's u_ref (the default)        */
#define HMPC_UREF_PER_STAGE 1     /* the intended per-stage 2mg*C[k]             */

/* arithmetic of the solve (hmpc_set_precision) */
#define HMPC_PREC_F64 0           /* fp64; the dedicated kernel when N has one (default) */
#define HMPC_PREC_F32 1           /* fp32 arithmetic (BASELINE configs[4]: the tolerance/
                                     throughput trade-off): the dense kernel's fp32
                                     build where N has one (N = 10), else generic */
#define HMPC_PREC_F64_GENERIC 2   /* fp64 on the generic kernel (its fp32 twin's A/B) */
#define HMPC_PREC_F64_RICCATI 3   /* fp64 on the Riccati kernel (any N <= 64; the default
                                     for 10 < N <= 64)                            */
#define HMPC_PREC_F64_DENSE 4     /* fp64 on the dedicated dense kernel of N (compiled
                                     horizons only; the default for N <= 10)      */
#define HMPC_PREC_F32_GENERIC 5   /* fp32 on the generic kernel (round-1 configs[4]) */
#define HMPC_PREC_F32_REFINED 6   /* configs[4]'s fp32 + fp64 iterative refinement: the fp32
                                     dense kernel's factors and active set, then
                                     hmpc_set_refinement() corrections of that active set's
                                     KKT system with fp64 residuals; an instance whose fp64
                                     check fails goes to the fp64 overflow pass (N = 10) */

typedef struct hmpc_ctx hmpc_ctx;

/* ABI version (major*10000 + minor*100 + patch): 1.2.0 = 1.0 + the fp32 dense
   build, HMPC_PREC_F64_RICCATI / _F64_DENSE / _F32_GENERIC, hmpc_kernel_name,
   hmpc_active_capacity, hmpc_plan_batch, hmpc_gait_batch, HMPC_VARIANT_CAS;
   1.3.0 = + hmpc_solve_batch_stats, HMPC_PREC_F32_REFINED, hmpc_set_refinement;
   1.4.0 = + hmpc_set_order;
   1.5.0 = + hmpc_overflow_total;
   1.5.1 = hmpc_kernel_name / hmpc_active_capacity report the last solve's N = 60
           kernel (capacity 64 at small batches);
   1.5.2 = the cross-stream completion event is recorded at a stream switch,
           not after every call (the last call's stream must stay valid) */
int hmpc_version(void);

/* Which horizons have a dedicated (one- or two-wavefront) kernel for
   `variant`; writes up to `cap` values into `Ns`, returns the count.  Every
   other horizon 1 <= N <= 64 (e.g. the Runner's N = 60) is solved by the
   Riccati kernel (one wavefront per instance, the condensed Hessian factored
   by a backward Riccati recursion), 64 < N <= 128 by the generic dense kernel.
   Every solve with N <= 64 re-solves the rare instances whose active set
   outgrows its kernel's capacity in an overflow pass (capacity 6N).  The
   context's workspaces and counters are shared by its calls, so the context
   orders them itself: a call on a different stream than the context's last
   one first records an event on that last stream and makes its own stream
   wait for it (hipStreamWaitEvent), so the stream of a context's last call
   must stay valid until the context's next call (or hmpc_overflow_total,
   which synchronises it).  Eager calls on one context never overlap; use one
   context per stream for concurrent solves.  Calls enqueued while their stream
   captures a HIP graph are outside this ordering (a replay runs whenever the
   caller launches it): the caller orders a graph's replays against the
   context's other streams, e.g. by synchronising the replay stream before
   the next eager call elsewhere (hmpc_runner.Runner does). */
int hmpc_supported_horizons(int variant, int* Ns, int cap);

/* Mpc.__init__: t = MPC sampling time (s), N = horizon, m (kg), g (m/s^2),
   mu = friction coefficient used when a batch passes mu == NULL,
   Jinv = inverse inertia (row-major 3x3), rh = hip offset (3).
   device = HIP device ordinal to bind the context to. */
int hmpc_create(hmpc_ctx** out, int variant, int N, double t, double m, double g,
                double mu, const double* Jinv, const double* rh, int uref_mode,
                int device);

int hmpc_destroy(hmpc_ctx* ctx);

/* One QP per instance on the given linearisation x_lin (device pointers).
     x_in  [B,12]       initial state (constraint x[0] == x_in)
     x_lin [B,N+1,12]   linearisation trajectory (rows 0..N-1, cols 0:3 and 5 used)
     x_ref [B,N,12]     reference trajectory
     pf    [B,N,3]      footstep plan
     C     [B,N]        contact schedule (0.0 swing / 1.0 stance)
     mu    [B] or NULL  friction coefficient per instance
   outputs
     u     [B,N,6]      optimal inputs u*
     x     [B,N+1,12]   optimal states x* (may be NULL)
     obj   [B]          optimal objective incl. its constant term (may be NULL)
     status[B]          HMPC_SOLVED / ...
     iters [B]          active-set iterations (may be NULL)
   `stream` is a hipStream_t (NULL = default stream).  Asynchronous. */
int hmpc_solve_batch(hmpc_ctx* ctx, int64_t B,
                     const double* x_in, const double* x_lin, const double* x_ref,
                     const double* pf, const double* C, const double* mu,
                     double* u, double* x, double* obj, int32_t* status, int32_t* iters,
                     void* stream);

/* hmpc_solve_batch plus one more output: active [B] receives each
   instance's final active-set size (the number of inequality rows active at
   the optimum the solver certifies; may be NULL).  The bench feeds its mean
   into the algorithmic flop count (bench.algorithmic_flops). */
int hmpc_solve_batch_stats(hmpc_ctx* ctx, int64_t B,
                           const double* x_in, const double* x_lin, const double* x_ref,
                           const double* pf, const double* C, const double* mu,
                           double* u, double* x, double* obj, int32_t* status, int32_t* iters,
                           int32_t* active, void* stream);

/* Same with host pointers; synchronous. */
int hmpc_solve_batch_host(hmpc_ctx* ctx, int64_t B,
                          const double* x_in, const double* x_lin, const double* x_ref,
                          const double* pf, const double* C, const double* mu,
                          double* u, double* x, double* obj, int32_t* status, int32_t* iters);

/* Mpc.mpcontrol for B independent controllers (device pointers).
   x_prev [B,N+1,12] is read when init == 0 (the previous x*) and always
   overwritten with the new x*.  u [B,N,6] receives the control.  Status is
   the worst status over the (1 or 2) solves.  Asynchronous. */
int hmpc_mpcontrol_batch(hmpc_ctx* ctx, int64_t B, int init,
                         const double* x_in, const double* x_ref, const double* pf,
                         const double* C, const double* mu,
                         double* x_prev, double* u, double* obj, int32_t* status,
                         int32_t* iters, void* stream);

/* Mpc.mpcontrol for B robots against a plan resident on the device
   (src/robotrunner.py:98-107).  x_ref_plan [T,12] and pf_plan [T,3] are the
   Runner's path_plan_init output (one per robot when plan_bstride = T rows,
   shared when 0); robot b's window is rows k, k + f, ..., k + (N-1) f
   (path_plan_grab, f = mpc_factor), which must lie inside [0, T).  C [N] is
   gait_map(N, mpc_dt, t, t0), shared by the batch when C_bstride = 0.
   Otherwise as hmpc_mpcontrol_batch.  Asynchronous. */
int hmpc_mpcontrol_plan_batch(hmpc_ctx* ctx, int64_t B, int init,
                              const double* x_in, const double* x_ref_plan,
                              const double* pf_plan, int64_t T, int64_t plan_bstride,
                              int64_t k, int mpc_factor,
                              const double* C, int64_t C_bstride, const double* mu,
                              double* x_prev, double* u, double* obj, int32_t* status,
                              int32_t* iters, void* stream);

/* The Runner's plant between two MPC solves, for B robots on the device:
   n_steps RK4 steps of dynamics_ct with step dt and the input held
   (src/robotrunner.py:104-113,126-164).  X [B,13] (p, q = [w,x,y,z], v, w:
   the simulator's SE(3) state) is advanced in place.  The held input of robot
   b is U[b*U_bstride .. +6) (pass the mpcontrol output u with U_bstride = 6N
   to take its first row, as the Runner does).  Step s uses the foot position
   pf[b*pf_bstride + s*pf_sstride .. +3) (the Runner's pf_ref[k + s]).
   J [9] is the body inertia (host pointer); m, g, rh and J^-1 come from the
   context.  X_hist [B,n_steps,13] (optional) receives every step's state,
   x_out [B,12] (optional) convert(X) after the last one.  Asynchronous. */
int hmpc_plant_batch(hmpc_ctx* ctx, int64_t B, int n_steps, double dt, const double* J,
                     double* X, const double* U, int64_t U_bstride,
                     const double* pf, int64_t pf_bstride, int64_t pf_sstride,
                     double* X_hist, double* x_out, void* stream);

/* x [B,12] = convert(X [B,13]) (src/robotrunner.py:19-28).  Asynchronous. */
int hmpc_convert_batch(hmpc_ctx* ctx, int64_t B, const double* X, double* x, void* stream);

/* Runner.path_plan_init (src/robotrunner.py:182-226) for B robots on the
   device: robot b's plan from its own start x_in[b] and goal xf[b] (convert()ed
   MPC states, [B,12] device) into x_ref [B,T,12] and pf_ref [B,T,3], T = N_run +
   N_k (N_k = N * mpc_factor: the MPC horizon in low-level steps).  curve != 0 is
   the --curve plan with the reference's quirks (:193-201).  t_p, phi_switch,
   t_start and step_adjustment are the Runner's gait constants (:44-49,78-79);
   C_map [T] (optional) receives gait_map(T, dt, t_start, 0) (:213).  Feeds
   hmpc_mpcontrol_plan_batch with plan_bstride = T.  Synchronous on `stream`
   (once per run): returns HMPC_ERR_ARG where the reference raises IndexError
   (a footstep peak moved outside the plan by step_adjustment, or a footstep
   counter past the end of idx_pf, :211-223) or a robot has more than 64
   footstep peaks; the plan is then not valid. */
int hmpc_plan_batch(hmpc_ctx* ctx, int64_t B, int N_run, int N_k, double dt, int curve, double t_p,
                    double phi_switch, double t_start, int step_adjustment, const double* x_in,
                    const double* xf, double* x_ref, double* pf_ref, double* C_map, void* stream);

/* The Runner loop's gait schedule (src/robotrunner.py:92-101,166-180) on the
   device: t = t_start; for step k < n_steps: t += dt, s_hist[k] =
   gait_scheduler(t, t0) (optional output), and at every MPC call (k % mpc_factor
   == 0) the row C_calls[p] = gait_map(N, mpc_dt, t, t0) of [n_calls, N], with
   the reference's float64 time accumulation.  Asynchronous. */
int hmpc_gait_batch(hmpc_ctx* ctx, int n_steps, int mpc_factor, int N, double dt, double mpc_dt, double t_p,
                    double phi_switch, double t_start, double t0, double* C_calls, double* s_hist,
                    void* stream);

/* Arithmetic of every later solve on this context (HMPC_PREC_*; inputs and
   outputs stay fp64 at the ABI).  BASELINE configs[4] asks for fp32 vs fp64:
   fp32 loses most of the 1e-6 tolerance on this ill-conditioned problem
   (reduced Hessian condition ~3e6), see DESIGN.md. */
int hmpc_set_precision(hmpc_ctx* ctx, int precision);

/* Number of fp64 corrections HMPC_PREC_F32_REFINED runs (0..16, default 5:
   each contracts the error by ~cond x eps32, measured max|du| 1.7e-3 / 7.4e-5 /
   3.1e-6 / 1.3e-7 / 6.4e-9 after 2 / 3 / 4 / 5 / 6 on configs[4]; each costs an
   fp64 rollout + adjoint and two fp32 sweeps per instance).  An instance is
   accepted only when its last correction is below 4e-6 (converged), so with
   fewer than about 4 corrections -- 0 included -- nearly every instance fails
   that check and is re-solved by the fp64 overflow pass: the results stay
   exact, the cost is that of the fp64 pass for the whole batch. */
int hmpc_set_refinement(hmpc_ctx* ctx, int corrections);

/* Instance order of later solves (results do not depend on it):
     HMPC_ORDER_AUTO            longest-first for small batches, where the
                                instances that start last set the step time
                                (dense split B <= 8192; Riccati kernel up to 8
                                instances per resident workgroup), else index
     HMPC_ORDER_INDEX           batch index order
     HMPC_ORDER_LONGEST_FIRST   stance-stage buckets, most stance stages first
   Longest-first measured +21 % at configs[1] (B = 4096) and +12 % at the
   Runner's N = 60 (B = 4096); -0.4 % at configs[2], -6 % at configs[3]. */
#define HMPC_ORDER_AUTO 0
#define HMPC_ORDER_INDEX 1
#define HMPC_ORDER_LONGEST_FIRST 2
int hmpc_set_order(hmpc_ctx* ctx, int order);

/* Name of the solve kernel this context's (variant, N, precision) runs on,
   as rocprofv3 demangles it, e.g. "hmpc::ric_kernel<3, 2, 0, 0, 0>" (the Riccati
   horizons above 24 run "hmpc::ric_factor_kernel<...> + hmpc::ric_kernel<..., 2>"); a split launch names
   every class kernel, "hmpc::solve_kernel<3, 10, double, 48, 13> + hmpc::solve_kernel<3, 10,
   double, 0, 0>" (the narrowest first; 2f's full class is the 5N-wide
   "hmpc::solve_kernel<2, 10, double, 50, 20>"; the fp32 builds list the fp64
   "hmpc::swing_kernel<10, 13>" class first).  N = 60 names the last solve's
   kernel: batches up to three workgroups per CU run the capacity-64
   "hmpc::ric_kernel<3, 1, 60, 64, 2>".  Static string, "" when none.  For
   benchmark records and profiles. */
const char* hmpc_kernel_name(hmpc_ctx* ctx);

/* Active-set capacity of that kernel's main pass (-1 when none): instances
   whose active set grows beyond it are re-solved by the overflow pass
   (capacity 6N) inside the same call, so this is a performance figure, not a
   limit (0 for the generic kernel, which has no overflow pass).  N = 60: the
   last solve's (64 for small batches, else 47, whose overflows go first to a
   capacity-64 second tier). */
int hmpc_active_capacity(hmpc_ctx* ctx);

/* Instances the overflow pass has re-solved on this context since it was
   created: the active sets that outgrew the main pass's capacity, and (the
   fp32 + fp64 refinement build) the instances whose fp64 check or
   convergence test failed.  Waits for the context's last solve.  No
   reference analogue: it reports where the GPU path spends its slow pass. */
int hmpc_overflow_total(hmpc_ctx* ctx, int64_t* total);

/* Last HIP error string of this context ("" if none). */
const char* hmpc_last_error(hmpc_ctx* ctx);

/* Kernel-level timing support for benchmarks: launches the solve kernel
   `reps` times on `stream` between two HIP events and returns the mean
   kernel time in milliseconds through *ms (device pointers as in
   hmpc_solve_batch). */
int hmpc_time_solve_batch(hmpc_ctx* ctx, int64_t B,
                          const double* x_in, const double* x_lin, const double* x_ref,
                          const double* pf, const double* C, const double* mu,
                          double* u, double* x, double* obj, int32_t* status, int32_t* iters,
                          int reps, void* stream, double* ms);

#ifdef __cplusplus
}
#endif

#endif /* HMPC_H */
