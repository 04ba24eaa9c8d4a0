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

/* u_ref semantics */
#define HMPC_UREF_ALIASED 0       /* what cvxpy actually solves: every stage sees
                                     the last stage's u_ref (the default)        */
#define HMPC_UREF_PER_STAGE 1     /* the intended per-stage 2mg*C[k]             */

typedef struct hmpc_ctx hmpc_ctx;

/* ABI version (major*10000 + minor*100 + patch) */
int hmpc_version(void);

/* Which horizons have a compiled kernel for `variant`; writes up to `cap`
   values into `Ns`, returns the count. */
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
