/*
 * indy7_mpc.h — C-ABI of the MI355X-native batched SQP-MPC solver (libindy7mpc.so).
 *
 * Plain C: pointers, sizes, int status codes. No torch / HIP types in any signature
 * (streams are passed as opaque `void*` = hipStream_t).
 *
 * Each entry point replaces a piece of the reference's Python/pinocchio/OSQP hot path
 * (reference A2R-Lab/indy7-mpc @ 2025-05-23, paths relative to its root):
 *
 *   i7m_create / i7m_destroy   OSQPSolver.__init__            src/osqp_solver.py:7-46
 *                              (dims, costs, templates, osqp.setup once; here: device
 *                               buffers for max_batch problems, model constants)
 *   i7m_solve / _device        SQP_OSQP.sqp                   src/osqp_sqp.py:76-93
 *                              — the whole <=2-iteration SQP (linearise, QP, line search,
 *                               step) for B independent problems, batch axis of
 *                               src/gato_mpc_batch.py:38-43,97-99
 *   i7m_qp                     OSQPSolver.setup_and_solve_qp  src/osqp_solver.py:137-143
 *                              (returns the QP minimiser sol.x, solved exactly; with
 *                               qp_mode = I7M_QP_BOX the QP also carries box rows on q, v, u
 *                               — SURVEY.md §8d config 4, an extension without a reference
 *                               counterpart; see oracle/box_ipm.py for its definition; with
 *                               qp_mode = I7M_QP_ADMM it is OSQP's iterate, as the reference's
 *                               osqp.solve() returns it, src/osqp_solver.py:38-40,140-143)
 *   i7m_admm_reset             a fresh OSQP object / batch_sqp resetRho, resetLambda
 *                                                             gato_controller.py:132-138
 *   i7m_linearize              update_constraint_matrix + update_cost_matrix
 *                                                             src/osqp_solver.py:70-135
 *   i7m_merit                  SQP_OSQP.eepos_cost + integrator_err
 *                                                             src/osqp_sqp.py:13-47
 *   i7m_linesearch             SQP_OSQP.linesearch            src/osqp_sqp.py:49-74
 *   i7m_eepos                  OSQPSolver.eepos / d_eepos     src/osqp_solver.py:146-155
 *   i7m_aba                    pin.aba (+f_ext)               src/osqp_sqp.py:40, src/utils.py:5
 *   i7m_aba_derivatives        pin.computeABADerivatives      src/osqp_solver.py:71,76
 *   i7m_rk4                    utils.rk4 (plant)              src/utils.py:3-18
 *   i7m_set_external_wrench    batch_sqp.set_external_wrench_batch  gato_controller.py:129
 *   i7m_mpc_run                MPC_OSQP.run_mpc over B instances     src/osqp_mpc.py:14-72
 *                              (batch axis of src/gato_mpc_batch.py:76-217)
 *
 * Layouts (all fp64, C-contiguous, row = problem):
 *   XU    (B, T)  T = 18N-6, [x_0,u_0,x_1,u_1,...,x_{N-1}], x=[q(6),v(6)]  src/osqp_solver.py:22
 *   xcur  (B, 12)
 *   goals (B, N*goal_stride), goal_stride 3 (OSQP surface, src/osqp_solver.py:111) or
 *         6 (batch_sqp surface, gato_controller.py:180-183; first 3 of each 6 used)
 *
 * QP modes (SURVEY.md §8(b) `qp_mode {direct, admm}`):
 *   - I7M_QP_DIRECT solves each SQP subproblem QP exactly (the optimum OSQP's ADMM approximates to
 *     eps 1e-3, src/osqp_solver.py:39-41) and keeps no state between calls;
 *   - I7M_QP_ADMM runs OSQP's algorithm itself (oracle/osqp_admm.py, pinned by the reference's
 *     printed closed loop): per problem a solver state (iterates, rho, the previous QP's linear
 *     cost) carried from call to call like the reference's osqp.OSQP object — i7m_reset or
 *     i7m_admm_reset start it afresh;
 *   - I7M_QP_BOX (config 4) adds box rows, solved by an interior point whose Newton steps are the
 *     exact solve (ADMM needed 40-4700 iterations on those problems).
 * Precision: i7m_config.precision exists; only I7M_PREC_F64 is built, and
 * i7m_create refuses I7M_PREC_F32 with I7M_EINVAL — every kernel computes in fp64.  The drop-in
 * batch_sqp module keeps the reference's SQPSolverfloat_* class names (gato_controller.py:54-62)
 * so callers run unchanged, but it also solves (and returns) fp64.
 *
 * Status: 0 = OK, <0 = error (see I7M_E*), message via i7m_last_error() (thread-local).
 * Threading: a handle is not re-entrant (like the reference's stateful OSQPSolver);
 * use one handle per (host thread, device).
 */
#ifndef INDY7_MPC_H
#define INDY7_MPC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define I7M_NJ 6
#define I7M_NX 12
#define I7M_NU 6
#define I7M_MAX_SQP 8
#define I7M_MAX_N 64

/* ABI revision, returned by i7m_abi_version(); bumped whenever an existing signature, struct
 * layout, field meaning or enum count changes.  6: i7m_get_admm_status has the value 2 ("solved
 * inaccurate") and, after admm_max_iter, runs OSQP's closing tests (0.6 builds).  5: i7m_get_admm_status and i7m_get_admm_dual
 * (appended); i7m_get_admm_stats' iteration record is reset to -1 at the start of every solve
 * (0.5 builds).  4: I7M_QP_ADMM and i7m_config's admm_* fields
 * (appended), I7M_K_COUNT 10 (I7M_K_ADMM, I7M_K_ADMM_PREP), i7m_admm_reset / i7m_get_admm_stats /
 * i7m_get_admm_state, the `precision` field in the former admm_pad slot (0.4 builds).  3: i7m_config's former `pad` is `h2h_chunks` (a
 * nonzero value changes how i7m_solve runs; outside [0, 64] it is refused) and I7M_K_COUNT is 8
 * (I7M_K_LINESEARCH_TAIL added) — size timing arrays from I7M_K_COUNT of this header (0.3 builds).
 * 2: i7m_aba / i7m_rk4 take a wrench `frame` before their outputs and i7m_set_external_wrench a
 * trailing `frame` (0.2 builds); 1 had neither.  A caller built against another revision must not
 * call through this library: compare first. */
#define I7M_ABI_VERSION 6

#define I7M_OK 0
#define I7M_EINVAL -1   /* bad argument (size, null pointer, unsupported N) */
#define I7M_EHIP -2     /* HIP runtime error */
#define I7M_ENOMEM -3   /* device allocation failed */
#define I7M_ENODEV -4   /* no usable gfx950 device */

enum { I7M_QP_DIRECT = 0, I7M_QP_BOX = 1, I7M_QP_ADMM = 2 };
/* How a solve is launched (I7M_QP_DIRECT): FUSED = one kernel per solve (a workgroup per
 * problem runs every SQP iteration's linearisation, QP and line search), FUSED_ITER = that kernel
 * once per SQP iteration, SPLIT = three kernels per SQP iteration; AUTO = SPLIT at every batch
 * size (the fused kernel measured slower at every size).  Bit-identical results
 * in every mode. */
enum { I7M_PIPE_AUTO = 0, I7M_PIPE_SPLIT = 1, I7M_PIPE_FUSED = 2, I7M_PIPE_FUSED_ITER = 3 };
enum { I7M_PREC_F64 = 0, I7M_PREC_F32 = 1 };
#define I7M_BOX_Q 1     /* q_lower <= q <= q_upper    description/indy7.urdf:203-238 <limit> */
#define I7M_BOX_V 2     /* |v| <= velocity limit */
#define I7M_BOX_U 4     /* |u| <= effort limit */

/* 6-DOF serial chain of revolute joints about local +z. Layout == RobotModel.packed(). */
typedef struct i7m_model {
  double placement_R[6][9];   /* joint frame in parent joint frame, row-major */
  double placement_t[6][3];
  double mass[6];
  double com[6][3];           /* in the joint frame */
  double inertia[6][6];       /* about the COM: xx xy xz yy yz zz */
  double gravity[3];          /* (0,0,-9.81), src/osqp_mpc.py:8-9 */
  double q_lower[6], q_upper[6], v_limit[6], effort_limit[6];
} i7m_model;

typedef struct i7m_config {
  int32_t N;            /* knot points (<= I7M_MAX_N), default 32   src/osqp_solver.py:7 */
  int32_t regularize;   /* default 1 */
  double dt;            /* default 0.01 */
  double dQ_cost;       /* default 0.01 */
  double R_cost;        /* default 1e-5 */
  double QN_cost;       /* default 100 */
  double eps;           /* default 1 */
  double mu;            /* merit penalty, 10          src/osqp_sqp.py:50 */
  double step_tol;      /* SQP break tolerance, 1e-3  src/osqp_sqp.py:90 */
  int32_t max_sqp_iters;/* 2                          src/osqp_sqp.py:77 */
  int32_t max_batch;    /* device buffers are sized for this many problems */
  int32_t device_id;
  int32_t qp_mode;      /* I7M_QP_DIRECT: exact block-tridiagonal (Riccati) KKT solve;
                           I7M_QP_BOX: + box rows on q, v, u (interior point, Riccati Newton steps);
                           I7M_QP_ADMM: OSQP's ADMM with its warm-started state */
  i7m_model model;
  /* I7M_QP_BOX only (appended: the offsets above are unchanged) */
  int32_t box_mask;     /* which rows: I7M_BOX_Q | I7M_BOX_V | I7M_BOX_U (default all) */
  int32_t box_max_iters;/* interior-point iterations per QP, default 30 */
  double box_tol;       /* stop when mu < tol and the residuals shrank by tol, default 1e-8 */
  int32_t pipeline;     /* I7M_PIPE_* (appended), default I7M_PIPE_AUTO */
  int32_t h2h_chunks;   /* i7m_solve (host buffers): split the batch into this many chunks, copies in,
                           solves and copies out pipelined on three streams so copies overlap
                           solves; 0 = automatic (was `pad`: same layout) */
  /* I7M_QP_ADMM only (appended): OSQP's settings; defaults (i7m_config_default) are OSQP's own
     with the duality-gap test on and no rho adaptation — the combination that reproduces the
     reference's printed closed loop (oracle/osqp_admm.py) */
  double admm_rho;              /* 0.1; equality rows use 1e3 rho (all of this QP's rows) */
  double admm_sigma;            /* 1e-6 */
  double admm_alpha;            /* relaxation, 1.6 */
  double admm_eps_abs;          /* 1e-3 */
  double admm_eps_rel;          /* 1e-3 */
  int32_t admm_max_iter;        /* 4000 */
  int32_t admm_check_termination; /* 25: residuals are tested every this many iterations */
  int32_t admm_scaling;         /* Ruiz passes, 10 */
  int32_t admm_check_dualgap;   /* 1: OSQP 1.x's duality-gap test */
  int32_t admm_adaptive_rho_interval; /* 0: never adapt rho; else every this many iterations */
  int32_t precision;    /* arithmetic of every kernel (SURVEY.md 8b's ABI sketch): I7M_PREC_F64 (0, the
                           only one built: the reference's OSQP path computes in double);
                           I7M_PREC_F32 (GATO's float, gato_controller.py:54-62) is refused by
                           i7m_create with I7M_EINVAL.  (Was admm_pad: same layout.) */
  double admm_adaptive_rho_tolerance; /* 5 */
} i7m_config;

/* Per-problem SQP statistics (keys of SQP_OSQP.stats, src/osqp_sqp.py:7-11). */
typedef struct i7m_problem_stats {
  int32_t qp_iters;                 /* qp+1 at loop exit                 */
  int32_t n_alphas;                 /* entries of linesearch_alphas       */
  int32_t n_steps;                  /* entries of sqp_stepsizes           */
  int32_t pad;
  double alphas[I7M_MAX_SQP];
  double stepsizes[I7M_MAX_SQP];
} i7m_problem_stats;

typedef struct i7m_handle i7m_handle;

const char* i7m_last_error(void);
const char* i7m_version(void);
int i7m_abi_version(void);                        /* == I7M_ABI_VERSION of the header it was built with */
int i7m_config_default(i7m_config* cfg);          /* fills everything but `model` */
int i7m_device_count(int* n);

/* In ADMM mode the handle's OSQP state (about 4 KB x N per problem) must stay under 2 GiB: the
   iteration kernel addresses it with 32-bit offsets; a larger max_batch x N is refused with
   I7M_EINVAL (shard the batch over handles instead). */
int i7m_create(const i7m_config* cfg, i7m_handle** out);
void i7m_destroy(i7m_handle* h);
/* NULL -> the handle's own stream, a blocking stream (ordered with the legacy null stream) */
int i7m_set_stream(i7m_handle* h, void* stream);
/* Back to the post-create solver state (batch_sqp reset / resetRho / resetLambda,
 * gato_controller.py:132-138): waits for the handle's stream, drops captured solve graphs and
 * zeroes the kernel timing sums; I7M_QP_ADMM: every problem's OSQP state starts afresh
 * (i7m_admm_reset(h, max_batch, I7M_ADMM_RESET_ALL)).  The exact modes carry no warm start,
 * penalty or dual state across calls.  The external wrench is caller input like the model and is
 * kept: clear it with i7m_set_external_wrench(h, 0, NULL, 0). */
int i7m_reset(i7m_handle* h);
int i7m_synchronize(i7m_handle* h);

/* External wrench [force; torque] acting on joint 6's body.  Frames:
 *   I7M_WRENCH_WORLD  a spatial force in the WORLD frame, about the world origin, as the
 *                     reference's callers draw it (gato_controller.py:77-81,120-129;
 *                     src/gato_mpc_batch_sample.py:37-40).  Every dynamics evaluation converts
 *                     it to joint 6's frame at that evaluation's configuration with
 *                     oMi[6].actInv (src/gato_mpc_batch_sample.py:151-161,270-279), and the
 *                     linearisation differentiates that conversion too.  i7m_rk4 converts once
 *                     at the start configuration and holds it over the four stages, as the
 *                     reference's host plant does (:270-279).
 *   I7M_WRENCH_LOCAL  constant in joint 6's LOCAL frame (pinocchio's f_ext[6] as it is). */
#define I7M_WRENCH_LOCAL 0
#define I7M_WRENCH_WORLD 1
/* One wrench per problem, used by every dynamics evaluation of subsequent solves
 * (linearisation and merit).  fext (B, 6); NULL clears it.  Backs
 * batch_sqp.set_external_wrench_batch (gato_controller.py:129). */
int i7m_set_external_wrench(i7m_handle* h, int32_t B, const double* fext, int32_t frame);

/* Full SQP solve, host buffers in/out (H2D + kernels + D2H, synchronous). */
int i7m_solve(i7m_handle* h, int32_t B, const double* xu_in, const double* xcur, const double* goals,
              int32_t goal_stride, double* xu_out, i7m_problem_stats* stats);

/* Full SQP solve on device-resident buffers, asynchronous on the handle's stream.
 * d_stats may be NULL. xu_in may alias xu_out (in-place); otherwise xu_in is only read and every
 * row of xu_out is written (no staging copy). */
int i7m_solve_device(i7m_handle* h, int32_t B, const double* d_xu_in, const double* d_xcur,
                     const double* d_goals, int32_t goal_stride, double* d_xu_out,
                     i7m_problem_stats* d_stats);

/* One QP (linearise at xu, solve exactly): sol (B, T). */
int i7m_qp(i7m_handle* h, int32_t B, const double* xu, const double* xcur, const double* goals,
           int32_t goal_stride, double* sol);

/* The QP's optimal cost-to-go at the first knot (the Riccati value function V~_0 in homogeneous
 * coordinates x~ = [x_0; 1], as the backward sweep ends with it): V0 (B, 13, 13) row-major, the
 * quadratic form the exact solve of i7m_qp minimises over the rest of the trajectory given x_0
 * — its 12 x 12 block is d^2 J* / d x_0^2 (the sensitivity of the optimal QP cost to the initial
 * state, the derivative of the equality multiplier of the x_0 rows l[:12] = -xs of
 * src/osqp_solver.py:85), its last column the linear part.  Diagnostic / test hook (the reference
 * has no counterpart; OSQP returns the multipliers `y`, src/osqp_solver.py:143).  Returned as
 * the recursion computes it except row 12, which the kernel mirrors from column 12 (the linear
 * part); the 12 x 12 block is symmetric only to the recursion's accuracy.  I7M_QP_DIRECT only,
 * N >= 10 (checked before any work). */
int i7m_qp_value(i7m_handle* h, int32_t B, const double* xu, const double* xcur, const double* goals,
                 int32_t goal_stride, double* V0);

/* I7M_QP_BOX: interior-point record of the most recent QP of problems [0, B) (the last
 * i7m_qp, or the last SQP iteration of i7m_solve): corrector steps taken, 1 if converged
 * (mu < box_tol and residuals reduced by box_tol), final mu.  Any output may be NULL. */
int i7m_get_box_stats(i7m_handle* h, int32_t B, int32_t* iters, int32_t* converged, double* mu);

/* I7M_QP_ADMM: start the OSQP state of problems [0, B) afresh.  what: I7M_ADMM_RESET_RHO (rho back
 * to admm_rho; batch_sqp resetRho), _DUAL (y = 0; resetLambda), _PRIMAL (x = z = 0 and the
 * remembered linear cost = 0), _ALL (a new OSQP object: the state right after create). */
#define I7M_ADMM_RESET_RHO 1
#define I7M_ADMM_RESET_DUAL 2
#define I7M_ADMM_RESET_PRIMAL 4
#define I7M_ADMM_RESET_ALL 7
int i7m_admm_reset(i7m_handle* h, int32_t B, int32_t what);
/* I7M_QP_ADMM: OSQP iterations of every SQP iteration of the last solve (B, I7M_MAX_SQP; -1 where
 * the problem ran no QP) and the current rho (B).  Either may be NULL. */
int i7m_get_admm_stats(i7m_handle* h, int32_t B, int32_t* iters, double* rho);
/* I7M_QP_ADMM: the carried OSQP state of problems [0, B) in OSQP's scaled coordinates: x (B, T),
 * z, y (B, 12N), the previous QP's linear cost, unscaled (B, T), rho (B).  Any may be NULL. */
int i7m_get_admm_state(i7m_handle* h, int32_t B, double* x, double* z, double* y, double* q, double* rho);
/* I7M_QP_ADMM (ABI 6): OSQP's result status of every SQP iteration's QP in the last solve
 * (B, I7M_MAX_SQP): 1 "solved" (its termination test passed), 2 "solved inaccurate" and 0
 * "maximum iterations reached" (admm_max_iter came first: as OSQP, the test is run once more at
 * the final iterate unless the last iteration ran it, then with eps_abs and eps_rel x 10, which
 * gives 2), -1 the problem ran no QP at that iteration.  The reference's solve() returns it in
 * .info.status (src/osqp_solver.py:143). */
int i7m_get_admm_status(i7m_handle* h, int32_t B, int32_t* status);
/* I7M_QP_ADMM (ABI 5): the dual y of each problem's last QP, unscaled as OSQP returns it in
 * result.y (y = E y_s / c: the carried scaled y with that QP's row scaling E and cost scale c),
 * (B, 12N). */
int i7m_get_admm_dual(i7m_handle* h, int32_t B, double* y);

/* Raw linearisation at xu.  lin (B, N-1, 114): per knot Aq(6x6,row-major, =dt*da/dq),
 * Av (=I+dt*da/dv), Bu (=dt*Minv), a (=ABA(q,v,u)); cost (B, N, 10): j = J^T e (6),
 * Qm, dQm, Rm, |e|.  Either output may be NULL. */
int i7m_linearize(i7m_handle* h, int32_t B, const double* xu, const double* goals, int32_t goal_stride,
                  double* lin, double* cost);

/* Merit pieces of XU (relative to XU_ref for the initial-state term): out (B, 5) =
 * qcost, vcost, ucost, integrator_err, |XU[:12]-XU_ref[:12]|. */
int i7m_merit(i7m_handle* h, int32_t B, const double* xu, const double* xu_ref, const double* goals,
              int32_t goal_stride, double* out);

/* Backtracking line search of src/osqp_sqp.py:49-74 (no step applied): alpha (B). */
int i7m_linesearch(i7m_handle* h, int32_t B, const double* xu, const double* xu_full,
                   const double* goals, int32_t goal_stride, double* alpha);

/* Kinematics / dynamics hooks, Bq independent queries (q,v,tau: (Bq,6)). */
int i7m_eepos(i7m_handle* h, int32_t Bq, const double* q, double* p_out, double* J_out /*(Bq,3,6) or NULL*/);
int i7m_aba(i7m_handle* h, int32_t Bq, const double* q, const double* v, const double* tau,
            const double* fext /*(Bq,6) spatial force on joint 6, or NULL*/, int32_t frame /*I7M_WRENCH_**/,
            double* a_out);
int i7m_aba_derivatives(i7m_handle* h, int32_t Bq, const double* q, const double* v, const double* tau,
                        double* dq /*(Bq,6,6)*/, double* dv, double* Minv, double* a);
int i7m_rk4(i7m_handle* h, int32_t Bq, const double* q, const double* v, const double* u, double dt,
            const double* fext, int32_t frame, double* q_out, double* v_out);

/* Closed-loop MPC of B independent instances on the device: MPC_OSQP.run_mpc
 * (src/osqp_mpc.py:14-72) per instance — goal = endpoints[0] tiled, XU = 0, an initial solve,
 * then per step: goal distance of xcur (cyclic switch below 0.1, the instance stops above 1.1),
 * xu_new = SQP solve, the rk4 plant over 0.01 s with the PREVIOUS trajectory's controls, the
 * warm-start shift and the first / last state pins — all batched, state resident in HBM; the
 * batch-axis analogue of src/gato_mpc_batch.py:76-217.  xstart (B, 12), endpoints (E, 3);
 * dist_out (num_steps, B) goal distances (NaN once an instance has stopped); q_out
 * (num_steps, B, 6) q after each step's plant, xcur_out (B, 12), xu_out (B, T) the final state
 * and warm start: each may be NULL but dist_out.  Synchronous.  I7M_EINVAL if the handle has an
 * external wrench set (MPC_OSQP's loop has none, src/osqp_mpc.py:56). */
int i7m_mpc_run(i7m_handle* h, int32_t B, const double* xstart, const double* endpoints, int32_t n_endpoints,
                int32_t num_steps, double* dist_out, double* q_out, double* xcur_out, double* xu_out);

/* Per-kernel device timing with HIP events on the launch stream. */
enum { I7M_K_LIN = 0, I7M_K_RICCATI = 1, I7M_K_LINESEARCH = 2, I7M_K_RICCATI_BOX = 3, I7M_K_IPM = 4, I7M_K_IPM_FUSED = 5,
       I7M_K_SQP_FUSED = 6, I7M_K_LINESEARCH_TAIL = 7 /* second launch of a split line search */, I7M_K_ADMM = 8 /* OSQP iterations */,
       I7M_K_ADMM_PREP = 9 /* the QP's scaling and factor */, I7M_K_COUNT = 10 };
int i7m_set_timing(i7m_handle* h, int enable);
/* Sums (ms) and launch counts per kernel id since the last reset; synchronises. */
int i7m_get_kernel_times(i7m_handle* h, double* ms_sum, int32_t* counts, int32_t n);
int i7m_reset_kernel_times(i7m_handle* h);

#ifdef __cplusplus
}
#endif

#endif /* INDY7_MPC_H */
