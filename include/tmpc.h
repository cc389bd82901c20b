/*
 * tmpc.h -- C ABI of the MI355X-native batched trajectory-optimisation solver
 * (libtmpc.so).  Drop-in boundary for the hot path of
 * VCA-EPFL/TrajoptMPCReference:
 *
 *   TrajoptMPCReference.SQP(x, u, N, dt, METHOD, options)   TrajoptMPCReference.py:510-760
 *     formKKTSystemBlocks                                    TrajoptMPCReference.py:200-271
 *     solveKKTSystem_Schur (+ PCG)                           TrajoptMPCReference.py:415-455
 *   PCG(A, b, block_size, Nblocks, guess, options).solve()   GBD-PCG-Python/PCG.py:5-16,66-111,214
 *   URDFPlant.forward_dynamics / forward_dynamics_gradient   TrajoptPlant.py:283-323
 *   TrajoptPlant.integrator (Euler, type 0)                  TrajoptPlant.py:83-108
 *
 * The reference has no FFI of its own (it is pure Python); these are the
 * entry points a ctypes binding of that Python surface needs (see
 * INTEGRATION.md).  Conventions:
 *   - every entry point returns 0 on success and < 0 on error; the message is
 *     available from tmpc_last_error(ctx) (the reference print()s and exit()s);
 *   - host pointers are caller-owned and only accessed during the call;
 *     "_device" entry points take device pointers obtained from
 *     tmpc_device_alloc on the same context;
 *   - one context per GPU, used by one host thread; calls are synchronous on
 *     the context's HIP stream;
 *   - all arithmetic is IEEE fp64, as in the reference, unless tmpc_options.precision selects
 *     fp32 dynamics (TMPC_PRECISION_F32 / _MIXED).
 *
 * Array layouts follow the reference's NumPy arrays in C order:
 *   x: [B][nx][N] (state column per knot), u: [B][nu][N-1],
 *   per-knot matrices row-major [K][rows][cols].
 */
#ifndef TMPC_H
#define TMPC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TMPC_ABI_VERSION 10  /* 10: tmpc_*_solve_stream_device; 9: tmpc_pcg_dense_batch; 8: tmpc_qp_blocks_batch */

/* SQPSolverMethods (TrajoptMPCReference.py:13-18). */
#define TMPC_LINSYS_S 1      /* Schur complement, direct block-tridiagonal solve (:441-446; np.linalg.solve in the reference) */
#define TMPC_LINSYS_PCG_J 2  /* PCG, Jacobi preconditioner            PCG.py:168-169 */
#define TMPC_LINSYS_PCG_BJ 3 /* PCG, block-Jacobi preconditioner      PCG.py:171-179 */
#define TMPC_LINSYS_PCG_SS 4 /* PCG, symmetric-stair preconditioner   PCG.py:181-212 */
#define TMPC_LINSYS_PCG_0 5  /* PCG, no preconditioner ('0', identity) PCG.py:114-118 (no SQPSolverMethods member;
                                reachable through solveKKTSystem_Schur's options['preconditioner_type']) */
#define TMPC_LINSYS_N 6      /* N, the reference's default: the dense KKT solve [G + rho I, C^T; C, 0] [dxu; lambda] =
                                [g; c] (solveKKTSystem :313-359).  Its solution is the Schur complement's
                                (lambda = S^-1 gamma, dxu = G^-1 (g - C^T lambda)), so it runs the direct Schur
                                path of method S; where the KKT matrix is singular the reference takes lstsq
                                (:353-357) and so does this path (trace.singular; the zero-row and duplicate-row
                                cases of hard limits, see tmpc_hard.hip) -- the KKT least-squares answer equals the
                                Schur one for consistent constraint sets and for FULL_SET's zero rows. */

/* preconditioner ids for tmpc_pcg_batch (PCG options['preconditioner_type']) */
#define TMPC_PRECOND_J 1
#define TMPC_PRECOND_BJ 2
#define TMPC_PRECOND_SS 3
#define TMPC_PRECOND_NONE 4  /* '0' */

/* joint types of the model arrays */
#define TMPC_JOINT_REVOLUTE 0  /* X(q) = X0 + cos(q) Xa + sin(q) Xb */
#define TMPC_JOINT_PRISMATIC 1 /* X(q) = X0 + q Xa                  */

/* box-limit modes (BoxConstraint modes, TrajoptConstraint.py:27-35).  Soft: penalty terms in the
 * cost and the augmented-Lagrangian outer loop.  Hard: rows of C / c per knot
 * (TrajoptMPCReference.py:238-248) -- ACTIVE_SET the violated entries, FULL_SET all of them (the
 * inactive ones with zero jacobian rows: S is then singular, which the reference's PCG preconditioner
 * rejects with LinAlgError and its method S answers with lstsq; here FULL_SET runs with method S and
 * gives the inactive rows lambda = 0, the minimum-norm least-squares solution). */
#define TMPC_LIMIT_NONE 0
#define TMPC_LIMIT_QUADRATIC_PENALTY 1
#define TMPC_LIMIT_AUGMENTED_LAGRANGIAN 2
#define TMPC_LIMIT_ACTIVE_SET 3
#define TMPC_LIMIT_FULL_SET 4

typedef struct tmpc_ctx tmpc_ctx;

/* Every key of TrajoptMPCReference.set_default_options (TrajoptMPCReference.py:91-115)
 * that the unconstrained SQP path reads, plus the PCG keys (PCG.py:19-25). */
typedef struct tmpc_options {
  double exit_tolerance_linSys;          /* 1e-6   */
  int32_t max_iter_linSys;               /* 100    */
  int32_t max_iter_SQP_DDP;              /* 100    */
  double exit_tolerance_SQP_DDP;         /* 1e-6   */
  double alpha_factor_SQP_DDP;           /* 0.5    */
  double alpha_min_SQP_DDP;              /* 0.005  */
  double rho_factor_SQP_DDP;             /* 4      */
  double rho_min_SQP_DDP;                /* 1e-3   */
  double rho_max_SQP_DDP;                /* 1e3    */
  double rho_init_SQP_DDP;               /* 1e-3   */
  double expected_reduction_min_SQP_DDP; /* 0.05   */
  double expected_reduction_max_SQP_DDP; /* 3      */
  double merit_mu;                       /* 10 (fixed in the reference, :545-546) */
  int32_t profile;                       /* 1: time kernels with HIP events (tmpc_kernel_stats) */
  int32_t max_iter_softConstraints;      /* 10     */
  double exit_tolerance_softConstraints; /* 1e-6   */
  /* PCG warm start (options['guess'] -> PCG.update_guess, TrajoptMPCReference.py:439-440; the reference's
   * SQP never forwards it, :512-519, so 0 is the reference behaviour): 1 = each QP's PCG starts from the
   * previous QP's lambda of the same problem, and in tmpc_mpc_batch the first QP of an MPC step starts
   * from the previous step's last lambda shifted by one knot (oracle/mpc.py). */
  int32_t pcg_warm_start;                /* 0      */
  /* Arithmetic precision (BASELINE configs 3 and 5; the reference is fp64 throughout):
   * TMPC_PRECISION_F64   everything fp64 (default, the reference's arithmetic);
   * TMPC_PRECISION_F32   the dynamics' derivatives (M^-1, RNEA gradient: A_k, B_k of the QP build and
   *                      of the iLQR linearisation) and the iLQR Riccati sweep in fp32; every
   *                      trajectory evaluation (the QP's defects, line-search trials, iLQR rollouts) in
   *                      fp64, so costs, merit and the exit tests are the fp64 ones (round 6);
   * TMPC_PRECISION_MIXED rigid-body dynamics (derivatives and trajectory evaluations) in fp32, Schur
   *                      complement / PCG and Riccati in fp64.
   * In every mode the buffers, the merit / cost sums, the acceptance tests and the MPC loop's
   * simulated plant step are fp64; the standalone dynamics entry points (tmpc_rollout_batch_device,
   * tmpc_fd_batch, tmpc_fd_grad_batch) evaluate in fp32 under F32 and MIXED. */
  int32_t precision;                     /* 0      */
} tmpc_options;

#define TMPC_PRECISION_F64 0
#define TMPC_PRECISION_F32 1
#define TMPC_PRECISION_MIXED 2

/* Box limits of TrajoptConstraint (set_joint_limits / set_velocity_limits / set_torque_limits,
 * TrajoptConstraint.py:190-206) in a soft or hard mode, with the BoxConstraint options (:38-46).
 * Index 0 = joint (q), 1 = velocity (qd), 2 = torque (u); lb/ub have n entries.
 * Vector semantics for constraint_size > 1 and the other corrections of SURVEY F6 are
 * documented in oracle/soft.py. */
typedef struct tmpc_box_limits {
  int32_t mode[3];
  int32_t reserved;
  double lb[3][8];
  double ub[3][8];
  double mu_init[3];    /* quadratic_penalty_mu_init        1e-2 */
  double mu_factor[3];  /* quadratic_penalty_mu_factor      10   */
  double mu_max[3];     /* quadratic_penalty_mu_max         1e12 */
  double phi_init[3];   /* augmentated_lagrangian_phi_init   1e-2 */
  double phi_factor[3]; /* augmentated_lagrangian_phi_factor 10   */
} tmpc_box_limits;

/* Per-problem SQP trace, the numeric fields of self.trace (TrajoptMPCReference.py:555-569,691-743).
 * Every member is nullable; each array is [B][max_iter_SQP_DDP + 1]; row 0 is the initial entry,
 * row i+1 the entry appended by SQP iteration i; rows used = sqp_iter + 1. */
typedef struct tmpc_trace {
  int32_t* iteration;
  int32_t* line_search_iteration;
  double* alpha;
  double* rho;
  double* J;
  double* c;
  double* merit;
  double* D;               /* NaN in row 0 (None in the reference) */
  double* reduction_ratio; /* NaN in row 0 */
  int32_t* succeeded_line_search;
  int32_t* pcg_iters;      /* PCG iterations of the QP solved in that SQP iteration (0 in row 0) */
  int32_t* singular;       /* 1: that QP's direct solve took the least-squares answer (S / KKT singular: the
                              reference's lstsq fallback, :353-357, 431-436; its self.singular is this flag
                              made sticky) */
  uint64_t* hard_active;   /* [B][max_iter_SQP_DDP + 1][N] (hard box limits only, else zeros): the active set of
                              that QP per knot, bit t * 2n + e for limit kind t (0 joint, 1 velocity, 2 torque)
                              and entry e of [z - lb; ub - z] (e < n lower, e >= n upper) when that entry is
                              violated -- ACTIVE_SET's rows, FULL_SET's nonzero rows (TrajoptConstraint.py:64-68,
                              110-111; TrajoptMPCReference.py:238-248) */
} tmpc_trace;

int tmpc_abi_version(void);
int tmpc_device_count(int* count);
int tmpc_create(int device, tmpc_ctx** out);
void tmpc_destroy(tmpc_ctx* ctx);
const char* tmpc_last_error(const tmpc_ctx* ctx);

/* Robot model in DFS order, as built by the reference's URDF parser
 * (GRiD/URDFParser/URDFParser.py:227-435): parent[n] (-1 = base), joint type,
 * index of the unit motion-subspace vector S (0..5), transform coefficient
 * matrices X0/Xa/Xb [n][6][6] and spatial inertias I [n][6][6]; gravity is
 * options['gravity'] (TrajoptPlant.py:31, -9.81).  Replaces URDFPlant.__init__
 * (TrajoptPlant.py:275-281) + RBDReference(robot) state.  1 <= n <= 12: up to 7 joints every solver, limit
 * kind and precision mode; 8..12 joints ("wide" models, round 6) the dynamics entry points, the SQP
 * (N * 2n <= 1024 Schur rows) and iLQR (QuadraticCost, fp64, no box limits) on the runtime-model kernels --
 * the other entry points fail with a message naming the limit. */
int tmpc_set_model(tmpc_ctx* ctx, int n, const int32_t* parent, const int32_t* jtype, const int32_t* saxis,
                   const double* X0, const double* Xa, const double* Xb, const double* I, double gravity);

/* QuadraticCost(Q, QF, R, xg, QF_start) (TrajoptCost.py:24-47); QF_start < 0 means None. */
int tmpc_set_cost_quadratic(tmpc_ctx* ctx, int nx, int nu, const double* Q, const double* QF, const double* R,
                            const double* xg, int32_t QF_start);

/* UrdfCost(plant, Q, QF, R, xg, QF_start) (TrajoptCost.py:371-569): the quadratic form acts on the
 * end-effector task state [p(q); J(q) qd] (RBDReference.py:123-148, 313-387), Gauss-Newton hessian
 * (hess_mode 0, :490-492).  2-link arms only (nx = 4, nu = 2), as the reference.  H0 / Ha / Hb:
 * [2][4][4] row-major coefficients of each joint's homogeneous transform
 * H_j(q) = H0 + cos q Ha + sin q Hb (Joint.py:91-97).  Supported by tmpc_sqp_solve_batch[_device];
 * iLQR, the MPC loop and tmpc_qp_batch reject it. */
int tmpc_set_cost_ee(tmpc_ctx* ctx, int nx, int nu, const double* Q, const double* QF, const double* R,
                     const double* xg, int32_t QF_start, const double* H0, const double* Ha, const double* Hb);

void tmpc_default_options(tmpc_options* opts);
int tmpc_set_options(tmpc_ctx* ctx, const tmpc_options* opts);

/* Soft box limits for the following solves (NULL: unconstrained, the reference default
 * TrajoptConstraint()).  Resets the soft-constraint state. */
int tmpc_set_box_limits(tmpc_ctx* ctx, const tmpc_box_limits* limits);

/* The per-problem augmented-Lagrangian constants -- the reference keeps them in the
 * BoxConstraint objects (quadratic_penalty_mu, augmented_lagrangian_lambda / _phi, :21-24)
 * and SQP updates them in place (:137-166).  Layout [B][N][6 n]: knot k, slot t*2n + e with
 * t = 0 joint / 1 velocity / 2 torque, e < n the lower-bound half, e >= n the upper half.
 * set: NULL arrays take the defaults (mu_init, 0, phi_init).  The state persists in the
 * context across solves of the same (B, N), like the reference object's. */
int tmpc_set_soft_state(tmpc_ctx* ctx, int B, int N, const double* mu, const double* lam, const double* phi);
int tmpc_get_soft_state(tmpc_ctx* ctx, int B, int N, double* mu, double* lam, double* phi);

/* Batched TrajoptMPCReference.SQP (TrajoptMPCReference.py:510-760) for B independent problems,
 * with the soft-constraint outer loop (:483-508) when box limits are set.  x [B][nx][N] and u [B][nu][N-1] are read as the
 * initial trajectory and overwritten with the result; per-problem outputs mirror the returned
 * tuple (x, u, exit_sqp, exit_soft, outer_iter, sqp_iter).  trace is nullable. */
int tmpc_sqp_solve_batch(tmpc_ctx* ctx, int B, int N, double dt, int linsys, double* x, double* u,
                         int32_t* exit_sqp, int32_t* exit_soft, int32_t* outer_iter, int32_t* sqp_iter,
                         tmpc_trace* trace);

/* Same solve with x/u already resident in device memory (tmpc_device_alloc); exit_sqp and
 * sqp_iter are host arrays [B] (nullable). */
int tmpc_sqp_solve_batch_device(tmpc_ctx* ctx, int B, int N, double dt, int linsys, double* d_x, double* d_u,
                                int32_t* exit_sqp, int32_t* sqp_iter);

/* Batched iLQR (the reference has only the MPCSolverMethods.iLQR enum value,
 * TrajoptMPCReference.py:21-27): Riccati backward sweep + closed-loop forward rollouts with the
 * SQP's *_SQP_DDP options, rho schedule and exit codes, and the soft-constraint outer loop when box
 * limits are set.  Algorithm: oracle/ilqr.py.  x is replaced by the rollout of u from x[:, 0]
 * before the first iteration.  exit_code: 1 converged (dJ < tol), 2 rho > rho_max, 3 max_iter.
 * trace as tmpc_sqp_solve_batch (c = 0, merit = J, D = dV1 of the backward sweep). */
int tmpc_ilqr_solve_batch(tmpc_ctx* ctx, int B, int N, double dt, double* x, double* u, int32_t* exit_code,
                          int32_t* exit_soft, int32_t* outer_iter, int32_t* iters, tmpc_trace* trace);
int tmpc_ilqr_solve_batch_device(tmpc_ctx* ctx, int B, int N, double dt, double* d_x, double* d_u,
                                 int32_t* exit_code, int32_t* iters);

/* Continuous batching (ABI 10): `problems` independent problems solved through `slots` resident slots.
 * The batch entry points above run B problems in lock step until the slowest one exits, so the GPU's
 * work per batch iteration shrinks to a few problems in the tail.  Here a slot whose problem finishes
 * (its last outer pass, i.e. its exit) takes the next pending problem in the same batch iteration, so
 * every batch iteration runs `slots` problems until the stream drains.  This is how the reference's own
 * drivers use the solver: a pool of independent problems (examples/test_multiple.py:123-128).  Each
 * problem's operations are those of a batch solve from the same input, so its results (x, u, exit
 * codes, iteration counts, trace) are bitwise those of tmpc_sqp_solve_batch / tmpc_ilqr_solve_batch;
 * with soft limits every problem starts from the limits' initial constants (a fresh BoxConstraint).
 * All arrays are device memory (tmpc_device_alloc):
 *   x_in [period][nx][N], u_in [period][nu][N-1]   problem p starts from input p % period (iLQR: only
 *                                                   x_in[:, :, 0] and u_in are read, as tmpc_ilqr_solve_batch);
 *   x_out [problems][nx][N], u_out [problems][nu][N-1]   results (nullable);
 *   status [problems][4]   exit code, iterations, exit_soft, outer_iter (nullable);
 *   trace                  device arrays [problems][max_iter_SQP_DDP + 1] per field (each nullable;
 *                          hard_active must be NULL).
 * The context's soft-constraint state is left unset (tmpc_get_soft_state fails until the next solve).
 * Work counters (tmpc_solve_counters) and kernel timings sum over the sub-streams. */
typedef struct tmpc_stream {
  int32_t problems;
  int32_t slots;
  int32_t period;
  int32_t substreams;   /* 0 / 1: one stream; K = 2..8: K concurrent sub-streams (own HIP stream, slots / K slots,
                           a contiguous 1 / K of the problems each), whose kernels overlap on the GPU */
  const double* x_in;
  const double* u_in;
  double* x_out;
  double* u_out;
  int32_t* status;
  tmpc_trace trace;
} tmpc_stream;
int tmpc_sqp_solve_stream_device(tmpc_ctx* ctx, int N, double dt, int linsys, const tmpc_stream* stream);
int tmpc_ilqr_solve_stream_device(tmpc_ctx* ctx, int N, double dt, const tmpc_stream* stream);

/* Receding-horizon MPC loop for B problems (the reference has only the hooks --
 * shift_QF_start, shift_soft_constraint_constants -- and no loop, F1; algorithm: oracle/mpc.py).
 * Per step: solve the horizon (solver = TMPC_LINSYS_* for SQP, or TMPC_SOLVER_ILQR) warm-started
 * from (x, u); apply u[:, 0] to the plant (one Euler step); shift x, u by one knot (last kept) with
 * x[:, 0] = the new state; QF_start -= 1 (floor 0) when set; soft-limit constants shifted.
 * Outputs: the executed states x_exec [B][nx][steps+1] and controls u_exec [B][nu][steps], per-step
 * exit codes and iteration counts [B][steps] (all nullable); x, u hold the final shifted horizon.
 * SQP horizons: the fused QP up to N * nx = 1536 (past 1024 rows the PCG keeps S in HBM); past that the banded
 * path of the hard-limit kernels with no constraint rows, PCG up to N * nx = 4096 and the direct methods (S, N)
 * up to the banded Schur kernel's LDS (arm6 N <= 650, a 7-joint arm N <= 556; fewer with hard-limit rows -- a
 * longer horizon fails with the largest supported N in the message); pcg_warm_start is refused there (the banded
 * PCG takes no guess).  iLQR has no horizon limit. */
#define TMPC_SOLVER_ILQR 16
int tmpc_mpc_batch(tmpc_ctx* ctx, int B, int N, double dt, int solver, int steps, double* x, double* u,
                   double* x_exec, double* u_exec, int32_t* exit_codes, int32_t* iters);
int tmpc_mpc_batch_device(tmpc_ctx* ctx, int B, int N, double dt, int solver, int steps, double* d_x, double* d_u,
                          double* d_x_exec, double* d_u_exec, int32_t* d_exit_codes, int32_t* d_iters);

/* Euler rollout x_{k+1} = f(x_k, u_k) from x[:, 0] (device pointers), the §8d initial trajectory. */
int tmpc_rollout_batch_device(tmpc_ctx* ctx, int B, int N, double dt, double* d_x, const double* d_u);

/* ---- kernel-level entry points (unit parity) ---- */

/* URDFPlant.forward_dynamics + Euler integrator for K independent knots
 * (TrajoptPlant.py:92-99,283-299): x [K][nx], u [K][nu] -> xnext [K][nx], qdd [K][n],
 * Minv [K][n][n] (outputs nullable). */
int tmpc_fd_batch(tmpc_ctx* ctx, int K, double dt, const double* x, const double* u, double* xnext, double* qdd,
                  double* Minv);

/* URDFPlant.forward_dynamics_gradient + integrator(return_gradient=True)
 * (TrajoptPlant.py:100-108,301-323): -> A [K][nx][nx], B [K][nx][nu], dqdd [K][n][3n] (nullable). */
int tmpc_fd_grad_batch(tmpc_ctx* ctx, int K, double dt, const double* x, const double* u, double* A, double* B,
                       double* dqdd);

/* One QP of the SQP loop for B problems: formKKTSystemBlocks + solveKKTSystem_Schur with PCG
 * (TrajoptMPCReference.py:200-271,415-455) at the given trajectories and regularisation rho[B];
 * xs [B][nx] (nullable: x[:, :, 0]) is the SQP's initial state, the initial-state row's c_0 = x_0 - xs.
 * guess [B][N nx] (nullable) is the PCG initial iterate, options['guess'] of solveKKTSystem_Schur (:439-440).
 * dxul [B][n_xu(N-1)+nx + nx N] in the reference's interleaved order [x0,u0,x1,...,x_{N-1}; lambda].
 * S_diag [B][N][nx][nx], S_lo [B][N-1][nx][nx] (= S_{k+1,k}), gamma [B][N nx], P_diag [B][N][nx][nx]
 * are optional (nullable) copies of the intermediate blocks.
 * With hard box limits (ACTIVE_SET / FULL_SET) the knots' constraint rows join the QP
 * (TrajoptMPCReference.py:238-248): the lambda part of dxul then holds the multipliers of the
 * N nx dynamics / initial-state rows in knot order (the hard rows' multipliers are dropped), and
 * guess, S_diag, S_lo, gamma, P_diag must be NULL (S is banded with variable blocks).
 * With soft box limits the QP carries their jacobian terms (:220-225, :255-259) at the context's soft state
 * (mu / lambda per knot, tmpc_set_soft_state).  That state is kept per (B, N): when the last
 * tmpc_set_soft_state or solve was for a different B or N, it is first reset to the limits' initial
 * constants -- so set it (tmpc_set_soft_state with this B, N) right before a tmpc_qp_batch that must see a
 * particular mu / lambda (the Python drop-in's solveKKTSystem(_Schur) always does). */
int tmpc_qp_batch(tmpc_ctx* ctx, int B, int N, double dt, int linsys, const double* rho, const double* x,
                  const double* u, const double* xs, const double* guess, double* dxul, int32_t* pcg_iters,
                  double* S_diag, double* S_lo, double* gamma, double* P_diag);

/* solveKKTSystem / solveKKTSystem_Schur (TrajoptMPCReference.py:313-455) on the blocks of formKKTSystemBlocks
 * (:118-271) as the caller's own plugin hooks formed them -- the QP of the drop-in's plugin-hook path, for
 * TrajoptCost / TrajoptPlant subclasses whose hooks have no device implementation.  n = nx + nu with
 * nx = 2 nu (1 <= nu <= 7), N nx <= 1024:
 *   G [B][N][n][n]   cost Hessian per knot, soft-limit outer products included, WITHOUT rho (knot N-1:
 *                    its nx x nx block in the top-left corner; the rest is ignored), x-u coupling allowed;
 *   g [B][N][n]      cost gradient (+ soft-limit jacobian) per knot (knot N-1: the first nx entries);
 *   A [B][N-1][nx][nx], Bm [B][N-1][nx][nu]   integrator Jacobians (C rows [-A_k -B_k I]);
 *   c [B][N][nx]     c_0 = x_0 - xs, c_{k+1} = x_{k+1} - f(x_k, u_k);
 *   rho [B]          the regularisation added to G in place (:419-420);
 *   linsys           TMPC_LINSYS_N / _S (direct) or _PCG_J / _BJ / _SS / _0;
 *   guess [B][N nx]  PCG initial iterate (nullable: zeros).
 * Outputs dxul [B][n(N-1)+nx + nx N] ([x0,u0,...,x_{N-1}; lambda], the reference's order), pcg_iters [B]
 * (0 for the direct methods), S_diag / S_lo / gamma (nullable).  (G_k + rho I)^-1 is formed by Gauss-Jordan
 * with partial pivoting (np.linalg.inv's LU pivots the same way; an indefinite plugin Hessian is fine): a zero or
 * non-finite pivot -- G_k + rho I exactly singular, np.linalg.inv's LinAlgError -- is an error. */
int tmpc_qp_blocks_batch(tmpc_ctx* ctx, int B, int N, int nx, int nu, int linsys, const double* G, const double* g,
                         const double* A, const double* Bm, const double* c, const double* rho, const double* guess,
                         double* dxul, int32_t* pcg_iters, double* S_diag, double* S_lo, double* gamma);

/* The plugin-hook QP on the banded path (ABI 10): solveKKTSystem / solveKKTSystem_Schur
 * (TrajoptMPCReference.py:313-455) on the caller's formKKTSystemBlocks blocks (:200-271) WITH hard rows
 * (ACTIVE_SET / FULL_SET, :238-248) and / or past tmpc_qp_blocks_batch's 1024 rows.  G, g, A, Bm, c, rho as
 * tmpc_qp_blocks_batch; the hard rows of each knot in the reference's order, from the caller's constraint
 * hooks (value_hard_constraints / jacobian_hard_constraints): hcnt [B][N] rows per knot, hcol [B][N][rmax]
 * the row's column in [x_k; u_k], hsgn [B][N][rmax] its jacobian entry (+1 / -1, or 0 for a FULL_SET row that
 * is not violated), hval [B][N][rmax] its value; every row a box row (one entry of [x_k; u_k]), which is what
 * the reference's BoxConstraint produces.  Outputs: dxul [B][n(N-1)+nx + nx N] (the lambda part: the N nx
 * dynamics / initial-state rows' multipliers in knot order), pcg_iters [B], lambda_hard [B][N][rmax] the hard
 * rows' multipliers, singular [B] (the direct methods' least-squares flag); all nullable.  The banded kernels of
 * the device path (k_hard_schur / k_hard_pcg / k_hard_direct / k_hard_dxu) with the caller's full
 * (G_k + rho I)^-1 blocks (partial-pivoting Gauss-Jordan) and gradient; summation order oracle/hard.py. */
int tmpc_qp_blocks_banded_batch(tmpc_ctx* ctx, int B, int N, int nx, int nu, int linsys, const double* G,
                                const double* g, const double* A, const double* Bm, const double* c,
                                const int32_t* hcnt, const int32_t* hcol, const double* hsgn, const double* hval,
                                int rmax, const double* rho, double* dxul, int32_t* pcg_iters, double* lambda_hard,
                                int32_t* singular);

/* Hard-limit detail of the last tmpc_qp_batch call with hard box limits, or of the last
 * tmpc_qp_blocks_banded_batch call (same B, N; there the bits and slots are t * 2 nu + e over the given
 * rows' columns, 6 n slots of the context's model): sizes[2] = {dmax, W} of
 * the banded Schur complement (rows padded to dmax, half band W), dim [B] its dimension per problem
 * (N nx + hard rows), active [B][N] the per-knot active-set bitmasks (as tmpc_trace.hard_active),
 * lambda_hard [B][N][6 n] the hard rows' multipliers by slot t * 2n + e (0 where no row), S_band
 * [B][dmax][2W+1] (row a, column a - W + o at offset o) and gamma [B][dmax] in the reference's row order
 * R_0 | R_1 H_0 | ... | R_{N-1} H_{N-2} H_{N-1}, singular [B] (the direct solve's least-squares flag).
 * Every output is nullable. */
int tmpc_qp_hard_info(tmpc_ctx* ctx, int B, int N, int32_t* sizes, int32_t* dim, uint64_t* active,
                      double* lambda_hard, double* S_band, double* gamma, int32_t* singular);

/* The hard-limit QP's PCG (GBD-PCG-Python/PCG.py:66-212 on the banded S of dimension dim[b], nx-aligned
 * preconditioner blocks from row 0, n_blocks = floor(dim / nx), PCG.py:182) on given systems: S_band
 * [B][dmax][2W+1], gamma [B][dmax] -> lambda [B][dmax], iters [B].  precond: TMPC_PRECOND_*.  Summation
 * order: the canonical one of oracle/hard.py pcg_canonical (bitwise reproducible on the CPU). */
int tmpc_hard_pcg_batch(tmpc_ctx* ctx, int B, int nx, int dmax, int W, const int32_t* dim, int precond,
                        const double* S_band, const double* gamma, double tol, int max_iter, double* lambda,
                        int32_t* iters);

/* PCG(S, gamma, nx, N, options={'preconditioner_type': J|BJ|SS, exit_tolerance, max_iter}).solve()
 * (GBD-PCG-Python/PCG.py:66-111) on B block-tridiagonal systems given by their blocks:
 * S_diag [B][N][nx][nx], S_lo [B][N-1][nx][nx] = S_{k+1,k}, S_up [B][N-1][nx][nx] = S_{k,k+1}
 * (nullable: S_lo^T is used), gamma [B][N nx], guess [B][N nx] (initial iterate, nullable = zeros,
 * PCG.py:11-12,33-34).  Outputs lambda [B][N nx], iters [B],
 * trace_nu / trace_res [B][max_iter+1] (|nu| and ||b - A x|| per iteration, nullable; entries past
 * iters[b] are left untouched), P_diag [B][N][nx][nx] (the inverted diagonal blocks, nullable). */
int tmpc_pcg_batch(tmpc_ctx* ctx, int B, int N, int nx, int precond, const double* S_diag, const double* S_lo,
                   const double* S_up, const double* gamma, const double* guess, double tol, int max_iter,
                   double* lambda, int32_t* iters, double* trace_nu, double* trace_res, double* P_diag);

/* PCG.pcg(A, b, Pinv, guess, options) (GBD-PCG-Python/PCG.py:66-111) on B dense systems with ANY
 * preconditioner matrix: A [B][D][D], b [B][D], Pinv [B][D][D] (row-major; replaces the reference's
 * dense Pinv argument).  Pinv = NULL: PCG.solve's own preconditioner (compute_preconditioner,
 * PCG.py:113-212) is built on the device from A -- precond TMPC_PRECOND_* with block size nx (1..16;
 * the floor(D / nx) nx-aligned blocks from row 0, rows past the last full block unpreconditioned).
 * guess [B][D] the initial iterate (nullable = zeros).  Outputs: x [B][D], iters [B], trace_nu /
 * trace_res [B][max_iter+1] (|nu| and ||b - A x|| per iteration as PCG.py:82-95, nullable: without
 * trace_res the explicit residual's extra product is skipped), Pinv_out [B][D][D] (nullable: the
 * preconditioner matrix the solve used).  Any D >= 1 (B D^2 <= 2^34 entries, i.e. the device memory of
 * three B x D x D matrices): no block-tridiagonal structure is assumed, the arbitrary-Pinv and the
 * past-1024-row forms of the reference's PCG class.  Up to 4096 rows one workgroup per system holds the
 * vectors (registers + LDS); past that each iteration's products and updates are separate launches with
 * the vectors in HBM (host-synchronous every 4 iterations), the same operation order.  Summation order:
 * oracle/dense.py (bitwise reproducible on the CPU). */
int tmpc_pcg_dense_batch(tmpc_ctx* ctx, int B, int D, const double* A, const double* b, const double* Pinv,
                         int precond, int nx, const double* guess, double tol, int max_iter, double* x,
                         int32_t* iters, double* trace_nu, double* trace_res, double* Pinv_out);

/* ---- device memory / timing helpers (the bench keeps inputs resident in HBM) ---- */
int tmpc_device_alloc(tmpc_ctx* ctx, size_t bytes, void** ptr);
int tmpc_device_free(tmpc_ctx* ctx, void* ptr);
int tmpc_memcpy_h2d(tmpc_ctx* ctx, void* dst, const void* src, size_t bytes);
int tmpc_memcpy_d2h(tmpc_ctx* ctx, void* dst, const void* src, size_t bytes);
int tmpc_memcpy_d2d(tmpc_ctx* ctx, void* dst, const void* src, size_t bytes);
int tmpc_synchronize(tmpc_ctx* ctx);

/* Kernel timing collected with HIP events on the context stream when options.profile = 1.
 * name: "qp_fd", "qp_minv", "qp_grad", "ginv", "qp" (the fused Schur + PCG + dxu kernel), "schur",
 * "btsolve", "dxu", "ls_terms", "ls_decide", "hard_schur", "hard_pcg" (also tmpc_hard_pcg_batch),
 * "hard_direct", "ilqr_backward", "ilqr_forward", "ilqr_decide", "mpc_shift", "pcg" (tmpc_pcg_batch),
 * "pcg_dense" (tmpc_pcg_dense_batch: transposes, preconditioner build and PCG). */
int tmpc_kernel_stats(tmpc_ctx* ctx, const char* name, int64_t* launches, double* total_ms);
/* Bytes a counting kernel reads and writes beyond its registers and LDS (its algorithmic memory traffic,
 * served by L2 / Infinity Cache / HBM), summed over its launches since the last
 * tmpc_reset_stats (any options.profile): "hard_pcg" (the hard-limit PCG of tmpc_sqp_solve_batch* /
 * tmpc_qp_batch: per launch and problem 8 B x (2 D + iterations x band entries + (iterations + 1) x
 * distinct preconditioner entries + setup blocks)).  Other names fail. */
int tmpc_kernel_bytes(tmpc_ctx* ctx, const char* name, double* bytes);
int tmpc_reset_stats(tmpc_ctx* ctx);

/* Work counters of the last solve call on this context: [0] problem-QPs solved (iLQR: problem-
 * iterations), [1] total PCG iterations, [2] QPs that recomputed the dynamics gradient, [3] line-search
 * trials per QP.  After tmpc_mpc_batch[_device], [0..2] are summed over all its horizon solves. */
int tmpc_solve_counters(tmpc_ctx* ctx, int64_t* counters);

/* ---- multi-GPU: one process per GPU, RCCL over xGMI ----
 * The reference has no distributed path (independent problems in a multiprocessing.Pool,
 * examples/test_multiple.py:123-128).  Problems shard by contiguous batch slices with no exchange
 * inside a solve; the communicator carries the initial states broadcast from rank 0 and the
 * per-problem summaries gathered back.  Rank 0 calls tmpc_comm_get_unique_id and shares the id
 * out of band before every rank calls tmpc_comm_create: trajoptmpcreference_amd/dist.py serves it over
 * TCP at MASTER_ADDR : MASTER_PORT + 1 together with a hash of each rank's run configuration (rank 0
 * answers every rank only after reading all requests: the id to all, or a refusal to all), or through a
 * launcher-provided file (TMPC_COMM_ID_FILE).  Buffers are device memory; every call is synchronous on
 * the ctx stream. */
#define TMPC_COMM_ID_BYTES 128
typedef struct tmpc_comm tmpc_comm;
int tmpc_comm_get_unique_id(uint8_t* id /* [TMPC_COMM_ID_BYTES] */);
int tmpc_comm_create(tmpc_ctx* ctx, int nranks, int rank, const uint8_t* id, tmpc_comm** out);
void tmpc_comm_destroy(tmpc_comm* comm);
int tmpc_comm_size(const tmpc_comm* comm, int* nranks, int* rank);
int tmpc_comm_broadcast(tmpc_comm* comm, void* d_buf, size_t bytes, int root);      /* in place */
int tmpc_comm_allgather(tmpc_comm* comm, const void* d_send, void* d_recv, size_t bytes_per_rank);
int tmpc_comm_allreduce_max_f64(tmpc_comm* comm, double* d_buf, size_t count);     /* in place */
int tmpc_comm_barrier(tmpc_comm* comm);

#ifdef __cplusplus
}
#endif
#endif /* TMPC_H */
