// Internal declarations shared by the kernels (tmpc_kernels.hip) and the
// C-ABI / solver driver (tmpc_api.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "tmpc_device.h"
#include "tmpc_models.h"

struct tmpc_ctx;

namespace tmpc {

// context accessors for the other translation units (tmpc_comm.cpp)
int ctx_fail(tmpc_ctx* ctx, const char* fmt, ...);
int ctx_device(const tmpc_ctx* ctx);
hipStream_t ctx_stream(const tmpc_ctx* ctx);

// The problems a batch-iteration launch visits: launches over B problems take (PList, nb) and visit
// problems P.at(p) for p < nb (and p < *P.cnt).  idx null: the identity, nb = B.  Otherwise idx is the
// ascending list of the problems still alive in the lock-step loop (k_alive_list, rebuilt at the end of
// every batch iteration on the stream, so exact when a launch reads it) and nb the host's upper bound
// of its length (the count of two iterations before: aliveness only ever ends).  Every kernel still
// tests its own per-problem mask (active / need_grad / ...): the list only drops the problems that can
// no longer be active, so the lock-step tail stops dispatching thousands of early-exit workgroups.
struct PList {
  const int* idx;
  const int* cnt;
  __device__ __forceinline__ int at(int p) const { return idx ? idx[p] : p; }
  __device__ __forceinline__ bool has(int p, int nb) const { return p < nb && (!cnt || p < *cnt); }
};
void launch_alive_list(hipStream_t s, int B, const int* alive, int* idx, int* cnt, int* host_slot);

// PRECOND_NONE: the identity preconditioner '0' (PCG.py:114-118)
enum { PRECOND_J = 1, PRECOND_BJ = 2, PRECOND_SS = 3, PRECOND_NONE = 4 };
enum { LS_MODE_INIT = 0, LS_MODE_STEP = 1 };
enum { QP_MODE_PCG = 0, QP_MODE_SCHUR = 1, QP_MODE_DXU = 2 };

// set_default_options (TrajoptMPCReference.py:91-115) + the fixed merit
// weight mu = 10 (:545-546)
struct SolverOpts {
  double exit_tol_sqp;
  double alpha_factor;
  double alpha_min;
  double rho_factor;
  double rho_min;
  double rho_max;
  double rho_init;
  double exp_red_min;
  double exp_red_max;
  double mu;
  int max_iter_sqp;
  int pad;
};

// per-problem solver state (device arrays, SoA)
struct ProbState {
  double* rho;
  double* drho;
  double* J;
  double* c;
  double* merit;
  int* iter;
  int* active;
  int* need_grad;
  int* exit_sqp;
};

// per-problem trace rows [B][max_iter_sqp + 1] (self.trace, :555-569, :691-743)
struct TraceDev {
  int* iteration;
  int* ls_iter;
  double* alpha;
  double* rho;
  double* J;
  double* c;
  double* merit;
  double* D;
  double* ratio;
  int* accepted;
  int* pcg_iters;
  int* singular;                  // the QP took the least-squares answer (reference: self.singular)
  unsigned long long* hard_active;   // [B][W][N] per-knot active-set bitmasks of the QP (nullable)
};

// f32: rigid-body dynamics (and, for launch_ilqr_backward, the Riccati sweep) in fp32 --
// tmpc_options.precision F32 / MIXED; every buffer stays fp64
int launch_qp_fd(bool f32, hipStream_t s, int nj, bool chain, int mid, const ModelDev* M, PList P, int B, int N, double dt, const double* x,
                 const double* u, const double* xs, const int* need, double* qdd, double* cvec);
int launch_qp_minv(bool f32, hipStream_t s, int nj, bool chain, int mid, const ModelDev* M, PList P, int B, int N, const double* x,
                   const int* need, double* minv);
int launch_qp_grad(bool f32, hipStream_t s, int nj, bool chain, int mid, const ModelDev* M, PList P, int B, int N, double dt, const double* x,
                   const int* need, const double* qdd, const double* minv, double* A, double* Bm);
int launch_ls_terms(bool f32, hipStream_t s, int nj, bool chain, int mid, const ModelDev* M, const CostDev* C, const ConstrDev* Cs,
                    const double* mu, const double* lam, PList P, int B, int N, int T, double dt, const double* alphas,
                    const double* x, const double* u, const double* xs, const double* dx, const double* du,
                    const int* active, double* terms);
int launch_unit_fd(bool f32, hipStream_t s, int nj, bool chain, int mid, const ModelDev* M, int K, double dt, const double* x,
                   const double* u, double* xnext, double* qdd);
int launch_unit_minv(bool f32, hipStream_t s, int nj, bool chain, int mid, const ModelDev* M, int K, const double* x, double* minv);
int launch_unit_grad(bool f32, hipStream_t s, int nj, bool chain, int mid, const ModelDev* M, int K, double dt, const double* x,
                     const double* qdd, const double* minv, double* A, double* Bm, double* dqdd);
// P / mask: the problems to roll out (the identity and every problem by default; the stream's refilled
// slots: the alive list and act_init)
int launch_rollout(bool f32, hipStream_t s, int nj, bool chain, int mid, const ModelDev* M, int B, int N, double dt, double* x,
                   const double* u, PList P = PList{nullptr, nullptr}, const int* mask = nullptr);
int launch_ginv(hipStream_t s, int nj, const CostDev* C, PList P, int B, const double* rho, const int* active, double* G);
// dt: the Euler step of A_k / B_k (their structural rows are not read, tmpc_kernels.hip qp_schur_row)
int launch_qp(hipStream_t s, int nj, const CostDev* C, PList P, int B, int N, double dt, int precond, int mode,
              const double* x, const double* u,
              const int* active, const double* G, const double* A, const double* Bm, const double* cvec, double tol,
              int max_iter, int* iters, double* dx, double* du, double* lam, double* Sd, double* Sl, double* gam,
              double* Pd, const double* jsoft, const double* guess, double* Sg);
// largest Schur dimension N nx of the fused QP: up to 1024 rows S / P^-1 stay in registers, up to
// QP_MAX_ROWS (the GM kernels: two rows per lane, 12 waves = 3 per SIMD, i.e. 168 VGPRs) in HBM
// scratch Sg of qp_gm_doubles(B, N, nx) doubles.  1536 = arm6 at N = 128 (BASELINE config 5).
constexpr int QP_MAX_ROWS = 1536;
inline size_t qp_gm_doubles(int B, int N, int nx) { return (size_t)B * 4 * nx * (size_t)N * nx; }
// rows from which the QP takes the GM kernel: 1025, or TMPC_QP_GM_MIN_ROWS (parity tests run the GM
// kernel on the reference's N = 64 fixtures this way)
inline int qp_gm_min_rows() {
  const char* e = getenv("TMPC_QP_GM_MIN_ROWS");
  const int v = e ? atoi(e) : 0;
  return v > 0 ? v : 1025;
}
int launch_ginv_soft(hipStream_t s, int nj, const CostDev* C, const ConstrDev* Cs, PList P, int B, int N, const double* rho,
                     const int* active, const double* x, const double* u, const double* mu, const double* lam,
                     double* Gk, double* jsoft);
int launch_pcg(hipStream_t s, int nx, int B, int N, int precond, const double* Sd, const double* Sl,
               const double* Su, const double* gam, const double* guess, double tol, int max_iter, double* lam,
               int* iters, double* tnu, double* tres, double* Pd);
// plugin-hook QP on caller-formed blocks (tmpc_hooks.hip)
int launch_ghat_full(hipStream_t s, int nj, int B, int N, const double* G, const double* rho, double* Gh, int* err);
int launch_qp_blocks(hipStream_t s, int nj, int B, int N, int precond, int mode, const double* Gh, const double* g,
                     const double* A, const double* Bm, const double* c, const int* err, double tol, int max_iter,
                     const double* guess, int* iters, double* dx, double* du, double* lam, double* Sd, double* Sl,
                     double* gam);
int qp_blocks_set_max_lds();
int launch_btsolve(hipStream_t s, int nx, int B, int N, const int* active, const double* Sd, const double* Sl,
                   const double* gam, double* U, double* Y, double* lam);
int pcg_set_max_lds();
void launch_sum_counters(hipStream_t s, int B, const unsigned long long* pc, unsigned long long* out);
// Continuous batching (tmpc_sqp_solve_stream_device / tmpc_ilqr_solve_stream_device): B resident slots
// work through a stream of P problems.  The workgroup of k_soft_outer that ends a problem's outer loop
// (outer_active 1 -> 0) writes the problem's results to its output rows and, when a problem is pending
// (one atomic on `next`; which slot gets which problem changes no problem's results), loads the next
// one's inputs with the state a fresh solve starts from -- act_init, so its initial merit / cost is
// evaluated in the same batch iteration.  Each problem's own operation sequence is the one of a batch
// solve, so its results are bitwise those of tmpc_*_solve_batch.
struct StreamDev {
  int P, period, NX, NU, N, W, MC;   // problems, input period, sizes, trace rows, soft slots per knot (6 n)
  int pbase;                         // global index of this (sub-)stream's problem 0 (inputs and output rows)
  const double* x_in;                // [period][NX][N]: problem p starts from input (pbase + p) % period
  const double* u_in;                // [period][NU][N-1]
  double* x_out;                     // [pbase + P][NX][N] (nullable): problem p's row is pbase + p
  double* u_out;                     // [pbase + P][NU][N-1] (nullable)
  int* status;                       // [pbase + P][4]: exit code, iterations, exit_soft, outer_iter (nullable)
  TraceDev tr_out;                   // [pbase + P][W] per field (each nullable; hard_active unused)
  int* slot_pid;                     // [B] problem in the slot (-1: none)
  int* next;                         // [1] next pending problem
};
void launch_stream_init(hipStream_t s, int B, const StreamDev& sd, double* x, double* u);

void launch_ls_decide(hipStream_t s, PList P, int B, int N, int NX, int NU, int T, int mode, int soft, const double* alphas,
                      const SolverOpts& o, const double* terms, double* x, double* u, const double* dx,
                      const double* du, const ProbState& st, const int* pcg_iters, const TraceDev& tr,
                      int* active_count, unsigned long long* counters, const double* hterms,
                      const int* qp_singular = nullptr, int* activate = nullptr);   // activate: as launch_ilqr_decide
void launch_init_state(hipStream_t s, int B, double rho_init, const ProbState& st, const int* outer_active);
// st / act_init / rho_init: the per-problem outer loop (null act_init: lock-step, tmpc_kernels.hip);
// sd / xs / tr / lam_warm: a stream's hand-over of finished slots (nullable; per-problem mode only)
void launch_soft_outer(hipStream_t s, const ConstrDev* Cs, PList P, int B, int N, int nj, double tol, int max_iter,
                       double* x, double* u, double* mu, double* lam, double* phi, int* outer_active,
                       int* outer_iter, int* exit_soft, int* outer_count, const ProbState* st = nullptr,
                       int* act_init = nullptr, double rho_init = 0.0, const StreamDev* sd = nullptr,
                       double* xs = nullptr, const TraceDev* tr = nullptr, double* lam_warm = nullptr);


int launch_ilqr_backward(bool f32, hipStream_t s, int nj, const CostDev* C, const ConstrDev* Cs, PList P, int B, int N, const double* x,
                         const double* u, const double* rho, const int* active, const double* A, const double* Bm,
                         const double* mu, const double* lam, double* jscratch, double* K, double* d, double* dV,
                         int* ok);
int launch_ilqr_forward(bool f32, hipStream_t s, int nj, bool chain, int mid, const ModelDev* M, const CostDev* C, const ConstrDev* Cs,
                        const double* mu, const double* lam, PList P, int B, int N, int T, double dt, int init,
                        const double* alphas, const double* x, const double* u, const double* K, const double* d,
                        const int* active, const int* ok, double* xt, double* ut, double* Jt);
int launch_ilqr_init_cost(hipStream_t s, int nj, const CostDev* C, const ConstrDev* Cs, const double* mu,
                          const double* lam, PList P, int B, int N, const double* x, const double* u, const int* mask,
                          double* Jt);
// counters: per-problem tallies [B][3] (problem-iterations, -, fresh gradients), summed by
// launch_sum_counters; activate (init only, nullable): the real active flags -- st.active is then the
// act_init mask, cleared as the problem enters its inner loop
void launch_ilqr_decide(hipStream_t s, PList P, int B, int N, int NX, int NU, int T, int init, const double* alphas,
                        const SolverOpts& o, const double* Jt, const double* dV, const int* ok, const double* xt,
                        const double* ut, double* x, double* u, const ProbState& st, const TraceDev& tr,
                        int* active_count, unsigned long long* counters, int* activate = nullptr);
int launch_mpc_shift(hipStream_t s, int nj, bool chain, int mid, const ModelDev* M, int B, int N, double dt, int step,
                     int steps, double* x, double* u, double* xe, double* ue);
void launch_soft_shift(hipStream_t s, const ConstrDev* Cs, int B, int N, int nj, double* mu, double* lam,
                       double* phi);
void launch_outer_init(hipStream_t s, int B, int* outer_active, int* outer_iter, int* exit_soft);
void launch_soft_init(hipStream_t s, const ConstrDev* Cs, size_t total, int MC, double* mu, double* lam,
                      double* phi);

// Hard box constraints (tmpc_hard.hip): one argument block for its four launch phases
// (0 rows + layout + Schur band, 1 PCG / direct solve, 2 dxu, 3 line-search terms).
struct HardArgs {
  int B, N, T, phase, precond, rmax, dmax, W, per_knot, max_iter;
  double tol;
  const ConstrDev* Cs;
  const CostDev* C;
  const double *x, *u, *Ghat, *A, *Bm, *cvec, *jsoft, *alphas;
  const int* active;
  int *cnt, *hcol, *roff, *hoff, *dim, *rkind, *rknot, *ridx, *PK, *iters;
  double *hsgn, *hval, *Y, *Sb, *gam, *Pd, *Pl, *Ptr, *M, *rhs, *lam, *dx, *du, *hterms;
  int* hslot;                     // [B][N][rmax] t * 2n + e of each row
  unsigned long long* amask;      // [B][N] active-set bitmask per knot (bit t * 2n + e)
  int* sing;                      // [B] the direct solve took the least-squares answer (singular S)
  int* rng;                       // [B][dmax][2] first / last structurally nonzero column of each row of S
  const int* iter;                // per-problem SQP iteration (trace row iter + 1)
  int Wtr;                        // trace row stride (max_iter_SQP_DDP + 1)
  unsigned long long* tr_active;  // [B][Wtr][N] trace copy of amask (nullable)
  double* work;                   // [B] algorithmic HBM bytes of k_hard_pcg, accumulated per problem (nullable)
  // the plugin-hook QP (tmpc_qp_blocks_banded_batch): per_knot = 2 -- Ghat holds full (G_k + rho I)^-1 blocks
  // [B][N][nx+nu][nx+nu] -- the caller's cost gradient gvec [B][N][nx+nu] (null: the context's cost), and
  // rows_given: cnt / hcol / hsgn / hval were filled from the caller's constraint hooks (k_hard_rows skipped)
  const double* gvec;
  int rows_given;
};
// k_hard_pcg: 1024 threads per problem, row a on thread a % 1024 (row slot a / 1024, at most 4 slots)
constexpr int HARD_PCG_THREADS = 1024, HARD_PCG_MAX_SLOTS = 4;
constexpr int HARD_PCG_MAX_ROWS = HARD_PCG_THREADS * HARD_PCG_MAX_SLOTS;
constexpr int HARD_PCG_LDS_BYTES = 160 * 1024;   // all of a CU's LDS: vectors + preconditioner-block cache
int launch_hard(hipStream_t s, int nj, const HardArgs& h);
// dynamic LDS of k_hard_schur (one workgroup per problem): the cost gradient / piece record per knot
// (3 nj doubles + 2 ints), the rows' piece knots (2 dmax ints, 16-byte rounded) and the shared Ghat
// blocks (2 (2 nj)^2 + nj^2 doubles).  It grows with N: setup_hard refuses a horizon past the CU's LDS.
inline size_t hard_schur_lds_bytes(int N, int nj, int dmax) {
  return (size_t)N * (3 * nj * sizeof(double) + 2 * sizeof(int)) + (size_t)((dmax * 2 + 3) & ~3) * sizeof(int) +
         (size_t)(2 * 4 * nj * nj + nj * nj) * sizeof(double);
}
constexpr size_t CU_LDS_BYTES = 160 * 1024;   // gfx950: 160 KB of LDS per CU
int hard_set_max_lds();

// the dense PCG of tmpc_pcg_dense_batch (tmpc_hard.hip): PCG.pcg with any A / Pinv, D <= HARD_PCG_MAX_ROWS.
// A row-major [B][D][D] (the preconditioner builders read it), AT / PT column-major (A^T, Pinv^T: the PCG
// reads columns), Pd [B][D / nx][nx][nx] the builders' diagonal blocks
struct DenseArgs {
  int B, D, nx, precond, max_iter;
  double tol;
  const double *A, *b, *guess;
  double *AT, *PT, *Pd, *x, *trace_nu, *trace_res;
  int* iters;
  // past HARD_PCG_MAX_ROWS (launch_pcg_dense_big): the vectors in HBM scratch [B][D] and per-system state
  double *r, *p, *y, *q, *nu;
  int *done;
};
int launch_dense_transpose(hipStream_t s, int B, int D, const double* in, double* out);
int launch_dense_precond(hipStream_t s, const DenseArgs& a);
int launch_pcg_dense(hipStream_t s, const DenseArgs& a);
// the same PCG past HARD_PCG_MAX_ROWS rows: one launch per product / update phase, vectors in HBM, the same
// operation order (oracle/dense.py); host-synchronous every few iterations to stop once every system is done
int launch_pcg_dense_big(hipStream_t s, const DenseArgs& a);
int dense_set_max_lds();

}  // namespace tmpc
