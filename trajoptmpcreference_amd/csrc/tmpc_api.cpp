// C ABI (include/tmpc.h) and the batched SQP driver.
//
// The driver is the host half of TrajoptMPCReference.SQP
// (TrajoptMPCReference.py:510-760): it launches, per SQP iteration, the
// masked device phases QP-build (dynamics + gradients) -> Schur -> PCG ->
// dxu -> line-search terms -> decision, and stops when no problem of the
// batch is active.  All per-problem branching lives on the device
// (k_ls_decide); the host reads back one integer per iteration.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "../../include/tmpc.h"
#include "tmpc_internal.h"

using namespace tmpc;

namespace {

struct DevBuf {
  void* ptr = nullptr;
  size_t bytes = 0;
};

struct Stat {
  int64_t launches = 0;
  double total_ms = 0.0;
};

struct PendingTiming {
  std::string name;
  hipEvent_t start, stop;
};

}  // namespace

struct tmpc_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  bool has_model = false, has_cost = false;
  ModelDev hmodel{};
  CostDev hcost{};
  ConstrDev hlim{};
  ModelDev* dmodel = nullptr;
  CostDev* dcost = nullptr;
  ConstrDev* dlim = nullptr;
  int soft_B = -1, soft_N = -1;   // shape of the valid soft-constraint state (-1: none)
  int model_id = 0;               // compiled model (tmpc_models.h) equal to the set model; 0 = runtime model
  tmpc_options opts{};
  std::map<std::string, DevBuf> bufs;
  std::map<std::string, Stat> stats;
  std::vector<PendingTiming> pending;
  std::vector<hipEvent_t> event_pool;
  int* h_count = nullptr;  // pinned
  int64_t last_counters[4] = {0, 0, 0, 0};
  // shape of the last tmpc_qp_batch with hard box limits (tmpc_qp_hard_info); B = 0: none
  // the last tmpc_qp_batch with hard limits (tmpc_qp_hard_info reads its hd_* buffers); cleared by every
  // other user of those buffers (setup_hard) and by a change of the limits, so stale data is refused
  struct { int B, N, dmax, W, rmax; } hard_last{0, 0, 0, 0, 0};
  std::map<std::string, double> kbytes;   // bytes beyond registers / LDS of counting kernels since tmpc_reset_stats
  std::vector<tmpc_ctx*> subs;            // a stream's concurrent sub-streams (tmpc_stream.substreams): own HIP
                                          // stream and buffers each, the configuration copied from this context
};

static int fail(tmpc_ctx* c, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (c) c->err = buf;
  return -1;
}

namespace tmpc {
int ctx_fail(tmpc_ctx* ctx, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (ctx) ctx->err = buf;
  return -1;
}
int ctx_device(const tmpc_ctx* ctx) { return ctx->device; }
hipStream_t ctx_stream(const tmpc_ctx* ctx) { return ctx->stream; }
}  // namespace tmpc

#define HIP_OK(call)                                                                        \
  do {                                                                                      \
    hipError_t e_ = (call);                                                                 \
    if (e_ != hipSuccess) return fail(ctx, "%s failed: %s", #call, hipGetErrorString(e_)); \
  } while (0)

#define LAUNCH_OK(call)                                                                       \
  do {                                                                                        \
    int r_ = (call);                                                                          \
    if (r_ != 0) return fail(ctx, "unsupported size for %s (code %d)", #call, r_);           \
    hipError_t e_ = hipGetLastError();                                                        \
    if (e_ != hipSuccess) return fail(ctx, "launch %s failed: %s", #call, hipGetErrorString(e_)); \
  } while (0)

static hipEvent_t get_event(tmpc_ctx* ctx) {
  if (!ctx->event_pool.empty()) {
    hipEvent_t e = ctx->event_pool.back();
    ctx->event_pool.pop_back();
    return e;
  }
  hipEvent_t e;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

// RAII timing of one launch on the context stream (options.profile)
struct Timed {
  tmpc_ctx* ctx;
  PendingTiming pt;
  bool on;
  Timed(tmpc_ctx* c, const char* name) : ctx(c), on(c->opts.profile != 0) {
    if (!on) return;
    pt.name = name;
    pt.start = get_event(ctx);
    pt.stop = get_event(ctx);
    hipEventRecord(pt.start, ctx->stream);
  }
  ~Timed() {
    if (!on) return;
    hipEventRecord(pt.stop, ctx->stream);
    ctx->pending.push_back(pt);
  }
};

static void resolve_timings(tmpc_ctx* ctx) {
  for (auto& p : ctx->pending) {
    float ms = 0.f;
    if (hipEventSynchronize(p.stop) == hipSuccess && hipEventElapsedTime(&ms, p.start, p.stop) == hipSuccess) {
      Stat& s = ctx->stats[p.name];
      s.launches += 1;
      s.total_ms += ms;
    }
    ctx->event_pool.push_back(p.start);
    ctx->event_pool.push_back(p.stop);
  }
  ctx->pending.clear();
}

template <typename T>
static T* buf(tmpc_ctx* ctx, const char* name, size_t count) {
  DevBuf& b = ctx->bufs[name];
  const size_t bytes = count * sizeof(T);
  if (b.bytes < bytes) {
    if (b.ptr) hipFree(b.ptr);
    b.ptr = nullptr;
    b.bytes = 0;
    if (hipMalloc(&b.ptr, bytes) != hipSuccess) {
      b.ptr = nullptr;
      return nullptr;
    }
    b.bytes = bytes;
  }
  return static_cast<T*>(b.ptr);
}

#define BUF(T, name, count)                                                            \
  T* name = buf<T>(ctx, #name, (size_t)(count));                                       \
  if (!name) return fail(ctx, "device allocation of %s (%zu elements) failed", #name, \
                         (size_t)(count));

// precision modes (tmpc_options.precision): the dynamics' derivatives (M^-1, RNEA gradient: A_k, B_k) in
// fp32 for F32 and MIXED; the trajectory values (the QP's defects, line-search trials, iLQR rollouts) in
// fp32 for MIXED only -- F32 evaluates every trajectory, cost and merit in fp64, so its exit tests see the
// fp64 objective; the Riccati sweep in fp32 for F32 only; Schur / PCG, merit sums and decisions stay fp64
static bool dyn32(const tmpc_ctx* ctx) { return ctx->opts.precision != TMPC_PRECISION_F64; }
static bool val32(const tmpc_ctx* ctx) { return ctx->opts.precision == TMPC_PRECISION_MIXED; }
static bool ric32(const tmpc_ctx* ctx) { return ctx->opts.precision == TMPC_PRECISION_F32; }

static SolverOpts solver_opts(const tmpc_options& o) {
  SolverOpts s{};
  s.exit_tol_sqp = o.exit_tolerance_SQP_DDP;
  s.alpha_factor = o.alpha_factor_SQP_DDP;
  s.alpha_min = o.alpha_min_SQP_DDP;
  s.rho_factor = o.rho_factor_SQP_DDP;
  s.rho_min = o.rho_min_SQP_DDP;
  s.rho_max = o.rho_max_SQP_DDP;
  s.rho_init = o.rho_init_SQP_DDP;
  s.exp_red_min = o.expected_reduction_min_SQP_DDP;
  s.exp_red_max = o.expected_reduction_max_SQP_DDP;
  s.mu = o.merit_mu;
  s.max_iter_sqp = o.max_iter_SQP_DDP;
  return s;
}

// alpha schedule of the line search (:606, :712-718): 1, f, f^2, ... while alpha > alpha_min
static std::vector<double> alpha_list(const tmpc_options& o) {
  std::vector<double> a;
  double al = 1.0;
  a.push_back(al);
  while (al > o.alpha_min_SQP_DDP && a.size() < 64) {
    al *= o.alpha_factor_SQP_DDP;
    a.push_back(al);
  }
  return a;
}

// 0 = method S (direct block-tridiagonal solve, k_btsolve); method N (the dense KKT solve) has the
// same solution and takes the same direct path (include/tmpc.h)
static int precond_of(int linsys) {
  switch (linsys) {
    case TMPC_LINSYS_S: return 0;
    case TMPC_LINSYS_N: return 0;
    case TMPC_LINSYS_PCG_J: return PRECOND_J;
    case TMPC_LINSYS_PCG_BJ: return PRECOND_BJ;
    case TMPC_LINSYS_PCG_SS: return PRECOND_SS;
    case TMPC_LINSYS_PCG_0: return PRECOND_NONE;
    default: return -1;
  }
}

// A wide model (NJ_FULL < n <= NJMAX joints) runs the dynamics on the runtime model, the SQP with the fused
// register / two-rows-per-lane QP (N * nx <= 1024 rows) and iLQR with the VALU Riccati sweep and the plain
// rollout: fp64, QuadraticCost, no box limits (the MFMA sweep's tiles and the fp32 / soft / hard / HBM-row
// instances exist for up to NJ_FULL joints)
static int wide_ok(tmpc_ctx* ctx, const char* what) {
  const int n = ctx->hmodel.n;
  if (n <= NJ_FULL) return 0;
  if (ctx->opts.precision != TMPC_PRECISION_F64)
    return fail(ctx, "%s: %d joints run in fp64 only (precision modes up to %d joints)", what, n, NJ_FULL);
  return 0;
}

static int check_ready(tmpc_ctx* ctx, int B, int N, bool qp = true) {
  if (!ctx) return -1;
  if (!ctx->has_model) return fail(ctx, "no model: call tmpc_set_model first");
  if (ctx->hmodel.n > NJ_FULL) {
    const int n = ctx->hmodel.n;
    if (int rc = wide_ok(ctx, qp ? "SQP" : "iLQR")) return rc;
    if (ctx->hlim.any)
      return fail(ctx, "box constraints with %d joints: supported up to %d joints (the soft / hard limit kernels)", n,
                  NJ_FULL);
    if (ctx->has_cost && ctx->hcost.kind != COST_QUADRATIC) return fail(ctx, "%d joints: QuadraticCost only", n);
    if (qp && N * 2 * n > 1024)
      return fail(ctx, "%d joints: the QP takes N * nx <= 1024 rows (N <= %d; got N = %d)", n, 1024 / (2 * n), N);
  }
  if (!ctx->has_cost) return fail(ctx, "no cost: call tmpc_set_cost_quadratic first");
  if (ctx->hcost.nx != 2 * ctx->hmodel.n || ctx->hcost.nu != ctx->hmodel.n)
    return fail(ctx, "cost sizes (nx=%d, nu=%d) do not match the model (n=%d)", ctx->hcost.nx, ctx->hcost.nu,
                ctx->hmodel.n);
  if (B < 1) return fail(ctx, "batch size must be >= 1 (got %d)", B);
  if (N < 2) return fail(ctx, "N must be >= 2 (got %d)", N);
  (void)qp;   // QPs past the fused kernel's QP_MAX_ROWS take the banded path (qp_banded)
  return 0;
}

// The QP takes the banded variable-block path of tmpc_hard.hip -- built for hard box constraints --
// with hard limits, and also without them past the fused k_qp's QP_MAX_ROWS (1536) rows: there the
// Schur complement is the same block-tridiagonal S with no constraint rows (every knot's row count 0),
// which the banded kernels solve up to HARD_PCG_MAX_ROWS rows by PCG (and by the direct banded
// elimination up to k_hard_schur's LDS bound, checked in setup_hard), in their own canonical order
// (oracle/hard.py pcg_canonical).
static bool qp_banded(const tmpc_ctx* ctx, int N) {
  return ctx->hlim.any_hard || N * 2 * ctx->hmodel.n > QP_MAX_ROWS;
}

// ------------------------------------------------------------------ QP phase (shared by SQP and tmpc_qp_batch)
struct Work {
  double *xs, *qdd, *minv, *cvec, *A, *Bm, *G, *Sd, *Sl, *gam, *lam, *dx, *du, *Pd;
  int* iters;
  double *U, *Y;   // method S scratch (k_btsolve)
  double *Gk, *jsoft, *smu, *slam;   // soft limits: per-knot Ghat, jacobian, AL constants
  const double* guess;               // PCG initial iterate [B][N nx] (nullable)
  double* lam_keep;                  // where the PCG path stores lambda (nullable; warm start)
  HardArgs* hard;                    // hard box constraints: the variable-row QP (tmpc_hard.hip)
  double* Sg;                        // S / P^-1 rows in HBM past 1024 rows (k_qp<..., GM>), else null
  unsigned long long* tr_active;     // hard limits: per-QP active-set bitmasks into the trace (nullable)
  int Wtr;                           // trace row stride
};

// P / nb: the problems the batch launches visit (tmpc_internal.h PList; the identity and B outside the
// lock-step loop)
static int run_qp(tmpc_ctx* ctx, int B, int N, double dt, int precond, const double* d_x, const double* d_u,
                  const ProbState& st, Work& w, bool keep_blocks, PList P, int nb) {
  const int nj = ctx->hmodel.n;
  const bool chain = ctx->hmodel.chain != 0;
  const bool soft = w.jsoft != nullptr;
  const double* G = soft ? w.Gk : w.G;
  {
    Timed t(ctx, "qp_fd");
    LAUNCH_OK(launch_qp_fd(val32(ctx), ctx->stream, nj, chain, ctx->model_id, ctx->dmodel, P, nb, N, dt, d_x, d_u, w.xs, st.need_grad,
                           w.qdd, w.cvec));
  }
  {
    Timed t(ctx, "qp_minv");
    LAUNCH_OK(launch_qp_minv(dyn32(ctx), ctx->stream, nj, chain, ctx->model_id, ctx->dmodel, P, nb, N, d_x, st.need_grad,
                             w.minv));
  }
  {
    Timed t(ctx, "qp_grad");
    LAUNCH_OK(launch_qp_grad(dyn32(ctx), ctx->stream, nj, chain, ctx->model_id, ctx->dmodel, P, nb, N, dt, d_x, st.need_grad, w.qdd, w.minv,
                             w.A, w.Bm));
  }
  if (soft) {
    Timed t(ctx, "ginv");
    LAUNCH_OK(launch_ginv_soft(ctx->stream, nj, ctx->dcost, ctx->dlim, P, nb, N, st.rho, st.active, d_x, d_u, w.smu,
                               w.slam, w.Gk, w.jsoft));
  } else {
    Timed t(ctx, "ginv");
    LAUNCH_OK(launch_ginv(ctx->stream, nj, ctx->dcost, P, nb, st.rho, st.active, w.G));
  }
  if (w.hard) {   // hard box constraints: rows of C per knot, banded S (tmpc_hard.hip)
    HardArgs h = *w.hard;
    h.precond = precond;
    h.Ghat = G;
    h.per_knot = soft || ctx->hcost.kind == COST_EE;
    h.A = w.A;
    h.Bm = w.Bm;
    h.cvec = w.cvec;
    h.jsoft = w.jsoft;
    h.x = d_x;
    h.u = d_u;
    h.active = st.active;
    h.iters = w.iters;
    h.dx = w.dx;
    h.du = w.du;
    h.tol = ctx->opts.exit_tolerance_linSys;
    h.max_iter = ctx->opts.max_iter_linSys;
    h.iter = st.iter;
    h.Wtr = w.Wtr;
    h.tr_active = w.tr_active;
    HIP_OK(hipMemsetAsync(w.iters, 0, sizeof(int) * B, ctx->stream));
    const char* names[3] = {"hard_schur", precond == 0 ? "hard_direct" : "hard_pcg", "dxu"};
    for (int ph = 0; ph < 3; ++ph) {
      Timed t(ctx, names[ph]);
      h.phase = ph;
      LAUNCH_OK(launch_hard(ctx->stream, nj, h));
    }
    return 0;
  }
  if (precond == 0) {   // method S: Schur blocks -> direct solve -> dxu
    {
      Timed t(ctx, "schur");
      LAUNCH_OK(launch_qp(ctx->stream, nj, ctx->dcost, P, nb, N, dt, PRECOND_SS, QP_MODE_SCHUR, d_x, d_u, st.active, G,
                          w.A, w.Bm, w.cvec, 0.0, 0, w.iters, w.dx, w.du, nullptr, w.Sd, w.Sl, w.gam, nullptr,
                          w.jsoft, nullptr, nullptr));
    }
    {
      Timed t(ctx, "btsolve");
      LAUNCH_OK(launch_btsolve(ctx->stream, 2 * nj, B, N, st.active, w.Sd, w.Sl, w.gam, w.U, w.Y, w.lam));
    }
    {
      Timed t(ctx, "dxu");
      LAUNCH_OK(launch_qp(ctx->stream, nj, ctx->dcost, P, nb, N, dt, PRECOND_SS, QP_MODE_DXU, d_x, d_u, st.active, G, w.A,
                          w.Bm, w.cvec, 0.0, 0, w.iters, w.dx, w.du, w.lam, nullptr, nullptr, nullptr, nullptr,
                          w.jsoft, nullptr, nullptr));
    }
    return 0;
  }
  {
    Timed t(ctx, "qp");
    LAUNCH_OK(launch_qp(ctx->stream, nj, ctx->dcost, P, nb, N, dt, precond, QP_MODE_PCG, d_x, d_u, st.active, G, w.A,
                        w.Bm, w.cvec, ctx->opts.exit_tolerance_linSys, ctx->opts.max_iter_linSys, w.iters, w.dx,
                        w.du, keep_blocks ? w.lam : w.lam_keep, keep_blocks ? w.Sd : nullptr,
                        keep_blocks ? w.Sl : nullptr, keep_blocks ? w.gam : nullptr, keep_blocks ? w.Pd : nullptr,
                        w.jsoft, w.guess, w.Sg));
  }
  return 0;
}

static int alloc_work(tmpc_ctx* ctx, int B, int N, Work& w, bool with_blocks) {
  const int nj = ctx->hmodel.n, nx = 2 * nj, K = N - 1;
  BUF(double, xs, (size_t)B * nx);
  BUF(double, qdd, (size_t)B * K * nj);
  BUF(double, minv, (size_t)B * K * nj * nj);
  BUF(double, cvec, (size_t)B * N * nx);
  BUF(double, Amat, (size_t)B * K * nx * nx);
  BUF(double, Bmat, (size_t)B * K * nx * nj);
  BUF(double, Ginv, (size_t)B * 3 * nx * nx);
  BUF(double, dx, (size_t)B * N * nx);
  BUF(double, du, (size_t)B * K * nj);
  BUF(int, iters, (size_t)B);
  w = Work{xs, qdd, minv, cvec, Amat, Bmat, Ginv, nullptr, nullptr, nullptr, nullptr, dx, du, nullptr, iters,
           nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0};
  if (N * nx >= qp_gm_min_rows() && !qp_banded(ctx, N)) {   // the GM QP kernel's rows of S / P^-1
    BUF(double, qp_gm, qp_gm_doubles(B, N, nx));
    w.Sg = qp_gm;
  }
  if (with_blocks) {
    BUF(double, Sdiag, (size_t)B * N * nx * nx);
    BUF(double, Slo, (size_t)B * (K > 0 ? K : 1) * nx * nx);
    BUF(double, gam, (size_t)B * N * nx);
    BUF(double, lam, (size_t)B * N * nx);
    BUF(double, Pdiag, (size_t)B * N * nx * nx);
    w.Sd = Sdiag;
    w.Sl = Slo;
    w.gam = gam;
    w.lam = lam;
    w.Pd = Pdiag;
    BUF(double, btU, (size_t)B * (K > 0 ? K : 1) * nx * nx);
    BUF(double, btY, (size_t)B * N * nx);
    w.U = btU;
    w.Y = btY;
  }
  return 0;
}

static int alloc_state(tmpc_ctx* ctx, int B, ProbState& st) {
  BUF(double, st_rho, B);
  BUF(double, st_drho, B);
  BUF(double, st_J, B);
  BUF(double, st_c, B);
  BUF(double, st_merit, B);
  BUF(int, st_iter, B);
  BUF(int, st_active, B);
  BUF(int, st_need, B);
  BUF(int, st_exit, B);
  st = ProbState{st_rho, st_drho, st_J, st_c, st_merit, st_iter, st_active, st_need, st_exit};
  return 0;
}

static int alloc_trace(tmpc_ctx* ctx, int B, int W, TraceDev& tr) {
  BUF(int, tr_iteration, (size_t)B * W);
  BUF(int, tr_ls, (size_t)B * W);
  BUF(double, tr_alpha, (size_t)B * W);
  BUF(double, tr_rho, (size_t)B * W);
  BUF(double, tr_J, (size_t)B * W);
  BUF(double, tr_c, (size_t)B * W);
  BUF(double, tr_merit, (size_t)B * W);
  BUF(double, tr_D, (size_t)B * W);
  BUF(double, tr_ratio, (size_t)B * W);
  BUF(int, tr_acc, (size_t)B * W);
  BUF(int, tr_pcg, (size_t)B * W);
  BUF(int, tr_sing, (size_t)B * W);
  HIP_OK(hipMemsetAsync(tr_sing, 0, (size_t)B * W * sizeof(int), ctx->stream));   // iLQR never sets it
  tr = TraceDev{tr_iteration, tr_ls, tr_alpha, tr_rho, tr_J, tr_c, tr_merit, tr_D, tr_ratio, tr_acc, tr_pcg, tr_sing,
                nullptr};
  return 0;
}

// soft-constraint state [B][N][6n] (mu, lambda, phi) and the per-knot QP terms
static int alloc_soft(tmpc_ctx* ctx, int B, int N, double** mu, double** lam, double** phi) {
  const size_t n = (size_t)B * N * 6 * ctx->hmodel.n;
  BUF(double, soft_mu, n);
  BUF(double, soft_lam, n);
  BUF(double, soft_phi, n);
  *mu = soft_mu;
  *lam = soft_lam;
  *phi = soft_phi;
  return 0;
}

// Buffers of the hard-constraint QP (tmpc_hard.hip) for B problems of N knots; T line-search trials.
// nj_given / rmax_given >= 0: the plugin-hook QP's joint count and rows per knot (its rows come from the
// caller's constraint hooks, not from the context's limits)
static int setup_hard(tmpc_ctx* ctx, int B, int N, int T, int precond, HardArgs& hard, int nj_given = -1,
                      int rmax_given = -1) {
  const int nj = nj_given >= 0 ? nj_given : ctx->hmodel.n, nx = 2 * nj;
  // rows per knot, at most: FULL_SET both bounds of every entry; ACTIVE_SET one per entry when lb < ub
  // (z - lb < 0 and ub - z < 0 cannot hold together), else both
  int rmax = 0;
  bool full = false;
  for (int t = 0; t < 3 && rmax_given < 0; ++t) {
    if (ctx->hlim.hard[t] == HARD_NONE) continue;
    bool ordered = ctx->hlim.hard[t] == HARD_ACTIVE;
    for (int i = 0; i < nj; ++i) ordered = ordered && ctx->hlim.lb[t][i] < ctx->hlim.ub[t][i];
    rmax += ordered ? nj : 2 * nj;
    if (ctx->hlim.hard[t] == HARD_FULL) full = true;
  }
  if (rmax_given >= 0) rmax = rmax_given;
  if (full && precond != 0)
    return fail(ctx, "FULL_SET box constraints with a PCG method: the inactive rows of C are zero, so S is "
                "singular and the reference's preconditioner raises LinAlgError (PCG.py:168-188); use method S");
  ctx->hard_last = {0, 0, 0, 0, 0};           // the hd_* buffers are about to be reused: no stale QP info
  hard = HardArgs{};
  hard.B = B;
  hard.N = N;
  hard.rmax = rmax;
  hard.dmax = nx * N + N * hard.rmax;
  const int gmax = nx + 2 * hard.rmax;         // the last group holds two knots' hard rows
  hard.W = 2 * gmax - 1;
  if (precond != 0 && hard.dmax > HARD_PCG_MAX_ROWS)
    return fail(ctx, "%s: Schur dimension up to %d exceeds the banded PCG's %d rows (methods S / N go further)",
                ctx->hlim.any_hard || rmax_given > 0 ? "hard constraints" : "N * nx past the fused QP's rows",
                hard.dmax, HARD_PCG_MAX_ROWS);
  if (hard.W > 1024) return fail(ctx, "hard constraints: band half-width %d > 1024", hard.W);
  if (hard_schur_lds_bytes(N, nj, hard.dmax) > CU_LDS_BYTES) {
    // the largest N whose k_hard_schur LDS fits: N (24 nj + 8) + 8 (nx + rmax) N + 72 nj^2 (+ 12 of rounding)
    int nmax = N;
    while (nmax > 2 && hard_schur_lds_bytes(nmax, nj, nx * nmax + nmax * hard.rmax) > CU_LDS_BYTES) --nmax;
    return fail(ctx, "%s: N = %d needs %zu bytes of LDS in the banded Schur kernel (k_hard_schur), more than a "
                "CU's %zu; the largest supported horizon for this robot%s is N = %d",
                ctx->hlim.any_hard ? "hard constraints" : "N * nx past the fused QP's rows", N,
                hard_schur_lds_bytes(N, nj, hard.dmax), CU_LDS_BYTES,
                ctx->hlim.any_hard ? " and these limits" : "", nmax);
  }
  const size_t BW = 2 * (size_t)hard.W + 1, nbmax = hard.dmax / nx + 1;
  hard.Cs = ctx->dlim;
  hard.C = ctx->dcost;
  const int rbuf = hard.rmax > 0 ? hard.rmax : 1;   // no hard limits (the banded path past QP_MAX_ROWS): rmax = 0
  BUF(int, hd_cnt, (size_t)B * N);
  BUF(int, hd_col, (size_t)B * N * rbuf);
  BUF(double, hd_sgn, (size_t)B * N * rbuf);
  BUF(double, hd_val, (size_t)B * N * rbuf);
  BUF(int, hd_roff, (size_t)B * N);
  BUF(int, hd_hoff, (size_t)B * N);
  BUF(int, hd_dim, (size_t)B);
  BUF(int, hd_rkind, (size_t)B * hard.dmax);
  BUF(int, hd_rknot, (size_t)B * hard.dmax);
  BUF(int, hd_ridx, (size_t)B * hard.dmax);
  BUF(int, hd_pk, (size_t)B * hard.dmax * 2);
  BUF(int, hd_slot, (size_t)B * N * rbuf);
  BUF(unsigned long long, hd_amask, (size_t)B * N);
  BUF(int, hd_sing, (size_t)B);
  HIP_OK(hipMemsetAsync(hd_sing, 0, (size_t)B * sizeof(int), ctx->stream));
  hard.hslot = hd_slot; hard.amask = hd_amask; hard.sing = hd_sing;
  BUF(int, hd_rng, (size_t)B * hard.dmax * 2);
  hard.rng = hd_rng;
  BUF(double, hd_Y, (size_t)B * hard.dmax * 2 * (nx + nj));
  BUF(double, hd_Sb, (size_t)B * hard.dmax * BW);
  BUF(double, hd_gam, (size_t)B * hard.dmax);
  BUF(double, hd_lam, (size_t)B * hard.dmax);
  hard.cnt = hd_cnt; hard.hcol = hd_col; hard.hsgn = hd_sgn; hard.hval = hd_val;
  hard.roff = hd_roff; hard.hoff = hd_hoff; hard.dim = hd_dim;
  hard.rkind = hd_rkind; hard.rknot = hd_rknot; hard.ridx = hd_ridx; hard.PK = hd_pk;
  hard.Y = hd_Y; hard.Sb = hd_Sb; hard.gam = hd_gam; hard.lam = hd_lam;
  if (precond == 0) {
    BUF(double, hd_M, (size_t)B * hard.dmax * BW);
    BUF(double, hd_rhs, (size_t)B * hard.dmax);
    hard.M = hd_M;
    hard.rhs = hd_rhs;
  } else {
    BUF(double, hd_Pd, (size_t)B * nbmax * nx * nx);
    BUF(double, hd_Pl, (size_t)B * nbmax * nx * nx);
    BUF(double, hd_Ptr, (size_t)B * nbmax * nx * nx);
    hard.Pd = hd_Pd; hard.Pl = hd_Pl; hard.Ptr = hd_Ptr;
  }
  BUF(double, hd_terms, (size_t)B * (T > 0 ? T : 1) * N);
  hard.hterms = hd_terms;
  if (precond != 0) {
    BUF(double, hd_work, (size_t)B);
    HIP_OK(hipMemsetAsync(hd_work, 0, (size_t)B * sizeof(double), ctx->stream));
    hard.work = hd_work;
  }
  return 0;
}

// add the per-problem algorithmic bytes k_hard_pcg counted in this solve to ctx->kbytes["hard_pcg"]
static int collect_hard_work(tmpc_ctx* ctx, const HardArgs& hard) {
  if (!hard.work) return 0;
  std::vector<double> w(hard.B);
  HIP_OK(hipMemcpyAsync(w.data(), hard.work, sizeof(double) * hard.B, hipMemcpyDeviceToHost, ctx->stream));
  HIP_OK(hipStreamSynchronize(ctx->stream));
  double sum = 0.0;
  for (double v : w) sum += v;
  ctx->kbytes["hard_pcg"] += sum;
  return 0;
}

// the hard box-constraint terms of the merit's violation at the line-search trial points
static int hard_ls(tmpc_ctx* ctx, int nj, const HardArgs& base, int B, int N, int T, const double* alphas, const double* x,
                   const double* u, double* dx, double* du, const int* active) {
  HardArgs h = base;
  h.phase = 3;
  h.B = B;
  h.N = N;
  h.T = T;
  h.alphas = alphas;
  h.x = x;
  h.u = u;
  h.dx = dx;
  h.du = du;
  h.active = active;
  return launch_hard(ctx->stream, nj, h);
}

// The problem list of the lock-step loop: mask = the per-problem "may still do work" flag (st.active
// without soft limits, outer_active with them: both only ever go 1 -> 0 inside the loop), idx / cnt
// its device list, P / nb what the iteration's launches take (tmpc_internal.h PList).
struct AliveList {
  const int* mask;
  int* idx;
  int* cnt;
  int B;
  PList P;
  int nb;
};

static int alloc_alive(tmpc_ctx* ctx, int B, const int* mask, AliveList& al) {
  BUF(int, alive_idx, B);
  BUF(int, alive_cnt, 1);
  al = AliveList{mask, alive_idx, alive_cnt, B, PList{nullptr, nullptr}, B};
  return 0;
}

// keep_warm: the PCG warm-start buffer already holds this batch's starting lambdas (MPC loop)
// Lock-step batch loop with a lag-1 termination test.  Each batch iteration writes its two flags
// (some problem continues its inner loop / some problem restarted an outer pass) and the length of
// the rebuilt problem list into its own slot of active_count[2][4]; the host copies them to pinned
// memory and tests iteration `it` only after iteration `it + 1` has been enqueued, so the GPU never
// idles while the host decides.  Every kernel masks itself with the per-problem state, so the one
// iteration enqueued after the batch finished is a no-op for every problem (need_grad / active /
// outer_active are all 0).  The launches of iteration `it` visit the problem list built at the end
// of `it - 1` (on the stream, so exact), with the grid sized by the list length the host last read,
// the one of iteration `it - 2` (an upper bound because the list only shrinks: the masks go 1 -> 0 inside
// the loop and never back -- k_alive_list flags any growth and the loop then fails instead of silently
// skipping problems); the tail of a batch whose problems converge at different iterations then
// dispatches only its live problems' workgroups.
template <class Body>
static int lockstep_loop(tmpc_ctx* ctx, long cap, int* active_count, AliveList& al, Body body) {
  hipEvent_t ev[2] = {get_event(ctx), get_event(ctx)};
  if (!ev[0] || !ev[1]) return fail(ctx, "hipEventCreate failed");
  int rc = 0;
  launch_alive_list(ctx->stream, al.B, al.mask, al.idx, al.cnt, nullptr);
  HIP_OK(hipGetLastError());
  al.P = PList{al.idx, al.cnt};
  al.nb = al.B;
  for (long it = 0; it < cap; ++it) {
    const int p = (int)(it & 1);
    int* ac = active_count + 4 * p;
    if (it >= 2) al.nb = std::max(1, std::min(al.nb, ctx->h_count[4 * p + 2]));   // synced at it - 1
    HIP_OK(hipMemsetAsync(ac, 0, 4 * sizeof(int), ctx->stream));
    if ((rc = body(ac))) break;
    launch_alive_list(ctx->stream, al.B, al.mask, al.idx, al.cnt, ac + 2);
    HIP_OK(hipGetLastError());
    HIP_OK(hipMemcpyAsync(ctx->h_count + 4 * p, ac, 4 * sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    HIP_OK(hipEventRecord(ev[p], ctx->stream));
    if (it > 0) {
      HIP_OK(hipEventSynchronize(ev[p ^ 1]));
      const int* h = ctx->h_count + 4 * (p ^ 1);
      if (h[3] != 0) {   // k_alive_list: the list grew, so a grid sized by an older length skipped problems
        rc = fail(ctx, "internal: the problem list of the lock-step loop grew (a problem re-entered its loop); "
                  "the grid-size bound no longer holds");
        break;
      }
      if (h[0] == 0 && h[1] == 0) break;
    }
  }
  al.P = PList{nullptr, nullptr};
  al.nb = al.B;
  ctx->event_pool.push_back(ev[0]);
  ctx->event_pool.push_back(ev[1]);
  return rc;
}

// sd (nullable): continuous batching -- d_x, d_u are the B slots of a stream of sd->P problems
// (tmpc_sqp_solve_stream_device); each problem's results go to its rows of sd's outputs
static int sqp_device(tmpc_ctx* ctx, int B, int N, double dt, int linsys, double* d_x, double* d_u,
                      TraceDev* tr_out, bool keep_warm = false, bool hard_trace = false,
                      const StreamDev* sd = nullptr) {
  int rc = check_ready(ctx, B, N);
  if (rc) return rc;
  const int precond = precond_of(linsys);
  if (precond < 0)
    return fail(ctx, "linear system method %d is not available on the GPU (use S/PCG-J/BJ/SS = 1/2/3/4)", linsys);
  const int nj = ctx->hmodel.n, nx = 2 * nj;
  const bool chain = ctx->hmodel.chain != 0;
  const tmpc_options& o = ctx->opts;
  const SolverOpts so = solver_opts(o);
  const std::vector<double> al = alpha_list(o);
  const int T = (int)al.size();
  const int W = o.max_iter_SQP_DDP + 1;
  Work w;
  if ((rc = alloc_work(ctx, B, N, w, precond == 0))) return rc;
  ProbState st;
  if ((rc = alloc_state(ctx, B, st))) return rc;
  TraceDev tr;
  if ((rc = alloc_trace(ctx, B, W, tr))) return rc;
  BUF(double, alphas, T + 1);
  BUF(double, terms, (size_t)B * T * N * 4);   // [B][T][N][cost, violation, D, soft value]
  BUF(int, active_count, 8);   // [2][4] (lag-1 double buffer): [0] some problem in its inner loop, [1] some problem restarted a pass, [2] problem-list length
  BUF(unsigned long long, counters, 4);
  BUF(unsigned long long, prob_counters, (size_t)B * 3);   // per-problem tallies of k_ls_decide
  BUF(int, outer_active, B);
  BUF(int, outer_iter, B);
  BUF(int, exit_soft, B);
  const bool soft = ctx->hlim.any != 0;
  // the outer loop per problem (k_soft_outer with act_init): soft limits, and every stream (a slot's problem
  // is finished when it leaves its outer loop, which without soft limits is check_and_update's exit 1)
  const bool per_problem = soft || sd;
  AliveList alv;
  if ((rc = alloc_alive(ctx, B, per_problem ? outer_active : st.active, alv))) return rc;
  // UrdfCost has a state-dependent Hessian: it takes the per-knot Ghat path of the soft limits
  const bool perknot = soft || ctx->hcost.kind == COST_EE;
  double *smu = nullptr, *slam = nullptr, *sphi = nullptr;
  if (perknot) {
    if ((rc = alloc_soft(ctx, B, N, &smu, &slam, &sphi))) return rc;
    if (sd || ctx->soft_B != B || ctx->soft_N != N) {   // a stream's problems start from the initial constants
      launch_soft_init(ctx->stream, ctx->dlim, (size_t)B * N * 6 * nj, 6 * nj, smu, slam, sphi);
      HIP_OK(hipGetLastError());
      ctx->soft_B = B;
      ctx->soft_N = N;
    }
    BUF(double, soft_Gk, (size_t)B * N * (nx * nx + nj * nj));
    BUF(double, soft_j, (size_t)B * N * (nx + nj));
    w.Gk = soft_Gk;
    w.jsoft = soft_j;
    w.smu = smu;
    w.slam = slam;
  }
  // hard box constraints (ACTIVE_SET / FULL_SET): per-knot rows, a banded Schur complement per problem
  HardArgs hard{};
  double* hterms = nullptr;
  const bool banded = qp_banded(ctx, N);
  if (banded) {
    if ((rc = setup_hard(ctx, B, N, T, precond, hard))) return rc;
    if (ctx->hlim.any_hard) hterms = hard.hterms;   // the limits' violation terms of the line search
    w.hard = &hard;
    w.Wtr = W;
    if (hard_trace && ctx->hlim.any_hard) {   // per-QP active-set bitmasks in the trace (tmpc_trace.hard_active)
      BUF(unsigned long long, tr_hard, (size_t)B * W * N);
      HIP_OK(hipMemsetAsync(tr_hard, 0, (size_t)B * W * N * sizeof(unsigned long long), ctx->stream));
      w.tr_active = tr_hard;
      tr.hard_active = tr_hard;
    }
  }
  if (o.pcg_warm_start && precond != 0 && banded)
    return fail(ctx, ctx->hlim.any_hard
                ? "pcg_warm_start with hard box constraints: the Schur dimension changes with the active set "
                  "from QP to QP, so a previous lambda is no PCG guess; unset pcg_warm_start"
                : "pcg_warm_start past the fused QP's rows: the banded PCG takes no guess; unset pcg_warm_start");
  if (o.pcg_warm_start && precond != 0) {
    // PCG warm start: each QP starts from the problem's previous lambda (in place: a workgroup reads
    // its guess before it writes its lambda)
    BUF(double, lam_warm, (size_t)B * N * nx);
    if (!keep_warm || sd) HIP_OK(hipMemsetAsync(lam_warm, 0, (size_t)B * N * nx * sizeof(double), ctx->stream));
    w.guess = lam_warm;
    w.lam_keep = lam_warm;
  }
  HIP_OK(hipMemsetAsync(counters, 0, 4 * sizeof(unsigned long long), ctx->stream));
  HIP_OK(hipMemsetAsync(prob_counters, 0, (size_t)B * 3 * sizeof(unsigned long long), ctx->stream));
  std::vector<double> al_h(al);
  al_h.push_back(0.0);  // slot T: alpha = 0 for the initial merit evaluation
  HIP_OK(hipMemcpyAsync(alphas, al_h.data(), al_h.size() * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
  if (sd) {   // slot s starts with problem s
    launch_stream_init(ctx->stream, B, *sd, d_x, d_u);
    HIP_OK(hipGetLastError());
  }
  // xs = x[:, 0] (:527)
  HIP_OK(hipMemcpy2DAsync(w.xs, sizeof(double), d_x, (size_t)N * sizeof(double), sizeof(double), (size_t)B * nx,
                          hipMemcpyDeviceToDevice, ctx->stream));
  launch_outer_init(ctx->stream, B, outer_active, outer_iter, exit_soft);
  launch_init_state(ctx->stream, B, o.rho_init_SQP_DDP, st, outer_active);
  // initial J, c, merit (:541-548) of the problems in `mask` (st.active: all; act_init: restarted passes
  // and a stream's new problems, which k_ls_decide then moves into their inner loop: activate = st.active)
  auto init_merit = [&](int* mask, int* ac, int* activate) -> int {
    ProbState sti = st;
    sti.active = mask;
    LAUNCH_OK(launch_ls_terms(val32(ctx), ctx->stream, nj, chain, ctx->model_id, ctx->dmodel, ctx->dcost, ctx->dlim, smu, slam,
                              alv.P, alv.nb, N, 1, dt, alphas + T, d_x, d_u, w.xs, nullptr, nullptr, mask, terms));
    if (hterms) LAUNCH_OK(hard_ls(ctx, nj, hard, B, N, 1, alphas + T, d_x, d_u, nullptr, nullptr, mask));
    launch_ls_decide(ctx->stream, alv.P, alv.nb, N, nx, nj, 1, LS_MODE_INIT, soft, alphas + T, so, terms, d_x, d_u, w.dx, w.du,
                     sti, nullptr, tr, ac, nullptr, hterms, nullptr, activate);
    HIP_OK(hipGetLastError());
    return 0;
  };
  // one SQP iteration (:550-757) of every problem in its inner loop; flags[0] = some problem continues
  auto sqp_iteration = [&](int* ac) -> int {
    int rc2 = run_qp(ctx, B, N, dt, precond, d_x, d_u, st, w, false, alv.P, alv.nb);
    if (rc2) return rc2;
    {
      Timed t(ctx, "ls_terms");
      LAUNCH_OK(launch_ls_terms(val32(ctx), ctx->stream, nj, chain, ctx->model_id, ctx->dmodel, ctx->dcost, ctx->dlim, smu, slam,
                                alv.P, alv.nb, N, T, dt, alphas, d_x, d_u, w.xs, w.dx, w.du, st.active, terms));
      if (hterms) LAUNCH_OK(hard_ls(ctx, nj, hard, B, N, T, alphas, d_x, d_u, w.dx, w.du, st.active));
    }
    Timed t(ctx, "ls_decide");
    launch_ls_decide(ctx->stream, alv.P, alv.nb, N, nx, nj, T, LS_MODE_STEP, soft, alphas, so, terms, d_x, d_u, w.dx, w.du,
                     st, w.iters, tr, ac, prob_counters, hterms, (w.hard && precond == 0) ? hard.sing : nullptr);
    HIP_OK(hipGetLastError());
    return 0;
  };
  HIP_OK(hipMemsetAsync(active_count, 0, 8 * sizeof(int), ctx->stream));
  if ((rc = init_merit(st.active, active_count, nullptr))) return rc;
  if (!per_problem) {
    // unconstrained: one inner loop (at most max_iter iterations, + 1 for the lag of the exit test);
    // check_and_update_soft_constraints then exits 1 (:531-757)
    rc = lockstep_loop(ctx, (long)o.max_iter_SQP_DDP + 1, active_count, alv, [&](int* ac) { return sqp_iteration(ac); });
    if (rc) return rc;
    launch_soft_outer(ctx->stream, ctx->dlim, PList{nullptr, nullptr}, B, N, nj, o.exit_tolerance_softConstraints, o.max_iter_softConstraints,
                      d_x, d_u, smu, slam, sphi, outer_active, outer_iter, exit_soft, active_count);
    HIP_OK(hipGetLastError());
  } else {
    // soft-constraint outer loop (:531-757), per problem: a problem whose inner loop exits runs
    // check_and_update_soft_constraints at once (k_soft_outer, per-problem mode) and starts its
    // next pass the following iteration, while the rest of the batch carries on.  Launches per
    // solve: the largest per-problem total of SQP iterations, not the sum over passes of each
    // pass's slowest problem (BASELINE config 4: 657 -> see DESIGN.md).  Each problem's own
    // sequence of operations is the lock-step one, so its results are identical.
    BUF(int, act_init, B);
    HIP_OK(hipMemsetAsync(act_init, 0, sizeof(int) * B, ctx->stream));
    const long per = (long)(o.max_iter_softConstraints + 1) * (o.max_iter_SQP_DDP + 1) + 3;
    // a stream: every batch iteration advances some problem by one iteration, so P x per bounds it
    const long cap = sd ? per * sd->P + 3 : per;
    rc = lockstep_loop(ctx, cap, active_count, alv, [&](int* ac) -> int {
      int r = sqp_iteration(ac);
      if (r) return r;
      {   // a stream: k_soft_outer also hands finished slots on (finished problems out, pending ones in)
        Timed t(ctx, "soft_outer");
        launch_soft_outer(ctx->stream, ctx->dlim, alv.P, alv.nb, N, nj, o.exit_tolerance_softConstraints,
                          o.max_iter_softConstraints, d_x, d_u, smu, slam, sphi, outer_active, outer_iter, exit_soft,
                          ac + 1, &st, act_init, o.rho_init_SQP_DDP, sd, w.xs, &tr, w.lam_keep);
        HIP_OK(hipGetLastError());
      }
      // restarted passes (act_init, set by k_soft_outer) and a stream's new problems: initial merit, then
      // into the inner loop; masked by act_init, so a no-op when no pass restarted
      Timed t(ctx, "init_merit");
      return init_merit(act_init, ac, st.active);
    });
    if (rc) return rc;
  }
  launch_sum_counters(ctx->stream, B, prob_counters, counters);
  unsigned long long hc[4] = {0, 0, 0, 0};
  HIP_OK(hipMemcpyAsync(hc, counters, sizeof(hc), hipMemcpyDeviceToHost, ctx->stream));
  HIP_OK(hipStreamSynchronize(ctx->stream));
  ctx->last_counters[0] = (int64_t)hc[0];
  ctx->last_counters[1] = (int64_t)hc[1];
  ctx->last_counters[2] = (int64_t)hc[2];
  ctx->last_counters[3] = (int64_t)T;
  if (w.hard && (rc = collect_hard_work(ctx, hard))) return rc;
  if (sd && perknot) ctx->soft_B = ctx->soft_N = -1;   // the slots' constants are no caller's state
  resolve_timings(ctx);
  if (tr_out) *tr_out = tr;
  return 0;
}

// ------------------------------------------------------------------ iLQR driver (oracle/ilqr.py)
static int ilqr_device(tmpc_ctx* ctx, int B, int N, double dt, double* d_x, double* d_u, TraceDev* tr_out,
                       const StreamDev* sd = nullptr) {
  int rc = check_ready(ctx, B, N, false);
  if (rc) return rc;
  if (ctx->hcost.kind != COST_QUADRATIC) return fail(ctx, "iLQR supports QuadraticCost only (UrdfCost: use SQP)");
  if (ctx->hlim.any_hard)
    return fail(ctx, "iLQR has no constraint rows: hard box constraints (ACTIVE_SET / FULL_SET) need SQP");
  const int nj = ctx->hmodel.n, nx = 2 * nj, K = N - 1;
  const bool chain = ctx->hmodel.chain != 0;
  const tmpc_options& o = ctx->opts;
  const SolverOpts so = solver_opts(o);
  const std::vector<double> al = alpha_list(o);
  const int T = (int)al.size();
  const int W = o.max_iter_SQP_DDP + 1;
  Work w;
  if ((rc = alloc_work(ctx, B, N, w, false))) return rc;
  ProbState st;
  if ((rc = alloc_state(ctx, B, st))) return rc;
  TraceDev tr;
  if ((rc = alloc_trace(ctx, B, W, tr))) return rc;
  BUF(double, alphas, T);
  BUF(double, il_K, (size_t)B * K * nj * nx);
  BUF(double, il_d, (size_t)B * K * nj);
  BUF(double, il_dV, (size_t)B * 2);
  BUF(int, il_ok, B);
  BUF(double, il_xt, (size_t)B * T * nx * N);
  BUF(double, il_ut, (size_t)B * T * nj * K);
  BUF(double, il_J, (size_t)B * T);
  BUF(int, active_count, 8);   // [2][4], as sqp_device
  BUF(int, outer_active, B);
  BUF(int, outer_iter, B);
  BUF(int, exit_soft, B);
  BUF(unsigned long long, counters, 4);
  BUF(unsigned long long, il_prob_counters, (size_t)B * 3);   // per-problem tallies of k_ilqr_decide
  HIP_OK(hipMemsetAsync(counters, 0, 4 * sizeof(unsigned long long), ctx->stream));
  HIP_OK(hipMemsetAsync(il_prob_counters, 0, (size_t)B * 3 * sizeof(unsigned long long), ctx->stream));
  const bool soft = ctx->hlim.any != 0;
  const bool per_problem = soft || sd;   // as sqp_device
  AliveList alv;
  if ((rc = alloc_alive(ctx, B, per_problem ? outer_active : st.active, alv))) return rc;
  double *smu = nullptr, *slam = nullptr, *sphi = nullptr, *il_jac = nullptr;
  if (soft) {
    if ((rc = alloc_soft(ctx, B, N, &smu, &slam, &sphi))) return rc;
    if (sd || ctx->soft_B != B || ctx->soft_N != N) {
      launch_soft_init(ctx->stream, ctx->dlim, (size_t)B * N * 6 * nj, 6 * nj, smu, slam, sphi);
      HIP_OK(hipGetLastError());
      ctx->soft_B = B;
      ctx->soft_N = N;
    }
    BUF(double, il_jac_buf, (size_t)B * N * 3 * nj);   // soft-limit jacobians of every knot (Riccati sweep)
    il_jac = il_jac_buf;
  }
  HIP_OK(hipMemcpyAsync(alphas, al.data(), al.size() * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
  StreamDev sdr{};
  if (sd) {
    // a stream's problems start from the rollout of u from x[:, 0] too: roll the `period` inputs out once
    // (the same kernel on the same x[:, 0], u as a batch solve's rollout, so the same trajectories) and
    // let the slots copy from there -- a pending problem then enters its slot without a serial rollout
    sdr = *sd;
    BUF(double, stream_xr, (size_t)sd->period * nx * N);
    HIP_OK(hipMemcpyAsync(stream_xr, sd->x_in, (size_t)sd->period * nx * N * sizeof(double), hipMemcpyDeviceToDevice,
                          ctx->stream));
    LAUNCH_OK(launch_rollout(val32(ctx), ctx->stream, nj, chain, ctx->model_id, ctx->dmodel, sd->period, N, dt,
                             stream_xr, sd->u_in));
    sdr.x_in = stream_xr;
    launch_stream_init(ctx->stream, B, sdr, d_x, d_u);   // slot s starts with problem s
    HIP_OK(hipGetLastError());
  } else {
    // iLQR iterates are rollouts: start from the rollout of u from x[:, 0]
    LAUNCH_OK(launch_rollout(val32(ctx), ctx->stream, nj, chain, ctx->model_id, ctx->dmodel, B, N, dt, d_x, d_u));
  }
  HIP_OK(hipMemcpy2DAsync(w.xs, sizeof(double), d_x, (size_t)N * sizeof(double), sizeof(double), (size_t)B * nx,
                          hipMemcpyDeviceToDevice, ctx->stream));
  launch_outer_init(ctx->stream, B, outer_active, outer_iter, exit_soft);
  launch_init_state(ctx->stream, B, o.rho_init_SQP_DDP, st, outer_active);
  // J at the current trajectory of the problems in `mask` (st.active: all; act_init: restarted passes and a
  // stream's new problems, moved into their inner loop by k_ilqr_decide: activate = st.active)
  auto init_cost = [&](int* mask, int* ac, int* activate) -> int {
    ProbState sti = st;
    sti.active = mask;
    LAUNCH_OK(launch_ilqr_init_cost(ctx->stream, nj, ctx->dcost, ctx->dlim, smu, slam, alv.P, alv.nb, N, d_x, d_u,
                                    mask, il_J));
    launch_ilqr_decide(ctx->stream, alv.P, alv.nb, N, nx, nj, 1, 1, alphas, so, il_J, il_dV, il_ok, il_xt, il_ut, d_x, d_u, sti,
                       tr, ac, nullptr, activate);
    HIP_OK(hipGetLastError());
    return 0;
  };
  // one iLQR iteration of every problem in its inner loop; flags[0] = some problem continues
  auto ilqr_iteration = [&](int* ac) -> int {
    {
      Timed t(ctx, "qp_fd");
      LAUNCH_OK(launch_qp_fd(val32(ctx), ctx->stream, nj, chain, ctx->model_id, ctx->dmodel, alv.P, alv.nb, N, dt, d_x, d_u,
                             w.xs, st.need_grad, w.qdd, w.cvec));
    }
    {
      Timed t(ctx, "qp_minv");
      LAUNCH_OK(launch_qp_minv(dyn32(ctx), ctx->stream, nj, chain, ctx->model_id, ctx->dmodel, alv.P, alv.nb, N, d_x,
                               st.need_grad, w.minv));
    }
    {
      Timed t(ctx, "qp_grad");
      LAUNCH_OK(launch_qp_grad(dyn32(ctx), ctx->stream, nj, chain, ctx->model_id, ctx->dmodel, alv.P, alv.nb, N, dt, d_x,
                               st.need_grad, w.qdd, w.minv, w.A, w.Bm));
    }
    {
      Timed t(ctx, "ilqr_backward");
      LAUNCH_OK(launch_ilqr_backward(ric32(ctx), ctx->stream, nj, ctx->dcost, ctx->dlim, alv.P, alv.nb, N, d_x, d_u,
                                     st.rho, st.active,
                                     w.A, w.Bm, smu, slam, il_jac, il_K, il_d, il_dV, il_ok));
    }
    {
      Timed t(ctx, "ilqr_forward");
      LAUNCH_OK(launch_ilqr_forward(val32(ctx), ctx->stream, nj, chain, ctx->model_id, ctx->dmodel, ctx->dcost, ctx->dlim, smu,
                                    slam, alv.P, alv.nb, N, T, dt, 0, alphas, d_x, d_u, il_K, il_d, st.active, il_ok, il_xt, il_ut,
                                    il_J));
    }
    Timed t(ctx, "ilqr_decide");
    launch_ilqr_decide(ctx->stream, alv.P, alv.nb, N, nx, nj, T, 0, alphas, so, il_J, il_dV, il_ok, il_xt, il_ut, d_x, d_u, st, tr,
                       ac, il_prob_counters);
    HIP_OK(hipGetLastError());
    return 0;
  };
  HIP_OK(hipMemsetAsync(active_count, 0, 8 * sizeof(int), ctx->stream));
  if ((rc = init_cost(st.active, active_count, nullptr))) return rc;
  if (!per_problem) {
    rc = lockstep_loop(ctx, (long)o.max_iter_SQP_DDP + 1, active_count, alv, [&](int* ac) { return ilqr_iteration(ac); });
    if (rc) return rc;
    launch_soft_outer(ctx->stream, ctx->dlim, PList{nullptr, nullptr}, B, N, nj, o.exit_tolerance_softConstraints,
                      o.max_iter_softConstraints, d_x, d_u, smu, slam, sphi, outer_active, outer_iter, exit_soft,
                      active_count);
    HIP_OK(hipGetLastError());
  } else {
    // soft-constraint outer loop per problem (as sqp_device): a problem starts its next pass as soon
    // as its own inner loop exits
    BUF(int, act_init, B);
    HIP_OK(hipMemsetAsync(act_init, 0, sizeof(int) * B, ctx->stream));
    const long per = (long)(o.max_iter_softConstraints + 1) * (o.max_iter_SQP_DDP + 1) + 3;
    const long cap = sd ? per * sd->P + 3 : per;   // as sqp_device
    rc = lockstep_loop(ctx, cap, active_count, alv, [&](int* ac) -> int {
      int r = ilqr_iteration(ac);
      if (r) return r;
      {   // a stream: k_soft_outer also hands finished slots on (pending problems from the rolled-out inputs)
        Timed t(ctx, "soft_outer");
        launch_soft_outer(ctx->stream, ctx->dlim, alv.P, alv.nb, N, nj, o.exit_tolerance_softConstraints,
                          o.max_iter_softConstraints, d_x, d_u, smu, slam, sphi, outer_active, outer_iter, exit_soft,
                          ac + 1, &st, act_init, o.rho_init_SQP_DDP, sd ? &sdr : nullptr, w.xs, &tr, nullptr);
        HIP_OK(hipGetLastError());
      }
      Timed t(ctx, "init_merit");
      return init_cost(act_init, ac, st.active);   // masked by act_init: a no-op when no pass restarted
    });
    if (rc) return rc;
  }
  launch_sum_counters(ctx->stream, B, il_prob_counters, counters);
  unsigned long long hc[4] = {0, 0, 0, 0};
  HIP_OK(hipMemcpyAsync(hc, counters, sizeof(hc), hipMemcpyDeviceToHost, ctx->stream));
  HIP_OK(hipStreamSynchronize(ctx->stream));
  for (int i = 0; i < 3; ++i) ctx->last_counters[i] = (int64_t)hc[i];
  ctx->last_counters[3] = (int64_t)T;
  if (sd && soft) ctx->soft_B = ctx->soft_N = -1;   // as sqp_device
  resolve_timings(ctx);
  if (tr_out) *tr_out = tr;
  return 0;
}

// ======================================================================= C ABI
extern "C" {

int tmpc_abi_version(void) { return TMPC_ABI_VERSION; }

int tmpc_device_count(int* count) {
  if (!count) return -1;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *count = n;
  return 0;
}

int tmpc_create(int device, tmpc_ctx** out) {
  if (!out) return -1;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return -2;
  if (device < 0 || device >= n) return -3;
  tmpc_ctx* ctx = new tmpc_ctx();
  ctx->device = device;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc(&ctx->dmodel, sizeof(ModelDev)) != hipSuccess || hipMalloc(&ctx->dcost, sizeof(CostDev)) != hipSuccess ||
      hipMalloc(&ctx->dlim, sizeof(ConstrDev)) != hipSuccess || hipMemset(ctx->dlim, 0, sizeof(ConstrDev)) != hipSuccess ||
      hipHostMalloc(&ctx->h_count, 8 * sizeof(int)) != hipSuccess) {
    delete ctx;
    return -4;
  }
  pcg_set_max_lds();
  hard_set_max_lds();
  dense_set_max_lds();
  qp_blocks_set_max_lds();
  tmpc_default_options(&ctx->opts);
  *out = ctx;
  return 0;
}

void tmpc_destroy(tmpc_ctx* ctx) {
  if (!ctx) return;
  hipSetDevice(ctx->device);
  if (ctx->stream) hipStreamSynchronize(ctx->stream);
  for (auto& p : ctx->pending) {
    hipEventDestroy(p.start);
    hipEventDestroy(p.stop);
  }
  for (auto e : ctx->event_pool) hipEventDestroy(e);
  for (tmpc_ctx* sub : ctx->subs) tmpc_destroy(sub);
  for (auto& kv : ctx->bufs)
    if (kv.second.ptr) hipFree(kv.second.ptr);
  if (ctx->dmodel) hipFree(ctx->dmodel);
  if (ctx->dcost) hipFree(ctx->dcost);
  if (ctx->dlim) hipFree(ctx->dlim);
  if (ctx->h_count) hipHostFree(ctx->h_count);
  if (ctx->stream) hipStreamDestroy(ctx->stream);
  delete ctx;
}

const char* tmpc_last_error(const tmpc_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int tmpc_set_model(tmpc_ctx* ctx, int n, const int32_t* parent, const int32_t* jtype, const int32_t* saxis,
                   const double* X0, const double* Xa, const double* Xb, const double* I, double gravity) {
  if (!ctx) return -1;
  if (n < 1 || n > NJMAX) return fail(ctx, "model must have 1..%d joints (got %d)", NJMAX, n);
  if (!parent || !jtype || !saxis || !X0 || !Xa || !Xb || !I) return fail(ctx, "null model array");
  ModelDev m{};
  m.n = n;
  m.gravity = gravity;
  bool chain = true;
  for (int j = 0; j < n; ++j) {
    if (parent[j] < -1 || parent[j] >= j)
      return fail(ctx, "parent[%d] = %d: joints must be in DFS order (parent id < child id)", j, parent[j]);
    if (jtype[j] != TMPC_JOINT_REVOLUTE && jtype[j] != TMPC_JOINT_PRISMATIC)
      return fail(ctx, "joint %d: unsupported joint type %d", j, jtype[j]);
    if (saxis[j] < 0 || saxis[j] > 5) return fail(ctx, "joint %d: motion subspace index %d out of range", j, saxis[j]);
    m.parent[j] = parent[j];
    m.jtype[j] = jtype[j];
    m.saxis[j] = saxis[j];
    if (parent[j] != j - 1) chain = false;
    for (int e = 0; e < 6; ++e) m.S[j][e] = (e == saxis[j]) ? 1.0 : 0.0;
    memcpy(m.X0[j], X0 + 36 * j, 36 * sizeof(double));
    memcpy(m.Xa[j], Xa + 36 * j, 36 * sizeof(double));
    memcpy(m.Xb[j], Xb + 36 * j, 36 * sizeof(double));
    memcpy(m.I[j], I + 36 * j, 36 * sizeof(double));
  }
  for (int j = n - 1; j >= 0; --j) {
    m.subtree[j] |= 1u << j;
    if (parent[j] >= 0) m.subtree[parent[j]] |= m.subtree[j];
  }
  m.chain = chain ? 1 : 0;
  // per-robot compiled kernels when the model is one of the bundled ones (tools/gen_models.py);
  // TMPC_GENERIC_MODEL=1 forces the runtime-coefficient kernels
  const char* gen = getenv("TMPC_GENERIC_MODEL");
  ctx->model_id = (gen && gen[0] == '1') ? 0 : match_static_model(m);
  ctx->soft_B = ctx->soft_N = -1;   // the soft-constraint state is sized per model (6 n slots per knot)
  hipSetDevice(ctx->device);
  HIP_OK(hipMemcpyAsync(ctx->dmodel, &m, sizeof(m), hipMemcpyHostToDevice, ctx->stream));
  HIP_OK(hipStreamSynchronize(ctx->stream));
  ctx->hmodel = m;
  ctx->has_model = true;
  return 0;
}

int tmpc_set_cost_quadratic(tmpc_ctx* ctx, int nx, int nu, const double* Q, const double* QF, const double* R,
                            const double* xg, int32_t QF_start) {
  if (!ctx) return -1;
  if (nx < 1 || nx > NXMAX || nu < 1 || nu > NJMAX) return fail(ctx, "cost sizes out of range (nx=%d, nu=%d)", nx, nu);
  if (!Q || !QF || !R || !xg) return fail(ctx, "null cost array");
  CostDev c{};
  c.nx = nx;
  c.nu = nu;
  c.QF_start = QF_start < 0 ? -1 : QF_start;
  memcpy(c.Q, Q, sizeof(double) * nx * nx);
  memcpy(c.QF, QF, sizeof(double) * nx * nx);
  memcpy(c.R, R, sizeof(double) * nu * nu);
  memcpy(c.xg, xg, sizeof(double) * nx);
  // diagonal Q, QF, R: the kernels' cost products take their exact-zero-free form (CostDev.diag);
  // TMPC_GENERIC_COST=1 keeps the dense form (tests compare the two bit for bit)
  const char* gc = getenv("TMPC_GENERIC_COST");
  c.diag = (gc && gc[0] == '1') ? 0 : 1;
  for (int r = 0; r < nx; ++r)
    for (int k = 0; k < nx; ++k)
      if (r != k && (Q[r * nx + k] != 0.0 || QF[r * nx + k] != 0.0)) c.diag = 0;
  for (int r = 0; r < nu; ++r)
    for (int k = 0; k < nu; ++k)
      if (r != k && R[r * nu + k] != 0.0) c.diag = 0;
  hipSetDevice(ctx->device);
  HIP_OK(hipMemcpyAsync(ctx->dcost, &c, sizeof(c), hipMemcpyHostToDevice, ctx->stream));
  HIP_OK(hipStreamSynchronize(ctx->stream));
  ctx->hcost = c;
  ctx->has_cost = true;
  return 0;
}

int tmpc_set_cost_ee(tmpc_ctx* ctx, int nx, int nu, const double* Q, const double* QF, const double* R,
                     const double* xg, int32_t QF_start, const double* H0, const double* Ha, const double* Hb) {
  if (!ctx) return -1;
  if (nx != 4 || nu != 2)
    return fail(ctx, "UrdfCost is defined for 2-link arms only (nx=4, nu=2; got nx=%d, nu=%d)", nx, nu);
  if (!Q || !QF || !R || !xg || !H0 || !Ha || !Hb) return fail(ctx, "null cost array");
  CostDev c{};
  c.nx = nx;
  c.nu = nu;
  c.kind = COST_EE;
  c.QF_start = QF_start < 0 ? -1 : QF_start;
  memcpy(c.Q, Q, sizeof(double) * nx * nx);
  memcpy(c.QF, QF, sizeof(double) * nx * nx);
  memcpy(c.R, R, sizeof(double) * nu * nu);
  memcpy(c.xg, xg, sizeof(double) * nx);
  memcpy(c.eeH0, H0, sizeof(double) * 32);
  memcpy(c.eeHa, Ha, sizeof(double) * 32);
  memcpy(c.eeHb, Hb, sizeof(double) * 32);
  hipSetDevice(ctx->device);
  HIP_OK(hipMemcpyAsync(ctx->dcost, &c, sizeof(c), hipMemcpyHostToDevice, ctx->stream));
  HIP_OK(hipStreamSynchronize(ctx->stream));
  ctx->hcost = c;
  ctx->has_cost = true;
  return 0;
}

void tmpc_default_options(tmpc_options* o) {
  if (!o) return;
  memset(o, 0, sizeof(*o));
  o->exit_tolerance_linSys = 1e-6;
  o->max_iter_linSys = 100;
  o->max_iter_SQP_DDP = 100;
  o->exit_tolerance_SQP_DDP = 1e-6;
  o->alpha_factor_SQP_DDP = 0.5;
  o->alpha_min_SQP_DDP = 0.005;
  o->rho_factor_SQP_DDP = 4;
  o->rho_min_SQP_DDP = 1e-3;
  o->rho_max_SQP_DDP = 1e3;
  o->rho_init_SQP_DDP = 0.001;
  o->expected_reduction_min_SQP_DDP = 0.05;
  o->expected_reduction_max_SQP_DDP = 3;
  o->merit_mu = 10.0;
  o->profile = 0;
  o->max_iter_softConstraints = 10;
  o->exit_tolerance_softConstraints = 1e-6;
}

int tmpc_set_box_limits(tmpc_ctx* ctx, const tmpc_box_limits* L) {
  if (!ctx) return -1;
  if (!ctx->has_model) return fail(ctx, "no model: call tmpc_set_model first");
  ctx->hard_last = {0, 0, 0, 0, 0};
  ConstrDev c{};
  if (L) {
    for (int t = 0; t < 3; ++t) {
      if (L->mode[t] < TMPC_LIMIT_NONE || L->mode[t] > TMPC_LIMIT_FULL_SET)
        return fail(ctx, "limit %d: mode %d (valid: 0 none, 1 QUADRATIC_PENALTY, 2 AUGMENTED_LAGRANGIAN, "
                    "3 ACTIVE_SET, 4 FULL_SET)", t, L->mode[t]);
      if (L->mode[t] <= TMPC_LIMIT_AUGMENTED_LAGRANGIAN) {
        c.mode[t] = L->mode[t];
        if (c.mode[t] != SOFT_NONE) c.any = 1;
      } else {
        c.hard[t] = L->mode[t] == TMPC_LIMIT_ACTIVE_SET ? HARD_ACTIVE : HARD_FULL;
        c.any_hard = 1;
      }
      constexpr int abi_row = (int)(sizeof(L->lb[0]) / sizeof(double));   // tmpc_box_limits rows: 8 joints
      for (int i = 0; i < NJMAX; ++i) {   // (limits are refused past NJ_FULL joints, check_ready)
        c.lb[t][i] = i < abi_row ? L->lb[t][i] : 0.0;
        c.ub[t][i] = i < abi_row ? L->ub[t][i] : 0.0;
      }
      c.mu_init[t] = L->mu_init[t];
      c.mu_factor[t] = L->mu_factor[t];
      c.mu_max[t] = L->mu_max[t];
      c.phi_init[t] = L->phi_init[t];
      c.phi_factor[t] = L->phi_factor[t];
    }
  }
  hipSetDevice(ctx->device);
  HIP_OK(hipMemcpyAsync(ctx->dlim, &c, sizeof(c), hipMemcpyHostToDevice, ctx->stream));
  HIP_OK(hipStreamSynchronize(ctx->stream));
  ctx->hlim = c;
  ctx->soft_B = ctx->soft_N = -1;
  return 0;
}

int tmpc_set_soft_state(tmpc_ctx* ctx, int B, int N, const double* mu, const double* lam, const double* phi) {
  if (!ctx) return -1;
  if (!ctx->has_model) return fail(ctx, "no model: call tmpc_set_model first");
  if (B < 1 || N < 2) return fail(ctx, "bad sizes B=%d N=%d", B, N);
  hipSetDevice(ctx->device);
  double *smu, *slam, *sphi;
  int rc = alloc_soft(ctx, B, N, &smu, &slam, &sphi);
  if (rc) return rc;
  const size_t n = (size_t)B * N * 6 * ctx->hmodel.n;
  launch_soft_init(ctx->stream, ctx->dlim, n, 6 * ctx->hmodel.n, smu, slam, sphi);
  HIP_OK(hipGetLastError());
  if (mu) HIP_OK(hipMemcpyAsync(smu, mu, n * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
  if (lam) HIP_OK(hipMemcpyAsync(slam, lam, n * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
  if (phi) HIP_OK(hipMemcpyAsync(sphi, phi, n * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
  HIP_OK(hipStreamSynchronize(ctx->stream));
  ctx->soft_B = B;
  ctx->soft_N = N;
  return 0;
}

int tmpc_get_soft_state(tmpc_ctx* ctx, int B, int N, double* mu, double* lam, double* phi) {
  if (!ctx) return -1;
  if (ctx->soft_B != B || ctx->soft_N != N)
    return fail(ctx, "no soft-constraint state for B=%d N=%d (solve or tmpc_set_soft_state first)", B, N);
  hipSetDevice(ctx->device);
  const size_t n = (size_t)B * N * 6 * ctx->hmodel.n;
  if (mu) HIP_OK(hipMemcpy(mu, ctx->bufs["soft_mu"].ptr, n * sizeof(double), hipMemcpyDeviceToHost));
  if (lam) HIP_OK(hipMemcpy(lam, ctx->bufs["soft_lam"].ptr, n * sizeof(double), hipMemcpyDeviceToHost));
  if (phi) HIP_OK(hipMemcpy(phi, ctx->bufs["soft_phi"].ptr, n * sizeof(double), hipMemcpyDeviceToHost));
  return 0;
}

int tmpc_set_options(tmpc_ctx* ctx, const tmpc_options* o) {
  if (!ctx || !o) return -1;
  if (o->max_iter_linSys < 1 || o->max_iter_SQP_DDP < 1 || o->max_iter_softConstraints < 1)
    return fail(ctx, "max_iter options must be >= 1");
  if (!(o->alpha_factor_SQP_DDP > 0.0 && o->alpha_factor_SQP_DDP < 1.0))
    return fail(ctx, "alpha_factor_SQP_DDP must be in (0, 1)");
  if (o->precision < TMPC_PRECISION_F64 || o->precision > TMPC_PRECISION_MIXED)
    return fail(ctx, "precision %d (valid: 0 F64, 1 F32, 2 MIXED)", o->precision);
  ctx->opts = *o;
  return 0;
}

int tmpc_sqp_solve_batch_device(tmpc_ctx* ctx, int B, int N, double dt, int linsys, double* d_x, double* d_u,
                                int32_t* exit_sqp, int32_t* sqp_iter) {
  if (!ctx) return -1;
  hipSetDevice(ctx->device);
  int rc = sqp_device(ctx, B, N, dt, linsys, d_x, d_u, nullptr);
  if (rc) return rc;
  if (exit_sqp) HIP_OK(hipMemcpy(exit_sqp, ctx->bufs["st_exit"].ptr, sizeof(int) * B, hipMemcpyDeviceToHost));
  if (sqp_iter) HIP_OK(hipMemcpy(sqp_iter, ctx->bufs["st_iter"].ptr, sizeof(int) * B, hipMemcpyDeviceToHost));
  return 0;
}

int tmpc_sqp_solve_batch(tmpc_ctx* ctx, int B, int N, double dt, int linsys, double* x, double* u,
                         int32_t* exit_sqp, int32_t* exit_soft, int32_t* outer_iter, int32_t* sqp_iter,
                         tmpc_trace* trace) {
  if (!ctx) return -1;
  int rc = check_ready(ctx, B, N);
  if (rc) return rc;
  if (!x || !u) return fail(ctx, "null x/u");
  hipSetDevice(ctx->device);
  const int nx = ctx->hcost.nx, nu = ctx->hcost.nu;
  const size_t xn = (size_t)B * nx * N, un = (size_t)B * nu * (N - 1);
  BUF(double, io_x, xn);
  BUF(double, io_u, un);
  HIP_OK(hipMemcpyAsync(io_x, x, xn * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
  HIP_OK(hipMemcpyAsync(io_u, u, un * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
  TraceDev tr;
  const bool hard_trace = trace && trace->hard_active && ctx->hlim.any_hard;
  if ((rc = sqp_device(ctx, B, N, dt, linsys, io_x, io_u, &tr, false, hard_trace))) return rc;
  HIP_OK(hipMemcpy(x, io_x, xn * sizeof(double), hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(u, io_u, un * sizeof(double), hipMemcpyDeviceToHost));
  if (exit_sqp) HIP_OK(hipMemcpy(exit_sqp, ctx->bufs["st_exit"].ptr, sizeof(int) * B, hipMemcpyDeviceToHost));
  if (sqp_iter) HIP_OK(hipMemcpy(sqp_iter, ctx->bufs["st_iter"].ptr, sizeof(int) * B, hipMemcpyDeviceToHost));
  if (exit_soft) HIP_OK(hipMemcpy(exit_soft, ctx->bufs["exit_soft"].ptr, sizeof(int) * B, hipMemcpyDeviceToHost));
  if (outer_iter) HIP_OK(hipMemcpy(outer_iter, ctx->bufs["outer_iter"].ptr, sizeof(int) * B, hipMemcpyDeviceToHost));
  if (trace) {
    const size_t n = (size_t)B * (ctx->opts.max_iter_SQP_DDP + 1);
#define CP(field, src, T) \
  if (trace->field) HIP_OK(hipMemcpy(trace->field, tr.src, n * sizeof(T), hipMemcpyDeviceToHost));
    CP(iteration, iteration, int)
    CP(line_search_iteration, ls_iter, int)
    CP(alpha, alpha, double)
    CP(rho, rho, double)
    CP(J, J, double)
    CP(c, c, double)
    CP(merit, merit, double)
    CP(D, D, double)
    CP(reduction_ratio, ratio, double)
    CP(succeeded_line_search, accepted, int)
    CP(pcg_iters, pcg_iters, int)
    CP(singular, singular, int)
#undef CP
    if (trace->hard_active) {
      if (hard_trace)
        HIP_OK(hipMemcpy(trace->hard_active, tr.hard_active, n * N * sizeof(unsigned long long), hipMemcpyDeviceToHost));
      else
        memset(trace->hard_active, 0, n * N * sizeof(uint64_t));
    }
  }
  return 0;
}

int tmpc_ilqr_solve_batch(tmpc_ctx* ctx, int B, int N, double dt, double* x, double* u, int32_t* exit_code,
                          int32_t* exit_soft, int32_t* outer_iter, int32_t* iters, tmpc_trace* trace) {
  if (!ctx) return -1;
  int rc = check_ready(ctx, B, N, false);
  if (rc) return rc;
  if (!x || !u) return fail(ctx, "null x/u");
  hipSetDevice(ctx->device);
  const int nx = ctx->hcost.nx, nu = ctx->hcost.nu;
  const size_t xn = (size_t)B * nx * N, un = (size_t)B * nu * (N - 1);
  BUF(double, io_x, xn);
  BUF(double, io_u, un);
  HIP_OK(hipMemcpyAsync(io_x, x, xn * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
  HIP_OK(hipMemcpyAsync(io_u, u, un * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
  TraceDev tr;
  if ((rc = ilqr_device(ctx, B, N, dt, io_x, io_u, &tr))) return rc;
  HIP_OK(hipMemcpy(x, io_x, xn * sizeof(double), hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(u, io_u, un * sizeof(double), hipMemcpyDeviceToHost));
  if (exit_code) HIP_OK(hipMemcpy(exit_code, ctx->bufs["st_exit"].ptr, sizeof(int) * B, hipMemcpyDeviceToHost));
  if (iters) HIP_OK(hipMemcpy(iters, ctx->bufs["st_iter"].ptr, sizeof(int) * B, hipMemcpyDeviceToHost));
  if (exit_soft) HIP_OK(hipMemcpy(exit_soft, ctx->bufs["exit_soft"].ptr, sizeof(int) * B, hipMemcpyDeviceToHost));
  if (outer_iter) HIP_OK(hipMemcpy(outer_iter, ctx->bufs["outer_iter"].ptr, sizeof(int) * B, hipMemcpyDeviceToHost));
  if (trace) {
    const size_t n = (size_t)B * (ctx->opts.max_iter_SQP_DDP + 1);
#define CP(field, src, T) \
  if (trace->field) HIP_OK(hipMemcpy(trace->field, tr.src, n * sizeof(T), hipMemcpyDeviceToHost));
    CP(iteration, iteration, int)
    CP(line_search_iteration, ls_iter, int)
    CP(alpha, alpha, double)
    CP(rho, rho, double)
    CP(J, J, double)
    CP(c, c, double)
    CP(merit, merit, double)
    CP(D, D, double)
    CP(reduction_ratio, ratio, double)
    CP(succeeded_line_search, accepted, int)
    CP(pcg_iters, pcg_iters, int)
    CP(singular, singular, int)
#undef CP
    if (trace->hard_active) memset(trace->hard_active, 0, n * N * sizeof(uint64_t));
  }
  return 0;
}

int tmpc_ilqr_solve_batch_device(tmpc_ctx* ctx, int B, int N, double dt, double* d_x, double* d_u,
                                 int32_t* exit_code, int32_t* iters) {
  if (!ctx) return -1;
  hipSetDevice(ctx->device);
  int rc = ilqr_device(ctx, B, N, dt, d_x, d_u, nullptr);
  if (rc) return rc;
  if (exit_code) HIP_OK(hipMemcpy(exit_code, ctx->bufs["st_exit"].ptr, sizeof(int) * B, hipMemcpyDeviceToHost));
  if (iters) HIP_OK(hipMemcpy(iters, ctx->bufs["st_iter"].ptr, sizeof(int) * B, hipMemcpyDeviceToHost));
  return 0;
}

// ------------------------------------------------------------------ continuous batching (include/tmpc.h, ABI 10)
// The stream's device descriptor and its B = min(slots, problems) slot buffers.
static int stream_setup(tmpc_ctx* ctx, int N, const tmpc_stream* s, StreamDev& sd, int& B, double** d_x,
                        double** d_u) {
  if (!s) return fail(ctx, "null stream");
  if (s->problems < 0 || s->slots < 1 || s->period < 1)
    return fail(ctx, "stream: problems %d (>= 0), slots %d and period %d (>= 1)", s->problems, s->slots, s->period);
  if (!s->x_in || !s->u_in) return fail(ctx, "stream: null x_in / u_in");
  if (s->trace.hard_active) return fail(ctx, "stream: trace.hard_active is not supported (set it to NULL)");
  if (s->substreams < 0 || s->substreams > 8) return fail(ctx, "stream: substreams %d (0..8)", s->substreams);
  B = std::min(s->slots, s->problems);
  const int nj = ctx->hmodel.n, nx = 2 * nj;
  BUF(double, stream_x, (size_t)std::max(B, 1) * nx * N);
  BUF(double, stream_u, (size_t)std::max(B, 1) * nj * (N - 1));
  BUF(int, stream_pid, std::max(B, 1));
  BUF(int, stream_next, 1);
  *d_x = stream_x;
  *d_u = stream_u;
  sd = StreamDev{};
  sd.P = s->problems;
  sd.pbase = 0;
  sd.period = s->period;
  sd.NX = nx;
  sd.NU = nj;
  sd.N = N;
  sd.W = ctx->opts.max_iter_SQP_DDP + 1;
  sd.MC = 6 * nj;
  sd.x_in = s->x_in;
  sd.u_in = s->u_in;
  sd.x_out = s->x_out;
  sd.u_out = s->u_out;
  sd.status = s->status;
  const tmpc_trace& t = s->trace;
  sd.tr_out = TraceDev{t.iteration, t.line_search_iteration, t.alpha, t.rho, t.J, t.c, t.merit, t.D,
                       t.reduction_ratio, t.succeeded_line_search, t.pcg_iters, t.singular, nullptr};
  sd.slot_pid = stream_pid;
  sd.next = stream_next;
  return 0;
}

// One (sub-)stream on one context: problems [pbase, pbase + s->problems) of the caller's stream.
static int stream_one(tmpc_ctx* ctx, int N, double dt, int linsys, const tmpc_stream* s, int pbase) {
  StreamDev sd;
  int B = 0;
  double *d_x = nullptr, *d_u = nullptr;
  int rc = stream_setup(ctx, N, s, sd, B, &d_x, &d_u);
  if (rc || B == 0) return rc;
  sd.pbase = pbase;
  return linsys < 0 ? ilqr_device(ctx, B, N, dt, d_x, d_u, nullptr, &sd)
                    : sqp_device(ctx, B, N, dt, linsys, d_x, d_u, nullptr, false, false, &sd);
}

// The stream, split over K = substreams concurrent sub-streams: sub-stream c has its own context (HIP stream,
// buffers, lock-step loop on its own host thread), slots / K of the slots and a contiguous 1 / K of the
// problems.  Their kernels run side by side on the GPU, so one sub-stream's latency-bound phases (a one-wave
// Riccati sweep, a rollout with fewer lanes than SIMDs) overlap the other's.  Each problem's operations are
// unchanged, so its results are too.  linsys < 0: iLQR.
static int stream_solve(tmpc_ctx* ctx, int N, double dt, int linsys, const tmpc_stream* s) {
  int rc = linsys < 0 ? check_ready(ctx, 1, N, false) : check_ready(ctx, 1, N);
  if (rc) return rc;
  if (!s) return fail(ctx, "null stream");
  hipSetDevice(ctx->device);
  const int K = std::max(1, std::min({s->substreams, s->slots, std::max(1, s->problems), 8}));
  if (K == 1 || s->substreams <= 1) return stream_one(ctx, N, dt, linsys, s, 0);
  if (s->slots < 1 || s->problems < 0 || s->period < 1 || !s->x_in || !s->u_in)
    return stream_one(ctx, N, dt, linsys, s, 0);   // the argument errors, as for one stream
  while ((int)ctx->subs.size() < K) {
    tmpc_ctx* sub = nullptr;
    if (tmpc_create(ctx->device, &sub) != 0) return fail(ctx, "stream: creating sub-stream context failed");
    ctx->subs.push_back(sub);
  }
  for (int c = 0; c < K; ++c) {   // the configuration of this context
    tmpc_ctx* sub = ctx->subs[c];
    sub->hmodel = ctx->hmodel;
    sub->hcost = ctx->hcost;
    sub->hlim = ctx->hlim;
    sub->model_id = ctx->model_id;
    sub->opts = ctx->opts;
    sub->has_model = ctx->has_model;
    sub->has_cost = ctx->has_cost;
    sub->soft_B = sub->soft_N = -1;
    sub->stats.clear();
    sub->kbytes.clear();
    sub->err.clear();
    HIP_OK(hipMemcpyAsync(sub->dmodel, &sub->hmodel, sizeof(ModelDev), hipMemcpyHostToDevice, sub->stream));
    HIP_OK(hipMemcpyAsync(sub->dcost, &sub->hcost, sizeof(CostDev), hipMemcpyHostToDevice, sub->stream));
    HIP_OK(hipMemcpyAsync(sub->dlim, &sub->hlim, sizeof(ConstrDev), hipMemcpyHostToDevice, sub->stream));
    HIP_OK(hipStreamSynchronize(sub->stream));
  }
  std::vector<tmpc_stream> part(K, *s);
  std::vector<int> pbase(K, 0), rcs(K, 0);
  for (int c = 0, p0 = 0; c < K; ++c) {
    part[c].problems = s->problems / K + (c < s->problems % K ? 1 : 0);
    part[c].slots = s->slots / K + (c < s->slots % K ? 1 : 0);
    part[c].substreams = 1;
    pbase[c] = p0;
    p0 += part[c].problems;
  }
  std::vector<std::thread> th;
  for (int c = 0; c < K; ++c)
    th.emplace_back([&, c]() {
      hipSetDevice(ctx->device);
      rcs[c] = stream_one(ctx->subs[c], N, dt, linsys, &part[c], pbase[c]);
    });
  for (auto& t : th) t.join();
  for (int c = 0; c < K; ++c)
    if (rcs[c]) return fail(ctx, "sub-stream %d: %s", c, ctx->subs[c]->err.c_str());
  for (int i = 0; i < 3; ++i) {
    ctx->last_counters[i] = 0;
    for (int c = 0; c < K; ++c) ctx->last_counters[i] += ctx->subs[c]->last_counters[i];
  }
  ctx->last_counters[3] = ctx->subs[0]->last_counters[3];
  for (int c = 0; c < K; ++c) {   // kernel timings and counted bytes of every sub-stream
    for (auto& kv : ctx->subs[c]->stats) {
      ctx->stats[kv.first].launches += kv.second.launches;
      ctx->stats[kv.first].total_ms += kv.second.total_ms;
    }
    for (auto& kv : ctx->subs[c]->kbytes) ctx->kbytes[kv.first] += kv.second;
  }
  ctx->soft_B = ctx->soft_N = -1;
  return 0;
}

int tmpc_sqp_solve_stream_device(tmpc_ctx* ctx, int N, double dt, int linsys, const tmpc_stream* stream) {
  if (!ctx) return -1;
  if (precond_of(linsys) < 0)
    return fail(ctx, "linear system method %d is not available on the GPU (use S/PCG-J/BJ/SS = 1/2/3/4)", linsys);
  return stream_solve(ctx, N, dt, linsys, stream);
}

int tmpc_ilqr_solve_stream_device(tmpc_ctx* ctx, int N, double dt, const tmpc_stream* stream) {
  if (!ctx) return -1;
  return stream_solve(ctx, N, dt, -1, stream);
}

// ------------------------------------------------------------------ receding-horizon MPC (oracle/mpc.py)
static int mpc_device(tmpc_ctx* ctx, int B, int N, double dt, int solver, int steps, double* d_x, double* d_u,
                      double* d_xe, double* d_ue, int* d_codes, int* d_iters) {
  const bool ilqr = solver == TMPC_SOLVER_ILQR;
  int rc = check_ready(ctx, B, N, !ilqr);
  if (rc) return rc;
  if (ctx->hmodel.n > NJ_FULL)
    return fail(ctx, "the MPC loop supports up to %d joints (got %d)", NJ_FULL, ctx->hmodel.n);
  if (ctx->hcost.kind != COST_QUADRATIC) return fail(ctx, "the MPC loop supports QuadraticCost only");
  if (steps < 1) return fail(ctx, "steps must be >= 1");
  if (!ilqr && precond_of(solver) < 0) return fail(ctx, "solver %d: use TMPC_LINSYS_* or TMPC_SOLVER_ILQR", solver);
  if (!ilqr && ctx->opts.pcg_warm_start && precond_of(solver) != 0 && qp_banded(ctx, N))
    return fail(ctx, "pcg_warm_start with hard box constraints or past the fused QP's rows: the banded PCG takes "
                "no guess; unset pcg_warm_start");
  const int nj = ctx->hmodel.n, nx = 2 * nj;
  const bool chain = ctx->hmodel.chain != 0;
  // work counters of the whole loop: the sum over its horizon solves (tmpc_solve_counters)
  int64_t sum_counters[3] = {0, 0, 0};
  // executed state 0 = x[:, 0]
  HIP_OK(hipMemcpy2DAsync(d_xe, (size_t)(steps + 1) * sizeof(double), d_x, (size_t)N * sizeof(double), sizeof(double),
                          (size_t)B * nx, hipMemcpyDeviceToDevice, ctx->stream));
  for (int s = 0; s < steps; ++s) {
    rc = ilqr ? ilqr_device(ctx, B, N, dt, d_x, d_u, nullptr)
              : sqp_device(ctx, B, N, dt, solver, d_x, d_u, nullptr, /*keep_warm=*/s > 0);
    if (rc) return rc;
    for (int i = 0; i < 3; ++i) sum_counters[i] += ctx->last_counters[i];
    if (!ilqr && ctx->opts.pcg_warm_start && precond_of(solver) != 0 && !qp_banded(ctx, N)) {
      // the next step's first PCG starts from this step's last lambda shifted by one knot
      // (lambda_k <- lambda_{k+1}, last block kept), as x and u are shifted (oracle/mpc.py)
      double* lw = (double*)ctx->bufs["lam_warm"].ptr;
      BUF(double, lam_tmp, (size_t)B * N * nx);
      const size_t row = (size_t)N * nx * sizeof(double), blk = (size_t)nx * sizeof(double);
      HIP_OK(hipMemcpyAsync(lam_tmp, lw, (size_t)B * row, hipMemcpyDeviceToDevice, ctx->stream));
      HIP_OK(hipMemcpy2DAsync(lw, row, (char*)lam_tmp + blk, row, row - blk, B, hipMemcpyDeviceToDevice, ctx->stream));
    }
    HIP_OK(hipMemcpy2DAsync(d_codes + s, (size_t)steps * sizeof(int), ctx->bufs["st_exit"].ptr, sizeof(int),
                            sizeof(int), B, hipMemcpyDeviceToDevice, ctx->stream));
    HIP_OK(hipMemcpy2DAsync(d_iters + s, (size_t)steps * sizeof(int), ctx->bufs["st_iter"].ptr, sizeof(int),
                            sizeof(int), B, hipMemcpyDeviceToDevice, ctx->stream));
    {
      Timed t(ctx, "mpc_shift");
      LAUNCH_OK(launch_mpc_shift(ctx->stream, nj, chain, ctx->model_id, ctx->dmodel, B, N, dt, s, steps, d_x, d_u,
                                 d_xe, d_ue));
    }
    // QuadraticCost.shift_QF_start(-1) (TrajoptCost.py:100-104)
    if (ctx->hcost.QF_start >= 0) {
      ctx->hcost.QF_start = ctx->hcost.QF_start > 0 ? ctx->hcost.QF_start - 1 : 0;
      HIP_OK(hipMemcpyAsync(ctx->dcost, &ctx->hcost, sizeof(CostDev), hipMemcpyHostToDevice, ctx->stream));
    }
    if (ctx->hlim.any) {
      launch_soft_shift(ctx->stream, ctx->dlim, B, N, nj, (double*)ctx->bufs["soft_mu"].ptr,
                        (double*)ctx->bufs["soft_lam"].ptr, (double*)ctx->bufs["soft_phi"].ptr);
      HIP_OK(hipGetLastError());
    }
  }
  HIP_OK(hipStreamSynchronize(ctx->stream));
  for (int i = 0; i < 3; ++i) ctx->last_counters[i] = sum_counters[i];
  return 0;
}

int tmpc_mpc_batch_device(tmpc_ctx* ctx, int B, int N, double dt, int solver, int steps, double* d_x, double* d_u,
                          double* d_x_exec, double* d_u_exec, int32_t* d_exit_codes, int32_t* d_iters) {
  if (!ctx) return -1;
  hipSetDevice(ctx->device);
  return mpc_device(ctx, B, N, dt, solver, steps, d_x, d_u, d_x_exec, d_u_exec, d_exit_codes, d_iters);
}

int tmpc_mpc_batch(tmpc_ctx* ctx, int B, int N, double dt, int solver, int steps, double* x, double* u,
                   double* x_exec, double* u_exec, int32_t* exit_codes, int32_t* iters) {
  if (!ctx) return -1;
  int rc = check_ready(ctx, B, N, solver != TMPC_SOLVER_ILQR);
  if (rc) return rc;
  if (!x || !u || steps < 1) return fail(ctx, "null x/u or steps < 1");
  hipSetDevice(ctx->device);
  const int nx = ctx->hcost.nx, nu = ctx->hcost.nu;
  const size_t xn = (size_t)B * nx * N, un = (size_t)B * nu * (N - 1);
  BUF(double, mpc_x, xn);
  BUF(double, mpc_u, un);
  BUF(double, mpc_xe, (size_t)B * nx * (steps + 1));
  BUF(double, mpc_ue, (size_t)B * nu * steps);
  BUF(int, mpc_codes, (size_t)B * steps);
  BUF(int, mpc_iters, (size_t)B * steps);
  HIP_OK(hipMemcpyAsync(mpc_x, x, xn * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
  HIP_OK(hipMemcpyAsync(mpc_u, u, un * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
  if ((rc = mpc_device(ctx, B, N, dt, solver, steps, mpc_x, mpc_u, mpc_xe, mpc_ue, mpc_codes, mpc_iters))) return rc;
  HIP_OK(hipMemcpy(x, mpc_x, xn * sizeof(double), hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(u, mpc_u, un * sizeof(double), hipMemcpyDeviceToHost));
  if (x_exec) HIP_OK(hipMemcpy(x_exec, mpc_xe, sizeof(double) * B * nx * (steps + 1), hipMemcpyDeviceToHost));
  if (u_exec) HIP_OK(hipMemcpy(u_exec, mpc_ue, sizeof(double) * B * nu * steps, hipMemcpyDeviceToHost));
  if (exit_codes) HIP_OK(hipMemcpy(exit_codes, mpc_codes, sizeof(int) * B * steps, hipMemcpyDeviceToHost));
  if (iters) HIP_OK(hipMemcpy(iters, mpc_iters, sizeof(int) * B * steps, hipMemcpyDeviceToHost));
  return 0;
}

int tmpc_rollout_batch_device(tmpc_ctx* ctx, int B, int N, double dt, double* d_x, const double* d_u) {
  if (!ctx) return -1;
  if (!ctx->has_model) return fail(ctx, "no model");
  if (int rc = wide_ok(ctx, "dynamics")) return rc;
  hipSetDevice(ctx->device);
  LAUNCH_OK(launch_rollout(dyn32(ctx), ctx->stream, ctx->hmodel.n, ctx->hmodel.chain != 0, ctx->model_id, ctx->dmodel, B, N, dt, d_x, d_u));
  HIP_OK(hipStreamSynchronize(ctx->stream));
  return 0;
}

int tmpc_fd_batch(tmpc_ctx* ctx, int K, double dt, const double* x, const double* u, double* xnext, double* qdd,
                  double* Minv) {
  if (!ctx) return -1;
  if (!ctx->has_model) return fail(ctx, "no model");
  if (int rc = wide_ok(ctx, "dynamics")) return rc;
  if (K < 1) return 0;
  hipSetDevice(ctx->device);
  const int nj = ctx->hmodel.n, nx = 2 * nj;
  BUF(double, u_x, (size_t)K * nx);
  BUF(double, u_u, (size_t)K * nj);
  BUF(double, u_xn, (size_t)K * nx);
  BUF(double, u_qdd, (size_t)K * nj);
  BUF(double, u_minv, (size_t)K * nj * nj);
  HIP_OK(hipMemcpyAsync(u_x, x, sizeof(double) * K * nx, hipMemcpyHostToDevice, ctx->stream));
  HIP_OK(hipMemcpyAsync(u_u, u, sizeof(double) * K * nj, hipMemcpyHostToDevice, ctx->stream));
  LAUNCH_OK(launch_unit_fd(dyn32(ctx), ctx->stream, nj, ctx->hmodel.chain != 0, ctx->model_id, ctx->dmodel, K, dt, u_x, u_u, u_xn, u_qdd));
  if (Minv) LAUNCH_OK(launch_unit_minv(dyn32(ctx), ctx->stream, nj, ctx->hmodel.chain != 0, ctx->model_id, ctx->dmodel, K, u_x, u_minv));
  HIP_OK(hipStreamSynchronize(ctx->stream));
  if (xnext) HIP_OK(hipMemcpy(xnext, u_xn, sizeof(double) * K * nx, hipMemcpyDeviceToHost));
  if (qdd) HIP_OK(hipMemcpy(qdd, u_qdd, sizeof(double) * K * nj, hipMemcpyDeviceToHost));
  if (Minv) HIP_OK(hipMemcpy(Minv, u_minv, sizeof(double) * K * nj * nj, hipMemcpyDeviceToHost));
  return 0;
}

int tmpc_fd_grad_batch(tmpc_ctx* ctx, int K, double dt, const double* x, const double* u, double* A, double* Bo,
                       double* dqdd) {
  if (!ctx) return -1;
  if (!ctx->has_model) return fail(ctx, "no model");
  if (int rc = wide_ok(ctx, "dynamics")) return rc;
  if (K < 1) return 0;
  hipSetDevice(ctx->device);
  const int nj = ctx->hmodel.n, nx = 2 * nj;
  const bool chain = ctx->hmodel.chain != 0;
  BUF(double, u_x, (size_t)K * nx);
  BUF(double, u_u, (size_t)K * nj);
  BUF(double, u_qdd, (size_t)K * nj);
  BUF(double, u_minv, (size_t)K * nj * nj);
  BUF(double, u_A, (size_t)K * nx * nx);
  BUF(double, u_B, (size_t)K * nx * nj);
  BUF(double, u_dqdd, (size_t)K * nj * 3 * nj);
  HIP_OK(hipMemcpyAsync(u_x, x, sizeof(double) * K * nx, hipMemcpyHostToDevice, ctx->stream));
  HIP_OK(hipMemcpyAsync(u_u, u, sizeof(double) * K * nj, hipMemcpyHostToDevice, ctx->stream));
  LAUNCH_OK(launch_unit_fd(dyn32(ctx), ctx->stream, nj, chain, ctx->model_id, ctx->dmodel, K, 0.0, u_x, u_u, nullptr, u_qdd));
  LAUNCH_OK(launch_unit_minv(dyn32(ctx), ctx->stream, nj, chain, ctx->model_id, ctx->dmodel, K, u_x, u_minv));
  LAUNCH_OK(launch_unit_grad(dyn32(ctx), ctx->stream, nj, chain, ctx->model_id, ctx->dmodel, K, dt, u_x, u_qdd, u_minv, u_A, u_B, u_dqdd));
  HIP_OK(hipStreamSynchronize(ctx->stream));
  if (A) HIP_OK(hipMemcpy(A, u_A, sizeof(double) * K * nx * nx, hipMemcpyDeviceToHost));
  if (Bo) HIP_OK(hipMemcpy(Bo, u_B, sizeof(double) * K * nx * nj, hipMemcpyDeviceToHost));
  if (dqdd) HIP_OK(hipMemcpy(dqdd, u_dqdd, sizeof(double) * K * nj * 3 * nj, hipMemcpyDeviceToHost));
  return 0;
}

int tmpc_qp_batch(tmpc_ctx* ctx, int B, int N, double dt, int linsys, const double* rho, const double* x,
                  const double* u, const double* xs, const double* guess, double* dxul, int32_t* pcg_iters,
                  double* S_diag, double* S_lo, double* gamma, double* P_diag) {
  if (!ctx) return -1;
  int rc = check_ready(ctx, B, N);
  if (rc) return rc;
  if (ctx->hcost.kind != COST_QUADRATIC) return fail(ctx, "tmpc_qp_batch supports QuadraticCost only");
  const bool banded = qp_banded(ctx, N);
  if (banded && guess)
    return fail(ctx, "tmpc_qp_batch: no PCG guess on the banded path (hard box constraints, or N * nx past %d)",
                QP_MAX_ROWS);
  if (banded && (S_diag || S_lo || gamma || P_diag))
    return fail(ctx, "tmpc_qp_batch: on the banded path (hard box constraints, or N * nx past %d) S is banded; "
                     "S_diag / S_lo / gamma / P_diag must be NULL (tmpc_qp_hard_info has S_band)", QP_MAX_ROWS);
  const int precond = precond_of(linsys);
  if (precond < 0) return fail(ctx, "linear system method %d is not available on the GPU", linsys);
  if (!rho || !x || !u) return fail(ctx, "null input");
  hipSetDevice(ctx->device);
  const int nj = ctx->hmodel.n, nx = 2 * nj, K = N - 1, nxu = nx + nj;
  Work w;
  if ((rc = alloc_work(ctx, B, N, w, true))) return rc;
  ProbState st;
  if ((rc = alloc_state(ctx, B, st))) return rc;
  BUF(double, io_x, (size_t)B * nx * N);
  BUF(double, io_u, (size_t)B * nj * K);
  HIP_OK(hipMemcpyAsync(io_x, x, sizeof(double) * B * nx * N, hipMemcpyHostToDevice, ctx->stream));
  HIP_OK(hipMemcpyAsync(io_u, u, sizeof(double) * B * nj * K, hipMemcpyHostToDevice, ctx->stream));
  HIP_OK(hipMemcpyAsync(st.rho, rho, sizeof(double) * B, hipMemcpyHostToDevice, ctx->stream));
  launch_init_state(ctx->stream, B, 0.0, ProbState{st.drho, st.drho, st.J, st.c, st.merit, st.iter, st.active,
                                                   st.need_grad, st.exit_sqp}, nullptr);
  if (xs)   // the SQP's initial state (solveKKTSystem_Schur's xs argument, :361): c_0 = x_0 - xs
    HIP_OK(hipMemcpyAsync(w.xs, xs, sizeof(double) * B * nx, hipMemcpyHostToDevice, ctx->stream));
  else
    HIP_OK(hipMemcpy2DAsync(w.xs, sizeof(double), io_x, (size_t)N * sizeof(double), sizeof(double), (size_t)B * nx,
                            hipMemcpyDeviceToDevice, ctx->stream));
  if (guess && precond != 0) {
    BUF(double, io_guess, (size_t)B * N * nx);
    HIP_OK(hipMemcpyAsync(io_guess, guess, sizeof(double) * B * N * nx, hipMemcpyHostToDevice, ctx->stream));
    w.guess = io_guess;
  }
  // soft limits: the QP of formKKTSystemBlocks carries their jacobian terms (:220-225, :255-259) at the
  // context's soft state (tmpc_set_soft_state; defaults if it was never set for this B, N)
  if (ctx->hlim.any) {
    double *smu = nullptr, *slam = nullptr, *sphi = nullptr;
    if ((rc = alloc_soft(ctx, B, N, &smu, &slam, &sphi))) return rc;
    if (ctx->soft_B != B || ctx->soft_N != N) {
      launch_soft_init(ctx->stream, ctx->dlim, (size_t)B * N * 6 * nj, 6 * nj, smu, slam, sphi);
      HIP_OK(hipGetLastError());
      ctx->soft_B = B;
      ctx->soft_N = N;
    }
    BUF(double, soft_Gk, (size_t)B * N * (nx * nx + nj * nj));
    BUF(double, soft_j, (size_t)B * N * (nx + nj));
    w.Gk = soft_Gk;
    w.jsoft = soft_j;
    w.smu = smu;
    w.slam = slam;
  }
  // hard box constraints: the QP with the knots' constraint rows (tmpc_hard.hip); the lambda part of
  // dxul then holds the multipliers of the N nx dynamics / initial-state rows, in knot order
  HardArgs hard{};
  if (banded) {
    if ((rc = setup_hard(ctx, B, N, 0, precond, hard))) return rc;
    w.hard = &hard;
  }
  ctx->hard_last = {0, 0, 0, 0, 0};
  if ((rc = run_qp(ctx, B, N, dt, precond, io_x, io_u, st, w, !banded, PList{nullptr, nullptr}, B)))
    return rc;
  HIP_OK(hipStreamSynchronize(ctx->stream));
  if (banded) {
    if ((rc = collect_hard_work(ctx, hard))) return rc;
    ctx->hard_last = {B, N, hard.dmax, hard.W, hard.rmax};
    std::vector<int> roff((size_t)B * N);
    std::vector<double> lh((size_t)B * hard.dmax);
    HIP_OK(hipMemcpy(roff.data(), hard.roff, roff.size() * sizeof(int), hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(lh.data(), hard.lam, lh.size() * sizeof(double), hipMemcpyDeviceToHost));
    std::vector<double> lr((size_t)B * N * nx);
    for (int b = 0; b < B; ++b)
      for (int j = 0; j < N; ++j)
        for (int i = 0; i < nx; ++i) lr[((size_t)b * N + j) * nx + i] = lh[(size_t)b * hard.dmax + roff[(size_t)b * N + j] + i];
    HIP_OK(hipMemcpy(w.lam, lr.data(), lr.size() * sizeof(double), hipMemcpyHostToDevice));
  }
  resolve_timings(ctx);
  if (dxul) {
    std::vector<double> dx((size_t)B * N * nx), du((size_t)B * K * nj), lam((size_t)B * N * nx);
    HIP_OK(hipMemcpy(dx.data(), w.dx, dx.size() * sizeof(double), hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(du.data(), w.du, du.size() * sizeof(double), hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(lam.data(), w.lam, lam.size() * sizeof(double), hipMemcpyDeviceToHost));
    const size_t L = (size_t)nxu * K + nx + (size_t)nx * N;
    for (int b = 0; b < B; ++b) {
      double* o = dxul + b * L;
      for (int k = 0; k < N; ++k) {
        for (int i = 0; i < nx; ++i) o[(size_t)k * nxu + i] = dx[((size_t)b * N + k) * nx + i];
        if (k < K)
          for (int i = 0; i < nj; ++i) o[(size_t)k * nxu + nx + i] = du[((size_t)b * K + k) * nj + i];
      }
      memcpy(o + (size_t)nxu * K + nx, lam.data() + (size_t)b * N * nx, sizeof(double) * N * nx);
    }
  }
  if (pcg_iters) HIP_OK(hipMemcpy(pcg_iters, w.iters, sizeof(int) * B, hipMemcpyDeviceToHost));
  if (S_diag) HIP_OK(hipMemcpy(S_diag, w.Sd, sizeof(double) * B * N * nx * nx, hipMemcpyDeviceToHost));
  if (S_lo) HIP_OK(hipMemcpy(S_lo, w.Sl, sizeof(double) * B * K * nx * nx, hipMemcpyDeviceToHost));
  if (gamma) HIP_OK(hipMemcpy(gamma, w.gam, sizeof(double) * B * N * nx, hipMemcpyDeviceToHost));
  if (P_diag && precond != PRECOND_J && precond != 0)
    HIP_OK(hipMemcpy(P_diag, w.Pd, sizeof(double) * B * N * nx * nx, hipMemcpyDeviceToHost));
  return 0;
}

int tmpc_qp_blocks_batch(tmpc_ctx* ctx, int B, int N, int nx, int nu, int linsys, const double* G, const double* g,
                         const double* A, const double* Bm, const double* c, const double* rho, const double* guess,
                         double* dxul, int32_t* pcg_iters, double* S_diag, double* S_lo, double* gamma) {
  if (!ctx) return -1;
  if (B < 1 || N < 2) return fail(ctx, "bad sizes B=%d N=%d (B >= 1, N >= 2)", B, N);
  if (nu < 1 || nu > 7 || nx != 2 * nu)
    return fail(ctx, "tmpc_qp_blocks_batch: nx = %d, nu = %d; the device QP takes nx = 2 nu, 1 <= nu <= 7", nx, nu);
  if (N * nx > 1024) return fail(ctx, "tmpc_qp_blocks_batch: N * nx = %d exceeds 1024 rows", N * nx);
  const int precond = precond_of(linsys);
  if (precond < 0) return fail(ctx, "linear system method %d is not available on the GPU", linsys);
  if (!G || !g || !A || !Bm || !c || !rho) return fail(ctx, "null input");
  hipSetDevice(ctx->device);
  const int n = nx + nu, K = N - 1;
  BUF(double, hb_G, (size_t)B * N * n * n);
  BUF(double, hb_Gh, (size_t)B * N * n * n);
  BUF(double, hb_g, (size_t)B * N * n);
  BUF(double, hb_A, (size_t)B * K * nx * nx);
  BUF(double, hb_B, (size_t)B * K * nx * nu);
  BUF(double, hb_c, (size_t)B * N * nx);
  BUF(double, hb_rho, (size_t)B);
  BUF(int, hb_err, (size_t)B);
  BUF(int, hb_it, (size_t)B);
  BUF(double, hb_dx, (size_t)B * N * nx);
  BUF(double, hb_du, (size_t)B * K * nu);
  BUF(double, hb_lam, (size_t)B * N * nx);
  BUF(double, hb_Sd, (size_t)B * N * nx * nx);
  BUF(double, hb_Sl, (size_t)B * K * nx * nx);
  BUF(double, hb_gam, (size_t)B * N * nx);
  double* hb_guess = nullptr;
  if (guess && precond != 0) {
    BUF(double, hb_x0, (size_t)B * N * nx);
    HIP_OK(hipMemcpyAsync(hb_x0, guess, sizeof(double) * B * N * nx, hipMemcpyHostToDevice, ctx->stream));
    hb_guess = hb_x0;
  }
  HIP_OK(hipMemcpyAsync(hb_G, G, sizeof(double) * B * N * n * n, hipMemcpyHostToDevice, ctx->stream));
  HIP_OK(hipMemcpyAsync(hb_g, g, sizeof(double) * B * N * n, hipMemcpyHostToDevice, ctx->stream));
  HIP_OK(hipMemcpyAsync(hb_A, A, sizeof(double) * B * K * nx * nx, hipMemcpyHostToDevice, ctx->stream));
  HIP_OK(hipMemcpyAsync(hb_B, Bm, sizeof(double) * B * K * nx * nu, hipMemcpyHostToDevice, ctx->stream));
  HIP_OK(hipMemcpyAsync(hb_c, c, sizeof(double) * B * N * nx, hipMemcpyHostToDevice, ctx->stream));
  HIP_OK(hipMemcpyAsync(hb_rho, rho, sizeof(double) * B, hipMemcpyHostToDevice, ctx->stream));
  HIP_OK(hipMemsetAsync(hb_err, 0, sizeof(int) * B, ctx->stream));
  {
    Timed t(ctx, "ghat_full");
    LAUNCH_OK(launch_ghat_full(ctx->stream, nu, B, N, hb_G, hb_rho, hb_Gh, hb_err));
  }
  const double tol = ctx->opts.exit_tolerance_linSys;
  const int max_iter = ctx->opts.max_iter_linSys;
  const bool keep = S_diag || S_lo || gamma;
  if (precond == 0) {   // methods S / N: Schur blocks -> block-Thomas -> dxu
    std::vector<int> act(B, 1);
    BUF(int, hb_act, (size_t)B);
    BUF(double, hb_U, (size_t)B * K * nx * nx);
    BUF(double, hb_Y, (size_t)B * N * nx);
    HIP_OK(hipMemcpyAsync(hb_act, act.data(), sizeof(int) * B, hipMemcpyHostToDevice, ctx->stream));
    {
      Timed t(ctx, "qp_blocks_schur");
      LAUNCH_OK(launch_qp_blocks(ctx->stream, nu, B, N, PRECOND_SS, QP_MODE_SCHUR, hb_Gh, hb_g, hb_A, hb_B, hb_c,
                                 hb_err, tol, max_iter, nullptr, hb_it, hb_dx, hb_du, hb_lam, hb_Sd, hb_Sl, hb_gam));
    }
    {
      Timed t(ctx, "btsolve");
      LAUNCH_OK(launch_btsolve(ctx->stream, nx, B, N, hb_act, hb_Sd, hb_Sl, hb_gam, hb_U, hb_Y, hb_lam));
    }
    {
      Timed t(ctx, "qp_blocks_dxu");
      LAUNCH_OK(launch_qp_blocks(ctx->stream, nu, B, N, PRECOND_SS, QP_MODE_DXU, hb_Gh, hb_g, hb_A, hb_B, hb_c,
                                 hb_err, tol, max_iter, nullptr, hb_it, hb_dx, hb_du, hb_lam, nullptr, nullptr,
                                 nullptr));
    }
  } else {
    Timed t(ctx, "qp_blocks");
    LAUNCH_OK(launch_qp_blocks(ctx->stream, nu, B, N, precond, QP_MODE_PCG, hb_Gh, hb_g, hb_A, hb_B, hb_c, hb_err,
                               tol, max_iter, hb_guess, hb_it, hb_dx, hb_du, hb_lam, keep ? hb_Sd : nullptr,
                               keep ? hb_Sl : nullptr, keep ? hb_gam : nullptr));
  }
  HIP_OK(hipStreamSynchronize(ctx->stream));
  resolve_timings(ctx);
  std::vector<int> err(B);
  HIP_OK(hipMemcpy(err.data(), hb_err, sizeof(int) * B, hipMemcpyDeviceToHost));
  for (int b = 0; b < B; ++b)
    if (err[b])
      return fail(ctx, "problem %d: G_k + rho I has a zero or non-finite pivot (singular matrix, the reference's "
                  "np.linalg.inv raises LinAlgError)", b);
  std::vector<double> dx((size_t)B * N * nx), du((size_t)B * K * nu), lam((size_t)B * N * nx);
  HIP_OK(hipMemcpy(dx.data(), hb_dx, dx.size() * sizeof(double), hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(du.data(), hb_du, du.size() * sizeof(double), hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(lam.data(), hb_lam, lam.size() * sizeof(double), hipMemcpyDeviceToHost));
  if (dxul) {
    const size_t L = (size_t)n * K + nx + (size_t)nx * N;
    for (int b = 0; b < B; ++b) {
      double* o = dxul + b * L;
      for (int k = 0; k < N; ++k) {
        for (int i = 0; i < nx; ++i) o[(size_t)k * n + i] = dx[((size_t)b * N + k) * nx + i];
        if (k < K)
          for (int i = 0; i < nu; ++i) o[(size_t)k * n + nx + i] = du[((size_t)b * K + k) * nu + i];
      }
      memcpy(o + (size_t)n * K + nx, lam.data() + (size_t)b * N * nx, sizeof(double) * N * nx);
    }
  }
  if (pcg_iters) HIP_OK(hipMemcpy(pcg_iters, hb_it, sizeof(int) * B, hipMemcpyDeviceToHost));
  if (S_diag) HIP_OK(hipMemcpy(S_diag, hb_Sd, sizeof(double) * B * N * nx * nx, hipMemcpyDeviceToHost));
  if (S_lo) HIP_OK(hipMemcpy(S_lo, hb_Sl, sizeof(double) * B * K * nx * nx, hipMemcpyDeviceToHost));
  if (gamma) HIP_OK(hipMemcpy(gamma, hb_gam, sizeof(double) * B * N * nx, hipMemcpyDeviceToHost));
  return 0;
}

int tmpc_qp_blocks_banded_batch(tmpc_ctx* ctx, int B, int N, int nx, int nu, int linsys, const double* G,
                                const double* g, const double* A, const double* Bm, const double* c,
                                const int32_t* hcnt, const int32_t* hcol, const double* hsgn, const double* hval,
                                int rmax, const double* rho, double* dxul, int32_t* pcg_iters, double* lambda_hard,
                                int32_t* singular) {
  if (!ctx) return -1;
  if (B < 1 || N < 2) return fail(ctx, "bad sizes B=%d N=%d (B >= 1, N >= 2)", B, N);
  if (nu < 1 || nu > 7 || nx != 2 * nu)
    return fail(ctx, "tmpc_qp_blocks_banded_batch: nx = %d, nu = %d; the device QP takes nx = 2 nu, 1 <= nu <= 7",
                nx, nu);
  const int n = nx + nu, K = N - 1;
  if (rmax < 0 || rmax > 2 * n) return fail(ctx, "tmpc_qp_blocks_banded_batch: rmax = %d (0..%d)", rmax, 2 * n);
  const int precond = precond_of(linsys);
  if (precond < 0) return fail(ctx, "linear system method %d is not available on the GPU", linsys);
  if (!G || !g || !A || !Bm || !c || !rho || (rmax > 0 && (!hcnt || !hcol || !hsgn || !hval)))
    return fail(ctx, "null input");
  const int rbuf = rmax > 0 ? rmax : 1;
  std::vector<int> cnt((size_t)B * N, 0);
  if (rmax > 0) memcpy(cnt.data(), hcnt, sizeof(int) * B * N);
  for (size_t e = 0; e < cnt.size(); ++e) {
    if (cnt[e] < 0 || cnt[e] > rmax) return fail(ctx, "hard rows: %d rows at (problem, knot) %zu (0..%d)", cnt[e], e, rmax);
    for (int r = 0; r < cnt[e]; ++r) {
      const int col = hcol[e * rmax + r];
      const double sg = hsgn[e * rmax + r];
      const int k = (int)(e % N);
      if (col < 0 || col >= (k < K ? n : nx) || !(sg == 1.0 || sg == -1.0 || sg == 0.0))
        return fail(ctx, "hard row %d at (problem, knot) %zu: column %d, sign %g -- the banded QP takes box rows "
                    "(+-1 or 0 times one entry of [x_k; u_k])", r, e, col, sg);
      if (sg == 0.0 && precond != 0)
        return fail(ctx, "FULL_SET box constraints with a PCG method: the inactive rows of C are zero, so S is "
                    "singular and the reference's preconditioner raises LinAlgError (PCG.py:168-188); use method S");
    }
  }
  hipSetDevice(ctx->device);
  BUF(double, hb_G, (size_t)B * N * n * n);
  BUF(double, hb_Gh, (size_t)B * N * n * n);
  BUF(double, hb_g, (size_t)B * N * n);
  BUF(double, hb_A, (size_t)B * K * nx * nx);
  BUF(double, hb_B, (size_t)B * K * nx * nu);
  BUF(double, hb_c, (size_t)B * N * nx);
  BUF(double, hb_rho, (size_t)B);
  BUF(int, hb_err, (size_t)B);
  BUF(int, hb_it, (size_t)B);
  BUF(int, hb_act, (size_t)B);
  BUF(double, hb_dx, (size_t)B * N * nx);
  BUF(double, hb_du, (size_t)B * K * nu);
  HIP_OK(hipMemcpyAsync(hb_G, G, sizeof(double) * B * N * n * n, hipMemcpyHostToDevice, ctx->stream));
  HIP_OK(hipMemcpyAsync(hb_g, g, sizeof(double) * B * N * n, hipMemcpyHostToDevice, ctx->stream));
  HIP_OK(hipMemcpyAsync(hb_A, A, sizeof(double) * B * K * nx * nx, hipMemcpyHostToDevice, ctx->stream));
  HIP_OK(hipMemcpyAsync(hb_B, Bm, sizeof(double) * B * K * nx * nu, hipMemcpyHostToDevice, ctx->stream));
  HIP_OK(hipMemcpyAsync(hb_c, c, sizeof(double) * B * N * nx, hipMemcpyHostToDevice, ctx->stream));
  HIP_OK(hipMemcpyAsync(hb_rho, rho, sizeof(double) * B, hipMemcpyHostToDevice, ctx->stream));
  HIP_OK(hipMemsetAsync(hb_err, 0, sizeof(int) * B, ctx->stream));
  HIP_OK(hipMemsetAsync(hb_it, 0, sizeof(int) * B, ctx->stream));
  std::vector<int> act(B, 1);
  HIP_OK(hipMemcpyAsync(hb_act, act.data(), sizeof(int) * B, hipMemcpyHostToDevice, ctx->stream));
  {
    Timed t(ctx, "ghat_full");
    LAUNCH_OK(launch_ghat_full(ctx->stream, nu, B, N, hb_G, hb_rho, hb_Gh, hb_err));
  }
  HardArgs hard{};
  int rc = setup_hard(ctx, B, N, 0, precond, hard, nu, rmax);
  if (rc) return rc;
  HIP_OK(hipMemcpyAsync(hard.cnt, cnt.data(), sizeof(int) * B * N, hipMemcpyHostToDevice, ctx->stream));
  // the per-knot active-set bitmasks (tmpc_qp_hard_info), bit t * 2 nu + e of the box row over [q; qd; u]
  // and each row's slot t * 2 nu + e (the lambda_hard layout)
  std::vector<unsigned long long> amask((size_t)B * N, 0ull);
  std::vector<int> hslot((size_t)B * N * std::max(rmax, 1), 0);
  for (size_t e = 0; e < amask.size(); ++e)
    for (int r = 0; r < cnt[e]; ++r) {
      const double sg = hsgn[e * rmax + r];
      const int col = hcol[e * rmax + r], t = col / nu, i = col % nu;
      hslot[e * rmax + r] = t * 2 * nu + (sg >= 0.0 ? i : nu + i);
      if (sg != 0.0) amask[e] |= 1ull << hslot[e * rmax + r];
    }
  HIP_OK(hipMemcpyAsync(hard.amask, amask.data(), sizeof(unsigned long long) * B * N, hipMemcpyHostToDevice,
                        ctx->stream));
  if (rmax > 0)
    HIP_OK(hipMemcpyAsync(hard.hslot, hslot.data(), sizeof(int) * B * N * rmax, hipMemcpyHostToDevice, ctx->stream));
  if (rmax > 0) {
    HIP_OK(hipMemcpyAsync(hard.hcol, hcol, sizeof(int) * B * N * rbuf, hipMemcpyHostToDevice, ctx->stream));
    HIP_OK(hipMemcpyAsync(hard.hsgn, hsgn, sizeof(double) * B * N * rbuf, hipMemcpyHostToDevice, ctx->stream));
    HIP_OK(hipMemcpyAsync(hard.hval, hval, sizeof(double) * B * N * rbuf, hipMemcpyHostToDevice, ctx->stream));
  }
  hard.rows_given = 1;
  hard.precond = precond;
  hard.Ghat = hb_Gh;
  hard.per_knot = 2;
  hard.gvec = hb_g;
  hard.A = hb_A;
  hard.Bm = hb_B;
  hard.cvec = hb_c;
  hard.x = hb_g;   // not read: the gradient is the caller's (gvec), the rows are given
  hard.u = hb_g;
  hard.jsoft = nullptr;
  hard.active = hb_act;
  hard.iters = hb_it;
  hard.dx = hb_dx;
  hard.du = hb_du;
  hard.tol = ctx->opts.exit_tolerance_linSys;
  hard.max_iter = ctx->opts.max_iter_linSys;
  const char* names[3] = {"hard_schur", precond == 0 ? "hard_direct" : "hard_pcg", "dxu"};
  for (int ph = 0; ph < 3; ++ph) {
    Timed t(ctx, names[ph]);
    hard.phase = ph;
    LAUNCH_OK(launch_hard(ctx->stream, nu, hard));
  }
  HIP_OK(hipStreamSynchronize(ctx->stream));
  if ((rc = collect_hard_work(ctx, hard))) return rc;
  resolve_timings(ctx);
  std::vector<int> err(B);
  HIP_OK(hipMemcpy(err.data(), hb_err, sizeof(int) * B, hipMemcpyDeviceToHost));
  for (int b = 0; b < B; ++b)
    if (err[b])
      return fail(ctx, "problem %d: G_k + rho I has a zero or non-finite pivot (singular matrix, the reference's "
                  "np.linalg.inv raises LinAlgError)", b);
  std::vector<int> roff((size_t)B * N), hoff((size_t)B * N);
  std::vector<double> lh((size_t)B * hard.dmax);
  HIP_OK(hipMemcpy(roff.data(), hard.roff, roff.size() * sizeof(int), hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(hoff.data(), hard.hoff, hoff.size() * sizeof(int), hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(lh.data(), hard.lam, lh.size() * sizeof(double), hipMemcpyDeviceToHost));
  if (dxul) {
    std::vector<double> dx((size_t)B * N * nx), du((size_t)B * K * nu);
    HIP_OK(hipMemcpy(dx.data(), hb_dx, dx.size() * sizeof(double), hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(du.data(), hb_du, du.size() * sizeof(double), hipMemcpyDeviceToHost));
    const size_t L = (size_t)n * K + nx + (size_t)nx * N;
    for (int b = 0; b < B; ++b) {
      double* o = dxul + b * L;
      for (int k = 0; k < N; ++k) {
        for (int i = 0; i < nx; ++i) o[(size_t)k * n + i] = dx[((size_t)b * N + k) * nx + i];
        if (k < K)
          for (int i = 0; i < nu; ++i) o[(size_t)k * n + nx + i] = du[((size_t)b * K + k) * nu + i];
        for (int i = 0; i < nx; ++i)
          o[(size_t)n * K + nx + (size_t)k * nx + i] = lh[(size_t)b * hard.dmax + roff[(size_t)b * N + k] + i];
      }
    }
  }
  if (lambda_hard)
    for (int b = 0; b < B; ++b)
      for (int k = 0; k < N; ++k)
        for (int r = 0; r < rbuf; ++r)
          lambda_hard[((size_t)b * N + k) * rbuf + r] =
              r < cnt[(size_t)b * N + k] ? lh[(size_t)b * hard.dmax + hoff[(size_t)b * N + k] + r] : 0.0;
  if (pcg_iters) HIP_OK(hipMemcpy(pcg_iters, hb_it, sizeof(int) * B, hipMemcpyDeviceToHost));
  if (singular) HIP_OK(hipMemcpy(singular, hard.sing, sizeof(int) * B, hipMemcpyDeviceToHost));
  ctx->hard_last = {B, N, hard.dmax, hard.W, hard.rmax};   // tmpc_qp_hard_info reads this QP's S band and gamma
  return 0;
}

int tmpc_qp_hard_info(tmpc_ctx* ctx, int B, int N, int32_t* sizes, int32_t* dim, uint64_t* active,
                      double* lambda_hard, double* S_band, double* gamma, int32_t* singular) {
  if (!ctx) return -1;
  const auto& hl = ctx->hard_last;
  if (hl.B == 0)
    return fail(ctx, "tmpc_qp_hard_info: the last tmpc_qp_batch did not take the banded path (hard box limits, or "
                "N * nx past %d rows)", QP_MAX_ROWS);
  if (hl.B != B || hl.N != N)
    return fail(ctx, "tmpc_qp_hard_info: the last hard-limit QP was B=%d N=%d, asked for B=%d N=%d", hl.B, hl.N, B, N);
  hipSetDevice(ctx->device);
  const int nj = ctx->hmodel.n, S6 = 6 * nj;
  if (sizes) {
    sizes[0] = hl.dmax;
    sizes[1] = hl.W;
  }
  auto dev = [&](const char* name) { return ctx->bufs[name].ptr; };
  if (dim) HIP_OK(hipMemcpy(dim, dev("hd_dim"), sizeof(int) * B, hipMemcpyDeviceToHost));
  if (active) HIP_OK(hipMemcpy(active, dev("hd_amask"), sizeof(uint64_t) * B * N, hipMemcpyDeviceToHost));
  if (singular) HIP_OK(hipMemcpy(singular, dev("hd_sing"), sizeof(int) * B, hipMemcpyDeviceToHost));
  const size_t BW = 2 * (size_t)hl.W + 1;
  if (S_band) {
    // device: row-start-relative [B][2W+1][dmax] (entry j of row a = column rng_a + j, tmpc_hard.hip),
    // written only inside each row's structural range (k_hard_schur); the ABI's band is row-major
    // [B][dmax][2W+1] (column c at a - W + o), zero outside the ranges
    std::vector<double> sbt((size_t)B * hl.dmax * BW);
    HIP_OK(hipMemcpy(sbt.data(), dev("hd_Sb"), sizeof(double) * sbt.size(), hipMemcpyDeviceToHost));
    std::vector<int> rg((size_t)B * hl.dmax * 2), dm(B);
    HIP_OK(hipMemcpy(rg.data(), dev("hd_rng"), rg.size() * sizeof(int), hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(dm.data(), dev("hd_dim"), B * sizeof(int), hipMemcpyDeviceToHost));
    for (int b = 0; b < B; ++b)
      for (int a = 0; a < hl.dmax; ++a) {
        double* row = S_band + ((size_t)b * hl.dmax + a) * BW;
        const int* r = rg.data() + ((size_t)b * hl.dmax + a) * 2;
        for (size_t o = 0; o < BW; ++o) {
          const int c = a - hl.W + (int)o;
          row[o] = (a >= dm[b] || c < r[0] || c > r[1]) ? 0.0 : sbt[((size_t)b * BW + (c - r[0])) * hl.dmax + a];
        }
      }
  }
  if (gamma) HIP_OK(hipMemcpy(gamma, dev("hd_gam"), sizeof(double) * B * hl.dmax, hipMemcpyDeviceToHost));
  if (lambda_hard) {
    // the hard rows' multipliers by slot t * 2n + e (0 where the slot has no row); rmax as hd_slot was laid out
    const int rmax = hl.rmax;
    std::vector<int> cnt((size_t)B * N), hoff((size_t)B * N), slot((size_t)B * N * rmax);
    std::vector<double> lam((size_t)B * hl.dmax);
    HIP_OK(hipMemcpy(cnt.data(), dev("hd_cnt"), cnt.size() * sizeof(int), hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(hoff.data(), dev("hd_hoff"), hoff.size() * sizeof(int), hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(slot.data(), dev("hd_slot"), slot.size() * sizeof(int), hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(lam.data(), dev("hd_lam"), lam.size() * sizeof(double), hipMemcpyDeviceToHost));
    memset(lambda_hard, 0, sizeof(double) * B * N * S6);
    for (int b = 0; b < B; ++b)
      for (int k = 0; k < N; ++k) {
        const size_t bk = (size_t)b * N + k;
        for (int r = 0; r < cnt[bk] && r < rmax; ++r) {
          const int sl = slot[bk * rmax + r];
          if (sl >= 0 && sl < S6) lambda_hard[bk * S6 + sl] = lam[(size_t)b * hl.dmax + hoff[bk] + r];
        }
      }
  }
  return 0;
}

int tmpc_hard_pcg_batch(tmpc_ctx* ctx, int B, int nx, int dmax, int W, const int32_t* dim, int precond,
                        const double* S_band, const double* gamma, double tol, int max_iter, double* lambda,
                        int32_t* iters) {
  if (!ctx) return -1;
  if (B < 1 || nx < 2 || nx > 14 || (nx & 1) || dmax < 1 || W < 0 || W > 1024)
    return fail(ctx, "bad sizes B=%d nx=%d dmax=%d W=%d", B, nx, dmax, W);
  if (precond != PRECOND_J && precond != PRECOND_BJ && precond != PRECOND_SS && precond != PRECOND_NONE)
    return fail(ctx, "preconditioner %d: valid are J=1, BJ=2, SS=3, 0=4 (PCG.py:52-55)", precond);
  if (dmax > HARD_PCG_MAX_ROWS) return fail(ctx, "dmax = %d exceeds the PCG's %d rows", dmax, HARD_PCG_MAX_ROWS);
  if (max_iter < 0) return fail(ctx, "max_iter must be >= 0");
  if (!dim || !S_band || !gamma) return fail(ctx, "null input");
  for (int b = 0; b < B; ++b)
    if (dim[b] < 1 || dim[b] > dmax) return fail(ctx, "dim[%d] = %d outside [1, %d]", b, dim[b], dmax);
  hipSetDevice(ctx->device);
  const size_t BW = 2 * (size_t)W + 1, nbmax = dmax / nx + 1;
  BUF(double, hp_Sb, (size_t)B * dmax * BW);
  BUF(double, hp_gam, (size_t)B * dmax);
  BUF(double, hp_lam, (size_t)B * dmax);
  BUF(int, hp_dim, (size_t)B);
  BUF(int, hp_act, (size_t)B);
  BUF(int, hp_it, (size_t)B);
  BUF(double, hp_Pd, (size_t)B * nbmax * nx * nx);
  BUF(double, hp_Pl, (size_t)B * nbmax * nx * nx);
  BUF(double, hp_Ptr, (size_t)B * nbmax * nx * nx);
  BUF(int, hp_rng, (size_t)B * dmax * 2);
  // each row's first / last nonzero column: the range the kernel's products visit (tmpc_hard.hip)
  std::vector<int> rg((size_t)B * dmax * 2);
  for (int b = 0; b < B; ++b)
    for (int a = 0; a < dmax; ++a) {
      const double* row = S_band + ((size_t)b * dmax + a) * BW;
      int lo = a, hi = a;
      for (size_t o = 0; o < BW; ++o) {
        const int c = a - W + (int)o;
        if (c < 0 || c >= dim[b] || row[o] == 0.0) continue;
        lo = std::min(lo, c);
        hi = std::max(hi, c);
      }
      rg[((size_t)b * dmax + a) * 2] = lo;
      rg[((size_t)b * dmax + a) * 2 + 1] = hi;
    }
  HIP_OK(hipMemcpyAsync(hp_rng, rg.data(), rg.size() * sizeof(int), hipMemcpyHostToDevice, ctx->stream));
  // the device band is row-start-relative ([B][2W+1][dmax], entry j of row a = column rg_a + j,
  // tmpc_hard.hip); the ABI's is row-major [B][dmax][2W+1]
  std::vector<double> sbt((size_t)B * dmax * BW, 0.0);
  for (int b = 0; b < B; ++b)
    for (int a = 0; a < dmax; ++a) {
      const int lo = rg[((size_t)b * dmax + a) * 2], hi = rg[((size_t)b * dmax + a) * 2 + 1];
      for (int c = lo; c <= hi; ++c)
        sbt[((size_t)b * BW + (c - lo)) * dmax + a] = S_band[((size_t)b * dmax + a) * BW + (c - a + W)];
    }
  HIP_OK(hipMemcpy(hp_Sb, sbt.data(), sizeof(double) * B * dmax * BW, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpyAsync(hp_gam, gamma, sizeof(double) * B * dmax, hipMemcpyHostToDevice, ctx->stream));
  HIP_OK(hipMemcpyAsync(hp_dim, dim, sizeof(int) * B, hipMemcpyHostToDevice, ctx->stream));
  std::vector<int> ones(B, 1);
  HIP_OK(hipMemcpyAsync(hp_act, ones.data(), sizeof(int) * B, hipMemcpyHostToDevice, ctx->stream));
  HardArgs h{};
  h.B = B;
  h.phase = 1;
  h.precond = precond;
  h.dmax = dmax;
  h.W = W;
  h.tol = tol;
  h.max_iter = max_iter;
  h.active = hp_act;
  h.dim = hp_dim;
  h.Sb = hp_Sb;
  h.gam = hp_gam;
  h.Pd = hp_Pd;
  h.Pl = hp_Pl;
  h.Ptr = hp_Ptr;
  h.lam = hp_lam;
  h.iters = hp_it;
  h.rng = hp_rng;
  int rc;
  BUF(double, hp_work, (size_t)B);
  HIP_OK(hipMemsetAsync(hp_work, 0, sizeof(double) * B, ctx->stream));
  h.work = hp_work;
  {
    Timed t(ctx, "hard_pcg");
    LAUNCH_OK(launch_hard(ctx->stream, nx / 2, h));
  }
  if ((rc = collect_hard_work(ctx, h))) return rc;
  resolve_timings(ctx);
  if (lambda) HIP_OK(hipMemcpy(lambda, hp_lam, sizeof(double) * B * dmax, hipMemcpyDeviceToHost));
  if (iters) HIP_OK(hipMemcpy(iters, hp_it, sizeof(int) * B, hipMemcpyDeviceToHost));
  return 0;
}

int tmpc_pcg_batch(tmpc_ctx* ctx, int B, int N, int nx, int precond, const double* S_diag, const double* S_lo,
                   const double* S_up, const double* gamma, const double* guess, double tol, int max_iter,
                   double* lambda,
                   int32_t* iters, double* trace_nu, double* trace_res, double* P_diag) {
  if (!ctx) return -1;
  if (B < 1 || N < 1 || nx < 1) return fail(ctx, "bad sizes B=%d N=%d nx=%d", B, N, nx);
  if (N * nx > 1024) return fail(ctx, "N * nx = %d exceeds 1024 rows", N * nx);
  if (precond != PRECOND_J && precond != PRECOND_BJ && precond != PRECOND_SS && precond != PRECOND_NONE)
    return fail(ctx, "preconditioner %d: valid are J=1, BJ=2, SS=3, 0=4 (PCG.py:52-55)", precond);
  if (max_iter < 0) return fail(ctx, "max_iter must be >= 0");
  if (!S_diag || !gamma || (N > 1 && !S_lo)) return fail(ctx, "null input");
  hipSetDevice(ctx->device);
  const int K = N - 1;
  BUF(double, p_Sd, (size_t)B * N * nx * nx);
  BUF(double, p_Sl, (size_t)B * (K > 0 ? K : 1) * nx * nx);
  BUF(double, p_Su, (size_t)B * (K > 0 ? K : 1) * nx * nx);
  BUF(double, p_g, (size_t)B * N * nx);
  BUF(double, p_lam, (size_t)B * N * nx);
  BUF(int, p_it, (size_t)B);
  BUF(double, p_tn, (size_t)B * (max_iter + 1));
  BUF(double, p_tr, (size_t)B * (max_iter + 1));
  BUF(double, p_Pd, (size_t)B * N * nx * nx);
  BUF(double, p_x0, (size_t)B * N * nx);
  if (guess) HIP_OK(hipMemcpyAsync(p_x0, guess, sizeof(double) * B * N * nx, hipMemcpyHostToDevice, ctx->stream));
  HIP_OK(hipMemcpyAsync(p_Sd, S_diag, sizeof(double) * B * N * nx * nx, hipMemcpyHostToDevice, ctx->stream));
  if (K > 0) HIP_OK(hipMemcpyAsync(p_Sl, S_lo, sizeof(double) * B * K * nx * nx, hipMemcpyHostToDevice, ctx->stream));
  if (K > 0 && S_up)
    HIP_OK(hipMemcpyAsync(p_Su, S_up, sizeof(double) * B * K * nx * nx, hipMemcpyHostToDevice, ctx->stream));
  HIP_OK(hipMemcpyAsync(p_g, gamma, sizeof(double) * B * N * nx, hipMemcpyHostToDevice, ctx->stream));
  {
    Timed t(ctx, "pcg");
    LAUNCH_OK(launch_pcg(ctx->stream, nx, B, N, precond, p_Sd, p_Sl, S_up ? p_Su : nullptr, p_g,
                         guess ? p_x0 : nullptr, tol,
                         max_iter, p_lam, p_it, trace_nu ? p_tn : nullptr, trace_res ? p_tr : nullptr,
                         P_diag ? p_Pd : nullptr));
  }
  HIP_OK(hipStreamSynchronize(ctx->stream));
  resolve_timings(ctx);
  if (lambda) HIP_OK(hipMemcpy(lambda, p_lam, sizeof(double) * B * N * nx, hipMemcpyDeviceToHost));
  if (iters) HIP_OK(hipMemcpy(iters, p_it, sizeof(int) * B, hipMemcpyDeviceToHost));
  if (trace_nu) HIP_OK(hipMemcpy(trace_nu, p_tn, sizeof(double) * B * (max_iter + 1), hipMemcpyDeviceToHost));
  if (trace_res) HIP_OK(hipMemcpy(trace_res, p_tr, sizeof(double) * B * (max_iter + 1), hipMemcpyDeviceToHost));
  if (P_diag && precond != PRECOND_J)
    HIP_OK(hipMemcpy(P_diag, p_Pd, sizeof(double) * B * N * nx * nx, hipMemcpyDeviceToHost));
  return 0;
}

int tmpc_pcg_dense_batch(tmpc_ctx* ctx, int B, int D, const double* A, const double* b, const double* Pinv,
                         int precond, int nx, const double* guess, double tol, int max_iter, double* x,
                         int32_t* iters, double* trace_nu, double* trace_res, double* Pinv_out) {
  if (!ctx) return -1;
  if (B < 1 || D < 1 || (size_t)B * D * D > ((size_t)1 << 34))
    return fail(ctx, "bad sizes B=%d D=%d (the dense PCG takes D >= 1 and B D^2 <= 2^34 entries)", B, D);
  if (!A || !b) return fail(ctx, "null input");
  if (max_iter < 0) return fail(ctx, "max_iter must be >= 0");
  if (!Pinv) {
    if (precond != PRECOND_J && precond != PRECOND_BJ && precond != PRECOND_SS && precond != PRECOND_NONE)
      return fail(ctx, "preconditioner %d: valid are J=1, BJ=2, SS=3, 0=4 (PCG.py:52-55)", precond);
    if ((precond == PRECOND_BJ || precond == PRECOND_SS) && (nx < 1 || nx > 16))
      return fail(ctx, "block size %d: the device preconditioner takes 1..16", nx);
  }
  hipSetDevice(ctx->device);
  const size_t DD = (size_t)B * D * D;
  BUF(double, dn_stage, DD);
  BUF(double, dn_AT, DD);
  BUF(double, dn_PT, DD);
  BUF(double, dn_b, (size_t)B * D);
  BUF(double, dn_x0, (size_t)B * D);
  BUF(double, dn_x, (size_t)B * D);
  BUF(int, dn_it, (size_t)B);
  BUF(double, dn_tn, (size_t)B * (max_iter + 1));
  BUF(double, dn_tr, (size_t)B * (max_iter + 1));
  const int nbk = (!Pinv && (precond == PRECOND_BJ || precond == PRECOND_SS)) ? D / nx : 0;
  BUF(double, dn_Pd, (size_t)B * (nbk + 1) * (nx > 0 ? nx * nx : 1));
  DenseArgs a{};
  a.B = B;
  a.D = D;
  a.nx = nx;
  a.precond = precond;
  a.max_iter = max_iter;
  a.tol = tol;
  a.A = dn_stage;
  a.b = dn_b;
  a.guess = guess ? dn_x0 : nullptr;
  a.AT = dn_AT;
  a.PT = dn_PT;
  a.Pd = dn_Pd;
  a.x = dn_x;
  a.iters = dn_it;
  a.trace_nu = trace_nu ? dn_tn : nullptr;
  a.trace_res = trace_res ? dn_tr : nullptr;
  const bool big = D > HARD_PCG_MAX_ROWS;   // past the one-workgroup kernel's registers / LDS
  if (big) {
    BUF(double, dn_r, (size_t)B * D);
    BUF(double, dn_p, (size_t)B * D);
    BUF(double, dn_y, (size_t)B * D);
    BUF(double, dn_q, (size_t)B * D);
    BUF(double, dn_nu, (size_t)B);
    BUF(int, dn_done, (size_t)B);
    a.r = dn_r;
    a.p = dn_p;
    a.y = dn_y;
    a.q = dn_q;
    a.nu = dn_nu;
    a.done = dn_done;
  }
  HIP_OK(hipMemcpyAsync(dn_stage, A, sizeof(double) * DD, hipMemcpyHostToDevice, ctx->stream));
  HIP_OK(hipMemcpyAsync(dn_b, b, sizeof(double) * B * D, hipMemcpyHostToDevice, ctx->stream));
  if (guess) HIP_OK(hipMemcpyAsync(dn_x0, guess, sizeof(double) * B * D, hipMemcpyHostToDevice, ctx->stream));
  {
    Timed t(ctx, "pcg_dense");
    LAUNCH_OK(launch_dense_transpose(ctx->stream, B, D, dn_stage, dn_AT));
    if (Pinv) {
      HIP_OK(hipMemcpyAsync(dn_stage, Pinv, sizeof(double) * DD, hipMemcpyHostToDevice, ctx->stream));
      LAUNCH_OK(launch_dense_transpose(ctx->stream, B, D, dn_stage, dn_PT));
    } else {
      HIP_OK(hipMemsetAsync(dn_PT, 0, sizeof(double) * DD, ctx->stream));
      LAUNCH_OK(launch_dense_precond(ctx->stream, a));   // reads A row-major from the stage
    }
    if (big) LAUNCH_OK(launch_pcg_dense_big(ctx->stream, a));
    else LAUNCH_OK(launch_pcg_dense(ctx->stream, a));
  }
  HIP_OK(hipStreamSynchronize(ctx->stream));
  resolve_timings(ctx);
  if (x) HIP_OK(hipMemcpy(x, dn_x, sizeof(double) * B * D, hipMemcpyDeviceToHost));
  if (iters) HIP_OK(hipMemcpy(iters, dn_it, sizeof(int) * B, hipMemcpyDeviceToHost));
  if (trace_nu) HIP_OK(hipMemcpy(trace_nu, dn_tn, sizeof(double) * B * (max_iter + 1), hipMemcpyDeviceToHost));
  if (trace_res) HIP_OK(hipMemcpy(trace_res, dn_tr, sizeof(double) * B * (max_iter + 1), hipMemcpyDeviceToHost));
  if (Pinv_out) {   // Pinv = PT^T: back through the transpose, into the stage
    LAUNCH_OK(launch_dense_transpose(ctx->stream, B, D, dn_PT, dn_stage));
    HIP_OK(hipMemcpyAsync(Pinv_out, dn_stage, sizeof(double) * DD, hipMemcpyDeviceToHost, ctx->stream));
    HIP_OK(hipStreamSynchronize(ctx->stream));
  }
  return 0;
}

int tmpc_device_alloc(tmpc_ctx* ctx, size_t bytes, void** ptr) {
  if (!ctx || !ptr) return -1;
  hipSetDevice(ctx->device);
  HIP_OK(hipMalloc(ptr, bytes));
  return 0;
}

int tmpc_device_free(tmpc_ctx* ctx, void* ptr) {
  if (!ctx) return -1;
  hipSetDevice(ctx->device);
  HIP_OK(hipFree(ptr));
  return 0;
}

int tmpc_memcpy_h2d(tmpc_ctx* ctx, void* dst, const void* src, size_t bytes) {
  if (!ctx) return -1;
  hipSetDevice(ctx->device);
  HIP_OK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
  HIP_OK(hipStreamSynchronize(ctx->stream));
  return 0;
}

int tmpc_memcpy_d2h(tmpc_ctx* ctx, void* dst, const void* src, size_t bytes) {
  if (!ctx) return -1;
  hipSetDevice(ctx->device);
  HIP_OK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
  HIP_OK(hipStreamSynchronize(ctx->stream));
  return 0;
}

int tmpc_memcpy_d2d(tmpc_ctx* ctx, void* dst, const void* src, size_t bytes) {
  if (!ctx) return -1;
  hipSetDevice(ctx->device);
  HIP_OK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, ctx->stream));
  HIP_OK(hipStreamSynchronize(ctx->stream));
  return 0;
}

int tmpc_synchronize(tmpc_ctx* ctx) {
  if (!ctx) return -1;
  hipSetDevice(ctx->device);
  HIP_OK(hipStreamSynchronize(ctx->stream));
  resolve_timings(ctx);
  return 0;
}

int tmpc_kernel_stats(tmpc_ctx* ctx, const char* name, int64_t* launches, double* total_ms) {
  if (!ctx || !name) return -1;
  resolve_timings(ctx);
  auto it = ctx->stats.find(name);
  if (launches) *launches = it == ctx->stats.end() ? 0 : it->second.launches;
  if (total_ms) *total_ms = it == ctx->stats.end() ? 0.0 : it->second.total_ms;
  return 0;
}

int tmpc_kernel_bytes(tmpc_ctx* ctx, const char* name, double* bytes) {
  if (!ctx || !name || !bytes) return -1;
  if (std::string(name) != "hard_pcg") return fail(ctx, "kernel '%s' does not count its bytes (counting: hard_pcg)", name);
  auto it = ctx->kbytes.find(name);
  *bytes = it == ctx->kbytes.end() ? 0.0 : it->second;
  return 0;
}

int tmpc_solve_counters(tmpc_ctx* ctx, int64_t* counters) {
  if (!ctx || !counters) return -1;
  for (int i = 0; i < 4; ++i) counters[i] = ctx->last_counters[i];
  return 0;
}

int tmpc_reset_stats(tmpc_ctx* ctx) {
  if (!ctx) return -1;
  resolve_timings(ctx);
  ctx->stats.clear();
  ctx->kbytes.clear();
  return 0;
}

}  // extern "C"
