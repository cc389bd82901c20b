// Hand-written gfx950 kernels for the batched SQP Schur-complement + GBD-PCG
// solve of TrajoptMPCReference (TrajoptMPCReference.py:510-760 and
// GBD-PCG-Python/PCG.py), redesigned for MI355X:
//
//   * per-knot work (forward dynamics, analytic gradients, merit terms) maps
//     one lane to one (problem, knot) -- or (problem, knot, derivative column)
//     -- with the whole rigid-body state in VGPRs (tmpc_device.h);
//   * the PCG solve maps one workgroup to one problem and one lane to one row
//     of the block-tridiagonal Schur complement S; each lane keeps its rows of
//     S and of P^-1 in registers for all iterations, vectors are exchanged
//     through LDS and the two dot products per iteration are wave64
//     shuffle reductions + an LDS fan-in (fixed order: deterministic);
//   * per-problem control flow (line search, rho schedule, exit codes) is
//     data, not host branches: every kernel takes the per-problem state and
//     masks itself, the host only loops until no problem is active.
//
// Layouts (per problem b): x[b][i][k] (nx x N, the reference's column-per-knot
// C order), u[b][i][k] (nu x N-1); per-knot matrices row-major
// [b][k][r][c]; Schur blocks S_diag[b][k][i][j], S_lo[b][k][i][j] = S_{k+1,k}.
#include "tmpc_internal.h"
#include "tmpc_pcg.h"
#include "tmpc_copy.h"

namespace tmpc {

// ======================================================================= analytic M^-1 columns
// lane = (knot, col), col < NJ; writes the full symmetric matrix (column col
// above the diagonal and row col left of it, :908-930).  x is [K][NX] rows
// with row stride `xstride` per knot and element stride `estride`.
template <int NJ, bool CHAIN, class R, class MT>
__device__ __forceinline__ void minv_lane_store(const MT& M, const double q[NJ], int col,
                                                double* __restrict__ Mo) {
  R cq[NJ], sq[NJ], mc[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) joint_cs(M, j, R(q[j]), cq[j], sq[j]);
  minv_column<NJ, CHAIN>(M, cq, sq, col, mc);
#pragma unroll
  for (int r = 0; r < NJ; ++r) {
    if (r <= col) {
      Mo[r * NJ + col] = double(mc[r]);
      Mo[col * NJ + r] = double(mc[r]);
    }
  }
}

template <int NJ, bool CHAIN, class MT, class R>
__global__ void __launch_bounds__(256) k_qp_minv(MT M, PList P, int B, int N,
                                                 const double* __restrict__ x, const int* __restrict__ need,
                                                 double* __restrict__ minv_out) {
  constexpr int NX = 2 * NJ;
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int K = N - 1;
  if (gid >= B * K * NJ) return;
  const int col = gid % NJ;
  const int pk = gid / NJ;
  const int p = pk / K, k = pk - p * K;
  if (!P.has(p, B)) return;
  const int b = P.at(p);
  if (!need[b]) return;
  const size_t bk = (size_t)b * K + k;
  const double* xb = x + (size_t)b * NX * N;
  double q[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) q[j] = xb[j * N + k];
  minv_lane_store<NJ, CHAIN, R>(M, q, col, minv_out + (size_t)bk * NJ * NJ);
}

// ======================================================================= gradient columns -> A, B
// lane = (b, k, col), col < 2 NJ.  dqdd[:, col] = -Minv dc[:, col]
// (TrajoptPlant.py:313-316); A = I + dt [[0, I], [dqdd_q, dqdd_qd]],
// B = dt [[0], [Minv]] (TrajoptPlant.py:100-108).
template <int NJ, bool CHAIN, class R, class MT>
__device__ __forceinline__ void grad_lane_store(const MT& M, double dt, const double q[NJ],
                                                const double qd[NJ], const double qdd[NJ],
                                                const double* __restrict__ Mi, int col, double* __restrict__ A,
                                                double* __restrict__ Bm, double* __restrict__ dqdd) {
  constexpr int NX = 2 * NJ;
  R cq[NJ], sq[NJ], dc[NJ], qdr[NJ], qddr[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    joint_cs(M, j, R(q[j]), cq[j], sq[j]);
    qdr[j] = R(qd[j]);
    qddr[j] = R(qdd[j]);
  }
  const bool colqd = col >= NJ;
  rnea_grad_column<NJ, CHAIN>(M, cq, sq, qdr, qddr, colqd ? col - NJ : col, colqd, dc);
#pragma unroll
  for (int r = 0; r < NJ; ++r) {
    R accr = 0.0;
#pragma unroll
    for (int m = 0; m < NJ; ++m) accr += (-R(Mi[r * NJ + m])) * dc[m];
    const double acc = double(accr);
    if (dqdd) {
      dqdd[r * 3 * NJ + col] = acc;
      if (col < NJ) dqdd[r * 3 * NJ + NX + col] = Mi[r * NJ + col];
    }
    if (A) {
      A[r * NX + col] = (r == col ? 1.0 : 0.0) + dt * (col == NJ + r ? 1.0 : 0.0);
      A[(NJ + r) * NX + col] = (NJ + r == col ? 1.0 : 0.0) + dt * acc;
    }
    if (Bm && col < NJ) {
      Bm[r * NJ + col] = 0.0;
      Bm[(NJ + r) * NJ + col] = dt * Mi[r * NJ + col];
    }
  }
}

template <int NJ, bool CHAIN, class MT, class R>
__global__ void __launch_bounds__(256) k_qp_grad(MT M, PList P, int B, int N, double dt,
                                                 const double* __restrict__ x, const int* __restrict__ need,
                                                 const double* __restrict__ qdd_in, const double* __restrict__ minv_in,
                                                 double* __restrict__ Aout, double* __restrict__ Bout) {
  constexpr int NX = 2 * NJ;
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int K = N - 1;
  if (gid >= B * K * NX) return;
  const int col = gid % NX;
  const int pk = gid / NX;
  const int p = pk / K, k = pk - p * K;
  if (!P.has(p, B)) return;
  const int b = P.at(p);
  if (!need[b]) return;
  const size_t bk = (size_t)b * K + k;
  const double* xb = x + (size_t)b * NX * N;
  double q[NJ], qd[NJ], qdd[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    q[j] = xb[j * N + k];
    qd[j] = xb[(NJ + j) * N + k];
    qdd[j] = qdd_in[(size_t)bk * NJ + j];
  }
  grad_lane_store<NJ, CHAIN, R>(M, dt, q, qd, qdd, minv_in + (size_t)bk * NJ * NJ, col,
                             Aout + (size_t)bk * NX * NX, Bout + (size_t)bk * NX * NJ, nullptr);
}

// ======================================================================= G-block inverses
// dpp_get: tmpc_pcg.h

// In-place Gauss-Jordan inverse of an SPD matrix (no pivoting needed), one
// 16-lane DPP row per matrix, lane r holding row r in a[]: pivot row p is
// broadcast with DPP row_newbcast:p (a VALU move, no LDS round trip), its
// reciprocal taken once.  Exact for diagonal inputs.  All 64 lanes must run it.
template <int P, int NX>
__device__ __forceinline__ void gj_pivot(double (&a)[NX], int r) {
  double pr[NX];
#pragma unroll
  for (int c = 0; c < NX; ++c) pr[c] = dpp_get<0x150 + P, 0xf>(a[c]);
  const double rp = 1.0 / pr[P];
#pragma unroll
  for (int c = 0; c < NX; ++c) pr[c] *= rp;
  const double f = a[P];
  if (r == P) {
#pragma unroll
    for (int c = 0; c < NX; ++c) a[c] = pr[c];
    a[P] = rp;
  } else {
#pragma unroll
    for (int c = 0; c < NX; ++c) a[c] = fma(-f, pr[c], a[c]);
    a[P] = -f * rp;
  }
}

template <int P, int NX>
struct GjSweep {
  static __device__ __forceinline__ void run(double (&a)[NX], int r) {
    gj_pivot<P, NX>(a, r);
    GjSweep<P + 1, NX>::run(a, r);
  }
};
template <int NX>
struct GjSweep<NX, NX> {
  static __device__ __forceinline__ void run(double (&)[NX], int) {}
};

// Ghat = (G_k + rho I)^-1 for the three distinct cost Hessian blocks of
// QuadraticCost (Q, QF, R; TrajoptCost.py:71-83); solveKKTSystem_Schur
// adds rho in place and inverts (TrajoptMPCReference.py:419-422).
// One 16-lane group per matrix, one row per lane (GjSweep).
template <int NJ>
__global__ void __launch_bounds__(64) k_ginv(const CostDev* __restrict__ C, PList P, int B,
                                             const double* __restrict__ rho, const int* __restrict__ active,
                                             double* __restrict__ Ginv) {
  constexpr int NX = 2 * NJ;
  const int lane = threadIdx.x & 63;
  const int slot = (blockIdx.x * blockDim.x + threadIdx.x) >> 4;   // one matrix per 16 lanes
  const int r = lane & 15;
  const int ps = slot / 3;
  const bool in_range = slot < B * 3 && P.has(ps, B);
  const int b = in_range ? P.at(ps) : 0, which = in_range ? slot - 3 * ps : 0;
  const bool act = in_range && active[b];
  const int n = which == 2 ? NJ : NX;
  const double* src = which == 0 ? C->Q : (which == 1 ? C->QF : C->R);
  if (!__any(act)) return;   // wave-uniform exit
  const double rh = act ? rho[b] : 0.0;
  double a[NX];
#pragma unroll
  for (int c = 0; c < NX; ++c)
    a[c] = (act && r < n && c < n) ? src[r * n + c] + (r == c ? rh : 0.0) : (r == c ? 1.0 : 0.0);
  GjSweep<0, NX>::run(a, r);
  if (act && r < n) {
    double* out = Ginv + ((size_t)b * 3 + which) * NX * NX;
#pragma unroll
    for (int c = 0; c < NX; ++c)
      if (c < n) out[r * n + c] = a[c];
  }
}

// k_ginv for the wide models (NX > 16): one 32-lane group per matrix, the pivot row
// broadcast by a lane shuffle instead of a 16-lane DPP row; the operations of gj_pivot, pivot by pivot.
template <int P, int NX>
__device__ __forceinline__ void gj_pivot_wide(double (&a)[NX], int r, int base) {
  double pr[NX];
#pragma unroll
  for (int c = 0; c < NX; ++c) pr[c] = __shfl(a[c], base + P, 64);
  const double rp = 1.0 / pr[P];
#pragma unroll
  for (int c = 0; c < NX; ++c) pr[c] *= rp;
  const double f = a[P];
  if (r == P) {
#pragma unroll
    for (int c = 0; c < NX; ++c) a[c] = pr[c];
    a[P] = rp;
  } else {
#pragma unroll
    for (int c = 0; c < NX; ++c) a[c] = fma(-f, pr[c], a[c]);
    a[P] = -f * rp;
  }
}
template <int P, int NX>
struct GjSweepWide {
  static __device__ __forceinline__ void run(double (&a)[NX], int r, int base) {
    gj_pivot_wide<P, NX>(a, r, base);
    GjSweepWide<P + 1, NX>::run(a, r, base);
  }
};
template <int NX>
struct GjSweepWide<NX, NX> {
  static __device__ __forceinline__ void run(double (&)[NX], int, int) {}
};
template <int NJ>
__global__ void __launch_bounds__(64) k_ginv_wide(const CostDev* __restrict__ C, PList P, int B,
                                                  const double* __restrict__ rho, const int* __restrict__ active,
                                                  double* __restrict__ Ginv) {
  constexpr int NX = 2 * NJ;
  static_assert(NX <= 32, "one matrix per 32 lanes");
  const int lane = threadIdx.x & 63;
  const int slot = (blockIdx.x * blockDim.x + threadIdx.x) >> 5;   // one matrix per 32 lanes
  const int r = lane & 31, base = lane & 32;
  const int ps = slot / 3;
  const bool in_range = slot < B * 3 && P.has(ps, B);
  const int b = in_range ? P.at(ps) : 0, which = in_range ? slot - 3 * ps : 0;
  const bool act = in_range && active[b];
  const int n = which == 2 ? NJ : NX;
  const double* src = which == 0 ? C->Q : (which == 1 ? C->QF : C->R);
  if (!__any(act)) return;   // wave-uniform exit
  const double rh = act ? rho[b] : 0.0;
  double a[NX];
#pragma unroll
  for (int c = 0; c < NX; ++c)
    a[c] = (act && r < n && c < n) ? src[r * n + c] + (r == c ? rh : 0.0) : (r == c ? 1.0 : 0.0);
  GjSweepWide<0, NX>::run(a, r, base);
  if (act && r < n) {
    double* out = Ginv + ((size_t)b * 3 + which) * NX * NX;
#pragma unroll
    for (int c = 0; c < NX; ++c)
      if (c < n) out[r * n + c] = a[c];
  }
}

// cost-to-go helpers (QuadraticCost.get_currQ, TrajoptCost.py:40-47)
__device__ __forceinline__ bool use_QF(const CostDev* C, int k, int N) {
  return (k == N - 1) || (C->QF_start >= 0 && k >= C->QF_start);
}

// Per-knot Ghat_k = (G_k + rho I)^-1 with soft limits: formKKTSystemBlocks adds
// outer(jac, jac) to the cost Hessian block and jac to its gradient
// (TrajoptMPCReference.py:220-225, :255-259), then solveKKTSystem_Schur adds rho
// (:419-422).  The per-type jacobians have disjoint supports on [q | qd | u], so
// G_k stays block-diagonal in (x, u) and each type's outer product lands in its
// own diagonal sub-block (oracle/soft.py).  One 16-lane group per (problem,
// knot, x|u block), one row per lane, Gauss-Jordan as k_ginv.  Also writes the
// summed jacobian (the g_k increment) to jsoft [B][N][NX + NU].
// Layout of Gk: [B][N][NX*NX + NU*NU] (x block, then the packed u block).
constexpr int GINV_SOFT_GROUPS = 2;
template <int NJ>
__global__ void __launch_bounds__(64) k_ginv_soft(const CostDev* __restrict__ C, const ConstrDev* __restrict__ Cs,
                                                  PList P, int B, int N, const double* __restrict__ rho,
                                                  const int* __restrict__ active, const double* __restrict__ x,
                                                  const double* __restrict__ u, const double* __restrict__ mu,
                                                  const double* __restrict__ lam, double* __restrict__ Gk,
                                                  double* __restrict__ jsoft) {
  constexpr int NX = 2 * NJ, NU = NJ, MC = 6 * NJ;
  // one workgroup per (problem, GINV_SOFT_GROUPS x 4 of its 2N matrices), over the launch's problem list
  // (PList: the lock-step tail no longer dispatches workgroups for problems that have finished, so the
  // groups per workgroup can stay few -- the tail's latency is one workgroup's sequential groups)
  const int lane = threadIdx.x & 63;
  const int r = lane & 15;
  const int wpp = (2 * N + 4 * GINV_SOFT_GROUPS - 1) / (4 * GINV_SOFT_GROUPS);
  const int pb = blockIdx.x / wpp;
  if (pb >= B || !P.has(pb, B)) return;   // workgroup-uniform exit
  const int b = P.at(pb);
  if (!active[b]) return;
  const int c0 = (blockIdx.x - pb * wpp) * 4 * GINV_SOFT_GROUPS;
  for (int grp = 0; grp < GINV_SOFT_GROUPS; ++grp) {
  const int rem = c0 + 4 * grp + (lane >> 4);
  const bool in_range = rem < 2 * N;
  if (!__any(in_range)) break;   // wave-uniform: past the problem's last matrix
  const int k = in_range ? rem >> 1 : 0, which = in_range ? rem & 1 : 0;
  const bool terminal = k == N - 1;
  const bool act = in_range && !(which == 1 && terminal);
  const int n = which ? NJ : NX;
  double z[3 * NJ], jac[3 * NJ];
  const double* xb = x + (size_t)b * NX * N;
  const double* ub = u + (size_t)b * NU * (N - 1);
#pragma unroll
  for (int m = 0; m < NX; ++m) z[m] = act ? xb[m * N + k] : 0.0;
#pragma unroll
  for (int m = 0; m < NU; ++m) z[NX + m] = (act && !terminal) ? ub[m * (N - 1) + k] : 0.0;
  const size_t ko = ((size_t)b * N + k) * MC;
  soft_knot<NJ>(Cs, mu + ko, lam + ko, terminal, z, jac);
  const double* src = which ? C->R : (use_QF(C, k, N) ? C->QF : C->Q);
  const double rh = act ? rho[b] : 0.0;
  // UrdfCost: state-dependent x block (Q Jt)^T Jt (hess_mode 0, TrajoptCost.py:490-492)
  // and its gradient (y^T Q) Jt (:449) joins the soft jacobian in jsoft
  // (2-link only, tmpc_set_cost_ee: compiled out of the other instances, whose registers it would
  // otherwise spill -- k_ginv_soft<6> carried 1168 B/lane of scratch for it)
  const bool ee = NJ == 2 && C->kind == COST_EE && which == 0;
  double eg[NX], hrow[NX];
#pragma unroll
  for (int c = 0; c < NX; ++c) eg[c] = hrow[c] = 0.0;
  if constexpr (NJ == 2) if (ee) {
    double Jt[NX * NX], qj[NX];
    ee_eval<NJ>(C, src, z, eg, Jt);
#pragma unroll
    for (int l = 0; l < NX; ++l) {   // (Q Jt)[l][r]
      double acc = 0.0;
#pragma unroll
      for (int m = 0; m < NX; ++m) {
        double jm = 0.0;
#pragma unroll
        for (int rr = 0; rr < NX; ++rr)
          if (rr == r) jm = Jt[m * NX + rr];
        acc += src[l * NX + m] * jm;
      }
      qj[l] = acc;
    }
#pragma unroll
    for (int c = 0; c < NX; ++c) {
      double acc = 0.0;
#pragma unroll
      for (int l = 0; l < NX; ++l) acc += qj[l] * Jt[l * NX + c];
      hrow[c] = acc;
    }
  }
  double a[NX];
#pragma unroll
  for (int c = 0; c < NX; ++c) {
    double outer = 0.0;
    if (which == 0) {
#pragma unroll
      for (int rr = 0; rr < NX; ++rr)
        if (rr == r && (rr / NJ) == (c / NJ)) outer = jac[rr] * jac[c];
    } else {
#pragma unroll
      for (int rr = 0; rr < NU; ++rr)
        if (rr == r && c < NU) outer = jac[NX + rr] * jac[NX + c];
    }
    const double h = ee ? hrow[c] : src[(r < n ? r : 0) * n + c];
    a[c] = (act && r < n && c < n) ? (h + outer) + (r == c ? rh : 0.0) : (r == c ? 1.0 : 0.0);
  }
  GjSweep<0, NX>::run(a, r);
  if (!in_range || r >= n) continue;
  if (act) {
    double* out = Gk + ((size_t)b * N + k) * (NX * NX + NU * NU) + (which ? NX * NX : 0);
#pragma unroll
    for (int c = 0; c < NX; ++c)
      if (c < n) out[r * n + c] = a[c];
  }
  double jr = 0.0;
#pragma unroll
  for (int m = 0; m < NX; ++m)
    if (m == (which ? NX + r : r)) jr = jac[m];
  if (ee) {
#pragma unroll
    for (int m = 0; m < NX; ++m)
      if (m == r) jr = eg[m] + jr;
  }
  if (which) {
#pragma unroll
    for (int m = 0; m < NU; ++m)
      if (m == r) jr = terminal ? 0.0 : jac[NX + m];
  }
  jsoft[((size_t)b * N + k) * (NX + NU) + (which ? NX : 0) + r] = jr;
  }   // grp
}

// ======================================================================= block-tridiagonal PCG: tmpc_pcg.h

// ---- standalone PCG on given blocks (tmpc_pcg_batch: the PCG class)
template <int NX, int RPL, int MAXT>
__global__ void __launch_bounds__(MAXT) k_pcg(int B, int N, int precond, const double* __restrict__ Sd,
                                              const double* __restrict__ Sl, const double* __restrict__ Su,
                                              const double* __restrict__ gam, const double* __restrict__ guess,
                                              double tol, int max_iter, double* __restrict__ lam,
                                              int* __restrict__ iters, double* __restrict__ trace_nu,
                                              double* __restrict__ trace_res, double* __restrict__ Pd_out) {
  const int b = blockIdx.x;
  extern __shared__ __align__(16) double lds[];
  const int rows = N * NX;
  pcg_lds_clear(lds, N, NX, 1024);
  const PcgLds L = pcg_lds(lds, N, NX, 1024);
  const PcgLane<NX, RPL> ln(threadIdx.x, N);
  const int k = ln.k, K = N - 1;
  PcgRow<NX> R[RPL];
  double bv[RPL];
#pragma unroll
  for (int m = 0; m < RPL; ++m) {
#pragma unroll
    for (int j = 0; j < NX; ++j) R[m].sd[j] = R[m].sl[j] = R[m].su[j] = R[m].pr[j] = 0.0;
    bv[m] = 0.0;
    if (!ln.valid) continue;
    const int i = ln.r(m);
    const double* d = Sd + (((size_t)b * N + k) * NX + i) * NX;
#pragma unroll
    for (int j = 0; j < NX; ++j) R[m].sd[j] = d[j];
    if (k > 0) {
      const double* l = Sl + (((size_t)b * K + (k - 1)) * NX + i) * NX;
#pragma unroll
      for (int j = 0; j < NX; ++j) R[m].sl[j] = l[j];
    }
    if (k < K) {
      if (Su) {
        const double* up = Su + (((size_t)b * K + k) * NX + i) * NX;
#pragma unroll
        for (int j = 0; j < NX; ++j) R[m].su[j] = up[j];
      } else {
        const double* l = Sl + ((size_t)b * K + k) * NX * NX;
#pragma unroll
        for (int j = 0; j < NX; ++j) R[m].su[j] = l[j * NX + i];
      }
    }
    bv[m] = gam[(size_t)b * rows + ln.row(m)];
  }
  pcg_precondition<NX, RPL>(R, precond, ln, N, L.piv, Pd_out ? Pd_out + ((size_t)b * N + k) * NX * NX : nullptr);
  int it_done = 0;
  double xv[RPL];
  pcg_dispatch<NX, RPL>(precond, R, ln, N, L, bv, guess ? guess + (size_t)b * rows : nullptr, tol, max_iter,
                        trace_nu ? trace_nu + (size_t)b * (max_iter + 1) : nullptr,
                        trace_res ? trace_res + (size_t)b * (max_iter + 1) : nullptr, &it_done, xv);
  if (ln.valid) {
#pragma unroll
    for (int m = 0; m < RPL; ++m) lam[(size_t)b * rows + ln.row(m)] = xv[m];
  }
  if (threadIdx.x == 0) iters[b] = it_done;
}

// ======================================================================= fused QP kernel
// One QP of the SQP loop for one problem per workgroup:
//   prologue  Schur blocks (blockwise form of
//             solveKKTSystem_Schur :419-424): each lane computes its rows of
//             S_kk, S_{k,k-1}, S_{k,k+1} and gamma_k straight into registers
//             from A, B (qp_grad), the defects c (qp_fd) and Ghat (ginv),
//             all staged once into LDS with coalesced loads;
//   body      preconditioner + PCG (pcg_precondition / pcg_run);
//   epilogue  dxu = Ghat (g - C^T lambda) (:449-452), with C^T lambda formed
//             once per knot in LDS.
// S and lambda never leave the chip.
// A_k / B_k are read from HBM (L2-resident, shared by the NX lanes of a knot), not staged:
// that keeps k_qp's LDS under 80 KB so two problems' workgroups share a CU.
__host__ __device__ inline size_t qp_stage_doubles(int N, int NX, int NU) {
  const size_t K = N - 1;
  return 3 * (size_t)NX * NX + (size_t)NX * N + (size_t)NU * K;
}

// LDS layout of k_qp: [staging area | lambda] is reused by the PCG buffers
// (which start at 0); the cost gradients g_k = [dx_k^T Q_k, u_k^T R] live past
// both because they must survive the PCG.  In the epilogue the x / u slots of
// the staging area hold C^T lambda.
__host__ __device__ inline size_t qp_g_offset(int N, int NX, int NU, int VR) {
  const size_t a = qp_stage_doubles(N, NX, NU) + (size_t)N * NX;
  const size_t p = pcg_lds_doubles(N, NX, VR);
  return a > p ? a : p;
}

__host__ __device__ inline size_t qp_lds_doubles(int N, int NX, int NU, int VR) {
  return qp_g_offset(N, NX, NU, VR) + (size_t)N * (NX + NU);
}

struct QpStage {
  const double *A, *B;      // global (this problem's A_k, B_k)
  double *G, *x, *u;        // LDS
};

__device__ __forceinline__ QpStage qp_stage(double* lds, int N, int NX, int NU, const double* A, const double* B) {
  QpStage S;
  S.A = A;
  S.B = B;
  S.G = lds;
  S.x = S.G + 3 * NX * NX;
  S.u = S.x + NX * N;
  return S;
}

__device__ __forceinline__ void lds_copy(double* dst, const double* __restrict__ src, int count) {
  for (int e = threadIdx.x; e < count; e += blockDim.x) dst[e] = src[e];
}

// Row i of block k of the Schur complement and gamma_k[i] into R (:419-424):
//   S_kk = -(A G A^T + B G B^T + Ghat_x,k), S_{k,k-1} = A_{k-1} Ghat_x,k-1,
//   S_{k,k+1} = (A_k Ghat_x,k)^T, gamma_k = c_k + [AB Ghat g]_{k-1} - (Ghat_k g_k)_x
// Ghat blocks: the three distinct cost blocks staged in LDS (QuadraticCost,
// no soft limits), or per knot from HBM (PK: soft limits, k_ginv_soft layout)
template <int NJ, bool PK>
struct GhatSrc {
  static constexpr int NX = 2 * NJ, NU = NJ, GS = NX * NX + NU * NU;
  const double* base;
  __device__ __forceinline__ const double* x(const CostDev* C, int k, int N) const {
    return PK ? base + (size_t)k * GS : base + (use_QF(C, k, N) ? NX * NX : 0);
  }
  __device__ __forceinline__ const double* u(int k) const {
    return PK ? base + (size_t)k * GS + NX * NX : base + 2 * NX * NX;
  }
};

// A_k, B_k of the Euler integrator (TrajoptPlant.py:92-108) as k_qp_grad writes them:
//   A_k = [[I, dt I], [dt dqdd_q, I + dt dqdd_qd]],   B_k = [[0], [dt M^-1]].
// Their first NJ rows are structural -- exactly 1, dt and 0 -- so the fused QP kernel reads only the
// bottom NJ rows: a product's chain keeps its order term by term, a structural 1 or dt
// is the same fma, a structural zero term is dropped (fma(0, g, acc) == acc for finite g, up to the
// sign of a zero).  Half of A_k / B_k never leaves HBM for the QP, prologue and epilogue alike.
template <int NJ, bool PK>
__device__ __forceinline__ double qp_schur_row(const CostDev* __restrict__ C, const QpStage& S,
                                               const GhatSrc<NJ, PK>& Gh, const double* __restrict__ g_lds,
                                               double c_ki, int k, int i, int N, double dt, PcgRow<2 * NJ>& R) {
  constexpr int NX = 2 * NJ, NU = NJ;
  const int K = N - 1;
  const double* Gxk = Gh.x(C, k, N);
  const double* gk = g_lds + k * (NX + NU);
  double gam = c_ki;
  {
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < NX; ++j) s += Gxk[i * NX + j] * gk[j];
    gam -= s;
  }
  if (k == 0) {
#pragma unroll
    for (int j = 0; j < NX; ++j) R.sd[j] = -Gxk[i * NX + j];
  } else {
    const int km = k - 1;
    const double* Gxm = Gh.x(C, km, N);
    const double* Gu = Gh.u(km);
    const double* gm = g_lds + km * (NX + NU);
    const double* A = S.A + km * NX * NX;
    const double* Bm = S.B + km * NX * NU;
    // R.sl = row i of A_{k-1} Ghat_{k-1}: a structural row i < NJ is e_i + dt e_{i+NJ}
    if (i < NJ) {
#pragma unroll
      for (int j = 0; j < NX; ++j) R.sl[j] = fma(dt, Gxm[(i + NJ) * NX + j], Gxm[i * NX + j] + 0.0);
    } else {
#pragma unroll
      for (int j = 0; j < NX; ++j) {
        double acc = 0.0;
#pragma unroll
        for (int m = 0; m < NX; ++m) acc += A[i * NX + m] * Gxm[m * NX + j];
        R.sl[j] = acc;
      }
    }
    // row i of B_{k-1} Ghat_u: zero for a structural row
    double BG[NU];
#pragma unroll
    for (int j = 0; j < NU; ++j) BG[j] = 0.0;
    if (i >= NJ) {
#pragma unroll
      for (int j = 0; j < NU; ++j) {
        double acc = 0.0;
#pragma unroll
        for (int m = 0; m < NU; ++m) acc += Bm[i * NU + m] * Gu[m * NU + j];
        BG[j] = acc;
      }
    }
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      double acc;
      if (j < NJ) {   // structural row j of A_{k-1}; row j of B_{k-1} is zero
        acc = fma(R.sl[j + NJ], dt, R.sl[j] + 0.0);
      } else {
        acc = 0.0;
#pragma unroll
        for (int m = 0; m < NX; ++m) acc += R.sl[m] * A[j * NX + m];
#pragma unroll
        for (int m = 0; m < NU; ++m) acc += BG[m] * Bm[j * NU + m];
      }
      R.sd[j] = -(acc + Gxk[i * NX + j]);
    }
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < NX; ++j) s += R.sl[j] * gm[j];
#pragma unroll
    for (int j = 0; j < NU; ++j) s += BG[j] * gm[NX + j];
    gam += s;
  }
  if (k < K) {
    const double* A = S.A + k * NX * NX;
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      double acc;
      if (j < NJ) {
        acc = fma(dt, Gxk[(j + NJ) * NX + i], Gxk[j * NX + i] + 0.0);
      } else {
        acc = 0.0;
#pragma unroll
        for (int m = 0; m < NX; ++m) acc += A[j * NX + m] * Gxk[m * NX + i];
      }
      R.su[j] = acc;
    }
  }
  return gam;
}

// mode: QP_MODE_PCG   prologue + PCG + epilogue (the fused path);
//       QP_MODE_SCHUR prologue only: S blocks and gamma to Sd_out / Sl_out / gam_out
//                     (method S: the direct solve k_btsolve runs next);
//       QP_MODE_DXU   epilogue only, lambda read from lam_out (method S, after k_btsolve).
//       GM: more than 1024 rows -- S and P^-1 rows in HBM (Sg, [B][4][NX/2][rows][2], PcgRowG), two rows
//           per lane, LDS vectors of QP_MAX_ROWS rows.
template <int NJ, int RPL, int MAXT, bool PK, int MODE, bool GM = false>
__global__ void __launch_bounds__(MAXT) k_qp(const CostDev* __restrict__ C, PList P, int B, int N, double dt, int precond,
                                             const double* __restrict__ x, const double* __restrict__ u,
                                             const int* __restrict__ active, const double* __restrict__ Ginv,
                                             const double* __restrict__ Aall, const double* __restrict__ Ball,
                                             const double* __restrict__ cvec, double tol, int max_iter,
                                             int* __restrict__ iters, double* __restrict__ dx,
                                             double* __restrict__ du, double* __restrict__ lam_out,
                                             double* __restrict__ Sd_out, double* __restrict__ Sl_out,
                                             double* __restrict__ gam_out, double* __restrict__ Pd_out,
                                             const double* __restrict__ jsoft, const double* __restrict__ guess,
                                             double* __restrict__ Sg) {
  constexpr int NX = 2 * NJ, NU = NJ;
  constexpr int VR = GM ? QP_MAX_ROWS : 1024;
  if (!P.has(blockIdx.x, B)) return;
  const int b = P.at(blockIdx.x);
  if (!active[b]) return;
  extern __shared__ __align__(16) double lds[];
  const int rows = N * NX;
  const PcgLane<NX, RPL> ln(threadIdx.x, N);
  const int k = ln.k;
  const int K = N - 1;
  const QpStage S = qp_stage(lds, N, NX, NU, Aall + (size_t)b * K * NX * NX, Ball + (size_t)b * K * NX * NU);
  double* lam_lds = S.u + NU * K;
  if (!PK) lds_copy(S.G, Ginv + (size_t)b * 3 * NX * NX, 3 * NX * NX);
  const GhatSrc<NJ, PK> Gh{PK ? Ginv + (size_t)b * N * GhatSrc<NJ, PK>::GS : S.G};
  lds_copy(S.x, x + (size_t)b * NX * N, NX * N);
  lds_copy(S.u, u + (size_t)b * NU * K, NU * K);
  __syncthreads();

  // cost gradients g_k = [(x_k - xg)^T Q_k, u_k^T R] (QuadraticCost.gradient, TrajoptCost.py:58-69)
  double* g_lds = lds + qp_g_offset(N, NX, NU, VR);    // [N][NX + NU]
  for (int e = threadIdx.x; e < N * (NX + NU); e += blockDim.x) {
    const int kk = e / (NX + NU), c = e - kk * (NX + NU);
    double g = 0.0;
    if (c < NX) {
      if (C->kind == COST_EE) { g_lds[e] = PK ? jsoft[(size_t)b * N * (NX + NU) + e] : 0.0; continue; }   // in jsoft
      const double* Qk = use_QF(C, kk, N) ? C->QF : C->Q;
#pragma unroll
      for (int m = 0; m < NX; ++m) g += (S.x[m * N + kk] - C->xg[m]) * Qk[m * NX + c];
    } else if (kk < K) {
#pragma unroll
      for (int m = 0; m < NU; ++m) g += S.u[m * K + kk] * C->R[m * NU + (c - NX)];
    }
    if (PK) g = g + jsoft[(size_t)b * N * (NX + NU) + e];   // soft-limit jacobian (:220-225)
    g_lds[e] = g;
  }
  __syncthreads();

  double xv[RPL];
  if constexpr (MODE == QP_MODE_DXU) {
#pragma unroll
    for (int m = 0; m < RPL; ++m) xv[m] = ln.valid ? lam_out[(size_t)b * rows + ln.row(m)] : 0.0;
    if (threadIdx.x == 0) iters[b] = 0;
  } else {
  PcgRow<NX> R[RPL];
  double bv[RPL];
  // GM: this lane's rows of S / P^-1 in HBM (invalid lanes point at slot m N L and never use it)
  double* const Sgb = GM ? Sg + (size_t)b * 4 * NX * rows : nullptr;
  // storage slot of this lane's row m: lane-major (m N L + lane), so that one wave instruction reads
  // 64 consecutive 16-byte pairs (1 KB, whole lines) whatever the rows' order inside a block
  auto g_at = [&](int q, int m) {
    return Sgb + (size_t)q * NX * rows + 2 * ((size_t)m * N * (NX / RPL) + (size_t)ln.k * (NX / RPL) + ln.i);
  };
  auto g_put = [&](int q, int m, int j, double v) { g_at(q, m)[(size_t)(j >> 1) * 2 * rows + (j & 1)] = v; };
#pragma unroll
  for (int m = 0; m < RPL; ++m) {
#pragma unroll
    for (int j = 0; j < NX; ++j) R[m].sd[j] = R[m].sl[j] = R[m].su[j] = R[m].pr[j] = 0.0;
    bv[m] = 0.0;
    if (!ln.valid) continue;
    const int i = ln.r(m);
    bv[m] = qp_schur_row<NJ, PK>(C, S, Gh, g_lds, cvec[(size_t)b * N * NX + k * NX + i], k, i, N, dt, R[m]);
    if (Sd_out) {
#pragma unroll
      for (int j = 0; j < NX; ++j) Sd_out[(((size_t)b * N + k) * NX + i) * NX + j] = R[m].sd[j];
      if (k > 0) {
#pragma unroll
        for (int j = 0; j < NX; ++j) Sl_out[(((size_t)b * K + k - 1) * NX + i) * NX + j] = R[m].sl[j];
      }
      gam_out[(size_t)b * rows + ln.row(m)] = bv[m];
    }
    if constexpr (GM && MODE == QP_MODE_PCG) {
      // off-diagonal rows to HBM now; the diagonal row stays for the preconditioner
#pragma unroll
      for (int j = 0; j < NX; ++j) {
        g_put(0, m, j, R[m].sd[j]);
        g_put(1, m, j, R[m].sl[j]);
        g_put(2, m, j, R[m].su[j]);
        R[m].sl[j] = R[m].su[j] = 0.0;
      }
    }
  }
  if constexpr (MODE == QP_MODE_SCHUR) {
    if (threadIdx.x == 0) iters[b] = 0;
    return;
  }
  __syncthreads();   // the PCG buffers alias the staging area
  pcg_lds_clear(lds, N, NX, VR);
  const PcgLds L = pcg_lds(lds, N, NX, VR);
  pcg_precondition<NX, RPL>(R, precond, ln, N, L.piv, Pd_out ? Pd_out + ((size_t)b * N + k) * NX * NX : nullptr);
  int it_done = 0;
  // PCG warm start (PCG.update_guess, TrajoptMPCReference.py:439-440): guess [B][N NX] or null
  if constexpr (GM) {
    PcgRowG<NX> RG[RPL];
#pragma unroll
    for (int m = 0; m < RPL; ++m) {
#pragma unroll
      for (int j = 0; j < NX; ++j) RG[m].pr[j] = R[m].pr[j];
      RG[m].sd = GRowRef{g_at(0, m), 2 * rows};
      RG[m].sl = GRowRef{g_at(1, m), 2 * rows};
      RG[m].su = GRowRef{g_at(2, m), 2 * rows};
    }
    pcg_dispatch<NX, RPL>(precond, RG, ln, N, L, bv, guess ? guess + (size_t)b * rows : nullptr, tol, max_iter,
                          nullptr, nullptr, &it_done, xv);
  } else {
    pcg_dispatch<NX, RPL>(precond, R, ln, N, L, bv, guess ? guess + (size_t)b * rows : nullptr, tol, max_iter,
                          nullptr, nullptr, &it_done, xv);
  }
  if (threadIdx.x == 0) iters[b] = it_done;
  }

  // ---- epilogue: dxu = Ghat (g - C^T lambda); Ghat re-staged into LDS
  __syncthreads();
  if (!PK) lds_copy(S.G, Ginv + (size_t)b * 3 * NX * NX, 3 * NX * NX);
  if (ln.valid) {
#pragma unroll
    for (int m = 0; m < RPL; ++m) {
      lam_lds[ln.row(m)] = xv[m];
      if (lam_out && MODE == QP_MODE_PCG) lam_out[(size_t)b * rows + ln.row(m)] = xv[m];
    }
  }
  __syncthreads();
  // C^T lambda per knot: x part lambda_k - A_k^T lambda_{k+1} (terminal: lambda_{N-1}),
  // u part -B_k^T lambda_{k+1}; stored in the (dead) x / u staging slots.  The structural rows m < NJ
  // of A_k (e_m + dt e_{m+NJ}) and B_k (0) are not read (qp_schur_row above): column j of A_k^T lambda
  // starts from its one structural term, lambda_j (j < NJ) or dt lambda_{j-NJ}, as the full chain would.
  double* ctl_x = S.x;   // [N][NX]
  double* ctl_u = S.u;   // [K][NU]
  for (int e = threadIdx.x; e < N * NX + K * NU; e += blockDim.x) {
    if (e < N * NX) {
      const int kk = e / NX, j = e - kk * NX;
      double atl = 0.0;
      if (kk < K) {
        const double* A = S.A + kk * NX * NX;
        const double* l1 = lam_lds + (kk + 1) * NX;
        atl = j < NJ ? l1[j] + 0.0 : fma(dt, l1[j - NJ], 0.0);
#pragma unroll
        for (int m = NJ; m < NX; ++m) atl += A[m * NX + j] * l1[m];
      }
      ctl_x[e] = lam_lds[e] - atl;
    } else {
      const int f = e - N * NX;
      const int kk = f / NU, j = f - kk * NU;
      const double* Bm = S.B + kk * NX * NU;
      const double* l1 = lam_lds + (kk + 1) * NX;
      double btl = 0.0;
#pragma unroll
      for (int m = NJ; m < NX; ++m) btl += Bm[m * NU + j] * l1[m];
      ctl_u[f] = -btl;
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < N * NX + K * NU; e += blockDim.x) {
    if (e < N * NX) {
      const int kk = e / NX, i = e - kk * NX;
      const double* Gxk = Gh.x(C, kk, N);
      const double* gk = g_lds + kk * (NX + NU);
      const double* ck = ctl_x + kk * NX;
      double acc = 0.0;
#pragma unroll
      for (int j = 0; j < NX; ++j) acc += Gxk[i * NX + j] * (gk[j] - ck[j]);
      dx[(size_t)b * N * NX + e] = acc;
    } else {
      const int f = e - N * NX;
      const int kk = f / NU, i = f - kk * NU;
      const double* Gu = Gh.u(kk);
      const double* gk = g_lds + kk * (NX + NU) + NX;
      const double* ck = ctl_u + kk * NU;
      double acc = 0.0;
#pragma unroll
      for (int j = 0; j < NU; ++j) acc += Gu[i * NU + j] * (gk[j] - ck[j]);
      du[(size_t)b * K * NU + f] = acc;
    }
  }
}

// ======================================================================= method S: direct block-tridiagonal solve
// solveKKTSystem_Schur with use_PCG = False (TrajoptMPCReference.py:441-446)
// solves S lambda = gamma by np.linalg.solve on the dense S.  S is exactly
// block-tridiagonal and negative definite, so the block
// Thomas recursion needs no pivoting:
//   D_0 = S_00, e_0 = gamma_0;   D_k = S_kk - S_{k,k-1} U_{k-1},  e_k = gamma_k - S_{k,k-1} y_{k-1}
//   [U_k | y_k] = D_k^-1 [S_{k,k+1} | e_k]                         (Gauss-Jordan)
//   lambda_{N-1} = y_{N-1},   lambda_k = y_k - U_k lambda_{k+1}
// One wave per problem, one lane per column of the augmented block
// [D_k | S_{k,k+1} | e_k] (2 NX + 1 <= 64 lanes).  The pivot column is
// broadcast with readlane, so the elimination is register-only; the S_{k,k-1}
// entries are wave-uniform (scalar loads).  U_k and y_k go to a per-problem
// scratch for the back substitution.
template <int NX>
__global__ void __launch_bounds__(64) k_btsolve(int N, const int* __restrict__ active, const double* __restrict__ Sd,
                                                const double* __restrict__ Sl, const double* __restrict__ gam,
                                                double* __restrict__ U, double* __restrict__ Y,
                                                double* __restrict__ lam) {
  static_assert(2 * NX + 1 <= 64, "augmented block must fit one wave");
  const int b = blockIdx.x;
  if (!active[b]) return;
  const int t = threadIdx.x;
  const int K = N - 1;
  const double* sd = Sd + (size_t)b * N * NX * NX;
  const double* sl = Sl + (size_t)b * (K > 0 ? K : 1) * NX * NX;
  const double* gm = gam + (size_t)b * N * NX;
  double* Ub = U + (size_t)b * (K > 0 ? K : 1) * NX * NX;
  double* Yb = Y + (size_t)b * N * NX;
  double a[NX], prev[NX];
#pragma unroll
  for (int r = 0; r < NX; ++r) prev[r] = 0.0;
  for (int k = 0; k < N; ++k) {
#pragma unroll
    for (int r = 0; r < NX; ++r) {
      double v = 0.0;
      if (t < NX)
        v = sd[((size_t)k * NX + r) * NX + t];
      else if (t < 2 * NX)
        v = k < K ? sl[((size_t)k * NX + (t - NX)) * NX + r] : 0.0;   // S_{k,k+1}[r][c] = S_{k+1,k}[c][r]
      else if (t == 2 * NX)
        v = gm[k * NX + r];
      a[r] = v;
    }
    if (k > 0 && (t < NX || t == 2 * NX)) {
      const double* L = sl + (size_t)(k - 1) * NX * NX;   // S_{k,k-1}, wave-uniform
#pragma unroll
      for (int r = 0; r < NX; ++r) {
        double acc = 0.0;
#pragma unroll
        for (int m = 0; m < NX; ++m) acc += L[r * NX + m] * prev[m];
        a[r] -= acc;
      }
    }
#pragma unroll
    for (int p = 0; p < NX; ++p) {
      double f[NX];
#pragma unroll
      for (int r = 0; r < NX; ++r) f[r] = readlane_f64(a[r], p);
      const double inv = 1.0 / f[p];
      a[p] *= inv;
#pragma unroll
      for (int r = 0; r < NX; ++r)
        if (r != p) a[r] -= f[r] * a[p];
    }
    if (t >= NX && t < 2 * NX && k < K) {
#pragma unroll
      for (int r = 0; r < NX; ++r) Ub[((size_t)k * NX + r) * NX + (t - NX)] = a[r];
    }
    if (t == 2 * NX) {
#pragma unroll
      for (int r = 0; r < NX; ++r) Yb[k * NX + r] = a[r];
    }
    // U_k column c moves to lane c for the next D; lane 2 NX keeps y_k
    const int src = t < NX ? t + NX : t;
#pragma unroll
    for (int r = 0; r < NX; ++r) {
      const int lo = __shfl(__double2loint(a[r]), src, 64);
      const int hi = __shfl(__double2hiint(a[r]), src, 64);
      prev[r] = __hiloint2double(hi, lo);
    }
  }
  __threadfence();
  // back substitution, lane r < NX owns row r of lambda_k
  double* lb = lam + (size_t)b * N * NX;
  double lv = (t < NX) ? Yb[K * NX + t] : 0.0;
  if (t < NX) lb[K * NX + t] = lv;
  for (int k = K - 1; k >= 0; --k) {
    double ur[NX];
#pragma unroll
    for (int c = 0; c < NX; ++c) ur[c] = t < NX ? Ub[((size_t)k * NX + t) * NX + c] : 0.0;
    double acc = 0.0;
#pragma unroll
    for (int c = 0; c < NX; ++c) acc += ur[c] * readlane_f64(lv, c);
    lv = (t < NX) ? Yb[k * NX + t] - acc : 0.0;
    if (t < NX) lb[k * NX + t] = lv;
  }
}

int launch_btsolve(hipStream_t s, int nx, int B, int N, const int* active, const double* Sd, const double* Sl,
                   const double* gam, double* U, double* Y, double* lam) {
  switch (nx) {
#define CASE_BT(V) \
  case V: hipLaunchKernelGGL((k_btsolve<V>), dim3(B), dim3(64), 0, s, N, active, Sd, Sl, gam, U, Y, lam); return 0;
    CASE_BT(2) CASE_BT(4) CASE_BT(6) CASE_BT(8) CASE_BT(10) CASE_BT(12) CASE_BT(14)
    CASE_BT(16) CASE_BT(18) CASE_BT(20) CASE_BT(22) CASE_BT(24)
#undef CASE_BT
    default: return -2;
  }
}

// ======================================================================= line-search decision + state machine
// One workgroup per problem.  Reproduces the accept test (:655-666), the
// alpha schedule (:712-718), reduce_regularization (:457-461) and
// check_for_exit_or_error (:463-481), applies the accepted step and records
// the trace row (:691-705 / :729-743).
__global__ void __launch_bounds__(64) k_ls_decide(PList P, int B, int N, int NX, int NU, int T, int mode, int soft,
                                                  const double* __restrict__ alphas, SolverOpts o,
                                                  const double* __restrict__ terms, double* __restrict__ x,
                                                  double* __restrict__ u, const double* __restrict__ dx,
                                                  const double* __restrict__ du, ProbState st,
                                                  const int* __restrict__ pcg_iters, TraceDev tr,
                                                  int* __restrict__ active_count,
                                                  unsigned long long* __restrict__ counters,
                                                  const double* __restrict__ hterms,
                                                  const int* __restrict__ qp_singular,
                                                  int* __restrict__ activate, int stage_bytes) {
  if (!P.has(blockIdx.x, B)) return;
  const int b = P.at(blockIdx.x);
  if (!st.active[b]) return;
  __shared__ double sJ[64], sC[64], sD[64], s_al[64];
  __shared__ int s_choice;
  const int t = threadIdx.x;
  if (t < T) s_al[t] = alphas[t];   // (published by the barrier after the sums)
  // the problem's line-search terms staged in LDS by all 64 lanes at once (dynamic LDS of T N 4 + T N
  // doubles when the launch gives it, LS_DECIDE_STAGE_MAX): one round of independent loads instead of the
  // trial lanes' serial walks through HBM; the sums below read the same values in the same order
  extern __shared__ double s_terms[];
  const bool staged = stage_bytes > 0;
  if (staged) {
    const double* src = terms + (size_t)b * T * N * 4;
    const int ne = T * N * 4;
    // 18 passes' loads in flight (36 per lane at T = 9, N = 64: two round trips; 8 took five)
#pragma unroll 18
    for (int e = t; e < ne; e += 64) s_terms[e] = src[e];
    if (hterms) {
      const double* hs = hterms + (size_t)b * T * N;
#pragma unroll 4
      for (int e = t; e < T * N; e += 64) s_terms[ne + e] = hs[e];
    }
    __syncthreads();
  }
  if (t < T) {
    const double* tm = staged ? s_terms + (size_t)t * N * 4 : terms + ((size_t)b * T + t) * N * 4;
    double J = 0.0, c = 0.0, D = 0.0;
    for (int k = 0; k < N - 1; ++k) J = J + tm[k * 4 + 0];
    J = J + tm[(N - 1) * 4 + 0];
    if (soft) {   // totalCost adds the soft values after the cost terms (:303-307)
      for (int k = 0; k < N - 1; ++k) J = J + tm[k * 4 + 3];
      J = J + tm[(N - 1) * 4 + 3];
    }
    c = tm[(N - 1) * 4 + 1];
    for (int k = 0; k < N - 1; ++k) c = c + tm[k * 4 + 1];
    for (int k = 0; k < N - 1; ++k) D += tm[k * 4 + 2];
    D += tm[(N - 1) * 4 + 2];
    if (hterms) {   // hard box-constraint terms after the dynamics ones, knot by knot (:286-293)
      const double* th = staged ? s_terms + (size_t)T * N * 4 + (size_t)t * N : hterms + ((size_t)b * T + t) * N;
      for (int k = 0; k < N; ++k) c = c + th[k];
    }
    sJ[t] = J;
    sC[t] = c;
    sD[t] = D;
  }
  __syncthreads();
  const int W = o.max_iter_sqp + 1;
  if (t == 0) {
    if (mode == LS_MODE_INIT) {
      const double J = sJ[0], c = sC[0];
      st.J[b] = J;
      st.c[b] = c;
      st.merit[b] = J + o.mu * c;
      const size_t e = (size_t)b * W;
      tr.iteration[e] = 0; tr.ls_iter[e] = 0; tr.alpha[e] = 1.0; tr.rho[e] = st.rho[b];
      tr.J[e] = J; tr.c[e] = c; tr.merit[e] = J + o.mu * c; tr.D[e] = __builtin_nan(""); tr.ratio[e] = __builtin_nan("");
      tr.accepted[e] = 0; tr.pcg_iters[e] = 0; tr.singular[e] = 0;
      if (activate) {   // a restarted pass / a stream's new problem enters its inner loop (st.active: act_init)
        st.active[b] = 0;
        activate[b] = 1;
      }
      s_choice = -2;
    } else {
      const double J = st.J[b], c = st.c[b], merit = st.merit[b];
      double rho = st.rho[b], drho = st.drho[b];
      int choice = -1;
      double D = 0.0, ratio = 0.0, Jn = 0.0, cn = 0.0, mn = 0.0, al = 1.0;
      int ls = 0;
      for (int tt = 0; tt < T; ++tt) {
        al = s_al[tt];
        ls = tt;
        Jn = sJ[tt];
        cn = sC[tt];
        D = sD[tt];
        mn = Jn + o.mu * cn;
        const double dmerit = merit - mn;
        const double expected = al * (D - o.mu * cn);
        ratio = dmerit / expected;
        if (dmerit >= 0.0 && ratio >= o.exp_red_min && ratio <= o.exp_red_max) {
          choice = tt;
          break;
        }
      }
      const int it = st.iter[b];
      const size_t e = (size_t)b * W + it + 1;
      if (counters) {
        // per-problem tallies [B][3], summed once per solve by k_sum_counters (one global
        // atomic per problem and iteration serialised thousands of blocks on one L2 line):
        // [0] problem-QPs solved, [1] PCG iterations, [2] QPs with a fresh dynamics gradient
        unsigned long long* pc = counters + (size_t)b * 3;
        pc[0] += 1ull;
        pc[1] += (unsigned long long)(pcg_iters ? pcg_iters[b] : 0);
        pc[2] += (unsigned long long)st.need_grad[b];
      }
      const bool error = choice < 0;
      double deltaJ = 0.0;
      if (!error) {
        deltaJ = J - Jn;
        st.J[b] = Jn;
        st.c[b] = cn;
        st.merit[b] = mn;
        drho = fmin(drho / o.rho_factor, 1.0 / o.rho_factor);
        rho = fmax(rho * drho, o.rho_min);
      }
      tr.iteration[e] = it; tr.ls_iter[e] = ls; tr.alpha[e] = al; tr.rho[e] = rho;
      tr.J[e] = error ? J : Jn; tr.c[e] = error ? c : cn; tr.merit[e] = error ? merit : mn;
      tr.D[e] = D; tr.ratio[e] = ratio; tr.accepted[e] = error ? 0 : 1;
      tr.pcg_iters[e] = pcg_iters ? pcg_iters[b] : 0;
      tr.singular[e] = qp_singular ? qp_singular[b] : 0;
      // check_for_exit_or_error
      bool done = false;
      if (error) {
        drho = fmax(drho * o.rho_factor, o.rho_factor);
        rho = fmax(rho * drho, o.rho_min);
        if (rho > o.rho_max) { st.exit_sqp[b] = 2; done = true; }
      } else if (deltaJ < o.exit_tol_sqp) {
        st.exit_sqp[b] = 1;
        done = true;
      }
      if (it == o.max_iter_sqp - 1) {
        st.exit_sqp[b] = 3;
        done = true;
      } else {
        st.iter[b] = it + 1;
      }
      st.rho[b] = rho;
      st.drho[b] = drho;
      st.need_grad[b] = (error || done) ? 0 : 1;
      if (done) st.active[b] = 0;
      else *active_count = 1;   // the host only tests for zero
      s_choice = choice;
    }
  }
  __syncthreads();
  const int choice = s_choice;
  if (choice >= 0) {
    const double al = alphas[choice];
    double* xb = x + (size_t)b * NX * N;
    const double* dxb = dx + (size_t)b * N * NX;
    // x - alpha dx, u - alpha du element by element, the loads of U passes ahead of their stores (tmpc_copy.h)
    wg_batched<12, double>(NX * N, t, blockDim.x, [&](int e) {
      const int m = e / N, k = e - m * N;
      return xb[e] - al * dxb[k * NX + m];
    }, [&](int e, double v) { xb[e] = v; });
    const int K = N - 1;
    double* ub = u + (size_t)b * NU * K;
    const double* dub = du + (size_t)b * K * NU;
    wg_batched<8, double>(NU * K, t, blockDim.x, [&](int e) {
      const int m = e / K, k = e - m * K;
      return ub[e] - al * dub[k * NU + m];
    }, [&](int e, double v) { ub[e] = v; });
  } else if (choice == -2 && t == 0) {
    *active_count = 1;
  }
}

// Sum the per-problem tallies of k_ls_decide into out[0..2] (256 atomics per solve).
__global__ void __launch_bounds__(256) k_sum_counters(int B, const unsigned long long* __restrict__ pc,
                                                      unsigned long long* __restrict__ out) {
  unsigned long long s0 = 0, s1 = 0, s2 = 0;
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    s0 += pc[(size_t)b * 3];
    s1 += pc[(size_t)b * 3 + 1];
    s2 += pc[(size_t)b * 3 + 2];
  }
  atomicAdd(&out[0], s0);
  atomicAdd(&out[1], s1);
  atomicAdd(&out[2], s2);
}

void launch_sum_counters(hipStream_t s, int B, const unsigned long long* pc, unsigned long long* out) {
  hipLaunchKernelGGL(k_sum_counters, dim3(1), dim3(256), 0, s, B, pc, out);
}

__global__ void k_init_state(int B, double rho_init, ProbState st, const int* __restrict__ outer_active) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  if (outer_active && !outer_active[b]) {
    st.active[b] = 0;
    return;
  }
  st.rho[b] = rho_init;
  st.drho[b] = 1.0;
  st.iter[b] = 0;
  st.active[b] = 1;
  st.need_grad[b] = 1;
  st.exit_sqp[b] = 0;
}

// ======================================================================= kernel-level entry points
// [K][nx] / [K][nu] row layout, one lane per knot (or per knot and column)
template <int NJ, bool CHAIN, class MT, class R>
__global__ void __launch_bounds__(256) k_unit_minv(MT M, int K, const double* __restrict__ x,
                                                   double* __restrict__ minv_out) {
  constexpr int NX = 2 * NJ;
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= K * NJ) return;
  const int col = gid % NJ, k = gid / NJ;
  double q[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) q[j] = x[(size_t)k * NX + j];
  minv_lane_store<NJ, CHAIN, R>(M, q, col, minv_out + (size_t)k * NJ * NJ);
}

template <int NJ, bool CHAIN, class MT, class R>
__global__ void __launch_bounds__(256) k_unit_grad(MT M, int K, double dt,
                                                   const double* __restrict__ x, const double* __restrict__ qdd_in,
                                                   const double* __restrict__ minv_in, double* __restrict__ Aout,
                                                   double* __restrict__ Bout, double* __restrict__ dqdd) {
  constexpr int NX = 2 * NJ;
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= K * NX) return;
  const int col = gid % NX, k = gid / NX;
  double q[NJ], qd[NJ], qdd[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    q[j] = x[(size_t)k * NX + j];
    qd[j] = x[(size_t)k * NX + NJ + j];
    qdd[j] = qdd_in[(size_t)k * NJ + j];
  }
  grad_lane_store<NJ, CHAIN, R>(M, dt, q, qd, qdd, minv_in + (size_t)k * NJ * NJ, col,
                             Aout ? Aout + (size_t)k * NX * NX : nullptr, Bout ? Bout + (size_t)k * NX * NJ : nullptr,
                             dqdd ? dqdd + (size_t)k * NJ * 3 * NJ : nullptr);
}

// ======================================================================= launchers
#define TMPC_GRID(n, bs) dim3(((n) + (bs) - 1) / (bs)), dim3(bs)

// f32: the dynamics in fp32 (tmpc_options.precision F32 / MIXED), fp64 in and out
template <int NJ, bool CHAIN, class MT>
struct Launch {
  static void qp_minv(bool f32, hipStream_t s, const ModelDev* M, PList P, int B, int N, const double* x,
                      const int* need, double* minv) {
    if constexpr (!kWide<NJ>) {   // fp32 instances for up to NJ_FULL joints only
      if (f32) {
        hipLaunchKernelGGL((k_qp_minv<NJ, CHAIN, MT, float>), TMPC_GRID(B * (N - 1) * NJ, 256), 0, s, MT::make(M), P, B, N,
                           x, need, minv);
        return;
      }
    }
    hipLaunchKernelGGL((k_qp_minv<NJ, CHAIN, MT, double>), TMPC_GRID(B * (N - 1) * NJ, 256), 0, s, MT::make(M), P, B, N,
                       x, need, minv);
  }
  // a runtime model (ModelRef) takes the general-topology gradient instance even for a chain: with runtime
  // coefficients the chain specialisation's unrolled recursion spills 2.5x more (k_qp_grad<6, chain,
  // ModelRef, double> 4.4 kB per lane against 1.7 kB; 2.7 -> 1.3 ms per headline launch)
  static constexpr bool GCHAIN = MT::STATIC ? CHAIN : false;
  static void qp_grad(bool f32, hipStream_t s, const ModelDev* M, PList P, int B, int N, double dt, const double* x,
                      const int* need, const double* qdd, const double* minv, double* A, double* Bm) {
    if constexpr (!kWide<NJ>) {   // fp32 instances for up to NJ_FULL joints only
      if (f32) {
        hipLaunchKernelGGL((k_qp_grad<NJ, GCHAIN, MT, float>), TMPC_GRID(B * (N - 1) * 2 * NJ, 256), 0, s, MT::make(M), P, B,
                           N, dt, x, need, qdd, minv, A, Bm);
        return;
      }
    }
    hipLaunchKernelGGL((k_qp_grad<NJ, GCHAIN, MT, double>), TMPC_GRID(B * (N - 1) * 2 * NJ, 256), 0, s, MT::make(M), P,
                       B, N, dt, x, need, qdd, minv, A, Bm);
  }
  static void unit_minv(bool f32, hipStream_t s, const ModelDev* M, int K, const double* x, double* minv) {
    if constexpr (!kWide<NJ>) {   // fp32 instances for up to NJ_FULL joints only
      if (f32) {
        hipLaunchKernelGGL((k_unit_minv<NJ, CHAIN, MT, float>), TMPC_GRID(K * NJ, 256), 0, s, MT::make(M), K, x, minv);
        return;
      }
    }
    hipLaunchKernelGGL((k_unit_minv<NJ, CHAIN, MT, double>), TMPC_GRID(K * NJ, 256), 0, s, MT::make(M), K, x, minv);
  }
  static void unit_grad(bool f32, hipStream_t s, const ModelDev* M, int K, double dt, const double* x, const double* qdd,
                        const double* minv, double* A, double* Bm, double* dqdd) {
    if constexpr (!kWide<NJ>) {   // fp32 instances for up to NJ_FULL joints only
      if (f32) {
        hipLaunchKernelGGL((k_unit_grad<NJ, GCHAIN, MT, float>), TMPC_GRID(K * 2 * NJ, 256), 0, s, MT::make(M), K, dt, x, qdd,
                           minv, A, Bm, dqdd);
        return;
      }
    }
    hipLaunchKernelGGL((k_unit_grad<NJ, GCHAIN, MT, double>), TMPC_GRID(K * 2 * NJ, 256), 0, s, MT::make(M), K, dt, x, qdd,
                       minv, A, Bm, dqdd);
  }
};

template <int NJ>
struct LaunchNJ {
  static void ginv(hipStream_t s, const CostDev* C, PList P, int B, const double* rho, const int* active, double* G) {
    if constexpr (2 * NJ > 16)
      hipLaunchKernelGGL((k_ginv_wide<NJ>), TMPC_GRID(B * 3 * 32, 64), 0, s, C, P, B, rho, active, G);
    else
      hipLaunchKernelGGL((k_ginv<NJ>), TMPC_GRID(B * 3 * 16, 64), 0, s, C, P, B, rho, active, G);
  }
  static void qp(hipStream_t s, const CostDev* C, PList P, int B, int N, double dt, int precond, int mode, const double* x,
                 const double* u,
                 const int* active, const double* G, const double* A, const double* Bm, const double* cvec, double tol,
                 int max_iter, int* iters, double* dx, double* du, double* lam, double* Sd, double* Sl, double* gam,
                 double* Pd, const double* jsoft, const double* guess, double* Sg) {
    constexpr int NX = 2 * NJ;
    const int rows = N * NX;
    // S / P^-1 rows in HBM (Sg), two rows per lane, up to 1024 lanes (method S past 1024 rows runs the
    // same instance for its prologue / epilogue modes, which never touch Sg)
    const bool gm = !kWide<NJ> && (rows > 1024 || (rows >= qp_gm_min_rows() && mode == QP_MODE_PCG));
    const int rpl = gm ? 2 : pcg_rpl(N, NX);
    const int threads = ((rows / rpl + 63) / 64) * 64;
    const size_t lds = qp_lds_doubles(N, NX, NJ, gm ? QP_MAX_ROWS : 1024) * sizeof(double);
#define TMPC_QP_ARGS s, C, P, B, N, dt, precond, x, u, active, G, A, Bm, cvec, tol, max_iter, iters, dx, du, lam, Sd, \
                     Sl, gam, Pd, jsoft, guess, Sg
#define TMPC_QP_LAUNCH(PKV, MODEV)                                                                        \
    if (gm)                                                                                                \
      hipLaunchKernelGGL((k_qp<NJ, 2, QP_MAX_ROWS / 2, PKV, MODEV, true>), dim3(B), dim3(threads), lds, TMPC_QP_ARGS); \
    else if (rpl == 1)                                                                                     \
      hipLaunchKernelGGL((k_qp<NJ, 1, 768, PKV, MODEV>), dim3(B), dim3(threads), lds, TMPC_QP_ARGS);        \
    else                                                                                                   \
      hipLaunchKernelGGL((k_qp<NJ, 2, 512, PKV, MODEV>), dim3(B), dim3(threads), lds, TMPC_QP_ARGS);
    if constexpr (kWide<NJ>) {   // a wide model: registers / two rows per lane, no soft limits (launch_qp checks)
#define TMPC_QP_LAUNCH_W(MODEV)                                                                            \
      if (rpl == 1)                                                                                        \
        hipLaunchKernelGGL((k_qp<NJ, 1, 768, false, MODEV>), dim3(B), dim3(threads), lds, TMPC_QP_ARGS);    \
      else                                                                                                 \
        hipLaunchKernelGGL((k_qp<NJ, 2, 512, false, MODEV>), dim3(B), dim3(threads), lds, TMPC_QP_ARGS);
      if (mode == QP_MODE_PCG) { TMPC_QP_LAUNCH_W(QP_MODE_PCG) }
      else if (mode == QP_MODE_SCHUR) { TMPC_QP_LAUNCH_W(QP_MODE_SCHUR) }
      else { TMPC_QP_LAUNCH_W(QP_MODE_DXU) }
#undef TMPC_QP_LAUNCH_W
    } else {
      // soft limits (jsoft != null): per-knot Ghat from HBM
      if (mode == QP_MODE_PCG) {
        if (jsoft) { TMPC_QP_LAUNCH(true, QP_MODE_PCG) } else { TMPC_QP_LAUNCH(false, QP_MODE_PCG) }
      } else if (mode == QP_MODE_SCHUR) {
        if (jsoft) { TMPC_QP_LAUNCH(true, QP_MODE_SCHUR) } else { TMPC_QP_LAUNCH(false, QP_MODE_SCHUR) }
      } else {
        if (jsoft) { TMPC_QP_LAUNCH(true, QP_MODE_DXU) } else { TMPC_QP_LAUNCH(false, QP_MODE_DXU) }
      }
    }
#undef TMPC_QP_LAUNCH
#undef TMPC_QP_ARGS
  }
  static void ginv_soft(hipStream_t s, const CostDev* C, const ConstrDev* Cs, PList P, int B, int N, const double* rho,
                        const int* active, const double* x, const double* u, const double* mu, const double* lam,
                        double* Gk, double* jsoft) {
    if constexpr (!kWide<NJ>) {   // no soft limits on a wide model (launch_ginv_soft refuses it)
      const int wpp = (2 * N + 4 * GINV_SOFT_GROUPS - 1) / (4 * GINV_SOFT_GROUPS);
      hipLaunchKernelGGL((k_ginv_soft<NJ>), dim3(B * wpp), dim3(64), 0, s, C, Cs, P, B, N, rho, active, x, u, mu, lam,
                         Gk, jsoft);
    }
  }
};

int pcg_set_max_lds() {
  const int bytes = 160 * 1024;
  int err = 0;
#define SETA(V)                                                                                                    \
  err |= (int)hipFuncSetAttribute((const void*)k_pcg<V, 1, 768>, hipFuncAttributeMaxDynamicSharedMemorySize, bytes); \
  err |= (int)hipFuncSetAttribute((const void*)k_pcg<V, 2, 512>, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
#ifdef TMPC_DEV_NJ
  SETA(2 * TMPC_DEV_NJ)
#else
  SETA(2) SETA(4) SETA(6) SETA(8) SETA(10) SETA(12) SETA(14) SETA(16)
#endif
#undef SETA
#define SETQ2(V, P, MD)                                                                                  \
  err |= (int)hipFuncSetAttribute((const void*)k_qp<V, 1, 768, P, MD>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                  bytes);                                                              \
  err |= (int)hipFuncSetAttribute((const void*)k_qp<V, 2, 512, P, MD>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                  bytes);                                                              \
  err |= (int)hipFuncSetAttribute((const void*)k_qp<V, 2, QP_MAX_ROWS / 2, P, MD, true>,                          \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
#define SETQ1(V, P) SETQ2(V, P, QP_MODE_PCG) SETQ2(V, P, QP_MODE_SCHUR) SETQ2(V, P, QP_MODE_DXU)
#define SETQ(V) SETQ1(V, false) SETQ1(V, true)
#ifdef TMPC_DEV_NJ
  SETQ(TMPC_DEV_NJ)
#else
  SETQ(1) SETQ(2) SETQ(3) SETQ(4) SETQ(5) SETQ(6) SETQ(7)
  // the wide models' instances (registers / two rows per lane, no soft limits)
#define SETQW1(V, MD)                                                                                    \
  err |= (int)hipFuncSetAttribute((const void*)k_qp<V, 1, 768, false, MD>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                  bytes);                                                              \
  err |= (int)hipFuncSetAttribute((const void*)k_qp<V, 2, 512, false, MD>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                  bytes);
#define SETQW(V) SETQW1(V, QP_MODE_PCG) SETQW1(V, QP_MODE_SCHUR) SETQW1(V, QP_MODE_DXU)
  SETQW(8) SETQW(9) SETQW(10) SETQW(11) SETQW(12)
#undef SETQW
#undef SETQW1
#endif
#undef SETQ
#undef SETQ1
#undef SETQ2
  return err;
}

template <int NX>
static void launch_pcg_nx(hipStream_t s, int B, int N, int precond, const double* Sd, const double* Sl,
                          const double* Su, const double* gam, const double* guess, double tol, int max_iter,
                          double* lam, int* iters, double* tnu, double* tres, double* Pd) {
  const int rows = N * NX;
  const int rpl = pcg_rpl(N, NX);
  const int threads = ((rows / rpl + 63) / 64) * 64;
  const size_t lds = pcg_lds_doubles(N, NX, 1024) * sizeof(double);
  if (rpl == 1)
    hipLaunchKernelGGL((k_pcg<NX, 1, 768>), dim3(B), dim3(threads), lds, s, B, N, precond, Sd, Sl, Su, gam, guess,
                       tol, max_iter, lam, iters, tnu, tres, Pd);
  else
    hipLaunchKernelGGL((k_pcg<NX, 2, 512>), dim3(B), dim3(threads), lds, s, B, N, precond, Sd, Sl, Su, gam, guess,
                       tol, max_iter, lam, iters, tnu, tres, Pd);
}

int launch_pcg(hipStream_t s, int nx, int B, int N, int precond, const double* Sd, const double* Sl,
               const double* Su, const double* gam, const double* guess, double tol, int max_iter, double* lam,
               int* iters, double* tnu, double* tres, double* Pd) {
  if (N * nx > 1024) return -1;
  switch (nx) {
#define CASE_NX(V) \
  case V: launch_pcg_nx<V>(s, B, N, precond, Sd, Sl, Su, gam, guess, tol, max_iter, lam, iters, tnu, tres, Pd); return 0;
#ifdef TMPC_DEV_NJ
    CASE_NX(2 * TMPC_DEV_NJ)
#else
    CASE_NX(2) CASE_NX(4) CASE_NX(6) CASE_NX(8) CASE_NX(10) CASE_NX(12) CASE_NX(14) CASE_NX(16)
#endif
#undef CASE_NX
    default: return -2;
  }
}

void launch_ls_decide(hipStream_t s, PList P, int B, int N, int NX, int NU, int T, int mode, int soft,
                      const double* alphas, const SolverOpts& o, const double* terms, double* x, double* u,
                      const double* dx, const double* du, const ProbState& st, const int* pcg_iters,
                      const TraceDev& tr, int* active_count, unsigned long long* counters, const double* hterms,
                      const int* qp_singular, int* activate) {
  // LDS staging of the terms up to LS_DECIDE_STAGE_MAX bytes (within the default dynamic-LDS limit; N = 64,
  // T = 9: 18 kB), the direct HBM walks past it
  constexpr size_t LS_DECIDE_STAGE_MAX = 60 * 1024;
  size_t stage = ((size_t)T * N * 4 + (hterms ? (size_t)T * N : 0)) * sizeof(double);
  if (stage > LS_DECIDE_STAGE_MAX) stage = 0;
  hipLaunchKernelGGL(k_ls_decide, dim3(B), dim3(64), stage, s, P, B, N, NX, NU, T, mode, soft, alphas, o, terms, x, u,
                     dx, du, st, pcg_iters, tr, active_count, counters, hterms, qp_singular, activate, (int)stage);
}

// The problems still alive in the lock-step loop (mask != 0), ascending, and their count: one
// 1024-lane workgroup, each lane a contiguous chunk of the batch, a block prefix sum of the chunk
// counts.  host_slot (nullable): the count also lands in the iteration's flag slot the host reads back.
__global__ void __launch_bounds__(1024) k_alive_list(int B, const int* __restrict__ alive, int* __restrict__ idx,
                                                     int* __restrict__ cnt, int* __restrict__ host_slot) {
  __shared__ int part[1024];
  const int t = threadIdx.x, nt = blockDim.x;
  const int chunk = (B + nt - 1) / nt;
  const int lo = t * chunk, hi = min(B, lo + chunk);
  int c = 0;
  for (int b = lo; b < hi; ++b) c += alive[b] != 0;
  part[t] = c;
  __syncthreads();
  for (int off = 1; off < nt; off <<= 1) {   // inclusive Hillis-Steele scan
    const int v = t >= off ? part[t - off] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int o = part[t] - c;
  for (int b = lo; b < hi; ++b)
    if (alive[b]) idx[o++] = b;
  if (t == nt - 1) {
    // the lock-step loop sizes its grids by an earlier length (tmpc_api.cpp lockstep_loop): valid only
    // while the list never grows -- host_slot[1] flags a violation, which the host turns into an error
    if (host_slot) {
      host_slot[0] = part[t];
      if (part[t] > *cnt) host_slot[1] = 1;
    }
    *cnt = part[t];
  }
}

void launch_alive_list(hipStream_t s, int B, const int* alive, int* idx, int* cnt, int* host_slot) {
  hipLaunchKernelGGL(k_alive_list, dim3(1), dim3(1024), 0, s, B, alive, idx, cnt, host_slot);
}

void launch_init_state(hipStream_t s, int B, double rho_init, const ProbState& st, const int* outer_active) {
  hipLaunchKernelGGL(k_init_state, TMPC_GRID(B, 256), 0, s, B, rho_init, st, outer_active);
}

// ======================================================================= soft-constraint outer loop
// check_and_update_soft_constraints (TrajoptMPCReference.py:483-508) for one
// problem per 64-lane workgroup, after its inner SQP loop exited:
//   max_c = max over types and knots of |min(v)|  (max_soft_constraint_value, :130-135)
//   exit 1 if max_c < tol; exit 2 at the last outer iteration (else outer_iter += 1);
//   otherwise update_soft_constraint_constants (:137-166) elementwise and exit 3
//   when no constant changed (all mu at their limit).
// Unconstrained problems (no soft type) take the reference's path: max_c = 0 -> exit 1.
// Two drivers:
//   lock-step (inner == null): every problem still in the outer loop, after the whole batch's
//     inner loops have exited; *outer_count = 1 when some problem continues;
//   per-problem (inner = the inner loop's active flags): only problems whose inner loop has just
//     exited (outer_active && !inner && !init); one that continues is reset for its next pass
//     (k_init_state's reset) and flagged in act_init for its initial merit evaluation, so each
//     problem runs its passes back to back instead of waiting for the batch's slowest pass.
__device__ __forceinline__ double soft_v(const ConstrDev* Cs, int t, int e, int n, double z) {
  const int i = e < n ? e : e - n;
  return e < n ? z - Cs->lb[t][i] : Cs->ub[t][i] - z;
}

// A stream's hand-over of slot s, whose problem has just left its outer loop (tmpc_internal.h StreamDev),
// by the workgroup of k_soft_outer that ended it: the finished problem's trajectory, status and trace rows
// to its output rows; then, when a problem is pending, its x, u, x[:, 0] and the state a fresh solve
// starts from -- k_init_state's reset, k_outer_init's, BoxConstraint.__init__'s constants (k_soft_init),
// a zero PCG warm start -- and act_init, so that its initial merit / cost is evaluated this iteration.
__device__ void stream_handover(int s, const StreamDev& sd, double* __restrict__ x, double* __restrict__ u,
                                double* __restrict__ xs, const ProbState& st, int* __restrict__ outer_active,
                                int* __restrict__ outer_iter, int* __restrict__ exit_soft,
                                int* __restrict__ act_init, double rho_init, const TraceDev& tr,
                                const ConstrDev* __restrict__ Cs, double* __restrict__ mu, double* __restrict__ lam,
                                double* __restrict__ phi, double* __restrict__ lam_warm) {
  __shared__ int s_next;
  const int t = threadIdx.x, nt = blockDim.x;
  const int old_l = sd.slot_pid[s];
  const int old = sd.pbase + old_l;   // the output row (global problem index)
  const int XN = sd.NX * sd.N, UN = sd.NU * (sd.N - 1), W = sd.W;
  double* xb = x + (size_t)s * XN;
  double* ub = u + (size_t)s * UN;
  if (t == 0) s_next = atomicAdd(sd.next, 1);
  if (old_l >= 0) {
    // the rows' loads batched ahead of their stores (tmpc_copy.h): 12 + 6 passes at arm6 N = 64 were
    // that many dependent round trips
    if (sd.x_out) wg_copy<12>(sd.x_out + (size_t)old * XN, xb, XN, t, nt);
    if (sd.u_out) wg_copy<8>(sd.u_out + (size_t)old * UN, ub, UN, t, nt);
    if (sd.status && t == 0) {
      int* so = sd.status + (size_t)old * 4;
      so[0] = st.exit_sqp[s];
      so[1] = st.iter[s];
      so[2] = exit_soft[s];
      so[3] = outer_iter[s];
    }
    const TraceDev& to = sd.tr_out;
    const size_t ri = (size_t)s * W, ro = (size_t)old * W;
#define TMPC_TR_COPY(f) \
  if (to.f) wg_copy<4>(to.f + ro, tr.f + ri, W, t, nt);
    TMPC_TR_COPY(iteration) TMPC_TR_COPY(ls_iter) TMPC_TR_COPY(alpha) TMPC_TR_COPY(rho) TMPC_TR_COPY(J)
    TMPC_TR_COPY(c) TMPC_TR_COPY(merit) TMPC_TR_COPY(D) TMPC_TR_COPY(ratio) TMPC_TR_COPY(accepted)
    TMPC_TR_COPY(pcg_iters) TMPC_TR_COPY(singular)
#undef TMPC_TR_COPY
  }
  __syncthreads();   // every read of the finished problem precedes the writes of the next one
  const int nw = s_next;
  if (nw >= sd.P) {
    if (t == 0) sd.slot_pid[s] = -1;
    return;
  }
  const size_t src = (size_t)((sd.pbase + nw) % sd.period);
  wg_copy<12>(xb, sd.x_in + src * XN, XN, t, nt);
  wg_copy<8>(ub, sd.u_in + src * UN, UN, t, nt);
  for (int m = t; m < sd.NX; m += nt) xs[(size_t)s * sd.NX + m] = sd.x_in[src * XN + (size_t)m * sd.N];
  if (mu) {
    const int MC = sd.MC;
    for (int i = t; i < sd.N * MC; i += nt) {
      const int ty = (i % MC) / (MC / 3);
      const size_t o = (size_t)s * sd.N * MC + i;
      mu[o] = Cs->mu_init[ty];
      lam[o] = 0.0;
      phi[o] = Cs->phi_init[ty];
    }
  }
  if (lam_warm)
    for (int e = t; e < sd.NX * sd.N; e += nt) lam_warm[(size_t)s * sd.NX * sd.N + e] = 0.0;
  if (t == 0) {
    st.rho[s] = rho_init;
    st.drho[s] = 1.0;
    st.iter[s] = 0;
    st.active[s] = 0;   // set by the initial merit's decision (act_init)
    st.need_grad[s] = 1;
    st.exit_sqp[s] = 0;
    outer_active[s] = 1;
    outer_iter[s] = 0;
    exit_soft[s] = 0;
    act_init[s] = 1;
    sd.slot_pid[s] = nw;
  }
}

__global__ void __launch_bounds__(64) k_soft_outer(const ConstrDev* __restrict__ Cs, PList P, int B, int N, int NJ,
                                                   double tol, int max_iter, double* __restrict__ x,
                                                   double* __restrict__ u, double* __restrict__ mu,
                                                   double* __restrict__ lam, double* __restrict__ phi,
                                                   int* __restrict__ outer_active, int* __restrict__ outer_iter,
                                                   int* __restrict__ exit_soft, int* __restrict__ outer_count,
                                                   ProbState st, int* __restrict__ act_init, double rho_init,
                                                   StreamDev sd, double* __restrict__ xs, TraceDev tr,
                                                   double* __restrict__ lam_warm) {
  if (!P.has(blockIdx.x, B)) return;
  const int b = P.at(blockIdx.x);
  if (!outer_active[b]) return;
  const bool per_problem = act_init != nullptr;
  if (per_problem && (st.active[b] || act_init[b])) return;
  const int t0 = threadIdx.x;
  const int NX = 2 * NJ, K = N - 1, MC = 6 * NJ;
  const double* xb = x + (size_t)b * NX * N;
  const double* ub = u + (size_t)b * NJ * K;
  auto zval = [&](int t, int i, int k) -> double {
    return t == 2 ? ub[i * K + k] : xb[(t * NJ + i) * N + k];
  };
  // max_c over (type, knot) pairs (the pair's 2 n values loaded together, then reduced in order); PB pairs'
  // loads per lane issued before any is reduced (one round trip for arm6 N = 64's three passes)
  double mx = 0.0;
  constexpr int PB = 4;
  for (int p0 = t0; p0 < 3 * N; p0 += 64 * PB) {
    double zz[PB][NJMAX];
    bool okp[PB];
#pragma unroll
    for (int j = 0; j < PB; ++j) {
      const int p = p0 + 64 * j;
      const int t = p / N, k = p - t * N;
      okp[j] = p < 3 * N && Cs->mode[t] != SOFT_NONE && !(t == 2 && k == K);
#pragma unroll
      for (int i = 0; i < NJMAX; ++i) zz[j][i] = (okp[j] && i < NJ) ? zval(t, i, k) : 0.0;
    }
#pragma unroll
    for (int j = 0; j < PB; ++j) {
      if (!okp[j]) continue;
      const int t = (p0 + 64 * j) / N;
      // the lower bounds' values, then the upper ones' (e = i, then NJ + i): the pair's order, with
      // static indices into zz (NJ is a launch argument: zz[e - NJ] had put zz in scratch)
      double mn = 0.0;
#pragma unroll
      for (int i = 0; i < NJMAX; ++i) {
        if (i >= NJ) break;
        const double v = soft_v(Cs, t, i, NJ, zz[j][i]);
        mn = i == 0 ? v : fmin(mn, v);
      }
#pragma unroll
      for (int i = 0; i < NJMAX; ++i) {
        if (i >= NJ) break;
        mn = fmin(mn, soft_v(Cs, t, NJ + i, NJ, zz[j][i]));
      }
      mx = fmax(mx, fabs(mn));
    }
  }
  __shared__ double smax[64];
  __shared__ int s_exit, s_changed, s_done;
  smax[t0] = mx;
  if (t0 == 0) s_changed = 0;
  __syncthreads();
  if (t0 == 0) {
    double m = 0.0;
    for (int i = 0; i < 64; ++i) m = fmax(m, smax[i]);
    int ex = 0;
    if (m < tol) ex = 1;
    const int it = outer_iter[b];
    if (it == max_iter - 1) ex = 2;
    else outer_iter[b] = it + 1;
    s_exit = ex;
  }
  __syncthreads();
  if (s_exit == 0) {
    // update_soft_constraint_constants entry by entry; OB entries per lane have their loads issued together
    // before any of them is updated (each entry's arithmetic is unchanged)
    constexpr int OB = 18;
    for (int p0 = t0; p0 < N * MC; p0 += 64 * OB) {
      double zv[OB], ph[OB], mv[OB], lv[OB];
      bool ok[OB];
#pragma unroll
      for (int j = 0; j < OB; ++j) {
        const int p = p0 + 64 * j;
        const int k = p / MC, sl = p - k * MC;
        const int t = sl / (2 * NJ), e = sl - t * 2 * NJ;
        ok[j] = p < N * MC && Cs->mode[t] != SOFT_NONE && !(t == 2 && k == K);
        zv[j] = ph[j] = mv[j] = lv[j] = 0.0;
        if (ok[j]) {
          const size_t o = ((size_t)b * N + k) * MC + sl;
          zv[j] = zval(t, e < NJ ? e : e - NJ, k);
          ph[j] = phi[o];
          mv[j] = mu[o];
          lv[j] = lam[o];
        }
      }
#pragma unroll
      for (int j = 0; j < OB; ++j) {
        if (!ok[j]) continue;
        const int p = p0 + 64 * j;
        const int k = p / MC, sl = p - k * MC;
        const int t = sl / (2 * NJ), e = sl - t * 2 * NJ;
        const double v = soft_v(Cs, t, e, NJ, zv[j]);
        const size_t o = ((size_t)b * N + k) * MC + sl;
        if (v < 0.0 && !(fabs(v) < ph[j])) {
          if (mv[j] < Cs->mu_max[t]) {
            s_changed = 1;
            mu[o] = fmin(Cs->mu_max[t], mv[j] * Cs->mu_factor[t]);
          }
        } else if (v < 0.0) {
          s_changed = 1;
          lam[o] = lv[j] + mv[j] * v;
          phi[o] = ph[j] / Cs->phi_factor[t];
        }
      }
    }
  }
  __syncthreads();
  if (t0 == 0) {
    int ex = s_exit;
    if (ex == 0 && !s_changed) ex = 3;
    s_done = ex != 0;
    if (ex) {
      exit_soft[b] = ex;
      outer_active[b] = 0;
    } else {
      *outer_count = 1;   // the host only tests for zero
      if (per_problem) {  // next pass: the reset of k_init_state, then the initial merit (act_init)
        st.rho[b] = rho_init;
        st.drho[b] = 1.0;
        st.iter[b] = 0;
        st.need_grad[b] = 1;
        st.exit_sqp[b] = 0;
        act_init[b] = 1;
      }
    }
  }
  if (sd.P > 0) {   // a stream (per-problem mode): a finished problem hands its slot on
    __syncthreads();
    if (s_done)
      stream_handover(b, sd, x, u, xs, st, outer_active, outer_iter, exit_soft, act_init, rho_init, tr, Cs, mu, lam,
                      phi, lam_warm);
  }
}

void launch_soft_outer(hipStream_t s, const ConstrDev* Cs, PList P, int B, int N, int nj, double tol, int max_iter,
                       double* x, double* u, double* mu, double* lam, double* phi, int* outer_active,
                       int* outer_iter, int* exit_soft, int* outer_count, const ProbState* st, int* act_init,
                       double rho_init, const StreamDev* sd, double* xs, const TraceDev* tr, double* lam_warm) {
  ProbState none{};
  StreamDev nosd{};
  TraceDev notr{};
  hipLaunchKernelGGL(k_soft_outer, dim3(B), dim3(64), 0, s, Cs, P, B, N, nj, tol, max_iter, x, u, mu, lam, phi,
                     outer_active, outer_iter, exit_soft, outer_count, st ? *st : none, act_init, rho_init,
                     sd ? *sd : nosd, xs, tr ? *tr : notr, lam_warm);
}

// BoxConstraint.__init__ (:21-24): mu = mu_init, lambda = 0, phi = phi_init
__global__ void k_soft_init(const ConstrDev* __restrict__ Cs, size_t total, int MC, double* __restrict__ mu,
                            double* __restrict__ lam, double* __restrict__ phi) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int t = (int)(i % MC) / (MC / 3);
  mu[i] = Cs->mu_init[t];
  lam[i] = 0.0;
  phi[i] = Cs->phi_init[t];
}

// BoxConstraint.shift_soft_constraint_constants(1) (TrajoptConstraint.py:168-176) on the
// [B][N][6n] state: arr[:, :-1] = arr[:, 1:]; arr[:, 1:] = init (the reference's semantics:
// every knot after the first returns to its initial value).  Torque limits span N-1 knots.
__global__ void k_soft_shift(const ConstrDev* __restrict__ Cs, int B, int N, int NJ, double* __restrict__ mu,
                             double* __restrict__ lam, double* __restrict__ phi) {
  const int MC = 6 * NJ;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * MC) return;
  const int b = i / MC, sl = i - b * MC, t = sl / (2 * NJ);
  const int T = t == 2 ? N - 1 : N;
  double* arrs[3] = {mu, lam, phi};
  const double init[3] = {Cs->mu_init[t], 0.0, Cs->phi_init[t]};
  for (int a = 0; a < 3; ++a) {
    double* v = arrs[a] + (size_t)b * N * MC + sl;
    if (T > 1) v[0] = v[MC];
    for (int k = 1; k < T; ++k) v[(size_t)k * MC] = init[a];
  }
}

void launch_soft_shift(hipStream_t s, const ConstrDev* Cs, int B, int N, int nj, double* mu, double* lam,
                       double* phi) {
  hipLaunchKernelGGL(k_soft_shift, TMPC_GRID(B * 6 * nj, 256), 0, s, Cs, B, N, nj, mu, lam, phi);
}

__global__ void k_outer_init(int B, int* __restrict__ outer_active, int* __restrict__ outer_iter,
                             int* __restrict__ exit_soft) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  outer_active[b] = 1;
  outer_iter[b] = 0;
  exit_soft[b] = 0;
}

void launch_outer_init(hipStream_t s, int B, int* outer_active, int* outer_iter, int* exit_soft) {
  hipLaunchKernelGGL(k_outer_init, TMPC_GRID(B, 256), 0, s, B, outer_active, outer_iter, exit_soft);
}

void launch_soft_init(hipStream_t s, const ConstrDev* Cs, size_t total, int MC, double* mu, double* lam,
                      double* phi) {
  hipLaunchKernelGGL(k_soft_init, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, Cs, total, MC, mu, lam,
                     phi);
}

// ======================================================================= continuous batching (tmpc_internal.h)
// slot s starts with problem s: one 256-thread workgroup per slot copies its inputs (x, u are read and
// written with unit stride, so a workgroup's loads and stores coalesce)
__global__ void __launch_bounds__(256) k_stream_init(int B, StreamDev sd, double* __restrict__ x,
                                                     double* __restrict__ u) {
  const int s = blockIdx.x, t = threadIdx.x;
  const int XN = sd.NX * sd.N, UN = sd.NU * (sd.N - 1);
  const size_t src = (size_t)((sd.pbase + s) % sd.period);
  wg_copy<4>(x + (size_t)s * XN, sd.x_in + src * XN, XN, t, blockDim.x);
  wg_copy<4>(u + (size_t)s * UN, sd.u_in + src * UN, UN, t, blockDim.x);
  if (t == 0) {
    sd.slot_pid[s] = s;
    if (s == 0) *sd.next = B;   // the next pending problem (stream_handover takes them with atomics)
  }
}

void launch_stream_init(hipStream_t s, int B, const StreamDev& sd, double* x, double* u) {
  hipLaunchKernelGGL(k_stream_init, dim3(B), dim3(256), 0, s, B, sd, x, u);
}


// dispatch tables over the joint count and the chain specialisation
#ifdef TMPC_DEV_NJ
#define TMPC_DISPATCH_NJ(nj, chain, CALL)                                          \
  if (nj != TMPC_DEV_NJ) return -2;                                                 \
  if (chain) Launch<TMPC_DEV_NJ, true, ModelRef>::CALL;                             \
  else Launch<TMPC_DEV_NJ, false, ModelRef>::CALL;                                  \
  return 0;
#else
#define TMPC_DISPATCH_NJ(nj, chain, CALL)                                                              \
  switch (mid) {                                                                                       \
    TMPC_STATIC_MODEL_CASES(Launch, CALL)                                                            \
    default: break;                                                                                    \
  }                                                                                                    \
  switch (nj) {                                                                                        \
    case 1: if (chain) Launch<1, true, ModelRef>::CALL; else Launch<1, false, ModelRef>::CALL; break;  \
    case 2: if (chain) Launch<2, true, ModelRef>::CALL; else Launch<2, false, ModelRef>::CALL; break;  \
    case 3: if (chain) Launch<3, true, ModelRef>::CALL; else Launch<3, false, ModelRef>::CALL; break;  \
    case 4: if (chain) Launch<4, true, ModelRef>::CALL; else Launch<4, false, ModelRef>::CALL; break;  \
    case 5: if (chain) Launch<5, true, ModelRef>::CALL; else Launch<5, false, ModelRef>::CALL; break;  \
    case 6: if (chain) Launch<6, true, ModelRef>::CALL; else Launch<6, false, ModelRef>::CALL; break;  \
    case 7: if (chain) Launch<7, true, ModelRef>::CALL; else Launch<7, false, ModelRef>::CALL; break;  \
    TMPC_WIDE_CASES(Launch, CALL)                                                                      \
    default: return -2;                                                                                \
  }                                                                                                    \
  return 0;
#endif

#ifdef TMPC_DEV_NJ
// experiment builds (make dev): one joint count only, a fraction of the compile time
#define TMPC_DISPATCH_NJ2(nj, CALL)                      \
  if (nj != TMPC_DEV_NJ) return -2;                      \
  LaunchNJ<TMPC_DEV_NJ>::CALL;                           \
  return 0;
#else
#define TMPC_DISPATCH_NJ2(nj, CALL)          \
  switch (nj) {                              \
    case 1: LaunchNJ<1>::CALL; break;        \
    case 2: LaunchNJ<2>::CALL; break;        \
    case 3: LaunchNJ<3>::CALL; break;        \
    case 4: LaunchNJ<4>::CALL; break;        \
    case 5: LaunchNJ<5>::CALL; break;        \
    case 6: LaunchNJ<6>::CALL; break;        \
    case 7: LaunchNJ<7>::CALL; break;        \
    case 8: LaunchNJ<8>::CALL; break;        \
    case 9: LaunchNJ<9>::CALL; break;        \
    case 10: LaunchNJ<10>::CALL; break;      \
    case 11: LaunchNJ<11>::CALL; break;      \
    case 12: LaunchNJ<12>::CALL; break;      \
    default: return -2;                      \
  }                                                                                \
  return 0;
#endif

int launch_qp_minv(bool f32, hipStream_t s, int nj, bool chain, int mid, const ModelDev* M, PList P, int B, int N,
                   const double* x, const int* need, double* minv) {
  TMPC_DISPATCH_NJ(nj, chain, qp_minv(f32, s, M, P, B, N, x, need, minv))
}
int launch_qp_grad(bool f32, hipStream_t s, int nj, bool chain, int mid, const ModelDev* M, PList P, int B, int N,
                   double dt, const double* x, const int* need, const double* qdd, const double* minv, double* A,
                   double* Bm) {
  TMPC_DISPATCH_NJ(nj, chain, qp_grad(f32, s, M, P, B, N, dt, x, need, qdd, minv, A, Bm))
}
int launch_unit_minv(bool f32, hipStream_t s, int nj, bool chain, int mid, const ModelDev* M, int K, const double* x,
                     double* minv) {
  TMPC_DISPATCH_NJ(nj, chain, unit_minv(f32, s, M, K, x, minv))
}
int launch_unit_grad(bool f32, hipStream_t s, int nj, bool chain, int mid, const ModelDev* M, int K, double dt,
                     const double* x, const double* qdd, const double* minv, double* A, double* Bm, double* dqdd) {
  TMPC_DISPATCH_NJ(nj, chain, unit_grad(f32, s, M, K, dt, x, qdd, minv, A, Bm, dqdd))
}
int launch_ginv(hipStream_t s, int nj, const CostDev* C, PList P, int B, const double* rho, const int* active,
                double* G) {
  TMPC_DISPATCH_NJ2(nj, ginv(s, C, P, B, rho, active, G))
}
int launch_qp(hipStream_t s, int nj, const CostDev* C, PList P, int B, int N, double dt, int precond, int mode,
              const double* x, const double* u,
              const int* active, const double* G, const double* A, const double* Bm, const double* cvec, double tol,
              int max_iter, int* iters, double* dx, double* du, double* lam, double* Sd, double* Sl, double* gam,
              double* Pd, const double* jsoft, const double* guess, double* Sg) {
  const int rows = N * 2 * nj;
  if (rows > QP_MAX_ROWS) return -1;
  if (nj > NJ_FULL && (rows > 1024 || jsoft)) return -2;   // a wide model: no HBM-row instance, no soft limits
  const bool gm = nj <= NJ_FULL && (rows > 1024 || (rows >= qp_gm_min_rows() && mode == QP_MODE_PCG));
  if (gm && mode == QP_MODE_PCG && !Sg) return -4;
  if (qp_lds_doubles(N, 2 * nj, nj, gm ? QP_MAX_ROWS : 1024) * sizeof(double) > 160 * 1024) return -3;
  TMPC_DISPATCH_NJ2(nj, qp(s, C, P, B, N, dt, precond, mode, x, u, active, G, A, Bm, cvec, tol, max_iter, iters, dx, du, lam,
                           Sd, Sl, gam, Pd, jsoft, guess, Sg))
}
int launch_ginv_soft(hipStream_t s, int nj, const CostDev* C, const ConstrDev* Cs, PList P, int B, int N,
                     const double* rho, const int* active, const double* x, const double* u, const double* mu,
                     const double* lam, double* Gk, double* jsoft) {
  if (nj > NJ_FULL) return -2;
  TMPC_DISPATCH_NJ2(nj, ginv_soft(s, C, Cs, P, B, N, rho, active, x, u, mu, lam, Gk, jsoft))
}

}  // namespace tmpc
