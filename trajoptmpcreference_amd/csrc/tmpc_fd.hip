// Per-knot forward-dynamics kernels (one lane per knot): the QP-build
// defects, the line-search merit terms, the unit-test entry point and the
// workload rollout.  Compiled in their own translation unit with the
// register-minimising scheduler (see Makefile): the fully unrolled
// articulated-body recursion for n = 6 otherwise spills to scratch.
#include "tmpc_internal.h"

namespace tmpc {

__device__ __forceinline__ bool use_QF(const CostDev* C, int k, int N) {
  return (k == N - 1) || (C->QF_start >= 0 && k >= C->QF_start);
}

// ======================================================================= per-knot forward dynamics
// Solver mode: lane = (b, k), k < N-1.  Writes qdd (the point the gradient is
// evaluated at, TrajoptPlant.py:313) and the dynamics defect
// c_{k+1} = x_{k+1} - f(x_k, u_k) (formKKTSystemBlocks :227-231); lane k = 0
// also writes c_0 = x_0 - xs (:213-214).
template <int NJ, bool CHAIN, class MT, class R>
__global__ void __launch_bounds__(256) k_qp_fd(MT M, PList P, int B, int N, double dt,
                                               const double* __restrict__ x, const double* __restrict__ u,
                                               const double* __restrict__ xs, const int* __restrict__ need,
                                               double* __restrict__ qdd_out, double* __restrict__ cvec) {
  constexpr int NX = 2 * NJ;
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int K = N - 1;
  if (gid >= B * K) return;
  const int p = gid / K, k = gid - p * K;
  if (!P.has(p, B)) return;
  const int b = P.at(p);
  if (!need[b]) return;
  const double* xb = x + (size_t)b * NX * N;
  const double* ub = u + (size_t)b * NJ * K;
  double q[NJ], qd[NJ], qdd[NJ];
  R qdr[NJ], ur[NJ], qddr[NJ], cq[NJ], sq[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    q[j] = xb[j * N + k];
    qd[j] = xb[(NJ + j) * N + k];
    qdr[j] = R(qd[j]);
    ur[j] = R(ub[j * K + k]);
    joint_cs(M, j, R(q[j]), cq[j], sq[j]);
  }
  fd_aba<NJ, CHAIN>(M, cq, sq, qdr, ur, qddr);
#pragma unroll
  for (int j = 0; j < NJ; ++j) qdd[j] = double(qddr[j]);
  const size_t kk = (size_t)b * K + k;
#pragma unroll
  for (int j = 0; j < NJ; ++j) qdd_out[kk * NJ + j] = qdd[j];
  double* cb = cvec + (size_t)b * N * NX;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    // x_{k+1} = x_k + dt * [qd; qdd]  (TrajoptPlant.py:95-97), rounded as NumPy does
    const double xq = __dadd_rn(q[j], __dmul_rn(dt, qd[j]));
    const double xv = __dadd_rn(qd[j], __dmul_rn(dt, qdd[j]));
    cb[(k + 1) * NX + j] = xb[j * N + k + 1] - xq;
    cb[(k + 1) * NX + NJ + j] = xb[(NJ + j) * N + k + 1] - xv;
  }
  if (k == 0) {
#pragma unroll
    for (int i = 0; i < NX; ++i) cb[i] = xb[i * N] - xs[(size_t)b * NX + i];
  }
}

// ======================================================================= line-search merit terms
// lane = (b, t, k): for trial step alpha_t evaluate the per-knot pieces of
// totalCost (:296-310), totalHardConstraintViolation (:273-294) and the
// directional derivative D (:635-648, gradient taken at x_new as the
// reference does).  Knot lane N-1 carries the terminal cost / D term and the
// |x_0 - xs| violation term.  SOFT: soft-limit value (slot 3, summed after
// the cost terms as totalCost does, :303-307) and jacobian . dxu added to D
// (:633-646).  terms: [B][T][N][4] = cost, violation, D, soft value.
// Two waves per SIMD (amdgpu_waves_per_eu(2)): left to itself the compiler took 256 VGPRs + 76 AGPRs, one
// wave per SIMD, with nothing to hide the dynamics' latencies; at two it spills 348 B/lane and the headline
// launch takes 0.142 ms instead of 0.195 (profiles/r04/ls_terms).
template <int NJ, bool CHAIN, bool SOFT, class MT, class R>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) k_ls_terms(MT M, const CostDev* __restrict__ C,
                                                  const ConstrDev* __restrict__ Cs, const double* __restrict__ mu,
                                                  const double* __restrict__ lam,
                                                  PList P, int B, int N, int T, double dt, const double* __restrict__ alphas,
                                                  const double* __restrict__ x, const double* __restrict__ u,
                                                  const double* __restrict__ xs, const double* __restrict__ dx,
                                                  const double* __restrict__ du, const int* __restrict__ active,
                                                  double* __restrict__ terms) {
  constexpr int NX = 2 * NJ, NU = NJ;
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= B * T * N) return;
  const int k = gid % N;
  const int pt = gid / N;
  const int p = pt / T, t = pt - p * T;
  if (!P.has(p, B)) return;
  const int b = P.at(p);
  if (!active[b]) return;
  const size_t bt = (size_t)b * T + t;
  const int K = N - 1;
  const double al = alphas[t];
  const double* xb = x + (size_t)b * NX * N;
  const double* ub = u + (size_t)b * NU * K;
  const double* dxb = dx ? dx + (size_t)b * N * NX : nullptr;
  const double* dub = du ? du + (size_t)b * K * NU : nullptr;
  double xk[NX], dxk[NX];
#pragma unroll
  for (int m = 0; m < NX; ++m) {
    dxk[m] = dxb ? dxb[k * NX + m] : 0.0;
    // x_new = x - alpha dx  (:619-622; alpha is a power of two: exact)
    xk[m] = dxb ? xb[m * N + k] - al * dxk[m] : xb[m * N + k];
  }
  const double* Qk = use_QF(C, k, N) ? C->QF : C->Q;
  double cost, Dk = 0.0;
  if (C->kind == COST_EE) {
    // UrdfCost value and gradient at the trial point (TrajoptCost.py:402-458)
    double gx[NX], Jt[NX * NX];
    cost = ee_eval<NJ>(C, Qk, xk, gx, Jt);
#pragma unroll
    for (int m = 0; m < NX; ++m) Dk += gx[m] * dxk[m];
  } else {
  double d[NX];
#pragma unroll
  for (int m = 0; m < NX; ++m) d[m] = xk[m] - C->xg[m];
  // value: 0.5 dx^T (Q dx) [+ 0.5 u^T (R u)]; gradient: [dx^T Q, u^T R]
  double vq = 0.0;
  if (C->diag) {   // the same chains without their exact-zero terms (CostDev.diag)
    const double pz = diag_poison(d, NX);
#pragma unroll
    for (int r = 0; r < NX; ++r) {
      const double qd = __fma_rn(Qk[r * NX + r], d[r], 0.0);
      vq = __fma_rn(d[r], qd, vq);
      Dk = __fma_rn(qd + pz, dxk[r], Dk);
    }
    vq = vq + pz;
  } else {
#pragma unroll
  for (int r = 0; r < NX; ++r) {
    double qd = 0.0, gq = 0.0;
#pragma unroll
    for (int c = 0; c < NX; ++c) {
      qd += Qk[r * NX + c] * d[c];
      gq += d[c] * Qk[c * NX + r];
    }
    vq += d[r] * qd;
    Dk += gq * dxk[r];
  }
  }
  cost = 0.5 * vq;
  }
  double viol = 0.0;
  double* out = terms + ((size_t)bt * N + k) * 4;
  double uk[NU], duk[NU];
#pragma unroll
  for (int m = 0; m < NU; ++m) uk[m] = duk[m] = 0.0;
  if (k < K) {
#pragma unroll
    for (int m = 0; m < NU; ++m) {
      duk[m] = dub ? dub[k * NU + m] : 0.0;
      uk[m] = dub ? ub[m * K + k] - al * duk[m] : ub[m * K + k];
    }
    double vr = 0.0;
    if (C->diag) {
      const double pz = diag_poison(uk, NU);
#pragma unroll
      for (int r = 0; r < NU; ++r) {
        const double ru = __fma_rn(C->R[r * NU + r], uk[r], 0.0);
        vr = __fma_rn(uk[r], ru, vr);
        Dk = __fma_rn(ru + pz, duk[r], Dk);
      }
      vr = vr + pz;
    } else {
#pragma unroll
    for (int r = 0; r < NU; ++r) {
      double ru = 0.0, gr = 0.0;
#pragma unroll
      for (int c = 0; c < NU; ++c) {
        ru += C->R[r * NU + c] * uk[c];
        gr += uk[c] * C->R[c * NU + r];
      }
      vr += uk[r] * ru;
      Dk += gr * duk[r];
    }
    }
    cost += 0.5 * vr;
    // dynamics defect at the trial point
    double qd[NJ], qdd[NJ];
    R cq[NJ], sq[NJ], qdr[NJ], ur[NJ], qddr[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      qd[j] = xk[NJ + j];
      qdr[j] = R(qd[j]);
      ur[j] = R(uk[j]);
      joint_cs(M, j, R(xk[j]), cq[j], sq[j]);
    }
    fd_aba<NJ, CHAIN>(M, cq, sq, qdr, ur, qddr);
#pragma unroll
    for (int j = 0; j < NJ; ++j) qdd[j] = double(qddr[j]);
#pragma unroll
    for (int m = 0; m < NX; ++m) {
      const double dxn = dxb ? dxb[(k + 1) * NX + m] : 0.0;
      const double xn = dxb ? xb[m * N + k + 1] - al * dxn : xb[m * N + k + 1];
      const double xdot = m < NJ ? qd[m] : qdd[m - NJ];
      const double f = __dadd_rn(xk[m], __dmul_rn(dt, xdot));
      viol += fabs(xn - f);
    }
  } else {
    // |x_0 - xs|_1 for the initial-state constraint
#pragma unroll
    for (int m = 0; m < NX; ++m) {
      const double x0 = dxb ? xb[m * N] - al * dxb[m] : xb[m * N];
      viol += fabs(x0 - xs[(size_t)b * NX + m]);
    }
  }
  double sv = 0.0;
  if (SOFT) {
    double z[3 * NJ], jac[3 * NJ];
#pragma unroll
    for (int m = 0; m < NX; ++m) z[m] = xk[m];
#pragma unroll
    for (int m = 0; m < NU; ++m) z[NX + m] = uk[m];
    const size_t ko = ((size_t)b * N + k) * 6 * NJ;
    sv = soft_knot<NJ>(Cs, mu + ko, lam + ko, k == K, z, jac);
    double Ds = 0.0;
#pragma unroll
    for (int m = 0; m < NX; ++m) Ds += jac[m] * dxk[m];
#pragma unroll
    for (int m = 0; m < NU; ++m) Ds += jac[NX + m] * duk[m];
    Dk = Dk + Ds;
  }
  out[0] = cost;
  out[1] = viol;
  out[2] = Dk;
  out[3] = sv;
}

// ======================================================================= kernel-level entry points
template <int NJ, bool CHAIN, class MT, class R>
__global__ void __launch_bounds__(256) k_unit_fd(MT M, int K, double dt,
                                                 const double* __restrict__ x, const double* __restrict__ u,
                                                 double* __restrict__ xnext, double* __restrict__ qdd_out) {
  constexpr int NX = 2 * NJ;
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  double q[NJ], qd[NJ], qdd[NJ];
  R qdr[NJ], ur[NJ], qddr[NJ], cq[NJ], sq[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    q[j] = x[(size_t)k * NX + j];
    qd[j] = x[(size_t)k * NX + NJ + j];
    qdr[j] = R(qd[j]);
    ur[j] = R(u[(size_t)k * NJ + j]);
    joint_cs(M, j, R(q[j]), cq[j], sq[j]);
  }
  fd_aba<NJ, CHAIN>(M, cq, sq, qdr, ur, qddr);
#pragma unroll
  for (int j = 0; j < NJ; ++j) qdd[j] = double(qddr[j]);
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    qdd_out[(size_t)k * NJ + j] = qdd[j];
    if (xnext) {
      xnext[(size_t)k * NX + j] = __dadd_rn(q[j], __dmul_rn(dt, qd[j]));
      xnext[(size_t)k * NX + NJ + j] = __dadd_rn(qd[j], __dmul_rn(dt, qdd[j]));
    }
  }
}

// sequential Euler rollout, one lane per problem (workload setup: §8d)
template <int NJ, bool CHAIN, class MT, class R>
__global__ void __launch_bounds__(64) k_rollout(MT M, PList P, int B, int N, double dt,
                                                double* __restrict__ x, const double* __restrict__ u,
                                                const int* __restrict__ mask) {
  constexpr int NX = 2 * NJ;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (!P.has(p, B)) return;
  const int b = P.at(p);
  if (mask && !mask[b]) return;
  const int K = N - 1;
  double* xb = x + (size_t)b * NX * N;
  const double* ub = u + (size_t)b * NJ * K;
  double q[NJ], qd[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) { q[j] = xb[j * N]; qd[j] = xb[(NJ + j) * N]; }
  for (int k = 0; k < K; ++k) {
    double qdd[NJ];
    R ur[NJ], qdr[NJ], qddr[NJ], cq[NJ], sq[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      ur[j] = R(ub[j * K + k]);
      qdr[j] = R(qd[j]);
      joint_cs(M, j, R(q[j]), cq[j], sq[j]);
    }
    fd_aba<NJ, CHAIN>(M, cq, sq, qdr, ur, qddr);
#pragma unroll
    for (int j = 0; j < NJ; ++j) qdd[j] = double(qddr[j]);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const double nq = __dadd_rn(q[j], __dmul_rn(dt, qd[j]));
      const double nv = __dadd_rn(qd[j], __dmul_rn(dt, qdd[j]));
      q[j] = nq;
      qd[j] = nv;
      xb[j * N + k + 1] = nq;
      xb[(NJ + j) * N + k + 1] = nv;
    }
  }
}

// ======================================================================= MPC step (oracle/mpc.py)
// One 64-lane workgroup per problem after a horizon solve: apply the first
// control to the plant, x_next = integrator(x_0, u_0) (TrajoptPlant.py:92-99),
// record it, and shift the trajectory by one knot for the warm start
// (x_k <- x_{k+1}, u_k <- u_{k+1}, last knot kept, x_0 <- x_next).
template <int NJ, bool CHAIN, class MT>
__global__ void __launch_bounds__(64) k_mpc_shift(MT M, int B, int N, double dt, int step, int steps,
                                                  double* __restrict__ x, double* __restrict__ u,
                                                  double* __restrict__ xe, double* __restrict__ ue) {
  constexpr int NX = 2 * NJ, NU = NJ;
  const int b = blockIdx.x, t = threadIdx.x;
  const int K = N - 1;
  double* xb = x + (size_t)b * NX * N;
  double* ub = u + (size_t)b * NU * K;
  __shared__ double xn[NX];
  if (t == 0) {
    // the simulated plant is fp64 in every precision mode
    double q[NJ], qd[NJ], uu[NJ], qdd[NJ], cq[NJ], sq[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      q[j] = xb[j * N];
      qd[j] = xb[(NJ + j) * N];
      uu[j] = ub[j * K];
      joint_cs(M, j, q[j], cq[j], sq[j]);
    }
    fd_aba<NJ, CHAIN>(M, cq, sq, qd, uu, qdd);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      xn[j] = __dadd_rn(q[j], __dmul_rn(dt, qd[j]));
      xn[NJ + j] = __dadd_rn(qd[j], __dmul_rn(dt, qdd[j]));
    }
#pragma unroll
    for (int m = 0; m < NX; ++m) xe[((size_t)b * NX + m) * (steps + 1) + step + 1] = xn[m];
#pragma unroll
    for (int m = 0; m < NU; ++m) ue[((size_t)b * NU + m) * steps + step] = uu[m];
  }
  __syncthreads();
  // shift each state / control row (rows are contiguous in the [nx][N] layout)
  for (int m = t; m < NX; m += 64) {
    double* row = xb + m * N;
    for (int k = 0; k < N - 1; ++k) row[k] = row[k + 1];
    row[0] = xn[m];
  }
  for (int m = t; m < NU; m += 64) {
    double* row = ub + m * K;
    for (int k = 0; k < K - 1; ++k) row[k] = row[k + 1];
  }
}

#define TMPC_GRID(n, bs) dim3(((n) + (bs) - 1) / (bs)), dim3(bs)

template <int NJ, bool CHAIN, class MT>
struct LaunchFD {
  static void qp_fd(bool f32, hipStream_t s, const ModelDev* M, PList P, int B, int N, double dt, const double* x,
                    const double* u, const double* xs, const int* need, double* qdd, double* cvec) {
    if constexpr (!kWide<NJ>) {   // fp32 instances for up to NJ_FULL joints only
      if (f32) {
        hipLaunchKernelGGL((k_qp_fd<NJ, CHAIN, MT, float>), TMPC_GRID(B * (N - 1), 256), 0, s, MT::make(M), P, B, N, dt, x, u,
                           xs, need, qdd, cvec);
        return;
      }
    }
    hipLaunchKernelGGL((k_qp_fd<NJ, CHAIN, MT, double>), TMPC_GRID(B * (N - 1), 256), 0, s, MT::make(M), P, B, N, dt, x, u,
                       xs, need, qdd, cvec);
  }
  // a runtime model (ModelRef) takes the general-topology line-search instance even for a chain: with
  // runtime coefficients the chain specialisation's unrolled recursion spills 9x more (k_ls_terms<6,
  // chain, ModelRef, double> 19 kB per lane against 2.2 kB; 11.2 -> 1.9 ms per headline launch, DESIGN.md
  // 4a); the other FD kernels keep the chain instance, which measured faster for them
  static constexpr bool LCHAIN = MT::STATIC ? CHAIN : false;
  static void ls_terms(bool f32, hipStream_t s, const ModelDev* M, const CostDev* C, const ConstrDev* Cs, const double* mu,
                       const double* lam, PList P, int B, int N, int T, double dt, const double* alphas, const double* x,
                       const double* u, const double* xs, const double* dx, const double* du, const int* active,
                       double* terms) {
#define TMPC_LS(SOFTV, RV)                                                                                        \
    hipLaunchKernelGGL((k_ls_terms<NJ, LCHAIN, SOFTV, MT, RV>), TMPC_GRID(B * T * N, 256), 0, s, MT::make(M), C, Cs, mu, \
                       lam, P, B, N, T, dt, alphas, x, u, xs, dx, du, active, terms);
    if constexpr (kWide<NJ>) {   // a wide model: fp64 without soft limits only (check_ready refuses the rest)
      TMPC_LS(false, double)
    } else {
      if (mu) { if (f32) { TMPC_LS(true, float) } else { TMPC_LS(true, double) } }
      else { if (f32) { TMPC_LS(false, float) } else { TMPC_LS(false, double) } }
    }
#undef TMPC_LS
  }
  static void unit_fd(bool f32, hipStream_t s, const ModelDev* M, int K, double dt, const double* x, const double* u,
                      double* xnext, double* qdd) {
    if constexpr (!kWide<NJ>) {   // fp32 instances for up to NJ_FULL joints only
      if (f32) {
        hipLaunchKernelGGL((k_unit_fd<NJ, CHAIN, MT, float>), TMPC_GRID(K, 256), 0, s, MT::make(M), K, dt, x, u, xnext, qdd);
        return;
      }
    }
    hipLaunchKernelGGL((k_unit_fd<NJ, CHAIN, MT, double>), TMPC_GRID(K, 256), 0, s, MT::make(M), K, dt, x, u, xnext, qdd);
  }
  static void mpc_shift(hipStream_t s, const ModelDev* M, int B, int N, double dt, int step, int steps, double* x,
                        double* u, double* xe, double* ue) {
    hipLaunchKernelGGL((k_mpc_shift<NJ, CHAIN, MT>), dim3(B), dim3(64), 0, s, MT::make(M), B, N, dt, step, steps, x,
                       u, xe, ue);
  }
  static void rollout(bool f32, hipStream_t s, const ModelDev* M, int B, int N, double dt, double* x, const double* u,
                      PList P, const int* mask) {
    if constexpr (!kWide<NJ>) {   // fp32 instances for up to NJ_FULL joints only
      if (f32) {
        hipLaunchKernelGGL((k_rollout<NJ, CHAIN, MT, float>), TMPC_GRID(B, 64), 0, s, MT::make(M), P, B, N, dt, x, u, mask);
        return;
      }
    }
    hipLaunchKernelGGL((k_rollout<NJ, CHAIN, MT, double>), TMPC_GRID(B, 64), 0, s, MT::make(M), P, B, N, dt, x, u, mask);
  }
};

// dispatch tables over the joint count and the chain specialisation
#define TMPC_DISPATCH_NJ(nj, chain, CALL)                                                              \
  switch (mid) {                                                                                       \
    TMPC_STATIC_MODEL_CASES(LaunchFD, CALL)                                                            \
    default: break;                                                                                    \
  }                                                                                                    \
  switch (nj) {                                                                                        \
    case 1: if (chain) LaunchFD<1, true, ModelRef>::CALL; else LaunchFD<1, false, ModelRef>::CALL; break;  \
    case 2: if (chain) LaunchFD<2, true, ModelRef>::CALL; else LaunchFD<2, false, ModelRef>::CALL; break;  \
    case 3: if (chain) LaunchFD<3, true, ModelRef>::CALL; else LaunchFD<3, false, ModelRef>::CALL; break;  \
    case 4: if (chain) LaunchFD<4, true, ModelRef>::CALL; else LaunchFD<4, false, ModelRef>::CALL; break;  \
    case 5: if (chain) LaunchFD<5, true, ModelRef>::CALL; else LaunchFD<5, false, ModelRef>::CALL; break;  \
    case 6: if (chain) LaunchFD<6, true, ModelRef>::CALL; else LaunchFD<6, false, ModelRef>::CALL; break;  \
    case 7: if (chain) LaunchFD<7, true, ModelRef>::CALL; else LaunchFD<7, false, ModelRef>::CALL; break;  \
    TMPC_WIDE_CASES(LaunchFD, CALL)                                                                    \
    default: return -2;                                                                                \
  }                                                                                                    \
  return 0;

int launch_qp_fd(bool f32, hipStream_t s, int nj, bool chain, int mid, const ModelDev* M, PList P, int B, int N,
                 double dt, const double* x, const double* u, const double* xs, const int* need, double* qdd,
                 double* cvec) {
  TMPC_DISPATCH_NJ(nj, chain, qp_fd(f32, s, M, P, B, N, dt, x, u, xs, need, qdd, cvec))
}
int launch_ls_terms(bool f32, hipStream_t s, int nj, bool chain, int mid, const ModelDev* M, const CostDev* C,
                    const ConstrDev* Cs, const double* mu, const double* lam, PList P, int B, int N, int T, double dt,
                    const double* alphas, const double* x, const double* u, const double* xs, const double* dx,
                    const double* du, const int* active, double* terms) {
  TMPC_DISPATCH_NJ(nj, chain, ls_terms(f32, s, M, C, Cs, mu, lam, P, B, N, T, dt, alphas, x, u, xs, dx, du, active,
                                       terms))
}
int launch_unit_fd(bool f32, hipStream_t s, int nj, bool chain, int mid, const ModelDev* M, int K, double dt,
                   const double* x, const double* u, double* xnext, double* qdd) {
  TMPC_DISPATCH_NJ(nj, chain, unit_fd(f32, s, M, K, dt, x, u, xnext, qdd))
}
int launch_rollout(bool f32, hipStream_t s, int nj, bool chain, int mid, const ModelDev* M, int B, int N, double dt,
                   double* x, const double* u, PList P, const int* mask) {
  TMPC_DISPATCH_NJ(nj, chain, rollout(f32, s, M, B, N, dt, x, u, P, mask))
}

int launch_mpc_shift(hipStream_t s, int nj, bool chain, int mid, const ModelDev* M, int B, int N, double dt, int step,
                     int steps, double* x, double* u, double* xe, double* ue) {
  TMPC_DISPATCH_NJ(nj, chain, mpc_shift(s, M, B, N, dt, step, steps, x, u, xe, ue))
}

}  // namespace tmpc
