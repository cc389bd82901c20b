// iLQR on the GPU.  The reference has no iLQR
// (MPCSolverMethods.iLQR is an enum value only, TrajoptMPCReference.py:21-27);
// the algorithm is defined in oracle/ilqr.py on the reference's plugin hooks
// and *_SQP_DDP option keys, and these kernels follow it step for step:
//
//   k_ilqr_backward  one 64-lane workgroup per problem walks k = N-2 .. 0:
//                    the Q-function products (V_xx [A B], [A B]^T (V_xx [A B]))
//                    as one-entry-per-lane dot products over LDS-resident
//                    12x12 / 12x6 tiles, the 6x6 Cholesky solve for [K | d] with
//                    one right-hand-side column per lane, and the value-function
//                    update; K_k, d_k go to HBM for the forward sweep;
//   k_ilqr_forward   lane = (problem, alpha trial): the sequential closed-loop
//                    rollout u^ = u + alpha d + K (x^ - x), x^+ = f(x^, u^) with
//                    the articulated-body dynamics in registers, and the trial
//                    cost; all trials alpha = 1, f, f^2, ... speculatively;
//   k_ilqr_decide    per problem: the acceptance test in the reference's alpha
//                    order, the rho schedule / exit codes of the SQP
//                    (:457-481), the trace row and the copy of the accepted
//                    trajectory.
#include "tmpc_internal.h"

namespace tmpc {

__device__ __forceinline__ bool use_QF(const CostDev* C, int k, int N) {
  return (k == N - 1) || (C->QF_start >= 0 && k >= C->QF_start);
}

// ======================================================================= backward (Riccati) sweep
template <int NJ, class R>
struct IlqrLds {
  static constexpr int NX = 2 * NJ, NU = NJ;
  R Vxx[NX * NX], Vx[NX];
  R A[NX * NX], Bm[NX * NU];
  R P[NX * NX], VB[NX * NU];        // V_xx A, V_xx B (P then holds the unsymmetrised V_xx)
  R Qxx[NX * NX], Qux[NU * NX], Quu[NU * NU], Qx[NX], Qu[NU];
  R KD[NU * (NX + 1)];              // [Q_uu^-1 Q_ux | Q_uu^-1 Q_u], row-major
  R lx[NX], lu[NU], jac[3 * NJ];
  R dv[2];
  int fail;
};

template <int NJ, class R>
__global__ void __launch_bounds__(64) k_ilqr_backward(const CostDev* __restrict__ C, const ConstrDev* __restrict__ Cs,
                                                      int B, int N, const double* __restrict__ x,
                                                      const double* __restrict__ u, const double* __restrict__ rho_in,
                                                      const int* __restrict__ active, const double* __restrict__ Aall,
                                                      const double* __restrict__ Ball, const double* __restrict__ mu,
                                                      const double* __restrict__ lam, double* __restrict__ Kout,
                                                      double* __restrict__ dout, double* __restrict__ dV,
                                                      int* __restrict__ ok) {
  constexpr int NX = 2 * NJ, NU = NJ, NC = NX + 1, MC = 6 * NJ;
  const int b = blockIdx.x;
  if (!active[b]) return;
  __shared__ IlqrLds<NJ, R> L;
  const int t = threadIdx.x;
  const int K = N - 1;
  const R rho = R(rho_in[b]);
  const double* xb = x + (size_t)b * NX * N;
  const double* ub = u + (size_t)b * NU * K;
  const bool soft = Cs->any != 0;

  // stage the cost derivatives of knot k (QuadraticCost.gradient / hessian, TrajoptCost.py:58-83,
  // plus the soft-limit jacobian, :220-225) into L.lx / L.lu / L.jac
  auto stage_l = [&](int k) {
    const bool term = k == K;
    if (soft && t == 0) {
      double z[3 * NJ], jac[3 * NJ];
#pragma unroll
      for (int m = 0; m < NX; ++m) z[m] = xb[m * N + k];
#pragma unroll
      for (int m = 0; m < NU; ++m) z[NX + m] = term ? 0.0 : ub[m * K + k];
      const size_t ko = ((size_t)b * N + k) * MC;
      soft_knot<NJ>(Cs, mu + ko, lam + ko, term, z, jac);
#pragma unroll
      for (int m = 0; m < 3 * NJ; ++m) L.jac[m] = jac[m];
    }
    if (!soft && t < 3 * NJ) L.jac[t] = 0.0;
    __syncthreads();
    const double* Qk = use_QF(C, k, N) ? C->QF : C->Q;
    if (t < NX) {
      R g = 0.0;
      for (int m = 0; m < NX; ++m) g += R(xb[m * N + k] - C->xg[m]) * R(Qk[m * NX + t]);
      L.lx[t] = g + L.jac[t];
    } else if (t < NX + NU && !term) {
      const int c = t - NX;
      R g = 0.0;
      for (int m = 0; m < NU; ++m) g += R(ub[m * K + k]) * R(C->R[m * NU + c]);
      L.lu[c] = g + L.jac[NX + c];
    }
  };
  // l_xx (+ per-type outer products on the q / qd diagonal blocks)
  auto lxx = [&](int k, int r, int c) -> R {
    const double* Qk = use_QF(C, k, N) ? C->QF : C->Q;
    const R o = (r / NJ == c / NJ) ? L.jac[r] * L.jac[c] : 0.0;
    return R(Qk[r * NX + c]) + o;
  };

  // terminal value function: V_x = l_x(N-1), V_xx = l_xx(N-1)
  stage_l(K);
  __syncthreads();
  for (int e = t; e < NX * NX; e += 64) L.Vxx[e] = lxx(K, e / NX, e % NX);
  if (t < NX) L.Vx[t] = L.lx[t];
  if (t == 0) {
    L.dv[0] = L.dv[1] = 0.0;
    L.fail = 0;
  }
  __syncthreads();

  for (int k = K - 1; k >= 0; --k) {
    for (int e = t; e < NX * NX; e += 64) L.A[e] = Aall[((size_t)b * K + k) * NX * NX + e];
    for (int e = t; e < NX * NU; e += 64) L.Bm[e] = Ball[((size_t)b * K + k) * NX * NU + e];
    stage_l(k);
    __syncthreads();
    // P = V_xx A, R = V_xx B; Q_x = l_x + A^T V_x, Q_u = l_u + B^T V_x
    for (int e = t; e < NX * NX + NX * NU + NX + NU; e += 64) {
      if (e < NX * NX) {
        const int r = e / NX, c = e % NX;
        R s = 0.0;
#pragma unroll
        for (int m = 0; m < NX; ++m) s += L.Vxx[r * NX + m] * L.A[m * NX + c];
        L.P[e] = s;
      } else if (e < NX * NX + NX * NU) {
        const int f = e - NX * NX, r = f / NU, c = f % NU;
        R s = 0.0;
#pragma unroll
        for (int m = 0; m < NX; ++m) s += L.Vxx[r * NX + m] * L.Bm[m * NU + c];
        L.VB[f] = s;
      } else if (e < NX * NX + NX * NU + NX) {
        const int r = e - NX * NX - NX * NU;
        R s = 0.0;
#pragma unroll
        for (int m = 0; m < NX; ++m) s += L.A[m * NX + r] * L.Vx[m];
        L.Qx[r] = L.lx[r] + s;
      } else {
        const int r = e - NX * NX - NX * NU - NX;
        R s = 0.0;
#pragma unroll
        for (int m = 0; m < NX; ++m) s += L.Bm[m * NU + r] * L.Vx[m];
        L.Qu[r] = L.lu[r] + s;
      }
    }
    __syncthreads();
    // Q_xx = l_xx + A^T P, Q_uu = l_uu + B^T R + rho I, Q_ux = B^T P
    for (int e = t; e < NX * NX + NU * NU + NU * NX; e += 64) {
      if (e < NX * NX) {
        const int r = e / NX, c = e % NX;
        R s = 0.0;
#pragma unroll
        for (int m = 0; m < NX; ++m) s += L.A[m * NX + r] * L.P[m * NX + c];
        L.Qxx[e] = lxx(k, r, c) + s;
      } else if (e < NX * NX + NU * NU) {
        const int f = e - NX * NX, r = f / NU, c = f % NU;
        R s = 0.0;
#pragma unroll
        for (int m = 0; m < NX; ++m) s += L.Bm[m * NU + r] * L.VB[m * NU + c];
        L.Quu[f] = (R(C->R[f]) + L.jac[NX + r] * L.jac[NX + c]) + s + (r == c ? rho : R(0));
      } else {
        const int f = e - NX * NX - NU * NU, r = f / NX, c = f % NX;
        R s = 0.0;
#pragma unroll
        for (int m = 0; m < NX; ++m) s += L.Bm[m * NU + r] * L.P[m * NX + c];
        L.Qux[f] = s;
      }
    }
    __syncthreads();
    // [K | d] = -Q_uu^-1 [Q_ux | Q_u]: Cholesky Q_uu = L L^T (every lane, from LDS), then lane c
    // solves its right-hand-side column c; Q_uu not positive definite -> backward failure
    if (t < NC) {
      R Lc[NU][NU];
      bool pd = true;
#pragma unroll
      for (int j = 0; j < NU; ++j) {
        R s = L.Quu[j * NU + j];
#pragma unroll
        for (int m = 0; m < j; ++m) s -= Lc[j][m] * Lc[j][m];
        pd = pd && (s > R(0));
        const R dj = sqrt(s);
        Lc[j][j] = dj;
#pragma unroll
        for (int i = j + 1; i < NU; ++i) {
          R v = L.Quu[i * NU + j];
#pragma unroll
          for (int m = 0; m < j; ++m) v -= Lc[i][m] * Lc[j][m];
          Lc[i][j] = v / dj;
        }
      }
      R y[NU];
#pragma unroll
      for (int i = 0; i < NU; ++i) {
        R v = t < NX ? L.Qux[i * NX + t] : L.Qu[i];
#pragma unroll
        for (int m = 0; m < i; ++m) v -= Lc[i][m] * y[m];
        y[i] = v / Lc[i][i];
      }
#pragma unroll
      for (int i = NU - 1; i >= 0; --i) {
        R v = y[i];
#pragma unroll
        for (int m = i + 1; m < NU; ++m) v -= Lc[m][i] * y[m];
        y[i] = v / Lc[i][i];
      }
#pragma unroll
      for (int i = 0; i < NU; ++i) L.KD[i * NC + t] = -y[i];
      if (t == 0 && !pd) L.fail = 1;
    }
    __syncthreads();
    if (L.fail) break;
    // V_x = Q_x + Q_ux^T d, M = Q_xx + Q_ux^T K; dV1 += d^T Q_u, dV2 += d^T Q_uu d / 2
    for (int e = t; e < NX * NX + NX; e += 64) {
      if (e < NX * NX) {
        const int r = e / NX, c = e % NX;
        R s = 0.0;
#pragma unroll
        for (int m = 0; m < NU; ++m) s += L.Qux[m * NX + r] * L.KD[m * NC + c];
        L.P[e] = L.Qxx[e] + s;
      } else {
        const int r = e - NX * NX;
        R s = 0.0;
#pragma unroll
        for (int m = 0; m < NU; ++m) s += L.Qux[m * NX + r] * L.KD[m * NC + NX];
        L.Vx[r] = L.Qx[r] + s;
      }
    }
    if (t == 63) {
      R s1 = 0.0, s2 = 0.0;
#pragma unroll
      for (int i = 0; i < NU; ++i) {
        const R di = L.KD[i * NC + NX];
        s1 += di * L.Qu[i];
        R qd = 0.0;
#pragma unroll
        for (int m = 0; m < NU; ++m) qd += L.Quu[i * NU + m] * L.KD[m * NC + NX];
        s2 += di * qd;
      }
      L.dv[0] += s1;
      L.dv[1] += R(0.5) * s2;
    }
    // K_k, d_k to HBM ([B][K][NU][NX], [B][K][NU])
    for (int e = t; e < NU * NC; e += 64) {
      const int i = e / NC, c = e % NC;
      if (c < NX)
        Kout[(((size_t)b * K + k) * NU + i) * NX + c] = double(L.KD[e]);
      else
        dout[((size_t)b * K + k) * NU + i] = double(L.KD[e]);
    }
    __syncthreads();
    for (int e = t; e < NX * NX; e += 64) {
      const int r = e / NX, c = e % NX;
      L.Vxx[e] = R(0.5) * (L.P[r * NX + c] + L.P[c * NX + r]);
    }
    __syncthreads();
  }
  if (t == 0) {
    ok[b] = L.fail ? 0 : 1;
    dV[2 * b] = double(L.dv[0]);
    dV[2 * b + 1] = double(L.dv[1]);
  }
}

// ======================================================================= forward sweep (closed-loop rollouts)
// lane = (b, trial t).  INIT: J at the current trajectory (no rollout).  Trial
// trajectories are kept ([B][T][nx][N], [B][T][nu][N-1]) so the decision kernel
// copies the accepted one.  Cost sums in totalCost's order (:296-310): the
// QuadraticCost terms, then the soft values.
template <int NJ, bool CHAIN, bool SOFT, class MT, class R>
__global__ void __launch_bounds__(64) k_ilqr_forward(MT Mg, const CostDev* __restrict__ C,
                                                     const ConstrDev* __restrict__ Cs, const double* __restrict__ mu,
                                                     const double* __restrict__ lam, int B, int N, int T, double dt,
                                                     int init, const double* __restrict__ alphas,
                                                     const double* __restrict__ x, const double* __restrict__ u,
                                                     const double* __restrict__ Kg, const double* __restrict__ dg,
                                                     const int* __restrict__ active, const int* __restrict__ ok,
                                                     double* __restrict__ xt, double* __restrict__ ut,
                                                     double* __restrict__ Jt) {
  // the runtime model is staged in LDS (tmpc_device.h, stage_model); compiled models need no data
  __shared__ ModelDev sM;
  MT M = Mg;
  if constexpr (!MT::STATIC) M = ModelRef{stage_model(Mg.p, &sM)};
  constexpr int NX = 2 * NJ, NU = NJ;
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= B * T) return;
  const int b = gid / T, tr = gid - b * T;
  if (!active[b] || (!init && !ok[b])) return;
  const int K = N - 1;
  const double al = init ? 0.0 : alphas[tr];
  const double* xb = x + (size_t)b * NX * N;
  const double* ub = u + (size_t)b * NU * K;
  double* xo = xt + (size_t)gid * NX * N;
  double* uo = ut + (size_t)gid * NU * K;
  double xh[NX];
#pragma unroll
  for (int m = 0; m < NX; ++m) xh[m] = xb[m * N];
  double J = 0.0;
  for (int k = 0; k <= K; ++k) {
    const bool term = k == K;
    double uh[NU];
    if (!init) {
#pragma unroll
      for (int m = 0; m < NX; ++m) xo[m * N + k] = xh[m];
    } else {
#pragma unroll
      for (int m = 0; m < NX; ++m) xh[m] = xb[m * N + k];
    }
    if (!term) {
      if (init) {
#pragma unroll
        for (int i = 0; i < NU; ++i) uh[i] = ub[i * K + k];
      } else {
        const double* Kk = Kg + ((size_t)b * K + k) * NU * NX;
        const double* dk = dg + ((size_t)b * K + k) * NU;
#pragma unroll
        for (int i = 0; i < NU; ++i) {
          double fb = 0.0;
#pragma unroll
          for (int m = 0; m < NX; ++m) fb += Kk[i * NX + m] * (xh[m] - xb[m * N + k]);
          uh[i] = (ub[i * K + k] + al * dk[i]) + fb;
          uo[i * K + k] = uh[i];
        }
      }
    }
    // QuadraticCost.value (TrajoptCost.py:49-56): 0.5 dx^T (Q dx) [+ 0.5 u^T (R u)]
    const double* Qk = use_QF(C, k, N) ? C->QF : C->Q;
    double vq = 0.0;
#pragma unroll
    for (int r = 0; r < NX; ++r) {
      double qd = 0.0;
#pragma unroll
      for (int c = 0; c < NX; ++c) qd += Qk[r * NX + c] * (xh[c] - C->xg[c]);
      vq += (xh[r] - C->xg[r]) * qd;
    }
    double cost = 0.5 * vq;
    if (!term) {
      double vr = 0.0;
#pragma unroll
      for (int r = 0; r < NU; ++r) {
        double ru = 0.0;
#pragma unroll
        for (int c = 0; c < NU; ++c) ru += C->R[r * NU + c] * uh[c];
        vr += uh[r] * ru;
      }
      cost += 0.5 * vr;
    }
    J = J + cost;
    if (!term && !init) {
      double qd[NJ], qdd[NJ];
      R cq[NJ], sq[NJ], qdr[NJ], ur[NJ], qddr[NJ];
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        qd[j] = xh[NJ + j];
        qdr[j] = R(qd[j]);
        ur[j] = R(uh[j]);
        joint_cs(M, j, R(xh[j]), cq[j], sq[j]);
      }
      fd_aba<NJ, CHAIN>(M, cq, sq, qdr, ur, qddr);
#pragma unroll
      for (int j = 0; j < NJ; ++j) qdd[j] = double(qddr[j]);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const double nq = __dadd_rn(xh[j], __dmul_rn(dt, qd[j]));
        const double nv = __dadd_rn(xh[NJ + j], __dmul_rn(dt, qdd[j]));
        xh[j] = nq;
        xh[NJ + j] = nv;
      }
    }
  }
  if (SOFT) {
    // value_soft_constraints per knot, summed after the cost terms
    const double* xs_ = init ? xb : xo;
    const double* us_ = init ? ub : uo;
    for (int k = 0; k <= K; ++k) {
      double z[3 * NJ], jac[3 * NJ];
#pragma unroll
      for (int m = 0; m < NX; ++m) z[m] = xs_[m * N + k];
#pragma unroll
      for (int m = 0; m < NU; ++m) z[NX + m] = k < K ? us_[m * K + k] : 0.0;
      const size_t ko = ((size_t)b * N + k) * 6 * NJ;
      J = J + soft_knot<NJ>(Cs, mu + ko, lam + ko, k == K, z, jac);
    }
  }
  Jt[gid] = J;
}

// ======================================================================= decision + state machine
// One 64-lane workgroup per problem.  Acceptance ratio (J - J^) / (-alpha (dV1 + alpha dV2)) in
// [exp_red_min, exp_red_max] in the reference's alpha order (oracle/ilqr.py), rho schedule and exit
// codes of reduce_regularization / check_for_exit_or_error (:457-481), trace row, trajectory copy.
__global__ void __launch_bounds__(64) k_ilqr_decide(int B, int N, int NX, int NU, int T, int init,
                                                    const double* __restrict__ alphas, SolverOpts o,
                                                    const double* __restrict__ Jt, const double* __restrict__ dV,
                                                    const int* __restrict__ okb, const double* __restrict__ xt,
                                                    const double* __restrict__ ut, double* __restrict__ x,
                                                    double* __restrict__ u, ProbState st, TraceDev tr,
                                                    int* __restrict__ active_count,
                                                    unsigned long long* __restrict__ counters) {
  const int b = blockIdx.x;
  if (!st.active[b]) return;
  __shared__ int s_choice;
  const int t = threadIdx.x;
  const int W = o.max_iter_sqp + 1;
  const int K = N - 1;
  if (t == 0) {
    if (init) {
      const double J = Jt[(size_t)b * T];
      st.J[b] = J;
      st.c[b] = 0.0;
      st.merit[b] = J;
      const size_t e = (size_t)b * W;
      tr.iteration[e] = 0; tr.ls_iter[e] = 0; tr.alpha[e] = 1.0; tr.rho[e] = st.rho[b];
      tr.J[e] = J; tr.c[e] = 0.0; tr.merit[e] = J; tr.D[e] = __builtin_nan(""); tr.ratio[e] = __builtin_nan("");
      tr.accepted[e] = 0; tr.pcg_iters[e] = 0;
      *active_count = 1;   // the host only tests for zero
      s_choice = -1;
    } else {
      const double J = st.J[b];
      double rho = st.rho[b], drho = st.drho[b];
      const bool bok = okb[b] != 0;
      const double dV1 = dV[2 * b], dV2 = dV[2 * b + 1];
      int choice = -1, ls = 0;
      double al = 0.0, ratio = __builtin_nan(""), Jn = J, deltaJ = 0.0;
      if (bok) {
        for (int tt = 0; tt < T; ++tt) {
          al = alphas[tt];
          ls = tt;
          Jn = Jt[(size_t)b * T + tt];
          deltaJ = J - Jn;
          ratio = deltaJ / (-al * (dV1 + al * dV2));
          if (ratio >= o.exp_red_min && ratio <= o.exp_red_max) {
            choice = tt;
            break;
          }
        }
      }
      const bool error = choice < 0;
      const int it = st.iter[b];
      const size_t e = (size_t)b * W + it + 1;
      if (counters) {
        // [0] problem-iterations, [2] iterations with a fresh dynamics gradient
        atomicAdd(&counters[0], 1ull);
        atomicAdd(&counters[2], (unsigned long long)st.need_grad[b]);
      }
      if (!error) {
        st.J[b] = Jn;
        st.merit[b] = Jn;
        drho = fmin(drho / o.rho_factor, 1.0 / o.rho_factor);
        rho = fmax(rho * drho, o.rho_min);
      }
      tr.iteration[e] = it; tr.ls_iter[e] = bok ? ls : 0; tr.alpha[e] = bok ? al : 0.0; tr.rho[e] = rho;
      tr.J[e] = error ? J : Jn; tr.c[e] = 0.0; tr.merit[e] = error ? J : Jn;
      tr.D[e] = bok ? dV1 : __builtin_nan(""); tr.ratio[e] = bok ? ratio : __builtin_nan("");
      tr.accepted[e] = error ? 0 : 1; tr.pcg_iters[e] = 0;
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
      else *active_count = 1;
      s_choice = choice;
    }
  }
  __syncthreads();
  const int choice = s_choice;
  if (choice >= 0) {
    const double* xs_ = xt + ((size_t)b * T + choice) * NX * N;
    const double* us_ = ut + ((size_t)b * T + choice) * NU * K;
    for (int e = t; e < NX * N; e += 64) x[(size_t)b * NX * N + e] = xs_[e];
    for (int e = t; e < NU * K; e += 64) u[(size_t)b * NU * K + e] = us_[e];
  }
}

// ======================================================================= launchers
#define TMPC_GRID(n, bs) dim3(((n) + (bs) - 1) / (bs)), dim3(bs)

template <int NJ, bool CHAIN, class MT>
struct LaunchIlqr {
  static void backward(bool f32, hipStream_t s, const CostDev* C, const ConstrDev* Cs, int B, int N, const double* x,
                       const double* u, const double* rho, const int* active, const double* A, const double* Bm,
                       const double* mu, const double* lam, double* K, double* d, double* dV, int* ok) {
    if (f32)
      hipLaunchKernelGGL((k_ilqr_backward<NJ, float>), dim3(B), dim3(64), 0, s, C, Cs, B, N, x, u, rho, active, A, Bm, mu,
                         lam, K, d, dV, ok);
    else
      hipLaunchKernelGGL((k_ilqr_backward<NJ, double>), dim3(B), dim3(64), 0, s, C, Cs, B, N, x, u, rho, active, A, Bm, mu,
                         lam, K, d, dV, ok);
  }
  static void forward(bool f32, hipStream_t s, const ModelDev* M, const CostDev* C, const ConstrDev* Cs, const double* mu,
                      const double* lam, int B, int N, int T, double dt, int init, const double* alphas,
                      const double* x, const double* u, const double* K, const double* d, const int* active,
                      const int* ok, double* xt, double* ut, double* Jt) {
#define TMPC_FWD(SOFTV, RV)                                                                                          \
    hipLaunchKernelGGL((k_ilqr_forward<NJ, CHAIN, SOFTV, MT, RV>), TMPC_GRID(B * T, 64), 0, s, MT::make(M), C, Cs, mu, \
                       lam, B, N, T, dt, init, alphas, x, u, K, d, active, ok, xt, ut, Jt);
    if (mu) { if (f32) { TMPC_FWD(true, float) } else { TMPC_FWD(true, double) } }
    else { if (f32) { TMPC_FWD(false, float) } else { TMPC_FWD(false, double) } }
#undef TMPC_FWD
  }
};

#define TMPC_DISPATCH_ILQR(nj, chain, CALL)                                                              \
  switch (mid) {                                                                                       \
    TMPC_STATIC_MODEL_CASES(LaunchIlqr, CALL)                                                            \
    default: break;                                                                                    \
  }                                                                                                    \
  switch (nj) {                                                                                        \
    case 1: if (chain) LaunchIlqr<1, true, ModelRef>::CALL; else LaunchIlqr<1, false, ModelRef>::CALL; break;  \
    case 2: if (chain) LaunchIlqr<2, true, ModelRef>::CALL; else LaunchIlqr<2, false, ModelRef>::CALL; break;  \
    case 3: if (chain) LaunchIlqr<3, true, ModelRef>::CALL; else LaunchIlqr<3, false, ModelRef>::CALL; break;  \
    case 4: if (chain) LaunchIlqr<4, true, ModelRef>::CALL; else LaunchIlqr<4, false, ModelRef>::CALL; break;  \
    case 5: if (chain) LaunchIlqr<5, true, ModelRef>::CALL; else LaunchIlqr<5, false, ModelRef>::CALL; break;  \
    case 6: if (chain) LaunchIlqr<6, true, ModelRef>::CALL; else LaunchIlqr<6, false, ModelRef>::CALL; break;  \
    case 7: if (chain) LaunchIlqr<7, true, ModelRef>::CALL; else LaunchIlqr<7, false, ModelRef>::CALL; break;  \
    default: return -2;                                                                                \
  }                                                                                                    \
  return 0;

int launch_ilqr_backward(bool f32, hipStream_t s, int nj, const CostDev* C, const ConstrDev* Cs, int B, int N,
                         const double* x, const double* u, const double* rho, const int* active, const double* A,
                         const double* Bm, const double* mu, const double* lam, double* K, double* d, double* dV,
                         int* ok) {
  const int mid = 0;
  TMPC_DISPATCH_ILQR(nj, true, backward(f32, s, C, Cs, B, N, x, u, rho, active, A, Bm, mu, lam, K, d, dV, ok))
}

int launch_ilqr_forward(bool f32, hipStream_t s, int nj, bool chain, int mid, const ModelDev* M, const CostDev* C,
                        const ConstrDev* Cs, const double* mu, const double* lam, int B, int N, int T, double dt,
                        int init, const double* alphas, const double* x, const double* u, const double* K,
                        const double* d, const int* active, const int* ok, double* xt, double* ut, double* Jt) {
  TMPC_DISPATCH_ILQR(nj, chain, forward(f32, s, M, C, Cs, mu, lam, B, N, T, dt, init, alphas, x, u, K, d, active, ok,
                                        xt, ut, Jt))
}

void launch_ilqr_decide(hipStream_t s, int B, int N, int NX, int NU, int T, int init, const double* alphas,
                        const SolverOpts& o, const double* Jt, const double* dV, const int* ok, const double* xt,
                        const double* ut, double* x, double* u, const ProbState& st, const TraceDev& tr,
                        int* active_count, unsigned long long* counters) {
  hipLaunchKernelGGL(k_ilqr_decide, dim3(B), dim3(64), 0, s, B, N, NX, NU, T, init, alphas, o, Jt, dV, ok, xt, ut, x,
                     u, st, tr, active_count, counters);
}

}  // namespace tmpc
