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
#include "tmpc_copy.h"

namespace tmpc {

__device__ __forceinline__ bool use_QF(const CostDev* C, int k, int N) {
  return (k == N - 1) || (C->QF_start >= 0 && k >= C->QF_start);
}

// ======================================================================= backward (Riccati) sweep
template <int NJ, class R>
struct IlqrLds {
  static constexpr int NX = 2 * NJ, NU = NJ;
  R Vxx[NX * NX], Vx[NX];
  R A[2][NX * NX], Bm[2][NX * NU];      // knot k's A_k, B_k and the prefetched A_{k-1}, B_{k-1}
  R P[NX * NX], VB[NX * NU];            // V_xx A, V_xx B (P then holds the unsymmetrised V_xx)
  R Qxx[NX * NX], Qux[NU * NX], Quu[NU * NU], Qx[NX], Qu[NU];
  R KD[NU * (NX + 1)];                  // [Q_uu^-1 Q_ux | Q_uu^-1 Q_u], row-major
  R lx[NX], lu[NU], jac[3 * NJ];
  R Q[NX * NX], QF[NX * NX], Rc[NU * NU];   // the cost's Hessian blocks, staged once
  double xg[NX];
  double z[2][NX + NU];                 // knot k's [x_k; u_k] and the prefetched knot's (fp64: the soft terms)
  int fail;
  R trash[64];                          // the stores of lanes without an output land here
};

// One 64-lane workgroup = one wave: LDS written by one lane is visible to the others once the
// wave's LDS operations have completed, so the phases below are ordered by `s_waitcnt lgkmcnt(0)`
// alone.  __syncthreads() would also drain the wave's outstanding global memory operations
// (vmcnt(0)): the K_k / d_k stores of the previous knot and the next knot's prefetch loads.
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// lane l's value of v, on every lane (v_readlane: no LDS round trip)
__device__ __forceinline__ double lane_val(double v, int l) {
  const long long bits = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)bits, l), hi = __builtin_amdgcn_readlane((int)(bits >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ float lane_val(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// Diagnostic build only (-DTMPC_ILQR_STAMPS): per-phase s_memtime cycle totals of block 0's
// backward sweep, printed at its end (tools/debug/ilqr_stamps.py).
#ifdef TMPC_ILQR_STAMPS
#define IL_STAMP(i)                                             \
  do {                                                          \
    const unsigned long long n_ = __builtin_amdgcn_s_memtime(); \
    st_[i] += n_ - st_prev_;                                    \
    st_prev_ = n_;                                              \
  } while (0)
#else
#define IL_STAMP(i) \
  do {              \
  } while (0)
#endif

// MF (fp64 only): the Q-function products on the fp64 matrix cores (v_mfma_f64_16x16x4f64, one
// wave): P|VB = V_xx [A B] with [Q_x; Q_u] - l as an extra row, then [A B]^T [P VB] taking the
// first product's accumulators as its B operand in place (the f64 C/D layout puts row 4s + lane/16
// of reg s on the lane the next MFMA's k-step s reads), then M | V_x = Q_ux^T [K d].  Every output
// is the same products summed in the same order as the VALU loops.
typedef double dbl4 __attribute__((ext_vector_type(4)));

template <int NJ, class R, bool MF>
__global__ void __launch_bounds__(64) k_ilqr_backward(const CostDev* __restrict__ C, const ConstrDev* __restrict__ Cs,
                                                      PList P, int B, int N, const double* __restrict__ x,
                                                      const double* __restrict__ u, const double* __restrict__ rho_in,
                                                      const int* __restrict__ active, const double* __restrict__ Aall,
                                                      const double* __restrict__ Ball, const double* __restrict__ mu,
                                                      const double* __restrict__ lam,
                                                      const double* __restrict__ jsoft, double* __restrict__ Kout,
                                                      double* __restrict__ dout, double* __restrict__ dV,
                                                      int* __restrict__ ok) {
  constexpr int NX = 2 * NJ, NU = NJ, NC = NX + 1;
  constexpr int NA = (NX * NX + 63) / 64, NB = (NX * NU + 63) / 64;   // prefetch slots per lane
  if (!P.has(blockIdx.x, B)) return;
  const int b = P.at(blockIdx.x);
  if (!active[b]) return;
  __shared__ IlqrLds<NJ, R> L;
  const int t = threadIdx.x;
  const int K = N - 1;
  const R rho = R(rho_in[b]);
  const double* xb = x + (size_t)b * NX * N;
  const double* ub = u + (size_t)b * NU * K;
  const bool soft = jsoft != nullptr;   // soft limits: their jacobians precomputed (k_ilqr_soft_jac)
  const int qf_start = C->QF_start;
  const bool diag = C->diag != 0;

  // the cost blocks once (QuadraticCost, TrajoptCost.py:71-83)
  for (int e = t; e < NX * NX; e += 64) {
    L.Q[e] = R(C->Q[e]);
    L.QF[e] = R(C->QF[e]);
  }
  for (int e = t; e < NU * NU; e += 64) L.Rc[e] = R(C->R[e]);
  if (t < NX) L.xg[t] = C->xg[t];
  auto use_qf = [&](int k) { return (k == N - 1) || (qf_start >= 0 && k >= qf_start); };
  // [x_k; u_k] of a knot, one entry per lane (u_{N-1} := 0)
  auto load_z = [&](int k) -> double {
    if (t < NX) return xb[t * N + k];
    if (t < NX + NU) return k < K ? ub[(t - NX) * K + k] : 0.0;
    return 0.0;
  };
  // prefetched A_k / B_k entries of this lane, and (soft limits) entry t of the knot's soft-limit
  // jacobian, precomputed for every knot by k_ilqr_soft_jac ([B][N][3 NJ])
  double pa[NA], pb[NB], pj = 0.0, pjn = 0.0;
  auto load_jac = [&](int k) -> double {
    return (soft && t < 3 * NJ) ? jsoft[((size_t)b * N + k) * 3 * NJ + t] : 0.0;
  };
  auto load_ab = [&](int k) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int e = t + 64 * i;
      pa[i] = e < NX * NX ? Aall[((size_t)b * K + k) * NX * NX + e] : 0.0;
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int e = t + 64 * i;
      pb[i] = e < NX * NU ? Ball[((size_t)b * K + k) * NX * NU + e] : 0.0;
    }
  };
  auto store_ab = [&](int slot) {
#pragma unroll
    for (int i = 0; i < NA; ++i)
      if (t + 64 * i < NX * NX) L.A[slot][t + 64 * i] = R(pa[i]);
#pragma unroll
    for (int i = 0; i < NB; ++i)
      if (t + 64 * i < NX * NU) L.Bm[slot][t + 64 * i] = R(pb[i]);
  };

  // stage the cost derivatives of knot k (QuadraticCost.gradient / hessian, TrajoptCost.py:58-83,
  // plus the soft-limit jacobian, :220-225) into L.lx / L.lu / L.jac; z = L.z[zs], and zr = this
  // lane's entry of it (lanes < NX: x_k[t], NX .. NX + NU - 1: u_k[t - NX])
  auto stage_l = [&](int k, int zs, double zr) {
    const bool term = k == K;
    const double* zk = L.z[zs];
    const R jt = R(pj);                  // this lane's entry of the knot's soft-limit jacobian
    if (t < 3 * NJ) L.jac[t] = jt;       // 0 without soft limits
    // lanes < NX: l_x[t], lanes NX .. NX + NU - 1: l_u[t - NX].  Both dot products on every lane and
    // one store: the wave would execute both sides of a divergent branch anyway, plus its exec
    // bookkeeping (one wave per problem: every instruction is on the critical path)
    const int tx = t < NX ? t : NX - 1;
    const bool isu = t >= NX && t < NX + NU;
    const int tu = isu ? t - NX : 0;
    R g = 0.0, gu = 0.0;
    if (diag) {
      // the same chains without their exact-zero terms (CostDev.diag), from registers: the lane's
      // own z entry and diagonal entries; the NaN a non-finite entry of y / w puts into every dense
      // row sum (0 * inf) is raised by a ballot over the wave (diag_poison's rule)
      const int tq = t < NX ? t : 0;
      const R qdg = (use_qf(k) ? L.QF : L.Q)[tq * NX + tq], rdg = L.Rc[tu * NU + tu];
      const R yt = R(zr - L.xg[tq]), wt = R(zr);
      const bool badx = __ballot(t < NX && !isfinite(yt)) != 0;
      const bool badu = __ballot(isu && !isfinite(wt)) != 0;
      g = fma_r(yt, qdg, R(0)) + ((badx && NX > 1) ? R(NAN) : R(0));
      gu = fma_r(wt, rdg, R(0)) + ((badu && NU > 1) ? R(NAN) : R(0));
    } else {
      wave_lds_sync();
      const R* Qk = use_qf(k) ? L.QF : L.Q;
#pragma unroll
      for (int m = 0; m < NX; ++m) g += R(zk[m] - L.xg[m]) * Qk[m * NX + tx];
#pragma unroll
      for (int m = 0; m < NU; ++m) gu += R(zk[NX + m]) * L.Rc[m * NU + tu];
    }
    const R vx = g + jt;                 // L.jac[t] (lanes < NX) / L.jac[NX + tu] (u lanes): jt
    const R vu = gu + jt;
    R* dst = t < NX ? &L.lx[t] : ((isu && !term) ? &L.lu[tu] : &L.trash[t]);
    *dst = t < NX ? vx : vu;
  };
  // l_xx (+ per-type outer products on the q / qd diagonal blocks)
  auto lxx = [&](int k, int r, int c) -> R {
    const R* Qk = use_qf(k) ? L.QF : L.Q;
    const R o = (r / NJ == c / NJ) ? L.jac[r] * L.jac[c] : 0.0;
    return Qk[r * NX + c] + o;
  };

  // terminal value function: V_x = l_x(N-1), V_xx = l_xx(N-1); A_{K-1}, B_{K-1} and z_{K-1} in flight
  double zr = 0.0;   // this lane's entry of the next knot to stage
  R dv0 = 0.0, dv1 = 0.0;   // the expected-reduction sums dV1, dV2 (lane NX)
  {
    const double zt = load_z(K);
    pj = load_jac(K);
    load_ab(K - 1);
    pjn = load_jac(K - 1);
    const double zn = load_z(K - 1);
    if (t < NX + NU) L.z[0][t] = zt;
    wave_lds_sync();
    stage_l(K, 0, zt);
    wave_lds_sync();
    for (int e = t; e < NX * NX; e += 64) L.Vxx[e] = lxx(K, e / NX, e % NX);
    if (t < NX) L.Vx[t] = L.lx[t];
    if (t == 0) {
      L.fail = 0;
    }
    store_ab(0);
    if (t < NX + NU) L.z[1][t] = zn;
    zr = zn;
    pj = pjn;
    wave_lds_sync();
  }

#ifdef TMPC_ILQR_STAMPS
  unsigned long long st_[8] = {}, st_prev_ = __builtin_amdgcn_s_memtime();
#endif
  for (int k = K - 1; k >= 0; --k) {
    IL_STAMP(7);
    const int cur = (K - 1 - k) & 1;
    const R* A = L.A[cur];
    const R* Bm = L.Bm[cur];
    // next knot's A, B, z: loads issued now, written to the other slot at the end of this knot
    double zn = 0.0;
    if (k > 0) {
      load_ab(k - 1);
      pjn = load_jac(k - 1);
      zn = load_z(k - 1);
    }
    stage_l(k, 1 - cur, zr);
    wave_lds_sync();
    IL_STAMP(0);
    if constexpr (MF) {
      // fragments: lane l = (row / col l & 15, k-offset l >> 4) of each 16x16x4 k-step
      constexpr int KS = (NX + 3) / 4;
      const int lo = t & 15, hi = t >> 4;
      double vf[KS], abf[2][KS];
      // each fragment entry is one LDS read from a selected, always valid address, then a select
      // against 0 (the nested conditional reads compiled to exec-masked branches with an LDS wait in
      // each); the same values
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int kk = 4 * s + hi, kc = kk < NX ? kk : NX - 1;
        const R* vp = lo < NX ? &L.Vxx[lo * NX + kc] : &L.Vx[kc];
        const double vv = double(*vp);
        vf[s] = (kk < NX && lo <= NX) ? vv : 0.0;
#pragma unroll
        for (int tl = 0; tl < 2; ++tl) {
          const int c = 16 * tl + lo;
          const R* ap = c < NX ? &A[kc * NX + c] : &Bm[kc * NU + (c < NX + NU ? c - NX : 0)];
          const double av = double(*ap);
          abf[tl][s] = (kk < NX && c < NX + NU) ? av : 0.0;
        }
      }
      // P | VB (rows < NX) and [A B]^T V_x (row NX) = V_xx' [A B]
      dbl4 pv[2];
#pragma unroll
      for (int tl = 0; tl < 2; ++tl) {
        pv[tl] = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int s = 0; s < KS; ++s) pv[tl] = __builtin_amdgcn_mfma_f64_16x16x4f64(vf[s], abf[tl][s], pv[tl], 0, 0, 0);
      }
      // row NX of the product (the [A B]^T V_x row) sits in reg NX / 4 of the lanes with hi = NX % 4
      constexpr int IR = NX / 4, HR = NX % 4;
#pragma unroll
      for (int tl = 0; tl < 2; ++tl) {
        const int c = 16 * tl + lo;
        const bool isx = c < NX, isu = !isx && c < NX + NU;
        const R base = isx ? L.lx[isx ? c : 0] : L.lu[isu ? c - NX : 0];
        R* dst = (hi == HR && isx) ? &L.Qx[isx ? c : 0] : ((hi == HR && isu) ? &L.Qu[isu ? c - NX : 0] : &L.trash[t]);
        *dst = base + R(pv[tl][IR]);
      }
      // [A B]^T [P VB]: tile (tr, tc); B operand of k-step s = reg s of pv[tc] (rows >= NX zeroed)
#pragma unroll
      for (int tr = 0; tr < 2; ++tr)
#pragma unroll
        for (int tc = 0; tc < 2; ++tc) {
          dbl4 q{0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int s = 0; s < KS; ++s) {
            const double bop = 4 * s + hi < NX ? pv[tc][s] : 0.0;
            q = __builtin_amdgcn_mfma_f64_16x16x4f64(abf[tr][s], bop, q, 0, 0, 0);
          }
          // element i of the tile: row 16 tr + hi + 4 i, column 16 tc + lo.  Which of Q_xx / Q_ux /
          // Q_uu it can belong to is fixed per (tr, tc, i) up to the lane's hi / lo: the impossible
          // cases drop out at compile time, the rest is one select-and-store (same expressions)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int r0 = 16 * tr + 4 * i, c0 = 16 * tc;          // compile-time after unrolling
            const bool can_rx = r0 < NX, can_ru = r0 + 3 >= NX && r0 < NX + NU;
            const bool can_cx = c0 < NX, can_cu = c0 + 15 >= NX && c0 < NX + NU;
            const bool can_xx = can_rx && can_cx, can_ux = can_ru && can_cx, can_uu = can_ru && can_cu;
            if (!(can_xx || can_ux || can_uu)) continue;
            const int r = r0 + hi, c = c0 + lo;
            const R v = R(q[i]);
            const bool rx = r < NX, ru = r >= NX && r < NX + NU, cx = c < NX, cu = c >= NX && c < NX + NU;
            const bool xx = can_xx && rx && cx, ux = can_ux && ru && cx, uu = can_uu && ru && cu;
            const int rr = ru ? r - NX : 0, cc = cu ? c - NX : 0;
            R val = v;
            if (can_xx) {
              const R vxx = lxx(k, rx ? r : 0, cx ? c : 0) + v;
              val = xx ? vxx : val;
            }
            if (can_uu) {
              const R vuu = (L.Rc[rr * NU + cc] + L.jac[NX + rr] * L.jac[NX + cc]) + v + (rr == cc ? rho : R(0));
              val = uu ? vuu : val;
            }
            R* dst = xx ? &L.Qxx[(rx ? r : 0) * NX + (cx ? c : 0)]
                        : (ux ? &L.Qux[rr * NX + (cx ? c : 0)] : (uu ? &L.Quu[rr * NU + cc] : &L.trash[t]));
            *dst = val;
          }
        }
      wave_lds_sync();
      IL_STAMP(1);
    } else {
    // P = V_xx A, R = V_xx B; Q_x = l_x + A^T V_x, Q_u = l_u + B^T V_x
    for (int e = t; e < NX * NX + NX * NU + NX + NU; e += 64) {
      if (e < NX * NX) {
        const int r = e / NX, c = e % NX;
        R s = 0.0;
#pragma unroll
        for (int m = 0; m < NX; ++m) s += L.Vxx[r * NX + m] * A[m * NX + c];
        L.P[e] = s;
      } else if (e < NX * NX + NX * NU) {
        const int f = e - NX * NX, r = f / NU, c = f % NU;
        R s = 0.0;
#pragma unroll
        for (int m = 0; m < NX; ++m) s += L.Vxx[r * NX + m] * Bm[m * NU + c];
        L.VB[f] = s;
      } else if (e < NX * NX + NX * NU + NX) {
        const int r = e - NX * NX - NX * NU;
        R s = 0.0;
#pragma unroll
        for (int m = 0; m < NX; ++m) s += A[m * NX + r] * L.Vx[m];
        L.Qx[r] = L.lx[r] + s;
      } else {
        const int r = e - NX * NX - NX * NU - NX;
        R s = 0.0;
#pragma unroll
        for (int m = 0; m < NX; ++m) s += Bm[m * NU + r] * L.Vx[m];
        L.Qu[r] = L.lu[r] + s;
      }
    }
    wave_lds_sync();
    IL_STAMP(1);
    // Q_xx = l_xx + A^T P, Q_uu = l_uu + B^T R + rho I, Q_ux = B^T P
    for (int e = t; e < NX * NX + NU * NU + NU * NX; e += 64) {
      if (e < NX * NX) {
        const int r = e / NX, c = e % NX;
        R s = 0.0;
#pragma unroll
        for (int m = 0; m < NX; ++m) s += A[m * NX + r] * L.P[m * NX + c];
        L.Qxx[e] = lxx(k, r, c) + s;
      } else if (e < NX * NX + NU * NU) {
        const int f = e - NX * NX, r = f / NU, c = f % NU;
        R s = 0.0;
#pragma unroll
        for (int m = 0; m < NX; ++m) s += Bm[m * NU + r] * L.VB[m * NU + c];
        L.Quu[f] = (L.Rc[f] + L.jac[NX + r] * L.jac[NX + c]) + s + (r == c ? rho : R(0));
      } else {
        const int f = e - NX * NX - NU * NU, r = f / NX, c = f % NX;
        R s = 0.0;
#pragma unroll
        for (int m = 0; m < NX; ++m) s += Bm[m * NU + r] * L.P[m * NX + c];
        L.Qux[f] = s;
      }
    }
    wave_lds_sync();
    }   // MF
    IL_STAMP(2);
    // [K | d] = -Q_uu^-1 [Q_ux | Q_u]: Cholesky Q_uu = L L^T (every lane, from LDS), then lane c
    // solves its right-hand-side column c; Q_uu not positive definite -> backward failure.
    // LAPACK's dpotf2 form (numpy.linalg.cholesky): column j scaled by the reciprocal 1 / L_jj,
    // and the substitutions multiply by it too -- 6 IEEE divisions on the knot's serial chain
    // instead of 27 (each a ~10-instruction dependent sequence)
    bool pd = true;
    R ds1 = 0.0, ds2 = 0.0;   // this knot's dV terms (meaningful on lane NX)
    {
      // every lane factors (the wave would anyway); lanes >= NC solve a copy of column NC - 1
      const int tc = t < NC ? t : NC - 1;
      R Lc[NU][NU], ri[NU];
#pragma unroll
      for (int j = 0; j < NU; ++j) {
        R s = L.Quu[j * NU + j];
#pragma unroll
        for (int m = 0; m < j; ++m) s -= Lc[j][m] * Lc[j][m];
        pd = pd && (s > R(0));
        const R dj = sqrt(s);
        Lc[j][j] = dj;
        ri[j] = R(1) / dj;
#pragma unroll
        for (int i = j + 1; i < NU; ++i) {
          R v = L.Quu[i * NU + j];
#pragma unroll
          for (int m = 0; m < j; ++m) v -= Lc[i][m] * Lc[j][m];
          Lc[i][j] = v * ri[j];
        }
      }
      R y[NU], qv[NU];
#pragma unroll
      for (int i = 0; i < NU; ++i) {
        const R vx = L.Qux[i * NX + (tc < NX ? tc : 0)], vu = L.Qu[i];
        qv[i] = vu;
        R v = tc < NX ? vx : vu;
#pragma unroll
        for (int m = 0; m < i; ++m) v -= Lc[i][m] * y[m];
        y[i] = v * ri[i];
      }
#pragma unroll
      for (int i = NU - 1; i >= 0; --i) {
        R v = y[i];
#pragma unroll
        for (int m = i + 1; m < NU; ++m) v -= Lc[m][i] * y[m];
        y[i] = v * ri[i];
      }
#pragma unroll
      for (int i = 0; i < NU; ++i) *(t < NC ? &L.KD[i * NC + tc] : &L.trash[t]) = -y[i];
      // dV terms on the lane of column NX, whose -y is d (dV1 += d^T Q_u, dV2 += d^T Q_uu d / 2): the
      // chains the wave formed from LDS copies after the next phase (d from KD, (Q_uu d)_i on lane i,
      // read back lane by lane), now from this lane's registers, operand for operand
      R s1 = 0.0, s2 = 0.0;
#pragma unroll
      for (int i = 0; i < NU; ++i) {
        R qd = 0.0;
#pragma unroll
        for (int m = 0; m < NU; ++m) qd += L.Quu[i * NU + m] * (-y[m]);
        const R di = -y[i];
        s1 += di * qv[i];
        s2 += di * qd;
      }
      ds1 = s1;
      ds2 = s2;
    }
    // every lane factored the same Q_uu: pd is wave-uniform, no LDS round trip for the exit test
    pd = __builtin_amdgcn_readfirstlane((int)pd) != 0;
    if (!pd) {
      if (t == 0) L.fail = 1;
      wave_lds_sync();
      break;
    }
    dv0 += ds1;
    dv1 += R(0.5) * ds2;
    wave_lds_sync();
    IL_STAMP(3);
    // V_x = Q_x + Q_ux^T d, M = Q_xx + Q_ux^T K
    if constexpr (MF) {
      // [M | V_x] - [Q_xx | Q_x] = Q_ux^T [K | d]: one 16-column tile, k over the NU controls
      constexpr int KU = (NU + 3) / 4;
      const int lo = t & 15, hi = t >> 4;
      dbl4 mv{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int s = 0; s < KU; ++s) {
        const int kk = 4 * s + hi;
        const double aop = (kk < NU && lo < NX) ? double(L.Qux[kk * NX + lo]) : 0.0;
        const double bop = (kk < NU && lo < NC) ? double(L.KD[kk * NC + lo]) : 0.0;
        mv = __builtin_amdgcn_mfma_f64_16x16x4f64(aop, bop, mv, 0, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (4 * i >= NX) continue;   // rows past NX: none
        const int r = hi + 4 * i, c = lo;
        const bool rx = r < NX, cx = c < NX, cv = c == NX;
        const int rs = rx ? r : 0;
        const R base = cx ? L.Qxx[rs * NX + (cx ? c : 0)] : L.Qx[rs];
        R* dst = (rx && cx) ? &L.P[rs * NX + (cx ? c : 0)] : ((rx && cv) ? &L.Vx[rs] : &L.trash[t]);
        *dst = base + R(mv[i]);
      }
    } else
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
    IL_STAMP(4);
    // K_k, d_k to HBM ([B][K][NU][NX], [B][K][NU]); not waited for (wave_lds_sync)
#pragma unroll
    for (int j = 0; j < (NU * NC + 63) / 64; ++j) {
      const int e = t + 64 * j, i = e / NC, c = e % NC;
      double* dst = c < NX ? Kout + (((size_t)b * K + k) * NU + i) * NX + c : dout + ((size_t)b * K + k) * NU + i;
      if (e < NU * NC) *dst = double(L.KD[e]);
    }
    wave_lds_sync();
#pragma unroll
    for (int j = 0; j < (NX * NX + 63) / 64; ++j) {
      const int e = t + 64 * j, r = e / NX, c = e % NX;
      if (e < NX * NX) L.Vxx[e] = R(0.5) * (L.P[r * NX + c] + L.P[c * NX + r]);
    }
    IL_STAMP(5);
    if (k > 0) {
      store_ab(1 - cur);
      if (t < NX + NU) L.z[cur][t] = zn;
      zr = zn;
      pj = pjn;
    }
    wave_lds_sync();
    IL_STAMP(6);
  }
#ifdef TMPC_ILQR_STAMPS
  if (b == 0 && t == 0)
    printf("ilqr_stamps K=%d prefetch+stage_l %llu P/VB/Qx/Qu %llu Qxx/Quu/Qux %llu chol %llu Vx/M/dv %llu "
           "Kstore/Vxx %llu store_ab %llu loop %llu\n", K, st_[0], st_[1], st_[2], st_[3], st_[4], st_[5], st_[6],
           st_[7]);
#endif
  if (t == 0) ok[b] = L.fail ? 0 : 1;
  if (t == NX) {
    dV[2 * b] = double(dv0);
    dV[2 * b + 1] = double(dv1);
  }
}

// QuadraticCost.value of one knot (TrajoptCost.py:49-56): 0.5 dx^T (Q dx) [+ 0.5 u^T (R u)], one
// expression shared by the rollouts and the INIT evaluation so both round alike
template <int NJ>
__device__ __forceinline__ double knot_quad_cost(const CostDev* __restrict__ C, int k, int N, const double* xh,
                                                 const double* uh, bool term) {
  constexpr int NX = 2 * NJ, NU = NJ;
  const double* Qk = use_QF(C, k, N) ? C->QF : C->Q;
  if (C->diag) {   // the same chains without their exact-zero terms (CostDev.diag)
    double y[NX];
#pragma unroll
    for (int r = 0; r < NX; ++r) y[r] = xh[r] - C->xg[r];
    double vq = 0.0;
#pragma unroll
    for (int r = 0; r < NX; ++r) vq = __fma_rn(y[r], __fma_rn(Qk[r * NX + r], y[r], 0.0), vq);
    double cost = 0.5 * (vq + diag_poison(y, NX));
    if (!term) {
      double vr = 0.0;
#pragma unroll
      for (int r = 0; r < NU; ++r) vr = __fma_rn(uh[r], __fma_rn(C->R[r * NU + r], uh[r], 0.0), vr);
      cost = __fma_rn(0.5, vr + diag_poison(uh, NU), cost);
    }
    return cost;
  }
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
  return cost;
}

// J at the current trajectory (the iLQR drivers' INIT evaluation, oracle/ilqr.py:130) of the
// problems in `mask`: one 64-lane workgroup per problem, lanes over knots for the per-knot cost
// and soft value (sc[k], sc[N + k]), then lane 0 sums them in knot order, the cost terms first --
// totalCost's order (:296-310) and the serial sums of k_ilqr_forward operand for operand.  Run
// under the act_init mask every outer-loop iteration, so it must be cheap when few problems
// restart (the serial INIT rollout lane took 0.19 ms per launch on average).
template <int NJ, bool SOFT>
__global__ void __launch_bounds__(64) k_ilqr_init_cost(const CostDev* __restrict__ C, const ConstrDev* __restrict__ Cs,
                                                       const double* __restrict__ mu, const double* __restrict__ lam,
                                                       PList P, int B, int N, const double* __restrict__ x,
                                                       const double* __restrict__ u, const int* __restrict__ mask,
                                                       double* __restrict__ Jt) {
  constexpr int NX = 2 * NJ, NU = NJ;
  if (!P.has(blockIdx.x, B)) return;
  const int b = P.at(blockIdx.x);
  if (!mask[b]) return;
  extern __shared__ double sc[];   // [2][N]
  const int K = N - 1;
  const double* xb = x + (size_t)b * NX * N;
  const double* ub = u + (size_t)b * NU * K;
  for (int k = threadIdx.x; k < N; k += 64) {
    const bool term = k == K;
    double xh[NX], uh[NU];
#pragma unroll
    for (int m = 0; m < NX; ++m) xh[m] = xb[m * N + k];
#pragma unroll
    for (int i = 0; i < NU; ++i) uh[i] = term ? 0.0 : ub[i * K + k];
    sc[k] = knot_quad_cost<NJ>(C, k, N, xh, uh, term);
    if (SOFT) {
      double z[3 * NJ], jac[3 * NJ];
#pragma unroll
      for (int m = 0; m < NX; ++m) z[m] = xh[m];
#pragma unroll
      for (int m = 0; m < NU; ++m) z[NX + m] = uh[m];
      const size_t ko = ((size_t)b * N + k) * 6 * NJ;
      sc[N + k] = soft_knot<NJ>(Cs, mu + ko, lam + ko, term, z, jac);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double J = 0.0;
    for (int k = 0; k < N; ++k) J = J + sc[k];
    if (SOFT)
      for (int k = 0; k < N; ++k) J = J + sc[N + k];
    Jt[b] = J;
  }
}

// ======================================================================= forward sweep (closed-loop rollouts)
// lane = (b, trial t).  INIT: J at the current trajectory (no rollout).  Trial
// trajectories are kept knot-major ([B][T][N][nx], [B][T][N-1][nu]: a lane's knot is one
// contiguous 96 + 48-byte run, where the reference's [nx][N] order made every knot 18 partial
// cache-line writes per lane) so the decision kernel copies (and transposes) the accepted one.  Cost sums in totalCost's order (:296-310): the
// QuadraticCost terms, then the soft values.
// Prefetch (PF) of the feedback law's operands: the knot loop is one serial chain per lane
// (~25k cycles per knot at one wave per SIMD, profiles/r02: ~40 % of it the loads of K_k, d_k,
// x_k, u_k), so the next knot's operands of every problem of the workgroup go global -> LDS by
// LDS-DMA (global_load_lds: no VGPRs, the kernel is at the register cap) while this knot's
// dynamics run.  Per problem and knot: K_k in 16-byte pieces, then d_k, x_k, u_k in dwords
// (x / u are strided by knot in the reference layout).  Buffer [2][nprob][SK + SS] doubles.
template <int NJ>
struct FwdPf {
  static constexpr int NX = 2 * NJ, NU = NJ;
  static constexpr int SK = NU * NX;            // K_k
  static constexpr int SS = NU + NX + NU;       // d_k, x_k, u_k
  static constexpr int CK = SK / 2;             // 16-byte pieces of K_k (SK is even)
  static __host__ __device__ int nprob(int T) { return 63 / T + 2; }   // problems a 64-lane group can touch
  // regions rounded up to whole wave-instructions (64 x 16 B, 64 x 4 B): the last instruction's
  // spare lanes land inside the region, not in the next one
  static __host__ __device__ size_t rk(int T) { return (size_t)((nprob(T) * CK + 63) / 64) * 128; }
  static __host__ __device__ size_t rs(int T) { return (size_t)((nprob(T) * 2 * SS + 63) / 64) * 32; }
  static __host__ __device__ size_t lds_doubles(int T) { return 2 * (rk(T) + rs(T)); }
};

// The knot loop's memory waits (config 3, profiles/r05/configs/c3_fwd_*_r05a[e-g]*; each switch 0 restores
// the round-4 form for comparison): the next knot's prefetch issued after this knot's stores and feedback
// reads (PF_LATE: in front of them, the compiler's wait pass put a vmcnt(0) before the feedback's LDS
// reads -- the LDS-DMA may alias them -- exposing the DMA's latency), explicit waits after the loads into
// xh / uh (WAITS), the DMA sources precomputed (PFR), the knot's wait through the builtin (BWAIT):
// ilqr_forward 0.472 -> 0.401 ms per launch, config 3 4.37k -> 4.65k solves/s
#ifndef TMPC_FWD_PF_LATE
#define TMPC_FWD_PF_LATE 1
#endif
#ifndef TMPC_FWD_WAITS
#define TMPC_FWD_WAITS 1
#endif
#ifndef TMPC_FWD_PFR
#define TMPC_FWD_PFR 1
#endif
#ifndef TMPC_FWD_BWAIT
#define TMPC_FWD_BWAIT 1
#endif
template <int NJ, bool CHAIN, bool SOFT, class MT, class R, bool PF>
__global__ void __launch_bounds__(64) k_ilqr_forward(MT Mg, const CostDev* __restrict__ C,
                                                     const ConstrDev* __restrict__ Cs, const double* __restrict__ mu,
                                                     const double* __restrict__ lam, PList P, int B, int N, int T,
                                                     double dt, int init, const double* __restrict__ alphas,
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
  using PF_ = FwdPf<NJ>;
  extern __shared__ __align__(16) double pfb[];
  const int lane = threadIdx.x;
  const int gid = blockIdx.x * blockDim.x + lane;
  // lanes over (listed problem p, trial); the problem list's last entry stands in for dead lanes
  const int np = P.cnt ? min(B, *P.cnt) : B;
  if (np <= 0) return;
  const int pt = min(gid, np * T - 1);
  const int pp = pt / T, tr = pt - pp * T;
  const int b = P.at(pp);
  const bool live = gid < np * T && active[b] && (init || ok[b]);
  const bool pf = PF && !init;
  if (pf) {
    if (__ballot(live) == 0) return;   // the whole wave: no work, no prefetch to share
  } else if (!live) {
    return;
  }
  const int K = N - 1;
  const double al = init ? 0.0 : alphas[tr];
  const double* xb = x + (size_t)b * NX * N;
  const double* ub = u + (size_t)b * NU * K;
  const size_t bt = (size_t)b * T + tr;   // this lane's trial slot
  double* xo = xt + bt * NX * N;
  double* uo = ut + bt * NU * K;
  // prefetch bookkeeping: listed problems [p0, p0 + nprob) of this group, this lane's problem slot pl.
  // Their batch indices are read from the problem list once, into LDS: an index load per piece
  // inside the knot loop would make every LDS-DMA issue wait for the one before it (vmcnt counts
  // both in issue order).
  const int p0 = (int)(blockIdx.x * blockDim.x) / T;
  const int npf = PF_::nprob(T);
  const int pl = pp - p0;
  __shared__ int s_pb[64];
  const int npt = min(npf, 64);   // the slots a lane can own (pl < 64); higher ones only pad
  if (pf) {
    if (lane < npt) s_pb[lane] = P.at(min(p0 + lane, np - 1));
    __syncthreads();
  }
  // TMPC_FWD_PFR: each lane's LDS-DMA sources for knot 0 computed once, here, while no LDS-DMA is in
  // flight (up to PFJ wave-instructions per kind: T >= 5 trials); knot kn's are base + kn x stride.
  // Reading the problem slot from LDS per instruction inside the prefetch made the compiler wait for
  // the previous LDS-DMA before every read (the DMA writes LDS): ~3.7k cycles per knot to issue 13
  // instructions (profiles/r05/configs/c3_fwd_stamps_r05ae.txt)
  constexpr int PFJ = 12;
  const int nkj = (npf * PF_::CK + 63) / 64, nsj = (npf * 2 * PF_::SS + 63) / 64;
  const bool pfr = TMPC_FWD_PFR && pf && nkj <= PFJ && nsj <= PFJ;
  const double* kbase[PFJ];
  const char* sbase[PFJ];
  int sstride[PFJ];   // bytes per knot
  if (pfr) {
#pragma unroll
    for (int j = 0; j < PFJ; ++j) {
      const int c = j * 64 + lane;
      const int p = c / PF_::CK, w = c - p * PF_::CK;
      const int bb = s_pb[min(p, npt - 1)];
      kbase[j] = Kg + (size_t)bb * K * PF_::SK + 2 * w;
      const int q = j * 64 + lane;
      const int ps = q / (2 * PF_::SS), r = q - ps * (2 * PF_::SS), item = r >> 1, half = r & 1;
      const int bs = s_pb[min(ps, npt - 1)];
      const double* src = item < NU ? dg + (size_t)bs * K * NU + item
                        : item < NU + NX ? x + ((size_t)bs * NX + (item - NU)) * N
                                         : u + ((size_t)bs * NU + (item - NU - NX)) * K;
      sbase[j] = (const char*)src + 4 * half;
      sstride[j] = item < NU ? NU * 8 : 8;
    }
  }
  auto prefetch = [&](int kn, int slot) {
    double* buf = pfb + (size_t)slot * (PF_::rk(T) + PF_::rs(T));
    if (pfr) {
#pragma unroll
      for (int j = 0; j < PFJ; ++j)
        if (j < nkj) {
          const double* src = kbase[j] + (size_t)kn * PF_::SK;
          __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(buf + (size_t)j * 128), 16, 0, 0);
        }
      double* sb = buf + PF_::rk(T);
#pragma unroll
      for (int j = 0; j < PFJ; ++j)
        if (j < nsj) {
          const char* src = sbase[j] + (size_t)kn * sstride[j];
          __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(sb + (size_t)j * 32), 4, 0, 0);
        }
      return;
    }
    // K_kn: 16-byte pieces, lane-linear destinations
    for (int j = 0; j * 64 < npf * PF_::CK; ++j) {
      const int c = j * 64 + lane;
      const int p = c / PF_::CK, w = c - p * PF_::CK;
      const int bb = s_pb[min(p, npt - 1)];
      const double* src = Kg + ((size_t)bb * K + kn) * PF_::SK + 2 * w;
      __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(buf + (size_t)j * 128), 16, 0, 0);
    }
    // d_kn, x_kn, u_kn: dwords
    double* sb = buf + PF_::rk(T);
    for (int j = 0; j * 64 < npf * 2 * PF_::SS; ++j) {
      const int q = j * 64 + lane;
      const int p = q / (2 * PF_::SS), r = q - p * (2 * PF_::SS), item = r >> 1, half = r & 1;
      const int bb = s_pb[min(p, npt - 1)];
      const double* src = item < NU ? dg + ((size_t)bb * K + kn) * NU + item
                        : item < NU + NX ? x + ((size_t)bb * NX + (item - NU)) * N + kn
                                         : u + ((size_t)bb * NU + (item - NU - NX)) * K + kn;
      __builtin_amdgcn_global_load_lds((const char*)src + 4 * half,
                                       (__attribute__((address_space(3))) void*)(sb + (size_t)j * 32), 4, 0, 0);
    }
  };
  if (pf) prefetch(0, 0);
  double xh[NX];
#pragma unroll
  for (int m = 0; m < NX; ++m) xh[m] = xb[m * N];
  // vmcnt(0) through the builtin (the compiler's wait pass sees it, an asm one it does not): loads
  // that could still be in flight into xh / uh when the loop's paths join made the pass put a full
  // vmcnt(0) inside the knot loop, which also waited for the next knot's prefetch (its latency on
  // every knot's critical path instead of under the dynamics)
  if (TMPC_FWD_WAITS) __builtin_amdgcn_s_waitcnt(0x0F70);
  double J = 0.0;
#ifdef TMPC_ILQR_STAMPS
  unsigned long long st_[8] = {}, st_prev_ = __builtin_amdgcn_s_memtime();
#endif
  for (int k = 0; k <= K; ++k) {
    IL_STAMP(7);
    const bool term = k == K;
    double uh[NU];
    if (pf && !term) {
      // knot k's operands have landed in LDS.  TMPC_FWD_BWAIT: through the builtin, which is no
      // compiler memory barrier (the asm's "memory" clobber made every knot reload the cost's
      // constants); the compiler's own wait pass orders LDS reads after the LDS-DMA writing them
      if (TMPC_FWD_BWAIT) __builtin_amdgcn_s_waitcnt(0x0F70);
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      IL_STAMP(4);
      if (!TMPC_FWD_PF_LATE && k + 1 < K) prefetch(k + 1, (k + 1) & 1);
      IL_STAMP(5);
    }
    if (live) {
    if (!init) {
#pragma unroll
      for (int m = 0; m < NX; ++m) xo[k * NX + m] = xh[m];
      IL_STAMP(6);
    } else {
#pragma unroll
      for (int m = 0; m < NX; ++m) xh[m] = xb[m * N + k];
      if (TMPC_FWD_WAITS) __builtin_amdgcn_s_waitcnt(0x0F70);
    }
    if (!term) {
      if (init) {
#pragma unroll
        for (int i = 0; i < NU; ++i) uh[i] = ub[i * K + k];
        if (TMPC_FWD_WAITS) __builtin_amdgcn_s_waitcnt(0x0F70);
      } else if (pf) {
        const double* buf = pfb + (size_t)(k & 1) * (PF_::rk(T) + PF_::rs(T));
        const double* Kk = buf + (size_t)pl * PF_::SK;
        const double* sk = buf + PF_::rk(T) + (size_t)pl * PF_::SS;   // d_k | x_k | u_k
        // the LDS reads issued ahead of their products: d_k, x_k, u_k and row 0 of K_k together, then
        // row i + 1 of K_k before row i's products (the scheduler fences keep them there; left alone it
        // put each read next to its product with a full LDS wait between, ~4k cycles per knot,
        // profiles/r05/configs/c3_fwd_stamps_r05ag.txt).  Same operands, same chains.
        double sv[PF_::SS], kr[2][NX];
#pragma unroll
        for (int m = 0; m < PF_::SS; ++m) sv[m] = sk[m];
#pragma unroll
        for (int m = 0; m < NX; ++m) kr[0][m] = Kk[m];
        __builtin_amdgcn_sched_barrier(0);
        double dx[NX];
#pragma unroll
        for (int m = 0; m < NX; ++m) dx[m] = xh[m] - sv[NU + m];
#pragma unroll
        for (int i = 0; i < NU; ++i) {
          if (i + 1 < NU) {
#pragma unroll
            for (int m = 0; m < NX; ++m) kr[(i + 1) & 1][m] = Kk[(i + 1) * NX + m];
          }
          __builtin_amdgcn_sched_barrier(0);
          double fb = 0.0;
#pragma unroll
          for (int m = 0; m < NX; ++m) fb += kr[i & 1][m] * dx[m];
          uh[i] = (sv[NU + NX + i] + al * sv[i]) + fb;
          uo[k * NU + i] = uh[i];
        }
      } else {
        const double* Kk = Kg + ((size_t)b * K + k) * NU * NX;
        const double* dk = dg + ((size_t)b * K + k) * NU;
#pragma unroll
        for (int i = 0; i < NU; ++i) {
          double fb = 0.0;
#pragma unroll
          for (int m = 0; m < NX; ++m) fb += Kk[i * NX + m] * (xh[m] - xb[m * N + k]);
          uh[i] = (ub[i * K + k] + al * dk[i]) + fb;
          uo[k * NU + i] = uh[i];
        }
      }
    }
    }   // live
    // TMPC_FWD_PF_LATE: the next knot's prefetch after this knot's stores
    if (TMPC_FWD_PF_LATE && pf && k + 1 < K) prefetch(k + 1, (k + 1) & 1);
    if (live) {
    IL_STAMP(0);
    J = J + knot_quad_cost<NJ>(C, k, N, xh, uh, term);
    IL_STAMP(1);
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
      IL_STAMP(2);
#pragma unroll
      for (int j = 0; j < NJ; ++j) qdd[j] = double(qddr[j]);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const double nq = __dadd_rn(xh[j], __dmul_rn(dt, qd[j]));
        const double nv = __dadd_rn(xh[NJ + j], __dmul_rn(dt, qdd[j]));
        xh[j] = nq;
        xh[NJ + j] = nv;
      }
      IL_STAMP(3);
    }
    }   // live
  }
  if (!live) return;
  if (SOFT) {
    // value_soft_constraints per knot, summed after the cost terms
    const double* xs_ = init ? xb : xo;
    const double* us_ = init ? ub : uo;
    for (int k = 0; k <= K; ++k) {
      double z[3 * NJ], jac[3 * NJ];
#pragma unroll
      for (int m = 0; m < NX; ++m) z[m] = init ? xs_[m * N + k] : xs_[k * NX + m];
#pragma unroll
      for (int m = 0; m < NU; ++m) z[NX + m] = k < K ? (init ? us_[m * K + k] : us_[k * NU + m]) : 0.0;
      const size_t ko = ((size_t)b * N + k) * 6 * NJ;
      J = J + soft_knot<NJ>(Cs, mu + ko, lam + ko, k == K, z, jac);
    }
  }
#ifdef TMPC_ILQR_STAMPS
  if (gid == 0 && !init)
    printf("ilqr_fwd_stamps K=%d wait %llu prefetch %llu xstore %llu feedback %llu cost %llu aba %llu euler %llu\n", K,
           st_[4] + st_[7], st_[5], st_[6], st_[0], st_[1], st_[2], st_[3]);
#endif
  Jt[bt] = J;
}

// trials per pass of k_ilqr_soft_add: as many [N + 1] LDS rows as fit in 48 KB
// (TMPC_SOFT_ADD_GROUP=g caps it: tests run the multi-pass form at small sizes)
static inline int soft_add_group(int T, int N) {
  int g = (48 * 1024) / ((N + 1) * (int)sizeof(double));
  const char* e = getenv("TMPC_SOFT_ADD_GROUP");
  if (e && atoi(e) > 0 && atoi(e) < g) g = atoi(e);
  return g < 1 ? 1 : (g < T ? g : T);
}

// The soft-limit values of the trial trajectories (value_soft_constraints, summed after the cost
// terms as totalCost does, :296-310): one 64-lane workgroup per problem, lanes over knots.  A lane
// reads its knot's mu / lambda once and evaluates soft_knot for every trial's trajectory (the trials
// share the constants: one workgroup per (problem, trial) read them T times); then lane tr adds
// trial tr's values to its rollout's cost sum in knot order -- the serial tail of k_ilqr_forward
// operand for operand, the T trials' chains side by side.
template <int NJ>
__global__ void __launch_bounds__(64) k_ilqr_soft_add(const ConstrDev* __restrict__ Cs, const double* __restrict__ mu,
                                                      const double* __restrict__ lam, PList P, int B, int N, int T,
                                                      int TG, const double* __restrict__ xt,
                                                      const double* __restrict__ ut, const int* __restrict__ active,
                                                      const int* __restrict__ ok, double* __restrict__ Jt) {
  constexpr int NX = 2 * NJ, NU = NJ, MC = 6 * NJ;
  if (!P.has(blockIdx.x, B)) return;
  const int b = P.at(blockIdx.x);
  if (!active[b] || !ok[b]) return;
  extern __shared__ double sv[];   // [TG][N + 1] (the pad puts the trials' rows on different banks)
  const int K = N - 1, ld = N + 1;
  // TG: trials per pass (the LDS rows of one pass, soft_add_group)
  for (int t0 = 0; t0 < T; t0 += TG) {
    const int tn = min(TG, T - t0);
    for (int k = threadIdx.x; k < N; k += 64) {
      const size_t ko = ((size_t)b * N + k) * MC;
      double mk[MC], lk[MC];
#pragma unroll
      for (int e = 0; e < MC; ++e) {
        mk[e] = mu[ko + e];
        lk[e] = lam[ko + e];
      }
      for (int q = 0; q < tn; ++q) {
        const size_t gid = (size_t)b * T + t0 + q;
        const double* xo = xt + gid * NX * N;
        const double* uo = ut + gid * NU * K;
        double z[3 * NJ], jac[3 * NJ];
#pragma unroll
        for (int m = 0; m < NX; ++m) z[m] = xo[k * NX + m];
#pragma unroll
        for (int m = 0; m < NU; ++m) z[NX + m] = k < K ? uo[k * NU + m] : 0.0;
        sv[q * ld + k] = soft_knot<NJ>(Cs, mk, lk, k == K, z, jac);
      }
    }
    __syncthreads();
    const int q = threadIdx.x;
    if (q < tn) {
      const size_t gid = (size_t)b * T + t0 + q;
      double J = Jt[gid];
      for (int k = 0; k < N; ++k) J = J + sv[q * ld + k];
      Jt[gid] = J;
    }
    __syncthreads();
  }
}

// The soft-limit jacobians of every knot of the current trajectory (BoxConstraint.jacobian,
// TrajoptConstraint.py:53-128, through soft_knot) for the Riccati sweep: lane = (problem, knot),
// [B][N][3 NJ].  The sweep used to evaluate them in lane 0 at each knot, one dependent round trip
// to mu / lambda in HBM per knot on its critical path; it now prefetches row k - 1 with A_{k-1}.
template <int NJ>
__global__ void __launch_bounds__(256) k_ilqr_soft_jac(const ConstrDev* __restrict__ Cs, const double* __restrict__ mu,
                                                       const double* __restrict__ lam, PList P, int B, int N,
                                                       const double* __restrict__ x, const double* __restrict__ u,
                                                       const int* __restrict__ active, double* __restrict__ jout) {
  constexpr int NX = 2 * NJ, NU = NJ;
  const int pk = blockIdx.x * blockDim.x + threadIdx.x;
  if (pk >= B * N) return;
  const int p = pk / N, k = pk - p * N;
  if (!P.has(p, B)) return;
  const int b = P.at(p);
  if (!active[b]) return;
  const size_t gid = (size_t)b * N + k;
  const int K = N - 1;
  const double* xb = x + (size_t)b * NX * N;
  const double* ub = u + (size_t)b * NU * K;
  double z[3 * NJ], jac[3 * NJ];
#pragma unroll
  for (int m = 0; m < NX; ++m) z[m] = xb[m * N + k];
#pragma unroll
  for (int m = 0; m < NU; ++m) z[NX + m] = k < K ? ub[m * K + k] : 0.0;
  const size_t ko = ((size_t)b * N + k) * 6 * NJ;
  soft_knot<NJ>(Cs, mu + ko, lam + ko, k == K, z, jac);
#pragma unroll
  for (int m = 0; m < 3 * NJ; ++m) jout[(size_t)gid * 3 * NJ + m] = jac[m];
}

// ======================================================================= decision + state machine
// One 64-lane workgroup per problem.  Acceptance ratio (J - J^) / (-alpha (dV1 + alpha dV2)) in
// [exp_red_min, exp_red_max] in the reference's alpha order (oracle/ilqr.py), rho schedule and exit
// codes of reduce_regularization / check_for_exit_or_error (:457-481), trace row, trajectory copy.
__global__ void __launch_bounds__(64) k_ilqr_decide(PList P, int B, int N, int NX, int NU, int T, int init,
                                                    const double* __restrict__ alphas, SolverOpts o,
                                                    const double* __restrict__ Jt, const double* __restrict__ dV,
                                                    const int* __restrict__ okb, const double* __restrict__ xt,
                                                    const double* __restrict__ ut, double* __restrict__ x,
                                                    double* __restrict__ u, ProbState st, TraceDev tr,
                                                    int* __restrict__ active_count,
                                                    unsigned long long* __restrict__ counters,
                                                    int* __restrict__ activate) {
  if (!P.has(blockIdx.x, B)) return;
  const int b = P.at(blockIdx.x);
  if (!st.active[b]) return;
  __shared__ int s_choice;
  __shared__ double s_al[64], s_J[64];
  const int t = threadIdx.x;
  const int W = o.max_iter_sqp + 1;
  const int K = N - 1;
  if (t < T) {   // the trials' alphas and costs loaded by their lanes at once (lane 0 walks them below)
    s_al[t] = alphas[t];
    s_J[t] = Jt[(size_t)b * T + t];
  }
  __syncthreads();
  if (t == 0) {
    if (init) {
      const double J = s_J[0];
      st.J[b] = J;
      st.c[b] = 0.0;
      st.merit[b] = J;
      const size_t e = (size_t)b * W;
      tr.iteration[e] = 0; tr.ls_iter[e] = 0; tr.alpha[e] = 1.0; tr.rho[e] = st.rho[b];
      tr.J[e] = J; tr.c[e] = 0.0; tr.merit[e] = J; tr.D[e] = __builtin_nan(""); tr.ratio[e] = __builtin_nan("");
      tr.accepted[e] = 0; tr.pcg_iters[e] = 0;
      *active_count = 1;   // the host only tests for zero
      if (activate) {      // a restarted pass / a stream's new problem enters its inner loop (st.active: act_init)
        st.active[b] = 0;
        activate[b] = 1;
      }
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
          al = s_al[tt];
          ls = tt;
          Jn = s_J[tt];
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
        // per-problem tallies [B][3], summed once per solve (k_sum_counters): [0] problem-iterations,
        // [2] iterations with a fresh dynamics gradient (same-address atomics serialised the launch)
        unsigned long long* pc = counters + (size_t)b * 3;
        pc[0] += 1ull;
        pc[2] += (unsigned long long)st.need_grad[b];
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
    // trial trajectories are knot-major ([k][m], see k_ilqr_forward); x / u the reference's [m][k]; the
    // loads of U passes ahead of their stores (tmpc_copy.h)
    double* xb = x + (size_t)b * NX * N;
    double* ub = u + (size_t)b * NU * K;
    wg_batched<12, double>(NX * N, t, 64, [&](int e) {
      const int m = e / N, k = e - m * N;
      return xs_[k * NX + m];
    }, [&](int e, double v) { xb[e] = v; });
    wg_batched<8, double>(NU * K, t, 64, [&](int e) {
      const int m = e / K, k = e - m * K;
      return us_[k * NU + m];
    }, [&](int e, double v) { ub[e] = v; });
  }
}

// ======================================================================= launchers
#define TMPC_GRID(n, bs) dim3(((n) + (bs) - 1) / (bs)), dim3(bs)

template <int NJ, bool CHAIN, class MT>
struct LaunchIlqr {
  static void backward(bool f32, hipStream_t s, const CostDev* C, const ConstrDev* Cs, PList P, int B, int N, const double* x,
                       const double* u, const double* rho, const int* active, const double* A, const double* Bm,
                       const double* mu, const double* lam, double* jscratch, double* K, double* d, double* dV,
                       int* ok) {
    if constexpr (kWide<NJ>) {   // a wide model: fp64 VALU sweep, no soft limits (check_ready refuses the rest)
      hipLaunchKernelGGL((k_ilqr_backward<NJ, double, false>), dim3(B), dim3(64), 0, s, C, Cs, P, B, N, x, u, rho, active,
                         A, Bm, mu, lam, nullptr, K, d, dV, ok);
    } else {
      // fp64: the matrix-core products (MF) unless TMPC_ILQR_VALU=1 (the VALU loops, for comparison)
      const char* v = getenv("TMPC_ILQR_VALU");
      const bool mf = !(v && v[0] == '1');
      // soft limits: every knot's jacobian first, in parallel ([B][N][3 NJ] in jscratch)
      const double* js = nullptr;
      if (mu) {
        hipLaunchKernelGGL((k_ilqr_soft_jac<NJ>), TMPC_GRID(B * N, 256), 0, s, Cs, mu, lam, P, B, N, x, u, active, jscratch);
        js = jscratch;
      }
      // fp32: the Riccati state in fp32; its Q products on the matrix cores from the fp32 operands (fp64 MFMA
      // accumulation, rounded to fp32) unless TMPC_ILQR_F32_VALU=1 (the fp32 VALU loops)
      const char* fv = getenv("TMPC_ILQR_F32_VALU");
      const bool f32mf = mf && !(fv && fv[0] == '1');
      if (f32 && f32mf)
        hipLaunchKernelGGL((k_ilqr_backward<NJ, float, true>), dim3(B), dim3(64), 0, s, C, Cs, P, B, N, x, u, rho, active, A,
                           Bm, mu, lam, js, K, d, dV, ok);
      else if (f32)
        hipLaunchKernelGGL((k_ilqr_backward<NJ, float, false>), dim3(B), dim3(64), 0, s, C, Cs, P, B, N, x, u, rho, active, A,
                           Bm, mu, lam, js, K, d, dV, ok);
      else if (mf)
        hipLaunchKernelGGL((k_ilqr_backward<NJ, double, true>), dim3(B), dim3(64), 0, s, C, Cs, P, B, N, x, u, rho, active, A,
                           Bm, mu, lam, js, K, d, dV, ok);
      else
        hipLaunchKernelGGL((k_ilqr_backward<NJ, double, false>), dim3(B), dim3(64), 0, s, C, Cs, P, B, N, x, u, rho, active, A,
                           Bm, mu, lam, js, K, d, dV, ok);
    }
  }
  static void forward(bool f32, hipStream_t s, const ModelDev* M, const CostDev* C, const ConstrDev* Cs, const double* mu,
                      const double* lam, PList P, int B, int N, int T, double dt, int init, const double* alphas,
                      const double* x, const double* u, const double* K, const double* d, const int* active,
                      const int* ok, double* xt, double* ut, double* Jt) {
    // the prefetching instance when its LDS buffers fit (T >= 2: <= 33 problems per group); init
    // evaluations (no feedback law) take the plain one.  TMPC_ILQR_NOPF=1: plain only (comparison)
    const char* npf = getenv("TMPC_ILQR_NOPF");
    const size_t pf_lds = FwdPf<NJ>::lds_doubles(T) * sizeof(double);
    const bool pf = !init && pf_lds <= 48 * 1024 && !(npf && npf[0] == '1');
    if constexpr (kWide<NJ>) {   // a wide model: fp64, no soft limits, the plain (non-prefetching) instance
      hipLaunchKernelGGL((k_ilqr_forward<NJ, CHAIN, false, MT, double, false>), TMPC_GRID(B * T, 64), 0, s, MT::make(M), C,
                         Cs, mu, lam, P, B, N, T, dt, init, alphas, x, u, K, d, active, ok, xt, ut, Jt);
      return;
    } else {
#define TMPC_FWD(SOFTV, RV)                                                                                          \
    if (pf)                                                                                                          \
      hipLaunchKernelGGL((k_ilqr_forward<NJ, CHAIN, SOFTV, MT, RV, true>), TMPC_GRID(B * T, 64), pf_lds, s,           \
                         MT::make(M), C, Cs, mu, lam, P, B, N, T, dt, init, alphas, x, u, K, d, active, ok, xt, ut, Jt); \
    else                                                                                                             \
      hipLaunchKernelGGL((k_ilqr_forward<NJ, CHAIN, SOFTV, MT, RV, false>), TMPC_GRID(B * T, 64), 0, s, MT::make(M),  \
                         C, Cs, mu, lam, P, B, N, T, dt, init, alphas, x, u, K, d, active, ok, xt, ut, Jt);
    // soft limits: the rollouts sum the cost terms, k_ilqr_soft_add the soft values (INIT: in the kernel)
    if (mu && init) { if (f32) { TMPC_FWD(true, float) } else { TMPC_FWD(true, double) } }
    else { if (f32) { TMPC_FWD(false, float) } else { TMPC_FWD(false, double) } }
#undef TMPC_FWD
    if (mu && !init) {
      const int tg = soft_add_group(T, N);
      hipLaunchKernelGGL((k_ilqr_soft_add<NJ>), dim3(B), dim3(64), (size_t)tg * (N + 1) * sizeof(double), s, Cs, mu, lam,
                         P, B, N, T, tg, xt, ut, active, ok, Jt);
    }
    }
  }
};

// (Unlike tmpc_fd.hip / tmpc_kernels.hip, a runtime chain model keeps the CHAIN instance here: the rollout
// measured 2.1 ms per launch on it against 3.2 ms on the general-topology one, arm6 B = 4096.)
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
    TMPC_WIDE_CASES(LaunchIlqr, CALL)                                                                  \
    default: return -2;                                                                                \
  }                                                                                                    \
  return 0;

int launch_ilqr_backward(bool f32, hipStream_t s, int nj, const CostDev* C, const ConstrDev* Cs, PList P, int B, int N,
                         const double* x, const double* u, const double* rho, const int* active, const double* A,
                         const double* Bm, const double* mu, const double* lam, double* jscratch, double* K,
                         double* d, double* dV, int* ok) {
  const int mid = 0;
  TMPC_DISPATCH_ILQR(nj, true, backward(f32, s, C, Cs, P, B, N, x, u, rho, active, A, Bm, mu, lam, jscratch, K, d, dV,
                                        ok))
}

int launch_ilqr_forward(bool f32, hipStream_t s, int nj, bool chain, int mid, const ModelDev* M, const CostDev* C,
                        const ConstrDev* Cs, const double* mu, const double* lam, PList P, int B, int N, int T,
                        double dt, int init, const double* alphas, const double* x, const double* u, const double* K,
                        const double* d, const int* active, const int* ok, double* xt, double* ut, double* Jt) {
  TMPC_DISPATCH_ILQR(nj, chain, forward(f32, s, M, C, Cs, mu, lam, P, B, N, T, dt, init, alphas, x, u, K, d, active, ok,
                                        xt, ut, Jt))
}

int launch_ilqr_init_cost(hipStream_t s, int nj, const CostDev* C, const ConstrDev* Cs, const double* mu,
                          const double* lam, PList P, int B, int N, const double* x, const double* u, const int* mask,
                          double* Jt) {
  const size_t lds = (size_t)2 * N * sizeof(double);
  if (lds > 64 * 1024) return -1;
#define TMPC_INIT_COST(V)                                                                                      \
  case V:                                                                                                      \
    if (mu)                                                                                                    \
      hipLaunchKernelGGL((k_ilqr_init_cost<V, true>), dim3(B), dim3(64), lds, s, C, Cs, mu, lam, P, B, N, x, u, mask, Jt); \
    else                                                                                                       \
      hipLaunchKernelGGL((k_ilqr_init_cost<V, false>), dim3(B), dim3(64), lds, s, C, Cs, mu, lam, P, B, N, x, u, mask, Jt); \
    return 0;
  switch (nj) {
    TMPC_INIT_COST(1) TMPC_INIT_COST(2) TMPC_INIT_COST(3) TMPC_INIT_COST(4) TMPC_INIT_COST(5) TMPC_INIT_COST(6)
    TMPC_INIT_COST(7)
#define TMPC_INIT_COST_WIDE(V)   /* a wide model: no soft limits */                                         \
  case V:                                                                                                      \
    if (mu) return -2;                                                                                         \
    hipLaunchKernelGGL((k_ilqr_init_cost<V, false>), dim3(B), dim3(64), lds, s, C, Cs, mu, lam, P, B, N, x, u, mask, Jt); \
    return 0;
    TMPC_INIT_COST_WIDE(8) TMPC_INIT_COST_WIDE(9) TMPC_INIT_COST_WIDE(10) TMPC_INIT_COST_WIDE(11)
    TMPC_INIT_COST_WIDE(12)
#undef TMPC_INIT_COST_WIDE
    default: return -2;
  }
#undef TMPC_INIT_COST
}

void launch_ilqr_decide(hipStream_t s, PList P, int B, int N, int NX, int NU, int T, int init, const double* alphas,
                        const SolverOpts& o, const double* Jt, const double* dV, const int* ok, const double* xt,
                        const double* ut, double* x, double* u, const ProbState& st, const TraceDev& tr,
                        int* active_count, unsigned long long* counters, int* activate) {
  hipLaunchKernelGGL(k_ilqr_decide, dim3(B), dim3(64), 0, s, P, B, N, NX, NU, T, init, alphas, o, Jt, dV, ok, xt, ut, x,
                     u, st, tr, active_count, counters, activate);
}

}  // namespace tmpc
