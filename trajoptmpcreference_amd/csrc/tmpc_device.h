// Device-side data structures and per-lane rigid-body routines for gfx950.
//
// One lane evaluates one knot -- or one (knot, column) of a knot's
// derivative / inverse-inertia matrix -- with all state in VGPRs.  To keep
// that state small enough for a no-spill register allocation:
//   * the joint transform X_j(q) = X0 + c Xa + s Xb is never materialised:
//     rows (for X v) or columns (for X^T f) are formed on the fly from the
//     wave-uniform model coefficients (scalar loads);
//   * the motion subspace S_j is a uniform 0/1 vector, so S-products are plain
//     FMAs with scalar operands (no runtime-indexed register arrays);
//   * symmetric 6x6 inertias are stored as 21-entry upper triangles;
//   * arrays are indexed by compile-time joint ids; serial chains are a
//     separate instantiation where parent(j) = j-1 is a constant.
//
// Algorithms (GRiD/RBDReference/RBDReference.py, TrajoptPlant.py):
//   fd_aba          qdd = M^-1 (u - c(q, qd))  -- articulated-body form of
//                   URDFPlant.forward_dynamics (TrajoptPlant.py:283-299),
//                   mathematically identical to rnea + minv (:399-559,
//                   :805-930), O(n) and with O(n) live state;
//   minv_column     column `col` of the analytic M^-1 exactly as minv_bpass /
//                   minv_fpass compute it (:805-906), one column per lane;
//   rnea_grad_column  column `col` of rnea_grad (:561-802) fused with the
//                   rnea passes that produce v, a and the accumulated f.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tmpc {

constexpr int NJMAX = 8;
constexpr int NXMAX = 2 * NJMAX;

struct ModelDev {
  int n;
  int chain;                  // 1 if parent[j] == j-1 for all j
  int parent[NJMAX];
  int jtype[NJMAX];           // 0 revolute (X = X0 + cos q Xa + sin q Xb), 1 prismatic (X = X0 + q Xa)
  int saxis[NJMAX];           // S = e_saxis
  uint32_t subtree[NJMAX];    // bit s set <=> s in subtree(j)
  double gravity;             // options['gravity'] (TrajoptPlant.py:31); a_base[5] = -gravity
  double S[NJMAX][6];         // motion subspace vectors (0/1)
  double X0[NJMAX][36];
  double Xa[NJMAX][36];
  double Xb[NJMAX][36];
  double I[NJMAX][36];
};

struct CostDev {            // QuadraticCost (TrajoptCost.py:24-104)
  int nx, nu;
  int QF_start;             // -1 = None
  int pad;
  double Q[NXMAX * NXMAX];
  double QF[NXMAX * NXMAX];
  double R[NJMAX * NJMAX];
  double xg[NXMAX];
};

// Soft box limits: BoxConstraint in QUADRATIC_PENALTY / AUGMENTED_LAGRANGIAN
// mode (TrajoptConstraint.py:53-166) with the vector semantics of
// oracle/soft.py.  Type t: 0 joint (q), 1 velocity (qd), 2 torque (u).  Per
// knot the constants mu / lambda / phi have 6 n slots, slot t*2n + e with
// e < n the lower half (v = z - lb) and e >= n the upper half (v = ub - z).
// Joint and velocity limits cover knots 0..N-1, torque limits 0..N-2.
enum { SOFT_NONE = 0, SOFT_QP = 1, SOFT_AL = 2 };

struct ConstrDev {
  int mode[3];              // SOFT_* per type
  int any;                  // some type is soft
  double lb[3][NJMAX], ub[3][NJMAX];
  double mu_init[3], mu_factor[3], mu_max[3], phi_init[3], phi_factor[3];   // BoxConstraint options (:38-46)
};

// Value (summed over types, value_soft_constraints :296-310) and the per-type
// jacobians of one knot.  z = [q; qd; u] (u unused at the terminal knot); the
// three jacobians have disjoint supports, so jac[3 NJ] holds all of them.
// Arithmetic as BoxConstraint.value / .jacobian (:53-128).
template <int NJ>
__device__ __forceinline__ double soft_knot(const ConstrDev* __restrict__ Cs, const double* __restrict__ mu,
                                            const double* __restrict__ lam, bool terminal, const double (&z)[3 * NJ],
                                            double (&jac)[3 * NJ]) {
  double value = 0.0;
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const int md = Cs->mode[t];
#pragma unroll
    for (int i = 0; i < NJ; ++i) jac[t * NJ + i] = 0.0;
    if (md == SOFT_NONE || (t == 2 && terminal)) continue;
    double sq = 0.0, lin = 0.0;
#pragma unroll
    for (int e = 0; e < 2 * NJ; ++e) {
      const int i = e < NJ ? e : e - NJ;
      const double zi = z[t * NJ + i];
      const double v = e < NJ ? zi - Cs->lb[t][i] : Cs->ub[t][i] - zi;
      const double m = mu[t * 2 * NJ + e];
      const double l = lam[t * 2 * NJ + e];
      sq += m * (v * v);
      lin += l * v;
      if (v < 0.0) {
        const double s = e < NJ ? 1.0 : -1.0;
        double coef = 2.0 * (m * (v * s));
        if (md == SOFT_AL) coef += l * s;
        jac[t * NJ + i] += coef;
      }
    }
    value += md == SOFT_AL ? sq + lin : sq;
  }
  return value;
}

// ----------------------------------------------------------------- helpers
template <bool CHAIN>
__device__ __forceinline__ int parent_of(const ModelDev* __restrict__ M, int j) {
  return CHAIN ? j - 1 : M->parent[j];
}

template <bool CHAIN>
__device__ __forceinline__ bool in_subtree(const ModelDev* __restrict__ M, int j, int s) {
  return CHAIN ? (s >= j) : ((M->subtree[j] >> s) & 1u);
}

__device__ __forceinline__ void joint_cs(const ModelDev* __restrict__ M, int j, double q, double& c, double& s) {
  if (M->jtype[j] == 0) {
    sincos(q, &s, &c);
  } else {
    c = q;
    s = 0.0;
  }
}

// Opaque copy: stops the compiler from CSE-ing X entries across passes
// (which would keep 36 doubles per joint live for the whole kernel).
__device__ __forceinline__ void opaque(double& c, double& s) { asm volatile("" : "+v"(c), "+v"(s)); }

// y = X v, rows formed on the fly
__device__ __forceinline__ void mvX(const ModelDev* __restrict__ M, int j, double c, double s, const double v[6],
                                    double y[6]) {
  opaque(c, s);
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    double acc = 0.0;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const double x = M->X0[j][r * 6 + k] + c * M->Xa[j][r * 6 + k] + s * M->Xb[j][r * 6 + k];
      acc += x * v[k];
    }
    y[r] = acc;
  }
}

// y += X^T f, columns formed on the fly
__device__ __forceinline__ void add_mtvX(const ModelDev* __restrict__ M, int j, double c, double s,
                                         const double f[6], double y[6]) {
  opaque(c, s);
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    double acc = 0.0;
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      const double x = M->X0[j][r * 6 + k] + c * M->Xa[j][r * 6 + k] + s * M->Xb[j][r * 6 + k];
      acc += x * f[r];
    }
    y[k] += acc;
  }
}

// o = I v, I a uniform model matrix
__device__ __forceinline__ void mvI(const double* __restrict__ I, const double v[6], double o[6]) {
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    double acc = 0.0;
#pragma unroll
    for (int k = 0; k < 6; ++k) acc += I[r * 6 + k] * v[k];
    o[r] = acc;
  }
}

// crm(w) S for a 0/1 subspace vector S (mxS, RBDReference.py:57-62)
__device__ __forceinline__ void crmS(const double w[6], const double* __restrict__ S, double o[6]) {
  o[0] = -w[2] * S[1] + w[1] * S[2];
  o[1] = w[2] * S[0] - w[0] * S[2];
  o[2] = -w[1] * S[0] + w[0] * S[1];
  o[3] = -w[5] * S[1] + w[4] * S[2] - w[2] * S[4] + w[1] * S[5];
  o[4] = w[5] * S[0] - w[3] * S[2] + w[2] * S[3] - w[0] * S[5];
  o[5] = -w[4] * S[0] + w[3] * S[1] - w[1] * S[3] + w[0] * S[4];
}

__device__ __forceinline__ double dotS(const double* __restrict__ S, const double v[6]) {
  double acc = 0.0;
#pragma unroll
  for (int k = 0; k < 6; ++k) acc += S[k] * v[k];
  return acc;
}

// o += fxv(f, t) = crf(f) t (RBDReference.py:71-91); vxIv(v, I) = fxv(v, I v) (:98-116)
__device__ __forceinline__ void add_fxv(const double f[6], const double t[6], double o[6]) {
  o[0] += -f[2] * t[1] + f[1] * t[2] - f[5] * t[4] + f[4] * t[5];
  o[1] += f[2] * t[0] - f[0] * t[2] + f[5] * t[3] - f[3] * t[5];
  o[2] += -f[1] * t[0] + f[0] * t[1] - f[4] * t[3] + f[3] * t[4];
  o[3] += -f[2] * t[4] + f[1] * t[5];
  o[4] += f[2] * t[3] - f[0] * t[5];
  o[5] += -f[1] * t[3] + f[0] * t[4];
}

// symmetric 6x6 upper-triangle storage
__device__ __forceinline__ constexpr int sidx(int r, int c) {
  return r <= c ? r * 6 - (r * (r - 1)) / 2 + (c - r) : c * 6 - (c * (c - 1)) / 2 + (r - c);
}

// out = X^T A X for symmetric A (21 entries).  Column-at-a-time so that only
// two 6-vectors of X and one of A X are live (X columns are recomputed).
__device__ __forceinline__ void Xcol(const ModelDev* __restrict__ M, int j, double c, double s, int k, double x[6]) {
#pragma unroll
  for (int r = 0; r < 6; ++r) x[r] = M->X0[j][r * 6 + k] + c * M->Xa[j][r * 6 + k] + s * M->Xb[j][r * 6 + k];
}

__device__ __forceinline__ void XtAX(const ModelDev* __restrict__ M, int j, double c, double s, const double A[21],
                                     double out[21]) {
  opaque(c, s);
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    double xk[6], z[6];
    Xcol(M, j, c, s, k, xk);
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      double acc = 0.0;
#pragma unroll
      for (int m = 0; m < 6; ++m) acc += A[sidx(r, m)] * xk[m];
      z[r] = acc;
    }
#pragma unroll
    for (int r = 0; r <= k; ++r) {
      double xr[6];
      if (r == k) {
#pragma unroll
        for (int m = 0; m < 6; ++m) xr[m] = xk[m];
      } else {
        Xcol(M, j, c, s, r, xr);
      }
      double acc = 0.0;
#pragma unroll
      for (int m = 0; m < 6; ++m) acc += xr[m] * z[m];
      out[sidx(r, k)] = acc;
    }
  }
}

// y1 = X v1, y2 = X v2 sharing the formation of each X row
__device__ __forceinline__ void mvX2(const ModelDev* __restrict__ M, int j, double c, double s, const double v1[6],
                                     const double v2[6], double y1[6], double y2[6]) {
  opaque(c, s);
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    double a1 = 0.0, a2 = 0.0;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const double x = M->X0[j][r * 6 + k] + c * M->Xa[j][r * 6 + k] + s * M->Xb[j][r * 6 + k];
      a1 += x * v1[k];
      a2 += x * v2[k];
    }
    y1[r] = a1;
    y2[r] = a2;
  }
}

// ----------------------------------------------------------------- forward dynamics (ABA)
// qdd = M(q)^-1 (tau - c(q, qd)), gravity as the fictitious base acceleration
// a_base[5] = -gravity (RBDReference.py:456).  With UNIT = true it returns
// M^-1 tau (qd = 0, no gravity).  Velocities are recomputed in pass 3
// instead of being kept from pass 1, so at most ~8 doubles per joint are
// stored across passes.
template <int NJ, bool CHAIN, bool UNIT = false>
__device__ __forceinline__ void fd_aba(const ModelDev* __restrict__ M, const double cq[NJ], const double sq[NJ],
                                       const double qd[NJ], const double tau[NJ], double qdd[NJ]) {
  double v[NJ][6];
  // pass 1: velocities
  if (!UNIT) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int p = parent_of<CHAIN>(M, j);
      if (p < 0) {
#pragma unroll
        for (int i = 0; i < 6; ++i) v[j][i] = 0.0;
      } else {
        mvX(M, j, cq[j], sq[j], v[p], v[j]);
      }
#pragma unroll
      for (int i = 0; i < 6; ++i) v[j][i] += M->S[j][i] * qd[j];
    }
  }
  // pass 2: articulated inertias / bias forces, leaf to root
  double chIA[NJ][21], chpA[NJ][6];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
#pragma unroll
    for (int e = 0; e < 21; ++e) chIA[j][e] = 0.0;
#pragma unroll
    for (int e = 0; e < 6; ++e) chpA[j][e] = 0.0;
  }
  double U[NJ][6], Dd[NJ], uu[NJ];
#pragma unroll
  for (int j = NJ - 1; j >= 0; --j) {
    double IA[21];
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
      for (int k = r; k < 6; ++k) IA[sidx(r, k)] = M->I[j][r * 6 + k] + chIA[j][sidx(r, k)];
    double pA[6], cj[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) pA[i] = chpA[j][i];
    if (!UNIT) {
      double Iv[6];
      mvI(M->I[j], v[j], Iv);
      add_fxv(v[j], Iv, pA);
      double cc[6];
      crmS(v[j], M->S[j], cc);
#pragma unroll
      for (int i = 0; i < 6; ++i) cj[i] = qd[j] * cc[i];
    } else {
#pragma unroll
      for (int i = 0; i < 6; ++i) cj[i] = 0.0;
    }
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      double acc = 0.0;
#pragma unroll
      for (int k = 0; k < 6; ++k) acc += IA[sidx(r, k)] * M->S[j][k];
      U[j][r] = acc;
    }
    Dd[j] = dotS(M->S[j], U[j]);
    uu[j] = tau[j] - dotS(M->S[j], pA);
    const int p = parent_of<CHAIN>(M, j);
    if (p >= 0) {
      const double dinv = 1.0 / Dd[j];
#pragma unroll
      for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int k = r; k < 6; ++k) IA[sidx(r, k)] -= U[j][r] * (dinv * U[j][k]);   // Ia
      double pa[6];
      const double ud = uu[j] * dinv;
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        double acc = pA[r] + U[j][r] * ud;
        if (!UNIT) {
#pragma unroll
          for (int k = 0; k < 6; ++k) acc += IA[sidx(r, k)] * cj[k];
        }
        pa[r] = acc;
      }
      double t[21];
      XtAX(M, j, cq[j], sq[j], IA, t);
#pragma unroll
      for (int e = 0; e < 21; ++e) chIA[p][e] += t[e];
      add_mtvX(M, j, cq[j], sq[j], pa, chpA[p]);
    }
  }
  // pass 3: accelerations, root to leaf (velocities recomputed)
  double v3[NJ][6], a[NJ][6];
  const double g[6] = {0.0, 0.0, 0.0, 0.0, 0.0, UNIT ? 0.0 : -M->gravity};
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int p = parent_of<CHAIN>(M, j);
    if (UNIT) {
      if (p < 0)
        mvX(M, j, cq[j], sq[j], g, a[j]);
      else
        mvX(M, j, cq[j], sq[j], a[p], a[j]);
    } else {
      if (p < 0) {
        mvX(M, j, cq[j], sq[j], g, a[j]);
#pragma unroll
        for (int i = 0; i < 6; ++i) v3[j][i] = 0.0;
      } else {
        mvX2(M, j, cq[j], sq[j], v3[p], a[p], v3[j], a[j]);
      }
#pragma unroll
      for (int i = 0; i < 6; ++i) v3[j][i] += M->S[j][i] * qd[j];
      double cc[6];
      crmS(v3[j], M->S[j], cc);
#pragma unroll
      for (int i = 0; i < 6; ++i) a[j][i] += qd[j] * cc[i];
    }
    qdd[j] = (uu[j] - dotS(U[j], a[j])) / Dd[j];
#pragma unroll
    for (int i = 0; i < 6; ++i) a[j][i] += M->S[j][i] * qdd[j];
  }
}

// ----------------------------------------------------------------- analytic M^-1, one column
// Computes Minv[r][col] for r <= col (the upper triangle the reference fills
// before symmetrising, :908-930) following minv_bpass / minv_fpass
// restricted to column `col` (F[:, :, col] is per column; IA, U, Dinv are
// recomputed per lane).
template <int NJ, bool CHAIN>
__device__ __forceinline__ void minv_column(const ModelDev* __restrict__ M, const double cq[NJ], const double sq[NJ],
                                            int col, double mcol[NJ]) {
  double chIA[NJ][21];
  double Fc[NJ][6];      // F[j][:, col]
  double U[NJ][6], Dinv[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    mcol[j] = 0.0;
#pragma unroll
    for (int e = 0; e < 21; ++e) chIA[j][e] = 0.0;
#pragma unroll
    for (int e = 0; e < 6; ++e) Fc[j][e] = 0.0;
  }
  // backward pass (:805-866)
#pragma unroll
  for (int j = NJ - 1; j >= 0; --j) {
    double IA[21];
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
      for (int k = r; k < 6; ++k) IA[sidx(r, k)] = M->I[j][r * 6 + k] + chIA[j][sidx(r, k)];
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      double acc = 0.0;
#pragma unroll
      for (int k = 0; k < 6; ++k) acc += IA[sidx(r, k)] * M->S[j][k];
      U[j][r] = acc;
    }
    Dinv[j] = 1.0 / dotS(M->S[j], U[j]);
    const bool mine = in_subtree<CHAIN>(M, j, col);
    if (j == col) mcol[j] = Dinv[j];
    if (mine) mcol[j] -= Dinv[j] * dotS(M->S[j], Fc[j]);
    const int p = parent_of<CHAIN>(M, j);
    if (p >= 0) {
      if (mine) {
#pragma unroll
        for (int r = 0; r < 6; ++r) Fc[j][r] += U[j][r] * mcol[j];
        add_mtvX(M, j, cq[j], sq[j], Fc[j], Fc[p]);
      }
      double Ia[21];
#pragma unroll
      for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int k = r; k < 6; ++k) Ia[sidx(r, k)] = IA[sidx(r, k)] - U[j][r] * (Dinv[j] * U[j][k]);
      double t[21];
      XtAX(M, j, cq[j], sq[j], Ia, t);
#pragma unroll
      for (int e = 0; e < 21; ++e) chIA[p][e] += t[e];
    }
  }
  // forward pass (:868-906), rows j <= col
  double Ff[NJ][6];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    if (j > col) break;
    const int p = parent_of<CHAIN>(M, j);
    if (p >= 0) {
      double XF[6];
      mvX(M, j, cq[j], sq[j], Ff[p], XF);   // X F[p][:, col]
      // (U^T X) F[p][:, col] == U^T (X F[p][:, col])
      mcol[j] -= Dinv[j] * dotS(U[j], XF);
#pragma unroll
      for (int r = 0; r < 6; ++r) Ff[j][r] = M->S[j][r] * mcol[j] + XF[r];
    } else {
#pragma unroll
      for (int r = 0; r < 6; ++r) Ff[j][r] = M->S[j][r] * mcol[j];
    }
  }
}

// ----------------------------------------------------------------- one derivative column
// d c / d q_col (colqd = false) or d c / d qd_col (colqd = true) at (q, qd, qdd):
// rnea_grad forward passes (:561-690) and backward passes (:692-771) for ONE
// column, fused with the RNEA passes that produce v, a and the accumulated f.
template <int NJ, bool CHAIN>
__device__ __forceinline__ void rnea_grad_column(const ModelDev* __restrict__ M, const double cq[NJ],
                                                 const double sq[NJ], const double qd[NJ], const double qdd[NJ],
                                                 int col, bool colqd, double dc[NJ]) {
  double v[NJ][6], a[NJ][6], f[NJ][6];
  double dv[NJ][6], da[NJ][6], df[NJ][6];
  const double g[6] = {0.0, 0.0, 0.0, 0.0, 0.0, -M->gravity};
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int p = parent_of<CHAIN>(M, j);
    const double* S = M->S[j];
    // ---- RNEA forward (with qdd)
    double Xvp[6], Xap[6];
    if (p < 0) {
#pragma unroll
      for (int i = 0; i < 6; ++i) Xvp[i] = 0.0;
      mvX(M, j, cq[j], sq[j], g, Xap);
    } else {
      mvX(M, j, cq[j], sq[j], v[p], Xvp);
      mvX(M, j, cq[j], sq[j], a[p], Xap);
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) v[j][i] = Xvp[i] + S[i] * qd[j];
    {
      double cc[6];
      crmS(v[j], S, cc);
#pragma unroll
      for (int i = 0; i < 6; ++i) a[j][i] = Xap[i] + qd[j] * cc[i] + S[i] * qdd[j];
    }
    double Iv[6];
    mvI(M->I[j], a[j], f[j]);
    mvI(M->I[j], v[j], Iv);
    add_fxv(v[j], Iv, f[j]);
    // ---- derivative forward pass for this column
    if (p >= 0) {
      mvX(M, j, cq[j], sq[j], dv[p], dv[j]);
      mvX(M, j, cq[j], sq[j], da[p], da[j]);
    } else {
#pragma unroll
      for (int i = 0; i < 6; ++i) { dv[j][i] = 0.0; da[j][i] = 0.0; }
    }
    if (j == col) {
      if (!colqd) {
        if (p >= 0) {
          double cc[6];
          crmS(Xvp, S, cc);
#pragma unroll
          for (int i = 0; i < 6; ++i) dv[j][i] += cc[i];
        }
      } else {
#pragma unroll
        for (int i = 0; i < 6; ++i) dv[j][i] += S[i];
      }
    }
    {
      double cc[6];
      crmS(dv[j], S, cc);
#pragma unroll
      for (int i = 0; i < 6; ++i) da[j][i] += qd[j] * cc[i];
    }
    if (j == col) {
      double cc[6];
      crmS(colqd ? v[j] : Xap, S, cc);  // mxS(S, v) or mxS(S, X a_parent) / mxS(S, X g)
#pragma unroll
      for (int i = 0; i < 6; ++i) da[j][i] += cc[i];
    }
    mvI(M->I[j], da[j], df[j]);
    add_fxv(dv[j], Iv, df[j]);
    double Idv[6];
    mvI(M->I[j], dv[j], Idv);
    add_fxv(v[j], Idv, df[j]);
  }
  // ---- fused backward passes
#pragma unroll
  for (int j = NJ - 1; j >= 0; --j) {
    const double* S = M->S[j];
    dc[j] = dotS(S, df[j]);
    const int p = parent_of<CHAIN>(M, j);
    if (p >= 0) {
      add_mtvX(M, j, cq[j], sq[j], df[j], df[p]);
      if (!colqd && j == col) {
        // delta = X^T fxS(S, f) = -X^T (crm(f) S)
        double cc[6];
        crmS(f[j], S, cc);
#pragma unroll
        for (int i = 0; i < 6; ++i) cc[i] = -cc[i];
        add_mtvX(M, j, cq[j], sq[j], cc, df[p]);
      }
      add_mtvX(M, j, cq[j], sq[j], f[j], f[p]);
    }
  }
}

}  // namespace tmpc
