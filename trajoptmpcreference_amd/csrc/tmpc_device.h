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

constexpr int NJMAX = 12;
constexpr int NXMAX = 2 * NJMAX;
// joint counts with every kernel instance (fp32 / mixed, soft and hard limits, iLQR, the HBM-row QP, ...);
// 8..NJMAX joints run the SQP on the runtime model (ModelRef), fp64, without box limits, up to 1024 Schur
// rows: a "wide" model
constexpr int NJ_FULL = 7;
template <int NJ>
constexpr bool kWide = NJ > NJ_FULL;
// dispatch-table cases of the wide joint counts: the runtime model's general-topology instance (a chain is
// a tree; one instance per joint count keeps the build's size)
#define TMPC_WIDE_CASES(LAUNCH, CALL)                  \
  case 8: LAUNCH<8, false, ModelRef>::CALL; break;     \
  case 9: LAUNCH<9, false, ModelRef>::CALL; break;     \
  case 10: LAUNCH<10, false, ModelRef>::CALL; break;   \
  case 11: LAUNCH<11, false, ModelRef>::CALL; break;   \
  case 12: LAUNCH<12, false, ModelRef>::CALL; break;

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

enum { COST_QUADRATIC = 0, COST_EE = 1 };

struct CostDev {            // QuadraticCost (TrajoptCost.py:24-104) or UrdfCost (:371-569)
  int nx, nu;
  int QF_start;             // -1 = None
  int kind;                 // COST_*
  // QuadraticCost with diagonal Q, QF and R (set by tmpc_set_cost_quadratic; the reference's own
  // workloads).  A dot product against such a row adds fma(0, y, acc) = acc for every
  // off-diagonal entry, so it reduces to its diagonal term bit for bit -- for finite y: a
  // non-finite entry makes every generic sum NaN (0 * inf) and diag_dot keeps that explicitly.
  int diag;
  double Q[NXMAX * NXMAX];
  double QF[NXMAX * NXMAX];
  double R[NJMAX * NJMAX];
  double xg[NXMAX];
  // COST_EE: homogeneous joint transforms H_j(q) = H0 + cos q Ha + sin q Hb (Joint.py:91-97),
  // row-major 4x4, joints 0 and 1 of the 2-link chain
  double eeH0[2][16], eeHa[2][16], eeHb[2][16];
};

// sum_c M[r][c] y[c] for a diagonal M of order n (CostDev.diag): the generic chain's value.
// poison: NaN when some y[c] is non-finite and n > 1 (then 0 * y[c] enters every generic row sum
// but the diagonal one), else 0 -- callers add it to the result the generic form would have poisoned
template <class T>
__device__ __forceinline__ T diag_poison(const T* y, int n) {
  bool fin = true;
  for (int c = 0; c < n; ++c) fin = fin && isfinite(y[c]);
  return (fin || n < 2) ? T(0) : T(NAN);
}

// UrdfCost task-space terms at one knot (2-link arms only, as the reference: SURVEY F5).
//   y = [p(q); J(q) qd] - xg          delta_x           TrajoptCost.py:425-435
//   p = (H_0 H_1 o)[0:2], o = [0,1,0,1]  end_effector_positions  RBDReference.py:123-148
//   J[:, d] = (chain with dH_d) o [0:2]  Jacobian               RBDReference.py:334-387
//   Jt = [[J, 0], [reshape(dJdq qd), J]] with the hand-coded dJdq pattern (:252-259, :313-331)
// Returns 0.5 y^T Q y (value, :415) and writes grad = (y^T Q) Jt (:449) and Jt.
template <int NJ>
__device__ __forceinline__ double ee_eval(const CostDev* __restrict__ C, const double* __restrict__ Qk,
                                          const double* xk, double* grad, double* Jt) {
  constexpr int NX = 2 * NJ;
  if constexpr (NJ != 2) {
    for (int m = 0; m < NX; ++m) grad[m] = 0.0;
    for (int m = 0; m < NX * NX; ++m) Jt[m] = 0.0;
    return 0.0;
  } else {
    double H[2][16], dH[2][16];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      double s, c;
      sincos(xk[j], &s, &c);
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        H[j][e] = C->eeH0[j][e] + c * C->eeHa[j][e] + s * C->eeHb[j][e];
        dH[j][e] = -s * C->eeHa[j][e] + c * C->eeHb[j][e];
      }
    }
    // o = [0, 1, 0, 1]: M o = column 1 + column 3
    double v1[4], w1[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      v1[r] = H[1][r * 4 + 1] + H[1][r * 4 + 3];
      w1[r] = dH[1][r * 4 + 1] + dH[1][r * 4 + 3];
    }
    double p[2], J[2][2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      double a = 0.0, b = 0.0, d = 0.0;
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        a += H[0][r * 4 + m] * v1[m];
        b += dH[0][r * 4 + m] * v1[m];
        d += H[0][r * 4 + m] * w1[m];
      }
      p[r] = a;
      J[r][0] = b;
      J[r][1] = d;
    }
    const double qd0 = xk[2], qd1 = xk[3];
    const double J2[2][2] = {{-J[1][0] * qd0 - J[1][1] * qd1, -J[1][1] * qd0 - J[1][1] * qd1},
                             {-J[0][0] * qd0 - J[0][1] * qd1, J[0][1] * qd0 + J[0][1] * qd1}};
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        Jt[r * 4 + c] = J[r][c];
        Jt[r * 4 + 2 + c] = 0.0;
        Jt[(2 + r) * 4 + c] = J2[r][c];
        Jt[(2 + r) * 4 + 2 + c] = J[r][c];
      }
    double y[4];
    y[0] = p[0] - C->xg[0];
    y[1] = p[1] - C->xg[1];
    y[2] = (J[0][0] * qd0 + J[0][1] * qd1) - C->xg[2];
    y[3] = (J[1][0] * qd0 + J[1][1] * qd1) - C->xg[3];
    double v = 0.0, gq[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      double qy = 0.0, yq = 0.0;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        qy += Qk[r * 4 + c] * y[c];
        yq += y[c] * Qk[c * 4 + r];
      }
      v += y[r] * qy;
      gq[r] = yq;
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      double g = 0.0;
#pragma unroll
      for (int l = 0; l < 4; ++l) g += gq[l] * Jt[l * 4 + c];
      grad[c] = g;
    }
    return 0.5 * v;
  }
}

// Soft box limits: BoxConstraint in QUADRATIC_PENALTY / AUGMENTED_LAGRANGIAN
// mode (TrajoptConstraint.py:53-166) with the vector semantics of
// oracle/soft.py.  Type t: 0 joint (q), 1 velocity (qd), 2 torque (u).  Per
// knot the constants mu / lambda / phi have 6 n slots, slot t*2n + e with
// e < n the lower half (v = z - lb) and e >= n the upper half (v = ub - z).
// Joint and velocity limits cover knots 0..N-1, torque limits 0..N-2.
enum { SOFT_NONE = 0, SOFT_QP = 1, SOFT_AL = 2 };
// hard modes (BoxConstraint ACTIVE_SET / FULL_SET, TrajoptConstraint.py:27-30,64-68,110-113):
// rows of C / c per knot, tmpc_hard.hip
enum { HARD_NONE = 0, HARD_ACTIVE = 1, HARD_FULL = 2 };

struct ConstrDev {
  int mode[3];              // SOFT_* per type
  int any;                  // some type is soft
  int hard[3];              // HARD_* per type (a type is soft or hard, not both)
  int any_hard;             // some type is hard
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

// The per-lane dynamics kernels read the model's coefficients (X0 / Xa / Xb /
// I: ~9 KB) with wave-uniform addresses.  From global memory they become
// scalar loads that the fully unrolled recursions hoist far ahead of use, and
// the SGPR file overflows into v_writelane / v_readlane spill traffic (15.6k
// v_readlane per k_qp_grad lane vs 5.5k fp64 FMAs).  Staging the model in LDS
// removes the spills but exposes an LDS round trip per coefficient: measured
// on MI355X (arm6, B = 4096) it is 3.5x / 10x slower for k_qp_grad /
// k_ls_terms (1 wave per SIMD, nothing hides the latency) and 1.2x faster for
// k_ilqr_forward, whose knot loop is not unrolled; only the latter uses it.
__device__ __forceinline__ const ModelDev* stage_model(const ModelDev* __restrict__ Mg, ModelDev* sM) {
  constexpr int W = (int)(sizeof(ModelDev) / sizeof(unsigned long long));
  static_assert(sizeof(ModelDev) % sizeof(unsigned long long) == 0, "ModelDev must be 8-byte sized");
  const unsigned long long* src = reinterpret_cast<const unsigned long long*>(Mg);
  unsigned long long* dst = reinterpret_cast<unsigned long long*>(sM);
  for (int i = threadIdx.x; i < W; i += blockDim.x) dst[i] = src[i];
  __syncthreads();
  return sM;
}

// ----------------------------------------------------------------- scalar type
// The dynamics routines below are templated on the arithmetic type R: double
// (the reference's fp64, bit-for-bit the untemplated code) or float (the
// fp32 / mixed precision modes of tmpc_options.precision).  Model
// coefficients are stored in double and rounded to R where they are used.
__device__ __forceinline__ void sincos_r(double q, double& s, double& c) { sincos(q, &s, &c); }
__device__ __forceinline__ void sincos_r(float q, float& s, float& c) { sincosf(q, &s, &c); }
__device__ __forceinline__ double fma_r(double a, double b, double c) { return __fma_rn(a, b, c); }
__device__ __forceinline__ float fma_r(float a, float b, float c) { return __fmaf_rn(a, b, c); }

// Products and sums with an operand that is a compile-time zero after inlining and unrolling (a
// structural zero of a compiled model propagated through the recursions: for the planar arms the
// out-of-plane block of the articulated inertias, of U and of the accelerations) are dropped.  The
// compiler cannot fold acc + 0 * x itself (0 * x is NaN for non-finite x, and -0 + 0 = +0); for
// finite operands the result is the same value (up to the sign of a zero), and the now-unused
// out-of-plane quantities are removed as dead code.  __builtin_constant_p is resolved after
// inlining (llvm.is.constant), so the test sees the propagated constants.
template <class R>
__device__ __forceinline__ bool czero(R a) {
  return __builtin_constant_p(a) && a == R(0);
}
// acc + a b  (contracted to one fma where the original `acc += a * b` is)
template <bool PR = true, class R>
__device__ __forceinline__ R madd(R acc, R a, R b) {
  if (PR && (czero(a) || czero(b))) return acc;
  if (PR && czero(acc)) return a * b;
  return acc + a * b;
}
// acc - a b
template <bool PR = true, class R>
__device__ __forceinline__ R msub(R acc, R a, R b) {
  if (PR && (czero(a) || czero(b))) return acc;
  return acc - a * b;
}
// a + b
template <bool PR = true, class R>
__device__ __forceinline__ R addz(R a, R b) {
  if (PR && czero(b)) return a;
  if (PR && czero(a)) return b;
  return a + b;
}
// a b (zero when either factor is a compile-time zero)
template <bool PR = true, class R>
__device__ __forceinline__ R mulz(R a, R b) {
  if (PR && (czero(a) || czero(b))) return R(0);
  return a * b;
}

// ----------------------------------------------------------------- model access
// The dynamics routines take the model as `const MT& M` and read it as
// `M->field`:
//   ModelRef  the runtime model (ModelDev in HBM, from tmpc_set_model): every
//             coefficient is a wave-uniform load;
//   Arm<N>    a compile-time model (tmpc_models.h, generated from the bundled
//             URDFs the way GRiD generates per-robot code): the same fields as
//             static constexpr arrays, so coefficients fold to literals and the
//             structural zeros of X(q), I and S drop out at compile time.
// The compile-time path performs the same floating-point operations on the
// nonzero terms (a skipped term is acc + x * 0 = acc), so both paths agree for
// finite inputs.
struct ModelRef {
  static constexpr bool STATIC = false;
  const ModelDev* p;
  __device__ __forceinline__ const ModelDev* operator->() const { return p; }
  static ModelRef make(const ModelDev* q) { return ModelRef{q}; }
};

// true unless `a` is a structural zero of a compile-time model
template <class MT>
__device__ __forceinline__ constexpr bool nz(double a) {
  return !MT::STATIC || a != 0.0;
}

template <bool CHAIN, class MT>
__device__ __forceinline__ int parent_of(const MT& M, int j) {
  return CHAIN ? j - 1 : M->parent[j];
}

template <bool CHAIN, class MT>
__device__ __forceinline__ bool in_subtree(const MT& M, int j, int s) {
  return CHAIN ? (s >= j) : ((M->subtree[j] >> s) & 1u);
}

template <class MT, class R>
__device__ __forceinline__ void joint_cs(const MT& M, int j, R q, R& c, R& s) {
  if (M->jtype[j] == 0) {
    sincos_r(q, s, c);
  } else {
    c = q;
    s = 0.0;
  }
}

// Opaque copy: stops the compiler from CSE-ing X entries across passes
// (which would keep 36 doubles per joint live for the whole kernel).
template <class R>
__device__ __forceinline__ void opaque(R& c, R& s) { asm volatile("" : "+v"(c), "+v"(s)); }

// entry e of X_j(q) = X0 + cos(q) Xa + sin(q) Xb; false for a structural zero
template <class MT, class R>
__device__ __forceinline__ bool xent(const MT& M, int j, int e, R c, R s, R& x) {
  const double a0 = M->X0[j][e], a1 = M->Xa[j][e], a2 = M->Xb[j][e];
  if (!MT::STATIC) {
    x = R(a0) + c * R(a1) + s * R(a2);
    return true;
  }
  if (a0 == 0.0 && a1 == 0.0 && a2 == 0.0) return false;
  R t = a0;
  if (a1 != 0.0) t = a0 != 0.0 ? fma_r(c, R(a1), R(a0)) : c * R(a1);
  if (a2 != 0.0) t = (a0 != 0.0 || a1 != 0.0) ? fma_r(s, R(a2), t) : s * R(a2);
  x = t;
  return true;
}

// y = X v, rows formed on the fly
template <bool PR = true, class MT, class R>
__device__ __forceinline__ void mvX(const MT& M, int j, R c, R s, const R v[6], R y[6]) {
  opaque(c, s);
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    R acc = 0.0;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      R x;
      if (xent(M, j, r * 6 + k, c, s, x)) acc = madd<PR>(acc, x, v[k]);
    }
    y[r] = acc;
  }
}

// y += X^T f, columns formed on the fly
template <bool PR = true, class MT, class R>
__device__ __forceinline__ void add_mtvX(const MT& M, int j, R c, R s, const R f[6], R y[6]) {
  opaque(c, s);
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    R acc = 0.0;
    bool any = false;
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      R x;
      if (xent(M, j, r * 6 + k, c, s, x)) {
        acc = madd<PR>(acc, x, f[r]);
        any = true;
      }
    }
    if (any) y[k] = addz<PR>(y[k], acc);
  }
}

// o = I_j v
template <bool PR = true, class MT, class R>
__device__ __forceinline__ void mvI(const MT& M, int j, const R v[6], R o[6]) {
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    R acc = 0.0;
#pragma unroll
    for (int k = 0; k < 6; ++k)
      if (nz<MT>(M->I[j][r * 6 + k])) acc = madd<PR>(acc, R(M->I[j][r * 6 + k]), v[k]);
    o[r] = acc;
  }
}

// crm(w) S_j for a 0/1 subspace vector S (mxS, RBDReference.py:57-62)
template <bool PR = true, class MT, class R>
__device__ __forceinline__ void crmS(const R w[6], const MT& M, int j, R o[6]) {
#define S_(i) R(M->S[j][i])
  if (!MT::STATIC) {
    o[0] = -w[2] * S_(1) + w[1] * S_(2);
    o[1] = w[2] * S_(0) - w[0] * S_(2);
    o[2] = -w[1] * S_(0) + w[0] * S_(1);
    o[3] = -w[5] * S_(1) + w[4] * S_(2) - w[2] * S_(4) + w[1] * S_(5);
    o[4] = w[5] * S_(0) - w[3] * S_(2) + w[2] * S_(3) - w[0] * S_(5);
    o[5] = -w[4] * S_(0) + w[3] * S_(1) - w[1] * S_(3) + w[0] * S_(4);
    return;
  }
  // S is a unit vector: each output has at most one term, and the products are exact
#define T_(acc, sign, wi, si) \
  if (S_(si) != 0.0) acc = madd<PR>(acc, mulz<PR>(R(sign), w[wi]), S_(si));
  R a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0, a4 = 0.0, a5 = 0.0;
  T_(a0, -1.0, 2, 1) T_(a0, 1.0, 1, 2)
  T_(a1, 1.0, 2, 0) T_(a1, -1.0, 0, 2)
  T_(a2, -1.0, 1, 0) T_(a2, 1.0, 0, 1)
  T_(a3, -1.0, 5, 1) T_(a3, 1.0, 4, 2) T_(a3, -1.0, 2, 4) T_(a3, 1.0, 1, 5)
  T_(a4, 1.0, 5, 0) T_(a4, -1.0, 3, 2) T_(a4, 1.0, 2, 3) T_(a4, -1.0, 0, 5)
  T_(a5, -1.0, 4, 0) T_(a5, 1.0, 3, 1) T_(a5, -1.0, 1, 3) T_(a5, 1.0, 0, 4)
#undef T_
#undef S_
  o[0] = a0; o[1] = a1; o[2] = a2; o[3] = a3; o[4] = a4; o[5] = a5;
}

// S_j . v
template <bool PR = true, class MT, class R>
__device__ __forceinline__ R dotS(const MT& M, int j, const R v[6]) {
  R acc = 0.0;
#pragma unroll
  for (int k = 0; k < 6; ++k)
    if (nz<MT>(M->S[j][k])) acc = madd<PR>(acc, R(M->S[j][k]), v[k]);
  return acc;
}

template <bool PR = true, class R>
__device__ __forceinline__ R dot6(const R a[6], const R b[6]) {
  R acc = 0.0;
#pragma unroll
  for (int k = 0; k < 6; ++k) acc = madd<PR>(acc, a[k], b[k]);
  return acc;
}

// o += fxv(f, t) = crf(f) t (RBDReference.py:71-91); vxIv(v, I) = fxv(v, I v) (:98-116)
template <bool PR = true, class R>
__device__ __forceinline__ void add_fxv(const R f[6], const R t[6], R o[6]) {
  if constexpr (!PR) {
    o[0] += -f[2] * t[1] + f[1] * t[2] - f[5] * t[4] + f[4] * t[5];
    o[1] += f[2] * t[0] - f[0] * t[2] + f[5] * t[3] - f[3] * t[5];
    o[2] += -f[1] * t[0] + f[0] * t[1] - f[4] * t[3] + f[3] * t[4];
    o[3] += -f[2] * t[4] + f[1] * t[5];
    o[4] += f[2] * t[3] - f[0] * t[5];
    o[5] += -f[1] * t[3] + f[0] * t[4];
    return;
  }
  // each row as clang contracts `o += a*b + c*d - ...`: the first product fused over the rounded
  // second, each later product fused onto the running sum, the total added to o
  R e;
  e = mulz<PR>(f[1], t[2]); e = madd<PR>(e, -f[2], t[1]); e = msub<PR>(e, f[5], t[4]); e = madd<PR>(e, f[4], t[5]);
  o[0] = addz<PR>(o[0], e);
  e = -mulz<PR>(f[0], t[2]); e = madd<PR>(e, f[2], t[0]); e = madd<PR>(e, f[5], t[3]); e = msub<PR>(e, f[3], t[5]);
  o[1] = addz<PR>(o[1], e);
  e = mulz<PR>(f[0], t[1]); e = madd<PR>(e, -f[1], t[0]); e = msub<PR>(e, f[4], t[3]); e = madd<PR>(e, f[3], t[4]);
  o[2] = addz<PR>(o[2], e);
  e = mulz<PR>(f[1], t[5]); e = madd<PR>(e, -f[2], t[4]);
  o[3] = addz<PR>(o[3], e);
  e = -mulz<PR>(f[0], t[5]); e = madd<PR>(e, f[2], t[3]);
  o[4] = addz<PR>(o[4], e);
  e = mulz<PR>(f[0], t[4]); e = madd<PR>(e, -f[1], t[3]);
  o[5] = addz<PR>(o[5], e);
}

// symmetric 6x6 upper-triangle storage
__device__ __forceinline__ constexpr int sidx(int r, int c) {
  return r <= c ? r * 6 - (r * (r - 1)) / 2 + (c - r) : c * 6 - (c * (c - 1)) / 2 + (r - c);
}

// column k of X_j (structural-zero mask in nzm)
template <class MT, class R>
__device__ __forceinline__ void Xcol(const MT& M, int j, R c, R s, int k, R x[6], bool nzm[6]) {
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    nzm[r] = xent(M, j, r * 6 + k, c, s, x[r]);
    if (!nzm[r]) x[r] = 0.0;
  }
}

// out = X^T A X for symmetric A (21 entries).  Column-at-a-time so that only
// two 6-vectors of X and one of A X are live (X columns are recomputed).
template <class MT, class R>
__device__ __forceinline__ void XtAX(const MT& M, int j, R c, R s, const R A[21], R out[21]) {
  opaque(c, s);
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    R xk[6], z[6];
    bool nk[6];
    Xcol(M, j, c, s, k, xk, nk);
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      R acc = 0.0;
#pragma unroll
      for (int m = 0; m < 6; ++m)
        if (nk[m]) acc = madd(acc, A[sidx(r, m)], xk[m]);
      z[r] = acc;
    }
#pragma unroll
    for (int r = 0; r <= k; ++r) {
      R xr[6];
      bool nr[6];
      if (r == k) {
#pragma unroll
        for (int m = 0; m < 6; ++m) {
          xr[m] = xk[m];
          nr[m] = nk[m];
        }
      } else {
        Xcol(M, j, c, s, r, xr, nr);
      }
      R acc = 0.0;
#pragma unroll
      for (int m = 0; m < 6; ++m)
        if (nr[m]) acc = madd(acc, xr[m], z[m]);
      out[sidx(r, k)] = acc;
    }
  }
}

// y1 = X v1, y2 = X v2 sharing the formation of each X row
template <class MT, class R>
__device__ __forceinline__ void mvX2(const MT& M, int j, R c, R s, const R v1[6], const R v2[6],
                                     R y1[6], R y2[6]) {
  opaque(c, s);
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    R a1 = 0.0, a2 = 0.0;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      R x;
      if (xent(M, j, r * 6 + k, c, s, x)) {
        a1 = madd(a1, x, v1[k]);
        a2 = madd(a2, x, v2[k]);
      }
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
template <int NJ, bool CHAIN, bool UNIT = false, class MT, class R>
__device__ __forceinline__ void fd_aba(const MT& M, const R cq[NJ], const R sq[NJ], const R qd[NJ],
                                       const R tau[NJ], R qdd[NJ]) {
  R v[NJ][6];
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
      for (int i = 0; i < 6; ++i)
        if (nz<MT>(M->S[j][i])) v[j][i] = madd(v[j][i], R(M->S[j][i]), qd[j]);
    }
  }
  // pass 2: articulated inertias / bias forces, leaf to root
  R chIA[NJ][21], chpA[NJ][6];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
#pragma unroll
    for (int e = 0; e < 21; ++e) chIA[j][e] = 0.0;
#pragma unroll
    for (int e = 0; e < 6; ++e) chpA[j][e] = 0.0;
  }
  R U[NJ][6], Dd[NJ], uu[NJ];
#pragma unroll
  for (int j = NJ - 1; j >= 0; --j) {
    R IA[21];
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
      for (int k = r; k < 6; ++k)
        IA[sidx(r, k)] = nz<MT>(M->I[j][r * 6 + k]) ? addz(R(M->I[j][r * 6 + k]), chIA[j][sidx(r, k)]) : chIA[j][sidx(r, k)];
    R pA[6], cj[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) pA[i] = chpA[j][i];
    if (!UNIT) {
      R Iv[6];
      mvI(M, j, v[j], Iv);
      add_fxv(v[j], Iv, pA);
      R cc[6];
      crmS(v[j], M, j, cc);
#pragma unroll
      for (int i = 0; i < 6; ++i) cj[i] = mulz(qd[j], cc[i]);
    } else {
#pragma unroll
      for (int i = 0; i < 6; ++i) cj[i] = 0.0;
    }
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      R acc = 0.0;
#pragma unroll
      for (int k = 0; k < 6; ++k)
        if (nz<MT>(M->S[j][k])) acc = madd(acc, IA[sidx(r, k)], R(M->S[j][k]));
      U[j][r] = acc;
    }
    Dd[j] = dotS(M, j, U[j]);
    uu[j] = tau[j] - dotS(M, j, pA);
    const int p = parent_of<CHAIN>(M, j);
    if (p >= 0) {
      const R dinv = R(1) / Dd[j];
#pragma unroll
      for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int k = r; k < 6; ++k) IA[sidx(r, k)] = msub(IA[sidx(r, k)], U[j][r], mulz(dinv, U[j][k]));   // Ia
      R pa[6];
      const R ud = uu[j] * dinv;
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        R acc = madd(pA[r], U[j][r], ud);
        if (!UNIT) {
#pragma unroll
          for (int k = 0; k < 6; ++k) acc = madd(acc, IA[sidx(r, k)], cj[k]);
        }
        pa[r] = acc;
      }
      R t[21];
      XtAX(M, j, cq[j], sq[j], IA, t);
#pragma unroll
      for (int e = 0; e < 21; ++e) chIA[p][e] = addz(chIA[p][e], t[e]);
      add_mtvX(M, j, cq[j], sq[j], pa, chpA[p]);
    }
  }
  // pass 3: accelerations, root to leaf (velocities recomputed)
  R v3[NJ][6], a[NJ][6];
  const R g[6] = {0.0, 0.0, 0.0, 0.0, 0.0, UNIT ? R(0) : -R(M->gravity)};
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
      for (int i = 0; i < 6; ++i)
        if (nz<MT>(M->S[j][i])) v3[j][i] = madd(v3[j][i], R(M->S[j][i]), qd[j]);
      R cc[6];
      crmS(v3[j], M, j, cc);
#pragma unroll
      for (int i = 0; i < 6; ++i) a[j][i] = madd(a[j][i], qd[j], cc[i]);
    }
    qdd[j] = (uu[j] - dot6(U[j], a[j])) / Dd[j];
#pragma unroll
    for (int i = 0; i < 6; ++i)
      if (nz<MT>(M->S[j][i])) a[j][i] = madd(a[j][i], R(M->S[j][i]), qdd[j]);
  }
}

// ----------------------------------------------------------------- analytic M^-1, one column
// Computes Minv[r][col] for r <= col (the upper triangle the reference fills
// before symmetrising, :908-930) following minv_bpass / minv_fpass
// restricted to column `col` (F[:, :, col] is per column; IA, U, Dinv are
// recomputed per lane).
template <int NJ, bool CHAIN, class MT, class R>
__device__ __forceinline__ void minv_column(const MT& M, const R cq[NJ], const R sq[NJ], int col,
                                            R mcol[NJ]) {
  R chIA[NJ][21];
  R Fc[NJ][6];      // F[j][:, col]
  R U[NJ][6], Dinv[NJ];
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
    R IA[21];
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
      for (int k = r; k < 6; ++k)
        IA[sidx(r, k)] = nz<MT>(M->I[j][r * 6 + k]) ? addz(R(M->I[j][r * 6 + k]), chIA[j][sidx(r, k)]) : chIA[j][sidx(r, k)];
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      R acc = 0.0;
#pragma unroll
      for (int k = 0; k < 6; ++k)
        if (nz<MT>(M->S[j][k])) acc = madd(acc, IA[sidx(r, k)], R(M->S[j][k]));
      U[j][r] = acc;
    }
    Dinv[j] = R(1) / dotS(M, j, U[j]);
    const bool mine = in_subtree<CHAIN>(M, j, col);
    if (j == col) mcol[j] = Dinv[j];
    if (mine) mcol[j] -= Dinv[j] * dotS(M, j, Fc[j]);
    const int p = parent_of<CHAIN>(M, j);
    if (p >= 0) {
      if (mine) {
#pragma unroll
        for (int r = 0; r < 6; ++r) Fc[j][r] += U[j][r] * mcol[j];
        add_mtvX(M, j, cq[j], sq[j], Fc[j], Fc[p]);
      }
      R Ia[21];
#pragma unroll
      for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int k = r; k < 6; ++k) Ia[sidx(r, k)] = IA[sidx(r, k)] - U[j][r] * (Dinv[j] * U[j][k]);
      R t[21];
      XtAX(M, j, cq[j], sq[j], Ia, t);
#pragma unroll
      for (int e = 0; e < 21; ++e) chIA[p][e] = addz(chIA[p][e], t[e]);
    }
  }
  // forward pass (:868-906), rows j <= col
  R Ff[NJ][6];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    if (j > col) break;
    const int p = parent_of<CHAIN>(M, j);
    if (p >= 0) {
      R XF[6];
      mvX(M, j, cq[j], sq[j], Ff[p], XF);   // X F[p][:, col]
      // (U^T X) F[p][:, col] == U^T (X F[p][:, col])
      mcol[j] -= Dinv[j] * dot6(U[j], XF);
#pragma unroll
      for (int r = 0; r < 6; ++r) Ff[j][r] = nz<MT>(M->S[j][r]) ? R(M->S[j][r]) * mcol[j] + XF[r] : XF[r];
    } else {
#pragma unroll
      for (int r = 0; r < 6; ++r) Ff[j][r] = nz<MT>(M->S[j][r]) ? R(M->S[j][r]) * mcol[j] : 0.0;
    }
  }
}

// ----------------------------------------------------------------- one derivative column
// d c / d q_col (colqd = false) or d c / d qd_col (colqd = true) at (q, qd, qdd):
// rnea_grad forward passes (:561-690) and backward passes (:692-771) for ONE
// column, fused with the RNEA passes that produce v, a and the accumulated f.
template <int NJ, bool CHAIN, class MT, class R>
__device__ __forceinline__ void rnea_grad_column(const MT& M, const R cq[NJ], const R sq[NJ],
                                                 const R qd[NJ], const R qdd[NJ], int col, bool colqd,
                                                 R dc[NJ]) {
  R v[NJ][6], a[NJ][6], f[NJ][6];
  R dv[NJ][6], da[NJ][6], df[NJ][6];
  const R g[6] = {0.0, 0.0, 0.0, 0.0, 0.0, -R(M->gravity)};
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int p = parent_of<CHAIN>(M, j);
    // ---- RNEA forward (with qdd)
    R Xvp[6], Xap[6];
    if (p < 0) {
#pragma unroll
      for (int i = 0; i < 6; ++i) Xvp[i] = 0.0;
      mvX<false>(M, j, cq[j], sq[j], g, Xap);
    } else {
      mvX<false>(M, j, cq[j], sq[j], v[p], Xvp);
      mvX<false>(M, j, cq[j], sq[j], a[p], Xap);
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) v[j][i] = nz<MT>(M->S[j][i]) ? Xvp[i] + R(M->S[j][i]) * qd[j] : Xvp[i];
    {
      R cc[6];
      crmS<false>(v[j], M, j, cc);
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        R t = Xap[i] + qd[j] * cc[i];
        if (nz<MT>(M->S[j][i])) t += R(M->S[j][i]) * qdd[j];
        a[j][i] = t;
      }
    }
    R Iv[6];
    mvI<false>(M, j, a[j], f[j]);
    mvI<false>(M, j, v[j], Iv);
    add_fxv<false>(v[j], Iv, f[j]);
    // ---- derivative forward pass for this column
    if (p >= 0) {
      mvX<false>(M, j, cq[j], sq[j], dv[p], dv[j]);
      mvX<false>(M, j, cq[j], sq[j], da[p], da[j]);
    } else {
#pragma unroll
      for (int i = 0; i < 6; ++i) { dv[j][i] = 0.0; da[j][i] = 0.0; }
    }
    if (j == col) {
      if (!colqd) {
        if (p >= 0) {
          R cc[6];
          crmS<false>(Xvp, M, j, cc);
#pragma unroll
          for (int i = 0; i < 6; ++i) dv[j][i] += cc[i];
        }
      } else {
#pragma unroll
        for (int i = 0; i < 6; ++i)
          if (nz<MT>(M->S[j][i])) dv[j][i] += R(M->S[j][i]);
      }
    }
    {
      R cc[6];
      crmS<false>(dv[j], M, j, cc);
#pragma unroll
      for (int i = 0; i < 6; ++i) da[j][i] += qd[j] * cc[i];
    }
    if (j == col) {
      R cc[6];
      crmS<false>(colqd ? v[j] : Xap, M, j, cc);  // mxS(S, v) or mxS(S, X a_parent) / mxS(S, X g)
#pragma unroll
      for (int i = 0; i < 6; ++i) da[j][i] += cc[i];
    }
    mvI<false>(M, j, da[j], df[j]);
    add_fxv<false>(dv[j], Iv, df[j]);
    R Idv[6];
    mvI<false>(M, j, dv[j], Idv);
    add_fxv<false>(v[j], Idv, df[j]);
  }
  // ---- fused backward passes
#pragma unroll
  for (int j = NJ - 1; j >= 0; --j) {
    dc[j] = dotS<false>(M, j, df[j]);
    const int p = parent_of<CHAIN>(M, j);
    if (p >= 0) {
      add_mtvX<false>(M, j, cq[j], sq[j], df[j], df[p]);
      if (!colqd && j == col) {
        // delta = X^T fxS(S, f) = -X^T (crm(f) S)
        R cc[6];
        crmS<false>(f[j], M, j, cc);
#pragma unroll
        for (int i = 0; i < 6; ++i) cc[i] = -cc[i];
        add_mtvX<false>(M, j, cq[j], sq[j], cc, df[p]);
      }
      add_mtvX<false>(M, j, cq[j], sq[j], f[j], f[p]);
    }
  }
}

}  // namespace tmpc
