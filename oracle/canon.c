/* ORACLE -- test infrastructure, not product code (see oracle/__init__.py).
 *
 * PCG.pcg / PCG.compute_preconditioner (GBD-PCG-Python/PCG.py:66-111, :166-212) on a
 * block-tridiagonal S, restated in ONE canonical operation order: the order of the GPU's
 * fused QP kernel (k_qp / k_pcg, csrc/tmpc_kernels.hip pcg_precondition / pcg_run, one row of S
 * per lane), so that on the same S and gamma the iteration count and lambda agree bit for bit.
 * Compiled with -ffp-contract=off: every fused multiply-add below is an explicit fma() (the
 * kernel's contracted updates), every other product and sum is rounded on its own.
 *
 *   preconditioner  J:  1 / S_ii;  BJ / SS: (S_kk)^-1 by in-place Gauss-Jordan without pivoting,
 *                   pivot row scaled by 1 / d (its own entry), the others a_j - f * pv_j (fma);
 *   S v             per row three chains over j (S_{k,k-1}, S_kk, S_{k,k+1} against v_{k-1}, v_k,
 *                   v_{k+1}), each fma(s_j, v_j, acc) from +0, summed (a0 + a1) + a2;
 *   P_kk v          two chains over even / odd j, a0 + a1;
 *   SS P^-1 r       w = P_kk r_k;  t = r - (S_{k,k-1} w_{k-1} + S_{k,k+1} w_{k+1}) (two chains);
 *                   z = P_kk t_k;  nu' = w . t  (= r^T P^-1 r for the symmetric stair);
 *   dot products    per row fma(a_i, b_i, +0), then a pairwise tree over 1024 leaves in row order
 *                   (zero-padded): the wave's DPP / permlane butterfly and the 16-slot fan-in;
 *   updates         r - Ap alpha, x + p alpha, z + p beta as one fma each.
 * Rows per lane: one (N nx <= 768, the only layout this restatement covers).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

enum { PRE_J = 1, PRE_BJ = 2, PRE_SS = 3, PRE_0 = 4 };
#define LEAVES 1024

static double tree_dot(const double* a, const double* b, int n, double* buf) {
  for (int i = 0; i < LEAVES; ++i) buf[i] = i < n ? fma(a[i], b[i], 0.0) : 0.0;
  for (int len = LEAVES; len > 1; len /= 2)
    for (int i = 0; i < len / 2; ++i) buf[i] = buf[2 * i] + buf[2 * i + 1];
  return buf[0];
}

/* S_{k,k+1}[i][j] = S_{k+1,k}[j][i] (the kernel's rows are these bits: same products, same order) */
static inline double s_up(const double* Sl, int nx, int k, int i, int j) { return Sl[((size_t)k * nx + j) * nx + i]; }
static inline double s_lo(const double* Sl, int nx, int k, int i, int j) { return Sl[((size_t)(k - 1) * nx + i) * nx + j]; }

/* w = P_kk v_k for every block (two chains) */
static void block_dot(const double* Pd, const double* v, int N, int nx, double* out) {
  for (int k = 0; k < N; ++k)
    for (int i = 0; i < nx; ++i) {
      const double* pr = Pd + ((size_t)k * nx + i) * nx;
      double a0 = 0.0, a1 = 0.0;
      for (int j = 0; j < nx; ++j) {
        if (j % 2 == 0) a0 = fma(pr[j], v[k * nx + j], a0);
        else a1 = fma(pr[j], v[k * nx + j], a1);
      }
      out[k * nx + i] = nx > 1 ? a0 + a1 : a0;
    }
}

static void spmv(const double* Sd, const double* Sl, const double* v, int N, int nx, double* out) {
  for (int k = 0; k < N; ++k)
    for (int i = 0; i < nx; ++i) {
      double a0 = 0.0, a1 = 0.0, a2 = 0.0;
      for (int j = 0; j < nx; ++j) {
        const double sl = k > 0 ? s_lo(Sl, nx, k, i, j) : 0.0, pm = k > 0 ? v[(k - 1) * nx + j] : 0.0;
        const double su = k < N - 1 ? s_up(Sl, nx, k, i, j) : 0.0, pp = k < N - 1 ? v[(k + 1) * nx + j] : 0.0;
        a0 = fma(sl, pm, a0);
        a1 = fma(Sd[((size_t)k * nx + i) * nx + j], v[k * nx + j], a1);
        a2 = fma(su, pp, a2);
      }
      out[k * nx + i] = (a0 + a1) + a2;
    }
}

/* t = r - (S_{k,k-1} w_{k-1} + S_{k,k+1} w_{k+1}) */
static void off(const double* Sl, const double* w, const double* r, int N, int nx, double* t) {
  for (int k = 0; k < N; ++k)
    for (int i = 0; i < nx; ++i) {
      double a0 = 0.0, a1 = 0.0;
      for (int j = 0; j < nx; ++j) {
        const double sl = k > 0 ? s_lo(Sl, nx, k, i, j) : 0.0, wl = k > 0 ? w[(k - 1) * nx + j] : 0.0;
        const double su = k < N - 1 ? s_up(Sl, nx, k, i, j) : 0.0, wu = k < N - 1 ? w[(k + 1) * nx + j] : 0.0;
        a0 = fma(sl, wl, a0);
        a1 = fma(su, wu, a1);
      }
      t[k * nx + i] = r[k * nx + i] - (a0 + a1);
    }
}

/* (S_kk)^-1 of every block by the kernel's in-place Gauss-Jordan (pcg_precondition) */
int canon_block_inverse(int N, int nx, const double* Sd, double* Pd) {
  double* pv = malloc(sizeof(double) * nx);
  if (!pv) return -1;
  for (int k = 0; k < N; ++k) {
    double* a = Pd + (size_t)k * nx * nx;
    memcpy(a, Sd + (size_t)k * nx * nx, sizeof(double) * nx * nx);
    for (int p = 0; p < nx; ++p) {
      double* ap = a + (size_t)p * nx;
      const double d = ap[p];
      for (int j = 0; j < nx; ++j) {
        ap[j] = (j == p) ? 1.0 / d : ap[j] / d;
        pv[j] = ap[j];
      }
      for (int i = 0; i < nx; ++i) {
        if (i == p) continue;
        double* ai = a + (size_t)i * nx;
        const double f = ai[p];
        ai[p] = 0.0;
        for (int j = 0; j < nx; ++j) ai[j] = fma(-f, pv[j], ai[j]);
      }
    }
  }
  free(pv);
  return 0;
}

/* PCG with x0 = 0; returns the iteration count (PCG.py:97: exit when |nu'| < tol), lambda in x,
 * |nu| per iteration in trace_nu (max_iter + 1 entries, nullable) */
int canon_pcg(int N, int nx, int precond, const double* Sd, const double* Sl, const double* b, double tol,
              int max_iter, double* x, double* trace_nu) {
  const int n = N * nx;
  if (n > 768 || n < 1) return -1;
  double* Pd = malloc(sizeof(double) * (size_t)N * nx * nx);
  double* pj = malloc(sizeof(double) * n);
  double* r = malloc(sizeof(double) * n);
  double* z = malloc(sizeof(double) * n);
  double* p = malloc(sizeof(double) * n);
  double* ap = malloc(sizeof(double) * n);
  double* w = malloc(sizeof(double) * n);
  double* t = malloc(sizeof(double) * n);
  double* buf = malloc(sizeof(double) * LEAVES);
  if (!Pd || !pj || !r || !z || !p || !ap || !w || !t || !buf) return -2;
  if (precond == PRE_BJ || precond == PRE_SS) canon_block_inverse(N, nx, Sd, Pd);
  if (precond == PRE_J)
    for (int k = 0; k < N; ++k)
      for (int i = 0; i < nx; ++i) pj[k * nx + i] = 1.0 / Sd[((size_t)k * nx + i) * nx + i];
  for (int i = 0; i < n; ++i) {
    x[i] = 0.0;
    r[i] = b[i];
  }
  double nu;
  /* z = P^-1 r, nu = r . z */
  if (precond == PRE_SS) {
    block_dot(Pd, r, N, nx, w);
    off(Sl, w, r, N, nx, t);
    nu = tree_dot(w, t, n, buf);
    block_dot(Pd, t, N, nx, z);
  } else {
    if (precond == PRE_BJ) block_dot(Pd, r, N, nx, z);
    for (int i = 0; i < n; ++i)
      if (precond == PRE_J) z[i] = pj[i] * r[i];
      else if (precond == PRE_0) z[i] = r[i];
    nu = tree_dot(r, z, n, buf);
  }
  memcpy(p, z, sizeof(double) * n);
  if (trace_nu) trace_nu[0] = fabs(nu);
  int it_done = max_iter;
  for (int it = 0; it < max_iter; ++it) {
    spmv(Sd, Sl, p, N, nx, ap);
    const double alpha = nu / tree_dot(p, ap, n, buf);
    if (precond == PRE_BJ || precond == PRE_SS) {
      /* every lane rebuilds its block's new r from the old r and Ap (the same fma), then w = P_kk r_k */
      for (int i = 0; i < n; ++i) r[i] = fma(-ap[i], alpha, r[i]);
      block_dot(Pd, r, N, nx, w);
    } else {
      for (int i = 0; i < n; ++i) r[i] = fma(-ap[i], alpha, r[i]);
    }
    for (int i = 0; i < n; ++i) x[i] = fma(p[i], alpha, x[i]);
    double nup;
    if (precond == PRE_SS) {
      off(Sl, w, r, N, nx, t);
      nup = tree_dot(w, t, n, buf);
      block_dot(Pd, t, N, nx, z);
    } else {
      for (int i = 0; i < n; ++i) z[i] = precond == PRE_BJ ? w[i] : (precond == PRE_J ? pj[i] * r[i] : r[i]);
      nup = tree_dot(r, z, n, buf);
    }
    if (trace_nu) trace_nu[it + 1] = fabs(nup);
    if (fabs(nup) < tol) {
      it_done = it + 1;
      break;
    }
    const double beta = nup / nu;
    for (int i = 0; i < n; ++i) p[i] = fma(p[i], beta, z[i]);
    nu = nup;
  }
  free(Pd); free(pj); free(r); free(z); free(p); free(ap); free(w); free(t); free(buf);
  return it_done;
}
