/* ORACLE -- test infrastructure, not product code (see oracle/__init__.py).
 *
 * PCG.pcg / PCG.compute_preconditioner (GBD-PCG-Python/PCG.py:66-111, :166-212) on a
 * block-tridiagonal S, restated in ONE canonical operation order: the order of the GPU's
 * fused QP kernel (k_qp / k_pcg, csrc/tmpc_kernels.hip pcg_precondition / pcg_run), so that on
 * the same S and gamma the iteration count and lambda agree bit for bit.
 * Compiled with -ffp-contract=off: every fused multiply-add below is an explicit fma() (the
 * kernel's contracted updates), every other product and sum is rounded on its own.
 *
 * The kernel has two lane layouts (rpl = rows of S per lane):
 *   rpl 1  lane t = row t                                  (register instance, <= 768 rows);
 *   rpl 2  lane t = rows k nx + i and k nx + i + nx/2 of block k = t / (nx/2), i = t mod (nx/2)
 *          (register instance for 769..1024 rows; the GM instance -- rows of S in HBM -- at every
 *          size it runs, 1025..1536 rows and wherever TMPC_QP_GM_MIN_ROWS forces it).
 * The layouts differ in the accumulation chains and in the leaves of the dot-product tree:
 *
 *   preconditioner  J:  1 / S_ii;  BJ / SS: (S_kk)^-1 by in-place Gauss-Jordan without pivoting,
 *                   pivot row scaled by 1 / d (its own entry), the others a_j - f * pv_j (fma);
 *   S v             rpl 1: per row three chains over j (S_{k,k-1}, S_kk, S_{k,k+1} against v_{k-1},
 *                   v_k, v_{k+1}), each fma(s_j, v_j, acc) from +0, summed (a0 + a1) + a2;
 *                   rpl 2: one chain, for each j the three fma in the order S_{k,k-1}, S_kk, S_{k,k+1};
 *   P_kk v          rpl 1: two chains over even / odd j, a0 + a1;  rpl 2: one chain;
 *   SS P^-1 r       w = P_kk r_k;  t = r - (S_{k,k-1} w_{k-1} + S_{k,k+1} w_{k+1})
 *                   (rpl 1: two chains, a0 + a1; rpl 2: one chain, for each j S_{k,k-1} then S_{k,k+1});
 *                   z = P_kk t_k;  nu' = w . t  (= r^T P^-1 r for the symmetric stair);
 *   dot products    per lane fma over its rows from +0 (rpl 2: row i, then row i + nx/2), then a
 *                   pairwise tree over 1024 leaves in lane order (zero-padded): the wave's DPP /
 *                   permlane butterfly and the 16-slot fan-in;
 *   updates         r - Ap alpha, x + p alpha, z + p beta as one fma each;
 *   warm start      x0 = guess, r = b - S x0 (a plain difference), PCG.py:11-12,76.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

enum { PRE_J = 1, PRE_BJ = 2, PRE_SS = 3, PRE_0 = 4 };
#define LEAVES 1024

/* lane geometry: row of S held by lane t's slot m */
typedef struct {
  int N, nx, rpl, L, lanes;
} Geo;

static inline int geo_row(const Geo* g, int t, int m) {
  if (g->rpl == 1) return t;
  const int k = t / g->L, i = t - k * g->L;
  return k * g->nx + i + m * g->L;
}

static double tree_dot(const Geo* g, const double* a, const double* b, double* buf) {
  for (int t = 0; t < LEAVES; ++t) {
    double s = 0.0;
    if (t < g->lanes)
      for (int m = 0; m < g->rpl; ++m) {
        const int r = geo_row(g, t, m);
        s = fma(a[r], b[r], s);
      }
    buf[t] = s;
  }
  for (int len = LEAVES; len > 1; len /= 2)
    for (int i = 0; i < len / 2; ++i) buf[i] = buf[2 * i] + buf[2 * i + 1];
  return buf[0];
}

/* S_{k,k+1}[i][j] = S_{k+1,k}[j][i] (the kernel's rows are these bits: same products, same order);
 * entries outside the band read 0, as the kernel's zero rows and zero vector pads */
static inline double s_up(const double* Sl, int N, int nx, int k, int i, int j) {
  return k < N - 1 ? Sl[((size_t)k * nx + j) * nx + i] : 0.0;
}
static inline double s_lo(const double* Sl, int nx, int k, int i, int j) {
  return k > 0 ? Sl[((size_t)(k - 1) * nx + i) * nx + j] : 0.0;
}
static inline double v_at(const double* v, int N, int nx, int k, int j) {
  return (k >= 0 && k < N) ? v[k * nx + j] : 0.0;
}

/* w = P_kk v_k for every block */
static void block_dot(const Geo* g, const double* Pd, const double* v, double* out) {
  const int N = g->N, nx = g->nx;
  for (int k = 0; k < N; ++k)
    for (int i = 0; i < nx; ++i) {
      const double* pr = Pd + ((size_t)k * nx + i) * nx;
      double a0 = 0.0, a1 = 0.0;
      for (int j = 0; j < nx; ++j) {
        if (g->rpl == 2 || j % 2 == 0) a0 = fma(pr[j], v[k * nx + j], a0);
        else a1 = fma(pr[j], v[k * nx + j], a1);
      }
      out[k * nx + i] = (g->rpl == 1 && nx > 1) ? a0 + a1 : a0;
    }
}

static void spmv(const Geo* g, const double* Sd, const double* Sl, const double* v, double* out) {
  const int N = g->N, nx = g->nx;
  for (int k = 0; k < N; ++k)
    for (int i = 0; i < nx; ++i) {
      double a0 = 0.0, a1 = 0.0, a2 = 0.0;
      for (int j = 0; j < nx; ++j) {
        const double sl = s_lo(Sl, nx, k, i, j), pm = v_at(v, N, nx, k - 1, j);
        const double sd = Sd[((size_t)k * nx + i) * nx + j], pc = v[k * nx + j];
        const double su = s_up(Sl, N, nx, k, i, j), pp = v_at(v, N, nx, k + 1, j);
        if (g->rpl == 1) {
          a0 = fma(sl, pm, a0);
          a1 = fma(sd, pc, a1);
          a2 = fma(su, pp, a2);
        } else {
          a0 = fma(sl, pm, a0);
          a0 = fma(sd, pc, a0);
          a0 = fma(su, pp, a0);
        }
      }
      out[k * nx + i] = g->rpl == 1 ? (a0 + a1) + a2 : a0;
    }
}

/* t = r - (S_{k,k-1} w_{k-1} + S_{k,k+1} w_{k+1}) */
static void off(const Geo* g, const double* Sl, const double* w, const double* r, double* t) {
  const int N = g->N, nx = g->nx;
  for (int k = 0; k < N; ++k)
    for (int i = 0; i < nx; ++i) {
      double a0 = 0.0, a1 = 0.0;
      for (int j = 0; j < nx; ++j) {
        const double sl = s_lo(Sl, nx, k, i, j), wl = v_at(w, N, nx, k - 1, j);
        const double su = s_up(Sl, N, nx, k, i, j), wu = v_at(w, N, nx, k + 1, j);
        if (g->rpl == 1) {
          a0 = fma(sl, wl, a0);
          a1 = fma(su, wu, a1);
        } else {
          a0 = fma(sl, wl, a0);
          a0 = fma(su, wu, a0);
        }
      }
      t[k * nx + i] = r[k * nx + i] - (g->rpl == 1 ? a0 + a1 : a0);
    }
}

/* (S_kk)^-1 of every block by the kernel's in-place Gauss-Jordan (pcg_precondition; the same
 * arithmetic in both lane layouts) */
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

/* PCG from x0 = guess (null: zeros) in lane layout rpl; returns the iteration count (PCG.py:97:
 * exit when |nu'| < tol), lambda in x, |nu| per iteration in trace_nu (max_iter + 1 entries,
 * nullable).  -1: a size the layout does not cover (more than 1024 lanes, odd nx with rpl 2). */
int canon_pcg_rpl(int N, int nx, int precond, int rpl, const double* Sd, const double* Sl, const double* b,
                  const double* guess, double tol, int max_iter, double* x, double* trace_nu) {
  const int n = N * nx;
  if (n < 1 || (rpl != 1 && rpl != 2) || (rpl == 2 && (nx & 1)) || n / rpl > LEAVES) return -1;
  const Geo g = {N, nx, rpl, nx / rpl, n / rpl};
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
    x[i] = guess ? guess[i] : 0.0;
    r[i] = b[i];
  }
  if (guess) {
    spmv(&g, Sd, Sl, x, ap);
    for (int i = 0; i < n; ++i) r[i] = b[i] - ap[i];
  }
  double nu;
  /* z = P^-1 r, nu = r . z */
  if (precond == PRE_SS) {
    block_dot(&g, Pd, r, w);
    off(&g, Sl, w, r, t);
    nu = tree_dot(&g, w, t, buf);
    block_dot(&g, Pd, t, z);
  } else {
    if (precond == PRE_BJ) block_dot(&g, Pd, r, z);
    for (int i = 0; i < n; ++i)
      if (precond == PRE_J) z[i] = pj[i] * r[i];
      else if (precond == PRE_0) z[i] = r[i];
    nu = tree_dot(&g, r, z, buf);
  }
  memcpy(p, z, sizeof(double) * n);
  if (trace_nu) trace_nu[0] = fabs(nu);
  int it_done = max_iter;
  for (int it = 0; it < max_iter; ++it) {
    spmv(&g, Sd, Sl, p, ap);
    const double alpha = nu / tree_dot(&g, p, ap, buf);
    /* BJ / SS: every lane rebuilds its block's new r from the old r and Ap (the same fma), then
     * w = P_kk r_k */
    for (int i = 0; i < n; ++i) r[i] = fma(-ap[i], alpha, r[i]);
    if (precond == PRE_BJ || precond == PRE_SS) block_dot(&g, Pd, r, w);
    for (int i = 0; i < n; ++i) x[i] = fma(p[i], alpha, x[i]);
    double nup;
    if (precond == PRE_SS) {
      off(&g, Sl, w, r, t);
      nup = tree_dot(&g, w, t, buf);
      block_dot(&g, Pd, t, z);
    } else {
      for (int i = 0; i < n; ++i) z[i] = precond == PRE_BJ ? w[i] : (precond == PRE_J ? pj[i] * r[i] : r[i]);
      nup = tree_dot(&g, r, z, buf);
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

/* the one-row-per-lane layout from zeros (the round-4 entry point, <= 768 rows) */
int canon_pcg(int N, int nx, int precond, const double* Sd, const double* Sl, const double* b, double tol,
              int max_iter, double* x, double* trace_nu) {
  if (N * nx > 768) return -1;
  return canon_pcg_rpl(N, nx, precond, 1, Sd, Sl, b, NULL, tol, max_iter, x, trace_nu);
}
