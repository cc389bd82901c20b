// The QP of solveKKTSystem_Schur (TrajoptMPCReference.py:361-455) on blocks the caller formed with
// its own plugin hooks: formKKTSystemBlocks (:118-271) evaluated by a TrajoptCost / TrajoptPlant
// subclass on the host -- per knot the cost Hessian G_k (n x n with n = nx + nu, the x-u coupling
// included; terminal nx x nx) and gradient g_k, the integrator's A_k, B_k and the defect c_k.  This is
// the plugin-hook path of the drop-in (solver.py _sqp_hooks): the built-in plugins never take it
// (their blocks are formed on the device, tmpc_kernels.hip k_qp), and the PCG is the same code
// (tmpc_pcg.h, restated by oracle/canon.c), so its counts are the fused kernel's.
//
//   k_ghat_full   (G_k + rho I)^-1 per (problem, knot): one wave per matrix, row r on lane r,
//                 Gauss-Jordan with partial pivoting (a non-convex plugin cost makes G + rho I indefinite;
//                 an exactly singular one -- np.linalg.inv's LinAlgError -- sets the problem's error flag);
//   k_qp_blocks   one workgroup per problem, one row of S per lane (the fused kernel's geometry):
//                 prologue S_kk, S_{k,k-1}, S_{k,k+1}, gamma_k from the full blocks Ghat_k
//                   S_kk = -(AB_{k-1} Ghat_{k-1} AB_{k-1}^T + E Ghat_k E^T),  S_{k,k-1} = AB_{k-1} Ghat_{k-1} E^T,
//                   gamma_k = c_k + AB_{k-1} Ghat_{k-1} g_{k-1} - E Ghat_k g_k   (AB = [A B], E = [I 0]);
//                 PCG (PCG-J / BJ / SS / 0) or, for methods S / N, the Schur blocks out for k_btsolve;
//                 epilogue dxu_k = Ghat_k (g_k - (C^T lambda)_k).
// Layouts (per problem b): G, Ghat [B][N][n][n] (knot N-1: its nx x nx block in the top-left corner),
// g [B][N][n], A [B][N-1][nx][nx], Bm [B][N-1][nx][nu], c [B][N][nx]; dx [B][N][nx], du [B][N-1][nu].
#include "tmpc_pcg.h"

namespace tmpc {

__device__ __forceinline__ double hk_readlane(double v, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}

// one 64-lane wave per (problem, knot); MAXN >= n.  Gauss-Jordan with partial pivoting, as np.linalg.inv's
// LU (LAPACK getrf: the largest |entry| of the pivot column, the first such row on a tie): at step p the
// row with the largest |a_rp| among rows p..m-1 is swapped into place (the two lanes trade rows), and the
// in-place inverse of the row-permuted matrix is unscrambled by swapping its columns back in reverse order
// (the inverse of P A is A^-1 P^-1).  A zero or non-finite pivot -- an exactly singular G + rho I, where
// np.linalg.inv raises LinAlgError -- sets the problem's error flag.
template <int MAXN>
__global__ void __launch_bounds__(64) k_ghat_full(int B, int N, int nx, int nu, const double* __restrict__ G,
                                                  const double* __restrict__ rho, double* __restrict__ Ghat,
                                                  int* __restrict__ err) {
  const int n = nx + nu;
  const int mat = blockIdx.x;
  if (mat >= B * N) return;
  const int b = mat / N, k = mat - b * N;
  const int m = k == N - 1 ? nx : n;   // the terminal block is nx x nx
  const int r = threadIdx.x;
  const double* src = G + (size_t)mat * n * n;
  const double rh = rho[b];
  double a[MAXN];
#pragma unroll
  for (int c = 0; c < MAXN; ++c)
    a[c] = (r < m && c < m) ? src[r * n + c] + (r == c ? rh : 0.0) : (r == c ? 1.0 : 0.0);
  __shared__ int perm[MAXN];   // the row swapped with row p at step p (one wave: written, then read, by it)
  bool bad = false;
  for (int p = 0; p < m; ++p) {
    // pivot search over rows p..m-1 of column p (lane order breaks ties: the first row, as getrf's idamax)
    double ap = 0.0;
#pragma unroll
    for (int c = 0; c < MAXN; ++c)
      if (c == p) ap = a[c];
    double best = (r >= p && r < m) ? fabs(ap) : -1.0;
    int q = r;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      const double ob = __shfl_xor(best, off);
      const int oq = __shfl_xor(q, off);
      if (ob > best || (ob == best && oq < q)) {
        best = ob;
        q = oq;
      }
    }
    q = __builtin_amdgcn_readfirstlane(q);
    if (r == 0) perm[p] = q;
    if (q != p) {   // lanes p and q trade rows
#pragma unroll
      for (int c = 0; c < MAXN; ++c) {
        const double vp = hk_readlane(a[c], p), vq = hk_readlane(a[c], q);
        if (r == p) a[c] = vq;
        else if (r == q) a[c] = vp;
      }
    }
    double pr[MAXN];
#pragma unroll
    for (int c = 0; c < MAXN; ++c) pr[c] = hk_readlane(a[c], p);
    const double d = pr[p];
    if (!(d != 0.0) || !isfinite(d)) bad = true;   // wave-uniform
    const double rp = 1.0 / d;
#pragma unroll
    for (int c = 0; c < MAXN; ++c) pr[c] *= rp;
    double f = 0.0;
#pragma unroll
    for (int c = 0; c < MAXN; ++c)
      if (c == p) f = a[c];
    if (r == p) {
#pragma unroll
      for (int c = 0; c < MAXN; ++c) a[c] = c == p ? rp : pr[c];
    } else {
#pragma unroll
      for (int c = 0; c < MAXN; ++c) a[c] = c == p ? -f * rp : fma(-f, pr[c], a[c]);
    }
  }
  __syncthreads();
  for (int p = m - 1; p >= 0; --p) {   // unscramble: columns p and perm[p], in reverse order
    const int q = __builtin_amdgcn_readfirstlane(perm[p]);
    if (q == p) continue;
    double vp = 0.0, vq = 0.0;
#pragma unroll
    for (int c = 0; c < MAXN; ++c) {
      if (c == p) vp = a[c];
      if (c == q) vq = a[c];
    }
#pragma unroll
    for (int c = 0; c < MAXN; ++c) {
      if (c == p) a[c] = vq;
      else if (c == q) a[c] = vp;
    }
  }
  double* out = Ghat + (size_t)mat * n * n;
  if (r < n) {
#pragma unroll
    for (int c = 0; c < MAXN; ++c)
      if (c < n) out[r * n + c] = (r < m && c < m) ? a[c] : 0.0;
  }
  if (bad && r == 0) err[b] = 1;
}

// LDS of k_qp_blocks: [PCG buffers | g (N n) | lambda (N NX) | C^T lambda x (N NX), u (K NU)]
__host__ __device__ inline size_t qpb_lds_doubles(int N, int NX, int NU) {
  return pcg_lds_doubles(N, NX, 1024) + (size_t)N * (NX + NU) + 2 * (size_t)N * NX + (size_t)(N - 1) * NU;
}

template <int NJ, int RPL, int MAXT, int MODE>
__global__ void __launch_bounds__(MAXT) k_qp_blocks(int B, int N, int precond, const double* __restrict__ Ghat,
                                                    const double* __restrict__ gv, const double* __restrict__ Aall,
                                                    const double* __restrict__ Ball,
                                                    const double* __restrict__ cvec, const int* __restrict__ err,
                                                    double tol, int max_iter, const double* __restrict__ guess,
                                                    int* __restrict__ iters, double* __restrict__ dx,
                                                    double* __restrict__ du, double* __restrict__ lam_io,
                                                    double* __restrict__ Sd_out, double* __restrict__ Sl_out,
                                                    double* __restrict__ gam_out) {
  constexpr int NX = 2 * NJ, NU = NJ, NN = NX + NU;
  const int b = blockIdx.x;
  if (b >= B || err[b]) return;   // workgroup-uniform
  extern __shared__ __align__(16) double lds[];
  const int K = N - 1, rows = N * NX;
  const PcgLane<NX, RPL> ln(threadIdx.x, N);
  const int k = ln.k;
  const double* Gh = Ghat + (size_t)b * N * NN * NN;
  const double* A = Aall + (size_t)b * K * NX * NX;
  const double* Bm = Ball + (size_t)b * K * NX * NU;
  double* g_lds = lds + pcg_lds_doubles(N, NX, 1024);   // [N][NN]
  double* lam_lds = g_lds + (size_t)N * NN;             // [N][NX]
  double* ctl_x = lam_lds + (size_t)N * NX;             // [N][NX]
  double* ctl_u = ctl_x + (size_t)N * NX;               // [K][NU]
  for (int e = threadIdx.x; e < N * NN; e += blockDim.x) g_lds[e] = gv[(size_t)b * N * NN + e];
  __syncthreads();
  // AB_k[r][m]: [A_k | B_k] row r, entry m < NN
  auto ab = [&](int kk, int r, int m) -> double {
    return m < NX ? A[((size_t)kk * NX + r) * NX + m] : Bm[((size_t)kk * NX + r) * NU + (m - NX)];
  };
  auto gh = [&](int kk, int r, int c) -> double { return Gh[((size_t)kk * NN + r) * NN + c]; };
  double xv[RPL];
  if constexpr (MODE == QP_MODE_DXU) {
#pragma unroll
    for (int m = 0; m < RPL; ++m) xv[m] = ln.valid ? lam_io[(size_t)b * rows + ln.row(m)] : 0.0;
    if (threadIdx.x == 0) iters[b] = 0;
  } else {
    PcgRow<NX> R[RPL];
    double bv[RPL];
#pragma unroll
    for (int m = 0; m < RPL; ++m) {
#pragma unroll
      for (int j = 0; j < NX; ++j) R[m].sd[j] = R[m].sl[j] = R[m].su[j] = R[m].pr[j] = 0.0;
      bv[m] = 0.0;
      if (!ln.valid) continue;
      const int i = ln.r(m);
      const double* gk = g_lds + (size_t)k * NN;
      double gam = cvec[((size_t)b * N + k) * NX + i];
      {
        double s = 0.0;
        const int mk = k == K ? NX : NN;   // the terminal block is nx x nx
        for (int j = 0; j < mk; ++j) s += gh(k, i, j) * gk[j];
        gam -= s;
      }
      if (k == 0) {
#pragma unroll
        for (int j = 0; j < NX; ++j) R[m].sd[j] = -gh(0, i, j);
      } else {
        const int km = k - 1;
        double abg[NN];   // row i of AB_{k-1} Ghat_{k-1}
#pragma unroll
        for (int c = 0; c < NN; ++c) {
          double acc = 0.0;
#pragma unroll
          for (int p = 0; p < NN; ++p) acc += ab(km, i, p) * gh(km, p, c);
          abg[c] = acc;
        }
#pragma unroll
        for (int j = 0; j < NX; ++j) R[m].sl[j] = abg[j];
#pragma unroll
        for (int j = 0; j < NX; ++j) {
          double acc = 0.0;
#pragma unroll
          for (int c = 0; c < NN; ++c) acc += abg[c] * ab(km, j, c);
          R[m].sd[j] = -(acc + gh(k, i, j));
        }
        const double* gm = g_lds + (size_t)km * NN;
        double s = 0.0;
#pragma unroll
        for (int c = 0; c < NN; ++c) s += abg[c] * gm[c];
        gam += s;
      }
      if (k < K) {
#pragma unroll
        for (int j = 0; j < NX; ++j) {
          double acc = 0.0;
#pragma unroll
          for (int c = 0; c < NN; ++c) acc += ab(k, j, c) * gh(k, c, i);
          R[m].su[j] = acc;
        }
      }
      bv[m] = gam;
      if (Sd_out) {
#pragma unroll
        for (int j = 0; j < NX; ++j) Sd_out[(((size_t)b * N + k) * NX + i) * NX + j] = R[m].sd[j];
        if (k > 0) {
#pragma unroll
          for (int j = 0; j < NX; ++j) Sl_out[(((size_t)b * K + k - 1) * NX + i) * NX + j] = R[m].sl[j];
        }
        gam_out[(size_t)b * rows + ln.row(m)] = gam;
      }
    }
    if constexpr (MODE == QP_MODE_SCHUR) {
      if (threadIdx.x == 0) iters[b] = 0;
      return;
    }
    pcg_lds_clear(lds, N, NX, 1024);
    const PcgLds L = pcg_lds(lds, N, NX, 1024);
    pcg_precondition<NX, RPL>(R, precond, ln, N, L.piv, nullptr);
    int it_done = 0;
    pcg_dispatch<NX, RPL>(precond, R, ln, N, L, bv, guess ? guess + (size_t)b * rows : nullptr, tol, max_iter,
                          nullptr, nullptr, &it_done, xv);
    if (threadIdx.x == 0) iters[b] = it_done;
  }
  // ---- epilogue: dxu = Ghat (g - C^T lambda)  (:449-452)
  __syncthreads();
  if (ln.valid) {
#pragma unroll
    for (int m = 0; m < RPL; ++m) {
      lam_lds[ln.row(m)] = xv[m];
      if (MODE == QP_MODE_PCG) lam_io[(size_t)b * rows + ln.row(m)] = xv[m];
    }
  }
  __syncthreads();
  // C^T lambda: x part lambda_k - A_k^T lambda_{k+1} (terminal: lambda_{N-1}), u part -B_k^T lambda_{k+1}
  for (int e = threadIdx.x; e < N * NX + K * NU; e += blockDim.x) {
    if (e < N * NX) {
      const int kk = e / NX, j = e - kk * NX;
      double atl = 0.0;
      if (kk < K) {
        const double* l1 = lam_lds + (kk + 1) * NX;
#pragma unroll
        for (int p = 0; p < NX; ++p) atl += A[((size_t)kk * NX + p) * NX + j] * l1[p];
      }
      ctl_x[e] = lam_lds[e] - atl;
    } else {
      const int f = e - N * NX;
      const int kk = f / NU, j = f - kk * NU;
      const double* l1 = lam_lds + (kk + 1) * NX;
      double btl = 0.0;
#pragma unroll
      for (int p = 0; p < NX; ++p) btl += Bm[((size_t)kk * NX + p) * NU + j] * l1[p];
      ctl_u[f] = -btl;
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < N * NX + K * NU; e += blockDim.x) {
    int kk, i;
    if (e < N * NX) {
      kk = e / NX;
      i = e - kk * NX;
    } else {
      const int f = e - N * NX;
      kk = f / NU;
      i = NX + (f - kk * NU);
    }
    const double* gk = g_lds + (size_t)kk * NN;
    const int mk = kk == K ? NX : NN;
    double acc = 0.0;
    for (int j = 0; j < mk; ++j) {
      const double cj = j < NX ? ctl_x[kk * NX + j] : ctl_u[kk * NU + (j - NX)];
      acc += gh(kk, i, j) * (gk[j] - cj);
    }
    if (e < N * NX)
      dx[(size_t)b * N * NX + e] = acc;
    else
      du[(size_t)b * K * NU + (e - N * NX)] = acc;
  }
}

template <int NJ>
struct LaunchHooks {
  static int ghat(hipStream_t s, int B, int N, const double* G, const double* rho, double* Gh, int* err) {
    constexpr int n = 3 * NJ;
    hipLaunchKernelGGL((k_ghat_full<n>), dim3(B * N), dim3(64), 0, s, B, N, 2 * NJ, NJ, G, rho, Gh, err);
    return 0;
  }
  static int qp(hipStream_t s, int B, int N, int precond, int mode, const double* Gh, const double* g,
                const double* A, const double* Bm, const double* c, const int* err, double tol, int max_iter,
                const double* guess, int* iters, double* dx, double* du, double* lam, double* Sd, double* Sl,
                double* gam) {
    constexpr int NX = 2 * NJ;
    const int rows = N * NX;
    const int rpl = pcg_rpl(N, NX);
    const int threads = ((rows / rpl + 63) / 64) * 64;
    const size_t lds = qpb_lds_doubles(N, NX, NJ) * sizeof(double);
#define TMPC_QPB_ARGS s, B, N, precond, Gh, g, A, Bm, c, err, tol, max_iter, guess, iters, dx, du, lam, Sd, Sl, gam
#define TMPC_QPB_LAUNCH(MD)                                                                                  \
    if (rpl == 1)                                                                                            \
      hipLaunchKernelGGL((k_qp_blocks<NJ, 1, 768, MD>), dim3(B), dim3(threads), lds, TMPC_QPB_ARGS);         \
    else                                                                                                     \
      hipLaunchKernelGGL((k_qp_blocks<NJ, 2, 512, MD>), dim3(B), dim3(threads), lds, TMPC_QPB_ARGS);
    if (mode == QP_MODE_PCG) {
      TMPC_QPB_LAUNCH(QP_MODE_PCG)
    } else if (mode == QP_MODE_SCHUR) {
      TMPC_QPB_LAUNCH(QP_MODE_SCHUR)
    } else {
      TMPC_QPB_LAUNCH(QP_MODE_DXU)
    }
#undef TMPC_QPB_LAUNCH
#undef TMPC_QPB_ARGS
    return 0;
  }
  static int set_lds(int bytes) {
    int e = 0;
#define TMPC_QPB_ATTR(R, T, MD) \
    e |= (int)hipFuncSetAttribute((const void*)k_qp_blocks<NJ, R, T, MD>, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    TMPC_QPB_ATTR(1, 768, QP_MODE_PCG) TMPC_QPB_ATTR(2, 512, QP_MODE_PCG)
    TMPC_QPB_ATTR(1, 768, QP_MODE_SCHUR) TMPC_QPB_ATTR(2, 512, QP_MODE_SCHUR)
    TMPC_QPB_ATTR(1, 768, QP_MODE_DXU) TMPC_QPB_ATTR(2, 512, QP_MODE_DXU)
#undef TMPC_QPB_ATTR
    return e;
  }
};

#ifdef TMPC_DEV_NJ
#define TMPC_HOOKS_NJ(nj, CALL)                 \
  if (nj != TMPC_DEV_NJ) return -2;              \
  return LaunchHooks<TMPC_DEV_NJ>::CALL;
#else
#define TMPC_HOOKS_NJ(nj, CALL)                  \
  switch (nj) {                                  \
    case 1: return LaunchHooks<1>::CALL;         \
    case 2: return LaunchHooks<2>::CALL;         \
    case 3: return LaunchHooks<3>::CALL;         \
    case 4: return LaunchHooks<4>::CALL;         \
    case 5: return LaunchHooks<5>::CALL;         \
    case 6: return LaunchHooks<6>::CALL;         \
    case 7: return LaunchHooks<7>::CALL;         \
    default: return -2;                          \
  }
#endif

int launch_ghat_full(hipStream_t s, int nj, int B, int N, const double* G, const double* rho, double* Gh, int* err) {
  TMPC_HOOKS_NJ(nj, ghat(s, B, N, G, rho, Gh, err))
}

int launch_qp_blocks(hipStream_t s, int nj, int B, int N, int precond, int mode, const double* Gh, const double* g,
                     const double* A, const double* Bm, const double* c, const int* err, double tol, int max_iter,
                     const double* guess, int* iters, double* dx, double* du, double* lam, double* Sd, double* Sl,
                     double* gam) {
  const int rows = N * 2 * nj;
  if (rows > 1024) return -1;
  if (qpb_lds_doubles(N, 2 * nj, nj) * sizeof(double) > 160 * 1024) return -3;
  TMPC_HOOKS_NJ(nj, qp(s, B, N, precond, mode, Gh, g, A, Bm, c, err, tol, max_iter, guess, iters, dx, du, lam, Sd,
                       Sl, gam))
}

int qp_blocks_set_max_lds() {
  const int bytes = 160 * 1024;
#ifdef TMPC_DEV_NJ
  return LaunchHooks<TMPC_DEV_NJ>::set_lds(bytes);
#else
  return LaunchHooks<1>::set_lds(bytes) | LaunchHooks<2>::set_lds(bytes) | LaunchHooks<3>::set_lds(bytes) |
         LaunchHooks<4>::set_lds(bytes) | LaunchHooks<5>::set_lds(bytes) | LaunchHooks<6>::set_lds(bytes) |
         LaunchHooks<7>::set_lds(bytes);
#endif
}

}  // namespace tmpc
