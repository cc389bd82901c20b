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

namespace tmpc {

// ======================================================================= per-knot forward dynamics
// Solver mode: lane = (b, k), k < N-1.  Writes qdd (the point the gradient is
// evaluated at, TrajoptPlant.py:313) and the dynamics defect
// c_{k+1} = x_{k+1} - f(x_k, u_k) (formKKTSystemBlocks :227-231); lane k = 0
// also writes c_0 = x_0 - xs (:213-214).
template <int NJ, bool CHAIN>
__global__ void __launch_bounds__(256) k_qp_fd(const ModelDev* __restrict__ M, int B, int N, double dt,
                                               const double* __restrict__ x, const double* __restrict__ u,
                                               const double* __restrict__ xs, const int* __restrict__ need,
                                               double* __restrict__ qdd_out, double* __restrict__ cvec) {
  constexpr int NX = 2 * NJ;
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int K = N - 1;
  if (gid >= B * K) return;
  const int b = gid / K, k = gid - b * K;
  if (!need[b]) return;
  const double* xb = x + (size_t)b * NX * N;
  const double* ub = u + (size_t)b * NJ * K;
  double q[NJ], qd[NJ], uu[NJ], qdd[NJ], cq[NJ], sq[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    q[j] = xb[j * N + k];
    qd[j] = xb[(NJ + j) * N + k];
    uu[j] = ub[j * K + k];
    joint_cs(M, j, q[j], cq[j], sq[j]);
  }
  fd_aba<NJ, CHAIN>(M, cq, sq, qd, uu, qdd);
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

// ======================================================================= analytic M^-1 columns
// lane = (knot, col), col < NJ; writes the full symmetric matrix (column col
// above the diagonal and row col left of it, :908-930).  x is [K][NX] rows
// with row stride `xstride` per knot and element stride `estride`.
template <int NJ, bool CHAIN>
__device__ __forceinline__ void minv_lane_store(const ModelDev* __restrict__ M, const double q[NJ], int col,
                                                double* __restrict__ Mo) {
  double cq[NJ], sq[NJ], mc[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) joint_cs(M, j, q[j], cq[j], sq[j]);
  minv_column<NJ, CHAIN>(M, cq, sq, col, mc);
#pragma unroll
  for (int r = 0; r < NJ; ++r) {
    if (r <= col) {
      Mo[r * NJ + col] = mc[r];
      Mo[col * NJ + r] = mc[r];
    }
  }
}

template <int NJ, bool CHAIN>
__global__ void __launch_bounds__(256) k_qp_minv(const ModelDev* __restrict__ M, int B, int N,
                                                 const double* __restrict__ x, const int* __restrict__ need,
                                                 double* __restrict__ minv_out) {
  constexpr int NX = 2 * NJ;
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int K = N - 1;
  if (gid >= B * K * NJ) return;
  const int col = gid % NJ;
  const int bk = gid / NJ;
  const int b = bk / K, k = bk - b * K;
  if (!need[b]) return;
  const double* xb = x + (size_t)b * NX * N;
  double q[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) q[j] = xb[j * N + k];
  minv_lane_store<NJ, CHAIN>(M, q, col, minv_out + (size_t)bk * NJ * NJ);
}

// ======================================================================= gradient columns -> A, B
// lane = (b, k, col), col < 2 NJ.  dqdd[:, col] = -Minv dc[:, col]
// (TrajoptPlant.py:313-316); A = I + dt [[0, I], [dqdd_q, dqdd_qd]],
// B = dt [[0], [Minv]] (TrajoptPlant.py:100-108).
template <int NJ, bool CHAIN>
__device__ __forceinline__ void grad_lane_store(const ModelDev* __restrict__ M, double dt, const double q[NJ],
                                                const double qd[NJ], const double qdd[NJ],
                                                const double* __restrict__ Mi, int col, double* __restrict__ A,
                                                double* __restrict__ Bm, double* __restrict__ dqdd) {
  constexpr int NX = 2 * NJ;
  double cq[NJ], sq[NJ], dc[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) joint_cs(M, j, q[j], cq[j], sq[j]);
  const bool colqd = col >= NJ;
  rnea_grad_column<NJ, CHAIN>(M, cq, sq, qd, qdd, colqd ? col - NJ : col, colqd, dc);
#pragma unroll
  for (int r = 0; r < NJ; ++r) {
    double acc = 0.0;
#pragma unroll
    for (int m = 0; m < NJ; ++m) acc += (-Mi[r * NJ + m]) * dc[m];
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

template <int NJ, bool CHAIN>
__global__ void __launch_bounds__(256) k_qp_grad(const ModelDev* __restrict__ M, int B, int N, double dt,
                                                 const double* __restrict__ x, const int* __restrict__ need,
                                                 const double* __restrict__ qdd_in, const double* __restrict__ minv_in,
                                                 double* __restrict__ Aout, double* __restrict__ Bout) {
  constexpr int NX = 2 * NJ;
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int K = N - 1;
  if (gid >= B * K * NX) return;
  const int col = gid % NX;
  const int bk = gid / NX;
  const int b = bk / K, k = bk - b * K;
  if (!need[b]) return;
  const double* xb = x + (size_t)b * NX * N;
  double q[NJ], qd[NJ], qdd[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    q[j] = xb[j * N + k];
    qd[j] = xb[(NJ + j) * N + k];
    qdd[j] = qdd_in[(size_t)bk * NJ + j];
  }
  grad_lane_store<NJ, CHAIN>(M, dt, q, qd, qdd, minv_in + (size_t)bk * NJ * NJ, col,
                             Aout + (size_t)bk * NX * NX, Bout + (size_t)bk * NX * NJ, nullptr);
}

// ======================================================================= G-block inverses
// Ghat = (G_k + rho I)^-1 for the three distinct cost Hessian blocks of
// QuadraticCost (Q, QF, R; TrajoptCost.py:71-83); solveKKTSystem_Schur
// adds rho in place and inverts (TrajoptMPCReference.py:419-422).
// Gauss-Jordan on an SPD matrix (no pivoting needed; exact for diagonal
// inputs), one 16-lane group per matrix, one row per lane, pivot rows
// broadcast with wave shuffles.
template <int NJ>
__global__ void __launch_bounds__(64) k_ginv(const CostDev* __restrict__ C, int B, const double* __restrict__ rho,
                                             const int* __restrict__ active, double* __restrict__ Ginv) {
  constexpr int NX = 2 * NJ;
  const int lane = threadIdx.x & 63;
  const int slot = (blockIdx.x * blockDim.x + threadIdx.x) >> 4;   // one matrix per 16 lanes
  const int r = lane & 15, base = lane & ~15;
  const bool in_range = slot < B * 3;
  const int b = in_range ? slot / 3 : 0, which = in_range ? slot - 3 * b : 0;
  const bool act = in_range && active[b];
  const int n = which == 2 ? NJ : NX;
  const double* src = which == 0 ? C->Q : (which == 1 ? C->QF : C->R);
  const double rh = act ? rho[b] : 0.0;
  double a[NX], inv[NX];
#pragma unroll
  for (int c = 0; c < NX; ++c) {
    a[c] = (act && r < n && c < n) ? src[r * n + c] + (r == c ? rh : 0.0) : (r == c ? 1.0 : 0.0);
    inv[c] = (r == c) ? 1.0 : 0.0;
  }
#pragma unroll
  for (int p = 0; p < NX; ++p) {
    double pa[NX], pi[NX];
#pragma unroll
    for (int c = 0; c < NX; ++c) {
      pa[c] = __shfl(a[c], base + p, 64);
      pi[c] = __shfl(inv[c], base + p, 64);
    }
    const double piv = pa[p];
    if (r == p) {
#pragma unroll
      for (int c = 0; c < NX; ++c) { a[c] = a[c] / piv; inv[c] = inv[c] / piv; }
    } else {
      const double f = a[p];
#pragma unroll
      for (int c = 0; c < NX; ++c) { a[c] -= f * (pa[c] / piv); inv[c] -= f * (pi[c] / piv); }
    }
  }
  if (act && r < n) {
    double* out = Ginv + ((size_t)b * 3 + which) * NX * NX;
#pragma unroll
    for (int c = 0; c < NX; ++c)
      if (c < n) out[r * n + c] = inv[c];
  }
}

// cost-to-go helpers (QuadraticCost.get_currQ, TrajoptCost.py:40-47)
__device__ __forceinline__ bool use_QF(const CostDev* C, int k, int N) {
  return (k == N - 1) || (C->QF_start >= 0 && k >= C->QF_start);
}

// ======================================================================= Schur blocks
// lane = (b, k, i): row i of S_kk, of S_{k,k-1} and gamma_k[i]
template <int NJ>
__global__ void __launch_bounds__(256) k_schur(const CostDev* __restrict__ C, int B, int N,
                                               const double* __restrict__ x, const double* __restrict__ u,
                                               const int* __restrict__ active, const double* __restrict__ Ginv,
                                               const double* __restrict__ Aall, const double* __restrict__ Ball,
                                               const double* __restrict__ cvec, double* __restrict__ Sd,
                                               double* __restrict__ Sl, double* __restrict__ gam) {
  constexpr int NX = 2 * NJ, NU = NJ;
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= B * N * NX) return;
  const int i = gid % NX;
  const int bk = gid / NX;
  const int b = bk / N, k = bk - b * N;
  if (!active[b]) return;
  const int K = N - 1;
  const double* xb = x + (size_t)b * NX * N;
  const double* ub = u + (size_t)b * NU * K;
  const double* G3 = Ginv + (size_t)b * 3 * NX * NX;
  const double* GxK = G3 + (use_QF(C, k, N) ? NX * NX : 0);
  const double* QK = use_QF(C, k, N) ? C->QF : C->Q;
  // gx_k = (x_k - xg)^T Q_k  (QuadraticCost.gradient, TrajoptCost.py:58-69)
  double dxk[NX], gxk[NX];
#pragma unroll
  for (int m = 0; m < NX; ++m) dxk[m] = xb[m * N + k] - C->xg[m];
#pragma unroll
  for (int j = 0; j < NX; ++j) {
    double acc = 0.0;
#pragma unroll
    for (int m = 0; m < NX; ++m) acc += dxk[m] * QK[m * NX + j];
    gxk[j] = acc;
  }
  double Gxg = 0.0;
#pragma unroll
  for (int j = 0; j < NX; ++j) Gxg += GxK[i * NX + j] * gxk[j];
  const double cki = cvec[(size_t)b * N * NX + k * NX + i];
  double* sdr = Sd + ((size_t)bk * NX + i) * NX;
  if (k == 0) {
#pragma unroll
    for (int j = 0; j < NX; ++j) sdr[j] = -GxK[i * NX + j];
    gam[(size_t)bk * NX + i] = cki - Gxg;
    return;
  }
  const int km = k - 1;
  const double* A = Aall + ((size_t)b * K + km) * NX * NX;
  const double* Bm = Ball + ((size_t)b * K + km) * NX * NU;
  const double* Gxm = G3 + (use_QF(C, km, N) ? NX * NX : 0);
  const double* Gu = G3 + 2 * NX * NX;
  const double* Qm = use_QF(C, km, N) ? C->QF : C->Q;
  double AG[NX], BG[NU];
#pragma unroll
  for (int j = 0; j < NX; ++j) {
    double acc = 0.0;
#pragma unroll
    for (int m = 0; m < NX; ++m) acc += A[i * NX + m] * Gxm[m * NX + j];
    AG[j] = acc;
  }
#pragma unroll
  for (int j = 0; j < NU; ++j) {
    double acc = 0.0;
#pragma unroll
    for (int m = 0; m < NU; ++m) acc += Bm[i * NU + m] * Gu[m * NU + j];
    BG[j] = acc;
  }
  double* slr = Sl + (((size_t)b * K + km) * NX + i) * NX;
#pragma unroll
  for (int j = 0; j < NX; ++j) slr[j] = AG[j];
#pragma unroll 1
  for (int j = 0; j < NX; ++j) {
    double acc = 0.0;
#pragma unroll
    for (int m = 0; m < NX; ++m) acc += AG[m] * A[j * NX + m];
#pragma unroll
    for (int m = 0; m < NU; ++m) acc += BG[m] * Bm[j * NU + m];
    sdr[j] = -(acc + GxK[i * NX + j]);
  }
  // gamma_k = c_k + AB_{k-1} Ghat_{k-1} g_{k-1} - E Ghat_k g_k
  double dxm[NX], um[NU];
#pragma unroll
  for (int m = 0; m < NX; ++m) dxm[m] = xb[m * N + km] - C->xg[m];
#pragma unroll
  for (int m = 0; m < NU; ++m) um[m] = ub[m * K + km];
  double s = 0.0;
#pragma unroll
  for (int j = 0; j < NX; ++j) {
    double g = 0.0;
#pragma unroll
    for (int m = 0; m < NX; ++m) g += dxm[m] * Qm[m * NX + j];
    s += AG[j] * g;
  }
#pragma unroll
  for (int j = 0; j < NU; ++j) {
    double g = 0.0;
#pragma unroll
    for (int m = 0; m < NU; ++m) g += um[m] * C->R[m * NU + j];
    s += BG[j] * g;
  }
  gam[(size_t)bk * NX + i] = cki + s - Gxg;
}

// ======================================================================= block-tridiagonal PCG
// One workgroup per problem, one lane per row of S (PCG.pcg, PCG.py:66-111).
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// every thread returns the same value; `red` must alternate between calls
__device__ __forceinline__ double block_sum(double v, double* red, int nwaves) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
  for (int i = 0; i < nwaves; ++i) s += red[i];
  return s;
}

template <int NX, int MAXT>
__global__ void __launch_bounds__(MAXT) k_pcg(int B, int N, int precond, const double* __restrict__ Sd,
                                              const double* __restrict__ Sl, const double* __restrict__ Su,
                                              const double* __restrict__ gam, const double* __restrict__ guess,
                                              const int* __restrict__ active, double tol, int max_iter,
                                              double* __restrict__ lam,
                                              int* __restrict__ iters, double* __restrict__ trace_nu,
                                              double* __restrict__ trace_res, double* __restrict__ Pd_out) {
  const int b = blockIdx.x;
  if (active && !active[b]) return;
  extern __shared__ __align__(16) double lds[];
  const int rows = N * NX;
  const int nwaves = (blockDim.x + 63) >> 6;
  double* pbuf = lds;
  double* rbuf = pbuf + rows;
  double* wbuf = rbuf + rows;
  double* tbuf = wbuf + rows;
  double* xbuf = tbuf + rows;
  double* red = xbuf + rows;          // 2 x 16
  double* piv = red + 32;             // 2 x N x 2NX
  const int t = threadIdx.x;
  const bool valid = t < rows;
  const int k = valid ? t / NX : 0;
  const int i = valid ? t - k * NX : 0;
  const int K = N - 1;

  double sd[NX], sl[NX], su[NX], pr[NX];
#pragma unroll
  for (int j = 0; j < NX; ++j) { sd[j] = 0.0; sl[j] = 0.0; su[j] = 0.0; pr[j] = 0.0; }
  if (valid) {
    const double* d = Sd + (((size_t)b * N + k) * NX + i) * NX;
#pragma unroll
    for (int j = 0; j < NX; ++j) sd[j] = d[j];
    if (k > 0) {
      const double* l = Sl + (((size_t)b * K + (k - 1)) * NX + i) * NX;
#pragma unroll
      for (int j = 0; j < NX; ++j) sl[j] = l[j];
    }
    if (k < K) {
      if (Su) {
        const double* up = Su + (((size_t)b * K + k) * NX + i) * NX;
#pragma unroll
        for (int j = 0; j < NX; ++j) su[j] = up[j];
      } else {
        const double* l = Sl + ((size_t)b * K + k) * NX * NX;
#pragma unroll
        for (int j = 0; j < NX; ++j) su[j] = l[j * NX + i];
      }
    }
  }

  // ---- preconditioner (compute_preconditioner, PCG.py:166-212)
  if (precond == PRECOND_J) {
    // inv(diag(diag(S)))  (PCG.py:168-169)
    double dii = 1.0;
#pragma unroll
    for (int j = 0; j < NX; ++j)
      if (j == i) dii = sd[j];
    if (valid) pr[0] = 1.0 / dii;
  } else {
    // Gauss-Jordan of the diagonal block, one row per lane, pivot rows via LDS
    double aug[2 * NX];
#pragma unroll
    for (int j = 0; j < NX; ++j) { aug[j] = sd[j]; aug[NX + j] = (j == i) ? 1.0 : 0.0; }
#pragma unroll
    for (int p = 0; p < NX; ++p) {
      double* pv = piv + ((p & 1) * N + k) * 2 * NX;
      if (valid && i == p) {
        const double d = aug[p];
#pragma unroll
        for (int j = 0; j < 2 * NX; ++j) { aug[j] = aug[j] / d; pv[j] = aug[j]; }
      }
      __syncthreads();
      if (valid && i != p) {
        const double f = aug[p];
#pragma unroll
        for (int j = 0; j < 2 * NX; ++j) aug[j] -= f * pv[j];
      }
    }
#pragma unroll
    for (int j = 0; j < NX; ++j) pr[j] = aug[NX + j];
    if (Pd_out && valid) {
      double* o = Pd_out + (((size_t)b * N + k) * NX + i) * NX;
#pragma unroll
      for (int j = 0; j < NX; ++j) o[j] = pr[j];
    }
  }

  // z = P r  (J: diagonal, BJ: block diagonal, SS: P_D (r - S_off P_D r))
  auto apply_P = [&](double r_i) -> double {
    if (precond == PRECOND_J) return pr[0] * r_i;
    if (valid) rbuf[t] = r_i;
    __syncthreads();
    double w = 0.0;
    if (valid) {
#pragma unroll
      for (int j = 0; j < NX; ++j) w += pr[j] * rbuf[k * NX + j];
    }
    if (precond == PRECOND_BJ) return w;
    if (valid) wbuf[t] = w;
    __syncthreads();
    double tv = 0.0;
    if (valid) {
      double acc = 0.0;
      if (k > 0) {
#pragma unroll
        for (int j = 0; j < NX; ++j) acc += sl[j] * wbuf[(k - 1) * NX + j];
      }
      if (k < K) {
#pragma unroll
        for (int j = 0; j < NX; ++j) acc += su[j] * wbuf[(k + 1) * NX + j];
      }
      tv = r_i - acc;
      tbuf[t] = tv;
    }
    __syncthreads();
    double z = 0.0;
    if (valid) {
#pragma unroll
      for (int j = 0; j < NX; ++j) z += pr[j] * tbuf[k * NX + j];
    }
    return z;
  };
  auto spmv = [&](const double* vbuf) -> double {
    double acc = 0.0;
    if (valid) {
      if (k > 0) {
#pragma unroll
        for (int j = 0; j < NX; ++j) acc += sl[j] * vbuf[(k - 1) * NX + j];
      }
#pragma unroll
      for (int j = 0; j < NX; ++j) acc += sd[j] * vbuf[k * NX + j];
      if (k < K) {
#pragma unroll
        for (int j = 0; j < NX; ++j) acc += su[j] * vbuf[(k + 1) * NX + j];
      }
    }
    return acc;
  };

  const double bi = valid ? gam[(size_t)b * rows + t] : 0.0;
  // x0 = guess (default zeros, PCG.py:11-12); r = b - A x0 (:76)
  double xi = 0.0, ri = bi;
  if (guess) {
    xi = valid ? guess[(size_t)b * rows + t] : 0.0;
    if (valid) xbuf[t] = xi;
    __syncthreads();
    ri = bi - spmv(xbuf);
    __syncthreads();
  }
  double zi = apply_P(ri);
  double pi = zi;
  int rsel = 0;
  double nu = block_sum(valid ? ri * zi : 0.0, red + 16 * rsel, nwaves);
  rsel ^= 1;
  double* tn = trace_nu ? trace_nu + (size_t)b * (max_iter + 1) : nullptr;
  double* tr = trace_res ? trace_res + (size_t)b * (max_iter + 1) : nullptr;
  auto true_residual = [&]() -> double {
    // ||b - A x|| (PCG.py:83,95), debug/trace only
    if (valid) xbuf[t] = xi;
    __syncthreads();
    const double e = valid ? bi - spmv(xbuf) : 0.0;
    const double s = block_sum(e * e, red + 16 * rsel, nwaves);
    rsel ^= 1;
    return sqrt(s);
  };
  if (tn && t == 0) tn[0] = fabs(nu);
  if (tr) {
    const double rn = true_residual();
    if (t == 0) tr[0] = rn;
  }
  int it_done = max_iter;
  for (int it = 0; it < max_iter; ++it) {
    if (valid) pbuf[t] = pi;
    __syncthreads();
    const double api = spmv(pbuf);
    const double pap = block_sum(valid ? pi * api : 0.0, red + 16 * rsel, nwaves);
    rsel ^= 1;
    const double alpha = nu / pap;
    ri = ri - api * alpha;
    xi = xi + pi * alpha;
    zi = apply_P(ri);
    const double nup = block_sum(valid ? ri * zi : 0.0, red + 16 * rsel, nwaves);
    rsel ^= 1;
    if (tn && t == 0) tn[it + 1] = fabs(nup);
    if (tr) {
      const double rn = true_residual();
      if (t == 0) tr[it + 1] = rn;
    }
    if (fabs(nup) < tol) {
      it_done = it + 1;
      break;
    }
    const double beta = nup / nu;
    pi = zi + pi * beta;
    nu = nup;
  }
  if (valid) lam[(size_t)b * rows + t] = xi;
  if (t == 0) iters[b] = it_done;
}

// ======================================================================= dxul recovery
// dxu = Ghat (g - C^T lambda)  (solveKKTSystem_Schur :449-452), lane = (b, k, i)
template <int NJ>
__global__ void __launch_bounds__(256) k_dxu(const CostDev* __restrict__ C, int B, int N,
                                             const double* __restrict__ x, const double* __restrict__ u,
                                             const int* __restrict__ active, const double* __restrict__ Ginv,
                                             const double* __restrict__ Aall, const double* __restrict__ Ball,
                                             const double* __restrict__ lam, double* __restrict__ dx,
                                             double* __restrict__ du) {
  constexpr int NX = 2 * NJ, NU = NJ, NXU = NX + NU;
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= B * N * NXU) return;
  const int i = gid % NXU;
  const int bk = gid / NXU;
  const int b = bk / N, k = bk - b * N;
  if (!active[b]) return;
  const int K = N - 1;
  if (k == K && i >= NX) return;
  const double* xb = x + (size_t)b * NX * N;
  const double* G3 = Ginv + (size_t)b * 3 * NX * NX;
  const double* L = lam + (size_t)b * N * NX;
  if (i < NX) {
    const double* Gx = G3 + (use_QF(C, k, N) ? NX * NX : 0);
    const double* Qk = use_QF(C, k, N) ? C->QF : C->Q;
    double dxk[NX], h[NX];
#pragma unroll
    for (int m = 0; m < NX; ++m) dxk[m] = xb[m * N + k] - C->xg[m];
    const double* A = (k < K) ? Aall + ((size_t)b * K + k) * NX * NX : nullptr;
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      double g = 0.0;
#pragma unroll
      for (int m = 0; m < NX; ++m) g += dxk[m] * Qk[m * NX + j];
      double atl = 0.0;
      if (k < K) {
#pragma unroll
        for (int m = 0; m < NX; ++m) atl += A[m * NX + j] * L[(k + 1) * NX + m];
      }
      h[j] = g - (L[k * NX + j] - atl);
    }
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < NX; ++j) acc += Gx[i * NX + j] * h[j];
    dx[(size_t)bk * NX + i] = acc;
  } else {
    const int iu = i - NX;
    const double* ub = u + (size_t)b * NU * K;
    const double* Gu = G3 + 2 * NX * NX;
    const double* Bm = Ball + ((size_t)b * K + k) * NX * NU;
    double uk[NU], h[NU];
#pragma unroll
    for (int m = 0; m < NU; ++m) uk[m] = ub[m * K + k];
#pragma unroll
    for (int j = 0; j < NU; ++j) {
      double g = 0.0;
#pragma unroll
      for (int m = 0; m < NU; ++m) g += uk[m] * C->R[m * NU + j];
      double btl = 0.0;
#pragma unroll
      for (int m = 0; m < NX; ++m) btl += Bm[m * NU + j] * L[(k + 1) * NX + m];
      h[j] = g - (-btl);
    }
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < NU; ++j) acc += Gu[iu * NU + j] * h[j];
    du[((size_t)b * K + k) * NU + iu] = acc;
  }
}

// ======================================================================= line-search merit terms
// lane = (b, t, k): for trial step alpha_t evaluate the per-knot pieces of
// totalCost (:296-310), totalHardConstraintViolation (:273-294) and the
// directional derivative D (:635-648, gradient taken at x_new as the
// reference does).  Knot lane N-1 carries the terminal cost / D term and the
// |x_0 - xs| violation term.
template <int NJ, bool CHAIN>
__global__ void __launch_bounds__(256) k_ls_terms(const ModelDev* __restrict__ M, const CostDev* __restrict__ C,
                                                  int B, int N, int T, double dt, const double* __restrict__ alphas,
                                                  const double* __restrict__ x, const double* __restrict__ u,
                                                  const double* __restrict__ xs, const double* __restrict__ dx,
                                                  const double* __restrict__ du, const int* __restrict__ active,
                                                  double* __restrict__ terms) {
  constexpr int NX = 2 * NJ, NU = NJ;
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= B * T * N) return;
  const int k = gid % N;
  const int bt = gid / N;
  const int b = bt / T, t = bt - b * T;
  if (!active[b]) return;
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
  double d[NX];
#pragma unroll
  for (int m = 0; m < NX; ++m) d[m] = xk[m] - C->xg[m];
  // value: 0.5 dx^T (Q dx) [+ 0.5 u^T (R u)]; gradient: [dx^T Q, u^T R]
  double vq = 0.0, Dk = 0.0;
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
  double cost = 0.5 * vq;
  double viol = 0.0;
  double* out = terms + ((size_t)bt * N + k) * 3;
  if (k < K) {
    double uk[NU], duk[NU];
#pragma unroll
    for (int m = 0; m < NU; ++m) {
      duk[m] = dub ? dub[k * NU + m] : 0.0;
      uk[m] = dub ? ub[m * K + k] - al * duk[m] : ub[m * K + k];
    }
    double vr = 0.0;
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
    cost += 0.5 * vr;
    // dynamics defect at the trial point
    double cq[NJ], sq[NJ], qd[NJ], qdd[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      qd[j] = xk[NJ + j];
      joint_cs(M, j, xk[j], cq[j], sq[j]);
    }
    fd_aba<NJ, CHAIN>(M, cq, sq, qd, uk, qdd);
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
  out[0] = cost;
  out[1] = viol;
  out[2] = Dk;
}

// ======================================================================= line-search decision + state machine
// One workgroup per problem.  Reproduces the accept test (:655-666), the
// alpha schedule (:712-718), reduce_regularization (:457-461) and
// check_for_exit_or_error (:463-481), applies the accepted step and records
// the trace row (:691-705 / :729-743).
__global__ void __launch_bounds__(64) k_ls_decide(int B, int N, int NX, int NU, int T, int mode,
                                                  const double* __restrict__ alphas, SolverOpts o,
                                                  const double* __restrict__ terms, double* __restrict__ x,
                                                  double* __restrict__ u, const double* __restrict__ dx,
                                                  const double* __restrict__ du, ProbState st,
                                                  const int* __restrict__ pcg_iters, TraceDev tr,
                                                  int* __restrict__ active_count,
                                                  unsigned long long* __restrict__ counters) {
  const int b = blockIdx.x;
  if (!st.active[b]) return;
  __shared__ double sJ[64], sC[64], sD[64];
  __shared__ int s_choice;
  const int t = threadIdx.x;
  if (t < T) {
    const double* tm = terms + ((size_t)b * T + t) * N * 3;
    double J = 0.0, c = 0.0, D = 0.0;
    for (int k = 0; k < N - 1; ++k) J = J + tm[k * 3 + 0];
    J = J + tm[(N - 1) * 3 + 0];
    c = tm[(N - 1) * 3 + 1];
    for (int k = 0; k < N - 1; ++k) c = c + tm[k * 3 + 1];
    for (int k = 0; k < N - 1; ++k) D += tm[k * 3 + 2];
    D += tm[(N - 1) * 3 + 2];
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
      tr.accepted[e] = 0; tr.pcg_iters[e] = 0;
      s_choice = -2;
    } else {
      const double J = st.J[b], c = st.c[b], merit = st.merit[b];
      double rho = st.rho[b], drho = st.drho[b];
      int choice = -1;
      double D = 0.0, ratio = 0.0, Jn = 0.0, cn = 0.0, mn = 0.0, al = 1.0;
      int ls = 0;
      for (int tt = 0; tt < T; ++tt) {
        al = alphas[tt];
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
        // [0] problem-QPs solved, [1] PCG iterations, [2] QPs with a fresh dynamics gradient
        atomicAdd(&counters[0], 1ull);
        atomicAdd(&counters[1], (unsigned long long)(pcg_iters ? pcg_iters[b] : 0));
        atomicAdd(&counters[2], (unsigned long long)st.need_grad[b]);
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
      else atomicAdd(active_count, 1);
      s_choice = choice;
    }
  }
  __syncthreads();
  const int choice = s_choice;
  if (choice >= 0) {
    const double al = alphas[choice];
    double* xb = x + (size_t)b * NX * N;
    const double* dxb = dx + (size_t)b * N * NX;
    for (int e = t; e < NX * N; e += blockDim.x) {
      const int m = e / N, k = e - m * N;
      xb[e] = xb[e] - al * dxb[k * NX + m];
    }
    const int K = N - 1;
    double* ub = u + (size_t)b * NU * K;
    const double* dub = du + (size_t)b * K * NU;
    for (int e = t; e < NU * K; e += blockDim.x) {
      const int m = e / K, k = e - m * K;
      ub[e] = ub[e] - al * dub[k * NU + m];
    }
  } else if (choice == -2 && t == 0) {
    atomicAdd(active_count, 1);
  }
}

__global__ void k_init_state(int B, double rho_init, ProbState st) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  st.rho[b] = rho_init;
  st.drho[b] = 1.0;
  st.iter[b] = 0;
  st.active[b] = 1;
  st.need_grad[b] = 1;
  st.exit_sqp[b] = 0;
}

// ======================================================================= kernel-level entry points
// [K][nx] / [K][nu] row layout, one lane per knot (or per knot and column)
template <int NJ, bool CHAIN>
__global__ void __launch_bounds__(256) k_unit_fd(const ModelDev* __restrict__ M, int K, double dt,
                                                 const double* __restrict__ x, const double* __restrict__ u,
                                                 double* __restrict__ xnext, double* __restrict__ qdd_out) {
  constexpr int NX = 2 * NJ;
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  double q[NJ], qd[NJ], uu[NJ], qdd[NJ], cq[NJ], sq[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    q[j] = x[(size_t)k * NX + j];
    qd[j] = x[(size_t)k * NX + NJ + j];
    uu[j] = u[(size_t)k * NJ + j];
    joint_cs(M, j, q[j], cq[j], sq[j]);
  }
  fd_aba<NJ, CHAIN>(M, cq, sq, qd, uu, qdd);
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    qdd_out[(size_t)k * NJ + j] = qdd[j];
    if (xnext) {
      xnext[(size_t)k * NX + j] = __dadd_rn(q[j], __dmul_rn(dt, qd[j]));
      xnext[(size_t)k * NX + NJ + j] = __dadd_rn(qd[j], __dmul_rn(dt, qdd[j]));
    }
  }
}

template <int NJ, bool CHAIN>
__global__ void __launch_bounds__(256) k_unit_minv(const ModelDev* __restrict__ M, int K, const double* __restrict__ x,
                                                   double* __restrict__ minv_out) {
  constexpr int NX = 2 * NJ;
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= K * NJ) return;
  const int col = gid % NJ, k = gid / NJ;
  double q[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) q[j] = x[(size_t)k * NX + j];
  minv_lane_store<NJ, CHAIN>(M, q, col, minv_out + (size_t)k * NJ * NJ);
}

template <int NJ, bool CHAIN>
__global__ void __launch_bounds__(256) k_unit_grad(const ModelDev* __restrict__ M, int K, double dt,
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
  grad_lane_store<NJ, CHAIN>(M, dt, q, qd, qdd, minv_in + (size_t)k * NJ * NJ, col,
                             Aout ? Aout + (size_t)k * NX * NX : nullptr, Bout ? Bout + (size_t)k * NX * NJ : nullptr,
                             dqdd ? dqdd + (size_t)k * NJ * 3 * NJ : nullptr);
}

// sequential Euler rollout, one lane per problem (workload setup: §8d)
template <int NJ, bool CHAIN>
__global__ void __launch_bounds__(64) k_rollout(const ModelDev* __restrict__ M, int B, int N, double dt,
                                                double* __restrict__ x, const double* __restrict__ u) {
  constexpr int NX = 2 * NJ;
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int K = N - 1;
  double* xb = x + (size_t)b * NX * N;
  const double* ub = u + (size_t)b * NJ * K;
  double q[NJ], qd[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) { q[j] = xb[j * N]; qd[j] = xb[(NJ + j) * N]; }
  for (int k = 0; k < K; ++k) {
    double uu[NJ], qdd[NJ], cq[NJ], sq[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      uu[j] = ub[j * K + k];
      joint_cs(M, j, q[j], cq[j], sq[j]);
    }
    fd_aba<NJ, CHAIN>(M, cq, sq, qd, uu, qdd);
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

// ======================================================================= launchers
#define TMPC_GRID(n, bs) dim3(((n) + (bs) - 1) / (bs)), dim3(bs)

template <int NJ, bool CHAIN>
struct Launch {
  static void qp_fd(hipStream_t s, const ModelDev* M, int B, int N, double dt, const double* x, const double* u,
                    const double* xs, const int* need, double* qdd, double* cvec) {
    hipLaunchKernelGGL((k_qp_fd<NJ, CHAIN>), TMPC_GRID(B * (N - 1), 256), 0, s, M, B, N, dt, x, u, xs, need, qdd,
                       cvec);
  }
  static void qp_minv(hipStream_t s, const ModelDev* M, int B, int N, const double* x, const int* need, double* minv) {
    hipLaunchKernelGGL((k_qp_minv<NJ, CHAIN>), TMPC_GRID(B * (N - 1) * NJ, 256), 0, s, M, B, N, x, need, minv);
  }
  static void qp_grad(hipStream_t s, const ModelDev* M, int B, int N, double dt, const double* x, const int* need,
                      const double* qdd, const double* minv, double* A, double* Bm) {
    hipLaunchKernelGGL((k_qp_grad<NJ, CHAIN>), TMPC_GRID(B * (N - 1) * 2 * NJ, 256), 0, s, M, B, N, dt, x, need,
                       qdd, minv, A, Bm);
  }
  static void ls_terms(hipStream_t s, const ModelDev* M, const CostDev* C, int B, int N, int T, double dt,
                       const double* alphas, const double* x, const double* u, const double* xs, const double* dx,
                       const double* du, const int* active, double* terms) {
    hipLaunchKernelGGL((k_ls_terms<NJ, CHAIN>), TMPC_GRID(B * T * N, 256), 0, s, M, C, B, N, T, dt, alphas, x, u,
                       xs, dx, du, active, terms);
  }
  static void unit_fd(hipStream_t s, const ModelDev* M, int K, double dt, const double* x, const double* u,
                      double* xnext, double* qdd) {
    hipLaunchKernelGGL((k_unit_fd<NJ, CHAIN>), TMPC_GRID(K, 256), 0, s, M, K, dt, x, u, xnext, qdd);
  }
  static void unit_minv(hipStream_t s, const ModelDev* M, int K, const double* x, double* minv) {
    hipLaunchKernelGGL((k_unit_minv<NJ, CHAIN>), TMPC_GRID(K * NJ, 256), 0, s, M, K, x, minv);
  }
  static void unit_grad(hipStream_t s, const ModelDev* M, int K, double dt, const double* x, const double* qdd,
                        const double* minv, double* A, double* Bm, double* dqdd) {
    hipLaunchKernelGGL((k_unit_grad<NJ, CHAIN>), TMPC_GRID(K * 2 * NJ, 256), 0, s, M, K, dt, x, qdd, minv, A, Bm,
                       dqdd);
  }
  static void rollout(hipStream_t s, const ModelDev* M, int B, int N, double dt, double* x, const double* u) {
    hipLaunchKernelGGL((k_rollout<NJ, CHAIN>), TMPC_GRID(B, 64), 0, s, M, B, N, dt, x, u);
  }
};

template <int NJ>
struct LaunchNJ {
  static void ginv(hipStream_t s, const CostDev* C, int B, const double* rho, const int* active, double* G) {
    hipLaunchKernelGGL((k_ginv<NJ>), TMPC_GRID(B * 3 * 16, 64), 0, s, C, B, rho, active, G);
  }
  static void schur(hipStream_t s, const CostDev* C, int B, int N, const double* x, const double* u,
                    const int* active, const double* G, const double* A, const double* Bm, const double* cvec,
                    double* Sd, double* Sl, double* gam) {
    hipLaunchKernelGGL((k_schur<NJ>), TMPC_GRID(B * N * 2 * NJ, 256), 0, s, C, B, N, x, u, active, G, A, Bm, cvec,
                       Sd, Sl, gam);
  }
  static void dxu(hipStream_t s, const CostDev* C, int B, int N, const double* x, const double* u, const int* active,
                  const double* G, const double* A, const double* Bm, const double* lam, double* dx, double* du) {
    hipLaunchKernelGGL((k_dxu<NJ>), TMPC_GRID(B * N * 3 * NJ, 256), 0, s, C, B, N, x, u, active, G, A, Bm, lam, dx,
                       du);
  }
};

int pcg_set_max_lds() {
  const int bytes = 160 * 1024;
  int err = 0;
#define SETA(V)                                                                                                 \
  err |= (int)hipFuncSetAttribute((const void*)k_pcg<V, 768>, hipFuncAttributeMaxDynamicSharedMemorySize, bytes); \
  err |= (int)hipFuncSetAttribute((const void*)k_pcg<V, 1024>, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  SETA(2) SETA(4) SETA(6) SETA(8) SETA(10) SETA(12) SETA(14) SETA(16)
#undef SETA
  return err;
}

template <int NX>
static void launch_pcg_nx(hipStream_t s, int B, int N, int precond, const double* Sd, const double* Sl,
                          const double* Su, const double* gam, const double* guess, const int* active, double tol, int max_iter,
                          double* lam, int* iters, double* tnu, double* tres, double* Pd) {
  const int rows = N * NX;
  const int threads = ((rows + 63) / 64) * 64;
  const size_t lds = (size_t)(5 * rows + 32 + 2 * N * 2 * NX) * sizeof(double);
  if (threads <= 768)
    hipLaunchKernelGGL((k_pcg<NX, 768>), dim3(B), dim3(threads), lds, s, B, N, precond, Sd, Sl, Su, gam, guess, active,
                       tol, max_iter, lam, iters, tnu, tres, Pd);
  else
    hipLaunchKernelGGL((k_pcg<NX, 1024>), dim3(B), dim3(threads), lds, s, B, N, precond, Sd, Sl, Su, gam, guess, active,
                       tol, max_iter, lam, iters, tnu, tres, Pd);
}

int launch_pcg(hipStream_t s, int nx, int B, int N, int precond, const double* Sd, const double* Sl,
               const double* Su, const double* gam, const double* guess, const int* active, double tol, int max_iter, double* lam,
               int* iters, double* tnu, double* tres, double* Pd) {
  if (N * nx > 1024) return -1;
  switch (nx) {
#define CASE_NX(V) \
  case V: launch_pcg_nx<V>(s, B, N, precond, Sd, Sl, Su, gam, guess, active, tol, max_iter, lam, iters, tnu, tres, Pd); return 0;
    CASE_NX(2) CASE_NX(4) CASE_NX(6) CASE_NX(8) CASE_NX(10) CASE_NX(12) CASE_NX(14) CASE_NX(16)
#undef CASE_NX
    default: return -2;
  }
}

void launch_ls_decide(hipStream_t s, int B, int N, int NX, int NU, int T, int mode, const double* alphas,
                      const SolverOpts& o, const double* terms, double* x, double* u, const double* dx,
                      const double* du, const ProbState& st, const int* pcg_iters, const TraceDev& tr,
                      int* active_count, unsigned long long* counters) {
  hipLaunchKernelGGL(k_ls_decide, dim3(B), dim3(64), 0, s, B, N, NX, NU, T, mode, alphas, o, terms, x, u, dx, du,
                     st, pcg_iters, tr, active_count, counters);
}

void launch_init_state(hipStream_t s, int B, double rho_init, const ProbState& st) {
  hipLaunchKernelGGL(k_init_state, TMPC_GRID(B, 256), 0, s, B, rho_init, st);
}

// dispatch tables over the joint count and the chain specialisation
#define TMPC_DISPATCH_NJ(nj, chain, CALL)                                          \
  switch (nj) {                                                                    \
    case 1: if (chain) Launch<1, true>::CALL; else Launch<1, false>::CALL; break;  \
    case 2: if (chain) Launch<2, true>::CALL; else Launch<2, false>::CALL; break;  \
    case 3: if (chain) Launch<3, true>::CALL; else Launch<3, false>::CALL; break;  \
    case 4: if (chain) Launch<4, true>::CALL; else Launch<4, false>::CALL; break;  \
    case 5: if (chain) Launch<5, true>::CALL; else Launch<5, false>::CALL; break;  \
    case 6: if (chain) Launch<6, true>::CALL; else Launch<6, false>::CALL; break;  \
    case 7: if (chain) Launch<7, true>::CALL; else Launch<7, false>::CALL; break;  \
    default: return -2;                                                            \
  }                                                                                \
  return 0;

#define TMPC_DISPATCH_NJ2(nj, CALL)          \
  switch (nj) {                              \
    case 1: LaunchNJ<1>::CALL; break;        \
    case 2: LaunchNJ<2>::CALL; break;        \
    case 3: LaunchNJ<3>::CALL; break;        \
    case 4: LaunchNJ<4>::CALL; break;        \
    case 5: LaunchNJ<5>::CALL; break;        \
    case 6: LaunchNJ<6>::CALL; break;        \
    case 7: LaunchNJ<7>::CALL; break;        \
    default: return -2;                      \
  }                                                                                \
  return 0;

int launch_qp_fd(hipStream_t s, int nj, bool chain, const ModelDev* M, int B, int N, double dt, const double* x,
                 const double* u, const double* xs, const int* need, double* qdd, double* cvec) {
  TMPC_DISPATCH_NJ(nj, chain, qp_fd(s, M, B, N, dt, x, u, xs, need, qdd, cvec))
}
int launch_qp_minv(hipStream_t s, int nj, bool chain, const ModelDev* M, int B, int N, const double* x,
                   const int* need, double* minv) {
  TMPC_DISPATCH_NJ(nj, chain, qp_minv(s, M, B, N, x, need, minv))
}
int launch_qp_grad(hipStream_t s, int nj, bool chain, const ModelDev* M, int B, int N, double dt, const double* x,
                   const int* need, const double* qdd, const double* minv, double* A, double* Bm) {
  TMPC_DISPATCH_NJ(nj, chain, qp_grad(s, M, B, N, dt, x, need, qdd, minv, A, Bm))
}
int launch_ls_terms(hipStream_t s, int nj, bool chain, const ModelDev* M, const CostDev* C, int B, int N, int T,
                    double dt, const double* alphas, const double* x, const double* u, const double* xs,
                    const double* dx, const double* du, const int* active, double* terms) {
  TMPC_DISPATCH_NJ(nj, chain, ls_terms(s, M, C, B, N, T, dt, alphas, x, u, xs, dx, du, active, terms))
}
int launch_unit_fd(hipStream_t s, int nj, bool chain, const ModelDev* M, int K, double dt, const double* x,
                   const double* u, double* xnext, double* qdd) {
  TMPC_DISPATCH_NJ(nj, chain, unit_fd(s, M, K, dt, x, u, xnext, qdd))
}
int launch_unit_minv(hipStream_t s, int nj, bool chain, const ModelDev* M, int K, const double* x, double* minv) {
  TMPC_DISPATCH_NJ(nj, chain, unit_minv(s, M, K, x, minv))
}
int launch_unit_grad(hipStream_t s, int nj, bool chain, const ModelDev* M, int K, double dt, const double* x,
                     const double* qdd, const double* minv, double* A, double* Bm, double* dqdd) {
  TMPC_DISPATCH_NJ(nj, chain, unit_grad(s, M, K, dt, x, qdd, minv, A, Bm, dqdd))
}
int launch_rollout(hipStream_t s, int nj, bool chain, const ModelDev* M, int B, int N, double dt, double* x,
                   const double* u) {
  TMPC_DISPATCH_NJ(nj, chain, rollout(s, M, B, N, dt, x, u))
}
int launch_ginv(hipStream_t s, int nj, const CostDev* C, int B, const double* rho, const int* active, double* G) {
  TMPC_DISPATCH_NJ2(nj, ginv(s, C, B, rho, active, G))
}
int launch_schur(hipStream_t s, int nj, const CostDev* C, int B, int N, const double* x, const double* u,
                 const int* active, const double* G, const double* A, const double* Bm, const double* cvec,
                 double* Sd, double* Sl, double* gam) {
  TMPC_DISPATCH_NJ2(nj, schur(s, C, B, N, x, u, active, G, A, Bm, cvec, Sd, Sl, gam))
}
int launch_dxu(hipStream_t s, int nj, const CostDev* C, int B, int N, const double* x, const double* u,
               const int* active, const double* G, const double* A, const double* Bm, const double* lam, double* dx,
               double* du) {
  TMPC_DISPATCH_NJ2(nj, dxu(s, C, B, N, x, u, active, G, A, Bm, lam, dx, du))
}

}  // namespace tmpc
