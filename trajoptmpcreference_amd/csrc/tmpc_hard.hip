// Hard box constraints (BoxConstraint ACTIVE_SET / FULL_SET) in the SQP QP, for gfx950.
//
// The reference appends each knot's constraint rows to C right after that knot's
// dynamics rows (formKKTSystemBlocks, TrajoptMPCReference.py:238-248, 262-270), so
// the Schur complement S = -C G^-1 C^T (:415-424) changes size every SQP iteration
// and per problem.  In that row order
//     R_0 | R_1 H_0 | R_2 H_1 | ... | R_{N-1} H_{N-2} H_{N-1}
// (R_j the nx dynamics rows that define x_j, H_k knot k's hard rows) the groups
// touch the knot variables {0}, {0,1}, {1,2}, ..., so S is block-tridiagonal with
// VARIABLE block sizes: every row couples only with rows less than twice the
// largest group away.  S is therefore stored per problem in a row-start-relative band
// (ELL): row a's structurally nonzero columns c in [lo_a, hi_a] (rng) at [c - lo_a][a] of
// a [2W+1][dmax] array, so that the rows of a wave read their j-th entries as one
// contiguous 512-byte piece, and a wave walks only its longest row's entries.
// The reference's PCG preconditioner, however, cuts S into nx-aligned blocks from
// row 0 (n_blocks = floor(dim / nx), PCG.py:182-212), which no longer line up with
// the groups; it is reproduced exactly on the band (trailing dim mod nx rows have
// zero preconditioner rows, as in the reference).
//
// Kernels (one problem per workgroup except the per-knot row selection):
//   k_hard_rows     lane = (problem, knot): the knot's rows in the reference's order
//                   (TrajoptConstraint.value_hard_constraints / jacobian_hard_constraints,
//                   :53-128, 210-274): joint, velocity, torque; [z - lb; ub - z];
//                   ACTIVE_SET keeps the entries < 0, FULL_SET all of them
//   k_hard_layout   row offsets of the groups, dim, and a per-row table (kind, knot, index)
//   k_hard_schur    per row its G^-1-weighted coefficient pieces, then the S band and gamma
//   k_hard_pcg      preconditioner (0 / J / BJ / SS on nx-aligned blocks) + PCG (PCG.py:66-111)
//   k_hard_direct   method S: banded elimination (S negative definite: no pivoting); FULL_SET's
//                   zero rows get lambda = 0 (the reference's lstsq fallback, :431-436)
//   k_hard_dxu      dxu_k = Ghat_k (g_k - (C^T lambda)_k)
//   k_hard_ls       the hard terms of totalHardConstraintViolation (:286-293) per trial point
// Parity of these semantics is pinned for the 1-link arm by tests/golden/hard_*.npz.
//
// Summation order.  PCG on these Schur complements is order sensitive (the trailing dim mod nx rows
// have no preconditioner rows): two valid orders stop up to 5 iterations apart on the same S.  Every
// kernel of this file therefore rounds each product and sum on its own (fp contraction off below) and
// k_hard_pcg sums in the canonical order that oracle/hard.py pcg_canonical restates -- sequential
// sums from 0.0, per-thread dot partials over 1024 threads, a 64-lane xor butterfly, a fan-in over the
// 16 waves -- so that on identical S and gamma the two are bitwise equal (tests/test_gpu_hard.py).
#include "tmpc_internal.h"
#include "tmpc_pcg.h"

#include <algorithm>
#include <cstdlib>
#include <vector>

#pragma clang fp contract(off)

namespace tmpc {

__device__ __forceinline__ bool h_use_QF(const CostDev* C, int k, int N) {
  return (k == N - 1) || (C->QF_start >= 0 && k >= C->QF_start);
}

// the knot's rows in the reference order; returns the count (<= rmax).  slot (nullable) = t * 2 NJ + e,
// the row's (limit kind, entry of [z - lb; ub - z]); *mask (nullable) = the active-set bitmask of the
// knot, bit slot set for every violated entry (ACTIVE_SET's rows, FULL_SET's nonzero rows)
template <int NJ>
__device__ __forceinline__ int hard_knot_rows(const ConstrDev* __restrict__ Cs, const double* z, bool terminal,
                                              int rmax, int* col, double* sgn, double* val, int* slot = nullptr,
                                              unsigned long long* mask = nullptr) {
  int m = 0;
  unsigned long long bits = 0ull;
  for (int t = 0; t < 3; ++t) {
    const int hm = Cs->hard[t];
    if (hm == HARD_NONE || (t == 2 && terminal)) continue;
    for (int e = 0; e < 2 * NJ; ++e) {
      const int i = e < NJ ? e : e - NJ;
      const double zi = z[t * NJ + i];
      const double v = e < NJ ? zi - Cs->lb[t][i] : Cs->ub[t][i] - zi;
      const bool act = v < 0.0;
      if (hm == HARD_ACTIVE && !act) continue;
      if (act) bits |= 1ull << (t * 2 * NJ + e);
      if (m < rmax) {
        col[m] = t * NJ + i;
        sgn[m] = act ? (e < NJ ? 1.0 : -1.0) : 0.0;
        val[m] = v;
        if (slot) slot[m] = t * 2 * NJ + e;
      }
      ++m;
    }
  }
  if (mask) *mask = bits;
  return m;
}

template <int NJ>
__global__ void __launch_bounds__(256) k_hard_rows(const ConstrDev* __restrict__ Cs, int B, int N, int rmax,
                                                   const double* __restrict__ x, const double* __restrict__ u,
                                                   const int* __restrict__ active, int* __restrict__ cnt,
                                                   int* __restrict__ hcol, double* __restrict__ hsgn,
                                                   double* __restrict__ hval, int* __restrict__ hslot,
                                                   unsigned long long* __restrict__ amask,
                                                   const int* __restrict__ iter, int Wtr,
                                                   unsigned long long* __restrict__ tr_active) {
  constexpr int NX = 2 * NJ;
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= B * N) return;
  const int b = gid / N, k = gid - b * N;
  if (!active[b]) return;
  const int K = N - 1;
  double z[3 * NJ];
  for (int m = 0; m < NX; ++m) z[m] = x[((size_t)b * NX + m) * N + k];
  for (int m = 0; m < NJ; ++m) z[NX + m] = k < K ? u[((size_t)b * NJ + m) * K + k] : 0.0;
  const size_t o = (size_t)gid * rmax;
  unsigned long long bits;
  cnt[gid] = hard_knot_rows<NJ>(Cs, z, k == K, rmax, hcol + o, hsgn + o, hval + o, hslot + o, &bits);
  amask[gid] = bits;
  // the QP's active set in the trace row of this SQP iteration (row iter + 1, as k_ls_decide's)
  if (tr_active) tr_active[((size_t)b * Wtr + iter[b] + 1) * N + k] = bits;
}

// Row layout of one problem: roff[j] = first row of R_j, hoff[k] = first row of H_k, dim;
// per row: kind (0 dynamics / initial, 1 hard), knot (j for R_j, k for H_k), index.
__global__ void __launch_bounds__(64) k_hard_layout(int B, int N, int NX, int rmax, const int* __restrict__ active,
                                                    const int* __restrict__ cnt, int* __restrict__ roff,
                                                    int* __restrict__ hoff, int* __restrict__ dim,
                                                    int* __restrict__ rkind, int* __restrict__ rknot,
                                                    int* __restrict__ ridx, int dmax) {
  const int b = blockIdx.x;
  if (!active[b]) return;
  __shared__ int s_dim;
  int* ro = roff + (size_t)b * N;
  int* ho = hoff + (size_t)b * N;
  const int* cb = cnt + (size_t)b * N;
  if (threadIdx.x == 0) {
    int row = 0;
    ro[0] = 0;
    row = NX;
    for (int j = 1; j < N; ++j) {
      ro[j] = row;
      row += NX;
      ho[j - 1] = row;
      row += cb[j - 1];
    }
    ho[N - 1] = row;
    row += cb[N - 1];
    dim[b] = row;
    s_dim = row;
  }
  __syncthreads();
  int* rk = rkind + (size_t)b * dmax;
  int* rn = rknot + (size_t)b * dmax;
  int* ri = ridx + (size_t)b * dmax;
  for (int j = 0; j < N; ++j) {
    for (int i = threadIdx.x; i < NX; i += blockDim.x) {
      rk[ro[j] + i] = 0;
      rn[ro[j] + i] = j;
      ri[ro[j] + i] = i;
    }
    for (int i = threadIdx.x; i < cb[j]; i += blockDim.x) {
      rk[ho[j] + i] = 1;
      rn[ho[j] + i] = j;
      ri[ho[j] + i] = i;
    }
  }
  (void)s_dim;
}

// Ghat blocks: the three distinct QuadraticCost blocks [B][3][NX*NX] (Q, QF, R), or per knot
// [B][N][NX*NX + NU*NU] with soft limits (k_ginv / k_ginv_soft layouts)
template <int NJ>
struct HGhat {
  static constexpr int NX = 2 * NJ, NU = NJ, GS = NX * NX + NU * NU;
  const double* base;
  bool pk;
  __device__ __forceinline__ const double* x(const CostDev* C, int k, int N) const {
    return pk ? base + (size_t)k * GS : base + (h_use_QF(C, k, N) ? NX * NX : 0);
  }
  __device__ __forceinline__ const double* u(int k) const {
    return pk ? base + (size_t)k * GS + NX * NX : base + 2 * NX * NX;
  }
};

// the cost gradient g_k = [(x_k - xg)^T Q_k, u_k^T R] (+ soft jacobian; UrdfCost's x part in jsoft)
template <int NJ>
__device__ __forceinline__ double hard_grad(const CostDev* __restrict__ C, const double* xb, const double* ub,
                                            const double* js, int N, int k, int c) {
  constexpr int NX = 2 * NJ, NU = NJ;
  const int K = N - 1;
  double g = 0.0;
  if (c < NX) {
    if (C->kind == COST_EE) return js ? js[k * (NX + NU) + c] : 0.0;
    const double* Qk = h_use_QF(C, k, N) ? C->QF : C->Q;
    for (int m = 0; m < NX; ++m) g += (xb[m * N + k] - C->xg[m]) * Qk[m * NX + c];
  } else if (k < K) {
    for (int m = 0; m < NU; ++m) g += ub[m * K + k] * C->R[m * NU + (c - NX)];
  }
  if (js) g = g + js[k * (NX + NU) + c];
  return g;
}

// pointers typed with their address space (LDS / HBM): a plain pointer that may point to either makes
// every read through it a flat load
typedef __attribute__((address_space(3))) const double lds_cdouble;
typedef __attribute__((address_space(1))) const double glb_cdouble;
__device__ __forceinline__ lds_cdouble* lds_ptr(const double* p) { return (lds_cdouble*)p; }
__device__ __forceinline__ glb_cdouble* glb_ptr(const double* p) { return (glb_cdouble*)p; }

// piece p of row a: the knot and the coefficient vector over [x_knot; u_knot]
//   R_0 row i: (0, e_i);  R_j row i: (j-1, -[A_{j-1} B_{j-1}] row i), (j, e_i);  H_k row s: (k, sgn e_col)
template <int NJ>
__device__ __forceinline__ int row_piece(int kind, int knot, int idx, int p, const double* __restrict__ A,
                                         const double* __restrict__ Bm, const int* hcol, const double* hsgn,
                                         double (&cf)[3 * NJ]) {
  constexpr int NX = 2 * NJ, NU = NJ, NXU = NX + NU;
  // unit vectors by compare-select over the (unrolled) entries: no dynamic index into cf (no scratch)
  if (kind == 1) {
    const int col = hcol[idx];
    const double sg = hsgn[idx];
#pragma unroll
    for (int m = 0; m < NXU; ++m) cf[m] = m == col ? sg : 0.0;
    return p ? -1 : knot;
  }
  if (knot == 0 || p == 1) {
#pragma unroll
    for (int m = 0; m < NXU; ++m) cf[m] = m == idx ? 1.0 : 0.0;
    return (knot == 0 && p == 1) ? -1 : knot;
  }
  const double* Ak = A + (size_t)(knot - 1) * NX * NX;
  const double* Bk = Bm + (size_t)(knot - 1) * NX * NU;
  for (int m = 0; m < NX; ++m) cf[m] = -Ak[idx * NX + m];
  for (int m = 0; m < NU; ++m) cf[NX + m] = -Bk[idx * NU + m];
  return knot - 1;
}

// s_pk entry of one row piece: (knot + 1) | unit code << 16, the unit code 0 for a -[A B] row, else
// 1 + 3 uc + (uv > 0 ? 1 : uv < 0 ? 2 : 0) for the unit piece uv e_uc (uv = a hard row's sign or 1)
__device__ __forceinline__ int pk_pack(int kp, int uc, double uv) {
  return (kp + 1) | (uc < 0 ? 0 : 1 + 3 * uc + (uv > 0.0 ? 1 : (uv < 0.0 ? 2 : 0))) << 16;
}
__device__ __forceinline__ int pk_knot(int v) { return (v & 0xffff) - 1; }
__device__ __forceinline__ int pk_unit(int v) { return v >> 16; }
__device__ __forceinline__ int pk_uc(int code) { return (code - 1) / 3; }
__device__ __forceinline__ double pk_uv(int code) {
  const int sc = (code - 1) % 3;
  return sc == 1 ? 1.0 : (sc == 2 ? -1.0 : 0.0);
}

// the unit piece of row (kind, knot, idx), piece p (row_piece): its entry (-1: a -[A B] row or no piece)
__device__ __forceinline__ int piece_unit(int kind, int knot, int idx, int p, const int* hc, const double* hs,
                                          double& uv) {
  uv = 1.0;
  if (kind == 1) {
    if (p) return -1;
    uv = hs[idx];
    return hc[idx];
  }
  if (knot == 0) return p ? -1 : idx;
  return p ? idx : -1;
}

// S band and gamma.  Phase 1: per row and piece, Y = Ghat cf (global scratch [dmax][2][NXU] per
// problem); phase 2: S_ab = -sum over shared knots cf_a . Y_b, gamma_a = c_a - sum_p Y_a . g.
#ifndef TMPC_SCHUR_WPE
#define TMPC_SCHUR_WPE 1
#endif
// S entries per step of k_hard_schur's phase 2 (their Y loads in flight together): 2 (four measured the
// same at NJ = 6, profiles/r05/hard/probe_r05s.txt, at 254 VGPRs)
#ifndef TMPC_SCHUR_EPS
#define TMPC_SCHUR_EPS 2
#endif
// Y scratch layout: 1 (shipped) [2][NXU][dmax], a wave's rows consecutive: phase 1's writes coalesce
// (row-major [dmax][2][NXU], 0: Y 84k -> 63k cycles per problem, hard_schur 0.48 -> 0.43 ms per launch at
// B = 4096, profiles/r05/hard/probe_r05z.txt; while phase 2 read a full Y row per entry and piece the
// row-major layout was the faster one, probe_r05w_ytransposed_rejected.txt)
#ifndef TMPC_SCHUR_YT
#define TMPC_SCHUR_YT 1
#endif
#if TMPC_SCHUR_YT
#define Y_AT(row, q, m) Yb[((size_t)(q) * NXU + (m)) * dmax + (row)]
#else
#define Y_AT(row, q, m) Yb[((size_t)(row) * 2 + (q)) * NXU + (m)]
#endif
template <int NJ>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(TMPC_SCHUR_WPE))) k_hard_schur(const CostDev* __restrict__ C, int B, int N, int W, int dmax,
                                                    int rmax, const int* __restrict__ active,
                                                    const double* __restrict__ Ghat, int per_knot,
                                                    const double* __restrict__ Aall, const double* __restrict__ Ball,
                                                    const double* __restrict__ cvec, const double* __restrict__ x,
                                                    const double* __restrict__ u, const double* __restrict__ jsoft,
                                                    const int* __restrict__ dim, const int* __restrict__ rkind,
                                                    const int* __restrict__ rknot, const int* __restrict__ ridx,
                                                    const int* __restrict__ hoff, const int* __restrict__ hcol,
                                                    const double* __restrict__ hsgn, const double* __restrict__ hval,
                                                    double* __restrict__ Y, int* __restrict__ PK,
                                                    double* __restrict__ Sb, double* __restrict__ gam,
                                                    int* __restrict__ rng, const double* __restrict__ gvec) {
#if TMPC_HX_STAMPS
  unsigned long long sc_[4] = {}, sc_prev_ = __builtin_amdgcn_s_memtime();
#define HS_STAMP(i_) { const unsigned long long n_ = __builtin_amdgcn_s_memtime(); sc_[i_] += n_ - sc_prev_; sc_prev_ = n_; }
#else
#define HS_STAMP(i_)
#endif
  constexpr int NX = 2 * NJ, NU = NJ, NXU = NX + NU;
  extern __shared__ double s_grad[];   // [N][NXU] cost gradient per knot, then s_piece
  int* s_piece = reinterpret_cast<int*>(s_grad + N * NXU);   // [N] first row, [N] last row touching each knot piece
  int* s_pk = s_piece + 2 * N;   // [dmax][2] each row's piece knots (PK), read by phase 2 for every S entry
  const int b = blockIdx.x;
  if (!active[b]) return;
  const int K = N - 1;
  const int D = dim[b];
  const double* A = Aall + (size_t)b * K * NX * NX;
  const double* Bm = Ball + (size_t)b * K * NX * NU;
  const double* xb = x + (size_t)b * NX * N;
  const double* ub = u + (size_t)b * NU * K;
  const double* js = jsoft ? jsoft + (size_t)b * N * NXU : nullptr;
  const HGhat<NJ> Gh{per_knot ? Ghat + (size_t)b * N * HGhat<NJ>::GS : Ghat + (size_t)b * 3 * NX * NX, per_knot != 0};
  // per_knot 2: the plugin-hook QP's full (G_k + rho I)^-1 blocks [N][NXU][NXU] (x-u coupling; the terminal
  // knot's NX x NX block top-left, k_ghat_full) and the caller's gradient gvec [N][NXU]
  const double* Gf = Ghat + (size_t)b * N * NXU * NXU;
  const int* rk = rkind + (size_t)b * dmax;
  const int* rn = rknot + (size_t)b * dmax;
  const int* ri = ridx + (size_t)b * dmax;
  double* Yb = Y + (size_t)b * dmax * 2 * NXU;
  int* PKb = PK + (size_t)b * dmax * 2;
  const size_t hb = (size_t)b * N * rmax;
  // phase 0: the cost gradient of every knot (0 for the terminal knot's u part)
  for (int e = threadIdx.x; e < N * NXU; e += blockDim.x) {
    const int k = e / NXU, m = e - k * NXU;
    s_grad[e] = (m < NX || k < K) ? (gvec ? gvec[(size_t)b * N * NXU + e] : hard_grad<NJ>(C, xb, ub, js, N, k, m))
                                  : 0.0;
  }
  __syncthreads();
  HS_STAMP(0);
  // phase 1.  With one shared Ghat (no per-knot soft blocks: Q, QF and R blocks, 2 NX^2 + NU^2 doubles)
  // the rows read it from an LDS copy; per-knot blocks stay in HBM.  (From HBM, each row's 2 x 18 Ghat
  // row loads were dependent round trips.)
  double* s_gh = reinterpret_cast<double*>(s_pk + ((dmax * 2 + 3) & ~3));
  constexpr int GH = 2 * NX * NX + NU * NU;
  if (!per_knot) {
    for (int e = threadIdx.x; e < GH; e += blockDim.x) s_gh[e] = Ghat[(size_t)b * 3 * NX * NX + e];
    __syncthreads();
  }
  auto phase1 = [&](auto gx_of, auto gu_of) {
    for (int a = threadIdx.x; a < D; a += blockDim.x) {
      const int kind = rk[a], knot = rn[a], idx = ri[a];
      const int* hc = hcol + hb + (size_t)knot * rmax;
      const double* hs = hsgn + hb + (size_t)knot * rmax;
      double g_dot = 0.0;
      for (int p = 0; p < 2; ++p) {
        double cf[3 * NJ];
        const int kp = row_piece<NJ>(kind, knot, idx, p, A, Bm, hc, hs, cf);
        PKb[a * 2 + p] = kp;
        double uv;
        const int uc = piece_unit(kind, knot, idx, p, hc, hs, uv);
        s_pk[a * 2 + p] = pk_pack(kp, uc, uv);
        if (kp < 0) continue;
        // y = Ghat_kp cf (terminal knot: x block only), written out row by row, and s = y . g in the
        // same order; the row loops stay rolled so one Ghat row's loads are live at a time
        double* yo = &Y_AT(a, p, 0);
        const size_t ys = TMPC_SCHUR_YT ? (size_t)dmax : 1;   // the stride of the entries
        const double* gk = s_grad + kp * NXU;
        const auto Gx = gx_of(kp);
        double s = 0.0;
#pragma unroll 1
        for (int r = 0; r < NX; ++r) {
          double acc = 0.0;
#pragma unroll
          for (int c = 0; c < NX; ++c) acc += Gx[r * NX + c] * cf[c];
          yo[r * ys] = acc;
          s += acc * gk[r];
        }
        const auto Gu = gu_of(kp);
#pragma unroll 1
        for (int r = 0; r < NU; ++r) {
          double acc = 0.0;
          if (kp < K) {
#pragma unroll
            for (int c = 0; c < NU; ++c) acc += Gu[r * NU + c] * cf[NX + c];
          }
          yo[(NX + r) * ys] = acc;
          s += acc * gk[NX + r];
        }
        g_dot += s;
      }
      double ca;
      if (kind == 0) ca = cvec[((size_t)b * N + knot) * NX + idx];
      else ca = hval[hb + (size_t)knot * rmax + idx];
      gam[(size_t)b * dmax + a] = ca - g_dot;
    }
  };
  if (per_knot == 2) {   // full blocks: y = Ghat_kp cf over all NXU entries (terminal: the NX x NX block)
    for (int a = threadIdx.x; a < D; a += blockDim.x) {
      const int kind = rk[a], knot = rn[a], idx = ri[a];
      const int* hc = hcol + hb + (size_t)knot * rmax;
      const double* hs = hsgn + hb + (size_t)knot * rmax;
      double g_dot = 0.0;
      for (int p = 0; p < 2; ++p) {
        double cf[3 * NJ];
        const int kp = row_piece<NJ>(kind, knot, idx, p, A, Bm, hc, hs, cf);
        PKb[a * 2 + p] = kp;
        double uv;
        const int uc = piece_unit(kind, knot, idx, p, hc, hs, uv);
        s_pk[a * 2 + p] = pk_pack(kp, uc, uv);
        if (kp < 0) continue;
        double* yo = &Y_AT(a, p, 0);
        const size_t ys = TMPC_SCHUR_YT ? (size_t)dmax : 1;
        const double* gk = s_grad + kp * NXU;
        glb_cdouble* G = glb_ptr(Gf + (size_t)kp * NXU * NXU);
        const int m = kp < K ? NXU : NX;
        double s = 0.0;
#pragma unroll 1
        for (int r = 0; r < NXU; ++r) {
          double acc = 0.0;
          if (r < m) {
#pragma unroll
            for (int c = 0; c < NXU; ++c)
              if (c < m) acc += G[r * NXU + c] * cf[c];
          }
          yo[r * ys] = acc;
          s += acc * gk[r];
        }
        g_dot += s;
      }
      double ca;
      if (kind == 0) ca = cvec[((size_t)b * N + knot) * NX + idx];
      else ca = hval[hb + (size_t)knot * rmax + idx];
      gam[(size_t)b * dmax + a] = ca - g_dot;
    }
  } else if (!per_knot) {
    lds_cdouble* gl = lds_ptr(s_gh);
    phase1([&](int kp) { return gl + (h_use_QF(C, kp, N) ? NX * NX : 0); }, [&](int) { return gl + 2 * NX * NX; });
  } else {
    phase1([&](int kp) { return glb_ptr(Gh.x(C, kp, N)); }, [&](int kp) { return glb_ptr(Gh.u(kp)); });
  }
  HS_STAMP(1);
  // the rows of each knot piece: S_ac is structurally nonzero only where rows a and c share a piece,
  // so row a's nonzeros lie in [min, max] of the rows of its pieces -- a much narrower range than
  // the worst-case band W, which the PCG's products and the elimination then stay inside
  for (int k = threadIdx.x; k < N; k += blockDim.x) {
    s_piece[k] = D;
    s_piece[N + k] = -1;
  }
  __syncthreads();
  for (int a = threadIdx.x; a < D; a += blockDim.x)
    for (int p = 0; p < 2; ++p) {
      const int kp = pk_knot(s_pk[a * 2 + p]);
      if (kp < 0) continue;
      atomicMin(&s_piece[kp], a);
      atomicMax(&s_piece[N + kp], a);
    }
  __syncthreads();
  int* rb = rng + (size_t)b * dmax * 2;
  for (int a = threadIdx.x; a < D; a += blockDim.x) {
    int lo = a, hi = a;
    for (int p = 0; p < 2; ++p) {
      const int kp = pk_knot(s_pk[a * 2 + p]);
      if (kp < 0) continue;
      lo = min(lo, s_piece[kp]);
      hi = max(hi, s_piece[N + kp]);
    }
    lo = max(lo, max(0, a - W));
    hi = min(hi, min(D - 1, a + W));
    rb[2 * a] = lo;
    rb[2 * a + 1] = hi;
  }
  __syncthreads();
  // phase 2: the band inside the row ranges, row a, column c = lo_a + j (stored at [j][a]); entries
  // outside the ranges are never read (band_at / the PCG product / k_hard_direct's copy).  Each thread
  // keeps its row's two coefficient vectors in registers and the wave walks j up to its longest row (the
  // stores of one j are contiguous); S_ac = -(sum over pieces p of a, q of c on one knot of cf_ap . Y_cq)
  HS_STAMP(2);
  const int BW = 2 * W + 1;
  double* S = Sb + (size_t)b * dmax * BW;
  for (int a0 = threadIdx.x & ~63; a0 < D; a0 += blockDim.x) {   // wave-uniform: the wave's first row
    const int a = a0 + (threadIdx.x & 63);
    const bool own = a < D;
    double cf0[3 * NJ];   // piece 0's coefficients (piece 1 is always a unit piece, or none: row_piece)
    int kp0 = -1, kp1 = -1, ol = BW, oh = -1;
    // the unit pieces (row_piece: e_idx, or sgn e_col for a hard row): entry uc of cf, value uv (-1: a
    // -[A B] row, the full product)
    int uc0 = -1, uc1 = -1;
    double uv0 = 0.0, uv1 = 0.0;
    if (own) {
      const int kind = rk[a], knot = rn[a], idx = ri[a];
      const int* hc = hcol + hb + (size_t)knot * rmax;
      const double* hs = hsgn + hb + (size_t)knot * rmax;
      kp0 = row_piece<NJ>(kind, knot, idx, 0, A, Bm, hc, hs, cf0);
      kp1 = kind == 1 || knot == 0 ? -1 : knot;   // row_piece(.., p = 1, ..)
      uc0 = piece_unit(kind, knot, idx, 0, hc, hs, uv0);
      uc1 = piece_unit(kind, knot, idx, 1, hc, hs, uv1);
      ol = 0;
      oh = rb[2 * a + 1] - rb[2 * a];
    }
    int l = ol, h = oh;
    for (int off = 32; off > 0; off >>= 1) {
      l = min(l, __shfl_xor(l, off, 64));
      h = max(h, __shfl_xor(h, off, 64));
    }
    l = __builtin_amdgcn_readfirstlane(l);
    h = __builtin_amdgcn_readfirstlane(h);
    // EPS entries per step, each piece's Y vectors of all of them loaded together (per entry and piece a
    // dependent HBM round trip kept one Y vector in flight per lane); S_ac = -(sum over the pieces p of a,
    // in order, of cf_ap . Y_cq for the piece q of c on a's knot kp_p), zero past the row up to the wave's
    // longest row (k_hard_pcg's products read it: exact zeros)
    constexpr int EPS = TMPC_SCHUR_EPS;
    const int lo_a = own ? rb[2 * a] : 0;
    for (int o = l; o <= h; o += EPS) {
      bool in[EPS];
      int pc0[EPS], pc1[EPS];
      double sm[EPS];
#pragma unroll
      for (int e = 0; e < EPS; ++e) {
        in[e] = own && o + e <= oh;
        const int c = lo_a + o + e;
        pc0[e] = in[e] ? s_pk[c * 2] : -1;   // packed (pk_pack); -1: no entry
        pc1[e] = in[e] ? s_pk[c * 2 + 1] : -1;
        sm[e] = 0.0;
      }
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int kp = p ? kp1 : kp0;
        const int uc = p ? uc1 : uc0;
        int q[EPS];
#pragma unroll
        for (int e = 0; e < EPS; ++e)
          q[e] = kp < 0 || pc0[e] < 0 ? -1 : (pk_knot(pc0[e]) == kp ? 0 : (pk_knot(pc1[e]) == kp ? 1 : -1));
        if (uc >= 0) {
          // a unit piece: of the product's sequential chain from +0 (d += cf_m y_m) only the one nonzero
          // term changes d, so d = uv y_uc + 0 exactly (for finite Y): one Y load instead of NXU
          const double uv = p ? uv1 : uv0;
          double yv[EPS];
#pragma unroll
          for (int e = 0; e < EPS; ++e) yv[e] = q[e] >= 0 ? Y_AT(lo_a + o + e, q[e], uc) : 0.0;
#pragma unroll
          for (int e = 0; e < EPS; ++e)
            if (q[e] >= 0) sm[e] += uv * yv[e] + 0.0;
        } else if (p == 0) {
          // a -[A B] row (piece 0 only).  Where c's piece is the unit uv e_uc, cf_ap . Y_cq = uv (Ghat cf_ap)_uc = uv Y_ap[uc]
          // (Ghat symmetric), one entry of row a's own Y; else the full product with c's Y vector
          double v[EPS][NXU], dv[EPS];
          bool full[EPS];
#pragma unroll
          for (int e = 0; e < EPS; ++e) {
            const int code = q[e] < 0 ? 0 : pk_unit(q[e] ? pc1[e] : pc0[e]);
            full[e] = q[e] >= 0 && code == 0;
            dv[e] = code ? pk_uv(code) * Y_AT(a, p, pk_uc(code)) + 0.0 : 0.0;
          }
#pragma unroll
          for (int e = 0; e < EPS; ++e) {
            if (full[e]) {
#pragma unroll
              for (int m = 0; m < NXU; ++m) v[e][m] = Y_AT(lo_a + o + e, q[e], m);
            }
          }
#pragma unroll
          for (int e = 0; e < EPS; ++e) {
            if (full[e]) {
              double d = 0.0;
#pragma unroll
              for (int m = 0; m < NXU; ++m) d += cf0[m] * v[e][m];
              sm[e] += d;
            } else if (q[e] >= 0) {
              sm[e] += dv[e];
            }
          }
        }
      }
#pragma unroll
      for (int e = 0; e < EPS; ++e)
        if (own && o + e <= h) S[(size_t)(o + e) * dmax + a] = o + e <= oh ? -sm[e] : 0.0;
    }
  }
  HS_STAMP(3);
#if TMPC_HX_STAMPS
  if (b == 0 && (threadIdx.x & 63) == 0)
    printf("hs_stamps wave %d D %d: grad %llu Y %llu ranges %llu S %llu\n", (int)(threadIdx.x >> 6), D, sc_[0], sc_[1],
           sc_[2], sc_[3]);
#endif
#undef HS_STAMP
#undef Y_AT
}

#ifndef TMPC_HX_NOSTREAM
#define TMPC_HX_NOSTREAM 0
#endif
#ifndef TMPC_HX_NOPREC
#define TMPC_HX_NOPREC 0
#endif
#ifndef TMPC_HX_STAMPS
#define TMPC_HX_STAMPS 0
#endif

// band entries of each slot-0 row (its first ones) k_hard_pcg holds in registers for the whole solve:
// 24 (48 VGPRs of its 128); fewer where that spills (nx = 8, 14: 20; nx = 2, 4: 16; 8 fewer in the three- and
// four-slot instances, which hold x of three / four rows)
#ifndef TMPC_HARD_REG
#define TMPC_HARD_REG 24
#endif
// streamed band entries per batch of loads in k_hard_pcg's product
#ifndef TMPC_HARD_U
#define TMPC_HARD_U 8
#endif
__host__ __device__ constexpr int hard_pcg_reg_diag(int nx, int slots) {
  return (nx <= 4 ? 16 : (nx >= 14 || nx == 8 ? TMPC_HARD_REG - 4 : TMPC_HARD_REG)) - (slots >= 3 ? 8 : 0);
}

// doubles of LDS k_hard_pcg uses before its reduction slots: r and p of dmax rows, z and S p of the rows
// past slot 0 (slot 0's are registers), and at least four nx x nx blocks (with their pivot rows /
// columns) for the preconditioner setup
// (p is followed by HARD_PCG_GUARD zeros: the register-held band entries past a row read them)
constexpr int HARD_PCG_GUARD = 24;
__host__ __device__ constexpr int hard_pcg_scratch(int dmax, int nx) {
  return 2 * dmax + HARD_PCG_GUARD + 2 * (dmax > HARD_PCG_THREADS ? dmax - HARD_PCG_THREADS : 0) >
                 4 * (nx * nx + 2 * nx)
             ? 2 * dmax + HARD_PCG_GUARD + 2 * (dmax > HARD_PCG_THREADS ? dmax - HARD_PCG_THREADS : 0)
             : 4 * (nx * nx + 2 * nx);
}
// doubles before k_hard_pcg's preconditioner-block cache: the scratch, 2 x 16 reduction slots, the rows'
// and the wave-slots' diagonal ranges (ints)
// (rounded up to 16 bytes: the cached blocks are read as 16-byte pieces)
__host__ __device__ constexpr int hard_pcg_cache_offset(int D, int nx, int slots) {
  return (hard_pcg_scratch(D, nx) + 32 + (D + 2 * slots * (HARD_PCG_THREADS / 64) + 1) / 2 + 1) & ~1;
}

// ---- workgroup sum (deterministic): wave DPP butterfly via shuffles + fixed-order fan-in
// Double-buffered form for a sequence of sums (k_hard_pcg): sum number k uses slots red[16 (k & 1) ..],
// so the barrier that protects a slot set from being overwritten while a slow wave still reads it is
// the NEXT sum's own barrier -- one barrier per sum instead of two.
// The 64-lane xor butterfly v += v[l ^ off] for off = 32, 16, 8, 4, 2, 1 (oracle/hard.py _dot) on the
// VALU: permlane swaps (32, 16), DPP row_ror:8, row_shl:4 / row_shr:4 picked by lane bit 2, quad_perm
// (2, 1).  Each step adds the same two values as the shuffle form (addition commutes), so the sums
// are bitwise those of __shfl_xor, without its six ds_bpermute round trips through the LDS unit.
#ifndef TMPC_HARD_DPP
#define TMPC_HARD_DPP 1
#endif
__device__ __forceinline__ double h_wave_butterfly(double v) {
#if TMPC_HARD_DPP
  v = perm_pair_sum32(v);
  v = perm_pair_sum16(v);
  v += dpp_get<0x128, 0xf>(v);   // row_ror:8: lane l reads l ^ 8
  {
    const double up = dpp_get<0x104, 0xf>(v);   // row_shl:4: lane l reads l + 4 (lanes with bit 2 clear)
    const double dn = dpp_get<0x114, 0xf>(v);   // row_shr:4: lane l reads l - 4 (bit 2 set)
    v += (threadIdx.x & 4) ? dn : up;
  }
  v += dpp_get<0x4E, 0xf>(v);    // quad_perm [2,3,0,1]: l ^ 2
  v += dpp_get<0xB1, 0xf>(v);    // quad_perm [1,0,3,2]: l ^ 1
#else
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
#endif
  return v;
}

// (k_hard_pcg's HARD_PCG_THREADS workgroup: the fan-in over its 16 waves unrolled)
__device__ __forceinline__ double h_block_sum_db(double v, double* red, int& k) {
  constexpr int NW = HARD_PCG_THREADS / 64;
  v = h_wave_butterfly(v);
  const int w = threadIdx.x >> 6;
  double* rs = red + 16 * (k & 1);
  ++k;
  if ((threadIdx.x & 63) == 0) rs[w] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < NW; ++i) s += rs[i];
  return s;
}
__device__ __forceinline__ double h_block_sum(double v, double* red) {
  v = h_wave_butterfly(v);
  const int w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
  for (int i = 0; i < nw; ++i) s += red[i];
  return s;
}

// A preconditioner block's row / column from the LDS cache or from HBM, through pointers typed with
// their address space: a plain pointer that may point to either (or two branches the compiler merges)
// makes every read a flat load, issued one at a time here.  s += M_ij r_j in j order (canonical).
// The LDS copies of the preconditioner blocks are row-major with each row's 16-byte pieces swizzled:
// piece c of row i of block k sits at c ^ sw, sw = bit 3 of the global row k NX + i (NX a multiple of 4,
// so that c ^ 1 stays in the row).  A wave reads its rows' pieces with ds_read_b128: the 16 lanes of a
// lane group hold 16 consecutive global rows mod 16, which the swizzle spreads over all 64 banks
// (unswizzled, rows r and r + 8 share banks: two LDS cycles per piece instead of one).
template <int NX>
__device__ __forceinline__ int hp_swz(int k, int i) {
  return NX % 4 == 0 ? ((k * NX + i) >> 3) & 1 : 0;
}
// offset of element (i, j) of block k in the swizzled layout
template <int NX>
__device__ __forceinline__ int hp_off(int k, int i, int j) {
  return k * NX * NX + i * NX + ((((j >> 1) ^ hp_swz<NX>(k, i)) << 1) | (j & 1));
}
// s += P_ij r_j over row i of block k of the swizzled LDS copy (16-byte pieces, j in order)
template <int NX>
__device__ __forceinline__ double hp_row_lds(const double* base, int k, int i, const double* r, double s) {
  typedef double d2v __attribute__((ext_vector_type(2)));
  typedef __attribute__((address_space(3))) const d2v lds_cd2v;
  lds_cd2v* row = (lds_cd2v*)(base + (size_t)k * NX * NX + i * NX);
  const int sw = hp_swz<NX>(k, i);
#pragma unroll
  for (int c = 0; c < NX / 2; ++c) {
    const d2v m = row[c ^ sw];
    s += m.x * r[2 * c];
    s += m.y * r[2 * c + 1];
  }
  return s;
}
// s += P_ji r_j over column i of block k of the swizzled LDS copy
template <int NX>
__device__ __forceinline__ double hp_col_lds(const double* base, int k, int i, const double* r, double s) {
  lds_cdouble* blk = lds_ptr(base);
#pragma unroll
  for (int j = 0; j < NX; ++j) s += blk[hp_off<NX>(k, j, i)] * r[j];
  return s;
}

// column i of M (row-major M, i.e. M_ji for j = 0 ..): the transposed blocks
template <int NX, class P>
__device__ __forceinline__ double hp_col(P M, int i, const double* r, double s) {
#pragma unroll
  for (int j = 0; j < NX; ++j) s += M[j * NX + i] * r[j];
  return s;
}
// row i of M
template <int NX, class P>
__device__ __forceinline__ double hp_row(P M, int i, const double* r, double s) {
#pragma unroll
  for (int j = 0; j < NX; ++j) s += M[i * NX + j] * r[j];
  return s;
}

// S_rc from the (row-start-relative) band; zero outside row r's structural range rg[2r .. 2r+1]
__device__ __forceinline__ double band_at(const double* S, const int* rg, int dmax, int r, int c) {
  return (c >= rg[2 * r] && c <= rg[2 * r + 1]) ? S[(size_t)(c - rg[2 * r]) * dmax + r] : 0.0;
}

// Preconditioner (compute_preconditioner on the dense S, PCG.py:113-212) + PCG (:66-111).
// Pd [nb][NX][NX] diagonal inverses, Pl [nb-1][NX][NX] = P_{k+1,k} (P_{k,k+1} = Pl[k]^T: the
// reference copies transposes); Ptr holds the transposed diagonal blocks (column j contiguous).  P^-1 r
// reads P_kk from Ptr and P_{k,k+1} = Pl[k]^T column-wise (both coalesced) and P_{k,k-1} = Pl[k-1]
// row-wise: the lines of Pl[k-1] are the ones block row k-1 reads in the same pass, so they come from
// cache, and Pl streams from HBM once per iteration instead of twice.
// Thread t owns rows t, t + 1024, ... (slot m = row / 1024 < SLOTS; one 16-wave workgroup per problem,
// so one problem's product has a whole CU's loads in flight): x of its rows stays in its registers;
// r and p, which other rows read, and z and S p are in LDS (4 D doubles), and the rest of the CU's LDS
// holds as many preconditioner blocks as fit.
// Every global read of the iterations is coalesced: S p walks the wave's diagonals of the band (each
// lane adds the diagonals inside its row's range, in column order), and the preconditioner rows are read
// from the transposed blocks.  Every sum keeps the canonical order (oracle/hard.py pcg_canonical).
template <int NX, int SLOTS>
__global__ void __launch_bounds__(HARD_PCG_THREADS) k_hard_pcg(int B, int W, int dmax, int precond,
                                                              const int* __restrict__ active,
                                                              const int* __restrict__ dim, const double* __restrict__ Sb,
                                                              const double* __restrict__ gam, double tol, int max_iter,
                                                              double* __restrict__ Pd, double* __restrict__ Pl,
                                                              double* __restrict__ Ptr,
                                                              double* __restrict__ lam, int* __restrict__ iters,
                                                              const int* __restrict__ rng, double* __restrict__ work,
                                                              int lds_bytes) {
  constexpr int REG = hard_pcg_reg_diag(NX, SLOTS);
  const int b = blockIdx.x;
  if (!active[b]) return;
#if TMPC_HX_STAMPS
  unsigned long long su_[8] = {}, su_prev_ = __builtin_amdgcn_s_memtime();
#define HX_SETUP(i_) { const unsigned long long n_ = __builtin_amdgcn_s_memtime(); su_[i_] += n_ - su_prev_; su_prev_ = n_; }
#else
#define HX_SETUP(i_)
#endif
  const int D = dim[b];
  const int BW = 2 * W + 1;
  const int nb = D / NX;
  const int t = threadIdx.x;
  const double* S = Sb + (size_t)b * dmax * BW;
  const int* rg = rng + (size_t)b * dmax * 2;
  const size_t nbmax = dmax / NX + 1;
  double* P = Pd + (size_t)b * nbmax * NX * NX;
  double* PL = Pl + (size_t)b * nbmax * NX * NX;
  double* PT = Ptr + (size_t)b * nbmax * NX * NX;
  // LDS (the whole allotment, lds_bytes; one workgroup per CU), laid out for this problem's D:
  //   r, p of the rows [2][D], z, S p of the rows past slot 0 [2][D - 1024] (read and written by the
  //   owner only; slot 0's live in registers) -- the setup's staging area before; 16 reduction slots; each row's diagonal range; each wave-slot's union;
  //   then as many preconditioner blocks as fit, transposed diagonal blocks first (ncd of them), then
  //   stair blocks Pl (ncl): those never stream from HBM during the iterations
  constexpr int B2 = NX * NX;
  extern __shared__ __align__(16) double sh[];
  double* rv = sh;
  double* pv = rv + D;
  const int ext = D > HARD_PCG_THREADS ? D - HARD_PCG_THREADS : 0;
  double* zl = pv + D + HARD_PCG_GUARD - HARD_PCG_THREADS;   // zl[a], al[a] for a >= 1024 only
  double* al = zl + ext;
  double* red = sh + hard_pcg_scratch(D, NX);
  int* rlh = reinterpret_cast<int*>(red + 32);   // [D] each row's last entry | first column << 16
  int* wlh = rlh + D;                            // [SLOTS][16 waves] each wave-slot's longest row (last entry)
  double* pcache = sh + hard_pcg_cache_offset(D, NX, SLOTS);
  const bool blocks = precond == PRECOND_BJ || precond == PRECOND_SS;
  const int ncap = max(0, (int)(lds_bytes / sizeof(double)) - hard_pcg_cache_offset(D, NX, SLOTS)) / B2;
  const int ncd = blocks ? min(nb, ncap) : 0;
  const int ncl = precond == PRECOND_SS && nb > 1 ? min(nb - 1, ncap - ncd) : 0;
  double* pcd = pcache;                    // [ncd][NX][NX] = PT blocks
  double* pcl = pcache + (size_t)ncd * B2; // [ncl][NX][NX] = Pl blocks
  if (blocks) {
    // The setup runs on the whole workgroup, element-parallel, staged in the LDS that r, p, z, S p use
    // later: each element of a block keeps the canonical (oracle/hard.py) operation sequence, so the
    // blocks equal the oracle's bit for bit.
    // (1) diagonal blocks: Gauss-Jordan on the augmented [M | I] without pivoting (oracle/hard.py
    //     _gj_inverse).  One row of one block per thread, in registers, each block inside one wave (64 / NX
    //     whole blocks per wave): per pivot p the owner of each block's row p scales it into LDS and every
    //     other row of the block takes it in with its own column-p entry as the snapshot -- the operation
    //     sequence of every element is the oracle's.  A wave's LDS accesses complete in order, so a pivot
    //     needs no workgroup barrier.  (Element-parallel through LDS with two barriers per pivot it took
    //     ~110k cycles at D = 768, profiles/r05/hard/stamps_r05m_setup.txt; rows in registers with one
    //     workgroup barrier per pivot ~35k, stamps_r05t.)
    constexpr int BPW = 64 / NX;                          // whole blocks per wave
    constexpr int BPP = (HARD_PCG_THREADS / 64) * BPW;    // blocks per pass
    const int lane = t & 63, bw = lane / NX, i = lane - bw * NX;
    const int kkp = (t >> 6) * BPW + bw;                  // this thread's block within the pass
    for (int k0 = 0; k0 < nb; k0 += BPP) {
      const int k = k0 + kkp;
      const bool own = bw < BPW && k < nb;
      double* pr = sh + (size_t)kkp * NX;   // the block's pivot row (scratch: at most D doubles per pass)
      double m[NX];
      if (own) {   // row i of S_kk (band_at), the row's range read once and its NX loads in flight together
        const int a = k * NX + i;
        const int lo = rg[2 * a], hi = rg[2 * a + 1];
#pragma unroll
        for (int j = 0; j < NX; ++j) {
          const int c = k * NX + j;
          const double v = S[(size_t)min(max(c - lo, 0), BW - 1) * dmax + a];
          m[j] = (c >= lo && c <= hi) ? v : 0.0;
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      HX_SETUP(4);
#pragma unroll
      for (int p = 0; p < NX; ++p) {
        if (own && i == p) {
          const double d = m[p];
#pragma unroll
          for (int j = 0; j < NX; ++j) {
            m[j] = (j == p) ? 1.0 / d : m[j] / d;
            pr[j] = m[j];
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (own && i != p) {
          const double f = m[p];
#pragma unroll
          for (int j = 0; j < NX; ++j) m[j] = ((j == p) ? 0.0 : m[j]) - f * pr[j];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
      HX_SETUP(5);
      if (own) {   // P_kk: its LDS copy where cached, else in HBM row-major (stairs) and transposed (P^-1 r)
#pragma unroll
        for (int j = 0; j < NX; ++j) {
          if (k < ncd) {
            pcd[hp_off<NX>(k, i, j)] = m[j];
          } else {
            P[(size_t)k * B2 + i * NX + j] = m[j];
            PT[(size_t)k * B2 + j * NX + i] = m[j];
          }
        }
      }
      __syncthreads();   // (the next pass reuses the pivot rows)
    }
    HX_SETUP(0);
    // (2) SS stair blocks (oracle/hard.py _neg_triple, both products summed in index order):
    //     odd k: P_{k,k-1} = -P_kk (S_{k,k-1} P_{k-1,k-1}); even k: P_{k-1,k} = -P_{k-1,k-1} (S_{k-1,k}
    //     P_kk), stored transposed.  Pl[k-1] = P_{k,k-1} row-major.  Per pass, one thread per (stair,
    //     row) stages row `rr` of Y = S_{yr,yc} in LDS (the row's range once, its NX loads together) --
    //     for the stairs the LDS block cache holds, in their own cache slots, which their results
    //     overwrite once every read is done; the others in the scratch -- then the same thread forms
    //     column c = rr of X (Y Z) from LDS (Y, and P_kk's cached copy where present), each yz_mc and each
    //     acc_rc summed in index order.  (With every Y entry read from HBM by its consumer it took
    //     180-230k cycles at D = 768, profiles/r05/hard/stamps_r05m_setup.txt.)
    if (precond == PRECOND_SS && nb > 1) {
      __syncthreads();   // P (global, this workgroup) and its LDS copies written
      constexpr int SPP = HARD_PCG_THREADS / NX;
      const int scap = hard_pcg_scratch(D, NX) / B2;
      for (int s0 = 0; s0 < nb - 1;) {
        const bool cached = s0 < ncl;
        const int s1 = cached ? min(ncl, s0 + SPP) : min(nb - 1, s0 + min(SPP, scap));
        double* stage = cached ? pcl + (size_t)s0 * B2 : sh;
        const int q = t / NX, rr = t - q * NX;
        const bool act = q < s1 - s0;
        const int k = s0 + q + 1;
        const bool odd = k & 1;
        const int yr = odd ? k : k - 1, yc = odd ? k - 1 : k;   // Y = S_{yr, yc}
        const int zk = odd ? k - 1 : k, xk = odd ? k : k - 1;   // Z, X = P_zk, P_xk
        double* Yq = stage + (size_t)q * B2;
        if (act) {
          const int a = yr * NX + rr;
          const int lo = rg[2 * a], hi = rg[2 * a + 1];
#pragma unroll
          for (int l = 0; l < NX; ++l) {
            const int col = yc * NX + l;
            const double v = S[(size_t)min(max(col - lo, 0), BW - 1) * dmax + a];
            Yq[rr * NX + l] = (col >= lo && col <= hi) ? v : 0.0;   // band_at
          }
        }
        __syncthreads();
        HX_SETUP(6);
        double acc[NX];
        if (act) {
          double z[NX];
          if (zk < ncd) {
#pragma unroll
            for (int l = 0; l < NX; ++l) z[l] = pcd[hp_off<NX>(zk, l, rr)];
          } else {
#pragma unroll
            for (int l = 0; l < NX; ++l) z[l] = P[(size_t)zk * B2 + l * NX + rr];
          }
#pragma unroll
          for (int r = 0; r < NX; ++r) acc[r] = 0.0;
#pragma unroll 1
          for (int m = 0; m < NX; ++m) {
            double yz = 0.0;
#pragma unroll
            for (int l = 0; l < NX; ++l) yz += Yq[m * NX + l] * z[l];
            if (xk < ncd) {   // (separate loops: a select between the LDS and the HBM copy made flat loads)
#pragma unroll
              for (int r = 0; r < NX; ++r) acc[r] += pcd[hp_off<NX>(xk, r, m)] * yz;
            } else {
#pragma unroll
              for (int r = 0; r < NX; ++r) acc[r] += P[(size_t)xk * B2 + r * NX + m] * yz;
            }
          }
        }
        HX_SETUP(7);
        __syncthreads();   // every read of this pass's staged Y done
        if (act) {
#pragma unroll
          for (int r = 0; r < NX; ++r) {
            const double v = -acc[r];
            const int pr = odd ? r : rr, pc = odd ? rr : r;   // element of P_{k,k-1}
            if (k - 1 < ncl) pcl[hp_off<NX>(k - 1, pr, pc)] = v;   // cached: LDS only
            else PL[(size_t)(k - 1) * B2 + pr * NX + pc] = v;
          }
        }
        s0 = s1;
      }
    }
    __syncthreads();
  }
  HX_SETUP(1);
  // z = P^-1 r for row a (r read from LDS)
  auto apply_P = [&](int a) -> double {
    if (precond == PRECOND_NONE || TMPC_HX_NOPREC) return rv[a];
    if (precond == PRECOND_J) return (1.0 / band_at(S, rg, dmax, a, a)) * rv[a];
    if (a >= nb * NX) return 0.0;   // rows past the last full block: not preconditioned (PCG.py:182)
    const int k = a / NX, i = a - k * NX;
    // MT[j NX + i] = P_kk[i][j]; L = P_{k,k-1}; U = P_{k+1,k} (U^T = P_{k,k+1}).  The LDS copy where
    // cached, else HBM -- in separate branches, so that each read is a ds_read or a global load: one
    // pointer that may point to either makes every read of the three blocks a flat load
    const double* rk = rv + k * NX;
    double s = 0.0;
    // (LDS copies: P_kk and P_{k+1,k} row-major swizzled, hp_off; HBM: P_kk transposed, Pl row-major)
    if (k < ncd) s = hp_row_lds<NX>(pcd, k, i, rk, s);
    else s = hp_col<NX>(glb_ptr(PT + (size_t)k * B2), i, rk, s);
    if (precond == PRECOND_SS) {
      if (k > 0) {
        if (k - 1 < ncl) s = hp_row_lds<NX>(pcl, k - 1, i, rk - NX, s);
        else s = hp_row<NX>(glb_ptr(PL + (size_t)(k - 1) * B2), i, rk - NX, s);
      }
      if (k + 1 < nb) {
        if (k < ncl) s = hp_col_lds<NX>(pcl, k, i, rk + NX, s);
        else s = hp_col<NX>(glb_ptr(PL + (size_t)k * B2), i, rk + NX, s);
      }
    }
    return s;
  };
  // (S p)_a over the row's structural range only, in column order (the terms left out are exact zeros):
  // the wave walks j = 0 .. its longest row's width - 1 (wave-uniform), each lane adding its row's
  // entries j <= hi (column c = lo_a + j, increasing with j).  S does not change during the solve: for
  // the rows of slot 0 the first REG entries were loaded into registers once (vc) and only
  // the rest stream from HBM, eight entries' loads in flight before their products are added; past the
  // wave's longest row the index is clamped and the product dropped.
  auto spmv = [&](int a, bool own, int jmax, int c0hi, bool cached, const double (&vc)[REG])
      -> double {
    const int c0 = c0hi >> 16;
    constexpr int U = TMPC_HARD_U;
    double s = 0.0;
    const double* Sa = S + (own ? a : 0);
    // The streamed entries (past the register-held ones, up to the wave's longest row; the band is zero
    // past each row: k_hard_schur fills it up to that row, tmpc_hard_pcg_batch's host copy is zero there)
    // in batches of U; the first batch's loads are in flight while the register-held entries are added.  p is clamped into range (a zero entry times a finite p).
    int j = cached ? REG : 0;
    double v[U];
    if (j <= jmax) {
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = Sa[(size_t)min(j + u, jmax) * dmax];
    }
    if (cached) {
      // Branch-free, no select: vc is zero past the row (set once), p is finite and the zero guard after
      // p covers c0 + u past D, so those products are exact zeros, and s + 0 = s bitwise (s starts at +0
      // and a sum of nonzero terms is never -0 in round-to-nearest): the row's own terms in column order.
      // (A branch per entry kept one LDS read in flight per wave.)
#pragma unroll
      for (int u = 0; u < REG; ++u) s = s + vc[u] * pv[c0 + u];
#if TMPC_HX_NOSTREAM   // timing experiment only (wrong answers): no streamed band entries
      return s;
#endif
    }
    while (j <= jmax) {
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (j + u <= jmax) s = s + v[u] * pv[min(c0 + j + u, D - 1)];   // wave-uniform test
      j += U;
      if (j <= jmax) {
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = Sa[(size_t)min(j + u, jmax) * dmax];
      }
    }
    return s;
  };
  // The per-row loops that read memory run one slot at a time (unroll 1), with z = P^-1 r and S p of
  // the thread's rows in LDS: unrolled over the slots they held every slot's loads and products in
  // registers at once (254 VGPRs, one wave per SIMD); x stays in registers.
  const int wbase = t & ~63;   // first row of this wave in slot 0
  // the row ranges, once: row a's first column lo_a and last entry hi_a = width - 1 (both < 2^15), each
  // wave-slot's longest row; slot 0's first REG entries into registers; the band entries
  // that stream from HBM every iteration (work accounting: the rest of slot 0's, all of the others')
  double vc[REG];
  double nnz = 0.0, nnz_reg = 0.0;
  int nsum = 0;   // workgroup sums so far (h_block_sum_db's slot parity)
#pragma unroll 1
  for (int m = 0; m < SLOTS; ++m) {
    const int a = t + m * HARD_PCG_THREADS;
    const int hi = a < D ? rg[2 * a + 1] - rg[2 * a] : -1;
    if (a < D) rlh[a] = hi | (rg[2 * a] << 16);
    int h = hi;
    for (int off = 32; off > 0; off >>= 1) h = max(h, __shfl_xor(h, off, 64));
    if ((t & 63) == 0) wlh[m * (HARD_PCG_THREADS / 64) + (t >> 6)] = h;
    if (m == 0) {
      const double* Sa = S + (a < D ? a : 0);
#pragma unroll
      for (int u = 0; u < REG; ++u) vc[u] = (a < D && u <= hi) ? Sa[(size_t)min(u, BW - 1) * dmax] : 0.0;
      if (a < D) {
        const int streamed = max(0, hi + 1 - REG);
        nnz += streamed;
        nnz_reg += hi + 1 - streamed;
      }
    } else if (a < D) {
      nnz += hi + 1;
    }
  }
  HX_SETUP(2);
  if (work) {
    nnz = h_block_sum_db(nnz, red, nsum);
    nnz_reg = h_block_sum_db(nnz_reg, red, nsum);
  }
  static_assert(hard_pcg_reg_diag(NX, SLOTS) <= HARD_PCG_GUARD, "the guard covers the register entries");
  for (int e = t; e < HARD_PCG_GUARD; e += HARD_PCG_THREADS) pv[D + e] = 0.0;   // (after the setup's staging)
  double xv[SLOTS];
  const double* g = gam + (size_t)b * dmax;
#pragma unroll
  for (int m = 0; m < SLOTS; ++m) {
    const int a = t + m * HARD_PCG_THREADS;
    xv[m] = 0.0;
    if (a < D) rv[a] = g[a];
  }
  __syncthreads();
  double part = 0.0;
  double z0 = 0.0, sp0 = 0.0;   // z and S p of the slot-0 row (the other slots': zl, al in LDS)
#pragma unroll 1
  for (int m = 0; m < SLOTS; ++m) {
    const int a = t + m * HARD_PCG_THREADS;
    if (a < D) {
      const double z = apply_P(a);
      if (m == 0) z0 = z;
      else zl[a] = z;
      pv[a] = z;
      part += rv[a] * z;
    }
  }
  double nu = h_block_sum_db(part, red, nsum);
  HX_SETUP(3);
  int it_done = max_iter;
#if TMPC_HX_STAMPS   // timing experiment: per-phase shader-clock sums of every wave of problem 0
  unsigned long long hs_[8] = {}, hs_prev_ = __builtin_amdgcn_s_memtime();
#define HX_STAMP(i_) { const unsigned long long n_ = __builtin_amdgcn_s_memtime(); hs_[i_] += n_ - hs_prev_; hs_prev_ = n_; }
#else
#define HX_STAMP(i_)
#endif
  for (int it = 0; it < max_iter; ++it) {
    __syncthreads();
    HX_STAMP(0);
    part = 0.0;
#pragma unroll 1
    for (int m = 0; m < SLOTS; ++m) {
      if (wbase + m * HARD_PCG_THREADS >= D) break;   // wave-uniform: no row of this wave's slot m
      const int a = t + m * HARD_PCG_THREADS;
      const int c0hi = a < D ? rlh[a] : 0;   // (rows past D: own = false, nothing added)
      const int jmax = __builtin_amdgcn_readfirstlane(wlh[m * (HARD_PCG_THREADS / 64) + (t >> 6)]);
      const double sp = spmv(a, a < D, jmax, c0hi, m == 0, vc);
      if (a < D) {
        if (m == 0) sp0 = sp;
        else al[a] = sp;
        part += pv[a] * sp;
      }
    }
    HX_STAMP(1);
    const double alpha = nu / h_block_sum_db(part, red, nsum);
    HX_STAMP(2);
#pragma unroll
    for (int m = 0; m < SLOTS; ++m) {
      const int a = t + m * HARD_PCG_THREADS;
      if (a < D) {
        rv[a] = rv[a] - (m == 0 ? sp0 : al[a]) * alpha;
        xv[m] = xv[m] + pv[a] * alpha;
      }
    }
    HX_STAMP(3);
    __syncthreads();
    HX_STAMP(4);
    part = 0.0;
#pragma unroll 1
    for (int m = 0; m < SLOTS; ++m) {
      const int a = t + m * HARD_PCG_THREADS;
      if (a < D) {
        const double z = apply_P(a);
        if (m == 0) z0 = z;
        else zl[a] = z;
        part += rv[a] * z;
      }
    }
    HX_STAMP(5);
    const double nup = h_block_sum_db(part, red, nsum);
    HX_STAMP(6);
    if (fabs(nup) < tol) {
      it_done = it + 1;
      break;
    }
    const double beta = nup / nu;
    // p is rewritten only after every thread's S p and P^-1 r reads of this iteration (h_block_sum's barriers)
#pragma unroll
    for (int m = 0; m < SLOTS; ++m) {
      const int a = t + m * HARD_PCG_THREADS;
      if (a < D) pv[a] = (m == 0 ? z0 : zl[a]) + pv[a] * beta;
    }
    nu = nup;
    HX_STAMP(7);
  }
#if TMPC_HX_STAMPS
  if (b == 0 && (t & 63) == 0 && t < D)
    printf("hx_stamps wave %d it %d D %d: top %llu spmv %llu sum_a %llu upd %llu bar %llu precond %llu sum_nu %llu pupd %llu\n",
           t >> 6, it_done, D, hs_[0], hs_[1], hs_[2], hs_[3], hs_[4], hs_[5], hs_[6], hs_[7]);
  if (b == 0 && t == 0)
    printf("hx_setup D %d: gj_loads %llu gj_pivots %llu gj_writes %llu stair_stage %llu stair_compute %llu "
           "stair_rest %llu ranges %llu z0 %llu\n", D, su_[4], su_[5], su_[0], su_[6], su_[7], su_[1], su_[2], su_[3]);
#endif
#undef HX_STAMP
#undef HX_SETUP
#pragma unroll
  for (int m = 0; m < SLOTS; ++m) {
    const int a = t + m * HARD_PCG_THREADS;
    if (a < D) lam[(size_t)b * dmax + a] = xv[m];
  }
  if (t == 0) iters[b] = it_done;
  if (work && t == 0) {
    // bytes of this launch beyond registers and LDS: gamma in, lambda out; per iteration the
    // band's structural entries (S p) not held in registers, and the distinct preconditioner entries
    // one P^-1 r needs that are not resident in LDS (SS: of the nb diagonal and nb - 1 stair blocks,
    // each once, all but the ncd + ncl cached ones), it_done + 1 of those; once: the register-held band
    // entries, and the setup's reads of the band's diagonal (and for SS sub-diagonal) blocks and its HBM
    // writes: the blocks the LDS cache does not hold (P_kk row-major and transposed, Pl)
    const double b2 = (double)NX * NX;
    double pnnz = 0.0, setup = 0.0;
    if (precond == PRECOND_J) pnnz = D;
    if (precond == PRECOND_BJ) { pnnz = (double)(nb - ncd) * b2; setup = (nb + 2.0 * (nb - ncd)) * b2; }
    if (precond == PRECOND_SS && nb > 0) {
      pnnz = (double)(2 * nb - 1 - ncd - ncl) * b2;
      setup = (2.0 * nb - 1.0 + 2.0 * (nb - ncd) + (nb - 1 - ncl)) * b2;
    }
    work[b] += 8.0 * (2.0 * D + it_done * nnz + (it_done + 1.0) * pnnz + setup + nnz_reg);
  }
}

// Method S (and N): S lambda = gamma by banded elimination (S is negative definite: no pivoting).
// Where S is singular the reference's np.linalg.solve raises and it takes lstsq's minimum-norm
// least-squares answer, setting `singular` (:353-357, 431-436).  S is singular in exactly two
// structural ways here, both handled in closed form before the elimination:
//   * identically zero rows (FULL_SET's inactive constraints): lambda = 0 for them, the minimum norm;
//   * a knot-0 hard row on a state entry (xs violates a joint / velocity limit) duplicates the
//     initial-state row R_0 of that entry up to its sign s: S row / column b = s row / column a
//     exactly.  The least-squares equations for the pair reduce to one, row a with gamma_a' =
//     (gamma_a + s gamma_b) / 2 on lambda' = lambda_a + s lambda_b, and the minimum-norm split is
//     lambda_a = lambda' / 2, lambda_b = s lambda' / 2 (the null vector e_b - s e_a is orthogonal).
// sing[b] = 1 when either happened (the trace's `singular`).
__global__ void __launch_bounds__(256) k_hard_direct(int B, int N, int NX, int W, int dmax, int rmax,
                                                     const int* __restrict__ active, const int* __restrict__ dim,
                                                     const int* __restrict__ hoff, const int* __restrict__ cnt,
                                                     const int* __restrict__ hcol, const double* __restrict__ hsgn,
                                                     const double* __restrict__ Sb, const double* __restrict__ gam,
                                                     double* __restrict__ M, double* __restrict__ rhs,
                                                     double* __restrict__ lam, int* __restrict__ sing,
                                                     const int* __restrict__ rng) {
  const int b = blockIdx.x;
  if (!active[b]) return;
  const int D = dim[b];
  const int BW = 2 * W + 1;
  const double* S = Sb + (size_t)b * dmax * BW;
  const int* rg = rng + (size_t)b * dmax * 2;
  double* Mb = M + (size_t)b * dmax * BW;
  double* y = rhs + (size_t)b * dmax;
  __shared__ double fcol[1024];
  __shared__ double red[16];
  __shared__ int s_dup_a[64], s_dup_b[64];
  __shared__ double s_dup_s[64];
  __shared__ int s_ndup, s_sing, s_wr;
  if (threadIdx.x == 0) s_wr = 0;
  __syncthreads();
  // M = S inside the row ranges, zero elsewhere; Wr = the half-bandwidth of those ranges, which the
  // elimination's fill-in never leaves (no pivoting)
  for (int e = threadIdx.x; e < D * BW; e += blockDim.x) {
    const int a = e / BW, o = e - a * BW, c = a - W + o;
    Mb[e] = (c >= rg[2 * a] && c <= rg[2 * a + 1]) ? S[(size_t)(c - rg[2 * a]) * dmax + a] : 0.0;
  }
  for (int a = threadIdx.x; a < D; a += blockDim.x) atomicMax(&s_wr, max(a - rg[2 * a], rg[2 * a + 1] - a));
  for (int a = threadIdx.x; a < D; a += blockDim.x) y[a] = gam[(size_t)b * dmax + a];
  if (threadIdx.x == 0) {
    // knot-0 hard rows on state entries: duplicates of R_0 rows (rows 0..NX-1)
    int nd = 0;
    const int c0 = cnt[(size_t)b * N], h0 = hoff[(size_t)b * N];
    const size_t hb = (size_t)b * N * rmax;
    for (int s = 0; s < c0 && s < rmax && nd < 64; ++s) {
      const double sg = hsgn[hb + s];
      const int col = hcol[hb + s];
      if (sg != 0.0 && col < NX) {
        s_dup_a[nd] = col;
        s_dup_b[nd] = h0 + s;
        s_dup_s[nd] = sg;
        ++nd;
      }
    }
    s_ndup = nd;
    s_sing = nd > 0;
  }
  __syncthreads();
  const int nd = s_ndup;
  if (nd > 0 && threadIdx.x == 0) {
    for (int i = 0; i < nd; ++i) {
      const int a = s_dup_a[i], bb = s_dup_b[i];
      y[a] = 0.5 * (y[a] + s_dup_s[i] * y[bb]);
      y[bb] = 0.0;
    }
  }
  __syncthreads();
  for (int i = 0; i < nd; ++i) {   // row and column b -> identity
    const int bb = s_dup_b[i];
    for (int o = threadIdx.x; o < BW; o += blockDim.x) {
      Mb[(size_t)bb * BW + o] = o == W ? 1.0 : 0.0;
      const int r = bb - W + o;    // column bb of row r sits at offset bb - r + W = 2W - o
      if (r >= 0 && r < D && r != bb) Mb[(size_t)r * BW + (2 * W - o)] = 0.0;
    }
  }
  __syncthreads();
  // zero rows -> identity rows with a zero right-hand side
  for (int a = threadIdx.x; a < D; a += blockDim.x) {
    bool zero = true;
    for (int o = 0; o < BW; ++o) zero = zero && Mb[(size_t)a * BW + o] == 0.0;
    if (zero) {
      Mb[(size_t)a * BW + W] = 1.0;
      y[a] = 0.0;
      s_sing = 1;
    }
  }
  __syncthreads();
  const int Wr = s_wr;
  for (int p = 0; p < D; ++p) {
    const int r1 = p + Wr < D - 1 ? p + Wr : D - 1;
    const double piv = Mb[(size_t)p * BW + W];
    for (int r = p + 1 + threadIdx.x; r <= r1; r += blockDim.x) fcol[r - p - 1] = Mb[(size_t)r * BW + (p - r + W)] / piv;
    __syncthreads();
    const int nr = r1 - p, nc = r1 - p + 1;
    for (int e = threadIdx.x; e < nr * nc; e += blockDim.x) {
      const int r = p + 1 + e / nc, c = p + e % nc;
      const int oc = c - r + W;
      if (oc < 0 || oc >= BW) continue;
      const double f = fcol[r - p - 1];
      Mb[(size_t)r * BW + oc] -= f * Mb[(size_t)p * BW + (c - p + W)];
    }
    for (int r = p + 1 + threadIdx.x; r <= r1; r += blockDim.x) y[r] -= fcol[r - p - 1] * y[p];
    __syncthreads();
  }
  // back substitution
  for (int p = D - 1; p >= 0; --p) {
    const int c1 = p + Wr < D - 1 ? p + Wr : D - 1;
    double part = 0.0;
    for (int c = p + 1 + threadIdx.x; c <= c1; c += blockDim.x) part += Mb[(size_t)p * BW + (c - p + W)] * y[c];
    const double s = h_block_sum(part, red);
    if (threadIdx.x == 0) y[p] = (y[p] - s) / Mb[(size_t)p * BW + W];
    __syncthreads();
  }
  if (threadIdx.x == 0) {   // the minimum-norm split of the merged duplicate pairs
    for (int i = 0; i < nd; ++i) {
      const double l = y[s_dup_a[i]];
      y[s_dup_a[i]] = 0.5 * l;
      y[s_dup_b[i]] = s_dup_s[i] * (0.5 * l);
    }
    sing[b] = s_sing;
  }
  __syncthreads();
  for (int a = threadIdx.x; a < D; a += blockDim.x) lam[(size_t)b * dmax + a] = y[a];
}

// dxu_k = Ghat_k (g_k - (C^T lambda)_k) (:449-452), lane = (problem, knot)
template <int NJ>
__global__ void __launch_bounds__(64) k_hard_dxu(const CostDev* __restrict__ C, int B, int N, int dmax, int rmax,
                                                 const int* __restrict__ active, const double* __restrict__ Ghat,
                                                 int per_knot, const double* __restrict__ Aall,
                                                 const double* __restrict__ Ball, const double* __restrict__ x,
                                                 const double* __restrict__ u, const double* __restrict__ jsoft,
                                                 const int* __restrict__ roff, const int* __restrict__ hoff,
                                                 const int* __restrict__ cnt, const int* __restrict__ hcol,
                                                 const double* __restrict__ hsgn, const double* __restrict__ lam,
                                                 double* __restrict__ dx, double* __restrict__ du,
                                                 const double* __restrict__ gvec) {
  constexpr int NX = 2 * NJ, NU = NJ, NXU = NX + NU;
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= B * N) return;
  const int b = gid / N, k = gid - b * N;
  if (!active[b]) return;
  const int K = N - 1;
  const double* L = lam + (size_t)b * dmax;
  const int* ro = roff + (size_t)b * N;
  const int* ho = hoff + (size_t)b * N;
  // every array index below is static once the loops are unrolled (round 6: the hard rows' column
  // index and the plugin block's runtime row count had put ctl / rhs in scratch, 304 B per lane at
  // arm6); a hard row's term goes to its column through a compare per column, the same update of the
  // same element
  double ctl[3 * NJ];
#pragma unroll
  for (int m = 0; m < NXU; ++m) ctl[m] = 0.0;
#pragma unroll
  for (int i = 0; i < NX; ++i) ctl[i] = L[ro[k] + i];
  if (k < K) {
    const double* A = Aall + ((size_t)b * K + k) * NX * NX;
    const double* Bk = Ball + ((size_t)b * K + k) * NX * NU;
    const double* l1 = L + ro[k + 1];
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      double atl = 0.0;
#pragma unroll
      for (int m = 0; m < NX; ++m) atl += A[m * NX + j] * l1[m];
      ctl[j] = ctl[j] - atl;
    }
#pragma unroll
    for (int j = 0; j < NU; ++j) {
      double btl = 0.0;
#pragma unroll
      for (int m = 0; m < NX; ++m) btl += Bk[m * NU + j] * l1[m];
      ctl[NX + j] = -btl;
    }
  }
  const size_t hb = ((size_t)b * N + k) * rmax;
  for (int s = 0; s < cnt[(size_t)b * N + k]; ++s) {
    const int col = hcol[hb + s];
    const double hs = hsgn[hb + s], lv = L[ho[k] + s];
#pragma unroll
    for (int c = 0; c < NXU; ++c)
      if (c == col) ctl[c] += hs * lv;
  }
  const HGhat<NJ> Gh{per_knot ? Ghat + (size_t)b * N * HGhat<NJ>::GS : Ghat + (size_t)b * 3 * NX * NX, per_knot != 0};
  const double* xb = x + (size_t)b * NX * N;
  const double* ub = u + (size_t)b * NU * K;
  const double* js = jsoft ? jsoft + (size_t)b * N * NXU : nullptr;
  double rhs[3 * NJ];
#pragma unroll
  for (int m = 0; m < NXU; ++m)
    rhs[m] = (m < NX || k < K) ? (gvec ? gvec[((size_t)b * N + k) * NXU + m] : hard_grad<NJ>(C, xb, ub, js, N, k, m))
                                     - ctl[m]
                               : 0.0;
  if (per_knot == 2) {   // the plugin-hook QP's full block (k_ghat_full): dxu_k = Ghat_k (g_k - (C^T lambda)_k)
    const double* G = Ghat + ((size_t)b * N + k) * NXU * NXU;
    const int m = k < K ? NXU : NX;
#pragma unroll
    for (int i = 0; i < NXU; ++i) {
      if (i >= m) break;
      double acc = 0.0;
#pragma unroll
      for (int j = 0; j < NXU; ++j) {
        if (j >= m) break;
        acc += G[i * NXU + j] * rhs[j];
      }
      if (i < NX) dx[((size_t)b * N + k) * NX + i] = acc;
      else du[((size_t)b * K + k) * NU + (i - NX)] = acc;
    }
    return;
  }
  const double* Gx = Gh.x(C, k, N);
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < NX; ++j) acc += Gx[i * NX + j] * rhs[j];
    dx[((size_t)b * N + k) * NX + i] = acc;
  }
  if (k < K) {
    const double* Gu = Gh.u(k);
#pragma unroll
    for (int i = 0; i < NU; ++i) {
      double acc = 0.0;
#pragma unroll
      for (int j = 0; j < NU; ++j) acc += Gu[i * NU + j] * rhs[NX + j];
      du[((size_t)b * K + k) * NU + i] = acc;
    }
  }
}

// totalHardConstraintViolation's hard terms (:286-293): per trial point and knot,
// sum(map(abs, value_hard_constraints)) in the reference's row order; hterms [B][T][N]
template <int NJ>
__global__ void __launch_bounds__(256) k_hard_ls(const ConstrDev* __restrict__ Cs, int B, int N, int T,
                                                 const double* __restrict__ alphas, const double* __restrict__ x,
                                                 const double* __restrict__ u, const double* __restrict__ dx,
                                                 const double* __restrict__ du, const int* __restrict__ active,
                                                 double* __restrict__ hterms) {
  constexpr int NX = 2 * NJ, NU = NJ;
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= B * T * N) return;
  const int k = gid % N, bt = gid / N, b = bt / T, t = bt - b * T;
  if (!active[b]) return;
  const int K = N - 1;
  const double al = alphas[t];
  double z[3 * NJ];
#pragma unroll
  for (int m = 0; m < NX; ++m) {
    const double xm = x[((size_t)b * NX + m) * N + k];
    z[m] = dx ? xm - al * dx[((size_t)b * N + k) * NX + m] : xm;
  }
#pragma unroll
  for (int m = 0; m < NU; ++m) {
    double um = k < K ? u[((size_t)b * NU + m) * K + k] : 0.0;
    if (dx && k < K) um = um - al * du[((size_t)b * K + k) * NU + m];
    z[NX + m] = um;
  }
  // hard_knot_rows' rows in its order (type, then lower / upper bound per joint), each |value| added as it
  // is formed: the same sum in the same order as summing its val[] afterwards.  Its row arrays, indexed
  // by the running row count, lived in scratch here (k_hard_ls averaged 0.29 ms, profiles/r06/counters);
  // unrolled in full every z index is static and the kernel keeps no arrays.
  const bool terminal = k == K;
  double s = 0.0;
#pragma unroll
  for (int ty = 0; ty < 3; ++ty) {
    const int hm = Cs->hard[ty];
    if (hm == HARD_NONE || (ty == 2 && terminal)) continue;
#pragma unroll
    for (int e = 0; e < 2 * NJ; ++e) {
      const int i = e < NJ ? e : e - NJ;
      const double zi = z[ty * NJ + i];
      const double v = e < NJ ? zi - Cs->lb[ty][i] : Cs->ub[ty][i] - zi;
      if (hm == HARD_ACTIVE && !(v < 0.0)) continue;
      s += fabs(v);
    }
  }
  hterms[gid] = s;
}

// ---------------------------------------------------------------- launchers
#define HGRID(n, bs) dim3(((n) + (bs) - 1) / (bs)), dim3(bs)

template <int NJ>
struct LaunchHard {
  static void run(hipStream_t s, const HardArgs& h) {
    constexpr int NX = 2 * NJ;
    const int B = h.B, N = h.N;
    if (h.phase == 0) {
      if (!h.rows_given)   // the plugin-hook QP brings its rows (cnt / hcol / hsgn / hval) from the host
        hipLaunchKernelGGL((k_hard_rows<NJ>), HGRID(B * N, 256), 0, s, h.Cs, B, N, h.rmax, h.x, h.u, h.active, h.cnt,
                           h.hcol, h.hsgn, h.hval, h.hslot, h.amask, h.iter, h.Wtr, h.tr_active);
      hipLaunchKernelGGL(k_hard_layout, dim3(B), dim3(64), 0, s, B, N, NX, h.rmax, h.active, h.cnt, h.roff, h.hoff,
                         h.dim, h.rkind, h.rknot, h.ridx, h.dmax);
      hipLaunchKernelGGL((k_hard_schur<NJ>), dim3(B), dim3(256), hard_schur_lds_bytes(N, NJ, h.dmax), s, h.C, B, N, h.W, h.dmax, h.rmax, h.active, h.Ghat,
                         h.per_knot, h.A, h.Bm, h.cvec, h.x, h.u, h.jsoft, h.dim, h.rkind, h.rknot, h.ridx, h.hoff,
                         h.hcol, h.hsgn, h.hval, h.Y, h.PK, h.Sb, h.gam, h.rng, h.gvec);
    } else if (h.phase == 1) {
      if (h.precond == 0) {
        hipLaunchKernelGGL(k_hard_direct, dim3(B), dim3(256), 0, s, B, N, NX, h.W, h.dmax, h.rmax, h.active, h.dim,
                           h.hoff, h.cnt, h.hcol, h.hsgn, h.Sb, h.gam, h.M, h.rhs, h.lam, h.sing,
                           h.rng);
      } else {
        // the whole LDS: one 16-wave workgroup per CU, the rest of it caches preconditioner blocks
        size_t lds = HARD_PCG_LDS_BYTES;
        if (const char* e = getenv("TMPC_HARD_PCG_LDS_KB"))   // dev: a smaller block cache (measurement)
          lds = std::min(lds, std::max((size_t)atoi(e) * 1024,
                                       (size_t)hard_pcg_cache_offset(h.dmax, NX, HARD_PCG_MAX_SLOTS) * sizeof(double)));
        const int slots = (h.dmax + HARD_PCG_THREADS - 1) / HARD_PCG_THREADS;
#define HPCG(SL) hipLaunchKernelGGL((k_hard_pcg<NX, SL>), dim3(B), dim3(HARD_PCG_THREADS), lds, s, B, h.W, h.dmax, \
                                    h.precond, h.active, h.dim, h.Sb, h.gam, h.tol, h.max_iter, h.Pd, h.Pl, \
                                    h.Ptr, h.lam, h.iters, h.rng, h.work, (int)lds)
        if (slots <= 1) HPCG(1);
        else if (slots <= 2) HPCG(2);
        else if (slots <= 3) HPCG(3);
        else HPCG(4);
#undef HPCG
      }
    } else if (h.phase == 2) {
      hipLaunchKernelGGL((k_hard_dxu<NJ>), HGRID(B * N, 64), 0, s, h.C, B, N, h.dmax, h.rmax, h.active, h.Ghat,
                         h.per_knot, h.A, h.Bm, h.x, h.u, h.jsoft, h.roff, h.hoff, h.cnt, h.hcol, h.hsgn, h.lam, h.dx,
                         h.du, h.gvec);
    } else {
      hipLaunchKernelGGL((k_hard_ls<NJ>), HGRID(B * h.T * N, 256), 0, s, h.Cs, B, N, h.T, h.alphas, h.x, h.u, h.dx,
                         h.du, h.active, h.hterms);
    }
  }
};

int launch_hard(hipStream_t s, int nj, const HardArgs& h) {
  switch (nj) {
    case 1: LaunchHard<1>::run(s, h); break;
    case 2: LaunchHard<2>::run(s, h); break;
    case 3: LaunchHard<3>::run(s, h); break;
    case 4: LaunchHard<4>::run(s, h); break;
    case 5: LaunchHard<5>::run(s, h); break;
    case 6: LaunchHard<6>::run(s, h); break;
    case 7: LaunchHard<7>::run(s, h); break;
    default: return -2;
  }
  return 0;
}

int hard_set_max_lds() {
  const int bytes = HARD_PCG_LDS_BYTES;
  int err = 0;
#define SETH1(V, SL) err |= (int)hipFuncSetAttribute((const void*)k_hard_pcg<V, SL>, \
                                                   hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
#define SETH(V) SETH1(V, 1) SETH1(V, 2) SETH1(V, 3) SETH1(V, 4)
  SETH(2) SETH(4) SETH(6) SETH(8) SETH(10) SETH(12) SETH(14)
#undef SETH
#undef SETH1
  return err;
}

}  // namespace tmpc

// ============================================================== dense PCG (tmpc_pcg_dense_batch)
// PCG.pcg(A, b, Pinv, guess, options) (GBD-PCG-Python/PCG.py:66-111) with any dense A and preconditioner
// matrix Pinv -- the caller's, or PCG.solve's block preconditioner (compute_preconditioner, PCG.py:113-212)
// built here from A -- for dimensions up to HARD_PCG_MAX_ROWS.  Operation order: oracle/dense.py (every
// matrix-vector product sequential over the columns, the dot products of k_hard_pcg).
namespace tmpc {

// out[b][c][r] = in[b][r][c] (D x D per system): the PCG reads column c of A and Pinv as one coalesced row
__global__ void __launch_bounds__(256) k_dense_transpose(int D, const double* __restrict__ in, double* __restrict__ out) {
  __shared__ double tile[32][33];
  const size_t off = (size_t)blockIdx.z * D * D;
  const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  for (int i = threadIdx.y; i < 32; i += 8) {
    const int r = r0 + i, c = c0 + threadIdx.x;
    if (r < D && c < D) tile[i][threadIdx.x] = in[off + (size_t)r * D + c];
  }
  __syncthreads();
  for (int i = threadIdx.y; i < 32; i += 8) {
    const int c = c0 + i, r = r0 + threadIdx.x;
    if (r < D && c < D) out[off + (size_t)c * D + r] = tile[threadIdx.x][i];
  }
}

// '0' / J: the diagonal of Pinv (PT is zero-filled before)
__global__ void __launch_bounds__(256) k_dense_diag(int D, int precond, const double* __restrict__ A, double* __restrict__ PT) {
  const size_t off = (size_t)blockIdx.x * D * D;
  for (int a = threadIdx.x; a < D; a += blockDim.x)
    PT[off + (size_t)a * D + a] = precond == PRECOND_J ? 1.0 / A[off + (size_t)a * D + a] : 1.0;
}

// BJ / SS diagonal blocks: Gauss-Jordan on the augmented [A_kk | I] without pivoting, the operation
// sequence of k_hard_pcg's setup (oracle/hard.py _gj_inverse); one 64-thread workgroup per (block, system).
// Pd [B][nb][NX][NX] row-major; PT[(k NX + j) D + k NX + i] = (P_kk)_ij.
template <int NX>
__global__ void __launch_bounds__(64) k_dense_gj(int D, int nb, const double* __restrict__ A, double* __restrict__ Pd,
                                                 double* __restrict__ PT) {
  constexpr int B2 = NX * NX;
  __shared__ double M[B2], prow[NX], fcol[NX];
  const int k = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  const size_t off = (size_t)b * D * D;
  for (int e = t; e < B2; e += 64) M[e] = A[off + (size_t)(k * NX + e / NX) * D + k * NX + e % NX];
  for (int p = 0; p < NX; ++p) {
    __syncthreads();
    for (int j = t; j < NX; j += 64) {
      const double d = M[p * NX + p];
      prow[j] = (j == p) ? 1.0 / d : M[p * NX + j] / d;
      fcol[j] = M[j * NX + p];
    }
    __syncthreads();
    for (int e = t; e < B2; e += 64) {
      const int r = e / NX, j = e - r * NX;
      if (r == p) {
        M[e] = prow[j];
      } else {
        const double f = fcol[r];
        const double m0 = (j == p) ? 0.0 : M[e];
        M[e] = m0 - f * prow[j];
      }
    }
  }
  __syncthreads();
  for (int e = t; e < B2; e += 64) {
    const int i = e / NX, j = e - i * NX;
    Pd[((size_t)b * nb + k) * B2 + e] = M[e];
    PT[off + (size_t)(k * NX + j) * D + k * NX + i] = M[e];
  }
}

// SS stair blocks (k_hard_pcg's setup (2), oracle/hard.py _neg_triple): odd k: P_{k,k-1} = -P_kk (S_{k,k-1}
// P_{k-1,k-1}); even k: P_{k-1,k} = -P_{k-1,k-1} (S_{k-1,k} P_kk); each mirrored by its transpose.  One
// workgroup per (k - 1, system).
template <int NX>
__global__ void __launch_bounds__(256) k_dense_stair(int D, int nb, const double* __restrict__ A,
                                                     const double* __restrict__ Pd, double* __restrict__ PT) {
  constexpr int B2 = NX * NX;
  __shared__ double yz[B2];
  const int k = blockIdx.x + 1, b = blockIdx.y, t = threadIdx.x;
  const size_t off = (size_t)b * D * D;
  const bool odd = k & 1;
  const int yr = odd ? k : k - 1, yc = odd ? k - 1 : k;   // Y = S_{yr, yc}
  const double* Z = Pd + ((size_t)b * nb + (odd ? k - 1 : k)) * B2;
  const double* X = Pd + ((size_t)b * nb + (odd ? k : k - 1)) * B2;
  for (int e = t; e < B2; e += blockDim.x) {
    const int r = e / NX, c = e - r * NX;
    double s = 0.0;
    for (int l = 0; l < NX; ++l) s += A[off + (size_t)(yr * NX + r) * D + yc * NX + l] * Z[l * NX + c];
    yz[e] = s;
  }
  __syncthreads();
  for (int e = t; e < B2; e += blockDim.x) {
    const int r = e / NX, c = e - r * NX;
    double acc = 0.0;
    for (int m = 0; m < NX; ++m) acc += X[r * NX + m] * yz[m * NX + c];
    const double v = -acc;
    const int pr = odd ? r : c, pc = odd ? c : r;   // element (pr, pc) of P_{k,k-1}
    PT[off + (size_t)((k - 1) * NX + pc) * D + k * NX + pr] = v;   // Pinv[k NX + pr][(k-1) NX + pc]
    PT[off + (size_t)(k * NX + pr) * D + (k - 1) * NX + pc] = v;   // its mirror P_{k-1,k}
  }
}

// The PCG: one 1024-thread workgroup per system, row a on thread a mod 1024 (slot a / 1024); p, r, x of
// every row in LDS (the products read them all), each thread's own rows' r, x, p, z, A p in registers.
// Column c of A / Pinv (AT / PT rows) is one coalesced read per wave, p / r / x[c] an LDS broadcast.
template <int SLOTS>
__global__ void __launch_bounds__(HARD_PCG_THREADS) k_pcg_dense(int D, const double* __restrict__ AT,
                                                               const double* __restrict__ PT,
                                                               const double* __restrict__ bv,
                                                               const double* __restrict__ guess, double tol,
                                                               int max_iter, double* __restrict__ xo,
                                                               int* __restrict__ iters, double* __restrict__ tnu,
                                                               double* __restrict__ tres) {
  constexpr int T = HARD_PCG_THREADS;
  const int b = blockIdx.x, t = threadIdx.x;
  const size_t DD = (size_t)D * D;
  const double* A = AT + b * DD;
  const double* P = PT + b * DD;
  const double* bb = bv + (size_t)b * D;
  extern __shared__ __align__(16) double sh[];
  double* pv = sh;
  double* rv = pv + D;
  double* xl = rv + D;
  double* red = xl + D;   // 2 x 16 reduction slots
  int nsum = 0;
  const int W = max_iter + 1;
  // y = M v for this thread's rows, sequential over the columns (rows past D read a clamped, in-range
  // entry and are never used)
  auto mv = [&](const double* M, const double* v, double (&y)[SLOTS]) {
#pragma unroll
    for (int m = 0; m < SLOTS; ++m) y[m] = 0.0;
    constexpr int UNR = SLOTS >= 3 ? 2 : 4;   // (4 x 4 slots of loads in flight spilled)
#pragma unroll UNR
    for (int c = 0; c < D; ++c) {
      const double vc = v[c];
      const double* col = M + (size_t)c * D;
#pragma unroll
      for (int m = 0; m < SLOTS; ++m) y[m] = y[m] + col[min(t + m * T, D - 1)] * vc;
    }
  };
  double xr[SLOTS], rr[SLOTS], pr[SLOTS], y[SLOTS];
#pragma unroll
  for (int m = 0; m < SLOTS; ++m) {
    const int a = t + m * T;
    xr[m] = (guess && a < D) ? guess[(size_t)b * D + a] : 0.0;
    if (a < D) xl[a] = xr[m];
  }
  __syncthreads();
  mv(A, xl, y);
  double part = 0.0;
#pragma unroll
  for (int m = 0; m < SLOTS; ++m) {
    const int a = t + m * T;
    rr[m] = a < D ? bb[a] - y[m] : 0.0;
    if (a < D) {
      rv[a] = rr[m];
      part = part + rr[m] * rr[m];
    }
  }
  const double res0 = h_block_sum_db(part, red, nsum);   // (its barrier also publishes r)
  if (t == 0 && tres) tres[(size_t)b * W] = sqrt(res0);
  mv(P, rv, y);
  part = 0.0;
#pragma unroll
  for (int m = 0; m < SLOTS; ++m) {
    const int a = t + m * T;
    pr[m] = y[m];
    if (a < D) {
      pv[a] = pr[m];
      part = part + rr[m] * y[m];
    }
  }
  double nu = h_block_sum_db(part, red, nsum);
  if (t == 0 && tnu) tnu[(size_t)b * W] = fabs(nu);
  int it_done = max_iter;
  for (int it = 0; it < max_iter; ++it) {
    __syncthreads();   // p published
    mv(A, pv, y);      // A p
    part = 0.0;
#pragma unroll
    for (int m = 0; m < SLOTS; ++m)
      if (t + m * T < D) part = part + pr[m] * y[m];
    const double alpha = nu / h_block_sum_db(part, red, nsum);
#pragma unroll
    for (int m = 0; m < SLOTS; ++m) {
      const int a = t + m * T;
      rr[m] = rr[m] - y[m] * alpha;
      xr[m] = xr[m] + pr[m] * alpha;
      if (a < D) {
        rv[a] = rr[m];
        xl[a] = xr[m];
      }
    }
    __syncthreads();   // r, x published
    mv(P, rv, y);      // z = Pinv r
    part = 0.0;
#pragma unroll
    for (int m = 0; m < SLOTS; ++m)
      if (t + m * T < D) part = part + rr[m] * y[m];
    const double nup = h_block_sum_db(part, red, nsum);
    if (tres) {        // ||b - A x|| of the explicit residual (PCG.py:95)
      double q[SLOTS];
      mv(A, xl, q);
      double pq = 0.0;
#pragma unroll
      for (int m = 0; m < SLOTS; ++m) {
        const int a = t + m * T;
        if (a < D) {
          const double e = bb[a] - q[m];
          pq = pq + e * e;
        }
      }
      const double rs = h_block_sum_db(pq, red, nsum);
      if (t == 0) tres[(size_t)b * W + it + 1] = sqrt(rs);
    }
    if (t == 0 && tnu) tnu[(size_t)b * W + it + 1] = fabs(nup);
    if (fabs(nup) < tol) {
      it_done = it + 1;
      break;
    }
    const double beta = nup / nu;
#pragma unroll
    for (int m = 0; m < SLOTS; ++m) {
      const int a = t + m * T;
      pr[m] = y[m] + pr[m] * beta;
      if (a < D) pv[a] = pr[m];
    }
    nu = nup;
  }
#pragma unroll
  for (int m = 0; m < SLOTS; ++m) {
    const int a = t + m * T;
    if (a < D) xo[(size_t)b * D + a] = xr[m];
  }
  if (t == 0) iters[b] = it_done;
}

// ---- the dense PCG past HARD_PCG_MAX_ROWS rows (launch_pcg_dense_big) ----
// Past 4096 rows the vectors of a system no longer fit the workgroup's registers and LDS, so each phase of an
// iteration is its own launch with the vectors in HBM scratch, every value in k_pcg_dense's order:
//   k_pdb_mv:   y = M v (M given transposed: column c = row c of MT), row a on one thread, sequential over
//               the columns from 0.0 -- the product of k_pcg_dense's mv; 64-thread workgroups so that a
//               system's rows spread over D / 64 CUs; z selects one of two (M, v, y) products per launch;
//   k_pdb_step: one HARD_PCG_THREADS workgroup per system, thread t over rows t, t + 1024, ... in order --
//               the per-thread partials, butterfly and fan-in of h_block_sum_db, i.e. k_pcg_dense's sums --
//               and the element updates of the phase.
// A system that has met the tolerance sets done[b]; every later launch returns at once for it.
__global__ void __launch_bounds__(64) k_pdb_mv(int D, const double* __restrict__ M0, const double* __restrict__ v0,
                                               double* __restrict__ y0, const double* M1, const double* v1,
                                               double* y1,
                                               const int* __restrict__ done) {
  const int b = blockIdx.y, a = blockIdx.x * 64 + threadIdx.x;
  if (done[b] || a >= D) return;
  const bool second = blockIdx.z == 1;
  const size_t DD = (size_t)D * D;
  const double* M = (second ? M1 : M0) + b * DD;
  const double* v = (second ? v1 : v0) + (size_t)b * D;
  double s = 0.0;
  int c = 0;
  for (; c + 4 <= D; c += 4) {   // four columns' loads in flight, summed in column order
    const double m0 = M[(size_t)c * D + a], m1 = M[(size_t)(c + 1) * D + a];
    const double m2 = M[(size_t)(c + 2) * D + a], m3 = M[(size_t)(c + 3) * D + a];
    s = s + m0 * v[c];
    s = s + m1 * v[c + 1];
    s = s + m2 * v[c + 2];
    s = s + m3 * v[c + 3];
  }
  for (; c < D; ++c) s = s + M[(size_t)c * D + a] * v[c];
  (second ? y1 : y0)[(size_t)b * D + a] = s;
}

enum { PDB_INIT_R = 0, PDB_INIT_P = 1, PDB_A = 2, PDB_B = 3 };

__global__ void __launch_bounds__(HARD_PCG_THREADS) k_pdb_step(int phase, int it, int D, const double* __restrict__ bv,
                                                              double* __restrict__ xv, double* __restrict__ rv,
                                                              double* __restrict__ pv, const double* __restrict__ yv,
                                                              const double* __restrict__ qv, double* __restrict__ nuv,
                                                              int* __restrict__ done, double tol, int max_iter,
                                                              int* __restrict__ iters, double* __restrict__ tnu,
                                                              double* __restrict__ tres) {
  constexpr int T = HARD_PCG_THREADS;
  __shared__ double red[32];
  const int b = blockIdx.x, t = threadIdx.x;
  if (done[b]) return;
  int nsum = 0;
  const size_t o = (size_t)b * D;
  const double* bb = bv + o;
  double* x = xv + o;
  double* r = rv + o;
  double* p = pv + o;
  const double* y = yv + o;
  const int W = max_iter + 1;
  double part = 0.0;
  if (phase == PDB_INIT_R) {         // r = b - A x0, ||r||
    for (int a = t; a < D; a += T) {
      const double e = bb[a] - y[a];
      r[a] = e;
      part = part + e * e;
    }
    const double res0 = h_block_sum_db(part, red, nsum);
    if (t == 0 && tres) tres[(size_t)b * W] = sqrt(res0);
  } else if (phase == PDB_INIT_P) {  // p = z = Pinv r, nu = r . z
    for (int a = t; a < D; a += T) {
      p[a] = y[a];
      part = part + r[a] * y[a];
    }
    const double nu = h_block_sum_db(part, red, nsum);
    if (t == 0) {
      nuv[b] = nu;
      if (tnu) tnu[(size_t)b * W] = fabs(nu);
    }
  } else if (phase == PDB_A) {       // alpha = nu / p . A p; r -= A p alpha; x += p alpha
    for (int a = t; a < D; a += T) part = part + p[a] * y[a];
    const double alpha = nuv[b] / h_block_sum_db(part, red, nsum);
    for (int a = t; a < D; a += T) {
      r[a] = r[a] - y[a] * alpha;
      x[a] = x[a] + p[a] * alpha;
    }
  } else {                           // nu' = r . z, ||b - A x||, the exit test, p = z + p beta
    for (int a = t; a < D; a += T) part = part + r[a] * y[a];
    const double nup = h_block_sum_db(part, red, nsum);
    if (tres) {
      double pq = 0.0;
      for (int a = t; a < D; a += T) {
        const double e = bb[a] - qv[o + a];
        pq = pq + e * e;
      }
      const double rs = h_block_sum_db(pq, red, nsum);
      if (t == 0) tres[(size_t)b * W + it + 1] = sqrt(rs);
    }
    if (t == 0 && tnu) tnu[(size_t)b * W + it + 1] = fabs(nup);
    if (fabs(nup) < tol) {
      __syncthreads();   // every thread has read nu / done before thread 0 changes them
      if (t == 0) {
        iters[b] = it + 1;
        done[b] = 1;
      }
      return;
    }
    const double beta = nup / nuv[b];
    for (int a = t; a < D; a += T) p[a] = y[a] + p[a] * beta;
    __syncthreads();   // every thread has read nu
    if (t == 0) nuv[b] = nup;
  }
}

int launch_pcg_dense_big(hipStream_t s, const DenseArgs& a) {
  const dim3 g1((a.D + 63) / 64, a.B, 1), g2((a.D + 63) / 64, a.B, 2);
  const size_t vb = sizeof(double) * a.B * a.D;
  if (a.guess) {
    if (hipMemcpyAsync(a.x, a.guess, vb, hipMemcpyDeviceToDevice, s) != hipSuccess) return -1;
  } else if (hipMemsetAsync(a.x, 0, vb, s) != hipSuccess) {
    return -1;
  }
  if (hipMemsetAsync(a.done, 0, sizeof(int) * a.B, s) != hipSuccess) return -1;
  std::vector<int> itn(a.B, a.max_iter), dn(a.B);
  if (hipMemcpyAsync(a.iters, itn.data(), sizeof(int) * a.B, hipMemcpyHostToDevice, s) != hipSuccess) return -1;
  auto mv = [&](const double* M, const double* v, double* y) {
    hipLaunchKernelGGL(k_pdb_mv, g1, dim3(64), 0, s, a.D, M, v, y, M, v, y, a.done);
  };
  auto step = [&](int phase, int it) {
    hipLaunchKernelGGL(k_pdb_step, dim3(a.B), dim3(HARD_PCG_THREADS), 0, s, phase, it, a.D, a.b, a.x, a.r, a.p, a.y,
                       a.q, a.nu, a.done, a.tol, a.max_iter, a.iters, a.trace_nu, a.trace_res);
  };
  mv(a.AT, a.x, a.y);
  step(PDB_INIT_R, 0);
  mv(a.PT, a.r, a.y);
  step(PDB_INIT_P, 0);
  constexpr int CHECK = 4;   // iterations between host checks (later launches of a done system return at once)
  for (int it = 0; it < a.max_iter; ++it) {
    mv(a.AT, a.p, a.y);
    step(PDB_A, it);
    if (a.trace_res)   // z = Pinv r and A x in one launch
      hipLaunchKernelGGL(k_pdb_mv, g2, dim3(64), 0, s, a.D, a.PT, a.r, a.y, a.AT, a.x, a.q, a.done);
    else
      mv(a.PT, a.r, a.y);
    step(PDB_B, it);
    if ((it + 1) % CHECK == 0 && it + 1 < a.max_iter) {
      if (hipMemcpyAsync(dn.data(), a.done, sizeof(int) * a.B, hipMemcpyDeviceToHost, s) != hipSuccess) return -1;
      if (hipStreamSynchronize(s) != hipSuccess) return -1;
      bool all = true;
      for (int v : dn) all = all && v;
      if (all) break;
    }
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

static size_t pcg_dense_lds(int D) { return ((size_t)3 * D + 32) * sizeof(double); }

template <int NX>
static void dense_blocks(hipStream_t s, const DenseArgs& a, int nb) {
  hipLaunchKernelGGL((k_dense_gj<NX>), dim3(nb, a.B), dim3(64), 0, s, a.D, nb, a.A, a.Pd, a.PT);
  if (a.precond == PRECOND_SS && nb > 1)
    hipLaunchKernelGGL((k_dense_stair<NX>), dim3(nb - 1, a.B), dim3(256), 0, s, a.D, nb, a.A, a.Pd, a.PT);
}

int launch_dense_precond(hipStream_t s, const DenseArgs& a) {
  if (a.precond == PRECOND_NONE || a.precond == PRECOND_J) {
    hipLaunchKernelGGL(k_dense_diag, dim3(a.B), dim3(256), 0, s, a.D, a.precond, a.A, a.PT);
    return 0;
  }
  const int nb = a.D / a.nx;
  if (nb < 1) return 0;   // no full block: no row is preconditioned (PCG.py:182)
  switch (a.nx) {
#define DB(V) case V: dense_blocks<V>(s, a, nb); break;
    DB(1) DB(2) DB(3) DB(4) DB(5) DB(6) DB(7) DB(8) DB(9) DB(10) DB(11) DB(12) DB(13) DB(14) DB(15) DB(16)
#undef DB
    default: return -2;
  }
  return 0;
}

int launch_dense_transpose(hipStream_t s, int B, int D, const double* in, double* out) {
  hipLaunchKernelGGL(k_dense_transpose, dim3((D + 31) / 32, (D + 31) / 32, B), dim3(32, 8), 0, s, D, in, out);
  return 0;
}

int launch_pcg_dense(hipStream_t s, const DenseArgs& a) {
  const int slots = (a.D + HARD_PCG_THREADS - 1) / HARD_PCG_THREADS;
  const size_t lds = pcg_dense_lds(a.D);
#define PD(SL) hipLaunchKernelGGL((k_pcg_dense<SL>), dim3(a.B), dim3(HARD_PCG_THREADS), lds, s, a.D, a.AT, a.PT, a.b, \
                                  a.guess, a.tol, a.max_iter, a.x, a.iters, a.trace_nu, a.trace_res)
  if (slots <= 1) PD(1);
  else if (slots <= 2) PD(2);
  else if (slots <= 3) PD(3);
  else if (slots <= 4) PD(4);
  else return -2;
#undef PD
  return 0;
}

int dense_set_max_lds() {
  const int bytes = (int)pcg_dense_lds(HARD_PCG_MAX_ROWS);
  int err = 0;
  err |= (int)hipFuncSetAttribute((const void*)k_pcg_dense<1>, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  err |= (int)hipFuncSetAttribute((const void*)k_pcg_dense<2>, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  err |= (int)hipFuncSetAttribute((const void*)k_pcg_dense<3>, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  err |= (int)hipFuncSetAttribute((const void*)k_pcg_dense<4>, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  return err;
}

}  // namespace tmpc
