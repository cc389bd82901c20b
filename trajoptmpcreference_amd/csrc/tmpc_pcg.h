// The block-tridiagonal PCG of the fused QP kernels (PCG.pcg / compute_preconditioner,
// GBD-PCG-Python/PCG.py:66-212): lane geometry, register rows of S, LDS vectors, the
// preconditioners, the products, the fixed-tree reductions and the CG iteration.  Shared by
// tmpc_kernels.hip (k_qp, k_pcg) and tmpc_hooks.hip (k_qp_blocks, the plugin-hook QP): one
// operation order, restated by oracle/canon.c.
#pragma once
#include "tmpc_internal.h"

namespace tmpc {

// lanes outside ROW_MASK read 0
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ double dpp_get(double v) {
  int lo, hi;
  if (ROW_MASK == 0xf) {
    lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xf, 0xf, false);
    hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xf, 0xf, false);
  } else {
    lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, ROW_MASK, 0xf, false);
    hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, ROW_MASK, 0xf, false);
  }
  return __hiloint2double(hi, lo);
}

// ======================================================================= block-tridiagonal PCG
// One workgroup per problem, one lane per row of S (PCG.pcg, PCG.py:66-111).
//
// Reductions are DPP / permlane butterflies inside the wave (VALU only;
// ds_bpermute shuffles cost an LDS round trip per step) and one LDS fan-in of
// the per-wave totals, reduced again by DPP: a fixed tree, so the result is
// deterministic and identical for a problem whatever its batch neighbours.
__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}

// every lane of each 16-lane row ends with the sum over its row
__device__ __forceinline__ double dpp_row_sum(double v) {
  v += dpp_get<0xB1, 0xf>(v);    // quad_perm [1,0,3,2]
  v += dpp_get<0x4E, 0xf>(v);    // quad_perm [2,3,0,1]
  v += dpp_get<0x141, 0xf>(v);   // row_half_mirror
  v += dpp_get<0x140, 0xf>(v);   // row_mirror
  return v;
}

// v_permlane16_swap / v_permlane32_swap of a double with itself (gfx950): lane l gets
// its own value and that of lane l ^ 16 (resp. l ^ 32), in a fixed (lower, upper) order
__device__ __forceinline__ double perm_pair_sum16(double v) {
  const auto lo = __builtin_amdgcn_permlane16_swap(__double2loint(v), __double2loint(v), false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap(__double2hiint(v), __double2hiint(v), false, false);
  return __hiloint2double(hi[0], lo[0]) + __hiloint2double(hi[1], lo[1]);
}
__device__ __forceinline__ double perm_pair_sum32(double v) {
  const auto lo = __builtin_amdgcn_permlane32_swap(__double2loint(v), __double2loint(v), false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap(__double2hiint(v), __double2hiint(v), false, false);
  return __hiloint2double(hi[0], lo[0]) + __hiloint2double(hi[1], lo[1]);
}

// wave64 sum in every lane: row sums R_q by DPP, then (R0 + R1) + (R2 + R3) by the
// two permlane swaps -- the tree of the row_bcast:15 / row_bcast:31 reduction, so
// bitwise the same total, without the readlane round trip through SGPRs.  (Both
// reductions on the fp64 matrix core -- two v_mfma_f64_16x16x4f64 with B = 1 per
// sum, 3 VALU adds instead of 18 -- measured 12 % slower per PCG-SS iteration:
// the MFMA latency sits on the barrier-to-barrier critical path.)
__device__ __forceinline__ double wave_sum(double v) {
  return perm_pair_sum32(perm_pair_sum16(dpp_row_sum(v)));
}

// Lane geometry of the one-workgroup-per-problem kernels: RPL rows of S per
// lane, L = NX / RPL lanes per block row; lane t owns rows i + m L (m < RPL)
// of block k = t / L.  Two rows per lane halve the LDS traffic of every
// vector exchange (each block vector a lane reads serves both of its rows).
template <int NX, int RPL>
struct PcgLane {
  static constexpr int L = NX / RPL;
  int t, k, i;
  bool valid;
  __device__ __forceinline__ PcgLane(int t_, int N) {
    t = t_;
    valid = t < N * L;
    k = valid ? t / L : 0;
    i = valid ? t - k * L : 0;
  }
  __device__ __forceinline__ int r(int m) const { return i + m * L; }            // row within block k
  __device__ __forceinline__ int row(int m) const { return k * NX + i + m * L; }  // row of S
};

// one row of S (and of P_kk^-1) kept in registers for the whole solve
template <int NX>
struct PcgRow {
  double sd[NX];   // S_kk row
  double sl[NX];   // S_{k,k-1} row   (0 for k = 0)
  double su[NX];   // S_{k,k+1} row   (0 for k = N-1)
  double pr[NX];   // (S_kk)^-1 row  (J: pr[0] = 1 / S_ii)
};

// Past 1024 rows the four rows per lane no longer fit the register file (arm6
// N = 128: 1536 rows x 48 doubles = 74k doubles > the CU's 64k-double VGPR
// file), so the GM kernels keep S and P^-1 in HBM (L2 / MALL resident while a
// problem is solved) and the lane reads its rows there every product.  Layout
// per problem entry-pair-major [4][NX / 2][rows][2] (sd, sl, su; the P_kk^-1
// row pr stays in registers, slot 3 is unused), rows in lane order: a lane reads entries j, j + 1 of its row as one 16-byte load, and
// for a fixed pair the lanes of a wave read 1 KB of consecutive slots.  Same
// interface as PcgRow.
struct GRowRef {
  const double* __restrict__ p;   // this row's first pair
  int stride;                     // doubles from one pair of the row to the next (2 rows)
  __device__ __forceinline__ double operator[](int j) const {
    const double2 v = *reinterpret_cast<const double2*>(p + (size_t)(j >> 1) * stride);
    return (j & 1) ? v.y : v.x;
  }
};
template <int NX>
struct PcgRowG {
  GRowRef sd, sl, su;
  double pr[NX];   // the P_kk^-1 row stays in registers: an SS iteration reads it twice (w, z)
};
// HBM rows: bound the loads in flight (the compiler would hoist all of a product's row loads, 2-4
// dozen doubles per row, past the 168-VGPR budget of the GM kernel's 3 waves per SIMD)
template <class RT> struct RowInHbm { static constexpr bool value = false; };
template <int NX> struct RowInHbm<PcgRowG<NX>> { static constexpr bool value = true; };
#define PCG_LOAD_FENCE(RT, j, acc)                                       \
  if (RowInHbm<RT>::value && ((j) % 4) == 3) {                           \
    _Pragma("unroll") for (int m_ = 0; m_ < RPL; ++m_)                   \
      asm volatile("" : "+v"(acc[m_])::"memory");                        \
  }

// LDS vectors are [pad NX | N*NX rows | pad NX]: the pads stay zero so the
// block-tridiagonal products need no edge branches.  r is double-buffered
// (rbuf[it & 1]): in the same phase every lane reads the old r of its block
// while the owners write the new one.
constexpr int PCG_NVEC = 7;
struct PcgLds {
  double *pbuf, *rbuf[2], *abuf, *wbuf, *tbuf, *xbuf, *red, *piv;
  int* flags;   // [2][16] per-wave epochs: p published (0..15), w published (16..31)
};

// Fixed stride (the VR-row maximum plus the pads) so that every buffer is a
// compile-time offset from one per-lane address: one address VGPR for all
// vector traffic instead of one per buffer.  VR = 1024 for the register-row
// kernels, QP_MAX_ROWS for the global-row ones (GM, more than 1024 rows).
__host__ __device__ constexpr size_t pcg_vec_doubles(int NX, int VR) { return (size_t)VR + 2 * NX; }
__host__ __device__ inline size_t pcg_lds_doubles(int N, int NX, int VR) {
  return PCG_NVEC * pcg_vec_doubles(NX, VR) + 64 + (size_t)2 * N * NX;
}

__device__ __forceinline__ PcgLds pcg_lds(double* lds, int N, int NX, int VR) {
  const size_t v = pcg_vec_doubles(NX, VR);
  PcgLds L;
  L.pbuf = lds + NX;
  L.rbuf[0] = L.pbuf + v;
  L.rbuf[1] = L.rbuf[0] + v;
  L.abuf = L.rbuf[1] + v;
  L.wbuf = L.abuf + v;
  L.tbuf = L.wbuf + v;
  L.xbuf = L.tbuf + v;
  L.red = lds + PCG_NVEC * v;   // 3 x 16 reduction slots
  L.flags = reinterpret_cast<int*>(L.red + 48);   // 32 ints (16 doubles)
  L.piv = L.red + 64;           // 2 x N x NX
  return L;
}

// zero the pads, the reduction slots and the neighbour flags (callers barrier before first use)
__device__ __forceinline__ void pcg_lds_clear(double* lds, int N, int NX, int VR) {
  const size_t v = pcg_vec_doubles(NX, VR);
  const int rows = N * NX;
  for (int e = threadIdx.x; e < PCG_NVEC * 2 * NX + 64; e += blockDim.x) {
    if (e < PCG_NVEC * 2 * NX) {
      const int buf = e / (2 * NX), o = e - buf * 2 * NX;
      lds[buf * v + (o < NX ? o : rows + o)] = 0.0;
    } else {
      lds[PCG_NVEC * v + (e - PCG_NVEC * 2 * NX)] = 0.0;
    }
  }
}

// compute_preconditioner (PCG.py:166-212): J -> 1/S_ii; BJ and SS -> the
// diagonal block inverses by in-place Gauss-Jordan (one row per lane slot,
// pivot rows broadcast through LDS; S_kk is negative definite: no pivoting).
// In place, the row holds the not-yet-eliminated columns of [S_kk | I] and
// the already-formed columns of the inverse; the arithmetic is operation for
// operation that of the augmented [S_kk | I] elimination.
template <int NX, int RPL>
__device__ __forceinline__ void pcg_precondition(PcgRow<NX> (&R)[RPL], int precond, const PcgLane<NX, RPL>& ln,
                                                 int N, double* piv, double* Pd_block) {
  if (precond == PRECOND_NONE) {   // '0': P^-1 = I
    if (Pd_block && ln.valid) {
#pragma unroll
      for (int m = 0; m < RPL; ++m)
#pragma unroll
        for (int j = 0; j < NX; ++j) Pd_block[ln.r(m) * NX + j] = (j == ln.r(m)) ? 1.0 : 0.0;
    }
    return;
  }
  if (precond == PRECOND_J) {
#pragma unroll
    for (int m = 0; m < RPL; ++m) {
      double dii = 1.0;
#pragma unroll
      for (int j = 0; j < NX; ++j)
        if (j == ln.r(m)) dii = R[m].sd[j];
      if (ln.valid) R[m].pr[0] = 1.0 / dii;
    }
    return;
  }
#pragma unroll
  for (int m = 0; m < RPL; ++m)
#pragma unroll
    for (int j = 0; j < NX; ++j) R[m].pr[j] = R[m].sd[j];
#pragma unroll
  for (int p = 0; p < NX; ++p) {
    double* pv = piv + ((p & 1) * N + ln.k) * NX;
#pragma unroll
    for (int m = 0; m < RPL; ++m) {
      if (ln.valid && ln.r(m) == p) {
        double* a = R[m].pr;
        const double d = a[p];
#pragma unroll
        for (int j = 0; j < NX; ++j) {
          a[j] = (j == p) ? 1.0 / d : a[j] / d;
          pv[j] = a[j];
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int m = 0; m < RPL; ++m) {
      if (ln.valid && ln.r(m) != p) {
        double* a = R[m].pr;
        const double f = a[p];
        a[p] = 0.0;
#pragma unroll
        for (int j = 0; j < NX; ++j) a[j] -= f * pv[j];
      }
    }
  }
  if (Pd_block && ln.valid) {
#pragma unroll
    for (int m = 0; m < RPL; ++m)
#pragma unroll
      for (int j = 0; j < NX; ++j) Pd_block[ln.r(m) * NX + j] = R[m].pr[j];
  }
}

// out[m] = (S v) for this lane's rows, each block-vector element read once for
// all RPL rows.  With one row per lane: three independent chains (latency);
// with two: one chain per row (the rows interleave, and the VGPR budget of a
// 2-waves-per-SIMD launch has no room for more accumulators).
template <int NX, int RPL, class RT>
__device__ __forceinline__ void pcg_spmv(const RT (&R)[RPL], const double* __restrict__ v, int kb,
                                         double (&out)[RPL]) {
  const double* vm = v + kb - NX;
  constexpr int NC = RPL == 1 ? 3 : 1;
  double a[NC][RPL];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int m = 0; m < RPL; ++m) a[c][m] = 0.0;
#pragma unroll
  for (int j = 0; j < NX; ++j) {
    const double p0 = vm[j], p1 = vm[NX + j], p2 = vm[2 * NX + j];
#pragma unroll
    for (int m = 0; m < RPL; ++m) {
      a[0][m] += R[m].sl[j] * p0;
      a[NC > 1 ? 1 : 0][m] += R[m].sd[j] * p1;
      a[NC > 2 ? 2 : 0][m] += R[m].su[j] * p2;
    }
    // two rows per lane: bound the LDS loads in flight (each b128 holds 4
    // VGPRs; all 18 hoisted would not fit next to the matrix rows): the
    // accumulators are pinned here, and loads may not cross the fence
    if (RPL > 1 && (j % 4) == 3) {
#pragma unroll
      for (int m = 0; m < RPL; ++m) asm volatile("" : "+v"(a[0][m])::"memory");
    }
  }
#pragma unroll
  for (int m = 0; m < RPL; ++m) out[m] = NC == 3 ? (a[0][m] + a[NC > 1 ? 1 : 0][m]) + a[NC > 2 ? 2 : 0][m] : a[0][m];
}

// out[m] = P_kk row . v_k
template <int NX, int RPL, class RT>
__device__ __forceinline__ void pcg_block_dot(const RT (&R)[RPL], const double* __restrict__ v,
                                              double (&out)[RPL]) {
  constexpr int NC = RPL == 1 ? 2 : 1;
  double a[NC][RPL];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int m = 0; m < RPL; ++m) a[c][m] = 0.0;
#pragma unroll
  for (int j = 0; j < NX; ++j) {
    const double vj = v[j];
#pragma unroll
    for (int m = 0; m < RPL; ++m) a[j % NC][m] += R[m].pr[j] * vj;
    PCG_LOAD_FENCE(RT, j, a[0])
  }
#pragma unroll
  for (int m = 0; m < RPL; ++m) out[m] = NC == 2 ? a[0][m] + a[NC - 1][m] : a[0][m];
}

// Diagnostic build only (-DTMPC_PCG_STAMPS, tools/pcg_microbench.py --stamps):
// per-phase s_memtime cycle totals of the first and last wave of each
// workgroup replace the |nu| trace; the true-residual trace is disabled.
#ifdef TMPC_PCG_STAMPS
#define PCG_STAMP(i)                                            \
  do {                                                          \
    const unsigned long long n_ = __builtin_amdgcn_s_memtime(); \
    st_[i] += n_ - st_prev_;                                    \
    st_prev_ = n_;                                              \
  } while (0)
#else
#define PCG_STAMP(i) \
  do {               \
  } while (0)
#endif

// Workgroup sums in two halves: red_put stores the wave's total in slot w of a
// 16-slot area (slots of absent waves hold 0); after the next barrier
// red_total reads all slots and reduces them by DPP.  A fixed tree: the result
// is deterministic and independent of the problem's batch neighbours.  Split
// this way, a reduction rides on a barrier the iteration needs anyway.  (Reading
// the slots as broadcast ds_read_b128 and adding them in the same tree measured
// slower: the compiler splits the reads into two dependent LDS round trips.)
__device__ __forceinline__ void red_put(double v, double* red) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
}
__device__ __forceinline__ double red_total(const double* red) {
  return readlane_f64(dpp_row_sum(red[threadIdx.x & 15]), 0);
}

// Neighbour flags instead of two of the iteration's workgroup barriers.  The products S p and
// S_{k,k+-1} w read block vectors of the lane's own block and of blocks k - 1, k + 1 only; the rows a
// wave reads past its own lie in the waves just before and after it (a block is at most NX <= 16 rows,
// a wave 64 lanes), so a wave needs the vector published by waves w - 1, w + 1 (its own writes precede
// its reads in program order), not by the whole workgroup.  The writer's release fence drains the
// wave's LDS writes (s_waitcnt lgkmcnt(0)) before lane 0 stores the epoch; the reader polls both
// neighbours' epochs (wave-uniform ds_read, s_sleep between polls) and acquires.  Write-after-read
// safety comes from the iteration's remaining full barriers (B2: alpha, B4: nu'), which lie between a
// vector's last readers of one iteration and its writers of the next.
// TMPC_PCG_NB: which of B1 (bit 0) / B3 (bit 1) become neighbour waits; TMPC_PCG_NB_SLEEP: s_sleep 1
// between polls (experiment builds)
#ifndef TMPC_PCG_NB
#define TMPC_PCG_NB 0
#endif
#ifndef TMPC_PCG_NB_SLEEP
#define TMPC_PCG_NB_SLEEP 1
#endif
__device__ __forceinline__ void nb_signal(int* flags, int epoch) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if ((threadIdx.x & 63) == 0) __hip_atomic_store(flags + (threadIdx.x >> 6), epoch, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void nb_wait(const int* flags, int epoch) {
  const int w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  const int lo = w > 0 ? w - 1 : w, hi = w + 1 < nw ? w + 1 : w;
  while (true) {
    const int a = __hip_atomic_load(flags + lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const int b = __hip_atomic_load(flags + hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (__builtin_amdgcn_readfirstlane(a < b ? a : b) >= epoch) break;
    if (TMPC_PCG_NB_SLEEP) __builtin_amdgcn_s_sleep(1);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// t = r - (S_{k,k-1} w_{k-1} + S_{k,k+1} w_{k+1}) for this lane's rows
template <int NX, int RPL, class RT>
__device__ __forceinline__ void pcg_off(const RT (&R)[RPL], const double* __restrict__ w, int kb,
                                        const double (&r)[RPL], double (&t)[RPL]) {
  const double* wm = w + kb - NX;
  constexpr int NC = RPL == 1 ? 2 : 1;
  double a[NC][RPL];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int m = 0; m < RPL; ++m) a[c][m] = 0.0;
#pragma unroll
  for (int j = 0; j < NX; ++j) {
    const double wl = wm[j], wu = wm[2 * NX + j];
#pragma unroll
    for (int m = 0; m < RPL; ++m) {
      a[0][m] += R[m].sl[j] * wl;
      a[NC - 1][m] += R[m].su[j] * wu;
    }
    PCG_LOAD_FENCE(RT, j, a[0])
  }
#pragma unroll
  for (int m = 0; m < RPL; ++m) t[m] = r[m] - (NC == 2 ? a[0][m] + a[NC - 1][m] : a[0][m]);
}

// The CG iteration (PCG.pcg, PCG.py:66-111), arranged around as few workgroup
// barriers as its data dependences allow -- SS 4 per iteration, BJ / J / 0 3:
//   B1  p visible       Ap = S p (own rows) to LDS, partial p.Ap
//   B2  p.Ap, Ap        alpha; every lane rebuilds r_k - Ap_k alpha for its whole
//                       block k from the LDS copies of r and Ap (the owners' update,
//                       operand for operand), x += p alpha, new r to the other r buffer;
//                       SS: w = P_kk r_k to LDS; BJ: z = P_kk r_k; J / 0: z = r / S_ii, r;
//                       BJ / J / 0: partial nu' = r.z
//   B3  SS: w           t = r - S_{k,k-1} w_{k-1} - S_{k,k+1} w_{k+1} to LDS,
//                       partial nu' = w.t  (= r^T P_kk t = r.z, P_kk symmetric)
//   B4  SS: t, nu'      z = P_kk t_k   (the symmetric-stair P^-1 r, PCG.py:181-212)
//   then                beta = nu'/nu, p = z + p beta to LDS -> B1
// The element updates are the reference's (r - Ap alpha, x + p alpha, z + p beta);
// hipcc contracts each into one fused multiply-add (__dmul_rn is a plain product
// here), one rounding where NumPy has two, and the summation order of the dot and
// block products differs -- iteration counts stay exact on every fixture.  x = the lane's
// entries of the solution.
template <int NX, int RPL, int PRE, class RT>
__device__ __forceinline__ void pcg_run(const RT (&R)[RPL], const PcgLane<NX, RPL>& ln, int N,
                                        const PcgLds& L, const double (&bv)[RPL], const double* guess_v, double tol,
                                        int max_iter, double* tn, double* tr, int* iters_out, double (&xv)[RPL]) {
  const int kb = ln.k * NX;
  const int t = ln.t;
#ifdef TMPC_PCG_STAMPS
  unsigned long long st_[16] = {}, st_prev_ = __builtin_amdgcn_s_memtime();
  double* const tn_st = tn;
  tn = nullptr;
  tr = nullptr;
#endif
  auto put = [&](double* buf, const double (&v)[RPL]) {
    if (ln.valid) {
#pragma unroll
      for (int m = 0; m < RPL; ++m) buf[ln.row(m)] = v[m];
    }
  };
  auto partial = [&](const double (&a)[RPL], const double (&b)[RPL]) -> double {
    double s = 0.0;
#pragma unroll
    for (int m = 0; m < RPL; ++m) s += a[m] * b[m];
    return ln.valid ? s : 0.0;
  };
  double* const redA = L.red;         // p.Ap
  double* const redB = L.red + 16;    // nu'
  double* const redC = L.red + 32;    // initial nu, true residual
  // With two rows per lane the search direction p and the iterate x live only
  // in LDS (own rows re-read where needed): the VGPR budget of 2 waves per SIMD
  // holds the 96 matrix doubles per lane and little else.
  constexpr bool IN_LDS = RPL > 1;
  double rv[RPL], zv[RPL], pv[RPL], av[RPL];
  __syncthreads();   // the caller's pcg_lds_clear (pads, reduction slots) is complete
  // x0 = guess (default zeros, PCG.py:11-12); r = b - A x0 (:76)
#pragma unroll
  for (int m = 0; m < RPL; ++m) {
    xv[m] = (guess_v && ln.valid) ? guess_v[ln.row(m)] : 0.0;
    rv[m] = bv[m];
  }
  if (guess_v || IN_LDS) put(L.xbuf, xv);
  if (guess_v) {
    __syncthreads();
    pcg_spmv<NX, RPL>(R, L.xbuf, kb, av);
#pragma unroll
    for (int m = 0; m < RPL; ++m) rv[m] = bv[m] - av[m];
  }
  auto true_residual = [&]() -> double {
    // ||b - A x|| (PCG.py:83,95), trace only; the barrier also orders x's LDS copy
    if (!IN_LDS) put(L.xbuf, xv);
    __syncthreads();
    double e[RPL];
    pcg_spmv<NX, RPL>(R, L.xbuf, kb, e);
#pragma unroll
    for (int m = 0; m < RPL; ++m) e[m] = bv[m] - e[m];
    red_put(partial(e, e), redC);
    __syncthreads();
    const double s = red_total(redC);
    __syncthreads();   // slot C is reused by the next call
    return sqrt(s);
  };
  // z = P^-1 r, nu = r^T z (:77-79)
  put(L.rbuf[0], rv);
  double nu;
  if (PRE == PRECOND_BJ || PRE == PRECOND_SS) {
    __syncthreads();
    double w[RPL];
    pcg_block_dot<NX, RPL>(R, L.rbuf[0] + kb, w);
    if (PRE == PRECOND_BJ) {
#pragma unroll
      for (int m = 0; m < RPL; ++m) zv[m] = w[m];
      red_put(partial(rv, zv), redC);
      __syncthreads();
    } else {
      put(L.wbuf, w);
      __syncthreads();
      double tv[RPL];
      pcg_off<NX, RPL>(R, L.wbuf, kb, rv, tv);
      put(L.tbuf, tv);
      red_put(partial(w, tv), redC);
      __syncthreads();
      pcg_block_dot<NX, RPL>(R, L.tbuf + kb, zv);
    }
  } else {
#pragma unroll
    for (int m = 0; m < RPL; ++m) zv[m] = PRE == PRECOND_J ? R[m].pr[0] * rv[m] : rv[m];
    red_put(partial(rv, zv), redC);
    __syncthreads();
  }
  nu = red_total(redC);
  __syncthreads();   // slot C free again
#pragma unroll
  for (int m = 0; m < RPL; ++m) pv[m] = zv[m];
  put(L.pbuf, pv);
  if (TMPC_PCG_NB & 1) nb_signal(L.flags, 1);
  if (tn && t == 0) tn[0] = fabs(nu);
  if (tr) {
    const double rn = true_residual();
    if (t == 0) tr[0] = rn;
  }
  int it_done = max_iter;
  int cur = 0;
  for (int it = 0; it < max_iter; ++it) {
    PCG_STAMP(0);
    if (TMPC_PCG_NB & 1)
      nb_wait(L.flags, it + 1);                        // B1: p of the neighbour waves
    else
      __syncthreads();                                 // B1: p
    PCG_STAMP(1);
    pcg_spmv<NX, RPL>(R, L.pbuf, kb, av);
    double po[RPL];
#pragma unroll
    for (int m = 0; m < RPL; ++m) po[m] = IN_LDS ? (ln.valid ? L.pbuf[ln.row(m)] : 0.0) : pv[m];
    if (PRE == PRECOND_BJ || PRE == PRECOND_SS) put(L.abuf, av);   // J / 0 need only their own rows
    red_put(partial(po, av), redA);
    PCG_STAMP(2);
    __syncthreads();                                   // B2: p.Ap, Ap
    PCG_STAMP(3);
    const double alpha = nu / red_total(redA);
    double w[RPL];
    if (PRE == PRECOND_BJ || PRE == PRECOND_SS) {
      // r_k - Ap_k alpha for the whole block; w = P_kk (new r_k); own rows kept
      const double* ro = (cur ? L.rbuf[1] : L.rbuf[0]) + kb;   // no dynamic index: keeps L out of scratch
      const double* ap = L.abuf + kb;
      constexpr int NC = RPL == 1 ? 2 : 1;
      double acc[NC][RPL];
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int m = 0; m < RPL; ++m) acc[c][m] = 0.0;
#pragma unroll
      for (int j = 0; j < NX; ++j) {
        const double rj = __dsub_rn(ro[j], __dmul_rn(ap[j], alpha));
#pragma unroll
        for (int m = 0; m < RPL; ++m) acc[j % NC][m] += R[m].pr[j] * rj;
        PCG_LOAD_FENCE(RT, j, acc[0])
      }
      // own rows from the registers: the same operands as the LDS copies
      // (ro[r(m)] = rv[m], ap[r(m)] = av[m]), the same expression, the same value
#pragma unroll
      for (int m = 0; m < RPL; ++m) rv[m] = __dsub_rn(rv[m], __dmul_rn(av[m], alpha));
#pragma unroll
      for (int m = 0; m < RPL; ++m) w[m] = NC == 2 ? acc[0][m] + acc[NC - 1][m] : acc[0][m];
    } else {
#pragma unroll
      for (int m = 0; m < RPL; ++m) rv[m] = __dsub_rn(rv[m], __dmul_rn(av[m], alpha));
    }
    if (IN_LDS) {
      if (ln.valid) {
#pragma unroll
        for (int m = 0; m < RPL; ++m) L.xbuf[ln.row(m)] = __dadd_rn(L.xbuf[ln.row(m)], __dmul_rn(po[m], alpha));
      }
    } else {
#pragma unroll
      for (int m = 0; m < RPL; ++m) xv[m] = __dadd_rn(xv[m], __dmul_rn(po[m], alpha));
    }
    if (PRE == PRECOND_BJ || PRE == PRECOND_SS) put(cur ? L.rbuf[0] : L.rbuf[1], rv);
    cur ^= 1;
    double nup;
    if (PRE == PRECOND_SS) {
      put(L.wbuf, w);
      if (TMPC_PCG_NB & 2) nb_signal(L.flags + 16, it + 1);
      PCG_STAMP(4);
      if (TMPC_PCG_NB & 2)
        nb_wait(L.flags + 16, it + 1);                 // B3: w of the neighbour waves
      else
        __syncthreads();                               // B3: w
      PCG_STAMP(5);
      double tv[RPL];
      pcg_off<NX, RPL>(R, L.wbuf, kb, rv, tv);
      put(L.tbuf, tv);
      red_put(partial(w, tv), redB);
      PCG_STAMP(6);
      __syncthreads();                                 // B4: t, nu'
      PCG_STAMP(7);
      nup = red_total(redB);
      pcg_block_dot<NX, RPL>(R, L.tbuf + kb, zv);
    } else {
#pragma unroll
      for (int m = 0; m < RPL; ++m)
        zv[m] = PRE == PRECOND_BJ ? w[m] : (PRE == PRECOND_J ? R[m].pr[0] * rv[m] : rv[m]);
      red_put(partial(rv, zv), redB);
      PCG_STAMP(4);
      __syncthreads();                                 // B3: nu'
      PCG_STAMP(5);
      nup = red_total(redB);
    }
    PCG_STAMP(8);
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
#pragma unroll
    for (int m = 0; m < RPL; ++m) pv[m] = __dadd_rn(zv[m], __dmul_rn(po[m], beta));
    put(L.pbuf, pv);
    if (TMPC_PCG_NB & 1) nb_signal(L.flags, it + 2);
    nu = nup;
    PCG_STAMP(9);
  }
  if (IN_LDS) {
    __syncthreads();
#pragma unroll
    for (int m = 0; m < RPL; ++m) xv[m] = ln.valid ? L.xbuf[ln.row(m)] : 0.0;
  }
#ifdef TMPC_PCG_STAMPS
  if (tn_st && (t == 0 || t == ((int)blockDim.x - 1) / 64 * 64)) {
    double* o = tn_st + (t == 0 ? 0 : 16);
    for (int i = 0; i < 16; ++i) o[i] = (double)st_[i];
  }
#endif
  *iters_out = it_done;
}

template <int NX, int RPL, class RT>
__device__ __forceinline__ void pcg_dispatch(int precond, const RT (&R)[RPL], const PcgLane<NX, RPL>& ln,
                                             int N, const PcgLds& L, const double (&bv)[RPL], const double* guess_v,
                                             double tol, int max_iter, double* tn, double* tr, int* iters_out,
                                             double (&xv)[RPL]) {
  if (precond == PRECOND_J)
    pcg_run<NX, RPL, PRECOND_J>(R, ln, N, L, bv, guess_v, tol, max_iter, tn, tr, iters_out, xv);
  else if (precond == PRECOND_BJ)
    pcg_run<NX, RPL, PRECOND_BJ>(R, ln, N, L, bv, guess_v, tol, max_iter, tn, tr, iters_out, xv);
  else if (precond == PRECOND_NONE)
    pcg_run<NX, RPL, PRECOND_NONE>(R, ln, N, L, bv, guess_v, tol, max_iter, tn, tr, iters_out, xv);
  else
    pcg_run<NX, RPL, PRECOND_SS>(R, ln, N, L, bv, guess_v, tol, max_iter, tn, tr, iters_out, xv);
}

// Rows per lane for an N x NX block system.  One row per lane up to 768 rows
// (12 waves, 3 per SIMD): measured fastest for PCG-SS at arm6 N = 64 (two rows
// per lane halve the LDS traffic but leave 2 waves per SIMD to hide the 9-cycle
// fp64 FMA latency, and the VGPR budget of 256 then barely holds the matrix
// rows).  Two rows per lane (<= 8 waves) for 769..1024 rows.
#ifndef TMPC_RPL1_MAX_ROWS
#define TMPC_RPL1_MAX_ROWS 768
#endif
__host__ __device__ inline int pcg_rpl(int N, int NX) { return (N * NX <= TMPC_RPL1_MAX_ROWS || (NX & 1)) ? 1 : 2; }

}  // namespace tmpc
