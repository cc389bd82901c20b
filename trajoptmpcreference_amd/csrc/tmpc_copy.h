// Workgroup copies for the per-problem decision / hand-over kernels (k_soft_outer's stream hand-over,
// k_ls_decide's and k_ilqr_decide's step application, k_stream_init).  One 64-lane workgroup moves a
// problem's rows (a trajectory is 768 doubles at arm6 N = 64): written as `for (e = t; e < n; e += nt)
// dst[e] = src[e]`, each pass's load waited for the previous pass's store whenever the compiler could not
// prove the two rows apart (struct members carry no __restrict__), so a row cost n / nt dependent memory
// round trips -- the slowest workgroup of these launches set their ~30-70 us (profiles/r06/counters).
// Here U passes' loads are issued before any of their stores: one round trip per U passes.  Every element
// is the same expression of the same operands, so the values are unchanged bit for bit.
#pragma once
#include <hip/hip_runtime.h>

namespace tmpc {

// for e in [0, n) step nt from t: st(e, ld(e)), U elements per lane loaded before any is stored
template <int U, class V, class LD, class ST>
__device__ __forceinline__ void wg_batched(int n, int t, int nt, LD ld, ST st) {
  for (int b0 = t; b0 < n; b0 += U * nt) {
    V v[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const int e = b0 + j * nt;
      v[j] = e < n ? ld(e) : V(0);
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const int e = b0 + j * nt;
      if (e < n) st(e, v[j]);
    }
  }
}

// dst[e] = src[e], e in [0, n)
template <int U, class V>
__device__ __forceinline__ void wg_copy(V* dst, const V* src, int n, int t, int nt) {
  wg_batched<U, V>(n, t, nt, [&](int e) { return src[e]; }, [&](int e, V v) { dst[e] = v; });
}

}  // namespace tmpc
