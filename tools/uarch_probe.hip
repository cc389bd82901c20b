// Micro-probes for the PCG kernel's design on gfx950: fp64 FMA issue rate and
// dependent latency per wave, and ds_read_b128 throughput for the broadcast
// pattern of the block-tridiagonal SpMV (12 lanes per block reading the same
// 16 B) vs lane-distinct addresses.  Prints cycles from s_memtime.
//   hipcc --offload-arch=gfx950 -O3 -o build_variants/uarch_probe tools/uarch_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                           \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                            \
    }                                                                      \
  } while (0)

// CH independent FMA chains per lane, ITER iterations each
template <int CH>
__global__ void fma_probe(double* out, long long* cyc, int iters, double a, double b) {
  double acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = threadIdx.x * 1e-3 + c;
  __syncthreads();
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int c = 0; c < CH; ++c) acc[c] = fma(acc[c], a, b);
  }
  const long long t1 = clock64();
  double s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// each lane reads NREAD x 16 B per iteration; MODE 0: lane group of 12 shares an
// address (block broadcast, as the SpMV), MODE 1: all lanes distinct, MODE 2: all same
template <int MODE>
__global__ void lds_probe(double* out, long long* cyc, int iters) {
  __shared__ __align__(16) double buf[8192];
  for (int e = threadIdx.x; e < 8192; e += blockDim.x) buf[e] = e * 1e-3;
  __syncthreads();
  const int t = threadIdx.x;
  int base;
  if (MODE == 0) base = (t / 12) * 12;        // doubles
  else if (MODE == 1) base = (t * 2) % 4096;
  else base = 0;
  double acc0 = 0, acc1 = 0;
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
    const double2* p = reinterpret_cast<const double2*>(buf + ((base + it * 2) & 4095));
#pragma unroll
    for (int r = 0; r < 18; ++r) {
      const double2 v = p[r * 6 % 96];
      acc0 += v.x;
      acc1 += v.y;
    }
  }
  const long long t1 = clock64();
  out[blockIdx.x * blockDim.x + t] = acc0 + acc1;
  if (t == 0) cyc[blockIdx.x] = t1 - t0;
}

template <typename K>
static int run(const char* name, K kern, int blocks, int threads, int iters, double per_iter_ops, const char* unit) {
  double* out;
  long long* cyc;
  CHECK(hipMalloc(&out, sizeof(double) * blocks * threads));
  CHECK(hipMalloc(&cyc, sizeof(long long) * blocks));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  kern(out, cyc, 10);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  kern(out, cyc, iters);
  CHECK(hipEventRecord(e1));
  CHECK(hipDeviceSynchronize());
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<long long> c(blocks);
  CHECK(hipMemcpy(c.data(), cyc, sizeof(long long) * blocks, hipMemcpyDeviceToHost));
  double avg = 0;
  for (auto v : c) avg += v;
  avg /= blocks;
  printf("%-34s blocks %5d threads %4d  cycles/iter %8.1f  %s %.2f  wall %.3f ms\n", name, blocks, threads,
         avg / iters, unit, avg / iters / per_iter_ops, ms);
  CHECK(hipFree(out));
  CHECK(hipFree(cyc));
  return 0;
}

int main() {
  const int it = 20000;
  // FMA: per iteration each lane issues 8*CH dependent-or-independent FMAs
  for (int threads : {64, 128, 256, 384, 512, 768}) {
    run("fma chains=1", [&](double* o, long long* c, int n) { hipLaunchKernelGGL(fma_probe<1>, dim3(256), dim3(threads), 0, 0, o, c, n, 1.0000001, 1e-9); }, 256, threads, it, 8.0, "cyc/fma(wave)");
    run("fma chains=4", [&](double* o, long long* c, int n) { hipLaunchKernelGGL(fma_probe<4>, dim3(256), dim3(threads), 0, 0, o, c, n, 1.0000001, 1e-9); }, 256, threads, it, 32.0, "cyc/fma(wave)");
    run("fma chains=8", [&](double* o, long long* c, int n) { hipLaunchKernelGGL(fma_probe<8>, dim3(256), dim3(threads), 0, 0, o, c, n, 1.0000001, 1e-9); }, 256, threads, it, 64.0, "cyc/fma(wave)");
  }
  for (int threads : {64, 256, 384, 768}) {
    run("lds b128 block-broadcast(12)", [&](double* o, long long* c, int n) { hipLaunchKernelGGL(lds_probe<0>, dim3(256), dim3(threads), 0, 0, o, c, n); }, 256, threads, 2000, 18.0, "cyc/read(wave)");
    run("lds b128 distinct", [&](double* o, long long* c, int n) { hipLaunchKernelGGL(lds_probe<1>, dim3(256), dim3(threads), 0, 0, o, c, n); }, 256, threads, 2000, 18.0, "cyc/read(wave)");
    run("lds b128 all-same", [&](double* o, long long* c, int n) { hipLaunchKernelGGL(lds_probe<2>, dim3(256), dim3(threads), 0, 0, o, c, n); }, 256, threads, 2000, 18.0, "cyc/read(wave)");
  }
  return 0;
}
