// ubench_rng.hip -- micro-benchmarks of the demand kernel's building blocks on gfx950.
// Each kernel runs N draws per lane (one lane = one env, 64-lane blocks) and reports ms.
//   gen        : PCG64 next64 -> double, summed (the LCG advance + XSL-RR + conversion)
//   gen2       : two independent PCG64 streams per lane (ILP x2), N/2 draws each
//   poisson    : gen + the Poisson multiplication test (prod *= U; prod > thr)
//   lds_u      : uniforms read from LDS instead of generated (the split kernel's parser input)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ubench_rng.hip -o tools/ubench_rng
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../marl-sc_amd/csrc/rng.hpp"
using namespace msc;

__global__ __launch_bounds__(64) void k_gen(int n, double* out) {
  Pcg64 r{};
  r.s_lo = blockIdx.x * 64 + threadIdx.x + 1; r.i_lo = 2 * r.s_lo + 1;
  double acc = 0;
  for (int i = 0; i < n; i++) acc += pcg_double(r);
  out[blockIdx.x * 64 + threadIdx.x] = acc;
}
__global__ __launch_bounds__(64) void k_gen2(int n, double* out) {
  Pcg64 a{}, b{};
  a.s_lo = blockIdx.x * 64 + threadIdx.x + 1; a.i_lo = 2 * a.s_lo + 1;
  b.s_lo = a.s_lo * 7; b.i_lo = 2 * b.s_lo + 1;
  double acc = 0, acc2 = 0;
  for (int i = 0; i < n / 2; i++) { acc += pcg_double(a); acc2 += pcg_double(b); }
  out[blockIdx.x * 64 + threadIdx.x] = acc + acc2;
}
__global__ __launch_bounds__(64) void k_poisson(int n, double thr, double* out) {
  Pcg64 r{};
  r.s_lo = blockIdx.x * 64 + threadIdx.x + 1; r.i_lo = 2 * r.s_lo + 1;
  double prod = 1.0; int x = 0, cnt = 0;
  for (int i = 0; i < n; i++) {
    const double pu = prod * pcg_double(r);
    const bool c = pu > thr;
    x += c; cnt += !c;
    prod = c ? pu : 1.0;
  }
  out[blockIdx.x * 64 + threadIdx.x] = x + cnt;
}
__global__ __launch_bounds__(64) void k_lds_u(int n, double thr, double* out) {
  __shared__ double ring[32 * 64];
  for (int i = 0; i < 32; i++) ring[i * 64 + threadIdx.x] = (i + 1) * 0.03;
  __syncthreads();
  double prod = 1.0; int x = 0, cnt = 0;
  for (int i = 0; i < n; i++) {
    const double pu = prod * ring[(i & 31) * 64 + threadIdx.x];
    const bool c = pu > thr;
    x += c; cnt += !c;
    prod = c ? pu : 1.0;
  }
  out[blockIdx.x * 64 + threadIdx.x] = x + cnt;
}

int main(int argc, char** argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 512, n = argc > 2 ? atoi(argv[2]) : 6720;
  double* out;
  hipMalloc(&out, sizeof(double) * blocks * 64);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  auto time = [&](const char* name, auto launch) {
    launch(); hipDeviceSynchronize();
    hipEventRecord(a);
    for (int i = 0; i < 5; i++) launch();
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    printf("%-8s blocks=%d n=%d  %.4f ms  (%.1f ns/draw/wave)\n", name, blocks, n, ms / 5, ms / 5 * 1e6 / n);
  };
  time("gen", [&] { hipLaunchKernelGGL(k_gen, dim3(blocks), dim3(64), 0, 0, n, out); });
  time("gen2", [&] { hipLaunchKernelGGL(k_gen2, dim3(blocks), dim3(64), 0, 0, n, out); });
  time("poisson", [&] { hipLaunchKernelGGL(k_poisson, dim3(blocks), dim3(64), 0, 0, n, exp(-5.0), out); });
  time("lds_u", [&] { hipLaunchKernelGGL(k_lds_u, dim3(blocks), dim3(64), 0, 0, n, exp(-5.0), out); });
  return 0;
}
