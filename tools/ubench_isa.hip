// ubench_isa.hip -- issue cost of the integer / f64 instructions the demand kernel's PCG64 generator
// and Poisson parser are made of, on gfx950. Each kernel runs N iterations of 8 independent
// instructions per lane (inline asm, so the compiler cannot fold them); cycles per instruction are
// measured with s_memtime per wave (lone wave per SIMD: 1 block of 64 threads per CU) and chip-wide
// (WPS waves per SIMD).
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_isa.hip -o tools/ubench_isa
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define REP8(x) x x x x x x x x
#define K_BODY(NAME, ASM)                                                                        \
  __global__ void NAME(int n, unsigned long long* cyc, unsigned* out) {                          \
    unsigned a0 = threadIdx.x + 1, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 9,            \
             a5 = a0 * 11, a6 = a0 * 13, a7 = a0 * 15, b = 0x9e3779b9u;                             \
    unsigned long long t0 = __builtin_readcyclecounter();                                        \
    for (int i = 0; i < n; i++) { ASM }                                                          \
    unsigned long long t1 = __builtin_readcyclecounter();                                        \
    if (threadIdx.x % 64 == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) / 64] = t1 - t0;      \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;          \
  }
#define ONE(op) asm volatile(op : "+v"(a0) : "v"(b)); asm volatile(op : "+v"(a1) : "v"(b)); \
  asm volatile(op : "+v"(a2) : "v"(b)); asm volatile(op : "+v"(a3) : "v"(b));              \
  asm volatile(op : "+v"(a4) : "v"(b)); asm volatile(op : "+v"(a5) : "v"(b));              \
  asm volatile(op : "+v"(a6) : "v"(b)); asm volatile(op : "+v"(a7) : "v"(b));
K_BODY(k_add, ONE("v_add_u32 %0, %0, %1"))
K_BODY(k_mullo, ONE("v_mul_lo_u32 %0, %0, %1"))
K_BODY(k_mulhi, ONE("v_mul_hi_u32 %0, %0, %1"))
K_BODY(k_mul24, ONE("v_mul_u32_u24 %0, %0, %1"))
K_BODY(k_mulhi24, ONE("v_mul_hi_u32_u24 %0, %0, %1"))

// 64-bit ops on register pairs
#define K64(NAME, OP)                                                                            \
  __global__ void NAME(int n, unsigned long long* cyc, unsigned* out) {                          \
    unsigned long long a[8];                                                                     \
    for (int j = 0; j < 8; j++) a[j] = (threadIdx.x + 1) * (j + 3);                              \
    unsigned bb = 0x9e3779b9u;                                                                   \
    double d[8];                                                                                 \
    for (int j = 0; j < 8; j++) d[j] = 1.0 + threadIdx.x * 1e-3 * (j + 1);                      \
    double dm = 0.999999;                                                                        \
    unsigned long long t0 = __builtin_readcyclecounter();                                        \
    for (int i = 0; i < n; i++) {                                                                \
      for (int j = 0; j < 8; j++) { OP }                                                         \
    }                                                                                            \
    unsigned long long t1 = __builtin_readcyclecounter();                                        \
    if (threadIdx.x % 64 == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) / 64] = t1 - t0;      \
    unsigned long long x = 0;                                                                    \
    for (int j = 0; j < 8; j++) x ^= a[j] ^ (unsigned long long)d[j];                           \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (unsigned)x;                                   \
  }
K64(k_mad64, asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(a[j]) : "v"((unsigned)a[j]), "v"(bb) : "vcc");)
K64(k_mulf64, asm volatile("v_mul_f64 %0, %0, %1" : "+v"(d[j]) : "v"(dm));)
K64(k_cmpf64, asm volatile("v_cmp_gt_f64 vcc, %0, %1\n\tv_cndmask_b32 %2, 0, 1, vcc" : "+v"(d[j]) : "v"(dm), "v"(bb) : "vcc");)
K64(k_lshr64, asm volatile("v_lshrrev_b64 %0, 3, %0" : "+v"(a[j]));)

typedef void (*KF)(int, unsigned long long*, unsigned*);
int main(int argc, char** argv) {
  const int n = 4096;
  int ncu = 256;
  unsigned long long* cyc;
  unsigned* out;
  hipMalloc(&cyc, sizeof(unsigned long long) * 256 * 64);
  hipMalloc(&out, sizeof(unsigned) * 256 * 1024 * 4);
  struct { const char* name; KF f; int per_iter; } ks[] = {
      {"v_add_u32", k_add, 8}, {"v_mul_lo_u32", k_mullo, 8}, {"v_mul_hi_u32", k_mulhi, 8},
      {"v_mul_u32_u24", k_mul24, 8}, {"v_mul_hi_u32_u24", k_mulhi24, 8}, {"v_mad_u64_u32", k_mad64, 8},
      {"v_mul_f64", k_mulf64, 8}, {"v_cmp_gt_f64+cndmask", k_cmpf64, 16}, {"v_lshrrev_b64", k_lshr64, 8}};
  unsigned long long h[256 * 16];
  for (auto& k : ks) {
    for (int wps : {1, 4}) {  // waves per SIMD: blocks of 64 * 4 * wps threads, one block per CU
      const int threads = 64 * 4 * wps;
      hipLaunchKernelGGL(k.f, dim3(ncu), dim3(threads), 0, 0, 64, cyc, out);  // warm
      hipEvent_t a, b;
      hipEventCreate(&a); hipEventCreate(&b);
      hipEventRecord(a);
      hipLaunchKernelGGL(k.f, dim3(ncu), dim3(threads), 0, 0, n, cyc, out);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      hipMemcpy(h, cyc, sizeof(unsigned long long) * ncu * (threads / 64), hipMemcpyDeviceToHost);
      double avg = 0; for (int i = 0; i < ncu * threads / 64; i++) avg += h[i]; avg /= ncu * threads / 64;
      // per-wave cycles per instruction; chip time per wave-instruction per SIMD
      const double ins = (double)n * k.per_iter;
      printf("%-24s wps=%d  wave cyc/inst %.2f   SIMD ns/wave-inst %.3f (%.2f cyc at 2.4GHz)\n", k.name, wps,
             avg / ins, ms * 1e6 / (ins * wps), ms * 1e6 / (ins * wps) * 2.4);
    }
  }
  return 0;
}
