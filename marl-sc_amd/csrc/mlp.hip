// Fused inference of the rollout's policy MLP: Linear -> ReLU -> Linear -> ReLU -> Linear
// (MLPArchitecture.build, src/algorithms/models/architectures/mlp.py:14-60, with the actor /
// critic configs of config_files/algorithms/{ippo,mappo}.yaml: hidden [256, 256] or [64, 64]) on
// the f32 MFMA of gfx950 (v_mfma_f32_32x32x2_f32: exact f32 products, f32 accumulation, the f32
// vector rate of 64 FLOP/clk/SIMD).
//
// One wave = 32 samples. Every layer is computed transposed, D = W * X^T (hidden units on the
// MFMA's row axis, samples on its column axis = the lane), because a 32x32 f32 accumulator holds
// column j on lane j & 31 and rows (r & 3) + 8 (r >> 2) + 4 (lane >> 5) in its 16 registers: used
// as the B operand of the next MFMA, register r of lane half h is exactly B[k = h][j] for the
// hidden pair {rho(r, 0), rho(r, 1)} of that tile. So the hidden activations never leave the
// registers (no LDS, no HBM round trip: hipBLASLt writes and re-reads 2 x 256 floats per sample),
// and only the weights are streamed, from L2, in the matching permuted k order: the host packs
// them once per weight version into lane-major fragments (w1p / w2p / w3p below) so that every
// weight load of a wave is one contiguous 1-KiB (float4 per lane) read.
//
// Per 32 samples at 34 -> 256 -> 256 -> 5: 8 x 17 + 8 x 128 + 128 MFMAs (the output layer padded
// to 32 rows), i.e. ~82 k MFMA cycles per wave. Biases initialise the accumulators, so every
// output is an f32 fma chain in k order (a different rounding order than hipBLASLt's: the
// tests compare with the torch layer sequence at f32 GEMM tolerance).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

namespace msc {

typedef float mlp_f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int mfma_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// NT1 / NT2: hidden tiles of 32 units; P: output tiles of layer 2 held at once (register budget:
// 16 NT1 + 16 P + 16 accumulators + 4 P weight registers per lane)
template <int NT1, int NT2, int P, int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) void mlp3_relu_kernel(
    const float* __restrict__ x, int64_t n, int L, int KS1, const float* __restrict__ w1p, const float* __restrict__ b1,
    const float4* __restrict__ w2p, const float* __restrict__ b2, const float4* __restrict__ w3p,
    const float* __restrict__ b3, int KO, float* __restrict__ out, int prio) {
  static_assert(NT2 % P == 0, "layer-2 passes");
  // the policy forward is on the rollout's critical path (step t + 1 needs its actions), the
  // pipelined demand kernel of step t + 1 (priorities 1-2) is not: issue ahead of it
  if (prio) __builtin_amdgcn_s_setprio(3);
  constexpr int S = NT1 * 16;  // layer-2 k steps (2 hidden units each)
  const int lane = threadIdx.x & 63, h = lane >> 5;
  const int64_t tile = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (tile * 32 >= n) return;  // wave-uniform (no block-level synchronisation below)
  const int64_t j = tile * 32 + (lane & 31);
  const bool jv = j < n;

  // layer 1: H1^T = W1 X^T + b1; lane half h feeds features [h KS1, h KS1 + KS1) of its sample
  mlp_f32x16 a1[NT1];
#pragma unroll
  for (int t = 0; t < NT1; t++)
#pragma unroll
    for (int r = 0; r < 16; r++) a1[t][r] = b1[t * 32 + mfma_row(r, h)];
  const float* xr = x + (jv ? j : 0) * (int64_t)L;
  for (int m = 0; m < KS1; m++) {
    const int k = h * KS1 + m;
    const float xv = (jv && k < L) ? xr[k] : 0.0f;
#pragma unroll
    for (int t = 0; t < NT1; t++)
      a1[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(w1p[((int64_t)t * KS1 + m) * 64 + lane], xv, a1[t], 0, 0, 0);
  }
#pragma unroll
  for (int t = 0; t < NT1; t++)
#pragma unroll
    for (int r = 0; r < 16; r++) a1[t][r] = fmaxf(a1[t][r], 0.0f);

  // layers 2 and 3 in passes of P output tiles: the output layer accumulates each pass's slice of
  // the hidden units as soon as it is final, so H2 is never held whole
  mlp_f32x16 a3;
#pragma unroll
  for (int r = 0; r < 16; r++) {
    const int row = mfma_row(r, h);
    a3[r] = row < KO ? b3[row] : 0.0f;
  }
#pragma unroll
  for (int p = 0; p < NT2 / P; p++) {
    mlp_f32x16 a2[P];
#pragma unroll
    for (int q = 0; q < P; q++)
#pragma unroll
      for (int r = 0; r < 16; r++) a2[q][r] = b2[(p * P + q) * 32 + mfma_row(r, h)];
#pragma unroll
    for (int s4 = 0; s4 < S / 4; s4++) {
      float4 w[P];
#pragma unroll
      for (int q = 0; q < P; q++) w[q] = w2p[((int64_t)(p * P + q) * (S / 4) + s4) * 64 + lane];
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int s = s4 * 4 + i;
        const float bv = a1[s / 16][s % 16];
#pragma unroll
        for (int q = 0; q < P; q++) {
          const float wv = i == 0 ? w[q].x : i == 1 ? w[q].y : i == 2 ? w[q].z : w[q].w;
          a2[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(wv, bv, a2[q], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < P; q++) {
#pragma unroll
      for (int r4 = 0; r4 < 4; r4++) {
        const float4 w = w3p[((int64_t)(p * P + q) * 4 + r4) * 64 + lane];
        a3 = __builtin_amdgcn_mfma_f32_32x32x2f32(w.x, fmaxf(a2[q][r4 * 4 + 0], 0.0f), a3, 0, 0, 0);
        a3 = __builtin_amdgcn_mfma_f32_32x32x2f32(w.y, fmaxf(a2[q][r4 * 4 + 1], 0.0f), a3, 0, 0, 0);
        a3 = __builtin_amdgcn_mfma_f32_32x32x2f32(w.z, fmaxf(a2[q][r4 * 4 + 2], 0.0f), a3, 0, 0, 0);
        a3 = __builtin_amdgcn_mfma_f32_32x32x2f32(w.w, fmaxf(a2[q][r4 * 4 + 3], 0.0f), a3, 0, 0, 0);
      }
    }
  }
  if (jv) {
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const int row = mfma_row(r, h);
      if (row < KO) out[j * KO + row] = a3[r];
    }
  }
}

// layer-2 output tiles per pass at 256 hidden units: 8 (all of H2 at once, 1 wave per SIMD, default:
// 1.547 vs 1.610 ms per rollout step) or 4 (<= 256 VGPRs, 2 waves per SIMD; MSC_MLP_P8=4, A/B)
static int mlp_p8() {
  static const int v = [] {
    const char* e = getenv("MSC_MLP_P8");
    return (e && atoi(e) == 4) ? 4 : 8;
  }();
  return v;
}
// wave priority 3 (MSC_MLP_PRIO=0: default priority, A/B)
static int mlp_prio() {
  static const int v = [] {
    const char* e = getenv("MSC_MLP_PRIO");
    return (e && atoi(e) == 0) ? 0 : 1;
  }();
  return v;
}

hipError_t launch_mlp3_relu(const float* x, int64_t n, int L, int H1, int H2, int KO, const float* w1p, const float* b1,
                            const float* w2p, const float* b2, const float* w3p, const float* b3, float* out,
                            hipStream_t st) {
  if (n == 0) return hipSuccess;
  const int KS1 = (L + 1) / 2;
  const int64_t tiles = (n + 31) / 32;
  const dim3 grid((unsigned)((tiles + 3) / 4)), block(256);
  const float4* w2 = reinterpret_cast<const float4*>(w2p);
  const float4* w3 = reinterpret_cast<const float4*>(w3p);
#define MSC_MLP_LAUNCH(NT1, NT2, P, WPE)                                                                          \
  hipLaunchKernelGGL((mlp3_relu_kernel<NT1, NT2, P, WPE>), grid, block, 0, st, x, n, L, KS1, w1p, b1, w2, b2, w3, b3, \
                     KO, out, mlp_prio())
  if (H1 == 256 && H2 == 256) {
    if (mlp_p8() == 8) MSC_MLP_LAUNCH(8, 8, 8, 1);
    else MSC_MLP_LAUNCH(8, 8, 4, 2);
  } else if (H1 == 128 && H2 == 128) {
    MSC_MLP_LAUNCH(4, 4, 4, 2);
  } else if (H1 == 64 && H2 == 64) {
    MSC_MLP_LAUNCH(2, 2, 2, 4);
  } else {
    return hipErrorInvalidValue;
  }
#undef MSC_MLP_LAUNCH
  return hipGetLastError();
}

}  // namespace msc
