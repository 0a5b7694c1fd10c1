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

#include "env.hpp"

namespace msc {

typedef float mlp_f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int mfma_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// Optional epilogue: the rollout's Gaussian action sampling (msc_gaussian_sample's arithmetic,
// operation for operation, so the results are bit-identical to the separate kernel) applied to the
// KO outputs of row j while they are in registers: one kernel launch and the mean's HBM round trip
// fewer per rollout step. act == nullptr: no sampling.
template <int VKO>
__device__ __forceinline__ void sample_row(const MlpSample& sm, int64_t j, int KO, const float (&m)[VKO]) {
  const float half_log_2pi = 0.91893853320467274178f;  // 0.5 * log(2 pi)
  const float* lsr = sm.log_std + (j % sm.ls_rows) * KO;
  float lp = 0.0f;
#pragma unroll
  for (int a = 0; a < VKO; a++) {
    if (a < KO) {
      const int64_t i = j * KO + a;
      const float ls = fmaxf(lsr[a], sm.floor_);
      const float sd = expf(ls);
      const float v = m[a] + sd * sm.eps[i];
      sm.act[i] = v;
      const float d = v - m[a];
      lp += (-(d * d) / (2.0f * sd * sd) - ls) - half_log_2pi;
      sm.clipped[i] = fminf(fmaxf(v, -1.0f), 1.0f);
    }
  }
  sm.logp[j] = lp;
}

// NT1 / NT2: hidden tiles of 32 units; P: output tiles of layer 2 held at once (register budget:
// 16 NT1 + 16 P + 16 accumulators + 2 x 4 P weight registers per lane).
// Weight fragments are software-pipelined one step ahead (the loads of step s + 1 are issued before
// the MFMAs of step s): with one wave per SIMD nothing else hides an L2 round trip, and a wait on
// each step's own loads cost ~35 % of the MFMA time.
// VKO > 0: the output layer (KO <= VKO <= 8 outputs) on the VALU instead of a 32-row MFMA tile
// padded from KO rows (an output MFMA tile of 5 actions is 84 % padding: 128 of the actor's 1,312
// MFMAs). Each lane accumulates its half of the hidden units into VKO f32 sums with the weights read
// from LDS (all lanes of a half read the same 32 bytes: broadcast), and the two halves are added
// with one lane exchange. The packed w3 is then [NT2 * 16][2][8] floats (zero past KO).
// IL (VKO > 0, P < NT2): the VALU output layer of pass p - 1 interleaved into the layer-2 MFMA stream
// of pass p (IPS units per k step), so its VALU work issues while the MFMAs execute instead of after
// them; only the last pass's output layer runs alone. Same accumulation order as IL = false.
template <int NT1, int NT2, int P, int WPE, int VKO, bool IL = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) void mlp3_relu_kernel(
    const float* __restrict__ x, int64_t n, int L, int KS1, const float4* __restrict__ w1p, const float* __restrict__ b1,
    const float4* __restrict__ w2p, const float* __restrict__ b2, const float4* __restrict__ w3p,
    const float* __restrict__ b3, int KO, float* __restrict__ out, const float* __restrict__ pre1, int grp, int prio,
    MlpSample sm) {
  static_assert(NT2 % P == 0, "layer-2 passes");
  static_assert(VKO >= 0 && VKO <= 8, "VALU output layer: at most 8 outputs");
  constexpr int S4 = NT1 * 4;  // layer-2 k steps of 4 MFMAs (2 hidden units each)
  // the policy forward is on the rollout's critical path (step t + 1 needs its actions), the
  // pipelined demand kernel of step t + 1 (priorities 1-2) is not: issue ahead of it
  if (prio) __builtin_amdgcn_s_setprio(3);
  const int lane = threadIdx.x & 63, h = lane >> 5;
  const int64_t tile = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  __shared__ float4 w3s[VKO > 0 ? NT2 * 16 * 2 * 2 : 1];  // [s][h][8 floats]
  if constexpr (VKO > 0) {
    for (int i = threadIdx.x; i < NT2 * 16 * 2 * 2; i += blockDim.x) w3s[i] = w3p[i];
    __syncthreads();
  }
  if (tile * 32 >= n) return;  // wave-uniform (no block-level synchronisation below)
  const int64_t j = tile * 32 + (lane & 31);
  const bool jv = j < n;
  const int M4 = (KS1 + 3) / 4;  // layer-1 k steps of 4 MFMAs

  // layer 1: H1^T = W1 X^T + b1 (+ pre1 of the sample's group); lane half h feeds features
  // h KS1 + m, m < KS1, of its sample
  // (registers 4g .. 4g + 3 of a tile hold rows 8g + 4h .. 8g + 4h + 3: one float4 per group)
  mlp_f32x16 a1[NT1];
#pragma unroll
  for (int t = 0; t < NT1; t++)
#pragma unroll
    for (int g = 0; g < 4; g++) {
      const float4 v = *reinterpret_cast<const float4*>(b1 + t * 32 + 8 * g + 4 * h);
      a1[t][4 * g] = v.x, a1[t][4 * g + 1] = v.y, a1[t][4 * g + 2] = v.z, a1[t][4 * g + 3] = v.w;
    }
  if (pre1 != nullptr) {  // a first-layer term shared by grp consecutive rows (MAPPO critic: the env's global block)
    const float* pg = pre1 + ((jv ? j : 0) / grp) * (int64_t)(NT1 * 32);
#pragma unroll
    for (int t = 0; t < NT1; t++)
#pragma unroll
      for (int g = 0; g < 4; g++) {
        const float4 v = *reinterpret_cast<const float4*>(pg + t * 32 + 8 * g + 4 * h);
        a1[t][4 * g] += v.x, a1[t][4 * g + 1] += v.y, a1[t][4 * g + 2] += v.z, a1[t][4 * g + 3] += v.w;
      }
  }
  const float* xr = x + (jv ? j : 0) * (int64_t)L;
  auto load_x = [&](int m4, float (&xv)[4]) {
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int m = m4 * 4 + i, k = h * KS1 + m;
      xv[i] = (jv && m < KS1 && k < L) ? xr[k] : 0.0f;
    }
  };
  {
    float xc[4], xn[4];
    float4 wc[NT1], wn[NT1];
    load_x(0, xc);
#pragma unroll
    for (int t = 0; t < NT1; t++) wc[t] = w1p[((int64_t)t * M4) * 64 + lane];
    for (int m4 = 0; m4 < M4; m4++) {
      const bool more = m4 + 1 < M4;
      if (more) {
        load_x(m4 + 1, xn);
#pragma unroll
        for (int t = 0; t < NT1; t++) wn[t] = w1p[((int64_t)t * M4 + m4 + 1) * 64 + lane];
      }
      __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of this step's MFMAs
#pragma unroll
      for (int t = 0; t < NT1; t++) {
        a1[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(wc[t].x, xc[0], a1[t], 0, 0, 0);
        a1[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(wc[t].y, xc[1], a1[t], 0, 0, 0);
        a1[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(wc[t].z, xc[2], a1[t], 0, 0, 0);
        a1[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(wc[t].w, xc[3], a1[t], 0, 0, 0);
      }
      if (more) {
#pragma unroll
        for (int i = 0; i < 4; i++) xc[i] = xn[i];
#pragma unroll
        for (int t = 0; t < NT1; t++) wc[t] = wn[t];
      }
    }
  }
#pragma unroll
  for (int t = 0; t < NT1; t++)
#pragma unroll
    for (int r = 0; r < 16; r++) a1[t][r] = fmaxf(a1[t][r], 0.0f);

  // layers 2 and 3 in passes of P output tiles: the output layer accumulates each pass's slice of
  // the hidden units as soon as it is final, so H2 is never held whole
  mlp_f32x16 a3;
  float o3[VKO > 0 ? VKO : 1];
  if constexpr (VKO > 0) {
#pragma unroll
    for (int a = 0; a < VKO; a++) o3[a] = (h == 0 && a < KO) ? b3[a] : 0.0f;
  } else {
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const int row = mfma_row(r, h);
      a3[r] = row < KO ? b3[row] : 0.0f;
    }
  }
  // one unit of the VALU output layer: hidden unit (tile q of pass pp, register r) into the outputs
  auto l3_unit = [&](const mlp_f32x16 (&src)[P], int pp, int q, int r) {
    if constexpr (VKO > 0) {
      const float hv = fmaxf(src[q][r], 0.0f);
      const int sidx = ((pp * P + q) * 16 + r) * 2 + h;
      const float4 wa = w3s[sidx * 2];
      const float wv[8] = {wa.x, wa.y, wa.z, wa.w, 0.f, 0.f, 0.f, 0.f};
      float wh[4] = {0.f, 0.f, 0.f, 0.f};
      if constexpr (VKO > 4) {
        const float4 wb = w3s[sidx * 2 + 1];
        wh[0] = wb.x, wh[1] = wb.y, wh[2] = wb.z, wh[3] = wb.w;
      }
#pragma unroll
      for (int a = 0; a < VKO; a++) o3[a] = fmaf(a < 4 ? wv[a] : wh[a - 4], hv, o3[a]);
    }
  };
  constexpr bool ILV = IL && VKO > 0 && P < NT2;
  constexpr int IPS = (P * 16 + S4 - 1) / S4;  // interleaved output-layer units per k step
  mlp_f32x16 a2p[ILV ? P : 1];                 // the previous pass's layer-2 sums (ILV)
  float4 w[2][P];  // [step parity][tile]: the fragments of step s4 and s4 + 1
#pragma unroll
  for (int q = 0; q < P; q++) w[0][q] = w2p[((int64_t)q * S4) * 64 + lane];
#pragma unroll
  for (int p = 0; p < NT2 / P; p++) {
    mlp_f32x16 a2[P];
#pragma unroll
    for (int q = 0; q < P; q++)
#pragma unroll
      for (int g = 0; g < 4; g++) {
        const float4 v = *reinterpret_cast<const float4*>(b2 + (p * P + q) * 32 + 8 * g + 4 * h);
        a2[q][4 * g] = v.x, a2[q][4 * g + 1] = v.y, a2[q][4 * g + 2] = v.z, a2[q][4 * g + 3] = v.w;
      }
#pragma unroll
    for (int s4 = 0; s4 < S4; s4++) {
      const int cb = (p * S4 + s4) & 1;
      // prefetch: the next step of this pass, or the first step of the next pass
      if (s4 + 1 < S4) {
#pragma unroll
        for (int q = 0; q < P; q++) w[cb ^ 1][q] = w2p[((int64_t)(p * P + q) * S4 + s4 + 1) * 64 + lane];
      } else if (p + 1 < NT2 / P) {
#pragma unroll
        for (int q = 0; q < P; q++) w[cb ^ 1][q] = w2p[((int64_t)((p + 1) * P + q) * S4) * 64 + lane];
      }
      // the scheduler would otherwise sink the prefetch into the registers this step frees last,
      // i.e. 8 MFMAs before their use instead of 4 P
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int s = s4 * 4 + i;
        const float bv = a1[s / 16][s % 16];
#pragma unroll
        for (int q = 0; q < P; q++) {
          const float4& wq = w[cb][q];
          const float wv = i == 0 ? wq.x : i == 1 ? wq.y : i == 2 ? wq.z : wq.w;
          a2[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(wv, bv, a2[q], 0, 0, 0);
        }
      }
      if constexpr (ILV) {  // the previous pass's output layer, IPS units behind these MFMAs
        if (p > 0) {
#pragma unroll
          for (int i = 0; i < IPS; i++) {
            const int u = s4 * IPS + i;
            if (u < P * 16) l3_unit(a2p, p - 1, u / 16, u % 16);
          }
        }
      }
    }
    if constexpr (VKO > 0) {  // layer 3 on the VALU: o[a] += W3[a][hidden] relu(h2) over this lane's half
      if constexpr (ILV) {
        if (p + 1 < NT2 / P) {  // (interleaved into the next pass)
#pragma unroll
          for (int q = 0; q < P; q++) a2p[q] = a2[q];
          continue;
        }
      }
#pragma unroll
      for (int q = 0; q < P; q++)
#pragma unroll
        for (int r = 0; r < 16; r++) l3_unit(a2, p, q, r);
      continue;
    }
    // layer 3 on this pass's slice: the fragments of tile q + 1 are in flight during tile q
    float4 w3[2][4];
#pragma unroll
    for (int r4 = 0; r4 < 4; r4++) w3[0][r4] = w3p[((int64_t)(p * P) * 4 + r4) * 64 + lane];
#pragma unroll
    for (int q = 0; q < P; q++) {
      if (q + 1 < P) {
#pragma unroll
        for (int r4 = 0; r4 < 4; r4++) w3[(q + 1) & 1][r4] = w3p[((int64_t)(p * P + q + 1) * 4 + r4) * 64 + lane];
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int r4 = 0; r4 < 4; r4++) {
        const float4 wq = w3[q & 1][r4];
        a3 = __builtin_amdgcn_mfma_f32_32x32x2f32(wq.x, fmaxf(a2[q][r4 * 4 + 0], 0.0f), a3, 0, 0, 0);
        a3 = __builtin_amdgcn_mfma_f32_32x32x2f32(wq.y, fmaxf(a2[q][r4 * 4 + 1], 0.0f), a3, 0, 0, 0);
        a3 = __builtin_amdgcn_mfma_f32_32x32x2f32(wq.z, fmaxf(a2[q][r4 * 4 + 2], 0.0f), a3, 0, 0, 0);
        a3 = __builtin_amdgcn_mfma_f32_32x32x2f32(wq.w, fmaxf(a2[q][r4 * 4 + 3], 0.0f), a3, 0, 0, 0);
      }
    }
  }
  if constexpr (VKO > 0) {
#pragma unroll
    for (int a = 0; a < VKO; a++) o3[a] += __shfl_xor(o3[a], 32);  // the other half's hidden units
    if (jv && h == 0) {
      if (out) {
#pragma unroll
        for (int a = 0; a < VKO; a++)
          if (a < KO) out[j * KO + a] = o3[a];
      }
      if constexpr (VKO > 0) {
        if (sm.act) sample_row<VKO>(sm, j, KO, o3);
      }
    }
  } else if (jv && out) {  // (no sampling epilogue on the MFMA output layer: the host checks)
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const int row = mfma_row(r, h);
      if (row < KO) out[j * KO + row] = a3[r];
    }
  }
}

// Fused Linear -> ReLU -> Linear (one hidden layer: the reference's IPPO actor / critic [256],
// config_files/algorithms/ippo.yaml:46,52; the test configs' [128] and [1024] heads): the hidden
// layer is produced TB tiles of 32 units at a time (layer 1 exactly as in mlp3_relu_kernel) and
// folded into the output accumulators as soon as it is final, so any hidden size up to 1024 runs
// with 16 TB accumulator registers. VKO > 0: output layer on the VALU (weights in LDS), else on
// the MFMA (fragments from L2, KO <= 32 rows).
template <int TB, int WPE, int VKO>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) void mlp2_relu_kernel(
    const float* __restrict__ x, int64_t n, int L, int KS1, int NT1, const float4* __restrict__ w1p,
    const float* __restrict__ b1, const float4* __restrict__ w3p, const float* __restrict__ b3, int KO,
    float* __restrict__ out, const float* __restrict__ pre1, int grp, int prio, MlpSample sm) {
  static_assert(VKO >= 0 && VKO <= 8, "VALU output layer: at most 8 outputs");
  if (prio) __builtin_amdgcn_s_setprio(3);
  const int lane = threadIdx.x & 63, h = lane >> 5;
  const int64_t tile = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  extern __shared__ float4 w3d[];  // VALU output layer: [NT1 * 16][2][8 floats]
  if constexpr (VKO > 0) {
    for (int i = threadIdx.x; i < NT1 * 16 * 2 * 2; i += blockDim.x) w3d[i] = w3p[i];
    __syncthreads();
  }
  if (tile * 32 >= n) return;  // wave-uniform
  const int64_t j = tile * 32 + (lane & 31);
  const bool jv = j < n;
  const int M4 = (KS1 + 3) / 4;
  const float* xr = x + (jv ? j : 0) * (int64_t)L;
  const float* pg = pre1 != nullptr ? pre1 + ((jv ? j : 0) / grp) * (int64_t)(NT1 * 32) : nullptr;
  auto load_x = [&](int m4, float (&xv)[4]) {
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int m = m4 * 4 + i, k = h * KS1 + m;
      xv[i] = (jv && m < KS1 && k < L) ? xr[k] : 0.0f;
    }
  };
  mlp_f32x16 a3;
  float o3[VKO > 0 ? VKO : 1];
  if constexpr (VKO > 0) {
#pragma unroll
    for (int a = 0; a < VKO; a++) o3[a] = (h == 0 && a < KO) ? b3[a] : 0.0f;
  } else {
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const int row = mfma_row(r, h);
      a3[r] = row < KO ? b3[row] : 0.0f;
    }
  }
  for (int g0 = 0; g0 < NT1; g0 += TB) {
    mlp_f32x16 a1[TB];
#pragma unroll
    for (int t = 0; t < TB; t++)
#pragma unroll
      for (int q = 0; q < 4; q++) {
        float4 v = *reinterpret_cast<const float4*>(b1 + (g0 + t) * 32 + 8 * q + 4 * h);
        if (pg != nullptr) {
          const float4 u = *reinterpret_cast<const float4*>(pg + (g0 + t) * 32 + 8 * q + 4 * h);
          v.x += u.x, v.y += u.y, v.z += u.z, v.w += u.w;
        }
        a1[t][4 * q] = v.x, a1[t][4 * q + 1] = v.y, a1[t][4 * q + 2] = v.z, a1[t][4 * q + 3] = v.w;
      }
    {
      float xc[4], xn[4];
      float4 wc[TB], wn[TB];
      load_x(0, xc);
#pragma unroll
      for (int t = 0; t < TB; t++) wc[t] = w1p[((int64_t)(g0 + t) * M4) * 64 + lane];
      for (int m4 = 0; m4 < M4; m4++) {
        const bool more = m4 + 1 < M4;
        if (more) {
          load_x(m4 + 1, xn);
#pragma unroll
          for (int t = 0; t < TB; t++) wn[t] = w1p[((int64_t)(g0 + t) * M4 + m4 + 1) * 64 + lane];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < TB; t++) {
          a1[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(wc[t].x, xc[0], a1[t], 0, 0, 0);
          a1[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(wc[t].y, xc[1], a1[t], 0, 0, 0);
          a1[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(wc[t].z, xc[2], a1[t], 0, 0, 0);
          a1[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(wc[t].w, xc[3], a1[t], 0, 0, 0);
        }
        if (more) {
#pragma unroll
          for (int i = 0; i < 4; i++) xc[i] = xn[i];
#pragma unroll
          for (int t = 0; t < TB; t++) wc[t] = wn[t];
        }
      }
    }
    // output layer over this group's hidden units (ReLU applied as they are read)
    if constexpr (VKO > 0) {
#pragma unroll
      for (int t = 0; t < TB; t++)
#pragma unroll
        for (int r = 0; r < 16; r++) {
          const float hv = fmaxf(a1[t][r], 0.0f);
          const int sidx = ((g0 + t) * 16 + r) * 2 + h;
          const float4 wa = w3d[sidx * 2];
          const float wv[4] = {wa.x, wa.y, wa.z, wa.w};
          float wh[4] = {0.f, 0.f, 0.f, 0.f};
          if constexpr (VKO > 4) {
            const float4 wb = w3d[sidx * 2 + 1];
            wh[0] = wb.x, wh[1] = wb.y, wh[2] = wb.z, wh[3] = wb.w;
          }
#pragma unroll
          for (int a = 0; a < VKO; a++) o3[a] = fmaf(a < 4 ? wv[a] : wh[a - 4], hv, o3[a]);
        }
    } else {
#pragma unroll
      for (int t = 0; t < TB; t++)
#pragma unroll
        for (int r4 = 0; r4 < 4; r4++) {
          const float4 wq = w3p[((int64_t)(g0 + t) * 4 + r4) * 64 + lane];
          a3 = __builtin_amdgcn_mfma_f32_32x32x2f32(wq.x, fmaxf(a1[t][r4 * 4 + 0], 0.0f), a3, 0, 0, 0);
          a3 = __builtin_amdgcn_mfma_f32_32x32x2f32(wq.y, fmaxf(a1[t][r4 * 4 + 1], 0.0f), a3, 0, 0, 0);
          a3 = __builtin_amdgcn_mfma_f32_32x32x2f32(wq.z, fmaxf(a1[t][r4 * 4 + 2], 0.0f), a3, 0, 0, 0);
          a3 = __builtin_amdgcn_mfma_f32_32x32x2f32(wq.w, fmaxf(a1[t][r4 * 4 + 3], 0.0f), a3, 0, 0, 0);
        }
    }
  }
  if constexpr (VKO > 0) {
#pragma unroll
    for (int a = 0; a < VKO; a++) o3[a] += __shfl_xor(o3[a], 32);
    if (jv && h == 0) {
      if (out) {
#pragma unroll
        for (int a = 0; a < VKO; a++)
          if (a < KO) out[j * KO + a] = o3[a];
      }
      if constexpr (VKO > 0) {
        if (sm.act) sample_row<VKO>(sm, j, KO, o3);
      }
    }
  } else if (jv && out) {  // (no sampling epilogue on the MFMA output layer: the host checks)
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const int row = mfma_row(r, h);
      if (row < KO) out[j * KO + row] = a3[r];
    }
  }
}

// layer-2 output tiles per pass at 256 hidden units, 1 wave per SIMD: 41 (default) = passes of 4
// tiles with the VALU output layer of each pass interleaved into the next pass's MFMAs (IL; C3 MAPPO
// rollout 1.139 -> 1.093 ms per step beside the demand kernel, profiles/r06/ab_mlp_il.txt), 21 = the
// same with passes of 2, 8 = all of H2 in one pass and the output layer after it (rounds 2-5);
// 4 / 2 = passes of 4 / 2 without interleaving at 2 waves per SIMD (<= 256 VGPRs, spills; A/B).
// MSC_MLP_P8, read at each launch (a test compares the forms)
static int mlp_p8() {
  const char* e = getenv("MSC_MLP_P8");
  const int v = e ? atoi(e) : 41;
  return (v == 8 || v == 4 || v == 2 || v == 41 || v == 21) ? v : 41;
}
// wave priority 3 (MSC_MLP_PRIO=0: default priority, A/B)
static int mlp_prio() {
  static const int v = [] {
    const char* e = getenv("MSC_MLP_PRIO");
    return (e && atoi(e) == 0) ? 0 : 1;
  }();
  return v;
}

// outputs of the VALU output layer for KO outputs (0: MFMA output layer); MSC_MLP_V3=0 forces the
// MFMA one (A/B). The host's weight packing must agree: msc_mlp3_w3_layout reports it.
int mlp3_valu_outputs(int KO) {
  static const int off = [] {
    const char* e = getenv("MSC_MLP_V3");
    return (e && atoi(e) == 0) ? 1 : 0;
  }();
  if (off || KO > 8) return 0;
  return KO <= 2 ? KO : KO <= 4 ? 4 : KO == 5 ? 5 : 8;
}

hipError_t launch_mlp3_relu(const float* x, int64_t n, int L, int H1, int H2, int KO, const float* w1p, const float* b1,
                            const float* w2p, const float* b2, const float* w3p, const float* b3, float* out,
                            const float* pre1, int grp, hipStream_t st, const MlpSample* smp) {
  if (n == 0) return hipSuccess;
  const MlpSample sm = smp ? *smp : MlpSample{};
  if (sm.act && mlp3_valu_outputs(KO) == 0) return hipErrorInvalidValue;  // sampling needs the VALU output layer
  const int KS1 = (L + 1) / 2;
  const int64_t tiles = (n + 31) / 32;
  const dim3 grid((unsigned)((tiles + 3) / 4)), block(256);
  const float4* w1 = reinterpret_cast<const float4*>(w1p);
  const float4* w2 = reinterpret_cast<const float4*>(w2p);
  const float4* w3 = reinterpret_cast<const float4*>(w3p);
#define MSC_MLP_LAUNCH_IL(NT1, NT2, P, WPE, VKO, IL)                                                                   \
  hipLaunchKernelGGL((mlp3_relu_kernel<NT1, NT2, P, WPE, VKO, IL>), grid, block, 0, st, x, n, L, KS1, w1, b1, w2, b2,   \
                     w3, b3, KO, out, pre1, grp, mlp_prio(), sm)
#define MSC_MLP_LAUNCH(NT1, NT2, P, WPE, VKO) MSC_MLP_LAUNCH_IL(NT1, NT2, P, WPE, VKO, false)
  // the output layer on the VALU for KO <= 8 (VKO = 1, 2, 4, 5 or 8: the next supported count >= KO)
  const int vko = mlp3_valu_outputs(KO);
#define MSC_MLP_VKO(NT1, NT2, P, WPE)                                 \
  switch (vko) {                                                      \
    case 1: MSC_MLP_LAUNCH(NT1, NT2, P, WPE, 1); break;               \
    case 2: MSC_MLP_LAUNCH(NT1, NT2, P, WPE, 2); break;               \
    case 4: MSC_MLP_LAUNCH(NT1, NT2, P, WPE, 4); break;               \
    case 5: MSC_MLP_LAUNCH(NT1, NT2, P, WPE, 5); break;               \
    case 8: MSC_MLP_LAUNCH(NT1, NT2, P, WPE, 8); break;               \
    default: MSC_MLP_LAUNCH(NT1, NT2, P, WPE, 0); break;              \
  }
#define MSC_MLP_VKO_IL(NT1, NT2, P, WPE)                                 \
  switch (vko) {                                                         \
    case 1: MSC_MLP_LAUNCH_IL(NT1, NT2, P, WPE, 1, true); break;         \
    case 2: MSC_MLP_LAUNCH_IL(NT1, NT2, P, WPE, 2, true); break;         \
    case 4: MSC_MLP_LAUNCH_IL(NT1, NT2, P, WPE, 4, true); break;         \
    case 5: MSC_MLP_LAUNCH_IL(NT1, NT2, P, WPE, 5, true); break;         \
    case 8: MSC_MLP_LAUNCH_IL(NT1, NT2, P, WPE, 8, true); break;         \
    default: MSC_MLP_LAUNCH(NT1, NT2, P, WPE, 0); break;                 \
  }
  // H1 held whole in registers, H2 in passes of P tiles; (NT1, P) sets the register budget
  // (16 NT1 + 24 P + ~48 per lane) and with it the waves per SIMD
  if (H1 == 256 && H2 == 256) {
    if (mlp_p8() == 41) MSC_MLP_VKO_IL(8, 8, 4, 1)
    else if (mlp_p8() == 21) MSC_MLP_VKO_IL(8, 8, 2, 1)
    else if (mlp_p8() == 8) MSC_MLP_VKO(8, 8, 8, 1)
    else if (mlp_p8() == 4) MSC_MLP_VKO(8, 8, 4, 2)
    else MSC_MLP_VKO(8, 8, 2, 2)
  } else if (H1 == 128 && H2 == 128) {
    MSC_MLP_VKO(4, 4, 4, 2)
  } else if (H1 == 64 && H2 == 64) {
    MSC_MLP_VKO(2, 2, 2, 4)
  } else if (H1 == 64 && H2 == 128) {
    MSC_MLP_VKO(2, 4, 2, 4)
  } else if (H1 == 64 && H2 == 256) {
    MSC_MLP_VKO(2, 8, 2, 4)
  } else if (H1 == 64 && H2 == 512) {
    MSC_MLP_VKO(2, 16, 2, 4)
  } else if (H1 == 128 && H2 == 64) {
    MSC_MLP_VKO(4, 2, 2, 2)
  } else if (H1 == 128 && H2 == 256) {
    MSC_MLP_VKO(4, 8, 4, 2)
  } else if (H1 == 128 && H2 == 512) {
    MSC_MLP_VKO(4, 16, 4, 2)
  } else if (H1 == 256 && H2 == 64) {
    MSC_MLP_VKO(8, 2, 2, 2)
  } else if (H1 == 256 && H2 == 128) {
    MSC_MLP_VKO(8, 4, 4, 2)
  } else if (H1 == 256 && H2 == 512) {
    MSC_MLP_VKO(8, 16, 8, 1)
  } else if (H1 == 512 && H2 == 64) {
    MSC_MLP_VKO(16, 2, 2, 1)
  } else if (H1 == 512 && H2 == 128) {
    MSC_MLP_VKO(16, 4, 4, 1)
  } else if (H1 == 512 && H2 == 256) {
    MSC_MLP_VKO(16, 8, 4, 1)
  } else if (H1 == 512 && H2 == 512) {
    MSC_MLP_VKO(16, 16, 4, 1)
  } else {
    return hipErrorInvalidValue;
  }
#undef MSC_MLP_VKO
#undef MSC_MLP_VKO_IL
#undef MSC_MLP_LAUNCH_IL
#undef MSC_MLP_LAUNCH
  return hipGetLastError();
}

// one hidden layer of H1 = 32 NT1 units (NT1 <= 32): TB tiles per group, the largest power of two
// <= 8 dividing NT1
bool mlp2_supported(int H1) { return H1 >= 32 && H1 <= 1024 && H1 % 32 == 0; }

hipError_t launch_mlp2_relu(const float* x, int64_t n, int L, int H1, int KO, const float* w1p, const float* b1,
                            const float* w3p, const float* b3, float* out, const float* pre1, int grp, hipStream_t st,
                            const MlpSample* smp) {
  if (n == 0) return hipSuccess;
  if (!mlp2_supported(H1)) return hipErrorInvalidValue;
  const MlpSample sm = smp ? *smp : MlpSample{};
  if (sm.act && mlp3_valu_outputs(KO) == 0) return hipErrorInvalidValue;
  const int KS1 = (L + 1) / 2, NT1 = H1 / 32;
  const int TB = NT1 % 8 == 0 ? 8 : NT1 % 4 == 0 ? 4 : NT1 % 2 == 0 ? 2 : 1;
  const int64_t tiles = (n + 31) / 32;
  const dim3 grid((unsigned)((tiles + 3) / 4)), block(256);
  const float4* w1 = reinterpret_cast<const float4*>(w1p);
  const float4* w3 = reinterpret_cast<const float4*>(w3p);
  const int vko = mlp3_valu_outputs(KO);
  const size_t lds = vko > 0 ? (size_t)NT1 * 16 * 2 * 2 * sizeof(float4) : 0;
#define MSC_MLP2_LAUNCH(TBV, WPE, VKO)                                                                              \
  hipLaunchKernelGGL((mlp2_relu_kernel<TBV, WPE, VKO>), grid, block, lds, st, x, n, L, KS1, NT1, w1, b1, w3, b3, KO, \
                     out, pre1, grp, mlp_prio(), sm)
#define MSC_MLP2_VKO(TBV, WPE)                  \
  switch (vko) {                                \
    case 1: MSC_MLP2_LAUNCH(TBV, WPE, 1); break; \
    case 2: MSC_MLP2_LAUNCH(TBV, WPE, 2); break; \
    case 4: MSC_MLP2_LAUNCH(TBV, WPE, 4); break; \
    case 5: MSC_MLP2_LAUNCH(TBV, WPE, 5); break; \
    case 8: MSC_MLP2_LAUNCH(TBV, WPE, 8); break; \
    default: MSC_MLP2_LAUNCH(TBV, WPE, 0); break; \
  }
  switch (TB) {
    case 8: MSC_MLP2_VKO(8, 2) break;
    case 4: MSC_MLP2_VKO(4, 4) break;
    case 2: MSC_MLP2_VKO(2, 4) break;
    default: MSC_MLP2_VKO(1, 4) break;
  }
#undef MSC_MLP2_VKO
#undef MSC_MLP2_LAUNCH
  return hipGetLastError();
}

}  // namespace msc
