// gae.hip -- advantage estimation for the rollout (RLlib 2.52.1's GAE connector, which the
// reference enables at src/algorithms/mappo.py:154-156 / ippo.py:157-159 and post-processes with
// src/algorithms/learners/hysteretic_learner.py:35-42).
//
// HBM-bound reverse scan over time: layout [T][N] (time-major) so each time row is read by
// consecutive lanes (coalesced 16-B-per-lane when vectorised by 4 sequences per lane).
// Per element: reward f32 + value f32 + done u8 (+ next_value on truncation rows) read,
// advantage f32 + target f32 written = 17 B. Statistics {sum A, sum A^2, n} are reduced per
// block in f64 and added with one f64 atomic per block for the cross-rank standardisation.
#include <hip/hip_runtime.h>

#include <stdlib.h>

#include "env.hpp"

namespace msc {

constexpr int GAE_BS = 256;
constexpr int GAE_MAX_GROUPS = 64;  // statistics groups (RLlib standardises per module: one per agent)

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  return v;
}

// Statistics groups: sequence n (= env * W + agent in the rollout's [T][E*W] layout) belongs to
// group n % G. G = 1 is one standardisation over the whole batch (the shared policy's single
// module); G = W standardises every agent's advantages with its own mean / std, as RLlib's GAE
// connector does for each module of a multi-agent batch when policies are not shared.
__global__ __launch_bounds__(GAE_BS) void gae_kernel(const float* __restrict__ r, const float* __restrict__ v,
                                                     const float* __restrict__ nv, const uint8_t* __restrict__ term,
                                                     const uint8_t* __restrict__ trunc, int64_t N, int32_t T,
                                                     float gamma, float lam, float* __restrict__ adv,
                                                     float* __restrict__ tgt, int32_t G, double* __restrict__ stats) {
  __shared__ double red[3][GAE_MAX_GROUPS];
  const int64_t n = (int64_t)blockIdx.x * GAE_BS + threadIdx.x;
  double s1 = 0.0, s2 = 0.0;
  if (n < N) {
    float a = 0.0f;
    float v_next = v[(int64_t)T * N + n];
    const float gl = gamma * lam;
    for (int t = T - 1; t >= 0; --t) {
      const int64_t i = (int64_t)t * N + n;
      const float vt = v[i];
      const bool te = term && term[i];
      const bool tr = trunc && trunc[i];
      float boot = tr ? (nv ? nv[i] : 0.0f) : v_next;
      if (te) boot = 0.0f;
      const float delta = r[i] + gamma * boot - vt;
      a = delta + ((te || tr) ? 0.0f : gl * a);
      adv[i] = a;
      if (tgt) tgt[i] = a + vt;
      s1 += (double)a;
      s2 += (double)a * (double)a;
      v_next = vt;
    }
  }
  if (!stats) return;
  if (G == 1) {
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    const int wid = threadIdx.x >> 6, ln = threadIdx.x & 63;
    if (ln == 0) {
      red[0][wid] = s1;
      red[1][wid] = s2;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      double a1 = 0.0, a2 = 0.0;
      for (int k = 0; k < GAE_BS / 64; k++) {
        a1 += red[0][k];
        a2 += red[1][k];
      }
      const int64_t cnt = (N - (int64_t)blockIdx.x * GAE_BS) < GAE_BS ? (N - (int64_t)blockIdx.x * GAE_BS) : GAE_BS;
      atomicAdd(&stats[0], a1);
      atomicAdd(&stats[1], a2);
      atomicAdd(&stats[2], (double)cnt * (double)T);
    }
    return;
  }
  for (int g = threadIdx.x; g < G; g += GAE_BS) red[0][g] = red[1][g] = red[2][g] = 0.0;
  __syncthreads();
  if (n < N) {
    const int g = (int)(n % G);
    atomicAdd(&red[0][g], s1);
    atomicAdd(&red[1][g], s2);
    atomicAdd(&red[2][g], (double)T);
  }
  __syncthreads();
  for (int g = threadIdx.x; g < G; g += GAE_BS) {
    if (red[2][g] > 0.0) {
      atomicAdd(&stats[3 * g + 0], red[0][g]);
      atomicAdd(&stats[3 * g + 1], red[1][g]);
      atomicAdd(&stats[3 * g + 2], red[2][g]);
    }
  }
}

// Vectorised variant (N % 4 == 0, term / trunc present): a lane owns 4 adjacent sequences (16-B
// loads and stores of every time row) and reads the rows of CT time steps back to back before it
// scans them, so each wave keeps ~CT x 3 KiB in flight instead of one dependent row at a time (the
// scalar kernel above is bound by one HBM round trip per time step: 34 % of 8 TB/s). Same f32
// arithmetic per element as gae_kernel; next_values is read only on truncated rows.
constexpr int GAE_CT = 8;
__global__ __launch_bounds__(GAE_BS) void gae4_kernel(const float4* __restrict__ r, const float4* __restrict__ v,
                                                      const float* __restrict__ nv, const uchar4* __restrict__ term,
                                                      const uchar4* __restrict__ trunc, int64_t N4, int32_t T,
                                                      float gamma, float lam, float4* __restrict__ adv,
                                                      float4* __restrict__ tgt, int32_t G, double* __restrict__ stats) {
  __shared__ double red[3][GAE_MAX_GROUPS];
  const int64_t q = (int64_t)blockIdx.x * GAE_BS + threadIdx.x;  // sequences 4q .. 4q + 3
  double s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
  if (q < N4) {
    float a[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    const float4 vl = v[(int64_t)T * N4 + q];
    float vn[4] = {vl.x, vl.y, vl.z, vl.w};
    const float gl = gamma * lam;
    for (int t0 = T - 1; t0 >= 0; t0 -= GAE_CT) {
      float4 R[GAE_CT], V[GAE_CT];
      uchar4 TE[GAE_CT], TR[GAE_CT];
#pragma unroll
      for (int j = 0; j < GAE_CT; j++) {
        const int t = t0 - j;
        if (t >= 0) {
          const int64_t i = (int64_t)t * N4 + q;
          R[j] = r[i];
          V[j] = v[i];
          TE[j] = term[i];
          TR[j] = trunc[i];
        }
      }
#pragma unroll
      for (int j = 0; j < GAE_CT; j++) {
        const int t = t0 - j;
        if (t < 0) break;
        const int64_t i = (int64_t)t * N4 + q;
        const float rr[4] = {R[j].x, R[j].y, R[j].z, R[j].w}, vv[4] = {V[j].x, V[j].y, V[j].z, V[j].w};
        const unsigned char te[4] = {TE[j].x, TE[j].y, TE[j].z, TE[j].w}, tr[4] = {TR[j].x, TR[j].y, TR[j].z, TR[j].w};
        float out_a[4], out_t[4];
#pragma unroll
        for (int c = 0; c < 4; c++) {
          float boot = tr[c] ? (nv ? nv[i * 4 + c] : 0.0f) : vn[c];
          if (te[c]) boot = 0.0f;
          const float delta = rr[c] + gamma * boot - vv[c];
          a[c] = delta + ((te[c] || tr[c]) ? 0.0f : gl * a[c]);
          out_a[c] = a[c];
          out_t[c] = a[c] + vv[c];
          s1[c] += (double)a[c];
          s2[c] += (double)a[c] * (double)a[c];
          vn[c] = vv[c];
        }
        adv[i] = make_float4(out_a[0], out_a[1], out_a[2], out_a[3]);
        if (tgt) tgt[i] = make_float4(out_t[0], out_t[1], out_t[2], out_t[3]);
      }
    }
  }
  if (!stats) return;
  if (G == 1) {
    double t1 = wave_sum((s1[0] + s1[1]) + (s1[2] + s1[3])), t2 = wave_sum((s2[0] + s2[1]) + (s2[2] + s2[3]));
    const int wid = threadIdx.x >> 6, ln = threadIdx.x & 63;
    if (ln == 0) {
      red[0][wid] = t1;
      red[1][wid] = t2;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      double a1 = 0.0, a2 = 0.0;
      for (int k = 0; k < GAE_BS / 64; k++) {
        a1 += red[0][k];
        a2 += red[1][k];
      }
      const int64_t rem = N4 - (int64_t)blockIdx.x * GAE_BS;
      const int64_t cnt = 4 * (rem < GAE_BS ? rem : GAE_BS);
      atomicAdd(&stats[0], a1);
      atomicAdd(&stats[1], a2);
      atomicAdd(&stats[2], (double)cnt * (double)T);
    }
    return;
  }
  for (int g = threadIdx.x; g < G; g += GAE_BS) red[0][g] = red[1][g] = red[2][g] = 0.0;
  __syncthreads();
  if (q < N4) {
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const int g = (int)((4 * q + c) % G);
      atomicAdd(&red[0][g], s1[c]);
      atomicAdd(&red[1][g], s2[c]);
      atomicAdd(&red[2][g], (double)T);
    }
  }
  __syncthreads();
  for (int g = threadIdx.x; g < G; g += GAE_BS) {
    if (red[2][g] > 0.0) {
      atomicAdd(&stats[3 * g + 0], red[0][g]);
      atomicAdd(&stats[3 * g + 1], red[1][g]);
      atomicAdd(&stats[3 * g + 2], red[2][g]);
    }
  }
}

// (A - mean_g) / max(1e-4, std_g) over the [T][N] advantages; element i is sequence i % N, whose
// group is (i % N) % G = i % G because the caller's N is a multiple of G.
__global__ void adv_norm_kernel(float* __restrict__ adv, int64_t n, int32_t G, const double* __restrict__ st) {
  __shared__ float mg[GAE_MAX_GROUPS], ig[GAE_MAX_GROUPS];
  for (int g = threadIdx.x; g < G; g += blockDim.x) {
    const double cnt = st[3 * g + 2] > 0 ? st[3 * g + 2] : 1.0;
    const double mean = st[3 * g] / cnt;
    double var = st[3 * g + 1] / cnt - mean * mean;
    var = var > 0 ? var : 0.0;
    double sd = sqrt(var);
    sd = sd > 1e-4 ? sd : 1e-4;
    mg[g] = (float)mean;
    ig[g] = (float)(1.0 / sd);
  }
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int g = G == 1 ? 0 : (int)(i % G);
    adv[i] = (adv[i] - mg[g]) * ig[g];
  }
}

hipError_t launch_gae(const float* r, const float* v, const float* nv, const uint8_t* term, const uint8_t* trunc,
                      int64_t N, int32_t T, float gamma, float lam, float* adv, float* tgt, int32_t G, double* stats,
                      hipStream_t st) {
  if (N == 0) return hipSuccess;
  if (G < 1 || G > GAE_MAX_GROUPS || N % G != 0) return hipErrorInvalidValue;
  const bool vec = N % 4 == 0 && term && trunc && ((uintptr_t)r | (uintptr_t)v | (uintptr_t)adv | (uintptr_t)tgt |
                                                   (uintptr_t)term | (uintptr_t)trunc) % 16 == 0 &&
                   ((uintptr_t)term | (uintptr_t)trunc) % 4 == 0 && getenv("MSC_GAE_SCALAR") == nullptr;
  if (vec) {
    const int64_t N4 = N / 4, blocks = (N4 + GAE_BS - 1) / GAE_BS;
    hipLaunchKernelGGL(gae4_kernel, dim3((unsigned)blocks), dim3(GAE_BS), 0, st, (const float4*)r, (const float4*)v,
                       nv, (const uchar4*)term, (const uchar4*)trunc, N4, T, gamma, lam, (float4*)adv, (float4*)tgt,
                       G, stats);
    return hipGetLastError();
  }
  const int64_t blocks = (N + GAE_BS - 1) / GAE_BS;
  hipLaunchKernelGGL(gae_kernel, dim3((unsigned)blocks), dim3(GAE_BS), 0, st, r, v, nv, term, trunc, N, T, gamma,
                     lam, adv, tgt, G, stats);
  return hipGetLastError();
}

hipError_t launch_adv_normalize(float* adv, int64_t n, int32_t G, const double* stats, hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (G < 1 || G > GAE_MAX_GROUPS || n % G != 0) return hipErrorInvalidValue;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(adv_norm_kernel, dim3((unsigned)blocks), dim3(256), 0, st, adv, n, G, stats);
  return hipGetLastError();
}

// Diagonal-Gaussian action sampling of the rollout (RLlib's TorchDiagGaussian over
// ACTION_DIST_INPUTS = [mean, log_std], rlmodules/base.py:480-557): one lane per (env, agent) row,
// a = mean + exp(max(log_std, floor)) * eps, logp = sum_k -(a - mean)^2 / (2 std^2) - log_std
// - log(sqrt(2 pi)), and the env's [-1, 1] clip of the action. Replaces a dozen elementwise
// passes over [N, K] per rollout step. HBM-bound: 16 B per row element (mean, eps in; a, clip out).
__global__ __launch_bounds__(256) void gauss_sample_kernel(const float* __restrict__ mean,
                                                           const float* __restrict__ log_std, int32_t ls_rows,
                                                           float floor_, const float* __restrict__ eps, int64_t N,
                                                           int32_t K,
                                                           float* __restrict__ act, float* __restrict__ logp,
                                                           float* __restrict__ clipped) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const float half_log_2pi = 0.91893853320467274178f;  // 0.5 * log(2 pi)
  const float* lsr = log_std + (n % ls_rows) * K;  // per-agent rows (n = env * W + agent) or one shared row
  float lp = 0.0f;
  for (int k = 0; k < K; k++) {
    const int64_t i = n * K + k;
    const float ls = fmaxf(lsr[k], floor_);
    const float sd = expf(ls);
    const float m = mean[i];
    const float a = m + sd * eps[i];
    act[i] = a;
    const float d = a - m;
    lp += (-(d * d) / (2.0f * sd * sd) - ls) - half_log_2pi;
    clipped[i] = fminf(fmaxf(a, -1.0f), 1.0f);
  }
  logp[n] = lp;
}

hipError_t launch_gauss_sample(const float* mean, const float* log_std, int32_t ls_rows, float floor_, const float* eps,
                               int64_t N, int32_t K, float* act, float* logp, float* clipped, hipStream_t st) {
  if (N == 0) return hipSuccess;
  hipLaunchKernelGGL(gauss_sample_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, st, mean, log_std, ls_rows,
                     floor_, eps, N, K, act, logp, clipped);
  return hipGetLastError();
}

// Rollout noise keyed by global env id: out[s][row][j] = N(0, 1) from Philox4x32-10 with key =
// seed and counter = {j / 2, global row (= row0 + row, 64 bit), step0 + s}, Box-Muller on two 32-bit
// uniforms giving elements j (cos) and j + 1 (sin). Every value depends only on (seed, global env id,
// rollout step, element), so a rank's envs draw the same noise whatever the sharding (the multi-rank
// training path equals the single-rank one, tests/test_gpu_train.py).
__device__ __forceinline__ void philox_round(uint32_t (&c)[4], uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint32_t h0 = __umulhi(M0, c[0]), l0 = M0 * c[0];
  const uint32_t h1 = __umulhi(M1, c[2]), l1 = M1 * c[2];
  const uint32_t n0 = h1 ^ c[1] ^ k0, n2 = h0 ^ c[3] ^ k1;
  c[0] = n0;
  c[1] = l1;
  c[2] = n2;
  c[3] = l0;
}

__global__ __launch_bounds__(256) void normal_keyed_kernel(float* __restrict__ out, int32_t n_steps, int64_t n_rows,
                                                           int32_t row_len, int64_t row0, uint64_t seed,
                                                           uint64_t step0) {
  const int pairs = (row_len + 1) / 2;
  const int64_t total = (int64_t)n_steps * n_rows * pairs;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int jp = (int)(i % pairs);
    const int64_t sr = i / pairs;
    const int64_t row = sr % n_rows;
    const int64_t st = sr / n_rows;
    const uint64_t g = (uint64_t)(row0 + row);
    uint32_t c[4] = {(uint32_t)jp, (uint32_t)g, (uint32_t)(g >> 32), (uint32_t)(step0 + (uint64_t)st)};
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
    for (int r = 0; r < 10; r++) {
      philox_round(c, k0, k1);
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    const float u1 = ((float)c[0] + 0.5f) * 2.3283064365386963e-10f;  // (0, 1]
    const float u2 = (float)c[1] * 2.3283064365386963e-10f;
    const float rad = sqrtf(-2.0f * logf(u1));
    float sn, cs;
    sincosf(6.283185307179586f * u2, &sn, &cs);
    float* o = out + (st * n_rows + row) * row_len + 2 * jp;
    o[0] = rad * cs;
    if (2 * jp + 1 < row_len) o[1] = rad * sn;
  }
}

hipError_t launch_normal_keyed(float* out, int32_t n_steps, int64_t n_rows, int32_t row_len, int64_t row0,
                               uint64_t seed, uint64_t step0, hipStream_t st) {
  const int64_t total = (int64_t)n_steps * n_rows * ((row_len + 1) / 2);
  if (total == 0) return hipSuccess;
  const int64_t blocks = (total + 255) / 256 < 16384 ? (total + 255) / 256 : 16384;
  hipLaunchKernelGGL(normal_keyed_kernel, dim3((unsigned)blocks), dim3(256), 0, st, out, n_steps, n_rows, row_len, row0,
                     seed, step0);
  return hipGetLastError();
}

}  // namespace msc
