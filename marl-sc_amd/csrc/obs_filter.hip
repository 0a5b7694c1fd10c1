// obs_filter.hip -- RLlib's MeanStdFilter env-to-module connector (obs_normalization: "meanstd",
// reference src/algorithms/mappo.py:170-171, ippo.py:173-175, evaluation with update=False at
// base.py:131-140 / :176-177) on the device. RLlib (ray 2.52.1, requirements.txt:81) is not part of
// the reference or of this image: the algorithm is ray.rllib.utils.filter's RunningStat /
// MeanStdFilter as published, restated in oracle/meanstd_ref.py (parity unpinned).
//
// Per column (agent, feature) a RunningStat {n, M, S}:
//   push(x):  n += 1; n == 1: M = x; else delta = x - M, M += delta / n, S += delta * delta * (n - 1) / n
//   var = S / (n - 1) if n > 1 else M^2;  y = clip((x - M) / (sqrt(var) + eps), -clip, clip)
// and every observation is pushed, then normalised with the statistics that include it; rows
// (envs) are pushed in order. The filter also keeps a buffer RunningStat of the pushes since the
// last synchronisation (merged across env runners / ranks by RunningStat.update, Chan et al.).
//
// On the device the E rows of a call are cut into P <= 64 segments of G rows:
//   of_segment_kernel  thread (segment p, column c): RunningStat of its G rows from zero;
//   of_apply_kernel    thread (p, c): the running state merged with segments 0 .. p-1, then its own
//                      rows pushed and normalised one by one (the reference's sequential update
//                      inside a segment, Chan merges across segment boundaries);
//   of_commit_kernel   thread c: the state after the last segment becomes the running state; the
//                      buffer absorbs the segments.
// Lanes are columns (rows are contiguous [E][C] f32), so every row read is coalesced. HBM traffic
// per call: the obs read twice and written once (12 B per element); the rest is per column.
#include <hip/hip_runtime.h>
#include <math.h>

#include "env.hpp"

namespace msc {

constexpr int OF_MAX_SEG = 64;
constexpr int OF_BS = 256;

__device__ __forceinline__ void rs_push(double& n, double& m, double& s, double x) {
  n += 1.0;
  if (n == 1.0) {
    m = x;
  } else {
    const double delta = x - m;
    m += delta / n;
    s += delta * delta * (n - 1.0) / n;
  }
}
// RunningStat.update(other): a <- a (+) b
__device__ __forceinline__ void rs_merge(double& n1, double& m1, double& s1, double n2, double m2, double s2) {
  const double n = n1 + n2;
  if (n == 0.0) return;
  const double delta = m1 - m2;
  const double delta2 = delta * delta;
  const double m = (n1 * m1 + n2 * m2) / n;
  const double s = s1 + s2 + (delta2 / n) * n1 * n2;
  n1 = n;
  m1 = m;
  s1 = s;
}
__device__ __forceinline__ float rs_normalize(double x, double n, double m, double s, double clip, double eps) {
  const double var = n > 1.0 ? s / (n - 1.0) : m * m;
  double y = (x - m) / (sqrt(var) + eps);
  if (clip > 0.0) y = y < -clip ? -clip : (y > clip ? clip : y);
  return (float)y;
}

// state: {run_n, buf_n, 0, 0, run_M[C], run_S[C], buf_M[C], buf_S[C]}; seg: [P][C][3]
__global__ __launch_bounds__(OF_BS) void of_segment_kernel(const float* __restrict__ x, int64_t E, int32_t C,
                                                         const uint8_t* __restrict__ mask, int64_t G, int32_t P,
                                                         double* __restrict__ seg) {
  const int64_t i = (int64_t)blockIdx.x * OF_BS + threadIdx.x;
  if (i >= (int64_t)P * C) return;
  const int c = (int)(i % C), p = (int)(i / C);
  const int64_t e0 = (int64_t)p * G, e1 = e0 + G < E ? e0 + G : E;
  double n = 0.0, m = 0.0, s = 0.0;
  for (int64_t e = e0; e < e1; e++)
    if (!mask || mask[e]) rs_push(n, m, s, (double)x[e * C + c]);
  double* o = seg + i * 3;
  o[0] = n;
  o[1] = m;
  o[2] = s;
}

__global__ __launch_bounds__(OF_BS) void of_apply_kernel(const float* __restrict__ x, float* __restrict__ out, int64_t E,
                                                       int32_t C, const uint8_t* __restrict__ mask, int64_t G,
                                                       int32_t P, const double* __restrict__ seg,
                                                       const double* __restrict__ state, double* __restrict__ fin,
                                                       int32_t update, double clip, double eps) {
  const int64_t i = (int64_t)blockIdx.x * OF_BS + threadIdx.x;
  if (i >= (int64_t)P * C) return;
  const int c = (int)(i % C), p = (int)(i / C);
  const int64_t e0 = (int64_t)p * G, e1 = e0 + G < E ? e0 + G : E;
  double n = state[0], m = state[4 + c], s = state[4 + C + c];
  if (update) {
    for (int q = 0; q < p; q++) {
      const double* g = seg + ((int64_t)q * C + c) * 3;
      rs_merge(n, m, s, g[0], g[1], g[2]);
    }
  }
  for (int64_t e = e0; e < e1; e++) {
    const double v = (double)x[e * C + c];
    if (update && (!mask || mask[e])) rs_push(n, m, s, v);
    out[e * C + c] = rs_normalize(v, n, m, s, clip, eps);
  }
  if (update && p == P - 1) {  // the running state after every row of the call
    fin[(int64_t)c * 3 + 0] = n;
    fin[(int64_t)c * 3 + 1] = m;
    fin[(int64_t)c * 3 + 2] = s;
  }
}

__global__ __launch_bounds__(OF_BS) void of_commit_kernel(int32_t C, int32_t P, const double* __restrict__ seg,
                                                        const double* __restrict__ fin, double* __restrict__ state) {
  const int c = (int)(blockIdx.x * OF_BS + threadIdx.x);
  if (c >= C) return;
  double bn = state[1], bm = state[4 + 2 * C + c], bs = state[4 + 3 * C + c];
  for (int q = 0; q < P; q++) {
    const double* g = seg + ((int64_t)q * C + c) * 3;
    rs_merge(bn, bm, bs, g[0], g[1], g[2]);
  }
  state[4 + c] = fin[(int64_t)c * 3 + 1];
  state[4 + C + c] = fin[(int64_t)c * 3 + 2];
  state[4 + 2 * C + c] = bm;
  state[4 + 3 * C + c] = bs;
  if (c == 0) {
    state[0] = fin[0];
    state[1] = bn;
  }
}

void meanstd_plan(int64_t E, int64_t* G, int32_t* P) {
  const int64_t p = E < OF_MAX_SEG ? E : OF_MAX_SEG;
  *G = (E + p - 1) / p;
  *P = (int32_t)((E + *G - 1) / *G);
}
int64_t meanstd_scratch_doubles(int64_t E, int32_t C) {
  int64_t G;
  int32_t P;
  meanstd_plan(E, &G, &P);
  return (int64_t)P * C * 3 + (int64_t)C * 3;
}

hipError_t launch_meanstd_filter(const float* x, float* out, int64_t E, int32_t C, const uint8_t* mask, int32_t update,
                                 double* state, double* scratch, double clip, double eps, hipStream_t st) {
  int64_t G;
  int32_t P;
  meanstd_plan(E, &G, &P);
  double* seg = scratch;
  double* fin = scratch + (int64_t)P * C * 3;
  const unsigned nb = (unsigned)(((int64_t)P * C + OF_BS - 1) / OF_BS);
  if (update) hipLaunchKernelGGL(of_segment_kernel, dim3(nb), dim3(OF_BS), 0, st, x, E, C, mask, G, P, seg);
  hipLaunchKernelGGL(of_apply_kernel, dim3(nb), dim3(OF_BS), 0, st, x, out, E, C, mask, G, P, seg, state, fin, update,
                     clip, eps);
  if (update)
    hipLaunchKernelGGL(of_commit_kernel, dim3((unsigned)((C + OF_BS - 1) / OF_BS)), dim3(OF_BS), 0, st, C, P, seg, fin,
                       state);
  return hipGetLastError();
}

}  // namespace msc
