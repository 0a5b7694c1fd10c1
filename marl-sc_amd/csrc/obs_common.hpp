// obs_common.hpp -- reset and observation building shared by the phase-C kernels
// (env_kernels.hip: step_c_kernel, reset_kernel; alloc_scan.hip: the scan allocator's fused phase C).
// _build_local_obs / _feature_block / _compute_pipeline (multi_env.py:577-745, 941-968), reset
// (multi_env.py:192-251). Included once per translation unit.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

#include "env.hpp"
#include "rng.hpp"
#include "demand_common.hpp"

namespace msc {

// numpy add.reduce order for n <= 128 float32 (pairwise_sum: sequential below 8, else eight
// strided accumulators over the whole 8-blocks, their fixed tree, then the tail sequentially)
template <int K>
__device__ __forceinline__ float np_sum_f32(const float (&a)[K]) {
  if constexpr (K < 8) {
    float s = 0.0f;
#pragma unroll
    for (int i = 0; i < K; i++) s += a[i];
    return s;
  } else {
    float r[8];
#pragma unroll
    for (int j = 0; j < 8; j++) r[j] = a[j];
#pragma unroll
    for (int i = 8; i + 8 <= K; i += 8)
#pragma unroll
      for (int j = 0; j < 8; j++) r[j] += a[i + j];
    float s = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
#pragma unroll
    for (int i = K - K % 8; i < K; i++) s += a[i];
    return s;
  }
}

// _rescale_actions_to_quantities (multi_env.py:795-848) of SKU sk: the action in [-1, 1], the
// incoming home demand of the previous step and the SKU's pending total -> the order quantity
__device__ __forceinline__ int rescale_action(const EnvConst& c, int sk, float a, int inc_old, int pend) {
  const double prm = c.act_param[sk];
  double q;
  if (c.action_type == MSC_ACTION_DIRECT) {
    q = rint((double)((a + 1.0f) / 2.0f) * prm);
    q = q < 0.0 ? 0.0 : (q > prm ? prm : q);
  } else if (c.action_type == MSC_ACTION_DEMAND_CENTERED) {
    q = rint(prm * (double)a) + (double)inc_old;
    q = q < 0.0 ? 0.0 : q;
  } else {
    const double target = (double)((a + 1.0f) / 2.0f) * prm;
    q = rint((target - (double)(float)inc_old) - (double)(float)pend);
    q = q < 0.0 ? 0.0 : q;
  }
  return (int)q;
}

// ------------------------------------------------------------------------------------------
// reset (multi_env.py:192-251, SeedManager.advance_episode / update_root_seed)
// ------------------------------------------------------------------------------------------
template <int K>
__device__ __noinline__ void reset_env(const EnvConst& c, const EnvState& s, int64_t e, int32_t flags,
                                       const uint32_t* new_root) {
  const int64_t E = c.E;
  const int WK = c.W * K;
  uint32_t root;
  if (new_root) {
    root = *new_root;
    s.orig_root[e] = root;
    s.counter[e] = 0;
  } else {
    int cnt = s.counter[e];
    if (c.num_eval > 0 && ((flags & MSC_RESET_EVAL_RESTART) || cnt >= c.num_eval)) cnt = 0;
    uint32_t w2[2] = {s.orig_root[e], (uint32_t)cnt};
    root = ss_u32(w2, 2);
    s.counter[e] = cnt + 1;
  }
  s.root[e] = root;
  Pcg64 r;
  pcg_seed_child(r, root, 2);  // 'demand_sampler'
  store_rng(s, 0, e, E, r);
  pcg_seed_child(r, root, 3);  // 'lead_time_sampler'
  store_rng(s, 1, e, E, r);
  if (c.init_type == MSC_INIT_UNIFORM) {
    pcg_seed_child(r, root, 1);  // 'inventory'
    for (int i = 0; i < WK; i++)
      s.inv[i * E + e] = (int32_t)bounded_int(r, c.init_min, (int64_t)c.init_max + 1);
  } else if (c.init_type == MSC_INIT_CUSTOM) {
    for (int i = 0; i < WK; i++) s.inv[i * E + e] = c.init_vals[i];
  } else {
    for (int i = 0; i < WK; i++) s.inv[i * E + e] = 0;
  }
  for (int i = 0; i < WK * c.RING; i++) s.ring_q[i * E + e] = 0;
  for (int i = 0; i < WK; i++) {
    s.inc[i * E + e] = 0;
    s.fc[i * E + e] = 0.0f;
  }
  s.t[e] = 0;
  s.emp_start[e] = -1;
}

// The feature vector of one agent from its gathered inputs (the second half of _build_local_obs):
// per-SKU inventory, incoming home demand dh, shipped home sh / away sa, forecast fc, rolling mean
// rm, pipeline total per SKU and expected lead times; pipe_at(l, sk) = pipeline bucket l of SKU sk,
// hist_at(a, sk) = the demand of age a (0 = this step's) for a < n_hist. Shared by step_c_kernel
// (inputs from HBM) and the fused phase C of the scan allocator (inputs from registers / LDS).
template <int K, typename PipeAt, typename HistAt>
__device__ __forceinline__ void obs_emit(const EnvConst& c, int w, int n_hist, const int (&inv)[K], const int (&dh)[K],
                                         const int (&sh)[K], const int (&sa)[K], const int (&pend_sum)[K],
                                         const int (&eltv)[K], const float (&rm)[K], const float (&fc)[K],
                                         PipeAt&& pipe_at, HistAt&& hist_at, float* out) {
  const int W = c.W, Lmax = c.Lmax;
  const uint32_t f = c.flags;
  const bool ratio = c.norm == MSC_OBS_RATIO, meanstd = c.norm == MSC_OBS_MEANSTD;
  const double eps = 1e-8;
  const float epsf = 1e-8f;
  float* o = out + (int64_t)w * c.L;
  int j = 0;  // feature index (excludes the one-hot)
  auto put = [&](double v) {
    float x = (float)v;
    if (meanstd) x = (x - c.obs_mean[j]) / c.obs_std[j];
    o[(c.wid ? W : 0) + j] = x;
    j++;
  };
  int pend_total = 0;
#pragma unroll
  for (int sk = 0; sk < K; sk++) pend_total += pend_sum[sk];
  if (c.wid)
    for (int k = 0; k < W; k++) o[k] = (k == w) ? 1.0f : 0.0f;
  double inv_total = 0.0, shipped_total = 0.0, sa_total = 0.0;
  float dh_total = 0.0f;
#pragma unroll
  for (int sk = 0; sk < K; sk++) {
    inv_total += (double)inv[sk];
    dh_total += (float)dh[sk];
    shipped_total += (double)(sh[sk] + sa[sk]);
    sa_total += (double)sa[sk];
  }
  const float rm_total = np_sum_f32<K>(rm);
  const float fc_total = np_sum_f32<K>(fc);

  if (f & MSC_F_INVENTORY) {
#pragma unroll
    for (int sk = 0; sk < K; sk++) put(ratio ? (double)inv[sk] / (inv_total + eps) : (double)inv[sk]);
    if (f & MSC_F_INVENTORY_AGG) put((double)(float)inv_total);
  }
  if (f & MSC_F_PIPELINE) {
    const float den = (float)((double)pend_total + eps);
    for (int l = 0; l < Lmax; l++)
#pragma unroll
      for (int sk = 0; sk < K; sk++) {
        float v = (float)pipe_at(l, sk);
        put(ratio ? (double)(v / den) : (double)v);
      }
    if (f & MSC_F_PIPELINE_AGG) put((double)pend_total);
  }
  if (f & MSC_F_INCOMING_HOME) {
    const float den = dh_total + epsf;
#pragma unroll
    for (int sk = 0; sk < K; sk++) put(ratio ? (double)((float)dh[sk] / den) : (double)dh[sk]);
    if (f & MSC_F_INCOMING_HOME_AGG) put((double)dh_total);
  }
  if (f & MSC_F_SHIPPED_HOME) {
    const double den = (double)(dh_total + epsf);
#pragma unroll
    for (int sk = 0; sk < K; sk++) put(ratio ? (double)sh[sk] / den : (double)sh[sk]);
  }
  if (f & MSC_F_SHIPPED_AWAY) {
#pragma unroll
    for (int sk = 0; sk < K; sk++) put(ratio ? (double)sa[sk] / (shipped_total + eps) : (double)sa[sk]);
    if (f & MSC_F_SHIPPED_AWAY_AGG) put((double)(float)(sa_total / (shipped_total + eps)));
  }
  if (f & MSC_F_STOCKOUT) {
    const float den = dh_total + epsf;
#pragma unroll
    for (int sk = 0; sk < K; sk++) {
      float so = (float)(dh[sk] - sh[sk] > 0 ? dh[sk] - sh[sk] : 0);
      put(ratio ? (double)(so / den) : (double)so);
    }
  }
  if (f & MSC_F_ROLLING_MEAN) {
    const float den = rm_total + epsf;
#pragma unroll
    for (int sk = 0; sk < K; sk++) put(ratio ? (double)(rm[sk] / den) : (double)rm[sk]);
    if (f & MSC_F_ROLLING_MEAN_AGG) put((double)rm_total);
  }
  if (f & MSC_F_FORECAST) {
    const float den = fc_total + epsf;
#pragma unroll
    for (int sk = 0; sk < K; sk++) put(ratio ? (double)(fc[sk] / den) : (double)fc[sk]);
    if (f & MSC_F_FORECAST_AGG) put((double)fc_total);
  }
  if (f & MSC_F_DAYS_OF_SUPPLY) {
#pragma unroll
    for (int sk = 0; sk < K; sk++) put((double)(float)((double)inv[sk] / (double)(rm[sk] > 1.0f ? rm[sk] : 1.0f)));
  }
  if (f & MSC_F_NET_POSITION) {
#pragma unroll
    for (int sk = 0; sk < K; sk++) {
      double v = ((double)inv[sk] + (double)pend_sum[sk]) - (double)fc[sk] * (double)eltv[sk];
      put((double)(float)v);
    }
  }
  if (f & MSC_F_DEMAND_VARIABILITY) {
#pragma unroll
    for (int sk = 0; sk < K; sk++) {
      float sd = 0.0f;
      if (n_hist > 1) {  // oldest first, as the deque (multi_env.py:776-789)
        float sum = 0.0f;
        for (int h = 0; h < n_hist; h++) sum += (float)hist_at(n_hist - 1 - h, sk);
        float mean = sum / (float)n_hist, ss = 0.0f;
        for (int h = 0; h < n_hist; h++) {
          float d = (float)hist_at(n_hist - 1 - h, sk) - mean;
          ss += d * d;
        }
        sd = sqrtf(ss / (float)n_hist);
      }
      put((double)sd);
    }
  }
  if (f & MSC_F_DEMAND_HISTORY) {
    for (int h = 0; h < MSC_HISTORY; h++)
#pragma unroll
      for (int sk = 0; sk < K; sk++) put((double)(h < n_hist ? hist_at(h, sk) : 0));
  }
}

// ------------------------------------------------------------------------------------------
// observations (_get_observations / _build_local_obs / _compute_pipeline, multi_env.py:548-745, 941-968)
//   t_now : timestep the observation is taken at (before the increment of step())
//   n_hist: entries in the demand-history deque (0 at reset)
//   shh/sht: per-lane LDS shipped-home / shipped-total of this step (null at reset)
// ------------------------------------------------------------------------------------------
//   shh/sht are indexed [(w * K + sku) * BS] from a pointer already offset to the env's column.
// One agent (warehouse w) per call: the step kernel builds the W agents of an env in parallel.
#ifndef MSC_OBS_RING_REG
#define MSC_OBS_RING_REG 4  // pending rings of up to this many slots (lead times <= 3) are read into registers
#endif
constexpr int OBS_RING_REG = MSC_OBS_RING_REG;
// RREG > 0: rings of up to RREG slots are read into registers (step_c with <= 8 waves per block;
// elsewhere the register budget is 128 and the ring is read where it is used)
template <int K, int RREG = 0, bool HIST_STATIC = false>
__device__ __forceinline__ void build_obs_agent(const EnvConst& c, const EnvState& s, int64_t e, int w, int t_now,
                                             int n_hist, const int32_t* shh, const int32_t* sht, int64_t sstride,
                                             float* out) {
  const int64_t E = c.E;
  const int W = c.W, RING = c.RING;
  {
    // Every state load is issued before the first observation store: vector-memory stores and loads
    // share one completion counter (vmcnt), so a load issued after stores waits for them all; the
    // pipeline buckets come from the pending ring held in registers (RING <= OBS_RING_REG) instead
    // of ring reads between the feature stores.
    int inv[K], dh[K], sh[K], sa[K], pend_sum[K], eltv[K];
    float rm[K], fc[K];
#pragma unroll
    for (int sk = 0; sk < K; sk++) {
      const int i = w * K + sk;
      eltv[sk] = c.elt[i];
      inv[sk] = s.inv[i * E + e];
      dh[sk] = s.inc[i * E + e];
      sh[sk] = shh ? shh[i * sstride] : 0;
      sa[sk] = sht ? sht[i * sstride] - sh[sk] : 0;
      fc[sk] = s.fc[i * E + e];
      int hs = 0;
      if constexpr (HIST_STATIC) {
        // the MSC_HISTORY slot loads issued together (a counted loop waits on each): slot q holds the
        // demand of age (t_now - q) mod MSC_HISTORY, in the window iff that age < n_hist (an integer
        // sum: the order of the terms does not matter)
        const int tm5 = t_now % MSC_HISTORY;
#pragma unroll
        for (int q = 0; q < MSC_HISTORY; q++) {
          const int age = tm5 - q >= 0 ? tm5 - q : tm5 - q + MSC_HISTORY;
          const int v = s.hist[((int64_t)q * W * K + i) * E + e];
          hs += age < n_hist ? v : 0;
        }
      } else {
        for (int h = 0; h < n_hist; h++) hs += s.hist[(((t_now - n_hist + 1 + h) % MSC_HISTORY) * W * K + i) * E + e];
      }
      rm[sk] = n_hist > 0 ? (float)hs / (float)n_hist : 0.0f;
      pend_sum[sk] = 0;
    }
    // pipeline buckets (_compute_pipeline, multi_env.py:956-966): an order of age a (ring slot
    // (t_now - a) mod RING) expects to arrive in elt - a steps and lands in bucket
    // max(1, elt - a) - 1, so bucket l >= 1 holds exactly the order of age elt - 1 - l and bucket 0
    // every order of age >= elt - 1 (due next step or overdue).
    constexpr int RR = RREG > 0 ? RREG : 1;
    const bool ring_reg = RREG > 0 && RING <= RREG;
    int rv[K][RR];  // ring slot q of SKU sk (ring_reg)
    int tm = t_now % RING;
    if (tm < 0) tm += RING;
    int pend_total = 0;
#pragma unroll
    for (int sk = 0; sk < K; sk++) {
      const int32_t* rq = s.ring_q + (int64_t)(w * K + sk) * RING * E + e;
      if (ring_reg) {
#pragma unroll
        for (int q = 0; q < RR; q++) rv[sk][q] = q < RING ? rq[q * E] : 0;
#pragma unroll
        for (int q = 0; q < RR; q++) pend_sum[sk] += rv[sk][q];
      } else {
        for (int jr = 0; jr < RING; jr++) pend_sum[sk] += rq[jr * E];
      }
      pend_total += pend_sum[sk];
    }
    auto pipe_at = [&](int l, int sk) -> int {
      const int elt = eltv[sk];
      if (ring_reg) {  // slot q (age (tm - q) mod RING) lands in bucket max(1, elt - age) - 1
        int v = 0;
#pragma unroll
        for (int q = 0; q < RR; q++) {
          const int age = tm - q >= 0 ? tm - q : tm - q + RING;
          const int b = elt - age > 1 ? elt - age - 1 : 0;
          v += (q < RING && b == l) ? rv[sk][q] : 0;
        }
        return v;
      }
      const int32_t* rq = s.ring_q + (int64_t)(w * K + sk) * RING * E + e;
      auto at_age = [&](int a) -> int {
        int jr = (t_now - a) % RING;
        if (jr < 0) jr += RING;
        return rq[jr * E];
      };
      if (l > 0) return l + 1 <= elt ? at_age(elt - 1 - l) : 0;
      int v = 0;
      for (int a = elt - 1 > 0 ? elt - 1 : 0; a < RING; a++) v += at_age(a);
      return v;
    };
    (void)pend_total;
    auto hist_at = [&](int a, int sk) -> int {  // the demand of age a (slot (t_now - a) mod 5)
      return s.hist[((((t_now - a) % MSC_HISTORY) * W * K) + w * K + sk) * E + e];
    };
    obs_emit<K>(c, w, n_hist, inv, dh, sh, sa, pend_sum, eltv, rm, fc, pipe_at, hist_at, out);
  }
}


}  // namespace msc
