// env_kernels.hip -- HIP kernels of the vectorised InventoryEnvironment (gfx950 / CDNA4).
//
// One lane = one environment. A step is two launches on the caller's stream:
//   1. demand_poisson_kernel  PoissonDemandSampler.sample   (demand_sampler.py:105-163)
//      draws every order of the step from the env's own PCG64 stream into a per-step order
//      buffer (records [slot][E], 16 B each), region-major exactly like the reference's list.
//   2. step_kernel            InventoryEnvironment.step     (multi_env.py:253-366)
//      rescale actions, lead times, orders/arrivals (phase A, coalesced over (w,s)),
//      greedy allocation streamed region by region with the lost-sales epilogue folded into
//      each region change (phase B, per-lane LDS for the (warehouse, SKU) arrays that the
//      cost ranking indexes dynamically), then inventory/history/forecast, rewards and the
//      per-agent observations (phase C), and an in-kernel reset when the episode truncates.
// Integer state is exact; f32 observation arithmetic follows numpy's dtype flow operation by
// operation (the library is built with -ffp-contract=off so no FMA contraction changes a
// rounding); rewards are f64.
#include <hip/hip_runtime.h>
#include <math.h>

#include "env.hpp"
#include "rng.hpp"

namespace msc {

// ------------------------------------------------------------------------------------------
// small helpers
// ------------------------------------------------------------------------------------------
template <int K>
struct Rec {
  static constexpr int NV = (1 + K + 7) / 8;  // uint4 words per order record
  uint16_t h[8 * NV];
};

template <int K>
__device__ __forceinline__ void load_rec(const uint4* p, int64_t stride, int& region, int (&q)[K]) {
  constexpr int NV = Rec<K>::NV;
  union {
    uint4 v[NV];
    uint16_t h[8 * NV];
  } u;
#pragma unroll
  for (int j = 0; j < NV; j++) u.v[j] = p[j * stride];
  region = u.h[0];
#pragma unroll
  for (int s = 0; s < K; s++) q[s] = u.h[1 + s];
}

template <int K>
__device__ __forceinline__ void store_rec(uint4* p, int64_t stride, int region, const int (&q)[K]) {
  constexpr int NV = Rec<K>::NV;
  union {
    uint4 v[NV];
    uint16_t h[8 * NV];
  } u;
#pragma unroll
  for (int j = 0; j < 8 * NV; j++) u.h[j] = 0;
  u.h[0] = (uint16_t)region;
#pragma unroll
  for (int s = 0; s < K; s++) u.h[1 + s] = (uint16_t)q[s];
#pragma unroll
  for (int j = 0; j < NV; j++) p[j * stride] = u.v[j];
}

__device__ __forceinline__ Pcg64 load_rng(const EnvState& s, int which, int64_t e, int64_t E) {
  Pcg64 r;
  const uint64_t* b = s.rng + (int64_t)which * 4 * E + e;
  r.s_hi = b[0];
  r.s_lo = b[E];
  r.i_hi = b[2 * E];
  r.i_lo = b[3 * E];
  r.has32 = s.rbuf[(int64_t)which * 2 * E + e];
  r.u32 = s.rbuf[(int64_t)which * 2 * E + E + e];
  return r;
}
__device__ __forceinline__ void store_rng(const EnvState& s, int which, int64_t e, int64_t E, const Pcg64& r) {
  uint64_t* b = s.rng + (int64_t)which * 4 * E + e;
  b[0] = r.s_hi;
  b[E] = r.s_lo;
  b[2 * E] = r.i_hi;
  b[3 * E] = r.i_lo;
  s.rbuf[(int64_t)which * 2 * E + e] = r.has32;
  s.rbuf[(int64_t)which * 2 * E + E + e] = r.u32;
}

// numpy add.reduce order for n <= 8 float32 (sequential below 8, 8-way pairwise at 8)
template <int K>
__device__ __forceinline__ float np_sum_f32(const float (&a)[K]) {
  if constexpr (K < 8) {
    float s = 0.0f;
#pragma unroll
    for (int i = 0; i < K; i++) s += a[i];
    return s;
  } else {
    return ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  }
}

// ------------------------------------------------------------------------------------------
// reset (multi_env.py:192-251, SeedManager.advance_episode / update_root_seed)
// ------------------------------------------------------------------------------------------
template <int K>
__device__ void reset_env(const EnvConst& c, const EnvState& s, int64_t e, int32_t flags, const uint32_t* new_root) {
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

// ------------------------------------------------------------------------------------------
// observations (_get_observations / _build_local_obs / _compute_pipeline, multi_env.py:548-745, 941-968)
//   t_now : timestep the observation is taken at (before the increment of step())
//   n_hist: entries in the demand-history deque (0 at reset)
//   shh/sht: per-lane LDS shipped-home / shipped-total of this step (null at reset)
// ------------------------------------------------------------------------------------------
template <int K>
__device__ void build_obs(const EnvConst& c, const EnvState& s, int64_t e, int t_now, int n_hist,
                          const int32_t* shh, const int32_t* sht, float* out) {
  const int64_t E = c.E;
  const int W = c.W, RING = c.RING, Lmax = c.Lmax;
  const uint32_t f = c.flags;
  const bool ratio = c.norm == MSC_OBS_RATIO, meanstd = c.norm == MSC_OBS_MEANSTD;
  const double eps = 1e-8;
  const float epsf = 1e-8f;
  for (int w = 0; w < W; w++) {
    float* o = out + (int64_t)w * c.L;
    int j = 0;  // feature index (excludes the one-hot)
    auto put = [&](double v) {
      float x = (float)v;
      if (meanstd) x = (x - c.obs_mean[j]) / c.obs_std[j];
      o[(c.wid ? W : 0) + j] = x;
      j++;
    };
    if (c.wid)
      for (int k = 0; k < W; k++) o[k] = (k == w) ? 1.0f : 0.0f;
    int inv[K], dh[K], sh[K], sa[K], pend_sum[K];
    float rm[K], fc[K];
#pragma unroll
    for (int sk = 0; sk < K; sk++) {
      const int i = w * K + sk;
      inv[sk] = s.inv[i * E + e];
      dh[sk] = s.inc[i * E + e];
      sh[sk] = shh ? shh[i * BS] : 0;
      sa[sk] = sht ? sht[i * BS] - sh[sk] : 0;
      fc[sk] = s.fc[i * E + e];
      int hs = 0;
      for (int h = 0; h < n_hist; h++) hs += s.hist[(((t_now - n_hist + 1 + h) % MSC_HISTORY) * W * K + i) * E + e];
      rm[sk] = n_hist > 0 ? (float)hs / (float)n_hist : 0.0f;
      pend_sum[sk] = 0;
    }
    // pipeline bucket of each pending order: expected arrival - t_now, overdue -> slot 0
    auto pipe_at = [&](int l, int sk) -> int {
      const int i = w * K + sk;
      const int elt = c.elt[i];
      int acc = 0;
      for (int jr = 0; jr < RING; jr++) {
        int q = s.ring_q[(i * RING + jr) * E + e];
        if (q == 0) continue;
        int age = (t_now - jr) % RING;
        if (age < 0) age += RING;
        int slot = elt - age;
        if (slot < 1) slot = 1;
        if (slot - 1 == l) acc += q;
      }
      return acc;
    };
    int pend_total = 0;
    for (int l = 0; l < Lmax; l++)
#pragma unroll
      for (int sk = 0; sk < K; sk++) {
        int v = pipe_at(l, sk);
        pend_total += v;
        pend_sum[sk] += v;
      }
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
        double v = ((double)inv[sk] + (double)pend_sum[sk]) - (double)fc[sk] * (double)c.elt[w * K + sk];
        put((double)(float)v);
      }
    }
    if (f & MSC_F_DEMAND_VARIABILITY) {
#pragma unroll
      for (int sk = 0; sk < K; sk++) {
        float sd = 0.0f;
        if (n_hist > 1) {
          const int i = w * K + sk;
          float sum = 0.0f;
          for (int h = 0; h < n_hist; h++)
            sum += (float)s.hist[(((t_now - n_hist + 1 + h) % MSC_HISTORY) * W * K + i) * E + e];
          float mean = sum / (float)n_hist, ss = 0.0f;
          for (int h = 0; h < n_hist; h++) {
            float d = (float)s.hist[(((t_now - n_hist + 1 + h) % MSC_HISTORY) * W * K + i) * E + e] - mean;
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
        for (int sk = 0; sk < K; sk++) {
          int v = 0;
          if (h < n_hist) v = s.hist[((((t_now - h) % MSC_HISTORY) * W * K) + w * K + sk) * E + e];
          put((double)v);
        }
    }
  }
}

// ------------------------------------------------------------------------------------------
// kernels
// ------------------------------------------------------------------------------------------
template <int K>
__global__ __launch_bounds__(BS) void reset_kernel(EnvConst c, EnvState s, const uint8_t* mask,
                                                   const uint32_t* new_roots, int32_t flags, float* obs) {
  const int64_t e = (int64_t)blockIdx.x * BS + threadIdx.x;
  if (e >= c.E) return;
  if (mask && !mask[e]) return;
  reset_env<K>(c, s, e, flags, new_roots ? new_roots + e : nullptr);
  if (obs) build_obs<K>(c, s, e, 0, 0, nullptr, nullptr, obs + e * c.W * c.L);
}

// PoissonDemandSampler.sample (demand_sampler.py:105-163): per region n ~ Poisson(lambda_o);
// per order K Bernoulli(p) SKU draws then max(1, Poisson(lambda_q)) for the selected SKUs.
template <int K>
__global__ __launch_bounds__(BS) void demand_poisson_kernel(EnvConst c, EnvState s) {
  const int64_t e = (int64_t)blockIdx.x * BS + threadIdx.x;
  if (e >= c.E) return;
  const int64_t E = c.E;
  constexpr int NV = Rec<K>::NV;
  Pcg64 rg = load_rng(s, 0, e, E);
  int n = 0;
  for (int r = 0; r < c.R; r++) {
    const double elo = c.enlam_o[r], p = c.p_sku[r];
    const int no = elo >= 1.0 ? 0 : poisson_mult(rg, elo);
    for (int k = 0; k < no; k++) {
      unsigned mask = 0;
#pragma unroll
      for (int sk = 0; sk < K; sk++) mask |= (pcg_double(rg) < p) ? (1u << sk) : 0u;
      int q[K];
#pragma unroll
      for (int sk = 0; sk < K; sk++) {
        q[sk] = 0;
        if (mask & (1u << sk)) {
          const double el = c.enlam_q[r * K + sk];
          int v = el >= 1.0 ? 0 : poisson_mult(rg, el);
          q[sk] = v > 1 ? v : 1;
        }
      }
      if (n < c.order_cap) store_rec<K>(s.orders + ((int64_t)n * E * NV) + e, E, r, q);
      n++;
    }
  }
  store_rng(s, 0, e, E, rg);
  if (n > c.order_cap) {
    atomicOr(s.err, ERR_ORDER_OVERFLOW);
    n = c.order_cap;
  }
  s.n_orders[e] = n;
}

// compare-and-swap of (cost, warehouse) pairs: ascending cost, lowest index first on ties
__device__ __forceinline__ void cas(double& ca, int& ia, double& cb, int& ib) {
  const bool sw = (cb < ca) || (cb == ca && ib < ia);
  const double tc = sw ? cb : ca;
  const int ti = sw ? ib : ia;
  cb = sw ? ca : cb;
  ib = sw ? ia : ib;
  ca = tc;
  ia = ti;
}
template <int WM>
__device__ __forceinline__ void sort_costs(double (&c)[WM], int (&ix)[WM]) {
  // odd-even transposition network: WM rounds, fully unrolled (all indices static)
#pragma unroll
  for (int round = 0; round < WM; round++)
#pragma unroll
    for (int a = round & 1; a + 1 < WM; a += 2) cas(c[a], ix[a], c[a + 1], ix[a + 1]);
}

template <int K, int WM>
__global__ __launch_bounds__(BS) void step_kernel(EnvConst c, EnvState s, StepIO io) {
  extern __shared__ __attribute__((aligned(16))) int32_t lds[];
  const int lane = threadIdx.x;
  const int64_t e = (int64_t)blockIdx.x * BS + lane;
  if (e >= c.E) return;
  const int64_t E = c.E;
  const int W = c.W, WK = W * K, R = c.R, RING = c.RING;
  int32_t* Linv = lds + lane;                 // [WK]  inventory
  int32_t* Lqsr = lds + 1 * WK * BS + lane;   // [WK]  shipped to the current region
  int32_t* Lsht = lds + 2 * WK * BS + lane;   // [WK]  shipped in total this step
  int32_t* Lshh = lds + 3 * WK * BS + lane;   // [WK]  shipped to the home region
  double* Lpen = reinterpret_cast<double*>(lds + 4 * WK * BS) + lane;  // [W] penalty cost
  double* Lout = Lpen + W * BS;                                        // [W] outbound cost
  double* Linb = Lout + W * BS;                                        // [W] inbound cost
  const msc_step_info& info = io.info;
  const bool dbg = io.has_info != 0;

  const int t = s.t[e];
  // ---- phase 0: state -> LDS --------------------------------------------------------------
  for (int i = 0; i < WK; i++) {
    const int v = s.inv[i * E + e];
    Linv[i * BS] = v;
    Lqsr[i * BS] = 0;
    Lsht[i * BS] = 0;
    Lshh[i * BS] = 0;
    if (dbg && info.inventory_before) info.inventory_before[e * WK + i] = v;
  }
  for (int w = 0; w < W; w++) {
    Lpen[w * BS] = 0.0;
    Lout[w * BS] = 0.0;
  }
  const bool stoch = c.lead_type == MSC_LEAD_STOCHASTIC;
  if (stoch) {  // lead_time_sampler.sample(): all W*K deviations drawn every step (multi_env.py:866)
    Pcg64 rl = load_rng(s, 1, e, E);
    if (c.dev_per_sku) {  // np.column_stack of per-SKU draws: SKU-major order (lead_time_sampler.py:181-185)
#pragma unroll
      for (int sk = 0; sk < K; sk++)
        for (int w = 0; w < W; w++)
          Lqsr[(w * K + sk) * BS] = (int32_t)bounded_int(rl, -c.maxdev[sk], (int64_t)c.maxdev[sk] + 1);
    } else {
      for (int i = 0; i < WK; i++) Lqsr[i * BS] = (int32_t)bounded_int(rl, -c.maxdev[0], (int64_t)c.maxdev[0] + 1);
    }
    store_rng(s, 1, e, E, rl);
  }

  // ---- phase A: actions -> orders, lead times, pending ring, arrivals -----------------------
  const int slot = t % RING;
  for (int w = 0; w < W; w++) {
    double inbF = 0.0, inbV = 0.0;
#pragma unroll
    for (int sk = 0; sk < K; sk++) {
      const int i = w * K + sk;
      const float a = io.actions[(e * W + w) * K + sk];
      const int inc_old = s.inc[i * E + e];
      int32_t* rq = s.ring_q + (int64_t)i * RING * E + e;
      int pend = 0;
      for (int jr = 0; jr < RING; jr++) pend += rq[jr * E];
      // _rescale_actions_to_quantities (multi_env.py:795-848)
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
      const int qi = (int)q;
      const int elt = c.elt[i];
      int lact = elt;
      if (stoch) {
        lact = elt + Lqsr[i * BS];
        lact = lact > 1 ? lact : 1;
      }
      // _apply_orders: the slot of order time t (its previous occupant arrived already)
      rq[slot * E] = qi;
      if (stoch) s.ring_l[((int64_t)i * RING + slot) * E + e] = (uint8_t)lact;
      // _apply_arrivals: orders whose actual arrival == t
      int inv = Linv[i * BS];
      for (int jr = 0; jr < RING; jr++) {
        if (jr == slot) continue;
        const int qq = rq[jr * E];
        if (qq == 0) continue;
        int age = (t - jr) % RING;
        if (age < 0) age += RING;
        const int l = stoch ? (int)s.ring_l[((int64_t)i * RING + jr) * E + e] : elt;
        if (l == age) {
          inv += qq;
          rq[jr * E] = 0;
        }
      }
      Linv[i * BS] = inv;
      s.inc[i * E + e] = 0;
      if (qi > 0) inbF += c.inF[i];
      inbV += ((double)qi * c.skw[sk]) * c.inV[i];
      if (dbg) {
        if (info.pending_total) info.pending_total[e * WK + i] = pend;
        if (info.order_quantities) info.order_quantities[e * WK + i] = qi;
      }
    }
    Linb[w * BS] = inbF + inbV;
  }
  if (stoch)
    for (int i = 0; i < WK; i++) Lqsr[i * BS] = 0;

  // ---- phase B: greedy allocation (demand_allocator.py:118-217) + per-region epilogue ------
  const uint4* src;
  int64_t stride;
  int n_orders;
  if (c.demand_type == MSC_DEMAND_EMPIRICAL) {  // demand_sampler.py:227-241
    int st0 = s.emp_start[e];
    if (st0 < 0) {
      Pcg64 rg = load_rng(s, 0, e, E);
      st0 = (int)bounded_int(rg, 0, (int64_t)(c.tr_rows - c.T) + 1);
      store_rng(s, 0, e, E, rg);
      s.emp_start[e] = st0;
    }
    const int64_t row = st0 + (t % c.T);
    const int64_t off = c.tr_off[row];
    n_orders = (int)(c.tr_off[row + 1] - off);
    src = c.tr_rec + off * Rec<K>::NV;
    stride = 1;
  } else {
    n_orders = s.n_orders[e];
    src = s.orders + e;
    stride = E;
  }
  if (dbg && info.n_orders) info.n_orders[e] = n_orders;
  const int64_t rec_step = stride * Rec<K>::NV;

  int cur = -1, lost_cnt = 0;
  unsigned touched = 0;
  int u[K], dsum[K];
#pragma unroll
  for (int sk = 0; sk < K; sk++) u[sk] = dsum[sk] = 0;

  // region epilogue: lost sales (lost_sales_handler.py) folded into the penalty cost, the
  // home-region features and, in diagnostic mode, the per-region infos.
  auto finalize = [&](int r) {
    if (lost_cnt > 0) {
      double upen = 0.0;
#pragma unroll
      for (int sk = 0; sk < K; sk++)
        upen += c.pen_per_sku ? (double)u[sk] * c.pen[sk] : ((double)u[sk] * c.skw[sk]) * c.pen_scalar;
      if (c.lost_type == MSC_LOST_CLOSEST) {
        const int w0 = c.closest[r];
        Lpen[w0 * BS] += upen;
        if (dbg && info.lost_sales)
#pragma unroll
          for (int sk = 0; sk < K; sk++) info.lost_sales[e * WK + w0 * K + sk] += (double)u[sk];
      } else if (c.lost_type == MSC_LOST_SHIPMENT) {
        double tot = 0.0;
        double qr[WM];
#pragma unroll
        for (int w = 0; w < WM; w++) {
          qr[w] = 0.0;
          if (w < W && (touched >> w & 1u)) {
            int acc = 0;
#pragma unroll
            for (int sk = 0; sk < K; sk++) acc += Lqsr[(w * K + sk) * BS];
            qr[w] = (double)acc;
          }
          tot += qr[w];
        }
        if (tot > 0.0) {
#pragma unroll
          for (int w = 0; w < WM; w++) {
            if (qr[w] > 0.0) {
              const double wt = qr[w] / tot;
              Lpen[w * BS] += wt * upen;
              if (dbg && info.lost_sales)
#pragma unroll
                for (int sk = 0; sk < K; sk++) info.lost_sales[e * WK + w * K + sk] += wt * (double)u[sk];
            }
          }
        } else {
          const int w0 = c.closest[r];
          Lpen[w0 * BS] += upen;
          if (dbg && info.lost_sales)
#pragma unroll
            for (int sk = 0; sk < K; sk++) info.lost_sales[e * WK + w0 * K + sk] += (double)u[sk];
        }
      } else {  // cost: softmax(-(of * lost_orders + ov * lost_weight) / alpha)
        double lw = 0.0;
#pragma unroll
        for (int sk = 0; sk < K; sk++) lw += (double)u[sk] * c.skw[sk];
        double lg[WM], mx = -INFINITY, se = 0.0;
#pragma unroll
        for (int w = 0; w < WM; w++) {
          lg[w] = w < W ? -(c.ofT[r * W + w] * (double)lost_cnt + c.ovT[r * W + w] * lw) / c.alpha : -INFINITY;
          mx = lg[w] > mx ? lg[w] : mx;
        }
#pragma unroll
        for (int w = 0; w < WM; w++) {
          lg[w] = w < W ? exp(lg[w] - mx) : 0.0;
          se += lg[w];
        }
#pragma unroll
        for (int w = 0; w < WM; w++) {
          if (w < W) {
            const double wt = lg[w] / se;
            Lpen[w * BS] += wt * upen;
            if (dbg && info.lost_sales)
#pragma unroll
              for (int sk = 0; sk < K; sk++) info.lost_sales[e * WK + w * K + sk] += wt * (double)u[sk];
          }
        }
      }
    }
    // home-region features: incoming demand and units shipped home (multi_env.py:767-773)
    unsigned hm = c.home_mask[r];
    while (hm) {
      const int w = __builtin_ctz(hm);
      hm &= hm - 1u;
#pragma unroll
      for (int sk = 0; sk < K; sk++) {
        s.inc[(int64_t)(w * K + sk) * E + e] = dsum[sk];
        Lshh[(w * K + sk) * BS] = Lqsr[(w * K + sk) * BS];
      }
    }
    if (dbg) {
#pragma unroll
      for (int sk = 0; sk < K; sk++) {
        if (info.demand_per_region) info.demand_per_region[(e * R + r) * K + sk] = dsum[sk];
        if (info.unfulfilled_demands) info.unfulfilled_demands[(e * R + r) * K + sk] = u[sk];
      }
      if (info.lost_order_counts) info.lost_order_counts[e * R + r] = lost_cnt;
    }
#pragma unroll
    for (int w = 0; w < WM; w++)
      if (w < W && (touched >> w & 1u))
#pragma unroll
        for (int sk = 0; sk < K; sk++) Lqsr[(w * K + sk) * BS] = 0;
  };

  const int maxwh = c.max_wh;
  for (int oi = 0; oi < n_orders; oi++) {
    int r, d[K];
    load_rec<K>(src + oi * rec_step, stride, r, d);
    if (r != cur) {
      if (cur >= 0) finalize(cur);
      cur = r;
      lost_cnt = 0;
      touched = 0;
#pragma unroll
      for (int sk = 0; sk < K; sk++) u[sk] = dsum[sk] = 0;
    }
    bool any_d = false;
    double tw = 0.0;
#pragma unroll
    for (int sk = 0; sk < K; sk++) {
      dsum[sk] += d[sk];
      any_d |= d[sk] > 0;
      tw += (double)d[sk] * c.skw[sk];
    }
    if (!any_d) continue;  // an empty order ships nothing and is never lost
    double cst[WM];
    int ix[WM];
#pragma unroll
    for (int w = 0; w < WM; w++) {
      cst[w] = w < W ? c.ofT[r * W + w] + c.ovT[r * W + w] * tw : INFINITY;
      ix[w] = w;
    }
    sort_costs<WM>(cst, ix);
    int rem[K];
#pragma unroll
    for (int sk = 0; sk < K; sk++) rem[sk] = d[sk];
    int used = 0;
#pragma unroll
    for (int k = 0; k < WM; k++) {
      if (k >= W || used >= maxwh) break;
      const int w = ix[k];
      int fl[K];
      bool any = false;
#pragma unroll
      for (int sk = 0; sk < K; sk++) {
        const int iv = Linv[(w * K + sk) * BS];
        fl[sk] = rem[sk] < iv ? rem[sk] : iv;
        any |= fl[sk] > 0;
      }
      if (!any) continue;
      double fw = 0.0;
      int fsum = 0;
      bool done = true;
#pragma unroll
      for (int sk = 0; sk < K; sk++) {
        const int idx = (w * K + sk) * BS;
        Linv[idx] -= fl[sk];
        Lqsr[idx] += fl[sk];
        Lsht[idx] += fl[sk];
        rem[sk] -= fl[sk];
        done &= rem[sk] <= 0;
        fsum += fl[sk];
        fw += (double)fl[sk] * c.skw[sk];
        if (dbg) {
          if (info.shipment_quantities_by_sku) info.shipment_quantities_by_sku[((e * W + w) * R + r) * K + sk] += fl[sk];
          if (info.fulfilled_per_warehouse) info.fulfilled_per_warehouse[e * WK + w * K + sk] += fl[sk];
        }
      }
      Lout[w * BS] += c.ofT[r * W + w] + c.ovT[r * W + w] * fw;
      touched |= 1u << w;
      used++;
      if (dbg) {
        if (info.shipment_counts) info.shipment_counts[(e * W + w) * R + r] += 1;
        if (info.shipment_quantities) info.shipment_quantities[(e * W + w) * R + r] += fsum;
      }
      if (done) break;
    }
    bool anyrem = false;
#pragma unroll
    for (int sk = 0; sk < K; sk++) {
      anyrem |= rem[sk] > 0;
      u[sk] += rem[sk] > 0 ? rem[sk] : 0;
    }
    lost_cnt += anyrem ? 1 : 0;
  }
  if (cur >= 0) finalize(cur);

  // ---- phase C: inventory, history, forecast, rewards, observations -------------------------
  const int hslot = t % MSC_HISTORY;
  for (int i = 0; i < WK; i++) {
    s.inv[i * E + e] = Linv[i * BS];
    const int v = s.inc[i * E + e];
    s.hist[((int64_t)hslot * WK + i) * E + e] = v;
    // EMA forecast in float32: 0.3 * x + 0.7 * f (python floats are weak scalars under NEP 50)
    s.fc[i * E + e] = 0.3f * (float)v + 0.7f * s.fc[i * E + e];
  }
  double rw[WM];
  double team = 0.0;
#pragma unroll
  for (int w = 0; w < WM; w++) {
    rw[w] = 0.0;
    if (w < W) {
      double hold = 0.0;
#pragma unroll
      for (int sk = 0; sk < K; sk++) {
        const double iv = (double)Linv[(w * K + sk) * BS];
        hold += c.hold_per_sku ? iv * c.hold[sk] : (iv * c.skw[sk]) * c.hold_scalar;
      }
      const double pen = Lpen[w * BS], out = Lout[w * BS], inb = Linb[w * BS];
      rw[w] = -((((hold + pen) + out) + inb) * c.scale);
      team += rw[w];
      if (dbg && info.costs) {
        info.costs[(e * 4 + 0) * W + w] = hold;
        info.costs[(e * 4 + 1) * W + w] = pen;
        info.costs[(e * 4 + 2) * W + w] = out;
        info.costs[(e * 4 + 3) * W + w] = inb;
      }
    }
  }
#pragma unroll
  for (int w = 0; w < WM; w++) {
    if (w < W) {
      const double v = c.scope == MSC_SCOPE_TEAM ? team : rw[w];
      io.rew[e * W + w] = (float)v;
      if (io.rew64) io.rew64[e * W + w] = v;
    }
  }
  const int n_hist = t + 1 < MSC_HISTORY ? t + 1 : MSC_HISTORY;
  const bool trunc = t + 1 >= c.T;
  io.trunc[e] = trunc ? 1 : 0;
  const int64_t obs_off = e * W * c.L;
  if (!trunc) {
    s.t[e] = t + 1;
    build_obs<K>(c, s, e, t, n_hist, Lshh, Lsht, io.obs + obs_off);
  } else {
    if (io.final_obs) build_obs<K>(c, s, e, t, n_hist, Lshh, Lsht, io.final_obs + obs_off);
    reset_env<K>(c, s, e, 0, nullptr);
    build_obs<K>(c, s, e, 0, 0, nullptr, nullptr, io.obs + obs_off);
  }
}

// flat per-agent obs [E][W][L(1+W)] = local_w || local_0 .. local_{W-1} (multi_env.py:566-573)
__global__ void obs_flat_kernel(const float* __restrict__ obs, float* __restrict__ flat, int64_t E, int W, int L) {
  const int64_t FL = (int64_t)L * (1 + W);
  const int64_t n = E * W * FL;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < n; idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = idx % FL, ew = idx / FL, e = ew / W;
    const int64_t w = ew % W;
    flat[idx] = j < L ? obs[(e * W + w) * L + j] : obs[e * W * L + (j - L)];
  }
}

// ------------------------------------------------------------------------------------------
// launchers: dispatch on (K, W bucket)
// ------------------------------------------------------------------------------------------
int order_record_vec4(int K) { return (1 + K + 7) / 8; }

size_t step_lds_bytes(const EnvConst& c) {
  return (size_t)BS * (4 * (size_t)c.W * c.K * sizeof(int32_t) + 3 * (size_t)c.W * sizeof(double));
}

#define MSC_K_SWITCH(KV, BODY) \
  switch (KV) {                \
    case 1: { constexpr int K = 1; BODY; } break; \
    case 2: { constexpr int K = 2; BODY; } break; \
    case 3: { constexpr int K = 3; BODY; } break; \
    case 4: { constexpr int K = 4; BODY; } break; \
    case 5: { constexpr int K = 5; BODY; } break; \
    case 6: { constexpr int K = 6; BODY; } break; \
    case 7: { constexpr int K = 7; BODY; } break; \
    case 8: { constexpr int K = 8; BODY; } break; \
    default: return hipErrorInvalidValue; \
  }

static dim3 grid_for(int64_t E) { return dim3((unsigned)((E + BS - 1) / BS)); }

hipError_t launch_reset(const EnvConst& c, const EnvState& s, const uint8_t* mask, const uint32_t* new_roots,
                        int32_t flags, float* obs, hipStream_t st) {
  MSC_K_SWITCH(c.K, hipLaunchKernelGGL(reset_kernel<K>, grid_for(c.E), dim3(BS), 0, st, c, s, mask, new_roots, flags, obs));
  return hipGetLastError();
}

hipError_t launch_demand(const EnvConst& c, const EnvState& s, hipStream_t st) {
  MSC_K_SWITCH(c.K, hipLaunchKernelGGL(demand_poisson_kernel<K>, grid_for(c.E), dim3(BS), 0, st, c, s));
  return hipGetLastError();
}

template <int K>
static hipError_t launch_step_k(const EnvConst& c, const EnvState& s, const StepIO& io, bool gen, hipStream_t st) {
  const size_t lds = step_lds_bytes(c);
  if (gen && c.demand_type == MSC_DEMAND_POISSON)
    hipLaunchKernelGGL(demand_poisson_kernel<K>, grid_for(c.E), dim3(BS), 0, st, c, s);
  if (c.W <= 4)
    hipLaunchKernelGGL((step_kernel<K, 4>), grid_for(c.E), dim3(BS), lds, st, c, s, io);
  else if (c.W <= 8)
    hipLaunchKernelGGL((step_kernel<K, 8>), grid_for(c.E), dim3(BS), lds, st, c, s, io);
  else
    hipLaunchKernelGGL((step_kernel<K, 16>), grid_for(c.E), dim3(BS), lds, st, c, s, io);
  return hipGetLastError();
}

hipError_t launch_step(const EnvConst& c, const EnvState& s, const StepIO& io, bool gen, hipStream_t st) {
  MSC_K_SWITCH(c.K, return launch_step_k<K>(c, s, io, gen, st));
  return hipSuccess;
}

hipError_t launch_obs_flat(const EnvConst& c, const float* obs, float* flat, hipStream_t st) {
  const int64_t n = c.E * c.W * (int64_t)c.L * (1 + c.W);
  const int64_t blocks = (n + 255) / 256 < 65536 ? (n + 255) / 256 : 65536;
  hipLaunchKernelGGL(obs_flat_kernel, dim3((unsigned)blocks), dim3(256), 0, st, obs, flat, c.E, c.W, c.L);
  return hipGetLastError();
}

}  // namespace msc
