/*
 * msc_oracle.c -- TEST INFRASTRUCTURE ONLY: the parity checker and the CPU baseline.
 *
 * A deliberately plain, scalar C restatement of the reference's environment hot path. Every
 * function follows one reference function and says which (paths relative to /root/reference).
 * numpy 2.2's Generator pieces are restated from their published algorithms (SeedSequence
 * hash-mix pool, PCG64 XSL-RR 128/64, next_double, Poisson multiplication method for lam < 10 and
 * PTRS for lam >= 10, 32-bit buffered Lemire bounded integers); pinned by tests/golden/rng_streams.npz
 * and tests/golden/poisson_ptrs.npz.
 *
 * dtype flow mirrors numpy exactly (f32 buffers where the reference keeps f32, f64 elsewhere),
 * and reductions use numpy's order (sequential for n < 8, 8-way unrolled pairwise blocks up to
 * 128) so that outputs are bit-identical to the golden fixtures where the reference is
 * deterministic. Build: oracle/Makefile (gcc -O2 -ffp-contract=off -fopenmp).
 */
#include "msc_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;

static __thread char g_err[512];
const char* orc_error(void) { return g_err; }
#define FAIL(...) do { snprintf(g_err, sizeof g_err, __VA_ARGS__); return NULL; } while (0)

/* ------------------------------------------------------------------------------------------
 * numpy SeedSequence (numpy/random/bit_generator.pyx: mix_entropy, generate_state, spawn)
 * ------------------------------------------------------------------------------------------ */
#define SS_INIT_A 0x43b0d7e5u
#define SS_MULT_A 0x931e8875u
#define SS_INIT_B 0x8b51f9ddu
#define SS_MULT_B 0x58f38dedu
#define SS_MIX_L 0xca01f9ddu
#define SS_MIX_R 0x4973f715u

static uint32_t ss_hashmix(uint32_t v, uint32_t* hc) {
  v ^= *hc;
  *hc *= SS_MULT_A;
  v *= *hc;
  v ^= v >> 16;
  return v;
}
static uint32_t ss_mix(uint32_t x, uint32_t y) {
  uint32_t r = SS_MIX_L * x - SS_MIX_R * y;
  r ^= r >> 16;
  return r;
}
/* entropy words (already coerced to uint32) + spawn key -> 4-word pool */
static void ss_pool(const uint32_t* ent, int n_ent, const uint32_t* key, int n_key, uint32_t pool[4]) {
  uint32_t buf[64];
  int n = 0;
  for (int i = 0; i < n_ent; i++) buf[n++] = ent[i];
  if (n_key > 0)
    while (n < 4) buf[n++] = 0; /* zero-pad run entropy to the pool size when spawned */
  for (int i = 0; i < n_key; i++) buf[n++] = key[i];
  uint32_t hc = SS_INIT_A;
  for (int i = 0; i < 4; i++) pool[i] = ss_hashmix(i < n ? buf[i] : 0u, &hc);
  for (int s = 0; s < 4; s++)
    for (int d = 0; d < 4; d++)
      if (s != d) pool[d] = ss_mix(pool[d], ss_hashmix(pool[s], &hc));
  for (int s = 4; s < n; s++)
    for (int d = 0; d < 4; d++) pool[d] = ss_mix(pool[d], ss_hashmix(buf[s], &hc));
}
static void ss_generate(const uint32_t pool[4], uint32_t* out, int n_words) {
  uint32_t hc = SS_INIT_B;
  for (int i = 0; i < n_words; i++) {
    uint32_t v = pool[i & 3];
    v ^= hc;
    hc *= SS_MULT_B;
    v *= hc;
    v ^= v >> 16;
    out[i] = v;
  }
}
void orc_seedseq_state(const uint32_t* ent, int32_t n_ent, const uint32_t* key, int32_t n_key, uint32_t* out,
                       int32_t n_words) {
  uint32_t pool[4];
  ss_pool(ent, n_ent, key, n_key, pool);
  ss_generate(pool, out, n_words);
}
uint32_t orc_seedseq_u32(const uint32_t* words, int32_t n) {
  uint32_t o;
  orc_seedseq_state(words, n, NULL, 0, &o, 1);
  return o;
}

/* ------------------------------------------------------------------------------------------
 * PCG64 (numpy/random/src/pcg64/pcg64.h) + distributions.c pieces
 * ------------------------------------------------------------------------------------------ */
typedef struct { u128 state, inc; int has32; uint32_t u32; } pcg64_t;
#define PCG_MULT ((((u128)2549297995355413924ULL) << 64) + 4865540595714422341ULL)

static inline void pcg_step(pcg64_t* r) { r->state = r->state * PCG_MULT + r->inc; }
static inline uint64_t pcg_next64(pcg64_t* r) {
  pcg_step(r);
  uint64_t x = (uint64_t)(r->state >> 64) ^ (uint64_t)r->state;
  unsigned rot = (unsigned)(r->state >> 122);
  return (x >> rot) | (x << ((64 - rot) & 63));
}
static inline uint32_t pcg_next32(pcg64_t* r) {
  if (r->has32) { r->has32 = 0; return r->u32; }
  uint64_t v = pcg_next64(r);
  r->has32 = 1;
  r->u32 = (uint32_t)(v >> 32);
  return (uint32_t)v;
}
static inline double pcg_double(pcg64_t* r) { return (double)(pcg_next64(r) >> 11) * (1.0 / 9007199254740992.0); }

/* PCG64(SeedSequence): generate_state(4, uint64) -> pcg64_set_seed(seed = w[0..1], inc = w[2..3]) */
static void pcg_from_pool(pcg64_t* r, const uint32_t pool[4]) {
  uint32_t w[8];
  ss_generate(pool, w, 8);
  uint64_t s[4];
  for (int i = 0; i < 4; i++) s[i] = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
  u128 initstate = ((u128)s[0] << 64) | s[1];
  u128 initseq = ((u128)s[2] << 64) | s[3];
  r->state = 0;
  r->inc = (initseq << 1) | 1u;
  pcg_step(r);
  r->state += initstate;
  pcg_step(r);
  r->has32 = 0;
  r->u32 = 0;
}

/* random_loggam (numpy/random/src/distributions/distributions.c, numpy 2.2): log Gamma(x) by the
 * Stirling series with the argument shifted to >= 7, used by the PTRS acceptance test. */
static double np_loggam(double x) {
  static const double a[10] = {8.333333333333333e-02, -2.777777777777778e-03, 7.936507936507937e-04,
                               -5.952380952380952e-04, 8.417508417508418e-04, -1.917526917526918e-03,
                               6.410256410256410e-03, -2.955065359477124e-02, 1.796443723688307e-01,
                               -1.39243221690590e+00};
  if (x == 1.0 || x == 2.0) return 0.0;
  int64_t n = x < 7.0 ? (int64_t)(7 - x) : 0;
  double x0 = x + n;
  const double x2 = (1.0 / x0) * (1.0 / x0);
  const double lg2pi = 1.8378770664093453e+00;
  double gl0 = a[9];
  for (int k = 8; k >= 0; k--) {
    gl0 *= x2;
    gl0 += a[k];
  }
  double gl = gl0 / x0 + 0.5 * lg2pi + (x0 - 0.5) * log(x0) - x0;
  if (x < 7.0) {
    for (int64_t k = 1; k <= n; k++) {
      gl -= log(x0 - 1.0);
      x0 -= 1.0;
    }
  }
  return gl;
}

/* random_poisson_ptrs (distributions.c): Hoermann's transformed rejection (Insurance: Mathematics
 * and Economics 12, 39-45, 1993), numpy's sampler for lam >= 10; two doubles per trial. */
static int64_t np_poisson_ptrs(pcg64_t* r, double lam) {
  const double slam = sqrt(lam), loglam = log(lam);
  const double b = 0.931 + 2.53 * slam;
  const double a = -0.059 + 0.02483 * b;
  const double invalpha = 1.1239 + 1.1328 / (b - 3.4);
  const double vr = 0.9277 - 3.6224 / (b - 2);
  for (;;) {
    const double U = pcg_double(r) - 0.5;
    const double V = pcg_double(r);
    const double us = 0.5 - fabs(U);
    const int64_t k = (int64_t)floor((2 * a / us + b) * U + lam + 0.43);
    if ((us >= 0.07) && (V <= vr)) return k;
    if ((k < 0) || ((us < 0.013) && (V > us))) continue;
    if ((log(V) + log(invalpha) - log(a / (us * us) + b)) <= (-lam + k * loglam - np_loggam(k + 1))) return k;
  }
}

/* random_poisson: multiplication method for 0 < lam < 10, PTRS for lam >= 10 (distributions.c). */
static int64_t np_poisson(pcg64_t* r, double lam, double enlam) {
  if (lam >= 10) return np_poisson_ptrs(r, lam);
  if (lam == 0) return 0;
  int64_t X = 0;
  double prod = 1.0;
  for (;;) {
    prod *= pcg_double(r);
    if (prod > enlam) X += 1;
    else return X;
  }
}
/* Generator.integers(low, high) int64: random_bounded_uint64 with the 32-bit Lemire path. */
static int64_t np_integers(pcg64_t* r, int64_t low, int64_t high_excl) {
  uint64_t rng = (uint64_t)(high_excl - 1 - low);
  if (rng == 0) return low;
  if (rng == 0xFFFFFFFFull) return low + (int64_t)pcg_next32(r);
  if (rng < 0xFFFFFFFFull) {
    uint32_t rng_excl = (uint32_t)rng + 1u;
    uint64_t m = (uint64_t)pcg_next32(r) * rng_excl;
    uint32_t left = (uint32_t)m;
    if (left < rng_excl) {
      uint32_t thr = (uint32_t)(0xFFFFFFFFu - (uint32_t)rng) % rng_excl;
      while (left < thr) {
        m = (uint64_t)pcg_next32(r) * rng_excl;
        left = (uint32_t)m;
      }
    }
    return low + (int64_t)(m >> 32);
  }
  /* 64-bit ranges never occur on this path (lead deviations, inventory bounds, trace windows) */
  uint64_t rng_excl = rng + 1;
  u128 m = (u128)pcg_next64(r) * rng_excl;
  uint64_t left = (uint64_t)m;
  if (left < rng_excl) {
    uint64_t thr = (UINT64_MAX - rng) % rng_excl;
    while (left < thr) {
      m = (u128)pcg_next64(r) * rng_excl;
      left = (uint64_t)m;
    }
  }
  return low + (int64_t)(m >> 64);
}

static void rng_export(const pcg64_t* p, uint64_t* w) {
  w[0] = (uint64_t)(p->state >> 64);
  w[1] = (uint64_t)p->state;
  w[2] = (uint64_t)(p->inc >> 64);
  w[3] = (uint64_t)p->inc;
  w[4] = (uint64_t)p->has32;
  w[5] = p->u32;
}
static void rng_import(pcg64_t* p, const uint64_t* w) {
  p->state = ((u128)w[0] << 64) | w[1];
  p->inc = ((u128)w[2] << 64) | w[3];
  p->has32 = (int)w[4];
  p->u32 = (uint32_t)w[5];
}
void orc_rng_seed(orc_rng* r, const uint32_t* ent, int32_t n_ent, const uint32_t* key, int32_t n_key) {
  uint32_t pool[4];
  pcg64_t p;
  ss_pool(ent, n_ent, key, n_key, pool);
  pcg_from_pool(&p, pool);
  rng_export(&p, r->w);
}
#define RNG_WRAP(body) pcg64_t p; rng_import(&p, r->w); body; rng_export(&p, r->w)
uint64_t orc_rng_next64(orc_rng* r) { uint64_t v; RNG_WRAP(v = pcg_next64(&p)); return v; }
double orc_rng_random(orc_rng* r) { double v; RNG_WRAP(v = pcg_double(&p)); return v; }
int64_t orc_rng_poisson(orc_rng* r, double lam) { int64_t v; RNG_WRAP(v = np_poisson(&p, lam, exp(-lam))); return v; }
/* n draws of Generator.poisson(lam[i % n_lam]) (numpy draws an array of rates element by element) */
void orc_rng_poisson_n(orc_rng* r, const double* lam, int64_t n_lam, int64_t n, int64_t* out) {
  RNG_WRAP(for (int64_t i = 0; i < n; i++) out[i] = np_poisson(&p, lam[i % n_lam], exp(-lam[i % n_lam])));
}
int64_t orc_rng_integers(orc_rng* r, int64_t lo, int64_t hi) { int64_t v; RNG_WRAP(v = np_integers(&p, lo, hi)); return v; }

/* numpy add.reduce order for a contiguous double/float vector (pairwise_sum, n <= 128 path). */
static double np_sum_f64(const double* a, int n, int stride) {
  if (n < 8) {
    double s = 0.0;
    for (int i = 0; i < n; i++) s += a[i * stride];
    return s;
  }
  if (n <= 128) {
    double r[8];
    for (int j = 0; j < 8; j++) r[j] = a[j * stride];
    int i;
    for (i = 8; i < n - (n % 8); i += 8)
      for (int j = 0; j < 8; j++) r[j] += a[(i + j) * stride];
    double s = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; i++) s += a[i * stride];
    return s;
  }
  int n2 = n / 2;
  n2 -= n2 % 8;
  return np_sum_f64(a, n2, stride) + np_sum_f64(a + n2 * stride, n - n2, stride);
}
static float np_sum_f32(const float* a, int n) {
  if (n < 8) {
    float s = 0.0f;
    for (int i = 0; i < n; i++) s += a[i];
    return s;
  }
  if (n <= 128) {
    float r[8];
    for (int j = 0; j < 8; j++) r[j] = a[j];
    int i;
    for (i = 8; i < n - (n % 8); i += 8)
      for (int j = 0; j < 8; j++) r[j] += a[i + j];
    float s = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; i++) s += a[i];
    return s;
  }
  int n2 = n / 2;
  n2 -= n2 % 8;
  return np_sum_f32(a, n2) + np_sum_f32(a + n2, n - n2);
}

/* ------------------------------------------------------------------------------------------
 * Environment
 * ------------------------------------------------------------------------------------------ */
typedef struct { double q; int32_t act, exp; } pend_t; /* PendingOrder, multi_env.py:22-35 */
typedef struct { int32_t region; double d[MSC_MAX_K]; } order_t; /* Order, demand_sampler.py:12-24 */

typedef struct {
  pcg64_t rd, rl;                   /* demand_sampler / lead_time_sampler generators */
  uint32_t orig_root, root;
  int32_t counter, t;
  int64_t emp_start;                /* EmpiricalDemandSampler._start_timestep index (-1: unset) */
  double* inv;                      /* [W*K] float64 */
  pend_t* pend;                     /* [W*K][cap] */
  int32_t* pend_n;                  /* [W*K] */
  float* inc_home;                  /* [W*K] f32 */
  double* ship_home;                /* [W*K] f64 */
  double* ship_away;                /* [W*K] f64 */
  float* stockout;                  /* [W*K] */
  float* roll_mean;                 /* [W*K] */
  float* forecast;                  /* [W*K] */
  float* hist;                      /* [5][W*K] ring, oldest at hist_head */
  int32_t hist_n, hist_head;
  order_t* orders;                  /* per-step scratch */
  int32_t orders_cap;
} env_t;

struct orc_env {
  msc_env_desc d;                   /* scalars; array pointers below are owned copies */
  int W, K, R, L, F, Lmax, pend_cap;
  double *act_param, *hold, *pen, *skw, *dist, *of, *ov, *inf, *inv_var;
  double *lo, *ps, *lq, *enlam_o, *enlam_q;
  int64_t* tr_off; int32_t *tr_reg, *tr_q;
  int32_t *elt, *maxdev, *init_vals;
  float *obs_mean, *obs_std;
  int32_t *home, *closest;
  int64_t E;
  env_t* envs;
};

#define DUP(dst, src, n, T)                                      \
  do {                                                             \
    (dst) = NULL;                                                  \
    if ((src) != NULL && (n) > 0) {                                \
      (dst) = (T*)malloc(sizeof(T) * (size_t)(n));                 \
      memcpy((dst), (src), sizeof(T) * (size_t)(n));               \
    }                                                              \
  } while (0)

static int feature_dim(const orc_env* o) {
  uint32_t f = o->d.feature_flags;
  int K = o->K, n = 0;
  if (f & MSC_F_INVENTORY) n += K + ((f & MSC_F_INVENTORY_AGG) ? 1 : 0);
  if (f & MSC_F_PIPELINE) n += o->Lmax * K + ((f & MSC_F_PIPELINE_AGG) ? 1 : 0);
  if (f & MSC_F_INCOMING_HOME) n += K + ((f & MSC_F_INCOMING_HOME_AGG) ? 1 : 0);
  if (f & MSC_F_SHIPPED_HOME) n += K;
  if (f & MSC_F_SHIPPED_AWAY) n += K + ((f & MSC_F_SHIPPED_AWAY_AGG) ? 1 : 0);
  if (f & MSC_F_STOCKOUT) n += K;
  if (f & MSC_F_ROLLING_MEAN) n += K + ((f & MSC_F_ROLLING_MEAN_AGG) ? 1 : 0);
  if (f & MSC_F_FORECAST) n += K + ((f & MSC_F_FORECAST_AGG) ? 1 : 0);
  if (f & MSC_F_DAYS_OF_SUPPLY) n += K;
  if (f & MSC_F_NET_POSITION) n += K;
  if (f & MSC_F_DEMAND_VARIABILITY) n += K;
  if (f & MSC_F_DEMAND_HISTORY) n += MSC_HISTORY * K;
  return n;
}

orc_env* orc_create(const msc_env_desc* d, int64_t E, uint32_t base_seed, uint32_t worker, int64_t off,
                    const uint32_t* env_seeds) {
  int W = d->n_warehouses, K = d->n_skus, R = d->n_regions;
  if (W < 1 || W > MSC_MAX_W || K < 1 || K > MSC_MAX_K || R < 1 || R > MSC_MAX_R) FAIL("bad dims");
  orc_env* o = (orc_env*)calloc(1, sizeof(orc_env));
  o->d = *d;
  o->W = W; o->K = K; o->R = R; o->E = E;
  DUP(o->act_param, d->action_param, K, double);
  DUP(o->hold, d->holding_cost, d->holding_per_sku ? K : 1, double);
  DUP(o->pen, d->penalty_cost, d->penalty_per_sku ? K : 1, double);
  DUP(o->skw, d->sku_weights, K, double);
  DUP(o->dist, d->distances, W * R, double);
  DUP(o->of, d->outbound_fixed, W * R, double);
  DUP(o->ov, d->outbound_variable, W * R, double);
  DUP(o->inf, d->inbound_fixed, W * K, double);
  DUP(o->inv_var, d->inbound_variable, W * K, double);
  DUP(o->elt, d->expected_lead_times, W * K, int32_t);
  DUP(o->maxdev, d->max_deviation, d->max_dev_per_sku ? K : 1, int32_t);
  DUP(o->init_vals, d->init_values, W * K, int32_t);
  if (d->demand_type == MSC_DEMAND_POISSON) {
    DUP(o->lo, d->lambda_orders, R, double);
    DUP(o->ps, d->probability_skus, R, double);
    DUP(o->lq, d->lambda_quantity, R * K, double);
    o->enlam_o = (double*)malloc(sizeof(double) * R);
    o->enlam_q = (double*)malloc(sizeof(double) * R * K);
    for (int r = 0; r < R; r++) {
      if (!(o->lo[r] < 1e6) || !(o->lo[r] >= 0.0)) FAIL("lambda_orders must be in [0, 1e6)");
      o->enlam_o[r] = exp(-o->lo[r]);
      for (int s = 0; s < K; s++) {
        if (!(o->lq[r * K + s] < 20000.0)) FAIL("lambda_quantity must be < 20000");
        o->enlam_q[r * K + s] = exp(-o->lq[r * K + s]);
      }
    }
  } else {
    int64_t n_ord = d->trace_offsets[d->trace_n_rows];
    DUP(o->tr_off, d->trace_offsets, d->trace_n_rows + 1, int64_t);
    DUP(o->tr_reg, d->trace_regions, n_ord, int32_t);
    DUP(o->tr_q, d->trace_quantities, n_ord * K, int32_t);
    if (d->trace_n_rows < d->episode_length) FAIL("trace shorter than episode_length");
  }
  o->Lmax = 0;
  int lact_max = 0;
  for (int i = 0; i < W * K; i++) {
    if (o->elt[i] > o->Lmax) o->Lmax = o->elt[i];
    int dv = d->lead_type == MSC_LEAD_STOCHASTIC ? (d->max_dev_per_sku ? o->maxdev[i % K] : o->maxdev[0]) : 0;
    if (o->elt[i] + dv > lact_max) lact_max = o->elt[i] + dv;
  }
  o->pend_cap = d->episode_length + 1;
  o->F = feature_dim(o);
  o->L = o->F + (d->include_warehouse_id ? W : 0);
  if (d->obs_norm == MSC_OBS_MEANSTD) {
    DUP(o->obs_mean, d->obs_mean, o->F, float);
    DUP(o->obs_std, d->obs_std, o->F, float);
  }
  /* home_regions = argmin(distances, axis=1) (multi_env.py:144);
   * closest_warehouses = argmin(distances, axis=0) (lost_sales_handler.py:36) */
  o->home = (int32_t*)malloc(sizeof(int32_t) * W);
  o->closest = (int32_t*)malloc(sizeof(int32_t) * R);
  for (int w = 0; w < W; w++) {
    int b = 0;
    for (int r = 1; r < R; r++)
      if (o->dist[w * R + r] < o->dist[w * R + b]) b = r;
    o->home[w] = b;
  }
  for (int r = 0; r < R; r++) {
    int b = 0;
    for (int w = 1; w < W; w++)
      if (o->dist[w * R + r] < o->dist[b * R + r]) b = w;
    o->closest[r] = b;
  }
  o->envs = (env_t*)calloc((size_t)E, sizeof(env_t));
  int WK = W * K;
  for (int64_t i = 0; i < E; i++) {
    env_t* e = &o->envs[i];
    if (env_seeds) e->orig_root = env_seeds[i];
    else {
      uint64_t idx = (uint64_t)(off + i);
      uint32_t words[4] = {base_seed, worker, (uint32_t)idx, (uint32_t)(idx >> 32)};
      e->orig_root = orc_seedseq_u32(words, idx >> 32 ? 4 : 3); /* derive_env_seed, seed_manager.py:165-186 */
    }
    e->root = e->orig_root;
    e->inv = (double*)calloc(WK, sizeof(double));
    e->pend = (pend_t*)calloc((size_t)WK * o->pend_cap, sizeof(pend_t));
    e->pend_n = (int32_t*)calloc(WK, sizeof(int32_t));
    e->inc_home = (float*)calloc(WK, sizeof(float));
    e->ship_home = (double*)calloc(WK, sizeof(double));
    e->ship_away = (double*)calloc(WK, sizeof(double));
    e->stockout = (float*)calloc(WK, sizeof(float));
    e->roll_mean = (float*)calloc(WK, sizeof(float));
    e->forecast = (float*)calloc(WK, sizeof(float));
    e->hist = (float*)calloc((size_t)MSC_HISTORY * WK, sizeof(float));
    e->orders_cap = 64;
    e->orders = (order_t*)malloc(sizeof(order_t) * e->orders_cap);
    e->emp_start = -1;
  }
  (void)lact_max;
  return o;
}

void orc_destroy(orc_env* o) {
  if (!o) return;
  for (int64_t i = 0; i < o->E; i++) {
    env_t* e = &o->envs[i];
    free(e->inv); free(e->pend); free(e->pend_n); free(e->inc_home); free(e->ship_home);
    free(e->ship_away); free(e->stockout); free(e->roll_mean); free(e->forecast); free(e->hist);
    free(e->orders);
  }
  free(o->envs);
  void* ptrs[] = {o->act_param, o->hold, o->pen, o->skw, o->dist, o->of, o->ov, o->inf, o->inv_var, o->lo,
                  o->ps, o->lq, o->enlam_o, o->enlam_q, o->tr_off, o->tr_reg, o->tr_q, o->elt, o->maxdev,
                  o->init_vals, o->obs_mean, o->obs_std, o->home, o->closest};
  for (size_t i = 0; i < sizeof ptrs / sizeof ptrs[0]; i++) free(ptrs[i]);
  free(o);
}

void orc_dims(const orc_env* o, int32_t* L, int32_t* F, int32_t* lmax) {
  if (L) *L = o->L;
  if (F) *F = o->F;
  if (lmax) *lmax = o->Lmax;
}

/* _compute_pipeline, multi_env.py:941-968 */
static void pipeline(const orc_env* o, const env_t* e, int w, float* pipe /*[Lmax][K]*/) {
  int K = o->K;
  memset(pipe, 0, sizeof(float) * o->Lmax * K);
  for (int s = 0; s < K; s++) {
    const pend_t* q = &e->pend[(size_t)(w * K + s) * o->pend_cap];
    for (int j = 0; j < e->pend_n[w * K + s]; j++) {
      int slot = q[j].exp - e->t;
      if (slot >= 1 && slot <= o->Lmax) pipe[(slot - 1) * K + s] += (float)q[j].q;
      else if (slot <= 0) pipe[s] += (float)q[j].q;
    }
  }
}

/* _build_local_obs, multi_env.py:577-710 (dtype flow of each block noted inline) */
static void build_local_obs(const orc_env* o, const env_t* e, int w, float* out) {
  const int K = o->K;
  const uint32_t f = o->d.feature_flags;
  const int ratio = o->d.obs_norm == MSC_OBS_RATIO;
  const double eps = 1e-8;
  const float epsf = (float)1e-8;
  double loc[1024];
  int n = 0;
  const double* inv = &e->inv[w * K];
  const float* dh = &e->inc_home[w * K];
  const double* sh = &e->ship_home[w * K];
  const double* sa = &e->ship_away[w * K];
  const float* so = &e->stockout[w * K];
  const float* rm = &e->roll_mean[w * K];
  const float* fc = &e->forecast[w * K];
  float pipe[64 * MSC_MAX_K];
  pipeline(o, e, w, pipe);
  int P = o->Lmax * K;
  float pending_total_f = np_sum_f32(pipe, P);
  double pending_total = (double)pending_total_f;
  double inv_total = np_sum_f64(inv, K, 1);
  float dh_total = np_sum_f32(dh, K);
  double shp[MSC_MAX_K] = {0};
  for (int s = 0; s < K; s++) shp[s] = sh[s] + sa[s];
  double shipped_total = np_sum_f64(shp, K, 1);
  float rm_total = np_sum_f32(rm, K);
  float fc_total = np_sum_f32(fc, K);

  if (f & MSC_F_INVENTORY) { /* f64 block */
    for (int s = 0; s < K; s++) loc[n++] = ratio ? inv[s] / (inv_total + eps) : inv[s];
    if (f & MSC_F_INVENTORY_AGG) loc[n++] = (double)(float)inv_total;
  }
  if (f & MSC_F_PIPELINE) { /* f32 / (python float -> f32) */
    float den = (float)(pending_total + eps);
    for (int i = 0; i < P; i++) loc[n++] = ratio ? (double)(pipe[i] / den) : (double)pipe[i];
    if (f & MSC_F_PIPELINE_AGG) loc[n++] = pending_total;
  }
  if (f & MSC_F_INCOMING_HOME) { /* f32 / f32(total + eps) */
    float den = dh_total + epsf;
    for (int s = 0; s < K; s++) loc[n++] = ratio ? (double)(dh[s] / den) : (double)dh[s];
    if (f & MSC_F_INCOMING_HOME_AGG) loc[n++] = (double)dh_total;
  }
  if (f & MSC_F_SHIPPED_HOME) { /* f64 / f64(f32(total + eps)) */
    double den = (double)(dh_total + epsf);
    for (int s = 0; s < K; s++) loc[n++] = ratio ? sh[s] / den : sh[s];
  }
  if (f & MSC_F_SHIPPED_AWAY) { /* f64 / f64 */
    for (int s = 0; s < K; s++) loc[n++] = ratio ? sa[s] / (shipped_total + eps) : sa[s];
    if (f & MSC_F_SHIPPED_AWAY_AGG) loc[n++] = (double)(float)(np_sum_f64(sa, K, 1) / (shipped_total + eps));
  }
  if (f & MSC_F_STOCKOUT) {
    float den = dh_total + epsf;
    for (int s = 0; s < K; s++) loc[n++] = ratio ? (double)(so[s] / den) : (double)so[s];
  }
  if (f & MSC_F_ROLLING_MEAN) {
    float den = rm_total + epsf;
    for (int s = 0; s < K; s++) loc[n++] = ratio ? (double)(rm[s] / den) : (double)rm[s];
    if (f & MSC_F_ROLLING_MEAN_AGG) loc[n++] = (double)rm_total;
  }
  if (f & MSC_F_FORECAST) {
    float den = fc_total + epsf;
    for (int s = 0; s < K; s++) loc[n++] = ratio ? (double)(fc[s] / den) : (double)fc[s];
    if (f & MSC_F_FORECAST_AGG) loc[n++] = (double)fc_total;
  }
  if (f & MSC_F_DAYS_OF_SUPPLY) /* inv(f64) / max(rolling(f32), 1.0) -> f32 */
    for (int s = 0; s < K; s++) loc[n++] = (double)(float)(inv[s] / (double)(rm[s] > 1.0f ? rm[s] : 1.0f));
  if (f & MSC_F_NET_POSITION) { /* inv + pipeline.sum(0) - forecast * lead (f64) */
    for (int s = 0; s < K; s++) {
      float ps = 0.0f;
      for (int l = 0; l < o->Lmax; l++) ps += pipe[l * K + s];
      double v = (inv[s] + (double)ps) - (double)fc[s] * (double)o->elt[w * K + s];
      loc[n++] = (double)(float)v;
    }
  }
  if (f & MSC_F_DEMAND_VARIABILITY) { /* np.std over history (f32), multi_env.py:682-688 */
    for (int s = 0; s < K; s++) {
      float sd = 0.0f;
      if (e->hist_n > 1) {
        float sum = 0.0f;
        for (int h = 0; h < e->hist_n; h++) sum += e->hist[((e->hist_head + h) % MSC_HISTORY) * o->W * K + w * K + s];
        float mean = sum / (float)e->hist_n;
        float ss = 0.0f;
        for (int h = 0; h < e->hist_n; h++) {
          float dv = e->hist[((e->hist_head + h) % MSC_HISTORY) * o->W * K + w * K + s] - mean;
          ss += dv * dv;
        }
        sd = sqrtf(ss / (float)e->hist_n);
      }
      loc[n++] = (double)sd;
    }
  }
  if (f & MSC_F_DEMAND_HISTORY) { /* most recent first, zero padded */
    for (int h = 0; h < MSC_HISTORY; h++)
      for (int s = 0; s < K; s++) {
        float v = 0.0f;
        if (h < e->hist_n) v = e->hist[((e->hist_head + e->hist_n - 1 - h) % MSC_HISTORY) * o->W * K + w * K + s];
        loc[n++] = (double)v;
      }
  }
  int off = 0;
  if (o->d.include_warehouse_id) {
    for (int j = 0; j < o->W; j++) out[j] = (j == w) ? 1.0f : 0.0f;
    off = o->W;
  }
  for (int i = 0; i < n; i++) {
    float v = (float)loc[i];
    if (o->d.obs_norm == MSC_OBS_MEANSTD) v = (v - o->obs_mean[i]) / o->obs_std[i];
    out[off + i] = v;
  }
}

static void get_obs(const orc_env* o, const env_t* e, float* out /*[W][L]*/) {
  for (int w = 0; w < o->W; w++) build_local_obs(o, e, w, out + (size_t)w * o->L);
}

/* reset, multi_env.py:192-251 with SeedManager (seed_manager.py:100-136, 207-224) */
static void reset_env(const orc_env* o, env_t* e, const uint32_t* new_root, int flags) {
  if (new_root) { /* update_root_seed */
    e->root = e->orig_root = *new_root;
    e->counter = 0;
  } else { /* advance_episode (construction-seeded path, with eval cycling) */
    if (o->d.num_eval_episodes > 0 && ((flags & MSC_RESET_EVAL_RESTART) || e->counter >= o->d.num_eval_episodes))
      e->counter = 0;
    uint32_t w2[2] = {e->orig_root, (uint32_t)e->counter};
    e->root = orc_seedseq_u32(w2, 2);
    e->counter += 1;
  }
  uint32_t pool[4], key;
  key = 2; ss_pool(&e->root, 1, &key, 1, pool); pcg_from_pool(&e->rd, pool); /* 'demand_sampler' */
  key = 3; ss_pool(&e->root, 1, &key, 1, pool); pcg_from_pool(&e->rl, pool); /* 'lead_time_sampler' */
  e->emp_start = -1;
  int W = o->W, K = o->K, WK = W * K;
  if (o->d.init_type == MSC_INIT_UNIFORM) { /* _initialize_inventory, multi_env.py:504-539 */
    pcg64_t ri;
    key = 1; ss_pool(&e->root, 1, &key, 1, pool); pcg_from_pool(&ri, pool);
    for (int i = 0; i < WK; i++) e->inv[i] = (double)np_integers(&ri, o->d.init_min, (int64_t)o->d.init_max + 1);
  } else if (o->d.init_type == MSC_INIT_CUSTOM) {
    for (int i = 0; i < WK; i++) e->inv[i] = (double)o->init_vals[i];
  } else {
    for (int i = 0; i < WK; i++) e->inv[i] = 0.0;
  }
  memset(e->pend_n, 0, sizeof(int32_t) * WK);
  memset(e->inc_home, 0, sizeof(float) * WK);
  memset(e->ship_home, 0, sizeof(double) * WK);
  memset(e->ship_away, 0, sizeof(double) * WK);
  memset(e->stockout, 0, sizeof(float) * WK);
  memset(e->roll_mean, 0, sizeof(float) * WK);
  memset(e->forecast, 0, sizeof(float) * WK);
  e->hist_n = 0;
  e->hist_head = 0;
  e->t = 0;
}

void orc_reset(orc_env* o, const uint8_t* mask, const uint32_t* new_roots, int32_t flags, float* obs) {
  size_t per = (size_t)o->W * o->L;
  for (int64_t i = 0; i < o->E; i++) {
    if (mask && !mask[i]) continue;
    reset_env(o, &o->envs[i], new_roots ? &new_roots[i] : NULL, flags);
    if (obs) get_obs(o, &o->envs[i], obs + per * i);
  }
}

static void push_order(env_t* e, int n, const order_t* ord) {
  if (n >= e->orders_cap) {
    e->orders_cap *= 2;
    e->orders = (order_t*)realloc(e->orders, sizeof(order_t) * e->orders_cap);
  }
  e->orders[n] = *ord;
}

/* step, multi_env.py:253-366 for one env */
static void step_env(const orc_env* o, env_t* e, int64_t ei, const float* act, float* obs, double* rew,
                     uint8_t* trunc, float* final_obs, const msc_step_info* info) {
  const int W = o->W, K = o->K, R = o->R, WK = W * K;
  const msc_env_desc* d = &o->d;
#define INFO(field, idx) (info && info->field ? &info->field[idx] : NULL)
  if (info) {
    if (info->inventory_before)
      for (int i = 0; i < WK; i++) info->inventory_before[ei * WK + i] = (int32_t)e->inv[i];
    if (info->pending_total)
      for (int i = 0; i < WK; i++) {
        float p = 0.0f;
        for (int j = 0; j < e->pend_n[i]; j++) p += (float)e->pend[(size_t)i * o->pend_cap + j].q;
        info->pending_total[ei * WK + i] = (int32_t)p;
      }
  }
  /* 1. _rescale_actions_to_quantities (multi_env.py:795-848) */
  double oq[MSC_MAX_W * MSC_MAX_K];
  for (int w = 0; w < W; w++)
    for (int s = 0; s < K; s++) {
      float a = act[w * K + s];
      double q;
      if (d->action_type == MSC_ACTION_DIRECT) {
        double scaled = (double)((a + 1.0f) / 2.0f) * o->act_param[s];
        q = rint(scaled);
        if (q < 0) q = 0;
        if (q > o->act_param[s]) q = o->act_param[s];
      } else if (d->action_type == MSC_ACTION_DEMAND_CENTERED) {
        double adj = rint(o->act_param[s] * (double)a);
        double dem = (double)(int64_t)e->inc_home[w * K + s];
        q = adj + dem;
        if (q < 0) q = 0;
      } else {
        double target = (double)((a + 1.0f) / 2.0f) * o->act_param[s];
        float pend = 0.0f;
        for (int j = 0; j < e->pend_n[w * K + s]; j++) pend += (float)e->pend[(size_t)(w * K + s) * o->pend_cap + j].q;
        double v = rint((target - (double)e->inc_home[w * K + s]) - (double)pend);
        q = v > 0 ? v : 0;
      }
      oq[w * K + s] = q;
    }
  /* 2. _apply_orders (multi_env.py:850-901) with lead_time_sampler.sample() drawn every step */
  int32_t lact[MSC_MAX_W * MSC_MAX_K];
  if (d->lead_type == MSC_LEAD_STOCHASTIC) {
    int32_t dev[MSC_MAX_W * MSC_MAX_K];
    if (d->max_dev_per_sku) { /* np.column_stack of per-SKU draws: SKU-major order */
      for (int s = 0; s < K; s++)
        for (int w = 0; w < W; w++) dev[w * K + s] = (int32_t)np_integers(&e->rl, -o->maxdev[s], (int64_t)o->maxdev[s] + 1);
    } else {
      for (int i = 0; i < WK; i++) dev[i] = (int32_t)np_integers(&e->rl, -o->maxdev[0], (int64_t)o->maxdev[0] + 1);
    }
    for (int i = 0; i < WK; i++) lact[i] = o->elt[i] + dev[i] > 1 ? o->elt[i] + dev[i] : 1;
  } else {
    for (int i = 0; i < WK; i++) lact[i] = o->elt[i];
  }
  double ordered[MSC_MAX_W * MSC_MAX_K];
  for (int i = 0; i < WK; i++) {
    ordered[i] = oq[i] > 0 ? oq[i] : 0.0;
    if (oq[i] > 0) {
      pend_t* p = &e->pend[(size_t)i * o->pend_cap + e->pend_n[i]++];
      p->q = oq[i];
      p->act = e->t + lact[i];
      p->exp = e->t + o->elt[i];
    }
  }
  if (info && info->order_quantities)
    for (int i = 0; i < WK; i++) info->order_quantities[ei * WK + i] = (int32_t)ordered[i];
  /* 3. _apply_arrivals (multi_env.py:903-919) */
  for (int i = 0; i < WK; i++) {
    pend_t* q = &e->pend[(size_t)i * o->pend_cap];
    int m = 0;
    for (int j = 0; j < e->pend_n[i]; j++) {
      if (q[j].act == e->t) e->inv[i] += q[j].q;
      else q[m++] = q[j];
    }
    e->pend_n[i] = m;
  }
  /* 4. demand_sampler.sample(t) */
  int n_orders = 0;
  order_t ord;
  if (d->demand_type == MSC_DEMAND_POISSON) { /* demand_sampler.py:105-163 */
    for (int r = 0; r < R; r++) {
      int64_t n = np_poisson(&e->rd, o->lo[r], o->enlam_o[r]);
      for (int64_t k = 0; k < n; k++) {
        int sel[MSC_MAX_K], ns = 0;
        for (int s = 0; s < K; s++)
          if (pcg_double(&e->rd) < o->ps[r]) sel[ns++] = s;
        ord.region = r;
        for (int s = 0; s < K; s++) ord.d[s] = 0.0;
        for (int j = 0; j < ns; j++) {
          int64_t q = np_poisson(&e->rd, o->lq[r * K + sel[j]], o->enlam_q[r * K + sel[j]]);
          ord.d[sel[j]] = (double)(q > 1 ? q : 1);
        }
        push_order(e, n_orders++, &ord);
      }
    }
  } else { /* demand_sampler.py:214-261 */
    if (e->emp_start < 0) e->emp_start = np_integers(&e->rd, 0, (int64_t)(d->trace_n_rows - d->episode_length) + 1);
    int64_t row = e->emp_start + (e->t % d->episode_length);
    for (int64_t i = o->tr_off[row]; i < o->tr_off[row + 1]; i++) {
      ord.region = o->tr_reg[i];
      for (int s = 0; s < K; s++) ord.d[s] = (double)o->tr_q[i * K + s];
      push_order(e, n_orders++, &ord);
    }
  }
  /* 5. GreedyDemandAllocator.allocate (demand_allocator.py:118-217) */
  static __thread double ship_q[MSC_MAX_W * MSC_MAX_R];
  static __thread int32_t ship_n[MSC_MAX_W * MSC_MAX_R];
  static __thread double unf[MSC_MAX_R * MSC_MAX_K];
  static __thread int32_t lost_n[MSC_MAX_R];
  static __thread double qbys[MSC_MAX_W * MSC_MAX_R * MSC_MAX_K];
  memset(ship_q, 0, sizeof(double) * W * R);
  memset(ship_n, 0, sizeof(int32_t) * W * R);
  memset(unf, 0, sizeof(double) * R * K);
  memset(lost_n, 0, sizeof(int32_t) * R);
  memset(qbys, 0, sizeof(double) * W * R * K);
  double fulfilled[MSC_MAX_W * MSC_MAX_K];
  memset(fulfilled, 0, sizeof fulfilled);
  int maxwh = d->max_splits + 1;
  for (int oi = 0; oi < n_orders; oi++) {
    const order_t* od = &e->orders[oi];
    int r = od->region;
    double tw = 0.0;
    for (int s = 0; s < K; s++) tw += od->d[s] * o->skw[s];
    double c[MSC_MAX_W];
    int idx[MSC_MAX_W];
    for (int w = 0; w < W; w++) {
      c[w] = o->of[w * R + r] + o->ov[w * R + r] * tw;
      idx[w] = w;
    }
    for (int i = 1; i < W; i++) { /* stable insertion sort == argsort for tie-free costs */
      int v = idx[i], j = i;
      while (j > 0 && c[idx[j - 1]] > c[v]) { idx[j] = idx[j - 1]; j--; }
      idx[j] = v;
    }
    double rem[MSC_MAX_K];
    for (int s = 0; s < K; s++) rem[s] = od->d[s];
    int used = 0;
    for (int k = 0; k < W; k++) {
      if (used >= maxwh) break;
      int w = idx[k];
      double f[MSC_MAX_K];
      int any = 0;
      for (int s = 0; s < K; s++) {
        f[s] = rem[s] < e->inv[w * K + s] ? rem[s] : e->inv[w * K + s];
        any |= f[s] > 0;
      }
      if (any) {
        ship_n[w * R + r] += 1;
        double fs = 0.0;
        for (int s = 0; s < K; s++) fs += f[s];
        ship_q[w * R + r] += fs;
        int all_done = 1;
        for (int s = 0; s < K; s++) {
          qbys[(w * R + r) * K + s] += f[s];
          fulfilled[w * K + s] += f[s];
          rem[s] -= f[s];
          e->inv[w * K + s] -= f[s];
          all_done &= rem[s] <= 0;
        }
        used++;
        if (all_done) break;
      }
    }
    int anyrem = 0;
    for (int s = 0; s < K; s++) anyrem |= rem[s] > 0;
    if (anyrem) {
      for (int s = 0; s < K; s++) unf[r * K + s] += rem[s];
      lost_n[r] += 1;
    }
  }
  /* 6. inventory = max(inventory - fulfilled, 0): the allocator's working copy (never < 0) */
  /* 7. _update_observations (multi_env.py:747-793) */
  static __thread float dpr[MSC_MAX_R * MSC_MAX_K];
  memset(dpr, 0, sizeof(float) * R * K);
  for (int oi = 0; oi < n_orders; oi++)
    for (int s = 0; s < K; s++) dpr[e->orders[oi].region * K + s] = (float)((double)dpr[e->orders[oi].region * K + s] + e->orders[oi].d[s]);
  for (int w = 0; w < W; w++)
    for (int s = 0; s < K; s++) {
      int i = w * K + s, hr = o->home[w];
      e->inc_home[i] = dpr[hr * K + s];
      e->ship_home[i] = qbys[(w * R + hr) * K + s];
      double tot = 0.0;
      for (int r = 0; r < R; r++) tot += qbys[(w * R + r) * K + s];
      e->ship_away[i] = tot - e->ship_home[i];
      double so = (double)e->inc_home[i] - e->ship_home[i];
      e->stockout[i] = (float)(so > 0.0 ? so : 0.0);
    }
  if (e->hist_n < MSC_HISTORY) {
    memcpy(&e->hist[((e->hist_head + e->hist_n) % MSC_HISTORY) * WK], e->inc_home, sizeof(float) * WK);
    e->hist_n++;
  } else {
    memcpy(&e->hist[e->hist_head * WK], e->inc_home, sizeof(float) * WK);
    e->hist_head = (e->hist_head + 1) % MSC_HISTORY;
  }
  for (int i = 0; i < WK; i++) {
    float sum = 0.0f;
    for (int h = 0; h < e->hist_n; h++) sum += e->hist[((e->hist_head + h) % MSC_HISTORY) * WK + i];
    e->roll_mean[i] = sum / (float)e->hist_n;
    e->forecast[i] = (float)0.3 * e->inc_home[i] + (float)(1.0 - 0.3) * e->forecast[i];
  }
  /* 8. lost_sales_handler.calculate_lost_sales (lost_sales_handler.py:71-210) */
  double lost[MSC_MAX_W * MSC_MAX_K];
  memset(lost, 0, sizeof lost);
  for (int r = 0; r < R; r++) {
    if (d->lost_type == MSC_LOST_CLOSEST) {
      for (int s = 0; s < K; s++) lost[o->closest[r] * K + s] += unf[r * K + s];
    } else if (d->lost_type == MSC_LOST_SHIPMENT) {
      double tot = np_sum_f64(&ship_q[r], W, R);
      double wts[MSC_MAX_W];
      for (int w = 0; w < W; w++) wts[w] = tot > 0 ? ship_q[w * R + r] / tot : (w == o->closest[r] ? 1.0 : 0.0);
      for (int s = 0; s < K; s++)
        for (int w = 0; w < W; w++) lost[w * K + s] += wts[w] * unf[r * K + s];
    } else {
      double lo_n = (double)lost_n[r], lw = 0.0;
      for (int s = 0; s < K; s++) lw += unf[r * K + s] * o->skw[s];
      double lg[MSC_MAX_W], mx = -INFINITY, se = 0.0;
      for (int w = 0; w < W; w++) {
        lg[w] = -(o->of[w * R + r] * lo_n + o->ov[w * R + r] * lw) / d->lost_alpha;
        if (lg[w] > mx) mx = lg[w];
      }
      for (int w = 0; w < W; w++) { lg[w] = exp(lg[w] - mx); se += lg[w]; }
      for (int w = 0; w < W; w++)
        for (int s = 0; s < K; s++) lost[w * K + s] += (lg[w] / se) * unf[r * K + s];
    }
  }
  /* 9. CostRewardCalculator.calculate (reward_calculator.py:96-190) */
  double cost[4][MSC_MAX_W], rw[MSC_MAX_W];
  for (int w = 0; w < W; w++) {
    double t1[MSC_MAX_K], t2[MSC_MAX_K], t3[MSC_MAX_K], t4[MSC_MAX_K];
    for (int s = 0; s < K; s++) {
      int i = w * K + s;
      t1[s] = d->holding_per_sku ? e->inv[i] * o->hold[s] : (e->inv[i] * o->skw[s]) * o->hold[0];
      t2[s] = d->penalty_per_sku ? lost[i] * o->pen[s] : (lost[i] * o->skw[s]) * o->pen[0];
      t3[s] = (double)(ordered[i] > 0) * o->inf[i];
      t4[s] = (ordered[i] * o->skw[s]) * o->inv_var[i];
    }
    static __thread double of_r[MSC_MAX_R], ov_r[MSC_MAX_R];
    for (int r = 0; r < R; r++) {
      double wsum[MSC_MAX_K];
      for (int s = 0; s < K; s++) wsum[s] = qbys[(w * R + r) * K + s] * o->skw[s];
      of_r[r] = (double)ship_n[w * R + r] * o->of[w * R + r];
      ov_r[r] = np_sum_f64(wsum, K, 1) * o->ov[w * R + r];
    }
    cost[0][w] = np_sum_f64(t1, K, 1);
    cost[1][w] = np_sum_f64(t2, K, 1);
    cost[2][w] = np_sum_f64(of_r, R, 1) + np_sum_f64(ov_r, R, 1);
    cost[3][w] = np_sum_f64(t3, K, 1) + np_sum_f64(t4, K, 1);
    double tot = ((cost[0][w] + cost[1][w]) + cost[2][w]) + cost[3][w];
    rw[w] = -(tot * d->reward_scale);
  }
  if (d->reward_scope == MSC_SCOPE_TEAM) {
    double s = np_sum_f64(rw, W, 1);
    for (int w = 0; w < W; w++) rw[w] = s;
  }
  for (int w = 0; w < W; w++) rew[w] = rw[w];
  if (info) {
    if (info->demand_per_region)
      for (int i = 0; i < R * K; i++) info->demand_per_region[ei * R * K + i] = (int32_t)dpr[i];
    if (info->fulfilled_per_warehouse)
      for (int i = 0; i < WK; i++) info->fulfilled_per_warehouse[ei * WK + i] = (int32_t)fulfilled[i];
    if (info->unfulfilled_demands)
      for (int i = 0; i < R * K; i++) info->unfulfilled_demands[ei * R * K + i] = (int32_t)unf[i];
    if (info->shipment_counts)
      for (int i = 0; i < W * R; i++) info->shipment_counts[ei * W * R + i] = ship_n[i];
    if (info->shipment_quantities)
      for (int i = 0; i < W * R; i++) info->shipment_quantities[ei * W * R + i] = (int32_t)ship_q[i];
    if (info->shipment_quantities_by_sku)
      for (int i = 0; i < W * R * K; i++) info->shipment_quantities_by_sku[ei * W * R * K + i] = (int32_t)qbys[i];
    if (info->lost_order_counts)
      for (int i = 0; i < R; i++) info->lost_order_counts[ei * R + i] = lost_n[i];
    if (info->n_orders) info->n_orders[ei] = n_orders;
    if (info->lost_sales)
      for (int i = 0; i < WK; i++) info->lost_sales[ei * WK + i] = lost[i];
    if (info->costs)
      for (int c = 0; c < 4; c++)
        for (int w = 0; w < W; w++) info->costs[(ei * 4 + c) * W + w] = cost[c][w];
  }
  /* 10. observations, then timestep += 1 and truncation (multi_env.py:322-327) */
  get_obs(o, e, obs);
  e->t += 1;
  int tr = e->t >= d->episode_length;
  *trunc = (uint8_t)tr;
  if (tr) {
    if (final_obs) memcpy(final_obs, obs, sizeof(float) * W * o->L);
    reset_env(o, e, NULL, 0);
    get_obs(o, e, obs);
  }
#undef INFO
}

void orc_step(orc_env* o, const float* actions, float* obs, double* rewards, uint8_t* trunc, float* final_obs,
              const msc_step_info* info, int32_t n_threads) {
  const size_t WK = (size_t)o->W * o->K, WL = (size_t)o->W * o->L;
  (void)n_threads;
#pragma omp parallel for schedule(static) num_threads(n_threads > 0 ? n_threads : 1)
  for (int64_t i = 0; i < o->E; i++)
    step_env(o, &o->envs[i], i, actions + WK * i, obs + WL * i, rewards + (size_t)o->W * i, trunc + i,
             final_obs ? final_obs + WL * i : NULL, info);
}

void orc_read_state(const orc_env* o, int32_t* inv, int32_t* ts, int32_t* ep, uint64_t* rng) {
  const int WK = o->W * o->K;
  for (int64_t i = 0; i < o->E; i++) {
    const env_t* e = &o->envs[i];
    if (inv)
      for (int j = 0; j < WK; j++) inv[i * WK + j] = (int32_t)e->inv[j];
    if (ts) ts[i] = e->t;
    if (ep) ep[i] = e->counter;
    if (rng) {
      rng_export(&e->rd, &rng[i * 12]);
      rng_export(&e->rl, &rng[i * 12 + 6]);
    }
  }
}
