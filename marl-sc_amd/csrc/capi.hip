// capi.hip -- the extern "C" boundary of libmarlsc.so (include/marlsc.h).
//
// Host responsibilities only: validate the descriptor (the reference's EnvironmentConfig shape
// rules, src/config/schema.py:664-890), precompute the read-only tables (home regions
// multi_env.py:144, closest warehouses lost_sales_handler.py:36, exp(-lambda) with the host libm
// exactly as numpy's random_poisson does, transposed outbound costs), derive per-env root seeds
// (SeedManager.derive_env_seed, seed_manager.py:165-186), own the HBM arenas and launch the
// kernels of env_kernels.hip / gae.hip on the caller's stream.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../include/marlsc.h"
#include "env.hpp"
#include "rng.hpp"

using namespace msc;

static thread_local char g_err[512] = "";

static int set_err(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
  return code;
}
#define HIP_TRY(x)                                                                   \
  do {                                                                               \
    hipError_t _e = (x);                                                             \
    if (_e != hipSuccess) return set_err(-2, "%s: %s", #x, hipGetErrorString(_e));   \
  } while (0)

struct msc_env {
  EnvConst c;
  EnvState s;
  int device;
  void* tables = nullptr;   // device copy of every static table
  void* arena = nullptr;    // persistent per-env state (checkpointed by save/load_state)
  size_t arena_bytes = 0;
  void* scratch = nullptr;    // two per-step order buffers (double-buffered for pipelining)
  size_t order_bytes = 0;     // bytes of one order buffer (records + counts)
  DevEnv* dev = nullptr;      // device copies of {c, s}: dev[b] points at order buffer b
  // Demand pipelining: the Poisson demand of step tau+1 depends only on each env's own demand
  // stream, so it is generated on a side stream while the step kernel of tau runs (their waves
  // co-reside on the CUs), unless step tau ends an episode (the in-kernel reset re-seeds the
  // demand stream) or the envs' timesteps are out of sync after a masked reset.
  hipStream_t side = nullptr;
  hipEvent_t ev_dem[2] = {nullptr, nullptr}, ev_step[2] = {nullptr, nullptr}, ev_reset = nullptr;
  // the stream each ev_dem was last recorded on (a wait from that same stream is already ordered),
  // and whether the side stream has waited on the latest ev_reset (a reset is recorded once)
  hipStream_t ev_dem_on[2] = {nullptr, nullptr};
  bool side_saw_reset = false;
  bool ev_elide = true;  // MSC_EV_ELIDE=0: every wait is issued (A/B)
  int64_t tau = 0;                // steps issued
  int t_sync = -1;                 // common timestep of every env, -1 if unknown
  bool ready[2] = {false, false};  // order buffer b holds the demand of the next step using it
  bool pipeline = true;
  // msc_env_set_timing: event pairs around demand / step launches (2 per launch)
  std::vector<hipEvent_t> tev_dem, tev_step;
  int t_cap = 0, n_tdem = 0, n_tstep = 0;
  // Episode-ahead demand (EA; few envs per GPU). A Poisson episode's orders
  // depend only on its seed (SeedSequence([root, counter]), seed_manager.py:100-120), not on
  // actions, so whole future episodes are generated on side streams while earlier ones step: slot
  // n % S holds episode n (counted from the snapshot taken when EA started, episode 0 = the one
  // running then, which keeps the per-step path). At the end of episode n its slot is refilled
  // with episode n + S. Any desynchronising event (masked reset, load_state, disabling) stops it;
  // it restarts at the next common episode start.
  int64_t ea_budget = 0, ea_bytes = 0;  // episode-ahead memory budget and bytes allocated (create time)
  bool ea_enabled = false;  // configured: Poisson demand, few envs (or MSC_EA=1), buffers allocated
  bool ea_paused = false;   // msc_env_set_episode_ahead(0): per-step demand until re-enabled
  int32_t obs_stage_pe = 0, chain_prio_pe = 0;  // step_c staging / chain priority of the per-step path
  bool ea_running = false;
  int64_t ea_n = 0;         // episode (relative to the snapshot) the envs are in
  int ea_cur = -1;          // slot of the current episode, -1: per-step demand
  void* ea_mem = nullptr;
  // One launch is a chain of T per-step parses (~60 ms at 8 x 64 x 5) whatever its lane count,
  // while the envs consume an episode in T steps: freed slots are refilled ea_batch at a time, in
  // one launch of ea_batch x E lanes on one stream (separate streams would share the process's few
  // hardware queues and serialise anyway).
  hipStream_t ea_stream = nullptr;
  int ea_batch = 1;         // slots per refill launch
  int ea_freed = 0;         // consumed slots not yet refilled
  // A generation runs as chunks of ea_chunk steps, each launched once the previous one has finished
  // (polled at every step call; flushed when a step needs the slot), so that the EA work queued on
  // the device at any time -- what a device-wide synchronize waits for -- is one short chunk.
  int ea_chunk = 50;
  struct EaItem { EaLaunch l; int wait_cons; };  // wait_cons: slot whose ev_cons precedes chunk 0 (-1: none)
  std::vector<EaItem> ea_q;  // generations not yet fully launched (head: the one in progress)
  bool ea_chunk_out = false; // a chunk of the head item is in flight (ev_chunk)
  hipEvent_t ev_chunk = nullptr;
  bool gen_pending[MSC_EA_MAX_S] = {};  // slot's generation not fully launched (ev_gen stale)
  hipEvent_t ev_gen[MSC_EA_MAX_S] = {}, ev_cons[MSC_EA_MAX_S] = {}, ev_snap = nullptr;
  std::vector<hipEvent_t> tev_ea;  // timing of EA launches (msc_env_set_timing)
  std::vector<double> tea_work;    // env-steps generated by each timed EA launch
  // demand work issued since create (msc_env_work_counters): episode-ahead generation launches
  // (chunks) and the env-steps of demand they draw; per-step demand launches (E env-steps each); steps
  int64_t cnt_ea_launch = 0, cnt_dem_launch = 0, cnt_steps = 0;
  double cnt_ea_work = 0.0;
  int n_tea = 0;
};

static void timing_free(msc_env* env) {
  for (hipEvent_t e : env->tev_dem) (void)hipEventDestroy(e);
  for (hipEvent_t e : env->tev_step) (void)hipEventDestroy(e);
  for (hipEvent_t e : env->tev_ea) (void)hipEventDestroy(e);
  env->tev_dem.clear();
  env->tev_step.clear();
  env->tev_ea.clear();
  env->t_cap = env->n_tdem = env->n_tstep = env->n_tea = 0;
}
// record event `i` (0 = before, 1 = after) of launch n of `v` on `st`, if timing is on
static hipError_t tmark(const msc_env* env, const std::vector<hipEvent_t>& v, int n, int i, hipStream_t st) {
  return n < env->t_cap ? hipEventRecord(v[2 * n + i], st) : hipSuccess;
}

// ---- episode-ahead demand (see msc_env) ----------------------------------------------------
// the EA stream waits for the work queued on `st` so far
static int ea_stream_wait(msc_env* env, hipStream_t st) {
  HIP_TRY(hipEventRecord(env->ev_snap, st));
  HIP_TRY(hipStreamWaitEvent(env->ea_stream, env->ev_snap, 0));
  return 0;
}
// `st` waits for the EA stream's work so far
static int wait_ea_stream(msc_env* env, hipStream_t st) {
  HIP_TRY(hipEventRecord(env->ev_snap, env->ea_stream));
  HIP_TRY(hipStreamWaitEvent(st, env->ev_snap, 0));
  return 0;
}
// one chunk [l.t0, l.t1) of a generation on the EA stream; after the last chunk the slots' ev_gen
static hipError_t ea_launch_chunk(msc_env* env, const EaLaunch& l) {
  hipStream_t es = env->ea_stream;
  const bool tm = env->n_tea < env->t_cap;
  if (tm) {
    (void)hipEventRecord(env->tev_ea[2 * env->n_tea], es);
    if ((int)env->tea_work.size() <= env->n_tea) env->tea_work.resize(env->n_tea + 1);
    env->tea_work[env->n_tea] = (double)l.nslots * (double)(l.t1 - l.t0) * (double)env->c.E;
  }
  hipError_t e = launch_demand_ea(env->c, env->dev, l, es);
  if (e != hipSuccess) return e;
  env->cnt_ea_launch++;
  env->cnt_ea_work += (double)l.nslots * (double)(l.t1 - l.t0) * (double)env->c.E;
  if (tm) (void)hipEventRecord(env->tev_ea[2 * env->n_tea++ + 1], es);
  if (l.t1 >= env->c.T) {
    for (int k = 0; k < l.nslots; k++) {
      const int slot = (l.slot0 + k) % env->c.ea_S;
      e = hipEventRecord(env->ev_gen[slot], es);
      if (e != hipSuccess) return e;
      env->gen_pending[slot] = false;
    }
  }
  return hipEventRecord(env->ev_chunk, es);
}
// launch the next chunk of the head generation if none is in flight (block: even if one is)
static hipError_t ea_pump(msc_env* env, bool block) {
  if (env->ea_q.empty()) return hipSuccess;
  if (env->ea_chunk_out && !block) {
    const hipError_t q = hipEventQuery(env->ev_chunk);
    if (q == hipErrorNotReady) return hipSuccess;
    if (q != hipSuccess) return q;
  }
  msc_env::EaItem& it = env->ea_q.front();
  EaLaunch& l = it.l;
  if (it.wait_cons >= 0) {  // a refill: after the step that read the slots' previous episodes
    const hipError_t w = hipStreamWaitEvent(env->ea_stream, env->ev_cons[it.wait_cons], 0);
    if (w != hipSuccess) return w;
    it.wait_cons = -1;
  }
  EaLaunch cl = l;
  cl.t1 = l.t0 + env->ea_chunk < env->c.T ? l.t0 + env->ea_chunk : env->c.T;
  const hipError_t e = ea_launch_chunk(env, cl);
  if (e != hipSuccess) return e;
  env->ea_chunk_out = true;
  l.t0 = cl.t1;
  if (l.t0 >= env->c.T) env->ea_q.erase(env->ea_q.begin());
  return hipSuccess;
}
// queue a generation (slots slot0 .. slot0 + nslots - 1, see EaLaunch)
static hipError_t ea_enqueue(msc_env* env, int slot0, int nslots, int from_slot, int iters0, int iters_step,
                             int wait_cons = -1) {
  env->ea_q.push_back({EaLaunch{slot0, nslots, from_slot, iters0, iters_step, 0, env->c.T}, wait_cons});
  for (int k = 0; k < nslots; k++) env->gen_pending[(slot0 + k) % env->c.ea_S] = true;
  return ea_pump(env, false);
}
// every chunk up to the generation of `slot` launched (its ev_gen is then current)
static hipError_t ea_flush_to(msc_env* env, int slot) {
  while (env->gen_pending[slot]) {
    if (env->ea_q.empty()) return hipErrorInvalidValue;  // (unreachable: pending slots are queued)
    const hipError_t e = ea_pump(env, true);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}
// Snapshot at a common episode start (t_sync == 0, after the reset): the SeedManager counter of
// the current episode -> slot 0's counter; episodes 1 .. S-1 follow from it, 1 .. B first (the
// envs need episode 1 when the per-step episode 0 ends), then B+1 .. S-1.
static int ea_start(msc_env* env, hipStream_t st) {
  const int S = env->c.ea_S, B = env->ea_batch;
  if (const int rc = wait_ea_stream(env, st)) return rc;  // EA work of an earlier run still reads ea_cnt
  HIP_TRY(hipMemcpyAsync(env->s.ea_cnt, env->s.counter, sizeof(int32_t) * env->c.E, hipMemcpyDeviceToDevice, st));
  if (const int rc = ea_stream_wait(env, st)) return rc;
  const int first = B < S - 1 ? B : S - 1;
  env->ea_q.clear();
  env->ea_chunk_out = false;
  for (int j = 0; j < S; j++) env->gen_pending[j] = false;
  HIP_TRY(ea_enqueue(env, 1, first, 0, 1, 1));
  if (first < S - 1) HIP_TRY(ea_enqueue(env, 1 + first, S - 1 - first, 0, 1 + first, 1));
  env->ea_freed = 0;
  env->ea_running = true;
  env->ea_n = 0;
  env->ea_cur = -1;
  return 0;
}
// The demand stream of the current EA episode into s.rng[0] (what the per-step path and
// read_state / save_state use), stream-ordered on st.
static int ea_materialize(const msc_env* env, hipStream_t st) {
  if (env->ea_running && env->ea_cur >= 0 && env->t_sync > 0)
    HIP_TRY(launch_ea_materialize(env->c, env->dev, env->ea_cur, env->t_sync, st));
  return 0;
}
static int ea_stop(msc_env* env, hipStream_t st, bool materialize) {
  if (!env->ea_running) return 0;
  if (materialize) {
    const int rc = ea_materialize(env, st);
    if (rc) return rc;
  }
  env->ea_running = false;
  env->ea_cur = -1;
  env->ea_q.clear();  // generations not launched yet are dropped (chunks in flight finish on the EA stream)
  for (int j = 0; j < MSC_EA_MAX_S; j++) env->gen_pending[j] = false;
  return 0;
}

extern "C" {

const char* msc_last_error(void) { return g_err; }
int msc_abi_version(void) { return MSC_ABI_VERSION; }

uint32_t msc_seedseq_u32(const uint32_t* words, int32_t n) { return ss_u32(words, n); }

static int feature_dim(const msc_env_desc* d, int Lmax) {
  const uint32_t f = d->feature_flags;
  const int K = d->n_skus;
  int n = 0;
  if (f & MSC_F_INVENTORY) n += K + ((f & MSC_F_INVENTORY_AGG) ? 1 : 0);
  if (f & MSC_F_PIPELINE) n += Lmax * K + ((f & MSC_F_PIPELINE_AGG) ? 1 : 0);
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

// Packs host vectors into one device allocation; returns device pointers by offset.
struct TablePack {
  std::vector<char> host;
  size_t add(const void* p, size_t bytes) {
    size_t off = (host.size() + 15) & ~size_t(15);
    host.resize(off + bytes);
    if (bytes) memcpy(host.data() + off, p, bytes);
    return off;
  }
};

int msc_env_create(const msc_env_desc* d, int device, int64_t n_envs, uint32_t base_seed, uint32_t worker_index,
                   int64_t env_index_offset, const uint32_t* env_seeds_host, msc_env** out) {
  if (!d || !out) return set_err(-1, "null argument");
  *out = nullptr;
  if (d->abi_version != MSC_ABI_VERSION) return set_err(-1, "abi_version %d != %d", d->abi_version, MSC_ABI_VERSION);
  const int W = d->n_warehouses, K = d->n_skus, R = d->n_regions;
  if (W < 1 || W > MSC_MAX_W) return set_err(-1, "n_warehouses must be in [1, %d]", MSC_MAX_W);
  if (K < 1 || K > MSC_MAX_K) return set_err(-1, "n_skus must be in [1, %d]", MSC_MAX_K);
  if (R < 1 || R > MSC_MAX_R) return set_err(-1, "n_regions must be in [1, %d]", MSC_MAX_R);
  if (d->episode_length < 1) return set_err(-1, "episode_length must be positive");
  if (n_envs < 1) return set_err(-1, "n_envs must be positive");
  if (d->max_splits < 0 || d->max_splits >= W) return set_err(-1, "max_splits must be < n_warehouses=%d", W);
  const int WK = W * K;

  // lead times -> pipeline horizon and pending ring size
  int Lmax = 0, lact_max = 0;
  for (int i = 0; i < WK; i++) {
    const int elt = d->expected_lead_times[i];
    if (elt < 1) return set_err(-1, "expected_lead_times must be positive");
    int dev = 0;
    if (d->lead_type == MSC_LEAD_STOCHASTIC) dev = d->max_dev_per_sku ? d->max_deviation[i % K] : d->max_deviation[0];
    if (dev < 0) return set_err(-1, "max_deviation must be non-negative");
    Lmax = elt > Lmax ? elt : Lmax;
    lact_max = elt + dev > lact_max ? elt + dev : lact_max;
  }
  const int RING = lact_max + 1;
  if (RING > MAX_RING) return set_err(-1, "max actual lead time %d exceeds %d", lact_max, MAX_RING - 1);

  EnvConst c{};
  c.W = W; c.K = K; c.R = R; c.T = d->episode_length; c.Lmax = Lmax; c.RING = RING;
  c.F = feature_dim(d, Lmax);
  c.L = c.F + (d->include_warehouse_id ? W : 0);
  c.action_type = d->action_type; c.lead_type = d->lead_type; c.dev_per_sku = d->max_dev_per_sku;
  c.lost_type = d->lost_type; c.scope = d->reward_scope; c.norm = d->obs_norm; c.wid = d->include_warehouse_id;
  c.num_eval = d->num_eval_episodes; c.max_wh = d->max_splits + 1; c.demand_type = d->demand_type;
  c.init_type = d->init_type; c.init_min = d->init_min; c.init_max = d->init_max;
  c.hold_per_sku = d->holding_per_sku; c.pen_per_sku = d->penalty_per_sku;
  c.flags = d->feature_flags; c.E = n_envs; c.scale = d->reward_scale; c.alpha = d->lost_alpha;
  c.hold_scalar = d->holding_per_sku ? 0.0 : d->holding_cost[0];
  c.pen_scalar = d->penalty_per_sku ? 0.0 : d->penalty_cost[0];
  if (c.lost_type == MSC_LOST_COST && !(c.alpha > 0)) return set_err(-1, "cost lost-sales alpha must be > 0");
  if (c.norm == MSC_OBS_MEANSTD && (!d->obs_mean || !d->obs_std)) return set_err(-1, "meanstd needs obs_mean/obs_std");
  if (d->init_type == MSC_INIT_UNIFORM && (d->init_min < 0 || d->init_min > d->init_max))
    return set_err(-1, "uniform initial inventory needs 0 <= min <= max");

  // ---- static tables ---------------------------------------------------------------------
  std::vector<double> zeros_k(K, 0.0), hold(K), pen(K), ofT((size_t)R * W), ovT((size_t)R * W);
  for (int s = 0; s < K; s++) {
    hold[s] = d->holding_per_sku ? d->holding_cost[s] : 0.0;
    pen[s] = d->penalty_per_sku ? d->penalty_cost[s] : 0.0;
  }
  for (int w = 0; w < W; w++)
    for (int r = 0; r < R; r++) {
      ofT[(size_t)r * W + w] = d->outbound_fixed[(size_t)w * R + r];
      ovT[(size_t)r * W + w] = d->outbound_variable[(size_t)w * R + r];
    }
  std::vector<uint32_t> home_mask(R, 0u);
  std::vector<int32_t> closest(R, 0), home_of(W, 0);
  for (int w = 0; w < W; w++) {  // argmin over regions (first minimum), multi_env.py:144
    int b = 0;
    for (int r = 1; r < R; r++)
      if (d->distances[(size_t)w * R + r] < d->distances[(size_t)w * R + b]) b = r;
    home_mask[b] |= 1u << w;
    home_of[w] = b;
  }
  c.shared_home = 0;
  for (int r = 0; r < R; r++) c.shared_home |= __builtin_popcount(home_mask[r]) > 1 ? 1 : 0;
  for (int r = 0; r < R; r++) {  // argmin over warehouses, lost_sales_handler.py:36
    int b = 0;
    for (int w = 1; w < W; w++)
      if (d->distances[(size_t)w * R + r] < d->distances[(size_t)b * R + r]) b = w;
    closest[r] = b;
  }
  std::vector<double> enlam_o(R, 1.0), p_sku(R, 0.0), p_skip(R, 0.0), enlam_q((size_t)R * K, 1.0);
  std::vector<PtrsConst> ptrs_o(R), ptrs_q((size_t)R * K);
  int order_cap = 1;
  int nv = order_record_vec4(K);
  std::vector<uint4> trec;
  std::vector<int64_t> toff;
  if (d->demand_type == MSC_DEMAND_POISSON) {
    double lam_sum = 0.0;
    for (int r = 0; r < R; r++) {
      const double lo = d->lambda_orders[r];
      // PositiveFloat in the reference schema (schema.py:191); >= 10 is numpy's PTRS branch
      if (!(lo > 0.0 && lo < 1e6)) return set_err(-1, "lambda_orders[%d]=%g: must be in (0, 1e6)", r, lo);
      enlam_o[r] = exp(-lo);
      ptrs_o[r] = ptrs_const_host(lo);
      if (lo >= 10.0) c.demand_ptrs = 1;
      if (lo > 0.0 && lo < 10.0 && enlam_o[r] >= 1.0) return set_err(-1, "lambda_orders[%d] too small", r);
      p_sku[r] = d->probability_skus[r];
      // random() draws are multiples of 2^-53: U < p <=> U < ceil53(p) <=> !(U > ceil53(p) - 2^-53)
      p_skip[r] = ldexp(ceil(ldexp(p_sku[r], 53)), -53) - 0x1p-53;
      lam_sum += lo;
      for (int s = 0; s < K; s++) {
        const double lq = d->lambda_quantity[(size_t)r * K + s];
        // quantities are stored as 16-bit record fields: rates far below 2^16
        if (!(lq > 0.0 && lq < 20000.0)) return set_err(-1, "lambda_quantity[%d,%d]=%g: must be in (0, 20000)", r, s, lq);
        enlam_q[(size_t)r * K + s] = exp(-lq);
        ptrs_q[(size_t)r * K + s] = ptrs_const_host(lq);
        if (lq >= 10.0) c.demand_ptrs = 1;
      }
    }
    // record capacity per env and step in int64 first: the kernels index records with int32, so a
    // configuration whose per-step capacity does not fit is rejected here (rates up to 1e6 x 4,096
    // regions would otherwise wrap the cast)
    const double cap_d = ceil(lam_sum + 12.0 * sqrt(lam_sum + 1.0) + 64.0);
    if (!(cap_d <= (double)MSC_ORDER_CAP_MAX))
      return set_err(-1, "sum of lambda_orders %g: per-step order capacity %.0f exceeds %d records per env", lam_sum,
                     cap_d, MSC_ORDER_CAP_MAX);
    order_cap = (int)cap_d;
    // equal parameters in every region (and SKU): the demand parser's constant-threshold variant
    c.demand_uni = 1;
    for (int r = 0; r < R; r++) {
      c.demand_uni &= enlam_o[r] == enlam_o[0] && p_skip[r] == p_skip[0] ? 1 : 0;
      for (int s = 0; s < K; s++) c.demand_uni &= enlam_q[(size_t)r * K + s] == enlam_q[0] ? 1 : 0;
    }
    if (const char* du = getenv("MSC_DEMAND_UNI")) c.demand_uni &= atoi(du) != 0 ? 1 : 0;
    c.uni_thr_o = enlam_o[0];
    c.uni_thr_m = p_skip[0];
    c.uni_thr_q = enlam_q[0];
    // demand_v2_kernel (demand_v2.hip): its f32 chain decides "prod > exp(-lambda)" only outside a
    // band of relative width 2^-16 around the threshold (both bounds rounded outward to f32); the SKU
    // draw U = k 2^-53 < p <=> k < ceil(p 2^53), exact on the integer
    auto f_up = [](double v) { float f = (float)v; return (double)f < v ? nextafterf(f, INFINITY) : f; };
    auto f_dn = [](double v) { float f = (float)v; return (double)f > v ? nextafterf(f, -INFINITY) : f; };
    // (MSC_V2_BAND=b widens the band to 2^-b, b in [2, 16]: tests drive the exact recomputation with it)
    int band = 16;
    if (const char* vb = getenv("MSC_V2_BAND")) band = atoi(vb) >= 2 && atoi(vb) <= 16 ? atoi(vb) : band;
    const double bw = ldexp(1.0, -band);
    c.v2_thr[0] = f_up(enlam_o[0] * (1.0 + bw));
    c.v2_thr[1] = f_dn(enlam_o[0] * (1.0 - bw));
    c.v2_thr[2] = f_up(enlam_q[0] * (1.0 + bw));
    c.v2_thr[3] = f_dn(enlam_q[0] * (1.0 - bw));
    c.v2_k53 = (uint64_t)ceil(ldexp(p_sku[0] < 2.0 ? p_sku[0] : 2.0, 53));
  } else if (d->demand_type == MSC_DEMAND_EMPIRICAL) {
    const int rows = d->trace_n_rows;
    if (rows < d->episode_length) return set_err(-1, "trace has %d timesteps < episode_length %d", rows, d->episode_length);
    const int64_t n_ord = d->trace_offsets[rows];
    toff.assign(d->trace_offsets, d->trace_offsets + rows + 1);
    trec.assign((size_t)(n_ord > 0 ? n_ord : 1) * nv, make_uint4(0, 0, 0, 0));
    for (int64_t j = 0; j < n_ord; j++) {
      uint16_t* h = reinterpret_cast<uint16_t*>(&trec[(size_t)j * nv]);
      const int reg = d->trace_regions[j];
      if (reg < 0 || reg >= R) return set_err(-1, "trace region %d out of range", reg);
      h[0] = (uint16_t)reg;
      for (int s = 0; s < K; s++) {
        const int q = d->trace_quantities[j * K + s];
        if (q < 0 || q > 65535) return set_err(-1, "trace quantity %d out of range", q);
        h[1 + s] = (uint16_t)q;
      }
    }
    c.tr_rows = rows;
  } else {
    return set_err(-1, "unknown demand_type %d", d->demand_type);
  }
  c.order_cap = order_cap;
  {
    // A/B knobs (timing experiments only; results are identical)
    const char* impl = getenv("MSC_DEMAND_IMPL");
    // default (0): the unit-per-round parser; "ab" the split chain / bookkeeper parser
    // (demand_ab_kernel: measured slower), "park4" the round-1 parser
    // default (9): the short-round unit parser (demand_v3.hip) where the sampler's parameters are equal
    // in every region and SKU, the unit parser otherwise (0, "unit" forces it; C3 demand 0.787 -> 0.758
    // ms, C2 205 -> 208.7 M, profiles/r06/ab_demand_v3.txt)
    c.demand_impl = !impl ? 9 : strcmp(impl, "park4") == 0 ? 5 : strcmp(impl, "ab") == 0 ? 7
                  : strcmp(impl, "v2") == 0 ? 8 : strcmp(impl, "v3") == 0 ? 9 : 0;
    // demand_v2_kernel's generator refill per chunk (positions per lane; the parser consumes ~18 at
    // 8 x 64 x 5): MSC_V2_QUOTA
    c.v2_quota = 20;
    if (const char* vq = getenv("MSC_V2_QUOTA")) c.v2_quota = atoi(vq) >= 8 && atoi(vq) <= 64 ? atoi(vq) : c.v2_quota;
    const char* gen = getenv("MSC_DEMAND_GEN");
    // (5 and 7: A/B instantiations for 5 SKUs only, more generator waves per 64 envs)
    c.demand_gen = gen && ((atoi(gen) >= 1 && atoi(gen) <= 3) || (K == 5 && (atoi(gen) == 5 || atoi(gen) == 7))) ? atoi(gen) : 3;
    const char* v = getenv("MSC_DEMAND_EPW");
    const int x = v ? atoi(v) : 64;
    c.epw_dem = x == 16 || x == 32 || x == 64 ? x : 64;
    const char* pm = getenv("MSC_PARK_MIN");
    c.park_min = pm && atoi(pm) >= 1 && atoi(pm) <= 64 ? atoi(pm) : 32;
    const char* prot = getenv("MSC_PARSER_ROT");
    c.parser_rot = prot ? atoi(prot) : 0;
    // step_c observation staging when the block's stage fits (C3: 8 x 64 x 35 floats = 70 KiB)
    // staged in two phases of ceil(W / 2) agents: half the LDS, so two step_c blocks fit beside the
    // pipelined demand kernel's (C3 MAPPO rollout 1.19 -> 1.14 ms per step; profiles/r03/ab_stage_phases.txt)
    c.obs_stage = (size_t)BS * ((c.W * c.L) | 1) * sizeof(float) <= 80 * 1024 ? (c.W >= 2 ? 2 : 1) : 0;
    // MSC_OBS_STAGE=0 | 1 | P: off / whole block / in P phases of ceil(W / P) agents (a P-th of the LDS)
    if (const char* os = getenv("MSC_OBS_STAGE")) c.obs_stage = c.obs_stage ? (atoi(os) > 0 ? atoi(os) : 0) : 0;
    if (c.obs_stage > c.W) c.obs_stage = c.W;
    // step_c with the pending ring in registers (8-wave blocks, up to 256 VGPRs): C2 (4,096 envs)
    // 152.7 -> 157.4 M agent-steps/s; at 32,768 envs the env line is unchanged and the MAPPO rollout
    // 1.165 -> 1.188 ms per step (fewer step_c blocks fit beside the demand kernel), so only below
    // the lane allocator's env count (profiles/r03/ab_ringreg.txt). MSC_OBS_RING_REG=0|1 forces it.
    c.obs_ring_reg = n_envs < 16384 ? 1 : 0;
    if (const char* orr = getenv("MSC_OBS_RING_REG")) c.obs_ring_reg = atoi(orr) != 0;
    // phase B: one env per lane (alloc_lane_kernel) when there are enough env chains to fill the
    // chip and the Poisson demand kernel of the next step runs beside it (it then needs the issue
    // slots the lane kernel leaves free: C3, 32768 envs: 0.80 vs 0.86 ms/step); otherwise the
    // group-per-env kernel, whose 8-16x more waves shorten each chain (C5, 8192 envs x 16
    // warehouses, empirical demand: 1.08 vs 1.71 ms/step). MSC_ALLOC_IMPL=lane|group forces one.
    c.alloc_impl = (d->demand_type == MSC_DEMAND_POISSON && n_envs >= 16384) ? 0 : 1;
    if (const char* al = getenv("MSC_ALLOC_IMPL")) {
      if (strcmp(al, "group") == 0) c.alloc_impl = 1;
      else if (strcmp(al, "lane") == 0) c.alloc_impl = 0;
    }
    if (W > 16 || K > 8) c.alloc_impl = 1;  // the lane allocator's instantiations stop at 16 x 8
    c.alloc_lpe = 0;
    if (const char* lp = getenv("MSC_ALLOC_LPE")) c.alloc_lpe = atoi(lp);
    // group kernel over empirical demand: a wave runs as many order iterations as its busiest env,
    // and trace order counts spread widely (C5: 200-1,000 per step), so the envs are visited in
    // descending order of this step's count (one counting-sort launch; results do not depend on
    // the order, every env is independent). MSC_ALLOC_SORT=0|1 forces it off / on.
    c.alloc_sort = (c.alloc_impl == 1 && d->demand_type == MSC_DEMAND_EMPIRICAL) ? 1 : 0;
    if (const char* so = getenv("MSC_ALLOC_SORT")) c.alloc_sort = c.alloc_impl == 1 && atoi(so) != 0 ? 1 : 0;
    int64_t maxc = order_cap;
    if (d->demand_type == MSC_DEMAND_EMPIRICAL) {
      maxc = 0;
      for (int i = 0; i < c.tr_rows; i++) maxc = std::max<int64_t>(maxc, toff[i + 1] - toff[i]);
    }
    c.sort_shift = 0;
    while ((maxc >> c.sort_shift) >= SORT_BUCKETS) c.sort_shift++;
    // few envs (BASELINE configs[1]: 4,096): the scan allocator (one env per wave, no
    // data-dependent loop per order) at <= 8 warehouses and <= 6 SKUs. It also runs 9-16 warehouses
    // (MSC_ALLOC_IMPL=scan) but loses there: at C5 (16 x 256, 8,192 envs, ~2.5 orders per region, so
    // about one order per batch) 1.78 against 0.89 ms per step for the group kernel
    // (profiles/r04/ab_c5_scan.txt). An explicit MSC_ALLOC_IMPL=group keeps the group kernel.
    const char* al_env = getenv("MSC_ALLOC_IMPL");
    if (c.alloc_impl == 1 && !al_env && W <= 8 && alloc_scan_supported(W, K)) c.alloc_impl = 2;
    if (al_env && strcmp(al_env, "scan") == 0) c.alloc_impl = alloc_scan_supported(W, K) ? 2 : 1;
    c.scan_defer = 1;
    // phase C inside the scan allocator (one env per wave: its obs, rewards and state updates from the
    // allocation's registers; no step_c launch). MSC_FUSE_C=0 keeps the step_c kernel.
    c.fuse_c = c.alloc_impl == 2 ? (alloc_scan_fuse_supported(W, K, RING) ? 1 : 0)
             : c.alloc_impl == 1 ? (K <= 8 && RING <= 4 ? 1 : 0)  // the group allocator's (step_b_phase_c)
             : 0;
    if (const char* fc = getenv("MSC_FUSE_C")) c.fuse_c = c.fuse_c && atoi(fc) != 0 ? 1 : 0;
    // phase A too when it has no per-env RNG work (fixed lead times; Poisson demand: the empirical
    // sampler draws its window start in phase A). MSC_FUSE_A=0 keeps the step_a kernel.
    c.fuse_a = c.alloc_impl == 2 && c.fuse_c && d->lead_type != MSC_LEAD_STOCHASTIC && d->demand_type == MSC_DEMAND_POISSON ? 1 : 0;
    c.sc_tab = 1;
    c.sc_form = 5;
    if (const char* sf = getenv("MSC_STEP_C_FORM")) c.sc_form = atoi(sf) == 4 ? 4 : 5;
    // alloc_lane's waves run above the parser of the next step's demand kernel for the first 12/16
    // of their orders, then below it: the pipelined C3 step is demand-bound with the allocation at
    // full priority (0.755 ms demand beside 0.64 ms of step kernels) and chain-bound below it (0.61
    // beside 0.86); 12/16 balances them (341 -> 349 M agent-steps/s, profiles/r06/ab_alloc_prio.txt)
    c.al_psplit = 12;
    if (const char* ps = getenv("MSC_AL_PRIO_SPLIT")) c.al_psplit = atoi(ps) >= 1 && atoi(ps) <= 16 ? atoi(ps) : 12;
    if (const char* st = getenv("MSC_SC_TAB")) c.sc_tab = atoi(st) != 0 ? 1 : 0;
    c.sb_gw = 0;
    if (const char* g = getenv("MSC_SB_GW")) {
      const int v = atoi(g);
      c.sb_gw = (v == 4 || v == 8 || v == 16 || v == 32) ? v : 0;
    }
    if (const char* fa = getenv("MSC_FUSE_A")) c.fuse_a = c.fuse_a && atoi(fa) != 0 ? 1 : 0;
    {
      // step_b's block tables ({of, ov} rows [2][R][W] f64 + closest [R] i32) in LDS: when small
      // (16 KB, room for the blocks of the pipelined demand kernel beside the step), or, with
      // empirical demand (no demand kernel beside the step), when the step_b blocks one CU holds at
      // this env count fit its 160 KB with them (C5, 8,192 envs x 16 warehouses: one 8-wave block per
      // CU, 32 KB of record windows + 66.5 KB of tables); otherwise each region change reads its cost
      // row from L2, and its wait also drains the record windows' LDS-DMA and the stores in flight
      int ncu = 256;
      if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || ncu < 1) ncu = 256;
      int gw = W <= 2 ? 2 : W <= 4 ? 4 : W <= 8 ? 8 : W <= 16 ? 16 : 32;
      if (c.sb_gw > gw) gw = c.sb_gw;  // (the validated MSC_SB_GW: the group width launch_step_k uses)
      // (blocks of 8 waves for 16- and 32-lane groups with the tables, else 4: step_b_waves)
      const int bw = gw >= 16 ? 8 : 4;
      const int64_t blocks = (n_envs * gw + 64 * bw - 1) / (64 * bw), per_cu = (blocks + ncu - 1) / ncu;
      const size_t tab = (size_t)2 * R * W * sizeof(double) + (size_t)R * sizeof(int32_t);
      const size_t blk = (size_t)bw * 2 * 128 * 16 + tab;  // waves x 2 windows x SB_REC records + tables
      c.sb_tab = tab <= 16 * 1024 ? 1
               : (d->demand_type == MSC_DEMAND_EMPIRICAL && blk <= 160 * 1024 && (int64_t)blk * per_cu <= 160 * 1024) ? 1 : 0;
      if (const char* st = getenv("MSC_SB_TAB")) c.sb_tab = atoi(st) != 0 && blk <= 160 * 1024 ? 1 : 0;
    }
    if (const char* sd = getenv("MSC_SCAN_DEFER")) c.scan_defer = atoi(sd) != 0 ? 1 : 0;
    // episode-ahead Poisson demand when the envs are too few to fill the chip with per-step demand
    // chains (MSC_EA=0|1 forces it off / on)
    c.ea_S = 0;
    if (d->demand_type == MSC_DEMAND_POISSON) {
      // (automatic below 8,193 envs; at 32,768 envs it wins only in steady state -- 0.81 -> 0.72 ms
      // per step once the generation pipeline is full, profiles/r04/ab_ea_c3.txt -- while the first
      // episodes pay for the bulk generation, so larger handles ask for it explicitly)
      bool want = d->episode_ahead < 0 ? n_envs <= 8192 : d->episode_ahead > 0;
      if (const char* ea = getenv("MSC_EA")) want = atoi(ea) != 0;
      // 16 slots: the generation runs further ahead of the step (C2 over 48 episodes: 175.5 M
      // agent-steps/s at 12 slots, 180-183 M at 16; profiles/r03/ab_ea_slots.txt); 29 GB at 4,096 envs
      // (the memory budget below may lower it)
      int S = 16;
      if (d->episode_ahead > 0 && d->episode_ahead < S) S = d->episode_ahead;
      if (const char* es = getenv("MSC_EA_SLOTS")) S = atoi(es);
      S = S < 2 ? 2 : (S > MSC_EA_MAX_S ? MSC_EA_MAX_S : S);
      if (want) {
        double lam_sum = 0.0, draws = 0.0;
        // expected uniforms per Poisson draw: lambda + 1 for the multiplication method, a few per
        // PTRS trial (two uniforms, acceptance > 0.5) at lambda >= 10
        auto per_draw = [](double lam) { return lam < 10.0 ? lam + 1.0 : 8.0; };
        for (int r = 0; r < R; r++) {
          const double lo = d->lambda_orders[r];
          lam_sum += lo;
          double per_order = K;  // the SKU mask's Bernoulli draws
          for (int s = 0; s < K; s++) per_order += d->probability_skus[r] * per_draw(d->lambda_quantity[(size_t)r * K + s]);
          draws += per_draw(lo) + lo * per_order;
        }
        const double m = lam_sum * d->episode_length;
        draws *= d->episode_length;
        const double cap_d = ceil(m + 12.0 * sqrt(m + 1.0) + 64.0);
        // slot record indices are int32 in the kernels and stream positions uint32: an episode whose
        // records or draws (with a 12-sigma margin) do not fit keeps per-step demand
        if (cap_d * nv <= (double)INT32_MAX && draws + 12.0 * sqrt(draws + 1.0) < 4294967295.0) {
          c.ea_S = S;
          c.ea_cap = (int64_t)cap_d;
        }
      }
    }
  }

  TablePack tp;
  std::vector<int32_t> zeros_wk(WK, 0);
  std::vector<float> zeros_f(c.F > 0 ? c.F : 1, 0.0f), ones_f(c.F > 0 ? c.F : 1, 1.0f);
  const size_t o_act = tp.add(d->action_param, sizeof(double) * K);
  const size_t o_init = tp.add(d->init_values ? d->init_values : zeros_wk.data(), sizeof(int32_t) * WK);
  const size_t o_hold = tp.add(hold.data(), sizeof(double) * K);
  const size_t o_pen = tp.add(pen.data(), sizeof(double) * K);
  const size_t o_skw = tp.add(d->sku_weights, sizeof(double) * K);
  const size_t o_ofT = tp.add(ofT.data(), sizeof(double) * ofT.size());
  const size_t o_ovT = tp.add(ovT.data(), sizeof(double) * ovT.size());
  const size_t o_inF = tp.add(d->inbound_fixed, sizeof(double) * WK);
  const size_t o_inV = tp.add(d->inbound_variable, sizeof(double) * WK);
  const size_t o_elo = tp.add(enlam_o.data(), sizeof(double) * R);
  const size_t o_ps = tp.add(p_sku.data(), sizeof(double) * R);
  const size_t o_pk = tp.add(p_skip.data(), sizeof(double) * R);
  const size_t o_elq = tp.add(enlam_q.data(), sizeof(double) * enlam_q.size());
  const size_t o_pto = tp.add(ptrs_o.data(), sizeof(PtrsConst) * ptrs_o.size());
  const size_t o_ptq = tp.add(ptrs_q.data(), sizeof(PtrsConst) * ptrs_q.size());
  const size_t o_elt = tp.add(d->expected_lead_times, sizeof(int32_t) * WK);
  const size_t o_md = tp.add(d->lead_type == MSC_LEAD_STOCHASTIC ? d->max_deviation : zeros_wk.data(),
                             sizeof(int32_t) * (d->lead_type == MSC_LEAD_STOCHASTIC && d->max_dev_per_sku ? K : 1));
  const size_t o_hm = tp.add(home_mask.data(), sizeof(uint32_t) * R);
  const size_t o_cl = tp.add(closest.data(), sizeof(int32_t) * R);
  const size_t o_ho = tp.add(home_of.data(), sizeof(int32_t) * W);
  const size_t o_mean = tp.add(c.norm == MSC_OBS_MEANSTD ? d->obs_mean : zeros_f.data(), sizeof(float) * zeros_f.size());
  const size_t o_std = tp.add(c.norm == MSC_OBS_MEANSTD ? d->obs_std : ones_f.data(), sizeof(float) * ones_f.size());
  size_t o_toff = 0, o_trec = 0;
  if (d->demand_type == MSC_DEMAND_EMPIRICAL) {
    o_toff = tp.add(toff.data(), sizeof(int64_t) * toff.size());
    o_trec = tp.add(trec.data(), sizeof(uint4) * trec.size());
  }

  HIP_TRY(hipSetDevice(device));
  msc_env* env = new msc_env();
  env->device = device;
  auto fail = [&](int rc) {
    if (env->tables) (void)hipFree(env->tables);
    if (env->arena) (void)hipFree(env->arena);
    if (env->scratch) (void)hipFree(env->scratch);
    if (env->dev) (void)hipFree(env->dev);
    if (env->ea_mem) (void)hipFree(env->ea_mem);
    delete env;
    return rc;
  };
  if (hipMalloc(&env->tables, tp.host.size()) != hipSuccess) return fail(set_err(-2, "hipMalloc(tables) failed"));
  if (hipMemcpy(env->tables, tp.host.data(), tp.host.size(), hipMemcpyHostToDevice) != hipSuccess)
    return fail(set_err(-2, "copy tables failed"));
  char* tb = static_cast<char*>(env->tables);
  c.act_param = (const double*)(tb + o_act);
  c.init_vals = (const int32_t*)(tb + o_init);
  c.hold = (const double*)(tb + o_hold);
  c.pen = (const double*)(tb + o_pen);
  c.skw = (const double*)(tb + o_skw);
  c.ofT = (const double*)(tb + o_ofT);
  c.ovT = (const double*)(tb + o_ovT);
  c.inF = (const double*)(tb + o_inF);
  c.inV = (const double*)(tb + o_inV);
  c.enlam_o = (const double*)(tb + o_elo);
  c.p_sku = (const double*)(tb + o_ps);
  c.p_skip = (const double*)(tb + o_pk);
  c.enlam_q = (const double*)(tb + o_elq);
  c.ptrs_o = (const double*)(tb + o_pto);
  c.ptrs_q = (const double*)(tb + o_ptq);
  c.elt = (const int32_t*)(tb + o_elt);
  c.maxdev = (const int32_t*)(tb + o_md);
  c.home_mask = (const uint32_t*)(tb + o_hm);
  c.closest = (const int32_t*)(tb + o_cl);
  c.home_of = (const int32_t*)(tb + o_ho);
  c.obs_mean = (const float*)(tb + o_mean);
  c.obs_std = (const float*)(tb + o_std);
  if (d->demand_type == MSC_DEMAND_EMPIRICAL) {
    c.tr_off = (const int64_t*)(tb + o_toff);
    c.tr_rec = (const uint4*)(tb + o_trec);
  }

  // ---- persistent state arena (SoA, env fastest) -----------------------------------------
  const int64_t E = n_envs;
  const bool stoch = d->lead_type == MSC_LEAD_STOCHASTIC;
  size_t off = 0;
  auto slot = [&](size_t bytes) {
    size_t o = off;
    off = (off + bytes + 255) & ~size_t(255);
    return o;
  };
  const size_t a_inv = slot(sizeof(int32_t) * WK * E);
  const size_t a_rq = slot(sizeof(int32_t) * (size_t)WK * RING * E);
  const size_t a_rl = slot(stoch ? (size_t)WK * RING * E : 1);
  const size_t a_hist = slot(sizeof(int32_t) * (size_t)MSC_HISTORY * WK * E);
  const size_t a_inc = slot(sizeof(int32_t) * WK * E);
  const size_t a_fc = slot(sizeof(float) * WK * E);
  const size_t a_rng = slot(sizeof(uint64_t) * 8 * E);
  const size_t a_rbuf = slot(sizeof(uint32_t) * 4 * E);
  const size_t a_rpre = slot(sizeof(uint64_t) * 4 * E);
  const size_t a_bpre = slot(sizeof(uint32_t) * 2 * E);
  const size_t a_t = slot(sizeof(int32_t) * E);
  const size_t a_cnt = slot(sizeof(int32_t) * E);
  const size_t a_orig = slot(sizeof(uint32_t) * E);
  const size_t a_root = slot(sizeof(uint32_t) * E);
  const size_t a_emp = slot(sizeof(int32_t) * E);
  const size_t a_perm = slot(sizeof(int32_t) * E);
  const size_t a_err = slot(sizeof(uint32_t) * 4);
  const size_t a_sht = slot(sizeof(int32_t) * WK * E);
  const size_t a_shh = slot(sizeof(int32_t) * WK * E);
  const size_t a_pen = slot(sizeof(double) * W * E);
  const size_t a_out = slot(sizeof(double) * W * E);
  const size_t a_inb = slot(sizeof(double) * W * E);
  env->arena_bytes = off;
  if (hipMalloc(&env->arena, off) != hipSuccess) return fail(set_err(-2, "hipMalloc(state arena, %zu B) failed", off));
  if (hipMemset(env->arena, 0, off) != hipSuccess) return fail(set_err(-2, "memset arena failed"));
  char* ab = static_cast<char*>(env->arena);
  EnvState s{};
  s.inv = (int32_t*)(ab + a_inv);
  s.ring_q = (int32_t*)(ab + a_rq);
  s.ring_l = (uint8_t*)(ab + a_rl);
  s.hist = (int32_t*)(ab + a_hist);
  s.inc = (int32_t*)(ab + a_inc);
  s.fc = (float*)(ab + a_fc);
  s.rng = (uint64_t*)(ab + a_rng);
  s.rbuf = (uint32_t*)(ab + a_rbuf);
  s.rng_pre = (uint64_t*)(ab + a_rpre);
  s.rbuf_pre = (uint32_t*)(ab + a_bpre);
  s.t = (int32_t*)(ab + a_t);
  s.counter = (int32_t*)(ab + a_cnt);
  s.orig_root = (uint32_t*)(ab + a_orig);
  s.root = (uint32_t*)(ab + a_root);
  s.emp_start = (int32_t*)(ab + a_emp);
  s.perm = (int32_t*)(ab + a_perm);
  s.err = (uint32_t*)(ab + a_err);
  s.sc_sht = (int32_t*)(ab + a_sht);
  s.sc_shh = (int32_t*)(ab + a_shh);
  s.sc_pen = (double*)(ab + a_pen);
  s.sc_out = (double*)(ab + a_out);
  s.sc_inb = (double*)(ab + a_inb);
  EnvState s2 = s;
  if (d->demand_type == MSC_DEMAND_POISSON) {
    const size_t rec_bytes = sizeof(uint4) * (size_t)nv * order_cap * E;
    env->order_bytes = (rec_bytes + sizeof(int32_t) * E + 255) & ~size_t(255);
    if (hipMalloc(&env->scratch, 2 * env->order_bytes) != hipSuccess)
      return fail(set_err(-2, "hipMalloc(order buffers, %zu B) failed", 2 * env->order_bytes));
    for (int b = 0; b < 2; b++) {
      char* base = (char*)env->scratch + b * env->order_bytes;
      EnvState& sb = b ? s2 : s;
      sb.orders = (uint4*)base;
      sb.n_orders = (int32_t*)(base + rec_bytes);
    }
  }
  if (c.ea_S > 0) {
    // episode-ahead memory budget: at most ea_mem_fraction (default 0.25, MSC_EA_MEM_FRAC) of the
    // memory free now, so the rollout / learner allocations that follow keep the rest; the slot
    // count shrinks to what fits, and below 2 slots EA stays off
    const int T = c.T;
    const size_t slot_bytes = sizeof(uint4) * (size_t)nv * c.ea_cap * E + sizeof(int32_t) * (size_t)(T + 1) * E +
                              sizeof(uint32_t) * (size_t)T * E + sizeof(int32_t) * (size_t)E;
    double frac = d->ea_mem_fraction > 0.0 ? d->ea_mem_fraction : 0.25;
    if (const char* mf = getenv("MSC_EA_MEM_FRAC")) frac = atof(mf);
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) {
      (void)hipGetLastError();
      free_b = 0;
    }
    const double budget = frac * (double)free_b;
    const int64_t fit = (int64_t)(budget / (double)(slot_bytes + 1024 /* alignment slack */));
    if (fit < c.ea_S) c.ea_S = fit < 2 ? 0 : (int)fit;
    env->ea_budget = (int64_t)budget;
  }
  if (c.ea_S > 0) {  // episode-ahead buffers; without the memory EA stays off
    const int S = c.ea_S, T = c.T;
    const size_t rec = sizeof(uint4) * (size_t)nv * c.ea_cap * S * E;
    const size_t offb = sizeof(int32_t) * (size_t)S * (T + 1) * E, posb = sizeof(uint32_t) * (size_t)S * T * E;
    const size_t cntb = sizeof(int32_t) * (size_t)S * E;
    auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
    env->ea_bytes = (int64_t)(al(rec) + al(offb) + al(posb) + al(cntb));
    if (hipMalloc(&env->ea_mem, al(rec) + al(offb) + al(posb) + al(cntb)) == hipSuccess) {
      char* b = (char*)env->ea_mem;
      s.ea_rec = s2.ea_rec = (uint4*)b;
      s.ea_off = s2.ea_off = (int32_t*)(b + al(rec));
      s.ea_pos = s2.ea_pos = (uint32_t*)(b + al(rec) + al(offb));
      s.ea_cnt = s2.ea_cnt = (int32_t*)(b + al(rec) + al(offb) + al(posb));
      env->ea_enabled = true;
      env->obs_stage_pe = c.obs_stage;
      env->chain_prio_pe = c.chain_prio;
      // refill batch: a batch freed by episodes n-B+1 .. n is needed S-B episodes later. A generation
      // chunk's duration is one lane's parse chain whatever the slots per launch, so the slots per
      // launch set the generation rate: at 4,096 envs 4 per launch (16,384 lanes) could not keep up
      // with the step (C2 sustained 173 M agent-steps/s over 96 episodes), 8 per launch can (207 M,
      // profiles/r05/ab_ea_batch.txt); at 32,768 envs a single slot per launch already fills the chip
      int B = E <= 8192 ? S / 2 : S / 4;
      B = B > 1 ? B : 1;
      if (const char* eb = getenv("MSC_EA_BATCH")) B = atoi(eb);
      env->ea_batch = B < 1 ? 1 : (B > S - 1 ? S - 1 : B);
      // step_c's observation staging (up to 80 KB of LDS per block) stalls behind a generation
      // chunk's pending blocks for the chunk's whole run (measured: 5.5 ms step_c launches right
      // after a chunk starts, none without staging): off with EA unless MSC_OBS_STAGE=1
      const char* os = getenv("MSC_OBS_STAGE");
      if (!(os && atoi(os) != 0)) c.obs_stage = 0;
      // the generation waves (parser 2, generators 1) are background work: the whole step chain
      // runs above them (the allocation kernels are at 3 already; MSC_CHAIN_PRIO=0 leaves step_a /
      // step_c at 0)
      const char* cp = getenv("MSC_CHAIN_PRIO");
      c.chain_prio = (cp && atoi(cp) == 0) ? 0 : 1;
      // chunk A/B at C2 (scripts/gpu_ab_eachunk.sh, steps per launch -> M agent-steps/s): 5 -> 149.6,
      // 10 -> 152.9, 20 -> 157.8, 34 -> 165.3, 50 -> 170.1, 100 -> 171.4 (fewer launch ramps and
      // tails beside the step kernels); 50 keeps the work a synchronize may wait for at half an episode
      // at 32,768 envs whole-episode launches: 0.72 ms per step against 0.78 with 50-step chunks
      // (profiles/r04/ab_ea_c3.txt)
      int ch = E > 8192 ? T : 50;
      if (const char* ec = getenv("MSC_EA_CHUNK")) ch = atoi(ec);
      env->ea_chunk = ch < 1 ? 1 : ch;
    } else {
      (void)hipGetLastError();
      env->ea_mem = nullptr;
      env->ea_bytes = 0;
      c.ea_S = 0;
    }
  }
  // root seeds: explicit, or SeedSequence([base_seed, worker_index, env_index])
  std::vector<uint32_t> roots(E);
  std::vector<int32_t> minus1(E, -1);
  for (int64_t i = 0; i < E; i++) {
    if (env_seeds_host) roots[i] = env_seeds_host[i];
    else {
      const uint64_t idx = (uint64_t)(env_index_offset + i);
      uint32_t words[4] = {base_seed, worker_index, (uint32_t)idx, (uint32_t)(idx >> 32)};
      roots[i] = ss_u32(words, (idx >> 32) ? 4 : 3);
    }
  }
  if (hipMemcpy(s.orig_root, roots.data(), sizeof(uint32_t) * E, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(s.root, roots.data(), sizeof(uint32_t) * E, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(s.emp_start, minus1.data(), sizeof(int32_t) * E, hipMemcpyHostToDevice) != hipSuccess)
    return fail(set_err(-2, "seed upload failed"));
  // The step kernel of step t runs concurrently with the demand kernel of step t+1 (pipelining):
  // stage the outbound cost table in LDS only when two blocks of each still fit one CU's LDS.
  // Otherwise the step kernel's blocks wait for the demand kernel's and nothing overlaps
  // (measured: 3.4 -> 2.2 ms per step at 8x64x5 with the table in global memory).
  env->c = c;
  env->s = s;
  {
    DevEnv hd[2] = {{c, s}, {c, s2}};
    if (hipMalloc(&env->dev, 2 * sizeof(DevEnv)) != hipSuccess ||
        hipMemcpy(env->dev, hd, 2 * sizeof(DevEnv), hipMemcpyHostToDevice) != hipSuccess)
      return fail(set_err(-2, "device descriptor upload failed"));
  }
  {
    const char* pl = getenv("MSC_PIPELINE");
    env->pipeline = !(pl && strcmp(pl, "0") == 0) && d->demand_type == MSC_DEMAND_POISSON;
  }
  if (hipStreamCreateWithFlags(&env->side, hipStreamNonBlocking) != hipSuccess)
    return fail(set_err(-2, "side stream creation failed"));
  // the pipelining events only order work between two streams of this device (no host waits on
  // them), so their records skip the system-scope fence: ~2 us less per record (tools/ev_gap.hip),
  // C2 224 -> 227 M, C3 +0.3 % (profiles/r06/ab_ev_nofence.txt). MSC_EV_SCOPE=system restores it,
  // =device records them with a device-scope release (A/B)
  unsigned evf = hipEventDisableTiming | hipEventDisableSystemFence;
  if (const char* es = getenv("MSC_EV_SCOPE"))
    evf = hipEventDisableTiming | (strcmp(es, "device") == 0   ? hipEventReleaseToDevice
                                   : strcmp(es, "system") == 0 ? 0u
                                                               : hipEventDisableSystemFence);
  for (int b = 0; b < 2; b++)
    if (hipEventCreateWithFlags(&env->ev_dem[b], evf) != hipSuccess ||
        hipEventCreateWithFlags(&env->ev_step[b], evf) != hipSuccess)
      return fail(set_err(-2, "event creation failed"));
  if (hipEventCreateWithFlags(&env->ev_reset, evf) != hipSuccess)
    return fail(set_err(-2, "event creation failed"));
  for (int b = 0; b < 2; b++) {  // recorded once so that every later wait is well-defined
    (void)hipEventRecord(env->ev_dem[b], env->side);
    env->ev_dem_on[b] = env->side;
    (void)hipEventRecord(env->ev_step[b], env->side);
  }
  (void)hipEventRecord(env->ev_reset, env->side);
  env->side_saw_reset = true;
  if (const char* el = getenv("MSC_EV_ELIDE")) env->ev_elide = strcmp(el, "0") != 0;
  if (env->ea_enabled) {
    // MSC_EA_PRIO=low|high: queue priority of the generation stream (A/B; default: normal)
    int ea_prio = 0, lo = 0, hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
    if (const char* ep = getenv("MSC_EA_PRIO")) ea_prio = strcmp(ep, "low") == 0 ? lo : strcmp(ep, "high") == 0 ? hi : 0;
    if (hipStreamCreateWithPriority(&env->ea_stream, hipStreamNonBlocking, ea_prio) != hipSuccess)
      return fail(set_err(-2, "EA stream creation failed"));
    for (int j = 0; j < MSC_EA_MAX_S; j++)
      if (hipEventCreateWithFlags(&env->ev_gen[j], hipEventDisableTiming) != hipSuccess ||
          hipEventCreateWithFlags(&env->ev_cons[j], hipEventDisableTiming) != hipSuccess)
        return fail(set_err(-2, "event creation failed"));
    if (hipEventCreateWithFlags(&env->ev_snap, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&env->ev_chunk, hipEventDisableTiming) != hipSuccess)
      return fail(set_err(-2, "event creation failed"));
    for (int j = 0; j < MSC_EA_MAX_S; j++) {
      (void)hipEventRecord(env->ev_gen[j], env->ea_stream);
      (void)hipEventRecord(env->ev_cons[j], env->ea_stream);
    }
  }
  *out = env;
  return 0;
}

void msc_env_destroy(msc_env* env) {
  if (!env) return;
  (void)hipSetDevice(env->device);
  (void)hipDeviceSynchronize();
  if (env->tables) (void)hipFree(env->tables);
  if (env->arena) (void)hipFree(env->arena);
  if (env->scratch) (void)hipFree(env->scratch);
  if (env->dev) (void)hipFree(env->dev);
  for (int b = 0; b < 2; b++) {
    if (env->ev_dem[b]) (void)hipEventDestroy(env->ev_dem[b]);
    if (env->ev_step[b]) (void)hipEventDestroy(env->ev_step[b]);
  }
  if (env->ev_reset) (void)hipEventDestroy(env->ev_reset);
  for (int j = 0; j < MSC_EA_MAX_S; j++) {
    if (env->ev_gen[j]) (void)hipEventDestroy(env->ev_gen[j]);
    if (env->ev_cons[j]) (void)hipEventDestroy(env->ev_cons[j]);
  }
  if (env->ev_snap) (void)hipEventDestroy(env->ev_snap);
  if (env->ev_chunk) (void)hipEventDestroy(env->ev_chunk);
  if (env->ea_mem) (void)hipFree(env->ea_mem);
  timing_free(env);
  if (env->side) (void)hipStreamDestroy(env->side);
  if (env->ea_stream) (void)hipStreamDestroy(env->ea_stream);
  delete env;
}

int msc_env_ea_memory(const msc_env* env, int64_t* budget_bytes, int64_t* allocated_bytes) {
  if (!env) return set_err(-1, "null env");
  if (budget_bytes) *budget_bytes = env->ea_budget;
  if (allocated_bytes) *allocated_bytes = env->ea_enabled ? env->ea_bytes : 0;
  return 0;
}

int msc_env_dims(const msc_env* env, int64_t* n_envs, int32_t* n_agents, int32_t* n_skus, int32_t* n_regions,
                 int32_t* local_obs_dim, int32_t* n_features, int32_t* max_lead, int32_t* ea_slots) {
  if (!env) return set_err(-1, "null env");
  if (n_envs) *n_envs = env->c.E;
  if (n_agents) *n_agents = env->c.W;
  if (n_skus) *n_skus = env->c.K;
  if (n_regions) *n_regions = env->c.R;
  if (local_obs_dim) *local_obs_dim = env->c.L;
  if (n_features) *n_features = env->c.F;
  if (max_lead) *max_lead = env->c.Lmax;
  if (ea_slots) *ea_slots = env->ea_enabled ? env->c.ea_S : 0;
  return 0;
}

int msc_env_kernel_choice(const msc_env* env, int32_t* out, int32_t n) {
  if (!env || (!out && n > 0)) return set_err(-1, "null argument");
  const EnvConst& c = env->c;
  const int W = c.W;
  int gw = W <= 2 ? 2 : W <= 4 ? 4 : W <= 8 ? 8 : W <= 16 ? 16 : 32;
  if (c.sb_gw > gw) gw = c.sb_gw;
  const int32_t v[9] = {c.alloc_impl, c.alloc_sort, c.fuse_a, c.fuse_c, c.sb_tab, c.alloc_impl == 1 ? gw : 0,
                        env->ea_enabled ? c.ea_S : 0, c.demand_impl, c.demand_uni};
  const int m = n < 9 ? n : 9;
  for (int i = 0; i < m; i++) out[i] = v[i];
  return m;
}

int msc_env_reset(msc_env* env, const uint8_t* mask, const uint32_t* new_root_seeds, int32_t flags, float* obs,
                  msc_stream_t stream) {
  if (!env) return set_err(-1, "null env");
  hipStream_t st = (hipStream_t)stream;
  // episode-ahead demand stops (it restarts at the next common episode start); envs outside a
  // mask keep their episode, so their demand stream is materialised first
  if (const int rc = ea_stop(env, st, mask != nullptr)) return rc;
  // a reset re-seeds the demand streams: drop any demand generated ahead, order after the
  // side stream's last use of the state
  HIP_TRY(hipStreamWaitEvent(st, env->ev_dem[0], 0));
  HIP_TRY(hipStreamWaitEvent(st, env->ev_dem[1], 0));
  if (env->ready[0] || env->ready[1]) {
    // envs outside the mask keep their episode: rewind their demand stream to before the
    // dropped generation (rng[0][4][E] / rbuf[0][2][E] lead the arena's RNG slots)
    const int64_t E = env->c.E;
    HIP_TRY(hipMemcpyAsync(env->s.rng, env->s.rng_pre, sizeof(uint64_t) * 4 * E, hipMemcpyDeviceToDevice, st));
    HIP_TRY(hipMemcpyAsync(env->s.rbuf, env->s.rbuf_pre, sizeof(uint32_t) * 2 * E, hipMemcpyDeviceToDevice, st));
  }
  env->ready[0] = env->ready[1] = false;
  env->t_sync = mask ? -1 : 0;
  HIP_TRY(launch_reset(env->c, env->dev, mask, new_root_seeds, flags, obs, st));
  HIP_TRY(hipEventRecord(env->ev_reset, st));
  env->side_saw_reset = false;
  return 0;
}

int msc_env_step(msc_env* env, const float* actions, float* obs, float* rewards, double* rewards_f64,
                 uint8_t* truncated, float* final_obs, const msc_step_info* info, msc_stream_t stream) {
  if (!env || !actions || !obs || !rewards || !truncated) return set_err(-1, "null argument");
  const EnvConst& c = env->c;
  hipStream_t st = (hipStream_t)stream;
  StepIO io{};
  io.actions = actions;
  io.obs = obs;
  io.rew = rewards;
  io.rew64 = rewards_f64;
  io.trunc = truncated;
  io.final_obs = final_obs;
  if (info) {
    io.info = *info;
    io.has_info = 1;
    const int64_t E = c.E, W = c.W, K = c.K, R = c.R;
    struct { void* p; size_t n; } z[] = {
        {info->fulfilled_per_warehouse, sizeof(int32_t) * E * W * K},
        {info->demand_per_region, sizeof(int32_t) * E * R * K},
        {info->unfulfilled_demands, sizeof(int32_t) * E * R * K},
        {info->shipment_counts, sizeof(int32_t) * E * W * R},
        {info->shipment_quantities, sizeof(int32_t) * E * W * R},
        {info->shipment_quantities_by_sku, sizeof(int32_t) * E * W * R * K},
        {info->lost_order_counts, sizeof(int32_t) * E * R},
        {info->lost_sales, sizeof(double) * E * W * K},
    };
    for (auto& q : z)
      if (q.p) HIP_TRY(hipMemsetAsync(q.p, 0, q.n, st));
  }
  const bool poisson = c.demand_type == MSC_DEMAND_POISSON;
  const int b = (int)(env->tau & 1);
  // episode-ahead demand: start at a common episode start; an episode n >= 1 reads its slot
  if (env->ea_enabled && !env->ea_paused && env->pipeline && !env->ea_running && env->t_sync == 0)
    if (const int rc = ea_start(env, st)) return rc;
  if (env->ea_running) HIP_TRY(ea_pump(env, false));
  if (env->ea_running && env->t_sync == 0) {
    env->ea_cur = env->ea_n >= 1 ? (int)(env->ea_n % c.ea_S) : -1;
    if (env->ea_cur >= 0) {
      HIP_TRY(ea_flush_to(env, env->ea_cur));
      HIP_TRY(hipStreamWaitEvent(st, env->ev_gen[env->ea_cur], 0));
    }
  }
  io.ea_slot = env->ea_running ? env->ea_cur : -1;
  io.ea_t = env->t_sync;
  const bool ea_step = io.ea_slot >= 0;
  if (poisson && !ea_step) {
    if (env->ready[b]) {
      HIP_TRY(hipStreamWaitEvent(st, env->ev_dem[b], 0));
    } else {
      HIP_TRY(tmark(env, env->tev_dem, env->n_tdem, 0, st));
      HIP_TRY(launch_demand(c, env->dev + b, st));
      env->cnt_dem_launch++;
      HIP_TRY(tmark(env, env->tev_dem, env->n_tdem++, 1, st));
      HIP_TRY(hipEventRecord(env->ev_dem[b], st));
      env->ev_dem_on[b] = st;
    }
  }
  HIP_TRY(tmark(env, env->tev_step, env->n_tstep, 0, st));
  HIP_TRY(launch_step(c, env->dev + b, io, false, st));
  env->cnt_steps++;
  HIP_TRY(tmark(env, env->tev_step, env->n_tstep++, 1, st));
  HIP_TRY(hipEventRecord(env->ev_step[b], st));
  env->ready[b] = false;
  const bool boundary = env->t_sync < 0 || env->t_sync + 1 >= c.T;
  if (env->ea_running && env->t_sync + 1 >= c.T) {
    // episode ea_n ends with this step: its slot is to be refilled with episode ea_n + S once the
    // step has read it; every ea_batch freed slots (consecutive mod S) go in one launch
    const int slot = (int)(env->ea_n % c.ea_S);
    HIP_TRY(hipEventRecord(env->ev_cons[slot], st));
    if (++env->ea_freed == env->ea_batch) {
      const int B = env->ea_batch;
      HIP_TRY(ea_enqueue(env, (slot - B + 1 + c.ea_S) % c.ea_S, B, -1, c.ea_S, 0, slot));
      env->ea_freed = 0;
    }
    env->ea_n++;
  }
  if (env->pipeline && !boundary && !ea_step) {
    // demand of step tau+1 into the other buffer, concurrently with this step kernel; that buffer
    // was last read by step tau-1, and the demand stream was last advanced by demand(tau)
    const int nb = b ^ 1;
    // (a wait already ordered by the side stream itself is not issued: each costs a barrier packet
    // the command processor retires between the demand launches, which bound a pipelined step)
    HIP_TRY(hipStreamWaitEvent(env->side, env->ev_step[nb], 0));
    if (!env->ev_elide || env->ev_dem_on[b] != env->side)
      HIP_TRY(hipStreamWaitEvent(env->side, env->ev_dem[b], 0));
    if (!env->ev_elide || !env->side_saw_reset) {
      HIP_TRY(hipStreamWaitEvent(env->side, env->ev_reset, 0));
      env->side_saw_reset = true;
    }
    HIP_TRY(tmark(env, env->tev_dem, env->n_tdem, 0, env->side));
    HIP_TRY(launch_demand(c, env->dev + nb, env->side));
    env->cnt_dem_launch++;
    HIP_TRY(tmark(env, env->tev_dem, env->n_tdem++, 1, env->side));
    HIP_TRY(hipEventRecord(env->ev_dem[nb], env->side));
    env->ev_dem_on[nb] = env->side;
    env->ready[nb] = true;
  }
  env->t_sync = env->t_sync < 0 ? -1 : (env->t_sync + 1 >= c.T ? 0 : env->t_sync + 1);
  env->tau++;
  return 0;
}

int msc_env_set_pipelining(msc_env* env, int32_t enabled) {
  if (!env) return set_err(-1, "null env");
  env->pipeline = enabled != 0 && env->c.demand_type == MSC_DEMAND_POISSON;
  if (!env->pipeline && env->ea_running) {  // back to per-step demand from the current step on
    HIP_TRY(hipSetDevice(env->device));
    HIP_TRY(hipDeviceSynchronize());
    if (const int rc = ea_stop(env, nullptr, true)) return rc;
    HIP_TRY(hipDeviceSynchronize());
  }
  return 0;
}

int msc_env_set_episode_ahead(msc_env* env, int32_t enabled) {
  if (!env) return set_err(-1, "null env");
  if (!env->ea_enabled) return 0;  // not configured at create (or no memory): nothing to switch
  const bool pause = enabled == 0;
  if (pause == env->ea_paused) return 0;
  HIP_TRY(hipSetDevice(env->device));
  HIP_TRY(hipDeviceSynchronize());
  if (pause && env->ea_running)  // per-step demand from the current step on
    if (const int rc = ea_stop(env, nullptr, true)) return rc;
  env->ea_paused = pause;
  // the per-step path's step_c staging and chain priority (EA runs without staging, chain above the
  // generation waves); patched into both device descriptors
  const int32_t stage = pause ? env->obs_stage_pe : 0;
  const int32_t prio = pause ? env->chain_prio_pe : 1;
  const char* os = getenv("MSC_OBS_STAGE");
  const char* cp = getenv("MSC_CHAIN_PRIO");
  env->c.obs_stage = (!pause && os && atoi(os) != 0) ? env->obs_stage_pe : stage;
  env->c.chain_prio = (!pause && cp && atoi(cp) == 0) ? 0 : prio;
  for (int b = 0; b < 2; b++) {
    HIP_TRY(hipMemcpy(&env->dev[b].c.obs_stage, &env->c.obs_stage, sizeof(int32_t), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(&env->dev[b].c.chain_prio, &env->c.chain_prio, sizeof(int32_t), hipMemcpyHostToDevice));
  }
  HIP_TRY(hipDeviceSynchronize());
  return 0;
}

int msc_env_set_chain_priority(msc_env* env, int32_t enabled) {
  if (!env) return set_err(-1, "null env");
  const int32_t v = enabled != 0 ? 1 : 0;
  env->c.chain_prio = v;
  HIP_TRY(hipSetDevice(env->device));
  HIP_TRY(hipDeviceSynchronize());  // no launch in flight reads the descriptors being patched
  for (int b = 0; b < 2; b++)
    HIP_TRY(hipMemcpy(&env->dev[b].c.chain_prio, &v, sizeof v, hipMemcpyHostToDevice));
  return 0;
}

int msc_env_set_option(msc_env* env, int32_t key, int32_t value) {
  if (!env) return set_err(-1, "null env");
  if (key == MSC_OPT_STEP_C_FORM) {
    if (value != 4 && value != 5) return set_err(-1, "MSC_OPT_STEP_C_FORM must be 4 or 5");
    env->c.sc_form = value;  // (host-side launch choice: the device descriptor does not carry it)
    return 0;
  }
  if (key == MSC_OPT_ALLOC_PRIO_SPLIT) {
    if (value < 1 || value > 16) return set_err(-1, "MSC_OPT_ALLOC_PRIO_SPLIT must be in 1 .. 16");
    if (env->c.al_psplit == value) return 0;
    env->c.al_psplit = value;
    HIP_TRY(hipSetDevice(env->device));
    HIP_TRY(hipDeviceSynchronize());  // no launch in flight reads the descriptors being patched
    for (int b = 0; b < 2; b++)
      HIP_TRY(hipMemcpy(&env->dev[b].c.al_psplit, &value, sizeof value, hipMemcpyHostToDevice));
    return 0;
  }
  return set_err(-1, "unknown option %d", key);
}

int msc_env_set_timing(msc_env* env, int32_t max_steps) {
  if (!env) return set_err(-1, "null env");
  if (max_steps < 0) return set_err(-1, "max_steps < 0");
  HIP_TRY(hipSetDevice(env->device));
  HIP_TRY(hipDeviceSynchronize());
  timing_free(env);
  for (int i = 0; i < 2 * max_steps; i++) {
    hipEvent_t a, b, x;
    HIP_TRY(hipEventCreate(&a));
    HIP_TRY(hipEventCreate(&b));
    HIP_TRY(hipEventCreate(&x));
    env->tev_dem.push_back(a);
    env->tev_step.push_back(b);
    env->tev_ea.push_back(x);
  }
  env->t_cap = max_steps;
  return 0;
}

int msc_env_read_timing(msc_env* env, double* demand_ms, double* step_ms, int64_t* n_demand, int64_t* n_step) {
  if (!env) return set_err(-1, "null env");
  auto mean = [&](const std::vector<hipEvent_t>& v, int n, double* out) -> hipError_t {
    n = n < env->t_cap ? n : env->t_cap;
    double sum = 0.0;
    for (int i = 0; i < n; i++) {
      hipError_t e = hipEventSynchronize(v[2 * i + 1]);
      if (e != hipSuccess) return e;
      float ms = 0.f;
      e = hipEventElapsedTime(&ms, v[2 * i], v[2 * i + 1]);
      if (e != hipSuccess) return e;
      sum += ms;
    }
    if (out) *out = n ? sum / n : 0.0;
    return hipSuccess;
  };
  HIP_TRY(mean(env->tev_dem, env->n_tdem, demand_ms));
  HIP_TRY(mean(env->tev_step, env->n_tstep, step_ms));
  if (n_demand) *n_demand = env->n_tdem < env->t_cap ? env->n_tdem : env->t_cap;
  if (n_step) *n_step = env->n_tstep < env->t_cap ? env->n_tstep : env->t_cap;
  return 0;
}

int msc_env_read_timing_ea(msc_env* env, double* ea_ms, int64_t* n_ea, int32_t* slots, int32_t* active,
                           double* env_steps_per_launch) {
  if (!env) return set_err(-1, "null env");
  const int n = env->n_tea < env->t_cap ? env->n_tea : env->t_cap;
  double sum = 0.0, work = 0.0;
  for (int i = 0; i < n; i++) {
    HIP_TRY(hipEventSynchronize(env->tev_ea[2 * i + 1]));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, env->tev_ea[2 * i], env->tev_ea[2 * i + 1]));
    sum += ms;
    work += i < (int)env->tea_work.size() ? env->tea_work[i] : 0.0;
  }
  if (ea_ms) *ea_ms = n ? sum / n : 0.0;
  if (env_steps_per_launch) *env_steps_per_launch = n ? work / n : 0.0;
  if (n_ea) *n_ea = n;
  if (slots) *slots = env->c.ea_S;
  if (active) *active = env->ea_running && env->ea_cur >= 0 ? 1 : 0;
  return 0;
}

int msc_env_work_counters(const msc_env* env, int64_t* ea_launches, double* ea_env_steps, int64_t* demand_launches,
                          int64_t* steps) {
  if (!env) return set_err(-1, "null env");
  if (ea_launches) *ea_launches = env->cnt_ea_launch;
  if (ea_env_steps) *ea_env_steps = env->cnt_ea_work;
  if (demand_launches) *demand_launches = env->cnt_dem_launch;
  if (steps) *steps = env->cnt_steps;
  return 0;
}

int msc_env_generate_demand(msc_env* env, msc_stream_t stream) {
  if (!env) return set_err(-1, "null env");
  if (env->c.demand_type != MSC_DEMAND_POISSON) return 0;
  // the next step reads an episode-ahead slot: nothing to generate
  if (env->ea_running && (env->t_sync == 0 ? env->ea_n >= 1 : env->ea_cur >= 0)) return 0;
  const int b = (int)(env->tau & 1);
  if (env->ready[b]) return 0;  // already generated ahead
  hipStream_t st = (hipStream_t)stream;
  HIP_TRY(hipStreamWaitEvent(st, env->ev_step[b], 0));     // last reader of buffer b
  HIP_TRY(hipStreamWaitEvent(st, env->ev_dem[b ^ 1], 0));  // last advance of the demand streams
  HIP_TRY(hipStreamWaitEvent(st, env->ev_reset, 0));
  HIP_TRY(launch_demand(env->c, env->dev + b, st));
  env->cnt_dem_launch++;
  HIP_TRY(hipEventRecord(env->ev_dem[b], st));
  env->ev_dem_on[b] = st;
  env->ready[b] = true;
  return 0;
}

int msc_env_obs_flat(const msc_env* env, const float* obs, float* flat, msc_stream_t stream) {
  if (!env || !obs || !flat) return set_err(-1, "null argument");
  HIP_TRY(launch_obs_flat(env->c, obs, flat, (hipStream_t)stream));
  return 0;
}

int msc_env_read_state(const msc_env* env, int32_t* inv, int32_t* ts, int32_t* ep, uint64_t* rng) {
  if (!env) return set_err(-1, "null env");
  const int64_t E = env->c.E, WK = (int64_t)env->c.W * env->c.K;
  HIP_TRY(hipDeviceSynchronize());
  if (rng && env->ea_running && env->ea_cur >= 0 && env->t_sync > 0) {
    if (const int rc = ea_materialize(env, nullptr)) return rc;
    HIP_TRY(hipDeviceSynchronize());
  }
  if (inv) {
    std::vector<int32_t> soa(WK * E);
    HIP_TRY(hipMemcpy(soa.data(), env->s.inv, sizeof(int32_t) * WK * E, hipMemcpyDeviceToHost));
    for (int64_t e = 0; e < E; e++)
      for (int64_t i = 0; i < WK; i++) inv[e * WK + i] = soa[i * E + e];
  }
  if (ts) HIP_TRY(hipMemcpy(ts, env->s.t, sizeof(int32_t) * E, hipMemcpyDeviceToHost));
  if (ep) HIP_TRY(hipMemcpy(ep, env->s.counter, sizeof(int32_t) * E, hipMemcpyDeviceToHost));
  if (rng) {
    std::vector<uint64_t> r(8 * E);
    std::vector<uint32_t> b(4 * E);
    HIP_TRY(hipMemcpy(r.data(), env->s.rng, sizeof(uint64_t) * 8 * E, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(b.data(), env->s.rbuf, sizeof(uint32_t) * 4 * E, hipMemcpyDeviceToHost));
    if (env->ready[env->tau & 1]) {
      // the next step's demand is already generated: report the demand stream as of before it
      HIP_TRY(hipMemcpy(r.data(), env->s.rng_pre, sizeof(uint64_t) * 4 * E, hipMemcpyDeviceToHost));
      HIP_TRY(hipMemcpy(b.data(), env->s.rbuf_pre, sizeof(uint32_t) * 2 * E, hipMemcpyDeviceToHost));
    }
    for (int64_t e = 0; e < E; e++)
      for (int k = 0; k < 2; k++) {
        for (int j = 0; j < 4; j++) rng[(e * 2 + k) * 6 + j] = r[(k * 4 + j) * E + e];
        rng[(e * 2 + k) * 6 + 4] = b[(k * 2 + 0) * E + e];
        rng[(e * 2 + k) * 6 + 5] = b[(k * 2 + 1) * E + e];
      }
  }
  return 0;
}

// Checkpoint blob: {magic, pending, t_sync, reserved} | state arena | [order buffer of the next
// step when its demand was already generated ahead (its RNG draws are then already consumed)].
struct StateHeader {
  uint32_t magic, pending;
  int32_t t_sync, reserved;
};
constexpr uint32_t STATE_MAGIC = 0x4d534331u;  // "MSC1"

int64_t msc_env_state_bytes(const msc_env* env) {
  return env ? (int64_t)(sizeof(StateHeader) + env->arena_bytes + env->order_bytes) : -1;
}

int msc_env_save_state(const msc_env* env, void* buf) {
  if (!env || !buf) return set_err(-1, "null argument");
  HIP_TRY(hipDeviceSynchronize());
  if (env->ea_running && env->ea_cur >= 0 && env->t_sync > 0) {  // the blob carries the demand stream
    if (const int rc = ea_materialize(env, nullptr)) return rc;
    HIP_TRY(hipDeviceSynchronize());
  }
  const int b = (int)(env->tau & 1);
  StateHeader h{STATE_MAGIC, env->ready[b] ? 1u : 0u, env->t_sync, 0};
  memcpy(buf, &h, sizeof h);
  char* p = (char*)buf + sizeof h;
  HIP_TRY(hipMemcpy(p, env->arena, env->arena_bytes, hipMemcpyDeviceToHost));
  if (h.pending)
    HIP_TRY(hipMemcpy(p + env->arena_bytes, (char*)env->scratch + b * env->order_bytes, env->order_bytes,
                      hipMemcpyDeviceToHost));
  return 0;
}

int msc_env_load_state(msc_env* env, const void* buf) {
  if (!env || !buf) return set_err(-1, "null argument");
  StateHeader h;
  memcpy(&h, buf, sizeof h);
  if (h.magic != STATE_MAGIC) return set_err(-1, "not a libmarlsc state blob");
  HIP_TRY(hipDeviceSynchronize());
  if (const int rc = ea_stop(env, nullptr, false)) return rc;  // restarts at the next episode start
  const char* p = (const char*)buf + sizeof h;
  HIP_TRY(hipMemcpy(env->arena, p, env->arena_bytes, hipMemcpyHostToDevice));
  const int b = (int)(env->tau & 1);
  env->ready[0] = env->ready[1] = false;
  if (h.pending) {
    HIP_TRY(hipMemcpy((char*)env->scratch + b * env->order_bytes, p + env->arena_bytes, env->order_bytes,
                      hipMemcpyHostToDevice));
    env->ready[b] = true;
    HIP_TRY(hipEventRecord(env->ev_dem[b], env->side));
    env->ev_dem_on[b] = env->side;
  }
  env->t_sync = h.t_sync;
  return 0;
}

int msc_env_check(msc_env* env) {
  if (!env) return set_err(-1, "null env");
  HIP_TRY(hipDeviceSynchronize());
  uint32_t err = 0;
  HIP_TRY(hipMemcpy(&err, env->s.err, sizeof err, hipMemcpyDeviceToHost));
  if (err & ERR_ORDER_OVERFLOW) return set_err(-3, "per-step order buffer overflow (capacity %d)", env->c.order_cap);
  return 0;
}

int msc_gae_grouped(const float* rewards, const float* values, const float* next_values, const uint8_t* terminated,
                    const uint8_t* truncated, int64_t n_seq, int32_t T, float gamma, float lam, float* advantages,
                    float* targets, int32_t n_groups, double* stats_out, msc_stream_t stream) {
  if (!rewards || !values || !advantages || n_seq < 0 || T < 0) return set_err(-1, "bad argument");
  if (n_groups < 1 || n_groups > 64 || n_seq % n_groups != 0)
    return set_err(-1, "n_groups %d must be in [1, 64] and divide n_seq %lld", n_groups, (long long)n_seq);
  HIP_TRY(launch_gae(rewards, values, next_values, terminated, truncated, n_seq, T, gamma, lam, advantages, targets,
                     n_groups, stats_out, (hipStream_t)stream));
  return 0;
}

int msc_gae(const float* rewards, const float* values, const float* next_values, const uint8_t* terminated,
            const uint8_t* truncated, int64_t n_seq, int32_t T, float gamma, float lam, float* advantages,
            float* targets, double* stats_out, msc_stream_t stream) {
  return msc_gae_grouped(rewards, values, next_values, terminated, truncated, n_seq, T, gamma, lam, advantages,
                         targets, 1, stats_out, stream);
}

int msc_gaussian_sample(const float* mean, const float* log_std, int32_t log_std_rows, float logstd_floor,
                        const float* eps, int64_t n_rows, int32_t k, float* actions, float* logp, float* clipped,
                        msc_stream_t stream) {
  if (!mean || !log_std || !eps || !actions || !logp || !clipped) return set_err(-1, "null argument");
  if (n_rows < 0 || k < 1 || log_std_rows < 1)
    return set_err(-1, "bad shape (n_rows %lld, k %d, log_std_rows %d)", (long long)n_rows, k, log_std_rows);
  HIP_TRY(launch_gauss_sample(mean, log_std, log_std_rows, logstd_floor, eps, n_rows, k, actions, logp, clipped,
                              (hipStream_t)stream));
  return 0;
}

int msc_poisson_draws(const uint64_t* state_host, const double* lam_host, int64_t n_lam, int64_t n,
                      int64_t* out_host, uint64_t* state_out_host) {
  if (!state_host || !lam_host || !out_host) return set_err(-1, "null argument");
  if (n_lam < 1 || n_lam > 4096 || n < 0) return set_err(-1, "bad shape (n_lam %lld, n %lld)", (long long)n_lam, (long long)n);
  std::vector<PtrsConst> pc(n_lam);
  std::vector<double> enlam(n_lam);
  for (int64_t i = 0; i < n_lam; i++) {
    if (!(lam_host[i] > 0.0 && lam_host[i] < 1e6)) return set_err(-1, "lam[%lld]=%g: must be in (0, 1e6)", (long long)i, lam_host[i]);
    pc[i] = ptrs_const_host(lam_host[i]);
    enlam[i] = exp(-lam_host[i]);
  }
  void* mem = nullptr;
  const size_t b_st = 6 * sizeof(uint64_t), b_pc = sizeof(PtrsConst) * n_lam, b_el = sizeof(double) * n_lam,
               b_out = sizeof(int64_t) * (n > 0 ? n : 1);
  if (hipMalloc(&mem, b_st + b_pc + b_el + b_out) != hipSuccess) {
    (void)hipGetLastError();
    return set_err(-2, "hipMalloc failed");
  }
  char* m = (char*)mem;
  int rc = 0;
  if (hipMemcpy(m, state_host, b_st, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(m + b_st, pc.data(), b_pc, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(m + b_st + b_pc, enlam.data(), b_el, hipMemcpyHostToDevice) != hipSuccess ||
      launch_poisson_draws((uint64_t*)m, (const PtrsConst*)(m + b_st), (const double*)(m + b_st + b_pc), n_lam, n,
                           (int64_t*)(m + b_st + b_pc + b_el), 0) != hipSuccess ||
      hipDeviceSynchronize() != hipSuccess ||
      (n > 0 && hipMemcpy(out_host, m + b_st + b_pc + b_el, sizeof(int64_t) * n, hipMemcpyDeviceToHost) != hipSuccess) ||
      (state_out_host && hipMemcpy(state_out_host, m, b_st, hipMemcpyDeviceToHost) != hipSuccess))
    rc = set_err(-2, "poisson draws: %s", hipGetErrorString(hipGetLastError()));
  (void)hipFree(mem);
  return rc;
}

int msc_normal_keyed(float* out, int32_t n_steps, int64_t n_rows, int32_t row_len, int64_t row0, uint64_t seed,
                     uint64_t step0, msc_stream_t stream) {
  if (!out) return set_err(-1, "null argument");
  if (n_steps < 0 || n_rows < 0 || row_len < 1 || row0 < 0)
    return set_err(-1, "bad shape (n_steps %d, n_rows %lld, row_len %d)", n_steps, (long long)n_rows, row_len);
  HIP_TRY(launch_normal_keyed(out, n_steps, n_rows, row_len, row0, seed, step0, (hipStream_t)stream));
  return 0;
}

int64_t msc_meanstd_scratch_doubles(int64_t n_rows, int32_t n_cols) {
  return n_rows >= 1 && n_cols >= 1 ? meanstd_scratch_doubles(n_rows, n_cols) : -1;
}

int msc_meanstd_filter(const float* obs, float* out, int64_t n_rows, int32_t n_cols, const uint8_t* mask,
                       int32_t update, double* state, double* scratch, double clip, double eps,
                       msc_stream_t stream) {
  if (!obs || !out || !state || (update && !scratch)) return set_err(-1, "null argument");
  if (n_rows < 1 || n_cols < 1) return set_err(-1, "bad shape (n_rows %lld, n_cols %d)", (long long)n_rows, n_cols);
  if (!(eps >= 0.0) || !(clip >= 0.0)) return set_err(-1, "eps and clip must be >= 0");
  HIP_TRY(launch_meanstd_filter(obs, out, n_rows, n_cols, mask, update ? 1 : 0, state, scratch, clip, eps,
                                (hipStream_t)stream));
  return 0;
}

int msc_mlp3_w3_layout(int32_t out_dim) { return out_dim >= 1 && out_dim <= 32 ? (mlp3_valu_outputs(out_dim) > 0 ? 1 : 0) : -1; }

static int mlp_sample_args(const msc_gaussian_epilogue* g, int out_dim, MlpSample* sm) {
  if (!g) return 0;
  if (!g->log_std || !g->eps || !g->actions || !g->logp || !g->clipped) return set_err(-1, "null sampling buffer");
  if (g->log_std_rows < 1) return set_err(-1, "log_std_rows %d must be >= 1", g->log_std_rows);
  if (mlp3_valu_outputs(out_dim) == 0)
    return set_err(-1, "sampling epilogue needs the VALU output layer (out_dim %d <= 8)", out_dim);
  *sm = MlpSample{g->log_std, g->log_std_rows, g->logstd_floor, g->eps, g->actions, g->logp, g->clipped};
  return 0;
}

static int mlp3_impl(const float* x, int64_t n_rows, int32_t in_dim, int32_t hidden1, int32_t hidden2, int32_t out_dim,
                     const float* w1p, const float* b1, const float* w2p, const float* b2, const float* w3p,
                     const float* b3, float* out, const float* pre1, int32_t pre1_group,
                     const msc_gaussian_epilogue* sample, msc_stream_t stream) {
  if (pre1 && pre1_group < 1) return set_err(-1, "pre1_group %d must be >= 1", pre1_group);
  // the kernel reads b1 / b2 / pre1 rows as float4
  if (((uintptr_t)b1 | (uintptr_t)b2 | (uintptr_t)pre1 | (uintptr_t)w1p | (uintptr_t)w2p | (uintptr_t)w3p) & 15)
    return set_err(-1, "b1, b2, pre1 and the packed weights must be 16-byte aligned");
  if (!x || !w1p || !b1 || !w2p || !b2 || !w3p || !b3 || (!out && !sample)) return set_err(-1, "null argument");
  if (n_rows < 0 || in_dim < 1 || in_dim > 1024 || out_dim < 1 || out_dim > 32)
    return set_err(-1, "bad shape (n_rows %lld, in_dim %d, out_dim %d)", (long long)n_rows, in_dim, out_dim);
  auto hs = [](int h) { return h == 64 || h == 128 || h == 256 || h == 512; };
  if (!(hs(hidden1) && hs(hidden2)))
    return set_err(-1, "hidden sizes %d, %d: the fused MLP supports [H1, H2] with H1, H2 in {64, 128, 256, 512}", hidden1, hidden2);
  MlpSample sm{};
  if (const int r = mlp_sample_args(sample, out_dim, &sm)) return r;
  HIP_TRY(launch_mlp3_relu(x, n_rows, in_dim, hidden1, hidden2, out_dim, w1p, b1, w2p, b2, w3p, b3, out, pre1,
                           pre1 ? pre1_group : 1, (hipStream_t)stream, sample ? &sm : nullptr));
  return 0;
}

int msc_mlp3_relu_forward(const float* x, int64_t n_rows, int32_t in_dim, int32_t hidden1, int32_t hidden2,
                          int32_t out_dim, const float* w1p, const float* b1, const float* w2p, const float* b2,
                          const float* w3p, const float* b3, float* out, const float* pre1, int32_t pre1_group,
                          msc_stream_t stream) {
  if (!out) return set_err(-1, "null argument");
  return mlp3_impl(x, n_rows, in_dim, hidden1, hidden2, out_dim, w1p, b1, w2p, b2, w3p, b3, out, pre1, pre1_group,
                   nullptr, stream);
}

int msc_mlp3_relu_forward_sampled(const float* x, int64_t n_rows, int32_t in_dim, int32_t hidden1, int32_t hidden2,
                                  int32_t out_dim, const float* w1p, const float* b1, const float* w2p,
                                  const float* b2, const float* w3p, const float* b3, float* out,
                                  const float* pre1, int32_t pre1_group, const msc_gaussian_epilogue* sample,
                                  msc_stream_t stream) {
  if (!sample) return set_err(-1, "null argument");
  return mlp3_impl(x, n_rows, in_dim, hidden1, hidden2, out_dim, w1p, b1, w2p, b2, w3p, b3, out, pre1, pre1_group,
                   sample, stream);
}

static int mlp2_impl(const float* x, int64_t n_rows, int32_t in_dim, int32_t hidden, int32_t out_dim, const float* w1p,
                     const float* b1, const float* w3p, const float* b3, float* out, const float* pre1,
                     int32_t pre1_group, const msc_gaussian_epilogue* sample, msc_stream_t stream) {
  if (pre1 && pre1_group < 1) return set_err(-1, "pre1_group %d must be >= 1", pre1_group);
  if (((uintptr_t)b1 | (uintptr_t)pre1 | (uintptr_t)w1p | (uintptr_t)w3p) & 15)
    return set_err(-1, "b1, pre1 and the packed weights must be 16-byte aligned");
  if (!x || !w1p || !b1 || !w3p || !b3 || (!out && !sample)) return set_err(-1, "null argument");
  if (n_rows < 0 || in_dim < 1 || in_dim > 1024 || out_dim < 1 || out_dim > 32)
    return set_err(-1, "bad shape (n_rows %lld, in_dim %d, out_dim %d)", (long long)n_rows, in_dim, out_dim);
  if (!mlp2_supported(hidden)) return set_err(-1, "hidden size %d: the fused MLP supports multiples of 32 up to 1024", hidden);
  MlpSample sm{};
  if (const int r = mlp_sample_args(sample, out_dim, &sm)) return r;
  HIP_TRY(launch_mlp2_relu(x, n_rows, in_dim, hidden, out_dim, w1p, b1, w3p, b3, out, pre1, pre1 ? pre1_group : 1,
                           (hipStream_t)stream, sample ? &sm : nullptr));
  return 0;
}

int msc_mlp2_relu_forward(const float* x, int64_t n_rows, int32_t in_dim, int32_t hidden, int32_t out_dim,
                          const float* w1p, const float* b1, const float* w3p, const float* b3, float* out,
                          const float* pre1, int32_t pre1_group, msc_stream_t stream) {
  if (!out) return set_err(-1, "null argument");
  return mlp2_impl(x, n_rows, in_dim, hidden, out_dim, w1p, b1, w3p, b3, out, pre1, pre1_group, nullptr, stream);
}

int msc_mlp2_relu_forward_sampled(const float* x, int64_t n_rows, int32_t in_dim, int32_t hidden, int32_t out_dim,
                                  const float* w1p, const float* b1, const float* w3p, const float* b3, float* out,
                                  const float* pre1, int32_t pre1_group, const msc_gaussian_epilogue* sample,
                                  msc_stream_t stream) {
  if (!sample) return set_err(-1, "null argument");
  return mlp2_impl(x, n_rows, in_dim, hidden, out_dim, w1p, b1, w3p, b3, out, pre1, pre1_group, sample, stream);
}

int msc_adv_normalize_grouped(float* adv, int64_t n, int32_t n_groups, const double* stats, msc_stream_t stream) {
  if (!adv || !stats || n < 0) return set_err(-1, "bad argument");
  if (n_groups < 1 || n_groups > 64 || n % n_groups != 0)
    return set_err(-1, "n_groups %d must be in [1, 64] and divide n %lld", n_groups, (long long)n);
  HIP_TRY(launch_adv_normalize(adv, n, n_groups, stats, (hipStream_t)stream));
  return 0;
}

int msc_adv_normalize(float* adv, int64_t n, const double* stats, msc_stream_t stream) {
  return msc_adv_normalize_grouped(adv, n, 1, stats, stream);
}

int msc_env_set_episode_counters(msc_env* env, const int32_t* counters_host) {
  if (!env || !counters_host) return set_err(-1, "null argument");
  const int64_t E = env->c.E;
  for (int64_t i = 0; i < E; i++)
    if (counters_host[i] < 0) return set_err(-1, "episode counter %d of env %lld is negative", counters_host[i], (long long)i);
  HIP_TRY(hipSetDevice(env->device));
  HIP_TRY(hipDeviceSynchronize());
  // episodes generated ahead assumed the old counters: stop (restarts at the next episode start)
  if (const int rc = ea_stop(env, nullptr, true)) return rc;
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(env->s.counter, counters_host, sizeof(int32_t) * E, hipMemcpyHostToDevice));
  return 0;
}

}  // extern "C"
