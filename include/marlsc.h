/*
 * marlsc.h -- C ABI of the MI355X-native vectorised supply-chain environment (libmarlsc.so).
 *
 * Drop-in boundary for the reference's env hot path. One `msc_env` handle owns E independent
 * copies of the reference's `InventoryEnvironment` (src/environment/envs/multi_env.py:38)
 * resident in HBM and steps them in lockstep on one GPU. Entry points and the reference
 * interface each one replaces:
 *
 *   msc_env_create   <- InventoryEnvironment.__init__(env_config, seed, env_meta)   multi_env.py:58-190
 *                       + per-env seeds of the RLlib env factory
 *                         SeedManager.derive_env_seed(base, worker_index, env_index)  seed_manager.py:165-186
 *                         (called from src/algorithms/base.py:413-419)
 *   msc_env_reset    <- InventoryEnvironment.reset(seed=None, options=None)          multi_env.py:192-251
 *                       (SeedManager.advance_episode / update_root_seed, seed_manager.py:100-136)
 *   msc_env_step     <- InventoryEnvironment.step(actions)                            multi_env.py:253-366
 *                       (the five components: demand_sampler.py:105-163 / :214-261,
 *                        demand_allocator.py:118-217, lead_time_sampler.py:97-108 / :169-197,
 *                        lost_sales_handler.py:71-210, reward_calculator.py:96-190)
 *                       plus RLlib's reset-after-truncation of the EnvRunner loop.
 *   msc_env_obs_flat <- the flat per-agent observation  local_i || concat_j local_j   multi_env.py:548-575
 *   msc_gae          <- RLlib 2.52.1 GAE + advantage standardisation (external to the reference;
 *                       enabled at src/algorithms/mappo.py:154-156)
 *
 * Conventions
 *   - Return value 0 = OK, negative = error; msc_last_error() gives a thread-local message.
 *   - All array arguments of msc_env_step / msc_env_reset / msc_gae are DEVICE pointers
 *     (e.g. torch data_ptr()) unless the parameter name ends in `_host`.
 *   - Every call is stream-ordered on the given hipStream_t (pass 0 for the null stream); no call
 *     synchronises the device except msc_env_create / msc_env_destroy / msc_env_read_state /
 *     msc_env_save_state / msc_env_load_state / msc_env_check / msc_env_set_timing /
 *     msc_env_read_timing.
 *   - The library owns the env state buffers; callers own every I/O buffer.
 *   - One handle per stream / host thread; a handle is not thread-safe (like the reference object).
 *   - Layouts are row-major: actions [E][W][K] f32, obs [E][W][L] f32, rewards [E][W].
 */
#ifndef MARLSC_H
#define MARLSC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct msc_env msc_env;
typedef struct ihipStream_t* msc_stream_t; /* == hipStream_t */

#define MSC_ABI_VERSION 2
#define MSC_MAX_W 32   /* warehouses (agents) per env (step kernels loop warehouses over <= 16 waves above 16) */
#define MSC_MAX_K 16   /* SKUs (above 8: the sequential demand sampler and the group allocator) */
#define MSC_MAX_R 4096 /* demand regions */
#define MSC_HISTORY 5  /* rolling window, multi_env.py:147 */
#define MSC_ORDER_CAP_MAX (1 << 24) /* Poisson order records per env and step: sum(lambda_orders) + 12 sqrt(.) + 64 */

/* Component `type` strings of the reference's registries (src/environment/registry.py:300-308). */
enum msc_demand_type   { MSC_DEMAND_POISSON = 0, MSC_DEMAND_EMPIRICAL = 1 };
enum msc_action_type   { MSC_ACTION_DIRECT = 0, MSC_ACTION_DEMAND_CENTERED = 1, MSC_ACTION_BASE_STOCK = 2 };
enum msc_init_type     { MSC_INIT_UNIFORM = 0, MSC_INIT_CUSTOM = 1, MSC_INIT_ZERO = 2 };
enum msc_lead_type     { MSC_LEAD_FIXED = 0, MSC_LEAD_STOCHASTIC = 1 };
enum msc_lost_type     { MSC_LOST_CLOSEST = 0, MSC_LOST_SHIPMENT = 1, MSC_LOST_COST = 2 };
enum msc_scope         { MSC_SCOPE_AGENT = 0, MSC_SCOPE_TEAM = 1 };
enum msc_obs_norm      { MSC_OBS_OFF = 0, MSC_OBS_RATIO = 1, MSC_OBS_MEANSTD = 2 };

/* Feature toggles (FeatureConfig, src/config/schema.py:595-639); order = block order of
 * _build_local_obs (multi_env.py:620-695). */
enum msc_feature_bits {
  MSC_F_INVENTORY = 1u << 0,            MSC_F_INVENTORY_AGG = 1u << 1,
  MSC_F_PIPELINE = 1u << 2,             MSC_F_PIPELINE_AGG = 1u << 3,
  MSC_F_INCOMING_HOME = 1u << 4,        MSC_F_INCOMING_HOME_AGG = 1u << 5,
  MSC_F_SHIPPED_HOME = 1u << 6,
  MSC_F_SHIPPED_AWAY = 1u << 7,         MSC_F_SHIPPED_AWAY_AGG = 1u << 8,
  MSC_F_STOCKOUT = 1u << 9,
  MSC_F_ROLLING_MEAN = 1u << 10,        MSC_F_ROLLING_MEAN_AGG = 1u << 11,
  MSC_F_FORECAST = 1u << 12,            MSC_F_FORECAST_AGG = 1u << 13,
  MSC_F_DAYS_OF_SUPPLY = 1u << 14,
  MSC_F_NET_POSITION = 1u << 15,
  MSC_F_DEMAND_VARIABILITY = 1u << 16,
  MSC_F_DEMAND_HISTORY = 1u << 17
};

/* Environment descriptor: the reference's EnvironmentConfig + env_meta flattened to plain
 * host arrays (all HOST pointers; copied by msc_env_create). Shapes use W = n_warehouses,
 * K = n_skus, R = n_regions. */
typedef struct msc_env_desc {
  int32_t abi_version;                 /* = MSC_ABI_VERSION */
  int32_t n_warehouses, n_skus, n_regions, episode_length;

  int32_t action_type;                 /* msc_action_type */
  const double* action_param;          /* [K]: max_order_quantities | max_quantity_adjustment | max_stock_level */

  int32_t init_type;                   /* msc_init_type */
  int32_t init_min, init_max;          /* uniform: integers(min, max+1, (W,K)) (multi_env.py:522-525) */
  const int32_t* init_values;          /* custom: [W*K] */

  int32_t holding_per_sku;             /* 1: holding_cost is [K]; 0: scalar x sku_weights */
  const double* holding_cost;
  int32_t penalty_per_sku;
  const double* penalty_cost;
  const double* sku_weights;           /* [K] */
  const double* distances;             /* [W*R] */
  const double* outbound_fixed;        /* [W*R] */
  const double* outbound_variable;     /* [W*R] */
  const double* inbound_fixed;         /* [W*K] */
  const double* inbound_variable;      /* [W*K] */

  int32_t demand_type;                 /* msc_demand_type */
  const double* lambda_orders;         /* poisson: [R] (scalar mode: broadcast by the caller) */
  const double* probability_skus;      /* [R] */
  const double* lambda_quantity;       /* [R*K] */
  /* empirical trace, CSR over the sorted available timesteps (demand_sampler.py:199-261):
   * orders of trace row i are [trace_offsets[i], trace_offsets[i+1]), each with a region and
   * K quantities, already grouped/sorted by (region_id, order_id). */
  int32_t trace_n_rows;
  const int64_t* trace_offsets;        /* [trace_n_rows + 1] */
  const int32_t* trace_regions;        /* [n_trace_orders] */
  const int32_t* trace_quantities;     /* [n_trace_orders * K] */

  int32_t max_splits;                  /* greedy allocator ("default" -> W-1) */

  int32_t lead_type;                   /* msc_lead_type */
  const int32_t* expected_lead_times;  /* [W*K] */
  int32_t max_dev_per_sku;             /* 1: max_deviation is [K] (SKU-major draws); 0: scalar */
  const int32_t* max_deviation;

  int32_t lost_type;                   /* msc_lost_type */
  double lost_alpha;                   /* softmax temperature for MSC_LOST_COST */

  int32_t reward_scope;                /* msc_scope */
  double reward_scale;

  uint32_t feature_flags;              /* msc_feature_bits */
  int32_t include_warehouse_id;        /* one-hot prefix (parameter sharing) */
  int32_t obs_norm;                    /* msc_obs_norm */
  const float* obs_mean;               /* [n_features] for MSC_OBS_MEANSTD */
  const float* obs_std;
  int32_t num_eval_episodes;           /* <= 0: no eval cycling (multi_env.py:164-168, 220-224) */
  /* Episode-ahead Poisson demand (no reference counterpart: a scheduling choice, results are
   * identical either way): -1 automatic (on for <= 8,192 envs), 0 off (short-lived envs, e.g. the
   * evaluation envs), n > 0 at most n slots (future episodes per env). Its buffers take at most
   * ea_mem_fraction (<= 0: 0.25) of the device memory free at create time; fewer slots, or none,
   * when the budget binds (msc_env_dims reports the slots chosen). */
  int32_t episode_ahead;
  double ea_mem_fraction;
} msc_env_desc;

/* Optional per-step diagnostics = the reference's collect_step_info dict (multi_env.py:330-361).
 * DEVICE pointers, any may be NULL. */
typedef struct msc_step_info {
  int32_t* inventory_before;           /* [E][W][K] */
  int32_t* pending_total;              /* [E][W][K] */
  int32_t* order_quantities;           /* [E][W][K] */
  int32_t* demand_per_region;          /* [E][R][K] */
  int32_t* fulfilled_per_warehouse;    /* [E][W][K] */
  int32_t* unfulfilled_demands;        /* [E][R][K] */
  int32_t* shipment_counts;            /* [E][W][R] */
  int32_t* shipment_quantities;        /* [E][W][R] */
  int32_t* shipment_quantities_by_sku; /* [E][W][R][K] */
  int32_t* lost_order_counts;          /* [E][R] */
  int32_t* n_orders;                   /* [E] */
  double* lost_sales;                  /* [E][W][K] */
  double* costs;                       /* [E][4][W]: holding, penalty, outbound, inbound */
} msc_step_info;

/* Create E = n_envs environments on `device`. Env i gets root seed
 *   env_seeds_host[i]                                    if env_seeds_host != NULL, else
 *   SeedSequence([base_seed, worker_index, env_index_offset + i]).generate_state(1)[0].
 * Nothing is reset yet: call msc_env_reset before the first step. */
int msc_env_create(const msc_env_desc* desc, int device, int64_t n_envs, uint32_t base_seed,
                   uint32_t worker_index, int64_t env_index_offset, const uint32_t* env_seeds_host,
                   msc_env** out);
void msc_env_destroy(msc_env* env);

/* Sizes of the I/O tensors, and the episode-ahead slots per env chosen at create time (0: off). */
int msc_env_dims(const msc_env* env, int64_t* n_envs, int32_t* n_agents, int32_t* n_skus,
                 int32_t* n_regions, int32_t* local_obs_dim, int32_t* n_features,
                 int32_t* max_expected_lead_time, int32_t* ea_slots);

/* Diagnostic (no reference counterpart: the reference has one code path): the kernels this handle
 * runs, chosen at create time from its shape and the MSC_* knobs. Writes up to n of
 * {alloc (0 lane, 1 group, 2 scan), envs sorted by order count, phase A fused, phase C fused,
 *  group kernel cost tables in LDS, lane-group width, episode-ahead slots, demand (0 unit parser,
 *  5 park4, 7 split parser, 8 f32-ring parser, 9 demand_v3), equal sampler parameters (UNI)}; returns the
 *  count written. */
int msc_env_kernel_choice(const msc_env* env, int32_t* out, int32_t n);

/* Kernel-form options of a handle that change no result (diagnostic / tuning; no reference
 * counterpart). MSC_OPT_STEP_C_FORM: the waves per SIMD the observation kernel is compiled for, 5
 * (default: beside the pipelined demand kernel) or 4 (no register spills; the rollout collector's
 * choice, with policy kernels between steps). MSC_OPT_ALLOC_PRIO_SPLIT: the share, in 16ths of its
 * busiest env's orders, that each one-env-per-lane allocation wave runs above the pipelined demand
 * kernel's parser (s_setprio 3) before it drops below it (1 .. 16; default 12; 16: the whole kernel,
 * the rollout collector's choice). Returns 0, or < 0 for an unknown key / value. */
#define MSC_OPT_STEP_C_FORM 1
#define MSC_OPT_ALLOC_PRIO_SPLIT 2
int msc_env_set_option(msc_env* env, int32_t key, int32_t value);

#define MSC_RESET_EVAL_RESTART 1  /* reset(seed=...) of a construction-seeded eval env: counter -> 0 */

/* Reset envs with mask[i] != 0 (mask == NULL: all). new_root_seeds == NULL follows the
 * construction-seeded path (advance_episode, with eval cycling); otherwise
 * update_root_seed(new_root_seeds[i]) (reset(seed=X) of an env created without a seed).
 * Writes the reset observation of every reset env into obs [E][W][L] (may be NULL). */
int msc_env_reset(msc_env* env, const uint8_t* mask, const uint32_t* new_root_seeds, int32_t flags,
                  float* obs, msc_stream_t stream);

/* One step of every env. actions [E][W][K] in [-1, 1]. Outputs obs [E][W][L] (local obs of
 * every agent), rewards [E][W] (f32, and optionally f64), truncated [E]. An env whose episode
 * ends is reset in the same call (RLlib's EnvRunner semantics): its terminal observation goes
 * to final_obs (if non-NULL) and obs receives the first observation of the next episode. */
int msc_env_step(msc_env* env, const float* actions, float* obs, float* rewards,
                 double* rewards_f64, uint8_t* truncated, float* final_obs,
                 const msc_step_info* info, msc_stream_t stream);

/* Optional split of msc_env_step: run the demand sampler of the NEXT step now (it depends only
 * on each env's own RNG stream, not on actions), e.g. on a side stream while the policy forward
 * runs. The following msc_env_step consumes these orders instead of generating them.
 * No-op for the empirical sampler. */
int msc_env_generate_demand(msc_env* env, msc_stream_t stream);

/* Automatic demand pipelining (default on for the Poisson sampler): msc_env_step also launches the
 * NEXT step's demand generation on a library-owned side stream, concurrent with the current step
 * kernel (skipped across episode boundaries and after masked resets). Results are identical either
 * way; 0 disables it (every step then runs demand + step back to back on the caller's stream). */
int msc_env_set_pipelining(msc_env* env, int32_t enabled);

/* Episode-ahead demand on / off at run time (no reference counterpart; results are identical either
 * way): 0 switches a handle whose EA buffers exist to per-step pipelined demand from the current step
 * on (e.g. a rollout whose policy kernels lose more to the background generation than the step
 * gains), != 0 lets it restart at the next common episode start. No-op without EA buffers.
 * Synchronises the device. */
int msc_env_set_episode_ahead(msc_env* env, int32_t enabled);

/* Wave priority of the step chain (no reference counterpart: a scheduling hint). With enabled != 0
 * the phase-A and phase-C kernels of msc_env_step run at s_setprio 3, like the allocation kernel,
 * ahead of the pipelined demand kernel of the next step. For callers that run their own work between
 * steps (a rollout's policy forward): the env step is then their critical path and the next step's
 * demand has slack. Default 0 (env-only stepping: the demand kernel is the critical path).
 * Synchronises the device. Results are identical either way. */
int msc_env_set_chain_priority(msc_env* env, int32_t enabled);

/* Per-launch device durations of the production path (for roofline accounting): with max_steps > 0
 * the next max_steps calls of msc_env_step bracket their demand launch and their step launch (the
 * step kernels of that call) with HIP events on the stream each runs on -- the caller's stream, or
 * the side stream for pipelined demand. 0 disables and frees the events. No reference
 * counterpart (instrumentation only). */
int msc_env_set_timing(msc_env* env, int32_t max_steps);
/* Mean device duration in ms of the recorded demand / step launches and their counts (waits for
 * the recorded events). */
int msc_env_read_timing(msc_env* env, double* demand_ms, double* step_ms, int64_t* n_demand,
                        int64_t* n_step);
/* Episode-ahead demand (few envs per GPU: E <= 8192 by default, MSC_EA=0|1 forces it): while
 * every env sits at the same timestep, the Poisson orders of whole future episodes are drawn on a
 * library-owned stream (an episode's demand depends only on its SeedSequence([root, counter]) seed,
 * src/utils/seed_manager.py:100-120, never on actions); each env step then reads its episode's
 * slot. Results are identical with and without it. Mean device duration of the episode generation
 * launches timed since msc_env_set_timing (one launch = one episode of every env in steady state),
 * their count, the slots per env (0: EA off), whether the current episode reads a slot, and the mean
 * env-steps of demand one timed launch generated (slots x steps x envs; for roofline accounting). */
int msc_env_read_timing_ea(msc_env* env, double* ea_ms, int64_t* n_ea, int32_t* slots, int32_t* active,
                           double* env_steps_per_launch);

/* Demand work issued by the handle since create (monotonic; differences bracket a timed window):
 * episode-ahead generation launches (chunks) and the env-steps of demand they drew, per-step demand
 * launches (E env-steps each), and msc_env_step calls. Everything issued before a device-wide
 * synchronize has finished after it. */
int msc_env_work_counters(const msc_env* env, int64_t* ea_launches, double* ea_env_steps, int64_t* demand_launches,
                          int64_t* steps);

/* Episode-ahead memory of the handle: the budget computed at create time (bytes; 0 when EA was not
 * requested) and the bytes allocated for the slots (0: EA off). */
int msc_env_ea_memory(const msc_env* env, int64_t* budget_bytes, int64_t* allocated_bytes);

/* Flat per-agent observation of the reference [E][W][L*(1+W)] = local_w || local_0..local_{W-1},
 * from the compact obs [E][W][L]. */
int msc_env_obs_flat(const msc_env* env, const float* obs, float* flat, msc_stream_t stream);

/* Host copies of the parity-relevant state (synchronous). Any pointer may be NULL.
 *   inventory [E][W][K] i32, timestep [E], episode_counter [E],
 *   rng [E][2][6] u64: {demand, lead_time} x {state_hi, state_lo, inc_hi, inc_lo, has_uint32, uinteger} */
int msc_env_read_state(const msc_env* env, int32_t* inventory_host, int32_t* timestep_host,
                       int32_t* episode_counter_host, uint64_t* rng_host);

/* Opaque checkpoint of the whole device state (synchronous): size query, save, restore. */
int64_t msc_env_state_bytes(const msc_env* env);
int msc_env_save_state(const msc_env* env, void* buf_host);
int msc_env_load_state(msc_env* env, const void* buf_host);

/* Set SeedManager._episode_counter of every env (counters_host [E], host, >= 0; synchronous).
 * Replaces the caller-side write `seed_manager._episode_counter = 0` (src/algorithms/base.py:81):
 * the next construction-seeded reset of env i derives its episode root from
 * SeedSequence([root_i, counters_host[i]]) (seed_manager.py:100-120), so E eval envs created with
 * the same root and counters 0..E-1 replay the reference eval env's episodes 0..E-1, which it runs
 * one after another with eval cycling (multi_env.py:220-224). */
int msc_env_set_episode_counters(msc_env* env, const int32_t* counters_host);

/* Synchronise and report device-side errors (order-buffer overflow, ...). */
int msc_env_check(msc_env* env);

/* Advantage estimation over T steps x N sequences (layout [T][N], time-major):
 *   delta_t = r_t + gamma * V_{t+1} * (1 - term_t) - V_t
 *   A_t     = delta_t + gamma * lam * (1 - term_t) * (1 - trunc_t) * A_{t+1}
 * where V_{t+1} = next_values[t] if trunc_t (bootstrap from the terminal obs) else values[t+1];
 * values[T] (row T of `values`, [T+1][N]) bootstraps the last row. targets = A + V.
 * stats_out (device f64[3]) receives {sum A, sum A^2, count} (accumulated, caller zeroes it)
 * for the cross-rank advantage standardisation. */
int msc_gae(const float* rewards, const float* values, const float* next_values,
            const uint8_t* terminated, const uint8_t* truncated, int64_t n_seq, int32_t T,
            float gamma, float lam, float* advantages, float* targets, double* stats_out,
            msc_stream_t stream);

/* In-place (A - mean) / max(1e-4, std) using stats {sum, sumsq, count} (device f64[3]). */
int msc_adv_normalize(float* advantages, int64_t n, const double* stats, msc_stream_t stream);

/* Per-module variants (RLlib's GAE connector standardises the advantages of every module of a
 * multi-agent batch on its own; with one policy per agent that is one group per agent):
 * sequence n belongs to group n % n_groups (the rollout's sequences are env * W + agent, so
 * n_groups = W gives one group per agent); n_groups in [1, 64] must divide n_seq.
 * stats_out is device f64 [n_groups][3] {sum A, sum A^2, count} (accumulated, caller zeroes it);
 * msc_adv_normalize_grouped standardises element i of the [T][n_seq] advantages with the
 * statistics of group i % n_groups. n_groups = 1 is msc_gae / msc_adv_normalize. */
int msc_gae_grouped(const float* rewards, const float* values, const float* next_values,
                    const uint8_t* terminated, const uint8_t* truncated, int64_t n_seq, int32_t T,
                    float gamma, float lam, float* advantages, float* targets, int32_t n_groups,
                    double* stats_out, msc_stream_t stream);
int msc_adv_normalize_grouped(float* advantages, int64_t n, int32_t n_groups, const double* stats,
                              msc_stream_t stream);

/* Rollout action sampling (RLlib TorchDiagGaussian, rlmodules/base.py:480-557) over N rows of K:
 *   std = exp(max(log_std[n % log_std_rows][k], logstd_floor)) (one shared row, or one per agent
 *   with rows n = env * W + agent), actions = mean + std * eps (eps: standard normal draws),
 *   logp[n] = sum_k -(a - mean)^2 / (2 std^2) - log(std) - log(sqrt(2 pi)),
 *   clipped = clip(actions, -1, 1) (what the env receives; the reference's EnvRunner clips too).
 * All f32 device buffers: mean / eps / actions / clipped [N][K], log_std [log_std_rows][K], logp [N]. */
int msc_gaussian_sample(const float* mean, const float* log_std, int32_t log_std_rows, float logstd_floor,
                        const float* eps, int64_t n_rows, int32_t k, float* actions, float* logp,
                        float* clipped, msc_stream_t stream);

/* Standard-normal rollout noise keyed by global env id (no reference counterpart: RLlib draws it from
 * torch's global generator per env runner). out [n_steps][n_rows][row_len] f32: element (s, row, j)
 * depends only on (seed, row0 + row, step0 + s, j) -- Philox4x32-10, Box-Muller -- so the noise of a
 * global env is the same whichever rank owns it and however the envs are sharded. */
int msc_normal_keyed(float* out, int32_t n_steps, int64_t n_rows, int32_t row_len, int64_t row0, uint64_t seed,
                     uint64_t step0, msc_stream_t stream);

/* RLlib's MeanStdFilter env-to-module connector (obs_normalization "meanstd", the reference's
 * src/algorithms/mappo.py:170-171 / ippo.py:173-175; evaluation applies it with update=False,
 * base.py:131-140, :176-177), one RunningStat per column (agent x feature) of obs [n_rows][n_cols]:
 *   update != 0: every row (in row order; only rows with mask[row] != 0 when mask is given) is
 *   pushed (n += 1; M += (x - M) / n; S += (x - M_old)^2 (n - 1) / n) and normalised with the
 *   statistics that include it; update == 0: normalised with the current statistics only.
 *   out = clip((x - M) / (sqrt(var) + eps), -clip, clip) with var = S / (n - 1) (M^2 while n <= 1);
 *   clip = 0 disables clipping. out may alias obs.
 * state (device f64 [4 + 4 n_cols]): {n, buffer n, 0, 0, M[n_cols], S[n_cols], buffer M[n_cols],
 * buffer S[n_cols]}; the buffer collects the pushes since the caller last cleared it (RLlib's filter
 * buffer, merged across env runners by RunningStat.update). scratch: device f64
 * [msc_meanstd_scratch_doubles(n_rows, n_cols)] (only with update). Rows are pushed sequentially
 * within segments of ceil(n_rows / 64) rows and segment statistics combined by Chan's merge, so
 * results match a sequential update to rounding (f64). */
int64_t msc_meanstd_scratch_doubles(int64_t n_rows, int32_t n_cols);
int msc_meanstd_filter(const float* obs, float* out, int64_t n_rows, int32_t n_cols, const uint8_t* mask,
                       int32_t update, double* state, double* scratch, double clip, double eps,
                       msc_stream_t stream);

/* Rollout policy inference (replaces the actor's torch layer sequence in the EnvRunner's
 * _forward_inference, rlmodules/base.py:480-557, for MLPArchitecture.build networks,
 * architectures/mlp.py:14-60): out = W3 relu(W2 relu(W1 x + b1) + b2) + b3 for n_rows rows of
 * in_dim floats, in one kernel on the f32 MFMA (hidden activations stay in registers).
 * hidden1, hidden2 in {64, 128, 256, 512} (equal or not); out_dim <= 32. Weights are passed in the packed fragment
 * order the kernel streams (marlsc/mlp.py:pack_mlp3 builds them from the torch [out, in] matrices):
 *   w1p [hidden1/32][ceil(ceil(in_dim/2)/4)][64][4], w2p [hidden2/32][hidden1/8][64][4], and w3p either
 *   [hidden2/8][64][4] (MFMA output layer) or [hidden2/2][2][8] (VALU output layer, out_dim <= 8):
 *   msc_mlp3_w3_layout(out_dim) says which (0 / 1; -1 for an unsupported out_dim);
 * biases b1 [hidden1], b2 [hidden2], b3 [out_dim] as in torch. x [n_rows][in_dim], out [n_rows][out_dim]:
 * f32 device buffers; stream-ordered. pre1 (optional, [n_rows / pre1_group][hidden1]) is added to
 * the first layer's pre-activation of every row n as pre1[n / pre1_group]: the MAPPO critic's
 * first layer over local_w || global (multi_env.py:566-573) is W_local x_w + (W_global g_env + b1),
 * with the global block computed once per env (pre1_group = agents). */
int msc_mlp3_w3_layout(int32_t out_dim);
int msc_mlp3_relu_forward(const float* x, int64_t n_rows, int32_t in_dim, int32_t hidden1, int32_t hidden2,
                          int32_t out_dim, const float* w1p, const float* b1, const float* w2p, const float* b2,
                          const float* w3p, const float* b3, float* out, const float* pre1, int32_t pre1_group,
                          msc_stream_t stream);

/* The one-hidden-layer form out = W3 relu(W1 x + b1) + b3 (MLPArchitecture.build with
 * hidden_sizes [H]: the reference IPPO actor / critic [256], config_files/algorithms/ippo.yaml:46,52,
 * and the test configs' [128] / [1024] heads), hidden a multiple of 32 up to 1024, out_dim <= 32:
 * the hidden layer is produced 256 units at a time and folded into the outputs in registers.
 * w1p as msc_mlp3_relu_forward's (hidden1 = hidden), w3p as its output layer with hidden2 = hidden
 * (layout by msc_mlp3_w3_layout(out_dim)); pre1 / pre1_group as there. */
int msc_mlp2_relu_forward(const float* x, int64_t n_rows, int32_t in_dim, int32_t hidden, int32_t out_dim,
                          const float* w1p, const float* b1, const float* w3p, const float* b3, float* out,
                          const float* pre1, int32_t pre1_group, msc_stream_t stream);

/* The actor forward and the rollout's action sampling in one launch: msc_mlp3_relu_forward /
 * msc_mlp2_relu_forward followed, while the out_dim means of each row are still in registers, by
 * msc_gaussian_sample's arithmetic (bit-identical to the separate call) into sample->actions /
 * logp / clipped. out (the means) may be NULL. Needs the VALU output layer (out_dim <= 8,
 * msc_mlp3_w3_layout(out_dim) == 1). Replaces the EnvRunner's _forward_inference -> TorchDiagGaussian
 * sample pair (rlmodules/base.py:480-557). */
typedef struct msc_gaussian_epilogue {
  const float* log_std;   /* [log_std_rows][out_dim]: row n % log_std_rows applies to row n */
  int32_t log_std_rows;
  float logstd_floor;
  const float* eps;       /* [n_rows][out_dim] standard-normal draws */
  float* actions;         /* [n_rows][out_dim] */
  float* logp;            /* [n_rows] */
  float* clipped;         /* [n_rows][out_dim] */
} msc_gaussian_epilogue;
int msc_mlp3_relu_forward_sampled(const float* x, int64_t n_rows, int32_t in_dim, int32_t hidden1, int32_t hidden2,
                                  int32_t out_dim, const float* w1p, const float* b1, const float* w2p,
                                  const float* b2, const float* w3p, const float* b3, float* out,
                                  const float* pre1, int32_t pre1_group, const msc_gaussian_epilogue* sample,
                                  msc_stream_t stream);
int msc_mlp2_relu_forward_sampled(const float* x, int64_t n_rows, int32_t in_dim, int32_t hidden, int32_t out_dim,
                                  const float* w1p, const float* b1, const float* w3p, const float* b3, float* out,
                                  const float* pre1, int32_t pre1_group, const msc_gaussian_epilogue* sample,
                                  msc_stream_t stream);

/* Utility: numpy's Generator.poisson on the device (synchronous; the env's own sampler, exposed for
 * known-answer tests): n draws with the rates lam_host[i % n_lam] (random_poisson: multiplication
 * method below 10, PTRS at or above, numpy/random/src/distributions/distributions.c) from the PCG64
 * state_host[6] {state_hi, state_lo, inc_hi, inc_lo, has_uint32, uinteger} (the layout of
 * msc_env_read_state's rng); draws -> out_host [n], the final state -> state_out_host (may be NULL). */
int msc_poisson_draws(const uint64_t* state_host, const double* lam_host, int64_t n_lam, int64_t n,
                      int64_t* out_host, uint64_t* state_out_host);

/* Utility: SeedSequence(words).generate_state(1, uint32)[0] (numpy-compatible), on the host. */
uint32_t msc_seedseq_u32(const uint32_t* words, int32_t n_words);

const char* msc_last_error(void);
int msc_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* MARLSC_H */
