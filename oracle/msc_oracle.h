/*
 * msc_oracle.h -- TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline), never shipped or
 * linked by the product library. Plain-C restatement of the reference's env hot path:
 *   InventoryEnvironment.reset/step     src/environment/envs/multi_env.py:192-366
 *   components                          src/environment/components/ (all five)
 *   SeedManager                         src/utils/seed_manager.py
 *   numpy 2.2 Generator pieces used by them (SeedSequence, PCG64, random, poisson, integers).
 * Pinned by the tests/golden fixtures, which were produced by importing the reference itself
 * (tests/golden/make_golden.py). Uses the product's public descriptor (include/marlsc.h) only
 * as a plain data struct.
 */
#ifndef MSC_ORACLE_H
#define MSC_ORACLE_H
#include <stdint.h>
#include "../include/marlsc.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_env orc_env;

orc_env* orc_create(const msc_env_desc* d, int64_t n_envs, uint32_t base_seed, uint32_t worker_index,
                    int64_t env_index_offset, const uint32_t* env_seeds);
void orc_destroy(orc_env* e);
const char* orc_error(void);
void orc_dims(const orc_env* e, int32_t* local_obs_dim, int32_t* n_features, int32_t* max_lead);

/* Same semantics as msc_env_reset / msc_env_step, HOST pointers (info fields too). */
void orc_reset(orc_env* e, const uint8_t* mask, const uint32_t* new_root_seeds, int32_t flags, float* obs);
void orc_step(orc_env* e, const float* actions, float* obs, double* rewards, uint8_t* truncated,
              float* final_obs, const msc_step_info* info, int32_t n_threads);
void orc_read_state(const orc_env* e, int32_t* inventory, int32_t* timestep, int32_t* episode_counter,
                    uint64_t* rng);

/* numpy RNG known-answer hooks (tests/golden/rng_streams.npz). */
uint32_t orc_seedseq_u32(const uint32_t* words, int32_t n_words);
void orc_seedseq_state(const uint32_t* entropy, int32_t n_entropy, const uint32_t* spawn_key,
                       int32_t n_spawn, uint32_t* out, int32_t n_words);
typedef struct orc_rng { uint64_t w[6]; } orc_rng; /* state_hi, state_lo, inc_hi, inc_lo, has32, u32 */
void orc_rng_seed(orc_rng* r, const uint32_t* entropy, int32_t n_entropy, const uint32_t* spawn_key, int32_t n_spawn);
uint64_t orc_rng_next64(orc_rng* r);
double orc_rng_random(orc_rng* r);
int64_t orc_rng_poisson(orc_rng* r, double lam);
void orc_rng_poisson_n(orc_rng* r, const double* lam, int64_t n_lam, int64_t n, int64_t* out);
int64_t orc_rng_integers(orc_rng* r, int64_t low, int64_t high_exclusive);

#ifdef __cplusplus
}
#endif
#endif
