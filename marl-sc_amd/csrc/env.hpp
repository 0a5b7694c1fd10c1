// env.hpp -- internal layout of libmarlsc's device-resident environments (not part of the ABI).
//
// HBM layout: every per-env state field is structure-of-arrays with the env index fastest,
// `field[i][E]`, so a wavefront (64 envs, one per lane) touching the same (warehouse, SKU)
// index i issues one coalesced 256-B access. Static tables (costs, rates, lead times) are
// read-only and shared by all envs (L2 / Infinity-Cache resident).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/marlsc.h"

namespace msc {

constexpr int BS = 64;          // threads per block of the env kernels (one wave: one env per lane)
constexpr int MAX_RING = 64;    // pending-order ring slots (max actual lead time + 1)

struct EnvConst {
  int32_t W, K, R, T, Lmax, RING, F, L, order_cap;
  int32_t action_type, lead_type, dev_per_sku, lost_type, scope, norm, wid, num_eval, max_wh;
  int32_t demand_type, init_type, init_min, init_max, hold_per_sku, pen_per_sku, tr_rows;
  uint32_t flags;
  int64_t E;
  double scale, alpha, hold_scalar, pen_scalar;
  const double* act_param;   // [K]
  const int32_t* init_vals;  // [W*K]
  const double* hold;        // [K]
  const double* pen;         // [K]
  const double* skw;         // [K]
  const double* ofT;         // [R][W] outbound fixed (transposed: one region's row is contiguous)
  const double* ovT;         // [R][W] outbound variable
  const double* inF;         // [W*K]
  const double* inV;         // [W*K]
  const double* enlam_o;     // [R]   exp(-lambda_orders) from the host libm
  const double* p_sku;       // [R]
  const double* enlam_q;     // [R*K] exp(-lambda_quantity)
  const int32_t* elt;        // [W*K] expected lead times
  const int32_t* maxdev;     // [K] or [1]
  const uint32_t* home_mask; // [R] bit w set <=> region r is warehouse w's home region
  const int32_t* closest;    // [R] closest warehouse of each region
  const float* obs_mean;     // [F]
  const float* obs_std;      // [F]
  const int64_t* tr_off;     // [tr_rows + 1]
  const uint4* tr_rec;       // [n_trace_orders][NV] packed order records
};

struct EnvState {
  int32_t* inv;        // [WK][E]
  int32_t* ring_q;     // [WK][RING][E] pending quantity by order time mod RING (0 = empty)
  uint8_t* ring_l;     // [WK][RING][E] actual lead time of that order (stochastic lead only)
  int32_t* hist;       // [5][WK][E]    incoming home demand of step tau at slot tau % 5
  int32_t* inc;        // [WK][E]       incoming home demand of the last step
  float* fc;           // [WK][E]       EMA demand forecast (f32, multi_env.py:789-793)
  uint64_t* rng;       // [2][4][E]     {demand, lead} x {s_hi, s_lo, i_hi, i_lo}
  uint32_t* rbuf;      // [2][2][E]     {demand, lead} x {has32, u32}
  int32_t* t;          // [E] timestep
  int32_t* counter;    // [E] SeedManager._episode_counter
  uint32_t* orig_root; // [E] SeedManager._original_root_seed
  uint32_t* root;      // [E] SeedManager.root_seed
  int32_t* emp_start;  // [E] EmpiricalDemandSampler window start row (-1: not drawn)
  uint4* orders;       // [order_cap][E][NV] per-step order records (Poisson sampler output)
  int32_t* n_orders;   // [E]
  uint32_t* err;       // [1] device error bits
};

struct StepIO {
  const float* actions;  // [E][W][K]
  float* obs;            // [E][W][L]
  float* rew;            // [E][W]
  double* rew64;         // [E][W] or null
  uint8_t* trunc;        // [E]
  float* final_obs;      // [E][W][L] or null
  msc_step_info info;    // device pointers or nulls
  int32_t has_info;
};

constexpr uint32_t ERR_ORDER_OVERFLOW = 1u;

// launchers (env_kernels.hip)
hipError_t launch_reset(const EnvConst& c, const EnvState& s, const uint8_t* mask, const uint32_t* new_roots,
                        int32_t flags, float* obs, hipStream_t st);
hipError_t launch_step(const EnvConst& c, const EnvState& s, const StepIO& io, bool gen_demand, hipStream_t st);
hipError_t launch_demand(const EnvConst& c, const EnvState& s, hipStream_t st);
hipError_t launch_obs_flat(const EnvConst& c, const float* obs, float* flat, hipStream_t st);
size_t step_lds_bytes(const EnvConst& c);
int order_record_vec4(int K);
// gae.hip
hipError_t launch_gae(const float* r, const float* v, const float* nv, const uint8_t* term, const uint8_t* trunc,
                      int64_t n, int32_t T, float gamma, float lam, float* adv, float* tgt, double* stats,
                      hipStream_t st);
hipError_t launch_adv_normalize(float* adv, int64_t n, const double* stats, hipStream_t st);

}  // namespace msc
