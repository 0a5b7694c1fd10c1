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
#include "rng.hpp"

namespace msc {

// Device compilation sees every buffer pointer of the descriptor as a GLOBAL (addrspace 1) pointer:
// loads through pointers fetched from the device-resident DevEnv are otherwise generic flat_*
// instructions, which also count against lgkmcnt (so every LDS wait would wait for them too).
#if defined(__HIP_DEVICE_COMPILE__)
#define MSC_G __attribute__((address_space(1)))
#else
#define MSC_G
#endif

constexpr int BS = 64;          // threads per block of the env kernels (one wave: one env per lane)
constexpr int MAX_RING = 64;    // pending-order ring slots (max actual lead time + 1)
#define MSC_EA_MAX_S 32   // episode-ahead demand: max episode slots per env

struct EnvConst {
  int32_t W, K, R, T, Lmax, RING, F, L, order_cap;
  int32_t action_type, lead_type, dev_per_sku, lost_type, scope, norm, wid, num_eval, max_wh;
  int32_t demand_type, init_type, init_min, init_max, hold_per_sku, pen_per_sku, tr_rows;
  int32_t demand_impl;  // 0 = generator waves + unit-per-round parser (default); 5 = park4 (A/B)
  int32_t demand_gen;   // generator waves per block of the split demand kernel (1, 2 or 3; 5 / 7 A/B at 5 SKUs)
  int32_t park_min;     // parked lanes that trigger a settle pass of the demand parser (MSC_PARK_MIN)
  int32_t parser_rot;   // which wave of a demand block parses: (wave + rot(block)) % (1 + G) == 0 (A/B knob)
  int32_t obs_stage;    // 1: step_c stages each wave's observations in LDS and writes them coalesced
  int32_t obs_ring_reg; // 1: step_a / step_c (<= 8 warehouses) read the pending ring into registers before their stores
  int32_t epw_dem;      // envs per 64-lane block of the demand kernel (64, 32 or 16; see launch_demand)
  int32_t shared_home;  // 1: some region is the home region of two or more warehouses
  int32_t demand_uni;   // 1: Poisson parameters equal across regions (demand_unit_kernel<UNI>)
  int32_t alloc_impl;   // phase B: 0 = one env per lane (alloc_lane_kernel); 1 = one env per lane group (step_b_kernel)
  int32_t alloc_lpe;    // alloc_lane_kernel lanes per env forced by MSC_ALLOC_LPE (1, 2, 4); 0 = by env count
  int32_t chain_prio;   // step_a / step_c waves at s_setprio 3 (msc_env_set_chain_priority)
  int32_t alloc_sort;   // step_b_kernel visits envs in descending order of this step's order count (perm)
  int32_t sort_shift;   // order count >> sort_shift = bucket (< SORT_BUCKETS)
  int32_t ea_S;         // episode-ahead demand: episode slots per env (0: off)
  int32_t scan_defer;   // alloc_scan_kernel: lost-sales shares deferred to a post-pass (MSC_SCAN_DEFER=0: inline)
  int32_t demand_ptrs;  // 1: some Poisson rate >= 10 (numpy's PTRS branch): the sequential sampler demand_seq_kernel
  int32_t sb_tab;       // 1: step_b_kernel stages the {of, ov} rows and closest warehouses in LDS (its TAB form)
  int32_t fuse_c;       // 1: the scan allocator also runs phase C (step_c_kernel's work) for its env
  int32_t fuse_a;       // 1: ... and phase A (step_a_kernel's work; fixed lead times, Poisson demand)
  int32_t sb_gw;        // step_b lane-group width forced wider than the warehouse count (MSC_SB_GW; 0: by W)
  int32_t sc_tab;       // alloc_scan_kernel stages the {of, ov} table in LDS (when it fits: TAB form)
  int32_t sc_form;      // step_c_kernel's 16-wave form: compiled for 5 (env stepping) or 4 (rollout) waves per SIMD
  int32_t al_psplit;    // alloc_lane: 16ths of the wave's busiest env's orders run at s_setprio 3, the rest at 1
  uint32_t flags;
  int64_t E;
  int64_t ea_cap;       // episode-ahead demand: order records per (slot, env) episode
  double scale, alpha, hold_scalar, pen_scalar;
  double uni_thr_o, uni_thr_m, uni_thr_q;  // demand_uni: exp(-lambda_orders), p_skip, exp(-lambda_quantity)
  // demand_v2_kernel (demand_v2.hip, f32 ring): the f32 chain's decision thresholds around exp(-lambda)
  // {orders hi, orders lo, quantity hi, quantity lo}, the exact SKU-draw bound ceil(p * 2^53) on the
  // 53-bit draw, and the generators' refill quota per chunk
  float v2_thr[4];
  uint64_t v2_k53;
  int32_t v2_quota;
  const MSC_G double* act_param;   // [K]
  const MSC_G int32_t* init_vals;  // [W*K]
  const MSC_G double* hold;        // [K]
  const MSC_G double* pen;         // [K]
  const MSC_G double* skw;         // [K]
  const MSC_G double* ofT;         // [R][W] outbound fixed (transposed: one region's row is contiguous)
  const MSC_G double* ovT;         // [R][W] outbound variable
  const MSC_G double* inF;         // [W*K]
  const MSC_G double* inV;         // [W*K]
  const MSC_G double* enlam_o;     // [R]   exp(-lambda_orders) from the host libm
  const MSC_G double* p_sku;       // [R]
  const MSC_G double* p_skip;      // [R]   U > p_skip[r] <=> U >= p_sku[r] (SKU not in the order), U in 2^-53 Z
  const MSC_G double* enlam_q;     // [R*K] exp(-lambda_quantity)
  const MSC_G double* ptrs_o;      // [R][8]   PtrsConst of lambda_orders (demand_ptrs)
  const MSC_G double* ptrs_q;      // [R*K][8] PtrsConst of lambda_quantity (demand_ptrs)
  const MSC_G int32_t* elt;        // [W*K] expected lead times
  const MSC_G int32_t* maxdev;     // [K] or [1]
  const MSC_G uint32_t* home_mask; // [R] bit w set <=> region r is warehouse w's home region
  const MSC_G int32_t* closest;    // [R] closest warehouse of each region
  const MSC_G int32_t* home_of;    // [W] home region of each warehouse (the bit set in home_mask)
  const MSC_G float* obs_mean;     // [F]
  const MSC_G float* obs_std;      // [F]
  const MSC_G int64_t* tr_off;     // [tr_rows + 1]
  const uint4* tr_rec;       // [n_trace_orders][NV] packed order records
};

struct EnvState {
  MSC_G int32_t* inv;        // [WK][E]
  MSC_G int32_t* ring_q;     // [WK][RING][E] pending quantity by order time mod RING (0 = empty)
  MSC_G uint8_t* ring_l;     // [WK][RING][E] actual lead time of that order (stochastic lead only)
  MSC_G int32_t* hist;       // [5][WK][E]    incoming home demand of step tau at slot tau % 5
  MSC_G int32_t* inc;        // [WK][E]       incoming home demand of the last step
  MSC_G float* fc;           // [WK][E]       EMA demand forecast (f32, multi_env.py:789-793)
  MSC_G uint64_t* rng;       // [2][4][E]     {demand, lead} x {s_hi, s_lo, i_hi, i_lo}
  MSC_G uint32_t* rbuf;      // [2][2][E]     {demand, lead} x {has32, u32}
  MSC_G uint64_t* rng_pre;   // [4][E] demand-stream state before the last demand generation
  MSC_G uint32_t* rbuf_pre;  // [2][E] (reported while the next step's demand is pre-generated)
  MSC_G int32_t* t;          // [E] timestep
  MSC_G int32_t* counter;    // [E] SeedManager._episode_counter
  MSC_G uint32_t* orig_root; // [E] SeedManager._original_root_seed
  MSC_G uint32_t* root;      // [E] SeedManager.root_seed
  MSC_G int32_t* emp_start;  // [E] EmpiricalDemandSampler window start row (-1: not drawn)
  MSC_G int32_t* perm;       // [E] allocation visiting order (alloc_sort): envs by descending order count
  uint4* orders;       // [order_cap][E][NV] per-step order records (Poisson sampler output)
  MSC_G int32_t* n_orders;   // [E]
  // step phase scratch (step_a/b/c kernels): shipped total / home [WK][E], penalty / outbound /
  // inbound cost [W][E]
  MSC_G int32_t* sc_sht;
  MSC_G int32_t* sc_shh;
  MSC_G double* sc_pen;
  MSC_G double* sc_out;
  MSC_G double* sc_inb;
  MSC_G uint32_t* err;       // [1] device error bits
  // episode-ahead demand (EA): the Poisson orders of whole future episodes,
  // generated on a side stream while earlier episodes step. Slot j of env e holds one episode:
  uint4* ea_rec;             // [S][E][ea_cap][NV] order records, each env's episode contiguous
  MSC_G int32_t* ea_off;     // [S][T + 1][E] first record of step t (off[T] = the episode's count)
  MSC_G uint32_t* ea_pos;    // [S][T][E]     demand-stream position (draws) after step t
  MSC_G int32_t* ea_cnt;     // [S][E]        SeedManager._episode_counter after the slot episode's reset
};

// one launch of the episode-ahead demand generator: lanes (k, e) for k < nslots generate the
// episode of slot (slot0 + k) % S; its SeedManager counter follows from the counter stored for
// from_slot (the lane's own slot when from_slot < 0) by iters0 + k * iters_step more resets
// (reset_env's eval cycling included). A launch parses steps [t0, t1) of those episodes: t0 > 0
// continues from the stream position / record count the launch of [.., t0) left in the slot.
struct EaLaunch {
  int32_t slot0, nslots, from_slot, iters0, iters_step, t0, t1;
};

// where an env's orders of this step are: record n, word v at base + n * nstep + v * vstep (uint4)
struct OrderSrc {
  const uint4* src;
  int64_t base, nstep, vstep;
  int n;
};

struct StepIO {
  const MSC_G float* actions;  // [E][W][K]
  MSC_G float* obs;            // [E][W][L]
  MSC_G float* rew;            // [E][W]
  MSC_G double* rew64;         // [E][W] or null
  MSC_G uint8_t* trunc;        // [E]
  MSC_G float* final_obs;      // [E][W][L] or null
  msc_step_info info;    // device pointers or nulls
  int32_t has_info;
  int32_t ea_slot;       // >= 0: this step's orders come from episode-ahead slot ea_slot, step ea_t
  int32_t ea_t;
};

// The orders of env e for this step (every allocation kernel reads them through this): the Poisson
// sampler's per-step buffer [order][NV][E], an episode-ahead slot, or the empirical trace row.
template <int NV>
__device__ __forceinline__ OrderSrc order_src(const EnvConst& c, const EnvState& s, const StepIO& io, int64_t e) {
  OrderSrc o;
  const int64_t E = c.E;
  if (c.demand_type == MSC_DEMAND_EMPIRICAL) {
    o.src = c.tr_rec;
    o.nstep = NV;
    o.vstep = 1;
    o.base = 0;
    o.n = 0;
    if (s.emp_start[e] >= 0) {
      const int64_t row = s.emp_start[e] + (s.t[e] % c.T);
      const int64_t off = c.tr_off[row];
      o.n = (int)(c.tr_off[row + 1] - off);
      o.base = off * NV;
    }
  } else if (io.ea_slot >= 0) {
    const int64_t le = (int64_t)io.ea_slot * E + e;
    const MSC_G int32_t* off = s.ea_off + ((int64_t)io.ea_slot * (c.T + 1) + io.ea_t) * E + e;
    const int o0 = off[0];
    o.src = s.ea_rec;
    o.n = off[E] - o0;
    o.base = (le * c.ea_cap + o0) * NV;
    o.nstep = NV;
    o.vstep = 1;
  } else {
    o.src = s.orders;
    o.n = s.n_orders[e];
    o.base = e;
    o.nstep = (int64_t)NV * E;
    o.vstep = E;
  }
  return o;
}

constexpr uint32_t ERR_ORDER_OVERFLOW = 1u;

// launchers (env_kernels.hip)
// The descriptor + state pointers live in device memory and kernels take a pointer to them:
// fields are then scalar-cache loads, and no address-taken kernel argument is copied to scratch.
struct DevEnv {
  EnvConst c;
  EnvState s;
};

hipError_t launch_reset(const EnvConst& c, const DevEnv* d, const uint8_t* mask, const uint32_t* new_roots,
                        int32_t flags, float* obs, hipStream_t st);
hipError_t launch_step(const EnvConst& c, const DevEnv* d, const StepIO& io, bool gen_demand, hipStream_t st);
hipError_t launch_demand(const EnvConst& c, const DevEnv* d, hipStream_t st);
hipError_t launch_demand_ea(const EnvConst& c, const DevEnv* d, const EaLaunch& ea, hipStream_t st);
hipError_t launch_ea_materialize(const EnvConst& c, const DevEnv* d, int slot, int t_done, hipStream_t st);
// alloc_scan.hip
hipError_t launch_alloc_scan(const EnvConst& c, const DevEnv* d, const StepIO& io, hipStream_t st);
bool alloc_scan_fuse_supported(int W, int K, int RING);
bool alloc_scan_supported(int W, int K);
constexpr int SORT_BUCKETS = 1024;
// alloc_kernels.hip
hipError_t launch_alloc_lane(const EnvConst& c, const DevEnv* d, const StepIO& io, hipStream_t st);
hipError_t launch_obs_flat(const EnvConst& c, const float* obs, float* flat, hipStream_t st);
size_t demand_lds_bytes(const EnvConst& c);  // per block of the production demand kernel
// demand_ab.hip: the split-parser Poisson demand kernel (equal sampler parameters in every region)
bool demand_ab_supported(const EnvConst& c);
hipError_t launch_demand_seq(const EnvConst& c, const DevEnv* d, hipStream_t st, const EaLaunch* ea);
hipError_t launch_poisson_draws(uint64_t* state, const PtrsConst* ptrs, const double* enlam, int64_t n_lam, int64_t n,
                                int64_t* out, hipStream_t st);
hipError_t launch_demand_ab(const EnvConst& c, const DevEnv* d, hipStream_t st, const EaLaunch* ea);
// demand_v2.hip: the f32-ring Poisson demand kernel (equal sampler parameters, <= 8 SKUs)
bool demand_v2_supported(const EnvConst& c);
hipError_t launch_demand_v2(const EnvConst& c, const DevEnv* d, hipStream_t st, const EaLaunch* ea);
// demand_v3.hip: the unit parser with a shorter round (equal sampler parameters, <= 8 SKUs), and the
// dispatcher of the alternative demand kernels (c.demand_impl 8 / 9)
bool demand_v3_supported(const EnvConst& c);
hipError_t launch_demand_v3(const EnvConst& c, const DevEnv* d, hipStream_t st, const EaLaunch* ea);
hipError_t launch_demand_alt(const EnvConst& c, const DevEnv* d, hipStream_t st, const EaLaunch* ea);
int order_record_vec4(int K);
// gae.hip
hipError_t launch_gae(const float* r, const float* v, const float* nv, const uint8_t* term, const uint8_t* trunc,
                      int64_t n, int32_t T, float gamma, float lam, float* adv, float* tgt, int32_t n_groups,
                      double* stats, hipStream_t st);
hipError_t launch_adv_normalize(float* adv, int64_t n, int32_t n_groups, const double* stats, hipStream_t st);
int mlp3_valu_outputs(int KO);
// the fused MLPs' optional Gaussian-sampling epilogue (msc_gaussian_epilogue); act == nullptr: none
struct MlpSample {
  const float* log_std;  // [ls_rows][KO]
  int ls_rows;
  float floor_;
  const float* eps;      // [n][KO]
  float* act;            // [n][KO]
  float* logp;           // [n]
  float* clipped;        // [n][KO]
};
hipError_t launch_mlp3_relu(const float* x, int64_t n, int L, int H1, int H2, int KO, const float* w1p, const float* b1,
                            const float* w2p, const float* b2, const float* w3p, const float* b3, float* out,
                            const float* pre1, int grp, hipStream_t st, const MlpSample* smp = nullptr);
hipError_t launch_mlp2_relu(const float* x, int64_t n, int L, int H1, int KO, const float* w1p, const float* b1,
                            const float* w3p, const float* b3, float* out, const float* pre1, int grp, hipStream_t st,
                            const MlpSample* smp = nullptr);
bool mlp2_supported(int H1);
hipError_t launch_normal_keyed(float* out, int32_t n_steps, int64_t n_rows, int32_t row_len, int64_t row0,
                               uint64_t seed, uint64_t step0, hipStream_t st);
hipError_t launch_meanstd_filter(const float* x, float* out, int64_t E, int32_t C, const uint8_t* mask, int32_t update,
                                 double* state, double* scratch, double clip, double eps, hipStream_t st);
int64_t meanstd_scratch_doubles(int64_t E, int32_t C);
hipError_t launch_gauss_sample(const float* mean, const float* log_std, int32_t ls_rows, float floor_, const float* eps,
                               int64_t N, int32_t K, float* act, float* logp, float* clipped, hipStream_t st);

}  // namespace msc
