// alloc_scan.hip -- phase B of InventoryEnvironment.step for few envs per GPU (BASELINE configs[1]:
// 4,096 envs): the greedy allocation (GreedyDemandAllocator.allocate, demand_allocator.py:118-217)
// as a prefix scan over the cost ranking, one env per wave.
//
// Why a scan. For one order with demand d_s, the reference walks the warehouses in ascending cost
// order (argsort of of[w, r] + ov[w, r] * (d . sku_weights), :168-173) and takes
// fill = min(remaining, inventory) from each (:186), skipping warehouses with nothing to give and
// stopping after max_splits + 1 contributing ones (:182). Without that stop the fill of SKU s at
// the warehouse of rank p is exactly
//     f_{p,s} = min(inv_{p,s}, max(0, d_s - sum_{q<p} inv_{q,s}))       (inventories >= 0),
// an exclusive prefix sum over the ranking: no data-dependent loop, and every (SKU, warehouse) pair
// is independent. With the stop, the fills before the (max_splits+1)-th contributing rank are the
// same and later ones are zero (a mask over the contributing ranks). The few-env configs have few
// allocation chains (4,096 at configs[1] vs 32,768 at configs[2]), so the chain length per order,
// not the issue rate, bounds the step: this kernel spends ~25 vector instructions per order on the
// chain where the group kernel (step_b_kernel) spends ~340.
//
// Thread mapping: one env per wave (4 per block), lane = s * GW + w (SKU s, warehouse w; GW = the
// warehouse count rounded up to 2 / 4 / 8, K * GW <= 64). Per order:
//   1. rank (off the chain): the wave first ranks a window of 64 orders, one order per lane (the
//      W costs and their order, packed as 4-bit ranks rho_w), into LDS;
//   2. ds_permute moves each lane's inventory to the lane of its warehouse's rank (rank space),
//   3. a 3-step DPP scan over the GW lanes of a SKU gives the exclusive prefix, the fill is one med3,
//   4. ds_bpermute brings each fill back to its warehouse's lane, which updates its inventory.
// Region epilogues (orders are region-major) fold the region into lost sales (shipment share /
// closest / cost softmax, lost_sales_handler.py:71-210), outbound costs (reward_calculator.py:
// 139-142: counts x fixed + (shipped . weights) x variable, per region as the reference sums them)
// and the home-region features (multi_env.py:767-773). Inputs: any order source (order_src: the
// Poisson step buffer, an episode-ahead slot, the empirical trace).
#include <hip/hip_runtime.h>
#include <math.h>

#include <type_traits>

#include "env.hpp"
#include "kcommon.hpp"
#include "obs_common.hpp"

namespace msc {

#ifdef MSC_PROF
// in-kernel cycle accounting (profiling build: make prof -> libmarlsc_prof.so, tools/prof_scan.py)
__device__ unsigned long long g_prof_scan[8];
#define SPROF(v) unsigned long long v = 0
#define SPROF_T(v) const unsigned long long v = (unsigned long long)clock64()
#define SPROF_ADD(v, x) (v) += (x)
#define SPROF_NOW() ((unsigned long long)clock64())
#define SPROF_FLUSH(i, v) \
  if (lane == 0) atomicAdd(&g_prof_scan[i], (v))
#else
#define SPROF(v)
#define SPROF_T(v)
#define SPROF_ADD(v, x)
#define SPROF_NOW() 0ull
#define SPROF_FLUSH(i, v)
#endif

constexpr int SC_WAVES = 4;  // envs (waves) per block
// waves per SIMD the <= 8-warehouse instantiations are register-budgeted for: 4 (<= 128 VGPRs). At
// 142 / 136 VGPRs (rounds 3-4) only 3 fit, so of configs[1]'s 4,096 one-env waves 3,072 ran and the
// last 1,024 started as they retired: the launch took two wave lifetimes (75 us each, 142 us)
#ifndef MSC_SC_WPE
#define MSC_SC_WPE 4
#endif
constexpr int SC_WIN = 64;   // orders ranked per window (one per lane)
#ifndef MSC_SC_PRIO
#define MSC_SC_PRIO 3  // s_setprio: the step chain is the critical path next to the demand generator
#endif

// Lost regions whose shipment / cost shares are deferred: the region epilogue (on the per-order
// chain) only records the region, its lost-order count, the units each warehouse shipped to it and the
// unfulfilled units per SKU; the shares and the lost-sales sums run after the order loop, eight regions
// per pass (lane = region slot x warehouse) and then one multiply-add per region and (SKU, warehouse)
// lane, in region order (the reference's summation order, lost_sales_handler.py:113-148 / :170-210).
// deferred regions per flush: 16 (a 1.25-KB block per wave; 64 in rounds 3-4, 5 KB) leaves more of a
// CU's 160 KB of LDS to the episode-ahead generation's blocks (37 KB each) running beside the scan
// blocks at configs[1]: C2 205.5 -> 208.4 M agent-steps/s (profiles/r05/ab_scan_lds.txt)
#ifndef MSC_SC_LR
#define MSC_SC_LR 16
#endif
constexpr int SC_LR = MSC_SC_LR;

// LDS per wave: the window's order records, epilogue scratch (64 entries per SKU slot, see NS)
template <int NS>
struct ScWaveLds {
  uint4 rec[SC_WIN];  // (also the outbound-variable partials at the end: 128 doubles)
  int32_t iscr[64 * NS];
  double dscr[64 * NS];
};
// and, when the lost-sales shares are deferred, the deferred lost regions (after the SC_WAVES
// ScWaveLds blocks; not allocated otherwise)
template <int GW>
struct ScLostLds {
  static constexpr int LA = GW > 8 ? 16 : 8;
  int32_t lr_acc[SC_LR * LA];  // [i][w] units warehouse w shipped to deferred region i
  int32_t lr_ug[SC_LR * 8];    // [i][s] unfulfilled units of SKU s (K <= 6)
  int32_t lr_r[SC_LR];         // region id
  int32_t lr_cnt[SC_LR];       // lost orders
  double lr_wt[64];            // one pass's shares [i % (64 / GW)][w]
};
// fused phase C: the per-(SKU, warehouse) inputs of the observation builder, [field][s * GW + w]
// (aliases the deferred-region block, flushed by then; allocated as the larger of the two)
constexpr int SC_FC_RING = 4;  // pending-ring slots staged (lead times <= 3)
// (the fields an agent's totals read across its SKU lanes; the ring, history and lead time a lane
// reads only for its own SKU stay in its registers)
enum : int { FC_INV, FC_DH, FC_SH, FC_SA, FC_PEND, FC_FC, FC_RM, FC_NF };
struct ScFcLds {
  int32_t v[FC_NF][64];
};
constexpr size_t sc_tab_bytes(int R, int GW) { return (size_t)(R | 1) * GW * 16; }
constexpr size_t SC_TAB_MAX = 32 * 1024;
// warehouse lanes per SKU group and SKU slots per lane: GW = the warehouse count rounded up to
// 2 / 4 / 8 / 16; a wave holds 64 / GW SKU groups, so above 4 SKUs at 16 warehouses each lane
// carries two (SKU, warehouse) slots (SKUs sg and 4 + sg)
__host__ __device__ constexpr int sc_gw(int W) { return W <= 2 ? 2 : W <= 4 ? 4 : W <= 8 ? 8 : 16; }
__host__ __device__ constexpr int sc_ns(int K, int GW) { return (K * GW + 63) / 64; }

// inclusive prefix sum over the GW lanes of each group (p = lane % GW), DPP row shifts inside the
// 16-lane rows with the lanes whose source belongs to the previous group masked
template <int GW>
__device__ __forceinline__ int group_scan(int x, int p) {
  int v = x;
  int t = __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, true);  // row_shr:1
  v += p >= 1 ? t : 0;
  if constexpr (GW >= 4) {
    t = __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, true);  // row_shr:2
    v += p >= 2 ? t : 0;
  }
  if constexpr (GW == 8) {
    // row_shr:4 into banks 1 and 3 only (lanes 4-7, 12-15 of a row: p >= 4); others add 0
    t = __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xA, false);
    v += t;
  }
  if constexpr (GW == 16) {  // a group is a whole row: row_shr:4 into banks 1-3, row_shr:8 into 2-3
    t = __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xE, false);
    v += t;
    t = __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xC, false);
    v += t;
  }
  return v;
}
// OR of a value over the 64 / GW groups (lanes p, p + GW, p + 2 GW, ...): row rotations inside the
// 16-lane rows, then the gfx950 row / half swaps across them
template <int GW>
__device__ __forceinline__ uint32_t or_groups(uint32_t v) {
  if constexpr (GW <= 2) v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x122, 0xF, 0xF, false);  // row_ror:2
  if constexpr (GW <= 4) v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xF, 0xF, false);  // row_ror:4
  if constexpr (GW <= 8) v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
  const auto a = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  v = a[0] | a[1];
  const auto b = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return b[0] | b[1];
}
// sum of a value over the 64 / GW groups (as or_groups): every lane gets the total of its lane % GW
template <int GW>
__device__ __forceinline__ int add_groups(int v) {
  if constexpr (GW <= 2) v += __builtin_amdgcn_update_dpp(0, v, 0x122, 0xF, 0xF, false);  // row_ror:2
  if constexpr (GW <= 4) v += __builtin_amdgcn_update_dpp(0, v, 0x124, 0xF, 0xF, false);  // row_ror:4
  if constexpr (GW <= 8) v += __builtin_amdgcn_update_dpp(0, v, 0x128, 0xF, 0xF, false);  // row_ror:8
  const auto a = __builtin_amdgcn_permlane16_swap((uint32_t)v, (uint32_t)v, false, false);
  v = (int)(a[0] + a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap((uint32_t)v, (uint32_t)v, false, false);
  return (int)(b[0] + b[1]);
}
// OR of the 64 / GW groups' GW-bit fields of a ballot
template <int GW>
__device__ __forceinline__ uint32_t fold_groups(uint64_t b) {
#pragma unroll
  for (int sh = 32; sh >= GW; sh >>= 1) b |= b >> sh;
  return (uint32_t)b & ((1u << GW) - 1u);
}
template <int GW, typename T, typename F>
__device__ __forceinline__ T sc_group_reduce(T v, F op) {
  v = op(v, dpp_x<0>(v));
  if constexpr (GW >= 4) v = op(v, dpp_x<1>(v));
  if constexpr (GW >= 8) v = op(v, dpp_x<2>(v));
  if constexpr (GW >= 16) v = op(v, dpp_x<3>(v));
  return v;
}

__device__ __forceinline__ uint32_t rec_field(const uint4& v, int h) {  // h: compile-time after unrolling
  const uint32_t w = h < 2 ? v.x : h < 4 ? v.y : h < 6 ? v.z : v.w;
  return (h & 1) ? (w >> 16) : (w & 0xffffu);
}

// 4-bit ranks of up to 8 warehouses in 32 bits, of 16 in 64
template <int GW>
using ScRho = typename std::conditional<(GW > 8), uint64_t, uint32_t>::type;
template <typename T>
__device__ __forceinline__ T sc_shfl_up1(T v) {
  if constexpr (sizeof(T) == 8) {
    const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)v, 1), hi = (uint32_t)__shfl_up((int)(uint32_t)(v >> 32), 1);
    return ((T)hi << 32) | lo;
  } else {
    return (T)__shfl_up((int)v, 1);
  }
}
template <typename T>
__device__ __forceinline__ T sc_readlane(T v, int l) {
  if constexpr (sizeof(T) == 8) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((T)hi << 32) | lo;
  } else {
    return (T)__builtin_amdgcn_readlane((int)v, l);
  }
}

__device__ __forceinline__ int hist_of(const int (&hv)[MSC_HISTORY], int a) {
  int v = 0;
#pragma unroll
  for (int q = 0; q < MSC_HISTORY; q++) v = q == a ? hv[q] : v;
  return v;
}
// Fused phase C: the observation of agent w written by lane (sk, w) -- SKU sk's value of every
// per-SKU feature block and, on lane sk == 0, the aggregates and the one-hot entries -- instead of
// one lane per agent (obs_emit, the same arithmetic value by value: _build_local_obs /
// _feature_block, multi_env.py:577-745). The agent's inputs are the staged ones (ScFcLds, lane
// s * GW + w); o points at the agent's vector.
template <int K, int GW>
__device__ __forceinline__ void fc_obs_lane(const EnvConst& c, const ScFcLds* Lf, int w, int sk, int tm, int n_hist,
                                            int elt, const int (&rv)[SC_FC_RING], const int (&hv)[MSC_HISTORY],
                                            float* o) {
  const int W = c.W, Lmax = c.Lmax, RING = c.RING;
  const uint32_t f = c.flags;
  const bool ratio = c.norm == MSC_OBS_RATIO, meanstd = c.norm == MSC_OBS_MEANSTD;
  const double eps = 1e-8;
  const float epsf = 1e-8f;
  const int l0 = sk * GW + w;
  const int inv = Lf->v[FC_INV][l0], dh = Lf->v[FC_DH][l0], sh = Lf->v[FC_SH][l0], sa = Lf->v[FC_SA][l0];
  const int pend = Lf->v[FC_PEND][l0];
  const float fc = __int_as_float(Lf->v[FC_FC][l0]), rm = __int_as_float(Lf->v[FC_RM][l0]);
  // the agent's totals (obs_emit's sums, SKU order)
  double inv_total = 0.0, shipped_total = 0.0, sa_total = 0.0;
  float dh_total = 0.0f, rm_a[K], fc_a[K];
  int pend_total = 0;
#pragma unroll
  for (int k = 0; k < K; k++) {
    const int l = k * GW + w;
    inv_total += (double)Lf->v[FC_INV][l];
    dh_total += (float)Lf->v[FC_DH][l];
    shipped_total += (double)(Lf->v[FC_SH][l] + Lf->v[FC_SA][l]);
    sa_total += (double)Lf->v[FC_SA][l];
    pend_total += Lf->v[FC_PEND][l];
    rm_a[k] = __int_as_float(Lf->v[FC_RM][l]);
    fc_a[k] = __int_as_float(Lf->v[FC_FC][l]);
  }
  const float rm_total = np_sum_f32<K>(rm_a);
  const float fc_total = np_sum_f32<K>(fc_a);
  const int base = c.wid ? W : 0;
  auto put = [&](int j, double v) {  // feature j (the one-hot excluded)
    float x = (float)v;
    if (meanstd) x = (x - c.obs_mean[j]) / c.obs_std[j];
    o[base + j] = x;
  };
  const bool lead = sk == 0;  // writes the aggregates and the one-hot
  if (c.wid)
    for (int k = sk; k < W; k += K) o[k] = (k == w) ? 1.0f : 0.0f;
  int j0 = 0;  // first feature index of the current block
  if (f & MSC_F_INVENTORY) {
    put(j0 + sk, ratio ? (double)inv / (inv_total + eps) : (double)inv);
    j0 += K;
    if (f & MSC_F_INVENTORY_AGG) {
      if (lead) put(j0, (double)(float)inv_total);
      j0++;
    }
  }
  if (f & MSC_F_PIPELINE) {
    const float den = (float)((double)pend_total + eps);
    for (int l = 0; l < Lmax; l++) {
      // bucket l of this SKU: the order in ring slot q (age (t - q) mod RING) lands in bucket
      // max(1, elt - age) - 1 (_compute_pipeline, multi_env.py:956-966)
      int pv = 0;
#pragma unroll
      for (int q = 0; q < SC_FC_RING; q++) {
        const int age = tm - q >= 0 ? tm - q : tm - q + RING;
        const int bk = elt - age > 1 ? elt - age - 1 : 0;
        pv += (q < RING && bk == l) ? rv[q] : 0;
      }
      const float v = (float)pv;
      put(j0 + l * K + sk, ratio ? (double)(v / den) : (double)v);
    }
    j0 += Lmax * K;
    if (f & MSC_F_PIPELINE_AGG) {
      if (lead) put(j0, (double)pend_total);
      j0++;
    }
  }
  if (f & MSC_F_INCOMING_HOME) {
    const float den = dh_total + epsf;
    put(j0 + sk, ratio ? (double)((float)dh / den) : (double)dh);
    j0 += K;
    if (f & MSC_F_INCOMING_HOME_AGG) {
      if (lead) put(j0, (double)dh_total);
      j0++;
    }
  }
  if (f & MSC_F_SHIPPED_HOME) {
    const double den = (double)(dh_total + epsf);
    put(j0 + sk, ratio ? (double)sh / den : (double)sh);
    j0 += K;
  }
  if (f & MSC_F_SHIPPED_AWAY) {
    put(j0 + sk, ratio ? (double)sa / (shipped_total + eps) : (double)sa);
    j0 += K;
    if (f & MSC_F_SHIPPED_AWAY_AGG) {
      if (lead) put(j0, (double)(float)(sa_total / (shipped_total + eps)));
      j0++;
    }
  }
  if (f & MSC_F_STOCKOUT) {
    const float den = dh_total + epsf;
    const float so = (float)(dh - sh > 0 ? dh - sh : 0);
    put(j0 + sk, ratio ? (double)(so / den) : (double)so);
    j0 += K;
  }
  if (f & MSC_F_ROLLING_MEAN) {
    const float den = rm_total + epsf;
    put(j0 + sk, ratio ? (double)(rm / den) : (double)rm);
    j0 += K;
    if (f & MSC_F_ROLLING_MEAN_AGG) {
      if (lead) put(j0, (double)rm_total);
      j0++;
    }
  }
  if (f & MSC_F_FORECAST) {
    const float den = fc_total + epsf;
    put(j0 + sk, ratio ? (double)(fc / den) : (double)fc);
    j0 += K;
    if (f & MSC_F_FORECAST_AGG) {
      if (lead) put(j0, (double)fc_total);
      j0++;
    }
  }
  if (f & MSC_F_DAYS_OF_SUPPLY) {
    put(j0 + sk, (double)(float)((double)inv / (double)(rm > 1.0f ? rm : 1.0f)));
    j0 += K;
  }
  if (f & MSC_F_NET_POSITION) {
    put(j0 + sk, (double)(float)(((double)inv + (double)pend) - (double)fc * (double)elt));
    j0 += K;
  }
  if (f & MSC_F_DEMAND_VARIABILITY) {
    float sd = 0.0f;
    if (n_hist > 1) {  // oldest first, as the deque (multi_env.py:776-789)
      float sum = 0.0f;
      for (int h = 0; h < n_hist; h++) sum += (float)hist_of(hv, n_hist - 1 - h);
      const float mean = sum / (float)n_hist;
      float ss = 0.0f;
      for (int h = 0; h < n_hist; h++) {
        const float d = (float)hist_of(hv, n_hist - 1 - h) - mean;
        ss += d * d;
      }
      sd = sqrtf(ss / (float)n_hist);
    }
    put(j0 + sk, (double)sd);
    j0 += K;
  }
  if (f & MSC_F_DEMAND_HISTORY) {
    for (int h = 0; h < MSC_HISTORY; h++) put(j0 + h * K + sk, (double)(h < n_hist ? hist_of(hv, h) : 0));
    j0 += MSC_HISTORY * K;
  }
}

// Orders of one region with the same cost ranking form a batch: greedy fills of consecutive orders
// over one ranking are the fills of their running demand total, so order k of a batch takes
//     f_{k,p,s} = a_k - a_{k-1},  a_k = min(inv_{p,s}, max(0, D_{k,s} - sum_{q<p} inv_{q,s})),
// D_k = d_1 + ... + d_k, and the whole batch needs one permute, one scan and one bpermute. As D_k
// only grows, the orders rank p fills from are the ones asking for s in the run
//     D_k > excl_p  and  D_{k-1} < incl_p     (inventory > 0)
// and the orders short of s (lost-order test) those asking for it with D_k > the SKU total: per
// order three threshold counts of D_k, the order masks follow per batch (batches of <= 16 orders;
// contribution and lost masks in one word OR-reduced over the SKU groups). (With max_splits
// limiting the warehouses per order every order is its own batch, with per-order ballots.)
// NS = 2 (16 warehouses, 5-6 SKUs): every per-(SKU, warehouse) quantity is a two-slot array; one
// ranking, one permute address and one contribution mask serve both slots.
// FC: phase C fused (step_c_kernel's work for the wave's env: forecast / history, rewards, the
// observations, the in-kernel reset at truncation; one slot per lane, rings of <= SC_FC_RING slots).
// FA (with FC): phase A fused too (step_a_kernel: action rescale, orders into the ring, arrivals,
// inbound cost) for fixed lead times and Poisson demand (no per-env RNG work in phase A)
template <int K, int GW, bool TAB, bool FC = false, bool FA = false, bool ND = false>
__global__ __launch_bounds__(64 * SC_WAVES) __attribute__((amdgpu_waves_per_eu(GW > 8 ? 3 : MSC_SC_WPE))) void alloc_scan_kernel(
    const DevEnv* __restrict__ dp, StepIO io) {
  constexpr int SPW = 64 / GW;        // SKU groups per wave
  constexpr int NS = sc_ns(K, GW);    // SKU slots per lane
  static_assert(K <= 6 && NS <= 2 && GW <= 16, "one uint4 per order record; <= 2 slots");
  static_assert(!FC || NS == 1, "the fused phase C takes one (SKU, warehouse) slot per lane");
  static_assert(!FA || FC, "phase A is fused only with phase C");
  using Rho = ScRho<GW>;
  const EnvConst& c = dp->c;
  const EnvState& s = dp->s;
  const int W = c.W, R = c.R, WK = W * K;
  const int64_t E = c.E;
  // (the wave index through readfirstlane: the compiler's divergence analysis would otherwise treat
  // the env and everything derived from it -- order counts, loop bounds -- as per-lane values)
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int64_t e = (int64_t)blockIdx.x * SC_WAVES + wave;
  const int sg = lane / GW, w = lane % GW;  // this lane's SKU group and warehouse (its rank p in rank space)
  int skj[NS];                              // slot j's SKU
  bool lvj[NS];
#pragma unroll
  for (int j = 0; j < NS; j++) {
    skj[j] = j * SPW + sg;
    lvj[j] = skj[j] < K && w < W;
  }
  const msc_step_info info = io.info;
  // ND: an instantiation without the step-info stores (io.has_info == 0): their pointers, flags and
  // branches out of the registers of the order loop
  const bool dbg = !ND && io.has_info != 0;
  if (MSC_SC_PRIO > 0) __builtin_amdgcn_s_setprio(MSC_SC_PRIO);

  extern __shared__ __attribute__((aligned(16))) char sc_lds[];
  double2* Ltab = reinterpret_cast<double2*>(sc_lds);  // [w][R | 1] {of, ov}
  int32_t* Lcl = reinterpret_cast<int32_t*>(sc_lds + (TAB ? sc_tab_bytes(R, GW) : 0));  // [R] closest warehouse
  ScWaveLds<NS>* Lw = reinterpret_cast<ScWaveLds<NS>*>(Lcl + ((R + 3) & ~3)) + wave;
  // per-wave tail: the deferred lost-sales regions, aliased by the fused phase C's staging (the stride
  // is the larger of the two, as alloc_scan_lds_bytes sizes it)
  constexpr size_t TAILB =
      FC && sizeof(ScFcLds) > sizeof(ScLostLds<GW>) ? sizeof(ScFcLds) : sizeof(ScLostLds<GW>);
  static_assert(TAILB % 16 == 0, "per-wave tail keeps 16-byte alignment");
  ScLostLds<GW>* Ll = reinterpret_cast<ScLostLds<GW>*>(
      reinterpret_cast<char*>(reinterpret_cast<ScWaveLds<NS>*>(Lcl + ((R + 3) & ~3)) + SC_WAVES) + wave * TAILB);
  constexpr int LA = ScLostLds<GW>::LA;
  const int RS = R | 1;
  if constexpr (TAB) {
    for (int i = threadIdx.x; i < R * GW; i += blockDim.x) {
      const int ww = i / R, r = i % R;
      Ltab[ww * RS + r] = ww < W ? make_double2(c.ofT[r * W + ww], c.ovT[r * W + ww]) : make_double2(0.0, 0.0);
    }
  }
  for (int i = threadIdx.x; i < R; i += blockDim.x) Lcl[i] = c.closest[i];
  __syncthreads();  // the only block barrier: waves (envs) are independent from here on
  if (e >= E) return;
  auto tab_at = [&](int r, int ww) -> double2 {
    if constexpr (TAB) {
      return Ltab[ww * RS + r];
    } else {
      const int wc = ww < W ? ww : W - 1;
      return make_double2(gp(c.ofT)[r * W + wc], gp(c.ovT)[r * W + wc]);
    }
  };
  // LDS written by some lanes and read by others of the same wave: a wave's LDS instructions execute
  // in order, so only the compiler must not move the accesses
  auto wave_sync = [] {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };

  // uniform constants in scalar registers
  double skw[K];
#pragma unroll
  for (int j = 0; j < K; j++) skw[j] = sgpr_d(c.skw[j]);
  const int lost_type = __builtin_amdgcn_readfirstlane(c.lost_type);
  const int maxwh = __builtin_amdgcn_readfirstlane(c.max_wh);
  const bool split = maxwh < W;
  const bool defer = __builtin_amdgcn_readfirstlane(c.scan_defer) != 0 && !dbg && lost_type != MSC_LOST_CLOSEST;
  const double alpha = sgpr_d(c.alpha);
  const int pps = c.pen_per_sku;
  const int myhome = w < W ? c.home_of[w] : -1;
  const bool lastp = w == GW - 1;  // the lane of the last rank of its SKU (holds the SKU's total)

  // per slot: [w*K + s][E] state index, inventory, shipped-to-region, unfulfilled (last rank lane),
  // incoming demand of the region; lost sales; outbound-variable accumulator; home features.
  // ofix: sum_r count * fixed; ovacc: sum_r shipped(w, r, s) * variable (the SKU weights applied once
  // at the end: out_var_w = sum_s w_s ovacc_s, reward_calculator.py:141-142 reordered)
  int64_t gi[NS];
  int inv[NS], inv0[NS], qsr[NS], u[NS], dsum[NS], inc_h[NS], shh_h[NS], fi[NS];
  double lost[NS], ovacc[NS];
  const int t_now = FC ? __builtin_amdgcn_readfirstlane(s.t[e]) : 0;
  // FA: phase A (step_a_kernel's per-(SKU, warehouse) work) on this lane's slot; the warehouse's
  // inbound cost reaches lane w (sg == 0). The updated ring goes back to global memory and phase C
  // reloads it after the allocation (the RING registers are not kept live across the order loop, whose
  // VGPR budget sets the waves per SIMD; the reload hits L2)
  double inb_a = 0.0;
  if constexpr (FA) {
    const int RING = c.RING, slot = t_now % RING;
    const int i = w * K + skj[0];
    const int64_t g = (int64_t)i * E + e;
    double tF = 0.0, tV = 0.0;
    int iv = 0;
    int ring_a[SC_FC_RING] = {};
    if (lvj[0]) {
      const float a = io.actions[(e * W + w) * K + skj[0]];
      const int inc_old = s.inc[g];
      iv = s.inv[g];
      int pend = 0;
#pragma unroll
      for (int q = 0; q < SC_FC_RING; q++) {
        ring_a[q] = q < RING ? s.ring_q[((int64_t)i * RING + q) * E + e] : 0;
        pend += ring_a[q];
      }
      const int qi = rescale_action(c, skj[0], a, inc_old, pend);
      const int elt = c.elt[i];
      if (dbg) {
        if (info.inventory_before) info.inventory_before[e * WK + i] = iv;
        if (info.pending_total) info.pending_total[e * WK + i] = pend;
        if (info.order_quantities) info.order_quantities[e * WK + i] = qi;
      }
      // _apply_arrivals: the orders whose actual lead time equals their age (arrival == t)
#pragma unroll
      for (int q = 0; q < SC_FC_RING; q++) {
        int age = (t_now - q) % RING;
        if (age < 0) age += RING;
        const bool arrive = q < RING && q != slot && ring_a[q] != 0 && elt == age;
        iv += arrive ? ring_a[q] : 0;
        if (arrive) {
          ring_a[q] = 0;
          s.ring_q[((int64_t)i * RING + q) * E + e] = 0;
        }
      }
#pragma unroll
      for (int q = 0; q < SC_FC_RING; q++) ring_a[q] = q == slot ? qi : ring_a[q];
      s.ring_q[((int64_t)i * RING + slot) * E + e] = qi;  // _apply_orders: the slot of order time t
      tF = qi > 0 ? c.inF[i] : 0.0;
      tV = ((double)qi * c.skw[skj[0]]) * c.inV[i];
    }
    inv[0] = iv;

    // inbound cost (reward_calculator.py:144-151): fixed and variable terms summed over SKUs in order
    Lw->dscr[lane] = tF;
    wave_sync();
    double sF = 0.0, sV = 0.0;
    if (sg == 0 && w < W)
#pragma unroll
      for (int j = 0; j < K; j++) sF += Lw->dscr[j * GW + w];
    wave_sync();
    Lw->dscr[lane] = tV;
    wave_sync();
    if (sg == 0 && w < W) {
#pragma unroll
      for (int j = 0; j < K; j++) sV += Lw->dscr[j * GW + w];
      inb_a = sF + sV;
    }
    wave_sync();
  }
#pragma unroll
  for (int j = 0; j < NS; j++) {
    gi[j] = (int64_t)(w * K + skj[j]) * E + e;
    if (!FA) inv[j] = lvj[j] ? s.inv[gi[j]] : 0;
    inv0[j] = inv[j];
    qsr[j] = u[j] = dsum[j] = inc_h[j] = shh_h[j] = 0;
    lost[j] = ovacc[j] = 0.0;
    fi[j] = skj[j] < K ? 1 + skj[j] : 7;  // this slot's 16-bit field of a record (field 7 is 0: K <= 6)
  }
  int cnt = 0, lost_cnt = 0;
  double ofix = 0.0, of_me = 0.0, ov_me = 0.0;
  bool home_done = false;
  int cur = -1;
  Rho cur_rho = ~Rho(0);

  const OrderSrc o = order_src<1>(c, s, io, e);
  const int n = __builtin_amdgcn_readfirstlane(o.n);
  const MSC_GLOBAL uint4* src = gp(o.src);
  if (dbg && lane == 0 && info.n_orders) info.n_orders[e] = n;

  // deferred lost regions (see SC_LR): their shares and lost-sales sums, in region order
  int nl = 0;
  auto flush_lost = [&]() {
    constexpr int RPP = 64 / GW;  // regions per share pass
    for (int i0 = 0; i0 < nl; i0 += RPP) {
      // shares: lane = (region slot ri, warehouse wl)
      const int ri = lane / GW, wl = lane % GW, i = i0 + ri;
      const bool iv = i < nl;
      const int rr = iv ? Ll->lr_r[i] : 0;
      double wt = 0.0;
      if (lost_type == MSC_LOST_COST) {  // softmax(-(of * lost_orders + ov * lost_weight) / alpha)
        double lw = 0.0;                 // unfulfilled[r] . sku_weights, SKU order
#pragma unroll
        for (int j = 0; j < K; j++) lw += (double)(iv ? Ll->lr_ug[i * 8 + j] : 0) * skw[j];
        const double2 t = tab_at(rr, wl);
        const double lg = wl < W ? -(t.x * (double)(iv ? Ll->lr_cnt[i] : 0) + t.y * lw) / alpha : -INFINITY;
        const double mx = sc_group_reduce<GW>(lg, [](double a, double b) { return b > a ? b : a; });
        const double ex = wl < W ? exp(lg - mx) : 0.0;
        wt = wl < W ? ex / group_np_sum<GW>(ex, W) : 0.0;
      } else {  // shipment shares; nothing shipped: the closest warehouse
        const int acc = iv ? Ll->lr_acc[i * LA + wl] : 0;
        const int tot = sc_group_reduce<GW>(acc, [](int a, int b) { return a + b; });
        wt = tot > 0 ? (acc > 0 ? (double)acc / (double)tot : 0.0) : (wl == Lcl[rr] ? 1.0 : 0.0);
      }
      Ll->lr_wt[lane] = wt;
      wave_sync();
      // lost[w][s] += share(w, r) * unfulfilled(r, s), region by region
      const int np = nl - i0 < RPP ? nl - i0 : RPP;
      for (int k = 0; k < np; k++) {
        const double wk = Ll->lr_wt[k * GW + w];
#pragma unroll
        for (int j = 0; j < NS; j++) {
          const int ug = Ll->lr_ug[(i0 + k) * 8 + (skj[j] < 8 ? skj[j] : 7)];
          if (wk != 0.0) lost[j] += wk * (double)ug;
        }
      }
      wave_sync();  // lr_wt is rewritten by the next pass
    }
    nl = 0;
  };

  // region epilogue: lost sales, outbound cost, home features of region r (uniform)
  auto epilogue = [&](int r) {
    ofix += (double)cnt * of_me;
#pragma unroll
    for (int j = 0; j < NS; j++) ovacc[j] += (double)qsr[j] * ov_me;
    if (r == myhome) {
#pragma unroll
      for (int j = 0; j < NS; j++) {
        inc_h[j] = dsum[j];
        shh_h[j] = qsr[j];
      }
      home_done = true;
    }
    if (lost_cnt > 0 && defer) {
      // shares deferred (flush_lost): record the region, its lost orders, the units each warehouse
      // shipped to it (summed over the SKU groups by DPP / permlane swaps) and the unfulfilled units
      int qs = 0;
#pragma unroll
      for (int j = 0; j < NS; j++) qs += qsr[j];
      const int acc = add_groups<GW>(qs);
      if (sg == 0) Ll->lr_acc[nl * LA + w] = acc;
#pragma unroll
      for (int j = 0; j < NS; j++)  // (the SKU's unfulfilled demand: its last rank lane)
        if (lastp && skj[j] < K) Ll->lr_ug[nl * 8 + skj[j]] = u[j];
      if (lane == 0) {
        Ll->lr_r[nl] = r;
        Ll->lr_cnt[nl] = lost_cnt;
      }
      if (++nl == SC_LR) {
        wave_sync();
        flush_lost();
      }
    } else if (lost_cnt > 0 || dbg) {
      int ug[NS];  // the SKU's unfulfilled demand (kept by its last rank lane)
#pragma unroll
      for (int j = 0; j < NS; j++) ug[j] = __shfl(u[j], sg * GW + GW - 1);
      if (lost_cnt > 0) {
        double wt = 0.0;
        if (lost_type == MSC_LOST_CLOSEST) {
          wt = w == Lcl[r] ? 1.0 : 0.0;
        } else {
#pragma unroll
          for (int j = 0; j < NS; j++) {  // [s * GW + w]: slot j's lanes at 64 j + lane
            Lw->iscr[j * 64 + lane] = qsr[j];
            if (lastp) Lw->dscr[skj[j]] = (double)ug[j];
          }
          wave_sync();
          int acc = 0;  // units this warehouse shipped to the region (shipment_quantities[w, r])
#pragma unroll
          for (int j = 0; j < K; j++) acc += Lw->iscr[j * GW + w];
          if (lost_type == MSC_LOST_COST) {  // softmax(-(of * lost_orders + ov * lost_weight) / alpha)
            double lw = 0.0;                 // unfulfilled[r] . sku_weights
#pragma unroll
            for (int j = 0; j < K; j++) lw += Lw->dscr[j] * skw[j];
            const double lg = w < W ? -(of_me * (double)lost_cnt + ov_me * lw) / alpha : -INFINITY;
            const double mx = sc_group_reduce<GW>(lg, [](double a, double b) { return b > a ? b : a; });
            const double ex = w < W ? exp(lg - mx) : 0.0;
            wt = w < W ? ex / group_np_sum<GW>(ex, W) : 0.0;
          } else {  // shipment shares; nothing shipped: the closest warehouse
            const int tot = sc_group_reduce<GW>(acc, [](int a, int b) { return a + b; });
            wt = tot > 0 ? (acc > 0 ? (double)acc / (double)tot : 0.0) : (w == Lcl[r] ? 1.0 : 0.0);
          }
          if (dbg && sg == 0 && w < W) {
            if (info.shipment_quantities) info.shipment_quantities[(e * W + w) * R + r] = acc;
          }
          wave_sync();  // iscr / dscr are rewritten by the next epilogue
        }
        if (wt != 0.0)
#pragma unroll
          for (int j = 0; j < NS; j++) lost[j] += wt * (double)ug[j];
      }
      if (dbg) {
#pragma unroll
        for (int j = 0; j < NS; j++) {
          if (w == 0 && skj[j] < K) {
            if (info.demand_per_region) info.demand_per_region[(e * R + r) * K + skj[j]] = dsum[j];
            if (info.unfulfilled_demands) info.unfulfilled_demands[(e * R + r) * K + skj[j]] = ug[j];
          }
          if (lvj[j] && info.shipment_quantities_by_sku)
            info.shipment_quantities_by_sku[((e * W + w) * R + r) * K + skj[j]] = qsr[j];
        }
        if (lane == 0 && info.lost_order_counts) info.lost_order_counts[e * R + r] = lost_cnt;
        if (lvj[0] && sg == 0 && info.shipment_counts) info.shipment_counts[(e * W + w) * R + r] = cnt;
        if (info.shipment_quantities && !(lost_cnt > 0 && lost_type != MSC_LOST_CLOSEST)) {
#pragma unroll
          for (int j = 0; j < NS; j++) Lw->iscr[j * 64 + lane] = qsr[j];
          wave_sync();
          int acc = 0;
#pragma unroll
          for (int j = 0; j < K; j++) acc += Lw->iscr[j * GW + w];
          if (sg == 0 && w < W) info.shipment_quantities[(e * W + w) * R + r] = acc;
          wave_sync();
        }
      }
    }
#pragma unroll
    for (int j = 0; j < NS; j++) qsr[j] = u[j] = dsum[j] = 0;
    cnt = 0;
    lost_cnt = 0;
  };

  // order ranks (demand_allocator.py:167-173): 4-bit rank of warehouse w at bits 4w (stable order:
  // lower index first on equal cost); padding warehouses w >= W keep rank w
  auto rank_of = [&](const uint4& rv) -> Rho {
    const int rr = (int)(rv.x & 0xffffu);
    double tw = 0.0;  // order.sku_demands.dot(sku_weights)
#pragma unroll
    for (int j = 0; j < K; j++) tw += (double)rec_field(rv, 1 + j) * skw[j];
    double cst[GW];
#pragma unroll
    for (int ww = 0; ww < GW; ww++) {
      const double2 t = tab_at(rr, ww);
      cst[ww] = t.x + t.y * tw;
    }
    Rho rho = 0;
    if constexpr (GW <= 8) {
      // up to 8 warehouses: the 4-bit ranks as one packed 32-bit sum (one select + add per pair)
#pragma unroll
      for (int a = 0; a < GW; a++)
#pragma unroll
        for (int b = a + 1; b < GW; b++)
          if (b < W) rho += cst[b] < cst[a] ? (1u << (4 * a)) : (1u << (4 * b));
#pragma unroll
      for (int ww = 0; ww < GW; ww++)
        if (ww >= W) rho |= (Rho)ww << (4 * ww);
    } else {
      // rank of a = the warehouses that sort before it; 32-bit counters per warehouse (a 64-bit
      // packed sum of 120 selected constants at 16 warehouses ran out of registers)
      int rk[GW];
#pragma unroll
      for (int a = 0; a < GW; a++) rk[a] = a < W ? 0 : a;
#pragma unroll
      for (int a = 0; a < GW; a++)
#pragma unroll
        for (int b = a + 1; b < GW; b++)
          if (b < W) {
            const bool lt = cst[b] < cst[a];
            rk[a] += lt ? 1 : 0;
            rk[b] += lt ? 0 : 1;
          }
#pragma unroll
      for (int a = 0; a < GW; a++) rho |= (Rho)rk[a] << (4 * a);
    }
    return rho;
  };

  SPROF(p_tot);
  SPROF(p_rank);
  SPROF(p_epi);
  SPROF(n_epi);
  SPROF(n_bat);
  SPROF_T(t_begin);
#ifdef MSC_PROF
  const unsigned long long rt_begin = (unsigned long long)wall_clock64();  // constant-rate (100 MHz) clock
#endif
  uint4 nxt = lane < n ? gload4(src, o.base + (int64_t)lane * o.nstep) : make_uint4(0u, 0u, 0u, 0u);
  for (int o0 = 0; o0 < n; o0 += SC_WIN) {
    const int nw = n - o0 < SC_WIN ? n - o0 : SC_WIN;
    const uint4 rv = nxt;
    if (o0 + SC_WIN < n) {  // next window's records in flight while this one is allocated
      const int oi = o0 + SC_WIN + lane;
      nxt = oi < n ? gload4(src, o.base + (int64_t)oi * o.nstep) : make_uint4(0u, 0u, 0u, 0u);
    }
    SPROF_T(t_r0);
    // this lane's order (o0 + lane): region, ranking; batch / region starts against the previous order
    const int rg = (int)(rv.x & 0xffffu);
    const Rho rho = lane < nw ? rank_of(rv) : Rho(0);
    int rg_prev = __shfl_up(rg, 1);
    Rho rho_prev = sc_shfl_up1(rho);
    if (lane == 0) {
      rg_prev = cur;
      rho_prev = cur_rho;
    }
    const bool inw = lane < nw;
    const uint64_t inwm = __ballot(inw);
    const uint64_t rstart = __ballot(inw && rg != rg_prev);
    const uint64_t bstart = split ? inwm
                                  : (__ballot(inw && (rg != rg_prev || rho != rho_prev)) | (inwm & 0x0001000100010000ull));
    uint64_t nzl[NS];  // the window's orders asking for each slot's SKU
#pragma unroll
    for (int j = 0; j < NS; j++) nzl[j] = 0;
#pragma unroll
    for (int q = 0; q < K; q++) {
      const uint64_t b = __ballot(inw && rec_field(rv, 1 + q) != 0u);
#pragma unroll
      for (int j = 0; j < NS; j++) nzl[j] = skj[j] == q ? b : nzl[j];
    }
    Lw->rec[lane] = rv;
    wave_sync();
    SPROF_ADD(p_rank, SPROF_NOW() - t_r0);
    const uint16_t* Lh = reinterpret_cast<const uint16_t*>(Lw->rec);
    for (int i0 = 0; i0 < nw;) {
      const uint64_t later = bstart & ~((2ull << i0) - 1ull);  // batch starts after i0
      const int i1 = __builtin_amdgcn_readfirstlane(later ? (int)__builtin_ctzll(later) : nw);
      const int r = __builtin_amdgcn_readlane(rg, i0);
      const Rho rho_b = sc_readlane(rho, i0);
      int dn[NS];
#pragma unroll
      for (int j = 0; j < NS; j++) dn[j] = Lh[i0 * 8 + fi[j]];
      if ((rstart >> i0) & 1ull) {  // region boundary (orders are region-major)
        SPROF_T(t_e0);
        if (cur >= 0) epilogue(cur);
        SPROF_ADD(p_epi, SPROF_NOW() - t_e0);
        SPROF_ADD(n_epi, 1);
        cur = r;
        const double2 t = tab_at(r, w);
        of_me = t.x;
        ov_me = t.y;
      }
      cur_rho = rho_b;
      SPROF_ADD(n_bat, 1);
      const int paddr = (sg * GW + (int)((rho_b >> (4 * w)) & 0xFu)) << 2;
      int x[NS], incl[NS], excl[NS], a_prev[NS];
#pragma unroll
      for (int j = 0; j < NS; j++) {
        x[j] = __builtin_amdgcn_ds_permute(paddr, inv[j]);  // rank space: inventory of the rank-w warehouse
        incl[j] = group_scan<GW>(x[j], w);
        excl[j] = incl[j] - x[j];
        a_prev[j] = 0;
      }
      int cnt_r = 0;
      if (!split) {
        int D[NS], c1[NS], c2[NS], c3[NS];  // orders with D <= excl, D < incl, D <= incl
#pragma unroll
        for (int j = 0; j < NS; j++) D[j] = c1[j] = c2[j] = c3[j] = 0;
        for (int k = i0; k < i1; k++) {
#pragma unroll
          for (int j = 0; j < NS; j++) {
            const int d = dn[j];
            dn[j] = Lh[(k + 1) * 8 + fi[j]];  // (k + 1 == 64: the scratch after the window, unused)
            D[j] += d;
            c1[j] += D[j] <= excl[j] ? 1 : 0;
            c2[j] += D[j] < incl[j] ? 1 : 0;
            c3[j] += D[j] <= incl[j] ? 1 : 0;
          }
        }
        const int L = i1 - i0;  // <= 16
        uint32_t cm = 0u, lm = 0u;
#pragma unroll
        for (int j = 0; j < NS; j++) {
          const uint32_t nzb = (uint32_t)(nzl[j] >> i0) & ((1u << L) - 1u);
          const int hi = c2[j] < L - 1 ? c2[j] : L - 1;  // fills from orders c1 .. hi (relative to i0)
          cm |= (x[j] > 0 && hi >= c1[j]) ? nzb & ((2u << hi) - 1u) & ~((1u << c1[j]) - 1u) : 0u;
          lm |= lastp ? nzb & ~((1u << c3[j]) - 1u) : 0u;
          const int need = D[j] - excl[j];
          a_prev[j] = need > 0 ? (need < x[j] ? need : x[j]) : 0;
          dsum[j] += D[j];
          u[j] += D[j] - incl[j] > 0 ? D[j] - incl[j] : 0;  // the batch's unfulfilled units (last rank lane)
        }
        const uint32_t both = or_groups<GW>(cm | (lm << 16));
        cnt_r = __builtin_popcount(both & 0xFFFFu);
        lost_cnt += __builtin_popcount((uint32_t)__builtin_amdgcn_readlane((int)both, GW - 1) >> 16);
      } else for (int k = i0; k < i1; k++) {
        int d[NS], f[NS];
        bool anyf = false;
#pragma unroll
        for (int j = 0; j < NS; j++) {
          d[j] = dn[j];
          if (k + 1 < i1) dn[j] = Lh[(k + 1) * 8 + fi[j]];
          const int need = d[j] - excl[j];  // demand left after the cheaper ranks (one-order batch)
          f[j] = need > 0 ? (need < x[j] ? need : x[j]) : 0;  // min(inv, max(0, d - prefix))
          anyf |= f[j] > 0;
        }
        {  // max_splits: only the first max_wh contributing ranks ship (a one-order batch)
          uint32_t m = fold_groups<GW>(__ballot(anyf));
          if (__builtin_popcount(m) > maxwh) {
            uint32_t keep = 0u;
            for (int q = 0; q < maxwh; q++) {
              keep |= m & (0u - m);
              m &= m - 1u;
            }
            m = keep;
          }
          cnt_r += (int)((m >> w) & 1u);
          bool short_any = false;
#pragma unroll
          for (int j = 0; j < NS; j++) {
            f[j] = ((m >> w) & 1u) ? f[j] : 0;
            a_prev[j] = f[j];
            const int rem = d[j] - group_scan<GW>(f[j], w);  // (this SKU's total in its last rank lane)
            u[j] += rem;
            short_any |= lastp && rem > 0;
            dsum[j] += d[j];
          }
          lost_cnt += __ballot(short_any) != 0 ? 1 : 0;
        }
      }
      // total fill and contribution count of the rank back to its warehouse's lane, one bpermute per
      // slot: fill < 2^24 (<= 64 orders of < 2^16 units), count <= 64
#pragma unroll
      for (int j = 0; j < NS; j++) {
        const int back = __builtin_amdgcn_ds_bpermute(paddr, (j == 0 ? cnt_r << 24 : 0) | a_prev[j]);
        const int fw = back & 0xFFFFFF;
        inv[j] -= fw;
        qsr[j] += fw;
        if (j == 0) cnt += (int)((uint32_t)back >> 24);
      }
      i0 = i1;
    }
    wave_sync();  // the window is rewritten next
  }
  SPROF_T(t_e1);
  if (cur >= 0) epilogue(cur);
  if (nl > 0) {
    wave_sync();
    flush_lost();
  }
  SPROF_ADD(p_epi, SPROF_NOW() - t_e1);
  SPROF_ADD(p_tot, SPROF_NOW() - t_begin);
  SPROF_FLUSH(0, p_tot);
  SPROF_FLUSH(1, p_rank);
  SPROF_FLUSH(2, p_epi);
  SPROF_FLUSH(3, n_epi);
  SPROF_FLUSH(4, (unsigned long long)n);
  SPROF_FLUSH(5, 1ull);
  SPROF_FLUSH(6, n_bat);
#ifdef MSC_PROF
  SPROF_FLUSH(7, (unsigned long long)wall_clock64() - rt_begin);
#endif

  // penalty (reward_calculator.py:134-137): (lost_sales * per-SKU cost, or * sku_weights * cost)
  // summed over SKUs in order; outbound variable cost: sum over SKUs of sku_weight * ovacc
  Lw->rec[lane] = make_uint4(0u, 0u, 0u, 0u);
  double* Lov = reinterpret_cast<double*>(Lw->rec);  // [s * GW + w] (128 doubles)
#pragma unroll
  for (int j = 0; j < NS; j++) {
    const double skw_me = skj[j] < K ? c.skw[skj[j]] : 0.0;
    const double pen_me = skj[j] < K ? (pps ? c.pen[skj[j]] : c.pen_scalar) : 0.0;
    Lw->dscr[j * 64 + lane] = pps ? lost[j] * pen_me : (lost[j] * skw_me) * pen_me;
    Lov[j * 64 + lane] = skw_me * ovacc[j];
  }
  wave_sync();
#pragma unroll
  for (int j = 0; j < NS; j++) {
    if (!lvj[j]) continue;
    s.inv[gi[j]] = inv[j];
    if (!FC) {  // (step_c's inputs)
      s.sc_sht[gi[j]] = inv0[j] - inv[j];  // shipped this step = the inventory drop
      s.sc_shh[gi[j]] = home_done ? shh_h[j] : 0;
    }
    if (FA) s.inc[gi[j]] = home_done ? inc_h[j] : 0;  // (phase A here: nobody zeroed it)
    else if (home_done) s.inc[gi[j]] = inc_h[j];  // (step_a zeroed it: a home region without orders leaves 0)
    if (dbg) {
      if (info.lost_sales) info.lost_sales[e * WK + w * K + skj[j]] = lost[j];
      if (info.fulfilled_per_warehouse) info.fulfilled_per_warehouse[e * WK + w * K + skj[j]] = inv0[j] - inv[j];
    }
  }
  double pen_w = 0.0, out_w = 0.0;  // (lanes sg == 0, w < W)
  if (sg == 0 && w < W) {
    double ovar = 0.0;
#pragma unroll
    for (int j = 0; j < K; j++) {
      pen_w += Lw->dscr[j * GW + w];
      ovar += Lov[j * GW + w];
    }
    out_w = ofix + ovar;
    if (!FC) {
      s.sc_pen[w * E + e] = pen_w;
      s.sc_out[w * E + e] = out_w;
    }
  }
  if constexpr (FC) {
    // ---- phase C (step_c_kernel, multi_env.py:307-327, 747-793; reward_calculator.py:96-190) for
    // this wave's env, its inputs in registers: lane (s, w) holds SKU s of warehouse w after the
    // allocation. The observation builder's per-SKU inputs are staged in LDS; lane w < W then
    // builds agent w's vector (obs_emit, the code step_c runs) and its reward.
    const int hslot = t_now % MSC_HISTORY, n_hist = t_now + 1 < MSC_HISTORY ? t_now + 1 : MSC_HISTORY;
    const int RING = c.RING, tm = t_now % RING;
    ScFcLds* Lf = reinterpret_cast<ScFcLds*>(Ll);
    const bool lv = lvj[0];
    const int i = w * K + skj[0];
    const int64_t g = gi[0];
    // loads first (one vmcnt for loads and stores): forecast, the 4 older history slots, the ring
    int hv[MSC_HISTORY], rv[SC_FC_RING];
    float fo = 0.0f;
    int eltv = 0;
    if (lv) {
      fo = s.fc[g];
      eltv = c.elt[i];
#pragma unroll
      for (int a = 1; a < MSC_HISTORY; a++) {  // age a: slot (t - a) mod 5
        const int q = (t_now - a) % MSC_HISTORY;
        hv[a] = a < n_hist ? s.hist[((int64_t)(q < 0 ? q + MSC_HISTORY : q) * WK + i) * E + e] : 0;
      }
#pragma unroll
      for (int q = 0; q < SC_FC_RING; q++) rv[q] = q < RING ? s.ring_q[((int64_t)i * RING + q) * E + e] : 0;
    }
    const int dh = home_done ? inc_h[0] : 0;  // this step's incoming home demand (step_a zeroed s.inc)
    const int sh = home_done ? shh_h[0] : 0, sa = (inv0[0] - inv[0]) - sh;
    hv[0] = dh;
    float fcn = 0.0f, rm = 0.0f;
    int pend = 0;
    if (lv) {
      s.hist[((int64_t)hslot * WK + i) * E + e] = dh;
      fcn = 0.3f * (float)dh + 0.7f * fo;  // EMA forecast (f32)
      s.fc[g] = fcn;
      int hs = 0;
#pragma unroll
      for (int a = 0; a < MSC_HISTORY; a++) hs += a < n_hist ? hv[a] : 0;
      rm = n_hist > 0 ? (float)hs / (float)n_hist : 0.0f;
#pragma unroll
      for (int q = 0; q < SC_FC_RING; q++) pend += rv[q];
    }
    // holding cost terms (reward_calculator.py:127-131), summed per warehouse in SKU order below
    const int sk0 = skj[0];
    double hterm = 0.0;
    if (lv)
      hterm = c.hold_per_sku ? (double)inv[0] * c.hold[sk0] : ((double)inv[0] * c.skw[sk0]) * c.hold_scalar;
    Lf->v[FC_INV][lane] = inv[0];
    Lf->v[FC_DH][lane] = dh;
    Lf->v[FC_SH][lane] = sh;
    Lf->v[FC_SA][lane] = sa;
    Lf->v[FC_PEND][lane] = pend;
    Lf->v[FC_FC][lane] = __float_as_int(fcn);
    Lf->v[FC_RM][lane] = __float_as_int(rm);
    Lw->dscr[lane] = hterm;
    wave_sync();
    const bool agent = sg == 0 && w < W;  // lane w builds agent w
    const bool trunc = t_now + 1 >= c.T;
    double rw = 0.0;
    if (agent) {
      double hold = 0.0;
#pragma unroll
      for (int j = 0; j < K; j++) hold += Lw->dscr[j * GW + w];
      const double inb = FA ? inb_a : s.sc_inb[w * E + e];
      rw = -((((hold + pen_w) + out_w) + inb) * c.scale);
      if (dbg && info.costs) {
        info.costs[(e * 4 + 0) * W + w] = hold;
        info.costs[(e * 4 + 1) * W + w] = pen_w;
        info.costs[(e * 4 + 2) * W + w] = out_w;
        info.costs[(e * 4 + 3) * W + w] = inb;
      }
    }
    Lov[lane] = rw;  // (the outbound partials are read)
    wave_sync();
    if (agent) {
      double v = rw;
      if (c.scope == MSC_SCOPE_TEAM) {  // team scope: sum over agents in agent order
        v = 0.0;
        for (int j = 0; j < W; j++) v += Lov[j];
      }
      io.rew[e * W + w] = (float)v;
      if (io.rew64) io.rew64[e * W + w] = v;
    }
    // the observation, every lane (s, w) writing SKU s's values of agent w (obs_emit's arithmetic
    // value by value; the agent's totals from the staged SKU values, in SKU order)
    float* dst = trunc ? io.final_obs : io.obs;
    if (dst && lv) fc_obs_lane<K, GW>(c, Lf, w, sk0, tm, n_hist, eltv, rv, hv, dst + (e * W + w) * (int64_t)c.L);
    // truncation: reset the env (one sequential RNG pass), then every agent's reset observation
    if (trunc) {
      if (lane == 0) reset_env<K>(c, s, e, 0, nullptr);
      __builtin_amdgcn_s_waitcnt(0);  // (the reset's state stores have landed before they are read)
      wave_sync();
      if (agent) build_obs_agent<K>(c, s, e, w, 0, 0, nullptr, nullptr, 0, io.obs + e * W * c.L);
    }
    if (lane == 0) {
      io.trunc[e] = trunc ? 1 : 0;
      if (!trunc) s.t[e] = t_now + 1;
    }
  }
}

static bool alloc_scan_tab(const EnvConst& c, int GW) { return c.sc_tab && sc_tab_bytes(c.R, GW) <= SC_TAB_MAX; }
size_t alloc_scan_lds_bytes(const EnvConst& c) {
  const int GW = sc_gw(c.W), NS = sc_ns(c.K, GW);
  const size_t wave_b = NS > 1 ? sizeof(ScWaveLds<2>) : sizeof(ScWaveLds<1>);
  const size_t lost_b = GW > 8 ? sizeof(ScLostLds<16>) : sizeof(ScLostLds<8>);
  // (the fused phase C stages its inputs where the deferred regions were)
  const size_t tail_b = c.fuse_c ? (lost_b > sizeof(ScFcLds) ? lost_b : sizeof(ScFcLds)) : (c.scan_defer ? lost_b : 0);
  return (alloc_scan_tab(c, GW) ? sc_tab_bytes(c.R, GW) : 0) + sizeof(int32_t) * ((c.R + 3) & ~3) +
         SC_WAVES * wave_b + SC_WAVES * tail_b;
}
// phase C fused into the scan allocator: one slot per lane (<= 8 warehouses), pending rings of at
// most SC_FC_RING slots
bool alloc_scan_fuse_supported(int W, int K, int RING) { return W <= 8 && K <= 6 && RING <= SC_FC_RING; }
// <= 8 warehouses with <= 6 SKUs (one slot per lane), 9-16 warehouses with <= 6 SKUs (two slots
// above 4 SKUs)
bool alloc_scan_supported(int W, int K) { return W <= 16 && K <= 6; }

#ifndef MSC_SC_ND
#define MSC_SC_ND 1  // the fused scan step without step info runs its no-info instantiation
#endif
template <int K>
static hipError_t launch_scan_k(const EnvConst& c, const DevEnv* d, const StepIO& io, hipStream_t st) {
  using KFn = void (*)(const DevEnv*, StepIO);
  const int GW = sc_gw(c.W);
  const bool t = alloc_scan_tab(c, GW);
  KFn f;
  if (c.fuse_c && c.fuse_a && MSC_SC_ND && !io.has_info) {
    f = GW == 2 ? (t ? (KFn)alloc_scan_kernel<K, 2, true, true, true, true> : (KFn)alloc_scan_kernel<K, 2, false, true, true, true>)
      : GW == 4 ? (t ? (KFn)alloc_scan_kernel<K, 4, true, true, true, true> : (KFn)alloc_scan_kernel<K, 4, false, true, true, true>)
                : (t ? (KFn)alloc_scan_kernel<K, 8, true, true, true, true> : (KFn)alloc_scan_kernel<K, 8, false, true, true, true>);
    if (GW > 8) return hipErrorInvalidValue;
  } else if (c.fuse_c && c.fuse_a) {
    f = GW == 2 ? (t ? (KFn)alloc_scan_kernel<K, 2, true, true, true> : (KFn)alloc_scan_kernel<K, 2, false, true, true>)
      : GW == 4 ? (t ? (KFn)alloc_scan_kernel<K, 4, true, true, true> : (KFn)alloc_scan_kernel<K, 4, false, true, true>)
                : (t ? (KFn)alloc_scan_kernel<K, 8, true, true, true> : (KFn)alloc_scan_kernel<K, 8, false, true, true>);
    if (GW > 8) return hipErrorInvalidValue;
  } else if (c.fuse_c) {
    f = GW == 2 ? (t ? (KFn)alloc_scan_kernel<K, 2, true, true> : (KFn)alloc_scan_kernel<K, 2, false, true>)
      : GW == 4 ? (t ? (KFn)alloc_scan_kernel<K, 4, true, true> : (KFn)alloc_scan_kernel<K, 4, false, true>)
                : (t ? (KFn)alloc_scan_kernel<K, 8, true, true> : (KFn)alloc_scan_kernel<K, 8, false, true>);
    if (GW > 8) return hipErrorInvalidValue;
  } else {
    f = GW == 2 ? (t ? (KFn)alloc_scan_kernel<K, 2, true> : (KFn)alloc_scan_kernel<K, 2, false>)
      : GW == 4 ? (t ? (KFn)alloc_scan_kernel<K, 4, true> : (KFn)alloc_scan_kernel<K, 4, false>)
      : GW == 8 ? (t ? (KFn)alloc_scan_kernel<K, 8, true> : (KFn)alloc_scan_kernel<K, 8, false>)
                : (t ? (KFn)alloc_scan_kernel<K, 16, true> : (KFn)alloc_scan_kernel<K, 16, false>);
  }
  const size_t lds = alloc_scan_lds_bytes(c);
  if (lds > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(f, dim3((unsigned)((c.E + SC_WAVES - 1) / SC_WAVES)), dim3(64 * SC_WAVES), lds, st, d, io);
  return hipGetLastError();
}

hipError_t launch_alloc_scan(const EnvConst& c, const DevEnv* d, const StepIO& io, hipStream_t st) {
  if (!alloc_scan_supported(c.W, c.K)) return hipErrorInvalidValue;
  switch (c.K) {
    case 1: return launch_scan_k<1>(c, d, io, st);
    case 2: return launch_scan_k<2>(c, d, io, st);
    case 3: return launch_scan_k<3>(c, d, io, st);
    case 4: return launch_scan_k<4>(c, d, io, st);
    case 5: return launch_scan_k<5>(c, d, io, st);
    case 6: return launch_scan_k<6>(c, d, io, st);
    default: return hipErrorInvalidValue;
  }
}

#ifdef MSC_PROF
extern "C" int msc_debug_prof_scan(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_prof_scan), sizeof(unsigned long long) * 8) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[8] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_prof_scan), z, sizeof z) != hipSuccess) return -1;
  }
  return 0;
}
#endif

}  // namespace msc
