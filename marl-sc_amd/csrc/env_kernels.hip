// env_kernels.hip -- HIP kernels of the vectorised InventoryEnvironment (gfx950 / CDNA4).
//
// A step is four launches on the caller's stream:
//   1. demand_unit_kernel  PoissonDemandSampler.sample (demand_sampler.py:105-163): generator
//      waves + a one-unit-per-round parser draw every order of the step from the env's own
//      PCG64 stream into a per-step order buffer (records [slot][E], 16 B each), region-major
//      exactly like the reference's list;
//   2-4. step_a / step_b / step_c  InventoryEnvironment.step (multi_env.py:253-366): actions,
//      lead times, orders and arrivals; the greedy allocation with the lost-sales epilogue;
//      inventory/history/forecast, rewards, observations and the in-kernel reset at truncation.
// Integer state is exact; f32 observation arithmetic follows numpy's dtype flow operation by
// operation (the library is built with -ffp-contract=off so no FMA contraction changes a
// rounding); rewards are f64.
#include <hip/hip_runtime.h>
#include <math.h>

#include "env.hpp"
#include "kcommon.hpp"
#include "rng.hpp"
#include "demand_common.hpp"
#include "obs_common.hpp"

namespace msc {

#if defined(MSC_PROF) && !defined(MSC_EK_WIDE)
// in-kernel cycle accounting (profiling builds only: make prof -> libmarlsc_prof.so; SKU counts <= 8)
__device__ unsigned long long g_prof[16];
#define PROF_DECL(v) unsigned long long v = 0
#define PROF_NOW() ((unsigned long long)clock64())
#define PROF_T(v) const unsigned long long v = PROF_NOW()
#define PROF_ADD(v, x) (v) += (x)
#define PROF_FLUSH(i, v) \
  if ((threadIdx.x & 63) == 0) atomicAdd(&g_prof[i], (v))
#else
#define PROF_DECL(v)
#define PROF_NOW() 0ull
#define PROF_T(v)
#define PROF_ADD(v, x)
#define PROF_FLUSH(i, v)
#endif

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


// all W agents of env e (reset path: one lane per env)
template <int K>
__device__ __forceinline__ void build_obs(const EnvConst& c, const EnvState& s, int64_t e, int t_now, int n_hist,
                                          const int32_t* shh, const int32_t* sht, float* out) {
  for (int w = 0; w < c.W; w++) build_obs_agent<K>(c, s, e, w, t_now, n_hist, shh, sht, BS, out);
}

// ------------------------------------------------------------------------------------------
// kernels
// ------------------------------------------------------------------------------------------
template <int K>
__global__ __launch_bounds__(BS) void reset_kernel(const DevEnv* __restrict__ dp, const uint8_t* mask,
                                                   const uint32_t* new_roots, int32_t flags, float* obs) {
  const EnvConst& c = dp->c;
  const EnvState& s = dp->s;
  const int64_t e = (int64_t)blockIdx.x * BS + threadIdx.x;
  if (e >= c.E) return;
  if (mask && !mask[e]) return;
  reset_env<K>(c, s, e, flags, new_roots ? new_roots + e : nullptr);
  if (obs) build_obs<K>(c, s, e, 0, 0, nullptr, nullptr, obs + e * c.W * c.L);
}

// PoissonDemandSampler.sample (demand_sampler.py:105-163), production version: a flat per-lane
// parser whose every iteration draws ONE uniform per active lane and then settles the zero-draw
// transitions in a single branch-free pass. The pass is complete because the reference schema
// requires every Poisson rate to be strictly positive (PositiveFloat, src/config/schema.py:191),
// so each chain qty-done -> emit -> next order / next region ends at a state that draws.
// The thresholds a lane may need in the NEXT pass (its next SKU's exp(-lambda_q), the next
// region's exp(-lambda_o) and p) are prefetched from LDS at the end of each pass, so the LDS
// latency hides under the following PCG64 draw. No branch except the order-record store.

// ------------------------------------------------------------------------------------------
// demand_park4_kernel: the parking parser with multi-draw hot steps (A/B baseline of
// demand_unit_kernel: MSC_DEMAND_IMPL=park4). Generators as in demand_unit_kernel; the parser parks
// a lane whose unit ended and settles parked lanes in batches of >= park_min.
//
// Same generator / parser split and settle pass as demand_park_kernel, but one hot step advances
// a lane's unit by up to PD = 4 draws at once: the Poisson products p1..p4 are chained
// (prod*U0, p1*U1, ...), compared in parallel, and the lane consumes the leading run of
// "continue" draws plus the ending draw; a mask unit takes min(4, K - k) Bernoulli draws (its
// running product is reset to 1 before every multiply). The per-step overhead (the park check, the
// LDS round trip for the lane's next uniforms) is thus paid once per ~3 draws instead of once per
// draw. The ring is lane-major [64][DCAP4 + 1] (padded: conflict-free 8-B reads) so the four
// consecutive positions a lane needs are independent reads issued right after the previous
// step, overlapping the park check. A chunk is HS4 hot steps (<= PD * HS4 draws per lane).
// ------------------------------------------------------------------------------------------
constexpr int PD = 4;                // draws per hot step
constexpr int HS4 = 4;               // hot steps per chunk
constexpr int DCAP4 = 2 * PD * HS4;  // per-lane ring capacity (2 x the max draws of one chunk)
constexpr int DSTR4 = DCAP4 + 1;     // padded lane stride (doubles)

__host__ __device__ constexpr size_t park4_lds_fixed() {
  return (size_t)BS * DSTR4 * sizeof(double) + (size_t)2 * BS * sizeof(int32_t);
}

template <int K, int G, bool LDS_TAB>
__global__ __launch_bounds__(BS * (1 + G)) void demand_park4_kernel(const DevEnv* __restrict__ dp) {
  const EnvConst& c = dp->c;
  const EnvState& s = dp->s;
  const int R = c.R;
  constexpr int NV = Rec<K>::NV;
  constexpr int NW = 4 * NV;
  extern __shared__ __attribute__((aligned(16))) double plds[];
  __shared__ int more[2];
  double* ring = plds;                                              // [BS][DSTR4]
  int32_t* rdv = reinterpret_cast<int32_t*>(plds + BS * DSTR4);     // [2][BS]
  const double* To = c.enlam_o;
  const double* Tk = c.p_skip;
  const double* Tq = c.enlam_q;
  if constexpr (LDS_TAB) {
    double* lo = plds + BS * DSTR4 + BS;
    double* lk = lo + R;
    double* lq = lk + R;
    for (int i = threadIdx.x; i < R; i += blockDim.x) {
      lo[i] = c.enlam_o[i];
      lk[i] = c.p_skip[i];
    }
    for (int i = threadIdx.x; i < R * K; i += blockDim.x) lq[i] = c.enlam_q[i];
    To = lo;
    Tk = lk;
    Tq = lq;
  }
  const int wave = threadIdx.x / BS, lane = threadIdx.x % BS;
  const int64_t E = c.E;
  const int64_t e = (int64_t)blockIdx.x * c.epw_dem + lane;
  const bool valid = lane < c.epw_dem && e < E;
  double* myring = ring + lane * DSTR4;

  if (wave > 0) {
    // ---------------- generator g: stream positions g, g + G, g + 2G, ...
    const int g = wave - 1;
    uint64_t th = 0, tl = 0, ih = 0, il = 1;
    if (valid) {
      Pcg64 rg = load_rng(s, 0, e, E);
      for (int j = 0; j <= g; j++) pcg_step(rg);
      th = rg.s_hi;
      tl = rg.s_lo;
      ih = rg.i_hi;
      il = rg.i_lo;
    }
    uint64_t mh = PCG_MUL_HI, ml = PCG_MUL_LO, ch = ih, cl = il;
    if constexpr (G > 1) pcg_jump_coeffs(G, ih, il, mh, ml, ch, cl);
    int pg = g;
    auto gen_to = [&](int target) {
      while (pg < target) {
        myring[pg & (DCAP4 - 1)] = u64_to_double(pcg_output(th, tl));
        uint64_t nh, nl;
        mul128(th, tl, mh, ml, nh, nl);
        add128(nh, nl, ch, cl);
        th = nh;
        tl = nl;
        pg += G;
      }
    };
    if (valid) gen_to(DCAP4);
    __syncthreads();
    for (int ci = 0;; ci++) {
      if (valid) gen_to(rdv[(ci & 1) * BS + lane] + DCAP4);
      __syncthreads();
      if (!more[ci & 1]) break;
    }
    return;
  }

  // ---------------- parser
  Pcg64 r0{};
  if (valid) {
    r0 = load_rng(s, 0, e, E);
    store_rng_pre(s, e, E, r0);
  }
  rdv[lane] = 0;
  int st = valid ? PS_ORD : PS_DONE, r = 0, x = 0, k = 0, left = 0, sq = 0, n = 0, rd = 0;
  unsigned mask = 0;
  int pk = 0, mf = 0, live = valid ? 1 : 0;
  uint32_t w[NW];
#pragma unroll
  for (int j = 0; j < NW; j++) w[j] = 0;
  const int cap = c.order_cap;
  const int pmin = c.park_min;
  MSC_GLOBAL uint4* out = gp(s.orders + e);
  __syncthreads();
  double prod = 1.0, thr = To[0];
  auto settle = [&]() {
    const bool is_ord = st == PS_ORD, is_qty = st == PS_QTY;
    const uint32_t v = (uint32_t)(x > 1 ? x : 1);  // max(1, Poisson(lambda_q))
    const int h = 1 + sq;
#pragma unroll
    for (int j = 0; j < NW; j++) w[j] |= (is_qty && (h >> 1) == j) ? v << (16 * (h & 1)) : 0u;
    mask = is_qty ? (mask & (mask - 1u)) : mask;
    const int nsq = mask ? __builtin_ctz(mask) : 0;
    const int rn = r + 1 < R ? r + 1 : r;
    const double q_thr = Tq[r * K + nsq], k_thr = Tk[r], o_thr = To[rn];
    const bool start_q = !is_ord && mask != 0;
    const bool emit = !is_ord && mask == 0;
    if (emit && n < cap) {
#pragma unroll
      for (int j = 0; j < NV; j++)
        gstore4(out, ((int64_t)n * NV + j) * E, make_uint4(w[4 * j], w[4 * j + 1], w[4 * j + 2], w[4 * j + 3]));
    }
    n += emit ? 1 : 0;
    left = is_ord ? x : left - (emit ? 1 : 0);
    const bool start_order = !start_q && left > 0;
    const bool next_region = !start_q && left <= 0;
    const bool start_region = next_region && r + 1 < R;
    r += start_region ? 1 : 0;
    sq = start_q ? nsq : sq;
    st = start_q ? PS_QTY : start_order ? PS_MASK : start_region ? PS_ORD : PS_DONE;
    thr = start_q ? q_thr : start_order ? k_thr : o_thr;
    mask = start_order ? 0u : mask;
#pragma unroll
    for (int j = 0; j < NW; j++) w[j] = start_order ? (j == 0 ? (uint32_t)r : 0u) : w[j];
    prod = 1.0;
    x = 0;
    k = 0;
    pk = 0;
    mf = st == PS_MASK ? 1 : 0;
    live = st != PS_DONE ? 1 : 0;
  };
  PROF_DECL(p_all);
  PROF_DECL(p_set);
  PROF_DECL(p_bar);
  PROF_DECL(n_set);
  PROF_DECL(n_round);
  PROF_DECL(n_chunk);
  PROF_T(t_start);
  for (int ci = 0;; ci++) {
    double u0 = myring[rd & (DCAP4 - 1)], u1 = myring[(rd + 1) & (DCAP4 - 1)];
    double u2 = myring[(rd + 2) & (DCAP4 - 1)], u3 = myring[(rd + 3) & (DCAP4 - 1)];
#pragma unroll
    for (int hs = 0; hs < HS4; hs++) {
      // ---- hot step: up to PD draws of the lane's current unit
      const int a = live & (pk ^ 1);
      const double one = 1.0;
      const double p1 = prod * u0;
      const double p2 = (mf ? one : p1) * u1;
      const double p3 = (mf ? one : p2) * u2;
      const double p4 = (mf ? one : p3) * u3;
      const int c1 = p1 > thr ? 1 : 0, c2 = p2 > thr ? 1 : 0, c3 = p3 > thr ? 1 : 0, c4 = p4 > thr ? 1 : 0;
      // Poisson unit: leading run of continues, then the ending draw
      const int n2 = c1 & c2, n3 = n2 & c3, n4 = n3 & c4;
      const int ncont = c1 + n2 + n3 + n4;
      // mask unit: take min(PD, K - k) Bernoulli draws; bit set = SKU drawn (U < p <=> !(U > p_skip))
      const int take = (K - k) < PD ? (K - k) : PD;
      const unsigned bits = (unsigned)((c1 ^ 1) | ((c2 ^ 1) << 1) | ((c3 ^ 1) << 2) | ((c4 ^ 1) << 3)) & ((1u << take) - 1u);
      const int am = a & mf, ap = a & (mf ^ 1);
      mask |= am ? bits << k : 0u;
      k += am ? take : 0;
      x += ap ? ncont : 0;
      prod = (ap & n4) ? p4 : prod;
      const int cons = mf ? take : (n4 ? PD : ncont + 1);
      pk |= (am & ((k + (64 - K)) >> 6)) | (ap & (n4 ^ 1));
      rd += a ? cons : 0;
      u0 = myring[rd & (DCAP4 - 1)];
      u1 = myring[(rd + 1) & (DCAP4 - 1)];
      u2 = myring[(rd + 2) & (DCAP4 - 1)];
      u3 = myring[(rd + 3) & (DCAP4 - 1)];
      const uint64_t pkm = __ballot(pk);
      if (pkm != 0 && (__popcll(pkm) >= pmin || pkm == __ballot(live))) {
        PROF_T(ts);
        if (pk) settle();
        PROF_ADD(p_set, PROF_NOW() - ts);
        PROF_ADD(n_set, 1);
      }
      PROF_ADD(n_round, 1);
    }
    const bool any = __ballot(st != PS_DONE) != 0;
    rdv[((ci + 1) & 1) * BS + lane] = rd;
    if (lane == 0) more[ci & 1] = any ? 1 : 0;
    PROF_T(tb);
    __syncthreads();
    PROF_ADD(p_bar, PROF_NOW() - tb);
    PROF_ADD(n_chunk, 1);
    if (!any) break;
  }
  PROF_ADD(p_all, PROF_NOW() - t_start);
  PROF_FLUSH(0, p_all);
  PROF_FLUSH(1, p_set);
  PROF_FLUSH(2, p_bar);
  PROF_FLUSH(3, n_set);
  PROF_FLUSH(4, n_round);
  PROF_FLUSH(5, n_chunk);
  PROF_FLUSH(6, 1ull);
  if (!valid) return;
  pcg_advance(r0, (uint64_t)rd);
  store_rng(s, 0, e, E, r0);
  if (n > cap) {
    atomicOr(s.err, ERR_ORDER_OVERFLOW);
    n = cap;
  }
  s.n_orders[e] = n;
}

// ------------------------------------------------------------------------------------------
// demand_unit_kernel: converged "one unit per round" parser (production default).
//
// Same generator waves as the parking kernels, but the parser no longer parks lanes: in every
// round EVERY live lane runs its current unit over the next UD = 8 uniforms at once and settles
// it in the same round. A Poisson unit (a region's order count or one SKU quantity) chains the
// UD products p_i = p_{i-1} * U_i (the reference's `prod *= U` in order, bit-exact), compares
// each against exp(-lambda) and takes the leading run of continues plus the ending draw; the
// rare unit that is still going after UD draws (X >= UD) carries its product into the next
// round. A mask unit compares min(UD, K - k) uniforms against the folded Bernoulli threshold.
// With no park check, no ballot and no lane-mask logic the round is straight-line code, and a
// wave runs for ~ max over its lanes of (units + overflow segments) ~ 1.4k rounds at 8x64x5
// instead of ~3k hot steps + ~1.5k settle passes of demand_park4_kernel.
// Ring: slot-major [USLOTS][64] (lane fastest), slot = position mod UCAP; slots 0..UD-2 are
// mirrored at UCAP.. so the UD reads of a round are one base address + immediate offsets (no wrap
// arithmetic). Every lane reads its own slot, and the lanes' slots differ, so only a layout whose
// bank depends on the lane alone is conflict-free: [slot][lane] maps lane l to banks 2l, 2l + 1
// (mod 64) whatever the slot, and the generator's writes of one position are one contiguous row.
// ------------------------------------------------------------------------------------------
// UNI: every region has the same lambda_orders, probability_skus and lambda_quantity (scalar
// sampler parameters, demand_sampler.py:99-102, or equal per-region arrays): the three thresholds
// live in scalar registers and the settle step needs no table reads or region-indexed addressing.
// EA (episode-ahead demand): lane = (slot, env) of a future episode; the
// parser runs all T steps of the episode back to back (at the end of a step's last region it starts
// region 0 of the next step) and writes the orders env-contiguously into the slot, with the record
// offset and stream position at every step boundary.
template <int K, int G, bool LDS_TAB, bool UNI, bool EA>
__global__ __launch_bounds__(BS * (1 + G)) __attribute__((amdgpu_waves_per_eu(MSC_DEM_WPE))) void demand_unit_kernel(
    const DevEnv* __restrict__ dp, EaLaunch ea) {
  const EnvConst& c = dp->c;
  const EnvState& s = dp->s;
  const int R = c.R;
  constexpr int NV = Rec<K>::NV;
  extern __shared__ __attribute__((aligned(16))) double plds[];
  __shared__ int more[2];
  double* ring = plds;                                             // [USLOTS][BS]
  int32_t* rdv = reinterpret_cast<int32_t*>(plds + BS * USLOTS);   // [2][BS]
  const double* To = c.enlam_o;
  const double* Tk = c.p_skip;
  const double* Tq = c.enlam_q;
  if constexpr (LDS_TAB) {
    double* lo = plds + BS * USLOTS + BS;
    double* lk = lo + R;
    double* lq = lk + R;
    for (int i = threadIdx.x; i < R; i += blockDim.x) {
      lo[i] = c.enlam_o[i];
      lk[i] = c.p_skip[i];
    }
    for (int i = threadIdx.x; i < R * K; i += blockDim.x) lq[i] = c.enlam_q[i];
    To = lo;
    Tk = lk;
    Tq = lq;
  }
  const int rot = c.parser_rot == 1 ? (int)(blockIdx.x >> 8) : c.parser_rot == 2 ? (int)blockIdx.x
                : c.parser_rot == 3 ? (int)(blockIdx.x >> 3) : 0;
  const int wave = ((int)(threadIdx.x / BS) + rot) % (1 + G), lane = threadIdx.x % BS;  // role 0 parses
  const int64_t E = c.E;
  const int64_t vlane = (int64_t)blockIdx.x * c.epw_dem + lane;
  int64_t e = vlane;
  int slot = 0, ea_k = 0;
  bool valid = lane < c.epw_dem && vlane < E;
  if constexpr (EA) {
    valid = lane < c.epw_dem && vlane < (int64_t)ea.nslots * E;
    ea_k = valid ? (int)(vlane / E) : 0;
    e = valid ? vlane - (int64_t)ea_k * E : 0;
    slot = (ea.slot0 + ea_k) % c.ea_S;
  }
  double* myring = ring + lane;
  int ea_cnt_new = 0;
  // EA chunk [t0, t1): stream position and record count where step t0 starts (0 for t0 == 0)
  uint32_t ea_p0 = 0;
  int ea_n0 = 0;
  if constexpr (EA) {
    if (valid && ea.t0 > 0) {
      ea_p0 = s.ea_pos[((int64_t)slot * c.T + (ea.t0 - 1)) * E + e];
      ea_n0 = s.ea_off[((int64_t)slot * (c.T + 1) + ea.t0) * E + e];
    }
  }
  auto start_rng = [&]() -> Pcg64 {
    if constexpr (EA) {
      uint32_t root;
      if (ea.t0 == 0) {
        root = ea_root(c, s, ea, e, ea_k, slot, ea_cnt_new);
      } else {  // the episode's counter is in the slot since its first chunk (wv = counter - 1)
        const uint32_t w2[2] = {s.orig_root[e], (uint32_t)(s.ea_cnt[(int64_t)slot * E + e] - 1)};
        root = ss_u32(w2, 2);
      }
      Pcg64 r;
      pcg_seed_child(r, root, 2);  // 'demand_sampler' child of the episode's root (seed_manager.py:100-120)
      if (ea_p0) pcg_advance(r, (uint64_t)ea_p0);
      return r;
    } else {
      return load_rng(s, 0, e, E);
    }
  };

  if (wave > 0) {
    // ---------------- generator g: stream positions g, g + G, g + 2G, ...
    if (MSC_GEN_PRIO > 0) __builtin_amdgcn_s_setprio(MSC_GEN_PRIO);
    const int g = wave - 1;
    uint64_t th = 0, tl = 0, ih = 0, il = 1;
    if (valid) {
      Pcg64 rg = start_rng();
      for (int j = 0; j <= g; j++) pcg_step(rg);
      th = rg.s_hi;
      tl = rg.s_lo;
      ih = rg.i_hi;
      il = rg.i_lo;
    }
    uint64_t mh = PCG_MUL_HI, ml = PCG_MUL_LO, ch = ih, cl = il;
    if constexpr (G > 1) pcg_jump_coeffs(G, ih, il, mh, ml, ch, cl);
    int pg = g;
    auto gen_to = [&](int target) {
      while (pg < target) {
        const double u = pcg_output_double(th, tl);
        const int slot = pg & (UCAP - 1);
        myring[slot * BS] = u;
        myring[(slot < UD - 1 ? slot + UCAP : USLOTS - 1) * BS] = u;  // mirror (or the dummy row)
        lcg128(th, tl, mh, ml, ch, cl);
        pg += G;
      }
    };
    // Refill by quota (see unit_quota): in phase ci the parser reads positions [rdp, rdp + UHS*UD)
    // of chunk ci, so positions up to rdp + UCAP are free; every lane gets at most QUOTA more, the
    // same for every lane, instead of exactly what it consumed (which makes each wave loop for its
    // busiest lane). A lane the next chunk could overrun is topped up behind one extra barrier.
    int tgt = UCAP;
    if (valid) gen_to(UCAP);
    __syncthreads();
    for (int ci = 0;; ci++) {
      const int rdp = rdv[(ci & 1) * BS + lane];
      tgt = unit_quota(tgt, rdp);
      if (valid) gen_to(tgt);
      __syncthreads();
      if (!more[ci & 1]) break;
      const int need = rdv[((ci + 1) & 1) * BS + lane] + UHS * UD;
      if (__ballot(valid && tgt < need) != 0) {
        tgt = tgt > need ? tgt : need;
        if (valid) gen_to(tgt);
        __syncthreads();
      }
    }
    return;
  }

  // ---------------- parser
  // Older and higher-priority waves win VALU issue arbitration on a SIMD (MI355X_MICROARCH.md,
  // wave scheduling): the parser is the per-env critical path, the generators only need to stay
  // a chunk ahead of it.
  __builtin_amdgcn_s_setprio(MSC_PARSER_PRIO);
  Pcg64 r0{};
  if (valid) {
    r0 = start_rng();
    if constexpr (!EA) store_rng_pre(s, e, E, r0);
  }
  rdv[lane] = 0;
  static_assert(K <= UD, "a mask unit completes in one round");
  int st = valid ? PS_ORD : PS_DONE, r = 0, x = 0, left = 0, sq = 0, n = ea_n0, rd = 0;
  int tstep = EA ? ea.t0 : 0;  // EA: step of the episode being parsed
  unsigned mask = 0;
  int mf = 0, live = valid ? 1 : 0, pend = 0;
  const int cap = EA ? (int)c.ea_cap : c.order_cap;
  // the current order's record: written as {region, 0, ..., 0} when the order starts, then each
  // SKU quantity is stored into its 16-bit field as its unit ends (same-lane stores to one
  // address stay in program order)
  const int64_t vstride = EA ? 16 : E * 16;       // bytes between the uint4 words of a record
  const int64_t rstride = (int64_t)NV * vstride;  // bytes between consecutive records of a lane
  MSC_GLOBAL char* recp = reinterpret_cast<MSC_GLOBAL char*>(
      gp(EA ? s.ea_rec + ((int64_t)slot * E + e) * c.ea_cap * NV : s.orders + e)) + (int64_t)(n - 1) * rstride;
  // EA step boundaries: record offset / stream position after each step of the episode
  decltype(s.ea_off) ea_offp = EA ? s.ea_off + (int64_t)slot * (c.T + 1) * E + e : nullptr;
  decltype(s.ea_pos) ea_posp = EA ? s.ea_pos + (int64_t)slot * c.T * E + e : nullptr;
  const int T_s = __builtin_amdgcn_readfirstlane(EA ? ea.t1 : c.T);  // EA: the chunk's last step + 1
  __syncthreads();
  if constexpr (EA) {
    // (after the barrier: every wave of the block has read the slot's previous counter)
    if (valid && ea.t0 == 0) {
      s.ea_cnt[(int64_t)slot * E + e] = ea_cnt_new;
      ea_offp[0] = 0;
    }
  }
  // p_skip[r] and exp(-lambda_o[r + 1]) of the current region in registers (reloaded when a
  // region starts, long before their first use); exp(-lambda_q[r, sku]) is read from the LDS
  // table when a quantity unit opens, while the round's ring reads are in flight
  double tk = Tk[0], to_next = To[R > 1 ? 1 : 0];
  double prod = 1.0, thr = To[0];
  // (scalar loads of the descriptor, consumed before the loop: a vector load here would leave its
  // wait, vmcnt(0), inside the loop, where it also waits for every record store in flight)
  const double u_thr_o = sgpr_d(c.uni_thr_o), u_thr_m = sgpr_d(c.uni_thr_m), u_thr_q = sgpr_d(c.uni_thr_q);
  const int R_s = __builtin_amdgcn_readfirstlane(R), cap_s = __builtin_amdgcn_readfirstlane(cap);
  const int64_t rstride_s = (int64_t)__builtin_amdgcn_readfirstlane((uint32_t)rstride) |
                            ((int64_t)__builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)rstride >> 32)) << 32);
  if constexpr (UNI) thr = u_thr_o;
  // UNI settle: the same transitions with constant thresholds
  auto settle_uni = [&]() {
    const int is_q = st == PS_QTY ? 1 : 0, is_o = st == PS_ORD ? 1 : 0;
    if (is_q & (n <= cap_s ? 1 : 0)) {
      const int h = 1 + sq;  // 16-bit field of the record (field 0 = region)
      MSC_GLOBAL char* fp = NV == 1 ? recp + h * 2 : recp + (int64_t)(h >> 3) * vstride + (h & 7) * 2;
      *reinterpret_cast<MSC_GLOBAL uint16_t*>(fp) = (uint16_t)(x > 1 ? x : 1);  // max(1, Poisson(lambda_q))
    }
    const unsigned m2 = is_q ? (mask & (mask - 1u)) : mask;  // a mask unit left its bits in mask
    const int has_q = (is_o ^ 1) & (m2 != 0u ? 1 : 0);
    const int left2 = (is_o ? x : left) - ((is_o | has_q) ^ 1);  // an order completed
    const int new_order = (has_q ^ 1) & (left2 > 0 ? 1 : 0);
    const int new_region = (has_q | new_order) ^ 1;
    sq = __builtin_ctz(m2 | (1u << K));
    int wrap = 0;  // EA: the step's last region ended and another step of the episode follows
    if constexpr (EA) {
      if (new_region & (r + 1 == R_s ? 1 : 0)) {
        ea_offp[(int64_t)(tstep + 1) * E] = n;
        ea_posp[(int64_t)tstep * E] = ea_p0 + (uint32_t)rd;
        wrap = tstep + 1 < T_s ? 1 : 0;
        tstep += wrap;
      }
    }
    st = has_q ? PS_QTY : new_order ? PS_MASK : ((r + new_region < R_s) | wrap ? PS_ORD : PS_DONE);
    // three-way threshold choice as a bit select (as a ?: chain the optimizer turns it into a lookup
    // table in scratch memory, which then keeps the whole parser state in scratch)
    {
      const uint64_t bo = (uint64_t)__double_as_longlong(u_thr_o), bm = (uint64_t)__double_as_longlong(u_thr_m),
                     bq = (uint64_t)__double_as_longlong(u_thr_q);
      const uint64_t mo = (uint64_t)0 - (uint64_t)new_order, mq = (uint64_t)0 - (uint64_t)has_q;
      uint64_t b = bo ^ ((bo ^ bm) & mo);
      b = b ^ ((b ^ bq) & mq);
      thr = __longlong_as_double((long long)b);
    }
    mask = new_order ? 0u : m2;
    left = left2;
    n += new_order;
    recp += new_order ? rstride_s : 0;
    if (new_order & (n <= cap_s ? 1 : 0)) {
#pragma unroll
      for (int j = 0; j < NV; j++)
        *reinterpret_cast<MSC_GLOBAL v4u*>(recp + (int64_t)j * vstride) = v4u{j == 0 ? (unsigned)r : 0u, 0u, 0u, 0u};
    }
    r = wrap ? 0 : r + new_region;
    prod = 1.0;
    x = 0;
    mf = st == PS_MASK ? 1 : 0;
    live = st != PS_DONE ? 1 : 0;
  };
  // a unit ended: book its result, open the next unit (straight-line, predicated; only the two
  // record stores are guarded)
  auto settle = [&]() {
    const int is_q = st == PS_QTY ? 1 : 0, is_o = st == PS_ORD ? 1 : 0;
    if (is_q & (n <= cap ? 1 : 0)) {
      const int h = 1 + sq;  // 16-bit field of the record (field 0 = region)
      *reinterpret_cast<MSC_GLOBAL uint16_t*>(recp + (int64_t)(h >> 3) * vstride + (h & 7) * 2) =
          (uint16_t)(x > 1 ? x : 1);  // max(1, Poisson(lambda_q))
    }
    const unsigned m2 = is_q ? (mask & (mask - 1u)) : mask;
    const int has_q = (is_o ^ 1) & (m2 != 0u ? 1 : 0);
    const int left2 = (is_o ? x : left) - ((is_o | has_q) ^ 1);  // an order completed
    const int new_order = (has_q ^ 1) & (left2 > 0 ? 1 : 0);
    int new_region = (has_q | new_order) ^ 1 ? (r + 1 < R ? 1 : 0) : 0;
    int nsq = __builtin_ctz(m2 | (1u << K));
    nsq = nsq < K ? nsq : K - 1;
    const double q_thr = Tq[r * K + nsq];
    int wrap = 0;  // EA: the step's last region ended and another step of the episode follows
    if constexpr (EA) {
      if (((has_q | new_order) ^ 1) & (r + 1 == R ? 1 : 0)) {
        ea_offp[(int64_t)(tstep + 1) * E] = n;
        ea_posp[(int64_t)tstep * E] = ea_p0 + (uint32_t)rd;
        wrap = tstep + 1 < T_s ? 1 : 0;
        tstep += wrap;
      }
    }
    st = has_q ? PS_QTY : new_order ? PS_MASK : (new_region | wrap) ? PS_ORD : PS_DONE;
    thr = has_q ? q_thr : new_order ? tk : wrap ? To[0] : to_next;
    sq = nsq;
    mask = new_order ? 0u : m2;
    left = left2;
    n += new_order;
    recp += new_order ? rstride : 0;
    if (new_order & (n <= cap ? 1 : 0)) {
#pragma unroll
      for (int j = 0; j < NV; j++)
        *reinterpret_cast<MSC_GLOBAL v4u*>(recp + (int64_t)j * vstride) = v4u{j == 0 ? (unsigned)r : 0u, 0u, 0u, 0u};
    }
    r = wrap ? 0 : r + new_region;
    tk = Tk[r];
    to_next = To[r + 1 < R ? r + 1 : r];
    prod = 1.0;
    x = 0;
    mf = st == PS_MASK ? 1 : 0;
    live = st != PS_DONE ? 1 : 0;
  };
  PROF_DECL(p_all);
  PROF_DECL(n_round);
  PROF_DECL(n_chunk);
  PROF_DECL(p_bar);
  PROF_T(t_start);
  int ptgt = UCAP, rd_start = 0;  // the generators' fill target and the chunk's start position
  for (int ci = 0;; ci++) {
#pragma unroll 1
    for (int hs = 0; hs < UHS; hs++) {
      // issue this round's ring reads first, then book the unit that ended last round (its
      // bookkeeping has no LDS dependence) while they are in flight
      const double* rp = myring + (rd & (UCAP - 1)) * BS;
      double u[UD];
#pragma unroll
      for (int i = 0; i < UD; i++) u[i] = rp[i * BS];
      if constexpr (UNI) {
        if (pend) settle_uni();
      } else {
        if (pend) settle();
      }
      // Poisson unit: p_i = p_{i-1} * U_i in draw order; U_i < 1 makes the products non-increasing,
      // so "p_i > exp(-lambda)" holds for a leading run only and its length is a plain count.
      // Mask unit: the K Bernoulli draws, bit i = SKU drawn <=> U_i < p <=> !(U_i > p_skip).
      double p = prod;
      int ncont = 0;
      unsigned bits = 0;
#pragma unroll
      for (int i = 0; i < UD; i++) {
        p = p * u[i];
        ncont += p > thr ? 1 : 0;
        if (i < K) bits |= u[i] > thr ? 0u : (1u << i);
      }
      const int go = ncont >= UD ? 1 : 0;  // Poisson unit still running after UD draws
      const int cons = mf ? K : (go ? UD : ncont + 1);
      mask = mf ? bits : mask;
      x += ncont;  // (a mask unit's x is unused and cleared by its settle)
      prod = p;
      rd += live ? cons : 0;
      pend = live & (mf | (go ^ 1));
      PROF_ADD(n_round, 1);
    }
    // a lane with a booked-but-unsettled unit is still live: it settles in the next round
    const bool any = __ballot(live) != 0;
    rdv[((ci + 1) & 1) * BS + lane] = rd;
    if (lane == 0) more[ci & 1] = any ? 1 : 0;
    PROF_T(tb);
    __syncthreads();
    PROF_ADD(p_bar, PROF_NOW() - tb);
    PROF_ADD(n_chunk, 1);
    if (!any) break;
    // the generators' refill decision, restated: their top-up barrier (if any) is joined here
    ptgt = unit_quota(ptgt, rd_start);
    const int need = rd + UHS * UD;
    if (__ballot(valid && ptgt < need) != 0) {
      ptgt = ptgt > need ? ptgt : need;
      __syncthreads();
    }
    rd_start = rd;
  }
  PROF_ADD(p_all, PROF_NOW() - t_start);
  PROF_FLUSH(0, p_all);
  PROF_FLUSH(2, p_bar);
  PROF_FLUSH(4, n_round);
  PROF_FLUSH(5, n_chunk);
  PROF_FLUSH(6, 1ull);
  if (!valid) return;
  if constexpr (EA) {
    if (n > cap) atomicOr(s.err, ERR_ORDER_OVERFLOW);
    return;
  }
  pcg_advance(r0, (uint64_t)rd);
  store_rng(s, 0, e, E, r0);
  if (n > cap) {
    atomicOr(s.err, ERR_ORDER_OVERFLOW);
    n = cap;
  }
  s.n_orders[e] = n;
}

// The demand stream of env e as of `t_done` steps into the episode held by EA slot `slot`
// (read_state / save_state / leaving EA mode): the 'demand_sampler' child of the episode's root
// (s.root, written by the reset that started it) advanced by the draws of those steps.
#ifndef MSC_EK_WIDE  // (defined once: env_kernels.hip proper)
__global__ void ea_materialize_kernel(const DevEnv* __restrict__ dp, int32_t slot, int32_t t_done) {
  const EnvConst& c = dp->c;
  const EnvState& s = dp->s;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= c.E || t_done < 1) return;
  Pcg64 r;
  pcg_seed_child(r, s.root[e], 2);
  pcg_advance(r, s.ea_pos[((int64_t)slot * c.T + (t_done - 1)) * c.E + e]);
  store_rng(s, 0, e, c.E, r);
}
#endif

// ------------------------------------------------------------------------------------------
// Production step: InventoryEnvironment.step (multi_env.py:253-366) as three launches.
//
//   step_a_kernel  (block = 64 envs x min(W, 16) waves; wave = warehouse, lane = env): per-env RNG work
//                  (stochastic lead deviations, empirical window), then orders / lead times /
//                  pending ring / arrivals / inbound cost for the lane's (w, s) pairs;
//   step_b_kernel  (group of GW >= W lanes = one env, lane = warehouse): the greedy allocation.
//                  Each lane keeps its warehouse's inventory / shipped-to-region / shipped-total /
//                  shipped-home in registers and computes its own ranking cost; the group finds the
//                  cheapest candidate with a butterfly (lowest index on ties = the stable argsort),
//                  and the region epilogue (lost sales, home features) is per-warehouse lane work;
//   step_c_kernel  (wave = warehouse, lane = env): inventory / history / forecast, rewards (team
//                  sum across the block's waves), observations, in-kernel reset on truncation.
// Splitting keeps each kernel's register footprint small (the fused version spilled) and gives
// every phase its own natural thread mapping; the phases exchange ~0.7 KB per env through HBM
// scratch (EnvState::sc_*), and [i][E] state stays coalesced for the wave = warehouse phases.
// ------------------------------------------------------------------------------------------
// ---- phase A ------------------------------------------------------------------------------
#ifndef MSC_SA_RING_REG
#define MSC_SA_RING_REG 4  // step_a: pending rings of up to this many slots are read into registers
#endif
constexpr int SA_RING_REG = MSC_SA_RING_REG;
// waves of a step_a / step_c block: one per warehouse up to 16 warehouses (LOOP = false: the
// kernel has no warehouse loop); above 16 warehouses (or above 8 SKUs, whose K-wide register
// arrays need the larger per-lane budget of a WB = 4-wave block) each wave takes warehouses
// w, w + WB, ... (LOOP = true)
constexpr int STEP_WAVES = 16;
template <int WB, bool LOOP, typename F>
__device__ __forceinline__ void each_warehouse(int wave, int W, F&& f) {
  if constexpr (LOOP) {
    for (int w = wave; w < W; w += WB) f(w);
  } else {
    if (wave < W) f(wave);
  }
}
// waves per block of the LOOP instantiations: 4 above 8 SKUs, else 16
__host__ __device__ constexpr int step_loop_waves(int K) { return K > 8 ? 4 : STEP_WAVES; }
// REG: the register-ring instantiation (the fixed-lead path holds the K rings in registers: ~2x the
// VGPRs, which costs co-residency beside the demand kernel at 32,768 envs; used with obs_ring_reg)
template <int K, bool DBG, bool REG = false, int WB = STEP_WAVES, bool LOOP = false>
__global__ __launch_bounds__(BS * WB) void step_a_kernel(const DevEnv* __restrict__ dp, StepIO io) {
  const EnvConst& c = dp->c;
  const EnvState& s = dp->s;
  __shared__ int32_t Lt[BS];
  const int W = c.W, WK = W * K, RING = c.RING;
  const int64_t E = c.E;
  const int wave = threadIdx.x / BS, lane = threadIdx.x % BS;
  const int64_t e = (int64_t)blockIdx.x * BS + lane;
  if (c.chain_prio) __builtin_amdgcn_s_setprio(3);  // the step chain is the caller's critical path
  const bool ev = e < E;
  const msc_step_info info = io.info;
  constexpr bool dbg = DBG;
  const bool stoch = c.lead_type == MSC_LEAD_STOCHASTIC;
  if (wave == 0 && ev) {  // per-env sequential RNG work
    const int t = s.t[e];
    Lt[lane] = t;
    if (stoch) {  // lead_time_sampler.sample(): all W*K deviations every step (multi_env.py:866)
      // each actual lead time max(1, elt + deviation) goes straight to the ring slot of this step's
      // order (the arrival pass of the warehouse waves skips that slot)
      const int slot = t % RING;
      auto put = [&](int i, int64_t dev) {
        const int l = c.elt[i] + (int)dev;
        s.ring_l[((int64_t)i * RING + slot) * E + e] = (uint8_t)(l > 1 ? l : 1);
      };
      Pcg64 rl = load_rng(s, 1, e, E);
      if (c.dev_per_sku) {  // SKU-major column_stack order (lead_time_sampler.py:181-185)
        for (int sk = 0; sk < K; sk++)
          for (int w = 0; w < W; w++) put(w * K + sk, bounded_int(rl, -c.maxdev[sk], (int64_t)c.maxdev[sk] + 1));
      } else {
        for (int i = 0; i < WK; i++) put(i, bounded_int(rl, -c.maxdev[0], (int64_t)c.maxdev[0] + 1));
      }
      store_rng(s, 1, e, E, rl);
    }
    if (c.demand_type == MSC_DEMAND_EMPIRICAL && s.emp_start[e] < 0) {  // demand_sampler.py:227-241
      Pcg64 rg = load_rng(s, 0, e, E);
      s.emp_start[e] = (int)bounded_int(rg, 0, (int64_t)(c.tr_rows - c.T) + 1);
      store_rng(s, 0, e, E, rg);
    }
  }
  __syncthreads();
  if (!ev) return;
  const int t = Lt[lane];
  const int slot = t % RING;
  // one warehouse per wave (LOOP: each wave takes w, w + WB, ...)
  auto warehouse = [&](const int w) {
    double inbF = 0.0, inbV = 0.0;
    if constexpr (REG && K <= 5) {
    if (RING <= SA_RING_REG && !stoch) {
      // (fixed lead times; <= 5 SKUs, whose rings fit the register budget) Every load of the K SKUs first, then the arithmetic, then the stores: vector loads and stores
      // retire through one counter (vmcnt), so a load issued after a store waits for it (the loop
      // below stores the new order before it reads the ring for arrivals, K times)
      float a[K];
      int inc_old[K], inv[K], rv[K][SA_RING_REG];
#pragma unroll
      for (int sk = 0; sk < K; sk++) {
        const int i = w * K + sk;
        a[sk] = io.actions[(e * W + w) * K + sk];
        inc_old[sk] = s.inc[i * E + e];
        inv[sk] = s.inv[i * E + e];
        const int32_t* rq = s.ring_q + (int64_t)i * RING * E + e;
#pragma unroll
        for (int q = 0; q < SA_RING_REG; q++) rv[sk][q] = q < RING ? rq[q * E] : 0;
      }
#pragma unroll
      for (int sk = 0; sk < K; sk++) {
        const int i = w * K + sk;
        int pend = 0;
#pragma unroll
        for (int q = 0; q < SA_RING_REG; q++) pend += rv[sk][q];
        const double prm = c.act_param[sk];  // _rescale_actions_to_quantities (multi_env.py:795-848)
        double q;
        if (c.action_type == MSC_ACTION_DIRECT) {
          q = rint((double)((a[sk] + 1.0f) / 2.0f) * prm);
          q = q < 0.0 ? 0.0 : (q > prm ? prm : q);
        } else if (c.action_type == MSC_ACTION_DEMAND_CENTERED) {
          q = rint(prm * (double)a[sk]) + (double)inc_old[sk];
          q = q < 0.0 ? 0.0 : q;
        } else {
          const double target = (double)((a[sk] + 1.0f) / 2.0f) * prm;
          q = rint((target - (double)(float)inc_old[sk]) - (double)(float)pend);
          q = q < 0.0 ? 0.0 : q;
        }
        const int qi = (int)q;
        const int elt = c.elt[i];
        int32_t* rq = s.ring_q + (int64_t)i * RING * E + e;
        if (dbg && info.inventory_before) info.inventory_before[e * WK + i] = inv[sk];
        // _apply_arrivals: orders whose actual lead time equals their age arrive (actual arrival == t)
        int iv = inv[sk];
#pragma unroll
        for (int jr = 0; jr < SA_RING_REG; jr++) {
          int age = (t - jr) % RING;
          if (age < 0) age += RING;
          const bool arrive = jr < RING && jr != slot && rv[sk][jr] != 0 && elt == age;
          iv += arrive ? rv[sk][jr] : 0;
          if (arrive) rq[jr * E] = 0;
        }
        rq[slot * E] = qi;  // _apply_orders: the slot of order time t
        s.inv[i * E + e] = iv;
        s.inc[i * E + e] = 0;
        if (qi > 0) inbF += c.inF[i];
        inbV += ((double)qi * c.skw[sk]) * c.inV[i];
        if (dbg) {
          if (info.pending_total) info.pending_total[e * WK + i] = pend;
          if (info.order_quantities) info.order_quantities[e * WK + i] = qi;
        }
      }
      s.sc_inb[w * E + e] = inbF + inbV;
      return;
    }
    }
    if (RING <= SA_RING_REG && !stoch) {
      // (the low-register form: one SKU at a time, each SKU's loads issued together before its stores)
#pragma unroll
      for (int sk = 0; sk < K; sk++) {
        const int i = w * K + sk;
        int32_t* rq = s.ring_q + (int64_t)i * RING * E + e;
        const float a = io.actions[(e * W + w) * K + sk];
        const int inc_old = s.inc[i * E + e];
        int iv = s.inv[i * E + e];
        int rv[SA_RING_REG];
#pragma unroll
        for (int q = 0; q < SA_RING_REG; q++) rv[q] = q < RING ? rq[q * E] : 0;
        int pend = 0;
#pragma unroll
        for (int q = 0; q < SA_RING_REG; q++) pend += rv[q];
        const double prm = c.act_param[sk];  // _rescale_actions_to_quantities (multi_env.py:795-848)
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
        if (dbg && info.inventory_before) info.inventory_before[e * WK + i] = iv;
#pragma unroll
        for (int jr = 0; jr < SA_RING_REG; jr++) {  // _apply_arrivals (actual arrival == t)
          int age = (t - jr) % RING;
          if (age < 0) age += RING;
          const bool arrive = jr < RING && jr != slot && rv[jr] != 0 && elt == age;
          iv += arrive ? rv[jr] : 0;
          if (arrive) rq[jr * E] = 0;
        }
        rq[slot * E] = qi;  // _apply_orders: the slot of order time t
        s.inv[i * E + e] = iv;
        s.inc[i * E + e] = 0;
        if (qi > 0) inbF += c.inF[i];
        inbV += ((double)qi * c.skw[sk]) * c.inV[i];
        if (dbg) {
          if (info.pending_total) info.pending_total[e * WK + i] = pend;
          if (info.order_quantities) info.order_quantities[e * WK + i] = qi;
        }
      }
      s.sc_inb[w * E + e] = inbF + inbV;
      return;
    }
#pragma unroll
    for (int sk = 0; sk < K; sk++) {
      const int i = w * K + sk;
      const float a = io.actions[(e * W + w) * K + sk];
      const int inc_old = s.inc[i * E + e];
      int32_t* rq = s.ring_q + (int64_t)i * RING * E + e;
      int pend = 0;
      for (int jr = 0; jr < RING; jr++) pend += rq[jr * E];
      const double prm = c.act_param[sk];  // _rescale_actions_to_quantities (multi_env.py:795-848)
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
      rq[slot * E] = qi;  // _apply_orders: the slot of order time t (its actual lead time: wave 0)
      int inv = s.inv[i * E + e];  // _apply_arrivals: actual arrival == t
      if (dbg && info.inventory_before) info.inventory_before[e * WK + i] = inv;
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
      s.inv[i * E + e] = inv;
      s.inc[i * E + e] = 0;
      if (qi > 0) inbF += c.inF[i];
      inbV += ((double)qi * c.skw[sk]) * c.inV[i];
      if (dbg) {
        if (info.pending_total) info.pending_total[e * WK + i] = pend;
        if (info.order_quantities) info.order_quantities[e * WK + i] = qi;
      }
    }
    s.sc_inb[w * E + e] = inbF + inbV;
  };
  each_warehouse<WB, LOOP>(wave, W, warehouse);
}

// ---- phase B ------------------------------------------------------------------------------
// (dpp_x: kcommon.hpp)
template <int GW, typename T, typename F>
__device__ __forceinline__ T group_reduce(T v, F op) {
  v = op(v, dpp_x<0>(v));
  if constexpr (GW >= 4) v = op(v, dpp_x<1>(v));
  if constexpr (GW >= 8) v = op(v, dpp_x<2>(v));
  if constexpr (GW >= 16) v = op(v, dpp_x<3>(v));
  if constexpr (GW >= 32) v = op(v, dpp_x<4>(v));
  return v;
}

// Order records reach the allocator through a wave-private, double-buffered LDS window filled by
// LDS-DMA (global_load_lds_dwordx4: no VGPR staging): while the wave allocates the SB_CH orders
// of one window, the next window is in flight, so the order loop has no global-memory wait (a
// register FIFO of prefetched records waited on its newest load at every shift).
#ifndef MSC_SB_REC
#define MSC_SB_REC 128
#endif
constexpr int SB_REC = MSC_SB_REC;  // records per window (16 B each), two windows per wave
__host__ __device__ constexpr int step_b_chunk(int GW, int NV) { return SB_REC / ((64 / GW) * NV); }
// block tables: outbound costs [2][R][W] f64 + closest warehouse [R], staged in LDS when small
__host__ __device__ constexpr size_t step_b_tab_bytes(int R, int W) {
  return (size_t)2 * R * W * sizeof(double) + (size_t)R * sizeof(int32_t);
}
// waves per block: 8 for 16- and 32-lane groups with the tables in LDS (C5: one block per CU holds
// the 66.5-KB table once for 8 waves' record windows; two 4-wave blocks per CU would need it twice),
// else 4
__host__ __device__ constexpr int step_b_waves(int GW, bool tab) { return GW >= 16 && tab ? 8 : 4; }
__host__ __device__ constexpr size_t step_b_lds_bytes(int R, int W, bool tab, int waves) {
  return (size_t)waves * 2 * SB_REC * 16 + (tab ? step_b_tab_bytes(R, W) : 0);
}

// (group_np_sum: kcommon.hpp)

// step_b waves per SIMD the register budget is sized for: 5 (<= 96 VGPRs) leaves room on each SIMD
// for a demand-kernel wave of the next step next to the four step_b waves of this one
#ifndef MSC_SC_PRIO
#define MSC_SC_PRIO 0  // s_setprio of the step_c waves
#endif
#ifndef MSC_SB_PRIO
#define MSC_SB_PRIO 3  // s_setprio of the step_b waves (above the next step's demand waves)
#endif
#ifndef MSC_SB_WPE
#define MSC_SB_WPE 5
#endif
// 16- and 32-lane groups (9-32 warehouses): 4 envs per wave or fewer, so 8,192 envs (C5) are 2,048
// waves, 2 per SIMD: a 96-VGPR budget only spilled the order loop to scratch (whose reloads wait on
// vmcnt, i.e. also for the record window's LDS-DMA in flight); 128 VGPRs hold it
#ifndef MSC_SB_WPE16
#define MSC_SB_WPE16 4
#endif
#ifndef MSC_SB_BPERM
#define MSC_SB_BPERM 0  // 1: winner's fill broadcast by ds_bpermute (A/B, lost at C5: 0.908 vs 0.903 ms/step)
#endif

// This step's order count of env e (what step_b_kernel iterates over).
__device__ __forceinline__ int step_order_count(const EnvConst& c, const EnvState& s, const StepIO& io, int64_t e) {
  return order_src<1>(c, s, io, e).n;
}

// Allocation visiting order: envs by descending order count of this step (counting sort over
// SORT_BUCKETS buckets of count >> sort_shift; the order within a bucket is arbitrary, as is any
// permutation: every env's allocation is independent of where it runs). One block; ~10 us at
// 8,192 envs. Busiest envs first also starts the longest waves first.
#ifndef MSC_EK_WIDE  // (defined once: env_kernels.hip proper)
__global__ __launch_bounds__(1024) void alloc_sort_kernel(const DevEnv* __restrict__ dp, StepIO io) {
  const EnvConst& c = dp->c;
  const EnvState& s = dp->s;
  const int64_t E = c.E;
  __shared__ int hist[SORT_BUCKETS];
  __shared__ int wsum[1024 / 64];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  auto key = [&](int64_t e) {
    const int b = step_order_count(c, s, io, e) >> c.sort_shift;
    return SORT_BUCKETS - 1 - (b < SORT_BUCKETS ? b : SORT_BUCKETS - 1);
  };
  for (int i = tid; i < SORT_BUCKETS; i += blockDim.x) hist[i] = 0;
  __syncthreads();
  for (int64_t e = tid; e < E; e += blockDim.x) atomicAdd(&hist[key(e)], 1);
  __syncthreads();
  // exclusive scan of the histogram: wave scans, then the wave totals
  static_assert(SORT_BUCKETS == 1024, "one bucket per thread");
  const int h = hist[tid];
  int v = h;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(v, o);
    v += lane >= o ? u : 0;
  }
  if (lane == 63) wsum[wv] = v;
  __syncthreads();
  int base = 0;
  for (int i = 0; i < wv; i++) base += wsum[i];
  __syncthreads();
  hist[tid] = base + v - h;
  __syncthreads();
  for (int64_t e = tid; e < E; e += blockDim.x) s.perm[atomicAdd(&hist[key(e)], 1)] = (int32_t)e;
}
#endif

// Phase C fused into the group allocator (c.fuse_c; step_c_kernel's work, multi_env.py:307-327,
// 747-793, reward_calculator.py:96-190): lane w of env e's group is agent w, its SKUs' inventory in
// registers after the allocation; the history, forecast and observation of agent w, the reward (team
// scope: the group's sum in agent order), and the in-kernel reset at truncation (the group's lane 0).
// This lane's home-region stores of the allocation (s.inc, s.sc_shh) are read back after a wait.
constexpr int SB_FC_RING = 4;  // pending-ring slots held in registers (lead times <= 3)
template <int K, int GW>
__device__ __forceinline__ void step_b_phase_c(const EnvConst& c, const EnvState& s, const StepIO& io, int64_t e, int w,
                                               bool ev, bool wl, int gbase, bool home_done, const int (&inv)[K],
                                               double pen, double out) {
  const int64_t E = c.E;
  const int W = c.W, WK = W * K, RING = c.RING;
  const bool on = ev && wl;
  const int t_now = ev ? s.t[e] : 0;
  const int hslot = t_now % MSC_HISTORY, n_hist = t_now + 1 < MSC_HISTORY ? t_now + 1 : MSC_HISTORY;
  const int tm = t_now % RING;
  const bool trunc = ev && t_now + 1 >= c.T;
  __builtin_amdgcn_s_waitcnt(0);  // (the allocation's stores of this lane have landed)
  int a_inv[K], a_dh[K], a_sh[K], a_sa[K], a_pend[K], a_elt[K], hv[K][MSC_HISTORY], rv[K][SB_FC_RING];
  float a_rm[K], a_fc[K], fo[K];
  double hold = 0.0;
  if (on) {
    // every load first (one vmcnt for loads and stores)
#pragma unroll
    for (int sk = 0; sk < K; sk++) {
      const int i = w * K + sk;
      const int64_t g = (int64_t)i * E + e;
      a_inv[sk] = inv[sk];
      a_sa[sk] = s.inv[g] - inv[sk];  // shipped this step (the inventory drop); minus home below
      a_dh[sk] = s.inc[g];            // this step's incoming home demand (0 unless the home region)
      a_sh[sk] = home_done ? s.sc_shh[g] : 0;
      fo[sk] = s.fc[g];
      a_elt[sk] = c.elt[i];
#pragma unroll
      for (int a = 1; a < MSC_HISTORY; a++) {
        const int q = (t_now - a) % MSC_HISTORY;
        hv[sk][a] = a < n_hist ? s.hist[((int64_t)(q < 0 ? q + MSC_HISTORY : q) * WK + i) * E + e] : 0;
      }
#pragma unroll
      for (int q = 0; q < SB_FC_RING; q++) rv[sk][q] = q < RING ? s.ring_q[((int64_t)i * RING + q) * E + e] : 0;
    }
#pragma unroll
    for (int sk = 0; sk < K; sk++) {
      const int i = w * K + sk;
      const int64_t g = (int64_t)i * E + e;
      a_sa[sk] -= a_sh[sk];
      hv[sk][0] = a_dh[sk];
      s.hist[((int64_t)hslot * WK + i) * E + e] = a_dh[sk];
      a_fc[sk] = 0.3f * (float)a_dh[sk] + 0.7f * fo[sk];  // EMA forecast (f32)
      s.fc[g] = a_fc[sk];
      s.inv[g] = inv[sk];
      int hs = 0, pend = 0;
#pragma unroll
      for (int a = 0; a < MSC_HISTORY; a++) hs += a < n_hist ? hv[sk][a] : 0;
      a_rm[sk] = n_hist > 0 ? (float)hs / (float)n_hist : 0.0f;
#pragma unroll
      for (int q = 0; q < SB_FC_RING; q++) pend += rv[sk][q];
      a_pend[sk] = pend;
      hold += c.hold_per_sku ? (double)inv[sk] * c.hold[sk] : ((double)inv[sk] * c.skw[sk]) * c.hold_scalar;
    }
  }
  const double inb = on ? s.sc_inb[w * E + e] : 0.0;
  const double rw = -((((hold + pen) + out) + inb) * c.scale);
  if (on && io.has_info && io.info.costs) {
    io.info.costs[(e * 4 + 0) * W + w] = hold;
    io.info.costs[(e * 4 + 1) * W + w] = pen;
    io.info.costs[(e * 4 + 2) * W + w] = out;
    io.info.costs[(e * 4 + 3) * W + w] = inb;
  }
  double v = rw;
  if (c.scope == MSC_SCOPE_TEAM) {  // (uniform) the group's sum in agent order, every lane active
    v = 0.0;
    for (int j = 0; j < W; j++) v += __shfl(rw, gbase + j);
  }
  if (on) {
    io.rew[e * W + w] = (float)v;
    if (io.rew64) io.rew64[e * W + w] = v;
    auto pipe_at = [&](int l, int sk) -> int {  // bucket max(1, elt - age) - 1 of ring slot q
      int v2 = 0;
#pragma unroll
      for (int q = 0; q < SB_FC_RING; q++) {
        const int age = tm - q >= 0 ? tm - q : tm - q + RING;
        const int b = a_elt[sk] - age > 1 ? a_elt[sk] - age - 1 : 0;
        v2 += (q < RING && b == l) ? rv[sk][q] : 0;
      }
      return v2;
    };
    auto hist_at = [&](int a, int sk) -> int {
      int v2 = 0;
#pragma unroll
      for (int q = 0; q < MSC_HISTORY; q++) v2 = q == a ? hv[sk][q] : v2;
      return v2;
    };
    float* dst = trunc ? io.final_obs : io.obs;
    if (dst) obs_emit<K>(c, w, n_hist, a_inv, a_dh, a_sh, a_sa, a_pend, a_elt, a_rm, a_fc, pipe_at, hist_at, dst + e * W * c.L);
  }
  // truncation: the group's lane 0 resets the env, then every agent's reset observation
  if (__ballot(trunc) != 0ull) {
    if (trunc && w == 0) reset_env<K>(c, s, e, 0, nullptr);
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (trunc && wl) build_obs_agent<K>(c, s, e, w, 0, 0, nullptr, nullptr, 0, io.obs + e * W * c.L);
  }
  if (ev && w == 0) {
    io.trunc[e] = trunc ? 1 : 0;
    if (!trunc) s.t[e] = t_now + 1;
  }
}

// (above 8 SKUs the K-wide register arrays of a lane need the larger budget of 2 waves per SIMD)
template <int K, int GW, bool DBG, bool TAB>
__global__ __launch_bounds__(64 * step_b_waves(GW, TAB)) __attribute__((amdgpu_waves_per_eu(K > 8 ? 2 : GW >= 16 ? MSC_SB_WPE16 : MSC_SB_WPE))) void step_b_kernel(const DevEnv* __restrict__ dp, StepIO io) {
  const EnvConst& c = dp->c;
  const EnvState& s = dp->s;
  const int W = c.W, WK = W * K, R = c.R;
  const int64_t E = c.E;
  const int w = threadIdx.x % GW;
  // visiting slot of this lane group: wave k of block b runs slot-wave k * gridDim.x + b, so with the
  // envs sorted by order count a block (one CU at C5) holds waves from the whole range of loads
  // instead of 8 consecutive ones -- the busiest envs' waves no longer share their CU's SIMDs only
  // with each other -- while a wave still holds consecutive (similar) envs
  const int64_t eg = ((int64_t)(threadIdx.x >> 6) * gridDim.x + blockIdx.x) * (64 / GW) + (threadIdx.x & 63) / GW;
  const int64_t e = (c.alloc_sort && eg < E) ? (int64_t)s.perm[eg] : eg;
  const bool ev = e < E, wl = w < W;
  const msc_step_info info = io.info;
  constexpr bool dbg = DBG;
  constexpr int NVR = Rec<K>::NV;
  constexpr int EPW = 64 / GW;                // envs per wave
  constexpr int CH = SB_REC / (EPW * NVR);    // orders per window
  constexpr int LPL = SB_REC / 64;            // LDS-DMA loads per lane per window
  static_assert(CH >= 1 && SB_REC % 64 == 0, "window layout");
  extern __shared__ __attribute__((aligned(16))) uint4 sb_lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, gbase = lane & ~(GW - 1);
  if (MSC_SB_PRIO > 0) __builtin_amdgcn_s_setprio(MSC_SB_PRIO);
  uint4* win = sb_lds + wave * 2 * SB_REC;  // this wave's two windows [2][CH][NVR][EPW]
  const MSC_GLOBAL int32_t* closest = gp(c.closest);
  double* lof = TAB ? reinterpret_cast<double*>(sb_lds + step_b_waves(GW, TAB) * 2 * SB_REC) : nullptr;
  double* lov = TAB ? lof + R * W : nullptr;
  int32_t* lcl = TAB ? reinterpret_cast<int32_t*>(lov + R * W) : nullptr;
  if constexpr (TAB) {
    for (int i = threadIdx.x; i < R * W; i += blockDim.x) {
      lof[i] = c.ofT[i];
      lov[i] = c.ovT[i];
    }
    for (int i = threadIdx.x; i < R; i += blockDim.x) lcl[i] = c.closest[i];
    __syncthreads();
  }
  auto cost_of = [&](int r) { return TAB ? lof[r * W + w] : gp(c.ofT)[r * W + w]; };
  auto cost_ov = [&](int r) { return TAB ? lov[r * W + w] : gp(c.ovT)[r * W + w]; };
  auto closest_of = [&](int r) { return TAB ? lcl[r] : closest[r]; };

  int inv[K], qsr[K];
  {  // unconditional loads at clamped indices (a lane-conditional load is a branch with its own wait)
    const int64_t ec = ev ? e : 0;
    const int wc = wl ? w : 0;
#pragma unroll
    for (int sk = 0; sk < K; sk++) {
      const int v = s.inv[(int64_t)(wc * K + sk) * E + ec];
      inv[sk] = (ev && wl) ? v : 0;
      qsr[sk] = 0;
    }
  }
  double pen = 0.0, out = 0.0, cof = 0.0, cov = 0.0;
  // record (n, v) of this lane's env at base + n * nstep + v * vstep (uint4 units)
  const OrderSrc osrc = order_src<NVR>(c, s, io, ev ? e : 0);
  const int n_orders = ev ? osrc.n : 0;
  const int64_t base = ev ? osrc.base : 0, nstep = osrc.nstep, vstep = osrc.vstep;
  const MSC_GLOBAL uint4* src = gp(osrc.src);
  if (dbg && ev && w == 0 && info.n_orders) info.n_orders[e] = n_orders;
  // loader role: lane l fetches records of env l % EPW of this wave (whose group leader is lane
  // (l % EPW) * GW); window slot q = j * 64 + l holds (order q / (EPW NVR), v, env q % EPW)
  const int ljj = lane % EPW;
  const int ln = __shfl(n_orders, ljj * GW);
  const int64_t lbase = __shfl(base, ljj * GW);
  int wmax = n_orders;  // orders of the wave's busiest env
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const int v = __shfl_xor(wmax, o);
    wmax = v > wmax ? v : wmax;
  }
  // (uniform after the butterfly; as a scalar, the order loop's exit and window tests are scalar
  // compares instead of lane masks merged at every order)
  wmax = __builtin_amdgcn_readfirstlane(wmax);
  // this warehouse's home region (argmin over regions of its distance row, multi_env.py:144)
  int myhome = wl ? c.home_of[w] : -1;
  // the loaded values the order loop reads, settled before the first window's LDS-DMA: the
  // compiler's wait for a load first used inside the loop is a vmcnt(0) there, which would also
  // wait for the record windows in flight
  myhome = vsettle(myhome);
#pragma unroll
  for (int sk = 0; sk < K; sk++) inv[sk] = vsettle(inv[sk]);
  auto issue = [&](int chunk) {  // LDS-DMA of window `chunk` into buffer chunk % 2
    uint4* dst = win + (chunk & 1) * SB_REC;
#pragma unroll
    for (int j = 0; j < LPL; j++) {
      const int ov = (j * 64 + lane) / EPW;
      const int n = chunk * CH + ov / NVR, v = ov % NVR;
      // (inline asm: with the builtin the compiler drains every LDS-DMA in flight before any LDS
      // read, i.e. at each order; the explicit counted waits below order the windows instead)
      const uint32_t lds = __builtin_amdgcn_readfirstlane(
          (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)(dst + j * 64));
      const MSC_GLOBAL uint4* g = src + lbase + n * nstep + v * vstep;
      if (n < ln) {
        uint32_t keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(g), "s"(lds)
                     : "memory");
      }
    }
  };
  issue(0);
  if (wmax > CH) {
    issue(1);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPL) : "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  // per-SKU constants and flags in registers (read once: the loop below stores to global memory,
  // so the compiler could not keep re-reading them through `c` out of the loop)
  const int maxwh = c.max_wh, lost_type = c.lost_type, pps = c.pen_per_sku;
  const double alpha = sgpr_d(c.alpha);
  double skw[K], penk[K];  // wave-uniform: moved to SGPRs (the loads themselves are vector loads)
#pragma unroll
  for (int sk = 0; sk < K; sk++) {
    skw[sk] = sgpr_d(c.skw[sk]);
    penk[sk] = sgpr_d(pps ? c.pen[sk] : c.pen_scalar);
  }
  int cur = -1, lost_cnt = 0;
  int home_done = 0;  // (an int, not a bool: a lane-varying bool lives in a lane mask that every
                     // exit of the order loop's branches merges again)
  int u[K], dsum[K];
#pragma unroll
  for (int sk = 0; sk < K; sk++) u[sk] = dsum[sk] = 0;

  // region epilogue: lost sales (lost_sales_handler.py) into the penalty cost, home-region
  // features, per-region infos; every lane handles its own warehouse
  auto finalize = [&](int r) {
    if (lost_cnt > 0) {
      double upen = 0.0;
#pragma unroll
      for (int sk = 0; sk < K; sk++) upen += pps ? (double)u[sk] * penk[sk] : ((double)u[sk] * skw[sk]) * penk[sk];
      double wt = 0.0;  // this warehouse's share of the region's lost sales
      if (lost_type == MSC_LOST_CLOSEST) {
        wt = (wl && w == closest_of(r)) ? 1.0 : 0.0;
      } else if (lost_type == MSC_LOST_SHIPMENT) {
        int acc = 0;
#pragma unroll
        for (int sk = 0; sk < K; sk++) acc += qsr[sk];
        acc = wl ? acc : 0;
        // integer-valued shares: the integer group sum is the f64 sum exactly
        const int tot = group_reduce<GW>(acc, [](int a, int b) { return a + b; });
        if (tot > 0) wt = acc > 0 ? (double)acc / (double)tot : 0.0;
        else wt = (wl && w == closest_of(r)) ? 1.0 : 0.0;
      } else {  // cost: softmax(-(of * lost_orders + ov * lost_weight) / alpha), numpy sum order
        double lw = 0.0;
#pragma unroll
        for (int sk = 0; sk < K; sk++) lw += (double)u[sk] * skw[sk];
        const double lg = wl ? -(cof * (double)lost_cnt + cov * lw) / alpha : -INFINITY;
        const double mx = group_reduce<GW>(lg, [](double a, double b) { return b > a ? b : a; });
        const double ex = wl ? exp(lg - mx) : 0.0;
        wt = wl ? ex / group_np_sum<GW>(ex, W) : 0.0;
      }
      // (a closest-warehouse share is 1.0 and 1.0 * x == x: one update form serves every type)
      // (unconditional: a zero share adds a zero product, which leaves pen (>= +0.0) unchanged)
      pen += wt * upen;
      if (dbg && info.lost_sales && wt != 0.0)
#pragma unroll
        for (int sk = 0; sk < K; sk++) info.lost_sales[e * WK + w * K + sk] += wt * (double)u[sk];
    }
    // home-region features: incoming demand and units shipped home (multi_env.py:767-773)
    if (r == myhome) {
#pragma unroll
      for (int sk = 0; sk < K; sk++) {
        s.inc[(int64_t)(w * K + sk) * E + e] = dsum[sk];
        s.sc_shh[(int64_t)(w * K + sk) * E + e] = qsr[sk];
      }
      home_done = 1;
    }
    if (dbg && w == 0) {
#pragma unroll
      for (int sk = 0; sk < K; sk++) {
        if (info.demand_per_region) info.demand_per_region[(e * R + r) * K + sk] = dsum[sk];
        if (info.unfulfilled_demands) info.unfulfilled_demands[(e * R + r) * K + sk] = u[sk];
      }
      if (info.lost_order_counts) info.lost_order_counts[e * R + r] = lost_cnt;
    }
#pragma unroll
    for (int sk = 0; sk < K; sk++) qsr[sk] = 0;
  };

  constexpr int NP = (K + 1) / 2;  // 32-bit words of a packed (16-bit per SKU) fill vector
  const int myjj = lane / GW;      // this group's env slot in the window
  PROF_DECL(q_all);
  PROF_DECL(q_fin);
  PROF_DECL(q_alloc);
  PROF_DECL(q_iter);
  PROF_DECL(q_nfin);
  PROF_T(q_t0);
  int wdue = CH;  // (wave-uniform) the next order index that opens a window
  for (int oi = 0; oi <= wmax; oi++) {
    if (oi == wdue) {  // wave-uniform: window oi / CH is due, start the one after
      wdue += CH;
      if (oi + CH <= wmax) {
        issue(oi / CH + 1);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPL) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    // (structured ifs, not `continue`: every exit of the body is a latch whose lane masks the loop
    // merges at each order)
    if (oi <= n_orders) {  // else this env is done (lanes of busier envs go on)
    int r = -1;
    int d[K];
    {
      union {
        uint4 v[NVR];
        uint16_t h[8 * NVR];
      } ur;
#pragma unroll
      for (int j = 0; j < NVR; j++) ur.v[j] = win[((oi / CH) & 1) * SB_REC + ((oi % CH) * NVR + j) * EPW + myjj];
      if (oi < n_orders) r = ur.h[0];
#pragma unroll
      for (int sk = 0; sk < K; sk++) d[sk] = ur.h[1 + sk];
    }
    // (prof build: the time of this block and its passes counted for the whole wave, i.e. also when
    // only another env of the wave changes region)
    PROF_T(q_f0);
#ifdef MSC_PROF
    PROF_ADD(q_nfin, __ballot(r != cur) != 0 ? 1ull : 0ull);
#endif
    if (r != cur) {
      if (cur >= 0) finalize(cur);
      {  // (at clamped indices, no branch: the values for r = -1 or a lane past W are never used)
        const int rr = r >= 0 ? r : 0, wc = wl ? w : 0;
        cof = TAB ? lof[rr * W + wc] : gp(c.ofT)[rr * W + wc];
        cov = TAB ? lov[rr * W + wc] : gp(c.ovT)[rr * W + wc];
      }
      cur = r;
      lost_cnt = 0;
#pragma unroll
      for (int sk = 0; sk < K; sk++) u[sk] = dsum[sk] = 0;
    }
    PROF_ADD(q_fin, PROF_NOW() - q_f0);
    if (oi < n_orders) {  // (at oi == n_orders only the last region's epilogue above)
    // (the weight sum starts at its first product: 0.0 + x == x for the products here, which are
    // never -0.0 -- quantities >= 0 times PositiveFloat weights, schema.py:174)
    double tw = (double)d[0] * skw[0];
#pragma unroll
    for (int sk = 0; sk < K; sk++) {
      dsum[sk] += d[sk];
      if (sk > 0) tw += (double)d[sk] * skw[sk];
    }
    // (an empty order needs no test of its own: no warehouse holds a needed SKU, so its first round
    // ends the loop, and with nothing unfulfilled it is never lost)
    int rem[K];
#pragma unroll
    for (int sk = 0; sk < K; sk++) rem[sk] = d[sk];
    unsigned dpk[NP];  // the order's quantities packed like the winners' fills
#pragma unroll
    for (int j = 0; j < NP; j++) dpk[j] = (unsigned)d[2 * j] | (2 * j + 1 < K ? (unsigned)d[2 * j + 1] << 16 : 0u);
    const double mycost = cof + cov * tw;  // demand_allocator.py:168-172
    // total-order key of the cost (negatives and -0.0 included), so the group min is an integer min
    const uint64_t cbits = (uint64_t)__double_as_longlong(mycost + 0.0);
    const uint64_t ckey = cbits ^ ((uint64_t)((int64_t)cbits >> 63) | 0x8000000000000000ull);
    int used = 0;
    bool open = true;
    PROF_T(q_a0);
    while (open) {
      PROF_ADD(q_iter, 1);
      // a warehouse that shipped already has nothing left that the order still needs
      // (fill = min(rem, inv) zeroes one of the two for every SKU), so "has" alone excludes it
      bool has = false;
#pragma unroll
      for (int sk = 0; sk < K; sk++) has |= rem[sk] > 0 && inv[sk] > 0;
      const uint64_t key = (has && wl) ? ckey : ~0ull;
      uint64_t mk = key;
      {
        auto step = [&](uint64_t o) { mk = o < mk ? o : mk; };
        auto dpp64 = [](auto f, uint64_t v) {
          const int lo = f((int)(unsigned)v), hi = f((int)(unsigned)(v >> 32));
          return ((uint64_t)(unsigned)hi << 32) | (unsigned)lo;
        };
        step(dpp64([](int v) { return dpp_x<0>(v); }, mk));
        if constexpr (GW >= 4) step(dpp64([](int v) { return dpp_x<1>(v); }, mk));
        if constexpr (GW >= 8) step(dpp64([](int v) { return dpp_x<2>(v); }, mk));
        if constexpr (GW >= 16) step(dpp64([](int v) { return dpp_x<3>(v); }, mk));
        if constexpr (GW >= 32) step(dpp64([](int v) { return dpp_x<4>(v); }, mk));
      }
      if (mk == ~0ull) {  // nobody holds a still-needed SKU: the order closes (an if/else, not a
        open = false;     // break: one loop exit, no lane masks merged from a second one per round)
      } else {
      // lowest warehouse among the group's minimum-cost lanes (argsort order on ties)
      const uint64_t tie = __ballot(key == mk);
      const int bw = __builtin_ctzll(tie >> gbase);
      const bool me = w == bw;
      int fl[K];
#pragma unroll
      for (int sk = 0; sk < K; sk++) fl[sk] = me ? (rem[sk] < inv[sk] ? rem[sk] : inv[sk]) : 0;
      // the winner's fill reaches every lane: 16-bit fields (fill <= order quantity < 2^16),
      // one nonzero contributor per group, so an OR reduction is the broadcast
      unsigned pk[NP];
#pragma unroll
      for (int j = 0; j < NP; j++)
        pk[j] = (unsigned)fl[2 * j] | (2 * j + 1 < K ? (unsigned)fl[2 * j + 1] << 16 : 0u);
#if MSC_SB_BPERM
      // one ds_bpermute per word from the winner lane (3 LDS-crossbar reads instead of an OR
      // butterfly of log2(GW) DPP steps per word)
      {
        const int src = (gbase + bw) << 2;
#pragma unroll
        for (int j = 0; j < NP; j++) pk[j] = (unsigned)__builtin_amdgcn_ds_bpermute(src, (int)pk[j]);
      }
#else
      // the NP words' OR butterflies interleaved stage by stage: each word's DPP reads a result two
      // instructions old instead of the one just written, so no s_nop fills the DPP hazard
      {
        auto stage = [&](auto f) {
#pragma unroll
          for (int j = 0; j < NP; j++) pk[j] |= (unsigned)f((int)pk[j]);
        };
        stage([](int v) { return dpp_x<0>(v); });
        if constexpr (GW >= 4) stage([](int v) { return dpp_x<1>(v); });
        if constexpr (GW >= 8) stage([](int v) { return dpp_x<2>(v); });
        if constexpr (GW >= 16) stage([](int v) { return dpp_x<3>(v); });
        if constexpr (GW >= 32) stage([](int v) { return dpp_x<4>(v); });
      }
#endif
      bool done = true;
#pragma unroll
      for (int sk = 0; sk < K; sk++) {
        rem[sk] -= (int)((pk[sk >> 1] >> (16 * (sk & 1))) & 0xffffu);
        done &= rem[sk] <= 0;
      }
      if (me) {
        int fsum = 0;
#pragma unroll
        for (int sk = 0; sk < K; sk++) {
          inv[sk] -= fl[sk];
          qsr[sk] += fl[sk];
          fsum += fl[sk];
        }
        bool whole = true;  // the fills are the whole order: their weight is tw, computed the same way
#pragma unroll
        for (int j = 0; j < NP; j++) whole &= pk[j] == dpk[j];
        if (whole) {
          out += mycost;
        } else {
          double fw = (double)fl[0] * skw[0];
#pragma unroll
          for (int sk = 1; sk < K; sk++) fw += (double)fl[sk] * skw[sk];
          out += fw == tw ? mycost : cof + cov * fw;  // whole order from here: the ranking cost bit for bit
        }
        if (dbg) {
#pragma unroll
          for (int sk = 0; sk < K; sk++) {
            if (info.shipment_quantities_by_sku) info.shipment_quantities_by_sku[((e * W + w) * R + r) * K + sk] += fl[sk];
            if (info.fulfilled_per_warehouse) info.fulfilled_per_warehouse[e * WK + w * K + sk] += fl[sk];
          }
          if (info.shipment_counts) info.shipment_counts[(e * W + w) * R + r] += 1;
          if (info.shipment_quantities) info.shipment_quantities[(e * W + w) * R + r] += fsum;
        }
      }
      used++;
      open = !done && used < maxwh;
      }
    }
    PROF_ADD(q_alloc, PROF_NOW() - q_a0);
    // (rem >= 0 throughout: every fill is min(rem, inv) with inv >= 0, so the unfulfilled units are
    // rem itself and "any left" is an OR of the words)
    int remor = 0;
#pragma unroll
    for (int sk = 0; sk < K; sk++) {
      remor |= rem[sk];
      u[sk] += rem[sk];
    }
    lost_cnt += remor != 0 ? 1 : 0;
    }
    }
  }
  PROF_ADD(q_all, PROF_NOW() - q_t0);
  PROF_FLUSH(10, q_all);
  PROF_FLUSH(11, q_fin);
  PROF_FLUSH(12, q_alloc);
  PROF_FLUSH(13, q_iter);
  PROF_FLUSH(14, q_nfin);
  PROF_FLUSH(15, 1ull);
  if constexpr (K <= 8) {
    if (c.fuse_c) {  // (uniform) phase C here: the step_c kernel is not launched
      step_b_phase_c<K, GW>(c, s, io, e, w, ev, wl, gbase, home_done != 0, inv, pen, out);
      return;
    }
  }
  if (ev && wl) {
#pragma unroll
    for (int sk = 0; sk < K; sk++) {
      const int64_t i = (int64_t)(w * K + sk) * E + e;
      s.sc_sht[i] = s.inv[i] - inv[sk];  // shipped this step = the inventory drop (only shipments lower it here)
      s.inv[i] = inv[sk];
      if (!home_done) s.sc_shh[i] = 0;
    }
    s.sc_pen[w * E + e] = pen;
    s.sc_out[w * E + e] = out;
  }
}

// ---- phase C ------------------------------------------------------------------------------
// WB: the most waves a block has; blocks of <= 8 waves get up to 256 VGPRs per lane, so the
// observation builder holds the pending ring in registers without spilling. One warehouse per wave
// up to STEP_WAVES warehouses (LOOP: each wave takes w, w + WB, ...; see each_warehouse)
#ifndef MSC_SC_WPE
// waves per SIMD the 16-wave step_c form is compiled for: 5 (<= 96 VGPRs, some spilled) lets two of
// its 8-wave blocks sit beside the pipelined demand kernel's waves on a CU; at 128 VGPRs only one did,
// and step_c ran in two rounds of blocks (C3 pipelined step: 300 -> 230 us, profiles/r06/ab_step_c_wpe.txt).
// In the rollout (policy kernels between steps) the 128-VGPR form without spills is faster (1.18 ->
// 1.14 ms per MAPPO step): c.sc_form picks it (msc_env_set_option MSC_OPT_STEP_C_FORM, set by the
// rollout collector)
#define MSC_SC_WPE 5
#endif
template <int K, bool DBG, int WB = STEP_WAVES, bool LOOP = false, int SCW = MSC_SC_WPE>
__global__ __launch_bounds__(BS * WB) __attribute__((amdgpu_waves_per_eu(WB == STEP_WAVES && !LOOP ? SCW : 1)))
void step_c_kernel(const DevEnv* __restrict__ dp, StepIO io) {
  constexpr int RREG = (WB <= 8 && K <= 8) ? OBS_RING_REG : 0;
  constexpr bool HSTAT = true;
  const EnvConst& c = dp->c;
  const EnvState& s = dp->s;
  extern __shared__ __attribute__((aligned(16))) double Lrw[];  // [W][BS] rewards (team sum)
  const int W = c.W, WK = W * K;
  const int64_t E = c.E;
  const int wave = threadIdx.x / BS, lane = threadIdx.x % BS;
  if (MSC_SC_PRIO > 0) __builtin_amdgcn_s_setprio(MSC_SC_PRIO);
  if (c.chain_prio) __builtin_amdgcn_s_setprio(3);  // the step chain is the caller's critical path
  const int64_t e = (int64_t)blockIdx.x * BS + lane;
  const bool ev = e < E;
  const msc_step_info info = io.info;
  constexpr bool dbg = DBG;
  const int t = ev ? s.t[e] : 0;
  if (ev) {
    const int hslot = t % MSC_HISTORY;
    each_warehouse<WB, LOOP>(wave, W, [&](const int w) {
      double hold = 0.0;
      // the loads first, then the stores (a load issued after a store waits for it: one vmcnt)
      int iv[K], v[K];
      float fo[K];
#pragma unroll
      for (int sk = 0; sk < K; sk++) {
        const int i = w * K + sk;
        iv[sk] = s.inv[i * E + e];
        v[sk] = s.inc[i * E + e];
        fo[sk] = s.fc[i * E + e];
      }
      const double pen = s.sc_pen[w * E + e], out = s.sc_out[w * E + e], inb = s.sc_inb[w * E + e];
#pragma unroll
      for (int sk = 0; sk < K; sk++) {
        const int i = w * K + sk;
        s.hist[((int64_t)hslot * WK + i) * E + e] = v[sk];
        s.fc[i * E + e] = 0.3f * (float)v[sk] + 0.7f * fo[sk];  // EMA forecast (f32)
        hold += c.hold_per_sku ? (double)iv[sk] * c.hold[sk] : ((double)iv[sk] * c.skw[sk]) * c.hold_scalar;
      }
      const double rw = -((((hold + pen) + out) + inb) * c.scale);
      Lrw[w * BS + lane] = rw;
      if (dbg && info.costs) {
        info.costs[(e * 4 + 0) * W + w] = hold;
        info.costs[(e * 4 + 1) * W + w] = pen;
        info.costs[(e * 4 + 2) * W + w] = out;
        info.costs[(e * 4 + 3) * W + w] = inb;
      }
    });
  }
  __syncthreads();
  const bool trunc = ev && t + 1 >= c.T;
  const int64_t obs_off = e * W * c.L;
  // observation staging: the block's 64 envs x W agents' vectors [env][W*L] (row stride W*L | 1,
  // odd: a wave's 64 lanes write 64 different banks), then written to HBM as the block's one
  // contiguous [64][W][L] range, every cache line whole (per-agent vectors of L floats at a
  // stride of W*L floats leave partly written lines per store)
  // obs_stage = P > 1: the agents staged in P phases of ceil(W / P) (a P-th of the LDS, so P times
  // as many blocks fit beside the demand kernel's; each phase's waves build, the block copies out)
  const int L = c.L, WL = W * L;
  const int P = c.obs_stage > 1 ? c.obs_stage : 1, WP = (W + P - 1) / P, RS = (WP * L) | 1;
  float* stg = reinterpret_cast<float*>(Lrw + W * BS);
  int32_t* Lskip = reinterpret_cast<int32_t*>(stg + BS * RS);  // [BS]: env's vector not staged
  // shipped home / total of this step, [(w*K+s) * E] from the env's column
  const int32_t* shh = s.sc_shh + e;
  const int32_t* sht = s.sc_sht + e;
  const int n_hist = t + 1 < MSC_HISTORY ? t + 1 : MSC_HISTORY;
  if (ev) {
    double team = 0.0;
    if (c.scope == MSC_SCOPE_TEAM)  // team scope: sum over agents in agent order
      for (int j = 0; j < W; j++) team += Lrw[j * BS + lane];
    each_warehouse<WB, LOOP>(wave, W, [&](const int w) {
      const double v = c.scope == MSC_SCOPE_TEAM ? team : Lrw[w * BS + lane];
      io.rew[e * W + w] = (float)v;
      if (io.rew64) io.rew64[e * W + w] = v;
      if (trunc && io.final_obs) build_obs_agent<K, RREG, HSTAT>(c, s, e, w, t, n_hist, shh, sht, E, io.final_obs + obs_off);
      if (!trunc && !c.obs_stage) build_obs_agent<K, RREG, HSTAT>(c, s, e, w, t, n_hist, shh, sht, E, io.obs + obs_off);
    });
  }
  if (c.obs_stage) {
    if (wave == 0) Lskip[lane] = (e >= E || trunc) ? 1 : 0;
    const int64_t e0 = (int64_t)blockIdx.x * BS;
    const int nenv = E - e0 < BS ? (int)(E - e0) : BS;
    const int nt = (int)blockDim.x;
    for (int p = 0; p < P; p++) {
      const int w0 = p * WP, nw = W - w0 < WP ? W - w0 : WP;
      if (nw <= 0) break;
      if (ev && !trunc)
        each_warehouse<WB, LOOP>(wave, W, [&](const int w) {
          if (w >= w0 && w < w0 + nw)  // (out + w * L lands at column (w - w0) * L)
            build_obs_agent<K, RREG, HSTAT>(c, s, e, w, t, n_hist, shh, sht, E, stg + lane * RS - w0 * L);
        });
      __syncthreads();
      const int NL = nw * L, n = nenv * NL;
      const int dq = nt / NL, dr = nt % NL;  // (env, column) step of the flat index per iteration
      int el = (int)threadIdx.x / NL, j = (int)threadIdx.x % NL;
      float* dst = io.obs + e0 * WL + w0 * L;
      for (int i = (int)threadIdx.x; i < n; i += nt) {
        if (!Lskip[el]) dst[(int64_t)el * WL + j] = stg[el * RS + j];
        j += dr;
        el += dq;
        if (j >= NL) {
          j -= NL;
          el += 1;
        }
      }
      if (p + 1 < P) __syncthreads();  // the next phase rewrites the stage
    }
  }
  // truncation: reset the env (one sequential RNG pass per env), then every agent's reset obs
  if (__syncthreads_or(trunc ? 1 : 0)) {
    if (ev && wave == 0) {
      io.trunc[e] = trunc ? 1 : 0;
      if (trunc) reset_env<K>(c, s, e, 0, nullptr);
      else s.t[e] = t + 1;
    }
    __syncthreads();
    if (trunc)
      each_warehouse<WB, LOOP>(wave, W, [&](const int w) {
        build_obs_agent<K>(c, s, e, w, 0, 0, nullptr, nullptr, 0, io.obs + obs_off);
      });
  } else if (ev && wave == 0) {
    io.trunc[e] = 0;
    s.t[e] = t + 1;
  }
}

// flat per-agent obs [E][W][L(1+W)] = local_w || local_0 .. local_{W-1} (multi_env.py:566-573)
#ifndef MSC_EK_WIDE  // (defined once: env_kernels.hip proper)
__global__ void obs_flat_kernel(const float* __restrict__ obs, float* __restrict__ flat, int64_t E, int W, int L) {
  const int64_t FL = (int64_t)L * (1 + W);
  const int64_t n = E * W * FL;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < n; idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = idx % FL, ew = idx / FL, e = ew / W;
    const int64_t w = ew % W;
    flat[idx] = j < L ? obs[(e * W + w) * L + j] : obs[e * W * L + (j - L)];
  }
}
#endif

// ------------------------------------------------------------------------------------------
// launchers: dispatch on (K, W bucket). The file is compiled three times (translation units that
// build in parallel): SKU counts 1-8 with every non-template kernel and entry point, and
// (env_kernels_wide.hip: MSC_EK_WIDE 1 / 2) SKU counts 9-12 / 13-16, whose *_w1 / *_w2 entry
// points the first part's switches call.
// ------------------------------------------------------------------------------------------
// (the cases are spelled out: a BODY holding a kernel launch cannot pass through a second macro)
#ifndef MSC_EK_WIDE
#define MSC_EK_FN(name) name
#define MSC_K_SWITCH(KV, BODY, W1, W2) \
  switch (KV) { \
    case 1: { constexpr int K = 1; BODY; } break; \
    case 2: { constexpr int K = 2; BODY; } break; \
    case 3: { constexpr int K = 3; BODY; } break; \
    case 4: { constexpr int K = 4; BODY; } break; \
    case 5: { constexpr int K = 5; BODY; } break; \
    case 6: { constexpr int K = 6; BODY; } break; \
    case 7: { constexpr int K = 7; BODY; } break; \
    case 8: { constexpr int K = 8; BODY; } break; \
    default: \
      if ((KV) > 8 && (KV) <= 12) { W1; } \
      if ((KV) > 12 && (KV) <= MSC_MAX_K) { W2; } \
      return hipErrorInvalidValue; \
  }
#define MSC_EK_DECL(S)                                                                                    \
  hipError_t launch_reset_##S(const EnvConst& c, const DevEnv* d, const uint8_t* mask, const uint32_t* new_roots, \
                              int32_t flags, float* obs, hipStream_t st);                                 \
  hipError_t launch_demand_##S(const EnvConst& c, const DevEnv* d, hipStream_t st);                       \
  hipError_t launch_demand_ea_##S(const EnvConst& c, const DevEnv* d, const EaLaunch& ea, hipStream_t st); \
  hipError_t launch_step_##S(const EnvConst& c, const DevEnv* d, const StepIO& io, bool gen, hipStream_t st);
MSC_EK_DECL(w1)
MSC_EK_DECL(w2)
#undef MSC_EK_DECL

int order_record_vec4(int K) { return (1 + K + 7) / 8; }

void launch_alloc_sort(const DevEnv* d, const StepIO& io, hipStream_t st) {
  hipLaunchKernelGGL(alloc_sort_kernel, dim3(1), dim3(1024), 0, st, d, io);
}
#elif MSC_EK_WIDE == 1
#define MSC_EK_FN(name) name##_w1
#define MSC_K_SWITCH(KV, BODY, W1, W2) \
  switch (KV) { \
    case 9: { constexpr int K = 9; BODY; } break; \
    case 10: { constexpr int K = 10; BODY; } break; \
    case 11: { constexpr int K = 11; BODY; } break; \
    case 12: { constexpr int K = 12; BODY; } break; \
    default: return hipErrorInvalidValue; \
  }
void launch_alloc_sort(const DevEnv* d, const StepIO& io, hipStream_t st);
#else
#define MSC_EK_FN(name) name##_w2
#define MSC_K_SWITCH(KV, BODY, W1, W2) \
  switch (KV) { \
    case 13: { constexpr int K = 13; BODY; } break; \
    case 14: { constexpr int K = 14; BODY; } break; \
    case 15: { constexpr int K = 15; BODY; } break; \
    case 16: { constexpr int K = 16; BODY; } break; \
    default: return hipErrorInvalidValue; \
  }
void launch_alloc_sort(const DevEnv* d, const StepIO& io, hipStream_t st);
#endif

static dim3 grid_for(int64_t E, int epw = BS) { return dim3((unsigned)((E + epw - 1) / epw)); }

hipError_t MSC_EK_FN(launch_reset)(const EnvConst& c, const DevEnv* d, const uint8_t* mask, const uint32_t* new_roots,
                                   int32_t flags, float* obs, hipStream_t st) {
  MSC_K_SWITCH(c.K, hipLaunchKernelGGL(reset_kernel<K>, grid_for(c.E), dim3(BS), 0, st, d, mask, new_roots, flags, obs),
               return launch_reset_w1(c, d, mask, new_roots, flags, obs, st),
               return launch_reset_w2(c, d, mask, new_roots, flags, obs, st));
  return hipGetLastError();
}

static size_t park_fixed(const EnvConst& c) { return c.demand_impl == 5 ? park4_lds_fixed() : unit_lds_fixed(); }
[[maybe_unused]] static bool park_lds_tables(const EnvConst& c) {
  return park_fixed(c) + (size_t)(2 + c.K) * c.R * sizeof(double) <= 40 * 1024;
}
#ifndef MSC_EK_WIDE
size_t demand_lds_bytes(const EnvConst& c) {
  return park_fixed(c) + (park_lds_tables(c) ? (size_t)(2 + c.K) * c.R * sizeof(double) : 0);
}
#endif

template <int K, int G>
static hipError_t launch_split_demand(const EnvConst& c, const DevEnv* d, hipStream_t st, const EaLaunch* ea) {
  using DFn = void (*)(const DevEnv*);
  using UFn = void (*)(const DevEnv*, EaLaunch);
  if (c.demand_ptrs) {  // a rate >= 10: numpy's PTRS branch, the sequential sampler (demand_ab.hip)
    return launch_demand_seq(c, d, st, ea);
  }
  if (G == 3 && c.demand_impl == 7 && demand_ab_supported(c)) {  // the split parser (demand_ab.hip, A/B)
    return launch_demand_ab(c, d, st, ea);
  }
  if (G == 3 && c.demand_impl >= 8) {  // the f32-ring / short-round parsers (demand_v2.hip, demand_v3.hip)
    const hipError_t ealt = launch_demand_alt(c, d, st, ea);
    if (ealt != hipErrorNotSupported) return ealt;
  }
  const size_t tab = (size_t)(2 + K) * c.R * sizeof(double);
  const bool t = park_lds_tables(c);
  const size_t lds = park_fixed(c) + (t && !c.demand_uni ? tab : 0);
  if (ea) {  // episode-ahead generation over nslots x E lanes
    const UFn fn = c.demand_uni ? (UFn)demand_unit_kernel<K, G, false, true, true>
                                : (t ? (UFn)demand_unit_kernel<K, G, true, false, true> : (UFn)demand_unit_kernel<K, G, false, false, true>);
    const size_t lds_u = unit_lds_fixed() + (t && !c.demand_uni ? tab : 0);
    hipLaunchKernelGGL(fn, grid_for((int64_t)ea->nslots * c.E, c.epw_dem), dim3(BS * (1 + G)), lds_u, st, d, *ea);
    return hipGetLastError();
  }
  if (c.demand_impl == 5) {  // 4-draw parking parser (A/B: MSC_DEMAND_IMPL=park4)
    const DFn fn = t ? (DFn)demand_park4_kernel<K, G, true> : (DFn)demand_park4_kernel<K, G, false>;
    hipLaunchKernelGGL(fn, grid_for(c.E, c.epw_dem), dim3(BS * (1 + G)), lds, st, d);
    return hipGetLastError();
  }
  const UFn fn = c.demand_uni ? (UFn)demand_unit_kernel<K, G, false, true, false>
                              : (t ? (UFn)demand_unit_kernel<K, G, true, false, false> : (UFn)demand_unit_kernel<K, G, false, false, false>);
  hipLaunchKernelGGL(fn, grid_for(c.E, c.epw_dem), dim3(BS * (1 + G)), lds, st, d, EaLaunch{0, 0, 0, 0, 0, 0, 0});
  return hipGetLastError();
}

template <int K>
static hipError_t launch_demand_k(const EnvConst& c, const DevEnv* d, hipStream_t st, const EaLaunch* ea = nullptr) {
  if constexpr (K > 8) {  // above 8 SKUs: the sequential sampler (demand_ab.hip), per step or episode-ahead
    return launch_demand_seq(c, d, st, ea);
  } else if (c.demand_gen == 1) {
    return launch_split_demand<K, 1>(c, d, st, ea);
  } else if (c.demand_gen == 2) {
    return launch_split_demand<K, 2>(c, d, st, ea);
  } else {
    if constexpr (K == 5) {  // (A/B: 5 and 7 generator waves per block, 5 SKUs only)
      if (c.demand_gen == 5) return launch_split_demand<K, 5>(c, d, st, ea);
      if (c.demand_gen == 7) return launch_split_demand<K, 7>(c, d, st, ea);
    }
    return launch_split_demand<K, 3>(c, d, st, ea);
  }
}

hipError_t MSC_EK_FN(launch_demand)(const EnvConst& c, const DevEnv* d, hipStream_t st) {
  MSC_K_SWITCH(c.K, return launch_demand_k<K>(c, d, st), return launch_demand_w1(c, d, st),
               return launch_demand_w2(c, d, st));
  return hipSuccess;
}

hipError_t MSC_EK_FN(launch_demand_ea)(const EnvConst& c, const DevEnv* d, const EaLaunch& ea, hipStream_t st) {
  if (ea.nslots < 1) return hipSuccess;
  MSC_K_SWITCH(c.K, return launch_demand_k<K>(c, d, st, &ea), return launch_demand_ea_w1(c, d, ea, st),
               return launch_demand_ea_w2(c, d, ea, st));
  return hipSuccess;
}

#ifndef MSC_EK_WIDE
hipError_t launch_ea_materialize(const EnvConst& c, const DevEnv* d, int slot, int t_done, hipStream_t st) {
  hipLaunchKernelGGL(ea_materialize_kernel, grid_for(c.E, 256), dim3(256), 0, st, d, slot, t_done);
  return hipGetLastError();
}
#endif

template <int K>
static hipError_t launch_step_k(const EnvConst& c, const DevEnv* d, const StepIO& io, bool gen, hipStream_t st) {
  if (gen && c.demand_type == MSC_DEMAND_POISSON) {  // the orders the step kernels below consume
    const hipError_t ed = launch_demand_k<K>(c, d, st);
    if (ed != hipSuccess) return ed;
  }
  using KFn = void (*)(const DevEnv*, StepIO);
  // three phase kernels, group-per-env allocation
  int GW = c.W <= 2 ? 2 : c.W <= 4 ? 4 : c.W <= 8 ? 8 : c.W <= 16 ? 16 : 32;
  if (c.sb_gw > GW) GW = c.sb_gw;  // (A/B: wider lane groups, fewer envs per wave)
  const bool dbg = io.has_info != 0;  // collect_step_info: the instrumented instantiations
  // step_a / step_c: one wave per warehouse, or (> 16 warehouses, > 8 SKUs) LW waves looping
  constexpr int LW = step_loop_waves(K);
  int nwv = c.W;
  KFn a, cc;
  auto loop_forms = [&] {
    nwv = c.W < LW ? c.W : LW;
    a = dbg ? (KFn)step_a_kernel<K, true, false, LW, true> : (KFn)step_a_kernel<K, false, false, LW, true>;
    cc = dbg ? (KFn)step_c_kernel<K, true, LW, true> : (KFn)step_c_kernel<K, false, LW, true>;
  };
  if constexpr (K > 8) {
    loop_forms();
  } else if (c.W > STEP_WAVES) {
    loop_forms();
  } else {
    a = c.obs_ring_reg ? (dbg ? (KFn)step_a_kernel<K, true, true> : (KFn)step_a_kernel<K, false, true>)
                       : (dbg ? (KFn)step_a_kernel<K, true> : (KFn)step_a_kernel<K, false>);
    cc = (c.W <= 8 && c.obs_ring_reg) ? (dbg ? (KFn)step_c_kernel<K, true, 8> : (KFn)step_c_kernel<K, false, 8>)
       : c.sc_form == 4 ? (dbg ? (KFn)step_c_kernel<K, true, STEP_WAVES, false, 4> : (KFn)step_c_kernel<K, false, STEP_WAVES, false, 4>)
                        : (dbg ? (KFn)step_c_kernel<K, true> : (KFn)step_c_kernel<K, false>);
  }
  const bool tab = c.sb_tab != 0;  // (capi.hip: small tables, or room at this occupancy)
  KFn b;
#define MSC_SB(GWV)                                                                                   \
  (dbg ? (tab ? (KFn)step_b_kernel<K, GWV, true, true> : (KFn)step_b_kernel<K, GWV, true, false>)   \
       : (tab ? (KFn)step_b_kernel<K, GWV, false, true> : (KFn)step_b_kernel<K, GWV, false, false>))
  b = GW == 2 ? MSC_SB(2) : GW == 4 ? MSC_SB(4) : GW == 8 ? MSC_SB(8) : GW == 16 ? MSC_SB(16) : MSC_SB(32);
#undef MSC_SB
  if (!(c.alloc_impl == 2 && c.fuse_a)) hipLaunchKernelGGL(a, grid_for(c.E), dim3(BS * nwv), 0, st, d, io);
  if (c.alloc_impl == 0) {
    const hipError_t ea = launch_alloc_lane(c, d, io, st);
    if (ea != hipSuccess) return ea;
  } else if (c.alloc_impl == 2) {
    const hipError_t ea = launch_alloc_scan(c, d, io, st);
    if (ea != hipSuccess) return ea;
  } else {
    if (c.alloc_sort) launch_alloc_sort(d, io, st);
    const int bt = 64 * step_b_waves(GW, tab);
    const size_t lds_b = step_b_lds_bytes(c.R, c.W, tab, bt / 64);
    if (lds_b > 64 * 1024) {
      const hipError_t e = hipFuncSetAttribute((const void*)b, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_b);
      if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(b, dim3((unsigned)((c.E * GW + bt - 1) / bt)), dim3(bt), lds_b, st, d, io);
  }
  if (c.fuse_c && c.alloc_impl != 0) return hipGetLastError();  // (phase C ran inside the allocator)
  const int stage_w = c.obs_stage ? (c.W + (c.obs_stage > 1 ? c.obs_stage : 1) - 1) / (c.obs_stage > 1 ? c.obs_stage : 1) : 0;
  const size_t lds_c = (size_t)c.W * BS * sizeof(double) +
                       (c.obs_stage ? (size_t)BS * ((stage_w * c.L) | 1) * sizeof(float) + BS * sizeof(int32_t) : 0);
  hipLaunchKernelGGL(cc, grid_for(c.E), dim3(BS * nwv), lds_c, st, d, io);
  return hipGetLastError();
}

hipError_t MSC_EK_FN(launch_step)(const EnvConst& c, const DevEnv* d, const StepIO& io, bool gen, hipStream_t st) {
  MSC_K_SWITCH(c.K, return launch_step_k<K>(c, d, io, gen, st), return launch_step_w1(c, d, io, gen, st),
               return launch_step_w2(c, d, io, gen, st));
  return hipSuccess;
}

#ifndef MSC_EK_WIDE
hipError_t launch_obs_flat(const EnvConst& c, const float* obs, float* flat, hipStream_t st) {
  const int64_t n = c.E * c.W * (int64_t)c.L * (1 + c.W);
  const int64_t blocks = (n + 255) / 256 < 65536 ? (n + 255) / 256 : 65536;
  hipLaunchKernelGGL(obs_flat_kernel, dim3((unsigned)blocks), dim3(256), 0, st, obs, flat, c.E, c.W, c.L);
  return hipGetLastError();
}
#endif

#if defined(MSC_PROF) && !defined(MSC_EK_WIDE)
extern "C" int msc_debug_prof(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_prof), sizeof(unsigned long long) * 16) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof z) != hipSuccess) return -1;
  }
  return 0;
}
#endif

}  // namespace msc
