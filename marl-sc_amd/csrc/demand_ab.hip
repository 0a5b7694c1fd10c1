// demand_ab.hip -- PoissonDemandSampler.sample (demand_sampler.py:105-163) for equal sampler
// parameters in every region (the scalar `params` form, demand_sampler.py:99-102, and every BASELINE
// config), with the per-env parse split over two waves.
//
// demand_unit_kernel<UNI> (env_kernels.hip) runs one parser wave per 64 envs whose every round
// resolves one unit (a region's order count, an order's SKU mask or one SKU quantity) and then
// settles it: books the result into the order record, opens the next unit. Measured, that wave is
// the kernel's critical path: ~1,490 dependent rounds of ~115 VALU at a lone wave's issue cadence
// (~4-5 cycles per instruction), ~850 cycles per round. Only part of a round feeds the next one:
// the ring reads, the product chain, the unit length and the state transition (which threshold and
// which unit kind come next). The bookkeeping -- record headers, the 16-bit quantity stores, the
// record pointer and count, the episode-ahead step boundaries -- does not.
//
// So each block runs
//   wave 0  chain parser A: per round the 8 ring reads, the chained f64 products, the unit length
//           or SKU-mask bits, the reduced transition; it logs one byte per round (the unit count or
//           the mask bits) into an LDS log;
//   wave 1  bookkeeper B: one chunk (UHS rounds) behind A, replays the same transition from the
//           logged bytes (deterministic: the same state machine on the same inputs) and does every
//           store;
//   waves 2.. generators: unchanged (stream positions g, g + G, ... into the [slot][lane] ring,
//           refilled by quota, demand_common.hpp).
// The log is double-buffered per chunk ([2][64 lanes][UHS] bytes: A writes byte hs of its lane's
// word, B reads the word); the chunk barrier that publishes A's positions to the generators also
// hands the chunk's log to B. Results are bit-identical to demand_unit_kernel (same arithmetic,
// same order of draws).
#include <hip/hip_runtime.h>

#include "demand_common.hpp"

namespace msc {

#ifdef MSC_PROF
// in-kernel cycle accounting (profiling build: make prof, tools/prof_demand.py): [0] A cycles, [1] A
// at barriers, [2] A rounds, [3] A waves, [4] B cycles, [5] B at barriers, [6] B replaying,
// [7] generator cycles, [8] generators at barriers, [9] generator waves
__device__ unsigned long long g_prof_ab[16];
#define ABP_T(v) const unsigned long long v = (unsigned long long)clock64()
#define ABP_DECL(v) unsigned long long v = 0
#define ABP_ADD(v, x) (v) += (x)
#define ABP_FLUSH(i, v) \
  if ((threadIdx.x & 63) == 0) atomicAdd(&g_prof_ab[i], (v))
#else
#define ABP_T(v)
#define ABP_DECL(v)
#define ABP_ADD(v, x)
#define ABP_FLUSH(i, v)
#endif

#ifndef MSC_BOOK_PRIO
#define MSC_BOOK_PRIO 2  // s_setprio of the bookkeeper wave
#endif

__host__ __device__ constexpr size_t ab_lds_fixed() {
  return unit_lds_fixed() + (size_t)2 * BS * UHS;  // + the unit log
}
static_assert(UHS == 4, "the bookkeeper reads a chunk's log bytes as one 32-bit word per lane");

// the state both A and B advance, unit by unit (settle_uni of demand_unit_kernel restated; BOOK =
// the bookkeeper's copy, which also stores)
template <int K, bool EA, bool BOOK>
struct ParseState {
  int st, r, x, left, tstep, rd, live, mf, pend;
  unsigned mask;
  // bookkeeper only
  int n, sq;
  MSC_GLOBAL char* recp;

  __device__ __forceinline__ void settle(int R_s, int T_s, int cap_s, int64_t rstride_s, int64_t vstride, int64_t E,
                                         decltype(EnvState::ea_off) ea_offp, decltype(EnvState::ea_pos) ea_posp,
                                         uint32_t ea_p0, double u_thr_o, double u_thr_m, double u_thr_q, double& thr,
                                         double& prod) {
    constexpr int NV = Rec<K>::NV;
    const int is_q = st == PS_QTY ? 1 : 0, is_o = st == PS_ORD ? 1 : 0;
    if constexpr (BOOK) {
      if (is_q & (n <= cap_s ? 1 : 0)) {
        const int h = 1 + sq;  // 16-bit field of the record (field 0 = region)
        MSC_GLOBAL char* fp = NV == 1 ? recp + h * 2 : recp + (int64_t)(h >> 3) * vstride + (h & 7) * 2;
        *reinterpret_cast<MSC_GLOBAL uint16_t*>(fp) = (uint16_t)(x > 1 ? x : 1);  // max(1, Poisson(lambda_q))
      }
    }
    const unsigned m2 = is_q ? (mask & (mask - 1u)) : mask;  // a mask unit left its bits in mask
    const int has_q = (is_o ^ 1) & (m2 != 0u ? 1 : 0);
    const int left2 = (is_o ? x : left) - ((is_o | has_q) ^ 1);  // an order completed
    const int new_order = (has_q ^ 1) & (left2 > 0 ? 1 : 0);
    const int new_region = (has_q | new_order) ^ 1;
    if constexpr (BOOK) sq = __builtin_ctz(m2 | (1u << K));
    int wrap = 0;  // EA: the step's last region ended and another step of the episode follows
    if constexpr (EA) {
      if (new_region & (r + 1 == R_s ? 1 : 0)) {
        if constexpr (BOOK) {
          ea_offp[(int64_t)(tstep + 1) * E] = n;
          ea_posp[(int64_t)tstep * E] = ea_p0 + (uint32_t)rd;
        }
        wrap = tstep + 1 < T_s ? 1 : 0;
        tstep += wrap;
      }
    }
    st = has_q ? PS_QTY : new_order ? PS_MASK : ((r + new_region < R_s) | wrap ? PS_ORD : PS_DONE);
    if constexpr (!BOOK) {
      // three-way threshold choice as a bit select (a ?: chain becomes a scratch lookup table)
      const uint64_t bo = (uint64_t)__double_as_longlong(u_thr_o), bm = (uint64_t)__double_as_longlong(u_thr_m),
                     bq = (uint64_t)__double_as_longlong(u_thr_q);
      const uint64_t mo = (uint64_t)0 - (uint64_t)new_order, mq = (uint64_t)0 - (uint64_t)has_q;
      uint64_t b = bo ^ ((bo ^ bm) & mo);
      b = b ^ ((b ^ bq) & mq);
      thr = __longlong_as_double((long long)b);
      prod = 1.0;
    }
    mask = new_order ? 0u : m2;
    left = left2;
    if constexpr (BOOK) {
      n += new_order;
      recp += new_order ? rstride_s : 0;
      if (new_order & (n <= cap_s ? 1 : 0)) {
#pragma unroll
        for (int j = 0; j < NV; j++)
          *reinterpret_cast<MSC_GLOBAL v4u*>(recp + (int64_t)j * vstride) = v4u{j == 0 ? (unsigned)r : 0u, 0u, 0u, 0u};
      }
    }
    r = wrap ? 0 : r + new_region;
    x = 0;
    mf = st == PS_MASK ? 1 : 0;
    live = st != PS_DONE ? 1 : 0;
  }

  // the round's outcome (ncont: leading products above the threshold; bits: the mask unit's SKU
  // draws), applied after the settle exactly as the chain parser applies it
  __device__ __forceinline__ void advance(int ncont, unsigned bits) {
    const int go = ncont >= UD ? 1 : 0;  // Poisson unit still running after UD draws
    const int cons = mf ? K : (go ? UD : ncont + 1);
    mask = mf ? bits : mask;
    x += ncont;  // (a mask unit's x is unused and cleared by its settle)
    rd += live ? cons : 0;
    pend = live & (mf | (go ^ 1));
  }
};

template <int K, int G, bool EA>
__global__ __launch_bounds__(BS * (2 + G)) __attribute__((amdgpu_waves_per_eu(MSC_DEM_WPE))) void demand_ab_kernel(
    const DevEnv* __restrict__ dp, EaLaunch ea) {
  const EnvConst& c = dp->c;
  const EnvState& s = dp->s;
  constexpr int NV = Rec<K>::NV;
  static_assert(K <= UD, "a mask unit completes in one round");
  extern __shared__ __attribute__((aligned(16))) double plds[];
  __shared__ int more[2];
  double* ring = plds;                                                        // [USLOTS][BS]
  int32_t* rdv = reinterpret_cast<int32_t*>(plds + BS * USLOTS);              // [2][BS]
  uint8_t* ulog = reinterpret_cast<uint8_t*>(rdv + 2 * BS);                   // [2][BS][UHS]
  const int wave = (int)(threadIdx.x / BS), lane = threadIdx.x % BS;          // 0: parser A, 1: bookkeeper B
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
  double* myring = ring + lane;

  if (wave >= 2) {
    // ---------------- generator g: stream positions g, g + G, g + 2G, ... (demand_unit_kernel's)
    if (MSC_GEN_PRIO > 0) __builtin_amdgcn_s_setprio(MSC_GEN_PRIO);
    const int g = wave - 2;
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
        const int sl = pg & (UCAP - 1);
        myring[sl * BS] = u;
        myring[(sl < UD - 1 ? sl + UCAP : USLOTS - 1) * BS] = u;  // mirror (or the dummy row)
        lcg128(th, tl, mh, ml, ch, cl);
        pg += G;
      }
    };
    int tgt = UCAP;
    ABP_T(g0);
    ABP_DECL(gbar);
    if (valid) gen_to(UCAP);
    __syncthreads();
    for (int ci = 0;; ci++) {
      const int rdp = rdv[(ci & 1) * BS + lane];
      tgt = unit_quota(tgt, rdp);
      if (valid) gen_to(tgt);
      ABP_T(gb0);
      __syncthreads();
      ABP_ADD(gbar, (unsigned long long)clock64() - gb0);
      if (!more[ci & 1]) break;
      const int need = rdv[((ci + 1) & 1) * BS + lane] + UHS * UD;
      if (__ballot(valid && tgt < need) != 0) {
        tgt = tgt > need ? tgt : need;
        if (valid) gen_to(tgt);
        ABP_T(gb1);
        __syncthreads();
        ABP_ADD(gbar, (unsigned long long)clock64() - gb1);
      }
    }
    ABP_FLUSH(7, (unsigned long long)clock64() - g0);
    ABP_FLUSH(8, gbar);
    ABP_FLUSH(9, 1ull);
    return;
  }

  // ---------------- parser A (wave 0) and bookkeeper B (wave 1)
  const double u_thr_o = sgpr_d(c.uni_thr_o), u_thr_m = sgpr_d(c.uni_thr_m), u_thr_q = sgpr_d(c.uni_thr_q);
  const int cap = EA ? (int)c.ea_cap : c.order_cap;
  const int R_s = __builtin_amdgcn_readfirstlane(c.R), cap_s = __builtin_amdgcn_readfirstlane(cap);
  const int T_s = __builtin_amdgcn_readfirstlane(EA ? ea.t1 : c.T);  // EA: the chunk's last step + 1
  const int64_t vstride = EA ? 16 : E * 16;       // bytes between the uint4 words of a record
  const int64_t rstride = (int64_t)NV * vstride;  // bytes between consecutive records of a lane
  const int64_t rstride_s = (int64_t)__builtin_amdgcn_readfirstlane((uint32_t)rstride) |
                            ((int64_t)__builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)rstride >> 32)) << 32);
  decltype(s.ea_off) ea_offp = EA ? s.ea_off + (int64_t)slot * (c.T + 1) * E + e : nullptr;
  decltype(s.ea_pos) ea_posp = EA ? s.ea_pos + (int64_t)slot * c.T * E + e : nullptr;

  if (wave == 1) {
    // ---------------- bookkeeper B: replays chunk ci - 1 while A parses chunk ci
    __builtin_amdgcn_s_setprio(MSC_BOOK_PRIO);
    ParseState<K, EA, true> b{};
    b.st = valid ? PS_ORD : PS_DONE;
    b.live = valid ? 1 : 0;
    b.n = ea_n0;
    b.recp = reinterpret_cast<MSC_GLOBAL char*>(
                 gp(EA ? s.ea_rec + ((int64_t)slot * E + e) * c.ea_cap * NV : s.orders + e)) + (int64_t)(b.n - 1) * rstride;
    b.tstep = EA ? ea.t0 : 0;
    double thr_d = 0.0, prod_d = 0.0;  // (unused by the bookkeeper's settle)
    auto replay = [&](int buf) {
      const uint32_t w = *reinterpret_cast<const uint32_t*>(ulog + (buf * BS + lane) * UHS);
#pragma unroll
      for (int hs = 0; hs < UHS; hs++) {
        if (b.pend)
          b.settle(R_s, T_s, cap_s, rstride_s, vstride, E, ea_offp, ea_posp, ea_p0, u_thr_o, u_thr_m, u_thr_q, thr_d,
                   prod_d);
        const unsigned v = (w >> (8 * hs)) & 0xffu;
        b.advance(b.mf ? 0 : (int)v, v);
      }
    };
    __syncthreads();  // the initial fill
    ABP_T(b0);
    ABP_DECL(bbar);
    ABP_DECL(brep);
    int ptgt = UCAP, rd_start = 0;  // the generators' fill target, restated (their top-up barrier)
    for (int ci = 0;; ci++) {
      ABP_T(br0);
      if (ci > 0) replay((ci - 1) & 1);
      ABP_T(bb0);
      ABP_ADD(brep, bb0 - br0);
      __syncthreads();
      ABP_ADD(bbar, (unsigned long long)clock64() - bb0);
      if (!more[ci & 1]) {
        replay(ci & 1);
        break;
      }
      const int rd_a = rdv[((ci + 1) & 1) * BS + lane];  // A's position after chunk ci
      ptgt = unit_quota(ptgt, rd_start);
      const int need = rd_a + UHS * UD;
      if (__ballot(valid && ptgt < need) != 0) {
        ptgt = ptgt > need ? ptgt : need;
        ABP_T(bb1);
        __syncthreads();
        ABP_ADD(bbar, (unsigned long long)clock64() - bb1);
      }
      rd_start = rd_a;
    }
    ABP_FLUSH(4, (unsigned long long)clock64() - b0);
    ABP_FLUSH(5, bbar);
    ABP_FLUSH(6, brep);
    if (!valid) return;
    if (b.n > cap) atomicOr(s.err, ERR_ORDER_OVERFLOW);
    if constexpr (!EA) s.n_orders[e] = b.n > cap ? cap : b.n;
    return;
  }

  // ---------------- chain parser A (wave 0)
  // Older and higher-priority waves win VALU issue arbitration on a SIMD (MI355X_MICROARCH.md, wave
  // scheduling): the parser is the per-env critical path, the generators only stay a chunk ahead.
  __builtin_amdgcn_s_setprio(MSC_PARSER_PRIO);
  Pcg64 r0{};
  if (valid) {
    r0 = start_rng();
    if constexpr (!EA) store_rng_pre(s, e, E, r0);
  }
  rdv[lane] = 0;
  ParseState<K, EA, false> a{};
  a.st = valid ? PS_ORD : PS_DONE;
  a.live = valid ? 1 : 0;
  a.tstep = EA ? ea.t0 : 0;
  double thr = u_thr_o, prod = 1.0;
  __syncthreads();
  if constexpr (EA) {
    // (after the barrier: every wave of the block has read the slot's previous counter)
    if (valid && ea.t0 == 0) {
      s.ea_cnt[(int64_t)slot * E + e] = ea_cnt_new;
      ea_offp[0] = 0;
    }
  }
  int ptgt = UCAP, rd_start = 0;  // the generators' fill target and the chunk's start position
  ABP_T(a0);
  ABP_DECL(abar);
  ABP_DECL(arounds);
  for (int ci = 0;; ci++) {
    ABP_ADD(arounds, UHS);
    uint8_t* lg = ulog + ((ci & 1) * BS + lane) * UHS;
#pragma unroll 1
    for (int hs = 0; hs < UHS; hs++) {
      // issue this round's ring reads first, then the transition of the unit that ended last round
      // (no LDS dependence) while they are in flight
      const double* rp = myring + (a.rd & (UCAP - 1)) * BS;
      double u[UD];
#pragma unroll
      for (int i = 0; i < UD; i++) u[i] = rp[i * BS];
      if (a.pend)
        a.settle(R_s, T_s, cap_s, rstride_s, vstride, E, ea_offp, ea_posp, ea_p0, u_thr_o, u_thr_m, u_thr_q, thr, prod);
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
      lg[hs] = (uint8_t)(a.mf ? bits : (unsigned)ncont);
      prod = p;
      a.advance(ncont, bits);
    }
    // a lane with a booked-but-unsettled unit is still live: it settles in the next round
    const bool any = __ballot(a.live) != 0;
    rdv[((ci + 1) & 1) * BS + lane] = a.rd;
    if (lane == 0) more[ci & 1] = any ? 1 : 0;
    ABP_T(ab0);
    __syncthreads();
    ABP_ADD(abar, (unsigned long long)clock64() - ab0);
    if (!any) break;
    // the generators' refill decision, restated: their top-up barrier (if any) is joined here
    ptgt = unit_quota(ptgt, rd_start);
    const int need = a.rd + UHS * UD;
    if (__ballot(valid && ptgt < need) != 0) {
      ptgt = ptgt > need ? ptgt : need;
      ABP_T(ab1);
      __syncthreads();
      ABP_ADD(abar, (unsigned long long)clock64() - ab1);
    }
    rd_start = a.rd;
  }
  ABP_FLUSH(0, (unsigned long long)clock64() - a0);
  ABP_FLUSH(1, abar);
  ABP_FLUSH(2, arounds);
  ABP_FLUSH(3, 1ull);
  if (!valid) return;
  if constexpr (!EA) {
    pcg_advance(r0, (uint64_t)a.rd);
    store_rng(s, 0, e, E, r0);
  }
}

// ------------------------------------------------------------------------------------------
// demand_seq_kernel: PoissonDemandSampler.sample for parameter sets with a rate >= 10 (numpy's PTRS
// branch, demand_sampler.py:138,153 call Generator.poisson with any rate). One lane per env (or per
// (slot, env) of an episode-ahead launch) walks the reference's loops draw by draw: a region's order
// count, each order's K Bernoulli SKU draws, each drawn SKU's max(1, Poisson) quantity, with
// random_poisson's branch per rate (multiplication method below 10, PTRS at or above). No generator
// waves: PTRS trials take two draws each and reject data-dependently, which the ring parser's
// fixed 8-draw rounds do not model; such configs are outside every BASELINE shape.
// ------------------------------------------------------------------------------------------
template <int K, bool EA>
__global__ __launch_bounds__(BS) void demand_seq_kernel(const DevEnv* __restrict__ dp, EaLaunch ea) {
  const EnvConst& c = dp->c;
  const EnvState& s = dp->s;
  constexpr int NV = Rec<K>::NV;
  const int64_t E = c.E;
  const int64_t vlane = (int64_t)blockIdx.x * BS + threadIdx.x;
  int64_t e = vlane;
  int slot = 0;
  if constexpr (EA) {
    if (vlane >= (int64_t)ea.nslots * E) return;
    const int k = (int)(vlane / E);
    e = vlane - (int64_t)k * E;
    slot = (ea.slot0 + k) % c.ea_S;
  } else if (vlane >= E) {
    return;
  }
  const int cap = EA ? (int)c.ea_cap : c.order_cap;
  const PtrsConst* pto = reinterpret_cast<const PtrsConst*>(c.ptrs_o);
  const PtrsConst* ptq = reinterpret_cast<const PtrsConst*>(c.ptrs_q);
  PcgCounted g{};
  int n = 0, t_begin = 0, t_end = 1;
  uint32_t p0 = 0;
  if constexpr (EA) {
    const int64_t k = vlane / E;
    t_begin = ea.t0;
    t_end = ea.t1;
    uint32_t root;
    if (ea.t0 > 0) {
      p0 = s.ea_pos[((int64_t)slot * c.T + (ea.t0 - 1)) * E + e];
      n = s.ea_off[((int64_t)slot * (c.T + 1) + ea.t0) * E + e];
      const uint32_t w2[2] = {s.orig_root[e], (uint32_t)(s.ea_cnt[(int64_t)slot * E + e] - 1)};
      root = ss_u32(w2, 2);
    } else {
      int cnt_new = 0;
      root = ea_root(c, s, ea, e, (int)k, slot, cnt_new);
      s.ea_cnt[(int64_t)slot * E + e] = cnt_new;
      s.ea_off[(int64_t)slot * (c.T + 1) * E + e] = 0;
    }
    pcg_seed_child(g.r, root, 2);  // 'demand_sampler' child of the episode's root (seed_manager.py:100-120)
    if (p0) pcg_advance(g.r, (uint64_t)p0);
  } else {
    g.r = load_rng(s, 0, e, E);
    store_rng_pre(s, e, E, g.r);
  }
  const double* enlam_o = c.enlam_o;
  const double* enlam_q = c.enlam_q;
  const double* p_skip = c.p_skip;
  for (int t = t_begin; t < t_end; t++) {
    for (int reg = 0; reg < c.R; reg++) {
      const int64_t no = poisson_any_g(g, enlam_o[reg], pto[reg]);
      for (int64_t o = 0; o < no; o++) {
        unsigned mask = 0;
#pragma unroll
        for (int k = 0; k < K; k++) mask |= g.next_double() > p_skip[reg] ? 0u : (1u << k);  // U < p
        union {
          uint4 v[NV];
          uint16_t h[8 * NV];
        } u;
#pragma unroll
        for (int j = 0; j < 8 * NV; j++) u.h[j] = 0;
        u.h[0] = (uint16_t)reg;
#pragma unroll
        for (int k = 0; k < K; k++) {
          if (mask & (1u << k)) {
            const int64_t q = poisson_any_g(g, enlam_q[reg * K + k], ptq[reg * K + k]);
            u.h[1 + k] = (uint16_t)(q > 1 ? q : 1);
          }
        }
        n++;
        if (n <= cap) {
#pragma unroll
          for (int j = 0; j < NV; j++) {
            if constexpr (EA)
              s.ea_rec[(((int64_t)slot * E + e) * c.ea_cap + (n - 1)) * NV + j] = u.v[j];
            else
              s.orders[((int64_t)(n - 1) * NV + j) * E + e] = u.v[j];
          }
        }
      }
    }
    if constexpr (EA) {
      s.ea_off[((int64_t)slot * (c.T + 1) + (t + 1)) * E + e] = n;
      s.ea_pos[((int64_t)slot * c.T + t) * E + e] = p0 + g.n;
    }
  }
  if (n > cap) {
    atomicOr(s.err, ERR_ORDER_OVERFLOW);
    n = cap;
  }
  if constexpr (!EA) {
    store_rng(s, 0, e, E, g.r);
    s.n_orders[e] = n;
  }
}

template <int K>
static void launch_seq_k(const EnvConst& c, const DevEnv* d, hipStream_t st, const EaLaunch* ea) {
  if (ea)
    hipLaunchKernelGGL((demand_seq_kernel<K, true>), dim3((unsigned)(((int64_t)ea->nslots * c.E + BS - 1) / BS)), dim3(BS),
                       0, st, d, *ea);
  else
    hipLaunchKernelGGL((demand_seq_kernel<K, false>), dim3((unsigned)((c.E + BS - 1) / BS)), dim3(BS), 0, st, d,
                       EaLaunch{0, 0, 0, 0, 0, 0, 0});
}

hipError_t launch_demand_seq(const EnvConst& c, const DevEnv* d, hipStream_t st, const EaLaunch* ea) {
  switch (c.K) {
    case 1: launch_seq_k<1>(c, d, st, ea); break;
    case 2: launch_seq_k<2>(c, d, st, ea); break;
    case 3: launch_seq_k<3>(c, d, st, ea); break;
    case 4: launch_seq_k<4>(c, d, st, ea); break;
    case 5: launch_seq_k<5>(c, d, st, ea); break;
    case 6: launch_seq_k<6>(c, d, st, ea); break;
    case 7: launch_seq_k<7>(c, d, st, ea); break;
    case 8: launch_seq_k<8>(c, d, st, ea); break;
    case 9: launch_seq_k<9>(c, d, st, ea); break;
    case 10: launch_seq_k<10>(c, d, st, ea); break;
    case 11: launch_seq_k<11>(c, d, st, ea); break;
    case 12: launch_seq_k<12>(c, d, st, ea); break;
    case 13: launch_seq_k<13>(c, d, st, ea); break;
    case 14: launch_seq_k<14>(c, d, st, ea); break;
    case 15: launch_seq_k<15>(c, d, st, ea); break;
    case 16: launch_seq_k<16>(c, d, st, ea); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// Generator.poisson known answers on the device (msc_poisson_draws): one lane draws n variates with
// the rates ptrs[i % n_lam] (PtrsConst + exp(-lam) per rate) from the PCG64 state[6]
// {s_hi, s_lo, i_hi, i_lo, has32, u32} and writes the state back.
__global__ void poisson_draws_kernel(uint64_t* state, const PtrsConst* ptrs, const double* enlam, int64_t n_lam,
                                     int64_t n, int64_t* out) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  Pcg64 r;
  r.s_hi = state[0];
  r.s_lo = state[1];
  r.i_hi = state[2];
  r.i_lo = state[3];
  r.has32 = (uint32_t)state[4];
  r.u32 = (uint32_t)state[5];
  PcgRef g{r};
  for (int64_t i = 0; i < n; i++) out[i] = poisson_any_g(g, enlam[i % n_lam], ptrs[i % n_lam]);
  state[0] = r.s_hi;
  state[1] = r.s_lo;
  state[2] = r.i_hi;
  state[3] = r.i_lo;
  state[4] = r.has32;
  state[5] = r.u32;
}

hipError_t launch_poisson_draws(uint64_t* state, const PtrsConst* ptrs, const double* enlam, int64_t n_lam, int64_t n,
                                int64_t* out, hipStream_t st) {
  hipLaunchKernelGGL(poisson_draws_kernel, dim3(1), dim3(64), 0, st, state, ptrs, enlam, n_lam, n, out);
  return hipGetLastError();
}

template <int K, int G>
static void launch_ab_k(const EnvConst& c, const DevEnv* d, hipStream_t st, const EaLaunch* ea) {
  if (ea) {
    hipLaunchKernelGGL((demand_ab_kernel<K, G, true>), dim3((unsigned)(((int64_t)ea->nslots * c.E + c.epw_dem - 1) / c.epw_dem)),
                       dim3(BS * (2 + G)), ab_lds_fixed(), st, d, *ea);
  } else {
    hipLaunchKernelGGL((demand_ab_kernel<K, G, false>), dim3((unsigned)((c.E + c.epw_dem - 1) / c.epw_dem)),
                       dim3(BS * (2 + G)), ab_lds_fixed(), st, d, EaLaunch{0, 0, 0, 0, 0, 0, 0});
  }
}

#ifdef MSC_PROF
extern "C" int msc_debug_prof_ab(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_prof_ab), sizeof(unsigned long long) * 16) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_prof_ab), z, sizeof z) != hipSuccess) return -1;
  }
  return 0;
}
#endif

bool demand_ab_supported(const EnvConst& c) { return c.demand_uni != 0 && c.K >= 1 && c.K <= UD && c.K <= 8; }

size_t demand_ab_lds_bytes() { return ab_lds_fixed(); }

hipError_t launch_demand_ab(const EnvConst& c, const DevEnv* d, hipStream_t st, const EaLaunch* ea) {
  switch (c.K) {
    case 1: launch_ab_k<1, 3>(c, d, st, ea); break;
    case 2: launch_ab_k<2, 3>(c, d, st, ea); break;
    case 3: launch_ab_k<3, 3>(c, d, st, ea); break;
    case 4: launch_ab_k<4, 3>(c, d, st, ea); break;
    case 5: launch_ab_k<5, 3>(c, d, st, ea); break;
    case 6: launch_ab_k<6, 3>(c, d, st, ea); break;
    case 7: launch_ab_k<7, 3>(c, d, st, ea); break;
    case 8: launch_ab_k<8, 3>(c, d, st, ea); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace msc
