// demand_v3.hip -- PoissonDemandSampler.sample (demand_sampler.py:105-163) for equal sampler
// parameters in every region and SKU (the scalar `params` form, demand_sampler.py:99-102, and every
// BASELINE config): demand_unit_kernel<UNI> (env_kernels.hip) with a shorter parser round.
//
// The unit parser's round (one unit of up to UD = 8 draws per lane) is the
// per-env critical path of the C3 step: ~1,490 dependent rounds per launch at a lone wave's issue
// cadence, so every instruction of the round costs ~0.7 % of the kernel. This form keeps its
// arithmetic (numpy's f64 chain, bit-exact) and its generators, ring and barriers, and trims the
// bookkeeping the round executes:
//  * the unit kind as three 0/1 flags (quantity, mask, order count) instead of a state enum compared
//    in every settle;
//  * the chain threshold chosen between exp(-lambda_o) and exp(-lambda_q) only (two selects, both
//    held in VGPRs); the SKU draws compare against p_skip in scalar registers (carrying the SKU draw
//    in the sign bit of the ring entry shortens the round by 15 instructions but costs the generators
//    a compare and its hazard wait per draw: the kernel got slower, 0.758 -> 0.784 ms,
//    profiles/r06/ab_demand_v3.txt -- the generators, not only the parser, set its pace);
//  * record addresses from a clamped record index by one 64-bit multiply-add at each store, so
//    neither store tests the capacity (an overflowing env rewrites its last record and raises the
//    error flag, as before);
//  * the generators' high word converted by one v_cvt_f64_u32 (laundered: the optimizer otherwise
//    widens it into a 64-bit conversion with an add).
#include <hip/hip_runtime.h>

#include "demand_common.hpp"

namespace msc {

#ifdef MSC_PROF
__device__ unsigned long long g_prof_v3[8];  // [0] parser rounds, [2] parser waves
#endif

template <int K, int G, bool EA>
__global__ __launch_bounds__(BS * (1 + G)) __attribute__((amdgpu_waves_per_eu(MSC_DEM_WPE))) void demand_v3_kernel(
    const DevEnv* __restrict__ dp, EaLaunch ea) {
  const EnvConst& c = dp->c;
  const EnvState& s = dp->s;
  constexpr int NV = Rec<K>::NV;
  extern __shared__ __attribute__((aligned(16))) double v3lds[];
  __shared__ int more[2];
  double* ring = v3lds;                                               // [USLOTS][BS]
  int32_t* rdv = reinterpret_cast<int32_t*>(v3lds + BS * USLOTS);    // [2][BS]
  const int wave = (int)(threadIdx.x / BS), lane = (int)(threadIdx.x % BS);  // wave 0 parses
  const int64_t E = c.E;
  const int64_t vlane = (int64_t)blockIdx.x * BS + lane;
  int64_t e = vlane;
  int slot = 0, ea_k = 0;
  bool valid = vlane < E;
  if constexpr (EA) {
    valid = vlane < (int64_t)ea.nslots * E;
    ea_k = valid ? (int)(vlane / E) : 0;
    e = valid ? vlane - (int64_t)ea_k * E : 0;
    slot = (ea.slot0 + ea_k) % c.ea_S;
  }
  double* myring = ring + lane;
  int ea_cnt_new = 0;
  uint32_t ea_p0 = 0;  // EA chunk [t0, t1): stream position and record count where step t0 starts
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
    // ---------------- generator g: stream positions g, g + G, g + 2G, ... (demand_unit_kernel's)
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
        // numpy random(): (x >> 11) 2^-53 of the XSL-RR output x, as the top 32 bits 2^-32 plus the
        // next 21 bits 2^-53 (one exact fma, pcg_output_double)
        const uint64_t x = pcg_output(th, tl);
        const double hi = (double)(uint32_t)vsettle((int)(uint32_t)(x >> 32));
        const double u = fma(hi, 0x1p-32, (double)((uint32_t)x >> 11) * 0x1p-53);
        const int sl = pg & (UCAP - 1);
        myring[sl * BS] = u;
        myring[(sl < UD - 1 ? sl + UCAP : USLOTS - 1) * BS] = u;  // mirror (or the dummy row)
        lcg128(th, tl, mh, ml, ch, cl);
        pg += G;
      }
    };
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

  // ---------------- parser (priority above the generators: it is the per-env critical path)
  __builtin_amdgcn_s_setprio(MSC_PARSER_PRIO);
  Pcg64 r0{};
  if (valid) {
    r0 = start_rng();
    if constexpr (!EA) store_rng_pre(s, e, E, r0);
  }
  rdv[lane] = 0;
  static_assert(K <= UD, "a mask unit completes in one round");
  // unit kind: qf (an SKU quantity), mf (an order's SKU mask), of (a region's order count); none: done
  int qf = 0, mf = 0, of = valid ? 1 : 0, live = of;
  int r = 0, x = 0, left = 0, sq = 0, n = ea_n0, rd = 0, pend = 0;
  int tstep = EA ? ea.t0 : 0;
  unsigned mask = 0;
  const int cap = EA ? (int)c.ea_cap : c.order_cap;
  const int64_t vstride = EA ? 16 : E * 16;       // bytes between the uint4 words of a record
  const int64_t rstride = (int64_t)NV * vstride;  // bytes between consecutive records of a lane
  MSC_GLOBAL char* const recb = reinterpret_cast<MSC_GLOBAL char*>(
      gp(EA ? s.ea_rec + ((int64_t)slot * E + e) * c.ea_cap * NV : s.orders + e));
  decltype(s.ea_off) ea_offp = EA ? s.ea_off + (int64_t)slot * (c.T + 1) * E + e : nullptr;
  decltype(s.ea_pos) ea_posp = EA ? s.ea_pos + (int64_t)slot * c.T * E + e : nullptr;
  const int T_s = __builtin_amdgcn_readfirstlane(EA ? ea.t1 : c.T);
  __syncthreads();
  if constexpr (EA) {
    if (valid && ea.t0 == 0) {
      s.ea_cnt[(int64_t)slot * E + e] = ea_cnt_new;
      ea_offp[0] = 0;
    }
  }
  // (scalar loads of the descriptor, consumed before the loop: a vector load here would leave its
  // wait, vmcnt(0), inside the loop, where it also waits for every record store in flight)
  // (the two chain thresholds held in VGPRs: the per-round select would otherwise copy them from
  // scalar registers every settle)
  double thr_o = sgpr_d(c.uni_thr_o), thr_q = sgpr_d(c.uni_thr_q);
  asm volatile("" : "+v"(thr_o), "+v"(thr_q));
  const double thr_m = sgpr_d(c.uni_thr_m);
  const int R_s = __builtin_amdgcn_readfirstlane(c.R), cap_s = __builtin_amdgcn_readfirstlane(cap);
  const uint32_t rs32 = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)rstride);  // (< 2^32: E * 16 * NV)
  // the current record: index min(n, cap) - 1 (clamped: an overflow rewrites the last record)
  auto rec_at = [&](int idx) -> MSC_GLOBAL char* { return recb + (int64_t)((uint64_t)(uint32_t)idx * rs32); };
  int ridx = (n < cap_s ? n : cap_s) - 1;
  double thr = thr_o, prod = 1.0;
  // a unit ended: book its result, open the next unit (straight-line, predicated; the two record
  // stores are guarded)
  auto settle = [&]() {
    if (qf) {
      const int h = 1 + sq;  // 16-bit field of the record (field 0 = region)
      MSC_GLOBAL char* fp = NV == 1 ? rec_at(ridx) + h * 2 : rec_at(ridx) + (int64_t)(h >> 3) * vstride + (h & 7) * 2;
      *reinterpret_cast<MSC_GLOBAL uint16_t*>(fp) = (uint16_t)(x > 1 ? x : 1);  // max(1, Poisson(lambda_q))
    }
    const unsigned m2 = qf ? (mask & (mask - 1u)) : mask;  // a mask unit left its bits in mask
    const int has_q = (of ^ 1) & (m2 != 0u ? 1 : 0);
    const int left2 = (of ? x : left) - ((of | has_q) ^ 1);  // an order completed
    const int new_order = (has_q ^ 1) & (left2 > 0 ? 1 : 0);
    const int new_region = (has_q | new_order) ^ 1;
    int wrap = 0;  // EA: the step's last region ended and another step of the episode follows
    if constexpr (EA) {
      if (new_region & (r + 1 == R_s ? 1 : 0)) {
        ea_offp[(int64_t)(tstep + 1) * E] = n;
        ea_posp[(int64_t)tstep * E] = ea_p0 + (uint32_t)rd;
        wrap = tstep + 1 < T_s ? 1 : 0;
        tstep += wrap;
      }
    }
    sq = __builtin_ctz(m2 | (1u << K));
    qf = has_q;
    mf = new_order;
    of = new_region & ((r + 1 < R_s ? 1 : 0) | wrap);
    live = qf | mf | of;
    thr = has_q ? thr_q : thr_o;  // (a mask unit's draws compare against thr_m)
    mask = new_order ? 0u : m2;
    left = left2;
    n += new_order;
    ridx = (n < cap_s ? n : cap_s) - 1;
    if (new_order) {
      MSC_GLOBAL char* rp = rec_at(ridx);
#pragma unroll
      for (int j = 0; j < NV; j++)
        *reinterpret_cast<MSC_GLOBAL v4u*>(rp + (int64_t)j * vstride) = v4u{j == 0 ? (unsigned)r : 0u, 0u, 0u, 0u};
    }
    r = wrap ? 0 : r + new_region;
    prod = 1.0;
    x = 0;
  };
#ifdef MSC_PROF
  unsigned long long n_round = 0;
#endif
  int ptgt = UCAP, rd_start = 0;  // the generators' fill target and the chunk's start position
  for (int ci = 0;; ci++) {
#pragma unroll 1
    for (int hs = 0; hs < UHS; hs++) {
      // issue this round's ring reads first, then book the unit that ended last round while they
      // are in flight
      const double* rp = myring + (rd & (UCAP - 1)) * BS;
      double u[UD];
#pragma unroll
      for (int i = 0; i < UD; i++) u[i] = rp[i * BS];
      if (pend) settle();
      // Poisson unit: p_i = p_{i-1} U_i in draw order (bit-exact with numpy); U_i < 1 makes the
      // products non-increasing, so "p_i > exp(-lambda)" holds for a leading run and its length is a
      // plain count. Mask unit: bit i = SKU drawn <=> U_i < p <=> !(U_i > p_skip).
      double p = prod;
      int ncont = 0;
      unsigned bits = 0;
#pragma unroll
      for (int i = 0; i < UD; i++) {
        p = p * u[i];
        ncont += p > thr ? 1 : 0;
        if (i < K) bits |= u[i] > thr_m ? 0u : (1u << i);
      }
      const int go = ncont >= UD ? 1 : 0;  // Poisson unit still running after UD draws
      const int cons = mf ? K : (go ? UD : ncont + 1);
      mask = mf ? bits : mask;
      x += ncont;  // (a mask unit's x is unused and cleared by its settle)
      prod = p;
      rd += live ? cons : 0;
      pend = live & (mf | (go ^ 1));
#ifdef MSC_PROF
      n_round++;
#endif
    }
    // a lane with a booked-but-unsettled unit is still live: it settles in the next round
    const bool any = __ballot(live) != 0;
    rdv[((ci + 1) & 1) * BS + lane] = rd;
    if (lane == 0) more[ci & 1] = any ? 1 : 0;
    __syncthreads();
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
#ifdef MSC_PROF
  if (lane == 0) {
    atomicAdd(&g_prof_v3[0], n_round);
    atomicAdd(&g_prof_v3[2], 1ull);
  }
#endif
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

bool demand_v3_supported(const EnvConst& c) {
  // (record strides NV * E * 16 bytes below 2^32: the address multiply-add is 32 x 32 bits)
  return c.demand_uni != 0 && c.demand_ptrs == 0 && c.K >= 1 && c.K <= UD && c.K <= 8 && c.epw_dem == BS &&
         (uint64_t)c.E * 32u < (1ull << 32);
}

// the alternative Poisson demand kernels selected by c.demand_impl (8: demand_v2.hip, 9: this file);
// hipErrorNotSupported when the handle's sampler has no such form (the caller runs the unit parser)
hipError_t launch_demand_alt(const EnvConst& c, const DevEnv* d, hipStream_t st, const EaLaunch* ea) {
  if (c.demand_impl == 9 && demand_v3_supported(c)) return launch_demand_v3(c, d, st, ea);
  if (c.demand_impl == 8 && demand_v2_supported(c)) return launch_demand_v2(c, d, st, ea);
  return hipErrorNotSupported;
}

template <int K>
static void launch_v3_k(const EnvConst& c, const DevEnv* d, hipStream_t st, const EaLaunch* ea) {
  constexpr int G = 3;
  if (ea) {
    hipLaunchKernelGGL((demand_v3_kernel<K, G, true>), dim3((unsigned)(((int64_t)ea->nslots * c.E + BS - 1) / BS)),
                       dim3(BS * (1 + G)), unit_lds_fixed(), st, d, *ea);
  } else {
    hipLaunchKernelGGL((demand_v3_kernel<K, G, false>), dim3((unsigned)((c.E + BS - 1) / BS)), dim3(BS * (1 + G)),
                       unit_lds_fixed(), st, d, EaLaunch{0, 0, 0, 0, 0, 0, 0});
  }
}

hipError_t launch_demand_v3(const EnvConst& c, const DevEnv* d, hipStream_t st, const EaLaunch* ea) {
  switch (c.K) {
    case 1: launch_v3_k<1>(c, d, st, ea); break;
    case 2: launch_v3_k<2>(c, d, st, ea); break;
    case 3: launch_v3_k<3>(c, d, st, ea); break;
    case 4: launch_v3_k<4>(c, d, st, ea); break;
    case 5: launch_v3_k<5>(c, d, st, ea); break;
    case 6: launch_v3_k<6>(c, d, st, ea); break;
    case 7: launch_v3_k<7>(c, d, st, ea); break;
    case 8: launch_v3_k<8>(c, d, st, ea); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

#ifdef MSC_PROF
extern "C" int msc_debug_prof_v3(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_prof_v3), sizeof(unsigned long long) * 8) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[8] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_prof_v3), z, sizeof z) != hipSuccess) return -1;
  }
  return 0;
}
#endif

}  // namespace msc
