// demand_v2.hip -- PoissonDemandSampler.sample (demand_sampler.py:105-163) for equal sampler
// parameters in every region and SKU (the scalar `params` form, demand_sampler.py:99-102, and every
// BASELINE config) with a 4-byte ring: the round-6 production kernel at <= 8 SKUs.
//
// demand_unit_kernel<UNI> (env_kernels.hip) keeps numpy's random() doubles in an LDS ring of 64
// positions per env, [slot][lane], filled by three generator waves and read by one parser wave per
// 64 envs. Two of its costs come from the 8-byte entries:
//  * the ring is 64 positions deep (37 KB per block: two blocks per CU beside two allocation blocks).
//    The generators refill every lane by a fixed quota per chunk, so a generator wave loops for the
//    quota while lanes whose ring is full are masked off: ~1.34x the draws the parser consumes;
//  * the parser's chained products and compares are f64 (two issue cycles of a 32-bit op each).
// Here every ring entry is one f32: the draw's value rounded to f32, |f| = fl32(U), and its sign bit
// = the Bernoulli SKU draw (U < p, decided exactly on the 53-bit integer: U = k 2^-53 < p <=>
// k < ceil(p 2^53)). 128 positions fit the same 35 KB, the quota can sit near the mean consumption,
// and the parser runs the Poisson chain p_i = p_{i-1} |f_i| in f32.
//
// Exactness. numpy decides `prod > exp(-lam)` on the f64 chain P~ (one rounding per product). The
// f32 chain p of n draws satisfies |p / P - 1| <= n (2^-23 + 2^-24) (each |f| within 2^-23 of U,
// each f32 product rounded once; P the exact real product) and |P~ / P - 1| <= n 2^-53. With the
// host's thresholds hi >= exp(-lam) (1 + 2^-16) and lo <= exp(-lam) (1 - 2^-16) (rounded outward):
// p > hi proves "continue", p <= lo proves "end" for any unit of n <= 32 draws (n 1.8e-7 < 1.5e-5).
// A lane whose round holds a product in (lo, hi], or whose unit reaches 24 draws, recomputes the
// unit exactly: the PCG64 state of the unit's first draw by jump-ahead from the launch's start state,
// then numpy's f64 chain draw by draw. Per comparison that band has probability ~1.5e-6 (about one
// exact recomputation per 64-env wave every two steps at 8 x 64 x 5).
//
// Everything else -- unit-per-round parse, straight-line settle, chunk barriers, the generators'
// stream positions, the record format, the episode-ahead (EA) plumbing -- is demand_unit_kernel's.
#include <hip/hip_runtime.h>

#include "demand_common.hpp"

namespace msc {

#ifndef MSC_V2_UCAP
#define MSC_V2_UCAP 128
#endif
constexpr int V2_UCAP = MSC_V2_UCAP;          // ring capacity (positions)
constexpr int V2_ROWS = V2_UCAP + UD;         // + the UD - 1 mirrored rows + a dummy row
static_assert((V2_UCAP & (V2_UCAP - 1)) == 0 && V2_UCAP >= 2 * UD * UHS, "ring layout");
constexpr int V2_INIT = 2 * UD * UHS;      // positions drawn before the parser starts (two chunks)
constexpr int V2_LONG = 24;                   // a unit of >= this many continues is decided exactly
#ifndef MSC_V2_WPE
// <= 80 VGPRs: within 64 the exact recomputation's registers pushed the parser's chunk-loop values
// into scratch, and the reload's vmcnt(0) after every chunk also waited for all record stores in
// flight (+30 % per launch); two demand waves per SIMD still leave room for the allocation's waves
#define MSC_V2_WPE 6
#endif

__host__ __device__ constexpr size_t v2_lds_bytes() {
  return (size_t)BS * V2_ROWS * sizeof(float) + (size_t)2 * BS * sizeof(int32_t);
}

#ifdef MSC_PROF
// [0] parser rounds, [1] exact recomputations (lanes), [2] parser waves
__device__ unsigned long long g_prof_v2[8];
#endif

// the generators' fill target for the next phase: quota more positions, capped by the ring slots the
// parser's current chunk (starting at rdp) cannot read
__device__ __forceinline__ int v2_quota_target(int tgt, int rdp, int quota) {
  const int q = tgt + quota, cap = rdp + V2_UCAP;
  return q < cap ? q : cap;
}

template <int K, int G, bool EA>
__global__ __launch_bounds__(BS * (1 + G)) __attribute__((amdgpu_waves_per_eu(MSC_V2_WPE))) void demand_v2_kernel(
    const DevEnv* __restrict__ dp, EaLaunch ea) {
  const EnvConst& c = dp->c;
  const EnvState& s = dp->s;
  const int R = c.R;
  constexpr int NV = Rec<K>::NV;
  extern __shared__ __attribute__((aligned(16))) float v2lds[];
  __shared__ int more[2];
  float* ring = v2lds;                                                // [V2_ROWS][BS]
  int32_t* rdv = reinterpret_cast<int32_t*>(v2lds + BS * V2_ROWS);   // [2][BS]
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
  float* myring = ring + lane;
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
  const int quota = __builtin_amdgcn_readfirstlane(c.v2_quota);

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
    // (readfirstlane returns int: each half goes through uint32_t, or the low word would sign-extend)
    const uint32_t k53_hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(c.v2_k53 >> 32));
    const uint32_t k53_lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)c.v2_k53);
    const uint64_t k53 = ((uint64_t)k53_hi << 32) | k53_lo;
    int pg = g;
    auto gen_to = [&](int target) {
      while (pg < target) {
        // numpy random(): U = (x >> 11) 2^-53 of the XSL-RR output x. |f| = fl32(U) from the two
        // halves (the high word rounded to f32, the next 21 bits exact, one fma: within 2^-23 of U);
        // sign = the Bernoulli SKU draw U < p, exact on the 53-bit integer
        const uint64_t x = pcg_output(th, tl);
        // (the high word laundered: the optimizer would otherwise convert x >> 32 as a 64-bit integer,
        // a normalise-and-ldexp sequence instead of one v_cvt_f32_u32)
        const float hi = (float)(uint32_t)vsettle((int)(uint32_t)(x >> 32)), lo = (float)((uint32_t)x >> 11);
        const float f = fmaf(hi, 0x1p21f, lo) * 0x1p-53f;
        const float v = (x >> 11) < k53 ? -f : f;
        const int sl = pg & (V2_UCAP - 1);
        myring[sl * BS] = v;
        myring[(sl < UD - 1 ? sl + V2_UCAP : V2_ROWS - 1) * BS] = v;  // mirror (or the dummy row)
        lcg128(th, tl, mh, ml, ch, cl);
        pg += G;
      }
    };
    int tgt = V2_INIT;
    if (valid) gen_to(V2_INIT);
    __syncthreads();
    for (int ci = 0;; ci++) {
      const int rdp = rdv[(ci & 1) * BS + lane];
      tgt = v2_quota_target(tgt, rdp, quota);
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
  int st = valid ? PS_ORD : PS_DONE, r = 0, x = 0, left = 0, sq = 0, n = ea_n0, rd = 0, us = 0;
  int tstep = EA ? ea.t0 : 0;
  unsigned mask = 0;
  int mf = 0, live = valid ? 1 : 0, pend = 0;
  const int cap = EA ? (int)c.ea_cap : c.order_cap;
  const int64_t vstride = EA ? 16 : E * 16;       // bytes between the uint4 words of a record
  const int64_t rstride = (int64_t)NV * vstride;  // bytes between consecutive records of a lane
  MSC_GLOBAL char* recp = reinterpret_cast<MSC_GLOBAL char*>(
      gp(EA ? s.ea_rec + ((int64_t)slot * E + e) * c.ea_cap * NV : s.orders + e)) + (int64_t)(n - 1) * rstride;
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
  const float o_hi = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, c.v2_thr[0])));
  const float o_lo = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, c.v2_thr[1])));
  const float q_hi = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, c.v2_thr[2])));
  const float q_lo = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, c.v2_thr[3])));
  const double en_o = sgpr_d(c.uni_thr_o), en_q = sgpr_d(c.uni_thr_q);
  const int R_s = __builtin_amdgcn_readfirstlane(R), cap_s = __builtin_amdgcn_readfirstlane(cap);
  const int64_t rstride_s = (int64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)rstride) |
                            ((int64_t)__builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)rstride >> 32)) << 32);
  float thi = o_hi, tlo = o_lo, prod = 1.0f;
  // a unit ended: book its result, open the next unit (straight-line, predicated; only the two
  // record stores are guarded)
  auto settle = [&]() {
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
    thi = has_q ? q_hi : o_hi;  // (a mask unit ignores them)
    tlo = has_q ? q_lo : o_lo;
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
    prod = 1.0f;
    x = 0;
    us = rd;
    mf = st == PS_MASK ? 1 : 0;
    live = st != PS_DONE ? 1 : 0;
  };
#ifdef MSC_PROF
  unsigned long long n_round = 0, n_exact = 0;
#endif
  int ptgt = V2_INIT, rd_start = 0;  // the generators' fill target and the chunk's start position
  for (int ci = 0;; ci++) {
#pragma unroll 1
    for (int hs = 0; hs < UHS; hs++) {
      // issue this round's ring reads first, then book the unit that ended last round while they
      // are in flight
      const float* rp = myring + (rd & (V2_UCAP - 1)) * BS;
      float u[UD];
#pragma unroll
      for (int i = 0; i < UD; i++) u[i] = rp[i * BS];
      if (pend) settle();
      // Poisson unit: p_i = p_{i-1} |f_i|, non-increasing, so "p_i > lo" holds for a leading run and
      // its length is a plain count; a product in (lo, hi] leaves the round undecided (exact path).
      // Mask unit: bit i = the sign of f_i.
      float p = prod;
      int ncont = 0;
      unsigned bits = 0;
      bool band = false;
#pragma unroll
      for (int i = 0; i < UD; i++) {
        p = p * fabsf(u[i]);
        const bool cl = p > tlo;
        ncont += cl ? 1 : 0;
        band |= cl & !(p > thi);
        if (i < K) bits |= (__float_as_uint(u[i]) >> 31) << i;
      }
      // undecided: a product in the band, or a unit long enough that the f32 bound no longer holds
      const bool exact = live && !mf && (band || x >= V2_LONG);
      if (__ballot(exact) != 0) {
        if (exact) {
          // numpy's chain of this unit from its first draw (position us) through this round's
          // window: the state of position j is step^(j + 1) of the launch's start state
          Pcg64 q = r0;
          pcg_advance(q, (uint64_t)us + 1u);
          const double en = st == PS_ORD ? en_o : en_q;
          double P = 1.0;
          int j = us;
          bool ended = false;
          for (; j < rd + UD; j++) {
            P *= pcg_output_double(q.s_hi, q.s_lo);
            if (!(P > en)) {
              ended = true;
              break;
            }
            lcg128(q.s_hi, q.s_lo, PCG_MUL_HI, PCG_MUL_LO, q.i_hi, q.i_lo);
          }
          ncont = ended ? (j > rd ? j - rd : 0) : UD;  // (j >= rd: the earlier rounds were decided)
          p = (float)P;
#ifdef MSC_PROF
          n_exact++;
#endif
        }
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
    ptgt = v2_quota_target(ptgt, rd_start, quota);
    const int need = rd + UHS * UD;
    if (__ballot(valid && ptgt < need) != 0) {
      ptgt = ptgt > need ? ptgt : need;
      __syncthreads();
    }
    rd_start = rd;
  }
#ifdef MSC_PROF
  if (lane == 0) {
    atomicAdd(&g_prof_v2[0], n_round);
    atomicAdd(&g_prof_v2[2], 1ull);
  }
  atomicAdd(&g_prof_v2[1], n_exact);
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

#ifdef MSC_PROF
extern "C" int msc_debug_prof_v2(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_prof_v2), sizeof(unsigned long long) * 8) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[8] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_prof_v2), z, sizeof z) != hipSuccess) return -1;
  }
  return 0;
}
#endif

bool demand_v2_supported(const EnvConst& c) {
  return c.demand_uni != 0 && c.demand_ptrs == 0 && c.K >= 1 && c.K <= UD && c.K <= 8 && c.epw_dem == BS &&
         c.v2_quota > 0;
}

size_t demand_v2_lds_bytes() { return v2_lds_bytes(); }

template <int K>
static void launch_v2_k(const EnvConst& c, const DevEnv* d, hipStream_t st, const EaLaunch* ea) {
  constexpr int G = 3;
  if (ea) {
    hipLaunchKernelGGL((demand_v2_kernel<K, G, true>), dim3((unsigned)(((int64_t)ea->nslots * c.E + BS - 1) / BS)),
                       dim3(BS * (1 + G)), v2_lds_bytes(), st, d, *ea);
  } else {
    hipLaunchKernelGGL((demand_v2_kernel<K, G, false>), dim3((unsigned)((c.E + BS - 1) / BS)), dim3(BS * (1 + G)),
                       v2_lds_bytes(), st, d, EaLaunch{0, 0, 0, 0, 0, 0, 0});
  }
}

hipError_t launch_demand_v2(const EnvConst& c, const DevEnv* d, hipStream_t st, const EaLaunch* ea) {
  switch (c.K) {
    case 1: launch_v2_k<1>(c, d, st, ea); break;
    case 2: launch_v2_k<2>(c, d, st, ea); break;
    case 3: launch_v2_k<3>(c, d, st, ea); break;
    case 4: launch_v2_k<4>(c, d, st, ea); break;
    case 5: launch_v2_k<5>(c, d, st, ea); break;
    case 6: launch_v2_k<6>(c, d, st, ea); break;
    case 7: launch_v2_k<7>(c, d, st, ea); break;
    case 8: launch_v2_k<8>(c, d, st, ea); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace msc
