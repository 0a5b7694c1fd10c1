// alloc_kernels.hip -- phase B of InventoryEnvironment.step with one env per lane: the greedy
// allocation (GreedyDemandAllocator.allocate, demand_allocator.py:118-217), the inventory update
// (multi_env.py:307), the lost-sales handlers (lost_sales_handler.py:71-210) folded into the
// penalty cost, the outbound cost (reward_calculator.py:143-150) and the home-region features of
// _update_observations (multi_env.py:767-773).
//
// Thread mapping: lane = env, 64 envs per wave, one wave per block. The reference walks each
// env's order list sequentially (an order's ranking and fills depend on the inventory the previous
// order left), so every env is one dependent chain; giving each chain one lane (instead of one
// lane per warehouse) makes the per-order bookkeeping (record unpack, ranking weight, unfulfilled
// demand, region epilogue) one instruction for 64 envs instead of one per 8, i.e. ~10x fewer
// wave-instructions per order than the group-per-env step_b_kernel (kept for A/B:
// MSC_ALLOC_IMPL=group).
//
// Per lane: the current order's W ranking costs and the K-bit per-SKU stock masks (bit w of
// stock[s] <=> warehouse w holds SKU s) live in registers; everything indexed by the warehouse a
// fill lands on (inventory, shipped home, outbound cost, shipped-to-region) lives in LDS at
// [index][lane], so a lane-varying warehouse index is one conflict-free LDS access. Order records
// ([order][NV][E], env fastest: one 1-KiB coalesced load per wave per order) arrive in windows of
// AL_CH orders: the next window's loads are in flight in registers while the current one is read
// from LDS (a register FIFO rotated every order would wait on its newest load at each shift).
#include <hip/hip_runtime.h>
#include <math.h>

#include "env.hpp"
#include "kcommon.hpp"

namespace msc {

#ifndef MSC_AL_CH
#define MSC_AL_CH 8  // order records per window: window k + 1 is in flight (registers) while window k
                     // is allocated from LDS
#endif
constexpr int AL_CH = MSC_AL_CH;
template <int K>
hipError_t launch_alloc_lane_k(const EnvConst& c, const DevEnv* d, const StepIO& io, hipStream_t st);
#ifndef MSC_AL_PRIO
#define MSC_AL_PRIO 3  // s_setprio: the step chain is the critical path next to the demand waves
#endif
#ifndef MSC_AL_PRIO2
#define MSC_AL_PRIO2 1  // the priority after c.al_psplit 16ths of the orders: below the demand parser (2)
#endif

// LDS layout of one block (64 envs); word offsets
struct AlLds {
  int rec, inv, shh, qs, out, pen, tab, hm, cl, total;  // rec: uint4, out / pen: doubles, tab: double2
  // MWL: warehouses owned by one lane (MW / lanes per env); per-lane arrays are indexed by the
  // lane's local warehouse index i
  __host__ __device__ static AlLds make(int MWL, int MW, int K, int R, bool tab, bool SH) {
    AlLds L{};
    int o = 0;
    L.rec = o; o += AL_CH * ((1 + K + 7) / 8) * 64 * 4;  // [j][v][lane] order-record window
    L.inv = o; o += MWL * K * 64;   // [i*K+s][lane] inventory
    L.shh = o; o += SH ? MWL * K * 64 : 0;  // [i*K+s][lane] shipped home (only when home regions are shared)
    L.qs = o;  o += MWL * 64;       // [i][lane] units shipped by the warehouse to the current region
    o = (o + 3) & ~3;
    L.out = o; o += MWL * 64 * 2;   // [i][lane] outbound cost (f64)
    L.pen = o; o += MWL * 64 * 2;   // [i][lane] penalty cost (f64)
    L.tab = o; o += tab ? (R | 1) * MW * 4 : 0;  // [w][r] {of, ov} (f64 pairs), row stride R | 1
    L.hm = o;  o += R;             // [r] home mask
    L.cl = o;  o += R;             // [r] closest warehouse
    L.total = o;
    return L;
  }
};
// cost table in LDS up to this size (C3: 8 KiB; C5 16 x 256: 64 KiB -> read from L2 instead)
constexpr size_t AL_TAB_MAX = 32 * 1024;

// EXACT: n_warehouses == MW (compile-time W: no per-warehouse `w < W` masking).
// LPE: lanes per env (1, 2, 4). Lane j of an env owns warehouses w = i * LPE + j (i < MW / LPE):
// their ranking costs, stock bits and LDS rows. Each allocation round takes the cheapest candidate
// over the group (DPP butterfly on (cost, w), lowest w on ties), the owning lane computes the fills
// and the group ORs them (non-owners contribute 0), so every lane keeps the env's remaining demand.
// With fewer envs than lanes on the chip this multiplies the waves (C5: 8192 envs = 128 one-env-per
// -lane waves for 256 CUs) at the price of the butterfly per round.
template <int K, int MW, bool DBG, bool TAB, bool SH, bool EXACT, int LPE>
__global__ __launch_bounds__(64) void alloc_lane_kernel(const DevEnv* __restrict__ dp, StepIO io) {
  static_assert(LPE == 1 || LPE == 2 || LPE == 4, "lanes per env");
  static_assert(MW % LPE == 0, "warehouses per lane");
  constexpr int MWL = MW / LPE, EPB = 64 / LPE, LSH = LPE == 1 ? 0 : LPE == 2 ? 1 : 2;
  constexpr int SENT = 0x7fff;  // no candidate
  const EnvConst& c = dp->c;
  const EnvState& s = dp->s;
  const int W = EXACT ? MW : c.W, R = c.R, WK = W * K;
  const int64_t E = c.E;
  const int lane = threadIdx.x, jl = lane & (LPE - 1);
  const int64_t e = (int64_t)blockIdx.x * EPB + (lane >> LSH);
  const bool ev = e < E;
  const msc_step_info info = io.info;
  constexpr bool dbg = DBG;
  constexpr int NVR = Rec<K>::NV;
  if (MSC_AL_PRIO > 0) __builtin_amdgcn_s_setprio(MSC_AL_PRIO);
  auto gw = [&](int i) { return i * LPE + jl; };  // global index of local warehouse i

  extern __shared__ __attribute__((aligned(16))) int32_t al_lds[];
  const AlLds L = AlLds::make(MWL, MW, K, R, TAB, SH);
  int32_t* Linv = al_lds + L.inv + lane;
  int32_t* Lshh = al_lds + L.shh + lane;
  uint4* Lrec = reinterpret_cast<uint4*>(al_lds + L.rec) + lane;
  double* Lout = reinterpret_cast<double*>(al_lds + L.out) + lane;
  double* Lpen = reinterpret_cast<double*>(al_lds + L.pen) + lane;
  int32_t* Lqs = al_lds + L.qs + lane;
  // pointers used inside the order loop, read once (the loop stores to global memory, so fields
  // read through `s` would be re-loaded after every store)
  MSC_GLOBAL int32_t* const incp = gp(s.inc);
  const double2* Ltab = TAB ? reinterpret_cast<const double2*>(al_lds + L.tab) : nullptr;
  // table rows are warehouse-major with an odd stride (in 16-byte entries): the lanes' regions differ,
  // and with [r][w] rows (a 128-byte stride at MW 8) every even region falls on the same banks (up to
  // 8-way conflicts per 16-lane phase of the ds_read_b128); [w][r] puts consecutive regions on
  // consecutive banks, and the odd stride spreads the warehouses of one region (LPE > 1)
  const int RS = R | 1;
  const uint32_t* Lhm = reinterpret_cast<const uint32_t*>(al_lds + L.hm);
  const int32_t* Lcl = al_lds + L.cl;
  {
    double2* tw_ = reinterpret_cast<double2*>(al_lds + L.tab);
    if constexpr (TAB) {
      for (int i = lane; i < R * MW; i += 64) {
        const int w = i / R, r = i % R;
        tw_[w * RS + r] = w < W ? make_double2(c.ofT[r * W + w], c.ovT[r * W + w]) : make_double2(0.0, 0.0);
      }
    }
    uint32_t* hm_ = reinterpret_cast<uint32_t*>(al_lds + L.hm);
    int32_t* cl_ = al_lds + L.cl;
    for (int i = lane; i < R; i += 64) {
      hm_[i] = c.home_mask[i];
      cl_[i] = c.closest[i];
    }
  }
  auto tab_at = [&](int r, int w) -> double2 {
    if constexpr (TAB) return Ltab[w * RS + r];
    else return make_double2(gp(c.ofT)[r * W + w], gp(c.ovT)[r * W + w]);
  };

  // inventory after step_a's arrivals -> LDS; per-SKU stock masks (bit i: local warehouse i)
  uint32_t stock[K];
#pragma unroll
  for (int sk = 0; sk < K; sk++) stock[sk] = 0u;
  // every load issued unconditionally (clamped indices, the value masked after): a load under a
  // lane condition became a branch with its own wait, i.e. MWL * K serial round trips per launch
  int invv[MWL][K];
  {
    const int64_t ec = ev ? e : 0;
#pragma unroll
    for (int i = 0; i < MWL; i++) {
      const int w = gw(i), wc = w < W ? w : W - 1;
#pragma unroll
      for (int sk = 0; sk < K; sk++) invv[i][sk] = gp(s.inv)[(int64_t)(wc * K + sk) * E + ec];
    }
  }
#pragma unroll
  for (int i = 0; i < MWL; i++) {
    const int w = gw(i);
#pragma unroll
    for (int sk = 0; sk < K; sk++) {
      const int v = (ev && w < W) ? invv[i][sk] : 0;
      Linv[(i * K + sk) * 64] = v;
      if (SH) Lshh[(i * K + sk) * 64] = 0;
      stock[sk] |= v > 0 ? (1u << i) : 0u;
    }
    Lout[i * 64] = 0.0;
    Lpen[i * 64] = 0.0;
    Lqs[i * 64] = 0;
  }
  __syncthreads();  // tables

  // this env's order list: record (n, v) at base + n * nstep + v * vstep (uint4 units)
  const OrderSrc osrc = order_src<NVR>(c, s, io, ev ? e : 0);
  const int n_orders = ev ? osrc.n : 0;
  const int64_t base = ev ? osrc.base : 0, nstep = osrc.nstep, vstep = osrc.vstep;
  const MSC_GLOBAL uint4* src = gp(osrc.src);
  if (dbg && ev && jl == 0 && info.n_orders) info.n_orders[e] = n_orders;
  int wmax = n_orders;  // orders of the wave's busiest env
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const int v = __shfl_xor(wmax, o);
    wmax = v > wmax ? v : wmax;
  }
  wmax = __builtin_amdgcn_readfirstlane(wmax);  // (uniform: a scalar loop bound, no lane masks per order)

  const int maxwh = c.max_wh, lost_type = c.lost_type, pps = c.pen_per_sku;
  const double alpha = sgpr_d(c.alpha);
  double skw[K], penk[K];
#pragma unroll
  for (int sk = 0; sk < K; sk++) {
    skw[sk] = sgpr_d(c.skw[sk]);
    penk[sk] = sgpr_d(pps ? c.pen[sk] : c.pen_scalar);
  }

  // warehouses (global bit w) this lane owns
  const uint32_t ownw = LPE == 1 ? ~0u : (LPE == 2 ? 0x55555555u : 0x11111111u) << jl;
  int cur = -1, lost_cnt = 0;
  uint32_t hm = 0;     // warehouses whose home region is the current region (global bits)
  int hw = -1;         // the one warehouse whose home it is (!SH: every region is home to at most one)
  uint32_t smask = 0;  // own warehouses that shipped to the current region (local bits)
  int rtot = 0;        // units the env shipped to the current region
  int u[K], dsum[K], shc[K];  // shc: shipped by hw to its home region (!SH)
#pragma unroll
  for (int sk = 0; sk < K; sk++) u[sk] = dsum[sk] = shc[sk] = 0;
  // shipped home (multi_env.py:770-773) is stored when the home region ends; zero for a home region
  // without orders
  MSC_GLOBAL int32_t* const shhp = gp(s.sc_shh);
  if (!SH && ev)
    for (int i = 0; i < MWL; i++) {
      const int w = gw(i);
      if (w < W)
        for (int sk = 0; sk < K; sk++) shhp[(int64_t)(w * K + sk) * E + e] = 0;
    }

  // region epilogue (lost_sales_handler.py:71-210 into the penalty; home-region features). Only
  // nonzero shares are visited: the closest warehouse's, or those of the warehouses that shipped to
  // the region (a bit loop: most iterations end some lane's region, so this runs nearly every order)
  auto add_pen = [&](int i, double wt, double upen) {
    Lpen[i * 64] += wt * upen;
    if (dbg && info.lost_sales)
#pragma unroll
      for (int sk = 0; sk < K; sk++) info.lost_sales[e * WK + gw(i) * K + sk] += wt * (double)u[sk];
  };
  auto finalize = [&](int r) {
    if (lost_cnt > 0) {
      double upen = 0.0;
#pragma unroll
      for (int sk = 0; sk < K; sk++) upen += pps ? (double)u[sk] * penk[sk] : ((double)u[sk] * skw[sk]) * penk[sk];
      if (lost_type == MSC_LOST_COST) {  // softmax(-(of * lost_orders + ov * lost_weight) / alpha)
        if constexpr (LPE == 1) {  // (the launcher keeps LPE 1 for this handler)
          double lw = 0.0;
#pragma unroll
          for (int sk = 0; sk < K; sk++) lw += (double)u[sk] * skw[sk];
          double lg[16], mx = -INFINITY;
#pragma unroll
          for (int w = 0; w < 16; w++) {
            lg[w] = -INFINITY;
            if (w < MW && w < W) {
              const double2 t = tab_at(r, w);
              lg[w] = -(t.x * (double)lost_cnt + t.y * lw) / alpha;
              mx = lg[w] > mx ? lg[w] : mx;
            }
          }
          double ex[16];
#pragma unroll
          for (int w = 0; w < 16; w++) ex[w] = (w < MW && w < W) ? exp(lg[w] - mx) : 0.0;
          const double sum = np_sum_f64_16(ex, W);
#pragma unroll
          for (int w = 0; w < MW; w++) {
            const double wt = w < W ? ex[w] / sum : 0.0;
            if (wt != 0.0) add_pen(w, wt, upen);
          }
        }
      } else if (lost_type == MSC_LOST_SHIPMENT && rtot > 0) {
        // shares of the units shipped to the region (integer-valued: the integer sum is the f64 sum
        // exactly; x * (1 / tot) is within an ulp of x / tot)
        const double dt = (double)rtot;
        for (uint32_t m = smask; m != 0u; m &= m - 1u) {
          const int i = __builtin_ctz(m);
          add_pen(i, (double)Lqs[i * 64] / dt, upen);
        }
      } else {  // closest warehouse (also shipment with nothing shipped); 1.0 * x == x
        const int cw = Lcl[r];
        if ((cw & (LPE - 1)) == jl) add_pen(cw >> LSH, 1.0, upen);
      }
    }
    for (uint32_t m = smask; m != 0u; m &= m - 1u) Lqs[__builtin_ctz(m) * 64] = 0;
    if (!SH && hw >= 0 && (hw & (LPE - 1)) == jl)
#pragma unroll
      for (int sk = 0; sk < K; sk++) shhp[(int64_t)(hw * K + sk) * E + e] = shc[sk];
    // a home region: its demand is the incoming home demand of its warehouses (multi_env.py:767-769;
    // step_a zeroed s.inc, so a home region without orders leaves 0)
    for (uint32_t m = hm & ownw; m != 0u; m &= m - 1u) {
      const int w = __builtin_ctz(m);
#pragma unroll
      for (int sk = 0; sk < K; sk++) incp[(int64_t)(w * K + sk) * E + e] = dsum[sk];
    }
    if (dbg && jl == 0) {
#pragma unroll
      for (int sk = 0; sk < K; sk++) {
        if (info.demand_per_region) info.demand_per_region[(e * R + r) * K + sk] = dsum[sk];
        if (info.unfulfilled_demands) info.unfulfilled_demands[(e * R + r) * K + sk] = u[sk];
      }
      if (info.lost_order_counts) info.lost_order_counts[e * R + r] = lost_cnt;
    }
  };

  // order-record windows: window k in LDS, window k + 1 in flight in registers
  uint4 nxt[AL_CH][NVR];
  auto fetch = [&](int win) {
#pragma unroll
    for (int j = 0; j < AL_CH; j++) {
      const int oi = win * AL_CH + j;
#pragma unroll
      for (int v = 0; v < NVR; v++)
        nxt[j][v] = oi < n_orders ? gload4(src, base + oi * nstep + v * vstep) : make_uint4(0u, 0u, 0u, 0u);
    }
  };
  auto publish = [&]() {
#pragma unroll
    for (int j = 0; j < AL_CH; j++)
#pragma unroll
      for (int v = 0; v < NVR; v++) Lrec[(j * NVR + v) * 64] = nxt[j][v];
  };
  fetch(0);
  publish();
  fetch(1);

  // the first c.al_psplit 16ths of the orders above the next step's demand parser, the rest below it
  // (msc_env_set_option MSC_OPT_ALLOC_PRIO_SPLIT; 16: all of them)
  const int aps = __builtin_amdgcn_readfirstlane(c.chain_prio ? 16 : c.al_psplit);
  const int psplit = MSC_AL_PRIO > 0 && aps < 16 ? (wmax * aps) >> 4 : -1;
  for (int oi = 0; oi <= wmax; oi++) {
    if (oi == psplit) __builtin_amdgcn_s_setprio(MSC_AL_PRIO2);
    const int jw = oi % AL_CH;
    if (jw == 0 && oi > 0) {  // wave-uniform: window oi / AL_CH is due, start the one after
      publish();
      fetch(oi / AL_CH + 1);
    }
    union {
      uint4 v[NVR];
      uint16_t h[8 * NVR];
    } ur;
#pragma unroll
    for (int v = 0; v < NVR; v++) ur.v[v] = Lrec[(jw * NVR + v) * 64];
    const int r = oi < n_orders ? (int)ur.h[0] : -1;
    if (r != cur) {  // region boundary (orders are region-major) or end of this env's list
#ifndef MSC_AL_ABL_NOFIN  // (timing ablation only: results wrong)
      if (cur >= 0) finalize(cur);
#endif
      cur = r;
      lost_cnt = 0;
#pragma unroll
      for (int sk = 0; sk < K; sk++) u[sk] = dsum[sk] = 0;
      hm = r >= 0 ? Lhm[r] : 0u;
      hw = hm != 0u ? __builtin_ctz(hm) : -1;
      smask = 0u;
      rtot = 0;
#pragma unroll
      for (int sk = 0; sk < K; sk++) shc[sk] = 0;
    }
    // (structured ifs and one exit per loop, not continue / break: every exit is a latch whose lane
    // masks the loops merge at each order and round; an empty order needs no test of its own -- no
    // candidate, so its first round ends the loop, and with nothing unfulfilled it is never lost)
    if (oi < n_orders) {
    int d[K], rem[K];
    double tw = 0.0;  // order.sku_demands.dot(sku_weights) (demand_allocator.py:167)
#pragma unroll
    for (int sk = 0; sk < K; sk++) {
      d[sk] = ur.h[1 + sk];
      rem[sk] = d[sk];
      dsum[sk] += d[sk];
      tw += (double)d[sk] * skw[sk];
    }
    // demand_allocator.py:168-172; every row is read first (unconditionally: the LDS table is
    // padded to MW, the global one clamped), so the loads overlap instead of each waiting alone
    double2 trow[MWL];
#pragma unroll
    for (int i = 0; i < MWL; i++) trow[i] = tab_at(r, TAB ? gw(i) : (gw(i) < W ? gw(i) : W - 1));
    double cost[MWL];
#pragma unroll
    for (int i = 0; i < MWL; i++) cost[i] = gw(i) < W ? trow[i].x + trow[i].y * tw : INFINITY;
    int used = 0;
    bool open = true;
    while (open) {
      // candidates: warehouses holding a still-needed SKU (a warehouse that shipped already has
      // nothing left the order needs: fill = min(rem, inv) zeroes one of the two for every SKU;
      // a warehouse with nothing to give is skipped without counting towards max_splits)
      uint32_t cand = 0u;
#pragma unroll
      for (int sk = 0; sk < K; sk++) cand |= rem[sk] > 0 ? stock[sk] : 0u;
      if (LPE == 1 && cand == 0u) {
        open = false;
      } else {
      // cheapest candidate, lowest index on ties (the stable argsort order the fixtures assert)
      double best = INFINITY;
      int b = LPE == 1 ? 0 : SENT;
#pragma unroll
      for (int i = 0; i < MWL; i++) {
        const bool take = ((cand >> i) & 1u) && cost[i] < best;
        best = take ? cost[i] : best;
        b = take ? gw(i) : b;
      }
      if constexpr (LPE > 1) {
        auto mn = [&](double ob, int o) {
          const bool t = ob < best || (ob == best && o < b);
          best = t ? ob : best;
          b = t ? o : b;
        };
        mn(dpp_x<0>(best), dpp_x<0>(b));
        if constexpr (LPE == 4) mn(dpp_x<1>(best), dpp_x<1>(b));
      }
      if (LPE > 1 && b == SENT) {  // nobody in the group holds a still-needed SKU
        open = false;
      } else {
      const bool own = (b & (LPE - 1)) == jl;
      const int ib = b >> LSH;
      // every LDS value of warehouse b is read in one batch (one wait), then written back: shipped
      // home is accumulated unconditionally (+0 when r is not b's home region)
      int iv[K], sh[K];
#pragma unroll
      for (int sk = 0; sk < K; sk++) {
        iv[sk] = Linv[(ib * K + sk) * 64];
        sh[sk] = SH ? Lshh[(ib * K + sk) * 64] : 0;
      }
      const bool home_b = (hm >> b) & 1u;
      const double out_b = Lout[ib * 64];
      const int qs_b = Lqs[ib * 64];
      const double2 tb = tab_at(r, b);
      int f[K], fs = 0;
#pragma unroll
      for (int sk = 0; sk < K; sk++) f[sk] = own ? (rem[sk] < iv[sk] ? rem[sk] : iv[sk]) : 0;
      if constexpr (LPE > 1) {  // the owner's fills to the group (16-bit fields: fills <= demand < 2^16)
        constexpr int NP = (K + 1) / 2;
        uint32_t pk[NP];
#pragma unroll
        for (int p = 0; p < NP; p++)
          pk[p] = (uint32_t)f[2 * p] | (2 * p + 1 < K ? (uint32_t)f[2 * p + 1] << 16 : 0u);
#pragma unroll
        for (int p = 0; p < NP; p++) {
          pk[p] |= (uint32_t)dpp_x<0>((int)pk[p]);
          if constexpr (LPE == 4) pk[p] |= (uint32_t)dpp_x<1>((int)pk[p]);
        }
#pragma unroll
        for (int sk = 0; sk < K; sk++) f[sk] = (int)((pk[sk / 2] >> (16 * (sk & 1))) & 0xffffu);
      }
      double fw = 0.0;
      bool done = true;
#pragma unroll
      for (int sk = 0; sk < K; sk++) {
        rem[sk] -= f[sk];
        done &= rem[sk] <= 0;
        fs += f[sk];
        fw += (double)f[sk] * skw[sk];
        if (!SH) shc[sk] += home_b ? f[sk] : 0;
      }
      // outbound cost of this shipment; the whole order from here: the ranking cost bit for bit
      const double oc = fw == tw ? best : tb.x + tb.y * fw;
      if (own) {
#pragma unroll
        for (int sk = 0; sk < K; sk++) {
          const int left = iv[sk] - f[sk];
          stock[sk] &= left > 0 ? ~0u : ~(1u << ib);
          Linv[(ib * K + sk) * 64] = left;
          if (SH) Lshh[(ib * K + sk) * 64] = sh[sk] + (home_b ? f[sk] : 0);
        }
        Lout[ib * 64] = out_b + oc;
        Lqs[ib * 64] = qs_b + fs;
        smask |= 1u << ib;
        if (dbg) {
#pragma unroll
          for (int sk = 0; sk < K; sk++) {
            if (info.shipment_quantities_by_sku) info.shipment_quantities_by_sku[((e * W + b) * R + r) * K + sk] += f[sk];
            if (info.fulfilled_per_warehouse) info.fulfilled_per_warehouse[e * WK + b * K + sk] += f[sk];
          }
          if (info.shipment_counts) info.shipment_counts[(e * W + b) * R + r] += 1;
          if (info.shipment_quantities) info.shipment_quantities[(e * W + b) * R + r] += fs;
        }
      }
      rtot += fs;
      used++;
      open = !(done || used >= maxwh);
#ifdef MSC_AL_ABL_ONEROUND  // (timing ablation only: results wrong)
      open = false;
#endif
      }
      }
    }
    // (rem >= 0 throughout: every fill is min(rem, inv) with inv >= 0)
    int remor = 0;
#pragma unroll
    for (int sk = 0; sk < K; sk++) {
      remor |= rem[sk];
      u[sk] += rem[sk];
    }
    lost_cnt += remor != 0 ? 1 : 0;
    }
  }

  if (!ev) return;
#pragma unroll
  for (int i = 0; i < MWL; i++) {
    const int w = gw(i);
    if (w < W) {
#pragma unroll
      for (int sk = 0; sk < K; sk++) {
        const int64_t g = (int64_t)(w * K + sk) * E + e;
        const int left = Linv[(i * K + sk) * 64];
        s.sc_sht[g] = s.inv[g] - left;  // shipped this step = the inventory drop (only shipments lower it here)
        s.inv[g] = left;
        if (SH) s.sc_shh[g] = Lshh[(i * K + sk) * 64];
      }
      s.sc_pen[w * E + e] = Lpen[i * 64];
      s.sc_out[w * E + e] = Lout[i * 64];
    }
  }
}

// shared home regions (a region that is home to two or more warehouses: possible when
// n_regions < n_warehouses) need the LDS shipped-home table; otherwise it stays in registers, which
// keeps the block at <= 39 KiB of LDS so two allocation blocks fit beside two demand blocks per CU
static bool shared_homes(const EnvConst& c) { return c.shared_home != 0; }
static size_t alloc_lane_lds_bytes(const EnvConst& c, int MW, int LPE, bool tab) {
  return (size_t)AlLds::make(MW / LPE, MW, c.K, c.R, tab, shared_homes(c)).total * sizeof(int32_t);
}
// cost table in LDS: when small (beside the demand kernel's blocks), or -- with empirical demand
// (no demand kernel beside this one) and at most one block per CU -- up to what the CU holds
// (C5, 16 x 256: 64 KiB of table; read from L2 instead, its latency sits on every order's chain)
static bool alloc_tab_in_lds(const EnvConst& c, int MW, int LPE) {
  if ((size_t)(c.R | 1) * MW * 16 <= AL_TAB_MAX) return true;
  const int64_t blocks = (c.E * LPE + 63) / 64;
  return c.demand_type == MSC_DEMAND_EMPIRICAL && blocks <= 256 &&
         alloc_lane_lds_bytes(c, MW, LPE, true) <= 160 * 1024;
}
template <typename F>
static hipError_t alloc_launch(F f, const EnvConst& c, const DevEnv* d, const StepIO& io, hipStream_t st, int lpe,
                               size_t lds) {
  if (lds > 64 * 1024) {  // above the default dynamic LDS limit (gfx950: 160 KiB per workgroup); set
                          // on every such launch: the attribute is per function and device
    const hipError_t e = hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(f, dim3((unsigned)((c.E * lpe + 63) / 64)), dim3(64), lds, st, d, io);
  return hipGetLastError();
}

// lanes per env: 1 unless MSC_ALLOC_LPE asks for 2 or 4 (measured slower at every BASELINE shape:
// DESIGN.md §3). Only the plain (non-debug, unshared-home, shipment / closest lost-sales)
// allocation is instantiated with LPE > 1.
static int alloc_lpe(const EnvConst& c, bool dbg, int MW) {
  int lpe = c.alloc_lpe;
  if (lpe != 2 && lpe != 4) lpe = 1;
  if (dbg || shared_homes(c) || c.lost_type == MSC_LOST_COST || MW < 8) lpe = 1;
  return lpe;
}

template <int K, int MW, bool EXACT>
hipError_t launch_alloc_mw(const EnvConst& c, const DevEnv* d, const StepIO& io, hipStream_t st) {
  using KFn = void (*)(const DevEnv*, StepIO);
  const bool dbg = io.has_info != 0;
  const int lpe = alloc_lpe(c, dbg, MW);
  const bool tab = alloc_tab_in_lds(c, MW, lpe);
  const size_t lds = alloc_lane_lds_bytes(c, MW, lpe, tab);
  KFn f;
#define MSC_AL(DB, TB, SHV, LP) (KFn)alloc_lane_kernel<K, MW, DB, TB, SHV, EXACT, LP>
  if constexpr (MW >= 8) {
    if (lpe > 1) {
      f = lpe == 4 ? (tab ? MSC_AL(false, true, false, 4) : MSC_AL(false, false, false, 4))
                   : (tab ? MSC_AL(false, true, false, 2) : MSC_AL(false, false, false, 2));
      return alloc_launch(f, c, d, io, st, lpe, lds);
    }
  }
  if (shared_homes(c))
    f = dbg ? (tab ? MSC_AL(true, true, true, 1) : MSC_AL(true, false, true, 1))
            : (tab ? MSC_AL(false, true, true, 1) : MSC_AL(false, false, true, 1));
  else
    f = dbg ? (tab ? MSC_AL(true, true, false, 1) : MSC_AL(true, false, false, 1))
            : (tab ? MSC_AL(false, true, false, 1) : MSC_AL(false, false, false, 1));
#undef MSC_AL
  return alloc_launch(f, c, d, io, st, 1, lds);
}

template <int K>
hipError_t launch_alloc_lane_k(const EnvConst& c, const DevEnv* d, const StepIO& io, hipStream_t st) {
  // exact instantiations for the warehouse counts of the BASELINE configs (2, 8, 16), masked ones
  // (next power of two) otherwise
  if (c.W == 2) return launch_alloc_mw<K, 2, true>(c, d, io, st);
  if (c.W <= 4) return launch_alloc_mw<K, 4, false>(c, d, io, st);
  if (c.W == 8) return launch_alloc_mw<K, 8, true>(c, d, io, st);
  if (c.W < 8) return launch_alloc_mw<K, 8, false>(c, d, io, st);
  if (c.W == 16) return launch_alloc_mw<K, 16, true>(c, d, io, st);
  return launch_alloc_mw<K, 16, false>(c, d, io, st);
}

// The kernels are instantiated in sixteen translation units so the build runs them in parallel:
// MSC_AL_PART = 2K - 1 holds the exact warehouse counts of SKU count K (and launch_alloc_lane_k<K>),
// 2K the masked ones (the Makefile compiles this file once per part); MSC_AL_PART 0 (a plain
// one-file build) instantiates all of them.
#ifndef MSC_AL_PART
#define MSC_AL_PART 0
#endif
#define MSC_AL_MW(KV, MWV, EX, KW) KW template hipError_t launch_alloc_mw<KV, MWV, EX>(const EnvConst&, const DevEnv*, const StepIO&, hipStream_t);
#define MSC_AL_EXACT(KV, KW) MSC_AL_MW(KV, 2, true, KW) MSC_AL_MW(KV, 8, true, KW) MSC_AL_MW(KV, 16, true, KW)
#define MSC_AL_MASKED(KV, KW) MSC_AL_MW(KV, 4, false, KW) MSC_AL_MW(KV, 8, false, KW) MSC_AL_MW(KV, 16, false, KW)
#define MSC_AL_K(KV) template hipError_t launch_alloc_lane_k<KV>(const EnvConst&, const DevEnv*, const StepIO&, hipStream_t);
#if MSC_AL_PART == 0
#define MSC_AL_ALL(KV) MSC_AL_EXACT(KV, ) MSC_AL_MASKED(KV, ) MSC_AL_K(KV)
MSC_AL_ALL(1) MSC_AL_ALL(2) MSC_AL_ALL(3) MSC_AL_ALL(4) MSC_AL_ALL(5) MSC_AL_ALL(6) MSC_AL_ALL(7) MSC_AL_ALL(8)
#undef MSC_AL_ALL
#elif MSC_AL_PART == 1  // + launch_alloc_lane, whose switch must not instantiate the other parts' K
MSC_AL_MASKED(1, extern)
MSC_AL_EXACT(1, )
MSC_AL_K(1)
extern MSC_AL_K(2) extern MSC_AL_K(3) extern MSC_AL_K(4) extern MSC_AL_K(5) extern MSC_AL_K(6) extern MSC_AL_K(7) extern MSC_AL_K(8)
#elif MSC_AL_PART % 2 == 1
MSC_AL_MASKED((MSC_AL_PART + 1) / 2, extern)
MSC_AL_EXACT((MSC_AL_PART + 1) / 2, )
MSC_AL_K((MSC_AL_PART + 1) / 2)
#else
MSC_AL_MASKED(MSC_AL_PART / 2, )
#endif
#undef MSC_AL_K
#undef MSC_AL_MASKED
#undef MSC_AL_EXACT
#undef MSC_AL_MW

#if MSC_AL_PART == 0 || MSC_AL_PART == 1
hipError_t launch_alloc_lane(const EnvConst& c, const DevEnv* d, const StepIO& io, hipStream_t st) {
  switch (c.K) {
    case 1: return launch_alloc_lane_k<1>(c, d, io, st);
    case 2: return launch_alloc_lane_k<2>(c, d, io, st);
    case 3: return launch_alloc_lane_k<3>(c, d, io, st);
    case 4: return launch_alloc_lane_k<4>(c, d, io, st);
    case 5: return launch_alloc_lane_k<5>(c, d, io, st);
    case 6: return launch_alloc_lane_k<6>(c, d, io, st);
    case 7: return launch_alloc_lane_k<7>(c, d, io, st);
    case 8: return launch_alloc_lane_k<8>(c, d, io, st);
    default: return hipErrorInvalidValue;
  }
}
#endif

}  // namespace msc
