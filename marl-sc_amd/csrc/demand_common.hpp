// demand_common.hpp -- pieces shared by the Poisson demand kernels (env_kernels.hip:
// demand_unit_kernel / demand_park4_kernel; demand_ab.hip: demand_ab_kernel): the PCG64 state I/O of
// the env's demand stream, the generator ring geometry and refill quota, the parser states, and the
// episode-ahead root derivation.
#pragma once
#include <hip/hip_runtime.h>

#include "env.hpp"
#include "kcommon.hpp"
#include "rng.hpp"

namespace msc {

__device__ __forceinline__ Pcg64 load_rng(const EnvState& s, int which, int64_t e, int64_t E) {
  Pcg64 r;
  const uint64_t* b = s.rng + (int64_t)which * 4 * E + e;
  r.s_hi = b[0];
  r.s_lo = b[E];
  r.i_hi = b[2 * E];
  r.i_lo = b[3 * E];
  r.has32 = s.rbuf[(int64_t)which * 2 * E + e];
  r.u32 = s.rbuf[(int64_t)which * 2 * E + E + e];
  return r;
}
// the demand stream as it was before this demand generation (see EnvState::rng_pre)
__device__ __forceinline__ void store_rng_pre(const EnvState& s, int64_t e, int64_t E, const Pcg64& r) {
  s.rng_pre[e] = r.s_hi;
  s.rng_pre[E + e] = r.s_lo;
  s.rng_pre[2 * E + e] = r.i_hi;
  s.rng_pre[3 * E + e] = r.i_lo;
  s.rbuf_pre[e] = r.has32;
  s.rbuf_pre[E + e] = r.u32;
}
__device__ __forceinline__ void store_rng(const EnvState& s, int which, int64_t e, int64_t E, const Pcg64& r) {
  uint64_t* b = s.rng + (int64_t)which * 4 * E + e;
  b[0] = r.s_hi;
  b[E] = r.s_lo;
  b[2 * E] = r.i_hi;
  b[3 * E] = r.i_lo;
  s.rbuf[(int64_t)which * 2 * E + e] = r.has32;
  s.rbuf[(int64_t)which * 2 * E + E + e] = r.u32;
}

constexpr int PS_MASK = 0, PS_ORD = 1, PS_QTY = 2, PS_DONE = 3;

#ifndef MSC_UD
#define MSC_UD 8
#endif
#ifndef MSC_UHS
#define MSC_UHS 4
#endif
constexpr int UD = MSC_UD;                  // uniforms per round
constexpr int UHS = MSC_UHS;                // rounds per chunk (<= UD * UHS draws per lane)
constexpr int pow2ceil(int x) { return x <= 1 ? 1 : 2 * pow2ceil((x + 1) / 2); }
#ifndef MSC_UCAP_X
#define MSC_UCAP_X 1  // A/B: ring capacity multiplier (deeper rings, fewer demand blocks per CU)
#endif
constexpr int UCAP = pow2ceil(2 * UD * UHS) * MSC_UCAP_X;  // ring capacity (positions), >= 2 chunks
constexpr int USLOTS = UCAP + UD;           // ring rows: UCAP + the UD - 1 mirrored ones + a dummy row
static_assert((UCAP & (UCAP - 1)) == 0, "ring layout");

#ifndef MSC_GEN_QUOTA
#define MSC_GEN_QUOTA 24  // positions added per lane per chunk (mean consumption ~18 at lambda 4-5)
#endif
// the generators' fill target for the next phase: QUOTA more positions, capped by the ring slots the
// parser's current chunk (starting at rdp) cannot read
__device__ __forceinline__ int unit_quota(int tgt, int rdp) {
  const int q = tgt + MSC_GEN_QUOTA, cap = rdp + UCAP;
  return q < cap ? q : cap;
}

// EA: the root seed of the episode a lane generates (reset_env's counter rule applied
// iters0 + k * iters_step times from the counter stored for from_slot, or for the lane's own slot
// when from_slot < 0); the counter after that reset goes to cnt_out
__device__ __forceinline__ uint32_t ea_root(const EnvConst& c, const EnvState& s, const EaLaunch& ea, int64_t e,
                                            int k, int slot, int& cnt_out) {
  int cnt = s.ea_cnt[(int64_t)(ea.from_slot < 0 ? slot : ea.from_slot) * c.E + e];
  const int iters = ea.iters0 + k * ea.iters_step;
  int wv = 0;
  for (int i = 0; i < iters; i++) {
    wv = (c.num_eval > 0 && cnt >= c.num_eval) ? 0 : cnt;
    cnt = wv + 1;
  }
  cnt_out = cnt;
  const uint32_t w2[2] = {s.orig_root[e], (uint32_t)wv};
  return ss_u32(w2, 2);
}

__host__ __device__ constexpr size_t unit_lds_fixed() {
  return (size_t)BS * USLOTS * sizeof(double) + (size_t)2 * BS * sizeof(int32_t);
}

#ifndef MSC_PARSER_PRIO
#define MSC_PARSER_PRIO 2  // s_setprio of the parser wave (generators: MSC_GEN_PRIO)
#endif
#ifndef MSC_GEN_PRIO
#define MSC_GEN_PRIO 1
#endif
#ifndef MSC_DEM_WPE
#define MSC_DEM_WPE 8  // <= 64 VGPRs: two demand waves fit beside four step_b waves on a SIMD
#endif

}  // namespace msc
