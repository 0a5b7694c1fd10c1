// rng.hpp -- numpy-2.x-compatible random streams for the device (and host) side of libmarlsc.
//
// The reference draws all env randomness from numpy Generators created by its SeedManager
// (src/utils/seed_manager.py:63-78, 100-120, 207-224): SeedSequence pools -> PCG64 -> random(),
// poisson() (multiplication method below lam = 10), integers() (32-bit buffered Lemire).
// Restated here on 64-bit limbs so a gfx950 lane advances a 128-bit LCG with 13 integer
// multiplies and no 128-bit emulation library. Every function is bit-exact with numpy; the
// parity tests compare the resulting PCG64 states after every step.
#pragma once
#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define MSC_HD __host__ __device__ __forceinline__
#else
#define MSC_HD inline
#endif

namespace msc {

// ---- SeedSequence (numpy/random/bit_generator.pyx) ------------------------------------------
constexpr uint32_t SS_INIT_A = 0x43b0d7e5u, SS_MULT_A = 0x931e8875u;
constexpr uint32_t SS_INIT_B = 0x8b51f9ddu, SS_MULT_B = 0x58f38dedu;
constexpr uint32_t SS_MIX_L = 0xca01f9ddu, SS_MIX_R = 0x4973f715u;

MSC_HD uint32_t ss_hashmix(uint32_t v, uint32_t& hc) {
  v ^= hc;
  hc *= SS_MULT_A;
  v *= hc;
  return v ^ (v >> 16);
}
MSC_HD uint32_t ss_mix(uint32_t x, uint32_t y) {
  uint32_t r = SS_MIX_L * x - SS_MIX_R * y;
  return r ^ (r >> 16);
}
// Pool of SeedSequence(entropy[0..n)) or, with spawn key k >= 0,
// SeedSequence(entropy, spawn_key=(k,)) (entropy zero-padded to 4 words first).
MSC_HD void ss_pool(const uint32_t* ent, int n_ent, int spawn_key, uint32_t pool[4]) {
  uint32_t buf[6];
  int n = 0;
  for (int i = 0; i < n_ent && i < 5; i++) buf[n++] = ent[i];
  if (spawn_key >= 0) {
    while (n < 4) buf[n++] = 0u;
    buf[n++] = (uint32_t)spawn_key;
  }
  uint32_t hc = SS_INIT_A;
#pragma unroll
  for (int i = 0; i < 4; i++) pool[i] = ss_hashmix(i < n ? buf[i] : 0u, hc);
#pragma unroll
  for (int s = 0; s < 4; s++)
#pragma unroll
    for (int d = 0; d < 4; d++)
      if (s != d) pool[d] = ss_mix(pool[d], ss_hashmix(pool[s], hc));
  for (int s = 4; s < n; s++)
#pragma unroll
    for (int d = 0; d < 4; d++) pool[d] = ss_mix(pool[d], ss_hashmix(buf[s], hc));
}
MSC_HD void ss_generate(const uint32_t pool[4], uint32_t* out, int n_words) {
  uint32_t hc = SS_INIT_B;
  for (int i = 0; i < n_words; i++) {
    uint32_t v = pool[i & 3] ^ hc;
    hc *= SS_MULT_B;
    v *= hc;
    out[i] = v ^ (v >> 16);
  }
}
MSC_HD uint32_t ss_u32(const uint32_t* words, int n) {
  uint32_t pool[4], o;
  ss_pool(words, n, -1, pool);
  ss_generate(pool, &o, 1);
  return o;
}

// ---- PCG64 (XSL-RR 128/64) ------------------------------------------------------------------
constexpr uint64_t PCG_MUL_HI = 2549297995355413924ULL;
constexpr uint64_t PCG_MUL_LO = 4865540595714422341ULL;

struct Pcg64 {
  uint64_t s_hi, s_lo, i_hi, i_lo;  // state, increment
  uint32_t has32, u32;               // numpy's buffered upper half for next_uint32
};

MSC_HD uint64_t mulhi64(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul64hi(a, b);
#else
  return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}

MSC_HD void pcg_step(Pcg64& r) {
  uint64_t lo = r.s_lo * PCG_MUL_LO;
  uint64_t hi = r.s_hi * PCG_MUL_LO + r.s_lo * PCG_MUL_HI + mulhi64(r.s_lo, PCG_MUL_LO);
  uint64_t nlo = lo + r.i_lo;
  hi += r.i_hi + (nlo < lo ? 1u : 0u);
  r.s_lo = nlo;
  r.s_hi = hi;
}
MSC_HD uint64_t pcg_next64(Pcg64& r) {
  pcg_step(r);
  uint64_t x = r.s_hi ^ r.s_lo;
  unsigned rot = (unsigned)(r.s_hi >> 58);
  return (x >> rot) | (x << ((64u - rot) & 63u));
}
MSC_HD uint32_t pcg_next32(Pcg64& r) {
  if (r.has32) {
    r.has32 = 0;
    return r.u32;
  }
  uint64_t v = pcg_next64(r);
  r.has32 = 1;
  r.u32 = (uint32_t)(v >> 32);
  return (uint32_t)v;
}
MSC_HD double pcg_double(Pcg64& r) { return (double)(pcg_next64(r) >> 11) * (1.0 / 9007199254740992.0); }

// ---- 128-bit LCG algebra for split / jump-ahead generation ----------------------------------
// low 128 bits of (ah:al) * (bh:bl)
MSC_HD void mul128(uint64_t ah, uint64_t al, uint64_t bh, uint64_t bl, uint64_t& rh, uint64_t& rl) {
  const uint64_t lo = al * bl;
  rh = mulhi64(al, bl) + ah * bl + al * bh;
  rl = lo;
}
MSC_HD void add128(uint64_t& ah, uint64_t& al, uint64_t bh, uint64_t bl) {
  const uint64_t lo = al + bl;
  ah += bh + (lo < bl ? 1u : 0u);
  al = lo;
}
// XSL-RR output of a state and numpy's random() of it
MSC_HD uint64_t pcg_output(uint64_t s_hi, uint64_t s_lo) {
  const uint64_t x = s_hi ^ s_lo;
  const unsigned rot = (unsigned)(s_hi >> 58);
  return (x >> rot) | (x << ((64u - rot) & 63u));
}
MSC_HD double u64_to_double(uint64_t v) { return (double)(v >> 11) * (1.0 / 9007199254740992.0); }

// The same double from the state directly (XSL-RR output >> 11 as 2^-53 units): the top 32 bits of
// the rotated word scaled by 2^-32 plus its next 21 bits scaled by 2^-53, one exact fma (the sum is
// k * 2^-53 with k < 2^53, representable). Fewer instructions than the 64-bit shift + two
// conversions + two scalings of u64_to_double(pcg_output(..)); bit-identical.
MSC_HD double pcg_output_double(uint64_t s_hi, uint64_t s_lo) {
  const uint64_t r = pcg_output(s_hi, s_lo);
  return fma((double)(uint32_t)(r >> 32), 0x1p-32, (double)((uint32_t)r >> 11) * 0x1p-53);
}

// s <- s * m + c (mod 2^128) as one 128-bit integer expression: the backend emits the partial
// products and a single add-with-carry chain (fewer instructions than mul128 + add128).
MSC_HD void lcg128(uint64_t& sh, uint64_t& sl, uint64_t mh, uint64_t ml, uint64_t ch, uint64_t cl) {
  const unsigned __int128 s = ((unsigned __int128)sh << 64) | sl;
  const unsigned __int128 m = ((unsigned __int128)mh << 64) | ml;
  const unsigned __int128 c = ((unsigned __int128)ch << 64) | cl;
  const unsigned __int128 n = s * m + c;
  sh = (uint64_t)(n >> 64);
  sl = (uint64_t)n;
}

// Affine map s -> A*s + C of `n` PCG64 steps for increment (ih:il) (Brown, "Random number
// generation with arbitrary strides"; numpy's pcg64_advance uses the same recurrence).
MSC_HD void pcg_jump_coeffs(uint64_t n, uint64_t ih, uint64_t il, uint64_t& ah, uint64_t& al, uint64_t& ch,
                            uint64_t& cl) {
  uint64_t am_h = 0, am_l = 1, ap_h = 0, ap_l = 0;                 // accumulated map (identity)
  uint64_t cm_h = PCG_MUL_HI, cm_l = PCG_MUL_LO, cp_h = ih, cp_l = il;  // map of 2^k steps
  while (n) {
    if (n & 1) {
      uint64_t th, tl;
      mul128(am_h, am_l, cm_h, cm_l, am_h, am_l);
      mul128(ap_h, ap_l, cm_h, cm_l, th, tl);
      add128(th, tl, cp_h, cp_l);
      ap_h = th;
      ap_l = tl;
    }
    uint64_t mh = cm_h, ml = cm_l;  // cp = (cm + 1) * cp ; cm = cm * cm
    add128(mh, ml, 0, 1);
    mul128(mh, ml, cp_h, cp_l, cp_h, cp_l);
    mul128(cm_h, cm_l, cm_h, cm_l, cm_h, cm_l);
    n >>= 1;
  }
  ah = am_h;
  al = am_l;
  ch = ap_h;
  cl = ap_l;
}
// advance the stream by n draws of next64 (the 32-bit buffer is left as it is)
MSC_HD void pcg_advance(Pcg64& r, uint64_t n) {
  uint64_t ah, al, ch, cl, sh, sl;
  pcg_jump_coeffs(n, r.i_hi, r.i_lo, ah, al, ch, cl);
  mul128(ah, al, r.s_hi, r.s_lo, sh, sl);
  add128(sh, sl, ch, cl);
  r.s_hi = sh;
  r.s_lo = sl;
}

// PCG64(SeedSequence pool): generate_state(4, uint64) = {seed_hi, seed_lo, inc_hi, inc_lo}
MSC_HD void pcg_seed_pool(Pcg64& r, const uint32_t pool[4]) {
  uint32_t w[8];
  ss_generate(pool, w, 8);
  uint64_t s0 = (uint64_t)w[0] | ((uint64_t)w[1] << 32), s1 = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
  uint64_t q0 = (uint64_t)w[4] | ((uint64_t)w[5] << 32), q1 = (uint64_t)w[6] | ((uint64_t)w[7] << 32);
  // inc = (initseq << 1) | 1 over 128 bits
  r.i_hi = (q0 << 1) | (q1 >> 63);
  r.i_lo = (q1 << 1) | 1u;
  r.s_hi = 0;
  r.s_lo = 0;
  pcg_step(r);
  uint64_t lo = r.s_lo + s1;
  r.s_hi += s0 + (lo < s1 ? 1u : 0u);
  r.s_lo = lo;
  pcg_step(r);
  r.has32 = 0;
  r.u32 = 0;
}
// Generator of SeedManager child `key` of root seed `root` (spawn_key=(key,))
MSC_HD void pcg_seed_child(Pcg64& r, uint32_t root, int key) {
  uint32_t pool[4];
  ss_pool(&root, 1, key, pool);
  pcg_seed_pool(r, pool);
}

// random_poisson for 0 <= lam < 10: multiplication method; enlam = exp(-lam) from the host libm.
MSC_HD int poisson_mult(Pcg64& r, double enlam) {
  int x = 0;
  double prod = 1.0;
  for (;;) {
    prod *= pcg_double(r);
    if (prod > enlam) x += 1;
    else return x;
  }
}

// ---- random_poisson_ptrs (numpy/random/src/distributions/distributions.c, numpy 2.2): lam >= 10 --
// Hoermann's transformed rejection. The per-rate constants come from the host libm (as numpy's own
// computation: sqrt, log of the rate and of invalpha), laid out as 8 doubles per rate.
struct PtrsConst {
  double lam, slam, loglam, b, a, invalpha, vr, log_invalpha;
};
static_assert(sizeof(PtrsConst) == 8 * sizeof(double), "PtrsConst layout");
inline PtrsConst ptrs_const_host(double lam) {
  PtrsConst p;
  p.lam = lam;
  p.slam = sqrt(lam);
  p.loglam = log(lam);
  p.b = 0.931 + 2.53 * p.slam;
  p.a = -0.059 + 0.02483 * p.b;
  p.invalpha = 1.1239 + 1.1328 / (p.b - 3.4);
  p.vr = 0.9277 - 3.6224 / (p.b - 2);
  p.log_invalpha = log(p.invalpha);
  return p;
}
// random_loggam (distributions.c): Stirling series with the argument shifted to >= 7
MSC_HD double np_loggam(double x) {
  const double a0 = 8.333333333333333e-02, a1 = -2.777777777777778e-03, a2 = 7.936507936507937e-04,
               a3 = -5.952380952380952e-04, a4 = 8.417508417508418e-04, a5 = -1.917526917526918e-03,
               a6 = 6.410256410256410e-03, a7 = -2.955065359477124e-02, a8 = 1.796443723688307e-01,
               a9 = -1.39243221690590e+00;
  if (x == 1.0 || x == 2.0) return 0.0;
  const int64_t n = x < 7.0 ? (int64_t)(7 - x) : 0;
  double x0 = x + (double)n;
  const double x2 = (1.0 / x0) * (1.0 / x0);
  double gl0 = a9;
  gl0 *= x2; gl0 += a8;
  gl0 *= x2; gl0 += a7;
  gl0 *= x2; gl0 += a6;
  gl0 *= x2; gl0 += a5;
  gl0 *= x2; gl0 += a4;
  gl0 *= x2; gl0 += a3;
  gl0 *= x2; gl0 += a2;
  gl0 *= x2; gl0 += a1;
  gl0 *= x2; gl0 += a0;
  double gl = gl0 / x0 + 0.5 * 1.8378770664093453e+00 + (x0 - 0.5) * log(x0) - x0;
  for (int64_t k = 1; k <= n; k++) {
    gl -= log(x0 - 1.0);
    x0 -= 1.0;
  }
  return gl;
}
// the samplers below draw through a generator adaptor with next_double(): the plain stream, or one
// that also counts the draws (the episode-ahead demand records stream positions)
struct PcgRef {
  Pcg64& r;
  MSC_HD double next_double() { return pcg_double(r); }
};
struct PcgCounted {
  Pcg64 r;
  uint32_t n;
  MSC_HD double next_double() {
    n++;
    return pcg_double(r);
  }
};
template <class G>
MSC_HD int64_t poisson_mult_g(G& g, double enlam) {
  int64_t x = 0;
  double prod = 1.0;
  for (;;) {
    prod *= g.next_double();
    if (prod > enlam) x += 1;
    else return x;
  }
}
// two doubles per trial; the fast acceptance (~90 % of trials near lam = 10) needs no logarithm
template <class G>
MSC_HD int64_t poisson_ptrs_g(G& g, const PtrsConst& p) {
  for (;;) {
    const double U = g.next_double() - 0.5;
    const double V = g.next_double();
    const double us = 0.5 - fabs(U);
    const int64_t k = (int64_t)floor((2 * p.a / us + p.b) * U + p.lam + 0.43);
    if ((us >= 0.07) && (V <= p.vr)) return k;
    if ((k < 0) || ((us < 0.013) && (V > us))) continue;
    if ((log(V) + p.log_invalpha - log(p.a / (us * us) + p.b)) <= (-p.lam + (double)k * p.loglam - np_loggam((double)(k + 1))))
      return k;
  }
}
// random_poisson: PTRS for lam >= 10, multiplication method below (enlam = exp(-lam) from the host)
template <class G>
MSC_HD int64_t poisson_any_g(G& g, double enlam, const PtrsConst& p) {
  return p.lam >= 10.0 ? poisson_ptrs_g(g, p) : poisson_mult_g(g, enlam);
}

// Generator.integers(low, high_exclusive) for ranges < 2^32 (buffered 32-bit Lemire).
MSC_HD int64_t bounded_int(Pcg64& r, int64_t low, int64_t high_excl) {
  uint32_t rng = (uint32_t)(high_excl - 1 - low);
  if (rng == 0) return low;
  if (rng == 0xFFFFFFFFu) return low + (int64_t)pcg_next32(r);
  uint32_t rng_excl = rng + 1u;
  uint64_t m = (uint64_t)pcg_next32(r) * rng_excl;
  uint32_t left = (uint32_t)m;
  if (left < rng_excl) {
    uint32_t thr = (0xFFFFFFFFu - rng) % rng_excl;
    while (left < thr) {
      m = (uint64_t)pcg_next32(r) * rng_excl;
      left = (uint32_t)m;
    }
  }
  return low + (int64_t)(m >> 32);
}

}  // namespace msc
