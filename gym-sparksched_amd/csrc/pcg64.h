// pcg64.h — numpy Generator(PCG64) consumption model on device.
//
// Restates numpy/random/src/pcg64 (pcg_setseq_128_xsl_rr_64: step, then output) and the parts of
// numpy's distributions the reference sampler calls at step time:
//   Generator.random()            -> next_double          (tpch.py:225)
//   Generator.choice(list of n)   -> integers(0, n)       (tpch.py:211)  buffered 32-bit Lemire
//   Generator.integers(0, n)      -> same                  (tpch.py:177, reset-time)
//   Generator.exponential(scale)  -> scale * ziggurat standard exponential (tpch.py:70, reset-time)
// and the seeding of gymnasium's Env.reset(seed) (spark_sched_sim.py:130):
//   Generator(PCG64(SeedSequence(seed)))  -> Pcg64::from_seed
// Pinned against numpy by tests/test_kats.py (mixed random/choice/integers sequences, state round trips,
// exponential streams, seeds).
#pragma once
#include <stdint.h>

#include "fdlibm.h"
#include "ziggurat.h"

namespace ssim {

struct Pcg64 {
  uint64_t s_hi, s_lo, i_hi, i_lo;
  uint32_t has32, u32;

  __device__ __forceinline__ uint64_t next64() {
    typedef unsigned __int128 u128;
    const u128 mult = ((u128)0x2360ED051FC65DA4ULL << 64) | (u128)0x4385DF649FCCF645ULL;
    u128 s = ((u128)s_hi << 64) | (u128)s_lo;
    const u128 inc = ((u128)i_hi << 64) | (u128)i_lo;
    s = s * mult + inc;
    s_hi = (uint64_t)(s >> 64);
    s_lo = (uint64_t)s;
    const uint64_t x = s_hi ^ s_lo;
    const unsigned rot = (unsigned)(s_hi >> 58);
    return (x >> rot) | (x << ((64u - rot) & 63u));
  }

  __device__ __forceinline__ uint32_t next32() {
    if (has32) {
      has32 = 0;
      return u32;
    }
    const uint64_t v = next64();
    has32 = 1;
    u32 = (uint32_t)(v >> 32);
    return (uint32_t)v;
  }

  __device__ __forceinline__ void step128() {
    typedef unsigned __int128 u128;
    const u128 mult = ((u128)0x2360ED051FC65DA4ULL << 64) | (u128)0x4385DF649FCCF645ULL;
    u128 st = ((u128)s_hi << 64) | (u128)s_lo;
    st = st * mult + (((u128)i_hi << 64) | (u128)i_lo);
    s_hi = (uint64_t)(st >> 64);
    s_lo = (uint64_t)st;
  }

  // numpy SeedSequence(seed).generate_state(4, uint64) for a non-negative integer seed (no spawn key),
  // then pcg64_set_seed (pcg_setseq_128_srandom_r).
  __device__ __forceinline__ static Pcg64 from_seed(uint64_t seed) {
    const uint32_t kInitA = 0x43b0d7e5u, kMultA = 0x931e8875u, kInitB = 0x8b51f9ddu, kMultB = 0x58f38dedu,
                   kMixL = 0xca01f9ddu, kMixR = 0x4973f715u;
    uint32_t ent[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    const int n_ent = (seed >> 32) ? 2 : 1;
    uint32_t hc = kInitA;
    auto hashmix = [&](uint32_t v) {
      v ^= hc;
      hc *= kMultA;
      v *= hc;
      v ^= v >> 16;
      return v;
    };
    auto mix = [](uint32_t x, uint32_t y) {
      uint32_t r = kMixL * x - kMixR * y;
      r ^= r >> 16;
      return r;
    };
    uint32_t pool[4];
    for (int i = 0; i < 4; ++i) pool[i] = hashmix(i < n_ent ? ent[i] : 0u);
    for (int a = 0; a < 4; ++a)
      for (int b = 0; b < 4; ++b)
        if (a != b) pool[b] = mix(pool[b], hashmix(pool[a]));
    uint32_t w[8];
    uint32_t hb = kInitB;
    for (int i = 0; i < 8; ++i) {
      uint32_t v = pool[i & 3];
      v ^= hb;
      hb *= kMultB;
      v *= hb;
      v ^= v >> 16;
      w[i] = v;
    }
    const uint64_t st_hi = w[0] | ((uint64_t)w[1] << 32), st_lo = w[2] | ((uint64_t)w[3] << 32);
    const uint64_t sq_hi = w[4] | ((uint64_t)w[5] << 32), sq_lo = w[6] | ((uint64_t)w[7] << 32);
    Pcg64 r;
    r.has32 = 0;
    r.u32 = 0;
    r.i_hi = (sq_hi << 1) | (sq_lo >> 63);  // inc = (initseq << 1) | 1
    r.i_lo = (sq_lo << 1) | 1u;
    r.s_hi = 0;
    r.s_lo = 0;
    r.step128();
    const unsigned __int128 s = (((unsigned __int128)r.s_hi << 64) | r.s_lo) +
                                (((unsigned __int128)st_hi << 64) | st_lo);
    r.s_hi = (uint64_t)(s >> 64);
    r.s_lo = (uint64_t)s;
    r.step128();
    return r;
  }

  // Generator.random(): 53-bit double in [0, 1)
  __device__ __forceinline__ double random() { return (double)(next64() >> 11) * (1.0 / 9007199254740992.0); }

  // numpy random_standard_exponential (ziggurat, distributions.c). The tail uses fd_log1p (== the host libm
  // numpy links); the wedge test compares against exp(-x), where a last-bit difference between the device
  // and host exp could only flip the outcome for a uniform draw within an ulp of exp(-x) (never observed:
  // tests/test_kats.py and the GPU reset-parity tests compare whole streams).
  __device__ __forceinline__ double std_exponential() {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
    for (;;) {
      uint64_t ri = next64() >> 3;
      const int idx = (int)(ri & 0xFF);
      ri >>= 8;
      const double we = __builtin_bit_cast(double, kZigWeBits[idx]);
      const double x = (double)ri * we;
      if (ri < kZigKe[idx]) return x;
      if (idx == 0) return kZigExpR - fd_log1p(-random());
      const double fe0 = __builtin_bit_cast(double, kZigFeBits[idx - 1]);
      const double fe1 = __builtin_bit_cast(double, kZigFeBits[idx]);
      if ((fe0 - fe1) * random() + fe1 < exp(-x)) return x;
    }
  }

  // Generator.integers(0, n) / choice(<n items>) for 1 <= n <= 2^32-1: no draw when n == 1.
  __device__ __forceinline__ uint32_t bounded(uint32_t n) {
    const uint32_t rng = n - 1u;
    if (rng == 0u) return 0u;
    uint64_t m = (uint64_t)next32() * (uint64_t)n;
    uint32_t left = (uint32_t)m;
    if (left < n) {
      const uint32_t threshold = (0xFFFFFFFFu - rng) % n;
      while (left < threshold) {
        m = (uint64_t)next32() * (uint64_t)n;
        left = (uint32_t)m;
      }
    }
    return (uint32_t)(m >> 32);
  }
};

}  // namespace ssim
