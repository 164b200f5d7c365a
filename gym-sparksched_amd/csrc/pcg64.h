// pcg64.h — numpy Generator(PCG64) consumption model on device.
//
// Restates numpy/random/src/pcg64 (pcg_setseq_128_xsl_rr_64: step, then output) and the parts of
// numpy's distributions the reference sampler calls at step time:
//   Generator.random()            -> next_double          (tpch.py:225)
//   Generator.choice(list of n)   -> integers(0, n)       (tpch.py:211)  buffered 32-bit Lemire
//   Generator.integers(0, n)      -> same                  (tpch.py:177, reset-time)
// Pinned against numpy by tests/test_kats.py (mixed random/choice/integers sequences, state round trips).
#pragma once
#include <stdint.h>

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

  // Generator.random(): 53-bit double in [0, 1)
  __device__ __forceinline__ double random() { return (double)(next64() >> 11) * (1.0 / 9007199254740992.0); }

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
