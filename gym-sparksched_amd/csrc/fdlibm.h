// fdlibm.h — log1p as computed by the host C library numpy calls (glibc 2.35, sysdeps/ieee754/dbl-64/
// s_log1p.c: the fdlibm algorithm with the Estrin-form polynomial), so the device reproduces
// Generator.exponential's ziggurat tail (`ziggurat_exp_r - npy_log1p(-next_double())`) bit for bit.
// Plain IEEE double arithmetic with contraction disabled (an FMA would change the rounding).
// Pinned against the host libm by tests/test_kats.py (hostsim build of this same header).
#pragma once
#include <stdint.h>
#include <string.h>

namespace ssim {

__device__ __forceinline__ int32_t fd_hi(double x) {
  uint64_t b;
  __builtin_memcpy(&b, &x, 8);
  return (int32_t)(b >> 32);
}
__device__ __forceinline__ double fd_sethi(double x, int32_t h) {
  uint64_t b;
  __builtin_memcpy(&b, &x, 8);
  b = (b & 0xFFFFFFFFull) | ((uint64_t)(uint32_t)h << 32);
  __builtin_memcpy(&x, &b, 8);
  return x;
}

// log1p(x) for finite x > -1 (the sampler calls it with x in (-1, 0]); -1 -> -inf, < -1 -> NaN.
__device__ __forceinline__ double fd_log1p(double x) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  const double Lp1 = 6.666666666666735130e-01, Lp2 = 3.999999999940941908e-01, Lp3 = 2.857142874366239149e-01,
               Lp4 = 2.222219843214978396e-01, Lp5 = 1.818357216161805012e-01, Lp6 = 1.531383769920937332e-01,
               Lp7 = 1.479819860511658591e-01;
  double f = 0.0, c = 0.0, u;
  int32_t k = 1, hu = 0;
  const int32_t hx = fd_hi(x), ax = hx & 0x7fffffff;
  if (hx < 0x3FDA827A) {  // x < 0.41422
    if (ax >= 0x3ff00000) return x == -1.0 ? -__builtin_inf() : __builtin_nan("");
    if (ax < 0x3e200000) {  // |x| < 2**-29
      if (ax < 0x3c900000) return x;
      return x - x * x * 0.5;
    }
    if (hx > 0 || hx <= (int32_t)0xbfd2bec3) {  // -0.2929 < x < 0.41422
      k = 0;
      f = x;
      hu = 1;
    }
  } else if (hx >= 0x7ff00000) {
    return x + x;
  }
  if (k != 0) {
    if (hx < 0x43400000) {
      u = 1.0 + x;
      hu = fd_hi(u);
      k = (hu >> 20) - 1023;
      c = (k > 0) ? 1.0 - (u - x) : x - (u - 1.0);
      c /= u;
    } else {
      u = x;
      hu = fd_hi(u);
      k = (hu >> 20) - 1023;
      c = 0;
    }
    hu &= 0x000fffff;
    if (hu < 0x6a09e) {
      u = fd_sethi(u, hu | 0x3ff00000);
    } else {
      k += 1;
      u = fd_sethi(u, hu | 0x3fe00000);
      hu = (0x00100000 - hu) >> 2;
    }
    f = u - 1.0;
  }
  const double hfsq = 0.5 * f * f;
  if (hu == 0) {  // |f| < 2**-20
    if (f == 0.0) {
      if (k == 0) return 0.0;
      c += k * ln2_lo;
      return k * ln2_hi + c;
    }
    const double R = hfsq * (1.0 - 0.66666666666666666 * f);
    if (k == 0) return f - R;
    return k * ln2_hi - ((R - (k * ln2_lo + c)) - f);
  }
  const double s = f / (2.0 + f), z = s * s;
  const double R1 = z * Lp1, z2 = z * z, R2 = Lp2 + z * Lp3, z4 = z2 * z2, R3 = Lp4 + z * Lp5, z6 = z4 * z2,
               R4 = Lp6 + z * Lp7;
  const double R = R1 + z2 * R2 + z4 * R3 + z6 * R4;
  if (k == 0) return f - (hfsq - s * (hfsq + R));
  return k * ln2_hi - ((hfsq - (s * (hfsq + R) + (k * ln2_lo + c))) - f);
}

}  // namespace ssim
