/*
 * aero_math.h — the libm the demod kernels call, bit-for-bit the glibc 2.35
 * that the reference links, as an x86-64 host with FMA + AVX2 resolves it
 * (the decode/ sources call std::abs on complex -> hypot, std::arg -> atan2,
 * tanh, cos/sin pairs -> sincos, std::exp(i x) -> cexp -> sincos, log10).
 *
 * Compiles for host (g++/hipcc host pass) and device (gfx950).  Every file
 * that includes it must be built with -ffp-contract=off: the fused
 * multiply-adds are the explicit fma() calls, placed exactly where glibc's
 * FMA build has a vfmadd (atan2, log) and nowhere else (sincos, hypot,
 * tanh are glibc's SSE2 code, no fusion).  Constants and tables come from
 * the host libm itself (aero_glibc_tables.h, tools/gen_glibc_tables.cpp).
 *
 *  aero_hypot  : glibc 2.35 dbl-64 e_hypot.c (non-FMA kernel)
 *  aero_tanh   : fdlibm s_tanh.c on glibc's s_expm1.c (Estrin-form polynomial)
 *  aero_sincos : glibc s_sincos.c with s_sin.c's do_sin / do_cos /
 *                reduce_sincos (SSE2 build, the only sincos in 2.35's libm)
 *  aero_atan2  : __atan2_fma (e_atan2.c without its removed slow paths)
 *  aero_log    : __log_fma (e_log.c, ARM optimized-routines log, 128-entry
 *                table), aero_log10 the e_log10.c wrapper around it
 * tests/test_math_host.py checks every one bitwise against the host glibc;
 * tests/test_gpu_math.py checks the device build against the host build.
 *
 * License: these functions restate the GNU C Library's (glibc 2.35) math
 * routines -- e_atan2.c, s_sin.c / s_sincos.c, e_log.c / e_log10.c,
 * e_hypot.c, s_tanh.c / s_expm1.c (the last from Sun's fdlibm) -- and are a
 * derivative work of them.  The GNU C Library is free software; you can
 * redistribute it and/or modify it under the terms of the GNU Lesser General
 * Public License as published by the Free Software Foundation; either version
 * 2.1 of the License, or (at your option) any later version.  It is
 * distributed WITHOUT ANY WARRANTY; without even the implied warranty of
 * MERCHANTABILITY or FITNESS FOR A PARTICULAR PURPOSE.  See the GNU Lesser
 * General Public License for more details.  Portions: Copyright (C)
 * 1991-2022 Free Software Foundation, Inc.; IBM Accurate Mathematical
 * Library, Copyright (C) 2001-2022 Free Software Foundation, Inc.; ARM
 * optimized-routines log, Copyright (c) 2018 Arm Ltd.; fdlibm, Copyright
 * (C) 1993 by Sun Microsystems, Inc. (permission to use, copy, modify and
 * distribute this software is freely granted, provided that this notice is
 * preserved).
 */
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define AERO_HD __host__ __device__ __forceinline__
#define AERO_TABLE_DECL static __host__ __device__ constexpr
#else
#include <math.h>
#define AERO_HD static inline
#define AERO_TABLE_DECL static constexpr
#endif

#include "aero_glibc_tables.h"

namespace aero {

AERO_HD uint64_t d2u(double x) { return __builtin_bit_cast(uint64_t, x); }
AERO_HD double u2d(uint64_t u) { return __builtin_bit_cast(double, u); }
AERO_HD uint32_t hiw(double x) { return (uint32_t)(d2u(x) >> 32); }
AERO_HD uint32_t low(double x) { return (uint32_t)d2u(x); }
AERO_HD double sethi(double x, uint32_t hi) {
  return u2d((d2u(x) & 0xffffffffULL) | ((uint64_t)hi << 32));
}
AERO_HD double mkd(uint32_t hi, uint32_t lo) { return u2d(((uint64_t)hi << 32) | lo); }

/* ----------------------------------------------------- IEEE division
 * The same correctly rounded quotient as the `/` the compiler emits, in
 * fewer dependent operations, for operands whose range the caller knows
 * (host: the plain division):
 *
 *  div_c(a, c)     a / c for a compile-time constant c: q0 = RN(a rc) with
 *                  rc = RN(1/c) folded by the compiler, the residual a - c q0
 *                  exact by fma, q = RN(q0 + r rc) = RN(a / c) (Markstein's
 *                  theorem: rc within half an ulp of 1/c, q0 within one ulp
 *                  of a/c, no underflow).  3 dependent operations instead of
 *                  the 10 of a division; a power-of-two c is one product.
 *  rcp_div(b)      v_rcp_f64 and the two Newton steps of the compiler's f64
 *  div_r(a, b, r)  division, then its final q = a r, r' = a - b q, q + r' r:
 *                  that sequence instruction for instruction without
 *                  v_div_scale (the identity when b and 1/b are normal, the
 *                  quotient is normal and a's exponent exceeds -970) and
 *                  v_div_fixup (the identity for a finite nonzero quotient);
 *                  two divisions by one b share the reciprocal.
 *
 * Contract, argued at every call site: a is zero (its signed zero quotient
 * is selected, as IEEE gives) or |a| >= 2^-969 and the quotient is normal,
 * or the caller's next step absorbs any tiny quotient (a max with a floor,
 * a sum with a phase pointer).  No branch: a guarded version split the
 * demods' basic blocks and cost more than it saved.  tests/test_gpu_math.py
 * compares them with the IEEE division on the device. */
AERO_HD double div_c(double a, double c) {
#if defined(__HIP_DEVICE_COMPILE__)
  const double rc = 1.0 / c;  // folded: c is a literal at every call site
  if ((d2u(c) & 0x000fffffffffffffULL) == 0) return a * rc;  // a power of two: exact product (folded)
  const double q0 = a * rc;
  const double q = fma(fma(-c, q0, a), rc, q0);
  return a == 0.0 ? q0 : q;
#else
  return a / c;
#endif
}

/* div_c behind a wave-uniform test of its contract (every lane's numerator
 * zero or at least 2^-900 in magnitude), the IEEE division otherwise: for
 * numerators whose range is not argued, e.g. 360 x a phase pointer */
AERO_HD double div_cw(double a, double c) {
#if defined(__HIP_DEVICE_COMPILE__)
  const double m = __builtin_fabs(a);
  if (__builtin_expect(__all(m == 0.0 || m >= 0x1p-900), 1)) return div_c(a, c);
#endif
  return a / c;
}

AERO_HD double rcp_div(double b) {
#if defined(__HIP_DEVICE_COMPILE__)
  double r = __builtin_amdgcn_rcp(b);
  r = fma(r, fma(-b, r, 1.0), r);
  r = fma(r, fma(-b, r, 1.0), r);
  return r;
#else
  return 1.0 / b;  // unused on the host (div_r divides)
#endif
}

AERO_HD double div_r(double a, double b, double r) {
#if defined(__HIP_DEVICE_COMPILE__)
  const double q = a * r;  // a zero quotient keeps a r's sign, as IEEE 0 / b
  const double f = fma(fma(-b, q, a), r, q);
  return a == 0.0 ? q : f;
#else
  (void)r;
  return a / b;
#endif
}

AERO_HD double div_n(double a, double b) { return div_r(a, b, rcp_div(b)); }

/* ------------------------------------------------------------- hypot */
AERO_HD double hypot_kernel(double ax, double ay) {
  double t1, t2;
  double h = sqrt(ax * ax + ay * ay);
  if (h <= 2.0 * ay) {
    double delta = h - ay;
    t1 = ax * (2.0 * delta - ax);
    t2 = (delta - 2.0 * (ax - ay)) * delta;
  } else {
    double delta = h - ax;
    t1 = 2.0 * delta * (ax - 2.0 * ay);
    t2 = (4.0 * delta - ay) * ay + delta * delta;
  }
  h -= (t1 + t2) / (2.0 * h);
  return h;
}

AERO_HD double aero_hypot(double x, double y) {
  if (!__builtin_isfinite(x) || !__builtin_isfinite(y)) {
    if (__builtin_isinf(x) || __builtin_isinf(y)) return __builtin_inf();
    return x + y;
  }
  x = __builtin_fabs(x);
  y = __builtin_fabs(y);
  double ax = x < y ? y : x;
  double ay = x < y ? x : y;
  const double SCALE = 0x1p-600, LARGE_VAL = 0x1p+511, TINY_VAL = 0x1p-511, EPS = 0x1p-54;
  if (ax > LARGE_VAL) {
    if (ay <= ax * EPS) return ax + ay;
    return hypot_kernel(ax * SCALE, ay * SCALE) / SCALE;
  }
  if (ay < TINY_VAL) {
    if (ax >= ay / EPS) return ax + ay;
    return hypot_kernel(ax / SCALE, ay / SCALE) * SCALE;
  }
  if (ay <= ax * EPS) return ax + ay;
  return hypot_kernel(ax, ay);
}

/* aero_hypot for finite x, y with max(|x|, |y|) in [2^-200, 2^200], without
 * a branch (callers check the range for a whole wave and fall back to
 * aero_hypot otherwise): there glibc takes neither scaling path, the sum of
 * squares needs no sqrt range scaling, and the correction's quotient
 * (t1 + t2) / (2h) is zero or at least 2^-560 in magnitude (t1 + t2 is a
 * multiple of ulp(ay^2 / 4) >= 2^-562 unless ay <= ax 2^-54, whose kernel
 * result is discarded), so the division sequence needs neither v_div_scale
 * nor v_div_fixup.  Both sides of the kernel's h <= 2ay test are evaluated
 * and selected, as the wave executes both anyway when its lanes differ. */
AERO_HD double aero_hypot_nr(double x, double y) {
#if defined(__HIP_DEVICE_COMPILE__)
  x = __builtin_fabs(x);
  y = __builtin_fabs(y);
  const double ax = x < y ? y : x, ay = x < y ? x : y;
  const double s = ax * ax + ay * ay;
  const double rs = __builtin_amdgcn_rsq(s);
  double g = s * rs, hh = rs * 0.5;
  const double r0 = fma(-hh, g, 0.5);
  g = fma(g, r0, g);
  hh = fma(hh, r0, hh);
  g = fma(fma(-g, g, s), hh, g);
  const double h = fma(fma(-g, g, s), hh, g);  // sqrt(s), the compiler's sequence
  const double d1 = h - ay, d2 = h - ax;
  const double t1a = ax * (2.0 * d1 - ax), t2a = (d1 - 2.0 * (ax - ay)) * d1;
  const double t1b = 2.0 * d2 * (ax - 2.0 * ay), t2b = (4.0 * d2 - ay) * ay + d2 * d2;
  const bool near = h <= 2.0 * ay;
  const double num = (near ? t1a : t1b) + (near ? t2a : t2b), den = 2.0 * h;
  double r = __builtin_amdgcn_rcp(den);
  r = fma(r, fma(-den, r, 1.0), r);
  r = fma(r, fma(-den, r, 1.0), r);
  const double q0 = num * r;
  const double q = num == 0.0 ? q0 : fma(fma(-den, q0, num), r, q0);
  return ay <= ax * 0x1p-54 ? ax + ay : h - q;
#else
  return aero_hypot(x, y);
#endif
}

/* aero_hypot with aero_hypot_nr when every active lane of the wave is in its
 * range (one uniform branch), the general code otherwise */
AERO_HD double aero_hypot_w(double x, double y) {
#if defined(__HIP_DEVICE_COMPILE__)
  const double a = __builtin_fabs(x), b = __builtin_fabs(y);
  const bool nr = a <= 0x1p200 && b <= 0x1p200 && (a >= 0x1p-200 || b >= 0x1p-200);
  if (__builtin_expect(__all(nr), 1)) return aero_hypot_nr(x, y);
#endif
  return aero_hypot(x, y);
}

/* ------------------------------------------------------ expm1 / tanh */
AERO_HD double aero_expm1(double x) {
  const double o_threshold = 7.09782712893383973096e+02, ln2_hi = 6.93147180369123816490e-01,
               ln2_lo = 1.90821492927058770002e-10, invln2 = 1.44269504088896338700e+00,
               Q1 = -3.33333333333331316428e-02, Q2 = 1.58730158725481460165e-03,
               Q3 = -7.93650757867487942473e-05, Q4 = 4.00821782732936239552e-06,
               Q5 = -2.01099218183624371326e-07;
  double y, hi, lo, c = 0, t, e, hxs, hfx, r1, h2, h4, R1, R2, R3;
  int32_t k;
  uint32_t hx = hiw(x);
  uint32_t xsb = hx & 0x80000000u;
  hx &= 0x7fffffffu;
  if (hx >= 0x4043687Au) {
    if (hx >= 0x40862E42u) {
      if (hx >= 0x7ff00000u) {
        if (((hx & 0xfffffu) | low(x)) != 0) return x + x;
        return (xsb == 0) ? x : -1.0;
      }
      if (x > o_threshold) return __builtin_inf();
    }
    if (xsb != 0) return -1.0;
  }
  if (hx > 0x3fd62e42u) {
    if (hx < 0x3FF0A2B2u) {
      if (xsb == 0) {
        hi = x - ln2_hi;
        lo = ln2_lo;
        k = 1;
      } else {
        hi = x + ln2_hi;
        lo = -ln2_lo;
        k = -1;
      }
    } else {
      k = (int32_t)(invln2 * x + ((xsb == 0) ? 0.5 : -0.5));
      t = k;
      hi = x - t * ln2_hi;
      lo = t * ln2_lo;
    }
    x = hi - lo;
    c = (hi - x) - lo;
  } else if (hx < 0x3c900000u) {
    return x;
  } else {
    k = 0;
  }
  hfx = 0.5 * x;
  hxs = x * hfx;
  R1 = 1.0 + hxs * Q1;
  h2 = hxs * hxs;
  R2 = Q2 + hxs * Q3;
  h4 = h2 * h2;
  R3 = Q4 + hxs * Q5;
  r1 = R1 + h2 * R2 + h4 * R3;
  t = 3.0 - r1 * hfx;
  e = hxs * ((r1 - t) / (6.0 - x * t));
  if (k == 0) return x - (x * e - hxs);
  e = (x * (e - c) - c);
  e -= hxs;
  if (k == -1) return 0.5 * (x - e) - 0.5;
  if (k == 1) {
    if (x < -0.25) return -2.0 * (e - (x + 0.5));
    return 1.0 + 2.0 * (x - e);
  }
  if (k <= -2 || k > 56) {
    y = 1.0 - (e - x);
    if (k == 1024)
      y = y * 2.0 * 0x1p1023;
    else
      y = sethi(y, hiw(y) + ((uint32_t)k << 20));
    return y - 1.0;
  }
  if (k < 20) {
    t = mkd(0x3ff00000u - (0x200000u >> k), 0);
    y = t - (e - x);
    y = sethi(y, hiw(y) + ((uint32_t)k << 20));
  } else {
    t = mkd((uint32_t)((0x3ff - k) << 20), 0);
    y = x - (e + t);
    y += 1.0;
    y = sethi(y, hiw(y) + ((uint32_t)k << 20));
  }
  return y;
}

AERO_HD double aero_tanh(double x) {
  double t, z;
  int32_t jx = (int32_t)hiw(x), ix = jx & 0x7fffffff;
  if (ix >= 0x7ff00000) {
    if (jx >= 0) return 1.0 / x + 1.0;
    return 1.0 / x - 1.0;
  }
  if (ix < 0x40360000) {
    if ((ix | (int32_t)low(x)) == 0) return x;
    if (ix < 0x3c800000) return x * (1.0 + x);
    if (ix >= 0x3ff00000) {
      t = aero_expm1(2.0 * __builtin_fabs(x));
      z = 1.0 - 2.0 / (t + 2.0);
    } else {
      t = aero_expm1(-2.0 * __builtin_fabs(x));
      z = -t / (t + 2.0);
    }
  } else {
    z = 1.0 - 1e-300;
  }
  return (jx >= 0) ? z : -z;
}

/* The branch-free forms' fallbacks (a wave with an out-of-range lane): inline
 * by default; AERO_X_COLD (timing builds) calls them out of line instead */
#if defined(__HIP_DEVICE_COMPILE__) && defined(AERO_X_COLD)
#define AERO_COLD __device__ __noinline__
#else
#define AERO_COLD AERO_HD
#endif
AERO_COLD double aero_tanh_cold(double x) { return aero_tanh(x); }

/* aero_expm1 on the arguments aero_tanh gives it for 2^-55 <= |x| < 22:
 * a = 2|x| in [2, 44) or a = -2|x| in (-2, -2^-54], without a branch.  There
 * glibc returns none of its early values, and k is 0 (|a| <= 0x3fd62e42's
 * binade bound), -1 (forced, |a| below 0x3ff0a2b2), or (int)(a/ln2 -+ 1/2)
 * in {-3, -2, -1} and [3, 63]; its k = 1 case needs a positive a < 1.04 and
 * does not occur.  One reduction serves every k: t = k gives x - t ln2_hi =
 * x -+ ln2_hi and t ln2_lo = +-ln2_lo bit for bit for the forced k = +-1, and
 * x - 0 = x, c = (x - x) - 0 = +0 for k = 0, which is what glibc's
 * unreduced path holds.  The tail's five forms are evaluated side by side and
 * selected.  (r1 - t) / (6 - x t) is a division by div_n: the numerator is
 * about -2 and the divisor about 6 for every reduced x (|x| <= 0.35), inside
 * its contract. */
AERO_HD double g_expm1_tanh_bf(double x) {
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
               invln2 = 1.44269504088896338700e+00, Q1 = -3.33333333333331316428e-02,
               Q2 = 1.58730158725481460165e-03, Q3 = -7.93650757867487942473e-05,
               Q4 = 4.00821782732936239552e-06, Q5 = -2.01099218183624371326e-07;
  const uint32_t hx0 = hiw(x), xsb = hx0 & 0x80000000u, hx = hx0 & 0x7fffffffu;
  int32_t k = (int32_t)(invln2 * x + ((xsb == 0) ? 0.5 : -0.5));
  k = hx < 0x3FF0A2B2u ? ((xsb == 0) ? 1 : -1) : k;
  k = hx > 0x3fd62e42u ? k : 0;
  const double tk = k;
  const double hi = x - tk * ln2_hi, lo = tk * ln2_lo;
  x = hi - lo;
  const double c = (hi - x) - lo;
  const double hfx = 0.5 * x;
  const double hxs = x * hfx;
  const double R1 = 1.0 + hxs * Q1;
  const double h2 = hxs * hxs;
  const double R2 = Q2 + hxs * Q3;
  const double h4 = h2 * h2;
  const double R3 = Q4 + hxs * Q5;
  const double r1 = R1 + h2 * R2 + h4 * R3;
  const double t = 3.0 - r1 * hfx;
  const double e = hxs * div_n(r1 - t, 6.0 - x * t);
  const double r_k0 = x - (x * e - hxs);
  double e2 = (x * (e - c) - c);
  e2 -= hxs;
  const double r_m1 = 0.5 * (x - e2) - 0.5;
  const uint32_t kup = (uint32_t)k << 20;
  double yb = 1.0 - (e2 - x);
  yb = sethi(yb, hiw(yb) + kup);
  const double r_far = yb - 1.0;  // k <= -2 or k > 56 (k == 1024 does not occur)
  const int32_t ks = k < 0 ? 0 : (k > 19 ? 19 : k);  // the shift's count where it is selected
  double y1 = mkd(0x3ff00000u - (0x200000u >> ks), 0) - (e2 - x);
  y1 = sethi(y1, hiw(y1) + kup);  // 3 <= k < 20
  double y2 = x - (e2 + mkd((uint32_t)((0x3ff - k) << 20), 0));
  y2 += 1.0;
  y2 = sethi(y2, hiw(y2) + kup);  // 20 <= k <= 56
  return k == 0 ? r_k0 : (k == -1 ? r_m1 : ((k <= -2 || k > 56) ? r_far : (k < 20 ? y1 : y2)));
}

/* aero_tanh without branches when every active lane of the wave has
 * 2^-55 <= |x| < 22 (the demods' soft values, |x| < 4); the general code
 * otherwise.  Its two forms share one expm1 and one division:
 * 1 - 2 / (t + 2) with t = expm1(2|x|) for |x| >= 1, -t / (t + 2) with
 * t = expm1(-2|x|) below; both quotients are in div_r's contract (t + 2 in
 * (1.13, 2) or >= 8.3, the numerator 2 or |t| >= 2^-54). */
AERO_HD double aero_tanh_bf(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
  const int32_t jx = (int32_t)hiw(x), ix = jx & 0x7fffffff;
  const bool ok = ix < 0x40360000 && ix >= 0x3c800000;
  if (!__builtin_expect(__all(ok), 1)) return aero_tanh_cold(x);
  const bool big = ix >= 0x3ff00000;
  const double ax = __builtin_fabs(x);
  const double t = g_expm1_tanh_bf(big ? 2.0 * ax : -2.0 * ax);
  const double d = t + 2.0;
  const double q = div_r(big ? 2.0 : -t, d, rcp_div(d));
  const double z = big ? 1.0 - q : q;
  return (jx >= 0) ? z : -z;
#else
  return aero_tanh(x);
#endif
}

/* ------------------------------------------------------------ sincos
 * glibc 2.35 sincos (sysdeps/ieee754/dbl-64/s_sincos.c + the do_sin /
 * do_cos / reduce_sincos helpers of s_sin.c), SSE2 build: libm.so.6's
 * `sincos` is not an ifunc in 2.35, so every host runs this code.  Read
 * from its disassembly; the operation order below is the instructions'.
 * |x| >= 105414350 goes through __branred (g_branred), as glibc's does; the
 * demods' arguments never get there (loop corrections, |x| < 2 pi). */

/* TAYLOR_SIN(xx, a, da) */
AERO_HD double g_taylor_sin(double xx, double a, double da) {
  double p = AERO_G_S5 * xx + AERO_G_S4;
  p = p * xx - AERO_G_NS3;
  p = p * xx + AERO_G_S2;
  p = p * xx - AERO_G_NS1;
  const double t = (p * a - AERO_G_CS2 * da) * xx + da;
  return t + a;
}

AERO_HD double g_do_sin(double x, double dx, const double *sct) {
  if (__builtin_fabs(x) < 0.126) return g_taylor_sin(x * x, x, dx);
  const double xold = x;
  if (x <= 0) dx = -dx;
  const double u = AERO_G_BIG + __builtin_fabs(x);
  x = __builtin_fabs(x) - (u - AERO_G_BIG);
  const double xx = x * x;
  const double s = x + (dx + (x * xx) * (xx * AERO_G_SN5 - AERO_G_NSN3));
  const double c = x * dx + xx * ((xx * AERO_G_CS6 - AERO_G_NCS4) * xx + AERO_G_CS2);
  const int k = (int)(low(u) << 2);
  const double sn = sct[k], ssn = sct[k + 1], cs = sct[k + 2], ccs = sct[k + 3];
  const double cor = (ssn + s * ccs - sn * c) + cs * s;
  return __builtin_copysign(sn + cor, xold);
}

AERO_HD double g_do_cos(double x, double dx, const double *sct) {
  if (x < 0) dx = -dx;
  const double u = AERO_G_BIG + __builtin_fabs(x);
  x = __builtin_fabs(x) - (u - AERO_G_BIG) + dx;
  const double xx = x * x;
  const double s = x + (x * xx) * (xx * AERO_G_SN5 - AERO_G_NSN3);
  const double c = xx * ((xx * AERO_G_CS6 - AERO_G_NCS4) * xx + AERO_G_CS2);
  const int k = (int)(low(u) << 2);
  const double sn = sct[k], ssn = sct[k + 1], cs = sct[k + 2], ccs = sct[k + 3];
  const double cor = (ccs - s * ssn - cs * c) - sn * s;
  return cs + cor;
}

AERO_HD int g_reduce_sincos(double x, double &a, double &da) {
  const double t = x * AERO_G_HPINV + AERO_G_TOINT;
  const double xn = t - AERO_G_TOINT;
  const double y = (x - xn * AERO_G_MP1) - xn * AERO_G_MP2;
  const int n = (int)(low(t) & 3);
  double t1 = xn * AERO_G_PP3;
  const double t2 = y - t1;
  double db = (y - t2) - t1;
  t1 = xn * AERO_G_PP4;
  const double b = t2 - t1;
  db += (t2 - b) - t1;
  a = b;
  da = db;
  return n;
}

/* __branred (branred.c): x = N pi/2 + (a + aa) for |x| >= 105414350, N mod
 * 4 returned; x scaled by 2^-600 and split into two 26-bit halves, each
 * multiplied by 2/pi in 24-bit digits (toverp) from the digit its exponent
 * needs, the integer parts removed (+- big), the halves' fractions summed,
 * and the fraction times pi/2 in double-double.  Restated from the SSE2
 * build's disassembly (libm 0x6f180, called by sincos): its packed ops are
 * these operations two at a time; additions and products are commutative,
 * and every grouping below is the one its instruction sequence has. */
AERO_HD int g_branred(double x, double &a, double &aa) {
  x *= AERO_G_BR_TM600;
  double t = x * AERO_G_BR_SPLIT;
  const double xs[2] = {t - (t - x), 0.0};
  double hb[2], hbb[2], hsum[2];
  const double x2 = x - xs[0];
  for (int h = 0; h < 2; h++) {
    const double xh = h ? x2 : xs[0];
    int k = (int)((d2u(xh) >> 52) & 2047);
    k = (k - 450) / 24;
    if (k < 0) k = 0;
    double gor = mkd(0x63f00000u - ((uint32_t)(k * 24) << 20), 0);
    double r[6];
    for (int i = 0; i < 6; i++) {
      r[i] = xh * aero_g_toverp[k + i] * gor;
      gor *= AERO_G_BR_TM24;
    }
    double sum = 0, s;
    for (int i = 0; i < 3; i++) {
      s = (r[i] + AERO_G_BR_BIG) - AERO_G_BR_BIG;
      sum += s;
      r[i] -= s;
    }
    t = 0;
    for (int i = 0; i < 6; i++) t += r[5 - i];
    double bb = (((((r[0] - t) + r[1]) + r[2]) + r[3]) + r[4]) + r[5];
    s = (t + AERO_G_BR_BIG) - AERO_G_BR_BIG;
    sum += s;
    t -= s;
    const double b = t + bb;
    bb = (t - b) + bb;
    s = (sum + AERO_G_BR_BIG1) - AERO_G_BR_BIG1;
    sum -= s;
    hb[h] = b;
    hbb[h] = bb;
    hsum[h] = sum;
  }
  const double b1 = hb[0], bb1 = hbb[0], b2 = hb[1], bb2 = hbb[1];
  double sum = hsum[0] + hsum[1];
  double b = b1 + b2;
  double bb = (__builtin_fabs(b1) > __builtin_fabs(b2)) ? (b1 - b) + b2 : (b2 - b) + b1;
  if (b > 0.5) {
    b -= 1.0;
    sum += 1.0;
  } else if (b < -0.5) {
    b += 1.0;
    sum -= 1.0;
  }
  double s = b + (bb + bb1 + bb2);
  t = ((b - s) + bb) + (bb1 + bb2);
  b = s * AERO_G_BR_SPLIT;
  const double t1 = b - (b - s), t2 = s - t1;
  b = s * AERO_G_HPI;
  bb = (((t1 * AERO_G_MP1 - b) + t1 * AERO_G_BR_MP2) + t2 * AERO_G_MP1) +
       (t2 * AERO_G_BR_MP2 + s * AERO_G_HP1 + t * AERO_G_HPI);
  s = b + bb;
  t = (b - s) + bb;
  a = s;
  aa = t;
  return ((int)sum) & 3;
}

/* sct: __sincostab (aero_g_sincostab, 440 doubles) or a copy of it, e.g. in
 * LDS (aero_sincos_t); the results do not depend on where it lives */
AERO_HD void aero_sincos_t(double x, double &so, double &co, const double *sct) {
  const uint32_t k = hiw(x) & 0x7fffffffu;
  if (k < 0x400368fdu) {
    if (k < 0x3e400000u) {
      so = x;
      co = 1.0;
    } else if (k < 0x3feb6000u) {
      so = g_do_sin(x, 0.0, sct);
      co = g_do_cos(x, 0.0, sct);
    } else {
      const double y = AERO_G_HPI - __builtin_fabs(x);
      const double a = y + AERO_G_HP1;
      const double da = (y - a) + AERO_G_HP1;
      so = __builtin_copysign(g_do_cos(a, da, sct), x);
      co = g_do_sin(a, da, sct);
    }
    return;
  }
  if (k < 0x7ff00000u) {
    double a, da;
    const int n = k < 0x419921fbu ? g_reduce_sincos(x, a, da) : g_branred(x, a, da);
    if ((unsigned)(n - 1) <= 1u) {
      a = -a;
      da = -da;
    }
    const double s = g_do_sin(a, da, sct);
    double c = g_do_cos(a, da, sct);
    if (n & 2) c = -c;
    if (n & 1) {
      so = c;
      co = s;
    } else {
      so = s;
      co = c;
    }
    return;
  }
  so = co = x / x;
}
AERO_COLD void aero_sincos_cold(double x, double &so, double &co, const double *sct) { aero_sincos_t(x, so, co, sct); }

AERO_HD void aero_sincos(double x, double &so, double &co) { aero_sincos_t(x, so, co, aero_g_sincostab); }

/* aero_sincos_t without branches when every active lane of the wave has
 * |x| < 0.855469 (hi word below 0x3feb6000: the loop corrections and
 * rotator frequencies of the demods); the general code otherwise.  There
 * sincos is (x, 1) below 2^-27 and (do_sin(x, 0), do_cos(x, 0)) above, and
 * do_sin is the Taylor form below 0.126 and the table form above: all four
 * are evaluated and selected, the two table forms on the one row of
 * u = BIG + |x|. */
AERO_HD void aero_sincos_bf(double x, double &so, double &co, const double *sct) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t k = hiw(x) & 0x7fffffffu;
  if (!__builtin_expect(__all(k < 0x3feb6000u), 1)) {
    aero_sincos_cold(x, so, co, sct);
    return;
  }
  const double ax = __builtin_fabs(x);
  const double s_tay = g_taylor_sin(x * x, x, 0.0);
  const double dxs = x <= 0 ? -0.0 : 0.0;  // do_sin's dx = -dx for x <= 0
  const double u = AERO_G_BIG + ax;
  const double xs = ax - (u - AERO_G_BIG);
  const double xxs = xs * xs;
  const double ss = xs + (dxs + (xs * xxs) * (xxs * AERO_G_SN5 - AERO_G_NSN3));
  const double cs_ = xs * dxs + xxs * ((xxs * AERO_G_CS6 - AERO_G_NCS4) * xxs + AERO_G_CS2);
  const int row = (int)(low(u) << 2);
  const double sn = sct[row], ssn = sct[row + 1], cs = sct[row + 2], ccs = sct[row + 3];
  const double cor_s = (ssn + ss * ccs - sn * cs_) + cs * ss;
  const double s_tab = __builtin_copysign(sn + cor_s, x);
  // do_cos(x, 0): dx = -0 for x < 0, added to the reduced argument
  const double dxc = x < 0 ? -0.0 : 0.0;
  const double xc = ax - (u - AERO_G_BIG) + dxc;
  const double xxc = xc * xc;
  const double sc = xc + (xc * xxc) * (xxc * AERO_G_SN5 - AERO_G_NSN3);
  const double cc = xxc * ((xxc * AERO_G_CS6 - AERO_G_NCS4) * xxc + AERO_G_CS2);
  const double cor_c = (ccs - sc * ssn - cs * cc) - sn * sc;
  const double c_tab = cs + cor_c;
  const bool tiny = k < 0x3e400000u;
  so = tiny ? x : (ax < 0.126 ? s_tay : s_tab);
  co = tiny ? 1.0 : c_tab;
#else
  aero_sincos_t(x, so, co, sct);
#endif
}

AERO_HD double aero_sin(double x) {
  double s, c;
  aero_sincos(x, s, c);
  return s;
}
AERO_HD double aero_cos(double x) {
  double s, c;
  aero_sincos(x, s, c);
  return c;
}

/* ------------------------------------------------------------- atan2
 * glibc 2.35 __atan2_fma (sysdeps/ieee754/dbl-64/e_atan2.c built with
 * -mfma -mavx2, the ifunc target on FMA + AVX2 hosts; the multi-precision
 * slow paths were removed before 2.35).  Restated from its disassembly:
 * every fma() below is a vfmadd/vfmsub/vfnmadd there, every other product
 * and sum a separate rounding.  The x87-free SET_RESTORE_ROUND has no effect
 * in round-to-nearest. */
AERO_HD double g_atan2_poly(double v) {  // d3 + v (d5 + v (d7 + v (d9 + v (d11 + v d13))))
  double p = fma(v, AERO_G_D13, AERO_G_D11);
  p = fma(v, p, AERO_G_D9);
  p = fma(v, p, AERO_G_D7);
  p = fma(v, p, AERO_G_D5);
  return fma(v, p, AERO_G_D3);
}
AERO_HD int g_atan2_row(double u) { return (int)(fma(u, AERO_G_TWO8, AERO_G_TWO52) - AERO_G_TWO52) - 16; }
AERO_HD double g_atan2_tail(const double *c, double v) {  // c2 + v (c3 + v (c4 + v (c5 + v c6)))
  double p = fma(v, c[6], c[5]);
  p = fma(v, p, c[4]);
  p = fma(v, p, c[3]);
  return fma(v, p, c[2]);
}

/* cij: uatan2.tbl's cij[241][7] (aero_g_cij) or a copy of it, e.g. in LDS */
AERO_HD double aero_atan2_t(double y, double x, const double (*cij)[7]) {
  const uint32_t ux = hiw(x), dx = low(x), uy = hiw(y), dy = low(y);
  if ((ux & 0x7ff00000u) == 0x7ff00000u && ((ux & 0xfffffu) | dx) != 0) return x + y;
  if ((uy & 0x7ff00000u) == 0x7ff00000u && ((uy & 0xfffffu) | dy) != 0) return y + y;
  if (uy == 0 && dy == 0) return ((int32_t)ux < 0) ? AERO_G_OPI : 0.0;
  if (uy == 0x80000000u && dy == 0) return ((int32_t)ux < 0) ? AERO_G_MOPI : -0.0;
  if (x == 0) return ((int32_t)uy < 0) ? AERO_G_MHPI : AERO_G_HPI;
  bool special = true;  // the infinite cases; a y with dy != 0 there is a NaN (above)
  if (ux == 0x7ff00000u && dx == 0) {
    if (uy == 0x7ff00000u) {
      if (dy == 0) return AERO_G_QPI;
    } else if (uy == 0xfff00000u) {
      if (dy == 0) return AERO_G_MQPI;
    } else {
      return ((int32_t)uy < 0) ? -0.0 : 0.0;
    }
    special = false;
  } else if (ux == 0xfff00000u && dx == 0) {
    if (uy == 0x7ff00000u) {
      if (dy == 0) return AERO_G_TQPI;
    } else if (uy == 0xfff00000u) {
      if (dy == 0) return AERO_G_MTQPI;
    } else {
      return ((int32_t)uy < 0) ? AERO_G_MOPI : AERO_G_OPI;
    }
    special = false;
  }
  if (special) {
    if (uy == 0x7ff00000u) {
      if (dy == 0) return AERO_G_HPI;
    } else if (uy == 0xfff00000u && dy == 0) {
      return AERO_G_MHPI;
    }
  }

  double ax = x < 0 ? -x : x, ay = y < 0 ? -y : y;
  const int32_t de = (int32_t)((uy & 0x7ff00000u) - (ux & 0x7ff00000u));
  if (de >= 59768832) return (0 < y) ? AERO_G_HPI : AERO_G_MHPI;
  if (de <= -59768832) {
    if (!(x > 0)) return (0 < y) ? AERO_G_OPI : AERO_G_MOPI;
    return __builtin_copysign(ay / ax, y);
  }
  if (ax < AERO_G_TWOM500 || ay < AERO_G_TWOM500) {
    ax *= AERO_G_TWO500;
    ay *= AERO_G_TWO500;
  }
  if (ax > AERO_G_TWO500 || ay > AERO_G_TWO500) {
    ax *= AERO_G_TWOM500;
    ay *= AERO_G_TWOM500;
  }
  double u, du;
  {
    // u = a / b and du = ((a - v) - vv) / b: one reciprocal for both.  After
    // the early returns and the 2^+-500 scalings a, b are in [2^-574, 2^524]
    // within 57 binades, u in [2^-58, 1], and du's numerator (the exact
    // residual a - b u) is zero or at least a 2^-104, so div_r's contract
    // holds.
    const double a = ax > ay ? ay : ax, b = ax > ay ? ax : ay;
    const double r = rcp_div(b);
    u = div_r(a, b, r);
    const double v = b * u, vv = fma(b, u, -v);
    du = div_r((a - v) - vv, b, r);
  }
  double z;
  if (x > 0) {
    if (ax > ay) {  // atan(u)
      if (u < AERO_G_INV16) {
        const double v = u * u;
        const double zz = fma(u * v, g_atan2_poly(v), du);
        return __builtin_copysign(u + zz, y);
      }
      const double *c = cij[g_atan2_row(u)];
      const double t3 = u - c[0];
      const double v = t3 + du;
      const double dv = (__builtin_fabs(t3) > __builtin_fabs(du)) ? ((t3 - v) + du) : ((du - v) + t3);
      double p = fma(v, c[6], c[5]);
      p = fma(v, p, c[4]);
      p = fma(v, p, c[3]);
      const double zz = fma(v, c[2], fma(dv, c[2], (v * v) * p));
      return __builtin_copysign(zz + c[1], y);
    }
    // pi/2 - atan(u)
    if (u < AERO_G_INV16) {
      const double v = u * u;
      const double zz = (u * v) * g_atan2_poly(v);
      const double t = AERO_G_HPI - u;
      const double cor = (AERO_G_HPI > __builtin_fabs(u)) ? ((AERO_G_HPI - t) - u) : (AERO_G_HPI - (u + t));
      z = (((cor + AERO_G_HPI1) - du) - zz) + t;
    } else {
      const double *c = cij[g_atan2_row(u)];
      const double v = (u - c[0]) + du;
      z = (AERO_G_HPI - c[1]) + fma(-v, g_atan2_tail(c, v), AERO_G_HPI1);
    }
    return __builtin_copysign(__builtin_fabs(z), y);
  }
  if (ay > ax) {  // pi/2 + atan(u)
    if (u < AERO_G_INV16) {
      const double v = u * u;
      const double t = u + AERO_G_HPI;
      const double zz = (v * u) * g_atan2_poly(v);
      const double cor = (AERO_G_HPI > __builtin_fabs(u)) ? ((AERO_G_HPI - t) + u) : ((u - t) + AERO_G_HPI);
      z = (((cor + AERO_G_HPI1) + du) + zz) + t;
    } else {
      const double *c = cij[g_atan2_row(u)];
      const double v = (u - c[0]) + du;
      z = (AERO_G_HPI + c[1]) + fma(v, g_atan2_tail(c, v), AERO_G_HPI1);
    }
  } else {  // pi - atan(u)
    if (u < AERO_G_INV16) {
      const double v = u * u;
      const double zz = (v * u) * g_atan2_poly(v);
      const double t = AERO_G_OPI - u;
      const double cor = (AERO_G_OPI > __builtin_fabs(u)) ? ((AERO_G_OPI - t) - u) : (AERO_G_OPI - (t + u));
      z = (((cor + AERO_G_OPI1) - du) - zz) + t;
    } else {
      const double *c = cij[g_atan2_row(u)];
      const double v = (u - c[0]) + du;
      z = (AERO_G_OPI - c[1]) + fma(-v, g_atan2_tail(c, v), AERO_G_OPI1);
    }
  }
  return __builtin_copysign(__builtin_fabs(z), y);
}
AERO_COLD double aero_atan2_cold(double y, double x, const double (*cij)[7]) { return aero_atan2_t(y, x, cij); }

AERO_HD double aero_atan2(double y, double x) { return aero_atan2_t(y, x, aero_g_cij); }

/* aero_atan2_t without branches for the main path, when every active lane
 * of the wave has finite nonzero |x|, |y| in [2^-500, 2^500] within 56
 * binades of each other (no special case, no 2^+-500 scaling, none of the
 * extreme-ratio returns); the general code otherwise.  The main path's six
 * instruction sequences (x > 0 with |x| > |y|, or the pi/2 - , pi/2 + and
 * pi - forms; each with the small-ratio series or a table row) are the
 * ones aero_atan2_t runs, evaluated side by side and selected, because a
 * wave whose 64 channels spread over the quadrants would run them one
 * after another:
 *   - the three non-primary forms differ only in (K, K1, s) = (pi/2, hpi1,
 *     -1), (pi/2, hpi1, +1), (pi, opi1, -1): t = K + s u, cor = (K - t) + s u,
 *     z = (((cor + K1) + s du) + s zz) + t (series), z = (K + s c1) +
 *     fma(s v, P, K1) (table), where multiplying by s = +-1 is exact and
 *     x + (-y) is x - y bit for bit;
 *   - the table forms share v = (u - c0) + du and P = fma(v, p3, c2). */
AERO_HD double aero_atan2_bf(double y, double x, const double (*cij)[7]) {
#if defined(__HIP_DEVICE_COMPILE__)
  const double ax = __builtin_fabs(x), ay = __builtin_fabs(y);
  const int32_t de = (int32_t)((hiw(y) & 0x7ff00000u) - (hiw(x) & 0x7ff00000u));
  const bool ok = ax >= 0x1p-500 && ax <= 0x1p500 && ay >= 0x1p-500 && ay <= 0x1p500 && de < 59768832 &&
                  de > -59768832;
  if (!__builtin_expect(__all(ok), 1)) return aero_atan2_cold(y, x, cij);
  const bool gt = ax > ay;  // u = ay / ax, else u = ax / ay
  const double a = gt ? ay : ax, b = gt ? ax : ay;
  const double r = rcp_div(b);
  const double u = div_r(a, b, r);
  const double vb = b * u, vvb = fma(b, u, -vb);
  const double du = div_r((a - vb) - vvb, b, r);
  const bool pos = x > 0;
  const bool prim = pos && gt;
  const bool cpi = !pos && !(ay > ax);                 // pi - atan(u)
  const double K = cpi ? AERO_G_OPI : AERO_G_HPI, K1 = cpi ? AERO_G_OPI1 : AERO_G_HPI1;
  const double s = (!pos && ay > ax) ? 1.0 : -1.0;     // pi/2 + atan(u)
  // small-ratio series
  const double vs = u * u;
  const double poly = g_atan2_poly(vs);
  const double uv = u * vs;
  const double zp_s = u + fma(uv, poly, du);
  const double zz = uv * poly;
  const double ts = K + s * u;
  const double cor = (K - ts) + s * u;
  const double zg_s = (((cor + K1) + s * du) + s * zz) + ts;
  // table row
  int row = g_atan2_row(u);
  row = row < 0 ? 0 : row;  // u < 1/16: the row is not used
  const double *c = cij[row];
  const double t3 = u - c[0];
  const double v = t3 + du;
  const double dv = (__builtin_fabs(t3) > __builtin_fabs(du)) ? ((t3 - v) + du) : ((du - v) + t3);
  double p3 = fma(v, c[6], c[5]);
  p3 = fma(v, p3, c[4]);
  p3 = fma(v, p3, c[3]);
  const double zp_t = fma(v, c[2], fma(dv, c[2], (v * v) * p3)) + c[1];
  const double P = fma(v, p3, c[2]);
  const double zg_t = (K + s * c[1]) + fma(s * v, P, K1);
  const double z = u < AERO_G_INV16 ? (prim ? zp_s : zg_s) : (prim ? zp_t : zg_t);
  return __builtin_copysign(z, y);
#else
  return aero_atan2_t(y, x, cij);
#endif
}

/* --------------------------------------------------------------- log
 * glibc 2.35 __log_fma (sysdeps/ieee754/dbl-64/e_log.c built with -mfma
 * -mavx2: r = fma(z, invc, -1) and GCC's contractions, read from its
 * disassembly), the ifunc target the log10 wrapper calls on FMA hosts. */
AERO_HD double aero_log(double x) {
  const uint64_t ix = d2u(x);
  const uint32_t top = (uint32_t)(ix >> 48);
  if (ix - 0x3fee000000000000ULL < 0x3090000000000ULL) {  // |x - 1| < 0x1p-4 (LO..HI)
    if (ix == 0x3ff0000000000000ULL) return 0.0;
    const double *B = aero_g_log_poly1;
    const double r = x - 1.0;
    const double r2 = r * r, r3 = r * r2;
    double p9 = fma(r3, B[10], fma(r2, B[9], fma(r, B[8], B[7])));
    p9 = fma(p9, r3, fma(r2, B[6], fma(r, B[5], B[4])));
    const double p = fma(p9, r3, fma(r2, B[3], fma(r, B[2], B[1])));
    const double rhi = fma(-AERO_G_TWO27, r, fma(r, AERO_G_TWO27, r));
    const double rlo = r - rhi;
    const double hi = fma(rhi * rhi, B[0], r);
    double lo = fma(rhi * rhi, B[0], r - hi);
    lo = fma(B[0] * rlo, r + rhi, lo);
    return hi + fma(p, r3, lo);
  }
  uint64_t jx = ix;
  if (top - 0x0010u >= 0x7ff0u - 0x0010u) {
    if ((ix << 1) == 0) return -1.0 / 0.0;  // __math_divzero
    if (ix == 0x7ff0000000000000ULL) return x;
    if ((top & 0x8000u) || (top & 0x7ff0u) == 0x7ff0u) return (x - x) / (x - x);  // __math_invalid
    jx = d2u(x * 0x1p52) - (52ULL << 52);
  }
  const uint64_t tmp = jx - 0x3fe6000000000000ULL;
  const int i = (int)((tmp >> 45) & 127);
  const int k = (int)((int64_t)tmp >> 52);
  const double z = u2d(jx - (tmp & (0xfffULL << 52)));
  const double invc = aero_g_log_tab[i][0], logc = aero_g_log_tab[i][1];
  const double r = fma(z, invc, -1.0);
  const double kd = (double)k;
  const double w = fma(kd, AERO_G_LN2HI, logc);
  const double hi = w + r;
  const double lo = fma(kd, AERO_G_LN2LO, (w - hi) + r);
  const double r2 = r * r;
  const double *A = aero_g_log_poly;
  const double q = fma(fma(r, A[4], A[3]), r2, fma(r, A[2], A[1]));
  return fma(r * r2, q, fma(r2, A[0], lo)) + hi;
}

/* log10 (e_log10.c, __log10_finite: SSE2, no fusion) around __log_fma */
AERO_HD double aero_log10(double x) {
  const double two54 = 0x1p54;
  int64_t ix = (int64_t)d2u(x);
  int64_t k;
  if (ix > 0x000fffffffffffffLL) {
    k = -1023;
  } else {
    if ((ix & 0x7fffffffffffffffLL) == 0) return -two54 / __builtin_fabs(x);
    if (ix < 0) return (x - x) / (x - x);
    x *= two54;
    ix = (int64_t)d2u(x);
    k = -1023 - 54;
  }
  if ((uint64_t)ix > 0x7fefffffffffffffULL) return x + x;
  k += ix >> 52;
  const int64_t i = (int64_t)((uint64_t)k >> 63);
  const double y = (double)(k + i);
  x = u2d((uint64_t)(ix & 0x000fffffffffffffLL) | ((uint64_t)(0x3ff - i) << 52));
  const double z = y * AERO_G_LOG10_2LO + aero_log(x) * AERO_G_IVLN10;
  return z + y * AERO_G_LOG10_2HI;
}

}  // namespace aero
