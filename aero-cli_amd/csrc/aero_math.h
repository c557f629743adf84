/*
 * aero_math.h — the libm the demod kernels call, bit-compatible with the
 * host glibc 2.35 that the reference links (the decode/ sources call std::abs on
 * complex (-> hypot), std::arg (-> atan2), tanh, sin, cos, log10).
 *
 * Compiles for host (g++/hipcc host pass) and device (gfx950).  Every file
 * that includes it must be built with -ffp-contract=off; the only fused
 * operations are the explicit fma() calls of the double-double helpers,
 * which are exact by construction.
 *
 *  aero_hypot  : glibc 2.35 dbl-64 e_hypot.c algorithm (non-FMA kernel) ->
 *                bit-exact with glibc (tests/test_math.py, 2e7 samples).
 *  aero_tanh   : fdlibm s_tanh.c on glibc's s_expm1.c (Estrin-form
 *                polynomial) -> bit-exact with glibc.
 *  aero_atan2, aero_sin, aero_cos, aero_log10 : correctly rounded via
 *                double-double evaluation (~2^-100 relative); glibc's own
 *                results are correctly rounded in all but rare cases, the
 *                measured agreement is recorded by tests/test_math.py.
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

#include "aero_math_tables.h"

namespace aero {

AERO_HD uint64_t d2u(double x) { return __builtin_bit_cast(uint64_t, x); }
AERO_HD double u2d(uint64_t u) { return __builtin_bit_cast(double, u); }
AERO_HD uint32_t hiw(double x) { return (uint32_t)(d2u(x) >> 32); }
AERO_HD uint32_t low(double x) { return (uint32_t)d2u(x); }
AERO_HD double sethi(double x, uint32_t hi) {
  return u2d((d2u(x) & 0xffffffffULL) | ((uint64_t)hi << 32));
}
AERO_HD double mkd(uint32_t hi, uint32_t lo) { return u2d(((uint64_t)hi << 32) | lo); }

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

/* ---------------------------------------------------- double-double */
struct dd {
  double hi, lo;
};
AERO_HD dd two_sum(double a, double b) {
  double s = a + b;
  double bb = s - a;
  double e = (a - (s - bb)) + (b - bb);
  return {s, e};
}
AERO_HD dd quick_two_sum(double a, double b) {
  double s = a + b;
  return {s, b - (s - a)};
}
AERO_HD dd two_prod(double a, double b) {
  double p = a * b;
  return {p, fma(a, b, -p)};
}
AERO_HD dd dd_add(dd a, dd b) {
  dd s = two_sum(a.hi, b.hi);
  dd t = two_sum(a.lo, b.lo);
  s.lo += t.hi;
  s = quick_two_sum(s.hi, s.lo);
  s.lo += t.lo;
  return quick_two_sum(s.hi, s.lo);
}
AERO_HD dd dd_neg(dd a) { return {-a.hi, -a.lo}; }
AERO_HD dd dd_mul(dd a, dd b) {
  dd p = two_prod(a.hi, b.hi);
  p.lo += a.hi * b.lo + a.lo * b.hi;
  return quick_two_sum(p.hi, p.lo);
}
AERO_HD dd dd_mul_d(dd a, double b) {
  dd p = two_prod(a.hi, b);
  p.lo += a.lo * b;
  return quick_two_sum(p.hi, p.lo);
}
AERO_HD dd dd_div(dd a, dd b) {
  double q1 = a.hi / b.hi;
  dd r = dd_add(a, dd_neg(dd_mul_d(b, q1)));
  double q2 = r.hi / b.hi;
  r = dd_add(r, dd_neg(dd_mul_d(b, q2)));
  double q3 = r.hi / b.hi;
  dd q = quick_two_sum(q1, q2);
  return dd_add(q, dd{q3, 0.0});
}

/* atan(t), t = th + tl in [0, 1], returned as double-double */
AERO_HD dd dd_atan01(double th, double tl) {
  int k = (int)(th * 64.0 + 0.5);
  double c = (double)k * (1.0 / 64.0);
  dd num = two_sum(th - c, tl);              // th - c is exact (Sterbenz)
  dd den = dd_add(dd{1.0, 0.0}, dd_mul_d(dd{th, tl}, c));
  dd u = dd_div(num, den);                   // |u| <= 2^-7
  dd u2 = dd_mul(u, u);
  dd u3 = dd_mul(u2, u);
  dd u5 = dd_mul(u3, u2);
  double v = u2.hi;
  // tail: -u^7/7 + u^9/9 - ... + u^17/17 in double
  double tail = -1.0 / 7 + v * (1.0 / 9 + v * (-1.0 / 11 + v * (1.0 / 13 + v * (-1.0 / 15 + v * (1.0 / 17)))));
  tail = tail * (u5.hi * v);
  dd r = dd_add(u, dd_mul(u3, dd{-AERO_INV3_HI, -AERO_INV3_LO}));
  r = dd_add(r, dd_mul(u5, dd{AERO_INV5_HI, AERO_INV5_LO}));
  r = dd_add(r, dd{tail, 0.0});
  return dd_add(dd{aero_atan_tab[k][0], aero_atan_tab[k][1]}, r);
}

AERO_HD double aero_atan2_dd(double y, double x) {
  if (__builtin_isnan(x) || __builtin_isnan(y)) return x + y;
  bool ny = __builtin_signbit(y) != 0, nx = __builtin_signbit(x) != 0;
  double ay = __builtin_fabs(y), ax = __builtin_fabs(x);
  if (ay == 0.0) {
    if (!nx) return y;  // +-0
    return ny ? -AERO_PI_HI : AERO_PI_HI;
  }
  if (ax == 0.0) return ny ? -AERO_PI_2_HI : AERO_PI_2_HI;
  if (__builtin_isinf(ax)) {
    if (__builtin_isinf(ay)) {
      double r = nx ? 3.0 * AERO_PI_4_HI : AERO_PI_4_HI;
      return ny ? -r : r;
    }
    double r = nx ? AERO_PI_HI : 0.0;
    return ny ? -r : r;
  }
  if (__builtin_isinf(ay)) return ny ? -AERO_PI_2_HI : AERO_PI_2_HI;
  bool swap = ay > ax;
  double a = swap ? ax : ay, b = swap ? ay : ax;
  // scale to keep the residual computation away from under/overflow
  const int eb = (int)((hiw(b) >> 20) & 0x7ff) - 1023;
  if (eb > 500) {  // only the ratio matters: scale by powers of two (exact)
    a *= 0x1p-600;
    b *= 0x1p-600;
  } else if (eb < -500) {
    a *= 0x1p600;
    b *= 0x1p600;
  }
  double th = a / b;
  if (th < 0x1p-1000) {
    // tiny ratio: atan(t) = t to double precision
    double r = th;
    dd res = swap ? dd_add(dd{AERO_PI_2_HI, AERO_PI_2_LO}, dd{-r, 0.0}) : dd{r, 0.0};
    if (nx) res = dd_add(dd{AERO_PI_HI, AERO_PI_LO}, dd_neg(res));
    double out = res.hi + res.lo;
    return ny ? -out : out;
  }
  double tl = fma(-th, b, a) / b;
  dd r = dd_atan01(th, tl);
  if (swap) r = dd_add(dd{AERO_PI_2_HI, AERO_PI_2_LO}, dd_neg(r));
  if (nx) r = dd_add(dd{AERO_PI_HI, AERO_PI_LO}, dd_neg(r));
  double out = r.hi + r.lo;
  return ny ? -out : out;
}

/* reciprocal to ~2^-100 relative after two Newton steps (device: v_rcp_f64) */
AERO_HD double approx_rcp(double b) {
#if defined(__HIP_DEVICE_COMPILE__)
  double r = __builtin_amdgcn_rcp(b);
#else
  double r = 1.0 / b;
#endif
  r = fma(r, fma(-b, r, 1.0), r);
  r = fma(r, fma(-b, r, 1.0), r);
  return r;
}

/* atan2 fast path (Ziv): atan(t) = atan(k/64) + atan(u) evaluated to about
 * 2^-65 relative without any IEEE division, returned only when that bound
 * proves the rounding; otherwise (≈2^-10 of arguments, and every special or
 * extreme-exponent argument) the double-double path decides.  Same results
 * as aero_atan2_dd by construction (tests/test_math_host.py compares them).
 * The quadrant (pi/2 - r when |y| > |x|, pi - r when x < 0) is folded into
 * one table row, C + s atan(k/64) in double-double, so the result is
 * B + s (u + corr) with a single two_sum, and the series runs in fused
 * Horner form (both only tighten the bound the rounding test assumes). */
AERO_HD double aero_atan2(double y, double x) {
  const double ay = __builtin_fabs(y), ax = __builtin_fabs(x);
  if (!(ax >= 0x1p-500 && ax <= 0x1p500 && ay >= 0x1p-500 && ay <= 0x1p500)) return aero_atan2_dd(y, x);
  const bool swap = ay > ax;
  const double a = swap ? ax : ay, b = swap ? ay : ax;  // t = a/b in (0, 1]
  const double rb = approx_rcp(b);
  const double th = a * rb;
  const double tl = fma(-th, b, a) * rb;
  const int k = (int)(th * 64.0 + 0.5);
  const double c = (double)k * (1.0 / 64.0);
  // u = (t - c) / (1 + t c), |u| <= 2^-7
  const dd num = two_sum(th - c, tl);  // th - c exact (Sterbenz)
  const double ph = th * c, pl = fma(th, c, -ph);
  const dd den0 = quick_two_sum(1.0, ph);  // ph = t c <= 1
  const double dh = den0.hi, dl = den0.lo + (pl + tl * c);
  const double rd = approx_rcp(dh);
  const double uh = num.hi * rd;
  const double ul = ((fma(-uh, dh, num.hi) + num.lo) - uh * dl) * rd;
  // atan(u) - u = u^3 (-1/3 + u^2/5 - ...) - u^2 ul
  const double v = uh * uh;
  double p = fma(v, -1.0 / 15, 1.0 / 13);
  p = fma(v, p, -1.0 / 11);
  p = fma(v, p, 1.0 / 9);
  p = fma(v, p, -1.0 / 7);
  p = fma(v, p, 1.0 / 5);
  p = fma(v, p, -AERO_INV3_HI);
  const double corr = fma(v * uh, p, -v * ul);
  // atan2 = C + s (A + u + corr): (C, s) = (0, 1), (pi/2, -1), (pi, -1),
  // (pi/2, 1) for q = swap | 2 (x < 0); the row holds C + s A
  const int q = (swap ? 1 : 0) | (__builtin_signbit(x) ? 2 : 0);
  const double sg = (q == 1 || q == 2) ? -1.0 : 1.0;
  const int row = q * 65 + k;
  dd r = two_sum(aero_atan2_quad_tab[row][0], sg * uh);
  r.lo += aero_atan2_quad_tab[row][1] + sg * (ul + corr);
  r = quick_two_sum(r.hi, r.lo);
  const double e = 0x1p-63 * __builtin_fabs(r.hi);
  const double out = r.hi + r.lo;
  if (out != r.hi + (r.lo + e) || out != r.hi + (r.lo - e)) return aero_atan2_dd(y, x);
  return __builtin_signbit(y) ? -out : out;
}

/* sin/cos of r = rh + rl, |r| <= pi/4 + eps, as double-double */
AERO_HD void dd_sincos_small(double rh, double rl, dd &s, dd &c, bool want_s, bool want_c) {
  double ar = __builtin_fabs(rh);
  int k = (int)(ar * 64.0 + 0.5);
  if (k > 52) k = 52;
  double kc = (double)k * (1.0 / 64.0);
  double sgn = rh < 0 ? -1.0 : 1.0;
  // d = |r| - k/64
  dd d = two_sum(ar - kc, sgn * rl);
  dd d2 = dd_mul(d, d);
  double v = d2.hi;
  // sin(d) = d - d^3/6 + d^5/120 - [d^7/5040 - d^9/9! + d^11/11!]
  dd d3 = dd_mul(d2, d);
  dd d5 = dd_mul(d3, d2);
  double st = (-1.0 / 5040 + v * (1.0 / 362880 + v * (-1.0 / 39916800))) * (d5.hi * v);
  dd sd = dd_add(d, dd_mul(d3, dd{-AERO_INV6_HI, -AERO_INV6_LO}));
  sd = dd_add(sd, dd_mul(d5, dd{AERO_INV120_HI, AERO_INV120_LO}));
  sd = dd_add(sd, dd{st, 0.0});
  // cos(d) = 1 - d^2/2 + d^4/24 - [d^6/720 - d^8/8! + d^10/10!]
  dd d4 = dd_mul(d2, d2);
  double ct = (-1.0 / 720 + v * (1.0 / 40320 + v * (-1.0 / 3628800))) * (d4.hi * v);
  dd cd = dd_add(dd{1.0, 0.0}, dd_mul_d(d2, -0.5));
  cd = dd_add(cd, dd_mul(d4, dd{AERO_INV24_HI, AERO_INV24_LO}));
  cd = dd_add(cd, dd{ct, 0.0});
  dd sk = {aero_sin_tab[k][0], aero_sin_tab[k][1]};
  dd ck = {aero_cos_tab[k][0], aero_cos_tab[k][1]};
  if (want_s) {
    // sin(|r|) = sin(k)cos(d) + cos(k)sin(d)
    s = dd_add(dd_mul(sk, cd), dd_mul(ck, sd));
    if (sgn < 0) s = dd_neg(s);
  }
  if (want_c) c = dd_add(dd_mul(ck, cd), dd_neg(dd_mul(sk, sd)));
}

/* x = n*pi/2 + r (Cody-Waite, fdlibm split constants); valid for |x| < 2^20.
 * aero_sin/aero_cos/aero_sincos return NaN outside that domain (the demod's
 * argument is a moving average of clipped loop errors, |x| <= pi/2). */
AERO_HD int reduce_pio2(double x, double &rh, double &rl) {
  const double pio2_1 = 1.57079632673412561417e+00, pio2_2 = 6.07710050630396597660e-11,
               pio2_3 = 2.02226624871116645580e-21, pio2_3t = 8.47842766036889956997e-32;
  if (__builtin_fabs(x) <= AERO_PI_4_HI) {
    rh = x;
    rl = 0.0;
    return 0;
  }
  double fn = __builtin_rint(x * AERO_2_PI_HI);
  int n = (int)fn;
  double r = x - fn * pio2_1;  // exact
  double w = fn * pio2_2;      // exact for |n| < 2^20
  dd t = two_sum(r, -w);
  dd u = two_sum(t.hi, -fn * pio2_3);
  u.lo += t.lo - fn * pio2_3t;
  dd res = quick_two_sum(u.hi, u.lo);
  rh = res.hi;
  rl = res.lo;
  return n;
}

AERO_HD double aero_sin(double x) {
  if (!__builtin_isfinite(x)) return x - x;
  if (__builtin_fabs(x) >= 0x1p20) return __builtin_nan("");
  if (__builtin_fabs(x) < 0x1p-26) return x;
  double rh, rl;
  int n = reduce_pio2(x, rh, rl);
  dd s, c;
  if (n & 1)
    dd_sincos_small(rh, rl, s, c, false, true);
  else
    dd_sincos_small(rh, rl, s, c, true, false);
  double out;
  switch (n & 3) {
    case 0: out = s.hi + s.lo; break;
    case 1: out = c.hi + c.lo; break;
    case 2: out = -(s.hi + s.lo); break;
    default: out = -(c.hi + c.lo); break;
  }
  return out;
}

AERO_HD double aero_cos(double x) {
  if (!__builtin_isfinite(x)) return x - x;
  if (__builtin_fabs(x) >= 0x1p20) return __builtin_nan("");
  if (__builtin_fabs(x) < 0x1p-27) return 1.0;
  double rh, rl;
  int n = reduce_pio2(x, rh, rl);
  dd s, c;
  if (n & 1)
    dd_sincos_small(rh, rl, s, c, true, false);
  else
    dd_sincos_small(rh, rl, s, c, false, true);
  double out;
  switch (n & 3) {
    case 0: out = c.hi + c.lo; break;
    case 1: out = -(s.hi + s.lo); break;
    case 2: out = -(c.hi + c.lo); break;
    default: out = s.hi + s.lo; break;
  }
  return out;
}

/* sin and cos of x together (one reduction, one table lookup); the same
 * correctly-rounded results as aero_sin / aero_cos */
AERO_HD void aero_sincos_dd(double x, double &so, double &co) {
  if (!__builtin_isfinite(x) || __builtin_fabs(x) >= 0x1p20) {
    so = co = __builtin_nan("");
    return;
  }
  double rh, rl;
  int n = reduce_pio2(x, rh, rl);
  dd s, c;
  dd_sincos_small(rh, rl, s, c, true, true);
  const double sv = s.hi + s.lo, cv = c.hi + c.lo;
  switch (n & 3) {
    case 0: so = sv; co = cv; break;
    case 1: so = cv; co = -sv; break;
    case 2: so = -sv; co = -cv; break;
    default: so = -cv; co = sv; break;
  }
  if (__builtin_fabs(x) < 0x1p-26) so = x;
  if (__builtin_fabs(x) < 0x1p-27) co = 1.0;
}

/* sincos fast path (Ziv) for 2^-26 <= |x| <= 1/4, the demods' usual loop
 * corrections.  Taylor series around 0 with the terms that matter at 2^-70
 * kept exact or in double-double: x^2 exact by fma, x^3/6 and x^5/120 (sin),
 * x^2/2 and x^4/24 (cos) as double-double products, the rest (|.| <= 2^-24
 * |x| for sin, 2^-21 for cos) in double; their sum carries at most ~2^-72
 * relative error, so when hi + (lo +- 2^-69 |hi|) round alike, hi + lo is the
 * correctly rounded value (aero_sincos_dd's result).  Otherwise (and outside
 * the range) the double-double path decides.  No IEEE division. */
AERO_HD void aero_sincos(double x, double &so, double &co) {
  const double ax = __builtin_fabs(x);
  if (!(ax >= 0x1p-26 && ax <= 0.25)) {
    aero_sincos_dd(x, so, co);
    return;
  }
  const double x2 = ax * ax, x2l = fma(ax, ax, -x2);  // x^2 = x2 + x2l exactly
  // sin |x| = |x| - x^3/6 + x^5/120 + x^7 P(x^2)
  const double x3 = ax * x2, x3l = fma(ax, x2, -x3) + ax * x2l;
  const double t3 = x3 * -AERO_INV6_HI, t3l = fma(x3, -AERO_INV6_HI, -t3) + (x3 * -AERO_INV6_LO + x3l * -AERO_INV6_HI);
  const double x5 = x3 * x2, x5l = fma(x3, x2, -x5) + (x3 * x2l + x3l * x2);
  const double t5 = x5 * AERO_INV120_HI, t5l = fma(x5, AERO_INV120_HI, -t5) + (x5 * AERO_INV120_LO + x5l * AERO_INV120_HI);
  double p = fma(x2, 1.0 / 355687428096000.0, -1.0 / 1307674368000.0);
  p = fma(x2, p, 1.0 / 6227020800.0);
  p = fma(x2, p, -1.0 / 39916800.0);
  p = fma(x2, p, 1.0 / 362880.0);
  p = fma(x2, p, -1.0 / 5040.0);
  const double r7 = (x5 * x2) * p;
  const dd sa = two_sum(ax, t3);
  const dd sb = two_sum(sa.hi, t5);
  const double slo = (sa.lo + sb.lo) + ((t3l + t5l) + r7);
  // cos x = 1 - x^2/2 + x^4/24 + x^6 Q(x^2)
  const double h = 0.5 * x2, hl = 0.5 * x2l;  // exact
  const double x4 = x2 * x2, x4l = fma(x2, x2, -x4) + 2.0 * (x2 * x2l);
  const double t4 = x4 * AERO_INV24_HI, t4l = fma(x4, AERO_INV24_HI, -t4) + (x4 * AERO_INV24_LO + x4l * AERO_INV24_HI);
  double q = fma(x2, 1.0 / 20922789888000.0, -1.0 / 87178291200.0);
  q = fma(x2, q, 1.0 / 479001600.0);
  q = fma(x2, q, -1.0 / 3628800.0);
  q = fma(x2, q, 1.0 / 40320.0);
  q = fma(x2, q, -1.0 / 720.0);
  const double r6 = (x4 * x2) * q;
  const dd ca = two_sum(1.0, -h);
  const dd cb = two_sum(ca.hi, t4);
  const double clo = (ca.lo + cb.lo) + ((t4l - hl) + r6);
  const double sv = sb.hi + slo, cv = cb.hi + clo;
  const double es = 0x1p-69 * sb.hi, ec = 0x1p-69 * cb.hi;
  if (sv != sb.hi + (slo + es) || sv != sb.hi + (slo - es) || cv != cb.hi + (clo + ec) ||
      cv != cb.hi + (clo - ec)) {
    aero_sincos_dd(x, so, co);
    return;
  }
  so = __builtin_signbit(x) ? -sv : sv;
  co = cv;
}

/* natural log of m in [1, 2) as double-double */
AERO_HD dd dd_log12(double m) {
  int k = (int)((m - 1.0) * 64.0 + 0.5);
  double c = 1.0 + (double)k * (1.0 / 64.0);
  // log(m/c) = 2 atanh(u), u = (m - c)/(m + c)
  dd num = {m - c, 0.0};               // exact (Sterbenz)
  dd den = two_sum(m, c);
  dd u = dd_div(num, den);             // |u| <= 2^-8
  dd u2 = dd_mul(u, u);
  dd u3 = dd_mul(u2, u);
  dd u5 = dd_mul(u3, u2);
  double v = u2.hi;
  double tail = (1.0 / 7 + v * (1.0 / 9 + v * (1.0 / 11 + v * (1.0 / 13)))) * (u5.hi * v);
  dd r = dd_add(u, dd_mul(u3, dd{AERO_INV3_HI, AERO_INV3_LO}));
  r = dd_add(r, dd_mul(u5, dd{AERO_INV5_HI, AERO_INV5_LO}));
  r = dd_add(r, dd{tail, 0.0});
  r = dd_mul_d(r, 2.0);
  return dd_add(dd{aero_log_tab[k][0], aero_log_tab[k][1]}, r);
}

/* correctly rounded natural log, double-double evaluation */
AERO_HD double aero_log_dd(double x) {
  if (!(x > 0.0) || !__builtin_isfinite(x)) {
    if (x == 0.0) return -__builtin_inf();
    if (x < 0.0 || __builtin_isnan(x)) return (x - x) / (x - x);
    return x;  // +inf
  }
  uint64_t u = d2u(x);
  int e = (int)((u >> 52) & 0x7ff);
  int k = 0;
  if (e == 0) {  // subnormal
    x *= 0x1p54;
    u = d2u(x);
    e = (int)((u >> 52) & 0x7ff);
    k = -54;
  }
  k += e - 1023;
  double m = u2d((u & 0x000fffffffffffffULL) | 0x3ff0000000000000ULL);
  dd lm = dd_log12(m);
  dd r = dd_add(dd_mul_d(dd{AERO_LN2_HI, AERO_LN2_LO}, (double)k), lm);
  return r.hi + r.lo;
}

/* log fast path (Ziv): log(x) = k ln2 + log(c) + 2 atanh(u), u = (m-c)/(m+c),
 * evaluated to about 2^-66 without IEEE division; returned only when that
 * bound proves the rounding, otherwise aero_log_dd decides (same results). */
AERO_HD double aero_log(double x) {
  if (!(x >= 0x1p-1000 && x <= 0x1p1000)) return aero_log_dd(x);
  const uint64_t ux = d2u(x);
  const int k = (int)((ux >> 52) & 0x7ff) - 1023;
  const double m = u2d((ux & 0x000fffffffffffffULL) | 0x3ff0000000000000ULL);
  const int j = (int)((m - 1.0) * 64.0 + 0.5);
  const double c = 1.0 + (double)j * (1.0 / 64.0);
  const double nh = m - c;                 // exact (Sterbenz)
  const dd den = two_sum(m, c);
  const double rd = approx_rcp(den.hi);
  const double uh = nh * rd;               // |u| <= 2^-8
  const double ul = (fma(-uh, den.hi, nh) - uh * den.lo) * rd;
  const double v = uh * uh;
  double p = 1.0 / 13;
  p = 1.0 / 11 + v * p;
  p = 1.0 / 9 + v * p;
  p = 1.0 / 7 + v * p;
  p = 1.0 / 5 + v * p;
  p = AERO_INV3_HI + v * p;
  const double corr = 2.0 * ((v * uh) * p + v * ul);  // 2 atanh(u) - 2u
  // log(c) + 2u + corr + k ln2
  dd r = two_sum(aero_log_tab[j][0], 2.0 * uh);
  r.lo += aero_log_tab[j][1] + (2.0 * ul + corr);
  r = quick_two_sum(r.hi, r.lo);
  if (k) r = dd_add(dd_mul_d(dd{AERO_LN2_HI, AERO_LN2_LO}, (double)k), r);
  const double e = 0x1p-63 * __builtin_fabs(r.hi);
  const double out = r.hi + r.lo;
  if (out != r.hi + (r.lo + e) || out != r.hi + (r.lo - e)) return aero_log_dd(x);
  return out;
}

AERO_HD double aero_log10(double x) {
  const double two54 = 1.80143985094819840000e+16, ivln10 = 4.34294481903251816668e-01,
               log10_2hi = 3.01029995663611771306e-01, log10_2lo = 3.69423907715893078616e-13;
  double y, z;
  int32_t i, k, hx;
  hx = (int32_t)hiw(x);
  uint32_t lx = low(x);
  k = 0;
  if (hx < 0x00100000) {
    if (((hx & 0x7fffffff) | (int32_t)lx) == 0) return -two54 / __builtin_fabs(x);
    if (hx < 0) return (x - x) / (x - x);
    k -= 54;
    x *= two54;
    hx = (int32_t)hiw(x);
  }
  if (hx >= 0x7ff00000) return x + x;
  k += (hx >> 20) - 1023;
  i = (int32_t)(((uint32_t)k & 0x80000000u) >> 31);
  hx = (hx & 0x000fffff) | ((0x3ff - i) << 20);
  y = (double)(k + i);
  x = sethi(x, (uint32_t)hx);
  z = y * log10_2lo + ivln10 * aero_log(x);
  return z + y * log10_2hi;
}

}  // namespace aero
