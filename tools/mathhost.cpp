// Host build of aero-cli_amd/csrc/aero_math.h (g++, -ffp-contract=off) for
// tests/test_math_host.py (bitwise against the host glibc) and the
// device-vs-host check in tests/test_gpu_math.py.
#include <cmath>
#include <cstddef>

#include "../aero-cli_amd/csrc/aero_math.h"

extern "C" void aero_math_host_eval(int fn, const double *x, const double *y, double *out, size_t n) {
  for (size_t i = 0; i < n; i++) {
    const double a = x[i], b = y[i];
    double r = 0;
    switch (fn) {
      case 0: r = aero::aero_hypot(a, b); break;
      case 1: r = aero::aero_atan2(a, b); break;
      case 2: r = aero::aero_tanh(a); break;
      case 3: r = aero::aero_sin(a); break;
      case 4: r = aero::aero_cos(a); break;
      case 5: r = aero::aero_log10(a); break;
      case 6: r = std::sqrt(a); break;
      case 7: r = std::fmod(a, 360.0); break;
      case 8: r = a / b; break;
      case 9: { double s, c; aero::aero_sincos(a, s, c); r = s; break; }
      case 10: { double s, c; aero::aero_sincos(a, s, c); r = c; break; }
      case 12: r = aero::aero_log(a); break;
      default: break;
    }
    out[i] = r;
  }
}

// glibc reference values: the entry points the reference's loops reach
// (sin/cos pairs of one argument compile to sincos; log10 calls log)
extern "C" void aero_math_glibc_eval(int fn, const double *x, const double *y, double *out, size_t n) {
  for (size_t i = 0; i < n; i++) {
    const double a = x[i], b = y[i];
    volatile double va = a;  // keep GCC from merging the separate sin/cos calls
    double r = 0, s, c;
    switch (fn) {
      case 0: r = hypot(a, b); break;
      case 1: r = atan2(a, b); break;
      case 2: r = tanh(a); break;
      case 3: sincos(a, &s, &c); r = s; break;
      case 4: sincos(a, &s, &c); r = c; break;
      case 5: r = log10(a); break;
      case 6: r = sqrt(a); break;
      case 7: r = fmod(a, 360.0); break;
      case 8: r = a / b; break;
      case 9: sincos(a, &s, &c); r = s; break;
      case 10: sincos(a, &s, &c); r = c; break;
      case 12: r = log(a); break;
      case 13: r = sin(va); break;  // the ifunc'd __sin_fma (host tables only)
      case 14: r = cos(va); break;
      default: break;
    }
    out[i] = r;
  }
}
