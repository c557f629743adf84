/*
 * oracle/ref_shim.cpp — TEST INFRASTRUCTURE ONLY.
 *
 * A C ABI over the two reference sources on this path that compile without
 * Qt or any other external library: decode/jfft.cpp (JFFT, the coarse
 * estimator's FFT; its Qt conveniences are behind QT_CORE_LIB) and
 * publish/oscillator.cpp (the channeliser's VFO mixer).  oracle/Makefile's
 * `ref` target compiles them straight from /root/reference into
 * oracle/_ref/libref.so; tests/test_oracle_ref.py checks the oracle's
 * restatements against them bit for bit.  Nothing else loads it.
 */
#include <complex>

#include "jfft.h"
#include "oscillator.h"

extern "C" {

/* JFFT::fft in place on nfft interleaved complex doubles */
void ref_jfft(double *x, int nfft, int inverse) {
  JFFT f;
  int n = nfft;
  f.init(n);
  f.fft(reinterpret_cast<std::complex<double> *>(x), nfft, inverse ? JFFT::INVERSE : JFFT::FORWARD);
}

/* Oscillator(fs, freq): _vector before each of n ticks, interleaved floats */
void ref_osc(double fs, double freq, float *dst, int n) {
  Oscillator o(fs, freq);
  for (int i = 0; i < n; ++i) {
    dst[2 * i] = o._vector.real();
    dst[2 * i + 1] = o._vector.imag();
    o.tick();
  }
}

}  // extern "C"
