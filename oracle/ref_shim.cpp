/*
 * oracle/ref_shim.cpp — TEST INFRASTRUCTURE ONLY.
 *
 * A C ABI over the two reference sources on this path that compile without
 * Qt or any other external library: decode/jfft.cpp (JFFT, the coarse
 * estimator's FFT, its real FFT that the burst trident check runs through
 * FFTrWrapper, and JFastFir, the fast convolution under the burst front
 * end's QJHilbertFilter; its Qt conveniences are behind QT_CORE_LIB) and
 * publish/oscillator.cpp (the channeliser's VFO mixer).  oracle/Makefile's
 * `ref` target compiles them straight from /root/reference into
 * oracle/_ref/libref.so; tests/test_oracle_ref.py checks the oracle's
 * restatements against them bit for bit.  Nothing else loads it.
 */
#include <complex>
#include <cstring>
#include <vector>

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

/* JFFT::fft_real through its std::vector convenience (as FFTrWrapper's
 * QVector one: init(n / 2)): n reals in, n interleaved complex out */
void ref_fft_real(const double *real, double *out, int n) {
  JFFT f;
  std::vector<double> r(real, real + n);
  std::vector<std::complex<double>> c;
  f.fft_real(r, c);
  memcpy(out, c.data(), sizeof(std::complex<double>) * (size_t)n);
}

/* JFastFir::SetKernel(kernel) then update() per sample, interleaved complex */
void ref_fastfir(const double *kernel, int klen, const double *in, double *out, int n) {
  JFastFir f;
  std::vector<std::complex<double>> k(reinterpret_cast<const std::complex<double> *>(kernel),
                                      reinterpret_cast<const std::complex<double> *>(kernel) + klen);
  f.SetKernel(k);
  for (int i = 0; i < n; ++i) {
    const std::complex<double> y = f.update(std::complex<double>(in[2 * i], in[2 * i + 1]));
    out[2 * i] = y.real();
    out[2 * i + 1] = y.imag();
  }
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
