/*
 * tables_host.cpp — host-computed constant tables of the engine.  Compiled
 * with g++ (-O2 -ffp-contract=off, baseline x86-64) like the reference, so
 * the std::complex arithmetic and every glibc call happen exactly as in the
 * reference's own table code.
 */
#include "tables_host.h"

#include <cmath>
#include <complex>
#include <cstring>

namespace aero {

void host_cis(double *cis) {  // TrigLookUp::TrigLookUp (decode/DSP.cpp:10-33)
  for (int i = 0; i < 19999; i++) {
    cis[2 * i + 1] = sin(2 * M_PI * ((double)i) / 19999);
    cis[2 * i] = sin(M_PI_2 + 2 * M_PI * ((double)i) / 19999);
  }
}

void host_twiddles(int nfft, double *tw, double *twi) {  // JFFT::init (decode/jfft.cpp:13-53)
  typedef std::complex<double> cpx;
  const cpx imag = cpx(0, 1);
  memset(tw, 0, sizeof(double) * 2 * nfft);
  memset(twi, 0, sizeof(double) * 2 * nfft);
  int w = 0;
  for (int N = 2; N <= nfft; N <<= 1) {
    for (int i = 0; i < N / 2; i++) {
      cpx twiddle = std::exp(-2.0 * imag * M_PI * ((double)i) / ((double)N));
      cpx twiddle_inv = std::exp(2.0 * imag * M_PI * ((double)i) / ((double)N));
      tw[2 * w] = twiddle.real();
      tw[2 * w + 1] = twiddle.imag();
      twi[2 * w] = twiddle_inv.real();
      twi[2 * w + 1] = twiddle_inv.imag();
      w++;
    }
  }
}

int host_rrc(double alpha, int firsize, double samplerate, double symbol_freq, double *Points) {
  // RootRaisedCosine::design (decode/DSP.h:325-351)
  if ((firsize % 2) == 0) firsize += 1;
  double T = (samplerate) / (symbol_freq);
  double fi;
  for (int i = 0; i < firsize; i++) {
    if (i == ((firsize - 1) / 2))
      Points[i] = (4.0 * alpha + M_PI - M_PI * alpha) / (M_PI * sqrt(T));
    else {
      fi = (((double)i) - ((double)(firsize - 1)) / 2.0);
      if (fabs(1.0 - pow(4.0 * alpha * fi / T, 2)) < 0.0000000001)
        Points[i] = (alpha *
                     ((M_PI - 2.0) * cos(M_PI / (4.0 * alpha)) +
                      (M_PI + 2.0) * sin(M_PI / (4.0 * alpha))) /
                     (M_PI * sqrt(2.0 * T)));
      else
        Points[i] = (4.0 * alpha / (M_PI * sqrt(T)) *
                     (cos((1.0 + alpha) * M_PI * fi / T) +
                      T / (4.0 * alpha * fi) * sin((1.0 - alpha) * M_PI * fi / T)) /
                     (1.0 - pow(4.0 * alpha * fi / T, 2)));
    }
  }
  return firsize;
}

bool host_delay(double fractdelay, DelayDesc &d) {
  // Delay<double>::setdelay/update (decode/DSP.h:358-384) evaluated for every
  // write pointer; the kernel keeps the ring as a shift register
  const int size = (int)std::ceil(fractdelay) + 1;
  if (size > 4) return false;
  memset(&d, 0, sizeof d);
  d.size = size;
  for (int p = 0; p < size; p++) {
    double dptr = ((double)p) - fractdelay;
    while (std::floor(dptr) < 0) dptr += ((double)size);
    const int iptr = (int)std::floor(dptr);
    const double weighting = dptr - ((double)iptr);
    const int a_old = ((p - iptr) % size + size) % size;
    const int a_new = ((p - (iptr + 1) % size) % size + size) % size;
    if (p == 0) {
      d.age_old = a_old;
      d.age_new = a_new;
    } else if (a_old != d.age_old || a_new != d.age_new) {
      return false;
    }
    d.w[p] = weighting;
    d.omw[p] = (1.0 - weighting);
  }
  return true;
}

bool host_delay_uniform(double fractdelay, int &size, int &age_old, int &age_new, double &w, double &omw) {
  size = (int)std::ceil(fractdelay) + 1;
  for (int p = 0; p < size; p++) {
    double dptr = ((double)p) - fractdelay;
    while (std::floor(dptr) < 0) dptr += ((double)size);
    const int iptr = (int)std::floor(dptr);
    const double weighting = dptr - ((double)iptr);
    const int a_old = ((p - iptr) % size + size) % size;
    const int a_new = ((p - (iptr + 1) % size) % size + size) % size;
    if (p == 0) {
      age_old = a_old;
      age_new = a_new;
      w = weighting;
      omw = (1.0 - weighting);
    } else if (a_old != age_old || a_new != age_new || memcmp(&w, &weighting, 8)) {
      return false;
    }
  }
  return true;
}

void host_msk_taps(int sps, double *taps) {
  const double SamplesPerSymbol = sps;
  for (int i = 0; i < 2 * sps; i++) taps[i] = sin(M_PI * i / (2.0 * SamplesPerSymbol)) / (2.0 * SamplesPerSymbol);
}

void host_scrambler(uint8_t *pre) {  // AeroLScrambler::AeroLScrambler (decode/aerol.h:408-427)
  int st[15] = {1, 1, 0, 1, 0, 0, 1, 0, 1, 0, 1, 1, 0, 0, 1};
  for (int a = 0; a < 5000; a++) {
    const int val0 = st[0] ^ st[14];
    pre[a] = (uint8_t)val0;
    for (int i = 14; i > 0; i--) st[i] = st[i - 1];
    st[0] = val0;
  }
}

}  // namespace aero

extern "C" {
/* exported for tests/test_tables.py: the engine's tables vs the oracle's */
void aero_host_tables(double *cis, double *tw, double *twi, double *taps, int *ntaps) {
  aero::host_cis(cis);
  aero::host_twiddles(16384, tw, twi);
  *ntaps = aero::host_rrc(1.0, 55, 48000, 10500 / 2, taps);
}
/* MSK groups: 8192-point twiddles and the 2*sps-tap matched filter */
void aero_host_msk_tables(int sps, double *tw, double *twi, double *taps) {
  aero::host_twiddles(8192, tw, twi);
  aero::host_msk_taps(sps, taps);
}
}
