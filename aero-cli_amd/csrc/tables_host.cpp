/*
 * tables_host.cpp — host-computed constant tables of the engine.  Compiled
 * with g++ (-O2 -ffp-contract=off, baseline x86-64) like the reference, so
 * the std::complex arithmetic and every glibc call happen exactly as in the
 * reference's own table code.
 */
#include "tables_host.h"

#include <algorithm>
#include <cmath>
#include <complex>
#include <cstring>
#include <vector>

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

// JFFT::fft (decode/jfft.cpp:114-212) on interleaved (re, im) doubles with
// the tables of host_twiddles; the inverse scales by 1/N as JFFT does
void host_jfft(double *xd, int nfft, bool inverse, const double *tw, const double *twi) {
  typedef std::complex<double> cpx;
  cpx *x = reinterpret_cast<cpx *>(xd);
  const cpx *TW = reinterpret_cast<const cpx *>(inverse ? twi : tw);
  int pw = 0;
  while ((1 << pw) < nfft) pw++;
  for (uint32_t i = 0; i < (uint32_t)nfft; ++i) {
    uint32_t y = i;
    y = (((y & 0xaaaaaaaa) >> 1) | ((y & 0x55555555) << 1));
    y = (((y & 0xcccccccc) >> 2) | ((y & 0x33333333) << 2));
    y = (((y & 0xf0f0f0f0) >> 4) | ((y & 0x0f0f0f0f) << 4));
    y = (((y & 0xff00ff00) >> 8) | ((y & 0x00ff00ff) << 8));
    y = ((y >> 16) | (y << 16)) >> (32 - pw);
    if (y > i) std::swap(x[i], x[y]);
  }
  for (int n = 1; n < nfft; n <<= 1)
    for (int g = 0; g < nfft; g += 2 * n)
      for (int j = 0; j < n; j++) {
        const cpx y = TW[n - 1 + j] * x[g + n + j];
        x[g + n + j] = x[g + j] - y;
        x[g + j] += y;
      }
  if (inverse)
    for (int i = 0; i < nfft; ++i) x[i] *= (1.0 / ((double)nfft));
}

// CoarseFreqEstimate::setSettings' raised-cosine window (decode/coarsefreqestimate.cpp:56-74)
void host_coarse_window(int nfft, double lockingbw, double fs, double *window) {
  const double hzperbin = fs / ((double)nfft);
  const int startbin = (int)std::max(round(lockingbw / hzperbin), 1.0);
  for (int i = 0; i < nfft; i++) window[i] = 0;
  window[0] = 1;
  for (int i = 1; i <= startbin; i++) {
    double val = cos(M_PI_2 * ((double)i) / ((double)startbin));
    val *= val;
    if ((nfft - i) < 0) break;
    if (i >= nfft) break;
    window[nfft - i] = val;
    window[i] = val;
  }
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


// Delay<T>::update (decode/DSP.h:365-384) for every write pointer p: the slot
// of the older sample and the weights (weighting, 1 - weighting).  Returns the
// ring size ceil(fd) + 1, or -1 when it exceeds cap.
int host_delay_table(double fractdelay, double *w, double *omw, int *iold, int cap) {
  const int size = (int)std::ceil(fractdelay) + 1;
  if (size > cap) return -1;
  for (int p = 0; p < size; p++) {
    double dptr = ((double)p) - fractdelay;
    while (std::floor(dptr) < 0) dptr += ((double)size);
    const int iptr = (int)std::floor(dptr);
    const double weighting = dptr - ((double)iptr);
    w[p] = weighting;
    omw[p] = (1.0 - weighting);
    iold[p] = iptr;
  }
  return size;
}

// FFTrWrapper split tables DA/DB (decode/fftrwrapper.cpp:13-24, JFFT::init
// real path decode/jfft.cpp:54-67), nfft = complex FFT size
void host_fftr_split(int nfft, double *da, double *db) {
  typedef std::complex<double> cpx;
  const cpx imag = cpx(0, 1);
  for (int i = 0; i < nfft; i++) {
    const cpx a = 0.5 * (1.0 - imag * std::exp(-2.0 * imag * M_PI * ((double)i) / ((double)(2 * nfft))));
    const cpx b = 0.5 * (1.0 + imag * std::exp(-2.0 * imag * M_PI * ((double)i) / ((double)(2 * nfft))));
    da[2 * i] = a.real();
    da[2 * i + 1] = a.imag();
    db[2 * i] = b.real();
    db[2 * i + 1] = b.imag();
  }
}

// QJHilbertFilter's 2048-tap analytic-signal kernel (decode/DSP.cpp:730-761)
// zero-padded to the 8192-point JFastFir block (decode/jfft.cpp:322-374)
void host_hilbert_kernel(double *k) {
  typedef std::complex<double> cpx;
  const int N = 2048;
  memset(k, 0, sizeof(double) * 2 * 8192);
  for (int i = 0; i < N; i++) {
    cpx v;
    if (i == N / 2)
      v = cpx(-1, 0);
    else if ((i % 2) == 0)
      v = cpx(0, 0);
    else
      v = cpx(0, (2.0 / ((double)N)) / (std::tan(M_PI * (((double)i) / ((double)N) - 0.5))));
    k[2 * i] = v.real();
    k[2 * i + 1] = v.imag();
  }
}

/* ------------------------------------------ aero-publish channeliser (FP32) */
int host_pub_osc_len(double sampleRate) { return (int)sampleRate; }

// Oscillator::Oscillator (publish/oscillator.cpp:4-28): queue[i] is the
// rotator after i+1 renormalised steps, in std::complex<float> as there
void host_pub_osc(double sampleRate, double frequency, float *queue) {
  typedef std::complex<float> cpxf;
  const double anglePerSample = 2.0 * M_PI * frequency / sampleRate;
  const cpxf rotation((float)cos(anglePerSample), (float)sin(anglePerSample));
  cpxf v(1.0f, 0);
  const int length = (int)sampleRate;
  for (int i = 0; i < length; i++) {
    v *= rotation;
    const float norm = 1.95f - (v.real() * v.real() + v.imag() * v.imag());
    v = v * norm;
    queue[2 * i] = v.real();
    queue[2 * i + 1] = v.imag();
  }
}

// FIRHilbert::FIRHilbert (publish/dsp.cpp:181-215).  `sqrt` of the float sum
// resolves to the float overload there (`using namespace std`, dsp.cpp:30).
void host_pub_hilbert(int len, int Fs, float *points) {
  std::vector<float> tempCoeffs(len);
  float sumofsquares = 0;
  for (int n = 0; n < len; n++) {
    if (n == len / 2)
      tempCoeffs[n] = 0;
    else
      tempCoeffs[n] = Fs / (M_PI * (n - len / 2)) * (1 - cos(M_PI * (n - len / 2)));
    sumofsquares += tempCoeffs[n] * tempCoeffs[n];
  }
  const double gain = std::sqrt(sumofsquares);
  for (int i = 0; i < len; i++) points[i] = tempCoeffs[len - i - 1] / gain;
}

// firfilter::low_pass with WIN_HAMMING (publish/firfilter.cpp:47-99, 186-193)
int host_pub_low_pass(double gain, double fs, double cutoff, double tw, float *taps, int cap) {
  int ntaps = (int)(53.0 * fs / (22.0 * tw));  // compute_ntaps, max_attenuation(HAMMING) = 53
  if ((ntaps & 1) == 0) ntaps++;
  if (ntaps > cap) return -1;
  std::vector<float> w(ntaps);
  const float Mf = static_cast<float>(ntaps - 1);
  for (int n = 0; n < ntaps; n++) w[n] = 0.54 - 0.46 * cos((2 * M_PI * n) / Mf);
  const int M = (ntaps - 1) / 2;
  const double fwT0 = 2 * M_PI * cutoff / fs;
  for (int n = -M; n <= M; n++) {
    if (n == 0)
      taps[n + M] = fwT0 / M_PI * w[n + M];
    else
      taps[n + M] = sin(n * fwT0) / (n * M_PI) * w[n + M];
  }
  double fmax = taps[0 + M];
  for (int n = 1; n <= M; n++) fmax += 2 * taps[n + M];
  gain /= fmax;
  for (int i = 0; i < ntaps; i++) taps[i] *= gain;
  return ntaps;
}

}  // namespace aero

extern "C" {
/* burst tables, for tests/test_abi.py */
void aero_host_fftr_split(int nfft, double *da, double *db) { aero::host_fftr_split(nfft, da, db); }
void aero_host_hilbert_kernel(double *k) { aero::host_hilbert_kernel(k); }
/* channeliser designs, for tests/test_abi.py (engine tables vs the oracle's) */
void aero_host_pub_osc(double fs, double freq, float *queue) { aero::host_pub_osc(fs, freq, queue); }
void aero_host_pub_hilbert(int len, int fs, float *points) { aero::host_pub_hilbert(len, fs, points); }
int aero_host_pub_low_pass(double gain, double fs, double cutoff, double tw, float *taps, int cap) {
  return aero::host_pub_low_pass(gain, fs, cutoff, tw, taps, cap);
}
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
