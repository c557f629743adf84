#pragma once
#include <stdint.h>

namespace aero {

// keep in sync with engine_common.h (no HIP types here: g++ compiles this)
struct DelayDesc {
  int size, age_old, age_new, pad;
  double w[4], omw[4];
};

void host_cis(double *cis);                                     // [19999][2] (cos, sin)
void host_twiddles(int nfft, double *tw, double *twi);          // [nfft][2] each
int host_rrc(double alpha, int firsize, double samplerate, double symbol_freq, double *points);
bool host_delay(double fractdelay, DelayDesc &d);
// Delay<double> of any length whose weights do not depend on the write pointer
bool host_delay_uniform(double fractdelay, int &size, int &age_old, int &age_new, double &w, double &omw);
// MskDemodulator matched filter, 2*sps taps (decode/mskdemodulator.cpp:126-133)
void host_jfft(double *x, int nfft, bool inverse, const double *tw, const double *twi);  // JFFT::fft, interleaved
void host_coarse_window(int nfft, double lockingbw, double fs, double *window);       // CoarseFreqEstimate window
void host_msk_taps(int sps, double *taps);
void host_scrambler(uint8_t *pre);                              // [5000]

// burst OQPSK: Delay<T> per-pointer weights and older slot, FFTrWrapper split
// tables, the Hilbert fast-FIR kernel (time domain, 8192 complex)
int host_delay_table(double fractdelay, double *w, double *omw, int *iold, int cap);
void host_fftr_split(int nfft, double *da, double *db);  // [nfft][2] each
void host_hilbert_kernel(double *k);                    // [8192][2]

// aero-publish channeliser designs (publish/oscillator.cpp:4-28,
// publish/dsp.cpp:181-215, publish/firfilter.cpp:47-99): FP32 as there
int host_pub_osc_len(double sampleRate);
void host_pub_osc(double sampleRate, double frequency, float *queue);  // [(int)sampleRate][2]
void host_pub_hilbert(int len, int Fs, float *points);                 // [len]
int host_pub_low_pass(double gain, double fs, double cutoff, double tw, float *taps, int cap);

}  // namespace aero
