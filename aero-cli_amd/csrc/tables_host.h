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
void host_scrambler(uint8_t *pre);                              // [5000]

}  // namespace aero
