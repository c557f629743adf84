// hostcheck.cpp — CPU harness over the engine's host-side C++ (no GPU):
// aero-cli_amd/csrc/acars_host.cpp (SU dispatch, ISU reassembly, ACARS
// parsing and defragmenting, PChannelHost) and tables_host.cpp (the tables
// the kernels read: CIS, JFFT twiddles, RRC, MSK taps, scrambler, the
// aero-publish channeliser designs).  tests/test_hostcheck.py feeds it the
// oracle's CRC-checked frames and R/T packets and compares the items and
// tables with the oracle's; built plain and, by `build.py --asan`, with
// AddressSanitizer + UndefinedBehaviorSanitizer.
#include <cstring>
#include <vector>

#include "../aero-cli_amd/csrc/acars_host.h"
#include "../aero-cli_amd/csrc/tables_host.h"

extern "C" {

void *hc_create(int disable_reassembly) { return new aero::PChannelHost(disable_reassembly != 0); }
void hc_destroy(void *h) { delete static_cast<aero::PChannelHost *>(h); }
void hc_frame(void *h, const uint8_t *info, int len, uint32_t okmask, int formatid) {
  static_cast<aero::PChannelHost *>(h)->frame(info, len, okmask, formatid);
}
void hc_rt_packet(void *h, int r_packet, const uint8_t *info, int len, int nsus) {
  static_cast<aero::PChannelHost *>(h)->rt_packet(r_packet != 0, info, len, nsus);
}
// pops up to cap items (emission order); returns the number copied
size_t hc_items(void *h, aero_acars_item *dst, size_t cap) {
  auto &v = static_cast<aero::PChannelHost *>(h)->items;
  const size_t n = v.size() < cap ? v.size() : cap;
  for (size_t i = 0; i < n; i++) dst[i] = v[i];
  v.erase(v.begin(), v.begin() + (long)n);
  return n;
}

void hc_cis(double *cis) { aero::host_cis(cis); }
void hc_twiddles(int nfft, double *tw, double *twi) { aero::host_twiddles(nfft, tw, twi); }
int hc_rrc(double alpha, int firsize, double fs, double symfreq, double *pts) {
  return aero::host_rrc(alpha, firsize, fs, symfreq, pts);
}
void hc_msk_taps(int sps, double *taps) { aero::host_msk_taps(sps, taps); }
void hc_scrambler(uint8_t *pre) { aero::host_scrambler(pre); }
int hc_pub_low_pass(double gain, double fs, double cutoff, double tw, float *taps, int cap) {
  return aero::host_pub_low_pass(gain, fs, cutoff, tw, taps, cap);
}
void hc_pub_hilbert(int len, int fs, float *pts) { aero::host_pub_hilbert(len, fs, pts); }
int hc_pub_osc_len(double fs) { return aero::host_pub_osc_len(fs); }
void hc_pub_osc(double fs, double freq, float *q) { aero::host_pub_osc(fs, freq, q); }
}
