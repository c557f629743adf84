/*
 * aero_synth.cpp — synthetic Aero P-channel transmitter (test/bench input).
 *
 * Produces what aero-publish would hand aero-decode for one VFO: 48 kHz real
 * int16 PCM of a 10500-bps OQPSK P-channel (SURVEY.md §8(d) C1/C2 input).
 * It inverts the receive chain of decode/aerol.cpp so that the reference
 * decoder recovers every signal unit it carries:
 *   SUs (12 B, CRC-16/X-25 LE, aerol.h:332-367) -> 26 per 0.5 s frame
 *   -> LSB-first bits (aerol.cpp:1509-1520) -> scrambler (aerol.h:406-440)
 *   -> K=7 r=1/2 {109,79} encoder, continuous across frames
 *      (jconvolutionalcodec.cpp:146-198, libcorrect conventions)
 *   -> 64x78 interleaver, inverse of deinterleave_ba (aerol.cpp:594-613)
 *   -> frame = 16 header + 178 dummy + 4992 data + 64 UW (aerol.cpp:1012-1021,
 *      UW 0xE15AE893 on both arms, aerol.cpp:933-936)
 *   -> OQPSK: even channel bits on Q, odd on I, Q leading I by T/2
 *      (oqpskdemodulator.cpp:437-445), RRC alpha=1, real carrier, AWGN.
 * ACARS payloads follow ParserISU's layout (aerol.cpp:333-489).
 *
 * Not part of the product path: tests/ and bench.py use it to make inputs.
 */
#include <cmath>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

extern "C" {
typedef struct {
  double fs;          /* 48000 */
  double carrier_hz;  /* e.g. 12037.5 */
  double phase0;      /* carrier phase, rad */
  double amplitude;   /* baseband scale (full scale = 1) */
  double ebn0_db;     /* >= 99: noiseless */
  uint64_t seed;
  double msg_rate;    /* probability of a new ACARS message when the SU queue is empty */
  int lead_in;        /* samples of noise before the first frame */
} aero_synth_cfg;

size_t aero_synth_p10500(const aero_synth_cfg *cfg, int16_t *pcm, size_t nsamples,
                         uint8_t *frames, size_t frames_cap);
/* 600/1200-bps MSK P-channel (cfg->fs = 12000 / 24000); frames: 72 info bytes each */
size_t aero_synth_msk(const aero_synth_cfg *cfg, int bitrate, int baud, int16_t *pcm, size_t nsamples,
                      uint8_t *frames, size_t frames_cap);
/* 8400-bps C channel; frames: 36 SU bytes + 300 voice bytes each */
size_t aero_synth_c8400(const aero_synth_cfg *cfg, int16_t *pcm, size_t nsamples, uint8_t *frames,
                        size_t frames_cap);
}

namespace {

struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed ? seed : 0x9E3779B97F4A7C15ULL) {}
  uint64_t next() {  // splitmix64
    uint64_t z = (s += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
  }
  double uniform() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
  int below(int n) { return (int)(uniform() * n); }
  double gauss() {
    double u1 = uniform(), u2 = uniform();
    if (u1 < 1e-300) u1 = 1e-300;
    return sqrt(-2.0 * log(u1)) * cos(2.0 * M_PI * u2);
  }
};

uint16_t crc16(const uint8_t *b, int n) {
  uint16_t crc = 0xFFFF;
  for (int i = 0; i < n; i++) {
    unsigned m = b[i];
    for (int k = 0; k < 8; k++) {
      unsigned bit = m & 1;
      m >>= 1;
      unsigned cb = crc & 1;
      crc >>= 1;
      if (cb ^ bit) crc ^= 0x8408;
    }
  }
  return (uint16_t)~crc;
}

uint8_t odd(uint8_t c) {
  c &= 0x7F;
  return (__builtin_popcount(c) & 1) ? c : (uint8_t)(c | 0x80);
}

struct SU {
  uint8_t b[12];
};

SU make_su(const uint8_t *ten) {
  SU s;
  memcpy(s.b, ten, 10);
  uint16_t c = crc16(ten, 10);
  s.b[10] = c & 0xFF;
  s.b[11] = c >> 8;
  return s;
}

struct Tx {
  aero_synth_cfg cfg;
  Rng rng;
  std::vector<SU> queue;
  std::vector<int> scr;
  int perm[64];
  unsigned enc_reg = 0;
  int frame_no = 0;
  std::vector<int> chan;  // channel bits of the current frame
  unsigned aes_pool[8];
  uint8_t refno = 0;

  explicit Tx(const aero_synth_cfg &c) : cfg(c), rng(c.seed) {
    std::vector<int> st = {1, 1, 0, 1, 0, 0, 1, 0, 1, 0, 1, 1, 0, 0, 1};
    scr.resize(5000);
    for (int a = 0; a < 5000; a++) {
      int v = st[0] ^ st[14];
      scr[a] = v;
      for (int i = 14; i > 0; i--) st[i] = st[i - 1];
      st[0] = v;
    }
    for (int i = 0; i < 64; i++) perm[i] = (i * 27) % 64;
    for (auto &a : aes_pool) a = 0x400000u + (unsigned)rng.below(0x3FFFFF);
  }

  void push_acars(unsigned aes, uint8_t ges, const std::string &reg, const std::string &label,
                  uint8_t bi, const std::string &text, bool more) {
    std::vector<uint8_t> ud;
    ud.push_back(0xFF);
    ud.push_back(0xFF);
    ud.push_back(odd(0x01));
    ud.push_back(odd('2'));
    for (int i = 0; i < 7; i++) ud.push_back(odd(i < (int)reg.size() ? reg[i] : '.'));
    ud.push_back(odd(0x15));
    ud.push_back(odd(label[0]));
    ud.push_back(odd(label[1]));
    ud.push_back(odd(bi));
    ud.push_back(odd(0x02));
    for (char ch : text) ud.push_back(odd((uint8_t)ch));
    ud.push_back(more ? 0x97 : 0x83);
    ud.push_back((uint8_t)rng.below(256));
    ud.push_back((uint8_t)rng.below(256));
    ud.push_back(0x7F);
    // ISU 0x71 + SSUs (ISUData::update, aerol.cpp:158-227)
    int rest = (int)ud.size() - 2;
    int m = (rest + 7) / 8;  // SSUs
    int r = rest - 8 * (m - 1);
    uint8_t qno = (uint8_t)rng.below(16), ref = (uint8_t)(refno++ & 0x0F);
    uint8_t isu[10] = {0x71, (uint8_t)(aes >> 16), (uint8_t)(aes >> 8), (uint8_t)aes, ges,
                       (uint8_t)((qno << 4) | ref), (uint8_t)(m & 0x3F), (uint8_t)(r << 4), ud[0], ud[1]};
    queue.push_back(make_su(isu));
    size_t p = 2;
    for (int s = m - 1; s >= 0; s--) {
      uint8_t ssu[10] = {(uint8_t)(0xC0 | s), (uint8_t)((qno << 4) | ref), 0, 0, 0, 0, 0, 0, 0, 0};
      int nb = s == 0 ? r : 8;
      for (int i = 0; i < nb; i++) ssu[2 + i] = ud[p++];
      for (int i = nb; i < 8; i++) ssu[2 + i] = (uint8_t)rng.below(256);
      queue.push_back(make_su(ssu));
    }
  }

  std::string rand_text(int n) {
    static const char *alpha = "ABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789 /.-,:";
    std::string t;
    for (int i = 0; i < n; i++) t += alpha[rng.below((int)strlen(alpha))];
    if (n > 20) t[n / 2] = '\r', t[n / 2 + 1] = '\n';
    return t;
  }

  void refill() {
    double u = rng.uniform();
    unsigned aes = aes_pool[rng.below(8)];
    uint8_t ges = (uint8_t)(0x80 + rng.below(8));
    if (u < cfg.msg_rate) {
      static const char *labels[] = {"H1", "SA", "_d", "Q0", "B6", "10", "5Z", "AA"};
      char reg[8];
      snprintf(reg, sizeof reg, ".N%05u", (unsigned)(aes % 100000));
      std::string label = labels[rng.below(8)];
      if (rng.uniform() < 0.15) {  // two-fragment message (ACARSDefragmenter)
        push_acars(aes, ges, reg, label, 'A', rand_text(40 + rng.below(60)), true);
        push_acars(aes, ges, reg, label, 'B', rand_text(10 + rng.below(40)), false);
      } else {
        push_acars(aes, ges, reg, label, (uint8_t)('A' + rng.below(26)),
                   rand_text(rng.below(180)), false);
      }
    } else if (u < cfg.msg_rate + 0.05) {  // log-on confirm (aerol.cpp:1730-1733)
      uint8_t su[10] = {0x11, (uint8_t)(aes >> 16), (uint8_t)(aes >> 8), (uint8_t)aes, ges, 0, 0, 0, 0, 0};
      for (int i = 5; i < 10; i++) su[i] = (uint8_t)rng.below(256);
      queue.push_back(make_su(su));
    } else if (u < cfg.msg_rate + 0.10) {  // C channel assignment (aerol.cpp:1804-1812)
      uint8_t su[10] = {0x34, (uint8_t)(aes >> 16), (uint8_t)(aes >> 8), (uint8_t)aes, ges, 0, 0, 0, 0, 0};
      for (int i = 5; i < 10; i++) su[i] = (uint8_t)rng.below(256);
      queue.push_back(make_su(su));
    } else {  // fill-in signal unit
      uint8_t su[10] = {0x01};
      for (int i = 1; i < 10; i++) su[i] = (uint8_t)rng.below(256);
      queue.push_back(make_su(su));
    }
  }

  // 600/1200-bps frame (aerol.cpp:975-993): 16 header + 1152 data (blocks of
  // N x 64, N = 6 / 9) + 32-bit UW at the end; 6 SUs = 72 info bytes
  void next_frame_msk(int N, uint8_t *info72) {
    uint8_t info[72];
    for (int k = 0; k < 6; k++) {
      while (queue.empty()) refill();
      memcpy(info + 12 * k, queue.front().b, 12);
      queue.erase(queue.begin());
    }
    if (info72) memcpy(info72, info, 72);
    int ibits[576];
    for (int h = 0; h < 576; h++) ibits[h] = ((info[h / 8] >> (h % 8)) & 1) ^ scr[h];
    int coded[1152];
    for (int t = 0; t < 576; t++) {
      enc_reg = ((enc_reg << 1) | (unsigned)ibits[t]) & 127;
      coded[2 * t] = __builtin_popcount(enc_reg & 109) & 1;
      coded[2 * t + 1] = __builtin_popcount(enc_reg & 79) & 1;
    }
    chan.assign(1200, 0);
    unsigned fc = (unsigned)(frame_no & 0xF);
    unsigned hdr = 0x1000u | ((unsigned)((frame_no >> 4) & 0xF) << 8) | (fc << 4) | fc;
    for (int b = 0; b < 16; b++) chan[b] = (hdr >> (15 - b)) & 1;
    const int B = N * 64;
    for (int b0 = 0; b0 < 1152; b0 += B)
      for (int j = 0; j < N; j++)
        for (int i = 0; i < 64; i++) chan[16 + b0 + perm[i] * N + j] = coded[b0 + j * 64 + i];
    const uint32_t uw = 0xE15AE893u;
    for (int j = 0; j < 32; j++) chan[1168 + j] = (uw >> (31 - j)) & 1;
    frame_no++;
  }

  // builds chan[] (5250 bits) for the next frame; info bytes to *info312
  void next_frame(uint8_t *info312) {
    uint8_t info[312];
    for (int k = 0; k < 26; k++) {
      while (queue.empty()) refill();
      memcpy(info + 12 * k, queue.front().b, 12);
      queue.erase(queue.begin());
    }
    if (info312) memcpy(info312, info, 312);
    // LSB-first bits, scrambled from position 0 (reset each frame)
    int ibits[2496];
    for (int h = 0; h < 2496; h++) ibits[h] = ((info[h / 8] >> (h % 8)) & 1) ^ scr[h];
    // encoder: table[r] bit j = parity(r & poly[j]); symbol j <-> poly[j]
    int coded[4992];
    for (int t = 0; t < 2496; t++) {
      enc_reg = ((enc_reg << 1) | (unsigned)ibits[t]) & 127;
      coded[2 * t] = __builtin_popcount(enc_reg & 109) & 1;
      coded[2 * t + 1] = __builtin_popcount(enc_reg & 79) & 1;
    }
    int blk[4992];
    for (int j = 0; j < 78; j++)
      for (int i = 0; i < 64; i++) blk[perm[i] * 78 + j] = coded[j * 64 + i];
    chan.assign(5250, 0);
    unsigned fc = (unsigned)(frame_no & 0xF);
    unsigned hdr = 0x1000u | ((unsigned)((frame_no >> 4) & 0xF) << 8) | (fc << 4) | fc;
    for (int b = 0; b < 16; b++) chan[b] = (hdr >> (15 - b)) & 1;
    for (int b = 16; b < 194; b++) chan[b] = rng.below(2);
    for (int b = 0; b < 4992; b++) chan[194 + b] = blk[b];
    const uint32_t uw = 0xE15AE893u;
    for (int j = 0; j < 32; j++) {
      int u = (uw >> (31 - j)) & 1;
      chan[5186 + 2 * j] = u;
      chan[5186 + 2 * j + 1] = u;
    }
    frame_no++;
  }
};

// RRC (alpha = 1) continuous pulse at t (in symbol periods)
double rrc1(double x) {
  const double a = 1.0;
  if (fabs(x) < 1e-12) return 1.0 - a + 4.0 * a / M_PI;
  if (fabs(fabs(x) - 0.25) < 1e-12)
    return a / sqrt(2.0) * ((1 + 2 / M_PI) * sin(M_PI / 4) + (1 - 2 / M_PI) * cos(M_PI / 4));
  return (sin(M_PI * x * (1 - a)) + 4 * a * x * cos(M_PI * x * (1 + a))) /
         (M_PI * x * (1 - 16 * a * a * x * x));
}

}  // namespace

extern "C" size_t aero_synth_p10500(const aero_synth_cfg *cfg, int16_t *pcm, size_t nsamples,
                                    uint8_t *frames, size_t frames_cap) {
  Tx tx(*cfg);
  const double Fs = cfg->fs, Ts = Fs / 5250.0;  // samples per arm symbol
  const int SPAN = 8;                           // +- symbols
  const int OS = 256;                           // table oversampling
  std::vector<double> tab(2 * SPAN * OS + 2);
  double energy = 0;
  for (size_t i = 0; i < tab.size(); i++) {
    tab[i] = rrc1((double)i / OS - SPAN);
  }
  for (int i = 0; i < 2 * SPAN * OS; i++) energy += tab[i] * tab[i];
  energy /= OS;  // integral of h^2 over symbol periods
  auto pulse = [&](double x) {
    double p = (x + SPAN) * OS;
    if (p <= 0 || p >= 2 * SPAN * OS) return 0.0;
    int ip = (int)p;
    double f = p - ip;
    return tab[ip] * (1 - f) + tab[ip + 1] * f;
  };
  // symbols: q[k] from chan bit 2k, i[k] from chan bit 2k+1, generated lazily
  std::vector<double> qs, is;
  size_t nframes = 0;
  auto ensure = [&](size_t k) {
    while (qs.size() <= k) {
      uint8_t *dst = (frames && nframes < frames_cap) ? frames + 312 * nframes : nullptr;
      tx.next_frame(dst);
      nframes++;
      for (int b = 0; b < 5250; b += 2) {
        qs.push_back(tx.chan[b] ? 1.0 : -1.0);
        is.push_back(tx.chan[b + 1] ? 1.0 : -1.0);
      }
    }
  };
  // power: A^2 * (E[I^2]+E[Q^2]) / 2 ; E[I^2] = energy (unit symbols, 1 per period)
  double A = cfg->amplitude;
  double P = A * A * (2.0 * energy) / 2.0;
  double sigma = 0;
  if (cfg->ebn0_db < 99) {
    double Eb = P / 10500.0;
    double N0 = Eb / pow(10.0, cfg->ebn0_db / 10.0);
    sigma = sqrt(N0 / 2.0 * Fs);
  }
  Rng nrng(cfg->seed ^ 0xA5A5A5A55A5A5A5AULL);
  const double w = 2.0 * M_PI * cfg->carrier_hz / Fs;
  for (size_t n = 0; n < nsamples; n++) {
    double x = 0;
    long long nn = (long long)n - cfg->lead_in;
    if (nn >= 0) {
      double t = (double)nn / Ts;  // in symbol periods; Q symbol k centred at k, I at k+0.5
      long long k0 = (long long)floor(t) - SPAN, k1 = (long long)floor(t) + SPAN + 1;
      if (k0 < 0) k0 = 0;
      ensure((size_t)k1 + 1);
      double I = 0, Q = 0;
      for (long long k = k0; k <= k1; k++) {
        Q += qs[k] * pulse(t - (double)k);
        I += is[k] * pulse(t - (double)k - 0.5);
      }
      double ph = w * (double)nn + cfg->phase0;
      x = A * (I * cos(ph) + Q * sin(ph));
    }
    if (sigma > 0) x += sigma * nrng.gauss();
    double v = floor(x * 32768.0 + 0.5);
    if (v > 32767) v = 32767;
    if (v < -32768) v = -32768;
    pcm[n] = (int16_t)v;
  }
  return nframes;
}

/* MSK: channel bits b_n are differentially encoded onto alternating arms so
 * that MskDemodulator's DiffDecode (decode/DSP.cpp:523-548) and its negated
 * real arm (decode/mskdemodulator.cpp:387-401) give them back: on the arm the
 * receiver reads first (imag) a 1 is a sign change, on the other a 1 is no
 * change.  Half-sine pulses over two bit periods (the receiver's matched
 * filter, mskdemodulator.cpp:126-133), arms offset by one bit period. */
extern "C" size_t aero_synth_msk(const aero_synth_cfg *cfg, int bitrate, int baud, int16_t *pcm, size_t nsamples,
                                 uint8_t *frames, size_t frames_cap) {
  // bitrate selects the frame layout (N = 6 / 9), baud the modulation rate.
  // aero-decode -b 1200 demodulates at fb = 600 (decode/decode.cpp:142-150
  // never sets fb), so only 600-baud input exercises its 1200 framing.
  Tx tx(*cfg);
  const int N = bitrate == 600 ? 6 : 9;
  const double Fs = cfg->fs, Tb = Fs / (double)baud;
  std::vector<double> arm;  // +-1 per channel bit
  size_t nframes = 0;
  double last = 1.0;
  auto ensure = [&](size_t k) {
    while (arm.size() <= k) {
      uint8_t *dst = (frames && nframes < frames_cap) ? frames + 72 * nframes : nullptr;
      tx.next_frame_msk(N, dst);
      nframes++;
      for (int b = 0; b < 1200; b++) {
        const size_t n = arm.size();
        const bool flip = (n % 2 == 0) ? !tx.chan[b] : tx.chan[b];
        last = flip ? -last : last;
        arm.push_back(last);
      }
    }
  };
  const double A = cfg->amplitude;
  const double P = A * A / 2.0;  // half-sine arms: E[I^2] = E[Q^2] = 1/2
  double sigma = 0;
  if (cfg->ebn0_db < 99) {
    double Eb = P / (double)baud;
    double N0 = Eb / pow(10.0, cfg->ebn0_db / 10.0);
    sigma = sqrt(N0 / 2.0 * Fs);
  }
  Rng nrng(cfg->seed ^ 0xA5A5A5A55A5A5A5AULL);
  const double w = 2.0 * M_PI * cfg->carrier_hz / Fs;
  for (size_t n = 0; n < nsamples; n++) {
    double x = 0;
    long long nn = (long long)n - cfg->lead_in;
    if (nn >= 0) {
      const double t = (double)nn / Tb;  // in bit periods
      const long long k1 = (long long)floor(t), k0 = k1 - 1;
      ensure((size_t)k1 + 1);
      double I = 0, Q = 0;
      for (long long k = k0; k <= k1; k++) {
        if (k < 0) continue;
        const double p = sin(M_PI * (t - (double)k) / 2.0);  // pulse over [k, k+2)
        if (k % 2 == 0)
          I += arm[k] * p;
        else
          Q += arm[k] * p;
      }
      const double ph = w * (double)nn + cfg->phase0;
      x = A * (I * cos(ph) + Q * sin(ph));
    }
    if (sigma > 0) x += sigma * nrng.gauss();
    double v = floor(x * 32768.0 + 0.5);
    if (v > 32767) v = 32767;
    if (v < -32768) v = -32768;
    pcm[n] = (int16_t)v;
  }
  return nframes;
}

/* ------------------------------------------------------------------ bursts
 * 10500-bps burst OQPSK (R / T channels, aero-decode --burst): per burst
 * 128 symbols of unmodulated carrier, 128 symbols of symbol tone, the UW on
 * both arms, then one R or T packet (decode/aerol.h:755-836 inverted):
 *   R: 17 bytes (RISU user-data SU, decode/aerol.cpp:32-119) + CRC = 152 bits
 *   T: 4-byte header + CRC, then S >= 2 SUs of 10 bytes + CRC (0x71 ISU + SSUs)
 * -> LSB-first bits, scrambled from 0, zero-padded to blockptr/2 - 6 bits, six
 * zero flush bits, K=7 {109,79} encoding (libcorrect, decode/jconvolutionalcodec.cpp:88-119)
 * -> 64 x (blockptr/64) interleaver, blockptr = 320 + 192 (S - 1).
 * Bursts are 1-3 s apart.  packets[] receives, per
 * burst, 2 x uint32 (kind 'R'/'T', byte count) + the packet bytes (<= 392). */
namespace {
struct BurstTx {
  Tx tx;
  unsigned risu_ref = 0;
  explicit BurstTx(const aero_synth_cfg &c) : tx(c) {}

  std::vector<uint8_t> acars_ud(unsigned aes, int maxtext) {
    char reg[8];
    snprintf(reg, sizeof reg, ".N%05u", (unsigned)(aes % 100000));
    static const char *labels[] = {"H1", "SA", "_d", "Q0", "B6", "10", "5Z", "AA"};
    const char *label = labels[tx.rng.below(8)];
    std::string text = tx.rand_text(1 + tx.rng.below(maxtext));
    std::vector<uint8_t> ud = {0xFF, 0xFF, odd(0x01), odd('2')};
    for (int i = 0; i < 7; i++) ud.push_back(odd(i < (int)strlen(reg) ? reg[i] : '.'));
    ud.push_back(odd(0x15));
    ud.push_back(odd(label[0]));
    ud.push_back(odd(label[1]));
    ud.push_back(odd((uint8_t)('A' + tx.rng.below(26))));
    ud.push_back(odd(0x02));
    for (char ch : text) ud.push_back(odd((uint8_t)ch));
    ud.push_back(0x83);
    ud.push_back((uint8_t)tx.rng.below(256));
    ud.push_back((uint8_t)tx.rng.below(256));
    ud.push_back(0x7F);
    return ud;
  }

  // queued packets (bytes incl. CRCs) + kind
  std::vector<std::pair<char, std::vector<uint8_t>>> pending;

  int t_maxtext = 40;  // T-packet text length bound (MSK bursts: the SU count must fit the burst window)
  void refill() {
    unsigned aes = tx.aes_pool[tx.rng.below(8)];
    uint8_t ges = (uint8_t)(0x80 + tx.rng.below(8));
    const double u = tx.rng.uniform();
    if (u < 0.35) {
      // a one-SU R user-data packet (SEQINDICATOR 1): too short for ACARS,
      // ParserISU reports it as a non-ACARS item (decode/aerol.cpp:471-488)
      uint8_t b[19] = {0};
      const int nb = 1 + tx.rng.below(11);
      b[0] = (uint8_t)((1 << 4) | nb);
      b[1] = (uint8_t)((tx.rng.below(16) << 4) | 0x08 | (risu_ref++ & 7));
      b[2] = (uint8_t)(aes >> 16);
      b[3] = (uint8_t)(aes >> 8);
      b[4] = (uint8_t)aes;
      b[5] = ges;
      for (int i = 0; i < 11; i++) b[6 + i] = (uint8_t)tx.rng.below(256);
      const uint16_t c = crc16(b, 17);
      b[17] = c & 0xFF;
      b[18] = c >> 8;
      pending.push_back({'R', std::vector<uint8_t>(b, b + 19)});
    } else if (u < 0.55) {
      // one ACARS message over three R bursts: SEQINDICATOR 4/5/6, 11 + 11 + r bytes
      std::vector<uint8_t> ud = acars_ud(aes, 13);
      while (ud.size() < 23) ud.insert(ud.end() - 4, odd('X'));  // keep the third SU non-empty
      const int r = (int)ud.size() - 22;
      const uint8_t qno = (uint8_t)tx.rng.below(16), ref = (uint8_t)(risu_ref++ & 7);
      for (int k = 0; k < 3; k++) {
        const int nb = k < 2 ? 11 : r;
        uint8_t b[19] = {0};
        b[0] = (uint8_t)(((4 + k) << 4) | nb);
        b[1] = (uint8_t)((qno << 4) | 0x08 | ref);
        b[2] = (uint8_t)(aes >> 16);
        b[3] = (uint8_t)(aes >> 8);
        b[4] = (uint8_t)aes;
        b[5] = ges;
        for (int i = 0; i < 11; i++) b[6 + i] = i < nb ? ud[11 * k + i] : (uint8_t)tx.rng.below(256);
        const uint16_t c = crc16(b, 17);
        b[17] = c & 0xFF;
        b[18] = c >> 8;
        pending.push_back({'R', std::vector<uint8_t>(b, b + 19)});
      }
    } else {
      // T packet: header + 0x71 ISU + SSUs (ISUData, decode/aerol.cpp:158-227)
      std::vector<uint8_t> ud = acars_ud(aes, t_maxtext);
      tx.queue.clear();
      // reuse the P-channel ISU/SSU builder on this message's user data
      const int rest = (int)ud.size() - 2;
      const int m = (rest + 7) / 8;
      const int r = rest - 8 * (m - 1);
      const uint8_t qno = (uint8_t)tx.rng.below(16), ref = (uint8_t)(tx.refno++ & 0x0F);
      std::vector<uint8_t> pkt;
      uint8_t hdr[4] = {(uint8_t)(aes >> 16), (uint8_t)(aes >> 8), (uint8_t)aes, ges};
      pkt.insert(pkt.end(), hdr, hdr + 4);
      uint16_t c = crc16(hdr, 4);
      pkt.push_back(c & 0xFF);
      pkt.push_back(c >> 8);
      uint8_t isu[10] = {0x71, (uint8_t)(aes >> 16), (uint8_t)(aes >> 8), (uint8_t)aes, ges,
                         (uint8_t)((qno << 4) | ref), (uint8_t)(m & 0x3F), (uint8_t)(r << 4), ud[0], ud[1]};
      SU s = make_su(isu);
      pkt.insert(pkt.end(), s.b, s.b + 12);
      size_t p = 2;
      for (int q = m - 1; q >= 0; q--) {
        uint8_t ssu[10] = {(uint8_t)(0xC0 | q), (uint8_t)((qno << 4) | ref), 0, 0, 0, 0, 0, 0, 0, 0};
        const int nb = q == 0 ? r : 8;
        for (int i = 0; i < nb; i++) ssu[2 + i] = ud[p++];
        for (int i = nb; i < 8; i++) ssu[2 + i] = (uint8_t)tx.rng.below(256);
        s = make_su(ssu);
        pkt.insert(pkt.end(), s.b, s.b + 12);
      }
      pending.push_back({'T', pkt});
    }
  }

  // channel bits of the next burst's packet part (after the UW).  MSK bursts
  // (decode/aerol.h:614-753) carry a T packet of S SUs in 320 + 192 S bits,
  // interleaved as a 64 x 5 section and then 64 x 3 sections
  // (AeroLInterleaver::deinterleaveMSK_ba, decode/aerol.cpp:651-686).
  std::vector<int> next_packet(char &kind, std::vector<uint8_t> &bytes, bool msk = false) {
    if (pending.empty()) refill();
    kind = pending.front().first;
    bytes = pending.front().second;
    pending.erase(pending.begin());
    const int nbytes = (int)bytes.size();
    const int S = kind == 'T' ? (nbytes - 6) / 12 : 1;
    const int blockptr = kind == 'R' ? 320 : 320 + 192 * (msk ? S : S - 1);
    const int dbits = blockptr / 2;
    std::vector<int> in(dbits, 0);
    for (int h = 0; h < 8 * nbytes && h < dbits - 6; h++) in[h] = ((bytes[h / 8] >> (h % 8)) & 1) ^ tx.scr[h];
    for (int h = 8 * nbytes; h < dbits - 6; h++) in[h] = tx.scr[h];  // decodes to zero pad bits
    std::vector<int> coded(blockptr);
    unsigned reg = 0;
    for (int t = 0; t < dbits; t++) {
      reg = ((reg << 1) | (unsigned)in[t]) & 127;
      coded[2 * t] = __builtin_popcount(reg & 109) & 1;
      coded[2 * t + 1] = __builtin_popcount(reg & 79) & 1;
    }
    const int cols = blockptr / 64;
    std::vector<int> blk(blockptr);
    if (!msk) {
      for (int j = 0; j < cols; j++)
        for (int i = 0; i < 64; i++) blk[tx.perm[i] * cols + j] = coded[j * 64 + i];
    } else {
      int k = 0;
      for (int j = 0; j < 5; j++)
        for (int i = 0; i < 64; i++) blk[tx.perm[i] * 5 + j] = coded[k++];
      for (int pb = 5; k < blockptr; pb += 3)
        for (int j = 0; j < 3; j++)
          for (int i = 0; i < 64; i++) blk[64 * pb + tx.perm[i] * 3 + j] = coded[k++];
    }
    return blk;
  }
};
}  // namespace

extern "C" size_t aero_synth_burst(const aero_synth_cfg *cfg, int16_t *pcm, size_t nsamples, uint8_t *packets,
                                   size_t packets_cap, size_t *npackets) {
  BurstTx bt(*cfg);
  const double Fs = cfg->fs, Ts = Fs / 5250.0;
  const int SPAN = 8, OS = 256;
  std::vector<double> tab(2 * SPAN * OS + 2);
  double energy = 0;
  for (size_t i = 0; i < tab.size(); i++) tab[i] = rrc1((double)i / OS - SPAN);
  for (int i = 0; i < 2 * SPAN * OS; i++) energy += tab[i] * tab[i];
  energy /= OS;
  auto pulse = [&](double x) {
    double p = (x + SPAN) * OS;
    if (p <= 0 || p >= 2 * SPAN * OS) return 0.0;
    int ip = (int)p;
    double f = p - ip;
    return tab[ip] * (1 - f) + tab[ip + 1] * f;
  };
  // symbol streams over the whole recording; 0 = silence
  const size_t nsym = (size_t)(nsamples / Ts) + 2 * SPAN + 4;
  std::vector<double> qs(nsym, 0.0), is(nsym, 0.0);
  size_t k = (size_t)(cfg->lead_in / Ts), np = 0, used = 0;
  while (true) {
    char kind;
    std::vector<uint8_t> bytes;
    std::vector<int> pk = bt.next_packet(kind, bytes);
    const size_t len = 256 + 32 + pk.size() / 2 + 16;
    if (k + len + 2 * SPAN >= nsym) break;
    for (int s = 0; s < 128; s++) qs[k + s] = is[k + s] = 1.0;  // carrier
    // symbol tone: Q alternates, I stays (of the four I/Q alternation patterns
    // this is the one BurstOqpskDemodulator's x4 symbol-tone PLL and arm
    // resolution lock to on every burst, burstoqpskdemodulator.cpp:466-493, 551-569)
    for (int s = 0; s < 128; s++) {
      qs[k + 128 + s] = (s & 1) ? -1.0 : 1.0;
      is[k + 128 + s] = 1.0;
    }
    size_t at = k + 256;
    const uint32_t uw = 0xE15AE893u;
    for (int j = 0; j < 32; j++, at++) qs[at] = is[at] = ((uw >> (31 - j)) & 1) ? 1.0 : -1.0;
    for (size_t b = 0; b < pk.size(); b += 2, at++) {
      qs[at] = pk[b] ? 1.0 : -1.0;
      is[at] = pk[b + 1] ? 1.0 : -1.0;
    }
    for (int s = 0; s < 16; s++, at++) {
      qs[at] = bt.tx.rng.below(2) ? 1.0 : -1.0;
      is[at] = bt.tx.rng.below(2) ? 1.0 : -1.0;
    }
    if (packets && used + 8 + bytes.size() <= packets_cap) {
      uint32_t h[2] = {(uint32_t)kind, (uint32_t)bytes.size()};
      memcpy(packets + used, h, 8);
      memcpy(packets + used + 8, bytes.data(), bytes.size());
      used += 8 + bytes.size();
    }
    np++;
    // next burst 1-3 s later
    k += (size_t)((1.0 + 2.0 * bt.tx.rng.uniform()) * 5250.0);
  }
  if (npackets) *npackets = np;
  double A = cfg->amplitude;
  double P = A * A * (2.0 * energy) / 2.0;
  double sigma = 0;
  if (cfg->ebn0_db < 99) {
    double Eb = P / 10500.0;
    double N0 = Eb / pow(10.0, cfg->ebn0_db / 10.0);
    sigma = sqrt(N0 / 2.0 * Fs);
  }
  Rng nrng(cfg->seed ^ 0xA5A5A5A55A5A5A5AULL);
  const double w = 2.0 * M_PI * cfg->carrier_hz / Fs;
  for (size_t n = 0; n < nsamples; n++) {
    const double t = (double)n / Ts;
    long long k0 = (long long)floor(t) - SPAN, k1 = (long long)floor(t) + SPAN + 1;
    if (k0 < 0) k0 = 0;
    if (k1 >= (long long)nsym) k1 = (long long)nsym - 1;
    double I = 0, Q = 0;
    for (long long kk = k0; kk <= k1; kk++) {
      if (qs[kk] != 0.0) Q += qs[kk] * pulse(t - (double)kk);
      if (is[kk] != 0.0) I += is[kk] * pulse(t - (double)kk - 0.5);
    }
    const double ph = w * (double)n + cfg->phase0;
    double x = A * (I * cos(ph) + Q * sin(ph));
    if (sigma > 0) x += sigma * nrng.gauss();
    double v = floor(x * 32768.0 + 0.5);
    if (v > 32767) v = 32767;
    if (v < -32768) v = -32768;
    pcm[n] = (int16_t)v;
  }
  return used;
}

/* 600/1200-bps burst MSK (R / T channels, aero-decode -b 600|1200 --burst).
 * aero-decode demodulates both rates with one fb = 1200 BurstMskDemodulator at
 * 48 kHz (decode/decode.cpp:123-132), so bursts are 1200-baud MSK: P1 bit
 * periods of unmodulated carrier (the trident check's "start tone",
 * decode/burstmskdemodulator.cpp:437-446), P2 of alternating frequency (the
 * 0-1 preamble whose lines sit fb/2 either side, :448-473), the UW, the packet
 * and a few random bits.  Data bits are differentially encoded onto
 * alternating half-sine arms exactly as aero_synth_msk does, generated as the
 * equivalent continuous-phase signal (+-90 degrees per bit period) so the
 * preamble and the data join without a phase step.  bitrate selects the
 * AeroL window (1800 / 3600 bits, decode/aerol.cpp:1031-1038) and so the
 * largest T packet; packets[] as aero_synth_burst. */
extern "C" size_t aero_synth_burst_msk(const aero_synth_cfg *cfg, int bitrate, int p1, int p2, int alt_sign,
                                       int16_t *pcm, size_t nsamples, uint8_t *packets, size_t packets_cap,
                                       size_t *npackets) {
  BurstTx bt(*cfg);
  bt.t_maxtext = bitrate == 600 ? 12 : 40;
  const double Fs = cfg->fs, T = Fs / 1200.0;
  const size_t nbits = (size_t)(nsamples / T) + 4;
  // phase (in quarter turns) at every bit boundary; NaN-free: silent bits flagged
  std::vector<int> quarter(nbits + 1, 0);
  std::vector<char> on(nbits, 0);
  size_t k = (size_t)(cfg->lead_in / T), np = 0, used = 0;
  int q = 0;
  while (true) {
    char kind;
    std::vector<uint8_t> bytes;
    std::vector<int> pk = bt.next_packet(kind, bytes, true);
    std::vector<int> data;
    const uint32_t uw = 0xE15AE893u;
    for (int j = 0; j < 32; j++) data.push_back((uw >> (31 - j)) & 1);
    data.insert(data.end(), pk.begin(), pk.end());
    for (int s = 0; s < 16; s++) data.push_back(bt.tx.rng.below(2));
    const size_t len = (size_t)p1 + (size_t)p2 + data.size();
    if (k + len + 2 >= nbits) break;
    size_t at = k;
    quarter[at] = q;
    for (int s = 0; s < p1; s++, at++) {  // carrier
      on[at] = 1;
      quarter[at + 1] = q;
    }
    for (int s = 0; s < p2; s++, at++) {  // alternating frequency
      on[at] = 1;
      q += ((s & 1) ? -alt_sign : alt_sign);
      quarter[at + 1] = q;
    }
    // data: arms a[n] (I on even n, Q on odd n), a 1 is a sign change on the
    // arm read first and no change on the other (aero_synth_msk); baseband
    // I - iQ turns by +90 deg * a[n] * a[n-1] over an even bit, -90 deg * ...
    // over an odd one
    int last = 1;
    for (size_t b = 0; b < data.size(); b++, at++) {
      const bool flip = (b % 2 == 0) ? !data[b] : data[b];
      const int a = flip ? -last : last;
      const int dq = ((b % 2 == 0) ? 1 : -1) * a * last;
      last = a;
      on[at] = 1;
      q += dq;
      quarter[at + 1] = q;
    }
    if (packets && used + 8 + bytes.size() <= packets_cap) {
      uint32_t h[2] = {(uint32_t)kind, (uint32_t)bytes.size()};
      memcpy(packets + used, h, 8);
      memcpy(packets + used + 8, bytes.data(), bytes.size());
      used += 8 + bytes.size();
    }
    np++;
    k = at + (size_t)((1.0 + 2.0 * bt.tx.rng.uniform()) * 1200.0);  // next burst 1-3 s later
    if (k >= nbits) break;
    for (size_t z = at + 1; z <= k && z <= nbits; z++) quarter[z] = q;
  }
  if (npackets) *npackets = np;
  const double A = cfg->amplitude;
  const double P = A * A / 2.0;
  double sigma = 0;
  if (cfg->ebn0_db < 99) {
    const double Eb = P / 1200.0;
    const double N0 = Eb / pow(10.0, cfg->ebn0_db / 10.0);
    sigma = sqrt(N0 / 2.0 * Fs);
  }
  Rng nrng(cfg->seed ^ 0xA5A5A5A55A5A5A5AULL);
  const double w = 2.0 * M_PI * cfg->carrier_hz / Fs;
  for (size_t n = 0; n < nsamples; n++) {
    const double t = (double)n / T;
    const size_t b = (size_t)t;
    double x = 0;
    if (b < nbits && on[b]) {
      const double u = t - (double)b;
      const double ph = (M_PI / 2.0) * ((double)quarter[b] * (1.0 - u) + (double)quarter[b + 1] * u);
      x = A * cos(w * (double)n + cfg->phase0 + ph);
    }
    if (sigma > 0) x += sigma * nrng.gauss();
    double v = floor(x * 32768.0 + 0.5);
    if (v > 32767) v = 32767;
    if (v < -32768) v = -32768;
    pcm[n] = (int16_t)v;
  }
  return used;
}

/* C channel (8400 bps OQPSK, AeroL::DecodeC, decode/aerol.cpp:2145-2415),
 * inverting the receive chain:
 *   three 12-byte SUs (CRC-16/X-25) at bits 109 y + 97 .. + 108 (y < 24) and
 *   25 x 96 voice bits at 109 y + 1 .. + 96 of a 2714-bit payload, scrambled
 *   from position 0 (reset at each UW, :2227)
 *   -> 2730 encoder input bits per frame: the receiver's Decode_Continuous
 *      window starts 6 bits before the frame's first bit and its 2708-bit
 *      delay line (:994-999) then hands back payload bits 0..2707 from
 *      positions 0..2707 of the previous frame and bits 2708..2713 from
 *      positions 2724..2729 (positions 2708..2723 are dummy)
 *   -> K=7 r=1/2 {109,79}, continuous; rate 3/4 by deleting every fourth
 *      symbol (PuncturedCode::depunture_soft_block(.., 4), :2417-2432), 4095
 *      symbols + 1 filler the receiver drops
 *   -> 16 interleaver blocks of 4 x 64 (deinterleave_ba(block, 4))
 *   -> frame: 52-bit preambles (0xC53D1C96ECD5 on Q, 0xAB376938BCA30 on I,
 *      :920-928), then the 4096 data bits: 4200 bits = 0.5 s
 *   -> OQPSK, RRC alpha = 0.6 (the receiver's prefilter, oqpskdemodulator.cpp:228-236).
 * frames: per frame 36 SU bytes + 300 voice bytes. */
namespace {
double rrc_a(double x, double a) {
  if (fabs(x) < 1e-12) return 1.0 - a + 4.0 * a / M_PI;
  if (fabs(fabs(x) - 1.0 / (4.0 * a)) < 1e-9)
    return a / sqrt(2.0) * ((1 + 2 / M_PI) * sin(M_PI / (4 * a)) + (1 - 2 / M_PI) * cos(M_PI / (4 * a)));
  return (sin(M_PI * x * (1 - a)) + 4 * a * x * cos(M_PI * x * (1 + a))) / (M_PI * x * (1 - 16 * a * a * x * x));
}

struct CTx {
  Tx tx;  // scrambler, interleaver permutation, encoder register, RNG
  explicit CTx(const aero_synth_cfg &c) : tx(c) {}
  std::vector<int> chan;
  // builds chan[] (4200 bits) for the next frame; SU and voice bytes to *rec336
  void next_frame(uint8_t *rec336) {
    uint8_t su[36], voice[300];
    for (int k = 0; k < 3; k++) {
      uint8_t ten[10];
      const double u = tx.rng.uniform();
      const unsigned aes = tx.aes_pool[tx.rng.below(8)];
      if (u < 0.4) {  // Call_progress (AEROTypeC, aerol.h:42-48): AES, GES
        ten[0] = 0x30;
        ten[1] = (uint8_t)(aes >> 16), ten[2] = (uint8_t)(aes >> 8), ten[3] = (uint8_t)aes;
        ten[4] = (uint8_t)(0x80 + tx.rng.below(8));
        for (int i = 5; i < 10; i++) ten[i] = (uint8_t)tx.rng.below(256);
      } else if (u < 0.55) {  // Telephony_acknowledge
        ten[0] = 0x60;
        for (int i = 1; i < 10; i++) ten[i] = (uint8_t)tx.rng.below(256);
      } else {  // fill-in
        ten[0] = 0x01;
        for (int i = 1; i < 10; i++) ten[i] = (uint8_t)tx.rng.below(256);
      }
      SU s = make_su(ten);
      memcpy(su + 12 * k, s.b, 12);
    }
    for (int i = 0; i < 300; i++) voice[i] = (uint8_t)tx.rng.below(256);
    if (rec336) {
      memcpy(rec336, su, 36);
      memcpy(rec336 + 36, voice, 300);
    }
    int pay[2714];
    for (int q = 0; q < 2714; q++) pay[q] = tx.rng.below(2);
    for (int b = 0; b < 288; b++) {  // LSB-first bytes
      const int y = b / 12, h = y * 109 + 97 + b % 12;
      pay[h] = (su[b / 8] >> (b % 8)) & 1;
    }
    for (int b = 0; b < 2400; b++) {
      const int y = b / 96, h = y * 109 + 1 + b % 96;
      pay[h] = (voice[b / 8] >> (b % 8)) & 1;
    }
    int ibits[2730];
    for (int q = 0; q < 2708; q++) ibits[q] = pay[q] ^ tx.scr[q];
    for (int q = 2708; q < 2724; q++) ibits[q] = tx.rng.below(2);
    for (int r = 0; r < 6; r++) ibits[2724 + r] = pay[2708 + r] ^ tx.scr[2708 + r];
    int coded[5460];
    for (int t = 0; t < 2730; t++) {
      tx.enc_reg = ((tx.enc_reg << 1) | (unsigned)ibits[t]) & 127;
      coded[2 * t] = __builtin_popcount(tx.enc_reg & 109) & 1;
      coded[2 * t + 1] = __builtin_popcount(tx.enc_reg & 79) & 1;
    }
    int deint[4096];
    int d = 0;
    for (int m = 0; m < 5460; m++)
      if (m % 4 != 3) deint[d++] = coded[m];
    deint[4095] = tx.rng.below(2);
    chan.assign(4200, 0);
    const uint64_t pq = 216866263330005ULL, pi = 3012071630031408ULL;
    for (int k = 0; k < 52; k++) {
      chan[2 * k] = (int)((pq >> (51 - k)) & 1);
      chan[2 * k + 1] = (int)((pi >> (51 - k)) & 1);
    }
    for (int b = 0; b < 16; b++)
      for (int j = 0; j < 4; j++)
        for (int i = 0; i < 64; i++) chan[104 + b * 256 + tx.perm[i] * 4 + j] = deint[b * 256 + j * 64 + i];
  }
};
}  // namespace

extern "C" size_t aero_synth_c8400(const aero_synth_cfg *cfg, int16_t *pcm, size_t nsamples, uint8_t *frames,
                                   size_t frames_cap) {
  CTx ct(*cfg);
  const double Fs = cfg->fs, Ts = Fs / 4200.0;  // samples per arm symbol
  const int SPAN = 10, OS = 256;
  std::vector<double> tab(2 * SPAN * OS + 2);
  double energy = 0;
  for (size_t i = 0; i < tab.size(); i++) tab[i] = rrc_a((double)i / OS - SPAN, 0.6);
  for (int i = 0; i < 2 * SPAN * OS; i++) energy += tab[i] * tab[i];
  energy /= OS;
  auto pulse = [&](double x) {
    double p = (x + SPAN) * OS;
    if (p <= 0 || p >= 2 * SPAN * OS) return 0.0;
    int ip = (int)p;
    double f = p - ip;
    return tab[ip] * (1 - f) + tab[ip + 1] * f;
  };
  std::vector<double> qs, is;
  size_t nframes = 0;
  auto ensure = [&](size_t k) {
    while (qs.size() <= k) {
      uint8_t *dst = (frames && nframes < frames_cap) ? frames + 336 * nframes : nullptr;
      ct.next_frame(dst);
      nframes++;
      for (int b = 0; b < 4200; b += 2) {
        qs.push_back(ct.chan[b] ? 1.0 : -1.0);
        is.push_back(ct.chan[b + 1] ? 1.0 : -1.0);
      }
    }
  };
  const double A = cfg->amplitude;
  const double P = A * A * (2.0 * energy) / 2.0;
  double sigma = 0;
  if (cfg->ebn0_db < 99) {
    const double Eb = P / 8400.0;
    const double N0 = Eb / pow(10.0, cfg->ebn0_db / 10.0);
    sigma = sqrt(N0 / 2.0 * Fs);
  }
  Rng nrng(cfg->seed ^ 0xC8400C8400C84001ULL);
  const double w = 2.0 * M_PI * cfg->carrier_hz / Fs;
  for (size_t n = 0; n < nsamples; n++) {
    double x = 0;
    const long long nn = (long long)n - cfg->lead_in;
    if (nn >= 0) {
      const double t = (double)nn / Ts;
      long long k0 = (long long)floor(t) - SPAN, k1 = (long long)floor(t) + SPAN + 1;
      if (k0 < 0) k0 = 0;
      ensure((size_t)k1 + 1);
      double I = 0, Q = 0;
      for (long long k = k0; k <= k1; k++) {
        Q += qs[k] * pulse(t - (double)k);
        I += is[k] * pulse(t - (double)k - 0.5);
      }
      const double ph = w * (double)nn + cfg->phase0;
      x = A * (I * cos(ph) + Q * sin(ph));
    }
    if (sigma > 0) x += sigma * nrng.gauss();
    double v = floor(x * 32768.0 + 0.5);
    if (v > 32767) v = 32767;
    if (v < -32768) v = -32768;
    pcm[n] = (int16_t)v;
  }
  return nframes;
}
