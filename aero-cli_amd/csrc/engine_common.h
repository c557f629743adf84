/*
 * engine_common.h — device-side state layout of the Aero engine (10500-bps
 * continuous OQPSK, decode/oqpskdemodulator.cpp + decode/aerol.cpp).
 *
 * One channel (VFO) per lane.  All per-channel state is struct-of-arrays in
 * HBM: field f of channel c lives at base[f * C + c], so a wavefront loads
 * and stores 64 consecutive channels with one coalesced access.  Rings whose
 * pointer advances in lockstep for every channel (AGC) are time-major; rings
 * whose pointer depends on each channel's symbol clock (moving averages,
 * delay lines, the coarse-estimator history) are channel-major so a lane's
 * successive accesses stay in one cache line.
 */
#pragma once
#include <stdint.h>

#include "aero_math.h"    // div_cw (set_phase_ptr)
#include "tables_host.h"  // DelayDesc

namespace aero {

constexpr int WTSIZE = 19999;         // decode/DSP.h:21
constexpr int NTAPS = 55;             // RRC taps (decode/oqpskdemodulator.cpp:177)
constexpr int AGC_LEN = 192000;       // AGC(4, 48000) (decode/DSP.cpp:361)
constexpr int MARG_LEN = 800;         // MovingAverage(800) (oqpskdemodulator.cpp:41)
constexpr int DT_LEN = 401;           // DelayThing.setLength(400) (oqpskdemodulator.cpp:42)
constexpr int MSE_LEN = 400;          // MSEcalc(400) (oqpskdemodulator.cpp:50)
constexpr int NFFT = 16384;           // coarse estimator 2^14 (decode/decode.cpp:152)
constexpr int HOP = 4096;             // 75 % overlap (oqpskdemodulator.cpp:357)
constexpr int SOFT_RING = 4096;       // per-channel soft-bit ring (power of 2)
constexpr int Y_LO = 2815, Y_HI = 13568;  // y[] bins the fold search reads
constexpr int Y_LEN = Y_HI - Y_LO + 1;
constexpr int BLOCK = 4992;           // 78 x 64 interleaver block (aerol.cpp:1012-1016)
constexpr int DL2_LEN = 4987;         // DelayLine setLength(4992-6) (aerol.cpp:1015)
constexpr int VIT_MAX = 5078;         // 62 overlap + 4992 + 24 pad
constexpr int JOB_OUT = 328;          // 312 infofield + len + mask + formatid + channel
constexpr int DCD_TICK_RING = 4;      // LS_TICK_SOFT0.. entries (ticks recorded, not yet applied)

// channel kinds, one engine group per kind: 10500-bps OQPSK, and continuous
// MSK per (demodulator sample rate, AeroL bit rate).  aero-decode configures
// 600 bps at 12 kHz and 1200 bps at 24 kHz (decode/decode.cpp:142-150); a
// message at another rate re-applies the MSK settings at that rate
// (MskDemodulator::dataReceived, decode/mskdemodulator.cpp:473-481, settings
// :94-218) and the channel moves to the group of that rate (engine.hip
// msk_migrate).  12000, 24000 and 48000 (the VFO rates aero-publish is
// configured with by default, publish/publisher.cpp:164-176) have groups of
// their own, compiled for that rate; every other rate in [MSK_FS_MIN,
// MSK_FS_MAX] runs in a group of the generic-rate kernels (MODE_MSKG600 /
// MODE_MSKG1200, rate-dependent constants in DevState::mg).
enum Mode : int {
  MODE_OQPSK = 0,
  MODE_MSK600 = 1,       // 600 bps, 12 kHz
  MODE_MSK1200 = 2,      // 1200 bps, 24 kHz
  MODE_MSK600_24K = 3,
  MODE_MSK600_48K = 4,
  MODE_MSK1200_12K = 5,
  MODE_MSK1200_48K = 6,
  MODE_COUNT = 7
};
// the kernel families of the generic-rate MSK groups (engine group ids of
// such groups are above MODE_COUNT; Group::mode holds one of these)
constexpr int MODE_MSKG600 = 8, MODE_MSKG1200 = 9;
constexpr bool msk_generic(int m) { return m == MODE_MSKG600 || m == MODE_MSKG1200; }
// The C channel (8400 bps OQPSK, AeroL::DecodeC): its own
// kernel family and a fixed engine group slot after the fixed-rate MSK ones
// (generic-rate MSK groups are appended after it).  OqpskDemodulator at
// fb = 8400 (decode/oqpskdemodulator.cpp:136-254, 284-560) prefilters every
// message with a JFastFir between a down- and an up-mix by mixer_fir_pre and
// retunes that mixer to the message's mean carrier, so unlike the P channel
// its output depends on the message boundaries: the group keeps them.
constexpr int MODE_C8400 = 10;
constexpr int GID_C8400 = MODE_COUNT;
constexpr int C_FRAME = 4096;         // AERO_SPEC_NumberOfBits (aerol.cpp:994-1004)
constexpr int C_BLOCK = 5460;         // depunctured frame: 4095 soft bits + 1365 erasures (aerol.cpp:2417-2432)
constexpr int C_DL2_LEN = 2709;       // dl2.setLength(2714 - 6) + 1
constexpr int C_PAYLOAD = 2714;       // deconvol.resize(2714) (aerol.cpp:2249)
constexpr int C_FIR_N = 4096;         // fir_pre.SetKernel(RRC 0.6 x 2049 taps, 4096) (oqpskdemodulator.cpp:228-236)
constexpr int C_FIR_SNZ = 2048;       // signal_non_zero_size = 4096 + 1 - 2049 (jfft.cpp:347-352)
constexpr int C_OUT_RING = 32768;     // prefiltered (before the up-mix) samples per channel: one message, <= half the PCM ring
constexpr int C_IN_RING = 65536;      // down-mix words per channel: a message plus the block it starts in
constexpr int JOB_OUT_C = 352;        // 36 SU bytes + 300 voice bytes + len, mask, AES, channel
// MSK sample rates served.  Below 12000 the coarse estimator's fold search
// would read y bins outside the range every MSK group keeps (MSK_YLO..MSK_YHI,
// which a channel carries over a rate change); aero-publish's VFO rate is
// at least the configured out_rate (its decimation count is
// int(log2(Fs / out_rate)), publish/publisher.cpp:196-210), 12000 by default
// for 600 bps.  Above 96000 the per-channel AGC ring (Fs doubles) and matched
// filter (2 Fs / 600 taps) grow past what a group is sized for; aero-publish
// produces less than twice out_rate (48000 at most by default).
constexpr int MSK_FS_MIN = 12000, MSK_FS_MAX = 96000;
constexpr int msk_fs(int m) {
  return (m == MODE_MSK600 || m == MODE_MSK1200_12K) ? 12000
                                                      : ((m == MODE_MSK1200 || m == MODE_MSK600_24K) ? 24000 : 48000);
}
constexpr int msk_bitrate(int m) {
  return (m == MODE_MSK600 || m == MODE_MSK600_24K || m == MODE_MSK600_48K || m == MODE_MSKG600) ? 600 : 1200;
}
// the fixed-rate MSK group of (AeroL bit rate, sample rate), or -1 (a
// generic-rate group serves the rate, or none)
inline int msk_mode(int bitrate, int fs) {
  for (int m = MODE_MSK600; m < MODE_COUNT; ++m)
    if (msk_bitrate(m) == bitrate && msk_fs(m) == fs) return m;
  return -1;
}

// continuous MSK (MskDemodulator as Decoder configures it, decode/decode.cpp:142-150,
// decode/mskdemodulator.cpp:94-218): fb stays 600 whatever the bit rate, so the
// demodulator depends on Fs only (SPS = Fs / 600, matched filter 2 SPS taps,
// AGC(1, Fs), the st resonator design and IfHavePassedPoint point chosen by
// Fs, :177-203); the AeroL framing on the bit rate
template <int M>
struct MskK {
  static constexpr int FS = msk_fs(M), SPS = FS / 600, BITRATE = msk_bitrate(M), LEAVER = BITRATE == 600 ? 6 : 9,
                       WG = SPS == 20 ? 256 : (SPS == 40 ? 128 : 64);
  static constexpr bool F48 = FS == 48000;  // "300hz / 4hz / 48000" design, else "300hz / 4hz / 12000"
  static constexpr double SR_B0 = F48 ? 1.308825621597620e-04 : 5.233248111921052e-04;
  static constexpr double SR_B2 = -SR_B0;
  static constexpr double SR_A1 = F48 ? -1.998196509168551 : -1.974342917561558;
  static constexpr double SR_A2 = F48 ? 0.999738234875681 : 0.998953350377616;
  static constexpr double EE = F48 ? 0.025 : 0.0125;
};
constexpr int MAX_TAPS = 2 * (MSK_FS_MAX / 600);  // matched filter / RRC taps a group table holds (MSK 96 kHz: 320)
constexpr int MSK_NFFT = 8192;          // coarsefreqest_fft_power 13 (mskdemodulator.h:26)
constexpr int MSK_HOP = 2048;           // 75 % overlap (mskdemodulator.cpp:289-291)
constexpr int MSK_MSEMA = 600;          // msema = MovingAverage(600) (mskdemodulator.cpp:57)
constexpr int MSK_BLOCK_MAX = 9 * 64;   // 576
constexpr int MSK_DL2_LEN = 571;        // dl2.setLength(576 - 6) (aerol.cpp:979,988)
// y[] bins every MSK group keeps: the fold search at 12 kHz reads
// round(+-lockingbw/hzperbin + nfft/2) +- (expectedpeakbin + 1), and the
// ranges at 24 and 48 kHz lie inside it, so a channel that changes rate finds
// the history it needs (the reference keeps y over a rate change,
// coarsefreqestimate.cpp:39-76 only resizes it)
constexpr int MSK_YLO = 3276, MSK_YHI = 4915;

// per-mode geometry shared by the host layout and the kernels
struct ModeGeom {
  int fs, nfft, hop, agc_len, ntaps, marg_len, dt_len, ms_len, dsm_len, d8_len, block, leaver, dl2_len, y_lo,
      y_hi, soft_group;
};
// MSK at sample rate fs: SPS = int(Fs / fb) (mskdemodulator.cpp:110), the
// matched filter 2 SPS taps, AGC(1, Fs), marg SPS, dt SPS/2 (+1 slot),
// delayedsmpl SPS (+1), delayt8 ceil(SPS/2) + 1 (DSP.h:360-362)
inline ModeGeom msk_geom(int bitrate, int fs) {
  const int sps = fs / 600, leaver = bitrate == 600 ? 6 : 9;
  return {fs,      MSK_NFFT,          MSK_HOP,     fs,          2 * sps, sps,     sps / 2 + 1, MSK_MSEMA,
          sps + 1, (sps + 1) / 2 + 1, leaver * 64, leaver, MSK_DL2_LEN, MSK_YLO, MSK_YHI, 12};
}
inline ModeGeom mode_geom(int m) {
  if (m == MODE_OQPSK) return {48000, 16384, 4096, 192000, 55, 800, 401, 400, 0, 0, 4992, 78, 4987, 2815, 13568, 32};
  if (m == MODE_C8400) return {48000, 16384, 4096, 192000, 55, 800, 401, 400, 0, 0, C_BLOCK, 4, C_DL2_LEN, 2815, 13568, 32};
  return msk_geom(msk_bitrate(m), msk_fs(m));
}

// the rate-dependent constants of a generic-rate MSK group, host-computed as
// MskDemodulator::setSettings (decode/mskdemodulator.cpp:94-218, fb 600) and
// CoarseFreqEstimate::setSettings(13, 900, 600, Fs)
// (decode/coarsefreqestimate.cpp:39-76) compute them
struct MskGen {
  double fs;
  double sr_b0, sr_b2, sr_a1, sr_a2;  // st_iir_resonator ("300hz / 4hz / 12000" design: Fs != 48000)
  double ee;                          // IfHavePassedPoint(ee)
  double d8w, d8omw;                  // delayt8 weights (the same at every ring pointer)
  int sps, d8_old, d8_new;            // delayt8 ages of older / newer
  int start, stop, ilo, ihi, epb;     // boxcar startbin..stopbin, fold [ilo, ihi), expectedpeakbin
};

// double state fields
enum DS : int {
  DS_M2_PTR, DS_M2_STEP, DS_M2_FREQ,
  DS_MC_PTR, DS_MC_STEP, DS_MC_FREQ,
  DS_SO_PTR, DS_SO_LAST, DS_SO_STEP, DS_SO_FREQ,
  DS_AGC_SUM,
  DS_D1_0, DS_D1_1,
  DS_D41_0, DS_D41_1, DS_D41_2, DS_D41_3,
  DS_D42_0, DS_D42_1, DS_D42_2, DS_D42_3,
  DS_D8_0, DS_D8_1, DS_D8_2,
  DS_SR_X1, DS_SR_X2, DS_SR_Y1, DS_SR_Y2,
  DS_CT_X1, DS_CT_X2, DS_CT_Y1, DS_CT_Y2,
  DS_MARG_SUM, DS_PM_SUM, DS_MS_SUM,
  DS_MSE,
  DS_PTD_RE, DS_PTD_IM, DS_S2L_RE, DS_S2L_IM,
  DS_DIFF_LAST,   // MSK DiffDecode::lastsoftstate (decode/DSP.cpp:517-520)
  // SignalHunter::newFreqCenter values (decode/hunter.cpp:34-40) of the last
  // eight steps: step k (1-based) at DS_HUNT_FC0 + ((k - 1) & 7)
  DS_HUNT_FC0, DS_HUNT_FC_END = DS_HUNT_FC0 + 7,
  // C channel: mixer_fir_pre (phase pointer, step, Hz) and the message's
  // running sum of mixer2's frequency (oqpskdemodulator.cpp:385, 557)
  DS_FP_PTR, DS_FP_STEP, DS_FP_FREQ, DS_M2_FSUM,
  DS_COUNT
};

// int state fields
enum IS : int {
  IS_AGC_PTR, IS_D1_P, IS_D41_P, IS_D42_P, IS_D8_P,
  IS_MARG_P, IS_DT_P, IS_PM_P, IS_MS_P,
  IS_YUI, IS_S2L_INIT,
  // hop / hunter state (decode/oqpskdemodulator.cpp:572,586; decode/hunter.cpp)
  IS_COUNTDOWN2, IS_COUNTDOWN, IS_HUNT_ITER, IS_HUNT_SCANS, IS_EMPTYCD, IS_YRESET,
  IS_HOPS_DONE,
  // AeroL framing (decode/aerol.cpp:1060-2038)
  IS_RI, IS_CNTR, IS_GSL, IS_UWI, IS_UWR, IS_UWI_INV, IS_UWR_INV,
  IS_FRAMEINFO, IS_LASTFRAMEINFO, IS_FORMATID, IS_DATACD, IS_DATACDCD,
  IS_SCR_POS, IS_BLKBUF, IS_HAS_OVERLAP, IS_DL2_PTR,
  IS_MSK_PD,      // MSK PreambleDetector shift register (aerol.cpp:716-725)
  IS_BLK_SINCE_CLEAR,  // blocks appended to the infofield since cntr == 0
  // decoder status events (decode/decode.cpp:429-439): DataCarrierDetect
  // changes as SignalHunter::handleDcd sees them, newFreqCenter emissions
  IS_DCD_EDGES, IS_HUNT_STEPS,
  // MSK: msema's slot offset (its pointer keeps running over a rate change
  // while marg and dt restart with the event counter)
  IS_MS_OFF,
  // AeroL's 1 s DCD timer on the sample clock (AERO_F_DCD_TICK, continuous
  // OQPSK; decode/aerol.cpp:900-902, 1043-1058): datacdcountdown; a frame
  // whose SU CRCs the framing has not seen yet (the Viterbi writes its CRC-ok
  // mask and SU count); ticks the demod recorded and the framing applied
  IS_DCD_COUNT, IS_CRC_PEND, IS_CRC_OKM, IS_CRC_NSU, IS_TICK_REC, IS_TICK_DONE,
  // C channel framing: the 4 x 64 block index (AeroL ctor: index = 0, aerol.cpp:931)
  IS_C_INDEX,
  IS_COUNT
};

// 64-bit counters
enum LS : int {
  LS_NSAMP,       // samples demodulated
  LS_AVAIL,       // samples pushed
  LS_FILLED,      // coarse-ring entries written (samples < filled)
  LS_ZERO_BEFORE, // coarse-ring entries of samples < this are zero
  LS_SOFT_P,      // soft bits produced
  LS_SOFT_C,      // soft bits consumed by AeroL
  LS_PT_N,        // pt trace records
  LS_EVENTS,      // MSK symbol events (ring pointer of marg / dt / msema)
  // DCD tick k (k = 0, 1, ...: after (k + 1) * 48000 samples) happens before
  // delivered soft bit LS_TICK_SOFT0 + (k & 3) (a multiple of 32)
  LS_TICK_SOFT0, LS_TICK_SOFT_END = LS_TICK_SOFT0 + 3,
  // C channel: samples prefiltered (the demod stops there: a message end),
  // the current message's first sample; the 52-bit shift registers of the
  // two dual-preamble detectors (real: r1, r2; imag: i1, i2, aerol.cpp:782-877)
  LS_PRE_END, LS_MSG_START, LS_C_R1, LS_C_R2, LS_C_I1, LS_C_I2,
  LS_COUNT
};


struct DevTables {
  const double2 *cis;      // [WTSIZE] (CosWT, SinWT)   decode/DSP.cpp:10-33
  const double2 *tw;       // [NFFT] forward twiddles   decode/jfft.cpp:41-53
  const double2 *twi;      // [NFFT] inverse twiddles
  const double2 *twg;      // the coarse transforms' stages past the LDS copy, permuted to the threads' order (fft_layout.h)
  const double2 *twgi;     // the same of the inverse table
  const uint8_t *scr;      // [5000] scrambler bits      decode/aerol.h:408-427
  const double *taps;      // [ntaps] RRC (OQPSK) / half-sine matched filter (MSK)
  // C channel: JFastFir kernel spectrum and the 4096-point twiddles
  // (decode/jfft.cpp:324-367), the coarse estimator's raised-cosine window
  // (decode/coarsefreqestimate.cpp:60-74)
  const double2 *cker, *tw4, *twi4;
  const double *cwin;
};

struct DevState {
  int C;                   // channel stride
  int mode;                // Mode
  int dcd_tick;            // AERO_F_DCD_TICK on a continuous OQPSK group
  ModeGeom g;              // ring and block sizes of this group
  MskGen mg;               // generic-rate MSK groups: the rate's constants
  double *ds;              // [DS_COUNT][C]
  int *is;                 // [IS_COUNT][C]
  long long *ls;           // [LS_COUNT][C]
  double *fir;             // [2*NTAPS][C] transposed-FIR partial sums
  double *agc;             // [agc_len][C]
  double2 *dsm;            // MSK delayedsmpl ring [dsm_len][C] (time-major, slot = n % len)
  double *d8;              // MSK delayt8 ring [d8_len][C] (time-major)
  double *marg;            // [C][marg_len]
  double2 *dt;             // [C][dt_len]
  double *pm, *ms;         // OQPSK: pm = [C][ms_len] (pm, ms) double2 pairs; MSK: ms = msema [C][ms_len]
  int16_t *pcm;            // [PCM_CAP][C] input ring (time-major)
  long long pcm_cap;       // power of 2
  uint32_t *cring;         // [C][nfft] coarse ring: cis index | pcm << 16 (demod-written)
                           // CIS * pcm / 32768 (coarse-written, one hop per run)
  double *y;               // [C][y_hi - y_lo + 1] coarse smoothing state
  uint8_t *soft;           // [C][SOFT_RING]
  double2 *pt;             // [C][pt_cap] (trace only)
  long long pt_cap;
  double *hops;            // [C][hop_cap][6] per-run hop trace
  int hop_cap;
  int *hop_n;              // [C]
  uint8_t *block;          // [C][2][block] double-buffered interleaver block
  uint8_t *overlap;        // [C][64]
  uint8_t *dl2;            // [C][dl2_len]
  int *jobs;               // [C] job list: channel | (buf << 24)
  int *njobs;              // [1]
  uint8_t *jobout;         // [C][JOB_OUT] (the Viterbi writes it in pinned host memory)
  int *njobs_host;         // [1] pinned host copy of the job count, written by the Viterbi kernel
  uint8_t *blocks_dbg;     // [C][2500] decoded bits (trace)
  uint32_t *cin;           // C channel: [C][C_IN_RING] the down-mix's table index | pcm << 16 per sample
  double2 *cout;           // C channel: [C][C_OUT_RING] JFastFir outputs (the up-mix is the demod's)
  double2 *csig;           // C channel: [C][C_FIR_SNZ] outputs of the last block transform (samples past its message)
  double2 *crem;           // C channel: [C][C_FIR_N - C_FIR_SNZ] JFastFir remainder
  int *err;                // [1] mapped pinned device-error word (DERR_*), sticky; read by the host
};

#if defined(__HIPCC__)
// WaveTable's pointer wraps (DSP.h:59-65's loops) with their first iteration
// as a select and the rest behind a wave-uniform test: the same iterations in
// the same order (a peeled loop), without a divergent loop's exec-mask
// bookkeeping on the per-sample path
__device__ __forceinline__ void wt_wrap(double &ptr) {
  ptr = ptr >= WTSIZE ? ptr - WTSIZE : ptr;
  if (__builtin_expect(__any(ptr >= WTSIZE), 0))
    while (ptr >= WTSIZE) ptr -= WTSIZE;
  ptr = ptr < 0 ? ptr + WTSIZE : ptr;
  if (__builtin_expect(__any(ptr < 0), 0))
    while (ptr < 0) ptr += WTSIZE;
}
// WTnextFrame's wrap (DSP.cpp:71-79), peeled the same way
__device__ __forceinline__ void wt_wrap_int(double &ptr) {
  ptr = ((int)ptr) >= WTSIZE ? ptr - WTSIZE : ptr;
  if (__builtin_expect(__any(((int)ptr) >= WTSIZE), 0))
    while (((int)ptr) >= WTSIZE) ptr -= WTSIZE;
}
// SetPhaseDeg (DSP.cpp:177-187): fmod(x, 360), the loop that adds 360 while
// negative, and the pointer (phase / 360) W.  For -360 < x < 720 fmod is x or
// the exact x - 360 (Sterbenz), and its remainder is above -360, so the loop
// adds at most once; other waves take fmod.  The quotient by div_cw.
__device__ __forceinline__ double set_phase_ptr(double x) {
  const bool in = x > -360.0 && x < 720.0;
  double r = x >= 360.0 ? x - 360.0 : x;
  if (__builtin_expect(__any(!in), 0)) r = in ? r : fmod(x, 360.0);
  r = r < 0 ? r + 360.0 : r;
  return div_cw(r, 360.0) * ((double)WTSIZE);
}
#endif

// device error codes (DevState::err)
constexpr int DERR_HANDOFF = 1;  // a demod wave pair's LDS hand-off timed out
constexpr int DERR_TICKS = 2;    // DCD ticks recorded faster than the framing applied them

}  // namespace aero
