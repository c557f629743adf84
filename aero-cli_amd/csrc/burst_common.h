/*
 * burst_common.h — layout shared by the burst-mode kernels (burst.hip:
 * 10500-bps OQPSK, burst_msk.hip: 600/1200-bps MSK) and their host
 * (burst_engine.hip).  OQPSK geometry from BurstOqpskDemodulator's constructor
 * and setSettings (decode/burstoqpskdemodulator.cpp:5-232) at Fs 48000,
 * fb 10500 (SamplesPerSymbol = 9.142857); MSK geometry from
 * BurstMskDemodulator::setSettings (decode/burstmskdemodulator.cpp:119-297) at
 * Fs 48000, fb 1200 (SamplesPerSymbol = 40, the fb >= 1200 branch, which
 * aero-decode uses for both MSK bit rates, decode/decode.cpp:123-132); AeroL's
 * R/T block (decode/aerol.h:614-836).
 */
#pragma once
#include <stdint.h>

namespace aero {

constexpr int HB_N = 8192;       // JFastFir block (decode/jfft.cpp:322-374): nfft >= 4 * 2048
constexpr int HB_SNZ = 6145;     // signal_non_zero_size = nfft + 1 - 2048
constexpr int HB_REM = 2047;     // remainder_size
constexpr int ANA_LEN = 65536;   // analytic-signal ring (time-major), >= PCM ring + 2 blocks
constexpr int B_AGC = 48000;     // agc.init(1, Fs)
constexpr int B_AGC2 = 585;      // agc2.init(SPS * 64 / Fs, Fs)
constexpr int B_D1 = 2736;       // d1.setLength(SPS * 128 * 2.5 - 190) + 1
constexpr int B_D2 = 2634;       // d2.setLength(tridentbuffer_sz) + 1
constexpr int B_TRI = 2633;      // tridentbuffer_sz = qRound(288 * SPS)
constexpr int B_TRI_HALF = 1170; // qRound(128 * SPS): base / top halves of the trident check
constexpr int B_MA = 1170;       // bt_ma1 (complex) and mav1 lengths
constexpr int B_PD1 = 1171, B_PD2 = 586, B_PD3 = 1171;  // PeakDetector d1 / d2 / d3 (length 585)
// d1 and d2 are read from d3's ring (burst.hip front_burst_kernel)
static_assert(B_PD1 == B_PD3 && B_PD2 <= B_PD3, "peak detector rings");
constexpr int B_PD_MAXCD = 1170; // 2 * length
constexpr int B_MSEMA = 128;
constexpr int B_STARTSTOP = 9600;  // SPS * 1050
constexpr int B_SOFT_RING = 16384; // int16 entries: 0..255 soft, 0x100 start of packet, |0x200 last of a group
constexpr int B_SOFT_MARK = 0x100, B_SOFT_LAST = 0x200;
constexpr int CHUNK_RING = 256;  // message start samples (lastmse, burstoqpskdemodulator.cpp:264)
constexpr int RT_BLOCK = 6080;   // 64 x 95 R/T block
constexpr int RT_JOB_OUT = 400;  // int4 header + decoded bits, MSB first
constexpr int RT_TESTS_PER_PASS = 8;
constexpr int TRI_N = 16384;     // complex FFT inside FFTrWrapper<double>(32768)
// The front end (AGC, burst statistic, peak detector, trident buffer) runs
// ahead of the demodulator proper: d2's output, the demodulator's input
// val_to_demod, goes to a time-indexed ring (B_D2 - 1 samples of delay plus
// the run-ahead), and every completed trident buffer to one of TRI_SLOTS
// slots with the sample the reference checks it at.
constexpr int TRI_SLOTS = 4;     // trident checks a channel may have recorded and not yet applied
constexpr int BV_LEN = 16384;    // OQPSK val_to_demod ring (>= B_D2 - 1 + a pass of 12000 samples)
constexpr int MV_LEN = 32768;    // MSK (M_D2 - 1 = 7680)
constexpr int CHK_REC = 8;       // doubles per trident decision record
constexpr int TRI_GRID = 1024;   // trident workgroups (each loops over the pass's checks)

// Delay<T> instances (ring size, fractional delay): delays(1), delayt41/42(T/4),
// delayt8(T/8), a1(T/2), bt_d1(T, complex), bt_ma_diff(128 T)
enum BurstDelay { BDL_S = 0, BDL_41, BDL_42, BDL_8, BDL_A1, BDL_BT, BDL_MADIFF, BDL_COUNT };
// ring sizes ceil(delay) + 1 of the part-B delays the demodulator keeps in
// registers (delays 1, SPS/4, SPS/4, SPS/8, SPS/2 with SPS = 2 * 48000 /
// 10500; burst_engine.hip checks them against the host tables)
constexpr int BDL_N_S = 2, BDL_N_41 = 4, BDL_N_42 = 4, BDL_N_8 = 3, BDL_N_A1 = 6;
// the front end's bt_d1 (one symbol, complex) in registers too
constexpr int BDL_N_BT = 11;

// double state fields
enum BDS : int {
  BD_M2_PTR, BD_M2_STEP, BD_M2_FREQ,
  BD_SO_PTR, BD_SO_LAST, BD_SO_STEP, BD_SO_FREQ,
  BD_Q_PTR, BD_Q_STEP,
  BD_AGC_SUM, BD_AGC2_SUM, BD_MA1_RE, BD_MA1_IM, BD_MAV1_SUM,
  BD_PD_LASTDY, BD_VOL_GAIN,
  BD_SR_X1, BD_SR_X2, BD_SR_Y1, BD_SR_Y2,
  BD_AVE_RE, BD_AVE_IM, BD_ROT_RE, BD_ROT_IM, BD_STR_RE, BD_STR_IM,
  BD_PTD_RE, BD_PTD_IM, BD_S2L_RE, BD_S2L_IM, BD_ROTF,
  BD_MSE, BD_LASTMSE, BD_MSEMA_SUM,
  BD_COUNT
};

// int state fields
enum BIS : int {
  BI_AGC_P, BI_AGC2_P, BI_D1_P, BI_MA1_P, BI_MAV1_P,
  BI_DL_P0,  // .. BI_DL_P0 + BDL_COUNT - 1: Delay write pointers
  BI_PD1_P = BI_DL_P0 + BDL_COUNT, BI_PD2_P, BI_PD3_P, BI_PD_CNTDOWN, BI_PD_MAXPOSCD,
  BI_TRI_PTR, BI_MSEMA_P,
  BI_STARTSTOP, BI_CNTR, BI_INSERTPRE, BI_YUI,
  // AeroL burst framing
  BI_RI, BI_MUW, BI_FCNTR, BI_GSL, BI_UWI, BI_UWR, BI_UWI_INV, BI_UWR_INV, BI_DATACD, BI_BLOCKPTR, BI_BURST_ID,
  BI_SKIP_GROUP,
  BI_DCD_EDGES,  // DataCarrierDetect changes (SignalHunter::handleDcd, decode/hunter.cpp:14-19)
  BI_COUNT
};

// ---- burst MSK (burst_msk.hip)
constexpr int M_NT = 80;           // matched filter taps, 2 * SPS (:142-149)
constexpr int M_D1 = 11581;        // d1.setLength(289 * SPS + 20) + 1
constexpr int M_D2 = 7681;         // d2.setLength((72 + 120) * SPS) + 1
constexpr int M_TRI = 8000;        // tridentbuffer_sz = qRound(200 * SPS)
constexpr int M_TRI_BASE = 5040;   // qRound(126 * SPS): start tone window
constexpr int M_TRI_TOP = 2960;    // qRound(74 * SPS): 0-1 preamble window
constexpr int M_MA = 5040;         // bt_ma1 (complex) and mav1: 126 * SPS
constexpr int M_MADIFF = 5041;     // bt_ma_diff.setdelay(126 * SPS): ceil + 1 slots
constexpr int M_BTD = 41;          // bt_d1.setdelay(SPS) (complex)
constexpr int M_A1 = 21, M_D8 = 21;  // a1 / delayt8 .setdelay(SPS / 2)
constexpr int M_DSM = 41;          // delayedsmpl.setLength(SPS)
constexpr int M_PD1 = 5041, M_PD2 = 2521, M_PD3 = 5041;  // PeakDetector(2520, 0.1)
static_assert(M_PD1 == M_PD3 && M_PD2 <= M_PD3, "peak detector rings (read from d3's)");
constexpr int M_PD_MAXCD = 5040;
constexpr int M_AGC2 = 5120;       // AGC(SPS * 128 / Fs, Fs)
constexpr int M_MSEMA = 75;
constexpr int M_STARTSTOP = 20000; // SPS * 500
constexpr int M_SOFT_GROUP = 12;   // RxDataBits emitted at >= 12 entries (:689-692)

enum BMDS : int {
  BM_M2_PTR, BM_M2_STEP, BM_M2_FREQ,
  BM_SO_PTR, BM_SO_LAST, BM_SO_STEP, BM_SH_PTR, BM_SH_STEP,
  BM_AGC_SUM, BM_AGC2_SUM, BM_MA1_RE, BM_MA1_IM, BM_MAV1_SUM,
  BM_PD_LASTDY, BM_VOL_GAIN,
  BM_SR_X1, BM_SR_X2, BM_SR_Y1, BM_SR_Y2,
  BM_AVE_RE, BM_AVE_IM, BM_ROT_RE, BM_ROT_IM, BM_STR_RE, BM_STR_IM, BM_ROTF,
  BM_MSE, BM_MSEMA_SUM, BM_DIFF_LAST,
  BM_COUNT
};
enum BMIS : int {
  BMI_AGC_P, BMI_AGC2_P, BMI_D1_P, BMI_MA1_P, BMI_MAV1_P, BMI_MADIFF_P, BMI_BTD_P, BMI_A1_P, BMI_D8_P,
  BMI_DSM_P, BMI_PD1_P, BMI_PD2_P, BMI_PD3_P, BMI_PD_CNTDOWN, BMI_PD_MAXPOSCD,
  BMI_TRI_PTR, BMI_MSEMA_P, BMI_STARTSTOP, BMI_CNTR,
  // AeroL MSK burst framing
  BMI_MUW, BMI_FCNTR, BMI_UW, BMI_UW_INV, BMI_BLOCKPTR, BMI_BURST_ID, BMI_SKIP_GROUP, BMI_TOTAL,
  BMI_DATACD, BMI_DCD_EDGES,  // AeroL datacd (aerol.cpp:2010-2028) and its changes
  BMI_COUNT
};
constexpr int BURST_DS_COUNT = BD_COUNT > BM_COUNT ? BD_COUNT : BM_COUNT;
constexpr int BURST_IS_COUNT = BI_COUNT > BMI_COUNT ? BI_COUNT : BMI_COUNT;

// 64-bit counters
enum BLS : int {
  BL_NSAMP,    // samples demodulated
  BL_AVAIL,    // samples pushed
  BL_HB_DONE,  // Hilbert blocks processed
  BL_SP,       // soft entries written (uncommitted included)
  BL_SCOMMIT,  // soft entries committed (emitted groups)
  BL_SCONS,    // soft entries consumed by the framing
  BL_CHUNK_N,  // message starts recorded
  BL_CHUNK_H,  // message starts passed
  BL_NSAMP_A,  // samples through the front end
  BL_CHK_N,    // trident checks recorded by the front end
  BL_CHK_DONE, // trident decisions applied by the demodulator
  BL_COUNT
};

struct BurstState {
  int C;
  int *hop_n;       // [C] trident records written this pass
  double *ds;
  int *is;
  long long *ls;
  double *fir;      // [2 * 55][C] transposed RRC partial sums (MSK: [2 * 80][C] matched filter)
  double2 *ana;     // [ANA_LEN / 4][C][4] analytic signal (ana_idx)
  int16_t *pcm;     // [C][pcm_cap], channel-major (burst_engine.hip b_batch_scatter_kernel)
  long long pcm_cap;
  double2 *hb_rem;  // [C][HB_REM]
  double *agc, *agc2;           // [len][C]
  double *d1;                   // [B_D1][C] d1's real part (its only output read: val_to_demod, the trident buffer)
  double *vring;                // [BV_LEN or MV_LEN][C] val_to_demod of sample n at n & (len - 1)
  double2 *ma1;                 // [B_MA][C]
  double *mav1;                 // [B_MA][C]
  double *dl[BDL_COUNT];        // Delay rings [size][C] (BDL_BT holds double2); MSK: bt_d1 (double2),
                                // bt_ma_diff, a1, delayt8, delayedsmpl (double2) in slots 0-4
  double *pd3;                  // [len][C] PeakDetector d3 (d1 and d2 read from it)
  double *tri;                  // [C][TRI_SLOTS][B_TRI or M_TRI] completed trident buffers
  long long *chk_n;             // [C][TRI_SLOTS] sample of each recorded check
  double *chk;                  // [C][TRI_SLOTS][CHK_REC] its decision (trident kernels)
  int *tjobs;                   // [C * TRI_SLOTS] this pass's checks: channel | slot << 24
  int *ntjobs;
  double *msema;                // [C][B_MSEMA]
  long long *chunks;            // [C][CHUNK_RING]
  int16_t *soft;                // [C][B_SOFT_RING]
  double *hops;                 // [C][hop_cap][6]
  int hop_cap;
  uint8_t *rtblock;             // [C][RT_BLOCK]
  int *jobs;                    // [C * RT_TESTS_PER_PASS] int4 (c, blockptr, burst id, 0)
  int *njobs;
  uint8_t *jobout;              // [C * RT_TESTS_PER_PASS][RT_JOB_OUT]
  double *tri_abs;              // [TRI_GRID][TRI_N] |base| scratch of the trident check
};

struct BurstTables {
  const double2 *cis;     // [WTSIZE]
  const double2 *tw8, *twi8, *tw16;
  const double2 *hk;      // [HB_N] Hilbert kernel spectrum
  const double2 *hk_time; // [HB_N] Hilbert kernel, time domain
  const double2 *da, *db; // [TRI_N]
  const double *taps;     // RRC
  const double *dw[BDL_COUNT], *domw[BDL_COUNT];
  const int *dio[BDL_COUNT];
  int dsize[BDL_COUNT];
};

// The analytic-signal ring: a channel's samples in runs of 2^ANA_LB (the
// runs of all channels side by side, then the next run), so the Hilbert
// stage's stores of consecutive samples fill whole runs; the front ends'
// lanes (one channel each) read 16 B at a 2^ANA_LB x 16 B stride.  Runs of
// 1 / 2 / 4 / 8 measured hilbert 17.2 / 16.3 / 15.5 / 15.0 ms per C4 step,
// front_burst 26.1 / 26.2 / 26.3 / 26.9.
#ifndef AERO_ANA_LB
#define AERO_ANA_LB 2
#endif
constexpr int ANA_LB = AERO_ANA_LB;
__device__ __forceinline__ size_t ana_idx(long long s, int c, int C) {
  const size_t q = (size_t)(s & (ANA_LEN - 1));
  return ((((q >> ANA_LB) * (size_t)C) + (size_t)c) << ANA_LB) | (q & ((1u << ANA_LB) - 1));
}

// Workgroup -> channel map for kernels with one workgroup per channel that
// read or write time-major [sample][C] arrays (a 128-B line holds 64 int16
// or 8 complex samples of neighbouring channels).  Workgroups are dealt to
// the 8 XCDs round-robin (blockIdx % 8), each with its own L2, so the
// identity map has every line fetched (or partially written) by all 8 L2s;
// this bijection of [0, n) gives XCD x the contiguous channels
// [x q + min(x, r), ...) (q = n / 8, r = n % 8), so neighbouring channels
// share one L2.
__device__ __forceinline__ int xcd_channel(int b, int n) {
  const int x = b & 7, k = b >> 3, q = n >> 3, r = n & 7;
  return x * q + (x < r ? x : r) + k;
}

}  // namespace aero
