/*
 * burst_common.h — layout shared by the burst-mode 10500-bps OQPSK kernels
 * (burst.hip) and the engine host (engine.hip).  Geometry from
 * BurstOqpskDemodulator's constructor and setSettings
 * (decode/burstoqpskdemodulator.cpp:5-232) at Fs 48000, fb 10500
 * (SamplesPerSymbol = 9.142857), and AeroL's burst R/T block
 * (decode/aerol.h:755-836).
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

// Delay<T> instances (ring size, fractional delay): delays(1), delayt41/42(T/4),
// delayt8(T/8), a1(T/2), bt_d1(T, complex), bt_ma_diff(128 T)
enum BurstDelay { BDL_S = 0, BDL_41, BDL_42, BDL_8, BDL_A1, BDL_BT, BDL_MADIFF, BDL_COUNT };

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
  BD_RESUME_VAL,
  BD_TRI_MINVAL, BD_TRI_MAXVAL, BD_TRI_BRE, BD_TRI_BIM,
  BD_COUNT
};

// int state fields
enum BIS : int {
  BI_AGC_P, BI_AGC2_P, BI_D1_P, BI_D2_P, BI_MA1_P, BI_MAV1_P,
  BI_DL_P0,  // .. BI_DL_P0 + BDL_COUNT - 1: Delay write pointers
  BI_PD1_P = BI_DL_P0 + BDL_COUNT, BI_PD2_P, BI_PD3_P, BI_PD_CNTDOWN, BI_PD_MAXPOSCD,
  BI_TRI_PTR, BI_MSEMA_P,
  BI_STARTSTOP, BI_CNTR, BI_INSERTPRE, BI_YUI,
  BI_PEND,  // 0 running, 1 trident check requested, 2 trident decision ready
  BI_TRI_DET, BI_TRI_MINBIN, BI_TRI_MAXBIN,
  // AeroL burst framing
  BI_RI, BI_MUW, BI_FCNTR, BI_GSL, BI_UWI, BI_UWR, BI_UWI_INV, BI_UWR_INV, BI_DATACD, BI_BLOCKPTR, BI_BURST_ID,
  BI_SKIP_GROUP,
  BI_HOP_N,
  BI_COUNT
};

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
  BL_COUNT
};

struct BurstState {
  int C;
  double *ds;
  int *is;
  long long *ls;
  double *fir;      // [2 * 55][C] transposed RRC partial sums
  double2 *ana;     // [ANA_LEN][C] analytic signal
  int16_t *pcm;     // [pcm_cap][C]
  long long pcm_cap;
  double2 *hb_rem;  // [C][HB_REM]
  double *agc, *agc2;           // [len][C]
  double2 *d1;                  // [B_D1][C]
  double *d2;                   // [B_D2][C]
  double2 *ma1;                 // [B_MA][C]
  double *mav1;                 // [B_MA][C]
  double *dl[BDL_COUNT];        // Delay rings [size][C] (BDL_BT holds double2)
  double *pd1, *pd2, *pd3;      // [len][C]
  double *tri;                  // [C][B_TRI]
  double *msema;                // [C][B_MSEMA]
  long long *chunks;            // [C][CHUNK_RING]
  int16_t *soft;                // [C][B_SOFT_RING]
  double *hops;                 // [C][hop_cap][6]
  int hop_cap;
  uint8_t *rtblock;             // [C][RT_BLOCK]
  int *jobs;                    // [C * RT_TESTS_PER_PASS] int4 (c, blockptr, burst id, 0)
  int *njobs;
  uint8_t *jobout;              // [C * RT_TESTS_PER_PASS][RT_JOB_OUT]
  double *tri_abs;              // [C][TRI_N] |base| scratch of the trident check
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

}  // namespace aero
