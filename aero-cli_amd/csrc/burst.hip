/*
 * burst.hip — burst-mode 10500-bps OQPSK on gfx950 (aero-decode --burst):
 * BurstOqpskDemodulator::writeDataSlot (decode/burstoqpskdemodulator.cpp:262-703)
 * and the burst branch of AeroL::Decode with RTChannelDeleaveFECScram
 * (decode/aerol.cpp:1060-1240, decode/aerol.h:755-836).
 *
 *  hilbert_kernel      QJHilbertFilter on JFastFir (decode/DSP.cpp:730-761,
 *                      decode/jfft.cpp:445-495): 8192-point overlap-add blocks of
 *                      6145 samples, one workgroup per channel, into a
 *                      time-major analytic-signal ring.
 *  front_burst_kernel  part A of the per-sample recurrence (AGC, d1/d2, burst
 *                      statistic, peak detector, trident buffer), one channel
 *                      per lane, ahead of the demodulator: it never reads the
 *                      demodulator's state.  It records each completed trident
 *                      buffer and the sample the reference checks it at
 *                      (burstoqpskdemodulator.cpp:343-440).
 *  trident_kernel      FFTrWrapper<double>(32768) of both trident halves (a
 *                      16384-point JFFT + split), |top| - |base|, the +-1792-bin
 *                      trident search and the strongest base bin; one
 *                      1024-thread workgroup per recorded check.
 *  demod_burst_kernel  part B, one channel per lane, from the front end's
 *                      val_to_demod ring, each trident decision applied at
 *                      its sample.
 *  frame_burst_kernel  AeroL burst framing (UW tolerance 4 within the muw window,
 *                      dummy header, R/T block fill, tests at blockptr 320+192k).
 *  rt_viterbi_kernel   one wave per R/T test: deinterleave 64 x blockptr/64 and
 *                      Decode_soft of the whole block (jconvolutionalcodec.cpp:88-119).
 * CRC checks and R/T packet handling run on the host (engine.hip).
 *
 * Bit-exactness rules as in demod_oqpsk.hip: -ffp-contract=off, reference
 * operation order, GCC complex products, aero_math.h for libm.
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>

#include "aero_math.h"
#include "burst_common.h"
#include "engine_common.h"
#include "fft_dit.h"
#include "viterbi_dev.h"
#include "burst_dev.h"

namespace aero {

namespace {

constexpr double SPS = 2.0 * 48000.0 / 10500.0;  // SamplesPerSymbol
constexpr uint32_t BUW = 0xE15AE893u;

__constant__ double c_bsr_b[3];  // st_iir_resonator (burstoqpskdemodulator.cpp:220-227)
__constant__ double c_bsr_a[3];
__constant__ double c_btaps[NTAPS];  // RRC (burstoqpskdemodulator.cpp:199-201)

}  // namespace

// ------------------------------------------------------------ Hilbert FIR
// Kernel spectrum: JFFT of the zero-padded 2048-tap kernel (JFastFir ctor).
__global__ __launch_bounds__(512) void hk_spectrum_kernel(BurstTables T, double2 *hk) {
  constexpr int L = 13, PADDED = HB_N + HB_N / 16;
  __shared__ double lds[PADDED];
  __shared__ double2 s_tw[TwLds<L>::LEN];
  const int t = threadIdx.x;
  load_tw_lds<L>(s_tw, T.tw8, t, 512);
  __syncthreads();
  double2 x[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = T.hk_time[bitrev<L>(epos<L, 0>(t, i))];
  fft_dit<L, false>(x, t, lds, T.tw8, s_tw);
#pragma unroll
  for (int i = 0; i < 16; ++i) hk[epos<L, 3>(t, i)] = x[i];
}

// JFastFir::update (decode/jfft.cpp:445-495): for every complete block j of
// 6145 inputs (pcm / 32768, 0): y = IFFT(FFT(block, zeros) * K) (JFFT scales
// the inverse by 1/N); y[0 .. 2047) += previous remainder; outputs y[0 .. 6145)
// are the analytic samples of inputs (j + 1) * 6145 + p; y[6145 ..) is the
// next remainder.  Inputs 0 .. 6144 come out as zeros (the initial buffer).
__global__ __launch_bounds__(512) void hilbert_kernel(BurstState S, BurstTables T, int nch) {
  constexpr int L = 13, PADDED = HB_N + HB_N / 16;
  __shared__ double lds[PADDED];
  __shared__ double2 s_tw[TwLds<L>::LEN];
  const int c = xcd_channel(blockIdx.x, gridDim.x), t = threadIdx.x;
  if (c >= nch) return;
  const int C = S.C;
  load_tw_lds<L>(s_tw, T.tw8, t, 512);
  __syncthreads();
  long long j = S.ls[BL_HB_DONE * C + c];
  const long long avail = S.ls[BL_AVAIL * C + c];
  const long long capm = S.pcm_cap - 1;
  double2 *rem = S.hb_rem + (size_t)c * HB_REM;
  const int16_t *pcm = S.pcm + (size_t)c * S.pcm_cap;  // this channel's run of the ring
  for (; (j + 1) * HB_SNZ <= avail; ++j) {
    double2 x[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int p = bitrev<L>(epos<L, 0>(t, i));
      x[i] = p < HB_SNZ ? make_double2(((double)pcm[(j * HB_SNZ + p) & capm]) / 32768.0, 0.0)
                        : make_double2(0.0, 0.0);
    }
    fft_dit<L, false>(x, t, lds, T.tw8, s_tw);
#pragma unroll
    for (int i = 0; i < 16; ++i) {  // sigspace[k] *= kernel[k]
      const double2 k = T.hk[epos<L, 3>(t, i)];
      x[i] = make_double2(x[i].x * k.x - x[i].y * k.y, x[i].x * k.y + x[i].y * k.x);
    }
    exchange<L, 3, 0, true>(x, t, lds);
    fft_dit<L, true>(x, t, lds, T.twi8, s_tw);
    double2 r[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      x[i].x *= (1.0 / ((double)HB_N));
      x[i].y *= (1.0 / ((double)HB_N));
      const int p = epos<L, 3>(t, i);
      r[i] = p < HB_REM ? rem[p] : make_double2(0.0, 0.0);
    }
    __syncthreads();  // every old remainder read before it is replaced
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int p = epos<L, 3>(t, i);
      if (p < HB_SNZ) {
        double2 y = x[i];
        if (p < HB_REM) y = make_double2(y.x + r[i].x, y.y + r[i].y);
        const long long s = (j + 1) * HB_SNZ + p;
        S.ana[ana_idx(s, c, C)] = y;
      } else {
        rem[p - HB_SNZ] = x[i];
      }
    }
    __syncthreads();
  }
  if (t == 0) S.ls[BL_HB_DONE * C + c] = j;
}

// ----------------------------------------------------------------- demod
// One wave per workgroup, at most 40 KB of LDS per wave, so four waves (one
// per SIMD) share a CU and 65536 channels run in one round instead of two.
//
// The RRC (FIR::FIRUpdateAndProcess, transposed form: the output is
// ((0 + h0 d[n-55]) + h1 d[n-54]) + ... + h54 d[n-1], oldest term first).
// The partial sum of the oldest BD_LDS_TAPS taps is formed directly, oldest
// first, from a per-lane LDS line of the last BD_LDS_TAPS mixer outputs d
// (one 16-B read per tap and one write per sample); the line slides back
// every BD_DBLK samples.  The same products are added in the same order as in
// the transposed form, so every partial sum is the same double.  The newest
// taps keep their transposed partial sums in registers.  The state between
// launches holds the line (oldest first) in place of those taps' partial
// sums: all zero at start in either form.
constexpr int BD_BLOCK = 64;
constexpr int BD_LDS_TAPS = 36, BD_REG_TAPS = NTAPS - BD_LDS_TAPS;
constexpr int BD_DBLK = 40 - BD_LDS_TAPS;  // samples per slide of the line
#ifndef AERO_X_BD_DCH
constexpr int BD_DCH = 8;                  // line entries read per chunk
#else
constexpr int BD_DCH = AERO_X_BD_DCH;      // timing builds: other chunk sizes
#endif

// AERO_X_BSTAMPS (diagnostic build only): s_memtime cycle totals per section
// of the demod loop, each wave's maximum over its lanes (the wave's time in
// the section while the lane was in the loop), summed over waves: [0] loop
// control, [1] message start + val_to_demod, [3] trident decision, [4] part
// B loads + RRC, [5] PLL, rotators, AGC2, clip, [2] symbol timing, [6]
// symbol step + NCOs, [7] entry + exit (state); counters summed over lanes: [8] samples
// advanced, [10] lanes that entered the loop, [11] waves, [12] loop
// iterations (max over the wave's lanes)
#ifdef AERO_X_BSTAMPS
__device__ unsigned long long g_bstamps[16];
#define BSTAMP(k)                                                  \
  do {                                                             \
    __builtin_amdgcn_sched_barrier(0);                             \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();    \
    bst_[k] += t_ - btime_;                                        \
    btime_ = t_;                                                   \
    __builtin_amdgcn_sched_barrier(0);                             \
  } while (0)
#define BCOUNT(k, v) (bcnt_[k] += (v))
#else
#define BSTAMP(k) \
  do {            \
  } while (0)
#define BCOUNT(k, v) \
  do {               \
  } while (0)
#endif

// ------------------------------------------------------------- front end
// Part A of BurstOqpskDemodulator::writeDataSlot (decode/burstoqpskdemodulator.cpp:
// 300-345): AGC, the delays d1 / d2, the burst-timing statistic, the peak
// detector and the trident buffer.  It reads the analytic signal only, never
// the demodulator's state, so it runs ahead of the demodulator proper over
// the pass's samples: d2's output (val_to_demod, the demodulator's input
// B_D2 - 1 samples later) goes to a ring indexed by sample, and each
// completed trident buffer stays in its own slot with the sample at which
// the reference checks it, for trident_kernel to decide before the
// demodulator reaches that sample.  One channel per lane, no LDS.
__global__ __launch_bounds__(64) void front_burst_kernel(BurstState S, BurstTables T, int nch) {
  const int c = blockIdx.x * 64 + threadIdx.x;
  if (c >= nch) return;
  const int C = S.C;
  double *ds = S.ds + c;
  int *is = S.is + c;
  long long *ls = S.ls + c;
  const long long n0 = ls[BL_NSAMP_A * C];
  long long end = ls[BL_AVAIL * C];
  // the ring keeps what the demodulator has not read yet
  const long long lim = ls[BL_NSAMP * C] + (BV_LEN - (B_D2 - 1));
  if (end > lim) end = lim;
  long long chk_n = ls[BL_CHK_N * C];
  const long long chk_done = ls[BL_CHK_DONE * C];
  if (n0 >= end) return;
  double agc_sum = ds[BD_AGC_SUM * C];
  double ma1r = ds[BD_MA1_RE * C], ma1i = ds[BD_MA1_IM * C], mav1_sum = ds[BD_MAV1_SUM * C];
  double pd_lastdy = ds[BD_PD_LASTDY * C];
  int agc_p = is[BI_AGC_P * C], d1_p = is[BI_D1_P * C];
  int ma1_p = is[BI_MA1_P * C], mav1_p = is[BI_MAV1_P * C];
  int dl_bt = is[(BI_DL_P0 + BDL_BT) * C], dl_md = is[(BI_DL_P0 + BDL_MADIFF) * C];
  int pd3_p = is[BI_PD3_P * C];
  int pd_cntdown = is[BI_PD_CNTDOWN * C], pd_maxposcd = is[BI_PD_MAXPOSCD * C];
  int tri_ptr = is[BI_TRI_PTR * C];
  double *tri = S.tri + ((size_t)c * TRI_SLOTS + (chk_n & (TRI_SLOTS - 1))) * B_TRI;
  const DlyRef dMD = dref(T, BDL_MADIFF);
  double *mdr = S.dl[BDL_MADIFF] + c;
  // bt_d1 (a complex delay of one symbol, 11 slots) in registers: its
  // weights do not depend on the write pointer (host-checked)
  double2 *btr = reinterpret_cast<double2 *>(S.dl[BDL_BT]) + c;
  double2 hBT[BDL_N_BT];
  dly_regs_load2(hBT, btr, C, dl_bt);
  const double wBT = T.dw[BDL_BT][0], oBT = T.domw[BDL_BT][0];
  long long n = n0;
  // the analytic sample and the AGC slot it replaces are loaded one sample
  // ahead: the sample's whole chain starts from them
  double2 a_n = S.ana[ana_idx(n, c, C)];
  double agc_n = S.agc[(size_t)agc_p * C + c];
  // so are the ring slots the sample reads (none is a slot the sample before
  // writes: every ring is longer than 3); bt_ma_diff's "newer" slot is the
  // next sample's "older"
  auto nxt = [](int p, int len) { return p + 1 == len ? 0 : p + 1; };
  auto pd2_slot = [](int p3) { return p3 >= B_PD2 - 1 ? p3 - (B_PD2 - 1) : p3 + B_PD3 - (B_PD2 - 1); };
  double cvd_n = S.d1[(size_t)nxt(d1_p, B_D1) * C + c];
  double2 ma_n = S.ma1[(size_t)ma1_p * C + c];
  double mv_n = S.mav1[(size_t)mav1_p * C + c];
  double md_older = mdr[(size_t)nxt(dl_md, dMD.size) * C];
  double md_newer = mdr[(size_t)nxt(nxt(dl_md, dMD.size), dMD.size) * C];
  double pd1_n = S.pd3[(size_t)nxt(pd3_p, B_PD3) * C + c], pd2_n = S.pd3[(size_t)pd2_slot(pd3_p) * C + c];
  while (n < end) {
    // every slot holds a check the demodulator has not applied: the buffer
    // this sample may start filling is one of them
    if (chk_n - chk_done >= TRI_SLOTS) break;
    // every ring slot (and Delay weight) this sample reads, loaded before any
    // of its stores so the round trips overlap; none is the slot written
    // this sample (burst_dev.h dly_pre)
    const int d1r = nxt(d1_p, B_D1);
    // the peak detector's d1 (same length as d3) and d2 (half) see the same
    // values as d3, so their outputs are d3's slots: the oldest one and the
    // one written B_PD2 - 1 updates ago
    const int p1r = nxt(pd3_p, B_PD3);
    const double2 a = a_n;
    const double agc_old = agc_n;
    const double cvd = cvd_n;  // real(d1.update_dont_touch(cval)): the only part read
    const double2 ma_old = ma_n;
    const double mv_old = mv_n;
    const double pd1_old = pd1_n, pd2_old = pd2_n;
    const DlyPre mdp = {dMD.w[dl_md], dMD.omw[dl_md], md_older, md_newer, nxt(dl_md, dMD.size), false};
    // the next sample's slots
    a_n = S.ana[ana_idx(n + 1, c, C)];  // past the Hilbert stage's output: unused
    cvd_n = S.d1[(size_t)nxt(d1r, B_D1) * C + c];
    ma_n = S.ma1[(size_t)nxt(ma1_p, B_MA) * C + c];
    mv_n = S.mav1[(size_t)nxt(mav1_p, B_MA) * C + c];
    const double md_next = mdr[(size_t)nxt(nxt(mdp.next, dMD.size), dMD.size) * C];
    pd1_n = S.pd3[(size_t)nxt(p1r, B_PD3) * C + c];
    pd2_n = S.pd3[(size_t)pd2_slot(p1r) * C + c];
    double cr = a.x, ci = a.y;
    {  // agc.Update(|cval|); cval *= AGCVal (:316-317)
      const double av = B_HYPOT(cr, ci);
      agc_sum = agc_sum - agc_old;
      agc_sum = agc_sum + fabs(av);
      S.agc[(size_t)agc_p * C + c] = fabs(av);
      agc_p = agc_p + 1 == B_AGC ? 0 : agc_p + 1;
      agc_n = S.agc[(size_t)agc_p * C + c];  // written B_AGC samples ago
      // short exact divisions (aero_math.h): a tiny agc_sum / B_AGC is floored at 1e-6
      double g = div_n(1.414213562, fmax(div_c(agc_sum, ((double)B_AGC)), 0.000001));
      g = fmax(g, 0.000001);
      cr *= g;
      ci *= g;
    }
    S.d1[(size_t)d1_p * C + c] = cr;
    d1_p = d1r;
    // d2.update_dont_touch(real(cval_d)): the demodulator reads it back B_D2 - 1 samples later
    S.vring[(size_t)(n & (BV_LEN - 1)) * C + c] = cvd;
    double fastarm;
    {  // burst-timing statistic (:326-339)
      const double2 bd = dly_reg2(hBT, wBT, oBT, make_double2(cr, ci));
      const double pr = cr * bd.x - ci * (-bd.y), pi = cr * (-bd.y) + ci * bd.x;  // cval * conj(bd)
      ma1r = ma1r - ma_old.x;
      ma1i = ma1i - ma_old.y;
      ma1r = ma1r + pr;
      ma1i = ma1i + pi;
      S.ma1[(size_t)ma1_p * C + c] = make_double2(pr, pi);
      ma1_p = ma1_p + 1 == B_MA ? 0 : ma1_p + 1;
      // div_c (aero_math.h): the running sums are zero or far above 2^-969
      // (int16 PCM through the Hilbert transform, the AGC gain and two
      // products stay on a grid of about 2^-400), so the contract holds
      fastarm = B_HYPOT(div_c(ma1r, (double)B_MA), div_c(ma1i, (double)B_MA));
      mav1_sum = mav1_sum - mv_old;
      mav1_sum = mav1_sum + (fastarm);
      S.mav1[(size_t)mav1_p * C + c] = fastarm;
      mav1_p = mav1_p + 1 == B_MA ? 0 : mav1_p + 1;
      fastarm = div_c(mav1_sum, (double)B_MA);
      fastarm -= dly_commit(mdr, C, dl_md, mdp, fastarm);
      md_older = md_newer;
      md_newer = md_next;
      if (fastarm < 0) fastarm = 0;
    }
    double bt = fastarm * fastarm;
    if (bt > 500) bt = 500;
    {  // PeakDetector::update (DSP.h:491-566)
      double val = bt;
      S.pd3[(size_t)pd3_p * C + c] = val;  // d3 (and so d1, d2)
      pd3_p = p1r;
      const double dy = val - pd1_old;     // d1.update_dont_touch(val)
      val = pd2_old;                       // d2.update(val)
      if ((!pd_cntdown) && (val > 0.2) && ((pd_lastdy >= 0 && dy < 0))) {
        pd_cntdown = B_PD_MAXCD;
        pd_maxposcd = pd3_findmaxpos(S.pd3 + c, C, pd3_p, B_PD3);
      }
      if (pd_cntdown > 0) pd_cntdown--;
      pd_lastdy = dy;
      bool hit = false;
      if (!pd_maxposcd) {
        pd_maxposcd--;
        hit = true;
      } else if (pd_maxposcd > 0) {
        pd_maxposcd--;
      }
      if (hit) tri_ptr = 0;
    }
    if (tri_ptr < B_TRI) {
      tri[tri_ptr] = cvd;
      tri_ptr++;
    } else if (tri_ptr == B_TRI) {
      // the reference checks the buffer at this sample (:343-440); the
      // demodulator applies trident_kernel's decision before its part B here
      tri_ptr++;
      const int slot = (int)(chk_n & (TRI_SLOTS - 1));
      S.chk_n[(size_t)c * TRI_SLOTS + slot] = n;
      S.tjobs[atomicAdd(S.ntjobs, 1)] = c | (slot << 24);
      chk_n++;
      tri = S.tri + ((size_t)c * TRI_SLOTS + (chk_n & (TRI_SLOTS - 1))) * B_TRI;
    }
    n++;
  }
  ds[BD_AGC_SUM * C] = agc_sum;
  ds[BD_MA1_RE * C] = ma1r;
  ds[BD_MA1_IM * C] = ma1i;
  ds[BD_MAV1_SUM * C] = mav1_sum;
  ds[BD_PD_LASTDY * C] = pd_lastdy;
  is[BI_AGC_P * C] = agc_p;
  is[BI_D1_P * C] = d1_p;
  is[BI_MA1_P * C] = ma1_p;
  is[BI_MAV1_P * C] = mav1_p;
  dly_regs_store2(hBT, btr, C);
  is[(BI_DL_P0 + BDL_BT) * C] = 0;
  is[(BI_DL_P0 + BDL_MADIFF) * C] = dl_md;
  is[BI_PD3_P * C] = pd3_p;
  is[BI_PD_CNTDOWN * C] = pd_cntdown;
  is[BI_PD_MAXPOSCD * C] = pd_maxposcd;
  is[BI_TRI_PTR * C] = tri_ptr;
  ls[BL_NSAMP_A * C] = n;
  ls[BL_CHK_N * C] = chk_n;
}

// ----------------------------------------------------------------- demod
// Part B of writeDataSlot (:450-702) from the front end's val_to_demod, the
// trident decisions applied at the samples the front end recorded.  One
// wave per workgroup.  The transposed RRC partial sums of taps
// [BD_LDS_TAPS, 55) live in registers, the rest (real and imaginary) in LDS.
__global__ __launch_bounds__(BD_BLOCK) void demod_burst_kernel(BurstState S, BurstTables T, int nch, int trace) {
  __shared__ double2 s_d[BD_LDS_TAPS + BD_DBLK][BD_BLOCK];  // [slot][lane]: d of past samples
  const int c = blockIdx.x * BD_BLOCK + threadIdx.x, col = threadIdx.x;
  if (c >= nch) return;
#ifdef AERO_X_BSTAMPS
  unsigned long long bst_[8] = {0, 0, 0, 0, 0, 0, 0, 0}, bcnt_[5] = {0, 0, 0, 0, 0};
  unsigned long long btime_ = __builtin_amdgcn_s_memtime();
  bool bactive_ = false;
#endif
  const int C = S.C;
  double *ds = S.ds + c;
  int *is = S.is + c;
  long long *ls = S.ls + c;
  const long long n0 = ls[BL_NSAMP * C];
  const long long end = ls[BL_NSAMP_A * C];  // the front end's progress
#ifdef AERO_X_BSTAMPS
  // every lane reaches the wave reduction at the end
  if (n0 < end) {
    bactive_ = true;
#else
  if (n0 >= end) return;
  {
#endif
  double m2_ptr = ds[BD_M2_PTR * C], m2_step = ds[BD_M2_STEP * C], m2_freq = ds[BD_M2_FREQ * C];
  double so_ptr = ds[BD_SO_PTR * C], so_last = ds[BD_SO_LAST * C], so_step = ds[BD_SO_STEP * C];
  double so_freq = ds[BD_SO_FREQ * C];
  double q_ptr = ds[BD_Q_PTR * C], q_step = ds[BD_Q_STEP * C];
  double agc2_sum = ds[BD_AGC2_SUM * C], vol_gain = ds[BD_VOL_GAIN * C];
  double srx1 = ds[BD_SR_X1 * C], srx2 = ds[BD_SR_X2 * C], sry1 = ds[BD_SR_Y1 * C], sry2 = ds[BD_SR_Y2 * C];
  double ave_r = ds[BD_AVE_RE * C], ave_i = ds[BD_AVE_IM * C], rot_r = ds[BD_ROT_RE * C], rot_i = ds[BD_ROT_IM * C];
  double str_r = ds[BD_STR_RE * C], str_i = ds[BD_STR_IM * C];
  double ptd_r = ds[BD_PTD_RE * C], ptd_i = ds[BD_PTD_IM * C], s2l_r = ds[BD_S2L_RE * C], s2l_i = ds[BD_S2L_IM * C];
  double rotf = ds[BD_ROTF * C], mse = ds[BD_MSE * C], lastmse = ds[BD_LASTMSE * C];
  // exp(i rotator_freq) changes only with rotator_freq (a symbol step or a
  // trident decision), so it is kept rather than evaluated every sample
  double rf_c, rf_s;
  b_cexp_i(rotf, rf_c, rf_s);
  double msema_sum = ds[BD_MSEMA_SUM * C];
  int agc2_p = is[BI_AGC2_P * C];
  int dl_s = is[(BI_DL_P0 + BDL_S) * C], dl_41 = is[(BI_DL_P0 + BDL_41) * C], dl_42 = is[(BI_DL_P0 + BDL_42) * C];
  int dl_8 = is[(BI_DL_P0 + BDL_8) * C], dl_a1 = is[(BI_DL_P0 + BDL_A1) * C];
  int msema_p = is[BI_MSEMA_P * C];
  int startstop = is[BI_STARTSTOP * C], cntr = is[BI_CNTR * C], insertpre = is[BI_INSERTPRE * C];
  int yui = is[BI_YUI * C];
  int hop_n = S.hop_n[c];
  long long sp = ls[BL_SP * C], scommit = ls[BL_SCOMMIT * C];
  const long long scons = ls[BL_SCONS * C];
  long long chunk_h = ls[BL_CHUNK_H * C];
  const long long chunk_n = ls[BL_CHUNK_N * C];
  long long chk_done = ls[BL_CHK_DONE * C];
  const long long chk_n = ls[BL_CHK_N * C];
  long long next_chk = chk_done < chk_n ? S.chk_n[(size_t)c * TRI_SLOTS + (chk_done & (TRI_SLOTS - 1))] : LLONG_MAX;
#pragma unroll 1
  for (int j = 0; j < BD_LDS_TAPS; ++j)
    s_d[j][col] = make_double2(S.fir[(size_t)j * C + c], S.fir[(size_t)(NTAPS + j) * C + c]);
  int dt = 0;  // the line's oldest entry is slot dt
  double hre[BD_REG_TAPS], him[BD_REG_TAPS];  // partial sums of taps BD_LDS_TAPS..54
#pragma unroll
  for (int j = 0; j < BD_REG_TAPS; ++j) {
    hre[j] = S.fir[(size_t)(BD_LDS_TAPS + j) * C + c];
    him[j] = S.fir[(size_t)(NTAPS + BD_LDS_TAPS + j) * C + c];
  }
  int16_t *soft = S.soft + (size_t)c * B_SOFT_RING;
  const long long *chunks = S.chunks + (size_t)c * CHUNK_RING;
  const double PT = 0.4 * WTSIZE;  // IfHavePassedPoint(ee), ee = 0.4
  // the short delays in registers (burst_dev.h dly_reg); their weights are
  // the same for every write pointer
  double hS[BDL_N_S], h41[BDL_N_41], h42[BDL_N_42], h8[BDL_N_8], hA1[BDL_N_A1];
  dly_regs_load(hS, S.dl[BDL_S] + c, C, dl_s);
  dly_regs_load(h41, S.dl[BDL_41] + c, C, dl_41);
  dly_regs_load(h42, S.dl[BDL_42] + c, C, dl_42);
  dly_regs_load(h8, S.dl[BDL_8] + c, C, dl_8);
  dly_regs_load(hA1, S.dl[BDL_A1] + c, C, dl_a1);
  const double wS = T.dw[BDL_S][0], oS = T.domw[BDL_S][0], w41 = T.dw[BDL_41][0], o41 = T.domw[BDL_41][0];
  const double w42 = T.dw[BDL_42][0], o42 = T.domw[BDL_42][0], w8 = T.dw[BDL_8][0], o8 = T.domw[BDL_8][0];
  const double wA1 = T.dw[BDL_A1][0], oA1 = T.domw[BDL_A1][0];

  long long n = n0;
  // the loads a sample's FIR and AGC2 need are issued one sample ahead (their
  // indices advance by one per sample; a trident decision that moves mixer2
  // reloads its table entry): val_to_demod (front end's ring), mixer2's cis
  // entry, the agc2 slot about to be replaced
  auto vtd_at = [&](long long k) {
    return k >= B_D2 - 1 ? S.vring[(size_t)((k - (B_D2 - 1)) & (BV_LEN - 1)) * C + c] : 0.0;
  };
  double vtd_n = vtd_at(n);
  double2 m2_n = T.cis[b_cis_index(m2_ptr)];
  double2 so_n = T.cis[b_cis_index(so_ptr)];  // st_osc's entry (reloaded where the phase is set)
  double agc2_n = S.agc2[(size_t)agc2_p * C + c];
  // the symbol-tone PLL's table entry and the msema slot an update replaces
  // are loaded ahead too (q_ptr's entry after each NCO step, the slot after
  // each update): with 64 channels a wave, some lane is in the PLL window or
  // at a symbol step nearly every sample, so a load waited for there is
  // waited for every sample
  double2 q_n = T.cis[b_cis_index(q_ptr)];
  double *const mm = S.msema + (size_t)c * B_MSEMA;
  double mm_n = mm[msema_p];
  BSTAMP(7);
  while (n < end) {
    BSTAMP(0);
    BCOUNT(4, 1);
    if (sp - scons > B_SOFT_RING - 64) break;  // soft ring full: framing frees it next
    // lastmse is captured at the start of every message (burstoqpskdemodulator.cpp:264)
    while (chunk_h < chunk_n && chunks[chunk_h & (CHUNK_RING - 1)] == n) {
      lastmse = mse;
      chunk_h++;
    }
    // val_to_demod = d2.update_dont_touch(...): the front end's value of B_D2 - 1 samples ago (zeros before)
    const double vtd = vtd_n;
    vtd_n = vtd_at(n + 1);  // past the front end's progress: unused
    BSTAMP(1);
    if (n == next_chk) {
      // trident decision (burstoqpskdemodulator.cpp:393-411), computed by trident_kernel
      const double *r = S.chk + ((size_t)c * TRI_SLOTS + (chk_done & (TRI_SLOTS - 1))) * CHK_REC;
      if (r[0] != 0.0) {
        const double carrierphase = aero_atan2(r[6], r[5]) - (M_PI / 4.0);
        b_set_freq(m2_freq, m2_step, (48000.0 / 32768.0) * r[1]);
        b_set_phase_deg(m2_ptr, (180.0 / M_PI) * carrierphase);
        m2_n = T.cis[b_cis_index(m2_ptr)];
        vol_gain = 1.4142 * 500.0 / r[3];
        b_set_freq(so_freq, so_step, 10500.0);
        b_set_phase_deg(so_ptr, 0);
        so_n = T.cis[b_cis_index(so_ptr)];
        srx1 = srx2 = sry1 = sry2 = 0;
        startstop = B_STARTSTOP;
        cntr = 0;
        rot_r = 1;
        rot_i = 0;
        insertpre = 1;
        rotf = 0;
        b_cexp_i(rotf, rf_c, rf_s);
        ave_r = 1;
        ave_i = 0;
        mse = 0;
        for (int k = 0; k < B_MSEMA; k++) mm[k] = 0;
        msema_sum = 0;
        msema_p = 0;
        mm_n = 0;
      }
      if (trace && hop_n < S.hop_cap) {
        double *h = S.hops + ((size_t)c * S.hop_cap + hop_n) * 6;
        h[0] = (double)n;
        h[1] = r[0] != 0.0 ? 1.0 : 0.0;
        h[2] = m2_freq;
        h[3] = vol_gain;
        h[4] = r[4];
        h[5] = r[1];
      }
      hop_n++;
      chk_done++;
      next_chk = chk_done < chk_n ? S.chk_n[(size_t)c * TRI_SLOTS + (chk_done & (TRI_SLOTS - 1))] : LLONG_MAX;
    }
    BSTAMP(3);
    // ---- part B (:450-702); its ring and weight reads first (a1's whatever
    // the symbol-tone window says: a read changes nothing)
    const double agc2_old = agc2_n;
    double s2r, s2i;
    {
      // the taps are reloaded (scalar loads) every sample rather than held
      // in 110 SGPRs across the loop, which spilled: the laundered value is
      // a zero offset, not the pointer, so the loads stay scalar loads from
      // constant memory (a laundered pointer loses its address space and
      // turns them into flat vector loads, each waited for in turn)
      // (the offset is laundered again after each chunk of taps, so a chunk's
      // scalar loads are issued when it is due and 16 SGPRs hold its taps)
      int tz = 0;
      asm volatile("" : "+s"(tz));
      const double2 m2 = m2_n;
      const double sc = vol_gain * vtd;
      const double ddr = m2.x * sc, ddi = m2.y * sc;
      // RRC (FIR::FIRUpdateAndProcess reads the 55 samples before the newest)
      // partial sum of taps 0..BD_LDS_TAPS-1 at sample n-1, oldest term first
      const int lbase = dt * BD_BLOCK + col;  // element index of the oldest entry in s_d
      double ar = 0.0, ai = 0.0;
      {
        // in chunks of BD_DCH entries, each chunk's reads issued after the
        // previous chunk's sums (the scheduler would otherwise issue all
        // reads at once and hold 4 registers per tap); the laundered value is
        // an index, so the reads stay LDS reads
        const double2 *sd = &s_d[0][0];
        int lp = lbase;
#pragma unroll
        for (int i0 = 0; i0 < BD_LDS_TAPS; i0 += BD_DCH) {
          double2 v[BD_DCH];
#pragma unroll
          for (int u = 0; u < BD_DCH; ++u)
            if (i0 + u < BD_LDS_TAPS) v[u] = sd[lp + (i0 + u) * BD_BLOCK];
#pragma unroll
          for (int u = 0; u < BD_DCH; ++u) {
            if (i0 + u >= BD_LDS_TAPS) break;
            const double tap = c_btaps[tz + i0 + u];
            if (i0 + u == 0) {
              ar = 0.0 + tap * v[0].x;
              ai = 0.0 + tap * v[0].y;
            } else {
              ar = ar + tap * v[u].x;
              ai = ai + tap * v[u].y;
            }
          }
          asm volatile("" : "+v"(lp), "+s"(tz) : "v"(ar), "v"(ai));
        }
      }
      const double *tp = c_btaps + tz;
      s2r = hre[BD_REG_TAPS - 1];
      s2i = him[BD_REG_TAPS - 1];
#pragma unroll
      for (int j = NTAPS - 1; j > BD_LDS_TAPS; --j) {  // register part, descending: q[j - 1] read before rewritten
        hre[j - BD_LDS_TAPS] = hre[j - 1 - BD_LDS_TAPS] + tp[j] * ddr;
        him[j - BD_LDS_TAPS] = him[j - 1 - BD_LDS_TAPS] + tp[j] * ddi;
        if ((NTAPS - 1 - j) % 8 == 7) {
          asm volatile("" : "+s"(tz) : "v"(hre[j - BD_LDS_TAPS]));
          tp = c_btaps + tz;
        }
      }
      hre[0] = ar + tp[BD_LDS_TAPS] * ddr;
      him[0] = ai + tp[BD_LDS_TAPS] * ddi;
      (&s_d[0][0])[lbase + BD_LDS_TAPS * BD_BLOCK] = make_double2(ddr, ddi);
      if (++dt == BD_DBLK) {  // slide the line back to slot 0 (ascending: no entry overwritten before it is moved)
        dt = 0;
#pragma unroll 8
        for (int i = 0; i < BD_LDS_TAPS; ++i) s_d[i][col] = s_d[BD_DBLK + i][col];
      }
    }
    BSTAMP(4);
    if (startstop > 0) {
      startstop--;
      if (cntr < 1000000) cntr++;
      if (mse < 0.75) startstop = B_STARTSTOP;
    }
    if (startstop == 0) startstop--;
    if ((cntr > ((256 - 10) * SPS)) && insertpre) {
      soft[sp & (B_SOFT_RING - 1)] = B_SOFT_MARK;
      sp++;
      insertpre = 0;
    }
    if ((cntr > SPS * (128 + 10)) && (cntr < ((256 - 10) * SPS))) {  // symbol-tone PLL (:462-474)
      const double progress =
          div_c(((double)cntr) - (SPS * (128 + 10)), (double)(((256 - 10) * SPS) - (SPS * (128 + 10))));  // integer numerator
      const double t1r = s2r * str_r - s2i * str_i, t1i = s2r * str_i + s2i * str_r;
      const double spr = t1r * 0.0 - t1i * 1.0, spi = t1r * 1.0 + t1i * 0.0;  // * imag
      const double er = aero_tanh_bf(spi) * (spr);
      double ec, es;
      b_cexp_i(er * 0.01, ec, es);
      const double nr = str_r * ec - str_i * es, ni = str_r * es + str_i * ec;
      str_r = nr;
      str_i = ni;
      ave_r = ave_r * 0.95 + 0.05 * str_r;
      ave_i = ave_i * 0.95 + 0.05 * str_i;
      const double spi2 = dly_reg(hA1, wA1, oA1, spr);
      const double2 qv = q_n;
      const double er_r = qv.x * spr - qv.y * (-spi2), er_i = qv.x * (-spi2) + qv.y * spr;
      double st_err = B_ATAN2(er_i, er_r);
      st_err *= 1.5 * (1.0 - progress * progress);
      b_advance(q_ptr, -(1.0 / (2.0 * M_PI)) * st_err * 0.1);
      b_set_phase_deg_pos(so_ptr, div_cw(360.0 * q_ptr, (double)WTSIZE) * 4.0 + (360.0 * 0.4));
      so_n = T.cis[b_cis_index(so_ptr)];
    }
    {  // sig2 *= symboltone_averotator; rotator *= exp(i rotator_freq); sig2 *= rotator
      const double ar = s2r * ave_r - s2i * ave_i, ai = s2r * ave_i + s2i * ave_r;
      double ec, es;
      ec = rf_c;
      es = rf_s;
      const double rr = rot_r * ec - rot_i * es, ri = rot_r * es + rot_i * ec;
      rot_r = rr;
      rot_i = ri;
      s2r = ar * rot_r - ai * rot_i;
      s2i = ar * rot_i + ai * rot_r;
    }
    {  // agc2 (AGC(SPS*64/Fs)) and clip (:478-481)
      const double sa = B_HYPOT(s2r, s2i);
      agc2_sum = agc2_sum - agc2_old;
      agc2_sum = agc2_sum + fabs(sa);
      S.agc2[(size_t)agc2_p * C + c] = fabs(sa);
      agc2_p = agc2_p + 1 == B_AGC2 ? 0 : agc2_p + 1;
      agc2_n = S.agc2[(size_t)agc2_p * C + c];  // written B_AGC2 samples ago
      double g = div_n(1.414213562, fmax(div_c(agc2_sum, ((double)B_AGC2)), 0.000001));  // as the AGC above
      g = fmax(g, 0.000001);
      s2r *= g;
      s2i *= g;
    }
    const double abval = B_HYPOT(s2r, s2i);
    if (abval > 2.84) {
      const double k = div_n(2.84, abval);  // abval > 2.84
      s2r = k * s2r;
      s2i = k * s2i;
    }
    BSTAMP(5);
    {  // symbol timing (:482-496)
      const double st_diff = dly_reg(hS, wS, oS, abval * abval) - (abval * abval);
      const double st_d1out = dly_reg(h41, w41, o41, st_diff);
      const double st_d2out = dly_reg(h42, w42, o42, st_d1out);
      double st_eta = (st_d2out - st_diff) * st_d1out;
      {  // st_iir_resonator.update(st_eta)
        double y = 0;
        y += srx2 * c_bsr_b[2];
        y += srx1 * c_bsr_b[1];
        y += st_eta * c_bsr_b[0];
        y -= sry2 * c_bsr_a[2];
        y -= sry1 * c_bsr_a[1];
        srx2 = srx1;
        srx1 = st_eta;
        sry2 = sry1;
        sry1 = y;
        if (cntr > SPS * (128 + 128)) st_eta = y;
      }
      const double m1r = st_eta, m1i = -dly_reg(h8, w8, o8, st_eta);
      const double2 so = so_n;
      const double ore = so.x * m1r - so.y * m1i, oim = so.x * m1i + so.y * m1r;
      const double st_angle_error = B_ATAN2(oim, ore);
      if (cntr > SPS * (128 + 64)) {
        b_set_freq(so_freq, so_step, -st_angle_error * 0.00000001 + so_freq);
        b_advance(so_ptr, div_c(-st_angle_error * 0.01, 360.0));  // a tiny quotient vanishes in so_ptr + x W
      }
      if (so_freq < (10500.0 - 0.1)) b_set_freq(so_freq, so_step, (10500.0 - 0.1));
      if (so_freq > (10500.0 + 0.1)) b_set_freq(so_freq, so_step, (10500.0 + 0.1));
    }
    BSTAMP(2);
    {  // IfHavePassedPoint(ee) (DSP.cpp:222-238) and the symbol step (:497-554)
      double tl = so_last - PT, tw = so_ptr - PT;
      if (tl < 0.0) tl += WTSIZE;
      if (tw < 0.0) tw += WTSIZE;
      if ((tl > 3.0 * WTSIZE / 4.0) && (tw < 1.0 * WTSIZE / 4.0)) {
        const double pt_last = div_n(tw, so_step);  // tw: 0 or >= 2^-40, so_step ~4375
        const double pt_this = 1.0 - pt_last;
        const double ptr_ = pt_this * s2r + pt_last * s2l_r, pti = pt_this * s2i + pt_last * s2l_i;
        // the remainder of a value in [72, 792): 0 or a multiple of ulp(72), in div_c's contract
        const double twospeed =
            -4.0 * (div_c(b_fmod360(div_cw(360.0 * q_ptr, (double)WTSIZE) * 2.0 + (360.0 * 0.4 * 0.5)), 360.0) -
                    (0.34046 + 0.4111 * 0.4));
        const bool even = !(twospeed < 0);
        yui++;
        yui %= 2;
        if (cntr < ((128 + 128) * SPS)) {
          if ((even && yui == 1) || (!even && yui == 0)) {
            yui++;
            yui %= 2;
          }
        }
        if (!yui) {
          ptd_r = ptr_;
          ptd_i = pti;
        } else {
          const double qr = ptr_, qi = ptd_i;  // pt_qpsk
          const double ct_xt = aero_tanh_bf(pti) * ptr_;
          const double ct_xt_d = aero_tanh_bf(ptd_r) * ptd_i;
          double ct_ec = ct_xt_d - ct_xt;
          if (ct_ec > M_PI) ct_ec = M_PI;
          if (ct_ec < -M_PI) ct_ec = -M_PI;
          if (ct_ec > M_PI_2) ct_ec = M_PI_2;
          if (ct_ec < -M_PI_2) ct_ec = -M_PI_2;
          if (cntr > ((128 + 10) * SPS)) {
            double ec, es;
            b_cexp_i(ct_ec * 0.1, ec, es);
            const double rr = rot_r * ec - rot_i * es, ri = rot_r * es + rot_i * ec;
            rot_r = rr;
            rot_i = ri;
            rotf = rotf + ct_ec * 0.0001;
            b_cexp_i(rotf, rf_c, rf_s);
          }
          if (cntr > ((128 + 10) * SPS)) {  // msema.Update (DSP.cpp:405-416)
            const double tda = (fabs(qr) - 1.0), tdb = (fabs(qi) - 1.0);
            const double v = (tda * tda) + (tdb * tdb);
            msema_sum = msema_sum - mm_n;
            msema_sum = msema_sum + fabs(v);
            mm[msema_p] = fabs(v);
            msema_p = msema_p + 1 == B_MSEMA ? 0 : msema_p + 1;
            mm_n = mm[msema_p];  // written B_MSEMA updates ago
            mse = div_c(msema_sum, ((double)B_MSEMA));
          }
          if (startstop > 0) {
            int ibit = b_qround(0.75 * qi * 127.0 + 128.0);
            if (ibit > 255) ibit = 255;
            if (ibit < 0) ibit = 0;
            soft[sp & (B_SOFT_RING - 1)] = (int16_t)ibit;
            sp++;
            ibit = b_qround(0.75 * qr * 127.0 + 128.0);
            if (ibit > 255) ibit = 255;
            if (ibit < 0) ibit = 0;
            // RxDataBits emitted or dropped as a group (:548-551): the group's
            // last entry carries the mark in the same store
            const long long sp1 = sp;
            sp++;
            if (sp - scommit >= 32) {
              if (mse < 0.6 || lastmse < 0.6) {
                ibit |= B_SOFT_LAST;
                scommit = sp;
              } else {
                sp = scommit;
              }
            }
            soft[sp1 & (B_SOFT_RING - 1)] = (int16_t)ibit;
          }
        }
      }
    }
    s2l_r = s2r;
    s2l_i = s2i;
    b_nco_next(m2_ptr, m2_step);
    m2_n = T.cis[b_cis_index(m2_ptr)];
    so_last = so_ptr;
    b_nco_next(so_ptr, so_step);
    so_n = T.cis[b_cis_index(so_ptr)];
    b_nco_next(q_ptr, q_step);
    q_n = T.cis[b_cis_index(q_ptr)];
    n++;
    BSTAMP(6);
  }
  BCOUNT(0, (unsigned long long)(n - n0));
  // state back
#pragma unroll 1
  for (int j = 0; j < BD_LDS_TAPS; ++j) {
    const double2 v = s_d[dt + j][col];
    S.fir[(size_t)j * C + c] = v.x;
    S.fir[(size_t)(NTAPS + j) * C + c] = v.y;
  }
#pragma unroll
  for (int j = 0; j < BD_REG_TAPS; ++j) {
    S.fir[(size_t)(BD_LDS_TAPS + j) * C + c] = hre[j];
    S.fir[(size_t)(NTAPS + BD_LDS_TAPS + j) * C + c] = him[j];
  }
  ds[BD_M2_PTR * C] = m2_ptr;
  ds[BD_M2_STEP * C] = m2_step;
  ds[BD_M2_FREQ * C] = m2_freq;
  ds[BD_SO_PTR * C] = so_ptr;
  ds[BD_SO_LAST * C] = so_last;
  ds[BD_SO_STEP * C] = so_step;
  ds[BD_SO_FREQ * C] = so_freq;
  ds[BD_Q_PTR * C] = q_ptr;
  ds[BD_Q_STEP * C] = q_step;
  ds[BD_AGC2_SUM * C] = agc2_sum;
  ds[BD_VOL_GAIN * C] = vol_gain;
  ds[BD_SR_X1 * C] = srx1;
  ds[BD_SR_X2 * C] = srx2;
  ds[BD_SR_Y1 * C] = sry1;
  ds[BD_SR_Y2 * C] = sry2;
  ds[BD_AVE_RE * C] = ave_r;
  ds[BD_AVE_IM * C] = ave_i;
  ds[BD_ROT_RE * C] = rot_r;
  ds[BD_ROT_IM * C] = rot_i;
  ds[BD_STR_RE * C] = str_r;
  ds[BD_STR_IM * C] = str_i;
  ds[BD_PTD_RE * C] = ptd_r;
  ds[BD_PTD_IM * C] = ptd_i;
  ds[BD_S2L_RE * C] = s2l_r;
  ds[BD_S2L_IM * C] = s2l_i;
  ds[BD_ROTF * C] = rotf;
  ds[BD_MSE * C] = mse;
  ds[BD_LASTMSE * C] = lastmse;
  ds[BD_MSEMA_SUM * C] = msema_sum;
  is[BI_AGC2_P * C] = agc2_p;
  dly_regs_store(hS, S.dl[BDL_S] + c, C);
  dly_regs_store(h41, S.dl[BDL_41] + c, C);
  dly_regs_store(h42, S.dl[BDL_42] + c, C);
  dly_regs_store(h8, S.dl[BDL_8] + c, C);
  dly_regs_store(hA1, S.dl[BDL_A1] + c, C);
  is[(BI_DL_P0 + BDL_S) * C] = 0;
  is[(BI_DL_P0 + BDL_41) * C] = 0;
  is[(BI_DL_P0 + BDL_42) * C] = 0;
  is[(BI_DL_P0 + BDL_8) * C] = 0;
  is[(BI_DL_P0 + BDL_A1) * C] = 0;
  is[BI_MSEMA_P * C] = msema_p;
  is[BI_STARTSTOP * C] = startstop;
  is[BI_CNTR * C] = cntr;
  is[BI_INSERTPRE * C] = insertpre;
  is[BI_YUI * C] = yui;
  S.hop_n[c] = hop_n;
  ls[BL_NSAMP * C] = n;
  ls[BL_SP * C] = sp;
  ls[BL_SCOMMIT * C] = scommit;
  ls[BL_CHUNK_H * C] = chunk_h;
  ls[BL_CHK_DONE * C] = chk_done;
  BSTAMP(7);
  }
#ifdef AERO_X_BSTAMPS
  {  // per wave: section maxima over lanes, counters summed
    unsigned long long v[13];
    for (int k = 0; k < 8; k++) v[k] = bst_[k];
    v[8] = bcnt_[0];
    v[9] = 0;
    v[10] = bactive_ ? 1 : 0;
    v[11] = 0;
    v[12] = bcnt_[4];
    for (int off = 32; off > 0; off >>= 1) {
      for (int k = 0; k < 13; k++) {
        const unsigned long long o = __shfl_xor(v[k], off, 64);
        v[k] = (k < 8 || k == 12) ? (o > v[k] ? o : v[k]) : v[k] + o;
      }
    }
    if (threadIdx.x == 0 && v[10]) {
      for (int k = 0; k < 8; k++) atomicAdd(&g_bstamps[k], v[k]);
      atomicAdd(&g_bstamps[8], v[8]);
      atomicAdd(&g_bstamps[9], v[9]);
      atomicAdd(&g_bstamps[10], v[10]);
      atomicAdd(&g_bstamps[11], 1ull);
      atomicAdd(&g_bstamps[12], v[12]);
    }
  }
#endif
}

void burst_read_stamps(unsigned long long *out) {
#ifdef AERO_X_BSTAMPS
  hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bstamps), sizeof(unsigned long long) * 16);
  unsigned long long z[16] = {0};
  hipMemcpyToSymbol(HIP_SYMBOL(g_bstamps), z, sizeof z);
#else
  for (int k = 0; k < 16; ++k) out[k] = 0;
#endif
}

// --------------------------------------------------------- trident check
// burstoqpskdemodulator.cpp:343-392 for every check the front end recorded
// this pass (S.tjobs); each workgroup takes checks blockIdx.x, + gridDim.x, ...
__global__ __launch_bounds__(1024) void trident_kernel(BurstState S, BurstTables T) {
  constexpr int L = 14, N = TRI_N, FT = N / 16, PADDED = N + N / 16;
  __shared__ double lds[PADDED];
  __shared__ double2 s_tw[TwLds<L>::LEN];
  __shared__ double red_v[FT / 64];
  __shared__ int red_i[FT / 64];
  __shared__ double2 s_best;
  const int t = threadIdx.x;
  const int njobs = *S.ntjobs;  // uniform
  if ((int)blockIdx.x >= njobs) return;
  load_tw_lds<L>(s_tw, T.tw16, t, FT);
  double *absb = S.tri_abs + (size_t)blockIdx.x * N;
  for (int job = blockIdx.x; job < njobs; job += gridDim.x) {
  const int c = S.tjobs[job] & 0xFFFFFF, slot = S.tjobs[job] >> 24;
  const double *tb = S.tri + ((size_t)c * TRI_SLOTS + slot) * B_TRI;
  // block reduction: larger value, then smaller index
  auto reduce = [&](double v, int idx, double &bv, int &bi) {
    for (int off = 32; off > 0; off >>= 1) {
      const double ov = __shfl_down(v, off, 64);
      const int oi = __shfl_down(idx, off, 64);
      if (ov > v || (ov == v && oi < idx)) {
        v = ov;
        idx = oi;
      }
    }
    __syncthreads();
    if ((t & 63) == 0) {
      red_v[t >> 6] = v;
      red_i[t >> 6] = idx;
    }
    __syncthreads();
    bv = red_v[0];
    bi = red_i[0];
    for (int w = 1; w < FT / 64; ++w)
      if (red_v[w] > bv || (red_v[w] == bv && red_i[w] < bi)) {
        bv = red_v[w];
        bi = red_i[w];
      }
  };
  double minval = 0;
  int minbin = 0;
  for (int pass = 0; pass < 2; ++pass) {
    // FFTrWrapper: F[i] = (real[2i], real[2i+1]) of the 32768 reals (1170 trident samples, zeros)
    const int off = pass ? B_TRI_HALF : 0;
    double2 x[16];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int j = bitrev<L>(epos<L, 0>(t, i));
      const double a = 2 * j < B_TRI_HALF ? tb[off + 2 * j] : 0.0;
      const double b = 2 * j + 1 < B_TRI_HALF ? tb[off + 2 * j + 1] : 0.0;
      x[i] = make_double2(a, b);
    }
    fft_dit<L, false>(x, t, lds, T.tw16, s_tw);
    // out[i] = F[i] * DA[i] + DB[i] * conj(F[(N - i) % N])
    double2 g[16];
#pragma unroll
    for (int part = 0; part < 2; ++part) {
      __syncthreads();
#pragma unroll
      for (int i = 0; i < 16; ++i) lds[pad(epos<L, 3>(t, i))] = part ? x[i].y : x[i].x;
      __syncthreads();
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const double v = lds[pad((N - epos<L, 3>(t, i)) & (N - 1))];
        if (part)
          g[i].y = v;
        else
          g[i].x = v;
      }
    }
    __syncthreads();
    double lv = -1.0;
    int li = 0x7fffffff;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int p = epos<L, 3>(t, i);
      const double2 da = T.da[p], db = T.db[p];
      const double ar = x[i].x * da.x - x[i].y * da.y, ai = x[i].x * da.y + x[i].y * da.x;
      const double br = db.x * g[i].x - db.y * (-g[i].y), bi = db.x * (-g[i].y) + db.y * g[i].x;
      const double orr = ar + br, oi = ai + bi;
      const double ab = B_HYPOT(orr, oi);
      x[i] = make_double2(orr, oi);
      if (pass == 0) {
        absb[p] = ab;
        if (ab > lv || (ab == lv && p < li)) {
          lv = ab;
          li = p;
        }
      } else {
        lds[pad(p)] = ab - absb[p];  // out_abs_diff
      }
    }
    if (pass == 0) {
      // strongest base bin, first on ties (:377-383)
      double bv;
      int bi;
      reduce(lv, li, bv, bi);
      minval = bv;
      minbin = bi;
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if (epos<L, 3>(t, i) == minbin) s_best = x[i];
      __syncthreads();
    }
  }
  __syncthreads();
  // trident search: testval(i) = d[i-b] + d[i+b] - d[i], i in [b, N - b), b = 1792 (:369-376)
  constexpr int B = 1792;
  double lv = -1e308;
  int li = 0x7fffffff;
  for (int i = B + t; i < N - B; i += FT) {
    const double tv = lds[pad(i - B)] + lds[pad(i + B)] - lds[pad(i)];
    if (tv > lv) {
      lv = tv;
      li = i;
    }
  }
  double maxval;
  int maxbin;
  reduce(lv, li, maxval, maxbin);
  if (t == 0) {  // the decision record demod_burst_kernel applies at the check's sample
    const double hzperbin = 48000.0 / 32768.0;
    const int det = (maxval > 500.0) && (fabs((((double)maxbin - (double)minbin)) * hzperbin) < 20.0);
    double *r = S.chk + ((size_t)c * TRI_SLOTS + slot) * CHK_REC;
    r[0] = det;
    r[1] = minbin;
    r[2] = maxbin;
    r[3] = minval;
    r[4] = maxval;
    r[5] = s_best.x;
    r[6] = s_best.y;
  }
  __syncthreads();  // the LDS and s_best are the next check's
  }
}

// -------------------------------------------------------- AeroL framing
// AeroL::Decode, burst branch (decode/aerol.cpp:1060-1240, 2014-2030): the
// start-of-packet marker resets muw; the phase-invariant UW detectors take 4
// bit errors and must fire within |muw - 80| <= 150; a sync starts a packet
// with a dummy header (cntr jumps to 16) and every soft bit then fills the
// R/T block, tested at blockptr = 320 + 192 k (C remainder: also at 128); a
// burst window ends after 10500 bits, dropping the rest of that group.
// A lane stops before a new packet would overwrite the block of tests it
// queued this pass, and after RT_TESTS_PER_PASS tests.
__global__ __launch_bounds__(256) void frame_burst_kernel(BurstState S, int nch) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nch) return;
  const int C = S.C;
  int *is = S.is + c;
  long long *ls = S.ls + c;
  const long long E = ls[BL_SCOMMIT * C];
  long long q = ls[BL_SCONS * C];
  if (q >= E) return;
  int realimag = is[BI_RI * C], muw = is[BI_MUW * C], cntr = is[BI_FCNTR * C], gsl = is[BI_GSL * C];
  uint32_t uwi = (uint32_t)is[BI_UWI * C], uwr = (uint32_t)is[BI_UWR * C];
  int inv_i = is[BI_UWI_INV * C], inv_r = is[BI_UWR_INV * C];
  int datacd = is[BI_DATACD * C], blockptr = is[BI_BLOCKPTR * C], burst = is[BI_BURST_ID * C];
  int skip = is[BI_SKIP_GROUP * C];
  const int16_t *soft = S.soft + (size_t)c * B_SOFT_RING;
  uint8_t *blk = S.rtblock + (size_t)c * RT_BLOCK;
  int emitted = 0;
  for (; q < E; ++q) {
    const int e = soft[q & (B_SOFT_RING - 1)];
    const bool last = (e & B_SOFT_LAST) != 0;
    const int v = e & 0x1FF;
    if (skip) {
      if (last) skip = 0;
      continue;
    }
    if (v == B_SOFT_MARK) {
      muw = 0;
      continue;
    }
    if ((cntr == -1 && emitted) || emitted >= RT_TESTS_PER_PASS) break;
    int bit = v >= 128 ? 1 : 0, soft_bit = v;
    if (muw < 100000) muw++;
    realimag++;
    realimag %= 2;
    int gotsync;
    if (cntr > 4992 - 68 || cntr <= 0 || !datacd) {
      uint32_t &reg = realimag ? uwi : uwr;
      int &inv = realimag ? inv_i : inv_r;
      reg = (reg << 1) | (uint32_t)bit;
      const int xs = __builtin_popcount(reg ^ BUW);
      int g = 0;
      if (xs >= 32 - 4) {
        inv = 1;
        g = 1;
      } else if (xs <= 4) {
        inv = 0;
        g = 1;
      }
      gotsync = g;
      if (!gsl) {
        gsl = gotsync;
        gotsync = 0;
      } else
        gsl = 0;
    } else {
      gotsync = 0;
      gsl = 0;
    }
    if (gotsync && abs(muw - 80) > 150) gotsync = 0;
    if (realimag ? inv_i : inv_r) {
      bit = 1 - bit;
      if (soft_bit != 128) soft_bit = 255 - soft_bit;
    }
    if (cntr < 1000000000) cntr++;
    if (cntr == 0) {  // dummy header, rtchanneldeleavefecscram.resetblockptr()
      cntr = 16;
      blockptr = 0;
      burst++;
    }
    if (cntr >= 16 && blockptr < RT_BLOCK) {  // RTChannelDeleaveFECScram::update
      blk[blockptr] = (uint8_t)soft_bit;
      blockptr++;
      if (((blockptr - (64 * 5)) % (64 * 3)) == 0) {
        const int j = atomicAdd(S.njobs, 1);
        reinterpret_cast<int4 *>(S.jobs)[j] = make_int4(c, blockptr, burst, 0);
        emitted++;
      }
    }
    if (gotsync) {
      cntr = -1;
      if (!datacd) is[BI_DCD_EDGES * C]++;
      datacd = 1;
    }
    if (cntr + 1 == 10500) {  // end of the burst window: Decode returns
      cntr = 1000000000;
      if (datacd) is[BI_DCD_EDGES * C]++;
      datacd = 0;
      if (!last) skip = 1;
    }
  }
  ls[BL_SCONS * C] = q;
  is[BI_RI * C] = realimag;
  is[BI_MUW * C] = muw;
  is[BI_FCNTR * C] = cntr;
  is[BI_GSL * C] = gsl;
  is[BI_UWI * C] = (int)uwi;
  is[BI_UWR * C] = (int)uwr;
  is[BI_UWI_INV * C] = inv_i;
  is[BI_UWR_INV * C] = inv_r;
  is[BI_DATACD * C] = datacd;
  is[BI_BLOCKPTR * C] = blockptr;
  is[BI_BURST_ID * C] = burst;
  is[BI_SKIP_GROUP * C] = skip;
}

// one wave per R/T test: del[j*64 + i] = block[((i*27) % 64) * cols + j]
// (OQPSK, AeroLInterleaver::deinterleave_ba, decode/aerol.cpp:594-613), or
// for MSK jobs (w = 1) a 64 x 5 section then 64 x 3 sections
// (deinterleaveMSK_ba, decode/aerol.cpp:651-686); Decode_soft over blockptr
// soft values, decoded bits MSB-first
__global__ __launch_bounds__(64) void rt_viterbi_kernel(BurstState S) {
  __shared__ uint8_t sbuf[RT_BLOCK];
  __shared__ unsigned long long ow[64];  // decoded bit b: bit b & 63 of ow[b >> 6]
  static_assert(RT_BLOCK / 2 <= 64 * 64, "decoded bits fit one 64-bit word per lane");
  const int njobs = *S.njobs;
  const int lane = threadIdx.x;
  for (int job = blockIdx.x; job < njobs; job += gridDim.x) {
    __syncthreads();
    const int4 jd = reinterpret_cast<const int4 *>(S.jobs)[job];
    const int c = jd.x, bp = jd.y, cols = bp / 64;
    const uint8_t *blk = S.rtblock + (size_t)c * RT_BLOCK;
    if (!jd.w) {
      for (int k = lane; k < bp; k += 64) {
        const int j = k / 64, i = k % 64;
        sbuf[k] = blk[((i * 27) % 64) * cols + j];
      }
    } else {
      for (int k = lane; k < bp; k += 64) {
        const int j = k / 64, i = k % 64;
        if (k < 320) {
          sbuf[k] = blk[((i * 27) % 64) * 5 + j];
        } else {
          const int sec = (k - 320) / 192, jj = ((k - 320) % 192) / 64;
          sbuf[k] = blk[64 * (5 + 3 * sec) + ((i * 27) % 64) * 3 + jj];
        }
      }
    }
    __syncthreads();
    // the register-history decoder (viterbi_dev.h), the same decoder as
    // viterbi_decode_wave: the trellis steps need no LDS store or barrier
    uint64_t obw;
    viterbi_decode_regs(sbuf, bp, obw, lane);
    ow[lane] = obw;
    __syncthreads();
    uint8_t *out = S.jobout + (size_t)job * RT_JOB_OUT;
    const int nbits = bp / 2;
    if (lane == 0) *reinterpret_cast<int4 *>(out) = make_int4(c, bp, jd.z, nbits);
    for (int b = lane; b < (nbits + 7) / 8; b += 64) {
      // bits 8b .. 8b+7 (one byte of one word), first bit as the MSB
      const int byte = (int)((ow[b >> 3] >> (8 * (b & 7))) & 0xFFULL);
      int v = 0;
      for (int m = 0; m < 8; ++m)
        if (8 * b + m < nbits) v |= ((byte >> m) & 1) << (7 - m);
      out[16 + b] = (uint8_t)v;
    }
  }
}

// ------------------------------------------------------------ launchers
void burst_upload_constants(const double *sr_b, const double *sr_a, const double *taps) {
  hipMemcpyToSymbol(HIP_SYMBOL(c_btaps), taps, sizeof(double) * NTAPS);
  hipMemcpyToSymbol(HIP_SYMBOL(c_bsr_b), sr_b, sizeof(double) * 3);
  hipMemcpyToSymbol(HIP_SYMBOL(c_bsr_a), sr_a, sizeof(double) * 3);
}

void launch_hk_spectrum(hipStream_t st, const BurstTables &T, double2 *hk) {
  hipLaunchKernelGGL(hk_spectrum_kernel, dim3(1), dim3(512), 0, st, T, hk);
}

void launch_hilbert(hipStream_t st, const BurstState &S, const BurstTables &T, int nch) {
  hipLaunchKernelGGL(hilbert_kernel, dim3(nch), dim3(512), 0, st, S, T, nch);
}

void launch_front_burst(hipStream_t st, const BurstState &S, const BurstTables &T, int nch) {
  hipLaunchKernelGGL(front_burst_kernel, dim3((nch + 63) / 64), dim3(64), 0, st, S, T, nch);
}

void launch_demod_burst(hipStream_t st, const BurstState &S, const BurstTables &T, int nch, int trace) {
  hipLaunchKernelGGL(demod_burst_kernel, dim3((nch + BD_BLOCK - 1) / BD_BLOCK), dim3(BD_BLOCK), 0, st, S, T, nch,
                     trace);
}

void launch_trident(hipStream_t st, const BurstState &S, const BurstTables &T, int nch) {
  hipLaunchKernelGGL(trident_kernel, dim3(std::min(nch * TRI_SLOTS, TRI_GRID)), dim3(1024), 0, st, S, T);
}

void launch_frame_burst(hipStream_t st, const BurstState &S, int nch) {
  hipLaunchKernelGGL(frame_burst_kernel, dim3((nch + 255) / 256), dim3(256), 0, st, S, nch);
}

void launch_rt_viterbi(hipStream_t st, const BurstState &S, int max_jobs) {
  const int g = max_jobs < 16384 ? (max_jobs > 0 ? max_jobs : 1) : 16384;
  hipLaunchKernelGGL(rt_viterbi_kernel, dim3(g), dim3(64), 0, st, S);
}

}  // namespace aero
