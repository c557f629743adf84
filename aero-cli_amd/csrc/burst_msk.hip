/*
 * burst_msk.hip — burst-mode 600/1200-bps MSK on gfx950 (aero-decode -b 600|1200
 * --burst): BurstMskDemodulator::writeData (decode/burstmskdemodulator.cpp:328-704)
 * as Decoder configures it (decode/decode.cpp:123-132: Fs 48000, fb 1200 for
 * both bit rates, freq_center 1000, AFC on, dcd never set) and the MSK burst
 * branch of AeroL::Decode (decode/aerol.cpp:1155-1178, 1234-1252, 2014-2030)
 * with RTChannelDeleaveFECScram::updateMSK (decode/aerol.h:614-753).
 *
 *  hilbert_kernel         shared with burst OQPSK (burst.hip): the same
 *                         2048-tap QJHilbertFilter.
 *  front_bmsk_kernel      the front end, one channel per lane, ahead of the
 *                         demodulator (it never reads its state): AGC, the d1 /
 *                         d2 alignment delays (d2's output to a ring indexed by
 *                         sample), the burst-timing statistic and peak detector,
 *                         trident-buffer fill; each completed buffer is kept
 *                         with the sample the reference checks it at.
 *  trident_bmsk_kernel    FFTrWrapper<double>(32768) of the start-tone window
 *                         (5040 samples) and the 0-1 preamble window (2960): the
 *                         strongest base bin and the strongest top bins either
 *                         side of it (:414-473); one 1024-thread workgroup per
 *                         recorded check.  The detection decision needs cntr
 *                         and runs in the demodulator.
 *  demod_bmsk_kernel      the demodulator, one channel per lane: at each
 *                         check's sample the trident decision, and while a
 *                         burst is on (startstop > 0 || mse < 0.6) the 80-tap
 *                         matched filter (transposed form, partial sums of taps
 *                         0-39 in LDS [tap][lane], 40-79 in registers),
 *                         symbol-tone PLL, carrier rotation, AGC2, symbol timing
 *                         and the differential soft bits, grouped 12 at a time.
 *  frame_bmsk_kernel      AeroL MSK burst framing: phase-invariant UW (4 bit
 *                         errors) accepted within 250 bits of the start-of-burst
 *                         marker, dummy header, R/T block fill, Viterbi jobs at
 *                         blockptr 320 + 192 k (the host keeps those updateMSK
 *                         tests: blocks 5, 11, 50 and the T packet's target).
 * The R/T Viterbi is burst.hip's rt_viterbi_kernel with the MSK deinterleave.
 *
 * Bit-exactness rules as demod_oqpsk.hip: -ffp-contract=off, reference
 * operation order, GCC complex products, aero_math.h for libm.
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>

#include "aero_math.h"
#include "burst_common.h"
#include "burst_dev.h"
#include "engine_common.h"
#include "fft_dit.h"

namespace aero {

namespace {

constexpr double MSPS = 40.0;  // SamplesPerSymbol = int(Fs / fb)
constexpr uint32_t MUW = 0xE15AE893u;
constexpr double M_EE = 0.025;
constexpr int M_START = 120, M_ENDROT = (120 + 37) * 40;

__constant__ double c_msr_b[3];  // st_iir_resonator, 600 Hz at 48 kHz (burstmskdemodulator.cpp:214-227)
__constant__ double c_msr_a[3];
__constant__ double c_mtaps[M_NT];  // matched filter (:142-149); LDS and registers hold only the partial sums

__device__ __forceinline__ double m_diff_soft(double &last, double soft) {  // DiffDecode::UpdateSoft (DSP.cpp:523-548)
  double retval;
  if (soft < 0 && last < 0) {
    retval = last;
  } else if (soft > 0 && last > 0) {
    retval = -last;
  } else {
    retval = fabs(last);
  }
  last = soft;
  return retval;
}

}  // namespace

// ----------------------------------------------------------------- demod
// channels per workgroup (one wave).  The matched filter's transposed partial
// sums of taps [BM_LDS_TAPS, 80) live in registers, the rest (real and
// imaginary) in LDS: 40 KB per wave, four waves per CU.
constexpr int BM_BLOCK = 64;
constexpr int BM_LDS_TAPS = 40, BM_REG_TAPS = M_NT - BM_LDS_TAPS;

// ------------------------------------------------------------- front end
// The part of BurstMskDemodulator::writeData before the demodulator proper
// (decode/burstmskdemodulator.cpp:356-413): AGC, d1 / d2, the burst-timing
// statistic, the peak detector and the trident buffer.  It never reads the
// demodulator's state and runs ahead of it (as burst.hip's
// front_burst_kernel): val_to_demod to a ring indexed by sample, completed
// trident buffers to slots with the sample the reference checks them at.
__global__ __launch_bounds__(64) void front_bmsk_kernel(BurstState S, BurstTables T, int nch) {
  const int c = blockIdx.x * 64 + threadIdx.x;
  if (c >= nch) return;
  const int C = S.C;
  double *ds = S.ds + c;
  int *is = S.is + c;
  long long *ls = S.ls + c;
  const long long n0 = ls[BL_NSAMP_A * C];
  long long end = ls[BL_AVAIL * C];
  const long long lim = ls[BL_NSAMP * C] + (MV_LEN - (M_D2 - 1));  // what the demodulator has not read
  if (end > lim) end = lim;
  long long chk_n = ls[BL_CHK_N * C];
  const long long chk_done = ls[BL_CHK_DONE * C];
  if (n0 >= end) return;
  double agc_sum = ds[BM_AGC_SUM * C];
  double ma1r = ds[BM_MA1_RE * C], ma1i = ds[BM_MA1_IM * C], mav1_sum = ds[BM_MAV1_SUM * C];
  double pd_lastdy = ds[BM_PD_LASTDY * C];
  int agc_p = is[BMI_AGC_P * C], d1_p = is[BMI_D1_P * C];
  int ma1_p = is[BMI_MA1_P * C], mav1_p = is[BMI_MAV1_P * C], madiff_p = is[BMI_MADIFF_P * C];
  int btd_p = is[BMI_BTD_P * C];
  int pd3_p = is[BMI_PD3_P * C];
  int pd_cntdown = is[BMI_PD_CNTDOWN * C], pd_maxposcd = is[BMI_PD_MAXPOSCD * C];
  int tri_ptr = is[BMI_TRI_PTR * C];
  double *tri = S.tri + ((size_t)c * TRI_SLOTS + (chk_n & (TRI_SLOTS - 1))) * M_TRI;
  double2 *btd = reinterpret_cast<double2 *>(S.dl[0]) + c;
  double *madiff = S.dl[1] + c;
  // both whole-sample delays read two slots per sample; the one read as
  // "newer" is the next sample's "older" (nothing writes it in between), so
  // it is carried in a register and each sample loads one slot per ring
  double2 bt_older = btd[(size_t)(btd_p + 1 == M_BTD ? 0 : btd_p + 1) * C];
  double md_older = madiff[(size_t)(madiff_p + 1 == M_MADIFF ? 0 : madiff_p + 1) * C];
  long long n = n0;
  // the analytic sample and the AGC slot it replaces are loaded one sample
  // ahead: the sample's whole chain starts from them
  double2 a_n = S.ana[ana_idx(n, c, C)];
  double agc_n = S.agc[(size_t)agc_p * C + c];
  while (n < end) {
    if (chk_n - chk_done >= TRI_SLOTS) break;  // every slot holds a check not yet applied
    // every ring slot this sample reads, loaded before any of its stores so
    // the round trips overlap; no slot read here is the one written this
    // sample (rings hold > 2 slots)
    const int d1r = d1_p + 1 == M_D1 ? 0 : d1_p + 1;
    const int bto = btd_p + 1 == M_BTD ? 0 : btd_p + 1, btn = bto + 1 == M_BTD ? 0 : bto + 1;
    const int mdo = madiff_p + 1 == M_MADIFF ? 0 : madiff_p + 1, mdn = mdo + 1 == M_MADIFF ? 0 : mdo + 1;
    // the peak detector's d1 (same length as d3) and d2 (half) see the same
    // values as d3, so their outputs are d3's slots: the oldest one and the
    // one written M_PD2 - 1 updates ago
    const int p1r = pd3_p + 1 == M_PD3 ? 0 : pd3_p + 1;
    const int p2r = pd3_p >= M_PD2 - 1 ? pd3_p - (M_PD2 - 1) : pd3_p + M_PD3 - (M_PD2 - 1);
    const double2 a = a_n;
    const double agc_old = agc_n;
    a_n = S.ana[ana_idx(n + 1, c, C)];  // past the Hilbert stage's output: unused
    const double cvd = S.d1[(size_t)d1r * C + c];  // real(d1.update_dont_touch(cval)): the only part read
    const double2 bt_old = bt_older, bt_new = btd[(size_t)btn * C];
    const double2 ma_old = S.ma1[(size_t)ma1_p * C + c];
    const double mv_old = S.mav1[(size_t)mav1_p * C + c];
    const double md_old = md_older, md_new = madiff[(size_t)mdn * C];
    const double pd1_old = S.pd3[(size_t)p1r * C + c], pd2_old = S.pd3[(size_t)p2r * C + c];
    double cr = a.x, ci = a.y;
    {  // agc->Update(abs(cval)); cval *= agc->AGCVal (:366-368)
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
    // d2.update_dont_touch(real(cval_d)): the demodulator reads it back M_D2 - 1 samples later
    S.vring[(size_t)(n & (MV_LEN - 1)) * C + c] = cvd;
    double fastarm;
    {  // burst-timing statistic (:376-385); bt_d1 = Delay(SPS): weights 0 / 1 (dly_int2)
      btd[(size_t)btd_p * C] = make_double2(cr, ci);
      btd_p = bto;
      bt_older = bt_new;
      const double2 bd = make_double2(0.0 * bt_new.x + (1.0 - 0.0) * bt_old.x,
                                      0.0 * bt_new.y + (1.0 - 0.0) * bt_old.y);
      const double pr = cr * bd.x - ci * (-bd.y), pi = cr * (-bd.y) + ci * bd.x;  // cval * conj(bd)
      ma1r = ma1r - ma_old.x;
      ma1i = ma1i - ma_old.y;
      ma1r = ma1r + pr;
      ma1i = ma1i + pi;
      S.ma1[(size_t)ma1_p * C + c] = make_double2(pr, pi);
      ma1_p = ma1_p + 1 == M_MA ? 0 : ma1_p + 1;
      // div_c (aero_math.h): the running sums are zero or far above 2^-969
      // (int16 PCM through the Hilbert transform, the AGC gain and two
      // products stay on a grid of about 2^-400), so the contract holds
      fastarm = B_HYPOT(div_c(ma1r, (double)M_MA), div_c(ma1i, (double)M_MA));
      mav1_sum = mav1_sum - mv_old;
      mav1_sum = mav1_sum + (fastarm);
      S.mav1[(size_t)mav1_p * C + c] = fastarm;
      mav1_p = mav1_p + 1 == M_MA ? 0 : mav1_p + 1;
      fastarm = div_c(mav1_sum, (double)M_MA);
      madiff[(size_t)madiff_p * C] = fastarm;  // bt_ma_diff.update(fastarm), whole-sample delay
      madiff_p = mdo;
      md_older = md_new;
      fastarm -= (0.0 * md_new + (1.0 - 0.0) * md_old);
      if (fastarm < 0) fastarm = 0;
    }
    double bt = fastarm * fastarm;
    if (bt > 500) bt = 500;
    {  // PeakDetector::update (DSP.h:491-566), setSettings(2520, 0.1)
      double val = bt;
      S.pd3[(size_t)pd3_p * C + c] = val;  // d3 (and so d1, d2)
      pd3_p = p1r;
      const double dy = val - pd1_old;     // d1.update_dont_touch(val)
      val = pd2_old;                       // d2.update(val)
      if ((!pd_cntdown) && (val > 0.1) && ((pd_lastdy >= 0 && dy < 0))) {
        pd_cntdown = M_PD_MAXCD;
        pd_maxposcd = pd3_findmaxpos(S.pd3 + c, C, pd3_p, M_PD3);
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
    if (tri_ptr < M_TRI) {
      tri[tri_ptr] = cvd;
      tri_ptr++;
    } else if (tri_ptr == M_TRI) {
      // the reference computes the trident spectra at this sample
      // (:414-473); the demodulator takes the decision before the rest of it
      tri_ptr++;
      const int slot = (int)(chk_n & (TRI_SLOTS - 1));
      S.chk_n[(size_t)c * TRI_SLOTS + slot] = n;
      S.tjobs[atomicAdd(S.ntjobs, 1)] = c | (slot << 24);
      chk_n++;
      tri = S.tri + ((size_t)c * TRI_SLOTS + (chk_n & (TRI_SLOTS - 1))) * M_TRI;
    }
    n++;
  }
  ds[BM_AGC_SUM * C] = agc_sum;
  ds[BM_MA1_RE * C] = ma1r;
  ds[BM_MA1_IM * C] = ma1i;
  ds[BM_MAV1_SUM * C] = mav1_sum;
  ds[BM_PD_LASTDY * C] = pd_lastdy;
  is[BMI_AGC_P * C] = agc_p;
  is[BMI_D1_P * C] = d1_p;
  is[BMI_MA1_P * C] = ma1_p;
  is[BMI_MAV1_P * C] = mav1_p;
  is[BMI_MADIFF_P * C] = madiff_p;
  is[BMI_BTD_P * C] = btd_p;
  is[BMI_PD3_P * C] = pd3_p;
  is[BMI_PD_CNTDOWN * C] = pd_cntdown;
  is[BMI_PD_MAXPOSCD * C] = pd_maxposcd;
  is[BMI_TRI_PTR * C] = tri_ptr;
  ls[BL_NSAMP_A * C] = n;
  ls[BL_CHK_N * C] = chk_n;
}

__global__ __launch_bounds__(BM_BLOCK) void demod_bmsk_kernel(BurstState S, BurstTables T, int nch, int trace) {
  __shared__ double s_qre[BM_LDS_TAPS][BM_BLOCK];
  __shared__ double s_qim[BM_LDS_TAPS][BM_BLOCK];
  const int c = blockIdx.x * BM_BLOCK + threadIdx.x, col = threadIdx.x;
  if (c >= nch) return;
  const int C = S.C;
  double *ds = S.ds + c;
  int *is = S.is + c;
  long long *ls = S.ls + c;
  const long long n0 = ls[BL_NSAMP * C];
  const long long end = ls[BL_NSAMP_A * C];  // the front end's progress
  if (n0 >= end) return;

  double m2_ptr = ds[BM_M2_PTR * C], m2_step = ds[BM_M2_STEP * C], m2_freq = ds[BM_M2_FREQ * C];
  double so_ptr = ds[BM_SO_PTR * C], so_last = ds[BM_SO_LAST * C], so_step = ds[BM_SO_STEP * C];
  double sh_ptr = ds[BM_SH_PTR * C], sh_step = ds[BM_SH_STEP * C];
  double agc2_sum = ds[BM_AGC2_SUM * C], vol_gain = ds[BM_VOL_GAIN * C];
  double srx1 = ds[BM_SR_X1 * C], srx2 = ds[BM_SR_X2 * C], sry1 = ds[BM_SR_Y1 * C], sry2 = ds[BM_SR_Y2 * C];
  double ave_r = ds[BM_AVE_RE * C], ave_i = ds[BM_AVE_IM * C], rot_r = ds[BM_ROT_RE * C], rot_i = ds[BM_ROT_IM * C];
  double str_r = ds[BM_STR_RE * C], str_i = ds[BM_STR_IM * C], rotf = ds[BM_ROTF * C];
  // exp(i rotator_freq) changes only with rotator_freq (a symbol step or a
  // trident decision), so it is kept rather than evaluated every sample
  double rf_c, rf_s;
  b_cexp_i(rotf, rf_c, rf_s);
  double mse = ds[BM_MSE * C], msema_sum = ds[BM_MSEMA_SUM * C], diff_last = ds[BM_DIFF_LAST * C];
  int agc2_p = is[BMI_AGC2_P * C];
  int a1_p = is[BMI_A1_P * C], d8_p = is[BMI_D8_P * C], dsm_p = is[BMI_DSM_P * C];
  int msema_p = is[BMI_MSEMA_P * C];
  int startstop = is[BMI_STARTSTOP * C], cntr = is[BMI_CNTR * C];
  int hop_n = S.hop_n[c];
  long long sp = ls[BL_SP * C], scommit = ls[BL_SCOMMIT * C];
  const long long scons = ls[BL_SCONS * C];
  long long chk_done = ls[BL_CHK_DONE * C];
  const long long chk_n = ls[BL_CHK_N * C];
  long long next_chk = chk_done < chk_n ? S.chk_n[(size_t)c * TRI_SLOTS + (chk_done & (TRI_SLOTS - 1))] : LLONG_MAX;
#pragma unroll 1
  for (int j = 0; j < BM_LDS_TAPS; ++j) {
    s_qre[j][col] = S.fir[(size_t)j * C + c];
    s_qim[j][col] = S.fir[(size_t)(M_NT + j) * C + c];
  }
  double hre[BM_REG_TAPS], him[BM_REG_TAPS];  // partial sums of taps BM_LDS_TAPS..79
#pragma unroll
  for (int j = 0; j < BM_REG_TAPS; ++j) {
    hre[j] = S.fir[(size_t)(BM_LDS_TAPS + j) * C + c];
    him[j] = S.fir[(size_t)(M_NT + BM_LDS_TAPS + j) * C + c];
  }
  int16_t *soft = S.soft + (size_t)c * B_SOFT_RING;
  double *a1 = S.dl[2] + c, *d8 = S.dl[3] + c;
  double2 *dsm = reinterpret_cast<double2 *>(S.dl[4]) + c;
  const double PT = M_EE * WTSIZE;  // IfHavePassedPoint(ee)

  long long n = n0;
  // loads issued one sample ahead, as in demod_burst_kernel: val_to_demod,
  // mixer2's cis entry (reloaded when a decision moves mixer2), the agc2 slot
  auto vtd_at = [&](long long k) {
    return k >= M_D2 - 1 ? S.vring[(size_t)((k - (M_D2 - 1)) & (MV_LEN - 1)) * C + c] : 0.0;
  };
  double vtd_n = vtd_at(n);
  double2 m2_n = T.cis[b_cis_index(m2_ptr)];
  double2 so_n = T.cis[b_cis_index(so_ptr)];  // st_osc's entry (reloaded where the phase is set)
  double agc2_n = S.agc2[(size_t)agc2_p * C + c];
  // the symbol-tone PLL's table entry and the msema slot an update replaces,
  // ahead as well (see demod_burst_kernel)
  double2 h_n = T.cis[b_cis_index(sh_ptr)];
  double *const mm = S.msema + (size_t)c * M_MSEMA;
  double mm_n = mm[msema_p];
  while (n < end) {
    if (sp - scons > B_SOFT_RING - 64) break;  // soft ring full: framing frees it next
    // val_to_demod = d2.update_dont_touch(...): the front end's value M_D2 - 1 samples ago (zeros before)
    const double vtd = vtd_n;
    vtd_n = vtd_at(n + 1);  // past the front end's progress: unused
    if (n == next_chk) {
      // trident decision (burstmskdemodulator.cpp:475-522) from trident_bmsk_kernel's spectra; dcd is false
      const double *r = S.chk + ((size_t)c * TRI_SLOTS + (chk_done & (TRI_SLOTS - 1))) * CHK_REC;
      const double minval = r[0];
      const int minvalbin = (int)r[1], maxtoppos = (int)r[2];
      const int maxtopposhigh = (int)r[3];
      const double hzperbin = 48000.0 / 32768.0;
      constexpr int peakspacingbins = 410;  // qRound((0.5 * fb) / hzperbin)
      const int distfrompeak = abs(maxtoppos - minvalbin);
      const bool det = minval > 500.0 && abs(distfrompeak - peakspacingbins) < abs(peakspacingbins / 20) &&
                       !(cntr > 0 && cntr < (500 * MSPS));
      if (det) {
        vol_gain = 1.4142 * (500.0 / (minval / 3));
        const double carrierphase = aero_atan2(r[5], r[4]) - (M_PI / 4.0);
        b_set_phase_deg(m2_ptr, (180.0 / M_PI) * carrierphase);
        m2_n = T.cis[b_cis_index(m2_ptr)];
        // mixer2.SetFreq, then CenterFreqChangedSlot (:299-317) puts mixer2 on
        // mixer_center's clamped frequency
        double fc = ((maxtopposhigh + maxtoppos) / 2) * hzperbin;
        if (fc < (0.75 * 1200.0)) fc = 0.75 * 1200.0;
        if (fc > (48000.0 / 2.0 - 0.75 * 1200.0)) fc = 48000.0 / 2.0 - 0.75 * 1200.0;
        b_set_freq(m2_freq, m2_step, fc);
        startstop = M_STARTSTOP;
        cntr = 0;
        sp = scommit;  // RxDataBits.clear()
        soft[sp & (B_SOFT_RING - 1)] = B_SOFT_MARK;  // start of burst
        sp++;
        mse = 0;
        for (int k = 0; k < M_MSEMA; k++) mm[k] = 0;
        msema_sum = 0;
        msema_p = 0;
        mm_n = 0;
        ave_r = 1;
        ave_i = 0;
        str_r = 1;
        str_i = 0;
        rot_r = 1;
        rot_i = 0;
        rotf = 0;
        b_cexp_i(rotf, rf_c, rf_s);
        srx1 = srx2 = sry1 = sry2 = 0;
        b_set_phase_deg(so_ptr, 0);
        so_n = T.cis[b_cis_index(so_ptr)];
        b_set_phase_deg(sh_ptr, 0);
        h_n = T.cis[b_cis_index(sh_ptr)];
      }
      if (trace && hop_n < S.hop_cap) {
        double *h = S.hops + ((size_t)c * S.hop_cap + hop_n) * 6;
        h[0] = (double)n;
        h[1] = det ? 1.0 : 0.0;
        h[2] = m2_freq;
        h[3] = vol_gain;
        h[4] = minval;
        h[5] = (double)minvalbin + 65536.0 * (double)maxtoppos;
      }
      hop_n++;
      chk_done++;
      next_chk = chk_done < chk_n ? S.chk_n[(size_t)c * TRI_SLOTS + (chk_done & (TRI_SLOTS - 1))] : LLONG_MAX;
    }
    // sample counting and the signal-status timeout (:525-545)
    if (startstop > 0) {
      if (cntr >= (M_START * MSPS)) startstop--;
      if (cntr < 1000000) cntr++;
      if (mse < 0.6) startstop = M_STARTSTOP;
    }
    if (startstop == 0) {
      startstop--;
      cntr = 0;
      mse = 1;
    }
    if (startstop > 0 || mse < 0.6) {  // the demodulator proper (:547-700)
      // this part's ring reads first, as in the front end
      const bool tone = cntr > (M_START * MSPS) && cntr < M_ENDROT;
      const int dsr = dsm_p + 1 == M_DSM ? 0 : dsm_p + 1;
      const int d8o = d8_p + 1 == M_D8 ? 0 : d8_p + 1, d8n = d8o + 1 == M_D8 ? 0 : d8o + 1;
      const int a1o = a1_p + 1 == M_A1 ? 0 : a1_p + 1, a1n = a1o + 1 == M_A1 ? 0 : a1o + 1;
      const double agc2_old = agc2_n;
      const double2 pd_slot = dsm[(size_t)dsr * C];
      const double d8_old = d8[(size_t)d8o * C], d8_new = d8[(size_t)d8n * C];
      double a1_old = 0.0, a1_new = 0.0;
      if (tone) {
        a1_old = a1[(size_t)a1o * C];
        a1_new = a1[(size_t)a1n * C];
      }
      double s2r, s2i;
      {
        const double2 m2 = m2_n;
        double cr = m2.x * vtd, ci = m2.y * vtd;  // mixer2.WTCISValue() * (val_to_demod) * vol_gain
        cr = cr * vol_gain;
        ci = ci * vol_gain;
        // matched filter, transposed form (FIR::FIRUpdateAndProcess reads the 80 samples before the newest);
        // taps reloaded by scalar loads every sample, 8 at a time (a zero
        // offset laundered after each 8 taps: held across the loop they took
        // 160 SGPRs and spilled)
        int tz = 0;
        asm volatile("" : "+s"(tz));
        const double *tp = c_mtaps + tz;
        s2r = hre[BM_REG_TAPS - 1];
        s2i = him[BM_REG_TAPS - 1];
#pragma unroll
        for (int j = M_NT - 1; j > BM_LDS_TAPS; --j) {  // register part, descending: q[j - 1] read before rewritten
          hre[j - BM_LDS_TAPS] = hre[j - 1 - BM_LDS_TAPS] + tp[j] * cr;
          him[j - BM_LDS_TAPS] = him[j - 1 - BM_LDS_TAPS] + tp[j] * ci;
          if ((M_NT - 1 - j) % 8 == 7) {
            asm volatile("" : "+s"(tz) : "v"(hre[j - BM_LDS_TAPS]));
            tp = c_mtaps + tz;
          }
        }
        hre[0] = s_qre[BM_LDS_TAPS - 1][col] + tp[BM_LDS_TAPS] * cr;
        him[0] = s_qim[BM_LDS_TAPS - 1][col] + tp[BM_LDS_TAPS] * ci;
        for (int j = BM_LDS_TAPS - 1; j >= 1; --j) {
          s_qre[j][col] = s_qre[j - 1][col] + tp[j] * cr;
          s_qim[j][col] = s_qim[j - 1][col] + tp[j] * ci;
          if ((BM_LDS_TAPS - 1 - j) % 8 == 7) {
            asm volatile("" : "+s"(tz) : "v"(cr));
            tp = c_mtaps + tz;
          }
        }
        s_qre[0][col] = 0.0 + tp[0] * cr;
        s_qim[0][col] = 0.0 + tp[0] * ci;
      }
      if (tone) {  // symbol-tone x4 PLL (:555-578)
        const double t1r = s2r * str_r - s2i * str_i, t1i = s2r * str_i + s2i * str_r;
        const double spr = t1r * 0.0 - t1i * 1.0, spi = t1r * 1.0 + t1i * 0.0;  // * imag
        const double er = aero_tanh_bf(spi) * (spr);
        double ec, es;
        b_cexp_i(er * 0.5, ec, es);
        const double nr = str_r * ec - str_i * es, ni = str_r * es + str_i * ec;
        str_r = nr;
        str_i = ni;
        ave_r = ave_r * 0.999 + 0.001 * str_r;
        ave_i = ave_i * 0.999 + 0.001 * str_i;
        a1[(size_t)a1_p * C] = spr;  // a1.update(spr), whole-sample delay (dly_int)
        a1_p = a1o;
        const double spi2 = (0.0 * a1_new + (1.0 - 0.0) * a1_old);
        double progress = (double)cntr - (MSPS * (M_START));
        const double goal = M_ENDROT - (MSPS * M_START);
        progress = div_c(progress, goal);  // goal a compile-time constant, progress an integer
        const double2 hv = h_n;
        const double er_r = hv.x * spr - hv.y * (-spi2), er_i = hv.x * (-spi2) + hv.y * spr;
        double st_err = B_ATAN2(er_i, er_r);
        st_err *= 0.5 * (1.0 - progress * progress);
        b_advance(sh_ptr, -(1.0 / (2.0 * M_PI)) * st_err * 0.05);
        b_set_phase_deg_pos(so_ptr, div_cw(360.0 * sh_ptr, (double)WTSIZE) + (360.0 * (1.0 - M_EE)));  // in [351, 711)
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
      {  // agc2 and clip (:592-598)
        const double sa = B_HYPOT(s2r, s2i);
        agc2_sum = agc2_sum - agc2_old;
        agc2_sum = agc2_sum + fabs(sa);
        S.agc2[(size_t)agc2_p * C + c] = fabs(sa);
        agc2_p = agc2_p + 1 == M_AGC2 ? 0 : agc2_p + 1;
        agc2_n = S.agc2[(size_t)agc2_p * C + c];  // written M_AGC2 samples ago
        double g = div_n(1.414213562, fmax(div_c(agc2_sum, ((double)M_AGC2)), 0.000001));  // as above
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
      double pdr, pdi;  // pt_d = delayedsmpl.update_dont_touch(sig2)
      {
        dsm[(size_t)dsm_p * C] = make_double2(s2r, s2i);
        dsm_p = dsr;
        pdr = pd_slot.x;
        pdi = pd_slot.y;
      }
      double st_eta = B_HYPOT(s2r, pdi);  // abs(pt_msk), pt_msk = (sig2.re, pt_d.im)
      {  // st_iir_resonator.update (DSP.cpp:635-685)
        double y = 0;
        y += srx2 * c_msr_b[2];
        y += srx1 * c_msr_b[1];
        y += st_eta * c_msr_b[0];
        y -= sry2 * c_msr_a[2];
        y -= sry1 * c_msr_a[1];
        y /= c_msr_a[0];
        srx2 = srx1;
        srx1 = st_eta;
        sry2 = sry1;
        sry1 = y;
        st_eta = y;
      }
      d8[(size_t)d8_p * C] = st_eta;  // delayt8.update(st_eta), whole-sample delay (dly_int)
      d8_p = d8o;
      const double m1r = st_eta, m1i = -(0.0 * d8_new + (1.0 - 0.0) * d8_old);
      const double2 so = so_n;
      const double ore = so.x * m1r - so.y * m1i, oim = so.x * m1i + so.y * m1r;
      const double st_angle_error = B_ATAN2(oim, ore);
      if (cntr > M_ENDROT) b_advance(so_ptr, div_c(-st_angle_error * 0.002, 360.0));  // tiny: vanishes in so_ptr
      {  // IfHavePassedPoint(ee) (DSP.cpp:222-238) and the symbol step (:617-693)
        double tl = so_last - PT, tw = so_ptr - PT;
        if (tl < 0.0) tl += WTSIZE;
        if (tw < 0.0) tw += WTSIZE;
        if ((tl > 3.0 * WTSIZE / 4.0) && (tw < 1.0 * WTSIZE / 4.0)) {
          const double ct_xt = aero_tanh_bf(s2i) * s2r;
          const double ct_xt_d = aero_tanh_bf(pdr) * pdi;
          double ct_ec = ct_xt_d - ct_xt;
          if (ct_ec > M_PI) ct_ec = M_PI;
          if (ct_ec < -M_PI) ct_ec = -M_PI;
          if (ct_ec > M_PI_2) ct_ec = M_PI_2;
          if (ct_ec < -M_PI_2) ct_ec = -M_PI_2;
          if (cntr > (M_START * MSPS)) {
            double ec, es;
            b_cexp_i(ct_ec * 0.25, ec, es);
            const double rr = rot_r * ec - rot_i * es, ri = rot_r * es + rot_i * ec;
            rot_r = rr;
            rot_i = ri;
            if (cntr > M_ENDROT) {
              rotf = rotf + ct_ec * 0.0001;
              b_cexp_i(rotf, rf_c, rf_s);
            }
          }
          if (cntr > (M_START * MSPS)) {  // msema->Update (DSP.cpp:409-416)
            const double tda = (fabs(s2r * 0.75) - 1.0);
            const double tdb = (fabs(pdi * 0.75) - 1.0);
            const double v = (tda * tda) + (tdb * tdb);
            msema_sum = msema_sum - mm_n;
            msema_sum = msema_sum + fabs(v);
            mm[msema_p] = fabs(v);
            msema_p = msema_p + 1 == M_MSEMA ? 0 : msema_p + 1;
            mm_n = mm[msema_p];  // written M_MSEMA updates ago
            mse = msema_sum / ((double)M_MSEMA);
          }
          {  // differential soft bits, imag first, real negated (:664-686)
            const double imagin = m_diff_soft(diff_last, pdi);
            int ibit = b_qround((imagin) * 127.0 + 128.0);
            if (ibit > 255) ibit = 255;
            if (ibit < 0) ibit = 0;
            soft[sp & (B_SOFT_RING - 1)] = (int16_t)ibit;
            sp++;
            double real = m_diff_soft(diff_last, s2r);
            real = -real;
            ibit = b_qround((real) * 127.0 + 128.0);
            if (ibit > 255) ibit = 255;
            if (ibit < 0) ibit = 0;
            // emit processDemodulatedSoftBits (:689-692): the group's last
            // entry carries the mark in the same store
            const long long sp1 = sp;
            sp++;
            if (sp - scommit >= M_SOFT_GROUP) {
              ibit |= B_SOFT_LAST;
              scommit = sp;
            }
            soft[sp1 & (B_SOFT_RING - 1)] = (int16_t)ibit;
          }
        }
      }
      so_last = so_ptr;
      b_nco_next(so_ptr, so_step);
      so_n = T.cis[b_cis_index(so_ptr)];
      b_nco_next(sh_ptr, sh_step);
      h_n = T.cis[b_cis_index(sh_ptr)];
      b_nco_next(m2_ptr, m2_step);
      m2_n = T.cis[b_cis_index(m2_ptr)];
    }
    n++;
  }
  // state back
#pragma unroll 1
  for (int j = 0; j < BM_LDS_TAPS; ++j) {
    S.fir[(size_t)j * C + c] = s_qre[j][col];
    S.fir[(size_t)(M_NT + j) * C + c] = s_qim[j][col];
  }
#pragma unroll
  for (int j = 0; j < BM_REG_TAPS; ++j) {
    S.fir[(size_t)(BM_LDS_TAPS + j) * C + c] = hre[j];
    S.fir[(size_t)(M_NT + BM_LDS_TAPS + j) * C + c] = him[j];
  }
  ds[BM_M2_PTR * C] = m2_ptr;
  ds[BM_M2_STEP * C] = m2_step;
  ds[BM_M2_FREQ * C] = m2_freq;
  ds[BM_SO_PTR * C] = so_ptr;
  ds[BM_SO_LAST * C] = so_last;
  ds[BM_SH_PTR * C] = sh_ptr;
  ds[BM_AGC2_SUM * C] = agc2_sum;
  ds[BM_VOL_GAIN * C] = vol_gain;
  ds[BM_SR_X1 * C] = srx1;
  ds[BM_SR_X2 * C] = srx2;
  ds[BM_SR_Y1 * C] = sry1;
  ds[BM_SR_Y2 * C] = sry2;
  ds[BM_AVE_RE * C] = ave_r;
  ds[BM_AVE_IM * C] = ave_i;
  ds[BM_ROT_RE * C] = rot_r;
  ds[BM_ROT_IM * C] = rot_i;
  ds[BM_STR_RE * C] = str_r;
  ds[BM_STR_IM * C] = str_i;
  ds[BM_ROTF * C] = rotf;
  ds[BM_MSE * C] = mse;
  ds[BM_MSEMA_SUM * C] = msema_sum;
  ds[BM_DIFF_LAST * C] = diff_last;
  is[BMI_AGC2_P * C] = agc2_p;
  is[BMI_A1_P * C] = a1_p;
  is[BMI_D8_P * C] = d8_p;
  is[BMI_DSM_P * C] = dsm_p;
  is[BMI_MSEMA_P * C] = msema_p;
  is[BMI_STARTSTOP * C] = startstop;
  is[BMI_CNTR * C] = cntr;
  S.hop_n[c] = hop_n;
  ls[BL_NSAMP * C] = n;
  ls[BL_SP * C] = sp;
  ls[BL_SCOMMIT * C] = scommit;
  ls[BL_CHK_DONE * C] = chk_done;
}

// --------------------------------------------------------- trident check
// burstmskdemodulator.cpp:414-473 for every channel waiting on it: base =
// FFTr of tridentbuffer[0, 5040), top = FFTr of [5040, 8000); the first
// strict maximum of |base| over bins [0, 16384), and of |top| over bins
// (50, minvalbin - 205) and (minvalbin + 205, 16384), each starting from 0.
__global__ __launch_bounds__(1024) void trident_bmsk_kernel(BurstState S, BurstTables T) {
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
  for (int job = blockIdx.x; job < njobs; job += gridDim.x) {
  const int c = S.tjobs[job] & 0xFFFFFF, slot = S.tjobs[job] >> 24;
  const double *tb = S.tri + ((size_t)c * TRI_SLOTS + slot) * M_TRI;
  // block reduction of (value, bin) candidates: larger value, then smaller bin
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
  // a candidate only if strictly above the running 0 start (the loops' initial maximum)
  auto offer = [](double ab, int p, double &lv, int &li) {
    if (ab > 0.0 && (ab > lv || (ab == lv && p < li))) {
      lv = ab;
      li = p;
    }
  };
  constexpr int NONE = 0x7fffffff;
  double minval = 0;
  int minbin = 0;
  int toplo = 0, tophi = 0;
  for (int pass = 0; pass < 2; ++pass) {
    const int off = pass ? M_TRI_BASE : 0, len = pass ? M_TRI_TOP : M_TRI_BASE;
    double2 x[16];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int j = bitrev<L>(epos<L, 0>(t, i));
      const double a = 2 * j < len ? tb[off + 2 * j] : 0.0;
      const double b = 2 * j + 1 < len ? tb[off + 2 * j + 1] : 0.0;
      x[i] = make_double2(a, b);
    }
    fft_dit<L, false>(x, t, lds, T.tw16, s_tw);
    // out[i] = F[i] * DA[i] + DB[i] * conj(F[(N - i) % N]) (fftrwrapper.cpp)
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
    double lv = 0.0, hv = 0.0;
    int li = NONE, hi = NONE;
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
        offer(ab, p, lv, li);
      } else if (p > 50) {
        if (p < minbin - (410 / 2)) offer(ab, p, lv, li);
        if (p > minbin + (410 / 2)) offer(ab, p, hv, hi);
      }
    }
    if (pass == 0) {
      double bv;
      int bi;
      reduce(lv, li, bv, bi);
      minval = bi == NONE ? 0.0 : bv;
      minbin = bi == NONE ? 0 : bi;
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if (epos<L, 3>(t, i) == minbin) s_best = x[i];
      __syncthreads();
    } else {
      double bv;
      int bi;
      reduce(lv, li, bv, bi);
      toplo = bi == NONE ? 0 : bi;
      reduce(hv, hi, bv, bi);
      tophi = bi == NONE ? 0 : bi;
    }
  }
  if (t == 0) {  // the record demod_bmsk_kernel decides on at the check's sample
    double *r = S.chk + ((size_t)c * TRI_SLOTS + slot) * CHK_REC;
    r[0] = minval;
    r[1] = minbin;
    r[2] = toplo;
    r[3] = tophi;
    r[4] = s_best.x;
    r[5] = s_best.y;
  }
  __syncthreads();  // the LDS and s_best are the next check's
  }
}

// -------------------------------------------------------- AeroL framing
// AeroL::Decode, MSK burst branch (decode/aerol.cpp:1155-1178, 1183-1252,
// 2014-2030): the start-of-burst marker resets muw; mskBurstDetector takes 4
// bit errors either polarity, a sync more than 250 bits after the marker is
// dropped and its polarity change undone; a sync starts a packet with a dummy
// header (cntr jumps to 16) and every soft bit then fills the R/T block; a
// burst window ends after ifb * 3 bits, dropping the rest of that group.
// A lane stops before a new packet would overwrite the block of tests it
// queued this pass, and after RT_TESTS_PER_PASS tests.
__global__ __launch_bounds__(256) void frame_bmsk_kernel(BurstState S, int nch) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nch) return;
  const int C = S.C;
  int *is = S.is + c;
  long long *ls = S.ls + c;
  const long long E = ls[BL_SCOMMIT * C];
  long long q = ls[BL_SCONS * C];
  if (q >= E) return;
  int muw = is[BMI_MUW * C], cntr = is[BMI_FCNTR * C];
  uint32_t uw = (uint32_t)is[BMI_UW * C];
  int inv = is[BMI_UW_INV * C], blockptr = is[BMI_BLOCKPTR * C], burst = is[BMI_BURST_ID * C];
  int skip = is[BMI_SKIP_GROUP * C];
  const int total = is[BMI_TOTAL * C];
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
    const int inv_before = inv;
    uw = (uw << 1) | (uint32_t)bit;
    const int xs = __builtin_popcount(uw ^ MUW);
    int gotsync = 0;
    if (xs >= 32 - 4) {
      inv = 1;
      gotsync = 1;
    } else if (xs <= 4) {
      inv = 0;
      gotsync = 1;
    }
    if (muw > 250 && gotsync) {
      inv = inv_before;
      gotsync = 0;
    }
    if (inv) {
      bit = 1 - bit;
      if (soft_bit != 128) soft_bit = 255 - soft_bit;
    }
    if (cntr < 1000000000) cntr++;
    if (cntr == 0) {  // dummy header, rtchanneldeleavefecscram.resetblockptr()
      cntr = 16;
      blockptr = 0;
      burst++;
    }
    if (cntr >= 16 && blockptr < RT_BLOCK) {  // RTChannelDeleaveFECScram::updateMSK
      blk[blockptr] = (uint8_t)soft_bit;
      blockptr++;
      if (blockptr >= 64 * 5 && ((blockptr - (64 * 5)) % (64 * 3)) == 0) {
        const int j = atomicAdd(S.njobs, 1);
        reinterpret_cast<int4 *>(S.jobs)[j] = make_int4(c, blockptr, burst, 1);
        emitted++;
      }
    }
    if (gotsync) {
      cntr = -1;
      if (!is[BMI_DATACD * C]) {  // datacd = true (aerol.cpp:2010-2012), a change for SignalHunter::handleDcd
        is[BMI_DATACD * C] = 1;
        is[BMI_DCD_EDGES * C]++;
      }
    }
    if (cntr + 1 == total) {  // end of the burst window: Decode returns
      cntr = 1000000000;
      if (is[BMI_DATACD * C]) {  // datacd = false (aerol.cpp:2021-2028)
        is[BMI_DATACD * C] = 0;
        is[BMI_DCD_EDGES * C]++;
      }
      if (!last) skip = 1;
    }
  }
  ls[BL_SCONS * C] = q;
  is[BMI_MUW * C] = muw;
  is[BMI_FCNTR * C] = cntr;
  is[BMI_UW * C] = (int)uw;
  is[BMI_UW_INV * C] = inv;
  is[BMI_BLOCKPTR * C] = blockptr;
  is[BMI_BURST_ID * C] = burst;
  is[BMI_SKIP_GROUP * C] = skip;
}

// ------------------------------------------------------------ launchers
void burst_msk_upload_constants(const double *sr_b, const double *sr_a, const double *taps) {
  hipMemcpyToSymbol(HIP_SYMBOL(c_msr_b), sr_b, sizeof(double) * 3);
  hipMemcpyToSymbol(HIP_SYMBOL(c_msr_a), sr_a, sizeof(double) * 3);
  hipMemcpyToSymbol(HIP_SYMBOL(c_mtaps), taps, sizeof(double) * M_NT);
}

void launch_front_bmsk(hipStream_t st, const BurstState &S, const BurstTables &T, int nch) {
  hipLaunchKernelGGL(front_bmsk_kernel, dim3((nch + 63) / 64), dim3(64), 0, st, S, T, nch);
}

void launch_demod_bmsk(hipStream_t st, const BurstState &S, const BurstTables &T, int nch, int trace) {
  hipLaunchKernelGGL(demod_bmsk_kernel, dim3((nch + BM_BLOCK - 1) / BM_BLOCK), dim3(BM_BLOCK), 0, st, S, T, nch,
                     trace);
}

void launch_trident_bmsk(hipStream_t st, const BurstState &S, const BurstTables &T, int nch) {
  hipLaunchKernelGGL(trident_bmsk_kernel, dim3(std::min(nch * TRI_SLOTS, TRI_GRID)), dim3(1024), 0, st, S, T);
}

void launch_frame_bmsk(hipStream_t st, const BurstState &S, int nch) {
  hipLaunchKernelGGL(frame_bmsk_kernel, dim3((nch + 255) / 256), dim3(256), 0, st, S, nch);
}

}  // namespace aero
