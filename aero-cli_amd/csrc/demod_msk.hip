/*
 * demod_msk.hip — batched continuous MSK demodulator (600 / 1200 bps) for
 * gfx950: MskDemodulator::writeData (decode/mskdemodulator.cpp:252-428) as
 * aero-decode configures it (decode/decode.cpp:142-150: Fs 12000 / 24000,
 * fb stays 600, freq_center 0, AFC on, dcd never set), and at any other
 * rate after a rate change (mskdemodulator.cpp:473-481): one kernel per Fs
 * for 12, 24 and 48 kHz (MskK), a generic-rate kernel for the others.
 *
 * One VFO channel per lane, thousands side by side, the same structure as
 * demod_oqpsk.hip:
 *   - the 2*SPS-tap half-sine matched filter runs in transposed form, real
 *     partial sums in VGPRs, imaginary ones in LDS [tap][lane];
 *   - the per-sample delay lines (delayedsmpl, delayt8) and the AGC ring are
 *     time-major HBM rings indexed by sample number, so channels that move in
 *     step read and write one coalesced row;
 *   - the symbol event (carrier loop, rotation, MSE, differential soft bits)
 *     runs once per st_osc cycle, 1 sample in 2*SPS; lanes run their samples
 *     up to their next event (inner loop) and the event step then runs for
 *     all lanes together, so a wave does not pay for one lane's event every
 *     sample.  Per lane, operations and their order are the reference's.
 *
 * Bit-exactness rules as demod_oqpsk.hip (-ffp-contract=off, reference
 * operation order, std::complex products expanded as GCC does, libm from
 * aero_math.h).  std::sqrt is IEEE (correctly rounded) on both sides.
 */
#include <hip/hip_runtime.h>

#include "aero_math.h"
#include "engine_common.h"

namespace aero {

__constant__ double c_msk_d8w[2];   // delayt8 weights {weighting, 1 - weighting} (pointer-independent, host-checked)

namespace {

__device__ __forceinline__ int cis_index(double WTptr) {  // WaveTable::WTCISValue (DSP.cpp:81-88)
  int tint = (int)WTptr;
  if (tint >= WTSIZE) tint = 0;
  if (tint < 0) tint = WTSIZE - 1;
  return tint;
}

__device__ __forceinline__ void nco_next(double &ptr, double &step) {  // WTnextFrame (DSP.cpp:71-79)
  if (step < 0) step = 0;
  ptr += step;
  wt_wrap_int(ptr);
}

__device__ __forceinline__ int qround(double d) {  // qRound (Qt 5.9 qglobal.h:525)
  return d >= 0.0 ? int(d + 0.5) : int(d - double(int(d - 1)) + 0.5) + int(d - 1);
}

__device__ __forceinline__ double diff_soft(double &last, double soft) {  // DiffDecode::UpdateSoft (DSP.cpp:523-548)
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

template <int M>
__global__ __launch_bounds__(MskK<M>::WG) void demod_msk_kernel(DevState S, DevTables T, int nch, int flush) {
  using K = MskK<M>;
  constexpr int WG = K::WG;
  constexpr int SPS = K::SPS;
  constexpr int NT = 2 * SPS;            // matched filter taps (mskdemodulator.cpp:126-133)
  constexpr int AGC = K::FS;             // AGC(1, Fs) (mskdemodulator.cpp:135)
  constexpr int DSM = SPS + 1;           // delayedsmpl.setLength(SPS)
  constexpr int D8 = SPS / 2 + 1;        // delayt8.setdelay(SPS / 2.0): ceil + 1 slots
  constexpr int DTL = SPS / 2 + 1;       // dt.setLength(SPS / 2)
  constexpr int MARG = SPS;              // marg = MovingAverage(SPS)
  constexpr double FS = (double)K::FS;
  static_assert(DSM >= 3 && D8 >= 4, "one-sample-ahead ring loads never read a slot the sample before writes");
  // imaginary matched-filter partial sums: registers at 12 kHz (40 taps,
  // ~400 of the 512 registers with the real ones), LDS at 24 / 48 kHz (80 /
  // 160 taps would not fit); at 48 kHz the oldest 100 real ones are LDS too.
  // At 24 kHz the newest two stay in registers: 78 x 128 channels + the taps
  // is 80.5 KB, so two workgroups (four waves) share a CU's LDS and 65536
  // channels run in one round instead of two
  constexpr bool QREG = NT <= 40;
  constexpr int NRL = NT > 80 ? NT - 60 : 0;  // real partial sums 0..NRL-1 in LDS
  constexpr int NIL = QREG ? 0 : (NT == 80 ? NT - 2 : NT);  // imaginary partial sums 0..NIL-1 in LDS
  __shared__ double s_qim[NIL > 0 ? NIL : 1][WG];
  __shared__ double s_qre[NRL > 0 ? NRL : 1][WG];
  __shared__ double s_taps[NT];
  // at 12 kHz (one 256-lane workgroup per CU, LDS to spare) the libm tables
  // the chain gathers from (atan2's cij rows every sample, sincos's table
  // every event) are copied to LDS; the 24 kHz workgroups pack two per CU
  // and the 48 kHz ones fill it, so those read the global copies
  constexpr bool LTAB = SPS == 20;
  __shared__ double s_cij[LTAB ? 241 : 1][7];
  __shared__ double s_sct[LTAB ? 440 : 1];
  for (int l = threadIdx.x; l < NT; l += WG) s_taps[l] = T.taps[l];
  if (LTAB) {
    for (int k = threadIdx.x; k < 241 * 7; k += WG) (&s_cij[0][0])[k] = (&aero_g_cij[0][0])[k];
    for (int k = threadIdx.x; k < 440; k += WG) s_sct[k] = aero_g_sincostab[k];
  }
  __syncthreads();
  const int c = blockIdx.x * WG + threadIdx.x;
  const int lane = threadIdx.x;
  if (c >= nch) return;
  const int C = S.C;
  const int HOPN = MSK_HOP, NF = MSK_NFFT;

  const long long n0 = S.ls[LS_NSAMP * C + c];
  const long long avail = S.ls[LS_AVAIL * C + c];
  const long long filled0 = S.ls[LS_FILLED * C + c];
  const int hops_done = S.is[IS_HOPS_DONE * C + c];
  const long long boundary = (long long)HOPN * (hops_done + 1) - 1;
  long long end = avail < boundary ? avail : boundary;
  if (!flush && avail <= boundary) end = n0;
  const int capm = (int)S.pcm_cap - 1;
  const int ia = (int)(avail - n0);
  const int ie = (int)(end - n0);
  int ifl = (int)(filled0 - n0);

  double mc_ptr = S.ds[DS_MC_PTR * C + c], mc_step = S.ds[DS_MC_STEP * C + c];
  if (ifl == 0 && ia > 0) {  // coarse-ring entry of sample n0
    const int16_t x = S.pcm[(size_t)(n0 & capm) * C + c];
    S.cring[(size_t)c * NF + (n0 & (NF - 1))] = (uint32_t)cis_index(mc_ptr) | ((uint32_t)(uint16_t)x << 16);
    ifl = 1;
  }
  if (ie <= 0) {
    S.ls[LS_FILLED * C + c] = n0 + ifl;
    return;
  }

  double m2_ptr = S.ds[DS_M2_PTR * C + c], m2_step = S.ds[DS_M2_STEP * C + c];
  double m2_freq = S.ds[DS_M2_FREQ * C + c];
  double so_ptr = S.ds[DS_SO_PTR * C + c], so_last = S.ds[DS_SO_LAST * C + c];
  const double so_step = S.ds[DS_SO_STEP * C + c];
  double agc_sum = S.ds[DS_AGC_SUM * C + c];
  double srx1 = S.ds[DS_SR_X1 * C + c], srx2 = S.ds[DS_SR_X2 * C + c];
  double sry1 = S.ds[DS_SR_Y1 * C + c], sry2 = S.ds[DS_SR_Y2 * C + c];
  double marg_sum = S.ds[DS_MARG_SUM * C + c], ms_sum = S.ds[DS_MS_SUM * C + c];
  double mse = S.ds[DS_MSE * C + c], diff_last = S.ds[DS_DIFF_LAST * C + c];
  long long ev = S.ls[LS_EVENTS * C + c];
  const int ms_off = S.is[IS_MS_OFF * C + c];  // msema's slot offset (see IS_MS_OFF)
  long long softp = S.ls[LS_SOFT_P * C + c];
  long long ptn = S.ls[LS_PT_N * C + c];

  double qr[NT - NRL];
  double qi[NT - NIL > 0 ? NT - NIL : 1];
  auto QI = [&](int j) -> double & {
    if (j < NIL)
      return s_qim[j < NIL ? j : 0][lane];
    else
      return qi[j - NIL];
  };
  auto Q = [&](int j) -> double & {
    if (j < NRL)
      return s_qre[j < NRL ? j : 0][lane];
    else
      return qr[j - NRL];
  };
#pragma unroll
  for (int j = 0; j < NT; ++j) Q(j) = S.fir[(size_t)j * C + c];
#pragma unroll
  for (int j = 0; j < NT; ++j) QI(j) = S.fir[(size_t)(NT + j) * C + c];

  const double PT = K::EE * WTSIZE;  // IfHavePassedPoint(ee) (mskdemodulator.cpp:177-203)
  const double d8w = c_msk_d8w[0], d8omw = c_msk_d8w[1];

  int i = 0;
  // event operands carried out of the sample loop
  double e_s2r = 0, e_s2i = 0, e_pdr = 0, e_pdi = 0;
  // PCM words two samples ahead (the coarse-ring entry staged during sample
  // n holds sample n+1's word; loaded one sample ahead it would be waited for
  // at once)
  int16_t pcm_a = S.pcm[(size_t)(n0 & capm) * C + c];
  int16_t pcm_b = S.pcm[(size_t)((n0 + 1) & capm) * C + c];
  // at 12 kHz a sample's AGC, delayedsmpl and delayt8 ring slots are loaded
  // one sample ahead (an HBM round trip each, which the sample would
  // otherwise wait for); none is a slot the sample before writes, and
  // delayt8's "newer" slot is the next sample's "older".  (At 24 / 48 kHz the
  // five extra live values spill: there they are loaded at the sample's top.)
  constexpr bool AHEAD = QREG;
  double agc_nx = S.agc[(size_t)(n0 % AGC) * C + c];
  double2 dsm_nx = S.dsm[(size_t)((n0 + 1) % DSM) * C + c];
  double d8o_nx = S.d8[(size_t)((n0 + 1) % D8) * C + c];
  double d8n_nx = S.d8[(size_t)((n0 + 2) % D8) * C + c];
  while (i < ie) {
    bool pend = false;
    do {
      const long long n = n0 + i;
      // this sample's ring reads before any of its stores, so their round
      // trips overlap (the rings are distinct, the compiler cannot prove it);
      // no slot read is the slot written this sample
      const int16_t xs = pcm_a;
      pcm_a = pcm_b;
      pcm_b = S.pcm[(size_t)((n + 2) & capm) * C + c];  // past the pushed samples: unused
      double agc_old, d8_older, d8_newer;
      double2 dsm_old;
      if constexpr (AHEAD) {
        agc_old = agc_nx;
        dsm_old = dsm_nx;
        d8_older = d8o_nx;
        d8_newer = d8n_nx;
        agc_nx = S.agc[(size_t)((n + 1) % AGC) * C + c];
        dsm_nx = S.dsm[(size_t)((n + 2) % DSM) * C + c];
        d8o_nx = d8n_nx;
        d8n_nx = S.d8[(size_t)((n + 3) % D8) * C + c];
      } else {
        agc_old = S.agc[(size_t)(n % AGC) * C + c];
        dsm_old = S.dsm[(size_t)((n + 1) % DSM) * C + c];
        d8_older = S.d8[(size_t)((n + 1) % D8) * C + c];
        d8_newer = S.d8[(size_t)((n + 2) % D8) * C + c];
      }
      const double dval = ((double)xs) / 32768.0;
      const double2 cm = T.cis[cis_index(m2_ptr)];
      const double cv = cm.x * dval, cvi = cm.y * dval;  // mixer2.WTCISValue() * dval
      // matched filter: FIRUpdateAndProcess reads the 2*SPS samples before the newest
      double s2r = Q(NT - 1), s2i = QI(NT - 1);
#pragma unroll
      for (int j = NT - 1; j >= 1; --j) {
        Q(j) = Q(j - 1) + s_taps[j] * cv;
        if (NRL > 0 && j < NRL && (j & 7) == 0) asm volatile("" : : : "memory");
      }
      Q(0) = 0.0 + s_taps[0] * cv;
#pragma unroll
      for (int j = NT - 1; j >= 1; --j) {
        QI(j) = QI(j - 1) + s_taps[j] * cvi;
        if (!QREG && (j & 7) == 0) asm volatile("" : : : "memory");
      }
      QI(0) = 0.0 + s_taps[0] * cvi;
      const double dab = sqrt(s2r * s2r + s2i * s2i);
      {  // AGC::Update (DSP.cpp:371-380)
        agc_sum = agc_sum - agc_old;
        agc_sum = agc_sum + fabs(dab);
        S.agc[(size_t)(n % AGC) * C + c] = fabs(dab);
        // short exact divisions (aero_math.h): a tiny agc_sum / AGC is floored at 1e-6
        double g = div_n(1.414213562, fmax(div_c(agc_sum, ((double)AGC)), 0.000001));
        g = fmax(g, 0.000001);
        s2r *= g;
        s2i *= g;
      }
      const double ab = sqrt(s2r * s2r + s2i * s2i);
      if (ab > 2.84) {
        const double k = div_n(2.84, ab);  // ab > 2.84
        s2r = k * s2r;
        s2i = k * s2i;
      }
      // pt_d = delayedsmpl.update_dont_touch(sig2) (DSP.h:468-473)
      double pdr, pdi;
      {
        S.dsm[(size_t)(n % DSM) * C + c] = make_double2(s2r, s2i);
        pdr = dsm_old.x;
        pdi = dsm_old.y;
      }
      // st_eta = resonator(|pt_msk|), pt_msk = (sig2.re, pt_d.im)
      double st_eta;
      {
        const double sig = aero_hypot_w(s2r, pdi);
        double y = 0;
        y += srx2 * K::SR_B2;
        y += srx1 * 0.0;
        y += sig * K::SR_B0;
        y -= sry2 * K::SR_A2;
        y -= sry1 * K::SR_A1;
        srx2 = srx1;
        srx1 = sig;
        sry2 = sry1;
        sry1 = y;
        st_eta = y;
      }
      // delayt8.update(st_eta) (DSP.h:365-384): ages SPS/2 and SPS/2 - 1
      double d8v;
      {
        S.d8[(size_t)(n % D8) * C + c] = st_eta;
        d8v = (d8w * d8_newer + d8omw * d8_older);
      }
      const double m1r = st_eta, m1i = -d8v;
      const double2 so = T.cis[cis_index(so_ptr)];
      const double ore = so.x * m1r - so.y * m1i, oim = so.x * m1i + so.y * m1r;
      const double ang = LTAB ? aero_atan2_bf(oim, ore, s_cij) : aero_atan2_bf(oim, ore, aero_g_cij);
      const double weighting = fabs(aero_tanh_bf(ang));
      {  // st_osc.AdvanceFractionOfWave (DSP.h:59-65), dcd false
        so_ptr += (-(1.0 - weighting) * ang * (0.05 / 360.0)) * WTSIZE;
        wt_wrap(so_ptr);
      }
      {  // IfHavePassedPoint (DSP.cpp:222-238)
        double tl = so_last - PT, tw = so_ptr - PT;
        if (tl < 0.0) tl += WTSIZE;
        if (tw < 0.0) tw += WTSIZE;
        if ((tl > 3.0 * WTSIZE / 4.0) && (tw < 1.0 * WTSIZE / 4.0)) {
          pend = true;
          e_s2r = s2r;
          e_s2i = s2i;
          e_pdr = pdr;
          e_pdi = pdi;
        }
      }
      // the coarse-ring entry of the next sample (mskdemodulator.cpp:284-287)
      nco_next(mc_ptr, mc_step);
      so_last = so_ptr;
      {
        double st = so_step;
        nco_next(so_ptr, st);
      }
      if (i + 1 < ia) {
        const long long n1 = n + 1;
        const int16_t x1 = pcm_a;
        S.cring[(size_t)c * NF + (n1 & (NF - 1))] = (uint32_t)cis_index(mc_ptr) | ((uint32_t)(uint16_t)x1 << 16);
        ifl = i + 2;
      }
      if (!pend) {
        nco_next(m2_ptr, m2_step);
        ++i;
      }
    } while (!pend && i < ie);
    if (pend) {
      // carrier tracking (mskdemodulator.cpp:333-357)
      const double ct_xt = aero_tanh_bf(e_s2i) * e_s2r;
      const double ct_xt_d = aero_tanh_bf(e_pdr) * e_pdi;
      double ct_ec = ct_xt_d - ct_xt;
      if (ct_ec > M_PI) ct_ec = M_PI;
      if (ct_ec < -M_PI) ct_ec = -M_PI;
      if (ct_ec > M_PI_2) ct_ec = M_PI_2;
      if (ct_ec < -M_PI_2) ct_ec = -M_PI_2;
      const double carrier_aggression = 12.0 * 1.0;  // correctionfactor 1.0 (fb < 1200)
      {  // mixer2.IncresePhaseDeg (DSP.cpp:177-187)
        double phase_deg = carrier_aggression * 1.0 * ct_ec;
        phase_deg += div_cw(360.0 * m2_ptr, (double)WTSIZE);
        m2_ptr = set_phase_ptr(phase_deg);
      }
      {  // mixer2.IncreseFreqHz -> SetFreq(double) (DSP.cpp:163-175)
        double f = carrier_aggression * 0.01 * ct_ec;
        f += m2_freq;
        m2_freq = f;
        if (m2_freq < 0) m2_freq = 0;
        m2_step = (m2_freq) * ((double)WTSIZE) / FS;
      }
      int cl = c;
      asm volatile("" : "+v"(cl));
      // marg->UpdateSigned(ct_ec / 2.0) (DSP.cpp:419-427)
      double mval;
      {
        double *mb = S.marg + (size_t)cl * MARG;
        const int p = (int)(ev % MARG);
        const double nv = ct_ec / 2.0;
        marg_sum = marg_sum - mb[p];
        marg_sum = marg_sum + (nv);
        mb[p] = nv;
        mval = marg_sum / ((double)MARG);
      }
      // dt.update(pt_msk) (DSP.h:463-467)
      double pr, pi;
      {
        double2 *db = S.dt + (size_t)cl * DTL;
        db[ev % DTL] = make_double2(e_s2r, e_pdi);
        const double2 o = db[(ev + 1) % DTL];
        pr = o.x;
        pi = o.y;
      }
      {  // pt_msk *= cpx(cos(marg->Val), sin(marg->Val))
        double rs, rc;
        if (LTAB)
          aero_sincos_bf(mval, rs, rc, s_sct);
        else
          aero_sincos_bf(mval, rs, rc, aero_g_sincostab);
        const double rr = pr * rc - pi * rs, ri = pr * rs + pi * rc;
        pr = rr;
        pi = ri;
      }
      if (S.pt_cap) {
        if (ptn < S.pt_cap) S.pt[(size_t)cl * S.pt_cap + ptn] = make_double2(pr, pi);
        ptn++;
      }
      {  // mse = msema->Update(tda^2 + tdb^2) (DSP.cpp:405-413)
        const double tda = (fabs((pr) * 0.75) - 1.0);
        const double tdb = (fabs((pi) * 0.75) - 1.0);
        const double v = (tda * tda) + (tdb * tdb);
        double *mb = S.ms + (size_t)cl * MSK_MSEMA;
        const int p = (int)((ev + ms_off) % MSK_MSEMA);
        ms_sum = ms_sum - mb[p];
        ms_sum = ms_sum + fabs(v);
        mb[p] = fabs(v);
        mse = ms_sum / ((double)MSK_MSEMA);
      }
      {  // differential soft bits, imag first, real negated (mskdemodulator.cpp:381-401)
        const double imagin = diff_soft(diff_last, pi);
        int ibit = qround((imagin) * 127.0 + 128.0);
        if (ibit > 255) ibit = 255;
        if (ibit < 0) ibit = 0;
        double real = diff_soft(diff_last, pr);
        real = -real;
        int rbit = qround((real) * 127.0 + 128.0);
        if (rbit > 255) rbit = 255;
        if (rbit < 0) rbit = 0;
        uint8_t *soft = S.soft + (size_t)cl * SOFT_RING;
        soft[softp & (SOFT_RING - 1)] = (uint8_t)ibit;
        soft[(softp + 1) & (SOFT_RING - 1)] = (uint8_t)rbit;
        softp += 2;
      }
      ev++;
      nco_next(m2_ptr, m2_step);
      ++i;
    }
  }

  int cl = c;
  asm volatile("" : "+v"(cl));
  {
    double *fir = S.fir + cl;
#pragma unroll
    for (int j = 0; j < NT; ++j) fir[(size_t)j * C] = Q(j);
#pragma unroll
    for (int j = 0; j < NT; ++j) fir[(size_t)(NT + j) * C] = QI(j);
  }
  double *ds = S.ds + cl;
  long long *ls = S.ls + cl;
  ls[LS_NSAMP * C] = n0 + i;
  ls[LS_FILLED * C] = n0 + ifl;
  ls[LS_SOFT_P * C] = softp;
  ls[LS_EVENTS * C] = ev;
  if (S.pt_cap) ls[LS_PT_N * C] = ptn;
  ds[DS_M2_PTR * C] = m2_ptr;
  ds[DS_M2_STEP * C] = m2_step;
  ds[DS_M2_FREQ * C] = m2_freq;
  ds[DS_MC_PTR * C] = mc_ptr;
  ds[DS_MC_STEP * C] = mc_step;
  ds[DS_SO_PTR * C] = so_ptr;
  ds[DS_SO_LAST * C] = so_last;
  ds[DS_AGC_SUM * C] = agc_sum;
  ds[DS_SR_X1 * C] = srx1;
  ds[DS_SR_X2 * C] = srx2;
  ds[DS_SR_Y1 * C] = sry1;
  ds[DS_SR_Y2 * C] = sry2;
  ds[DS_MARG_SUM * C] = marg_sum;
  ds[DS_MS_SUM * C] = ms_sum;
  ds[DS_MSE * C] = mse;
  ds[DS_DIFF_LAST * C] = diff_last;
}

// The generic-rate kernel: MskDemodulator at any other Fs in [MSK_FS_MIN,
// MSK_FS_MAX] (setSettings, decode/mskdemodulator.cpp:94-218, applied with
// that Fs), the same per-sample and per-event arithmetic as demod_msk_kernel
// with the rate's constants from S.mg and S.g: the matched filter's 2 SPS
// partial sums stay in their HBM rows (S.fir, [tap][C]) through the segment,
// every ring is read at the top of its sample, the libm tables are the
// global copies.  One 64-lane workgroup per 64 channels.
constexpr int MSKG_WG = 64;
__global__ __launch_bounds__(MSKG_WG) void demod_mskg_kernel(DevState S, DevTables T, int nch, int flush) {
  const MskGen &G = S.mg;
  const int SPS = G.sps, NT = 2 * SPS, AGC = S.g.agc_len, DSM = S.g.dsm_len, D8 = S.g.d8_len, DTL = S.g.dt_len,
            MARG = S.g.marg_len;
  const double FS = G.fs;
  __shared__ double s_taps[MAX_TAPS];
  for (int l = threadIdx.x; l < NT; l += MSKG_WG) s_taps[l] = T.taps[l];
  __syncthreads();
  const int c = blockIdx.x * MSKG_WG + threadIdx.x;
  if (c >= nch) return;
  const int C = S.C;
  const int HOPN = MSK_HOP, NF = MSK_NFFT;

  const long long n0 = S.ls[LS_NSAMP * C + c];
  const long long avail = S.ls[LS_AVAIL * C + c];
  const long long filled0 = S.ls[LS_FILLED * C + c];
  const int hops_done = S.is[IS_HOPS_DONE * C + c];
  const long long boundary = (long long)HOPN * (hops_done + 1) - 1;
  long long end = avail < boundary ? avail : boundary;
  if (!flush && avail <= boundary) end = n0;
  const int capm = (int)S.pcm_cap - 1;
  const int ia = (int)(avail - n0);
  const int ie = (int)(end - n0);
  int ifl = (int)(filled0 - n0);

  double mc_ptr = S.ds[DS_MC_PTR * C + c], mc_step = S.ds[DS_MC_STEP * C + c];
  if (ifl == 0 && ia > 0) {  // coarse-ring entry of sample n0
    const int16_t x = S.pcm[(size_t)(n0 & capm) * C + c];
    S.cring[(size_t)c * NF + (n0 & (NF - 1))] = (uint32_t)cis_index(mc_ptr) | ((uint32_t)(uint16_t)x << 16);
    ifl = 1;
  }
  if (ie <= 0) {
    S.ls[LS_FILLED * C + c] = n0 + ifl;
    return;
  }

  double m2_ptr = S.ds[DS_M2_PTR * C + c], m2_step = S.ds[DS_M2_STEP * C + c];
  double m2_freq = S.ds[DS_M2_FREQ * C + c];
  double so_ptr = S.ds[DS_SO_PTR * C + c], so_last = S.ds[DS_SO_LAST * C + c];
  const double so_step = S.ds[DS_SO_STEP * C + c];
  double agc_sum = S.ds[DS_AGC_SUM * C + c];
  double srx1 = S.ds[DS_SR_X1 * C + c], srx2 = S.ds[DS_SR_X2 * C + c];
  double sry1 = S.ds[DS_SR_Y1 * C + c], sry2 = S.ds[DS_SR_Y2 * C + c];
  double marg_sum = S.ds[DS_MARG_SUM * C + c], ms_sum = S.ds[DS_MS_SUM * C + c];
  double mse = S.ds[DS_MSE * C + c], diff_last = S.ds[DS_DIFF_LAST * C + c];
  long long ev = S.ls[LS_EVENTS * C + c];
  const int ms_off = S.is[IS_MS_OFF * C + c];
  long long softp = S.ls[LS_SOFT_P * C + c];
  long long ptn = S.ls[LS_PT_N * C + c];
  double *qre = S.fir + c, *qim = S.fir + (size_t)NT * C + c;  // partial sum j at [j * C]

  const double PT = G.ee * WTSIZE;  // IfHavePassedPoint(ee) (mskdemodulator.cpp:177-203)
  for (int i = 0; i < ie; ++i) {
    const long long n = n0 + i;
    const int16_t xs = S.pcm[(size_t)(n & capm) * C + c];
    const double agc_old = S.agc[(size_t)(n % AGC) * C + c];
    const double2 dsm_old = S.dsm[(size_t)((n + 1) % DSM) * C + c];
    const double d8_older = S.d8[(size_t)((n - G.d8_old + D8) % D8) * C + c];
    const double d8_newer = S.d8[(size_t)((n - G.d8_new + D8) % D8) * C + c];
    const double dval = ((double)xs) / 32768.0;
    const double2 cm = T.cis[cis_index(m2_ptr)];
    const double cv = cm.x * dval, cvi = cm.y * dval;  // mixer2.WTCISValue() * dval
    // matched filter (transposed form): FIRUpdateAndProcess reads the 2*SPS samples before the newest
    double s2r = qre[(size_t)(NT - 1) * C], s2i = qim[(size_t)(NT - 1) * C];
    for (int j = NT - 1; j >= 1; --j) qre[(size_t)j * C] = qre[(size_t)(j - 1) * C] + s_taps[j] * cv;
    qre[0] = 0.0 + s_taps[0] * cv;
    for (int j = NT - 1; j >= 1; --j) qim[(size_t)j * C] = qim[(size_t)(j - 1) * C] + s_taps[j] * cvi;
    qim[0] = 0.0 + s_taps[0] * cvi;
    const double dab = sqrt(s2r * s2r + s2i * s2i);
    {  // AGC::Update (DSP.cpp:371-380)
      agc_sum = agc_sum - agc_old;
      agc_sum = agc_sum + fabs(dab);
      S.agc[(size_t)(n % AGC) * C + c] = fabs(dab);
      double g = 1.414213562 / fmax(agc_sum / ((double)AGC), 0.000001);
      g = fmax(g, 0.000001);
      s2r *= g;
      s2i *= g;
    }
    const double ab = sqrt(s2r * s2r + s2i * s2i);
    if (ab > 2.84) {
      const double k = 2.84 / ab;
      s2r = k * s2r;
      s2i = k * s2i;
    }
    // pt_d = delayedsmpl.update_dont_touch(sig2) (DSP.h:468-473)
    S.dsm[(size_t)(n % DSM) * C + c] = make_double2(s2r, s2i);
    const double pdr = dsm_old.x, pdi = dsm_old.y;
    // st_eta = resonator(|pt_msk|), pt_msk = (sig2.re, pt_d.im)
    double st_eta;
    {
      const double sig = aero_hypot_w(s2r, pdi);
      double y = 0;
      y += srx2 * G.sr_b2;
      y += srx1 * 0.0;
      y += sig * G.sr_b0;
      y -= sry2 * G.sr_a2;
      y -= sry1 * G.sr_a1;
      srx2 = srx1;
      srx1 = sig;
      sry2 = sry1;
      sry1 = y;
      st_eta = y;
    }
    // delayt8.update(st_eta) (DSP.h:365-384)
    S.d8[(size_t)(n % D8) * C + c] = st_eta;
    const double d8v = (G.d8w * d8_newer + G.d8omw * d8_older);
    const double m1r = st_eta, m1i = -d8v;
    const double2 so = T.cis[cis_index(so_ptr)];
    const double ore = so.x * m1r - so.y * m1i, oim = so.x * m1i + so.y * m1r;
    const double ang = aero_atan2_bf(oim, ore, aero_g_cij);
    const double weighting = fabs(aero_tanh_bf(ang));
    {  // st_osc.AdvanceFractionOfWave (DSP.h:59-65), dcd false
      so_ptr += (-(1.0 - weighting) * ang * (0.05 / 360.0)) * WTSIZE;
      wt_wrap(so_ptr);
    }
    bool pend = false;
    {  // IfHavePassedPoint (DSP.cpp:222-238)
      double tl = so_last - PT, tw = so_ptr - PT;
      if (tl < 0.0) tl += WTSIZE;
      if (tw < 0.0) tw += WTSIZE;
      pend = (tl > 3.0 * WTSIZE / 4.0) && (tw < 1.0 * WTSIZE / 4.0);
    }
    // the coarse-ring entry of the next sample (mskdemodulator.cpp:284-287)
    nco_next(mc_ptr, mc_step);
    so_last = so_ptr;
    {
      double st = so_step;
      nco_next(so_ptr, st);
    }
    if (i + 1 < ia) {
      const long long n1 = n + 1;
      const int16_t x1 = S.pcm[(size_t)(n1 & capm) * C + c];
      S.cring[(size_t)c * NF + (n1 & (NF - 1))] = (uint32_t)cis_index(mc_ptr) | ((uint32_t)(uint16_t)x1 << 16);
      ifl = i + 2;
    }
    if (pend) {
      // carrier tracking (mskdemodulator.cpp:333-357)
      const double ct_xt = aero_tanh_bf(s2i) * s2r;
      const double ct_xt_d = aero_tanh_bf(pdr) * pdi;
      double ct_ec = ct_xt_d - ct_xt;
      if (ct_ec > M_PI) ct_ec = M_PI;
      if (ct_ec < -M_PI) ct_ec = -M_PI;
      if (ct_ec > M_PI_2) ct_ec = M_PI_2;
      if (ct_ec < -M_PI_2) ct_ec = -M_PI_2;
      const double carrier_aggression = 12.0 * 1.0;  // correctionfactor 1.0 (fb < 1200)
      {  // mixer2.IncresePhaseDeg (DSP.cpp:177-187)
        double phase_deg = carrier_aggression * 1.0 * ct_ec;
        phase_deg += div_cw(360.0 * m2_ptr, (double)WTSIZE);
        m2_ptr = set_phase_ptr(phase_deg);
      }
      {  // mixer2.IncreseFreqHz -> SetFreq(double) (DSP.cpp:163-175)
        double f = carrier_aggression * 0.01 * ct_ec;
        f += m2_freq;
        m2_freq = f;
        if (m2_freq < 0) m2_freq = 0;
        m2_step = (m2_freq) * ((double)WTSIZE) / FS;
      }
      // marg->UpdateSigned(ct_ec / 2.0) (DSP.cpp:419-427)
      double mval;
      {
        double *mb = S.marg + (size_t)c * MARG;
        const int p = (int)(ev % MARG);
        const double nv = ct_ec / 2.0;
        marg_sum = marg_sum - mb[p];
        marg_sum = marg_sum + (nv);
        mb[p] = nv;
        mval = marg_sum / ((double)MARG);
      }
      // dt.update(pt_msk) (DSP.h:463-467)
      double pr, pi;
      {
        double2 *db = S.dt + (size_t)c * DTL;
        db[ev % DTL] = make_double2(s2r, pdi);
        const double2 o = db[(ev + 1) % DTL];
        pr = o.x;
        pi = o.y;
      }
      {  // pt_msk *= cpx(cos(marg->Val), sin(marg->Val))
        double rs, rc;
        aero_sincos_bf(mval, rs, rc, aero_g_sincostab);
        const double rr = pr * rc - pi * rs, ri = pr * rs + pi * rc;
        pr = rr;
        pi = ri;
      }
      if (S.pt_cap) {
        if (ptn < S.pt_cap) S.pt[(size_t)c * S.pt_cap + ptn] = make_double2(pr, pi);
        ptn++;
      }
      {  // mse = msema->Update(tda^2 + tdb^2) (DSP.cpp:405-413)
        const double tda = (fabs((pr) * 0.75) - 1.0);
        const double tdb = (fabs((pi) * 0.75) - 1.0);
        const double v = (tda * tda) + (tdb * tdb);
        double *mb = S.ms + (size_t)c * MSK_MSEMA;
        const int p = (int)((ev + ms_off) % MSK_MSEMA);
        ms_sum = ms_sum - mb[p];
        ms_sum = ms_sum + fabs(v);
        mb[p] = fabs(v);
        mse = ms_sum / ((double)MSK_MSEMA);
      }
      {  // differential soft bits, imag first, real negated (mskdemodulator.cpp:381-401)
        const double imagin = diff_soft(diff_last, pi);
        int ibit = qround((imagin) * 127.0 + 128.0);
        if (ibit > 255) ibit = 255;
        if (ibit < 0) ibit = 0;
        double real = diff_soft(diff_last, pr);
        real = -real;
        int rbit = qround((real) * 127.0 + 128.0);
        if (rbit > 255) rbit = 255;
        if (rbit < 0) rbit = 0;
        uint8_t *soft = S.soft + (size_t)c * SOFT_RING;
        soft[softp & (SOFT_RING - 1)] = (uint8_t)ibit;
        soft[(softp + 1) & (SOFT_RING - 1)] = (uint8_t)rbit;
        softp += 2;
      }
      ev++;
    }
    nco_next(m2_ptr, m2_step);
  }

  double *ds = S.ds + c;
  long long *ls = S.ls + c;
  ls[LS_NSAMP * C] = n0 + ie;
  ls[LS_FILLED * C] = n0 + ifl;
  ls[LS_SOFT_P * C] = softp;
  ls[LS_EVENTS * C] = ev;
  if (S.pt_cap) ls[LS_PT_N * C] = ptn;
  ds[DS_M2_PTR * C] = m2_ptr;
  ds[DS_M2_STEP * C] = m2_step;
  ds[DS_M2_FREQ * C] = m2_freq;
  ds[DS_MC_PTR * C] = mc_ptr;
  ds[DS_MC_STEP * C] = mc_step;
  ds[DS_SO_PTR * C] = so_ptr;
  ds[DS_SO_LAST * C] = so_last;
  ds[DS_AGC_SUM * C] = agc_sum;
  ds[DS_SR_X1 * C] = srx1;
  ds[DS_SR_X2 * C] = srx2;
  ds[DS_SR_Y1 * C] = sry1;
  ds[DS_SR_Y2 * C] = sry2;
  ds[DS_MARG_SUM * C] = marg_sum;
  ds[DS_MS_SUM * C] = ms_sum;
  ds[DS_MSE * C] = mse;
  ds[DS_DIFF_LAST * C] = diff_last;
}

// The few-channel kernel (a receiver's handful of VFOs, C5): one channel per
// 16 lanes.  A channel's chain is latency-bound, one sample after another;
// with few channels the GPU has lanes to spare, so the matched filter's
// partial sums are spread over the channel's 16 lanes (B taps each,
// right-aligned: lane k holds taps NT - (16 - k) B .. NT - (15 - k) B - 1, so
// lane 15 holds tap NT - 1) and updated in parallel, the one value that
// crosses a lane boundary per sample (R_{j-1}(n-1) of the lane below) taken
// by a shuffle before the update.  Every lane of the group runs the rest of
// the chain on the same values (bit-identical results), so the filter
// output needs only one broadcast; the lanes' stores to the channel's rings
// carry identical values and coalesce.  Same arithmetic, same state layout
// as demod_msk_kernel / demod_mskg_kernel (the partial sums at [tap][C]), so
// a group can switch between the kernels from one launch to the next.
constexpr int MSKW_G = 16, MSKW_WG = 64;
static_assert(MAX_TAPS <= 20 * MSKW_G, "launch_demod_msk's largest instance holds every tap");
template <int B>
__global__ __launch_bounds__(MSKW_WG) void demod_mskw_kernel(DevState S, DevTables T, int nch, int flush) {
  const MskGen &G = S.mg;
  const int SPS = G.sps, NT = 2 * SPS, AGC = S.g.agc_len, DSM = S.g.dsm_len, D8 = S.g.d8_len, DTL = S.g.dt_len,
            MARG = S.g.marg_len;
  const double FS = G.fs;
  // atan2's and sincos's glibc tables in LDS: their row gathers sit on the
  // chain every sample / every event
  __shared__ double s_cij[241][7];
  __shared__ double s_sct[440];
  for (int q = threadIdx.x; q < 241 * 7; q += MSKW_WG) (&s_cij[0][0])[q] = (&aero_g_cij[0][0])[q];
  for (int q = threadIdx.x; q < 440; q += MSKW_WG) s_sct[q] = aero_g_sincostab[q];
  __syncthreads();
  const int lane = threadIdx.x, k = lane & (MSKW_G - 1), top = (lane & ~(MSKW_G - 1)) + MSKW_G - 1;
  const int c = blockIdx.x * (MSKW_WG / MSKW_G) + lane / MSKW_G;
  if (c >= nch) return;  // the whole 16-lane group
  const int j0 = NT - (MSKW_G - k) * B;  // this lane's first tap (negative: slots without a tap)
  const int C = S.C;
  const int HOPN = MSK_HOP, NF = MSK_NFFT;

  const long long n0 = S.ls[LS_NSAMP * C + c];
  const long long avail = S.ls[LS_AVAIL * C + c];
  const long long filled0 = S.ls[LS_FILLED * C + c];
  const int hops_done = S.is[IS_HOPS_DONE * C + c];
  const long long boundary = (long long)HOPN * (hops_done + 1) - 1;
  long long end = avail < boundary ? avail : boundary;
  if (!flush && avail <= boundary) end = n0;
  const int capm = (int)S.pcm_cap - 1;
  const int ia = (int)(avail - n0);
  const int ie = (int)(end - n0);
  int ifl = (int)(filled0 - n0);

  double mc_ptr = S.ds[DS_MC_PTR * C + c], mc_step = S.ds[DS_MC_STEP * C + c];
  if (ifl == 0 && ia > 0) {  // coarse-ring entry of sample n0
    const int16_t x = S.pcm[(size_t)(n0 & capm) * C + c];
    S.cring[(size_t)c * NF + (n0 & (NF - 1))] = (uint32_t)cis_index(mc_ptr) | ((uint32_t)(uint16_t)x << 16);
    ifl = 1;
  }
  if (ie <= 0) {
    S.ls[LS_FILLED * C + c] = n0 + ifl;
    return;
  }

  double m2_ptr = S.ds[DS_M2_PTR * C + c], m2_step = S.ds[DS_M2_STEP * C + c];
  double m2_freq = S.ds[DS_M2_FREQ * C + c];
  double so_ptr = S.ds[DS_SO_PTR * C + c], so_last = S.ds[DS_SO_LAST * C + c];
  const double so_step = S.ds[DS_SO_STEP * C + c];
  double agc_sum = S.ds[DS_AGC_SUM * C + c];
  double srx1 = S.ds[DS_SR_X1 * C + c], srx2 = S.ds[DS_SR_X2 * C + c];
  double sry1 = S.ds[DS_SR_Y1 * C + c], sry2 = S.ds[DS_SR_Y2 * C + c];
  double marg_sum = S.ds[DS_MARG_SUM * C + c], ms_sum = S.ds[DS_MS_SUM * C + c];
  double mse = S.ds[DS_MSE * C + c], diff_last = S.ds[DS_DIFF_LAST * C + c];
  long long ev = S.ls[LS_EVENTS * C + c];
  const int ms_off = S.is[IS_MS_OFF * C + c];
  long long softp = S.ls[LS_SOFT_P * C + c];
  long long ptn = S.ls[LS_PT_N * C + c];
  double qre[B], qim[B], tp[B];
#pragma unroll
  for (int jj = 0; jj < B; ++jj) {
    const int j = j0 + jj;
    tp[jj] = j >= 0 ? T.taps[j] : 0.0;
    qre[jj] = j >= 0 ? S.fir[(size_t)j * C + c] : 0.0;
    qim[jj] = j >= 0 ? S.fir[(size_t)(NT + j) * C + c] : 0.0;
  }

  const double PT = G.ee * WTSIZE;  // IfHavePassedPoint(ee) (mskdemodulator.cpp:177-203)
  // a sample's PCM word and ring slots are loaded one sample ahead (their
  // HBM / L2 round trips would otherwise open every sample): none is a slot
  // the sample before writes (AGC >= 2, DSM > 2, delayt8 ages >= 2, host-checked)
  auto ld_pcm = [&](long long m) { return S.pcm[(size_t)(m & capm) * C + c]; };
  auto ld_agc = [&](long long m) { return S.agc[(size_t)(m % AGC) * C + c]; };
  auto ld_dsm = [&](long long m) { return S.dsm[(size_t)((m + 1) % DSM) * C + c]; };
  auto ld_d8 = [&](long long m, int age) { return S.d8[(size_t)((m - age + D8) % D8) * C + c]; };
  int16_t xs_nx = ld_pcm(n0);
  double agc_nx = ld_agc(n0), d8o_nx = ld_d8(n0, G.d8_old), d8n_nx = ld_d8(n0, G.d8_new);
  double2 dsm_nx = ld_dsm(n0);
  for (int i = 0; i < ie; ++i) {
    const long long n = n0 + i;
    const int16_t xs = xs_nx;
    const double agc_old = agc_nx;
    const double2 dsm_old = dsm_nx;
    const double d8_older = d8o_nx;
    const double d8_newer = d8n_nx;
    xs_nx = ld_pcm(n + 1);  // past the pushed samples: unused
    agc_nx = ld_agc(n + 1);
    dsm_nx = ld_dsm(n + 1);
    d8o_nx = ld_d8(n + 1, G.d8_old);
    d8n_nx = ld_d8(n + 1, G.d8_new);
    const double dval = ((double)xs) / 32768.0;
    const double2 cm = T.cis[cis_index(m2_ptr)];
    const double cv = cm.x * dval, cvi = cm.y * dval;  // mixer2.WTCISValue() * dval
    // matched filter (transposed form): the output is R_{NT-1}(n-1), lane
    // 15's last slot; each lane's lowest tap takes R_{j0-1}(n-1) from the
    // lane below, both read before any update
    double s2r = __shfl(qre[B - 1], top, 64), s2i = __shfl(qim[B - 1], top, 64);
    const double bre = __shfl_up(qre[B - 1], 1, MSKW_G), bim = __shfl_up(qim[B - 1], 1, MSKW_G);
#pragma unroll
    for (int jj = B - 1; jj >= 1; --jj) {
      const int j = j0 + jj;
      if (j > 0) {
        qre[jj] = qre[jj - 1] + tp[jj] * cv;
        qim[jj] = qim[jj - 1] + tp[jj] * cvi;
      } else if (j == 0) {
        qre[jj] = 0.0 + tp[jj] * cv;
        qim[jj] = 0.0 + tp[jj] * cvi;
      }
    }
    if (j0 > 0) {
      qre[0] = bre + tp[0] * cv;
      qim[0] = bim + tp[0] * cvi;
    } else if (j0 == 0) {
      qre[0] = 0.0 + tp[0] * cv;
      qim[0] = 0.0 + tp[0] * cvi;
    }
    const double dab = sqrt(s2r * s2r + s2i * s2i);
    {  // AGC::Update (DSP.cpp:371-380)
      agc_sum = agc_sum - agc_old;
      agc_sum = agc_sum + fabs(dab);
      S.agc[(size_t)(n % AGC) * C + c] = fabs(dab);
      double g = 1.414213562 / fmax(agc_sum / ((double)AGC), 0.000001);
      g = fmax(g, 0.000001);
      s2r *= g;
      s2i *= g;
    }
    const double ab = sqrt(s2r * s2r + s2i * s2i);
    if (ab > 2.84) {
      const double kk = 2.84 / ab;
      s2r = kk * s2r;
      s2i = kk * s2i;
    }
    // pt_d = delayedsmpl.update_dont_touch(sig2) (DSP.h:468-473)
    S.dsm[(size_t)(n % DSM) * C + c] = make_double2(s2r, s2i);
    const double pdr = dsm_old.x, pdi = dsm_old.y;
    // st_eta = resonator(|pt_msk|), pt_msk = (sig2.re, pt_d.im)
    double st_eta;
    {
      const double sig = aero_hypot_w(s2r, pdi);
      double y = 0;
      y += srx2 * G.sr_b2;
      y += srx1 * 0.0;
      y += sig * G.sr_b0;
      y -= sry2 * G.sr_a2;
      y -= sry1 * G.sr_a1;
      srx2 = srx1;
      srx1 = sig;
      sry2 = sry1;
      sry1 = y;
      st_eta = y;
    }
    // delayt8.update(st_eta) (DSP.h:365-384)
    S.d8[(size_t)(n % D8) * C + c] = st_eta;
    const double d8v = (G.d8w * d8_newer + G.d8omw * d8_older);
    const double m1r = st_eta, m1i = -d8v;
    const double2 so = T.cis[cis_index(so_ptr)];
    const double ore = so.x * m1r - so.y * m1i, oim = so.x * m1i + so.y * m1r;
    const double ang = aero_atan2_bf(oim, ore, s_cij);
    const double weighting = fabs(aero_tanh_bf(ang));
    {  // st_osc.AdvanceFractionOfWave (DSP.h:59-65), dcd false
      so_ptr += (-(1.0 - weighting) * ang * (0.05 / 360.0)) * WTSIZE;
      wt_wrap(so_ptr);
    }
    bool pend;
    {  // IfHavePassedPoint (DSP.cpp:222-238)
      double tl = so_last - PT, tw = so_ptr - PT;
      if (tl < 0.0) tl += WTSIZE;
      if (tw < 0.0) tw += WTSIZE;
      pend = (tl > 3.0 * WTSIZE / 4.0) && (tw < 1.0 * WTSIZE / 4.0);
    }
    // the coarse-ring entry of the next sample (mskdemodulator.cpp:284-287)
    nco_next(mc_ptr, mc_step);
    so_last = so_ptr;
    {
      double st = so_step;
      nco_next(so_ptr, st);
    }
    if (i + 1 < ia) {
      const long long n1 = n + 1;
      const int16_t x1 = S.pcm[(size_t)(n1 & capm) * C + c];
      S.cring[(size_t)c * NF + (n1 & (NF - 1))] = (uint32_t)cis_index(mc_ptr) | ((uint32_t)(uint16_t)x1 << 16);
      ifl = i + 2;
    }
    if (pend) {
      // carrier tracking (mskdemodulator.cpp:333-357)
      const double ct_xt = aero_tanh_bf(s2i) * s2r;
      const double ct_xt_d = aero_tanh_bf(pdr) * pdi;
      double ct_ec = ct_xt_d - ct_xt;
      if (ct_ec > M_PI) ct_ec = M_PI;
      if (ct_ec < -M_PI) ct_ec = -M_PI;
      if (ct_ec > M_PI_2) ct_ec = M_PI_2;
      if (ct_ec < -M_PI_2) ct_ec = -M_PI_2;
      const double carrier_aggression = 12.0 * 1.0;  // correctionfactor 1.0 (fb < 1200)
      {  // mixer2.IncresePhaseDeg (DSP.cpp:177-187)
        double phase_deg = carrier_aggression * 1.0 * ct_ec;
        phase_deg += div_cw(360.0 * m2_ptr, (double)WTSIZE);
        m2_ptr = set_phase_ptr(phase_deg);
      }
      {  // mixer2.IncreseFreqHz -> SetFreq(double) (DSP.cpp:163-175)
        double f = carrier_aggression * 0.01 * ct_ec;
        f += m2_freq;
        m2_freq = f;
        if (m2_freq < 0) m2_freq = 0;
        m2_step = (m2_freq) * ((double)WTSIZE) / FS;
      }
      // marg->UpdateSigned(ct_ec / 2.0) (DSP.cpp:419-427)
      double mval;
      {
        double *mb = S.marg + (size_t)c * MARG;
        const int p = (int)(ev % MARG);
        const double nv = ct_ec / 2.0;
        marg_sum = marg_sum - mb[p];
        marg_sum = marg_sum + (nv);
        mb[p] = nv;
        mval = marg_sum / ((double)MARG);
      }
      // dt.update(pt_msk) (DSP.h:463-467)
      double pr, pi;
      {
        double2 *db = S.dt + (size_t)c * DTL;
        db[ev % DTL] = make_double2(s2r, pdi);
        const double2 o = db[(ev + 1) % DTL];
        pr = o.x;
        pi = o.y;
      }
      {  // pt_msk *= cpx(cos(marg->Val), sin(marg->Val))
        double rs, rc;
        aero_sincos_bf(mval, rs, rc, s_sct);
        const double rr = pr * rc - pi * rs, ri = pr * rs + pi * rc;
        pr = rr;
        pi = ri;
      }
      if (S.pt_cap) {
        if (ptn < S.pt_cap) S.pt[(size_t)c * S.pt_cap + ptn] = make_double2(pr, pi);
        ptn++;
      }
      {  // mse = msema->Update(tda^2 + tdb^2) (DSP.cpp:405-413)
        const double tda = (fabs((pr) * 0.75) - 1.0);
        const double tdb = (fabs((pi) * 0.75) - 1.0);
        const double v = (tda * tda) + (tdb * tdb);
        double *mb = S.ms + (size_t)c * MSK_MSEMA;
        const int p = (int)((ev + ms_off) % MSK_MSEMA);
        ms_sum = ms_sum - mb[p];
        ms_sum = ms_sum + fabs(v);
        mb[p] = fabs(v);
        mse = ms_sum / ((double)MSK_MSEMA);
      }
      {  // differential soft bits, imag first, real negated (mskdemodulator.cpp:381-401)
        const double imagin = diff_soft(diff_last, pi);
        int ibit = qround((imagin) * 127.0 + 128.0);
        if (ibit > 255) ibit = 255;
        if (ibit < 0) ibit = 0;
        double real = diff_soft(diff_last, pr);
        real = -real;
        int rbit = qround((real) * 127.0 + 128.0);
        if (rbit > 255) rbit = 255;
        if (rbit < 0) rbit = 0;
        uint8_t *soft = S.soft + (size_t)c * SOFT_RING;
        soft[softp & (SOFT_RING - 1)] = (uint8_t)ibit;
        soft[(softp + 1) & (SOFT_RING - 1)] = (uint8_t)rbit;
        softp += 2;
      }
      ev++;
    }
    nco_next(m2_ptr, m2_step);
  }

#pragma unroll
  for (int jj = 0; jj < B; ++jj) {
    const int j = j0 + jj;
    if (j >= 0) {
      S.fir[(size_t)j * C + c] = qre[jj];
      S.fir[(size_t)(NT + j) * C + c] = qim[jj];
    }
  }
  double *ds = S.ds + c;
  long long *ls = S.ls + c;
  ls[LS_NSAMP * C] = n0 + ie;
  ls[LS_FILLED * C] = n0 + ifl;
  ls[LS_SOFT_P * C] = softp;
  ls[LS_EVENTS * C] = ev;
  if (S.pt_cap) ls[LS_PT_N * C] = ptn;
  ds[DS_M2_PTR * C] = m2_ptr;
  ds[DS_M2_STEP * C] = m2_step;
  ds[DS_M2_FREQ * C] = m2_freq;
  ds[DS_MC_PTR * C] = mc_ptr;
  ds[DS_MC_STEP * C] = mc_step;
  ds[DS_SO_PTR * C] = so_ptr;
  ds[DS_SO_LAST * C] = so_last;
  ds[DS_AGC_SUM * C] = agc_sum;
  ds[DS_SR_X1 * C] = srx1;
  ds[DS_SR_X2 * C] = srx2;
  ds[DS_SR_Y1 * C] = sry1;
  ds[DS_SR_Y2 * C] = sry2;
  ds[DS_MARG_SUM * C] = marg_sum;
  ds[DS_MS_SUM * C] = ms_sum;
  ds[DS_MSE * C] = mse;
  ds[DS_DIFF_LAST * C] = diff_last;
}

template <int M>
static void launch_msk_mode(hipStream_t st, const DevState &S, const DevTables &T, int nch, int flush) {
  constexpr int WG = MskK<M>::WG;
  hipLaunchKernelGGL(demod_msk_kernel<M>, dim3((nch + WG - 1) / WG), dim3(WG), 0, st, S, T, nch, flush);
}

// the few-channel kernel for nch <= wide_max (engine.hip: up to
// MSKW_MAX_DEFAULT channels unless AERO_MSK_WIDE says otherwise)
template <int B>
static void launch_mskw(hipStream_t st, const DevState &S, const DevTables &T, int nch, int flush) {
  constexpr int CPB = MSKW_WG / MSKW_G;
  hipLaunchKernelGGL(demod_mskw_kernel<B>, dim3((nch + CPB - 1) / CPB), dim3(MSKW_WG), 0, st, S, T, nch, flush);
}

void launch_demod_msk(hipStream_t st, int mode, const DevState &S, const DevTables &T, int nch, int flush,
                      bool wide) {
  if (wide) {
    const int nt = 2 * S.mg.sps, b = (nt + MSKW_G - 1) / MSKW_G;  // taps per lane
    if (b <= 3) return launch_mskw<3>(st, S, T, nch, flush);
    if (b <= 5) return launch_mskw<5>(st, S, T, nch, flush);
    if (b <= 10) return launch_mskw<10>(st, S, T, nch, flush);
    return launch_mskw<20>(st, S, T, nch, flush);  // MAX_TAPS / 16
  }
  switch (mode) {
    case MODE_MSK600: return launch_msk_mode<MODE_MSK600>(st, S, T, nch, flush);
    case MODE_MSK1200: return launch_msk_mode<MODE_MSK1200>(st, S, T, nch, flush);
    case MODE_MSK600_24K: return launch_msk_mode<MODE_MSK600_24K>(st, S, T, nch, flush);
    case MODE_MSK600_48K: return launch_msk_mode<MODE_MSK600_48K>(st, S, T, nch, flush);
    case MODE_MSK1200_12K: return launch_msk_mode<MODE_MSK1200_12K>(st, S, T, nch, flush);
    case MODE_MSK1200_48K: return launch_msk_mode<MODE_MSK1200_48K>(st, S, T, nch, flush);
    default:  // MODE_MSKG600, MODE_MSKG1200
      hipLaunchKernelGGL(demod_mskg_kernel, dim3((nch + MSKG_WG - 1) / MSKG_WG), dim3(MSKG_WG), 0, st, S, T, nch, flush);
  }
}

void upload_msk_constants(const double *d8w) {
  hipMemcpyToSymbol(HIP_SYMBOL(c_msk_d8w), d8w, sizeof(double) * 2);
}

}  // namespace aero
