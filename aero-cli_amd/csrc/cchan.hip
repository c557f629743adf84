/*
 * cchan.hip — the C channel: 8400-bps OQPSK (OqpskDemodulator at fb = 8400)
 * and AeroL::DecodeC on gfx950.
 *
 *  prefilter_dn_kernel  the per-message prefilter of OqpskDemodulator::writeData
 *  prefilter_blk_kernel (decode/oqpskdemodulator.cpp:292-324): down-mix by
 *                       mixer_fir_pre, JFastFir (RRC 0.6, 2049 taps, 4096-point
 *                       overlap-add blocks of 2048, decode/jfft.cpp:324-367,
 *                       445-495), up-mix by the conjugate from the phase saved
 *                       at the message start.  The down-mix's phase pointer on
 *                       one lane per channel, the block transforms by one
 *                       workgroup per channel in registers (fft_dit.h), the
 *                       up-mix in the demod as it reads each sample.
 *  demod_c_kernel     : the per-sample loop at fb = 8400 (:331-553): no RRC FIR
 *                       (the prefilter is the matched filter), its own timer
 *                       delays / resonator / ee, the carrier loop with faster
 *                       phase agility (:463-472), mixer2's frequency summed over
 *                       the message and mixer_fir_pre retuned to the mean at
 *                       its end (:555-557).  One lane per channel.
 *  frame_c_kernel     : AeroL::DecodeC's framing (decode/aerol.cpp:2145-2240):
 *                       the two dual-preamble detectors (52 bits, tolerance 6,
 *                       :782-877) on alternating soft bits, 16 blocks of 4 x 64
 *                       deinterleaved (deinterleave_ba(block, 4), :594-613) and
 *                       depunctured (PuncturedCode, :2417-2432) as they fill.
 *  viterbi_c_kernel   : Decode_Continuous of a 5460-symbol frame
 *                       (jconvolutionalcodec.cpp:146-198; the soft Viterbi of
 *                       viterbi_dev.h), the 2714-bit payload through dl2 and
 *                       the scrambler, the three 12-byte SUs and their CRCs and
 *                       the 300 voice bytes (:2249-2392) into the job record.
 *
 * Bit-exactness rules as in demod_oqpsk.hip: -ffp-contract=off, the
 * reference's operation order, GCC complex products, aero_math.h for libm;
 * the short exact divisions of aero_math.h where demod_oqpsk.hip uses them.
 */
#include <hip/hip_runtime.h>

#include <climits>

#include "aero_math.h"
#include "engine_common.h"
#include "fft_dit.h"
#include "viterbi_dev.h"

namespace aero {

struct CPreJob {  // one message of one channel: samples [s, e)
  int c, pad;
  long long s, e;
};

namespace {

__constant__ DelayDesc cc_dly[4];  // delays(1), delayt41(T/4), delayt42(T/4), delayt8(T/8), T = 48000 / 4200

__device__ __forceinline__ int c_cis_index(double WTptr) {  // WaveTable::WTCISValue (DSP.cpp:81-88)
  int tint = (int)WTptr;
  if (tint >= WTSIZE) tint = 0;
  if (tint < 0) tint = WTSIZE - 1;
  return tint;
}
__device__ __forceinline__ void c_nco_next(double &ptr, double &step) {  // WTnextFrame (DSP.cpp:71-79)
  if (step < 0) step = 0;
  ptr += step;
  wt_wrap_int(ptr);
}
__device__ __forceinline__ void c_set_freq(double &freq, double &step, double f) {  // SetFreq(double) (DSP.cpp:163-168)
  freq = f;
  if (freq < 0) freq = 0;
  step = div_c((freq) * ((double)WTSIZE), 48000.0);
}
// Delay<double>::update (DSP.h:365-384) as a shift register (h[0] newest)
// whose weights depend on the write pointer p (T/8 at 8400 bps does)
template <int N, int AGE_OLD, int AGE_NEW>
__device__ __forceinline__ double c_delay(double (&h)[N], int &p, const DelayDesc &d, double sig) {
#pragma unroll
  for (int i = N - 1; i > 0; --i) h[i] = h[i - 1];
  h[0] = sig;
  const double w = d.w[p], omw = d.omw[p];
  p = p + 1 == d.size ? 0 : p + 1;
  return (w * h[AGE_NEW] + omw * h[AGE_OLD]);
}
__device__ __forceinline__ double c_iir3(double &x1, double &x2, double &y1, double &y2, const double (&b)[3],
                                         const double (&a)[3], double sig) {  // IIR::update (DSP.cpp:635-685)
  double y = 0;
  y += x2 * b[2];
  y += x1 * b[1];
  y += sig * b[0];
  y -= y2 * a[2];
  y -= y1 * a[1];
  x2 = x1;
  x1 = sig;
  y2 = y1;
  y1 = y;
  return y;
}
__device__ __forceinline__ int c_qround(double d) {  // qRound (Qt 5.9 qglobal.h:525)
  return d >= 0.0 ? int(d + 0.5) : int(d - double(int(d - 1)) + 0.5) + int(d - 1);
}

}  // namespace

// The per-message prefilter (decode/oqpskdemodulator.cpp:292-324) in three
// parts, each in the layout its work wants:
//  1. prefilter_dn_kernel, one lane per channel: the down-mix's phase pointer
//     (a serial recurrence) over the message, with the PCM rows read
//     coalesced; each sample's table index and pcm word go to the channel's
//     run of `cin`.  It also restores the saved phase for the up-mix
//     (GetPhaseDeg / SetPhaseDeg, DSP.cpp:177-200) into DS_FP_PTR.
//  2. prefilter_blk_kernel, one 256-thread workgroup per channel: JFastFir
//     (jfft.cpp:445-495) block by block, each 4096-point transform pair in
//     registers (fft_dit.h); the outputs into the channel's run of `cout`.
//  3. the up-mix by WTCISValue_conj from the restored phase, in
//     demod_c_kernel as it reads each sample (the pointer advances with the
//     step the message started with; the demod retunes it only at the end).
__global__ __launch_bounds__(64) void prefilter_dn_kernel(DevState S, const CPreJob *jobs, int njobs) {
  const int q = blockIdx.x * 64 + threadIdx.x;
  if (q >= njobs) return;
  const CPreJob J = jobs[q];
  const int c = J.c, C = S.C;
  const long long capm = S.pcm_cap - 1;
  double fp_step = S.ds[DS_FP_STEP * C + c];
  double dn_ptr = S.ds[DS_FP_PTR * C + c];
  {  // savedphase = GetPhaseDeg() (DSP.cpp:200), SetPhaseDeg(savedphase) (:177-187)
    S.ds[DS_FP_PTR * C + c] = set_phase_ptr(div_cw(360.0 * dn_ptr, (double)WTSIZE));
  }
  uint32_t *cin = S.cin + (size_t)c * C_IN_RING;
  long long n = J.s;
  // eight PCM rows in flight ahead of the chain
  for (; n + 8 <= J.e; n += 8) {
    int16_t x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = S.pcm[(size_t)((n + k) & capm) * C + c];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      cin[(n + k) & (C_IN_RING - 1)] = (uint32_t)c_cis_index(dn_ptr) | ((uint32_t)(uint16_t)x[k] << 16);
      c_nco_next(dn_ptr, fp_step);
    }
  }
  for (; n < J.e; ++n) {
    const int16_t x = S.pcm[(size_t)(n & capm) * C + c];
    cin[n & (C_IN_RING - 1)] = (uint32_t)c_cis_index(dn_ptr) | ((uint32_t)(uint16_t)x << 16);
    c_nco_next(dn_ptr, fp_step);
  }
  S.ls[LS_PRE_END * C + c] = J.e;
  S.ls[LS_MSG_START * C + c] = J.s;
}

// JFastFir::update over one message [s, e): sample n's output is the value
// the block transform at 2048 * floor(n / 2048) left in sigspace (zero
// before the first); that transform runs before sample n = 2048 B > 0 is
// pushed, on the down-mixed inputs of samples [n - 2048, n) and zeros:
// y = IFFT(FFT(block) * K) / 4096; outputs y[k] + remainder[k] (k < 2048);
// the remainder becomes y[2048 + k].  Outputs of samples past the message
// wait in `csig` for the next one.
__global__ __launch_bounds__(256, 2) void prefilter_blk_kernel(DevState S, DevTables T, const CPreJob *jobs) {
  constexpr int L = 12, PADDED = C_FIR_N + C_FIR_N / 16;
  static_assert(C_FIR_N == 1 << L && C_FIR_SNZ == C_FIR_N / 2, "4096-point blocks of 2048 inputs");
  __shared__ double lds[PADDED];
  __shared__ double2 s_tw[TwLds<L>::LEN];
  const CPreJob J = jobs[blockIdx.x];
  const int c = J.c, t = threadIdx.x;
  load_tw_lds<L>(s_tw, T.tw4, t, 256);
  const uint32_t *cin = S.cin + (size_t)c * C_IN_RING;
  double2 *out = S.cout + (size_t)c * C_OUT_RING;
  double2 *pend = S.csig + (size_t)c * C_FIR_SNZ;
  double2 *rem = S.crem + (size_t)c * (C_FIR_N - C_FIR_SNZ);
  const long long s = J.s, e = J.e;
  if (s % C_FIR_SNZ != 0 || s == 0) {  // the samples before the message's first transform
    const long long be = (s / C_FIR_SNZ + 1) * C_FIR_SNZ < e ? (s / C_FIR_SNZ + 1) * C_FIR_SNZ : e;
    for (long long n = s + t; n < be; n += 256) out[n & (C_OUT_RING - 1)] = pend[n & (C_FIR_SNZ - 1)];
  }
  __syncthreads();
  for (long long p = (s + C_FIR_SNZ - 1) / C_FIR_SNZ * C_FIR_SNZ; p < e; p += C_FIR_SNZ) {
    if (p == 0) continue;
    double2 x[16];
    // (t laundered per loop: the compiler would otherwise keep every loop's
    // per-value addresses live across the transforms, which spills)
    const int t0 = fresh(t);
#pragma unroll
    for (int i = 0; i < 16; ++i) {  // inputs [p - 2048, p) (mixer_fir_pre.WTCISValue() * dval), then zeros
      const int q = bitrev<L>(epos<L, 0>(t0, i));
      if (q < C_FIR_SNZ) {
        const uint32_t w = cin[(p - C_FIR_SNZ + q) & (C_IN_RING - 1)];
        const double dval = ((double)(int16_t)(w >> 16)) / 32768.0;
        const double2 cs = T.cis[w & 0xFFFF];
        x[i] = make_double2(cs.x * dval, cs.y * dval);
      } else {
        x[i] = make_double2(0.0, 0.0);
      }
    }
    fft_dit<L, false>(x, t, lds, T.tw4, s_tw);
    const int t1 = fresh(t);
#pragma unroll
    for (int i = 0; i < 16; ++i) {  // *psigspace *= *pkernel
      const double2 k = T.cker[epos<L, 2>(t1, i)];
      x[i] = make_double2(x[i].x * k.x - x[i].y * k.y, x[i].x * k.y + x[i].y * k.x);
    }
    exchange<L, 2, 0, true>(x, t, lds);
    fft_dit<L, true>(x, t, lds, T.twi4, s_tw);
    // positions t + 256 i: registers 0-7 hold the outputs, 8-15 the next
    // remainder, so a thread reads and replaces only its own remainder slots
    const bool last = p + C_FIR_SNZ >= e;
    const int t2 = fresh(t);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int k = epos<L, 2>(t2, i);
      const double2 r = rem[k];
      const double2 y = make_double2(x[i].x * (1.0 / ((double)C_FIR_N)) + r.x, x[i].y * (1.0 / ((double)C_FIR_N)) + r.y);
      if (p + k < e) out[(p + k) & (C_OUT_RING - 1)] = y;
      if (last) pend[k] = y;
      rem[k] = make_double2(x[i + 8].x * (1.0 / ((double)C_FIR_N)), x[i + 8].y * (1.0 / ((double)C_FIR_N)));
    }
    __syncthreads();
  }
}

// OqpskDemodulator::writeData at fb = 8400 (decode/oqpskdemodulator.cpp:331-557)
template <bool TRACE>
__global__ __launch_bounds__(64) void demod_c_kernel(DevState S, DevTables T, int nch) {
  __shared__ double cij[241][7];
  __shared__ double sct[440];
  __shared__ DelayDesc sdly[4];  // the timer delays' pointer-indexed weights: an LDS read, not an L2 round trip
  for (int q = threadIdx.x; q < 241 * 7; q += 64) (&cij[0][0])[q] = (&aero_g_cij[0][0])[q];
  for (int q = threadIdx.x; q < 440; q += 64) sct[q] = aero_g_sincostab[q];
  if (threadIdx.x < 4) sdly[threadIdx.x] = cc_dly[threadIdx.x];
  __syncthreads();
  const int c = blockIdx.x * 64 + threadIdx.x;
  if (c >= nch) return;
  const int C = S.C;
  const long long n0 = S.ls[LS_NSAMP * C + c];
  const long long avail = S.ls[LS_AVAIL * C + c];
  const long long filled0 = S.ls[LS_FILLED * C + c];
  const long long pre_end = S.ls[LS_PRE_END * C + c];
  const int hops_done = S.is[IS_HOPS_DONE * C + c];
  const long long boundary = (long long)HOP * (hops_done + 1) - 1;
  const long long end = pre_end < boundary ? pre_end : boundary;
  const int capm = (int)S.pcm_cap - 1;
  const int ia = (int)(avail - n0);
  const int ie = (int)(end - n0);
  int ifl = (int)(filled0 - n0);
  double mc_ptr = S.ds[DS_MC_PTR * C + c], mc_step = S.ds[DS_MC_STEP * C + c];
  if (ifl == 0 && ia > 0) {  // coarse-ring entry of sample n0 (:351-356)
    const int16_t x = S.pcm[(size_t)(n0 & capm) * C + c];
    S.cring[(size_t)c * NFFT + (n0 & (NFFT - 1))] = (uint32_t)c_cis_index(mc_ptr) | ((uint32_t)(uint16_t)x << 16);
    ifl = 1;
  }
  if (ie <= 0) {
    S.ls[LS_FILLED * C + c] = n0 + ifl;
    return;
  }
  // the symbol-timer resonator at 8400 bps, the second ("10Hz bw") design (:196-214)
  const double sr_b[3] = {0.0012845857864470789, 0, -0.0012845857864470789};
  const double sr_a[3] = {1, -0.90681461999279889, 0.99743082842710584};
  const double ct_b[3] = {0.0010275610653672064, 0.0020551221307344128, 0.0010275610653672064};
  const double ct_a[3] = {1, -1.9207386815577139, 0.92509247310306331};
  const double SO_F = 8400.0;
  double m2_ptr = S.ds[DS_M2_PTR * C + c], m2_step = S.ds[DS_M2_STEP * C + c], m2_freq = S.ds[DS_M2_FREQ * C + c];
  double so_ptr = S.ds[DS_SO_PTR * C + c], so_last = S.ds[DS_SO_LAST * C + c];
  double so_step = S.ds[DS_SO_STEP * C + c], so_freq = S.ds[DS_SO_FREQ * C + c];
  double agc_sum = S.ds[DS_AGC_SUM * C + c], m2_fsum = S.ds[DS_M2_FSUM * C + c];
  double d1[2], d41[4], d42[4], d8[3];
#pragma unroll
  for (int q = 0; q < 2; ++q) d1[q] = S.ds[(DS_D1_0 + q) * C + c];
#pragma unroll
  for (int q = 0; q < 4; ++q) d41[q] = S.ds[(DS_D41_0 + q) * C + c];
#pragma unroll
  for (int q = 0; q < 4; ++q) d42[q] = S.ds[(DS_D42_0 + q) * C + c];
#pragma unroll
  for (int q = 0; q < 3; ++q) d8[q] = S.ds[(DS_D8_0 + q) * C + c];
  int p1 = S.is[IS_D1_P * C + c], p41 = S.is[IS_D41_P * C + c], p42 = S.is[IS_D42_P * C + c],
      p8 = S.is[IS_D8_P * C + c];
  double srx1 = S.ds[DS_SR_X1 * C + c], srx2 = S.ds[DS_SR_X2 * C + c];
  double sry1 = S.ds[DS_SR_Y1 * C + c], sry2 = S.ds[DS_SR_Y2 * C + c];
  double s2l_re = S.ds[DS_S2L_RE * C + c], s2l_im = S.ds[DS_S2L_IM * C + c];
  double ctx1 = S.ds[DS_CT_X1 * C + c], ctx2 = S.ds[DS_CT_X2 * C + c];
  double cty1 = S.ds[DS_CT_Y1 * C + c], cty2 = S.ds[DS_CT_Y2 * C + c];
  double marg_sum = S.ds[DS_MARG_SUM * C + c], pm_sum = S.ds[DS_PM_SUM * C + c];
  double ms_sum = S.ds[DS_MS_SUM * C + c], mse = S.ds[DS_MSE * C + c];
  double ptd_re = S.ds[DS_PTD_RE * C + c], ptd_im = S.ds[DS_PTD_IM * C + c];
  int agc_ptr = S.is[IS_AGC_PTR * C + c];
  int yui = S.is[IS_YUI * C + c], s2l_init = S.is[IS_S2L_INIT * C + c];
  int marg_p = S.is[IS_MARG_P * C + c], dt_p = S.is[IS_DT_P * C + c];
  int pm_p = S.is[IS_PM_P * C + c], ms_p = S.is[IS_MS_P * C + c];
  long long softp = S.ls[LS_SOFT_P * C + c];
  long long ptn = TRACE ? S.ls[LS_PT_N * C + c] : 0;
  double *marg = S.marg + (size_t)c * MARG_LEN;
  double2 *dtb = S.dt + (size_t)c * DT_LEN;
  double2 *pmsb = reinterpret_cast<double2 *>(S.pm) + (size_t)c * MSE_LEN;
  uint8_t *soft = S.soft + (size_t)c * SOFT_RING;
  const double2 *cout = S.cout + (size_t)c * C_OUT_RING;
  double up_ptr = S.ds[DS_FP_PTR * C + c], fp_step = S.ds[DS_FP_STEP * C + c];
  const double PT = 0.65 * WTSIZE;  // IfHavePassedPoint(ee), ee = 0.65 at 8400 (:213)
  // Event-aligned (as demod_oqpsk.hip): each lane runs its samples up to
  // its next carrier event, then the carrier step runs once for every lane
  // at one; a sample's mixer2 advance waits for its carrier step.  The
  // carrier step reads none of what the sample's other NCOs and the
  // coarse-ring entry change, so running those first keeps the order of
  // every value.
  // the table entries, prefiltered value and AGC slot a sample uses are
  // loaded a sample ahead (each would otherwise be an L2 round trip on the
  // sample's chain)
  double2 cm_next = T.cis[c_cis_index(m2_ptr)], so_next = T.cis[c_cis_index(so_ptr)];
  double2 cu_next = T.cis[c_cis_index(up_ptr)], o_next = cout[n0 & (C_OUT_RING - 1)];
  double agc_next = S.agc[(size_t)agc_ptr * C + c];
  // the PCM word of the coarse-ring entry a sample writes (the next
  // sample's) is loaded two samples ahead: one ahead it would be waited for
  // at once by the entry's store
  int16_t pcm_n1 = S.pcm[(size_t)((n0 + 1) & capm) * C + c], pcm_n2 = S.pcm[(size_t)((n0 + 2) & capm) * C + c];
  int i = 0;
  while (i < ie) {
    bool pend = false;
    double ev_pr = 0.0, ev_pi = 0.0;
    do {
      const long long n = n0 + i;
      double2 pre;
      {  // the prefilter's up-mix: *= mixer_fir_pre.WTCISValue_conj(), WTnextFrame() (:316-322)
        const double2 o = o_next, cu = cu_next;
        c_nco_next(up_ptr, fp_step);
        o_next = cout[(n + 1) & (C_OUT_RING - 1)];
        cu_next = T.cis[c_cis_index(up_ptr)];
        const double cr = cu.x, ci = -cu.y;
        pre = make_double2(o.x * cr - o.y * ci, o.x * ci + o.y * cr);
      }
      const double2 cm = cm_next;
      // mix only: sig2 = mixer2.WTCISValue() * cval_prefiltered[i] (:376-385)
      double s2r = cm.x * pre.x - cm.y * pre.y, s2i = cm.x * pre.y + cm.y * pre.x;
      m2_fsum += m2_freq;
      const double dab = sqrt(s2r * s2r + s2i * s2i);
      {  // AGC (DSP.cpp:371-380)
        const double agc_old = agc_next;
        agc_sum = agc_sum - agc_old;
        agc_sum = agc_sum + fabs(dab);
        S.agc[(size_t)agc_ptr * C + c] = fabs(dab);
        agc_ptr++;
        if (agc_ptr == AGC_LEN) agc_ptr = 0;
        agc_next = S.agc[(size_t)agc_ptr * C + c];
        // the short exact divisions of aero_math.h at the call sites whose
        // operand ranges demod_oqpsk.hip argues (the same expressions)
        double g = div_n(1.414213562, fmax(div_c(agc_sum, ((double)AGC_LEN)), 0.000001));
        g = fmax(g, 0.000001);
        s2r *= g;
        s2i *= g;
      }
      const double ab = aero_hypot_w(s2r, s2i);  // clipping (:408-410)
      if (ab > 2.84) {
        const double kk = div_n(2.84, ab);
        s2r = kk * s2r;
        s2i = kk * s2i;
      }
      // symbol timer (:413-426)
      const double st_diff = c_delay<2, 1, 0>(d1, p1, sdly[0], ab * ab) - (ab * ab);
      const double st_d1out = c_delay<4, 3, 2>(d41, p41, sdly[1], st_diff);
      const double st_d2out = c_delay<4, 3, 2>(d42, p42, sdly[2], st_d1out);
      double st_eta = (st_d2out - st_diff) * st_d1out;
      st_eta = c_iir3(srx1, srx2, sry1, sry2, sr_b, sr_a, st_eta);
      const double m1r = st_eta, m1i = -c_delay<3, 2, 1>(d8, p8, sdly[3], st_eta);
      const double2 so = so_next;
      const double ore = so.x * m1r - so.y * m1i, oim = so.x * m1i + so.y * m1r;
      const double st_angle_error = aero_atan2_bf(oim, ore, cij);
      c_set_freq(so_freq, so_step, -st_angle_error * 0.00000001 + so_freq);
      so_ptr += div_c(-st_angle_error * 0.01, 360.0) * WTSIZE;
      wt_wrap(so_ptr);
      if (so_freq < (SO_F - 0.1)) c_set_freq(so_freq, so_step, (SO_F - 0.1));
      if (so_freq > (SO_F + 0.1)) c_set_freq(so_freq, so_step, (SO_F + 0.1));
      if (!s2l_init) {
        s2l_re = s2r;
        s2l_im = s2i;
        s2l_init = 1;
      }
      {  // sample instant (:430) IfHavePassedPoint (DSP.cpp:222-238)
        double tl = so_last - PT, tw = so_ptr - PT;
        if (tl < 0.0) tl += WTSIZE;
        if (tw < 0.0) tw += WTSIZE;
        if ((tl > 3.0 * WTSIZE / 4.0) && (tw < 1.0 * WTSIZE / 4.0)) {
          const double pt_last = div_n(tw, so_step);  // tw: 0 or >= 2^-40, so_step ~3500
          const double pt_this = 1.0 - pt_last;
          const double pr = pt_this * s2r + pt_last * s2l_re;
          const double pi = pt_this * s2i + pt_last * s2l_im;
          yui++;
          yui %= 2;
          if (!yui) {
            ptd_re = pr;
            ptd_im = pi;
          } else {
            ev_pr = pr;
            ev_pi = pi;
            pend = true;
          }
        }
      }
      s2l_re = s2r;
      s2l_im = s2i;
      c_nco_next(mc_ptr, mc_step);
      so_last = so_ptr;
      c_nco_next(so_ptr, so_step);
      so_next = T.cis[c_cis_index(so_ptr)];
      if (i + 1 < ia) {  // coarse-ring entry of the next sample (:351-356)
        const long long n1 = n + 1;
        S.cring[(size_t)c * NFFT + (n1 & (NFFT - 1))] = (uint32_t)c_cis_index(mc_ptr) | ((uint32_t)(uint16_t)pcm_n1 << 16);
        ifl = i + 2;
      }
      pcm_n1 = pcm_n2;
      pcm_n2 = S.pcm[(size_t)((n + 3) & capm) * C + c];  // past the pushed samples: unused
      if (!pend) {
        c_nco_next(m2_ptr, m2_step);
        cm_next = T.cis[c_cis_index(m2_ptr)];
        ++i;
      }
    } while (!pend && i < ie);
    if (pend) {  // carrier step (:447-541)
      const int dt_rp = (dt_p + 1) % DT_LEN;
      const double marg_old = marg[marg_p];
      const double2 dv = dtb[dt_rp];
      const double2 pms_old = pmsb[pm_p];
      const double pr = ev_pr, pi = ev_pi;
      double qr = pr, qi = ptd_im;  // pt_qpsk
      const double ct_xt = aero_tanh_bf(pi) * pr;
      const double ct_xt_d = aero_tanh_bf(ptd_re) * ptd_im;
      double ct_ec = ct_xt_d - ct_xt;
      if (ct_ec > M_PI) ct_ec = M_PI;
      if (ct_ec < -M_PI) ct_ec = -M_PI;
      {  // 8400: mixer2.IncresePhaseDeg(1.0 * ct_ec) unfiltered (DSP.cpp:177-187)
        double phase_deg = 1.0 * ct_ec;
        phase_deg += div_cw(360.0 * m2_ptr, (double)WTSIZE);
        m2_ptr = set_phase_ptr(phase_deg);
      }
      // mixer2.IncreseFreqHz(0.5 * 0.01 * ct_iir_loopfilter.update(ct_ec)) (:470)
      c_set_freq(m2_freq, m2_step, 0.5 * 0.01 * c_iir3(ctx1, ctx2, cty1, cty2, ct_b, ct_a, ct_ec) + m2_freq);
      marg_sum = marg_sum - marg_old;  // marg->UpdateSigned (DSP.cpp:419-427)
      marg_sum = marg_sum + (ct_ec);
      marg[marg_p] = ct_ec;
      marg_p++;
      marg_p %= MARG_LEN;
      const double mval = marg_sum / ((double)MARG_LEN);
      dtb[dt_p] = make_double2(qr, qi);  // dt.update (DSP.h:456-461)
      dt_p = dt_rp;
      qr = dv.x;
      qi = dv.y;
      double rs, rc;
      aero_sincos_bf(mval, rs, rc, sct);
      const double rr = qr * rc - qi * rs, ri = qr * rs + qi * rc;
      qr = rr;
      qi = ri;
      if (TRACE) {
        if (ptn < S.pt_cap) S.pt[(size_t)c * S.pt_cap + ptn] = make_double2(qr, qi);
        ptn++;
      }
      {  // MSEcalc::Update (DSP.cpp:449-461)
        const double av = aero_hypot_w(qr, qi);
        pm_sum = pm_sum - pms_old.x;
        pm_sum = pm_sum + fabs(av);
        const int slot = pm_p;
        pm_p++;
        pm_p %= MSE_LEN;
        double mu = div_c(pm_sum, ((double)MSE_LEN));
        if (mu < 0.000001) mu = 0.000001;
        const double rmu = rcp_div(mu);  // mu >= 1e-6
        const double tr = div_r(1.4142135623730951 * qr, mu, rmu), ti = div_r(1.4142135623730951 * qi, mu, rmu);
        const double tda = (fabs(tr) - 1.0), tdb = (fabs(ti) - 1.0);
        const double v = (tda * tda) + (tdb * tdb);
        ms_sum = ms_sum - pms_old.y;
        ms_sum = ms_sum + fabs(v);
        pmsb[slot] = make_double2(fabs(av), fabs(v));
        ms_p++;
        ms_p %= MSE_LEN;
        mse = div_c(ms_sum, ((double)MSE_LEN));  // exact: ms_sum is 0 or a multiple of 2^-158
      }
      if (mse < 0.65) {  // soft bits, imag first (:516-530)
        int ibit = c_qround(0.75 * qi * 127.0 + 128.0);
        if (ibit > 255) ibit = 255;
        if (ibit < 0) ibit = 0;
        int rbit = c_qround(0.75 * qr * 127.0 + 128.0);
        if (rbit > 255) rbit = 255;
        if (rbit < 0) rbit = 0;
        soft[softp & (SOFT_RING - 1)] = (uint8_t)ibit;
        soft[(softp + 1) & (SOFT_RING - 1)] = (uint8_t)rbit;
        softp += 2;
      }
      c_nco_next(m2_ptr, m2_step);
      cm_next = T.cis[c_cis_index(m2_ptr)];
      ++i;
    }
  }
  double *ds = S.ds + c;
  int *is = S.is + c;
  long long *ls = S.ls + c;
  ds[DS_FP_PTR * C] = up_ptr;
  if (n0 + i == pre_end) {  // end of the message: mixer_fir_pre.SetFreq(mixer2_freq_sum / i) (:555-557)
    double f = m2_fsum / ((double)(pre_end - ls[LS_MSG_START * C]));
    double st = 0;
    c_set_freq(f, st, f);
    ds[DS_FP_FREQ * C] = f;
    ds[DS_FP_STEP * C] = st;
    m2_fsum = 0;
  }
  ls[LS_NSAMP * C] = n0 + i;
  ls[LS_FILLED * C] = n0 + ifl;
  ls[LS_SOFT_P * C] = softp;
  if (TRACE) ls[LS_PT_N * C] = ptn;
  ds[DS_M2_FSUM * C] = m2_fsum;
  ds[DS_CT_X1 * C] = ctx1;
  ds[DS_CT_X2 * C] = ctx2;
  ds[DS_CT_Y1 * C] = cty1;
  ds[DS_CT_Y2 * C] = cty2;
  ds[DS_MARG_SUM * C] = marg_sum;
  ds[DS_PM_SUM * C] = pm_sum;
  ds[DS_MS_SUM * C] = ms_sum;
  ds[DS_MSE * C] = mse;
  ds[DS_PTD_RE * C] = ptd_re;
  ds[DS_PTD_IM * C] = ptd_im;
  ds[DS_M2_FREQ * C] = m2_freq;
  ds[DS_M2_PTR * C] = m2_ptr;
  ds[DS_M2_STEP * C] = m2_step;
  ds[DS_MC_PTR * C] = mc_ptr;
  ds[DS_MC_STEP * C] = mc_step;
  ds[DS_SO_PTR * C] = so_ptr;
  ds[DS_SO_LAST * C] = so_last;
  ds[DS_SO_STEP * C] = so_step;
  ds[DS_SO_FREQ * C] = so_freq;
  ds[DS_AGC_SUM * C] = agc_sum;
#pragma unroll
  for (int q = 0; q < 2; ++q) ds[(DS_D1_0 + q) * C] = d1[q];
#pragma unroll
  for (int q = 0; q < 4; ++q) ds[(DS_D41_0 + q) * C] = d41[q];
#pragma unroll
  for (int q = 0; q < 4; ++q) ds[(DS_D42_0 + q) * C] = d42[q];
#pragma unroll
  for (int q = 0; q < 3; ++q) ds[(DS_D8_0 + q) * C] = d8[q];
  ds[DS_SR_X1 * C] = srx1;
  ds[DS_SR_X2 * C] = srx2;
  ds[DS_SR_Y1 * C] = sry1;
  ds[DS_SR_Y2 * C] = sry2;
  ds[DS_S2L_RE * C] = s2l_re;
  ds[DS_S2L_IM * C] = s2l_im;
  is[IS_AGC_PTR * C] = agc_ptr;
  is[IS_YUI * C] = yui;
  is[IS_S2L_INIT * C] = s2l_init;
  is[IS_MARG_P * C] = marg_p;
  is[IS_DT_P * C] = dt_p;
  is[IS_PM_P * C] = pm_p;
  is[IS_MS_P * C] = ms_p;
  is[IS_D1_P * C] = p1;
  is[IS_D41_P * C] = p41;
  is[IS_D42_P * C] = p42;
  is[IS_D8_P * C] = p8;
}

namespace {
// OQPSKPreambleDetectorAndAmbiguityCorrection::Update (decode/aerol.cpp:842-877)
// on 52-bit shift registers (newest bit lowest): preamble 1, and only if it
// does not match, preamble 2's buffer shifts and is checked
constexpr uint64_t C_PRE1 = 216866263330005ULL, C_PRE2 = 3012071630031408ULL;
constexpr uint64_t C_M52 = (1ULL << 52) - 1;
__device__ __forceinline__ int c_detect(uint64_t &r1, uint64_t &r2, int &inv, int bit) {
  const int tol = 6;  // AeroL::setSettings, continuous (aerol.cpp:972-973)
  r1 = ((r1 << 1) | (uint64_t)bit) & C_M52;
  int x = __builtin_popcountll(r1 ^ C_PRE1);
  if (x >= 52 - tol) {
    inv = 1;
    return 1;
  }
  if (x <= tol) {
    inv = 0;
    return 1;
  }
  r2 = ((r2 << 1) | (uint64_t)bit) & C_M52;
  x = __builtin_popcountll(r2 ^ C_PRE2);
  if (x >= 52 - tol) {
    inv = 1;
    return 1;
  }
  if (x <= tol) {
    inv = 0;
    return 1;
  }
  return 0;
}
}  // namespace

// AeroL::DecodeC's framing (decode/aerol.cpp:2145-2240); every completed
// frame becomes a Viterbi job over its depunctured block
__global__ __launch_bounds__(256) void frame_c_kernel(DevState S, int nch) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nch) return;
  const int C = S.C;
  int *is = S.is;
  long long *ls = S.ls;
  const long long P = ls[LS_SOFT_P * C + c];
  long long q = ls[LS_SOFT_C * C + c];
  const long long E = P & ~31LL;  // delivered in groups of 32 (oqpskdemodulator.cpp:534-540)
  if (q >= E) return;
  int realimag = is[IS_RI * C + c], cntr = is[IS_CNTR * C + c], gsl = is[IS_GSL * C + c];
  int inv_r = is[IS_UWR_INV * C + c], inv_i = is[IS_UWI_INV * C + c];
  int index = is[IS_C_INDEX * C + c];
  int blkbuf = is[IS_BLKBUF * C + c], has_ov = is[IS_HAS_OVERLAP * C + c];
  uint64_t r1 = (uint64_t)ls[LS_C_R1 * C + c], r2 = (uint64_t)ls[LS_C_R2 * C + c];
  uint64_t i1 = (uint64_t)ls[LS_C_I1 * C + c], i2 = (uint64_t)ls[LS_C_I2 * C + c];
  // the soft ring 16 bytes at a time, the next group in flight (as frame_kernel)
  const uint4 *soft16 = reinterpret_cast<const uint4 *>(S.soft + (size_t)c * SOFT_RING);
  constexpr int G16 = SOFT_RING / 16;
  long long grp = q >> 4;
  uint4 cur = soft16[grp & (G16 - 1)], nxt = soft16[(grp + 1) & (G16 - 1)];
  for (; q < E; ++q) {
    if ((q >> 4) != grp) {
      cur = nxt;
      grp++;
      nxt = soft16[(grp + 1) & (G16 - 1)];
    }
    const int wi = (int)(q >> 2) & 3;
    const uint32_t wd = wi == 0 ? cur.x : wi == 1 ? cur.y : wi == 2 ? cur.z : cur.w;
    const int sv = (int)((wd >> (8 * (q & 3))) & 0xFF);
    int bit = sv >= 128 ? 1 : 0;
    int soft_bit = sv;
    int gotsync = 0;
    realimag++;
    realimag %= 2;
    if (cntr > C_FRAME - 112 || cntr <= 0) {
      gotsync = realimag ? c_detect(r1, r2, inv_r, bit) : c_detect(i1, i2, inv_i, bit);
      if (!gsl) {
        gsl = gotsync;
        gotsync = 0;
      } else
        gsl = 0;
    } else {
      gotsync = 0;
      gsl = 0;
    }
    if (realimag ? inv_r : inv_i) {
      bit = 1 - bit;
      if (soft_bit != 128) soft_bit = 255 - soft_bit;
    }
    if (gotsync) {  // a new frame; deleaved / depunctured blocks cleared, scrambler reset
      cntr = -1;
      index = -1;
      continue;
    }
    if (cntr < 1000000000) cntr++;
    if (cntr <= C_FRAME - 1) {
      index++;
      // block kb of the frame, entry index = perm[i] * 4 + j -> deinterleaved
      // d = kb 256 + j 64 + i (perm[i] = 27 i mod 64, so i = 19 row mod 64),
      // depunctured d + d / 3; the frame's last value (d = 4095) is dropped
      const int kb = cntr >> 8;
      const int d = kb * 256 + (index & 3) * 64 + ((19 * (index >> 2)) & 63);
      if (d < C_FRAME - 1) S.block[((size_t)c * 2 + blkbuf) * C_BLOCK + d + d / 3] = (uint8_t)soft_bit;
    }
    if (index == 255) index = -1;
    if (cntr == C_FRAME - 1) {
      const int j = atomicAdd(S.njobs, 1);
      reinterpret_cast<int4 *>(S.jobs)[j] = make_int4(c, blkbuf | ((has_ov ? 0 : 1) << 1), 0, 0);
      has_ov = 1;
      blkbuf ^= 1;
      index = -1;
    }
  }
  ls[LS_SOFT_C * C + c] = q;
  is[IS_RI * C + c] = realimag;
  is[IS_CNTR * C + c] = cntr;
  is[IS_GSL * C + c] = gsl;
  is[IS_UWR_INV * C + c] = inv_r;
  is[IS_UWI_INV * C + c] = inv_i;
  is[IS_C_INDEX * C + c] = index;
  is[IS_BLKBUF * C + c] = blkbuf;
  is[IS_HAS_OVERLAP * C + c] = has_ov;
  ls[LS_C_R1 * C + c] = (long long)r1;
  ls[LS_C_R2 * C + c] = (long long)r2;
  ls[LS_C_I1 * C + c] = (long long)i1;
  ls[LS_C_I2 * C + c] = (long long)i2;
}

namespace {
// soft value p of a C job's decoder input: the previous frame's last 62
// depunctured values, the 5460 depunctured ones (erasures at 4k + 3), 24 erasures
struct CSoft {
  const uint8_t *blk;
  int ov, ovr;
  __device__ __forceinline__ int get(int p, bool may_ov) const {
    const int qq = p - ov;
    int v = 128;
    if (qq >= 0 && qq < C_BLOCK && (qq & 3) != 3) v = blk[qq];
    if (may_ov) {
      const int o = __builtin_amdgcn_ds_bpermute((p & 63) << 2, ovr);
      if (qq < 0) v = o;
    }
    return v;
  }
};
}  // namespace

__global__ __launch_bounds__(64) void viterbi_c_kernel(DevState S, DevTables T) {
  constexpr int NW = (62 + C_BLOCK + 24) / 2 / 64 + 1;
  __shared__ uint64_t obits[NW];
  __shared__ uint8_t pay[C_PAYLOAD];
  __shared__ uint8_t rec[336];
  const int njobs = *S.njobs;
  if (blockIdx.x == 0 && threadIdx.x == 0 && S.njobs_host) *S.njobs_host = njobs;
  const int lane = threadIdx.x, C = S.C;
  for (int job = blockIdx.x; job < njobs; job += gridDim.x) {
    __syncthreads();
    const int4 jd = reinterpret_cast<const int4 *>(S.jobs)[job];
    const int c = jd.x, buf = jd.y & 1, first = (jd.y >> 1) & 1;
    CSoft src;
    src.blk = S.block + ((size_t)c * 2 + buf) * C_BLOCK;
    src.ov = first ? 0 : 62;
    src.ovr = (!first && lane < 62) ? S.overlap[(size_t)c * 64 + lane] : 0;
    if (lane < 62) S.overlap[(size_t)c * 64 + lane] = (uint8_t)src.get(src.ov + C_BLOCK - 62 + lane, false);
    const int nsoft = src.ov + C_BLOCK + 24;
    uint64_t obw, unused;
    viterbi_decode_regs2(src, src, nsoft, obw, unused, lane);
    if (lane < NW) obits[lane] = obw;
    __syncthreads();
    // Decode_Continuous keeps bits [25, 25 + 2730), deconvol.resize(2714)
    // (jconvolutionalcodec.cpp:186-191, aerol.cpp:2249); DelayLine dl2
    // (aerol.h:464-471) out[q] = buffer[(p + q + 1) % L] before the q-th write,
    // i.e. an old value for q + 1 < L and in[q + 1 - L] after the wrap; then
    // AeroLScrambler from position 0 (reset at the frame's UW)
    uint8_t *dlg = S.dl2 + (size_t)c * C_DL2_LEN;
    const int p0 = S.is[IS_DL2_PTR * C + c];
    auto obit = [&](int k) { return (int)((obits[k >> 6] >> (k & 63)) & 1ULL); };
    for (int k = lane; k < C_PAYLOAD; k += 64) {
      int v;
      if (k + 1 < C_DL2_LEN) {
        int r = p0 + k + 1;
        r = r >= C_DL2_LEN ? r - C_DL2_LEN : r;
        v = dlg[r];
      } else {
        v = obit(25 + k + 1 - C_DL2_LEN);
      }
      pay[k] = (uint8_t)((v ^ T.scr[k]) & 1);
    }
    __syncthreads();  // every old delay-line value read
    for (int k = lane; k < C_PAYLOAD; k += 64) {
      if (k + C_DL2_LEN < C_PAYLOAD) continue;  // overwritten by a later input of this block
      int w = p0 + k;
      w %= C_DL2_LEN;
      dlg[w] = (uint8_t)obit(25 + k);
    }
    if (lane == 0) S.is[IS_DL2_PTR * C + c] = (p0 + C_PAYLOAD) % C_DL2_LEN;
    // three SUs from 24 sub-data fields of 12 bits at 109 y + 97, LSB-first
    // bytes (aerol.cpp:2262-2282); 25 voice frames of 96 bits at 109 y + 1 (:2362-2392)
    if (lane < 36) {
      int v = 0;
      for (int b = 0; b < 8; ++b) {
        const int kb = 8 * lane + b, y = kb / 12;
        v |= pay[y * 109 + 97 + kb % 12] << b;
      }
      rec[lane] = (uint8_t)v;
    }
    for (int byte = lane; byte < 300; byte += 64) {
      int v = 0;
      for (int b = 0; b < 8; ++b) {
        const int kb = 8 * byte + b, y = kb / 96;
        v |= pay[y * 109 + 1 + kb % 96] << b;
      }
      rec[36 + byte] = (uint8_t)v;
    }
    __syncthreads();
    bool ok = false;
    if (lane < 3) {  // AeroLcrc16::calcusingbytes (aerol.h:332-367), no all-zero exception here
      const uint8_t *su = rec + 12 * lane;
      unsigned crc = 0xFFFF;
      for (int k = 0; k < 10; ++k) {
        unsigned mb = su[k];
        for (int b = 0; b < 8; ++b) {
          const unsigned cb = crc & 1, bt = mb & 1;
          mb >>= 1;
          crc >>= 1;
          if (cb ^ bt) crc ^= 0x8408;
        }
      }
      ok = ((~crc) & 0xFFFF) == (((unsigned)su[11] << 8) | su[10]);
    }
    const unsigned long long okm = __ballot(ok);
    uint8_t *out = S.jobout + (size_t)job * JOB_OUT_C;
    for (int b = lane; b < 336; b += 64) out[b] = rec[b];
    if (lane == 0) {
      int *o = reinterpret_cast<int *>(out + 336);
      o[0] = 36;
      o[1] = (int)(okm & 7);
      o[2] = 0;
      o[3] = c;
    }
  }
}

void launch_prefilter_c(hipStream_t st, const DevState &S, const DevTables &T, const void *jobs, int njobs) {
  if (njobs <= 0) return;
  hipLaunchKernelGGL(prefilter_dn_kernel, dim3((njobs + 63) / 64), dim3(64), 0, st, S, (const CPreJob *)jobs, njobs);
  hipLaunchKernelGGL(prefilter_blk_kernel, dim3(njobs), dim3(256), 0, st, S, T, (const CPreJob *)jobs);
}
void launch_demod_c(hipStream_t st, const DevState &S, const DevTables &T, int nch, bool trace) {
  const dim3 g((nch + 63) / 64), b(64);
  if (trace)
    hipLaunchKernelGGL(demod_c_kernel<true>, g, b, 0, st, S, T, nch);
  else
    hipLaunchKernelGGL(demod_c_kernel<false>, g, b, 0, st, S, T, nch);
}
void launch_frame_c(hipStream_t st, const DevState &S, int nch) {
  hipLaunchKernelGGL(frame_c_kernel, dim3((nch + 255) / 256), dim3(256), 0, st, S, nch);
}
void launch_viterbi_c(hipStream_t st, const DevState &S, const DevTables &T, int max_jobs) {
  if (max_jobs <= 0) return;
  max_jobs = max_jobs < 16384 ? max_jobs : 16384;
  hipLaunchKernelGGL(viterbi_c_kernel, dim3(max_jobs), dim3(64), 0, st, S, T);
}
void upload_c_constants(const DelayDesc *dly) { hipMemcpyToSymbol(HIP_SYMBOL(cc_dly), dly, sizeof(DelayDesc) * 4); }
int c_prejob_bytes() { return (int)sizeof(CPreJob); }

}  // namespace aero
