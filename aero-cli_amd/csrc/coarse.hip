/*
 * coarse.hip — CoarseFreqEstimate::ProcessBasebandData
 * (decode/coarsefreqestimate.cpp:134-195) plus the hop-time control path
 * OqpskDemodulator::FreqOffsetEstimateSlot (decode/oqpskdemodulator.cpp:562-620),
 * SignalHunter::updatedSignalStatus (decode/hunter.cpp:21-42) and
 * CenterFreqChangedSlot (decode/oqpskdemodulator.cpp:256-280), for every
 * channel whose 4096-sample hop is due.
 *
 * One 1024-thread workgroup per channel.  The 16384-point FP64 FFTs keep 16
 * complex values per thread in registers and run JFFT's radix-2 DIT
 * butterflies (decode/jfft.cpp:114-212) chained through register stages, a
 * wave-local LDS transpose, lane permutes and one workgroup exchange per
 * transform (fft_chain.h); every butterfly uses the same operands and
 * twiddle as the reference, so the output is bit-identical regardless of how
 * butterflies are scheduled.
 */
#include <hip/hip_runtime.h>

#include <type_traits>

#include "aero_math.h"
#include "engine_common.h"
#include "fft_chain.h"

namespace aero {

#ifdef AERO_X_OCML  // timing experiment only (see demod_oqpsk.hip)
#define CO_HYPOT ::hypot
#define CO_HYPOT_NR ::hypot
#define CO_LOG10 ::log10
#else
#define CO_HYPOT aero_hypot
#define CO_HYPOT_NR aero_hypot_nr
#define CO_LOG10 aero_log10
#endif

// Geometry of one channel's coarse estimate (decode/coarsefreqestimate.cpp:39-76
// with the settings each demodulator applies).  OQPSK: setSettings(14, 10500,
// 10500, 48000); MSK: setSettings(13, 900, 600, Fs).
template <int M>
struct CoarseK;
template <>
struct CoarseK<MODE_OQPSK> {
  static constexpr int LOG2N = 14, HOPN = 4096, START = 3584, STOP = 12800, ILO = 4608, IHI = 11776, EPB = 1792;
  static constexpr int YLO = 2815, YHI = 13568;
  static constexpr double FS = 48000.0;
};
// the C channel: setSettings(14, 10500, 8400, 48000): the OQPSK bins, the
// expected peak at round(8400 / (2 hzperbin)) = 1434; the raised-cosine window
// in place of the boxcar (coarsefreqestimate.cpp:97-104)
template <>
struct CoarseK<MODE_C8400> {
  static constexpr int LOG2N = 14, HOPN = 4096, START = 3584, STOP = 12800, ILO = 4608, IHI = 11776, EPB = 1434;
  static constexpr int YLO = 2815, YHI = 13568;
  static constexpr double FS = 48000.0;
};
// MSK at Fs (setSettings(13, 900, 600, Fs)): hzperbin = Fs / 8192; startbin
// round(900 / hzperbin), stopbin nfft - startbin, the fold search over
// [round(-900 / hzperbin + 4096), round(900 / hzperbin + 4096)) with
// expectedpeakbin round(600 / (2 hzperbin)); y kept over MSK_YLO..MSK_YHI
template <int FS>
struct MskCoarseBins;
template <>
struct MskCoarseBins<12000> {
  static constexpr int START = 614, STOP = 7578, ILO = 3482, IHI = 4710, EPB = 205;
};
template <>
struct MskCoarseBins<24000> {
  static constexpr int START = 307, STOP = 7885, ILO = 3789, IHI = 4403, EPB = 102;
};
template <>
struct MskCoarseBins<48000> {
  static constexpr int START = 154, STOP = 8038, ILO = 3942, IHI = 4250, EPB = 51;
};
template <int M>
struct CoarseK {
  using B = MskCoarseBins<msk_fs(M)>;
  static constexpr int LOG2N = 13, HOPN = 2048, START = B::START, STOP = B::STOP, ILO = B::ILO, IHI = B::IHI,
                       EPB = B::EPB;
  static constexpr int YLO = MSK_YLO, YHI = MSK_YHI;
  static_assert(ILO - EPB - 1 >= YLO && IHI - 1 + EPB + 1 <= YHI, "fold search inside the kept y bins");
  static constexpr double FS = (double)msk_fs(M);
};

// the bins and rate one launch works with: compile-time for the fixed-rate
// groups, the group's MskGen for a generic-rate one
struct CoarseBins {
  int start, stop, ilo, ihi, epb;
  double fs;
};
template <int M>
__device__ __forceinline__ CoarseBins coarse_bins(const DevState &S) {
  using K = CoarseK<M>;
  if constexpr (msk_generic(M))
    return {S.mg.start, S.mg.stop, S.mg.ilo, S.mg.ihi, S.mg.epb, S.mg.fs};
  else
    return {K::START, K::STOP, K::ILO, K::IHI, K::EPB, K::FS};
}

__device__ __forceinline__ void set_freq1(double &freq, double &step, double f, double fs) {  // SetFreq (DSP.cpp:163-168)
  freq = f;
  if (freq < 0) freq = 0;
  step = (freq) * ((double)WTSIZE) / fs;
}

struct HopCtl {
  double m2f, m2s, mcf, mcs;
  int countdown2, countdown, ecd, yres_next;
  long long zb;
  bool stepped;  // SignalHunter emitted newFreqCenter(step_fc) this hop
  double step_fc;
};

// OqpskDemodulator::FreqOffsetEstimateSlot (decode/oqpskdemodulator.cpp:562-620),
// SignalHunter (decode/hunter.cpp:21-42; maxTries 15, params 0/25000/10500,
// decode/decode.cpp:161,169) and CenterFreqChangedSlot (:256-280).  dcd is
// never set (DCDstatSlot unconnected, decode/decode.cpp:168-241).
__device__ __forceinline__ bool hop_control_oqpsk(HopCtl &h, bool c8400, double est, double mse, unsigned &iter,
                                                  int &scans, long long nk) {
  const double thr = 0.65, lockingbw = 10500.0, Fs = 48000.0;
  if (mse < thr) {
    if (h.countdown2 > 0)
      h.countdown2--;
    else
      set_freq1(h.m2f, h.m2s, h.mcf + est, Fs);
  } else
    h.countdown2 = 5;
  if ((mse > thr) && (fabs(h.m2f - (h.mcf + est)) > 3.0)) set_freq1(h.m2f, h.m2s, h.mcf + est, Fs);
  if ((mse < thr) && (fabs(h.m2f - h.mcf) > 3.0)) {
    if (h.countdown > 0)
      h.countdown--;
    else {
      set_freq1(h.mcf, h.mcs, h.m2f, Fs);
      if (h.mcf < lockingbw / 2.0) set_freq1(h.mcf, h.mcs, lockingbw / 2.0, Fs);
      if (h.mcf > (Fs / 2.0 - lockingbw / 2.0)) set_freq1(h.mcf, h.mcs, Fs / 2.0 - lockingbw / 2.0, Fs);
      h.ecd = 4;  // bigchange (coarsefreqestimate.cpp:128-132)
      h.yres_next = 1;
      h.zb = nk + 1;  // bbcycbuff zeroed
    }
  } else
    h.countdown = 4;
  const bool gotasignal = !(mse > thr);
  if (gotasignal) {
    iter = 0;
  } else {
    iter++;
    if (iter > 0 && iter % 15u == 0) {
      double fc = 0u + (10500u >> 1) * (int)(iter / 15u);
      if (fc > 25000u - (10500u >> 1)) {
        fc = 0.0;
        iter = 0;
        scans++;
      }
      h.stepped = true;
      h.step_fc = fc;
      // CenterFreqChangedSlot, afc on; fb != 8400 clamps the centre
      // (oqpskdemodulator.cpp:256-265); fb is 10500 as aero-decode's Decoder
      // leaves it (decode/decode.cpp:152-159, oqpskdemodulator.h:24-32)
      if (!c8400) {
        if (fc < (0.5 * 10500.0)) fc = 0.5 * 10500.0;
        if (fc > (Fs / 2.0 - 0.5 * 10500.0)) fc = Fs / 2.0 - 0.5 * 10500.0;
      }
      set_freq1(h.mcf, h.mcs, fc, Fs);
      set_freq1(h.m2f, h.m2s, h.mcf, Fs);
      if ((h.m2f - h.mcf) > (lockingbw / 2.0)) set_freq1(h.m2f, h.m2s, h.mcf + (lockingbw / 2.0), Fs);
      if ((h.m2f - h.mcf) < (-lockingbw / 2.0)) set_freq1(h.m2f, h.m2s, h.mcf - (lockingbw / 2.0), Fs);
      h.zb = nk + 1;
    }
  }
  return gotasignal;
}

__device__ __forceinline__ bool hop_control(HopCtl &h, std::integral_constant<int, MODE_OQPSK>, double, double est,
                                            double mse, unsigned &iter, int &scans, long long nk) {
  return hop_control_oqpsk(h, false, est, mse, iter, scans, nk);
}
// the C channel: the same slot (its prefilter mixer's retune there is
// overridden by the message-end retune before any prefilter runs, :555-569)
__device__ __forceinline__ bool hop_control(HopCtl &h, std::integral_constant<int, MODE_C8400>, double, double est,
                                            double mse, unsigned &iter, int &scans, long long nk) {
  return hop_control_oqpsk(h, true, est, mse, iter, scans, nk);
}

// MskDemodulator::FreqOffsetEstimateSlot (decode/mskdemodulator.cpp:430-469;
// its AFC branch needs dcd, never set), SignalHunter with params 0/6000/900
// (decode/decode.cpp:193) and MskDemodulator::CenterFreqChangedSlot (:220-240).
template <int M>
__device__ __forceinline__ bool hop_control(HopCtl &h, std::integral_constant<int, M>, double Fs, double est,
                                            double mse, unsigned &iter, int &scans, long long nk) {
  const double thr = 0.5, lockingbw = 900.0, fb = 600.0;
  if ((mse > thr) && (fabs(h.m2f - (h.mcf + est)) > 0.0)) set_freq1(h.m2f, h.m2s, h.mcf + est, Fs);
  h.countdown = 4;
  const bool gotasignal = !(mse > thr);
  if (gotasignal) {
    iter = 0;
  } else {
    iter++;
    if (iter > 0 && iter % 15u == 0) {
      double fc = 0u + (900u >> 1) * (int)(iter / 15u);
      if (fc > 6000u - (900u >> 1)) {
        fc = 0.0;
        iter = 0;
        scans++;
      }
      h.stepped = true;
      h.step_fc = fc;
      if (fc < (0.75 * fb)) fc = 0.75 * fb;
      if (fc > (Fs / 2.0 - 0.75 * fb)) fc = Fs / 2.0 - 0.75 * fb;
      set_freq1(h.mcf, h.mcs, fc, Fs);
      set_freq1(h.m2f, h.m2s, h.mcf, Fs);
      if ((h.m2f - h.mcf) > (lockingbw / 2.0)) set_freq1(h.m2f, h.m2s, h.mcf + (lockingbw / 2.0), Fs);
      if ((h.m2f - h.mcf) < (-lockingbw / 2.0)) set_freq1(h.m2f, h.m2s, h.mcf - (lockingbw / 2.0), Fs);
      h.zb = nk + 1;
    }
  }
  return gotasignal;
}

// AERO_X_STAMPS (diagnostic build only): s_memtime cycle totals per section
// of wave 0 of every workgroup that ran a hop (prologue, ring to LDS +
// twiddles, table gathers + mix, FFT 1, boxcar+iFFT+square, FFT 3, |X|,
// log10 smoothing, fold search; slots 0-8), and the number of such
// workgroups (slot 11)
constexpr int CSTAMP_N = 12;
#ifdef AERO_X_STAMPS
__device__ unsigned long long g_cstamps[CSTAMP_N];
#define CSTAMP(k)                                                  \
  do {                                                             \
    __builtin_amdgcn_sched_barrier(0);                             \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();    \
    cst_[k] += t_ - ctime_;                                        \
    ctime_ = t_;                                                   \
    __builtin_amdgcn_sched_barrier(0);                             \
  } while (0)
#else
#define CSTAMP(k) \
  do {            \
  } while (0)
#endif

template <int M>
__global__ __launch_bounds__(1 << (CoarseK<M>::LOG2N - 4), CoarseK<M>::LOG2N == 13 ? 4 : 1) void coarse_kernel(DevState S, DevTables T, int nch) {
  using K = CoarseK<M>;
  const CoarseBins KB = coarse_bins<M>(S);
  constexpr int L = K::LOG2N, N = 1 << L, FT = N / 16, PADDED = N + N / 16;
  constexpr int YLEN = K::YHI - K::YLO + 1;
  __shared__ double lds[PADDED];
  __shared__ double2 s_tw[TwLds<L>::LEN];
  __shared__ double red_v[FT / 64];
  __shared__ int red_i[FT / 64];
  const int c = blockIdx.x;
  const int t = threadIdx.x;
  if (c >= nch) return;
  const int C = S.C;
  // hop due? sample n_k = HOP k - 1, demod stopped there and the ring holds it
  const long long nsamp = S.ls[LS_NSAMP * C + c];
  const long long filled = S.ls[LS_FILLED * C + c];
  const int hops_done = S.is[IS_HOPS_DONE * C + c];
  const long long nk = (long long)K::HOPN * (hops_done + 1) - 1;
  const long long avail = S.ls[LS_AVAIL * C + c];
  if (nsamp != nk || avail <= nk) return;
#ifdef AERO_X_STAMPS
  unsigned long long cst_[CSTAMP_N] = {}, ctime_ = __builtin_amdgcn_s_memtime();
#endif
  const long long zero_before = S.ls[LS_ZERO_BEFORE * C + c];
  if (filled <= nk && t == 0) {
    // ring entry of the hop sample not written yet (the demod segment ended
    // before the sample was pushed): mixer_center has not moved since
    const double mc_ptr = S.ds[DS_MC_PTR * C + c];
    int tint = (int)mc_ptr;
    if (tint >= WTSIZE) tint = 0;
    if (tint < 0) tint = WTSIZE - 1;
    const int16_t xs = S.pcm[(nk & (S.pcm_cap - 1)) * C + c];
    S.cring[(size_t)c * N + (nk & (N - 1))] = (uint32_t)tint | ((uint32_t)(uint16_t)xs << 16);
    S.ls[LS_FILLED * C + c] = nk + 1;
  }
  __syncthreads();
  CSTAMP(0);

  load_tw_lds<L>(s_tw, T.tw, t, FT);
  // ring words -> LDS (uint32, one pad word per 16: the bit-reversed gather
  // below reads 16-word strides, which would hit 4 of the 64 banks unpadded)
  uint32_t *ring_lds = reinterpret_cast<uint32_t *>(lds);
  const uint32_t *ring = S.cring + (size_t)c * N;
  for (int j = t; j < N; j += FT) ring_lds[j + (j >> 4)] = ring[j];
  __syncthreads();
  CSTAMP(1);
  double2 x[16];
  const long long s0 = nk - (N - 1);  // sample of snapshot element 0 (oqpskdemodulator.cpp:359-365)
  // every element's table entry is gathered before any is waited for (the
  // compiler would otherwise sink each gather into its element's branch
  // and wait for it there: 16 round trips one after another)
  double2 cs[16];
  double dval[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int q = (int)((s0 + bitrev<L>(epos<L, 0>(t, i))) & (N - 1));
    const uint32_t w = ring_lds[q + (q >> 4)];
    dval[i] = ((double)(int16_t)(w >> 16)) / 32768.0;
#ifdef AERO_X_CISLINE
    cs[i] = T.cis[w & 0x7];  // timing build: every gather on one line
#else
    cs[i] = T.cis[w & 0xFFFF];
#endif
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) asm volatile("" : "+v"(cs[i].x), "+v"(cs[i].y));
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    // entries below zero_before were cleared (AFC, CenterFreqChangedSlot);
    // entries of samples before the channel's first are the ring's own
    // contents (zero for a new channel: CIS[0] x 0; a channel that changed
    // rate keeps the ring it had, mskdemodulator.cpp:94-218)
    const long long s = s0 + bitrev<L>(epos<L, 0>(t, i));
    x[i] = s < zero_before ? make_double2(0.0, 0.0) : make_double2(cs[i].x * dval[i], cs[i].y * dval[i]);
  }
  __syncthreads();  // the ring image is read: the LDS is the transforms' from here on
  CSTAMP(2);
  // forward FFT
  chain::fft<L, true, false>(x, t, lds, T.tw, s_tw, T.twg);
  CSTAMP(3);
  // boxcar: zero bins startbin..stopbin (coarsefreqestimate.cpp:97-100);
  // the C channel multiplies by the raised-cosine window instead (:101-104)
  const int bin_t = chain::out_bin_thread<L>(t);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int p = bin_t | chain::out_bin_reg<L>(i);
    if constexpr (M == MODE_C8400) {
      const double w = T.cwin[i * FT + t];  // = window[p], stored in this layout's order (engine.hip)
      x[i] = make_double2(x[i].x * w, x[i].y * w);
    } else {
      if (p >= KB.start && p <= KB.stop) x[i] = make_double2(0.0, 0.0);
    }
  }
  // inverse FFT.  JFFT scales by 1/N and FFTWrapper multiplies by N
  // (jfft.cpp:206-212, fftwrapper.cpp:22-29): x * 2^-L * 2^L == x exactly for every
  // x with |x| >= 2^-1008, and a nonzero value of this path is far above that
  // (magnitudes >= ~2^-200: sums and products of pcm/32768, CIS and twiddle
  // values), so both multiplies are the identity here and are skipped.
  chain::fft<L, false, true>(x, t, lds, T.twi, s_tw, T.twgi);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    // square
    // (x*y + y*x: the two products are the same IEEE product, so the sum is
    // exactly 2 (x*y))
    const double r = x[i].x * x[i].x - x[i].y * x[i].y;
    const double im = 2.0 * (x[i].x * x[i].y);
    x[i] = make_double2(r, im);
  }
  CSTAMP(4);
  chain::fft<L, false, false>(x, t, lds, T.tw, s_tw, T.twg);
  CSTAMP(5);
  // fftshift + smoothing y = 0.9 y + 10 log10(max(|X|,1)) over the bins the
  // fold reads: |X| per bin to LDS first (keeps the log10 out of the
  // register-heavy FFT scope), then a dense log10 loop; the y history (HBM)
  // is read three iterations ahead of its update, the first loads
  // overlapping the |X| work.  (Round 5 measured the alternatives on one box:
  // the whole history brought into LDS by direct-to-LDS loads as the third
  // transform ends, |X| and log10 in registers meanwhile, 21.49 ms; plain
  // register loads of the whole history, 21.58 ms; this, 20.97 ms.  The
  // history's 86 KB take ~46k cycles from issue to arrival whichever way,
  // more than the |X| and log10 work that can overlap them.)
  double *yg = S.y + (size_t)c * YLEN;
  const int yreset = S.is[IS_YRESET * C + c];
#ifdef AERO_X_NOYREAD
  auto yload = [&](int k) { return 20.0 + 0.0 * k; };  // timing build: no y history reads
#else
  auto yload = [&](int k) { return (k < YLEN && !yreset) ? yg[k] : 20.0; };
#endif
  double yp0 = yload(t), yp1 = yload(t + FT);
  // no barrier here: the third transform's workgroup exchange ended with
  // one (chain::gx), after which every wave only works in registers, so the
  // LDS is free for |X| as soon as this wave gets here
  double *ylds = lds;  // bin k - YLO at ypad(k - YLO)
  auto ypad = [](int q) { return fftl::ypadn<6>(q); };
  // |X| by aero_hypot_nr when every value of the wave is in its range (the
  // usual case: |X| of a live channel is ~1e9), else by aero_hypot
  bool nr = true;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const double a = fabs(x[i].x), b = fabs(x[i].y);
    nr = nr && a <= 0x1p200 && b <= 0x1p200 && (a >= 0x1p-200 || b >= 0x1p-200);
  }
  if (__all(nr)) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int yi = (bin_t | chain::out_bin_reg<L>(i)) ^ (N / 2);
      if (yi >= K::YLO && yi <= K::YHI) ylds[ypad(yi - K::YLO)] = CO_HYPOT_NR(x[i].x, x[i].y);
    }
  } else {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int yi = (bin_t | chain::out_bin_reg<L>(i)) ^ (N / 2);
      if (yi >= K::YLO && yi <= K::YHI) ylds[ypad(yi - K::YLO)] = CO_HYPOT(x[i].x, x[i].y);
    }
  }
  double yp2 = yload(t + 2 * FT);
  __syncthreads();
  CSTAMP(6);
#pragma unroll 1
  for (int k = t; k < YLEN; k += FT) {
    const double yold = yp0;
    yp0 = yp1;
    yp1 = yp2;
    yp2 = yload(k + 3 * FT);
    const double ynew = yold * 0.9 + 0.1 * 10 * CO_LOG10(fmax(ylds[ypad(k)], 1.0));
    yg[k] = ynew;
    ylds[ypad(k)] = ynew;
  }
  __syncthreads();
  CSTAMP(7);
  // fold search (coarsefreqestimate.cpp:166-185): first strict maximum above 0
  double bv = 0.0;
  int bi = 0x7fffffff;
  for (int r = 0;; ++r) {
    const int i = KB.ilo + t + FT * r;
    if (i >= KB.ihi) break;
    double val = 0;
    for (int j = -1; j <= 1; j++)
      val += (ylds[ypad(i - KB.epb - j - K::YLO)] + ylds[ypad(i + KB.epb + j - K::YLO)]);
    if (val > bv) {
      bv = val;
      bi = i;
    }
  }
  // wave reduce: larger value, then smaller index
  for (int off = 32; off > 0; off >>= 1) {
    const double ov = __shfl_down(bv, off, 64);
    const int oi = __shfl_down(bi, off, 64);
    if (ov > bv || (ov == bv && oi < bi)) {
      bv = ov;
      bi = oi;
    }
  }
  if ((t & 63) == 0) {
    red_v[t >> 6] = bv;
    red_i[t >> 6] = bi;
  }
  __syncthreads();
  CSTAMP(8);
#ifdef AERO_X_STAMPS
  if (t == 0) {
    for (int k = 0; k < 9; ++k) atomicAdd(&g_cstamps[k], cst_[k]);
    atomicAdd(&g_cstamps[CSTAMP_N - 1], 1ull);
  }
#endif
  if (t != 0) return;
  for (int w = 1; w < FT / 64; ++w) {
    if (red_v[w] > bv || (red_v[w] == bv && red_i[w] < bi)) {
      bv = red_v[w];
      bi = red_i[w];
    }
  }
  const int zmaxloc = (bv > 0.0) ? bi : N / 2;
  const double nfft = (double)N;
  const double freq_offset_est = -((double)(zmaxloc - nfft / 2)) * (KB.fs / nfft) * 0.5;
  double est;
  int ecd = S.is[IS_EMPTYCD * C + c];
  if (ecd <= 0) {
    est = freq_offset_est;
  } else {
    ecd--;
    est = 0;
  }

  double *ds = S.ds;
  int *is = S.is;
  const double mse = ds[DS_MSE * C + c];
  HopCtl h;
  h.m2f = ds[DS_M2_FREQ * C + c];
  h.m2s = ds[DS_M2_STEP * C + c];
  h.mcf = ds[DS_MC_FREQ * C + c];
  h.mcs = ds[DS_MC_STEP * C + c];
  h.countdown2 = is[IS_COUNTDOWN2 * C + c];
  h.countdown = is[IS_COUNTDOWN * C + c];
  h.ecd = ecd;
  h.yres_next = 0;
  h.zb = zero_before;
  h.stepped = false;
  h.step_fc = 0.0;
  unsigned iter = (unsigned)is[IS_HUNT_ITER * C + c];
  int scans = is[IS_HUNT_SCANS * C + c];
  const bool gotasignal = hop_control(h, std::integral_constant<int, M>(), KB.fs, est, mse, iter, scans, nk);
  is[IS_HUNT_ITER * C + c] = (int)iter;
  is[IS_HUNT_SCANS * C + c] = scans;
  if (h.stepped) {
    const int k = is[IS_HUNT_STEPS * C + c];
    ds[(DS_HUNT_FC0 + (k & 7)) * C + c] = h.step_fc;
    is[IS_HUNT_STEPS * C + c] = k + 1;
  }
  ds[DS_M2_FREQ * C + c] = h.m2f;
  ds[DS_M2_STEP * C + c] = h.m2s;
  ds[DS_MC_FREQ * C + c] = h.mcf;
  ds[DS_MC_STEP * C + c] = h.mcs;
  is[IS_COUNTDOWN2 * C + c] = h.countdown2;
  is[IS_COUNTDOWN * C + c] = h.countdown;
  is[IS_EMPTYCD * C + c] = h.ecd;
  is[IS_YRESET * C + c] = h.yres_next;
  is[IS_HOPS_DONE * C + c] = hops_done + 1;
  S.ls[LS_ZERO_BEFORE * C + c] = h.zb;
  const int hn = S.hop_n[c];
  if (hn < S.hop_cap) {
    double *hr = S.hops + ((size_t)c * S.hop_cap + hn) * 6;
    hr[0] = (double)nk;
    hr[1] = est;
    hr[2] = h.m2f;
    hr[3] = h.mcf;
    hr[4] = mse;
    hr[5] = gotasignal ? 1.0 : 0.0;
  }
  S.hop_n[c] = hn + 1;
}

void coarse_read_stamps(unsigned long long *out) {
#ifdef AERO_X_STAMPS
  (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_cstamps), sizeof(unsigned long long) * CSTAMP_N);
  unsigned long long z[CSTAMP_N] = {0};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_cstamps), z, sizeof z);
#else
  for (int k = 0; k < CSTAMP_N; ++k) out[k] = 0;
#endif
}

void launch_coarse(hipStream_t st, int mode, const DevState &S, const DevTables &T, int nch) {
  switch (mode) {
    case MODE_OQPSK: hipLaunchKernelGGL(coarse_kernel<MODE_OQPSK>, dim3(nch), dim3(1024), 0, st, S, T, nch); break;
    case MODE_C8400: hipLaunchKernelGGL(coarse_kernel<MODE_C8400>, dim3(nch), dim3(1024), 0, st, S, T, nch); break;
    case MODE_MSK600: hipLaunchKernelGGL(coarse_kernel<MODE_MSK600>, dim3(nch), dim3(512), 0, st, S, T, nch); break;
    case MODE_MSK1200: hipLaunchKernelGGL(coarse_kernel<MODE_MSK1200>, dim3(nch), dim3(512), 0, st, S, T, nch); break;
    case MODE_MSK600_24K:
      hipLaunchKernelGGL(coarse_kernel<MODE_MSK600_24K>, dim3(nch), dim3(512), 0, st, S, T, nch);
      break;
    case MODE_MSK600_48K:
      hipLaunchKernelGGL(coarse_kernel<MODE_MSK600_48K>, dim3(nch), dim3(512), 0, st, S, T, nch);
      break;
    case MODE_MSK1200_12K:
      hipLaunchKernelGGL(coarse_kernel<MODE_MSK1200_12K>, dim3(nch), dim3(512), 0, st, S, T, nch);
      break;
    case MODE_MSK1200_48K:
      hipLaunchKernelGGL(coarse_kernel<MODE_MSK1200_48K>, dim3(nch), dim3(512), 0, st, S, T, nch);
      break;
    default:  // generic-rate MSK (the kernel does not depend on the bit rate)
      hipLaunchKernelGGL(coarse_kernel<MODE_MSKG600>, dim3(nch), dim3(512), 0, st, S, T, nch);
      break;
  }
}

}  // namespace aero
