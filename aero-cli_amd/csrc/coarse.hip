/*
 * coarse.hip — CoarseFreqEstimate::ProcessBasebandData
 * (decode/coarsefreqestimate.cpp:134-195) plus the hop-time control path
 * OqpskDemodulator::FreqOffsetEstimateSlot (decode/oqpskdemodulator.cpp:562-620),
 * SignalHunter::updatedSignalStatus (decode/hunter.cpp:21-42) and
 * CenterFreqChangedSlot (decode/oqpskdemodulator.cpp:256-280), for every
 * channel whose 4096-sample hop is due.
 *
 * One 1024-thread workgroup per channel.  The 16384-point FP64 FFT keeps 16
 * complex values per thread in registers and runs JFFT's radix-2 DIT
 * butterflies (decode/jfft.cpp:114-212) in four register phases (stages 0-3,
 * 4-7, 8-11, 12-13) with LDS transposes between them; every butterfly uses
 * the same operands and twiddle as the reference, so the output is
 * bit-identical regardless of how butterflies are scheduled.
 */
#include <hip/hip_runtime.h>

#include "aero_math.h"
#include "engine_common.h"

namespace aero {

constexpr int FT = 1024;  // threads per channel FFT
constexpr int PADDED = NFFT + NFFT / 16;

__device__ __forceinline__ int pad(int p) { return p + (p >> 4); }

template <int PH>
__device__ __forceinline__ int epos(int t, int i) {
  if (PH == 0) return (t << 4) | i;
  if (PH == 1) return (t & 15) | (i << 4) | ((t >> 4) << 8);
  if (PH == 2) return (t & 255) | (i << 8) | ((t >> 8) << 12);
  return (t & 1023) | ((i >> 2) << 10) | ((i & 3) << 12);
}

__device__ __forceinline__ int bitrev14(int p) { return (int)(__builtin_bitreverse32((uint32_t)p) >> 18); }

// one radix-2 DIT stage of half-size n on the thread's 16 values;
// `lb` is the bit of i that encodes the stage's position bit.
// `t` is laundered at every stage/exchange so the compiler recomputes the
// (cheap) per-thread positions instead of keeping hundreds of addresses live
// across the three transforms (that is what spilled).
__device__ __forceinline__ int fresh(int t) {
  asm volatile("" : "+v"(t));
  return t;
}

template <int PH>
__device__ __forceinline__ void stage(double2 (&x)[16], int t0, int lb, int n, const double2 *__restrict__ TW) {
  const int t = fresh(t0);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    if (i & (1 << lb)) continue;
    const int il = i | (1 << lb);
    const int pk = epos<PH>(t, i);
    const double2 w = TW[n - 1 + (pk & (n - 1))];
    const double yr = w.x * x[il].x - w.y * x[il].y;
    const double yi = w.x * x[il].y + w.y * x[il].x;
    x[il].x = x[i].x - yr;
    x[il].y = x[i].y - yi;
    x[i].x = x[i].x + yr;
    x[i].y = x[i].y + yi;
  }
}

// move values from layout PH_FROM to PH_TO through LDS (re then im);
// BR: the destination reads bit-reversed positions (start of a new transform)
template <int PH_FROM, int PH_TO, bool BR>
__device__ __forceinline__ void exchange(double2 (&x)[16], int t0, double *lds) {
#pragma unroll
  for (int part = 0; part < 2; ++part) {
    const int t = fresh(t0);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 16; ++i) lds[pad(epos<PH_FROM>(t, i))] = part ? x[i].y : x[i].x;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      int p = epos<PH_TO>(t, i);
      if (BR) p = bitrev14(p);
      const double v = lds[pad(p)];
      if (part)
        x[i].y = v;
      else
        x[i].x = v;
    }
  }
}

// full JFFT::fft on values already loaded in bit-reversed order in layout 0;
// leaves the natural-order result in layout 3
__device__ __forceinline__ void fft16k(double2 (&x)[16], int t, double *lds, const double2 *__restrict__ TW) {
  stage<0>(x, t, 0, 1, TW);
  stage<0>(x, t, 1, 2, TW);
  stage<0>(x, t, 2, 4, TW);
  stage<0>(x, t, 3, 8, TW);
  exchange<0, 1, false>(x, t, lds);
  stage<1>(x, t, 0, 16, TW);
  stage<1>(x, t, 1, 32, TW);
  stage<1>(x, t, 2, 64, TW);
  stage<1>(x, t, 3, 128, TW);
  exchange<1, 2, false>(x, t, lds);
  stage<2>(x, t, 0, 256, TW);
  stage<2>(x, t, 1, 512, TW);
  stage<2>(x, t, 2, 1024, TW);
  stage<2>(x, t, 3, 2048, TW);
  exchange<2, 3, false>(x, t, lds);
  stage<3>(x, t, 0, 4096, TW);
  stage<3>(x, t, 1, 8192, TW);
}

__device__ __forceinline__ void set_freq1(double &freq, double &step, double f) {  // SetFreq (DSP.cpp:163-168)
  freq = f;
  if (freq < 0) freq = 0;
  step = (freq) * ((double)WTSIZE) / 48000.0;
}

__global__ __launch_bounds__(FT) void coarse_kernel(DevState S, DevTables T, int nch) {
  __shared__ double lds[PADDED];
  __shared__ double red_v[FT / 64];
  __shared__ int red_i[FT / 64];
  const int c = blockIdx.x;
  const int t = threadIdx.x;
  if (c >= nch) return;
  const int C = S.C;
  // hop due? sample n_k = 4096 k - 1, demod stopped there and the ring holds it
  const long long nsamp = S.ls[LS_NSAMP * C + c];
  const long long filled = S.ls[LS_FILLED * C + c];
  const int hops_done = S.is[IS_HOPS_DONE * C + c];
  const long long nk = (long long)HOP * (hops_done + 1) - 1;
  const long long avail = S.ls[LS_AVAIL * C + c];
  if (nsamp != nk || avail <= nk) return;
  const long long zero_before = S.ls[LS_ZERO_BEFORE * C + c];
  if (filled <= nk && t == 0) {
    // ring entry of the hop sample not written yet (the demod segment ended
    // before the sample was pushed): mixer_center has not moved since
    const double mc_ptr = S.ds[DS_MC_PTR * C + c];
    int tint = (int)mc_ptr;
    if (tint >= WTSIZE) tint = 0;
    if (tint < 0) tint = WTSIZE - 1;
    const int16_t xs = S.pcm[(nk & (S.pcm_cap - 1)) * C + c];
    S.cring[(size_t)c * NFFT + (nk & (NFFT - 1))] = (uint32_t)tint | ((uint32_t)(uint16_t)xs << 16);
    S.ls[LS_FILLED * C + c] = nk + 1;
  }
  __syncthreads();

  // ring words -> LDS (as uint32 in the first 64 KB)
  uint32_t *ring_lds = reinterpret_cast<uint32_t *>(lds);
  const uint32_t *ring = S.cring + (size_t)c * NFFT;
  for (int j = t; j < NFFT; j += FT) ring_lds[j] = ring[j];
  __syncthreads();
  double2 x[16];
  const long long s0 = nk - (NFFT - 1);  // sample of snapshot element 0 (oqpskdemodulator.cpp:359-365)
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int j = bitrev14(epos<0>(t, i));
    const long long s = s0 + j;
    if (s < 0 || s < zero_before) {
      x[i] = make_double2(0.0, 0.0);
    } else {
      const uint32_t w = ring_lds[s & (NFFT - 1)];
      const double dval = ((double)(int16_t)(w >> 16)) / 32768.0;
      const double2 cs = T.cis[w & 0xFFFF];
      x[i] = make_double2(cs.x * dval, cs.y * dval);
    }
  }
  // forward FFT
  fft16k(x, t, lds, T.tw);
  // boxcar: zero bins startbin..stopbin (coarsefreqestimate.cpp:143-146)
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int p = epos<3>(t, i);
    if (p >= 3584 && p <= 12800) x[i] = make_double2(0.0, 0.0);
  }
  // inverse FFT (JFFT scales by 1/N, FFTWrapper multiplies by N)
  exchange<3, 0, true>(x, t, lds);
  fft16k(x, t, lds, T.twi);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    x[i].x *= (1.0 / ((double)NFFT));
    x[i].y *= (1.0 / ((double)NFFT));
    x[i].x *= (double)NFFT;
    x[i].y *= (double)NFFT;
    // square
    const double r = x[i].x * x[i].x - x[i].y * x[i].y;
    const double im = x[i].x * x[i].y + x[i].y * x[i].x;
    x[i] = make_double2(r, im);
  }
  exchange<3, 0, true>(x, t, lds);
  fft16k(x, t, lds, T.tw);
  // fftshift + smoothing y = 0.9 y + 10 log10(max(|X|,1)) over the bins the fold reads:
  // |X| per bin to LDS first (keeps the log10 out of the register-heavy FFT scope)
  __syncthreads();
  double *ylds = lds;  // [Y_LEN]
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int yi = epos<3>(t, i) ^ (NFFT / 2);
    if (yi >= Y_LO && yi <= Y_HI) ylds[yi - Y_LO] = aero_hypot(x[i].x, x[i].y);
  }
  __syncthreads();
  {
    double *yg = S.y + (size_t)c * Y_LEN;
    const int yreset = S.is[IS_YRESET * C + c];
#pragma unroll 1
    for (int k = t; k < Y_LEN; k += FT) {
      const double yold = yreset ? 20.0 : yg[k];
      const double ynew = yold * 0.9 + 0.1 * 10 * aero_log10(fmax(ylds[k], 1.0));
      yg[k] = ynew;
      ylds[k] = ynew;
    }
  }
  __syncthreads();
  // fold search (coarsefreqestimate.cpp:166-185): first strict maximum above 0
  double bv = 0.0;
  int bi = 0x7fffffff;
  for (int r = 0; r < 7; ++r) {
    const int i = 4608 + t + FT * r;
    if (i >= 11776) break;
    double val = 0;
    for (int j = -1; j <= 1; j++) val += (ylds[i - 1792 - j - Y_LO] + ylds[i + 1792 + j - Y_LO]);
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
  if (t != 0) return;
  for (int w = 1; w < FT / 64; ++w) {
    if (red_v[w] > bv || (red_v[w] == bv && red_i[w] < bi)) {
      bv = red_v[w];
      bi = red_i[w];
    }
  }
  const int zmaxloc = (bv > 0.0) ? bi : NFFT / 2;
  const double nfft = (double)NFFT;
  const double freq_offset_est = -((double)(zmaxloc - nfft / 2)) * (48000.0 / nfft) * 0.5;
  double est;
  int ecd = S.is[IS_EMPTYCD * C + c];
  if (ecd <= 0) {
    est = freq_offset_est;
  } else {
    ecd--;
    est = 0;
  }
  int yres_next = 0;

  // ---- FreqOffsetEstimateSlot (dcd never set: DCDstatSlot unconnected, decode.cpp:168-241)
  double *ds = S.ds;
  int *is = S.is;
  const double thr = 0.65, lockingbw = 10500.0, Fs = 48000.0;
  const double mse = ds[DS_MSE * C + c];
  double m2f = ds[DS_M2_FREQ * C + c], m2s = ds[DS_M2_STEP * C + c];
  double mcf = ds[DS_MC_FREQ * C + c], mcs = ds[DS_MC_STEP * C + c];
  int countdown2 = is[IS_COUNTDOWN2 * C + c], countdown = is[IS_COUNTDOWN * C + c];
  long long zb = zero_before;
  if (mse < thr) {
    if (countdown2 > 0)
      countdown2--;
    else
      set_freq1(m2f, m2s, mcf + est);
  } else
    countdown2 = 5;
  if ((mse > thr) && (fabs(m2f - (mcf + est)) > 3.0)) set_freq1(m2f, m2s, mcf + est);
  if ((mse < thr) && (fabs(m2f - mcf) > 3.0)) {
    if (countdown > 0)
      countdown--;
    else {
      set_freq1(mcf, mcs, m2f);
      if (mcf < lockingbw / 2.0) set_freq1(mcf, mcs, lockingbw / 2.0);
      if (mcf > (Fs / 2.0 - lockingbw / 2.0)) set_freq1(mcf, mcs, Fs / 2.0 - lockingbw / 2.0);
      ecd = 4;  // bigchange (coarsefreqestimate.cpp:128-132)
      yres_next = 1;
      zb = nk + 1;  // bbcycbuff zeroed
    }
  } else
    countdown = 4;
  // ---- SignalStatus -> SignalHunter (hunter.cpp:21-42, maxTries 15, params 0/25000/10500)
  const bool gotasignal = !(mse > thr);
  unsigned iter = (unsigned)is[IS_HUNT_ITER * C + c];
  if (gotasignal) {
    iter = 0;
  } else {
    iter++;
    if (iter > 0 && iter % 15u == 0) {
      double fc = 0u + (10500u >> 1) * (int)(iter / 15u);
      if (fc > 25000u - (10500u >> 1)) {
        fc = 0.0;
        iter = 0;
        is[IS_HUNT_SCANS * C + c]++;
      }
      // CenterFreqChangedSlot (oqpskdemodulator.cpp:256-280), fb != 8400, afc on
      if (fc < (0.5 * 10500.0)) fc = 0.5 * 10500.0;
      if (fc > (Fs / 2.0 - 0.5 * 10500.0)) fc = Fs / 2.0 - 0.5 * 10500.0;
      set_freq1(mcf, mcs, fc);
      set_freq1(m2f, m2s, mcf);
      if ((m2f - mcf) > (lockingbw / 2.0)) set_freq1(m2f, m2s, mcf + (lockingbw / 2.0));
      if ((m2f - mcf) < (-lockingbw / 2.0)) set_freq1(m2f, m2s, mcf - (lockingbw / 2.0));
      zb = nk + 1;
    }
  }
  is[IS_HUNT_ITER * C + c] = (int)iter;
  ds[DS_M2_FREQ * C + c] = m2f;
  ds[DS_M2_STEP * C + c] = m2s;
  ds[DS_MC_FREQ * C + c] = mcf;
  ds[DS_MC_STEP * C + c] = mcs;
  is[IS_COUNTDOWN2 * C + c] = countdown2;
  is[IS_COUNTDOWN * C + c] = countdown;
  is[IS_EMPTYCD * C + c] = ecd;
  is[IS_YRESET * C + c] = yres_next;
  is[IS_HOPS_DONE * C + c] = hops_done + 1;
  S.ls[LS_ZERO_BEFORE * C + c] = zb;
  const int hn = S.hop_n[c];
  if (hn < S.hop_cap) {
    double *h = S.hops + ((size_t)c * S.hop_cap + hn) * 6;
    h[0] = (double)nk;
    h[1] = est;
    h[2] = m2f;
    h[3] = mcf;
    h[4] = mse;
    h[5] = gotasignal ? 1.0 : 0.0;
  }
  S.hop_n[c] = hn + 1;
}

void launch_coarse(hipStream_t st, const DevState &S, const DevTables &T, int nch) {
  hipLaunchKernelGGL(coarse_kernel, dim3(nch), dim3(FT), 0, st, S, T, nch);
}

}  // namespace aero
