/*
 * fft_dit.h — JFFT's radix-2 decimation-in-time FFT (decode/jfft.cpp:114-212)
 * for one 4096-, 8192- or 16384-point transform per workgroup of N/16 threads
 * on gfx950: 16 complex FP64 values per thread in registers, three (4096) or
 * four register phases of up to four stages with padded LDS transposes
 * between them.  Every
 * butterfly uses the reference's operands and twiddle (TW[n - 1 + k]), so the
 * result is bit-identical to JFFT however the butterflies are scheduled.
 * Used by burst.hip (Hilbert fast-FIR blocks, trident check) and cchan.hip
 * (the C channel's 4096-point prefilter blocks).
 */
#pragma once
#include <hip/hip_runtime.h>

namespace aero {

// LDS padding of the transposes (1 -> 2, 2 -> 3, 3 -> 0): one double per 32 (one 64-bank row of
// dwords).  Contiguous 32-lane accesses (layouts 2, 3) stay conflict-free and
// the stride-16 ones (layout 0) spread over all banks; it is additive over
// bit-disjoint parts, which the base + immediate-offset addressing needs.
// (p + p/16 left 2-way conflicts on layouts 2/3 and the bit-reversed reads:
// SQ_LDS_BANK_CONFLICT ~= SQ_ACTIVE_INST_LDS on coarse_kernel.)
__device__ __forceinline__ int pad(int p) { return p + (p >> 5); }
// The 0 -> 1 transpose writes stride-16 positions (16-lane store groups hit
// 8 of the 16 double-banks under pad()) and reads two 16-position runs 256
// apart per 32-lane group (2-way under pad()); one double per 16 makes both
// conflict-free.  Each exchange picks its own map: only its writer and its
// reader share the layout.  Buffers hold N + N/16 doubles.
__device__ __forceinline__ int pad16(int p) { return p + (p >> 4); }
template <int PH_FROM, int PH_TO, bool BR>
__device__ __forceinline__ int xpad(int p) {
  return (PH_FROM == 0 && PH_TO == 1 && !BR) ? pad16(p) : pad(p);
}

// position of value i of thread t in register phase PH (4 FFT stages per
// phase; the last phase holds the LOG2N - 12 remaining stage bits in i's low bits)
template <int LOG2N, int PH>
__device__ __forceinline__ int epos(int t, int i) {
  constexpr int LFT = LOG2N - 4, R = LOG2N - 12;
  if (PH == 0) return (t << 4) | i;
  if (PH == 1) return (t & 15) | (i << 4) | ((t >> 4) << 8);
  if (PH == 2) return (t & 255) | (i << 8) | ((t >> 8) << 12);
  return (t & ((1 << LFT) - 1)) | ((i >> R) << LFT) | ((i & ((1 << R) - 1)) << (LOG2N - R));
}

template <int LOG2N>
__device__ __forceinline__ int bitrev(int p) { return (int)(__builtin_bitreverse32((uint32_t)p) >> (32 - LOG2N)); }

// one radix-2 DIT stage of half-size n on the thread's 16 values;
// `lb` is the bit of i that encodes the stage's position bit.
// `t` is laundered at every stage/exchange so the compiler recomputes the
// (cheap) per-thread positions instead of keeping hundreds of addresses live
// across the three transforms (that is what spilled).
__device__ __forceinline__ int fresh(int t) {
  asm volatile("" : "+v"(t));
  return t;
}

// Twiddles of the stages n <= TW_LDS<LOG2N> come from an LDS copy of the
// forward table (fewer L2 round trips per stage).  An inverse transform
// negates their imaginary parts: JFFT's inverse table is the forward one
// conjugated bit for bit (mirrored std::exp arguments, decode/jfft.cpp:41-53;
// tests/test_abi.py::test_twiddle_inverse_is_conjugate).
template <int LOG2N>
struct TwLds {
  static constexpr int N = LOG2N >= 14 ? 512 : 256;  // largest stage served from LDS
  static constexpr int LEN = 2 * N - 1;             // TW[0 .. 2N-2]
};

// twiddles of one stage's 8 butterflies (the values i with bit lb clear, in
// order).  epos(t, i) = epos(t, 0) | epos(0, i) with disjoint bits, so the
// index splits into a per-thread base plus a compile-time offset per value;
// duplicate indices (stages whose n spans fewer than 8 of the thread's
// butterflies) are the same load and fold away.
template <int LOG2N, int PH, bool INV>
__device__ __forceinline__ void tw_load(double2 (&w)[8], int t0, int lb, int n, const double2 *__restrict__ TW,
                                        const double2 *stw) {
  const int t = fresh(t0);
  const int wbase = n - 1 + (epos<LOG2N, PH>(t, 0) & (n - 1));
  int j = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    if (i & (1 << lb)) continue;
    const int widx = wbase + (epos<LOG2N, PH>(0, i) & (n - 1));
    if (n <= TwLds<LOG2N>::N) {
      w[j] = stw[widx];
      if (INV) w[j].y = -w[j].y;
    } else {
      w[j] = TW[widx];
    }
    ++j;
  }
}

// the stage's radix-2 DIT butterflies with JFFT's operand order
// (decode/jfft.cpp:176-204): y = w * x[il]; x[il] = x[i] - y; x[i] = x[i] + y
__device__ __forceinline__ void bfly(double2 (&x)[16], int lb, const double2 (&w)[8]) {
  int j = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    if (i & (1 << lb)) continue;
    const int il = i | (1 << lb);
    const double yr = w[j].x * x[il].x - w[j].y * x[il].y;
    const double yi = w[j].x * x[il].y + w[j].y * x[il].x;
    x[il].x = x[i].x - yr;
    x[il].y = x[i].y - yi;
    x[i].x = x[i].x + yr;
    x[i].y = x[i].y + yi;
    ++j;
  }
}

// one radix-2 DIT stage of half-size n on the thread's 16 values; `lb` is the
// bit of i that encodes the stage's position bit
template <int LOG2N, int PH, bool INV>
__device__ __forceinline__ void stage(double2 (&x)[16], int t, int lb, int n, const double2 *__restrict__ TW,
                                      const double2 *stw) {
  double2 w[8];
  tw_load<LOG2N, PH, INV>(w, t, lb, n, TW, stw);
  bfly(x, lb, w);
}

// move values from layout PH_FROM to PH_TO through LDS (re then im);
// BR: the destination reads bit-reversed positions (start of a new transform)
template <int LOG2N, int PH_FROM, int PH_TO, bool BR>
__device__ __forceinline__ void exchange(double2 (&x)[16], int t0, double *lds) {
#pragma unroll
  for (int part = 0; part < 2; ++part) {
    const int t = fresh(t0);
    // pad(A | B) = pad(A) + pad(B) for bit-disjoint A = epos(t, 0), B = epos(0, i)
    // (bit reversal permutes bits, so it keeps them disjoint): one base address
    // per thread, the per-value part is an immediate offset
    double *wb = lds + xpad<PH_FROM, PH_TO, BR>(epos<LOG2N, PH_FROM>(t, 0));
    int rp = epos<LOG2N, PH_TO>(t, 0);
    if (BR) rp = bitrev<LOG2N>(rp);
    const double *rb = lds + xpad<PH_FROM, PH_TO, BR>(rp);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 16; ++i) wb[xpad<PH_FROM, PH_TO, BR>(epos<LOG2N, PH_FROM>(0, i))] = part ? x[i].y : x[i].x;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      int p = epos<LOG2N, PH_TO>(0, i);
      if (BR) p = bitrev<LOG2N>(p);
      const double v = rb[xpad<PH_FROM, PH_TO, BR>(p)];
      if (part)
        x[i].y = v;
      else
        x[i].x = v;
    }
  }
}

// copy of the forward twiddles the LDS-served stages use (all threads call it)
template <int L>
__device__ __forceinline__ void load_tw_lds(double2 *stw, const double2 *__restrict__ TW, int t, int nthreads) {
  for (int j = t; j < TwLds<L>::LEN; j += nthreads) stw[j] = TW[j];
}

// A stage of register phase 0: epos(t, i) = (t << 4) | i, so the twiddle
// index k = i & (n - 1) is a compile-time constant per value and the k == 0
// butterflies (twiddle TW[n - 1] = exp(0) = (1, +-0) exactly) skip the
// multiply: 1*x - (+-0)*y == x for every nonzero x, so the results differ
// from JFFT's at most in the sign of an exact zero, which no later add,
// product, hypot or square can turn into a different nonzero value.
template <int LOG2N, bool INV, int LB>
__device__ __forceinline__ void stage0(double2 (&x)[16], int t0, const double2 *__restrict__ TW,
                                       const double2 *stw) {
  constexpr int n = 1 << LB;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    if (i & n) continue;
    const int il = i | n;
    const int k = i & (n - 1);
    double yr, yi;
    if (k == 0) {
      yr = x[il].x;
      yi = x[il].y;
    } else {
      double2 w = stw[n - 1 + k];  // n <= 8: the LDS copy of the forward table
      if (INV) w.y = -w.y;
      yr = w.x * x[il].x - w.y * x[il].y;
      yi = w.x * x[il].y + w.y * x[il].x;
    }
    x[il].x = x[i].x - yr;
    x[il].y = x[i].y - yi;
    x[i].x = x[i].x + yr;
    x[i].y = x[i].y + yi;
  }
}

// full JFFT::fft on values already loaded in bit-reversed order in layout 0;
// leaves the natural-order result in layout 3 (4096 points: layout 2, which
// is epos<12, 3> as well).  TW: this direction's table;
// stw: LDS copy of the forward table's first TwLds<L>::LEN entries.
// SKIP1: skip the exact-(1, +-0) twiddle multiplies of phase 0 (stage0);
// only for callers whose outputs are magnitudes / squares (coarse.hip), as
// the sign of an exact zero may differ from JFFT's.
template <int L, bool INV, bool SKIP1 = false>
__device__ __forceinline__ void fft_dit(double2 (&x)[16], int t, double *lds, const double2 *__restrict__ TW,
                                        const double2 *stw) {
  static_assert(L == 12 || L == 13 || L == 14, "register phases cover 12, 13 or 14 stages");
  if (SKIP1) {
    stage0<L, INV, 0>(x, t, TW, stw);
    stage0<L, INV, 1>(x, t, TW, stw);
    stage0<L, INV, 2>(x, t, TW, stw);
    stage0<L, INV, 3>(x, t, TW, stw);
  } else {
    stage<L, 0, INV>(x, t, 0, 1, TW, stw);
    stage<L, 0, INV>(x, t, 1, 2, TW, stw);
    stage<L, 0, INV>(x, t, 2, 4, TW, stw);
    stage<L, 0, INV>(x, t, 3, 8, TW, stw);
  }
  exchange<L, 0, 1, false>(x, t, lds);
  stage<L, 1, INV>(x, t, 0, 16, TW, stw);
  stage<L, 1, INV>(x, t, 1, 32, TW, stw);
  stage<L, 1, INV>(x, t, 2, 64, TW, stw);
  stage<L, 1, INV>(x, t, 3, 128, TW, stw);
  // the stages past TwLds read their twiddles from L2: each stage's loads are
  // issued one stage (or one LDS exchange) ahead of its butterflies, so their
  // latency overlaps work instead of stalling every wave of the workgroup
  double2 wa[8], wb[8];
  if (L == 14) {
    tw_load<L, 2, INV>(wa, t, 2, 1024, TW, stw);
    exchange<L, 1, 2, false>(x, t, lds);
    stage<L, 2, INV>(x, t, 0, 256, TW, stw);
    stage<L, 2, INV>(x, t, 1, 512, TW, stw);
    tw_load<L, 2, INV>(wb, t, 3, 2048, TW, stw);
    bfly(x, 2, wa);
    bfly(x, 3, wb);
    tw_load<L, 3, INV>(wa, t, 0, 4096, TW, stw);
    exchange<L, 2, 3, false>(x, t, lds);
    tw_load<L, 3, INV>(wb, t, 1, 8192, TW, stw);
    bfly(x, 0, wa);
    bfly(x, 1, wb);
  } else if (L == 12) {
    tw_load<L, 2, INV>(wa, t, 1, 512, TW, stw);
    exchange<L, 1, 2, false>(x, t, lds);
    stage<L, 2, INV>(x, t, 0, 256, TW, stw);
    tw_load<L, 2, INV>(wb, t, 2, 1024, TW, stw);
    bfly(x, 1, wa);
    tw_load<L, 2, INV>(wa, t, 3, 2048, TW, stw);
    bfly(x, 2, wb);
    bfly(x, 3, wa);
  } else {
    tw_load<L, 2, INV>(wa, t, 1, 512, TW, stw);
    exchange<L, 1, 2, false>(x, t, lds);
    stage<L, 2, INV>(x, t, 0, 256, TW, stw);
    tw_load<L, 2, INV>(wb, t, 2, 1024, TW, stw);
    bfly(x, 1, wa);
    tw_load<L, 2, INV>(wa, t, 3, 2048, TW, stw);
    bfly(x, 2, wb);
    tw_load<L, 3, INV>(wb, t, 0, 4096, TW, stw);
    bfly(x, 3, wa);
    exchange<L, 2, 3, false>(x, t, lds);
    bfly(x, 0, wb);
  }
}


}  // namespace aero
