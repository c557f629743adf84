/*
 * fft_dit.h — JFFT's radix-2 decimation-in-time FFT (decode/jfft.cpp:114-212)
 * for one 8192- or 16384-point transform per workgroup of N/16 threads on
 * gfx950: 16 complex FP64 values per thread in registers, four register
 * phases of up to four stages with padded LDS transposes between them.  Every
 * butterfly uses the reference's operands and twiddle (TW[n - 1 + k]), so the
 * result is bit-identical to JFFT however the butterflies are scheduled.
 * Used by coarse.hip (coarse frequency estimate) and burst.hip (Hilbert
 * fast-FIR blocks, trident check).
 */
#pragma once
#include <hip/hip_runtime.h>

namespace aero {

__device__ __forceinline__ int pad(int p) { return p + (p >> 4); }

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

template <int LOG2N, int PH, bool INV>
__device__ __forceinline__ void stage(double2 (&x)[16], int t0, int lb, int n, const double2 *__restrict__ TW,
                                      const double2 *stw) {
  const int t = fresh(t0);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    if (i & (1 << lb)) continue;
    const int il = i | (1 << lb);
    const int pk = epos<LOG2N, PH>(t, i);
    const int widx = n - 1 + (pk & (n - 1));
    double2 w;
    if (n <= TwLds<LOG2N>::N) {
      w = stw[widx];
      if (INV) w.y = -w.y;
    } else {
      w = TW[widx];
    }
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
template <int LOG2N, int PH_FROM, int PH_TO, bool BR>
__device__ __forceinline__ void exchange(double2 (&x)[16], int t0, double *lds) {
#pragma unroll
  for (int part = 0; part < 2; ++part) {
    const int t = fresh(t0);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 16; ++i) lds[pad(epos<LOG2N, PH_FROM>(t, i))] = part ? x[i].y : x[i].x;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      int p = epos<LOG2N, PH_TO>(t, i);
      if (BR) p = bitrev<LOG2N>(p);
      const double v = lds[pad(p)];
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

// full JFFT::fft on values already loaded in bit-reversed order in layout 0;
// leaves the natural-order result in layout 3.  TW: this direction's table;
// stw: LDS copy of the forward table's first TwLds<L>::LEN entries.
template <int L, bool INV>
__device__ __forceinline__ void fft_dit(double2 (&x)[16], int t, double *lds, const double2 *__restrict__ TW,
                                        const double2 *stw) {
  static_assert(L == 13 || L == 14, "register phases cover 13 or 14 stages");
  stage<L, 0, INV>(x, t, 0, 1, TW, stw);
  stage<L, 0, INV>(x, t, 1, 2, TW, stw);
  stage<L, 0, INV>(x, t, 2, 4, TW, stw);
  stage<L, 0, INV>(x, t, 3, 8, TW, stw);
  exchange<L, 0, 1, false>(x, t, lds);
  stage<L, 1, INV>(x, t, 0, 16, TW, stw);
  stage<L, 1, INV>(x, t, 1, 32, TW, stw);
  stage<L, 1, INV>(x, t, 2, 64, TW, stw);
  stage<L, 1, INV>(x, t, 3, 128, TW, stw);
  exchange<L, 1, 2, false>(x, t, lds);
  stage<L, 2, INV>(x, t, 0, 256, TW, stw);
  stage<L, 2, INV>(x, t, 1, 512, TW, stw);
  stage<L, 2, INV>(x, t, 2, 1024, TW, stw);
  stage<L, 2, INV>(x, t, 3, 2048, TW, stw);
  exchange<L, 2, 3, false>(x, t, lds);
  stage<L, 3, INV>(x, t, 0, 4096, TW, stw);
  if (L == 14) stage<L, 3, INV>(x, t, 1, 8192, TW, stw);
}


}  // namespace aero
