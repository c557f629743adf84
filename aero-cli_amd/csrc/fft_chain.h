/*
 * fft_chain.h — the coarse estimator's three chained JFFT transforms
 * (forward, inverse, forward: decode/coarsefreqestimate.cpp:134-160, JFFT
 * decode/jfft.cpp:114-212) for one 2^L-point channel-hop per workgroup of
 * 2^(L-4) threads on gfx950, 16 complex FP64 values per thread.
 *
 * Where the values live between stages is fft_layout.h (checked on the CPU
 * by tools/fft_chain_sim.cpp).  Per transform: four stages in registers, a
 * wave-local LDS transpose (no workgroup barrier: each wave uses its own
 * region, LDS operations of one wave execute in order), four stages,
 * v_permlane16_swap / v_permlane32_swap (no LDS at all), two stages, one
 * workgroup exchange through LDS for the wave bits (the only barriers), the
 * last L-10 stages.  The next transform starts where this one ends (it reads
 * the output in bit-reversed order, which is a relabelling of the bits), so
 * the chain of three needs three workgroup exchanges in all.
 *
 * Every butterfly takes JFFT's operands and twiddle TW[n - 1 + (a & (n - 1))]
 * for array index a, in JFFT's operation order, so each value is the
 * reference's bit for bit; the only liberty is the exact (1, +-0) twiddle of
 * the stages whose low array bits are all in registers (k == 0), whose
 * product is skipped (only the sign of an exact zero can differ).
 */
#pragma once
#include <hip/hip_runtime.h>

#include "fft_dit.h"  // TwLds, load_tw_lds
#include "fft_layout.h"

namespace aero {
namespace chain {

using namespace fftl;

// the twiddles of one stage's 8 butterflies (the values i with bit rb clear,
// in order); identical indices fold into one load.  Stages n <= TwLds<L>::N
// read the LDS copy of the forward table (an inverse negates the imaginary
// part: JFFT's inverse table is the forward one conjugated bit for bit,
// tests/test_abi.py::test_twiddle_inverse_is_conjugate); the later stages,
// all in the G layout, this direction's permuted copy TWG (fft_layout.h
// twg_build: one contiguous run per wave and row).
template <int L, uint64_t LAY, int S, bool INV>
__device__ __forceinline__ void tw_fetch(double2 (&w)[8], int athr_v, const double2 *__restrict__ TW,
                                         const double2 *stw, const double2 *__restrict__ TWG, int t) {
  constexpr int rb = sb(LAY, S), n = 1 << S, FT = 1 << (L - 4);
  constexpr bool lds_tw = n <= TwLds<L>::N;
  if constexpr (!lds_tw && LAY == lay_g<L>()) {
    // the laundered index keeps the compiler from computing every stage's
    // address up front and holding them all (that spills)
    const double2 *base = TWG + twg_base<L>(S) * FT + fresh(t);
    int j = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if (i & (1 << rb)) continue;
      w[j] = base[twg_row<L>(S, i) * FT];
      ++j;
    }
  } else {
    const double2 *base = (lds_tw ? stw : TW) + (n - 1) + (fresh(athr_v) & (n - 1));
    int j = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if (i & (1 << rb)) continue;
      w[j] = base[areg(LAY, L, i) & (n - 1)];
      if (lds_tw && INV) w[j].y = -w[j].y;
      ++j;
    }
  }
}

// JFFT's butterflies (decode/jfft.cpp:176-204): y = w x[il]; x[il] = x[i] - y;
// x[i] = x[i] + y; the product skipped where the twiddle is the exact TW[n-1]
template <int L, uint64_t LAY, int S>
__device__ __forceinline__ void bfly(double2 (&x)[16], const double2 (&w)[8]) {
  constexpr int rb = sb(LAY, S), n = 1 << S;
  constexpr bool thread_low = (thread_mask(LAY, L) & (n - 1)) != 0;
  int j = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    if (i & (1 << rb)) continue;
    const int il = i | (1 << rb);
    double yr, yi;
    if (!thread_low && (areg(LAY, L, i) & (n - 1)) == 0) {
      yr = x[il].x;
      yi = x[il].y;
    } else {
      yr = w[j].x * x[il].x - w[j].y * x[il].y;
      yi = w[j].x * x[il].y + w[j].y * x[il].x;
    }
    x[il].x = x[i].x - yr;
    x[il].y = x[i].y - yi;
    x[i].x = x[i].x + yr;
    x[i].y = x[i].y + yi;
    ++j;
  }
}

template <int L, uint64_t LAY, int S, bool INV>
__device__ __forceinline__ void stage(double2 (&x)[16], int athr_v, const double2 *__restrict__ TW,
                                      const double2 *stw) {
  double2 w[8];
  tw_fetch<L, LAY, S, INV>(w, athr_v, TW, stw, nullptr, 0);
  bfly<L, LAY, S>(x, w);
}

// v, laundered after the current value of x[0] (an ordering edge for the scheduler)
__device__ __forceinline__ int after(int v, double2 (&x)[16]) {
  asm volatile("" : "+v"(v), "+v"(x[0].x));
  return v;
}

// every value materialised here: no butterfly sinks past this point into the
// code after the transform (which raised the register pressure there)
__device__ __forceinline__ void pin(double2 (&x)[16]) {
#pragma unroll
  for (int i = 0; i < 16; ++i) asm volatile("" : "+v"(x[i].x), "+v"(x[i].y));
}

__device__ __forceinline__ void lds_fence() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// WL: register bit k <-> lane bit k (k < 4) through the wave's own LDS
// region, re then im; no workgroup barrier
__device__ __forceinline__ void wl(double2 (&x)[16], double *lds, int t) {
  t = fresh(t);
  const int lane = t & 63;
  double *base = lds + (t >> 6) * WL_REGION;
  double *wp = base + wl_w(lane, 0);
  const double *rp = base + wl_r(lane, 0);
#pragma unroll
  for (int part = 0; part < 2; ++part) {
#pragma unroll
    for (int i = 0; i < 16; ++i) wp[i] = part ? x[i].y : x[i].x;
    lds_fence();
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const double v = rp[i * 17];
      if (part)
        x[i].y = v;
      else
        x[i].x = v;
    }
    lds_fence();
  }
}

__device__ __forceinline__ uint64_t bits(double d) { return (uint64_t)__double_as_longlong(d); }
__device__ __forceinline__ double dbl(uint32_t lo, uint32_t hi) {
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
// v_permlane16_swap(vdst = a, src = b): rows 1, 3 of a <-> rows 0, 2 of b
__device__ __forceinline__ void pl16(double &a, double &b) {
  const uint64_t ua = bits(a), ub = bits(b);
  const auto lo = __builtin_amdgcn_permlane16_swap((uint32_t)ua, (uint32_t)ub, false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap((uint32_t)(ua >> 32), (uint32_t)(ub >> 32), false, false);
  a = dbl(lo[0], hi[0]);
  b = dbl(lo[1], hi[1]);
}
// v_permlane32_swap(vdst = a, src = b): lanes 32-63 of a <-> lanes 0-31 of b
__device__ __forceinline__ void pl32(double &a, double &b) {
  const uint64_t ua = bits(a), ub = bits(b);
  const auto lo = __builtin_amdgcn_permlane32_swap((uint32_t)ua, (uint32_t)ub, false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap((uint32_t)(ua >> 32), (uint32_t)(ub >> 32), false, false);
  a = dbl(lo[0], hi[0]);
  b = dbl(lo[1], hi[1]);
}
// PERM: lane bit 4 <-> register bit 2, lane bit 5 <-> register bit 3
__device__ __forceinline__ void perm(double2 (&x)[16]) {
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if (!(i & 4)) {
      pl16(x[i].x, x[i | 4].x);
      pl16(x[i].y, x[i | 4].y);
    }
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if (!(i & 8)) {
      pl32(x[i].x, x[i | 8].x);
      pl32(x[i].y, x[i | 8].y);
    }
}

// G: the workgroup exchange PERM -> G layout through LDS (re, then im);
// ends with a barrier so every wave has read before LDS is reused
template <int L, bool FIRST>
__device__ __forceinline__ void gx(double2 (&x)[16], double *lds, int t) {
  constexpr uint64_t P = lay_perm<L>(FIRST), G = lay_g<L>();
  t = fresh(t);
  double *wb = lds + gidx(athr<L, K_PERM, FIRST>(t));
  const double *rb = lds + gidx(athr<L, K_G, false>(t));
#pragma unroll
  for (int part = 0; part < 2; ++part) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 16; ++i) wb[gidx(areg(P, L, i))] = part ? x[i].y : x[i].x;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const double v = rb[gidx(areg(G, L, i))];
      if (part)
        x[i].y = v;
      else
        x[i].x = v;
    }
  }
  __syncthreads();
}

// one transform from its START layout to the G layout (the next one's START).
// TW: this direction's global table; stw: LDS copy of the forward table's
// first TwLds<L>::LEN entries; TWG: this direction's permuted copy for the
// stages after G.  Those twiddles are fetched before the exchange / one
// stage ahead.
template <int L, bool FIRST, bool INV>
__device__ __forceinline__ void fft(double2 (&x)[16], int t, double *lds, const double2 *__restrict__ TW,
                                    const double2 *stw, const double2 *__restrict__ TWG) {
  constexpr uint64_t S0 = lay_start<L>(FIRST), W = lay_wl<L>(FIRST), P = lay_perm<L>(FIRST), G = lay_g<L>();
  const int a0 = athr<L, K_START, FIRST>(t);
  stage<L, S0, 0, INV>(x, a0, TW, stw);
  stage<L, S0, 1, INV>(x, a0, TW, stw);
  stage<L, S0, 2, INV>(x, a0, TW, stw);
  stage<L, S0, 3, INV>(x, a0, TW, stw);
  wl(x, lds, t);
  const int a1 = athr<L, K_WL, FIRST>(t);
  stage<L, W, 4, INV>(x, a1, TW, stw);
  stage<L, W, 5, INV>(x, a1, TW, stw);
  stage<L, W, 6, INV>(x, a1, TW, stw);
  stage<L, W, 7, INV>(x, a1, TW, stw);
  perm(x);
  const int a2 = athr<L, K_PERM, FIRST>(t);
  stage<L, P, 8, INV>(x, a2, TW, stw);
  stage<L, P, 9, INV>(x, a2, TW, stw);
  const int a3 = athr<L, K_G, false>(t);
  double2 wa[8], wb[8];
  tw_fetch<L, G, 10, INV>(wa, a3, TW, stw, TWG, t);
  tw_fetch<L, G, 11, INV>(wb, a3, TW, stw, TWG, t);
  gx<L, FIRST>(x, lds, t);
  bfly<L, G, 10>(x, wa);
  // each later fetch is tied to the butterflies before it, so the scheduler
  // cannot issue all four stages' global twiddles at once (that spills)
  tw_fetch<L, G, 12, INV>(wa, after(a3, x), TW, stw, TWG, after(t, x));
  bfly<L, G, 11>(x, wb);
  if (L == 14) tw_fetch<L, G, (L == 14 ? 13 : 12), INV>(wb, after(a3, x), TW, stw, TWG, after(t, x));
  bfly<L, G, 12>(x, wa);
  if (L == 14) bfly<L, G, (L == 14 ? 13 : 12)>(x, wb);
  pin(x);
}

// natural (output) index of value i after a transform (G layout)
template <int L>
__device__ __forceinline__ int out_bin_thread(int t) {
  return athr<L, K_G, false>(t);
}
template <int L>
constexpr int out_bin_reg(int i) {
  return areg(lay_g<L>(), L, i);
}

}  // namespace chain
}  // namespace aero
