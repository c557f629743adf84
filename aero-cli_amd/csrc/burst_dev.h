/*
 * burst_dev.h — device helpers shared by the burst kernels (burst.hip,
 * burst_msk.hip): WaveTable operations (decode/DSP.cpp:35-262, DSP.h:59-65),
 * qRound, glibc cexp of a pure imaginary argument and Delay<T>::update
 * (DSP.h:365-384) on time-major rings.
 */
#pragma once
#include <hip/hip_runtime.h>

#include "aero_math.h"
#include "burst_common.h"
#include "engine_common.h"

// The per-sample libm of the burst demods: glibc's hypot as it is (the
// wave-uniform branch-free form measured 1.5% slower here), atan2's
// branch-free main path over the global cij table.  AERO_X_BURST_LIBM
// (timing builds only, bit-identical results): 1 the wave-uniform hypot,
// 2 general atan2, 3 both.
#if defined(AERO_X_BURST_LIBM) && (AERO_X_BURST_LIBM == 1 || AERO_X_BURST_LIBM == 3)
#define B_HYPOT aero_hypot_w
#else
#define B_HYPOT aero_hypot
#endif
#if defined(AERO_X_BURST_LIBM) && AERO_X_BURST_LIBM >= 2
#define B_ATAN2(y, x) aero_atan2(y, x)
#else
#define B_ATAN2(y, x) aero_atan2_bf(y, x, aero_g_cij)
#endif

namespace aero {
namespace {

__device__ __forceinline__ int b_cis_index(double WTptr) {  // WaveTable::WTCISValue (DSP.cpp:81-88)
  int tint = (int)WTptr;
  if (tint >= WTSIZE) tint = 0;
  if (tint < 0) tint = WTSIZE - 1;
  return tint;
}

// The wrap loops below run their first iteration as a select and the rest
// behind a wave-uniform test (the same iterations in the same order: a peeled
// loop); a step never exceeds a wave, so the rest never runs in practice, and
// the divergent loop's exec-mask bookkeeping is gone from the per-sample path.
__device__ __forceinline__ void b_nco_next(double &ptr, double &step) {  // WTnextFrame (DSP.cpp:71-79)
  if (step < 0) step = 0;
  ptr += step;
  ptr = ((int)ptr) >= WTSIZE ? ptr - WTSIZE : ptr;
  if (__builtin_expect(__any(((int)ptr) >= WTSIZE), 0))
    while (((int)ptr) >= WTSIZE) ptr -= WTSIZE;
}

__device__ __forceinline__ void b_set_freq(double &freq, double &step, double f) {  // SetFreq (DSP.cpp:163-168)
  freq = f;
  if (freq < 0) freq = 0;
  // freq: 10500 +- 0.1 (st_osc), a multiple of 48000 / 32768 (trident decisions) or 0
  step = div_c((freq) * ((double)WTSIZE), 48000.0);
}

// fmod(x, 360.0) for the phases of the per-sample path: for 0 <= x < 1800
// by repeated subtraction, which is exact there (x and 360 are multiples of
// ulp(x), and each difference is no larger than x) and so equals fmod's
// exact remainder; otherwise fmod itself
__device__ __forceinline__ double b_fmod360(double x) {
  const bool in = x >= 0.0 && x < 1800.0;
  double r = x;
#pragma unroll
  for (int i = 0; i < 4; ++i) r = r >= 360.0 ? r - 360.0 : r;  // the loop's (at most 4) iterations
  if (__builtin_expect(__any(!in), 0)) r = in ? r : fmod(x, 360.0);
  return r;
}

__device__ __forceinline__ void b_set_phase_deg(double &ptr, double phase_deg) {  // SetPhaseDeg (DSP.cpp:177-187)
  phase_deg = b_fmod360(phase_deg);
  // fmod's remainder is above -360: the loop adds 360 at most once
  phase_deg = phase_deg < 0 ? phase_deg + 360.0 : phase_deg;
  ptr = (phase_deg / 360.0) * ((double)WTSIZE);
}
// SetPhaseDeg for a phase in [0, 1800) made of pointer values (the symbol-tone
// PLL's 4 x (360 q_ptr / W) + 144): the remainder is 0 or a multiple of
// ulp(144) >= 2^-45, inside div_c's contract
__device__ __forceinline__ void b_set_phase_deg_pos(double &ptr, double phase_deg) {
  phase_deg = b_fmod360(phase_deg);
  phase_deg = phase_deg < 0 ? phase_deg + 360.0 : phase_deg;
  ptr = div_c(phase_deg, 360.0) * ((double)WTSIZE);
}

__device__ __forceinline__ void b_advance(double &ptr, double frac) {  // AdvanceFractionOfWave (DSP.h:59-65)
  ptr += frac * WTSIZE;
  ptr = ptr >= WTSIZE ? ptr - WTSIZE : ptr;
  if (__builtin_expect(__any(ptr >= WTSIZE), 0))
    while (ptr >= WTSIZE) ptr -= WTSIZE;
  ptr = ptr < 0 ? ptr + WTSIZE : ptr;
  if (__builtin_expect(__any(ptr < 0), 0))
    while (ptr < 0) ptr += WTSIZE;
}

__device__ __forceinline__ int b_qround(double d) {  // qRound (Qt 5.9 qglobal.h:525)
  return d >= 0.0 ? int(d + 0.5) : int(d - double(int(d - 1)) + 0.5) + int(d - 1);
}

// std::exp(complex(0 * y, y)) as glibc's cexp returns it: (cos y, sin y), or
// (1, y) when |y| <= DBL_MIN, which is also sincos's value there (below 2^-27
// it returns (y, 1)): sincos alone, branch-free for the small arguments of the
// loop corrections (aero_sincos_bf)
__device__ __forceinline__ void b_cexp_i(double y, double &c, double &s) {
  aero_sincos_bf(y, s, c, aero_g_sincostab);
}

// PeakDetector's d3.findmaxpos (DSP.h:491-566): the position of the first
// maximum of a time-major ring of len slots, scanning from the oldest slot p
// (the next one written); 16 slots are loaded at a time so their round trips
// overlap instead of one per slot
__device__ __forceinline__ int pd3_findmaxpos(const double *ring, int C, int p, int len) {
  double maxval = ring[(size_t)p * C];
  int maxpos = 0;
  for (int i0 = 0; i0 < len; i0 += 16) {
    double v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      int q = p + i0 + k;
      if (q >= len) q -= len;
      v[k] = i0 + k < len ? ring[(size_t)q * C] : -1.7976931348623157e308;
    }
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (v[k] > maxval) {
        maxval = v[k];
        maxpos = i0 + k;
      }
  }
  return maxpos;
}

// Delay<T>::update (DSP.h:365-384) on a time-major ring with per-pointer weights
struct DlyRef {
  const double *w, *omw;
  const int *io;
  int size;
};
__device__ __forceinline__ double dly_update(double *ring, int C, int &p, const DlyRef &d, double sig) {
  ring[(size_t)p * C] = sig;
  const int io = d.io[p], in = io + 1 == d.size ? 0 : io + 1;
  const double older = ring[(size_t)io * C], newer = ring[(size_t)in * C];
  const double w = d.w[p], om = d.omw[p];
  p = p + 1 == d.size ? 0 : p + 1;
  return (w * newer + om * older);
}
__device__ __forceinline__ double2 dly_update2(double2 *ring, int C, int &p, const DlyRef &d, double2 sig) {
  ring[(size_t)p * C] = sig;
  const int io = d.io[p], in = io + 1 == d.size ? 0 : io + 1;
  const double2 older = ring[(size_t)io * C], newer = ring[(size_t)in * C];
  const double w = d.w[p], om = d.omw[p];
  p = p + 1 == d.size ? 0 : p + 1;
  return make_double2(w * newer.x + om * older.x, w * newer.y + om * older.y);
}

__device__ __forceinline__ DlyRef dref(const BurstTables &T, int k) { return {T.dw[k], T.domw[k], T.dio[k], T.dsize[k]}; }


// Delay<T>::update split in two so a sample's ring reads can all be issued
// before its stores: dly_pre reads the slots the update at write pointer p
// will read (older = p + 1, newer = p + 2 mod size, which the host checks
// against the reference's pointer arithmetic, burst_engine.hip) and the
// pointer's weights; dly_commit writes sig and returns the weighted sum.  On a
// 2-slot ring "newer" is the slot written now: its value is sig.
struct DlyPre {
  double w, om, older, newer;
  int next;
  bool newer_is_sig;
};
__device__ __forceinline__ DlyPre dly_pre(const double *ring, int C, int p, const DlyRef &d) {
  const int io = p + 1 == d.size ? 0 : p + 1, in = io + 1 == d.size ? 0 : io + 1;
  return {d.w[p], d.omw[p], ring[(size_t)io * C], ring[(size_t)in * C], io, in == p};
}
__device__ __forceinline__ double dly_commit(double *ring, int C, int &p, const DlyPre &r, double sig) {
  ring[(size_t)p * C] = sig;
  p = r.next;
  const double newer = r.newer_is_sig ? sig : r.newer;
  return (r.w * newer + r.om * r.older);
}
// The demodulator's short fractional delays (sizes 2..6) held in registers,
// h[i] = the value written i updates ago (h[0] the newest): the update
// shifts and returns w * h[N-2] + om * h[N-1], exactly dly_commit's
// w * newer + om * older (older = the slot after the write pointer, i.e.
// N-1 updates old; newer = N-2 updates old, the value just written when
// N == 2).  The weights are the same for every write pointer (checked on
// the host, burst_engine.hip).  dly_regs_load / dly_regs_store convert
// from / to the ring [N][C] with write pointer p (stored back with p = 0).
template <int N>
__device__ __forceinline__ double dly_reg(double (&h)[N], double w, double om, double sig) {
#pragma unroll
  for (int i = N - 1; i > 0; --i) h[i] = h[i - 1];
  h[0] = sig;
  return (w * h[N - 2] + om * h[N - 1]);
}
template <int N>
__device__ __forceinline__ void dly_regs_load(double (&h)[N], const double *ring, int C, int p) {
#pragma unroll
  for (int i = 0; i < N; ++i) h[i] = ring[(size_t)(((p - 1 - i) % N + N) % N) * C];
}
template <int N>
__device__ __forceinline__ void dly_regs_store(const double (&h)[N], double *ring, int C) {
#pragma unroll
  for (int i = 0; i < N; ++i) ring[(size_t)(N - 1 - i) * C] = h[i];
}

// the same for a complex delay
template <int N>
__device__ __forceinline__ double2 dly_reg2(double2 (&h)[N], double w, double om, double2 sig) {
#pragma unroll
  for (int i = N - 1; i > 0; --i) h[i] = h[i - 1];
  h[0] = sig;
  return make_double2(w * h[N - 2].x + om * h[N - 1].x, w * h[N - 2].y + om * h[N - 1].y);
}
template <int N>
__device__ __forceinline__ void dly_regs_load2(double2 (&h)[N], const double2 *ring, int C, int p) {
#pragma unroll
  for (int i = 0; i < N; ++i) h[i] = ring[(size_t)(((p - 1 - i) % N + N) % N) * C];
}
template <int N>
__device__ __forceinline__ void dly_regs_store2(const double2 (&h)[N], double2 *ring, int C) {
#pragma unroll
  for (int i = 0; i < N; ++i) ring[(size_t)(N - 1 - i) * C] = h[i];
}

struct DlyPre2 {
  double w, om;
  double2 older, newer;
  int next;
};
__device__ __forceinline__ DlyPre2 dly_pre2(const double2 *ring, int C, int p, const DlyRef &d) {
  const int io = p + 1 == d.size ? 0 : p + 1, in = io + 1 == d.size ? 0 : io + 1;
  return {d.w[p], d.omw[p], ring[(size_t)io * C], ring[(size_t)in * C], io};
}
__device__ __forceinline__ double2 dly_commit2(double2 *ring, int C, int &p, const DlyPre2 &r, double2 sig) {
  ring[(size_t)p * C] = sig;
  p = r.next;
  return make_double2(r.w * r.newer.x + r.om * r.older.x, r.w * r.newer.y + r.om * r.older.y);
}

// Delay<T>::update with an integer delay D on a ring of D + 1 slots: the
// weighting is exactly 0, and the reference's sum is kept literally
// (0 * newer + 1 * older) so signed zeros come out the same
__device__ __forceinline__ double dly_int(double *ring, int C, int &p, int size, int D, double sig) {
  ring[(size_t)p * C] = sig;
  int io = p - D;
  if (io < 0) io += size;
  const int in = io + 1 == size ? 0 : io + 1;
  const double older = ring[(size_t)io * C], newer = ring[(size_t)in * C];
  p = p + 1 == size ? 0 : p + 1;
  return (0.0 * newer + (1.0 - 0.0) * older);
}
__device__ __forceinline__ double2 dly_int2(double2 *ring, int C, int &p, int size, int D, double2 sig) {
  ring[(size_t)p * C] = sig;
  int io = p - D;
  if (io < 0) io += size;
  const int in = io + 1 == size ? 0 : io + 1;
  const double2 older = ring[(size_t)io * C], newer = ring[(size_t)in * C];
  p = p + 1 == size ? 0 : p + 1;
  return make_double2(0.0 * newer.x + (1.0 - 0.0) * older.x, 0.0 * newer.y + (1.0 - 0.0) * older.y);
}

}  // namespace
}  // namespace aero
