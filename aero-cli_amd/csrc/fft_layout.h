/*
 * fft_layout.h — where each value of the coarse estimator's chained FFTs
 * lives (fft_chain.h), as plain constexpr index arithmetic shared by the
 * gfx950 kernel and the host model that checks it (tools/fft_chain_sim.cpp,
 * tests/test_fft_chain_sim.py).
 *
 * A 2^L-point JFFT (decode/jfft.cpp:114-212) runs on 2^(L-4) threads with 16
 * complex values each.  A value's "storage" index is
 *     S = i | lane << 4 | wave << 10      (i: register 0-15, lane 0-63)
 * i.e. storage bits 0-3 = register bits, 4-7 = lane bits 0-3 ("j"),
 * 8-9 = lane bits 4-5 ("h"), 10.. = wave bits.  The transform's array index
 * a (JFFT's index after its bit-reversal copy; stage s pairs a and a ^ 2^s)
 * is a bit permutation of S, the layout: for every array bit b, the storage
 * bit that holds it (4 bits per entry in a uint64_t).  A stage can run in
 * registers when its array bit sits in a register bit; the layout changes
 * move bits between storage classes:
 *
 *   START  stages 0-3 in registers
 *   WL     wave-local LDS transpose: register bit k <-> lane bit k (k < 4);
 *          stages 4-7
 *   PERM   v_permlane16_swap / v_permlane32_swap: lane bit 4 <-> register
 *          bit 2, lane bit 5 <-> register bit 3; stages 8-9
 *   G      workgroup LDS exchange: the wave bits (the last L-10 stages) into
 *          registers; stages 10..L-1
 *
 * Chaining: the next transform reads this one's output in bit-reversed
 * order, so its stage s works on this transform's array bit L-1-s.  G puts
 * the bits so that the next transform's START is where they already are
 * (registers: its stages 0-3 = this one's last four; lane bits 0-3: its
 * stages 4-7; lane bits 4-5: 8-9; wave bits: the rest), so no bit-reversal
 * pass is needed between the three transforms: one G exchange per transform.
 */
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define AERO_HD __host__ __device__
#else
#define AERO_HD
#endif

namespace aero {
namespace fftl {

constexpr int sb(uint64_t lay, int b) { return (int)((lay >> (4 * b)) & 15); }
constexpr uint64_t put(uint64_t lay, int b, int s) {
  return (lay & ~(15ull << (4 * b))) | ((uint64_t)s << (4 * b));
}

// START: the first transform holds array bits 0-3 in register bits 0-3, a
// chained one in register bits 3..0 (where the previous G left them)
template <int L>
constexpr uint64_t lay_start(bool first) {
  uint64_t a = 0;
  for (int k = 0; k < 4; k++) a = put(a, k, first ? k : 3 - k);
  for (int b = 4; b < L; b++) a = put(a, b, b);
  return a;
}
// WL: register bit k <-> lane bit k
template <int L>
constexpr uint64_t lay_wl(bool first) {
  uint64_t a = lay_start<L>(first);
  for (int b = 0; b < L; b++) {
    const int s = sb(a, b);
    if (s < 4)
      a = put(a, b, s + 4);
    else if (s < 8)
      a = put(a, b, s - 4);
  }
  return a;
}
// PERM: lane bit 4 (storage 8) <-> register bit 2, lane bit 5 (9) <-> 3
template <int L>
constexpr uint64_t lay_perm(bool first) {
  uint64_t a = lay_wl<L>(first);
  for (int b = 0; b < L; b++) {
    const int s = sb(a, b);
    if (s == 8)
      a = put(a, b, 2);
    else if (s == 9)
      a = put(a, b, 3);
    else if (s == 2)
      a = put(a, b, 8);
    else if (s == 3)
      a = put(a, b, 9);
  }
  return a;
}
// G: registers k = bit L-4+k, lane bits 0-3 = bits L-5..L-8, lane bits 4, 5 =
// bits L-9, L-10, wave bits = L-11..0: the next transform's START
template <int L>
constexpr uint64_t lay_g() {
  uint64_t a = 0;
  for (int k = 0; k < 4; k++) a = put(a, L - 4 + k, k);
  for (int k = 0; k < 4; k++) a = put(a, L - 5 - k, 4 + k);
  a = put(a, L - 9, 8);
  a = put(a, L - 10, 9);
  for (int k = 0; k < L - 10; k++) a = put(a, L - 11 - k, 10 + k);
  return a;
}

// the array-index bits a value's register index contributes
constexpr int areg(uint64_t lay, int L, int i) {
  int a = 0;
  for (int b = 0; b < L; b++)
    if (sb(lay, b) < 4 && ((i >> sb(lay, b)) & 1)) a |= 1 << b;
  return a;
}
// the array bits held by lanes and waves (as a mask)
constexpr int thread_mask(uint64_t lay, int L) {
  int m = 0;
  for (int b = 0; b < L; b++)
    if (sb(lay, b) >= 4) m |= 1 << b;
  return m;
}
// generic thread part (host model and the static checks of the kernel's
// closed forms below)
constexpr int athr_generic(uint64_t lay, int L, int t) {
  int a = 0;
  for (int b = 0; b < L; b++)
    if (sb(lay, b) >= 4 && ((t >> (sb(lay, b) - 4)) & 1)) a |= 1 << b;
  return a;
}

AERO_HD inline uint32_t brev32(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_bitreverse32(x);
#else
  uint32_t r = 0;
  for (int k = 0; k < 32; k++) r |= ((x >> k) & 1u) << (31 - k);
  return r;
#endif
}

enum Kind : int { K_START = 0, K_WL = 1, K_PERM = 2, K_G = 3 };

// the thread part of the array index in closed form (a few integer ops per
// layout change; == athr_generic, checked by tools/fft_chain_sim.cpp)
template <int L, int KIND, bool FIRST>
AERO_HD inline int athr(int t) {
  const int j = FIRST ? (t & 15) : (int)(brev32((uint32_t)(t & 15)) >> 28);
  if (KIND == K_START) return t << 4;
  if (KIND == K_WL) return j | ((t >> 4) << 8);
  if (KIND == K_PERM) return j | (((t >> 4) & 3) << 6) | ((t >> 6) << 10);
  return (int)(brev32((uint32_t)t) >> (32 - (L - 4)));
}

// LDS maps (doubles).  G exchange: array index -> slot, one pad per 32: the
// writers (16-lane groups over array bits 0-3) and the readers (32-lane
// groups over array bits L-5..L-9) are conflict-free; additive over disjoint
// bits, so a thread's slot is a base plus a per-register immediate.
AERO_HD constexpr int gidx(int a) { return a + (a >> 5); }
// WL transpose within a wave's 1088-double region: lane (h, j), register i
// writes [h][j][i] (rows of 17) and reads [h][i][j]; 16-lane write groups hit
// 16 distinct double-banks, 32-lane read groups all 64 banks
constexpr int WL_REGION = 1088;
AERO_HD constexpr int wl_w(int lane, int i) { return (lane >> 4) * 272 + (lane & 15) * 17 + i; }
AERO_HD constexpr int wl_r(int lane, int i) { return (lane >> 4) * 272 + i * 17 + (lane & 15); }
// the |X| bins after the last transform: lanes hold bin bits 4..9 (G
// layout), one pad per 64 keeps the 16-lane store groups on distinct banks
// the coarse kernel's |X| / y history in LDS: one pad double per 2^S
template <int S>
AERO_HD constexpr int ypadn(int q) { return q + (q >> S); }

// The L2-served stages of the G layout (S >= 10, past the LDS twiddle copy)
// read their twiddles from a copy permuted into the threads' order
// (DevTables::twg / twgi): row r of stage S holds, for every thread t in
// turn, the twiddle TW[n - 1 + ((athr_G(t) | r << (L - 4)) & (n - 1))] of
// the thread's butterflies whose register part of the array index below bit
// S is r << (L - 4).  A wave's load of one row is then one contiguous run
// instead of 64 lines (the G layout's lanes hold bit-reversed index bits).
template <int L>
AERO_HD constexpr int twg_rows(int S) {
  return 1 << (S - (L - 4));
}
template <int L>
AERO_HD constexpr int twg_base(int S) {
  int b = 0;
  for (int s = 10; s < S; s++) b += twg_rows<L>(s);
  return b;
}
template <int L>
AERO_HD constexpr int twg_row(int S, int i) {
  return (areg(lay_g<L>(), L, i) & ((1 << S) - 1)) >> (L - 4);
}
// the permuted table of one direction from JFFT's (tw: [2^L] complex as re, im pairs)
template <int L>
inline void twg_build(const double *tw, double *twg) {
  constexpr int FT = 1 << (L - 4);
  for (int S = 10; S < L; S++) {
    const int n = 1 << S;
    for (int r = 0; r < twg_rows<L>(S); r++)
      for (int t = 0; t < FT; t++) {
        const int k = n - 1 + ((athr<L, K_G, false>(t) | (r << (L - 4))) & (n - 1));
        const size_t o = (size_t)(twg_base<L>(S) + r) * FT + t;
        twg[2 * o] = tw[2 * k];
        twg[2 * o + 1] = tw[2 * k + 1];
      }
  }
}
static_assert(twg_base<14>(14) == 15 && twg_base<13>(13) == 14, "permuted twiddle rows");

// static checks of the closed forms for the two transform sizes in use
template <int L, int KIND, bool FIRST>
constexpr bool athr_ok() {
  const uint64_t lay = KIND == K_START ? lay_start<L>(FIRST)
                                       : KIND == K_WL ? lay_wl<L>(FIRST) : KIND == K_PERM ? lay_perm<L>(FIRST) : lay_g<L>();
  for (int t = 0; t < (1 << (L - 4)); t++) {
    const int j = FIRST ? (t & 15) : (((t & 1) << 3) | ((t & 2) << 1) | ((t & 4) >> 1) | ((t & 8) >> 3));
    int c = 0;
    if (KIND == K_START)
      c = t << 4;
    else if (KIND == K_WL)
      c = j | ((t >> 4) << 8);
    else if (KIND == K_PERM)
      c = j | (((t >> 4) & 3) << 6) | ((t >> 6) << 10);
    else {
      c = 0;
      for (int k = 0; k < L - 4; k++) c |= ((t >> k) & 1) << (L - 5 - k);
    }
    if (c != athr_generic(lay, L, t)) return false;
  }
  return true;
}
static_assert(athr_ok<14, K_START, true>(), "fft layout closed form");
static_assert(athr_ok<14, K_WL, true>(), "fft layout closed form");
static_assert(athr_ok<14, K_PERM, true>(), "fft layout closed form");
static_assert(athr_ok<14, K_START, false>(), "fft layout closed form");
static_assert(athr_ok<14, K_WL, false>(), "fft layout closed form");
static_assert(athr_ok<14, K_PERM, false>(), "fft layout closed form");
static_assert(athr_ok<14, K_G, false>(), "fft layout closed form");
static_assert(athr_ok<13, K_START, true>(), "fft layout closed form");
static_assert(athr_ok<13, K_WL, true>(), "fft layout closed form");
static_assert(athr_ok<13, K_PERM, true>(), "fft layout closed form");
static_assert(athr_ok<13, K_START, false>(), "fft layout closed form");
static_assert(athr_ok<13, K_WL, false>(), "fft layout closed form");
static_assert(athr_ok<13, K_PERM, false>(), "fft layout closed form");
static_assert(athr_ok<13, K_G, false>(), "fft layout closed form");
// G leaves the next transform's START: its array bit s = this one's L-1-s
template <int L>
constexpr bool chain_ok() {
  for (int s = 0; s < L; s++)
    if (sb(lay_g<L>(), L - 1 - s) != sb(lay_start<L>(false), s)) return false;
  return true;
}
static_assert(chain_ok<14>() && chain_ok<13>(), "G layout == next START");

}  // namespace fftl
}  // namespace aero
