/*
 * demod_oqpsk.hip — batched continuous 10500-bps OQPSK demodulator for
 * gfx950.  One VFO channel per lane; a channel's per-sample recurrence
 * (OqpskDemodulator::writeData, decode/oqpskdemodulator.cpp:284-560) runs
 * sequentially in its lane, thousands of channels run side by side.
 *
 * Bit-exactness rules: built with -ffp-contract=off; every
 * expression keeps the reference's operation order; std::complex products
 * are expanded as GCC does ((ac-bd), (ad+bc)); libm calls go to aero_math.h.
 *
 * One lane per channel, two waves per 64 channels on one SIMD: the chain
 * wave runs the per-sample recurrence; its helper, the FIR wave, keeps the
 * 55-tap RRC's transposed partial sums R_0..R_53 (60 in registers, 48 in
 * LDS) and updates them from the mixed samples the chain publishes in LDS,
 * handing R_53 back first so only R_54's update stays on the chain
 * (demod_fir_wave; the sequence-word protocol at DemodShared).  Each wave
 * fits the 256 VGPRs of two waves per SIMD.
 *
 * Segment contract: a launch advances every channel from nsamp up to (but
 * excluding) its next coarse-estimate hop sample, or to the pushed end; it
 * also writes the coarse-ring entry of the sample after each processed one
 * (ring fill precedes the hop that uses it, oqpskdemodulator.cpp:351-369).
 */
#include <hip/hip_runtime.h>

#include <climits>

#include "aero_math.h"
#include "engine_common.h"

namespace aero {

// Timing experiment only (never in the product build): AERO_X_OCML swaps the
// bit-exact libm for the device ocml one, to price exactness.
#ifdef AERO_X_OCML
#define DM_HYPOT ::hypot
#define DM_ATAN2 ::atan2
#define DM_TANH ::tanh
#define DM_SINCOS(x, s, c) ::sincos(x, &(s), &(c))
#else
#define DM_HYPOT aero_hypot_w
#define DM_ATAN2(y, x) aero_atan2_bf(y, x, sh.cij)
#define DM_TANH aero_tanh_bf
#define DM_SINCOS(x, s, c) aero_sincos_bf(x, s, c, sh.sct)
#endif
// AERO_X_DROP (diagnostic builds only, never bit-exact): leave out one
// buffer's HBM accesses to attribute the demod's PMC traffic buffer by buffer
// (scripts/pmc_demod_buffers.sh): 1 coarse-ring writes, 2 soft-bit writes,
// 4 the carrier event's rings (marg, dt, MSEcalc), 8 the AGC ring
#ifndef AERO_X_DROP
#define AERO_X_DROP 0
#endif
#define DM_DIVC(a, c) ((a) / (c))

// AERO_X_STAMPS (diagnostic build only): s_memtime cycle totals per loop
// section of wave 0 of workgroup 0, with scheduling barriers at the stamps
#ifdef AERO_X_STAMPS
__device__ unsigned long long g_stamps[8];
#define XSTAMP(k)                                         \
  do {                                                    \
    __builtin_amdgcn_sched_barrier(0);                    \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    xstamp_[k] += t_ - xtime_;                                     \
    xtime_ = t_;                                          \
    __builtin_amdgcn_sched_barrier(0);                    \
  } while (0)
#else
#define XSTAMP(k) \
  do {            \
  } while (0)
#endif

__constant__ double c_taps[NTAPS];
__constant__ DelayDesc c_dly[4];  // delays(1), delayt41(T/4), delayt42(T/4), delayt8(T/8)
__constant__ double c_sr_b[3];    // st resonator (oqpskdemodulator.cpp:218-223)
__constant__ double c_sr_a[3];
__constant__ double c_ct_b[3];    // carrier loop filter (oqpskdemodulator.cpp:92-99)
__constant__ double c_ct_a[3];

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

__device__ __forceinline__ void set_freq(double &freq, double &step, double f) {  // SetFreq (DSP.cpp:163-168)
  freq = f;
  if (freq < 0) freq = 0;
  step = DM_DIVC((freq) * ((double)WTSIZE), 48000.0);
}
// the same for st_osc, whose frequency stays within 10500 +- 0.1 (+ one
// nudge of at most pi 1e-8): the short exact division (aero_math.h div_c)
__device__ __forceinline__ void set_freq_st(double &freq, double &step, double f) {
  freq = f;
  if (freq < 0) freq = 0;
  step = div_c((freq) * ((double)WTSIZE), 48000.0);
}

// Delay<double>::update (DSP.h:365-384) as a shift register: h[0] is the
// newest sample.  The reference reads the ring at fixed ages behind its
// write pointer and weights them with per-pointer weights; at 48 kHz /
// 10500 bps the ages are compile-time constants and the weights do not
// depend on the pointer (engine.hip checks both at engine creation), so
// only the cells up to the oldest age read are kept.
template <int N, int AGE_OLD, int AGE_NEW>
__device__ __forceinline__ double delay_tap(double (&h)[N], const DelayDesc &d, double sig) {
  static_assert(AGE_OLD < N + 1 && AGE_NEW < N + 1, "ring ages");
#pragma unroll
  for (int i = N - 1; i > 0; --i) h[i] = h[i - 1];
  h[0] = sig;
  const double w = d.w[0], omw = d.omw[0];  // uniform: scalar loads
  return (w * h[AGE_NEW] + omw * h[AGE_OLD]);
}

// IIR::update with 3 b / 3 a coefficients (DSP.cpp:635-685), a[0] == 1
__device__ __forceinline__ double iir3(double &x1, double &x2, double &y1, double &y2, const double *b,
                                       const double *a, double sig) {
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

__device__ __forceinline__ int qround(double d) {  // qRound (Qt 5.9 qglobal.h:525)
  return d >= 0.0 ? int(d + 0.5) : int(d - double(int(d - 1)) + 0.5) + int(d - 1);
}

// carrier-step state kept in LDS (read and written once per carrier event,
// i.e. once per ~9 samples)
enum { PD_CTX1, PD_CTX2, PD_CTY1, PD_CTY2, PD_MARG_SUM, PD_PM_SUM, PD_MS_SUM, PD_MSE, PD_PTD_RE, PD_PTD_IM,
       PD_M2_FREQ, PD_N };
enum { PI_MARG_P, PI_DT_P, PI_PM_P, PI_MS_P, PI_N, PI_TICK = PI_N, PI_DTW0, PI_PMW0, PI_MGW0, PI_ALL };
enum { PL_SOFTP, PL_PTN, PL_N };

constexpr int DEMOD_BLOCK = 256;  // channels per workgroup
// Two waves per channel group: waves 0-3 run the per-sample chain of the
// block's 256 channels, waves 4-7 the RRC partial-sum update of the same
// channels (wave w + 4 serves wave w; the dispatcher places them on the same
// SIMD, tools/wave_place.hip)
constexpr int DEMOD_THREADS = 2 * DEMOD_BLOCK;
// coarse-ring entries staged per channel before one 32-byte write
constexpr int RING_GROUP = 8;
// chain -> FIR sequence word: iterations published, | CSEQ_DONE at the end
constexpr int CSEQ_DONE = 1 << 30;
// a wait that never ends (a broken hand-off) gives up after ~2^24 polls
// (about a second) instead of hanging the GPU, and raises the group's device
// error word: aero_run then fails with AERO_E_DEVICE instead of delivering
// the garbage the run produced.  AERO_X_HANDOFF_FAIL (diagnostic build only,
// tests/test_gpu_handoff.py) breaks the hand-off on purpose: the FIR waves
// return at once and the chain waves' wait gives up after 2^12 polls.
#ifdef AERO_X_HANDOFF_FAIL
constexpr int SPIN_LIMIT = 1 << 12;
#else
constexpr int SPIN_LIMIT = 1 << 24;
#endif

__device__ __forceinline__ void raise_device_error(const DevState &S, int code) {
  if (S.err) __hip_atomic_store(S.err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// AeroL's 1 s DCD QTimer on the sample clock (AERO_F_DCD_TICK): tick k fires
// after the first (k + 1) * Fs samples.  The framing must apply it after the
// soft bits delivered up to then and before the next ones, so the demod
// records, at its first carrier event of a sample >= the tick's (events come
// every ~9 samples; soft bits only at events), how many soft bits AeroL had
// received: groups of 32 (oqpskdemodulator.cpp:534-540).  The next tick's
// sample relative to the launch's first sample, or INT_MAX:
__device__ __forceinline__ int dcd_tick_rel(const DevState &S, int c, long long n0) {
  if (!S.dcd_tick) return INT_MAX;
  const long long d = (long long)(S.is[IS_TICK_REC * S.C + c] + 1) * 48000 - n0;
  return d < (long long)INT_MAX ? (int)d : INT_MAX;
}
__device__ __forceinline__ void dcd_tick_record(const DevState &S, int c, long long softp) {
  const int C = S.C;
  const int r = S.is[IS_TICK_REC * C + c];
  S.ls[(LS_TICK_SOFT0 + (r & (DCD_TICK_RING - 1))) * C + c] = softp & ~31LL;
  S.is[IS_TICK_REC * C + c] = r + 1;
}

// LDS ordering between the two waves of a pair: every LDS access issued
// before this has completed (the workgroup-scope release of the AMDGPU memory
// model, without the wait for outstanding global stores a release fence
// would add)
__device__ __forceinline__ void lds_release() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ int lds_load(const int *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// the LDS reads after a poll must not be hoisted above it (compiler barrier;
// the hardware returns a wave's LDS reads in order)
__device__ __forceinline__ void lds_acquire() { asm volatile("" ::: "memory"); }
__device__ __forceinline__ void lds_store(int *p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

constexpr int FIR_LDS_IM = 11, FIR_LDS_RE = 5;
// the carrier-event rings (dt, MSEcalc, marg) through LDS windows of
// DT_WIN / PM_WIN / MG_WIN events (the dt window holds one slot more: an
// event writes slot p and reads p + 1): one read and one write of the
// window's slots per window instead of a line fetched and written back per
// event
constexpr int DT_WIN = 4, PM_WIN = 4, MG_WIN = 4;

struct DemodShared {
  uint32_t ring[RING_GROUP][DEMOD_BLOCK];
  double pd[PD_N][DEMOD_BLOCK];
  long long pl[PL_N][DEMOD_BLOCK];
  int pi[PI_ALL][DEMOD_BLOCK];  // + PI_TICK: the next DCD tick's sample, relative to n0
  // chain -> FIR: the mixed sample of chain iteration it (slot it & 1) and
  // the lanes that produced one; FIR -> chain: R_53 after iteration it
  double2 x[2][DEMOD_BLOCK];
  double2 r53[2][DEMOD_BLOCK];
  unsigned long long mask[2][4];
  int cseq[4], fseq[4];
  // the FIR wave's oldest partial sums: imaginary R_0..R_10 and real
  // R_0..R_4 (the other 92 are registers; with the short division sequences
  // the kernel holds 227 VGPRs, and 4 sums fewer in LDS spill)
  double qil[FIR_LDS_IM][DEMOD_BLOCK];
  double qrl[FIR_LDS_RE][DEMOD_BLOCK];
  // the libm tables the chain gathers from every sample (atan2's cij rows,
  // sincos's __sincostab), copied from global memory once per launch: an
  // LDS gather instead of an L2 round trip on the per-sample chain
  double cij[241][7];
  double sct[440];
  // the soft-ring group (16 bytes) each channel is filling: written to the
  // ring as one 16-byte store when its last pair arrives, and at the end of
  // the launch (the group's earlier bytes are loaded at the start)
  uint32_t softw[4][DEMOD_BLOCK];
  double2 dtw[DT_WIN + 1][DEMOD_BLOCK];  // dt slots PI_DTW0 .. + DT_WIN
  double2 pmw[PM_WIN][DEMOD_BLOCK];      // MSEcalc slots PI_PMW0 .. + PM_WIN - 1
  double mgw[MG_WIN][DEMOD_BLOCK];       // marg slots PI_MGW0 .. + MG_WIN - 1
};

// dst += a (dst = a + b) for the lanes in m only, the rest keep dst: one
// EXEC-masked VALU op.  In C++ this is a divergent branch, and for values
// carried around the FIR loop the register allocator then keeps a second
// copy of every partial sum (the then- and bypass-values of the join), which
// does not fit; here the partial sum is updated in place.
__device__ __forceinline__ void add_masked(double &dst, double a, double b, unsigned long long m) {
  unsigned long long sv;
  asm volatile(
      "s_and_saveexec_b64 %0, %4\n\t"
      "v_add_f64 %1, %2, %3\n\t"
      "s_mov_b64 exec, %0"
      : "=&s"(sv), "+v"(dst)
      : "v"(a), "v"(b), "s"(m)
      : "scc");
}

// The RRC (FIR::FIRUpdateAndProcess, decode/DSP.cpp:290-304) in transposed
// form, R_j(n) = R_{j-1}(n-1) + h[j] x(n), j = 0..54: the filter output used
// at sample n is R_54(n-1), so only R_54's update is on the chain.  This wave
// holds R_0..R_53 of its 64 channels (real R_5..R_53 and imaginary
// R_11..R_53 in registers, the older ones in LDS) and, per chain iteration,
// takes the mixed samples the chain wave published, forms R_53 first and
// hands it back (the chain forms R_54 = R_53 + h[54] x itself), then updates
// the rest while the chain runs on.  h[j] == h[54 - j] bit for bit
// (host-checked), so the slots of a tap pair share one product; the
// additions are the reference's, term for term.  Lanes whose chain lane
// produced no sample in an iteration (waiting for their carrier event) keep
// their sums.
__device__ __forceinline__ void demod_fir_wave(const DevState &S, DemodShared &sh, int c, int pair, int wv,
                                               bool valid) {
  const int C = S.C;
  constexpr int NL = (NTAPS - 1) / 2;  // tap pairs k = 0..26, centre 27
  constexpr int NRL = FIR_LDS_RE, NIL = FIR_LDS_IM;
  // q[j]: R_j real (j >= NRL used); qi[j]: R_j imaginary (j >= NIL used)
  double q[NTAPS - 1], qi[NTAPS - 1];
  {
    // a lane past the last channel loads channel 0's sums (never used or stored)
    const double *fir = S.fir + (valid ? c : 0);
#pragma unroll
    for (int j = 0; j < NRL; ++j) sh.qrl[j][pair] = fir[(size_t)j * C];
#pragma unroll
    for (int j = NRL; j < NTAPS - 1; ++j) q[j] = fir[(size_t)j * C];
#pragma unroll
    for (int j = 0; j < NIL; ++j) sh.qil[j][pair] = fir[(size_t)(NTAPS + j) * C];
#pragma unroll
    for (int j = NIL; j < NTAPS - 1; ++j) qi[j] = fir[(size_t)(NTAPS + j) * C];
  }
  const unsigned long long vmask = __ballot(valid);
#ifdef AERO_X_HANDOFF_FAIL
  return;
#endif
  for (int it = 0;; ++it) {
    int cs;
    for (int spin = 0;; ++spin) {
      cs = __builtin_amdgcn_readfirstlane(lds_load(&sh.cseq[wv]));
      if ((cs & (CSEQ_DONE - 1)) > it || (cs & CSEQ_DONE)) break;
      if (spin > SPIN_LIMIT) {
        raise_device_error(S, DERR_HANDOFF);
        cs = CSEQ_DONE;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if ((cs & (CSEQ_DONE - 1)) <= it) break;  // the chain has finished and every iteration is handled
    lds_acquire();
    const int par = it & 1;
    const unsigned long long mv = sh.mask[par][wv];
    const unsigned long long m =
        (((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(mv >> 32)) << 32) |
         (unsigned)__builtin_amdgcn_readfirstlane((unsigned)mv)) & vmask;
    const double2 xv = sh.x[par][pair];
    const double cv = xv.x, cvi = xv.y;
    const double t1 = c_taps[1];
    const double pr1 = t1 * cv, pi1 = t1 * cvi;
    // R_53 first, for the chain
    add_masked(q[NTAPS - 2], q[NTAPS - 3], pr1, m);
    add_masked(qi[NTAPS - 2], qi[NTAPS - 3], pi1, m);
    sh.r53[par][pair] = make_double2(q[NTAPS - 2], qi[NTAPS - 2]);
    lds_release();
    lds_store(&sh.fseq[wv], it + 1);
    const bool act = (m >> (pair & 63)) & 1;
    // slot 54 - k and slot k share h[k] x (k = 0..26), then the centre;
    // slot 54 is the chain's, slot 53 was formed above.  The lower slots run
    // oldest-first, each taking the previous slot's value before this sample
    // (prev), so the LDS ones are read once and written once.
    double prev_re = 0.0, prev_im = 0.0;
#pragma unroll
    for (int k = 0; k <= NL; ++k) {
      const double t = c_taps[k];
      const double pr = k == 1 ? pr1 : t * cv, pim = k == 1 ? pi1 : t * cvi;
      if (k >= 2 && k < NL) {  // upper slot 54 - k (registers)
        add_masked(q[NTAPS - 1 - k], q[NTAPS - 2 - k], pr, m);
        add_masked(qi[NTAPS - 1 - k], qi[NTAPS - 2 - k], pim, m);
      }
      // lower slot k (the centre, k = 27, too)
      if (k < NRL) {
        const double old = sh.qrl[k][pair];
        const double nv = prev_re + pr;
        sh.qrl[k][pair] = act ? nv : old;
        prev_re = old;
      } else {
        const double old = q[k];
        add_masked(q[k], prev_re, pr, m);
        prev_re = old;
      }
      if (k < NIL) {
        const double old = sh.qil[k][pair];
        const double nv = prev_im + pim;
        sh.qil[k][pair] = act ? nv : old;
        prev_im = old;
      } else {
        const double old = qi[k];
        add_masked(qi[k], prev_im, pim, m);
        prev_im = old;
      }
    }
  }
  if (!valid) return;
  int cl = c;
  asm volatile("" : "+v"(cl));
  double *fir = S.fir + cl;
#pragma unroll
  for (int j = 0; j < NRL; ++j) fir[(size_t)j * C] = sh.qrl[j][pair];
#pragma unroll
  for (int j = NRL; j < NTAPS - 1; ++j) fir[(size_t)j * C] = q[j];
#pragma unroll
  for (int j = 0; j < NIL; ++j) fir[(size_t)(NTAPS + j) * C] = sh.qil[j][pair];
#pragma unroll
  for (int j = NIL; j < NTAPS - 1; ++j) fir[(size_t)(NTAPS + j) * C] = qi[j];
}

template <bool TRACE>
__device__ __forceinline__ void demod_chain_wave(const DevState &S, const DevTables &T, DemodShared &sh, int c,
                                                 int pair, int wv, bool valid, int flush) {
  const int C = S.C;
  // sample counters relative to n0 (a launch covers at most one hop)
  long long n0 = 0;
  int pb = 0, rb = 0, ia = 0, ie = 0, ifl = 0, capm = S.pcm_cap - 1;
  double mc_ptr = 0.0, mc_step = 0.0;
  if (valid) {
    n0 = S.ls[LS_NSAMP * C + c];
    const long long avail = S.ls[LS_AVAIL * C + c];
    const long long filled0 = S.ls[LS_FILLED * C + c];
    const int hops_done = S.is[IS_HOPS_DONE * C + c];
    const long long boundary = (long long)HOP * (hops_done + 1) - 1;
    long long end = avail < boundary ? avail : boundary;
    if (!flush && avail <= boundary) end = n0;  // wait for a whole segment + the hop's ring entry
    pb = (int)(n0 & capm);          // PCM ring row of sample n0
    rb = (int)(n0 & (NFFT - 1));    // coarse-ring slot of sample n0
    ia = (int)(avail - n0);         // pushed samples beyond n0 (<= ring size)
    ie = (int)(end - n0);
    ifl = (int)(filled0 - n0);      // coarse-ring entries written: samples < n0 + ifl
    mc_ptr = S.ds[DS_MC_PTR * C + c];
    mc_step = S.ds[DS_MC_STEP * C + c];
    // coarse-ring catch-up (entry of sample n0 not yet written)
    if (ifl == 0 && ia > 0) {
      const int16_t x = S.pcm[(size_t)pb * C + c];
      S.cring[(size_t)c * NFFT + rb] = (uint32_t)cis_index(mc_ptr) | ((uint32_t)(uint16_t)x << 16);
      ifl = 1;
    }
    if (ie <= 0) {
      S.ls[LS_FILLED * C + c] = n0 + ifl;
      ie = 0;
    }
  }
  const bool work = ie > 0;
  double m2_ptr = 0, m2_step = 0, so_ptr = 0, so_last = 0, so_step = 0, so_freq = 0, agc_sum = 0;
  double d1[2] = {0, 0}, d41[4] = {0, 0, 0, 0}, d42[4] = {0, 0, 0, 0}, d8[3] = {0, 0, 0};
  double srx1 = 0, srx2 = 0, sry1 = 0, sry2 = 0, s2l_re = 0, s2l_im = 0;
  double q54 = 0, q54i = 0;  // R_54: the filter output of the next sample
  int agc_ptr = 0, yui = 0, s2l_init = 0;
  int16_t pcm_next = 0, pcm_next2 = 0;
  double agc_next = 0;
  if (work) {
    m2_ptr = S.ds[DS_M2_PTR * C + c], m2_step = S.ds[DS_M2_STEP * C + c];
    so_ptr = S.ds[DS_SO_PTR * C + c], so_last = S.ds[DS_SO_LAST * C + c];
    so_step = S.ds[DS_SO_STEP * C + c], so_freq = S.ds[DS_SO_FREQ * C + c];
    agc_sum = S.ds[DS_AGC_SUM * C + c];
#pragma unroll
    for (int k = 0; k < 2; ++k) d1[k] = S.ds[(DS_D1_0 + k) * C + c];
#pragma unroll
    for (int k = 0; k < 4; ++k) d41[k] = S.ds[(DS_D41_0 + k) * C + c];
#pragma unroll
    for (int k = 0; k < 4; ++k) d42[k] = S.ds[(DS_D42_0 + k) * C + c];
#pragma unroll
    for (int k = 0; k < 3; ++k) d8[k] = S.ds[(DS_D8_0 + k) * C + c];
    srx1 = S.ds[DS_SR_X1 * C + c], srx2 = S.ds[DS_SR_X2 * C + c];
    sry1 = S.ds[DS_SR_Y1 * C + c], sry2 = S.ds[DS_SR_Y2 * C + c];
    s2l_re = S.ds[DS_S2L_RE * C + c], s2l_im = S.ds[DS_S2L_IM * C + c];
    agc_ptr = S.is[IS_AGC_PTR * C + c];
    yui = S.is[IS_YUI * C + c], s2l_init = S.is[IS_S2L_INIT * C + c];
    static constexpr int pd_src[PD_N] = {DS_CT_X1, DS_CT_X2, DS_CT_Y1, DS_CT_Y2, DS_MARG_SUM, DS_PM_SUM,
                                         DS_MS_SUM, DS_MSE, DS_PTD_RE, DS_PTD_IM, DS_M2_FREQ};
    static constexpr int pi_src[PI_N] = {IS_MARG_P, IS_DT_P, IS_PM_P, IS_MS_P};
#pragma unroll
    for (int k = 0; k < PD_N; ++k) sh.pd[k][pair] = S.ds[pd_src[k] * C + c];
#pragma unroll
    for (int k = 0; k < PI_N; ++k) sh.pi[k][pair] = S.is[pi_src[k] * C + c];
    sh.pl[PL_SOFTP][pair] = S.ls[LS_SOFT_P * C + c];
    sh.pl[PL_PTN][pair] = TRACE ? S.ls[LS_PT_N * C + c] : 0;
    {
      const uint4 g = *reinterpret_cast<const uint4 *>(S.soft + (size_t)c * SOFT_RING +
                                                       (sh.pl[PL_SOFTP][pair] & (SOFT_RING - 16)));
      sh.softw[0][pair] = g.x;
      sh.softw[1][pair] = g.y;
      sh.softw[2][pair] = g.z;
      sh.softw[3][pair] = g.w;
    }
    sh.pi[PI_TICK][pair] = dcd_tick_rel(S, c, n0);
    {  // the ring windows from the current slots
      const int dp = sh.pi[PI_DT_P][pair], pp = sh.pi[PI_PM_P][pair];
      const double2 *dtb = S.dt + (size_t)c * DT_LEN;
      const double2 *pmsb = reinterpret_cast<const double2 *>(S.pm) + (size_t)c * MSE_LEN;
#pragma unroll
      for (int k = 0; k <= DT_WIN; ++k)
        sh.dtw[k][pair] = (AERO_X_DROP & 4) ? make_double2(0.0, 0.0) : dtb[(dp + k) % DT_LEN];
#pragma unroll
      for (int k = 0; k < PM_WIN; ++k)
        sh.pmw[k][pair] = (AERO_X_DROP & 4) ? make_double2(0.0, 0.0) : pmsb[(pp + k) % MSE_LEN];
      sh.pi[PI_DTW0][pair] = dp;
      sh.pi[PI_PMW0][pair] = pp;
      const int mp = sh.pi[PI_MARG_P][pair];
      const double *mgb = S.marg + (size_t)c * MARG_LEN;
#pragma unroll
      for (int k = 0; k < MG_WIN; ++k) sh.mgw[k][pair] = (AERO_X_DROP & 4) ? 0.0 : mgb[(mp + k) % MARG_LEN];
      sh.pi[PI_MGW0][pair] = mp;
    }
    q54 = S.fir[(size_t)(NTAPS - 1) * C + c];
    q54i = S.fir[(size_t)(2 * NTAPS - 1) * C + c];
    // R_53 before the first sample: the slot chain iteration 0 reads
    sh.r53[1][pair] = make_double2(S.fir[(size_t)(NTAPS - 2) * C + c], S.fir[(size_t)(2 * NTAPS - 2) * C + c]);
    // sample n0+i's AGC ring slot is loaded one sample ahead, its PCM word two
    // samples ahead: the coarse-ring entry staged during sample i holds sample
    // i+1's PCM word, which one sample ahead would be waited for at once
    pcm_next = S.pcm[(size_t)pb * C + c];
    pcm_next2 = S.pcm[(size_t)((pb + 1) & capm) * C + c];
    agc_next = (AERO_X_DROP & 8) ? 0.0 : S.agc[(size_t)agc_ptr * C + c];
  }
  const double PT = 0.4 * WTSIZE;  // IfHavePassedPoint(ee) with ee = 0.4 (oqpskdemodulator.cpp:225)
  // the two CIS table entries a sample uses, gathered a sample ahead (an L2
  // round trip the chain would otherwise wait for at the top of every
  // sample): st_osc's once its pointer for the next sample is known (end of
  // the sample), mixer2's speculatively at the top of the previous sample
  // (its pointer then only advances by its step unless a carrier event
  // moves it, and the event step gathers it again)
  double2 cm_next = make_double2(0.0, 0.0), so_next = make_double2(0.0, 0.0);
  if (work) {
    cm_next = T.cis[cis_index(m2_ptr)];
    so_next = T.cis[cis_index(so_ptr)];
  }

  // Event-aligned iteration.  The carrier/MSE/soft-bit step runs at every
  // second sample instant (one channel in ~9 samples), but in lockstep
  // sample order some lane of a wave has one at almost every sample, so the
  // whole wave would pay for it every sample.  Instead each lane runs its
  // own samples until its next carrier event (inner loop), and the carrier
  // step then runs once for all lanes together.  Per lane the operations and
  // their order are exactly the reference's; only the interleaving of
  // different channels changes.  Every inner iteration hands the active
  // lanes' mixed samples to the FIR wave (`it` counts the wave's iterations).
  int i = 0, it = 0, spin_left = SPIN_LIMIT;
  double ev_pr = 0.0, ev_pi = 0.0;
#ifdef AERO_X_STAMPS
  unsigned long long xstamp_[8] = {0, 0, 0, 0, 0, 0, 0, 0}, xtime_ = __builtin_amdgcn_s_memtime();
#endif
  while (i < ie) {
    bool pend = false;
    it = __builtin_amdgcn_readfirstlane(lds_load(&sh.cseq[wv]));
    do {
      XSTAMP(0);  // loop control
      // the FIR wave's progress and R_53(n-1) (its iteration it - 1), read
      // first so their LDS latency passes while this sample is mixed
      const int fsv = lds_load(&sh.fseq[wv]);
      lds_acquire();  // the R_53 read below stays after the sequence-word read
      double2 r53 = sh.r53[(it & 1) ^ 1][pair];
      const int16_t xs = pcm_next;
      pcm_next = pcm_next2;
      const double agc_old = agc_next;
      // table lookups of this sample first, then the prefetch for the next
      const double2 cm = cm_next;
      const double2 so = so_next;
      {
        double p = m2_ptr, st = m2_step;
        nco_next(p, st);
        cm_next = T.cis[cis_index(p)];
      }
      {
        const int ap = agc_ptr + 1 == AGC_LEN ? 0 : agc_ptr + 1;
        pcm_next2 = S.pcm[(size_t)((pb + i + 2) & capm) * C + c];  // past the pushed samples: unused
        agc_next = (AERO_X_DROP & 8) ? 0.0 : S.agc[(size_t)ap * C + c];
      }
      const double dval = ((double)xs) / 32768.0;
      // mix (oqpskdemodulator.cpp:390): cval = CIS * dval, componentwise
      const double cv = cm.x * dval, cvi = cm.y * dval;
      // hand x(n) to the FIR wave (its slot was read: the FIR wave passed
      // iteration it - 2 before this wave's wait in iteration it - 1)
      {
        const int par = it & 1;
        sh.x[par][pair] = make_double2(cv, cvi);
        sh.mask[par][wv] = __builtin_amdgcn_read_exec();
        // no wait: a wave's LDS writes are performed in order, so the FIR
        // wave (on the same SIMD, LDS port) that sees the new sequence word
        // sees the sample; only the compiler must keep the order
        __atomic_signal_fence(__ATOMIC_RELEASE);
        lds_store(&sh.cseq[wv], it + 1);
      }
      // rrc output of this sample: R_54(n-1); then R_54(n) = R_53(n-1) + h[54] x(n)
      // with R_53(n-1) from the FIR wave's iteration it - 1
      double s2r = q54, s2i = q54i;
      {
        if (it > 0 && __builtin_amdgcn_readfirstlane(fsv) < it) {  // rare: the FIR wave is behind
          for (int spin = 0; __builtin_amdgcn_readfirstlane(lds_load(&sh.fseq[wv])) < it; ++spin) {
            if (spin > spin_left) {  // broken hand-off: stop waiting for good
              if (spin_left) raise_device_error(S, DERR_HANDOFF);
              spin_left = 0;
              break;
            }
            __builtin_amdgcn_s_sleep(1);
          }
          lds_acquire();
          r53 = sh.r53[(it & 1) ^ 1][pair];
        }
        const double t0 = c_taps[0];
        q54 = r53.x + t0 * cv;
        q54i = r53.y + t0 * cvi;
      }
      it = __builtin_amdgcn_readfirstlane(it + 1);
      // AGC (DSP.cpp:371-380) on |sig2| (oqpskdemodulator.cpp:399-405)
      const double dab = sqrt(s2r * s2r + s2i * s2i);
      {
        agc_sum = agc_sum - agc_old;
        agc_sum = agc_sum + fabs(dab);
        if (!(AERO_X_DROP & 8)) S.agc[(size_t)agc_ptr * C + c] = fabs(dab);
        agc_ptr++;
        if (agc_ptr == AGC_LEN) agc_ptr = 0;
        // short exact divisions: a tiny quotient of agc_sum is floored at 1e-6, so
        // the divisor of g is in [1e-6, ~10]
        double g = div_n(1.414213562, fmax(div_c(agc_sum, ((double)AGC_LEN)), 0.000001));
        g = fmax(g, 0.000001);
        s2r *= g;
        s2i *= g;
      }
      // clipping (:408-410)
      XSTAMP(1);  // loads, FIR hand-off, AGC
      const double ab = DM_HYPOT(s2r, s2i);
      if (ab > 2.84) {
        const double k = div_n(2.84, ab);
        s2r = k * s2r;
        s2i = k * s2i;
      }
      XSTAMP(2);  // hypot + clip
      // symbol timer (:413-426)
      const double st_diff = delay_tap<2, 1, 0>(d1, c_dly[0], ab * ab) - (ab * ab);
      const double st_d1out = delay_tap<4, 3, 2>(d41, c_dly[1], st_diff);
      const double st_d2out = delay_tap<4, 3, 2>(d42, c_dly[2], st_d1out);
      double st_eta = (st_d2out - st_diff) * st_d1out;
      st_eta = iir3(srx1, srx2, sry1, sry2, c_sr_b, c_sr_a, st_eta);
      const double m1r = st_eta, m1i = -delay_tap<3, 2, 1>(d8, c_dly[3], st_eta);
      const double ore = so.x * m1r - so.y * m1i, oim = so.x * m1i + so.y * m1r;
      const double st_angle_error = DM_ATAN2(oim, ore);
      set_freq_st(so_freq, so_step, -st_angle_error * 0.00000001 + so_freq);
      // (a quotient below 2^-969 could differ from IEEE in its last
      // subnormal bit, and vanishes in so_ptr + x W either way)
      so_ptr += div_c(-st_angle_error * 0.01, 360.0) * WTSIZE;
      wt_wrap(so_ptr);
      if (so_freq < (10500.0 - 0.1)) set_freq_st(so_freq, so_step, (10500.0 - 0.1));
      if (so_freq > (10500.0 + 0.1)) set_freq_st(so_freq, so_step, (10500.0 + 0.1));
      if (!s2l_init) {
        s2l_re = s2r;
        s2l_im = s2i;
        s2l_init = 1;
      }
      XSTAMP(3);  // timer: delays, resonator, atan2, NCO nudges
      // sample instant (:430) IfHavePassedPoint (DSP.cpp:222-238)
      double tl = so_last - PT, tw = so_ptr - PT;
      if (tl < 0.0) tl += WTSIZE;
      if (tw < 0.0) tw += WTSIZE;
      if ((tl > 3.0 * WTSIZE / 4.0) && (tw < 1.0 * WTSIZE / 4.0)) {
        const double pt_last = div_n(tw, so_step);  // tw: 0 or >= 2^-40 (a phase difference), so_step ~4375
        const double pt_this = 1.0 - pt_last;
        const double pr = pt_this * s2r + pt_last * s2l_re;
        const double pi = pt_this * s2i + pt_last * s2l_im;
        yui++;
        yui %= 2;
        if (!yui) {
          sh.pd[PD_PTD_RE][pair] = pr;
          sh.pd[PD_PTD_IM][pair] = pi;
        } else {
          ev_pr = pr;
          ev_pi = pi;
          pend = true;  // carrier step below, before mixer2 advances
        }
      }
      s2l_re = s2r;
      s2l_im = s2i;
      nco_next(mc_ptr, mc_step);
      so_last = so_ptr;
      nco_next(so_ptr, so_step);
      so_next = T.cis[cis_index(so_ptr)];
      // coarse-ring fill of the next sample (:351-356), staged in LDS
      if (i + 1 < ia) {
        const int m = rb + i + 1;  // ring slot before masking
        const int k = m & (RING_GROUP - 1);
        {
          sh.ring[k][pair] = (uint32_t)cis_index(mc_ptr) | ((uint32_t)(uint16_t)pcm_next << 16);
          if (k == RING_GROUP - 1 && !(AERO_X_DROP & 1)) {
            uint32_t *dst = S.cring + (size_t)c * NFFT + ((m - (RING_GROUP - 1)) & (NFFT - 1));
            if (i + 1 - (RING_GROUP - 1) >= 1) {  // the whole group was staged by this launch
#pragma unroll
              for (int q4 = 0; q4 < RING_GROUP / 4; ++q4)
                reinterpret_cast<uint4 *>(dst)[q4] = make_uint4(sh.ring[4 * q4][pair], sh.ring[4 * q4 + 1][pair],
                                                                sh.ring[4 * q4 + 2][pair], sh.ring[4 * q4 + 3][pair]);
            } else {
              for (int j = (RING_GROUP - 1) - i; j < RING_GROUP; ++j) dst[j] = sh.ring[j][pair];
            }
          }
        }
        ifl = i + 2;
      }
      if (!pend) {
        nco_next(m2_ptr, m2_step);
        ++i;
      }
      XSTAMP(4);  // sample instant, NCOs, coarse-ring staging
    } while (!pend && i < ie);
    XSTAMP(0);
    if (pend) {
      // channel-row pointers from a laundered index: recomputed here, not
      // kept live across the sample loop
      int cl = c;
      asm volatile("" : "+v"(cl));
      double *marg = S.marg + (size_t)cl * MARG_LEN;
      double2 *dtb = S.dt + (size_t)cl * DT_LEN;
      // MSEcalc's two moving averages advance together (pm_p == ms_p at
      // every event), so their slots share one 16-byte entry: one line per
      // event instead of two
      double2 *pmsb = reinterpret_cast<double2 *>(S.pm) + (size_t)cl * MSE_LEN;
      int marg_p = sh.pi[PI_MARG_P][pair], dt_p = sh.pi[PI_DT_P][pair];
      int pm_p = sh.pi[PI_PM_P][pair], ms_p = sh.pi[PI_MS_P][pair];
      const double pr = ev_pr, pi = ev_pi;
      // the four moving-average rings of this symbol, loaded together
      // before any ring store so their latencies overlap
      const int dt_rp = (dt_p + 1) % DT_LEN;
      const int dtw0 = sh.pi[PI_DTW0][pair], pmw0 = sh.pi[PI_PMW0][pair];
      int dk = dt_p - dtw0, pk = pm_p - pmw0;  // the slots' places in the windows
      if (dk < 0) dk += DT_LEN;
      if (pk < 0) pk += MSE_LEN;
      const int mgw0 = sh.pi[PI_MGW0][pair];
      int mk = marg_p - mgw0;
      if (mk < 0) mk += MARG_LEN;
      const double marg_old = sh.mgw[mk][pair];
      const double2 dv = sh.dtw[dk + 1][pair];
      const double2 pms_old = sh.pmw[pk][pair];
      const double pm_old = pms_old.x, ms_old = pms_old.y;
      double ctx1 = sh.pd[PD_CTX1][pair], ctx2 = sh.pd[PD_CTX2][pair];
      double cty1 = sh.pd[PD_CTY1][pair], cty2 = sh.pd[PD_CTY2][pair];
      double marg_sum = sh.pd[PD_MARG_SUM][pair], pm_sum = sh.pd[PD_PM_SUM][pair];
      double ms_sum = sh.pd[PD_MS_SUM][pair], mse;
      const double ptd_re = sh.pd[PD_PTD_RE][pair], ptd_im = sh.pd[PD_PTD_IM][pair];
      double m2_freq = sh.pd[PD_M2_FREQ][pair];
      double qr = pr, qi = ptd_im;  // pt_qpsk
      // carrier tracking (:456-470)
      const double ct_xt = DM_TANH(pi) * pr;
      const double ct_xt_d = DM_TANH(ptd_re) * ptd_im;
      double ct_ec = ct_xt_d - ct_xt;
      if (ct_ec > M_PI) ct_ec = M_PI;
      if (ct_ec < -M_PI) ct_ec = -M_PI;
      ct_ec = iir3(ctx1, ctx2, cty1, cty2, c_ct_b, c_ct_a, ct_ec);
      if (ct_ec > M_PI_2) ct_ec = M_PI_2;
      if (ct_ec < -M_PI_2) ct_ec = -M_PI_2;
      {  // mixer2.IncresePhaseDeg / SetPhaseDeg (DSP.cpp:177-187)
        double phase_deg = 1.0 * ct_ec;
        phase_deg += div_cw(360.0 * m2_ptr, (double)WTSIZE);
        m2_ptr = set_phase_ptr(phase_deg);
      }
      set_freq(m2_freq, m2_step, 0.01 * ct_ec + m2_freq);  // IncreseFreqHz
      // marg->UpdateSigned (DSP.cpp:419-427)
      marg_sum = marg_sum - marg_old;
      marg_sum = marg_sum + (ct_ec);
      sh.mgw[mk][pair] = ct_ec;
      marg_p++;
      marg_p %= MARG_LEN;
      const double mval = DM_DIVC(marg_sum, ((double)MARG_LEN));
      // dt.update (DSP.h:456-461): slot p written, slot p+1 read
      sh.dtw[dk][pair] = make_double2(qr, qi);
      dt_p = dt_rp;
      qr = dv.x;
      qi = dv.y;
      double rs, rc;
      DM_SINCOS(mval, rs, rc);
      const double rr = qr * rc - qi * rs, ri = qr * rs + qi * rc;
      qr = rr;
      qi = ri;
      if (TRACE) {
        const long long ptn = sh.pl[PL_PTN][pair];
        if (ptn < S.pt_cap) S.pt[(size_t)cl * S.pt_cap + ptn] = make_double2(qr, qi);
        sh.pl[PL_PTN][pair] = ptn + 1;
      }
      // MSEcalc::Update (DSP.cpp:449-461)
      {
        const double av = DM_HYPOT(qr, qi);
        pm_sum = pm_sum - pm_old;
        pm_sum = pm_sum + fabs(av);
        const int pms_slot = pm_p;
        pm_p++;
        pm_p %= MSE_LEN;
        double mu = div_c(pm_sum, ((double)MSE_LEN));  // a tiny mu is floored at 1e-6 below
        if (mu < 0.000001) mu = 0.000001;
        const double rmu = rcp_div(mu);  // mu >= 1e-6; one reciprocal for both quotients (a tiny one only
                                         // makes |t| - 1 == -1)
        const double tr = div_r(1.4142135623730951 * qr, mu, rmu), ti = div_r(1.4142135623730951 * qi, mu, rmu);
        const double tda = (fabs(tr) - 1.0), tdb = (fabs(ti) - 1.0);
        const double v = (tda * tda) + (tdb * tdb);
        ms_sum = ms_sum - ms_old;
        ms_sum = ms_sum + fabs(v);
        (void)pms_slot;
        sh.pmw[pk][pair] = make_double2(fabs(av), fabs(v));
        ms_p++;
        ms_p %= MSE_LEN;
        // ms_sum sums (|t| - 1)^2 terms: 0 or a multiple of 2^-158, so the short division is exact
        mse = div_c(ms_sum, ((double)MSE_LEN));
      }
      if (i >= sh.pi[PI_TICK][pair]) {  // the first event at or after the DCD tick's sample
        dcd_tick_record(S, cl, sh.pl[PL_SOFTP][pair]);
        sh.pi[PI_TICK][pair] = INT_MAX;
      }
      if (mse < 0.65) {  // soft bits, imag first (:516-530)
        int ibit = qround(0.75 * qi * 127.0 + 128.0);
        if (ibit > 255) ibit = 255;
        if (ibit < 0) ibit = 0;
        int rbit = qround(0.75 * qr * 127.0 + 128.0);
        if (rbit > 255) rbit = 255;
        if (rbit < 0) rbit = 0;
        const long long softp = sh.pl[PL_SOFTP][pair];
        // the pair into the channel's 16-byte group (softp is even), the
        // group to the ring once complete: one store per 8 pairs instead of
        // two 1-byte stores into the channel-major ring per pair
        reinterpret_cast<uint16_t *>(&sh.softw[(softp >> 2) & 3][pair])[(softp >> 1) & 1] =
            (uint16_t)(ibit | (rbit << 8));
        if ((softp & 15) == 14 && !(AERO_X_DROP & 2))
          *reinterpret_cast<uint4 *>(S.soft + (size_t)cl * SOFT_RING + (softp & (SOFT_RING - 16))) =
              make_uint4(sh.softw[0][pair], sh.softw[1][pair], sh.softw[2][pair], sh.softw[3][pair]);
        sh.pl[PL_SOFTP][pair] = softp + 2;
      }
      sh.pd[PD_CTX1][pair] = ctx1;
      sh.pd[PD_CTX2][pair] = ctx2;
      sh.pd[PD_CTY1][pair] = cty1;
      sh.pd[PD_CTY2][pair] = cty2;
      sh.pd[PD_MARG_SUM][pair] = marg_sum;
      sh.pd[PD_PM_SUM][pair] = pm_sum;
      sh.pd[PD_MS_SUM][pair] = ms_sum;
      sh.pd[PD_MSE][pair] = mse;
      sh.pd[PD_M2_FREQ][pair] = m2_freq;
      sh.pi[PI_MARG_P][pair] = marg_p;
      sh.pi[PI_DT_P][pair] = dt_p;
      sh.pi[PI_PM_P][pair] = pm_p;
      sh.pi[PI_MS_P][pair] = ms_p;
      if (dk == DT_WIN - 1) {  // the dt window written back, the next one read
        if (!(AERO_X_DROP & 4)) {
#pragma unroll
          for (int k = 0; k < DT_WIN; ++k) dtb[(dtw0 + k) % DT_LEN] = sh.dtw[k][pair];
#pragma unroll
          for (int k = 0; k <= DT_WIN; ++k) sh.dtw[k][pair] = dtb[(dtw0 + DT_WIN + k) % DT_LEN];
        }
        sh.pi[PI_DTW0][pair] = (dtw0 + DT_WIN) % DT_LEN;
      }
      if (mk == MG_WIN - 1) {  // the same for marg
        if (!(AERO_X_DROP & 4)) {
#pragma unroll
          for (int k = 0; k < MG_WIN; ++k) marg[(mgw0 + k) % MARG_LEN] = sh.mgw[k][pair];
#pragma unroll
          for (int k = 0; k < MG_WIN; ++k) sh.mgw[k][pair] = marg[(mgw0 + MG_WIN + k) % MARG_LEN];
        }
        sh.pi[PI_MGW0][pair] = (mgw0 + MG_WIN) % MARG_LEN;
      }
      if (pk == PM_WIN - 1) {  // the same for MSEcalc
        if (!(AERO_X_DROP & 4)) {
#pragma unroll
          for (int k = 0; k < PM_WIN; ++k) pmsb[(pmw0 + k) % MSE_LEN] = sh.pmw[k][pair];
#pragma unroll
          for (int k = 0; k < PM_WIN; ++k) sh.pmw[k][pair] = pmsb[(pmw0 + PM_WIN + k) % MSE_LEN];
        }
        sh.pi[PI_PMW0][pair] = (pmw0 + PM_WIN) % MSE_LEN;
      }
      nco_next(m2_ptr, m2_step);
      cm_next = T.cis[cis_index(m2_ptr)];  // the event moved mixer2
      ++i;
    }
    XSTAMP(5);  // carrier event step
  }
  // every lane of the wave passes here: the FIR wave may stop once it has
  // handled the iterations published so far
  lds_release();
  lds_store(&sh.cseq[wv], lds_load(&sh.cseq[wv]) | CSEQ_DONE);
#ifdef AERO_X_STAMPS
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    for (int k = 0; k < 6; ++k) g_stamps[k] += xstamp_[k];
    g_stamps[6] += (unsigned long long)i;  // samples
  }
#endif
  if (!work) return;
  // staged entries of an unfinished 16-sample group
  if (ifl - 1 >= 1 && ((rb + ifl - 1) & (RING_GROUP - 1)) != RING_GROUP - 1) {
    const int last = ifl - 1;                                // relative sample of the last staged entry
    const int g0 = last - ((rb + last) & (RING_GROUP - 1));  // relative sample of its group's slot 0
    uint32_t *dst = S.cring + (size_t)c * NFFT + ((rb + g0) & (NFFT - 1));
    for (int j = (g0 >= 1 ? 0 : 1 - g0); j <= last - g0; ++j) dst[j] = sh.ring[j][pair];
  }

  // epilogue addresses are recomputed from a laundered channel index so the
  // compiler cannot keep the prologue addresses live across the sample loop
  int cl = c;
  asm volatile("" : "+v"(cl));
  S.fir[(size_t)(NTAPS - 1) * C + cl] = q54;
  S.fir[(size_t)(2 * NTAPS - 1) * C + cl] = q54i;
  double *ds = S.ds + cl;
  int *is = S.is + cl;
  long long *ls = S.ls + cl;
  ls[LS_NSAMP * C] = n0 + i;
  ls[LS_FILLED * C] = n0 + ifl;
  ls[LS_SOFT_P * C] = sh.pl[PL_SOFTP][pair];
  if (TRACE) ls[LS_PT_N * C] = sh.pl[PL_PTN][pair];
  if (!(AERO_X_DROP & 4)) {  // the ring windows back (their unwritten slots hold what was read)
    double2 *dtb = S.dt + (size_t)cl * DT_LEN;
    double2 *pmsb = reinterpret_cast<double2 *>(S.pm) + (size_t)cl * MSE_LEN;
    const int dtw0 = sh.pi[PI_DTW0][pair], pmw0 = sh.pi[PI_PMW0][pair];
#pragma unroll
    for (int k = 0; k < DT_WIN; ++k) dtb[(dtw0 + k) % DT_LEN] = sh.dtw[k][pair];
#pragma unroll
    for (int k = 0; k < PM_WIN; ++k) pmsb[(pmw0 + k) % MSE_LEN] = sh.pmw[k][pair];
    double *mgb = S.marg + (size_t)cl * MARG_LEN;
    const int mgw0 = sh.pi[PI_MGW0][pair];
#pragma unroll
    for (int k = 0; k < MG_WIN; ++k) mgb[(mgw0 + k) % MARG_LEN] = sh.mgw[k][pair];
  }
  if ((sh.pl[PL_SOFTP][pair] & 15) && !(AERO_X_DROP & 2))  // the group being filled (bytes past softp are not read)
    *reinterpret_cast<uint4 *>(S.soft + (size_t)cl * SOFT_RING + (sh.pl[PL_SOFTP][pair] & (SOFT_RING - 16))) =
        make_uint4(sh.softw[0][pair], sh.softw[1][pair], sh.softw[2][pair], sh.softw[3][pair]);
  {
    static constexpr int pd_dst[PD_N] = {DS_CT_X1, DS_CT_X2, DS_CT_Y1, DS_CT_Y2, DS_MARG_SUM, DS_PM_SUM,
                                         DS_MS_SUM, DS_MSE, DS_PTD_RE, DS_PTD_IM, DS_M2_FREQ};
    static constexpr int pi_dst[PI_N] = {IS_MARG_P, IS_DT_P, IS_PM_P, IS_MS_P};
#pragma unroll
    for (int k = 0; k < PD_N; ++k) ds[pd_dst[k] * C] = sh.pd[k][pair];
#pragma unroll
    for (int k = 0; k < PI_N; ++k) is[pi_dst[k] * C] = sh.pi[k][pair];
  }
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
  for (int k = 0; k < 2; ++k) ds[(DS_D1_0 + k) * C] = d1[k];
#pragma unroll
  for (int k = 0; k < 4; ++k) ds[(DS_D41_0 + k) * C] = d41[k];
#pragma unroll
  for (int k = 0; k < 4; ++k) ds[(DS_D42_0 + k) * C] = d42[k];
#pragma unroll
  for (int k = 0; k < 3; ++k) ds[(DS_D8_0 + k) * C] = d8[k];
  ds[DS_SR_X1 * C] = srx1;
  ds[DS_SR_X2 * C] = srx2;
  ds[DS_SR_Y1 * C] = sry1;
  ds[DS_SR_Y2 * C] = sry2;
  ds[DS_S2L_RE * C] = s2l_re;
  ds[DS_S2L_IM * C] = s2l_im;
  is[IS_AGC_PTR * C] = agc_ptr;
  is[IS_YUI * C] = yui;
  is[IS_S2L_INIT * C] = s2l_init;
}

// One workgroup = 256 channels, two waves per 64 channels (chain + FIR).
// Segment contract: a launch advances every channel from nsamp up to (but
// excluding) its next coarse-estimate hop sample, or to the pushed end; it
// also writes the coarse-ring entry of the sample after each processed one
// (ring fill precedes the hop that uses it, oqpskdemodulator.cpp:351-369).
template <bool TRACE>
__global__ __launch_bounds__(DEMOD_THREADS) void demod_oqpsk_kernel(DevState S, DevTables T, int nch, int flush) {
  __shared__ DemodShared sh;
  const int pair = threadIdx.x & (DEMOD_BLOCK - 1);  // this channel's LDS column
  const int wv = pair >> 6;                          // channel wave of the block
  const int c = blockIdx.x * DEMOD_BLOCK + pair;
  const bool valid = c < nch;
  if (threadIdx.x < 4) {
    sh.cseq[threadIdx.x] = 0;
    sh.fseq[threadIdx.x] = 0;
  }
  for (int k = threadIdx.x; k < 241 * 7; k += DEMOD_THREADS) (&sh.cij[0][0])[k] = (&aero_g_cij[0][0])[k];
  for (int k = threadIdx.x; k < 440; k += DEMOD_THREADS) sh.sct[k] = aero_g_sincostab[k];
  __syncthreads();
  if (threadIdx.x >= DEMOD_BLOCK)
    demod_fir_wave(S, sh, c, pair, wv, valid);
  else
    demod_chain_wave<TRACE>(S, T, sh, c, pair, wv, valid, flush);
}

// The few-channel kernel (a receiver's handful of VFOs, C1 / C5): one channel
// per 16 lanes, no helper wave.  Lane k of a channel's group holds four of
// the RRC's transposed partial sums (right-aligned: lane 15 holds R_51..R_54,
// so R_54, the filter output, is its last slot); per sample the one partial
// sum that crosses a lane boundary moves by a shuffle before the update, and
// the output R_54(n-1) is broadcast from lane 15 first.  All 16 lanes run the
// chain on identical values (their identical stores coalesce).  The
// arithmetic is demod_chain_wave's and demod_fir_wave's operation for
// operation, and the state layout is theirs, so a group may switch kernels
// from one launch to the next.
constexpr int DMW_G = 16, DMW_WG = 64, DMW_B = 4;  // lanes per channel, workgroup, taps per lane
static_assert(DMW_G * DMW_B >= NTAPS, "every tap has a lane");
struct DemodWShared {
  double cij[241][7];
  double sct[440];
};
template <bool TRACE>
__global__ __launch_bounds__(DMW_WG) void demod_oqpskw_kernel(DevState S, DevTables T, int nch, int flush) {
  __shared__ DemodWShared sh;
  for (int q = threadIdx.x; q < 241 * 7; q += DMW_WG) (&sh.cij[0][0])[q] = (&aero_g_cij[0][0])[q];
  for (int q = threadIdx.x; q < 440; q += DMW_WG) sh.sct[q] = aero_g_sincostab[q];
  __syncthreads();
  const int lane = threadIdx.x, k = lane & (DMW_G - 1), top = (lane & ~(DMW_G - 1)) + DMW_G - 1;
  const int c = blockIdx.x * (DMW_WG / DMW_G) + lane / DMW_G;
  if (c >= nch) return;  // the whole 16-lane group
  const int j0 = NTAPS - (DMW_G - k) * DMW_B;  // this lane's first tap (negative: slots without one)
  const int C = S.C;
  const long long n0 = S.ls[LS_NSAMP * C + c];
  const long long avail = S.ls[LS_AVAIL * C + c];
  const long long filled0 = S.ls[LS_FILLED * C + c];
  const int hops_done = S.is[IS_HOPS_DONE * C + c];
  const long long boundary = (long long)HOP * (hops_done + 1) - 1;
  long long end = avail < boundary ? avail : boundary;
  if (!flush && avail <= boundary) end = n0;
  const int capm = (int)S.pcm_cap - 1;
  const int ia = (int)(avail - n0);
  const int ie = (int)(end - n0);
  int ifl = (int)(filled0 - n0);
  double mc_ptr = S.ds[DS_MC_PTR * C + c], mc_step = S.ds[DS_MC_STEP * C + c];
  if (ifl == 0 && ia > 0) {  // coarse-ring entry of sample n0
    const int16_t x = S.pcm[(size_t)(n0 & capm) * C + c];
    S.cring[(size_t)c * NFFT + (n0 & (NFFT - 1))] = (uint32_t)cis_index(mc_ptr) | ((uint32_t)(uint16_t)x << 16);
    ifl = 1;
  }
  if (ie <= 0) {
    S.ls[LS_FILLED * C + c] = n0 + ifl;
    return;
  }
  double m2_ptr = S.ds[DS_M2_PTR * C + c], m2_step = S.ds[DS_M2_STEP * C + c];
  double so_ptr = S.ds[DS_SO_PTR * C + c], so_last = S.ds[DS_SO_LAST * C + c];
  double so_step = S.ds[DS_SO_STEP * C + c], so_freq = S.ds[DS_SO_FREQ * C + c];
  double agc_sum = S.ds[DS_AGC_SUM * C + c];
  double d1[2], d41[4], d42[4], d8[3];
#pragma unroll
  for (int q = 0; q < 2; ++q) d1[q] = S.ds[(DS_D1_0 + q) * C + c];
#pragma unroll
  for (int q = 0; q < 4; ++q) d41[q] = S.ds[(DS_D41_0 + q) * C + c];
#pragma unroll
  for (int q = 0; q < 4; ++q) d42[q] = S.ds[(DS_D42_0 + q) * C + c];
#pragma unroll
  for (int q = 0; q < 3; ++q) d8[q] = S.ds[(DS_D8_0 + q) * C + c];
  double srx1 = S.ds[DS_SR_X1 * C + c], srx2 = S.ds[DS_SR_X2 * C + c];
  double sry1 = S.ds[DS_SR_Y1 * C + c], sry2 = S.ds[DS_SR_Y2 * C + c];
  double s2l_re = S.ds[DS_S2L_RE * C + c], s2l_im = S.ds[DS_S2L_IM * C + c];
  double ctx1 = S.ds[DS_CT_X1 * C + c], ctx2 = S.ds[DS_CT_X2 * C + c];
  double cty1 = S.ds[DS_CT_Y1 * C + c], cty2 = S.ds[DS_CT_Y2 * C + c];
  double marg_sum = S.ds[DS_MARG_SUM * C + c], pm_sum = S.ds[DS_PM_SUM * C + c];
  double ms_sum = S.ds[DS_MS_SUM * C + c], mse = S.ds[DS_MSE * C + c];
  double ptd_re = S.ds[DS_PTD_RE * C + c], ptd_im = S.ds[DS_PTD_IM * C + c];
  double m2_freq = S.ds[DS_M2_FREQ * C + c];
  int agc_ptr = S.is[IS_AGC_PTR * C + c];
  int yui = S.is[IS_YUI * C + c], s2l_init = S.is[IS_S2L_INIT * C + c];
  int marg_p = S.is[IS_MARG_P * C + c], dt_p = S.is[IS_DT_P * C + c];
  int pm_p = S.is[IS_PM_P * C + c], ms_p = S.is[IS_MS_P * C + c];
  long long softp = S.ls[LS_SOFT_P * C + c];
  long long ptn = TRACE ? S.ls[LS_PT_N * C + c] : 0;
  int tick_rel = dcd_tick_rel(S, c, n0);
  double qre[DMW_B], qim[DMW_B], tp[DMW_B];
#pragma unroll
  for (int jj = 0; jj < DMW_B; ++jj) {
    const int j = j0 + jj;
    tp[jj] = j >= 0 ? c_taps[j] : 0.0;
    qre[jj] = j >= 0 ? S.fir[(size_t)j * C + c] : 0.0;
    qim[jj] = j >= 0 ? S.fir[(size_t)(NTAPS + j) * C + c] : 0.0;
  }
  double *marg = S.marg + (size_t)c * MARG_LEN;
  double2 *dtb = S.dt + (size_t)c * DT_LEN;
  double2 *pmsb = reinterpret_cast<double2 *>(S.pm) + (size_t)c * MSE_LEN;
  uint8_t *soft = S.soft + (size_t)c * SOFT_RING;
  const double PT = 0.4 * WTSIZE;  // IfHavePassedPoint(ee) with ee = 0.4 (oqpskdemodulator.cpp:225)
  // a sample's PCM word and AGC slot, and its two table entries, loaded one
  // sample ahead (mixer2's speculatively: a carrier event reloads it)
  int16_t xs_nx = S.pcm[(size_t)(n0 & capm) * C + c];
  double agc_nx = S.agc[(size_t)agc_ptr * C + c];
  double2 cm_nx = T.cis[cis_index(m2_ptr)], so_nx = T.cis[cis_index(so_ptr)];
  int i = 0;
  for (; i < ie; ++i) {
    const long long n = n0 + i;
    const int16_t xs = xs_nx;
    const double agc_old = agc_nx;
    const double2 cm = cm_nx, so = so_nx;
    xs_nx = S.pcm[(size_t)((n + 1) & capm) * C + c];  // past the pushed samples: unused
    {
      const int ap = agc_ptr + 1 == AGC_LEN ? 0 : agc_ptr + 1;
      agc_nx = S.agc[(size_t)ap * C + c];
      double p = m2_ptr, st = m2_step;
      nco_next(p, st);
      cm_nx = T.cis[cis_index(p)];
    }
    const double dval = ((double)xs) / 32768.0;
    const double cv = cm.x * dval, cvi = cm.y * dval;  // mix (oqpskdemodulator.cpp:390)
    // RRC: output R_54(n-1) (lane 15's last slot), the boundary partial sums
    // of the lanes below, both before the update
    double s2r = __shfl(qre[DMW_B - 1], top, 64), s2i = __shfl(qim[DMW_B - 1], top, 64);
    const double bre = __shfl_up(qre[DMW_B - 1], 1, DMW_G), bim = __shfl_up(qim[DMW_B - 1], 1, DMW_G);
#pragma unroll
    for (int jj = DMW_B - 1; jj >= 1; --jj) {
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
    // AGC (DSP.cpp:371-380) on |sig2| (oqpskdemodulator.cpp:399-405)
    const double dab = sqrt(s2r * s2r + s2i * s2i);
    {
      agc_sum = agc_sum - agc_old;
      agc_sum = agc_sum + fabs(dab);
      S.agc[(size_t)agc_ptr * C + c] = fabs(dab);
      agc_ptr++;
      if (agc_ptr == AGC_LEN) agc_ptr = 0;
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
    const double st_diff = delay_tap<2, 1, 0>(d1, c_dly[0], ab * ab) - (ab * ab);
    const double st_d1out = delay_tap<4, 3, 2>(d41, c_dly[1], st_diff);
    const double st_d2out = delay_tap<4, 3, 2>(d42, c_dly[2], st_d1out);
    double st_eta = (st_d2out - st_diff) * st_d1out;
    st_eta = iir3(srx1, srx2, sry1, sry2, c_sr_b, c_sr_a, st_eta);
    const double m1r = st_eta, m1i = -delay_tap<3, 2, 1>(d8, c_dly[3], st_eta);
    const double ore = so.x * m1r - so.y * m1i, oim = so.x * m1i + so.y * m1r;
    const double st_angle_error = aero_atan2_bf(oim, ore, sh.cij);
    set_freq_st(so_freq, so_step, -st_angle_error * 0.00000001 + so_freq);
    so_ptr += div_c(-st_angle_error * 0.01, 360.0) * WTSIZE;
    wt_wrap(so_ptr);
    if (so_freq < (10500.0 - 0.1)) set_freq_st(so_freq, so_step, (10500.0 - 0.1));
    if (so_freq > (10500.0 + 0.1)) set_freq_st(so_freq, so_step, (10500.0 + 0.1));
    if (!s2l_init) {
      s2l_re = s2r;
      s2l_im = s2i;
      s2l_init = 1;
    }
    // sample instant (:430) IfHavePassedPoint (DSP.cpp:222-238)
    bool pend = false;
    double ev_pr = 0.0, ev_pi = 0.0;
    {
      double tl = so_last - PT, tw = so_ptr - PT;
      if (tl < 0.0) tl += WTSIZE;
      if (tw < 0.0) tw += WTSIZE;
      if ((tl > 3.0 * WTSIZE / 4.0) && (tw < 1.0 * WTSIZE / 4.0)) {
        const double pt_last = div_n(tw, so_step);
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
    nco_next(mc_ptr, mc_step);
    so_last = so_ptr;
    nco_next(so_ptr, so_step);
    so_nx = T.cis[cis_index(so_ptr)];
    if (i + 1 < ia) {  // coarse-ring entry of the next sample (:351-356)
      const long long n1 = n + 1;
      S.cring[(size_t)c * NFFT + (n1 & (NFFT - 1))] =
          (uint32_t)cis_index(mc_ptr) | ((uint32_t)(uint16_t)xs_nx << 16);
      ifl = i + 2;
    }
    if (pend) {  // carrier step (:455-541)
      const int dt_rp = (dt_p + 1) % DT_LEN;
      const double marg_old = marg[marg_p];
      const double2 dv = dtb[dt_rp];
      const double2 pms_old = pmsb[pm_p];
      const double pm_old = pms_old.x, ms_old = pms_old.y;
      const double pr = ev_pr, pi = ev_pi;
      double qr = pr, qi = ptd_im;  // pt_qpsk
      const double ct_xt = aero_tanh_bf(pi) * pr;
      const double ct_xt_d = aero_tanh_bf(ptd_re) * ptd_im;
      double ct_ec = ct_xt_d - ct_xt;
      if (ct_ec > M_PI) ct_ec = M_PI;
      if (ct_ec < -M_PI) ct_ec = -M_PI;
      ct_ec = iir3(ctx1, ctx2, cty1, cty2, c_ct_b, c_ct_a, ct_ec);
      if (ct_ec > M_PI_2) ct_ec = M_PI_2;
      if (ct_ec < -M_PI_2) ct_ec = -M_PI_2;
      {  // mixer2.IncresePhaseDeg / SetPhaseDeg (DSP.cpp:177-187)
        double phase_deg = 1.0 * ct_ec;
        phase_deg += div_cw(360.0 * m2_ptr, (double)WTSIZE);
        m2_ptr = set_phase_ptr(phase_deg);
      }
      set_freq(m2_freq, m2_step, 0.01 * ct_ec + m2_freq);  // IncreseFreqHz
      marg_sum = marg_sum - marg_old;  // marg->UpdateSigned (DSP.cpp:419-427)
      marg_sum = marg_sum + (ct_ec);
      marg[marg_p] = ct_ec;
      marg_p++;
      marg_p %= MARG_LEN;
      const double mval = DM_DIVC(marg_sum, ((double)MARG_LEN));
      dtb[dt_p] = make_double2(qr, qi);  // dt.update (DSP.h:456-461)
      dt_p = dt_rp;
      qr = dv.x;
      qi = dv.y;
      double rs, rc;
      aero_sincos_bf(mval, rs, rc, sh.sct);
      const double rr = qr * rc - qi * rs, ri = qr * rs + qi * rc;
      qr = rr;
      qi = ri;
      if (TRACE) {
        if (ptn < S.pt_cap) S.pt[(size_t)c * S.pt_cap + ptn] = make_double2(qr, qi);
        ptn++;
      }
      {  // MSEcalc::Update (DSP.cpp:449-461)
        const double av = aero_hypot_w(qr, qi);
        pm_sum = pm_sum - pm_old;
        pm_sum = pm_sum + fabs(av);
        const int pms_slot = pm_p;
        pm_p++;
        pm_p %= MSE_LEN;
        double mu = div_c(pm_sum, ((double)MSE_LEN));
        if (mu < 0.000001) mu = 0.000001;
        const double rmu = rcp_div(mu);
        const double tr = div_r(1.4142135623730951 * qr, mu, rmu), ti = div_r(1.4142135623730951 * qi, mu, rmu);
        const double tda = (fabs(tr) - 1.0), tdb = (fabs(ti) - 1.0);
        const double v = (tda * tda) + (tdb * tdb);
        ms_sum = ms_sum - ms_old;
        ms_sum = ms_sum + fabs(v);
        pmsb[pms_slot] = make_double2(fabs(av), fabs(v));
        ms_p++;
        ms_p %= MSE_LEN;
        mse = div_c(ms_sum, ((double)MSE_LEN));
      }
      if (i >= tick_rel) {  // the first event at or after the DCD tick's sample
        dcd_tick_record(S, c, softp);
        tick_rel = INT_MAX;
      }
      if (mse < 0.65) {  // soft bits, imag first (:516-530)
        int ibit = qround(0.75 * qi * 127.0 + 128.0);
        if (ibit > 255) ibit = 255;
        if (ibit < 0) ibit = 0;
        int rbit = qround(0.75 * qr * 127.0 + 128.0);
        if (rbit > 255) rbit = 255;
        if (rbit < 0) rbit = 0;
        soft[softp & (SOFT_RING - 1)] = (uint8_t)ibit;
        soft[(softp + 1) & (SOFT_RING - 1)] = (uint8_t)rbit;
        softp += 2;
      }
      nco_next(m2_ptr, m2_step);
      cm_nx = T.cis[cis_index(m2_ptr)];  // the event moved mixer2
    } else {
      nco_next(m2_ptr, m2_step);
    }
  }
#pragma unroll
  for (int jj = 0; jj < DMW_B; ++jj) {
    const int j = j0 + jj;
    if (j >= 0) {
      S.fir[(size_t)j * C + c] = qre[jj];
      S.fir[(size_t)(NTAPS + j) * C + c] = qim[jj];
    }
  }
  double *ds = S.ds + c;
  int *is = S.is + c;
  long long *ls = S.ls + c;
  ls[LS_NSAMP * C] = n0 + i;
  ls[LS_FILLED * C] = n0 + ifl;
  ls[LS_SOFT_P * C] = softp;
  if (TRACE) ls[LS_PT_N * C] = ptn;
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
  is[IS_MARG_P * C] = marg_p;
  is[IS_DT_P * C] = dt_p;
  is[IS_PM_P * C] = pm_p;
  is[IS_MS_P * C] = ms_p;
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
}

void launch_demod(hipStream_t st, const DevState &S, const DevTables &T, int nch, int flush, bool trace, bool wide) {
  if (wide) {
    constexpr int CPB = DMW_WG / DMW_G;
    dim3 grid((nch + CPB - 1) / CPB), block(DMW_WG);
    if (trace)
      hipLaunchKernelGGL(demod_oqpskw_kernel<true>, grid, block, 0, st, S, T, nch, flush);
    else
      hipLaunchKernelGGL(demod_oqpskw_kernel<false>, grid, block, 0, st, S, T, nch, flush);
    return;
  }
  dim3 grid((nch + DEMOD_BLOCK - 1) / DEMOD_BLOCK), block(DEMOD_THREADS);
  if (trace)
    hipLaunchKernelGGL(demod_oqpsk_kernel<true>, grid, block, 0, st, S, T, nch, flush);
  else
    hipLaunchKernelGGL(demod_oqpsk_kernel<false>, grid, block, 0, st, S, T, nch, flush);
}

// diagnostic build: cycle totals per section (7 values), then reset
void demod_read_stamps(unsigned long long *out) {
#ifdef AERO_X_STAMPS
  hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 7);
  unsigned long long z[8] = {0};
  hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof z);
#else
  for (int k = 0; k < 7; ++k) out[k] = 0;
#endif
}

void upload_demod_constants(const double *taps, const DelayDesc *dly, const double *sr_b, const double *sr_a,
                            const double *ct_b, const double *ct_a) {
  hipMemcpyToSymbol(HIP_SYMBOL(c_taps), taps, sizeof(double) * NTAPS);
  hipMemcpyToSymbol(HIP_SYMBOL(c_dly), dly, sizeof(DelayDesc) * 4);
  hipMemcpyToSymbol(HIP_SYMBOL(c_sr_b), sr_b, sizeof(double) * 3);
  hipMemcpyToSymbol(HIP_SYMBOL(c_sr_a), sr_a, sizeof(double) * 3);
  hipMemcpyToSymbol(HIP_SYMBOL(c_ct_b), ct_b, sizeof(double) * 3);
  hipMemcpyToSymbol(HIP_SYMBOL(c_ct_a), ct_a, sizeof(double) * 3);
}

}  // namespace aero
