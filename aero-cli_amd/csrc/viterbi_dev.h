// K=7 rate-1/2 soft-decision Viterbi, one wave64 per codeword: lane s owns
// state s. Restates libcorrect's convolutional_decode_soft as AeroL calls it
// (decode/jconvolutionalcodec.cpp:146-198 continuous blocks, :88-119 burst
// R/T packets): polys {109, 79}, warmup over the first 6 symbol pairs, uint16
// path metrics renormalised every 128 steps, history ring of 140 columns,
// traceback leaving 35 columns of depth, zero tail with the last 6 steps
// restricted to the states the tail can still reach, and a final traceback
// from state 0. Shared by aerol.hip (framing blocks) and burst.hip (R/T tests).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace aero {

__device__ __forceinline__ int conv_table(int r) {  // table[r]: bit j = parity(r & poly[j])
  return (__builtin_popcount(r & 109) & 1) | ((__builtin_popcount(r & 79) & 1) << 1);
}

__device__ __forceinline__ int soft_dist(int hard, int a, int b) {  // metric_soft_distance_linear
  const int x0 = (hard & 1) ? 255 : 0, x1 = (hard & 2) ? 255 : 0;
  const int d0 = a - x0, d1 = b - x1;
  return (d0 < 0 ? -d0 : d0) + (d1 < 0 ? -d1 : d1);
}

__device__ __forceinline__ int shfl_idx(int v, int src) { return __builtin_amdgcn_ds_bpermute(src << 2, v); }

constexpr int HCAP = 140, MINTB = 35, RENORM = 128;

// Decodes nsoft soft symbols from sbuf (LDS) into obits[0, nsoft/2) (LDS,
// one byte per bit, zeroed by the caller). hist: LDS, HCAP words. Every lane
// of the (single-wave) workgroup calls it; it contains __syncthreads().
__device__ __forceinline__ void viterbi_decode_wave(const uint8_t *sbuf, int nsoft, unsigned long long *hist,
                                                    uint8_t *obits, int lane) {
  const int sets = nsoft / 2;
  const int s = lane;
  const int tab_lo = conv_table(s), tab_hi = conv_table(s | 64);
  int m = 0;  // uint16 path metric of state s
  // warmup (decode.c convolutional_decode_warmup): states reachable from 0
  for (int i = 0; i < 6 && i < sets; ++i) {
    const int a = sbuf[2 * i], b = sbuf[2 * i + 1];
    const int prev = shfl_idx(m, s >> 1);
    if (s < (2 << i)) m = (soft_dist(conv_table(s), a, b) + prev) & 0xFFFF;
  }
  int index = 0, len = 0, renorm = 0, outpos = 0;
  auto search = [&](int skip) -> int {
    // least metric among states s % skip == 0, lowest index on ties
    int key = (s % skip == 0) ? ((m << 6) | s) : 0x7FFFFFFF;
    for (int off = 32; off > 0; off >>= 1) {
      const int o = __shfl_xor(key, off, 64);
      key = o < key ? o : key;
    }
    return key & 63;
  };
  auto traceback = [&](int bestpath, int mintb) {
    const int nout = len - mintb;
    if (lane == 0) {
      int idx = index;
      for (int j = 0; j < len; ++j) {
        idx = idx == 0 ? HCAP - 1 : idx - 1;
        const int hb = (int)((hist[idx] >> bestpath) & 1ULL);
        bestpath = (bestpath | (hb << 6)) >> 1;
        if (j >= mintb) obits[outpos + (nout - 1 - (j - mintb))] = (uint8_t)hb;
      }
    }
    outpos += nout;
    len -= nout;
    __syncthreads();
  };
  auto process = [&](int skip) {
    index++;
    if (index == HCAP) index = 0;
    renorm++;
    len++;
    if (renorm == RENORM) {
      renorm = 0;
      const int best = search(skip);
      const int mind = shfl_idx(m, best);
      m = (m - mind) & 0xFFFF;
      if (len == HCAP) traceback(best, MINTB);
    } else if (len == HCAP) {
      traceback(search(skip), MINTB);
    }
  };
  for (int i = 6; i < sets; ++i) {
    const int a = sbuf[2 * i], b = sbuf[2 * i + 1];
    const bool tail = i >= sets - 6;
    const int skip = tail ? (1 << (7 - (sets - i))) : 1;
    const int m0 = shfl_idx(m, s >> 1), m1 = shfl_idx(m, (s >> 1) | 32);
    const int e0 = (m0 + soft_dist(tab_lo, a, b)) & 0xFFFF;
    const int e1 = (m1 + soft_dist(tab_hi, a, b)) & 0xFFFF;
    const bool act = (s % skip) == 0;
    const int h = (e0 <= e1) ? 0 : 1;
    if (act) m = h ? e1 : e0;
    const unsigned long long mask = __ballot(act && h);
    if (lane == 0) hist[index] = mask;
    __syncthreads();
    process(skip);
  }
  traceback(0, 0);
}

}  // namespace aero

namespace aero {

// Same decoder as viterbi_decode_wave (same metrics, ties, renormalisation,
// 140-column history, 35-column traceback depth, restricted tail) with the
// history in registers (lane l holds columns l, l + 64, l + 128) instead of
// LDS, so a trellis step needs no LDS store and no barrier (two bpermutes,
// ~10 VALU and two v_writelane per step before the tail), and the traceback
// runs on the scalar unit (the path state is wave-uniform): two v_readlane
// per column instead of a dependent LDS read per column in lane 0.
// Decoded bit b lands in bit (b & 63) of obw in lane b >> 6.
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ void viterbi_decode_regs(const uint8_t *sbuf, int nsoft, uint64_t &obw, int lane) {
  const int sets = nsoft / 2;
  const int s = lane;
  const int tab_lo = conv_table(s), tab_hi = conv_table(s | 64);
  uint64_t h0 = 0, h1 = 0, h2 = 0;  // history columns lane, lane + 64, lane + 128
  obw = 0;
  int m = 0;
  for (int i = 0; i < 6 && i < sets; ++i) {
    const int a = sbuf[2 * i], b = sbuf[2 * i + 1];
    const int prev = shfl_idx(m, s >> 1);
    if (s < (2 << i)) m = (soft_dist(conv_table(s), a, b) + prev) & 0xFFFF;
  }
  int index = 0, len = 0, renorm = 0, outpos = 0;  // wave-uniform
  auto search = [&](int skip) -> int {
    int key = (s % skip == 0) ? ((m << 6) | s) : 0x7FFFFFFF;
    for (int off = 32; off > 0; off >>= 1) {
      const int o = __shfl_xor(key, off, 64);
      key = o < key ? o : key;
    }
    return __builtin_amdgcn_readfirstlane(key) & 63;
  };
  // Traceback on the scalar unit: per column two v_readlane and a few scalar
  // operations; the output bits (newest first, so bit b descends) are
  // gathered in a 64-bit scalar word and merged into lane b >> 6 once per
  // word.
  auto traceback = [&](int bestpath, int mintb) {
    const int nout = len - mintb;
    int idx = index;
    int j = 0;
    uint64_t acc = 0;
    int accw = -1;
    auto flush = [&]() {
      if (accw >= 0 && lane == accw) obw |= acc;
    };
    while (j < len) {
      idx = idx == 0 ? HCAP - 1 : idx - 1;
      int run = (idx & 63) + 1;  // columns idx, idx - 1, ... down to this register's first
      if (run > len - j) run = len - j;
      auto walk = [&](const uint64_t hw) {
        for (int k = 0; k < run; ++k, ++j) {
          const uint64_t hv = readlane64(hw, (idx - k) & 63);
          const int hb = (int)((hv >> bestpath) & 1ULL);
          bestpath = (bestpath | (hb << 6)) >> 1;
          if (j >= mintb) {
            const int bb = outpos + (nout - 1 - (j - mintb));
            if ((bb >> 6) != accw) {
              flush();
              accw = bb >> 6;
              acc = 0;
            }
            acc |= (uint64_t)hb << (bb & 63);
          }
        }
      };
      // uniform branch per register (a selected copy would go through scratch)
      const int w = __builtin_amdgcn_readfirstlane(idx >> 6);
      if (w == 0)
        walk(h0);
      else if (w == 1)
        walk(h1);
      else
        walk(h2);
      idx -= run - 1;
    }
    flush();
    outpos += nout;
    len -= nout;
  };
  auto process = [&](int skip) {
    index++;
    if (index == HCAP) index = 0;
    renorm++;
    len++;
    if (renorm == RENORM) {
      renorm = 0;
      const int best = search(skip);
      const int mind = __builtin_amdgcn_readlane(m, best);
      m = (m - mind) & 0xFFFF;
      if (len == HCAP) traceback(best, MINTB);
    } else if (len == HCAP) {
      traceback(search(skip), MINTB);
    }
  };
  // the soft pairs of the next 64 steps: lane l holds step i0 + l's pair
  // (a | b << 16); a step takes its pair with one v_readlane, so no LDS read
  // sits on the step's dependency chain
  auto pairs = [&](int i0) -> uint32_t {
    const int st = i0 + lane;
    return st < sets ? (uint32_t)sbuf[2 * st] | ((uint32_t)sbuf[2 * st + 1] << 16) : 0u;
  };
  // Steps before the restricted tail (every state active) in runs that no
  // event interrupts: a run ends where the column index leaves its register
  // (64, 128, the wrap at 140), at the renormalisation (every 128 steps), at
  // the traceback (140 columns held), at the end of the 64 buffered pairs
  // or at the tail; the events are handled between runs exactly as
  // process(1) handles them after a step.  Inside a run a step is: its pair
  // by v_readlane, the two predecessor metrics by ds_bpermute, the branch
  // metric soft_dist(tab_lo, a, b) = nbase - sa a - sb b (a, b in [0, 255];
  // the s | 64 edge carries the complementary code bits, as both
  // polynomials have bit 6 set: tab_hi == tab_lo ^ 3, so its metric is 510
  // minus that), the compare (the decision mask) and the minimum, the mask
  // into column index + k by two v_writelane.
  const int tail0 = sets - 6 > 6 ? sets - 6 : 6;
  {
    const int msa = (tab_lo & 1) ? 1 : -1, msb = (tab_lo & 2) ? 1 : -1;  // -sa, -sb
    typedef short v2s __attribute__((ext_vector_type(2)));
    const v2s coef = {(short)msa, (short)msb};
    const int nbase = -(((tab_lo & 1) ? 255 : 0) + ((tab_lo & 2) ? 255 : 0));
    const int src0 = (s >> 1) << 2, src1 = ((s >> 1) | 32) << 2;
    int i = 6;
    uint32_t pv = pairs(6);
    int pk = 0;  // step i's pair is lane pk of pv
    while (i < tail0) {
      const int idx = __builtin_amdgcn_readfirstlane(index);
      const int w = idx >> 6;
      int run = (w == 2 ? HCAP : 64 * (w + 1)) - idx;
      run = min(run, tail0 - i);
      run = min(run, RENORM - renorm);
      run = min(run, HCAP - len);
      run = min(run, 64 - pk);
      run = __builtin_amdgcn_readfirstlane(run);
      auto steps = [&](uint64_t &hw) {
        uint32_t lo = (uint32_t)hw, hi = (uint32_t)(hw >> 32);
        const int col0 = idx & 63;
        for (int k = 0; k < run; ++k) {
          const uint32_t ab = (uint32_t)__builtin_amdgcn_readlane((int)pv, pk + k);
          const int m0 = __builtin_amdgcn_ds_bpermute(src0, m), m1 = __builtin_amdgcn_ds_bpermute(src1, m);
          // -soft_dist(tab_lo, a, b) = nbase - sa a - sb b as one 16-bit dot
          // product (v_dot2c_i32_i16, exact integer arithmetic)
          const int nd = __builtin_amdgcn_sdot2(coef, __builtin_bit_cast(v2s, ab), nbase, false);
          const int e0 = (m0 - nd) & 0xFFFF;
          const int e1 = (m1 + 510 + nd) & 0xFFFF;
          const uint64_t mask = __ballot(e0 > e1);
          m = e0 < e1 ? e0 : e1;
          const int col = col0 + k;
          // the mask SGPRs were just written by a VALU compare: the hazard
          // recognizer does not see into inline asm, so the wait states the
          // v_writelane needs are explicit (without them the scheduler may
          // place the compare right before it and a stale mask is written)
          asm("s_nop 4\n\tv_writelane_b32 %0, %1, m0" : "+v"(lo) : "s"((uint32_t)mask), "{m0}"(col));
          asm("v_writelane_b32 %0, %1, m0" : "+v"(hi) : "s"((uint32_t)(mask >> 32)), "{m0}"(col));
        }
        hw = ((uint64_t)hi << 32) | lo;
      };
      if (w == 0)
        steps(h0);
      else if (w == 1)
        steps(h1);
      else
        steps(h2);
      i += run;
      pk += run;
      index = idx + run == HCAP ? 0 : idx + run;
      renorm += run;
      len += run;
      if (pk == 64) {
        pv = pairs(i);
        pk = 0;
      }
      if (renorm == RENORM) {
        renorm = 0;
        const int best = search(1);
        const int mind = __builtin_amdgcn_readlane(m, best);
        m = (m - mind) & 0xFFFF;
        if (len == HCAP) traceback(best, MINTB);
      } else if (len == HCAP) {
        traceback(search(1), MINTB);
      }
    }
  }
  int a = 0, b = 0;
  if (tail0 < sets) {
    a = sbuf[2 * tail0];
    b = sbuf[2 * tail0 + 1];
  }
  for (int i = tail0; i < sets; ++i) {
    // this step's symbols were read one step ahead (LDS latency off the chain)
    const int ca = a, cb = b;
    if (i + 1 < sets) {
      a = sbuf[2 * i + 2];
      b = sbuf[2 * i + 3];
    }
    const bool tail = i >= sets - 6;
    const int skip = tail ? (1 << (7 - (sets - i))) : 1;
    const int m0 = shfl_idx(m, s >> 1), m1 = shfl_idx(m, (s >> 1) | 32);
    const int e0 = (m0 + soft_dist(tab_lo, ca, cb)) & 0xFFFF;
    const int e1 = (m1 + soft_dist(tab_hi, ca, cb)) & 0xFFFF;
    const bool act = (s % skip) == 0;
    const int h = (e0 <= e1) ? 0 : 1;
    if (act) m = h ? e1 : e0;
    const uint64_t mask = __ballot(act && h);
    {
      const int w = __builtin_amdgcn_readfirstlane(index >> 6);
      const bool mine = lane == (index & 63);
      h0 = (mine && w == 0) ? mask : h0;
      h1 = (mine && w == 1) ? mask : h1;
      h2 = (mine && w == 2) ? mask : h2;
    }
    process(skip);
  }
  traceback(0, 0);
}

}  // namespace aero

namespace aero {

// Both codewords' tracebacks in one walk (their column schedule is the
// same): per column two v_readlane per codeword and a few scalar operations,
// the two path chains independent of each other.  Output bits (bit b
// descending) collect in one 64-bit scalar word per codeword, merged into
// lane b >> 6 of obw when the word is complete.  The caller advances outpos
// and len.
__device__ __forceinline__ void vit_traceback2(const uint64_t hA0, const uint64_t hA1, const uint64_t hA2,
                                               const uint64_t hB0, const uint64_t hB1, const uint64_t hB2,
                                               uint64_t &obwA, uint64_t &obwB, int bpA, int bpB, int mintb,
                                               int index, int len, int outpos, int lane) {
  const int nout = len - mintb;
  int idx = index;
  int j = 0;
  int bb = __builtin_amdgcn_readfirstlane(outpos + nout - 1);  // output bit of column j = mintb
  uint64_t accA = 0, accB = 0;
  auto flush = [&](int wd) {
    obwA = lane == wd ? (obwA | accA) : obwA;
    obwB = lane == wd ? (obwB | accB) : obwB;
    accA = 0;
    accB = 0;
  };
  while (j < len) {
    idx = idx == 0 ? HCAP - 1 : idx - 1;
    int run = (idx & 63) + 1;
    if (run > len - j) run = len - j;
    auto walk = [&](const uint64_t hwA, const uint64_t hwB) {
      for (int k = 0; k < run; ++k, ++j) {
        const int col = (idx - k) & 63;
        const uint64_t hvA = readlane64(hwA, col), hvB = readlane64(hwB, col);
        const int hbA = (int)((hvA >> bpA) & 1ULL), hbB = (int)((hvB >> bpB) & 1ULL);
        bpA = (bpA >> 1) | (hbA << 5);
        bpB = (bpB >> 1) | (hbB << 5);
        if (j >= mintb) {
          accA |= (uint64_t)hbA << (bb & 63);
          accB |= (uint64_t)hbB << (bb & 63);
          if ((bb & 63) == 0) flush(bb >> 6);
          --bb;
        }
      }
    };
    const int w = __builtin_amdgcn_readfirstlane(idx >> 6);
    if (w == 0)
      walk(hA0, hB0);
    else if (w == 1)
      walk(hA1, hB1);
    else
      walk(hA2, hB2);
    idx -= run - 1;
  }
  if (((bb + 1) & 63) != 0) flush((bb + 1) >> 6);  // the partly filled last word
}

// Two codewords of the same length in one wave: lane s holds state s's path
// metric of codeword A in its low 16 bits and of codeword B in its high 16
// bits.  The uint16 metric arithmetic of the single-codeword decoder is
// modulo 2^16, which is exactly what the packed 16-bit VALU operations
// compute, so one pair of bpermutes, one packed branch metric, two packed
// adds, a packed minimum and two compares advance both trellises a step; the
// renormalisation, traceback and output schedule depend only on the step
// count, so both codewords have their events at the same steps.  Same
// metrics, ties, renormalisation, history, traceback and tail as
// viterbi_decode_regs, so each codeword decodes to the same bits.
// Src::get(p, may_ov) returns soft value p of the codeword (called by every
// lane; may_ov: wave-uniform, p may fall in the overlap part); the soft
// pairs of the next 64 steps are fetched one run of 64 ahead, so the
// decoder needs no LDS.
template <class Src>
__device__ __forceinline__ void viterbi_decode_regs2(const Src &srcA, const Src &srcB, int nsoft, uint64_t &obwA,
                                                     uint64_t &obwB, int lane) {
  typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
  const int sets = nsoft / 2;
  const int s = lane;
  const int tab_lo = conv_table(s), tab_hi = conv_table(s | 64);
  uint64_t hA0 = 0, hA1 = 0, hA2 = 0, hB0 = 0, hB1 = 0, hB2 = 0;
  obwA = 0;
  obwB = 0;
  int mA = 0, mB = 0;
  for (int i = 0; i < 6 && i < sets; ++i) {
    const int pa = shfl_idx(mA, s >> 1), pb = shfl_idx(mB, s >> 1);
    const int aA = srcA.get(2 * i, true), bA = srcA.get(2 * i + 1, true);
    const int aB = srcB.get(2 * i, true), bB = srcB.get(2 * i + 1, true);
    if (s < (2 << i)) {
      mA = (soft_dist(conv_table(s), aA, bA) + pa) & 0xFFFF;
      mB = (soft_dist(conv_table(s), aB, bB) + pb) & 0xFFFF;
    }
  }
  int index = 0, len = 0, renorm = 0, outpos = 0;  // wave-uniform, shared by both codewords
  auto search = [&](int m, int skip) -> int {
    int key = (s % skip == 0) ? ((m << 6) | s) : 0x7FFFFFFF;
    for (int off = 32; off > 0; off >>= 1) {
      const int o = __shfl_xor(key, off, 64);
      key = o < key ? o : key;
    }
    return __builtin_amdgcn_readfirstlane(key) & 63;
  };
  auto traceback = [&](int bestA, int bestB, int mintb) {
    vit_traceback2(hA0, hA1, hA2, hB0, hB1, hB2, obwA, obwB, bestA, bestB, mintb, index, len, outpos, lane);
    const int nout = len - mintb;
    outpos += nout;
    len -= nout;
  };
  // process(skip) of the single decoder after its counters have advanced
  auto events = [&](int skip) {
    if (renorm == RENORM) {
      renorm = 0;
      const int bA = search(mA, skip), bB = search(mB, skip);
      mA = (mA - __builtin_amdgcn_readlane(mA, bA)) & 0xFFFF;
      mB = (mB - __builtin_amdgcn_readlane(mB, bB)) & 0xFFFF;
      if (len == HCAP) traceback(bA, bB, MINTB);
    } else if (len == HCAP) {
      traceback(search(mA, skip), search(mB, skip), MINTB);
    }
  };
  const int tail0 = sets - 6 > 6 ? sets - 6 : 6;
  {
    // branch metric soft_dist(tab_lo, a, b) = c0 + sa a + sb b with sa, sb =
    // +-1 (0xFFFF modulo 2^16); the s | 64 edge's metric is 510 minus it
    const unsigned short sa = (tab_lo & 1) ? 0xFFFF : 1, sb = (tab_lo & 2) ? 0xFFFF : 1;
    const unsigned short c0 = (unsigned short)(((tab_lo & 1) ? 255 : 0) + ((tab_lo & 2) ? 255 : 0));
    const u16x2 SA = {sa, sa}, SB = {sb, sb}, C0 = {c0, c0}, K510 = {510, 510};
    const int src0 = (s >> 1) << 2, src1 = ((s >> 1) | 32) << 2;
    // lane l: step i0 + l's a values (A low, B high) in pa, its b values in pb
    auto pairs = [&](int i0, uint32_t &pa, uint32_t &pb) {
      const int st = i0 + lane;
      const bool ov = 2 * i0 < 64;
      const uint32_t aA = (uint32_t)srcA.get(2 * st, ov), bA = (uint32_t)srcA.get(2 * st + 1, ov);
      const uint32_t aB = (uint32_t)srcB.get(2 * st, ov), bB = (uint32_t)srcB.get(2 * st + 1, ov);
      pa = st < sets ? aA | (aB << 16) : 0u;
      pb = st < sets ? bA | (bB << 16) : 0u;
    };
    uint32_t M = (uint32_t)mA | ((uint32_t)mB << 16);
    int i = 6;
    uint32_t pva, pvb, nva, nvb;
    pairs(6, pva, pvb);
    pairs(6 + 64, nva, nvb);
    int pk = 0;
    while (i < tail0) {
      const int idx = __builtin_amdgcn_readfirstlane(index);
      const int w = idx >> 6;
      int run = (w == 2 ? HCAP : 64 * (w + 1)) - idx;
      run = min(run, tail0 - i);
      run = min(run, RENORM - renorm);
      run = min(run, HCAP - len);
      run = min(run, 64 - pk);
      run = __builtin_amdgcn_readfirstlane(run);
      auto steps = [&](uint64_t &hwA, uint64_t &hwB) {
        uint32_t loA = (uint32_t)hwA, hiA = (uint32_t)(hwA >> 32);
        uint32_t loB = (uint32_t)hwB, hiB = (uint32_t)(hwB >> 32);
        const int col0 = idx & 63;
        for (int k = 0; k < run; ++k) {
          const uint32_t ap = (uint32_t)__builtin_amdgcn_readlane((int)pva, pk + k);
          const uint32_t bp = (uint32_t)__builtin_amdgcn_readlane((int)pvb, pk + k);
          const uint32_t m0 = (uint32_t)__builtin_amdgcn_ds_bpermute(src0, (int)M);
          const uint32_t m1 = (uint32_t)__builtin_amdgcn_ds_bpermute(src1, (int)M);
          const u16x2 d0 = SA * __builtin_bit_cast(u16x2, ap) + (SB * __builtin_bit_cast(u16x2, bp) + C0);
          u16x2 d1 = K510 - d0;
          asm volatile("" : "+v"(d1));  // both branch metrics off the metric chain
          const u16x2 e0 = __builtin_bit_cast(u16x2, m0) + d0, e1 = __builtin_bit_cast(u16x2, m1) + d1;
          const uint64_t maskA = __ballot(e0.x > e1.x), maskB = __ballot(e0.y > e1.y);
          M = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(e0, e1));
          const int col = col0 + k;
          // the mask SGPRs were just written by VALU compares: the wait
          // states the v_writelane needs are explicit (see viterbi_decode_regs)
          asm("s_nop 4\n\t"
              "v_writelane_b32 %0, %4, m0\n\t"
              "v_writelane_b32 %1, %5, m0\n\t"
              "v_writelane_b32 %2, %6, m0\n\t"
              "v_writelane_b32 %3, %7, m0"
              : "+v"(loA), "+v"(hiA), "+v"(loB), "+v"(hiB)
              : "s"((uint32_t)maskA), "s"((uint32_t)(maskA >> 32)), "s"((uint32_t)maskB),
                "s"((uint32_t)(maskB >> 32)), "{m0}"(col));
        }
        hwA = ((uint64_t)hiA << 32) | loA;
        hwB = ((uint64_t)hiB << 32) | loB;
      };
      if (w == 0)
        steps(hA0, hB0);
      else if (w == 1)
        steps(hA1, hB1);
      else
        steps(hA2, hB2);
      i += run;
      pk += run;
      index = idx + run == HCAP ? 0 : idx + run;
      renorm += run;
      len += run;
      if (pk == 64) {
        pva = nva;
        pvb = nvb;
        pairs(i + 64, nva, nvb);
        pk = 0;
      }
      if (renorm == RENORM || len == HCAP) {
        mA = (int)(M & 0xFFFFu);
        mB = (int)(M >> 16);
        events(1);
        M = (uint32_t)mA | ((uint32_t)mB << 16);
      }
    }
    mA = (int)(M & 0xFFFFu);
    mB = (int)(M >> 16);
  }
  for (int i = tail0; i < sets; ++i) {
    const int aA = srcA.get(2 * i, true), bA = srcA.get(2 * i + 1, true);
    const int aB = srcB.get(2 * i, true), bB = srcB.get(2 * i + 1, true);
    const bool tail = i >= sets - 6;
    const int skip = tail ? (1 << (7 - (sets - i))) : 1;
    const bool act = (s % skip) == 0;
    const int w = __builtin_amdgcn_readfirstlane(index >> 6);
    const bool mine = lane == (index & 63);
    {
      const int m0 = shfl_idx(mA, s >> 1), m1 = shfl_idx(mA, (s >> 1) | 32);
      const int e0 = (m0 + soft_dist(tab_lo, aA, bA)) & 0xFFFF, e1 = (m1 + soft_dist(tab_hi, aA, bA)) & 0xFFFF;
      const int h = (e0 <= e1) ? 0 : 1;
      if (act) mA = h ? e1 : e0;
      const uint64_t mask = __ballot(act && h);
      hA0 = (mine && w == 0) ? mask : hA0;
      hA1 = (mine && w == 1) ? mask : hA1;
      hA2 = (mine && w == 2) ? mask : hA2;
    }
    {
      const int m0 = shfl_idx(mB, s >> 1), m1 = shfl_idx(mB, (s >> 1) | 32);
      const int e0 = (m0 + soft_dist(tab_lo, aB, bB)) & 0xFFFF, e1 = (m1 + soft_dist(tab_hi, aB, bB)) & 0xFFFF;
      const int h = (e0 <= e1) ? 0 : 1;
      if (act) mB = h ? e1 : e0;
      const uint64_t mask = __ballot(act && h);
      hB0 = (mine && w == 0) ? mask : hB0;
      hB1 = (mine && w == 1) ? mask : hB1;
      hB2 = (mine && w == 2) ? mask : hB2;
    }
    index++;
    if (index == HCAP) index = 0;
    renorm++;
    len++;
    events(skip);
  }
  traceback(0, 0, 0);
}

}  // namespace aero
