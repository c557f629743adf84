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
