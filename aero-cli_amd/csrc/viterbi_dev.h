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
