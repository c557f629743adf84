/*
 * aerol.hip — AeroL P-channel link layer for 10500 bps on gfx950:
 *
 *  frame_kernel   : AeroL::Decode framing state machine, one channel per lane
 *                   (decode/aerol.cpp:1060-2038): phase-invariant UW search on
 *                   alternating arms, header, block fill; a full 64x78 block
 *                   becomes a Viterbi job (double-buffered per channel).
 *  viterbi_kernel : one wavefront per pair of jobs.  Deinterleave_ba on load
 *                   (decode/aerol.cpp:594-613), JConvolutionalCodec::
 *                   Decode_Continuous framing (decode/jconvolutionalcodec.cpp:
 *                   146-198) and the libcorrect soft Viterbi (r=1/2, K=7,
 *                   polys {109,79}; restated in oracle/aero_oracle.cpp): lane s
 *                   owns trellis state s of both codewords (16-bit metrics
 *                   packed in one register), predecessors arrive by
 *                   ds_bpermute, the 64 survivor decisions of a step are one
 *                   ballot word per codeword in registers.  Then DelayLine dl2, AeroLScrambler, LSB-first byte
 *                   packing and the per-SU CRC-16 (decode/aerol.cpp:1501-1556).
 *
 * The framing depends on the CRC results only through AeroL's data carrier
 * detect, and only when its 1 s DCD timer runs (AERO_F_DCD_TICK): datacd
 * gates the UW search (aerol.cpp:1096, 1108), the timer clears it once the
 * CRC failures have drained datacdcountdown (:1043-1058, :1545-1556).
 * Without the timer datacd becomes true at the first UW sync and stays true,
 * so the Viterbi/CRC work runs after the framing pass without changing any
 * framing decision.  With it, frame_kernel marks a completed frame's CRCs as
 * pending (its Viterbi runs after this framing pass) and stops a channel at
 * the first soft bit where they could matter: a DCD tick, or a bit whose UW
 * gate reads a datacd they could raise.  The next framing pass (after that
 * Viterbi, which leaves the frame's CRC-ok mask in IS_CRC_OKM) applies them
 * in the reference's order and goes on.  A UW sync in between overwrites
 * what they would have set (datacd = true, countdown = 12, :2010-2011).
 */
#include <hip/hip_runtime.h>

#include <climits>

#include "engine_common.h"
#include "viterbi_dev.h"

namespace aero {

constexpr uint32_t UW = 0xE15AE893u;  // 3780831379 (aerol.cpp:933-936)

// one SU CRC result on the DCD countdown (aerol.cpp:1545-1556); *edges
// counts datacd changes (SignalHunter::handleDcd)
__device__ __forceinline__ void dcd_su(bool ok, int &cd, int &datacd, int &edges) {
  if (ok) {
    if (cd < 12) cd += 2;
  } else {
    if (cd > 0) cd -= 3;
  }
  if (!datacd && cd > 2) {
    datacd = 1;
    edges++;
  }
}
// AeroL::updateDCD (aerol.cpp:1043-1058): a countdown of 2 goes to -1 and is
// clamped only at the next tick
__device__ __forceinline__ void dcd_tick(int &cd, int &datacd, int &edges) {
  if (cd > 0)
    cd -= 3;
  else if (cd < 0)
    cd = 0;
  if (datacd && !cd) {
    datacd = 0;
    edges++;
  }
}

__global__ __launch_bounds__(256) void frame_kernel(DevState S, int nch) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nch) return;
  const int C = S.C;
  int *is = S.is;
  long long *ls = S.ls;
  const long long P = ls[LS_SOFT_P * C + c];
  long long q = ls[LS_SOFT_C * C + c];
  const long long E = P & ~31LL;  // delivered in groups of 32 (oqpskdemodulator.cpp:534-540)
  const bool ticking = S.dcd_tick != 0;
  int tick_rec = 0, tick_done = 0, pend = 0;
  if (ticking) {
    tick_rec = is[IS_TICK_REC * C + c];
    tick_done = is[IS_TICK_DONE * C + c];
    pend = is[IS_CRC_PEND * C + c];
    if (tick_rec - tick_done > DCD_TICK_RING && S.err)  // cannot happen: the framing lags at most one pass
      __hip_atomic_store(S.err, DERR_TICKS, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (q >= E && tick_rec == tick_done && !pend) return;
  int realimag = is[IS_RI * C + c], cntr = is[IS_CNTR * C + c], gsl = is[IS_GSL * C + c];
  uint32_t uwi = (uint32_t)is[IS_UWI * C + c], uwr = (uint32_t)is[IS_UWR * C + c];
  int inv_i = is[IS_UWI_INV * C + c], inv_r = is[IS_UWR_INV * C + c];
  int frameinfo = is[IS_FRAMEINFO * C + c], lastframeinfo = is[IS_LASTFRAMEINFO * C + c];
  int formatid = is[IS_FORMATID * C + c], datacd = is[IS_DATACD * C + c];
  int scr_pos = is[IS_SCR_POS * C + c], blkbuf = is[IS_BLKBUF * C + c];
  int has_ov = is[IS_HAS_OVERLAP * C + c];
  int isu_reset = is[IS_DATACDCD * C + c];  // pending isudata.reset() for the next job
  int cd = is[IS_DCD_COUNT * C + c], edges = is[IS_DCD_EDGES * C + c];
  // the soft ring read 16 bytes at a time, the next group in flight (one
  // 1-byte load per bit, each waited for, was most of this kernel's time)
  const uint4 *soft16 = reinterpret_cast<const uint4 *>(S.soft + (size_t)c * SOFT_RING);
  constexpr int G16 = SOFT_RING / 16;
  long long grp = q >> 4;
  uint4 cur = soft16[grp & (G16 - 1)], nxt = soft16[(grp + 1) & (G16 - 1)];
  const int NumberOfBits = 4992, BitsInHeader = 194, Total = 5250;
  if (pend) {  // the last frame's SU CRCs, decoded since the previous pass
    const unsigned okm = (unsigned)is[IS_CRC_OKM * C + c];
    const int nsu = is[IS_CRC_NSU * C + c];
    for (int k = 0; k < nsu; ++k) dcd_su((okm >> k) & 1, cd, datacd, edges);
    pend = 0;
  }

  // the soft position of the next recorded tick, loaded once per tick (not per bit)
  auto tick_pos = [&](int k) {
    return k < tick_rec ? ls[(LS_TICK_SOFT0 + (k & (DCD_TICK_RING - 1))) * C + c] : LLONG_MAX;
  };
  long long tick_q = tick_pos(tick_done);
  for (;; ++q) {
    // DCD ticks due before soft bit q
    bool stop = false;
    while (tick_q <= q) {
      if (pend) {  // the countdown needs the CRCs of the frame that just ended
        stop = true;
        break;
      }
      dcd_tick(cd, datacd, edges);
      tick_done++;
      tick_q = tick_pos(tick_done);
    }
    if (stop || q >= E) break;
    // the gate below reads datacd, which pending CRCs could raise (a flywheel
    // frame after a tick cleared it); and a second frame end needs them too
    if (pend && ((!datacd && cntr >= 1 && cntr <= NumberOfBits - 68) || cntr + 1 - BitsInHeader == NumberOfBits - 1))
      break;
    if ((q >> 4) != grp) {  // q advances by one: the next group
      cur = nxt;
      grp++;
      nxt = soft16[(grp + 1) & (G16 - 1)];
    }
    const int wi = (int)(q >> 2) & 3;
    const uint32_t wd = wi == 0 ? cur.x : wi == 1 ? cur.y : wi == 2 ? cur.z : cur.w;
    const int sv = (int)((wd >> (8 * (q & 3))) & 0xFF);
    int bit = sv >= 128 ? 1 : 0;
    int soft_bit = sv;
    int gotsync;
    realimag++;
    realimag %= 2;
    const bool search = (cntr > NumberOfBits - 68 || cntr <= 0 || !datacd);
    if (search) {
      // PreambleDetectorPhaseInvariant::Update, tolerance 0 (aerol.cpp:757-777)
      uint32_t &reg = realimag ? uwi : uwr;
      int &inv = realimag ? inv_i : inv_r;
      reg = (reg << 1) | (uint32_t)bit;
      const int xorsum = __builtin_popcount(reg ^ UW);
      int g = 0;
      if (xorsum >= 32) {
        inv = 1;
        g = 1;
      } else if (xorsum <= 0) {
        inv = 0;
        g = 1;
      }
      gotsync = g;
      if (!gsl) {
        gsl = gotsync;
        gotsync = 0;
      } else
        gsl = 0;
    } else {
      gotsync = 0;
      gsl = 0;
    }
    if (realimag ? inv_i : inv_r) {
      bit = 1 - bit;
      if (soft_bit != 128) soft_bit = 255 - soft_bit;
    }
    if (cntr < 1000000000) cntr++;
    if (cntr < 16) {
      if (cntr == 0)
        frameinfo = bit;
      else
        frameinfo = ((frameinfo << 1) | bit) & 0xFFFF;
    }
    if (cntr == 15) {
      const int tval = frameinfo;
      frameinfo = lastframeinfo;
      lastframeinfo = tval;
      formatid = (frameinfo >> 12) & 0x000F;
    }
    if (cntr >= 16) {
      int idx = (cntr - BitsInHeader) % BLOCK;
      if (idx < 0) idx = 0;
      uint8_t *blk = S.block + ((size_t)c * 2 + blkbuf) * BLOCK;
      blk[idx] = (uint8_t)soft_bit;
      if (idx == BLOCK - 1) {
        const int j = atomicAdd(S.njobs, 1);
        int4 *jobs = reinterpret_cast<int4 *>(S.jobs);
        jobs[j] = make_int4(c, blkbuf | ((has_ov ? 0 : 1) << 1) | (isu_reset << 2), scr_pos,
                            ((cntr - BitsInHeader) == (NumberOfBits - 1) ? 0x100 : 0) | formatid);
        isu_reset = 0;
        scr_pos += has_ov ? 2496 : 2483;
        has_ov = 1;
        blkbuf ^= 1;
        // the SU CRCs of a completed frame update the DCD countdown
        // (aerol.cpp:1545-1556) once its Viterbi has run
        if (ticking && (cntr - BitsInHeader) == (NumberOfBits - 1)) pend = 1;
      }
    }
    if (gotsync) {
      if (cntr + 1 != Total) isu_reset = 1;
      cntr = -1;
      if (!datacd) edges++;  // SignalHunter::handleDcd: dcdChange(false, true)
      datacd = 1;
      cd = 12;
      pend = 0;  // what the pending CRCs would set, this overwrites
      scr_pos = 0;
    }
    if (cntr + 1 == Total) {
      scr_pos = 0;
      cntr = -1;
    }
  }
  ls[LS_SOFT_C * C + c] = q;
  is[IS_RI * C + c] = realimag;
  is[IS_CNTR * C + c] = cntr;
  is[IS_GSL * C + c] = gsl;
  is[IS_UWI * C + c] = (int)uwi;
  is[IS_UWR * C + c] = (int)uwr;
  is[IS_UWI_INV * C + c] = inv_i;
  is[IS_UWR_INV * C + c] = inv_r;
  is[IS_FRAMEINFO * C + c] = frameinfo;
  is[IS_LASTFRAMEINFO * C + c] = lastframeinfo;
  is[IS_FORMATID * C + c] = formatid;
  is[IS_DATACD * C + c] = datacd;
  is[IS_SCR_POS * C + c] = scr_pos;
  is[IS_BLKBUF * C + c] = blkbuf;
  is[IS_HAS_OVERLAP * C + c] = has_ov;
  is[IS_DATACDCD * C + c] = isu_reset;
  is[IS_DCD_COUNT * C + c] = cd;
  is[IS_DCD_EDGES * C + c] = edges;
  if (ticking) {
    is[IS_CRC_PEND * C + c] = pend;
    is[IS_TICK_DONE * C + c] = tick_done;
  }
}

// AeroL::Decode for continuous 600/1200 bps (decode/aerol.cpp:1060-2038 with
// useingOQPSK false, burstmode false): PreambleDetector::Update, an exact
// 32-bit UW match that clears its buffer on a hit (aerol.cpp:716-725), no
// phase inversion; 16 header bits + 1152 data bits in blocks of N x 64 +
// 32 UW bits per frame.  A job also carries whether the infofield was
// cleared (cntr == 0) since the previous block, so the host can assemble a
// frame's SUs from its blocks exactly as infofield is built (aerol.cpp:1509-1520).
template <int M>
__global__ __launch_bounds__(256) void frame_msk_kernel(DevState S, int nch) {
  constexpr int N = MskK<M>::LEAVER, B = N * 64;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nch) return;
  const int C = S.C;
  int *is = S.is;
  long long *ls = S.ls;
  const long long P = ls[LS_SOFT_P * C + c];
  long long q = ls[LS_SOFT_C * C + c];
  const long long E = P - P % 12;  // delivered in groups of 12 (mskdemodulator.cpp:404-407)
  if (q >= E) return;
  int cntr = is[IS_CNTR * C + c];
  uint32_t reg = (uint32_t)is[IS_MSK_PD * C + c];
  int frameinfo = is[IS_FRAMEINFO * C + c], lastframeinfo = is[IS_LASTFRAMEINFO * C + c];
  int formatid = is[IS_FORMATID * C + c];
  int scr_pos = is[IS_SCR_POS * C + c], blkbuf = is[IS_BLKBUF * C + c];
  int has_ov = is[IS_HAS_OVERLAP * C + c];
  int isu_reset = is[IS_DATACDCD * C + c];
  int since_clear = is[IS_BLK_SINCE_CLEAR * C + c];
  const uint8_t *soft = S.soft + (size_t)c * SOFT_RING;
  const int NumberOfBits = 1152, BitsInHeader = 16, Total = 16 + 1152 + 32;

  for (; q < E; ++q) {
    const int sv = soft[q & (SOFT_RING - 1)];
    const int bit = sv >= 128 ? 1 : 0;
    reg = (reg << 1) | (uint32_t)bit;
    const int gotsync = reg == UW;
    if (gotsync) reg = 0;
    if (cntr < 1000000000) cntr++;
    if (cntr < 16) {
      if (cntr == 0) {
        frameinfo = bit;
        since_clear = 0;  // infofield.clear()
      } else
        frameinfo = ((frameinfo << 1) | bit) & 0xFFFF;
    }
    if (cntr == 15) {
      const int tval = frameinfo;
      frameinfo = lastframeinfo;
      lastframeinfo = tval;
      formatid = (frameinfo >> 12) & 0x000F;
    }
    if (cntr >= 16) {
      int idx = (cntr - BitsInHeader) % B;
      if (idx < 0) idx = 0;
      uint8_t *blk = S.block + ((size_t)c * 2 + blkbuf) * B;
      blk[idx] = (uint8_t)sv;
      if (idx == B - 1) {
        const int j = atomicAdd(S.njobs, 1);
        int4 *jobs = reinterpret_cast<int4 *>(S.jobs);
        jobs[j] = make_int4(c, blkbuf | ((has_ov ? 0 : 1) << 1) | (isu_reset << 2) | ((since_clear == 0) << 3),
                            scr_pos, ((cntr - BitsInHeader) == (NumberOfBits - 1) ? 0x100 : 0) | formatid);
        isu_reset = 0;
        since_clear++;
        scr_pos += has_ov ? B / 2 : (B + 24) / 2 - 25;
        has_ov = 1;
        blkbuf ^= 1;
      }
    }
    if (gotsync) {
      if (cntr + 1 != Total) isu_reset = 1;
      cntr = -1;
      scr_pos = 0;
      if (!is[IS_DATACD * C + c]) {  // datacd = true (aerol.cpp:2010-2012), a change for SignalHunter::handleDcd
        is[IS_DATACD * C + c] = 1;
        is[IS_DCD_EDGES * C + c]++;
      }
    }
    if (cntr + 1 == Total) {
      scr_pos = 0;
      cntr = -1;
    }
  }
  ls[LS_SOFT_C * C + c] = q;
  is[IS_CNTR * C + c] = cntr;
  is[IS_MSK_PD * C + c] = (int)reg;
  is[IS_FRAMEINFO * C + c] = frameinfo;
  is[IS_LASTFRAMEINFO * C + c] = lastframeinfo;
  is[IS_FORMATID * C + c] = formatid;
  is[IS_SCR_POS * C + c] = scr_pos;
  is[IS_BLKBUF * C + c] = blkbuf;
  is[IS_HAS_OVERLAP * C + c] = has_ov;
  is[IS_DATACDCD * C + c] = isu_reset;
  is[IS_BLK_SINCE_CLEAR * C + c] = since_clear;
}

// ---------------------------------------------------------------- Viterbi
// BLK = interleaver block (N x 64 soft bits), N = BLK / 64; DL2 = dl2 length + 1.
// One wave per pair of jobs, ~1 KB of LDS and no per-step barrier
// (viterbi_decode_regs), launched between a coarse hop and a demod launch
// (engine.hip issue_viterbi).
#ifdef AERO_X_STAMPS
// diagnostic build only: s_memtime cycle totals of the Viterbi kernel's
// sections over every job (load + deinterleave, decode, post + record) and
// the job count
__device__ unsigned long long g_vstamps[4];
#define VSTAMP(k)                                               \
  do {                                                          \
    __builtin_amdgcn_sched_barrier(0);                          \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    vst_[k] += t_ - vtime_;                                     \
    vtime_ = t_;                                                \
    __builtin_amdgcn_sched_barrier(0);                          \
  } while (0)
#else
#define VSTAMP(k) \
  do {            \
  } while (0)
#endif

void viterbi_read_stamps(unsigned long long *out) {
#ifdef AERO_X_STAMPS
  hipMemcpyFromSymbol(out, HIP_SYMBOL(g_vstamps), sizeof(unsigned long long) * 4);
  unsigned long long z[4] = {0};
  hipMemcpyToSymbol(HIP_SYMBOL(g_vstamps), z, sizeof z);
#else
  for (int k = 0; k < 4; ++k) out[k] = 0;
#endif
}

// soft value p of a job's decoder input: the 62 overlap values of the
// previous block (lane p's ovr), then the block deinterleaved on the fly
// (deinterleave_ba, decode/aerol.cpp:594-613: position j * 64 + l comes from
// row (27 l) mod 64, column j), then erasures (128)
template <int BLK>
struct BlockSoft {
  const uint8_t *blk;
  int ov, ovr;
  // called by every lane; may_ov (wave-uniform): p may be an overlap position
  __device__ __forceinline__ int get(int p, bool may_ov) const {
    const int q = p - ov;
    int v = 128;
    if (q >= 0 && q < BLK) v = blk[(((q & 63) * 27) & 63) * (BLK / 64) + (q >> 6)];
    if (may_ov) {
      const int o = __builtin_amdgcn_ds_bpermute((p & 63) << 2, ovr);
      if (q < 0) v = o;
    }
    return v;
  }
};

template <int BLK, int DL2>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(6))) void viterbi_kernel(DevState S, DevTables T, int trace) {
  constexpr int NL = BLK / 64, HALF = BLK / 2;
  constexpr int NW = (62 + BLK + 24) / 2 / 64 + 1;  // 64-bit words of decoded bits
  __shared__ uint64_t obits[NW];
  __shared__ uint8_t info[320];
  // grid-stride over pairs of this pass's jobs (the job count stays on the
  // device, so the host launches without waiting for the framing kernel);
  // the two jobs of a pair decode in one wave (viterbi_decode_regs2) when
  // they have the same length and different channels, else one after the other
  const int njobs = *S.njobs;
  if (blockIdx.x == 0 && threadIdx.x == 0 && S.njobs_host) *S.njobs_host = njobs;
  const int lane = threadIdx.x;
  const int C = S.C;
  // a job's soft stream: overlap + deinterleaved block + 24 erasures, read by
  // the decoder straight from the block (no LDS copy); the old overlap is
  // taken into a register before this block's last 62 values replace it
  auto source = [&](int job) -> BlockSoft<BLK> {
    const int4 jd = reinterpret_cast<const int4 *>(S.jobs)[job];
    const int c = jd.x, buf = jd.y & 1, first = (jd.y >> 1) & 1;
    BlockSoft<BLK> b;
    b.blk = S.block + ((size_t)c * 2 + buf) * BLK;
    b.ov = first ? 0 : 62;
    b.ovr = (!first && lane < 62) ? S.overlap[(size_t)c * 64 + lane] : 0;
    if (lane < 62) S.overlap[(size_t)c * 64 + lane] = (uint8_t)b.get(b.ov + BLK - 62 + lane, false);
    return b;
  };
  // Decode_Continuous output, delay line, scrambler, SU CRCs and the job record
  auto post = [&](int job, int nsoft, uint64_t obw) {
    const int4 jd = reinterpret_cast<const int4 *>(S.jobs)[job];
    const int c = jd.x, reset = (jd.y >> 2) & 1, clear = (jd.y >> 3) & 1;
    const int scr_pos = jd.z, formatid = jd.w & 0xFF, frame_done = (jd.w >> 8) & 1;
    const int sets = nsoft / 2;
    __syncthreads();  // the previous post's reads of obits / info are done
    if (lane < NW) obits[lane] = obw;
    __syncthreads();
    auto obit = [&](int k) { return (int)((obits[k >> 6] >> (k & 63)) & 1ULL); };
    // Decode_Continuous: keep decoded bits [25, 25 + BLK/2) clipped to size/2
    const int nbits = (sets - 25) < HALF ? (sets - 25) : HALF;
    if (trace) {
      uint8_t *dbg = S.blocks_dbg + (size_t)c * 2500;
      if (lane == 0) *reinterpret_cast<int *>(dbg) = nbits;
      for (int k = lane; k < nbits; k += 64) dbg[4 + k] = (uint8_t)obit(25 + k);
    }
    // DelayLine dl2 (aerol.h:464-471): out[q] = old[(p+q+1)%L], new[(p+q)%L] = in[q]
    // (nbits < DL2: one wrap at most).  Each lane takes the eight bits of its
    // output bytes: all old values are read (and used) before any new one is
    // stored, as a neighbour's first read is this lane's last write.
    static_assert(HALF < DL2, "delay line longer than a block");
    uint8_t *dlg = S.dl2 + (size_t)c * DL2;
    const int p0 = S.is[IS_DL2_PTR * C + c];
    const int nbytes = nbits / 8;
    constexpr int BPL = (HALF / 8 + 63) / 64;  // output bytes per lane
    int bytev[BPL];
#pragma unroll
    for (int u = 0; u < BPL; ++u) {
      const int bb = lane + 64 * u;
      int v = 0;
      if (bb < nbytes) {
        // scrambler + LSB-first packing (aerol.cpp:1506-1520)
        for (int i = 0; i < 8; ++i) {
          int r = p0 + 8 * bb + i + 1;
          r = r >= DL2 ? r - DL2 : r;
          r = r >= DL2 ? r - DL2 : r;
          v |= ((dlg[r] ^ T.scr[scr_pos + 8 * bb + i]) & 1) << i;
        }
      }
      bytev[u] = v;
    }
#pragma unroll
    for (int u = 0; u < BPL; ++u) {
      const int bb = lane + 64 * u;
      if (bb < 312) info[bb] = (uint8_t)(bb < nbytes ? bytev[u] : 0);
    }
    for (int bb = lane + 64 * BPL; bb < 312; bb += 64) info[bb] = 0;
    __syncthreads();  // every old delay-line value read before the writes below
    for (int k = lane; k < nbits; k += 64) {
      int w = p0 + k;
      w = w >= DL2 ? w - DL2 : w;
      dlg[w] = (uint8_t)obit(25 + k);
    }
    if (lane == 0) S.is[IS_DL2_PTR * C + c] = (p0 + nbits) % DL2;
    // per-SU CRC (aerol.cpp:1531-1543); a 600/1200 frame spans 2-3 blocks and
    // its SUs are checked on the host once the frame's infofield is complete
    const int nsu = nbytes / 12;
    bool ok = false;
    if (lane < nsu && frame_done && BLK == BLOCK) {
      const uint8_t *su = info + 12 * lane;
      unsigned crc = 0xFFFF, sum = 0;
      for (int i = 0; i < 10; ++i) {
        unsigned mb = su[i];
        sum += mb;
        for (int k = 0; k < 8; ++k) {
          const unsigned bit = mb & 1;
          mb >>= 1;
          const unsigned cb = crc & 1;
          crc >>= 1;
          if (cb ^ bit) crc ^= 0x8408;
        }
      }
      unsigned calc = (~crc) & 0xFFFF;
      const unsigned rec = ((unsigned)su[11] << 8) | su[10];
      if (!rec && calc != rec && sum == 0) calc = 0;
      ok = calc == rec;
    }
    const unsigned long long okm = __ballot(ok);
    if (BLK == BLOCK && frame_done && lane == 0 && S.dcd_tick) {  // for frame_kernel's DCD countdown
      S.is[IS_CRC_OKM * C + c] = (int)(okm & 0x3FFFFFFULL);
      S.is[IS_CRC_NSU * C + c] = nsu;
    }
    uint8_t *out = S.jobout + (size_t)job * JOB_OUT;
    for (int b = lane; b < 312; b += 64) out[b] = info[b];
    if (lane == 0) {
      int *o = reinterpret_cast<int *>(out + 312);
      if (BLK == BLOCK) {
        o[0] = frame_done ? nbytes : -1;
        o[1] = (int)(okm & 0x3FFFFFFULL);
      } else {  // block bytes; bit 8: frame done, bit 9: infofield cleared before this block
        o[0] = nbytes | (frame_done << 8) | (clear << 9);
        o[1] = 0;
      }
      o[2] = formatid;
      o[3] = c | (reset << 30);
    }
  };
  for (int pj = blockIdx.x; 2 * pj < njobs; pj += gridDim.x) {
    __syncthreads();  // LDS of the previous pair fully consumed
#ifdef AERO_X_STAMPS
    unsigned long long vst_[4] = {0, 0, 0, 0}, vtime_ = __builtin_amdgcn_s_memtime();
#endif
    const int jobA = 2 * pj, jobB = 2 * pj + 1;
    bool paired = false;
    if (jobB < njobs) {
      const int4 ja = reinterpret_cast<const int4 *>(S.jobs)[jobA];
      const int4 jb = reinterpret_cast<const int4 *>(S.jobs)[jobB];
      // same length (both continue or both start a stream), different channels
      // (a channel's second block would read the overlap this one writes)
      paired = ja.x != jb.x && ((ja.y ^ jb.y) & 2) == 0;
    }
    if (paired) {
      const BlockSoft<BLK> sa = source(jobA), sb = source(jobB);
      const int nsoft = sa.ov + BLK + 24;
      VSTAMP(0);
      uint64_t obwA, obwB;
      viterbi_decode_regs2(sa, sb, nsoft, obwA, obwB, lane);
      VSTAMP(1);
      post(jobA, nsoft, obwA);
      post(jobB, nsoft, obwB);
      VSTAMP(2);
    } else {
      for (int job = jobA; job <= jobB && job < njobs; ++job) {
        const BlockSoft<BLK> sa = source(job);
        const int nsoft = sa.ov + BLK + 24;
        VSTAMP(0);
        uint64_t obw, unused;
        viterbi_decode_regs2(sa, sa, nsoft, obw, unused, lane);
        VSTAMP(1);
        post(job, nsoft, obw);
        VSTAMP(2);
      }
    }
#ifdef AERO_X_STAMPS
    if (lane == 0) {
      for (int k = 0; k < 3; ++k) atomicAdd(&g_vstamps[k], vst_[k]);
      atomicAdd(&g_vstamps[3], 1ull);
    }
#endif
  }  // pair loop
}

void launch_frame_c(hipStream_t st, const DevState &S, int nch);                             // cchan.hip
void launch_viterbi_c(hipStream_t st, const DevState &S, const DevTables &T, int max_jobs);  // cchan.hip

void launch_frame(hipStream_t st, int mode, const DevState &S, int nch) {
  const dim3 g((nch + 255) / 256), b(256);
  if (mode == MODE_C8400) return launch_frame_c(st, S, nch);
  // MSK framing depends on the AeroL bit rate only
  if (mode == MODE_OQPSK)
    hipLaunchKernelGGL(frame_kernel, g, b, 0, st, S, nch);
  else if (msk_bitrate(mode) == 600)
    hipLaunchKernelGGL(frame_msk_kernel<MODE_MSK600>, g, b, 0, st, S, nch);
  else
    hipLaunchKernelGGL(frame_msk_kernel<MODE_MSK1200>, g, b, 0, st, S, nch);
}

// max_jobs: an upper bound of the pass's job count (the count itself is read
// on the device); the grid is capped, blocks stride over the jobs
void launch_viterbi(hipStream_t st, int mode, const DevState &S, const DevTables &T, int max_jobs, int trace) {
  if (max_jobs <= 0) return;
  if (mode == MODE_C8400) return launch_viterbi_c(st, S, T, max_jobs);
  max_jobs = (max_jobs + 1) / 2;  // one block per pair of jobs
  max_jobs = max_jobs < 16384 ? max_jobs : 16384;
  if (mode == MODE_OQPSK)
    hipLaunchKernelGGL((viterbi_kernel<BLOCK, DL2_LEN>), dim3(max_jobs), dim3(64), 0, st, S, T, trace);
  else if (msk_bitrate(mode) == 600)
    hipLaunchKernelGGL((viterbi_kernel<6 * 64, MSK_DL2_LEN>), dim3(max_jobs), dim3(64), 0, st, S, T, trace);
  else
    hipLaunchKernelGGL((viterbi_kernel<9 * 64, MSK_DL2_LEN>), dim3(max_jobs), dim3(64), 0, st, S, T, trace);
}

}  // namespace aero
