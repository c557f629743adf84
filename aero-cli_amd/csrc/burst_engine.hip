/*
 * burst_engine.hip — host side of the burst-mode groups (aero-decode --burst,
 * decode/decode.cpp:123-140, 171-212): one group of 10500-bps OQPSK channels
 * and one of 600/1200-bps MSK channels.  Device layout and initial state
 * (BurstOqpskDemodulator ctor + setSettings, decode/burstoqpskdemodulator.cpp:5-232;
 * BurstMskDemodulator ctor + setSettings, decode/burstmskdemodulator.cpp:9-297;
 * AeroL::setSettings(fb, burst), decode/aerol.cpp:960-1039), one message per
 * push (the OQPSK lastmse gate makes its output depend on message boundaries,
 * burstoqpskdemodulator.cpp:264, 685), the pass loop over the kernels of
 * burst.hip / burst_msk.hip, and the R/T test results: descrambling, CRC
 * checks and packet handling of RTChannelDeleaveFECScram::update / updateMSK
 * (decode/aerol.h:614-836) and the R/T branch of AeroL::Decode
 * (decode/aerol.cpp:1240-1460).
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <map>
#include <string>
#include <vector>

#include "../../include/aero_engine.h"
#include "acars_host.h"
#include "burst_common.h"
#include "burst_engine.h"
#include "engine_common.h"
#include "host_pool.h"
#include "tables_host.h"

namespace aero {

void burst_upload_constants(const double *sr_b, const double *sr_a, const double *taps);
void launch_hk_spectrum(hipStream_t st, const BurstTables &T, double2 *hk);
void launch_hilbert(hipStream_t st, const BurstState &S, const BurstTables &T, int nch);
void launch_front_burst(hipStream_t st, const BurstState &S, const BurstTables &T, int nch);
void launch_demod_burst(hipStream_t st, const BurstState &S, const BurstTables &T, int nch, int trace);
void launch_trident(hipStream_t st, const BurstState &S, const BurstTables &T, int nch);
void launch_frame_burst(hipStream_t st, const BurstState &S, int nch);
void launch_rt_viterbi(hipStream_t st, const BurstState &S, int max_jobs);
void burst_msk_upload_constants(const double *sr_b, const double *sr_a, const double *taps);
void launch_front_bmsk(hipStream_t st, const BurstState &S, const BurstTables &T, int nch);
void launch_demod_bmsk(hipStream_t st, const BurstState &S, const BurstTables &T, int nch, int trace);
void launch_trident_bmsk(hipStream_t st, const BurstState &S, const BurstTables &T, int nch);
void launch_frame_bmsk(hipStream_t st, const BurstState &S, int nch);

namespace {

#define BCHK(x)                                                                        \
  do {                                                                                 \
    hipError_t err__ = (x);                                                            \
    if (err__ != hipSuccess) {                                                         \
      fprintf(stderr, "aero_engine(burst): %s failed: %s\n", #x, hipGetErrorString(err__)); \
      return AERO_E_HIP;                                                               \
    }                                                                                  \
  } while (0)

constexpr long long B_PCM_CAP = 32768;
constexpr int B_HOP_CAP = 256;

__global__ void b_scatter_kernel(int16_t *ring, long long cap, const int16_t *src, long long n, int c,
                                 long long start) {
  int16_t *row = ring + (size_t)c * cap;
  for (long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x; k < n; k += (long long)gridDim.x * blockDim.x)
    row[(start + k) & (cap - 1)] = src[k];
}

// lockstep batch of one message per channel: src time-major [n][ld], channel
// j < nch at its own pushed count (the device copy, stream-ordered).  The
// ring is channel-major (the Hilbert stage reads a channel's block as one
// run of lines), so each 64 x 64 tile goes through the LDS: read as rows of
// 64 channels (one line each), written as rows of 64 samples of one channel.
constexpr int BTILE = 64;
__global__ __launch_bounds__(256) void b_batch_scatter_kernel(int16_t *ring, long long cap, const int16_t *src,
                                                              long long n, long long ld, int nch,
                                                              const long long *avail) {
  __shared__ int16_t tile[BTILE][BTILE + 2];  // row stride 33 dwords: the column reads hit 64 banks
  const long long t0 = (long long)blockIdx.x * BTILE;
  const int j0 = blockIdx.y * BTILE;
  const int lane = threadIdx.x & 63, r0 = threadIdx.x >> 6;
  for (int r = r0; r < BTILE; r += 4) {
    const long long t = t0 + r;
    if (t < n && j0 + lane < nch) tile[r][lane] = src[t * ld + j0 + lane];
  }
  __syncthreads();
  for (int r = r0; r < BTILE; r += 4) {
    const int j = j0 + r;
    const long long t = t0 + lane;
    if (j < nch && t < n) ring[(size_t)j * cap + ((avail[j] + t) & (cap - 1))] = tile[lane][r];
  }
}

// the batch's message starts and pushed counts (after the scatter read them)
__global__ void b_batch_counts_kernel(long long *ls, long long *chunks, int C, int nch, long long n) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nch) return;
  const long long start = ls[(size_t)BL_AVAIL * C + j];
  const long long k = ls[(size_t)BL_CHUNK_N * C + j];
  chunks[(size_t)j * CHUNK_RING + (k & (CHUNK_RING - 1))] = start;
  ls[(size_t)BL_CHUNK_N * C + j] = k + 1;
  ls[(size_t)BL_AVAIL * C + j] = start + n;
}

template <class T>
T *carve(char *&p, size_t count) {
  T *r = reinterpret_cast<T *>(p);
  p += (count * sizeof(T) + 255) & ~size_t(255);
  return r;
}

// AeroLcrc16::calcusingbitsandcheck (decode/aerol.h:273-307)
bool crc_bits_check(const int *bits, int numberofbits) {
  uint16_t crc_rec = 0;
  for (int i = numberofbits - 1; i >= numberofbits - 16; i--) {
    crc_rec <<= 1;
    crc_rec |= bits[i];
  }
  numberofbits -= 16;
  uint16_t crc = 0xFFFF;
  for (int i = 0; i < numberofbits; i++) {
    const int crc_bit = crc & 1;
    crc >>= 1;
    if (crc_bit ^ bits[i]) crc = crc ^ 0x8408;
  }
  crc = ~crc;
  return crc_rec == crc;
}

// RTChannelDeleaveFECScram::packintobytes: LSB first
std::vector<uint8_t> pack_bits(const std::vector<int> &bits) {
  std::vector<uint8_t> out;
  int charptr = 0;
  uint8_t ch = 0;
  for (size_t h = 0; h < bits.size(); h++) {
    ch |= bits[h] * 128;
    charptr++;
    charptr %= 8;
    if (charptr == 0) {
      out.push_back(ch);
      ch = 0;
    } else {
      ch >>= 1;
    }
  }
  return out;
}

}  // namespace

struct BurstGroup {
  int device = 0, flags = 0, C = 0, nch = 0, kind = BURST_OQPSK;
  HostPool *hpool = nullptr;  // the engine's host threads (R/T tests by channel)
  std::vector<int> tsu, tblocks;  // MSK: updateMSK's targetSUSize / targetBlocks per channel
  hipStream_t st = nullptr;
  BurstState S{};
  BurstTables T{};
  void *pool = nullptr;
  std::vector<long long> avail, chunk_n;
  std::vector<std::unique_ptr<PChannelHost>> host;
  std::vector<int> ok_burst;
  std::vector<std::vector<int16_t>> soft_hold;
  std::vector<long long> soft_seen;
  std::vector<std::vector<double>> hop_hold;
  std::vector<int> hops_seen;
  std::vector<std::vector<uint8_t>> tests_hold, packets_hold;
  std::vector<uint8_t> scr;
  int16_t *d_scratch = nullptr;
  size_t scratch_cap = 0;
  uint64_t processed = 0;
  uint64_t st_tests = 0, st_packets = 0;  // aero_stat "rt_tests" / "rt_packets"
  uint64_t st_pass_max = 0;               // aero_stat "rt_pass_max": most R/T tests of one pass
  // AERO_F_TIMING: HIP-event milliseconds and launches per kernel name
  std::map<std::string, std::pair<double, long>> timing;
  std::vector<std::pair<std::string, std::pair<hipEvent_t, hipEvent_t>>> pending_ev;
  long long last_work = -1;
  std::vector<long long> hb_base;  // first sample the Hilbert stage still needs (host mirror)
  // initial state of channels [init_lo, nch), uploaded field by field before the next push or run
  int init_lo = 0;
  std::vector<double> init_ds;  // [field][channel - init_lo]
  std::vector<int> init_is;
  std::vector<int> since_run;      // messages pushed since the last run (message-start ring)
};

namespace {

size_t burst_layout(int kind, BurstState &S, BurstTables &T, int C, char *base, double2 **hk_out) {
  const bool msk = kind == BURST_MSK;
  char *p = base;
  S.C = C;
  S.hop_n = carve<int>(p, (size_t)C);
  S.ds = carve<double>(p, (size_t)BURST_DS_COUNT * C);
  S.is = carve<int>(p, (size_t)BURST_IS_COUNT * C);
  S.ls = carve<long long>(p, (size_t)BL_COUNT * C);
  S.fir = carve<double>(p, (size_t)2 * (msk ? M_NT : NTAPS) * C);
  S.ana = carve<double2>(p, (size_t)ANA_LEN * C);
  S.pcm = carve<int16_t>(p, (size_t)B_PCM_CAP * C);
  S.pcm_cap = B_PCM_CAP;
  S.hb_rem = carve<double2>(p, (size_t)HB_REM * C);
  S.agc = carve<double>(p, (size_t)B_AGC * C);
  S.agc2 = carve<double>(p, (size_t)(msk ? M_AGC2 : B_AGC2) * C);
  S.d1 = carve<double>(p, (size_t)(msk ? M_D1 : B_D1) * C);
  S.vring = carve<double>(p, (size_t)(msk ? MV_LEN : BV_LEN) * C);
  S.ma1 = carve<double2>(p, (size_t)(msk ? M_MA : B_MA) * C);
  S.mav1 = carve<double>(p, (size_t)(msk ? M_MA : B_MA) * C);
  if (msk) {  // bt_d1 (complex), bt_ma_diff, a1, delayt8, delayedsmpl (complex)
    const int sz[5] = {2 * M_BTD, M_MADIFF, M_A1, M_D8, 2 * M_DSM};
    for (int k = 0; k < 5; k++) S.dl[k] = carve<double>(p, (size_t)sz[k] * C);
  } else {
    for (int k = 0; k < BDL_COUNT; k++)  // sizes <= 1172 (bt_ma_diff); BDL_BT holds double2
      S.dl[k] = carve<double>(p, (size_t)(k == BDL_BT ? 2 : 1) * 1172 * C);
  }
  S.pd3 = carve<double>(p, (size_t)(msk ? M_PD3 : B_PD3) * C);
  S.tri = carve<double>(p, (size_t)TRI_SLOTS * (msk ? M_TRI : B_TRI) * C);
  S.chk_n = carve<long long>(p, (size_t)TRI_SLOTS * C);
  S.chk = carve<double>(p, (size_t)TRI_SLOTS * CHK_REC * C);
  S.tjobs = carve<int>(p, (size_t)TRI_SLOTS * C);
  S.ntjobs = carve<int>(p, 16);
  S.msema = carve<double>(p, (size_t)(msk ? M_MSEMA : B_MSEMA) * C);
  S.chunks = carve<long long>(p, (size_t)CHUNK_RING * C);
  S.soft = carve<int16_t>(p, (size_t)B_SOFT_RING * C);
  S.hop_cap = B_HOP_CAP;
  S.hops = carve<double>(p, (size_t)B_HOP_CAP * 6 * C);
  S.rtblock = carve<uint8_t>(p, (size_t)RT_BLOCK * C);
  S.jobs = carve<int>(p, (size_t)4 * RT_TESTS_PER_PASS * C);
  S.njobs = carve<int>(p, 16);
  S.jobout = carve<uint8_t>(p, (size_t)RT_JOB_OUT * RT_TESTS_PER_PASS * C);
  S.tri_abs = carve<double>(p, (size_t)(msk ? 1 : TRI_N) * TRI_GRID);
  T.cis = carve<double2>(p, WTSIZE);
  T.tw8 = carve<double2>(p, 8192);
  T.twi8 = carve<double2>(p, 8192);
  T.tw16 = carve<double2>(p, 16384);
  double2 *hk = carve<double2>(p, HB_N);
  T.hk = hk;
  if (hk_out) *hk_out = hk;
  T.hk_time = carve<double2>(p, HB_N);
  T.da = carve<double2>(p, TRI_N);
  T.db = carve<double2>(p, TRI_N);
  T.taps = carve<double>(p, 128);
  for (int k = 0; k < BDL_COUNT; k++) {
    T.dw[k] = carve<double>(p, 1172);
    T.domw[k] = carve<double>(p, 1172);
    T.dio[k] = carve<int>(p, 1172);
  }
  return (size_t)(p - base);
}

template <class V>
int h2d(const V *dst, const std::vector<V> &src) {
  BCHK(hipMemcpy((void *)dst, src.data(), src.size() * sizeof(V), hipMemcpyHostToDevice));
  return AERO_OK;
}

// times one launch (AERO_F_TIMING); collected after run_once's stream sync
template <class F>
void timed(BurstGroup *g, const char *name, F &&launch) {
  if (!(g->flags & AERO_F_TIMING)) {
    launch();
    return;
  }
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a, g->st);
  launch();
  hipEventRecord(b, g->st);
  g->pending_ev.push_back({name, {a, b}});
}

void collect_timing(BurstGroup *g) {
  for (auto &pe : g->pending_ev) {
    float ms = 0;
    hipEventSynchronize(pe.second.second);
    hipEventElapsedTime(&ms, pe.second.first, pe.second.second);
    auto &t = g->timing[pe.first];
    t.first += ms;
    t.second++;
    hipEventDestroy(pe.second.first);
    hipEventDestroy(pe.second.second);
  }
  g->pending_ev.clear();
}

// one pass's kernels (asynchronous)
int launch_pass(BurstGroup *g, bool trace) {
  const int nch = g->nch;
  const bool msk = g->kind == BURST_MSK;
  // Hilbert FIR -> front end (runs ahead, records the trident checks it
  // completes) -> the checks' decisions -> the demodulator up to the front
  // end, applying each decision at its sample
  timed(g, "burst_hilbert", [&] { launch_hilbert(g->st, g->S, g->T, nch); });
  BCHK(hipMemsetAsync(g->S.ntjobs, 0, sizeof(int), g->st));
  if (msk) {
    timed(g, "burst_front", [&] { launch_front_bmsk(g->st, g->S, g->T, nch); });
    timed(g, "burst_trident", [&] { launch_trident_bmsk(g->st, g->S, g->T, nch); });
    timed(g, "burst_demod", [&] { launch_demod_bmsk(g->st, g->S, g->T, nch, trace ? 1 : 0); });
  } else {
    timed(g, "burst_front", [&] { launch_front_burst(g->st, g->S, g->T, nch); });
    timed(g, "burst_trident", [&] { launch_trident(g->st, g->S, g->T, nch); });
    timed(g, "burst_demod", [&] { launch_demod_burst(g->st, g->S, g->T, nch, trace ? 1 : 0); });
  }
  BCHK(hipMemsetAsync(g->S.njobs, 0, sizeof(int), g->st));
  if (msk)
    timed(g, "burst_frame", [&] { launch_frame_bmsk(g->st, g->S, nch); });
  else
    timed(g, "burst_frame", [&] { launch_frame_burst(g->st, g->S, nch); });
  timed(g, "burst_viterbi", [&] { launch_rt_viterbi(g->st, g->S, nch * RT_TESTS_PER_PASS); });
  return AERO_OK;
}

// waits for the pass, takes its R/T test records and counters, runs the
// parity traces, and says whether another pass has work
int finish_pass(BurstGroup *g, bool trace, std::vector<uint8_t> &jobs, int &njobs, bool &progress) {
  const int nch = g->nch;
  BCHK(hipGetLastError());
  njobs = 0;
  BCHK(hipMemcpyAsync(&njobs, g->S.njobs, sizeof(int), hipMemcpyDeviceToHost, g->st));
  std::vector<long long> ls((size_t)BL_COUNT * g->C);
  BCHK(hipMemcpyAsync(ls.data(), g->S.ls, ls.size() * 8, hipMemcpyDeviceToHost, g->st));
  BCHK(hipStreamSynchronize(g->st));
  jobs.resize((size_t)std::max(njobs, 1) * RT_JOB_OUT);
  if (njobs > 0)
    BCHK(hipMemcpy(jobs.data(), g->S.jobout, (size_t)njobs * RT_JOB_OUT, hipMemcpyDeviceToHost));
  // traces: committed soft entries (with the start-of-packet markers) and trident records
  if (g->flags & AERO_F_TRACE_SOFT) {
    std::vector<int16_t> ring;
    for (int c = 0; c < nch; c++) {
      const long long com = ls[(size_t)BL_SCOMMIT * g->C + c];
      if (com <= g->soft_seen[c]) continue;
      if (ring.empty()) {
        ring.resize((size_t)B_SOFT_RING * nch);
        BCHK(hipMemcpy(ring.data(), g->S.soft, ring.size() * 2, hipMemcpyDeviceToHost));
      }
      for (long long k = g->soft_seen[c]; k < com; k++) {
        const int e = ring[(size_t)c * B_SOFT_RING + (k & (B_SOFT_RING - 1))] & 0x1FF;
        g->soft_hold[c].push_back(e == B_SOFT_MARK ? (int16_t)-1 : (int16_t)e);
      }
      g->soft_seen[c] = com;
    }
  }
  if (g->flags & AERO_F_TRACE_HOPS) {  // trident records of this pass, then the counters restart
    std::vector<int> hn(nch);
    BCHK(hipMemcpy(hn.data(), g->S.hop_n, sizeof(int) * nch, hipMemcpyDeviceToHost));
    std::vector<double> hops;
    for (int c = 0; c < nch; c++) {
      if (hn[c] <= 0) continue;
      if (hn[c] > B_HOP_CAP) return AERO_E_FULL;
      if (hops.empty()) {
        hops.resize((size_t)B_HOP_CAP * 6 * nch);
        BCHK(hipMemcpy(hops.data(), g->S.hops, hops.size() * 8, hipMemcpyDeviceToHost));
      }
      g->hop_hold[c].insert(g->hop_hold[c].end(), hops.begin() + (size_t)c * B_HOP_CAP * 6,
                            hops.begin() + ((size_t)c * B_HOP_CAP + hn[c]) * 6);
    }
    BCHK(hipMemset(g->S.hop_n, 0, sizeof(int) * nch));
  }
  // more passes while any channel has samples or committed soft bits left
  long long work = 0;
  for (int c = 0; c < nch; c++) {
    work += (g->avail[c] - ls[(size_t)BL_NSAMP * g->C + c]) +
            (ls[(size_t)BL_SCOMMIT * g->C + c] - ls[(size_t)BL_SCONS * g->C + c]);
  }
  progress = work > 0 && (work != g->last_work || njobs > 0);
  g->last_work = work;
  return AERO_OK;
}


// the host side of a pass's R/T tests (RTChannelDeleaveFECScram::update /
// updateMSK: descramble, CRCs, packet assembly, ACARS)
void process_tests(BurstGroup *g, const std::vector<uint8_t> &jobs, int njobs) {
  const int nch = g->nch;
  const bool msk = g->kind == BURST_MSK;
  // R/T tests in emission order (a channel's tests come from one lane, in
  // order).  Every piece of state a test touches is its channel's, so the
  // tests are split over the host pool by channel (c % T == t), each thread
  // taking its channels' tests in emission order.
  const int T = (g->hpool && njobs >= 256) ? std::min(g->hpool->size(), std::max(1, njobs / 128)) : 1;
  g->st_pass_max = std::max<uint64_t>(g->st_pass_max, (uint64_t)std::max(njobs, 0));
  std::vector<uint64_t> n_tests(T, 0), n_packets(T, 0);
  auto tests = [&](int t, int TT) {
  std::vector<int> deconvol;
  for (int j = 0; j < njobs; j++) {
    const uint8_t *rec = jobs.data() + (size_t)j * RT_JOB_OUT;
    int h[4];
    memcpy(h, rec, 16);
    const int c = h[0], bp = h[1], burst = h[2], nbits = h[3];
    if (c < 0 || c >= nch || c % TT != t) continue;
    if (burst == g->ok_burst[c]) continue;  // packet already decoded: the block is FULL
    deconvol.assign(nbits, 0);
    for (int b = 0; b < nbits; b++) deconvol[b] = ((rec[16 + b / 8] >> (7 - (b % 8))) & 1) ^ g->scr[b];
    enum { OK_R = 3, OK_T = 5, Bad = 0, Test_Failed = 32, Nothing = 8 };
    int result, nsus = 0;
    std::vector<uint8_t> info;
    if (msk) {
      // RTChannelDeleaveFECScram::updateMSK (decode/aerol.h:614-753): only
      // blocks 5, 11, 50 and the target block are tests
      const int blocks = bp / 64;
      int &tsu = g->tsu[c], &tb = g->tblocks[c];
      if (!(blocks == 5 || blocks == tb || blocks == 11 || blocks == 50)) continue;
      if (bp == 64 * 5) {
        tsu = 0;
        tb = 0;
        if (crc_bits_check(deconvol.data(), 8 * 19)) {
          info = pack_bits(deconvol);
          result = OK_R;
        } else {
          result = Nothing;
        }
      } else if (!crc_bits_check(deconvol.data(), 8 * 6)) {
        result = Bad;
      } else if (blocks == 11) {  // peek at the SU after the first for the SU count
        const int *isu = deconvol.data() + (8 * 6) + (8 * 12) * 1;
        int bin = 2;
        bin += ((isu[0] * 1) + (isu[1] * 2) + (isu[2] * 4) + (isu[3] * 8) + (isu[4] * 16) + (isu[5] * 32));
        tsu = bin;
        if (tsu >= 16) tsu = tsu / 2 + 1;
        tb = ((tsu + 1) * 3) + 2;
        result = Nothing;
      } else if (blocks == tb) {  // `ok <= targetSUSize` always holds
        info = pack_bits(deconvol);
        if (!info.empty()) info.pop_back();  // infofield.chop(1)
        nsus = tsu;
        result = OK_T;
      } else {
        result = Nothing;
      }
    } else if (bp == 64 * 5) {
      if (!crc_bits_check(deconvol.data(), 8 * 19)) {
        result = Test_Failed;
      } else {
        info = pack_bits(deconvol);
        result = OK_R;
      }
    } else if (!crc_bits_check(deconvol.data(), 8 * 6)) {
      result = bp >= RT_BLOCK ? Bad : Test_Failed;
    } else {
      nsus = 1 + (bp - (64 * 5)) / (64 * 3);
      result = OK_T;
      for (int i = 0; i < nsus; i++)
        if (!crc_bits_check(deconvol.data() + (8 * 6) + (8 * 12) * i, 8 * 12)) {
          result = bp >= RT_BLOCK ? Bad : Test_Failed;
          break;
        }
      if (result == OK_T) {
        info = pack_bits(deconvol);
        if (!info.empty()) info.pop_back();  // infofield.chop(1)
      }
    }
    n_tests[t]++;
    if (g->flags & AERO_F_TRACE_FRAMES) {
      const uint32_t t2[2] = {(uint32_t)bp, (uint32_t)result};
      g->tests_hold[c].insert(g->tests_hold[c].end(), (const uint8_t *)t2, (const uint8_t *)t2 + 8);
    }
    if (result == OK_R || result == OK_T) {
      n_packets[t]++;
      g->ok_burst[c] = burst;
      if (g->flags & AERO_F_TRACE_FRAMES) {
        const uint32_t p2[2] = {(uint32_t)(result == OK_R ? 'R' : 'T'), (uint32_t)info.size()};
        auto &ph = g->packets_hold[c];
        ph.insert(ph.end(), (const uint8_t *)p2, (const uint8_t *)p2 + 8);
        ph.insert(ph.end(), info.begin(), info.end());
      }
      g->host[c]->rt_packet(result == OK_R, info.data(), (int)info.size(), nsus);
    }
  }
  };
  if (T > 1) {
    g->hpool->submit(tests, T);
    g->hpool->wait();
  } else {
    tests(0, 1);
  }
  for (int t = 0; t < T; t++) {
    g->st_tests += n_tests[t];
    g->st_packets += n_packets[t];
  }
}

}  // namespace

int burst_group_create(int device, int flags, int max_channels, int kind, BurstGroup **out) {
  // every early return below releases what was already allocated
  std::unique_ptr<BurstGroup, void (*)(BurstGroup *)> g(new BurstGroup(), burst_group_destroy);
  g->device = device;
  g->flags = flags;
  g->kind = kind;
  const bool msk = kind == BURST_MSK;
  g->C = (max_channels + 63) & ~63;
  BurstState S{};
  BurstTables T{};
  const size_t bytes = burst_layout(kind, S, T, g->C, nullptr, nullptr) + 4096;
  if (hipMalloc(&g->pool, bytes) != hipSuccess) return AERO_E_NOMEM;
  BCHK(hipMemset(g->pool, 0, bytes));
  double2 *hk = nullptr;
  burst_layout(kind, g->S, g->T, g->C, reinterpret_cast<char *>(g->pool), &hk);
  BCHK(hipStreamCreateWithFlags(&g->st, hipStreamNonBlocking));
  // tables (host glibc, g++-compiled: tables_host.cpp)
  std::vector<double> cis(2 * WTSIZE), tw8(2 * 8192), twi8(2 * 8192), tw16(2 * 16384), twi16(2 * 16384);
  host_cis(cis.data());
  host_twiddles(8192, tw8.data(), twi8.data());
  host_twiddles(16384, tw16.data(), twi16.data());
  std::vector<double> hk_time(2 * HB_N), da(2 * TRI_N), db(2 * TRI_N), taps(128, 0.0);
  host_hilbert_kernel(hk_time.data());
  host_fftr_split(TRI_N, da.data(), db.data());
  if (msk)
    host_msk_taps(40, taps.data());  // matched filter, SamplesPerSymbol 40 (burstmskdemodulator.cpp:142-149)
  else if (host_rrc(1.0, 55, 48000, 10500 / 2.0, taps.data()) != NTAPS)
    return AERO_E_INVALID;
  if (int rc = h2d((const double *)g->T.cis, cis)) return rc;
  if (int rc = h2d((const double *)g->T.tw8, tw8)) return rc;
  if (int rc = h2d((const double *)g->T.twi8, twi8)) return rc;
  if (int rc = h2d((const double *)g->T.tw16, tw16)) return rc;
  if (int rc = h2d((const double *)g->T.hk_time, hk_time)) return rc;
  if (int rc = h2d((const double *)g->T.da, da)) return rc;
  if (int rc = h2d((const double *)g->T.db, db)) return rc;
  if (int rc = h2d(g->T.taps, taps)) return rc;
  // Delay<> instances (burstoqpskdemodulator.cpp:186-196, 213-216); the MSK
  // group's delays are whole samples (burst_dev.h dly_int)
  const double fds[BDL_COUNT] = {1.0, (2.0 * 48000.0 / 10500.0) / 4.0, (2.0 * 48000.0 / 10500.0) / 4.0,
                                 (2.0 * 48000.0 / 10500.0) / 8.0, (2.0 * 48000.0 / 10500.0) / 2.0,
                                 1.0 * (2.0 * 48000.0 / 10500.0), (2.0 * 48000.0 / 10500.0) * 128};
  for (int k = 0; k < BDL_COUNT && !msk; k++) {
    std::vector<double> w(1172), omw(1172);
    std::vector<int> io(1172);
    const int size = host_delay_table(fds[k], w.data(), omw.data(), io.data(), 1172);
    if (size <= 0) return AERO_E_INVALID;
    // burst_dev.h dly_pre reads slots p + 1 and p + 2: the reference's older
    // slot must be p + 1 for every write pointer p
    for (int q = 0; q < size; q++)
      if (io[q] != (q + 1) % size) return AERO_E_INVALID;
    if (k == BDL_BT && size <= 2) return AERO_E_INVALID;  // dly_pre2 has no newer-is-sig case
    // the part-B delays and the front end's bt_d1 live in registers
    // (burst.hip): their sizes are compile-time and their weights must not
    // depend on the write pointer
    const int reg_n[BDL_COUNT] = {BDL_N_S, BDL_N_41, BDL_N_42, BDL_N_8, BDL_N_A1, BDL_N_BT, 0};
    if (reg_n[k]) {
      if (size != reg_n[k]) return AERO_E_INVALID;
      for (int q = 1; q < size; q++)
        if (w[q] != w[0] || omw[q] != omw[0]) return AERO_E_INVALID;
    }
    g->T.dsize[k] = size;
    if (int rc = h2d(g->T.dw[k], w)) return rc;
    if (int rc = h2d(g->T.domw[k], omw)) return rc;
    if (int rc = h2d(g->T.dio[k], io)) return rc;
  }
  if (msk) {  // 600 Hz resonator at 48 kHz, 4 Hz bandwidth (burstmskdemodulator.cpp:214-227)
    const double sr_b[3] = {2.617308727964618e-04, 0, -2.617308727964618e-04};
    const double sr_a[3] = {1, -1.993312819378528, 0.999476538254407};
    burst_msk_upload_constants(sr_b, sr_a, taps.data());
  } else {
    const double sr_b[3] = {0.0048847995518126464, 0, -0.0048847995518126464};
    const double sr_a[3] = {1, -0.3882746897971619, 0.99023040089637471};
    burst_upload_constants(sr_b, sr_a, taps.data());
  }
  launch_hk_spectrum(g->st, g->T, hk);
  BCHK(hipGetLastError());
  BCHK(hipStreamSynchronize(g->st));
  g->scr.resize(5000);
  host_scrambler(g->scr.data());
  *out = g.release();
  return AERO_OK;
}

void burst_group_set_pool(BurstGroup *g, HostPool *pool) {
  if (g) g->hpool = pool;
}

void burst_group_destroy(BurstGroup *g) {
  if (!g) return;
  if (g->st) (void)hipStreamSynchronize(g->st);
  if (g->d_scratch) (void)hipFree(g->d_scratch);
  if (g->pool) (void)hipFree(g->pool);
  if (g->st) (void)hipStreamDestroy(g->st);
  delete g;
}

int burst_open(BurstGroup *g, int bitrate, bool disable_reassembly, int *local) {
  if (g->nch >= g->C) return AERO_E_FULL;
  const int c = g->nch;
  const int C = g->C;
  std::vector<double> ds(BURST_DS_COUNT, 0.0);
  std::vector<int> is(BURST_IS_COUNT, 0);
  if (g->kind == BURST_MSK) {
    if (bitrate != 600 && bitrate != 1200) return AERO_E_INVALID;
    // BurstMskDemodulator ctor + setSettings (burstmskdemodulator.cpp:9-297):
    // mixer2 at freq_center 1000, st_osc / st_osc_half at fb / 2; AeroL MSK
    // burst window ifb * 3 bits (aerol.cpp:1031-1038)
    ds[BM_M2_FREQ] = 1000;
    ds[BM_M2_STEP] = (1000.0) * ((double)WTSIZE) / ((float)48000);
    ds[BM_SO_STEP] = ds[BM_SH_STEP] = (1200 / 2.0) * ((double)WTSIZE) / ((float)48000);
    ds[BM_AVE_RE] = ds[BM_ROT_RE] = ds[BM_STR_RE] = 1;
    ds[BM_MSE] = 10.0;
    ds[BM_DIFF_LAST] = -1;  // DiffDecode lastsoftstate (DSP.h)
    is[BMI_PD_CNTDOWN] = M_PD_MAXCD;
    is[BMI_PD_MAXPOSCD] = -1;
    is[BMI_STARTSTOP] = -1;
    is[BMI_FCNTR] = 1000000000;
    is[BMI_TOTAL] = bitrate * 3;
  } else {
    if (bitrate != 10500) return AERO_E_INVALID;
    // BurstOqpskDemodulator ctor + setSettings (burstoqpskdemodulator.cpp:5-232) and AeroL burst state
    ds[BD_M2_FREQ] = 8000;  // freq_center (burstoqpskdemodulator.h:33)
    ds[BD_M2_STEP] = (8000.0) * ((double)WTSIZE) / ((float)48000);
    ds[BD_SO_FREQ] = 10500;
    ds[BD_SO_STEP] = (10500.0) * ((double)WTSIZE) / ((float)48000);
    ds[BD_Q_STEP] = (10500.0 / 4.0) * ((double)WTSIZE) / ((float)48000);
    ds[BD_VOL_GAIN] = 1;
    ds[BD_AVE_RE] = ds[BD_ROT_RE] = ds[BD_STR_RE] = 1;
    ds[BD_MSE] = 100;
    ds[BD_LASTMSE] = 100;
    is[BI_PD_CNTDOWN] = B_PD_MAXCD;
    is[BI_PD_MAXPOSCD] = -1;
    is[BI_STARTSTOP] = -1;
    is[BI_FCNTR] = 1000000000;
  }
  // the device copy waits for the next push or run (flush_init): one copy per
  // field for every channel opened since, not one per field per channel
  (void)C;
  g->init_ds.insert(g->init_ds.end(), ds.begin(), ds.end());
  g->init_is.insert(g->init_is.end(), is.begin(), is.end());
  g->nch++;
  g->avail.push_back(0);
  g->chunk_n.push_back(0);
  g->host.emplace_back(new PChannelHost(disable_reassembly));
  g->ok_burst.push_back(-1);
  g->soft_hold.emplace_back();
  g->soft_seen.push_back(0);
  g->hop_hold.emplace_back();
  g->hops_seen.push_back(0);
  g->tests_hold.emplace_back();
  g->packets_hold.emplace_back();
  g->hb_base.push_back(0);
  g->since_run.push_back(0);
  g->tsu.push_back(0);
  g->tblocks.push_back(0);
  *local = c;
  return AERO_OK;
}

// initial device state of the channels opened since the last push or run
static int flush_init(BurstGroup *g) {
  const int n = g->nch - g->init_lo;
  if (n <= 0) return AERO_OK;
  std::vector<double> col(n);
  std::vector<int> icol(n);
  for (int f = 0; f < BURST_DS_COUNT; f++) {
    for (int k = 0; k < n; k++) col[k] = g->init_ds[(size_t)k * BURST_DS_COUNT + f];
    BCHK(hipMemcpy(g->S.ds + (size_t)f * g->C + g->init_lo, col.data(), 8 * n, hipMemcpyHostToDevice));
  }
  for (int f = 0; f < BURST_IS_COUNT; f++) {
    for (int k = 0; k < n; k++) icol[k] = g->init_is[(size_t)k * BURST_IS_COUNT + f];
    BCHK(hipMemcpy(g->S.is + (size_t)f * g->C + g->init_lo, icol.data(), 4 * n, hipMemcpyHostToDevice));
  }
  g->init_lo = g->nch;
  g->init_ds.clear();
  g->init_is.clear();
  return AERO_OK;
}

int burst_run(BurstGroup *g, int flush) {
  (void)flush;  // every pushed sample is processed (burst output depends on message boundaries only)
  if (!g || !g->nch) return AERO_OK;
  BCHK(hipSetDevice(g->device));
  if (int rc = flush_init(g)) return rc;
  const bool trace = (g->flags & (AERO_F_TRACE_HOPS | AERO_F_TRACE_SOFT)) != 0;
  g->last_work = -1;
  std::vector<uint8_t> jobs;
  int njobs = 0;
  bool more = false;
  if (int rc = launch_pass(g, trace)) return rc;
  if (int rc = finish_pass(g, trace, jobs, njobs, more)) return rc;
  for (int guard = 0; guard < 100000; guard++) {
    // the next pass is launched before this pass's R/T tests are handled on
    // the host (they only touch host state), so that work overlaps the GPU;
    // parity traces read device state between passes and keep them apart
    if (more && !trace)
      if (int rc = launch_pass(g, trace)) return rc;
    process_tests(g, jobs, njobs);
    if (!more) break;
    if (trace)
      if (int rc = launch_pass(g, trace)) return rc;
    if (int rc = finish_pass(g, trace, jobs, njobs, more)) return rc;
  }
  for (int c = 0; c < g->nch; c++) {
    g->hb_base[c] = (g->avail[c] / HB_SNZ) * HB_SNZ;
    g->since_run[c] = 0;
  }
  return AERO_OK;
}

// one message (Decoder::audioReceived -> BurstOqpskDemodulator::dataReceived)
int burst_push(BurstGroup *g, int c, const int16_t *pcm, size_t n, bool dev, bool msg_start) {
  if (!n) return AERO_OK;
  BCHK(hipSetDevice(g->device));
  if (int rc = flush_init(g)) return rc;
  const int C = g->C;
  if ((long long)n > B_PCM_CAP / 2) return AERO_E_FULL;  // one message is at most 16384 samples here
  // never outrun the PCM ring (the Hilbert stage reads from hb_base on) or
  // the message-start ring: process what is pending first
  if (g->avail[c] + (long long)n - g->hb_base[c] > B_PCM_CAP - 2 || g->since_run[c] >= CHUNK_RING - 1)
    if (int rc = burst_run(g, 0)) return rc;
  const int16_t *src = pcm;
  if (!dev) {
    if (n > g->scratch_cap) {
      if (g->d_scratch) (void)hipFree(g->d_scratch);
      g->d_scratch = nullptr;
      g->scratch_cap = 0;
      BCHK(hipMalloc(&g->d_scratch, n * sizeof(int16_t)));
      g->scratch_cap = n;
    }
    BCHK(hipMemcpyAsync(g->d_scratch, pcm, n * sizeof(int16_t), hipMemcpyHostToDevice, g->st));
    src = g->d_scratch;
  }
  const long long start = g->avail[c];
  const int grid = (int)std::min<long long>(((long long)n + 255) / 256, 4096);
  hipLaunchKernelGGL(b_scatter_kernel, dim3(grid), dim3(256), 0, g->st, g->S.pcm, B_PCM_CAP, src, (long long)n, c,
                     start);
  BCHK(hipGetLastError());
  // message start (lastmse capture) and the new pushed count
  if (msg_start) {
    const long long k = g->chunk_n[c];
    BCHK(hipMemcpyAsync(g->S.chunks + (size_t)c * CHUNK_RING + (k & (CHUNK_RING - 1)), &start, 8,
                        hipMemcpyHostToDevice, g->st));
    g->chunk_n[c] = k + 1;
    g->since_run[c]++;
  }
  g->avail[c] = start + (long long)n;
  BCHK(hipMemcpyAsync(g->S.ls + (size_t)BL_CHUNK_N * C + c, &g->chunk_n[c], 8, hipMemcpyHostToDevice, g->st));
  BCHK(hipMemcpyAsync(g->S.ls + (size_t)BL_AVAIL * C + c, &g->avail[c], 8, hipMemcpyHostToDevice, g->st));
  BCHK(hipStreamSynchronize(g->st));  // the host values copied above and the caller's buffer are free again
  g->processed += n;
  return AERO_OK;
}

// aero_push_pcm_batch for burst channels [0, nch): one message of n samples
// per channel (the reference's message boundaries are what the caller's
// batch boundaries are), src a device pointer or host memory
int burst_push_batch(BurstGroup *g, const int16_t *src, size_t n, size_t ld, int nch, bool dev) {
  if (!n) return AERO_OK;
  if (nch > g->nch) return AERO_E_INVALID;
  BCHK(hipSetDevice(g->device));
  if (int rc = flush_init(g)) return rc;
  const int C = g->C;
  if ((long long)n > B_PCM_CAP / 2) return AERO_E_FULL;
  bool need_run = false;
  for (int c = 0; c < nch; c++)
    need_run |= g->avail[c] + (long long)n - g->hb_base[c] > B_PCM_CAP - 2 || g->since_run[c] >= CHUNK_RING - 1;
  if (need_run)
    if (int rc = burst_run(g, 0)) return rc;
  const int16_t *d = src;
  const size_t need = (n - 1) * ld + nch;
  if (!dev) {
    if (need > g->scratch_cap) {
      BCHK(hipStreamSynchronize(g->st));
      if (g->d_scratch) (void)hipFree(g->d_scratch);
      g->d_scratch = nullptr;
      g->scratch_cap = 0;
      BCHK(hipMalloc(&g->d_scratch, need * sizeof(int16_t)));
      g->scratch_cap = need;
    }
    BCHK(hipMemcpyAsync(g->d_scratch, src, need * sizeof(int16_t), hipMemcpyHostToDevice, g->st));
    d = g->d_scratch;
  }
  const dim3 tiles((unsigned)(((long long)n + BTILE - 1) / BTILE), (unsigned)((nch + BTILE - 1) / BTILE));
  hipLaunchKernelGGL(b_batch_scatter_kernel, tiles, dim3(256), 0, g->st, g->S.pcm, B_PCM_CAP, d, (long long)n,
                     (long long)ld, nch, (const long long *)(g->S.ls + (size_t)BL_AVAIL * C));
  hipLaunchKernelGGL(b_batch_counts_kernel, dim3((nch + 255) / 256), dim3(256), 0, g->st, g->S.ls, g->S.chunks, C,
                     nch, (long long)n);
  BCHK(hipGetLastError());
  for (int c = 0; c < nch; c++) {
    g->chunk_n[c]++;
    g->since_run[c]++;
    g->avail[c] += (long long)n;
  }
  BCHK(hipStreamSynchronize(g->st));  // the caller's buffer is free again
  g->processed += (uint64_t)n * nch;
  return AERO_OK;
}

template <class T>
static int pop_v(std::vector<T> &v, T *dst, size_t cap, size_t *n) {
  const size_t k = std::min(cap, v.size());
  if (dst && k) memcpy(dst, v.data(), k * sizeof(T));
  if (n) *n = k;
  v.erase(v.begin(), v.begin() + k);
  return AERO_OK;
}

int burst_pop_soft(BurstGroup *g, int c, int16_t *dst, size_t cap, size_t *n) {
  return pop_v(g->soft_hold[c], dst, cap, n);
}
int burst_pop_hops(BurstGroup *g, int c, double *dst, size_t cap_records, size_t *n) {
  size_t k = 0;
  int rc = pop_v(g->hop_hold[c], dst, cap_records * 6, &k);
  if (n) *n = k / 6;
  return rc;
}
int burst_pop_tests(BurstGroup *g, int c, uint8_t *dst, size_t cap, size_t *n) {
  return pop_v(g->tests_hold[c], dst, cap, n);
}
int burst_pop_packets(BurstGroup *g, int c, uint8_t *dst, size_t cap, size_t *n) {
  return pop_v(g->packets_hold[c], dst, cap, n);
}
std::vector<aero_acars_item> &burst_items(BurstGroup *g, int c) { return g->host[c]->items; }
uint64_t burst_processed(const BurstGroup *g) { return g ? g->processed : 0; }
int burst_dcd_edges(BurstGroup *g, int c, int64_t *edges) {
  if (!g || c < 0 || c >= g->nch) return AERO_E_INVALID;
  BCHK(hipSetDevice(g->device));
  if (int rc = flush_init(g)) return rc;
  BCHK(hipStreamSynchronize(g->st));
  const int f = g->kind == BURST_MSK ? BMI_DCD_EDGES : BI_DCD_EDGES;
  int v = 0;
  BCHK(hipMemcpy(&v, g->S.is + (size_t)f * g->C + c, sizeof(int), hipMemcpyDeviceToHost));
  *edges = v;
  return AERO_OK;
}

uint64_t burst_stat(const BurstGroup *g, int which) {
  if (!g) return 0;
  return which == 2 ? g->st_pass_max : (which ? g->st_packets : g->st_tests);
}
void burst_timing(BurstGroup *g, const char *name, double *ms, long *launches) {
  if (!g) return;
  collect_timing(g);
  auto it = g->timing.find(name);
  if (it == g->timing.end()) return;
  *ms += it->second.first;
  *launches += it->second.second;
}
void burst_timing_reset(BurstGroup *g) {
  if (!g) return;
  collect_timing(g);
  g->timing.clear();
}
int burst_sync(BurstGroup *g) {
  if (!g) return AERO_OK;
  BCHK(hipStreamSynchronize(g->st));
  return AERO_OK;
}

}  // namespace aero
