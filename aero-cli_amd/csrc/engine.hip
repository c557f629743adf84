/*
 * engine.hip — host side of the Aero engine: the C ABI of
 * include/aero_engine.h, device allocation, host-computed tables (the same
 * glibc calls the reference makes: decode/DSP.cpp:10-33, decode/DSP.h:325-351,
 * decode/jfft.cpp:13-67, decode/mskdemodulator.cpp:126-133) and the per-run
 * kernel schedule of each channel kind (10500 OQPSK, 600 / 1200 MSK)
 *
 *   [demod segment] -> [coarse hop + decision] -> [AeroL framing] -> [Viterbi+post]
 *
 * repeated until every channel has consumed its pushed samples up to a hop
 * boundary (aero_run) or to the end (aero_flush).
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <chrono>
#include <climits>
#include <deque>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <map>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../../include/aero_engine.h"
#include "acars_host.h"
#include "burst_engine.h"
#include "aero_math.h"
#include "engine_common.h"
#include "fft_layout.h"
#include "host_pool.h"
#include "engine_internal.h"
#include "tables_host.h"

namespace aero {
void launch_demod(hipStream_t, const DevState &, const DevTables &, int, int, bool, bool);
void upload_demod_constants(const double *, const DelayDesc *, const double *, const double *, const double *,
                            const double *);
void launch_demod_msk(hipStream_t, int, const DevState &, const DevTables &, int, int, bool);
void upload_msk_constants(const double *);
void demod_read_stamps(unsigned long long *);
void coarse_read_stamps(unsigned long long *);
void viterbi_read_stamps(unsigned long long *);
void burst_read_stamps(unsigned long long *);
void launch_coarse(hipStream_t, int, const DevState &, const DevTables &, int);
void launch_frame(hipStream_t, int, const DevState &, int);
void launch_viterbi(hipStream_t, int, const DevState &, const DevTables &, int, int);
// the C channel (cchan.hip)
void launch_prefilter_c(hipStream_t, const DevState &, const DevTables &, const void *, int);
void launch_demod_c(hipStream_t, const DevState &, const DevTables &, int, bool);
void upload_c_constants(const DelayDesc *);
int c_prejob_bytes();
}  // namespace aero

using namespace aero;

namespace {

constexpr int GENERIC_GROUP_CAP = 256;  // channels per generic-rate MSK group
constexpr long long PCM_CAP = 65536;  // per-channel PCM ring: a second of 48 kHz audio per run without an early pass
constexpr int PT_CAP = 4096;
constexpr int HOP_CAP = 64;

#define HIPCHK(x)                                   \
  do {                                              \
    hipError_t err__ = (x);                         \
    if (err__ != hipSuccess) {                      \
      fprintf(stderr, "aero_engine: %s failed: %s\n", #x, hipGetErrorString(err__)); \
      return AERO_E_HIP;                            \
    }                                               \
  } while (0)

__global__ void pcm_scatter_kernel(int16_t *ring, int C, long long capm, const int16_t *src, long long n, long long ld,
                                   int nch, int c0, long long start) {
  // src time-major [n][ld]; channel c0 + j, j < nch; ring slot (start + t) & capm
  const long long total = n * nch;
  for (long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x; k < total;
       k += (long long)gridDim.x * blockDim.x) {
    const long long t = k / nch;
    const int j = (int)(k - t * nch);
    ring[((start + t) & capm) * C + c0 + j] = src[t * ld + j];
  }
}

// one gather item: a device PCM run for one channel (aero_chan_feed, or a
// queued host message); `later` = a later job of the same launch sets the
// channel's counter (jobs run in parallel)
struct GatherJob {
  const int16_t *src;
  long long n, start, avail_after;
  int c, later;
};

__global__ void pcm_gather_kernel(int16_t *ring, int C, long long capm, long long *avail, const GatherJob *jobs) {
  const GatherJob j = jobs[blockIdx.y];
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < j.n; t += (long long)gridDim.x * blockDim.x)
    ring[((j.start + t) & capm) * C + j.c] = j.src[t];
  if (!j.later && blockIdx.x == 0 && threadIdx.x == 0) avail[j.c] = j.avail_after;  // LS_AVAIL row
}

__global__ void math_kernel(int fn, const double *x, const double *y, double *out, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double a = x[i], b = y[i];
  double r = 0;
  switch (fn) {
    case 0: r = aero_hypot(a, b); break;
    case 1: r = aero_atan2(a, b); break;
    case 2: r = aero_tanh(a); break;
    case 3: r = aero_sin(a); break;
    case 4: r = aero_cos(a); break;
    case 5: r = aero_log10(a); break;
    case 6: r = sqrt(a); break;
    case 7: r = fmod(a, 360.0); break;
    case 8: r = a / b; break;
    // the short exact division / sqrt sequences (aero_math.h) against the
    // IEEE operations above (tests/test_gpu_math.py)
    case 9: r = div_c(a, 48000.0); break;
    case 10: r = div_c(a, 360.0); break;
    case 11: r = div_n(a, b); break;
    case 13: r = div_c(a, 192000.0); break;
    case 14: r = aero_hypot_nr(a, b); break;
    case 15: r = aero_atan2_bf(a, b, aero_g_cij); break;
    case 16: r = aero_tanh_bf(a); break;
    case 17: { double sn, cs; aero_sincos_bf(a, sn, cs, aero_g_sincostab); r = sn; break; }
    case 18: { double sn, cs; aero_sincos_bf(a, sn, cs, aero_g_sincostab); r = cs; break; }
    case 19: r = div_cw(a, (double)WTSIZE); break;
    case 20: r = set_phase_ptr(a); break;
    default: break;
  }
  out[i] = r;
}

struct TimingSlot {
  double ms = 0;
  long launches = 0;
};

// wall-clock host section timer (AERO_F_TIMING), reported as "host_<name>"
struct HostTimer {
  std::map<std::string, TimingSlot> *t;
  const char *name;
  std::chrono::steady_clock::time_point t0;
  HostTimer(std::map<std::string, TimingSlot> *tm, const char *n) : t(tm), name(n) {
    if (t) t0 = std::chrono::steady_clock::now();
  }
  ~HostTimer() {
    if (!t) return;
    auto &slot = (*t)[name];
    slot.ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    slot.launches++;
  }
};
#define HT_CAT2(a, b) a##b
#define HT_CAT(a, b) HT_CAT2(a, b)
#define HOST_TIMER(e, n) HostTimer HT_CAT(_ht_, __LINE__)(((e)->flags & AERO_F_TIMING) ? &(e)->timing : nullptr, n)

}  // namespace


// One group per channel kind: OQPSK, each fixed-rate MSK Mode, and each
// (bit rate, Fs) of the generic-rate MSK kernels; its own device pool,
// stream, tables and kernels.  aero_engine routes every channel to its
// group (engine group id gid: the Mode for the fixed kinds, above MODE_COUNT
// for generic-rate groups).
struct Group {
  ~Group();  // releases every device/host resource (also on a failed group_create)
  int mode = MODE_OQPSK;  // kernel family: a Mode, MODE_MSKG600 or MODE_MSKG1200
  int gid = 0;            // engine group id
  // the few-channel demod kernels (16 lanes per channel, demod_oqpsk.hip /
  // demod_msk.hip) run while nch <= wide_max (AERO_OQPSK_WIDE /
  // AERO_MSK_WIDE, default WIDE_MAX_DEFAULT; 0: never)
  int wide_max = 0;
  ModeGeom g{};
  int device = 0, flags = 0, C = 0, nch = 0;
  std::string tag;  // timing-name prefix ("" for OQPSK, "msk600_", "msk1200_", "msk600_48k_", "msk600_16000_", ...)
  hipStream_t st = nullptr;
  DevState S{};
  DevTables T{};
  void *pool = nullptr;
  size_t pool_bytes = 0;
  HostPool *hpool = nullptr;  // the engine's
  std::vector<aero_channel_cfg> cfg;
  std::vector<int> gch;  // local -> engine channel id (-1: a free slot)
  // local slots an MSK channel left for another rate's group (msk_migrate),
  // reused by the next channel added to this group (group_add_channel)
  std::vector<int> free_slots;
  // host mirrors of the per-channel counters
  std::vector<long long> avail, nsamp, hops;
  std::vector<std::unique_ptr<PChannelHost>> host;
  std::vector<std::vector<uint8_t>> infofield;  // 600/1200: the frame being assembled from its blocks
  std::vector<std::vector<int16_t>> soft_hold;
  std::vector<std::vector<double>> hop_hold, pt_hold;
  std::vector<std::vector<uint8_t>> blk_hold, frame_hold;
  std::vector<long long> soft_seen;
  // samples the channel demodulated before it moved into this group (an MSK
  // rate change): hop records count from the channel's first sample
  std::vector<long long> hop_base;
  // the C channel (MODE_C8400): the pushed messages' ends not yet
  // prefiltered, the prefiltered end (host mirror of LS_PRE_END), decoded
  // Call_progress SUs and voice frames, AeroL's DCD countdown (aerol.cpp:2300-2315)
  int job_out = JOB_OUT;  // bytes per Viterbi job record
  std::vector<std::deque<long long>> msg_end;
  std::vector<long long> pre_end;
  std::vector<std::vector<uint8_t>> cunit_hold, voice_hold;
  std::vector<int> c_cd, c_dcd, c_edges;
  void *pin_cjobs[4] = {}, *d_cjobs[4] = {};
  hipEvent_t cjob_ev[4] = {};
  int next_cjob = 0;
  // aero_trace_select: host-side trace collection for these local channels
  // only (empty: every channel)
  bool trace_some = false;
  std::vector<int> trace_list;
  std::vector<uint8_t> trace_mask;
  bool traced(int c) const { return !trace_some || trace_mask[c]; }
  // scratch
  int16_t *d_scratch = nullptr;
  size_t scratch_cap = 0;
  std::vector<uint8_t> h_dbg;
  // Asynchronous frame hand-off.  A pass that demodulates lists its Viterbi
  // jobs in one of NSLOT slots; the Viterbi kernel writes the job records and
  // the job count straight into the slot's mapped pinned host buffers, and
  // the host SU/ACARS work for them starts once the slot's event (recorded
  // after that kernel) has completed, while the GPU runs on.  aero_run
  // therefore never waits for the GPU.
  struct JobSlot {
    int *d_n = nullptr;         // job count (device)
    int *d_jobs = nullptr;      // [C] int4 job list of this pass (device)
    hipEvent_t ev_vit = nullptr;  // this pass's Viterbi done (main stream)
    hipEvent_t ev_framed = nullptr;  // this pass's framing done (main stream)
    bool trace_blocks = false;
    // mapped pinned host records and job count, written by the Viterbi kernel
    // (system-scope stores); the host reads them only after `ev`, which the
    // main stream records after that kernel
    uint8_t *h_out = nullptr;
    int *h_n = nullptr;
    uint8_t *h_out_dev = nullptr;  // the same buffers as the device addresses them
    int *h_n_dev = nullptr;
    hipEvent_t ev = nullptr;
    bool pending = false;
  };
  static constexpr int NSLOT = 4;
  JobSlot slot[NSLOT];
  std::deque<int> pending_slots;
  int next_slot = 0, max_jobs_seen = 0;
  // device-error word (DevState::err): mapped pinned, set by a kernel that
  // gave up, checked by the host whenever a pass's slot completes
  int *h_err = nullptr, *h_err_dev = nullptr;
  // pinned staging for host->device counters and PCM (reused once its event completed)
  static constexpr int NPIN = 4;
  long long *pin_avail[NPIN] = {};
  hipEvent_t pin_ev[NPIN] = {};
  int next_pin = 0;
  int16_t *pin_pcm = nullptr;
  size_t pin_pcm_cap = 0;
  hipEvent_t pin_pcm_ev = nullptr;
  // device-pointer pushes: the caller's rows are copied straight into the PCM
  // ring on a high-priority side stream (the host waits for that copy only, so
  // it can run beside a coarse or demod launch); the copy first waits for the
  // demod launch that consumed the ring rows it overwrites: `consumed` holds
  // (least nsamp over the channels after a demod launch, event after it)
  hipStream_t st_in = nullptr;
  std::deque<std::pair<long long, hipEvent_t>> consumed;
  std::vector<hipEvent_t> ev_free;
  int vit_pending = -1;          // slot whose Viterbi launch is deferred
  hipEvent_t ev_in = nullptr;
  // gather job tables (aero_chan_feed, queued host messages; pinned ->
  // device, reused once their event completed), GJOB_MIN or C entries
  static constexpr int GJOB_MIN = 4096;
  GatherJob *pin_gjobs[NPIN] = {}, *d_gjobs[NPIN] = {};
  hipEvent_t gjob_ev[NPIN] = {};
  int next_gjob = 0;
  hipEvent_t ev_feed_done = nullptr;
  // queued host messages (single-channel pageable pushes, e.g. one ZeroMQ
  // message of one topic): copied into pinned staging when pushed, moved to
  // the PCM rings by one H2D copy and one gather launch when the group next
  // runs (hostq_flush) instead of a staged copy and a scatter launch each
  struct HqItem {
    int c;
    size_t off;
    long long n, start;
  };
  std::vector<HqItem> hq;
  // two pinned stagings, alternating at each flush (filling one never waits
  // for the copy out of the other); one device buffer (stream-ordered)
  int16_t *pin_hq[2] = {}, *d_hq = nullptr;
  size_t hq_cap = 0, hq_used = 0;
  int hq_buf = 0;
  hipEvent_t hq_ev[2] = {};  // after the last copy out of pin_hq[k]
  void *pin_stat = nullptr;  // aero_channel_stat staging
  std::map<std::string, TimingSlot> timing;
  std::vector<std::pair<std::string, std::pair<hipEvent_t, hipEvent_t>>> pending_ev;
  uint64_t processed = 0;
  // aero_stat counters: Viterbi jobs handed back, frames delivered to the
  // SU/ACARS host, SUs whose CRC checked
  std::atomic<uint64_t> st_jobs{0}, st_frames{0}, st_su_ok{0};
  int init_lo = 0;  // channels [init_lo, nch) await device state init
  std::vector<uint8_t> h_jobs_task, h_dbg_task;  // buffers owned by the running host task
};

// chmap kinds of burst-mode channels (burst_engine.hip): MODE_BURST + BurstKind
constexpr int MODE_BURST = 1 << 20;

struct aero_engine {
  int device = 0, flags = 0, max_channels = 0;
  // by gid: the fixed kinds (Mode), GID_C8400, then generic-rate MSK groups
  std::vector<std::unique_ptr<Group>> groups = std::vector<std::unique_ptr<Group>>(MODE_COUNT + 1);
  BurstGroup *burst[2] = {nullptr, nullptr};  // BURST_OQPSK, BURST_MSK
  std::vector<std::pair<int, int>> chmap;  // engine channel -> (gid or MODE_BURST + kind, local index)
  std::unique_ptr<HostPool> hpool;
  std::map<std::string, TimingSlot> timing;  // engine-level host sections
  uint64_t retired_jobs = 0, retired_frames = 0, retired_su_ok = 0;  // counters of released groups
};

namespace {

template <class T>
T *carve(char *&p, size_t count) {
  T *r = reinterpret_cast<T *>(p);
  size_t b = (count * sizeof(T) + 255) & ~size_t(255);
  p += b;
  return r;
}

size_t layout(DevState &S, DevTables &T, int mode, const ModeGeom &g, int C, int flags, char *base) {
  const bool msk = mode != MODE_OQPSK && mode != MODE_C8400;
  char *p = base;
  S.C = C;
  S.mode = mode;
  S.dcd_tick = (mode == MODE_OQPSK && (flags & AERO_F_DCD_TICK)) ? 1 : 0;
  S.g = g;
  S.ds = carve<double>(p, (size_t)DS_COUNT * C);
  S.is = carve<int>(p, (size_t)IS_COUNT * C);
  S.ls = carve<long long>(p, (size_t)LS_COUNT * C);
  S.fir = carve<double>(p, (size_t)2 * g.ntaps * C);
  S.agc = carve<double>(p, (size_t)g.agc_len * C);
  S.dsm = carve<double2>(p, msk ? (size_t)g.dsm_len * C : 1);
  S.d8 = carve<double>(p, msk ? (size_t)g.d8_len * C : 1);
  S.marg = carve<double>(p, (size_t)g.marg_len * C);
  S.dt = carve<double2>(p, (size_t)g.dt_len * C);
  // OQPSK: pm holds MSEcalc's (pm, ms) pairs, [C][ms_len] double2 (demod_oqpsk.hip); MSK: ms = msema
  S.pm = carve<double>(p, msk ? 1 : (size_t)2 * g.ms_len * C);
  S.ms = carve<double>(p, msk ? (size_t)g.ms_len * C : 1);
  S.pcm = carve<int16_t>(p, (size_t)PCM_CAP * C);
  S.pcm_cap = PCM_CAP;
  S.cring = carve<uint32_t>(p, (size_t)g.nfft * C);
  S.y = carve<double>(p, (size_t)(g.y_hi - g.y_lo + 1) * C);
  S.soft = carve<uint8_t>(p, (size_t)SOFT_RING * C);
  S.pt_cap = (flags & AERO_F_TRACE_PT) ? PT_CAP : 0;
  S.pt = carve<double2>(p, (size_t)S.pt_cap * C);
  S.hop_cap = HOP_CAP;
  S.hops = carve<double>(p, (size_t)HOP_CAP * 6 * C);
  S.hop_n = carve<int>(p, (size_t)C);
  S.block = carve<uint8_t>(p, (size_t)2 * g.block * C);
  S.overlap = carve<uint8_t>(p, (size_t)64 * C);
  S.dl2 = carve<uint8_t>(p, (size_t)g.dl2_len * C);
  S.jobs = carve<int>(p, (size_t)4 * C);
  S.njobs = carve<int>(p, 1);
  S.jobout = carve<uint8_t>(p, (size_t)JOB_OUT * C);
  S.blocks_dbg = carve<uint8_t>(p, (flags & AERO_F_TRACE_BLOCKS) ? (size_t)2500 * C : 1);
  const bool cch = mode == MODE_C8400;
  S.cin = carve<uint32_t>(p, cch ? (size_t)C_IN_RING * C : 1);
  S.cout = carve<double2>(p, cch ? (size_t)C_OUT_RING * C : 1);
  S.csig = carve<double2>(p, cch ? (size_t)C_FIR_SNZ * C : 1);
  S.crem = carve<double2>(p, cch ? (size_t)(C_FIR_N - C_FIR_SNZ) * C : 1);
  T.cker = carve<double2>(p, cch ? C_FIR_N : 1);
  T.tw4 = carve<double2>(p, cch ? C_FIR_N : 1);
  T.twi4 = carve<double2>(p, cch ? C_FIR_N : 1);
  T.cwin = carve<double>(p, cch ? NFFT : 1);
  T.cis = carve<double2>(p, WTSIZE);
  T.tw = carve<double2>(p, g.nfft);
  T.twi = carve<double2>(p, g.nfft);
  T.twg = carve<double2>(p, g.nfft);
  T.twgi = carve<double2>(p, g.nfft);
  T.scr = carve<uint8_t>(p, 5000);
  T.taps = carve<double>(p, MAX_TAPS);
  return (size_t)(p - base);
}

std::string tname(const Group *e, const char *name) { return e->tag + name; }

void ev_begin(Group *e, const char *name, hipEvent_t &a, hipEvent_t &b, hipStream_t st = nullptr) {
  if (!(e->flags & AERO_F_TIMING)) return;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a, st ? st : e->st);
  e->pending_ev.push_back({tname(e, name), {a, b}});
}
void ev_end(Group *e, hipEvent_t b, hipStream_t st = nullptr) {
  if (!(e->flags & AERO_F_TIMING)) return;
  hipEventRecord(b, st ? st : e->st);
}
void ev_collect(Group *e) {
  for (auto &pe : e->pending_ev) {
    float ms = 0;
    hipEventSynchronize(pe.second.second);
    hipEventElapsedTime(&ms, pe.second.first, pe.second.second);
    auto &slot = e->timing[pe.first];
    slot.ms += ms;
    slot.launches++;
    hipEventDestroy(pe.second.first);
    hipEventDestroy(pe.second.second);
  }
  e->pending_ev.clear();
}

// Per-channel scalar state as the demodulator ctor + setSettings leave it.
// OQPSK: decode/oqpskdemodulator.cpp:9-115, :136-254; MSK:
// decode/mskdemodulator.cpp:7-218 (both as Decoder applies them); AeroL ctor
// (decode/aerol.cpp:875-954).  Opened channels are initialised lazily, one
// strided copy per field for the whole pending range.
int init_scalars(Group *e, int lo, int hi) {
  const int C = e->C, k = hi - lo;
  std::vector<double> ds(DS_COUNT, 0.0);
  std::vector<int> is(IS_COUNT, 0);
  std::vector<long long> ls(LS_COUNT, 0);
  if (e->mode == MODE_OQPSK) {
    ds[DS_SO_FREQ] = 10500;
    ds[DS_SO_STEP] = (10500.0) * ((double)WTSIZE) / ((float)48000);
    ds[DS_MSE] = 100;
  } else if (e->mode == MODE_C8400) {
    // st_osc.SetFreq(fb = 8400, Fs) (oqpskdemodulator.cpp:225-227); the ctor's
    // mixer_fir_pre.SetFreq(freq_center = 8000, Fs) (:114), phase 0
    ds[DS_SO_FREQ] = 8400;
    ds[DS_SO_STEP] = (8400.0) * ((double)WTSIZE) / ((float)48000);
    ds[DS_MSE] = 100;
    ds[DS_FP_FREQ] = 8000;
    ds[DS_FP_STEP] = (8000.0) * ((double)WTSIZE) / ((float)48000);
  } else {
    // st_osc.SetFreq(fb / 2, Fs) (mskdemodulator.cpp:117); mse = 10.0 (:146);
    // DiffDecode::lastsoftstate = -1 (DSP.cpp:517-520)
    ds[DS_SO_FREQ] = 300;
    ds[DS_SO_STEP] = (300.0) * ((double)WTSIZE) / ((float)e->g.fs);
    ds[DS_MSE] = 10.0;
    ds[DS_DIFF_LAST] = -1;
  }
  is[IS_COUNTDOWN2] = 5;
  is[IS_COUNTDOWN] = 4;
  is[IS_EMPTYCD] = 1;
  is[IS_CNTR] = 1000000000;
  std::vector<double> vd(k);
  std::vector<int> vi(k);
  std::vector<long long> vl(k);
  for (int f = 0; f < DS_COUNT; f++) {
    std::fill(vd.begin(), vd.end(), ds[f]);
    HIPCHK(hipMemcpy(e->S.ds + (size_t)f * C + lo, vd.data(), 8 * (size_t)k, hipMemcpyHostToDevice));
  }
  for (int f = 0; f < IS_COUNT; f++) {
    std::fill(vi.begin(), vi.end(), is[f]);
    HIPCHK(hipMemcpy(e->S.is + (size_t)f * C + lo, vi.data(), 4 * (size_t)k, hipMemcpyHostToDevice));
  }
  for (int f = 0; f < LS_COUNT; f++) {
    std::fill(vl.begin(), vl.end(), ls[f]);
    HIPCHK(hipMemcpy(e->S.ls + (size_t)f * C + lo, vl.data(), 8 * (size_t)k, hipMemcpyHostToDevice));
  }
  return AERO_OK;
}

int flush_pending_init(Group *e) {
  const int lo = e->init_lo, hi = e->nch;
  if (lo >= hi) return AERO_OK;
  if (int rc = init_scalars(e, lo, hi)) return rc;
  e->init_lo = hi;
  return AERO_OK;
}

// A freed slot (free_slots) back to a new channel's state: every per-channel
// row zeroed, as the zeroed pool leaves a slot never used, then the scalar
// init.  The group is idle (its stream drained first).
int reset_slot(Group *e, int c) {
  const DevState &S = e->S;
  const ModeGeom &g = e->g;
  const size_t C = (size_t)e->C;
  const bool msk = e->mode != MODE_OQPSK;
  hipStream_t st = e->st;
  HIPCHK(hipStreamSynchronize(st));
  auto col = [&](void *base, size_t elem, size_t rows) {  // time-major [rows][C]: one element per row
    return hipMemset2DAsync((char *)base + elem * c, elem * C, 0, elem, rows, st);
  };
  auto row = [&](void *base, size_t bytes) {  // channel-major [C][len]
    return hipMemsetAsync((char *)base + bytes * c, 0, bytes, st);
  };
  HIPCHK(col(S.fir, 8, (size_t)2 * g.ntaps));
  HIPCHK(col(S.agc, 8, (size_t)g.agc_len));
  if (msk) {
    HIPCHK(col(S.dsm, 16, (size_t)g.dsm_len));
    HIPCHK(col(S.d8, 8, (size_t)g.d8_len));
    HIPCHK(row(S.ms, (size_t)8 * g.ms_len));
  } else {
    HIPCHK(row(S.pm, (size_t)16 * g.ms_len));
  }
  HIPCHK(col(S.pcm, 2, (size_t)PCM_CAP));
  HIPCHK(row(S.marg, (size_t)8 * g.marg_len));
  HIPCHK(row(S.dt, (size_t)16 * g.dt_len));
  HIPCHK(row(S.cring, (size_t)4 * g.nfft));
  HIPCHK(row(S.y, (size_t)8 * (g.y_hi - g.y_lo + 1)));
  HIPCHK(row(S.soft, (size_t)SOFT_RING));
  if (S.pt_cap) HIPCHK(row(S.pt, (size_t)16 * S.pt_cap));
  HIPCHK(row(S.hops, (size_t)8 * 6 * HOP_CAP));
  HIPCHK(row(S.hop_n, 4));
  HIPCHK(row(S.block, (size_t)2 * g.block));
  HIPCHK(row(S.overlap, 64));
  HIPCHK(row(S.dl2, (size_t)g.dl2_len));
  if (e->flags & AERO_F_TRACE_BLOCKS) HIPCHK(row(S.blocks_dbg, 2500));
  if (e->mode == MODE_C8400) {  // JFastFir's state: no outputs yet, no remainder
    HIPCHK(row(S.csig, (size_t)16 * C_FIR_SNZ));
    HIPCHK(row(S.crem, (size_t)16 * (C_FIR_N - C_FIR_SNZ)));
  }
  HIPCHK(hipStreamSynchronize(st));
  return init_scalars(e, c, c + 1);
}

// CRC-16 of one SU (AeroLcrc16::calcusingbytes, decode/aerol.h:332-367) and the
// all-zero special case (decode/aerol.cpp:1531-1543)
bool su_crc_ok(const uint8_t *su) {
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
  return calc == rec;
}

// Host SU/ACARS work for one completed job slot, on the worker pool
// (asynchronous; host_wait() joins it).  Slots are handled in launch order,
// and the pool finishes one slot's work before it starts the next, so a
// channel's frames keep their order.
int process_slot(Group *e, int si) {
  auto &sl = e->slot[si];
  const int C = e->C, nch = e->nch;
  const int njobs = *sl.h_n;
  // the slot's event follows this pass's demod: a hand-off that gave up in
  // it (or earlier) is visible now; the outputs of such a run are garbage
  if (*(volatile int *)e->h_err) return AERO_E_DEVICE;
  e->max_jobs_seen = std::max(e->max_jobs_seen, njobs);
  HOST_TIMER(e, "host_frames");
  e->hpool->wait();  // previous slot's frames first (per-channel order)
  const size_t JO = (size_t)e->job_out;
  e->h_jobs_task.resize((size_t)std::max(njobs, 1) * JO);
  if (njobs > 0) memcpy(e->h_jobs_task.data(), sl.h_out, (size_t)njobs * JO);
  sl.pending = false;
  const bool blocks = (e->flags & AERO_F_TRACE_BLOCKS) != 0 && e->mode != MODE_C8400;
  if (blocks) {
    // traces run synchronously (run_group waited for this slot): blocks_dbg is this pass's
    e->h_dbg_task.resize((size_t)2500 * C);
    if (!e->trace_some) {
      HIPCHK(hipMemcpy(e->h_dbg_task.data(), e->S.blocks_dbg, e->h_dbg_task.size(), hipMemcpyDeviceToHost));
    } else {
      for (int c : e->trace_list)
        HIPCHK(hipMemcpy(e->h_dbg_task.data() + (size_t)c * 2500, e->S.blocks_dbg + (size_t)c * 2500, 2500,
                         hipMemcpyDeviceToHost));
    }
  }
  if (njobs <= 0) return AERO_OK;
  e->st_jobs += (uint64_t)njobs;
  const bool msk = e->mode != MODE_OQPSK && e->mode != MODE_C8400;
  const bool cch = e->mode == MODE_C8400;
  // channels partitioned over workers (c % T): a channel's frames stay in
  // queue order and no two workers share state
  auto work = [e, njobs, nch, blocks, msk, cch, JO](int t, int T) {
    const uint8_t *jobs = e->h_jobs_task.data();
    uint64_t frames = 0, su_ok = 0;  // this worker's counts, added once (no shared atomics per job)
    for (int j = 0; j < njobs; j++) {
      const uint8_t *o = jobs + (size_t)j * JO;
      int meta[4];
      memcpy(meta, o + (cch ? 336 : 312), 16);
      const int c = meta[3] & 0x3FFFFFFF;
      const int reset = (meta[3] >> 30) & 1;
      if (c < 0 || c >= nch || c % T != t) continue;
      if (cch) {
        // AeroL::DecodeC's frame end (decode/aerol.cpp:2284-2405): per SU the DCD
        // countdown (+2 / -5) and datacd; Call_progress_Signal for a CRC-valid
        // Call_progress SU (0x30), whose AES tags the frame's Voicesignal
        const uint32_t mask = (uint32_t)meta[1];
        uint32_t aes = 0;
        for (int k = 0; k < 3; k++) {
          const bool ok = (mask >> k) & 1;
          int &cd = e->c_cd[c];
          if (ok) {
            if (cd < 12) cd += 2;
          } else {
            if (cd > 0) cd -= 5;
          }
          if (!e->c_dcd[c] && cd > 2) {
            e->c_dcd[c] = 1;
            e->c_edges[c]++;
          }
          const uint8_t *su = o + 12 * k;
          if (ok && su[0] == 0x30) {
            e->cunit_hold[c].insert(e->cunit_hold[c].end(), su, su + 12);
            aes = ((uint32_t)su[1] << 16) | ((uint32_t)su[2] << 8) | su[3];
          }
        }
        auto &v = e->voice_hold[c];
        v.insert(v.end(), (const uint8_t *)&aes, (const uint8_t *)&aes + 4);
        v.insert(v.end(), o + 36, o + 336);
        frames++;
        su_ok += (uint64_t)__builtin_popcount(mask);
        if ((e->flags & AERO_F_TRACE_FRAMES) && e->traced(c)) {
          uint8_t rec[320] = {0};
          memcpy(rec, o, 36);
          const uint32_t L = 36, M = mask;
          memcpy(rec + 312, &L, 4);
          memcpy(rec + 316, &M, 4);
          e->frame_hold[c].insert(e->frame_hold[c].end(), rec, rec + 320);
        }
        continue;
      }
      if (blocks && e->traced(c)) {
        const uint8_t *d = e->h_dbg_task.data() + (size_t)c * 2500;
        int nb;
        memcpy(&nb, d, 4);
        uint32_t L = (uint32_t)nb;
        auto &h = e->blk_hold[c];
        h.insert(h.end(), (uint8_t *)&L, (uint8_t *)&L + 4);
        h.insert(h.end(), d + 4, d + 4 + nb);
      }
      if (reset) e->host[c]->isu_reset();
      int flen = -1;
      uint32_t mask = (uint32_t)meta[1];
      const uint8_t *info = o;
      if (msk) {
        // 600/1200: a frame's infofield is the bytes of its blocks since the
        // last cntr == 0 (aerol.cpp:1247-1250, 1509-1520); SUs checked when done
        auto &inf = e->infofield[c];
        if (meta[0] & (1 << 9)) inf.clear();
        inf.insert(inf.end(), o, o + (meta[0] & 0xFF));
        if (meta[0] & (1 << 8)) {
          flen = (int)std::min<size_t>(inf.size(), 312);
          mask = 0;
          for (int k = 0; k < flen / 12; k++)
            if (su_crc_ok(inf.data() + 12 * k)) mask |= 1u << k;
          info = inf.data();
        }
      } else {
        flen = meta[0];
      }
      if (flen >= 0) {
        frames++;
        su_ok += (uint64_t)__builtin_popcount(mask);
        e->host[c]->frame(info, flen, mask, meta[2]);
        if ((e->flags & AERO_F_TRACE_FRAMES) && e->traced(c)) {
          uint8_t rec[320] = {0};
          memcpy(rec, info, flen);
          const uint32_t L = (uint32_t)flen, M = mask;
          memcpy(rec + 312, &L, 4);
          memcpy(rec + 316, &M, 4);
          e->frame_hold[c].insert(e->frame_hold[c].end(), rec, rec + 320);
        }
      }
    }
    e->st_frames += frames;
    e->st_su_ok += su_ok;
  };
  e->hpool->submit(work, std::max(1, std::min(njobs / 64, nch)));
  return AERO_OK;
}

// hands completed slots (all of them when `wait`) to the host workers, in order
int poll_slots(Group *e, bool wait) {
  while (!e->pending_slots.empty()) {
    const int si = e->pending_slots.front();
    if (wait) {
      HOST_TIMER(e, "host_wait_jobs");
      HIPCHK(hipEventSynchronize(e->slot[si].ev));
    } else if (hipEventQuery(e->slot[si].ev) != hipSuccess) {
      break;
    }
    e->pending_slots.pop_front();
    if (int rc = process_slot(e, si)) return rc;
  }
  return AERO_OK;
}

// joins the asynchronous host frame work (before any host-side output is read)
void host_wait(aero_engine *e) {
  if (e->hpool) e->hpool->wait();
}

int collect_traces(Group *e) {
  const int C = e->C, nch = e->nch;
  // the channels whose traces are kept (aero_trace_select), and whether
  // their rows are copied one by one (a few channels of a large group)
  std::vector<int> sel;
  if (!e->trace_some) {
    sel.resize(nch);
    for (int c = 0; c < nch; c++) sel[c] = c;
  } else {
    sel = e->trace_list;
  }
  const bool rows = e->trace_some;
  std::vector<int> hn(nch);
  if (e->flags & AERO_F_TRACE_HOPS) HIPCHK(hipMemcpy(hn.data(), e->S.hop_n, sizeof(int) * nch, hipMemcpyDeviceToHost));
  bool anyhop = false;
  for (int c = 0; c < nch; c++) anyhop |= hn[c] > 0;
  if (anyhop) {
    const size_t rec = (size_t)HOP_CAP * 6;
    std::vector<double> h(rec * (rows ? 1 : nch));
    if (!rows) HIPCHK(hipMemcpy(h.data(), e->S.hops, h.size() * 8, hipMemcpyDeviceToHost));
    for (int c : sel) {
      const int n = std::min(hn[c], HOP_CAP);
      if (n <= 0) continue;
      const double *src = h.data() + (rows ? 0 : (size_t)c * rec);
      if (rows) HIPCHK(hipMemcpy(h.data(), e->S.hops + (size_t)c * rec, (size_t)n * 6 * 8, hipMemcpyDeviceToHost));
      auto &hh = e->hop_hold[c];
      const size_t at = hh.size();
      hh.insert(hh.end(), src, src + (size_t)n * 6);
      if (e->hop_base[c])
        for (size_t r = at; r < hh.size(); r += 6) hh[r] += (double)e->hop_base[c];
    }
    HIPCHK(hipMemset(e->S.hop_n, 0, sizeof(int) * nch));
  }
  if (e->flags & AERO_F_TRACE_PT) {
    std::vector<long long> pn(nch);
    HIPCHK(hipMemcpy(pn.data(), e->S.ls + (size_t)LS_PT_N * C, 8 * nch, hipMemcpyDeviceToHost));
    std::vector<double2> pts((size_t)PT_CAP * (rows ? 1 : nch));
    if (!rows) HIPCHK(hipMemcpy(pts.data(), e->S.pt, pts.size() * sizeof(double2), hipMemcpyDeviceToHost));
    for (int c : sel) {
      if (pn[c] > PT_CAP) return AERO_E_FULL;
      if (pn[c] <= 0) continue;
      const double2 *src = pts.data() + (rows ? 0 : (size_t)c * PT_CAP);
      if (rows)
        HIPCHK(hipMemcpy(pts.data(), e->S.pt + (size_t)c * PT_CAP, (size_t)pn[c] * sizeof(double2),
                         hipMemcpyDeviceToHost));
      for (long long k = 0; k < pn[c]; k++) {
        e->pt_hold[c].push_back(src[k].x);
        e->pt_hold[c].push_back(src[k].y);
      }
    }
    HIPCHK(hipMemset(e->S.ls + (size_t)LS_PT_N * C, 0, 8 * nch));
  }
  // soft bits delivered to AeroL (groups of 32 / 12)
  if (!(e->flags & AERO_F_TRACE_SOFT)) return AERO_OK;
  std::vector<long long> sp(nch);
  HIPCHK(hipMemcpy(sp.data(), e->S.ls + (size_t)LS_SOFT_P * C, 8 * nch, hipMemcpyDeviceToHost));
  std::vector<uint8_t> ring;
  for (int c : sel) {
    const long long emitted = sp[c] - sp[c] % e->g.soft_group;
    if (emitted > e->soft_seen[c]) {
      const uint8_t *r;
      if (rows) {
        ring.resize(SOFT_RING);
        HIPCHK(hipMemcpy(ring.data(), e->S.soft + (size_t)c * SOFT_RING, SOFT_RING, hipMemcpyDeviceToHost));
        r = ring.data();
      } else {
        if (ring.empty()) {
          ring.resize((size_t)SOFT_RING * nch);
          HIPCHK(hipMemcpy(ring.data(), e->S.soft, ring.size(), hipMemcpyDeviceToHost));
        }
        r = ring.data() + (size_t)c * SOFT_RING;
      }
      for (long long k = e->soft_seen[c]; k < emitted; k++) e->soft_hold[c].push_back(r[k & (SOFT_RING - 1)]);
      e->soft_seen[c] = emitted;
    }
  }
  return AERO_OK;
}

// The Viterbi of a pass runs on the main stream, between the next pass's
// coarse hop and demod launch, with the whole GPU to itself.  (Measured, see
// beside the demod its waves take issue and LDS cycles from the
// latency-bound demod waves, which then lose as much time as the Viterbi
// takes; beside the coarse FFT there is no room.)  Its job records go to the
// host through mapped pinned memory the kernel writes itself.
int issue_viterbi(Group *e) {
  const int si = e->vit_pending;
  if (si < 0) return AERO_OK;
  e->vit_pending = -1;
  auto &sl = e->slot[si];
  DevState S2 = e->S;
  S2.njobs = sl.d_n;
  S2.jobs = sl.d_jobs;
  // The kernel writes the job records and their count straight into the
  // slot's pinned host buffers (3.6 MB per pass at the bench config, over
  // PCIe while it decodes): no device-to-host copy is queued.  A queued copy
  // waiting for this kernel held back the next push's host-to-device DMA
  // until the whole pass had finished (copies of the process run in order),
  // which serialised a host-pushed stream with the GPU work.
  S2.jobout = sl.h_out_dev;
  S2.njobs_host = sl.h_n_dev;
  hipEvent_t a, b;
  ev_begin(e, "viterbi", a, b);
  launch_viterbi(e->st, e->mode, S2, e->T, e->nch, sl.trace_blocks ? 1 : 0);
  ev_end(e, b);
  HIPCHK(hipEventRecord(sl.ev_vit, e->st));
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(sl.ev, e->st));
  sl.pending = true;
  e->pending_slots.push_back(si);
  return AERO_OK;
}

// after a demod launch: the ring rows of samples below every channel's new
// nsamp are free once the main stream has passed this point
int note_consumed(Group *e) {
  // a caught-up channel (nsamp == avail: an idle or never-pushed one) holds
  // no unconsumed rows, so only channels with samples still queued bound it
  long long mn = LLONG_MAX;
  for (int c = 0; c < e->nch; c++)
    if (e->avail[c] > e->nsamp[c]) mn = std::min(mn, e->nsamp[c]);
  hipEvent_t ev;
  if (e->ev_free.empty()) {
    HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  } else {
    ev = e->ev_free.back();
    e->ev_free.pop_back();
  }
  HIPCHK(hipEventRecord(ev, e->st));
  e->consumed.push_back({mn, ev});
  while (e->consumed.size() > 32) {  // older ones: a push that needs them waits for the stream instead
    e->ev_free.push_back(e->consumed.front().second);
    e->consumed.pop_front();
  }
  return AERO_OK;
}

size_t gjob_cap(const Group *e) { return (size_t)std::max(e->C, Group::GJOB_MIN); }

// a free gather-job table (pinned + device, gjob_cap entries)
int gather_table(Group *e, int &k) {
  k = e->next_gjob;
  e->next_gjob = (k + 1) % Group::NPIN;
  if (!e->pin_gjobs[k]) {
    if (hipHostMalloc(&e->pin_gjobs[k], sizeof(GatherJob) * gjob_cap(e)) != hipSuccess) return AERO_E_NOMEM;
    if (hipMalloc(&e->d_gjobs[k], sizeof(GatherJob) * gjob_cap(e)) != hipSuccess) return AERO_E_NOMEM;
    HIPCHK(hipEventCreateWithFlags(&e->gjob_ev[k], hipEventDisableTiming));
  }
  HIPCHK(hipEventSynchronize(e->gjob_ev[k]));  // the table NPIN launches ago has been read
  return AERO_OK;
}

// only a channel's last job of a launch writes its counter
void mark_last_jobs(GatherJob *jobs, size_t nj, int C) {
  std::vector<uint8_t> seen(C, 0);
  for (size_t i = nj; i-- > 0;) {
    jobs[i].later = seen[jobs[i].c];
    seen[jobs[i].c] = 1;
  }
}

// the queued host messages into the PCM rings: one H2D copy of the staging,
// one gather launch (stream-ordered before the group's next kernels)
int hostq_flush(Group *e) {
  if (e->hq.empty()) return AERO_OK;
  int k;
  if (int rc = gather_table(e, k)) return rc;
  const int b = e->hq_buf;
  HIPCHK(hipMemcpyAsync(e->d_hq, e->pin_hq[b], sizeof(int16_t) * e->hq_used, hipMemcpyHostToDevice, e->st));
  HIPCHK(hipEventRecord(e->hq_ev[b], e->st));
  long long mx = 0;
  const size_t nj = e->hq.size();
  for (size_t i = 0; i < nj; i++) {
    const Group::HqItem &it = e->hq[i];
    GatherJob &j = e->pin_gjobs[k][i];
    j.src = e->d_hq + it.off;
    j.n = it.n;
    j.start = it.start;
    j.avail_after = it.start + it.n;
    j.c = it.c;
    j.later = 0;
    mx = std::max(mx, it.n);
  }
  mark_last_jobs(e->pin_gjobs[k], nj, e->C);
  HIPCHK(hipMemcpyAsync(e->d_gjobs[k], e->pin_gjobs[k], sizeof(GatherJob) * nj, hipMemcpyHostToDevice, e->st));
  HIPCHK(hipEventRecord(e->gjob_ev[k], e->st));
  const unsigned gx = (unsigned)std::max<long long>(1, std::min<long long>((mx + 255) / 256, 64));
  hipLaunchKernelGGL(pcm_gather_kernel, dim3(gx, (unsigned)nj), dim3(256), 0, e->st, e->S.pcm, e->C,
                     (long long)PCM_CAP - 1, e->S.ls + (size_t)LS_AVAIL * e->C, (const GatherJob *)e->d_gjobs[k]);
  HIPCHK(hipGetLastError());
  e->hq.clear();
  e->hq_used = 0;
  e->hq_buf = b ^ 1;
  return AERO_OK;
}

// A run of a group is run_begin, passes until a pass has nothing to do,
// run_end.  run_group runs one group; run_impl interleaves the groups' passes
// so that each group's launches queue on its stream while the host waits for
// another group's old job slot (the kinds of a mixed engine, e.g. the C5
// receiver's OQPSK, MSK 600 and MSK 1200 groups, then run side by side).
int run_begin(Group *e) {
  HIPCHK(hipSetDevice(e->device));
  if (int rc = flush_pending_init(e)) return rc;
  if (int rc = hostq_flush(e)) return rc;
  return poll_slots(e, false);
}

int frame_round(Group *e, int flush, bool trace);

// one pass (coarse, the previous pass's Viterbi, demod, framing); *more is
// false when the group had nothing left to do
int run_pass(Group *e, int flush, bool *more) {
  HOST_TIMER(e, "host_run");
  *more = true;
  const int tflags = AERO_F_TRACE_PT | AERO_F_TRACE_BLOCKS | AERO_F_TRACE_SOFT | AERO_F_TRACE_HOPS;
  const bool trace = (e->flags & tflags) != 0;
  const long long HOPN = e->g.hop;
  const bool cch = e->mode == MODE_C8400;
  {
    // host mirror of the hop and segment rules of coarse.hip / demod_*.hip
    bool any_hop = false, progress = false;
    // the C channel: the next message of every channel whose demod has
    // reached the end of the prefiltered one (cchan.hip prefilter_dn_kernel, prefilter_blk_kernel)
    int ncj = 0, kcj = 0;
    if (cch) {
      kcj = e->next_cjob;
      struct HostCPreJob {
        int c, pad;
        long long s, e;
      };
      static_assert(sizeof(HostCPreJob) == 24, "CPreJob layout");
      HostCPreJob *jt = reinterpret_cast<HostCPreJob *>(e->pin_cjobs[kcj]);
      bool waited = false;
      for (int c = 0; c < e->nch; c++) {
        if (e->nsamp[c] != e->pre_end[c] || e->msg_end[c].empty()) continue;
        if (!waited) {  // the table of NPIN passes ago has been read
          HIPCHK(hipEventSynchronize(e->cjob_ev[kcj]));
          waited = true;
        }
        jt[ncj++] = {c, 0, e->pre_end[c], e->msg_end[c].front()};
        e->pre_end[c] = e->msg_end[c].front();
        e->msg_end[c].pop_front();
      }
      if (ncj) e->next_cjob = (kcj + 1) % Group::NPIN;
    }
    for (int c = 0; c < e->nch; c++) {
      const long long boundary = HOPN * (e->hops[c] + 1) - 1;
      if (e->nsamp[c] == boundary && e->avail[c] > boundary) {
        e->hops[c]++;
        any_hop = true;
      }
    }
    for (int c = 0; c < e->nch; c++) {
      const long long boundary = HOPN * (e->hops[c] + 1) - 1;
      long long end = std::min(e->avail[c], boundary);
      if (!flush && e->avail[c] <= boundary) end = e->nsamp[c];
      if (cch) end = std::min(e->pre_end[c], boundary);  // whole messages, prefiltered
      if (end > e->nsamp[c]) {
        e->processed += (uint64_t)(end - e->nsamp[c]);
        e->nsamp[c] = end;
        progress = true;
      }
    }
    if (!any_hop && !progress && !ncj) {
      *more = false;
      return AERO_OK;
    }
    hipEvent_t a, b;
    if (any_hop) {
      ev_begin(e, "coarse", a, b);
      launch_coarse(e->st, e->mode, e->S, e->T, e->nch);
      ev_end(e, b);
    }
    if (int rc = issue_viterbi(e)) return rc;  // the previous pass's decode, before this demod
    if (ncj) {
      HIPCHK(hipMemcpyAsync(e->d_cjobs[kcj], e->pin_cjobs[kcj], (size_t)c_prejob_bytes() * ncj,
                            hipMemcpyHostToDevice, e->st));
      HIPCHK(hipEventRecord(e->cjob_ev[kcj], e->st));
      ev_begin(e, "prefilter", a, b);
      launch_prefilter_c(e->st, e->S, e->T, e->d_cjobs[kcj], ncj);
      ev_end(e, b);
      HIPCHK(hipGetLastError());
    }
    if (!progress) return AERO_OK;  // no new soft bits: framing has nothing to do
    ev_begin(e, "demod", a, b);
    if (cch)
      launch_demod_c(e->st, e->S, e->T, e->nch, (e->flags & AERO_F_TRACE_PT) != 0);
    else if (e->mode == MODE_OQPSK)
      launch_demod(e->st, e->S, e->T, e->nch, flush, (e->flags & AERO_F_TRACE_PT) != 0, e->nch <= e->wide_max);
    else
      launch_demod_msk(e->st, e->mode, e->S, e->T, e->nch, flush, e->nch <= e->wide_max);
    ev_end(e, b);
    if (int rc = note_consumed(e)) return rc;
    if (int rc = frame_round(e, flush, trace)) return rc;
    // with the DCD timer a channel's framing may stop at a tick that needs the
    // CRCs of the frame this round completed (aerol.hip frame_kernel); a flush
    // has no next pass to resume it, so it frames once more after that Viterbi
    if (flush && e->S.dcd_tick)
      if (int rc = frame_round(e, flush, trace)) return rc;
  }
  return AERO_OK;
}

// framing + Viterbi into the next job slot (at most one job per channel per pass)
int frame_round(Group *e, int flush, bool trace) {
  hipEvent_t a, b;
  {
    const int si = e->next_slot;
    e->next_slot = (si + 1) % Group::NSLOT;
    auto &sl = e->slot[si];
    if (sl.pending) {  // four passes old: long done, hand it over first
      if (int rc = poll_slots(e, true)) return rc;
    }
    DevState S2 = e->S;
    S2.njobs = sl.d_n;
    S2.jobout = nullptr;  // framing lists jobs only; the Viterbi writes the records
    S2.jobs = sl.d_jobs;
    HIPCHK(hipMemsetAsync(sl.d_n, 0, sizeof(int), e->st));
    {
      // a channel refills its other interleaver buffer >= 5 passes after a
      // job took one; the Viterbi of two passes ago has read its buffer
      const auto &old = e->slot[(si + Group::NSLOT - 2) % Group::NSLOT];
      if (old.ev_vit) HIPCHK(hipStreamWaitEvent(e->st, old.ev_vit, 0));
    }
    ev_begin(e, "frame", a, b);
    launch_frame(e->st, e->mode, S2, e->nch);
    ev_end(e, b);
    HIPCHK(hipEventRecord(sl.ev_framed, e->st));
    sl.trace_blocks = (e->flags & AERO_F_TRACE_BLOCKS) != 0;
    e->vit_pending = si;
    if (trace || flush)  // parity traces run pass by pass; a flush has no next pass
      if (int rc = issue_viterbi(e)) return rc;
    if (trace) {  // parity traces: synchronous, pass by pass
      if (int rc = poll_slots(e, true)) return rc;
      if (int rc = collect_traces(e)) return rc;
    }
  }
  return AERO_OK;
}

// the deferral only reorders passes inside one run: the last pass's decode
// is launched before the run returns, so its items never wait for more audio
// (the reference emits them as soon as they are decoded)
int run_end(Group *e) { return issue_viterbi(e); }

int run_group(Group *e, int flush) {
  if (e->nch == 0) return AERO_OK;
  if (int rc = run_begin(e)) return rc;
  for (int guard = 0; guard < 1000000; guard++) {
    bool more;
    if (int rc = run_pass(e, flush, &more)) return rc;
    if (!more) break;
  }
  return run_end(e);
}

// waits for the group's GPU work and hands every completed slot over
int drain_group(Group *e) {
  HIPCHK(hipSetDevice(e->device));
  if (int rc = issue_viterbi(e)) return rc;
  // slot by slot as their records come back: the host work of each overlaps
  // the GPU's remaining passes
  if (int rc = poll_slots(e, true)) return rc;
  HIPCHK(hipStreamSynchronize(e->st));
  if (int rc = poll_slots(e, true)) return rc;
  if (e->flags & (AERO_F_TRACE_PT | AERO_F_TRACE_SOFT | AERO_F_TRACE_HOPS))
    if (int rc = collect_traces(e)) return rc;
  return AERO_OK;
}

// engine channel -> burst-group index (its group in *bg), or -1
int route_burst(aero_engine *e, int ch, BurstGroup **bg = nullptr) {
  if (!e || ch < 0 || ch >= (int)e->chmap.size()) return -1;
  const int k = e->chmap[ch].first - MODE_BURST;
  if (k < 0 || k > 1) return -1;
  if (bg) *bg = e->burst[k];
  return e->chmap[ch].second;
}

int run_impl(aero_engine *e, int flush) {
  for (BurstGroup *b : e->burst)
    if (b)
      if (int rc = burst_run(b, flush)) return rc;
  std::vector<Group *> act(e->groups.size());
  int na = 0;
  // a group whose channels have all moved to another rate's group (every
  // slot free, each drained when its channel left) is not launched
  for (auto &g : e->groups)
    if (g && g->nch && (int)g->free_slots.size() < g->nch) {
      if (int rc = run_begin(g.get())) return rc;
      act[na++] = g.get();
    }
  for (int guard = 0; na > 0 && guard < 1000000; guard++)
    for (int i = 0; i < na;) {
      bool more;
      if (int rc = run_pass(act[i], flush, &more)) return rc;
      if (more) {
        i++;
        continue;
      }
      if (int rc = run_end(act[i])) return rc;
      act[i] = act[--na];
    }
  if (flush)  // aero_flush returns with every output of the pushed samples available
    for (auto &g : e->groups)
      if (g) {
        int rc = drain_group(g.get());
        if (rc) return rc;
      }
  return AERO_OK;
}

// non-blocking: completed slots go to the host workers
void poll_all(aero_engine *e) {
  for (auto &g : e->groups)
    if (g) (void)poll_slots(g.get(), false);
}

template <class T>
int pop_vec(std::vector<T> &v, T *dst, size_t cap, size_t *n) {
  const size_t k = std::min(cap, v.size());
  if (dst && k) memcpy(dst, v.data(), k * sizeof(T));
  if (n) *n = k;
  v.erase(v.begin(), v.begin() + k);
  return AERO_OK;
}

// group tables and kernel constants (host glibc, g++-compiled: tables_host.cpp)
// the rate-dependent constants of a generic-rate MSK group at sample rate fs
// (MskDemodulator::setSettings with fb 600, decode/mskdemodulator.cpp:94-218;
// CoarseFreqEstimate::setSettings(13, 900, 600, Fs), coarsefreqestimate.cpp:39-76,
// and the fold search bounds of :166-185), or false when the kernels'
// assumptions do not hold at that rate
bool msk_gen_consts(int fs, MskGen &m) {
  if (fs < MSK_FS_MIN || fs > MSK_FS_MAX) return false;
  m = MskGen{};
  m.fs = fs;
  m.sps = fs / 600;
  // fb < 1200: the "300hz / 4hz / 48000" design at Fs 48000, else the
  // "300hz / 4hz / 12000" one (mskdemodulator.cpp:177-203)
  const bool f48 = fs == 48000;
  m.sr_b0 = f48 ? 1.308825621597620e-04 : 5.233248111921052e-04;
  m.sr_b2 = -m.sr_b0;
  m.sr_a1 = f48 ? -1.998196509168551 : -1.974342917561558;
  m.sr_a2 = f48 ? 0.999738234875681 : 0.998953350377616;
  m.ee = f48 ? 0.025 : 0.0125;
  int size;
  if (!host_delay_uniform(m.sps / 2.0, size, m.d8_old, m.d8_new, m.d8w, m.d8omw)) return false;
  // (ages >= 2: the few-channel kernel loads a sample's slots one sample ahead)
  if (size != msk_geom(600, fs).d8_len || m.d8_new < 2 || m.d8_old >= size) return false;
  const double nfft = MSK_NFFT, hzperbin = (double)fs / nfft, lockingbw = 900.0, fb = 600.0;
  const double startbin = std::max(std::round(lockingbw / hzperbin), 1.0);
  m.start = (int)startbin;
  m.stop = (int)(nfft - startbin);
  m.epb = (int)std::round(fb / (2.0 * hzperbin));
  m.ilo = (int)std::round((-lockingbw / hzperbin) + ((double)(MSK_NFFT / 2)));
  m.ihi = (int)std::round((lockingbw / hzperbin) + ((double)(MSK_NFFT / 2)));
  // every fold term inside the y bins an MSK group keeps (no "jic" skips)
  return m.ilo - m.epb - 1 >= MSK_YLO && m.ihi - 1 + m.epb + 1 <= MSK_YHI && m.ilo < m.ihi;
}

// the few-channel demod kernels' default limit: up to 4096 channels (1024
// waves of 16-lane groups) the chip has lanes to spare, and a channel's
// per-sample latency, not lane count, sets the time; above it the one-lane
// kernels' throughput wins (C2 / C3 at 65536 channels)
constexpr int WIDE_MAX_DEFAULT = 4096;

// gid: the group's engine id; fs: the sample rate of a generic-rate group
// (mode MODE_MSKG600 / MODE_MSKG1200), 0 for a fixed kind
int group_create(aero_engine *E, int mode, int gid, int fs, std::unique_ptr<Group> &out) {
  std::unique_ptr<Group> e(new Group());  // ~Group releases what an early return leaves allocated
  e->mode = mode;
  e->gid = gid;
  e->device = E->device;
  e->flags = E->flags;
  e->hpool = E->hpool.get();
  MskGen mg{};
  if (mode != MODE_OQPSK && mode != MODE_C8400) {
    // every MSK group carries its rate's constants (the generic-rate and the
    // few-channel kernels read them)
    if (!msk_gen_consts(msk_generic(mode) ? fs : msk_fs(mode), mg)) return AERO_E_RATE;
  }
  {
    const char *w = getenv(mode == MODE_OQPSK ? "AERO_OQPSK_WIDE" : "AERO_MSK_WIDE");
    e->wide_max = w ? atoi(w) : WIDE_MAX_DEFAULT;
  }
  if (msk_generic(mode)) {
    e->g = msk_geom(msk_bitrate(mode), fs);
    e->tag = "msk" + std::to_string(msk_bitrate(mode)) + "_" + std::to_string(fs) + "_";
  } else if (mode == MODE_C8400) {
    e->g = mode_geom(mode);
    e->tag = "c8400_";
    e->job_out = JOB_OUT_C;
  } else {
    static const char *const tags[MODE_COUNT] = {"", "msk600_", "msk1200_", "msk600_24k_", "msk600_48k_",
                                                  "msk1200_12k_", "msk1200_48k_"};
    e->g = mode_geom(mode);
    e->tag = tags[mode];
  }
  // a generic-rate MSK group serves the channels that happen to arrive at
  // its rate: a small pool (another group of the rate opens when it is
  // full), not max_channels (one 96 kHz channel of a 65536-channel engine
  // would otherwise ask for ~50 GB of AGC ring)
  e->C = (E->max_channels + 63) & ~63;
  if (msk_generic(mode)) e->C = std::min(e->C, GENERIC_GROUP_CAP);
  DevState S{};
  DevTables T{};
  const size_t bytes = layout(S, T, mode, e->g, e->C, e->flags, nullptr) + 4096;
  if (hipMalloc(&e->pool, bytes) != hipSuccess) return AERO_E_NOMEM;
  e->pool_bytes = bytes;
  HIPCHK(hipMemset(e->pool, 0, bytes));
  layout(e->S, e->T, mode, e->g, e->C, e->flags, reinterpret_cast<char *>(e->pool));
  e->S.mg = mg;
  HIPCHK(hipStreamCreateWithFlags(&e->st, hipStreamNonBlocking));
  if (hipHostMalloc(&e->h_err, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return AERO_E_NOMEM;
  *e->h_err = 0;
  HIPCHK(hipHostGetDevicePointer((void **)&e->h_err_dev, e->h_err, 0));
  e->S.err = e->h_err_dev;
  for (auto &sl : e->slot) {
    if (hipMalloc(&sl.d_n, 64) != hipSuccess) return AERO_E_NOMEM;
    // kernel-written zero-copy buffers: mapped (a device address for the
    // Viterbi kernel) and coherent (its system-scope stores reach host memory
    // without a cache flush); read by the host after the slot's event
    if (hipHostMalloc(&sl.h_out, (size_t)e->job_out * e->C, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
      return AERO_E_NOMEM;
    if (hipHostMalloc(&sl.h_n, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return AERO_E_NOMEM;
    HIPCHK(hipHostGetDevicePointer((void **)&sl.h_out_dev, sl.h_out, 0));
    HIPCHK(hipHostGetDevicePointer((void **)&sl.h_n_dev, sl.h_n, 0));
    if (hipMalloc(&sl.d_jobs, (size_t)16 * e->C) != hipSuccess) return AERO_E_NOMEM;
    HIPCHK(hipEventCreateWithFlags(&sl.ev, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&sl.ev_vit, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&sl.ev_framed, hipEventDisableTiming));
  }
  for (int k = 0; k < Group::NPIN; k++) {
    if (hipHostMalloc(&e->pin_avail[k], sizeof(long long) * e->C) != hipSuccess) return AERO_E_NOMEM;
    HIPCHK(hipEventCreateWithFlags(&e->pin_ev[k], hipEventDisableTiming));
  }
  HIPCHK(hipEventCreateWithFlags(&e->pin_pcm_ev, hipEventDisableTiming));
  if (hipHostMalloc(&e->pin_stat, 128) != hipSuccess) return AERO_E_NOMEM;
  // (st_in is created by the first batch push that needs it: HIP deals its
  // streams round-robin over GPU_MAX_HW_QUEUES hardware queues, 4 by default,
  // and a stream this group never uses would put two groups' kernel streams
  // on one queue, where they run one after the other)
  HIPCHK(hipEventCreateWithFlags(&e->ev_in, hipEventDisableTiming));
  const int nfft = e->g.nfft;
  std::vector<double> cis(2 * WTSIZE), tw(2 * nfft), twi(2 * nfft), taps(MAX_TAPS, 0.0);
  if (e->g.ntaps > MAX_TAPS) return AERO_E_INVALID;
  std::vector<uint8_t> scr(5000);
  host_cis(cis.data());
  host_twiddles(nfft, tw.data(), twi.data());
  host_scrambler(scr.data());
  HIPCHK(hipMemcpy((void *)e->T.cis, cis.data(), sizeof(double) * 2 * WTSIZE, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy((void *)e->T.tw, tw.data(), sizeof(double) * 2 * nfft, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy((void *)e->T.twi, twi.data(), sizeof(double) * 2 * nfft, hipMemcpyHostToDevice));
  {
    std::vector<double> pg(2 * nfft, 0.0), pgi(2 * nfft, 0.0);
    if (nfft == 16384) {
      fftl::twg_build<14>(tw.data(), pg.data());
      fftl::twg_build<14>(twi.data(), pgi.data());
    } else {
      fftl::twg_build<13>(tw.data(), pg.data());
      fftl::twg_build<13>(twi.data(), pgi.data());
    }
    HIPCHK(hipMemcpy((void *)e->T.twg, pg.data(), sizeof(double) * 2 * nfft, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy((void *)e->T.twgi, pgi.data(), sizeof(double) * 2 * nfft, hipMemcpyHostToDevice));
  }
  HIPCHK(hipMemcpy((void *)e->T.scr, scr.data(), 5000, hipMemcpyHostToDevice));
  if (mode == MODE_OQPSK) {
    if (host_rrc(1.0, 55, 48000, 10500 / 2, taps.data()) != NTAPS) return AERO_E_INVALID;
    const double T48 = 48000.0 / (10500.0 / 2);
    DelayDesc dly[4];
    if (!host_delay(1, dly[0]) || !host_delay(T48 / 4.0, dly[1]) || !host_delay(T48 / 4.0, dly[2]) ||
        !host_delay(T48 / 8.0, dly[3]))
      return AERO_E_INVALID;
    if (dly[0].size != 2 || dly[1].size != 4 || dly[2].size != 4 || dly[3].size != 3) return AERO_E_INVALID;
    // the demod kernel bakes in what these designs give at 48 kHz / 10500 bps:
    // the ring ages it reads (template arguments of delay_tap) and weights that
    // do not depend on the write pointer; refuse to run if that ever changes
    static const int ages[4][2] = {{1, 0}, {3, 2}, {3, 2}, {2, 1}};  // {age_old, age_new}
    for (int k = 0; k < 4; k++) {
      if (dly[k].age_old != ages[k][0] || dly[k].age_new != ages[k][1]) return AERO_E_INVALID;
      for (int p = 1; p < dly[k].size; p++)
        if (memcmp(&dly[k].w[p], &dly[k].w[0], 8) || memcmp(&dly[k].omw[p], &dly[k].omw[0], 8))
          return AERO_E_INVALID;
    }
    for (int j = 0; j < NTAPS; j++)  // the kernel stores the 28 distinct taps of the symmetric RRC
      if (memcmp(&taps[j], &taps[NTAPS - 1 - j], 8)) return AERO_E_INVALID;
    const double sr_b[3] = {0.00032714218939589035, 0, 0.00032714218939589035};
    const double sr_a[3] = {1, -0.39005299948210803, 0.99934571562120822};
    const double ct_b[3] = {0.0010275610653672064, 0.0020551221307344128, 0.0010275610653672064};
    const double ct_a[3] = {1, -1.9207386815577139, 0.92509247310306331};
    upload_demod_constants(taps.data(), dly, sr_b, sr_a, ct_b, ct_a);
  } else if (mode == MODE_C8400) {
    // the prefilter kernel: RRC(0.6, 2048 -> 2049 taps, 48000, 4200) into a
    // 4096-point block, its JFFT (oqpskdemodulator.cpp:228-236, jfft.cpp:324-367)
    std::vector<double> k(2 * C_FIR_N, 0.0), rrc(2049), t4(2 * C_FIR_N), ti4(2 * C_FIR_N);
    if (host_rrc(0.6, 2048, 48000, 8400 / 2, rrc.data()) != 2049) return AERO_E_INVALID;
    for (int j = 0; j < 2049; j++) k[2 * j] = rrc[j];
    host_twiddles(C_FIR_N, t4.data(), ti4.data());
    host_jfft(k.data(), C_FIR_N, false, t4.data(), ti4.data());
    std::vector<double> win(NFFT);
    host_coarse_window(NFFT, 10500.0, 48000.0, win.data());
    HIPCHK(hipMemcpy((void *)e->T.cker, k.data(), sizeof(double) * 2 * C_FIR_N, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy((void *)e->T.tw4, t4.data(), sizeof(double) * 2 * C_FIR_N, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy((void *)e->T.twi4, ti4.data(), sizeof(double) * 2 * C_FIR_N, hipMemcpyHostToDevice));
    // in the order the coarse kernel's threads hold the bins after the
    // forward transform (fft_layout.h, G layout): entry i * 1024 + t is bin
    // out_bin_thread(t) | out_bin_reg(i), so a wave's load of register i's
    // weights is one contiguous 512-byte run
    std::vector<double> wperm(NFFT);
    {
      constexpr int L = 14, FT = NFFT / 16;
      const uint64_t G = fftl::lay_g<L>();
      for (int t = 0; t < FT; t++)
        for (int i = 0; i < 16; i++) wperm[(size_t)i * FT + t] = win[fftl::athr<L, fftl::K_G, false>(t) | fftl::areg(G, L, i)];
    }
    HIPCHK(hipMemcpy((void *)e->T.cwin, wperm.data(), sizeof(double) * NFFT, hipMemcpyHostToDevice));
    // symbol timer delays at T = 48000 / 4200 (:186-190): the kernel reads ages
    // {1,0}, {3,2}, {3,2}, {2,1}; T/8's weights depend on the write pointer
    const double T84 = 48000.0 / (8400.0 / 2);
    DelayDesc dly[4];
    if (!host_delay(1, dly[0]) || !host_delay(T84 / 4.0, dly[1]) || !host_delay(T84 / 4.0, dly[2]) ||
        !host_delay(T84 / 8.0, dly[3]))
      return AERO_E_INVALID;
    static const int ages[4][3] = {{2, 1, 0}, {4, 3, 2}, {4, 3, 2}, {3, 2, 1}};  // {size, age_old, age_new}
    for (int j = 0; j < 4; j++)
      if (dly[j].size != ages[j][0] || dly[j].age_old != ages[j][1] || dly[j].age_new != ages[j][2])
        return AERO_E_INVALID;
    upload_c_constants(dly);
    for (int j = 0; j < Group::NPIN; j++) {
      if (hipHostMalloc(&e->pin_cjobs[j], (size_t)c_prejob_bytes() * e->C) != hipSuccess) return AERO_E_NOMEM;
      if (hipMalloc(&e->d_cjobs[j], (size_t)c_prejob_bytes() * e->C) != hipSuccess) return AERO_E_NOMEM;
      HIPCHK(hipEventCreateWithFlags(&e->cjob_ev[j], hipEventDisableTiming));
    }
  } else if (msk_generic(mode)) {
    host_msk_taps(e->g.fs / 600, taps.data());  // delayt8 ages and weights: S.mg
  } else {
    // matched filter sin(pi i / 2SPS) / 2SPS (mskdemodulator.cpp:126-133)
    const int sps = e->g.fs / 600;
    host_msk_taps(sps, taps.data());
    // delayt8.setdelay(SPS / 2.0) (mskdemodulator.cpp:215): the kernel reads
    // ages SPS/2 and SPS/2 - 1 with pointer-independent weights
    int size, age_old, age_new;
    double w, omw;
    if (!host_delay_uniform(sps / 2.0, size, age_old, age_new, w, omw)) return AERO_E_INVALID;
    if (size != e->g.d8_len || age_old != sps / 2 || age_new != sps / 2 - 1) return AERO_E_INVALID;
    const double d8w[2] = {w, omw};
    upload_msk_constants(d8w);  // the st resonator design is per Fs (MskK)
  }
  HIPCHK(hipMemcpy((void *)e->T.taps, taps.data(), sizeof(double) * MAX_TAPS, hipMemcpyHostToDevice));
  HIPCHK(hipGetLastError());
  HIPCHK(hipDeviceSynchronize());
  out = std::move(e);
  return AERO_OK;
}

void group_destroy(Group *e) {
  if (!e) return;
  if (e->st) hipStreamSynchronize(e->st);
  ev_collect(e);
  for (auto &sl : e->slot) {
    if (sl.d_n) (void)hipFree(sl.d_n);
    if (sl.d_jobs) (void)hipFree(sl.d_jobs);
    if (sl.ev_vit) (void)hipEventDestroy(sl.ev_vit);
    if (sl.ev_framed) (void)hipEventDestroy(sl.ev_framed);
    if (sl.h_out) (void)hipHostFree(sl.h_out);
    if (sl.h_n) (void)hipHostFree(sl.h_n);
    if (sl.ev) (void)hipEventDestroy(sl.ev);
  }
  if (e->h_err) (void)hipHostFree(e->h_err);
  for (int k = 0; k < Group::NPIN; k++) {
    if (e->pin_avail[k]) (void)hipHostFree(e->pin_avail[k]);
    if (e->pin_ev[k]) (void)hipEventDestroy(e->pin_ev[k]);
  }
  for (int k = 0; k < Group::NPIN; k++) {
    if (e->pin_gjobs[k]) (void)hipHostFree(e->pin_gjobs[k]);
    if (e->d_gjobs[k]) (void)hipFree(e->d_gjobs[k]);
    if (e->gjob_ev[k]) (void)hipEventDestroy(e->gjob_ev[k]);
  }
  if (e->ev_feed_done) (void)hipEventDestroy(e->ev_feed_done);
  for (int k = 0; k < 2; k++) {
    if (e->pin_hq[k]) (void)hipHostFree(e->pin_hq[k]);
    if (e->hq_ev[k]) (void)hipEventDestroy(e->hq_ev[k]);
  }
  if (e->d_hq) (void)hipFree(e->d_hq);
  for (int k = 0; k < Group::NPIN; k++) {
    if (e->pin_cjobs[k]) (void)hipHostFree(e->pin_cjobs[k]);
    if (e->d_cjobs[k]) (void)hipFree(e->d_cjobs[k]);
    if (e->cjob_ev[k]) (void)hipEventDestroy(e->cjob_ev[k]);
  }
  if (e->pin_stat) (void)hipHostFree(e->pin_stat);
  if (e->pin_pcm) (void)hipHostFree(e->pin_pcm);
  if (e->pin_pcm_ev) (void)hipEventDestroy(e->pin_pcm_ev);
  if (e->st_in) hipStreamSynchronize(e->st_in);
  if (e->ev_in) (void)hipEventDestroy(e->ev_in);
  for (auto &pr : e->consumed) (void)hipEventDestroy(pr.second);
  for (auto ev : e->ev_free) (void)hipEventDestroy(ev);
  if (e->st_in) (void)hipStreamDestroy(e->st_in);
  if (e->d_scratch) (void)hipFree(e->d_scratch);
  if (e->pool) (void)hipFree(e->pool);
  if (e->st) (void)hipStreamDestroy(e->st);
}

}  // namespace

Group::~Group() { group_destroy(this); }

namespace {

// engine channel -> (group, local index); nullptr if out of range
Group *route(aero_engine *e, int ch, int &local) {
  if (!e || ch < 0 || ch >= (int)e->chmap.size() || e->chmap[ch].first >= MODE_BURST) return nullptr;
  local = e->chmap[ch].second;
  return e->groups[e->chmap[ch].first].get();
}

}  // namespace

// A device pointer this process's HIP runtime does not know (e.g. allocated
// by a second runtime copy loaded into the process, aero_engine.py
// load_library) cannot be copied from: refuse it loudly.
int check_dev_ptr(const void *p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    fprintf(stderr, "aero_engine: %p is not a device pointer of this process's HIP runtime\n", p);
    return AERO_E_INVALID;
  }
  return AERO_OK;
}

namespace {

// host memory the HIP runtime has pinned (hipHostMalloc / hipHostRegister,
// e.g. a torch pin_memory() tensor): the DMA engines read it directly
bool is_pinned_host(const void *p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

// one pageable single-channel message into the queue (hostq_flush)
int hostq_push(Group *e, const int16_t *src, size_t n, int c) {
  if (e->hq.size() >= gjob_cap(e) || e->hq_used + n > e->hq_cap)
    if (int rc = hostq_flush(e)) return rc;
  for (int k = 0; k < 2; k++)
    if (!e->hq_ev[k]) HIPCHK(hipEventCreateWithFlags(&e->hq_ev[k], hipEventDisableTiming));
  if (n > e->hq_cap) {
    const size_t cap = std::max<size_t>(n, std::max<size_t>((size_t)1 << 22, 2 * e->hq_cap));
    HIPCHK(hipStreamSynchronize(e->st));  // the last copies and gathers have used them
    for (int k = 0; k < 2; k++) {
      if (e->pin_hq[k]) (void)hipHostFree(e->pin_hq[k]);
      e->pin_hq[k] = nullptr;
    }
    if (e->d_hq) (void)hipFree(e->d_hq);
    e->d_hq = nullptr;
    e->hq_cap = 0;
    for (int k = 0; k < 2; k++)
      if (hipHostMalloc(&e->pin_hq[k], sizeof(int16_t) * cap) != hipSuccess) return AERO_E_NOMEM;
    if (hipMalloc(&e->d_hq, sizeof(int16_t) * cap) != hipSuccess) return AERO_E_NOMEM;
    e->hq_cap = cap;
  }
  // the copy out of this staging two flushes ago is done
  if (e->hq_used == 0) HIPCHK(hipEventSynchronize(e->hq_ev[e->hq_buf]));
  memcpy(e->pin_hq[e->hq_buf] + e->hq_used, src, sizeof(int16_t) * n);
  e->hq.push_back({c, e->hq_used, (long long)n, e->avail[c]});
  e->hq_used += n;
  e->avail[c] += (long long)n;
  return AERO_OK;
}

int push_common(Group *e, const int16_t *src, size_t n, size_t ld, int nch, int c0, bool dev) {
  HOST_TIMER(e, "host_push");
  if (dev)
    if (int rc = check_dev_ptr(src)) return rc;
  // pinned host input goes straight into the PCM ring rows (a DMA on the
  // input stream, overlapping the kernels already queued: one 1-D copy when
  // the batch is whole ring rows, a 2-D copy otherwise), as a device source
  // does; a single channel's pageable message is queued (hostq_push), a
  // pageable batch staged
  const bool pinned = !dev && nch >= 64 && is_pinned_host(src);
  const hipMemcpyKind kind = dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
  if (pinned) dev = true;
  if (int rc = flush_pending_init(e)) return rc;
  // keep the ring from overrunning unprocessed samples
  for (int j = 0; j < nch; j++) {
    const int c = c0 + j;
    if (e->avail[c] + (long long)n - e->nsamp[c] > PCM_CAP - 2) {
      int rc = run_group(e, 0);
      if (rc) return rc;
      if (e->avail[c] + (long long)n - e->nsamp[c] > PCM_CAP - 2) return AERO_E_FULL;
    }
  }
  if (!dev && nch == 1) return hostq_push(e, src, n, c0);
  if (int rc = hostq_flush(e)) return rc;  // ring writes and counters in push order
  const int16_t *dsrc = src;
  if (!dev) {
    // the caller's buffer is copied before returning: into pinned staging
    // (after the previous copy out of it has completed), then async to HBM
    const size_t need = n * ld;
    HIPCHK(hipEventSynchronize(e->pin_pcm_ev));
    if (need > e->scratch_cap) {
      if (e->d_scratch) (void)hipFree(e->d_scratch);
      e->d_scratch = nullptr;
      e->scratch_cap = 0;
      HIPCHK(hipStreamSynchronize(e->st));
      HIPCHK(hipMalloc(&e->d_scratch, need * sizeof(int16_t)));
      e->scratch_cap = need;
    }
    if (need > e->pin_pcm_cap) {
      if (e->pin_pcm) (void)hipHostFree(e->pin_pcm);
      e->pin_pcm = nullptr;
      e->pin_pcm_cap = 0;
      HIPCHK(hipHostMalloc(&e->pin_pcm, need * sizeof(int16_t)));
      e->pin_pcm_cap = need;
    }
    memcpy(e->pin_pcm, src, need * sizeof(int16_t));
    HIPCHK(hipMemcpyAsync(e->d_scratch, e->pin_pcm, need * sizeof(int16_t), hipMemcpyHostToDevice, e->st));
    HIPCHK(hipEventRecord(e->pin_pcm_ev, e->st));
    dsrc = e->d_scratch;
  } else {
    const long long start = e->avail[c0];
    for (int j = 1; j < nch; j++)
      if (e->avail[c0 + j] != start) return AERO_E_INVALID;  // batch pushes are lockstep
    if (!e->st_in) {
      int lo = 0, hi = 0;
      HIPCHK(hipDeviceGetStreamPriorityRange(&lo, &hi));
      HIPCHK(hipStreamCreateWithPriority(&e->st_in, hipStreamNonBlocking, hi));
    }
    // rows of samples [start, start + n) overwrite those of samples below
    // start + n - PCM_CAP: wait for the demod launch that consumed them
    const long long need = start + (long long)n - PCM_CAP;
    if (need > 0) {
      hipEvent_t w = nullptr;
      while (!e->consumed.empty() && e->consumed.front().first < need) {
        e->ev_free.push_back(e->consumed.front().second);
        e->consumed.pop_front();
      }
      if (!e->consumed.empty()) w = e->consumed.front().second;
      if (w) {
        HIPCHK(hipStreamWaitEvent(e->st_in, w, 0));
      } else {
        HIPCHK(hipEventRecord(e->ev_in, e->st));  // not tracked: after all enqueued work
        HIPCHK(hipStreamWaitEvent(e->st_in, e->ev_in, 0));
      }
    }
    const long long r0 = start & (PCM_CAP - 1);
    const size_t n1 = (size_t)std::min<long long>((long long)n, PCM_CAP - r0);
    // whole rows (every channel of the group, the source as wide as the ring)
    // are one contiguous block: a 1-D copy, which the DMA engines run beside
    // the kernels (a 2-D copy is a blit kernel that waits for CUs)
    const bool rows = c0 == 0 && nch == e->C && ld == (size_t)e->C;
    auto copy = [&](int16_t *dst, const int16_t *from, size_t nrows) -> hipError_t {
      if (rows) return hipMemcpyAsync(dst, from, sizeof(int16_t) * e->C * nrows, kind, e->st_in);
      return hipMemcpy2DAsync(dst, sizeof(int16_t) * e->C, from, sizeof(int16_t) * ld, sizeof(int16_t) * nch, nrows,
                              kind, e->st_in);
    };
    HIPCHK(copy(e->S.pcm + r0 * e->C + c0, src, n1));
    if (n1 < n) HIPCHK(copy(e->S.pcm + c0, src + n1 * ld, n - n1));
    HIPCHK(hipEventRecord(e->ev_in, e->st_in));
    {
      HOST_TIMER(e, "host_push_copy");
      HIPCHK(hipEventSynchronize(e->ev_in));  // the caller's buffer is free again
    }
    HIPCHK(hipStreamWaitEvent(e->st, e->ev_in, 0));
    for (int j = 0; j < nch; j++) e->avail[c0 + j] += (long long)n;
  }
  if (!dev) {
    const long long start = e->avail[c0];
    for (int j = 1; j < nch; j++)
      if (e->avail[c0 + j] != start) return AERO_E_INVALID;  // batch pushes are lockstep
    const long long total = (long long)n * nch;
    const int grid = (int)std::min<long long>((total + 255) / 256, 65536);
    hipLaunchKernelGGL(pcm_scatter_kernel, dim3(grid), dim3(256), 0, e->st, e->S.pcm, e->C, (long long)PCM_CAP - 1,
                       dsrc, (long long)n, (long long)ld, nch, c0, start);
    HIPCHK(hipGetLastError());
    for (int j = 0; j < nch; j++) e->avail[c0 + j] += (long long)n;
  }
  // device copy of the counters, from pinned staging (stream-ordered before the next demod)
  const int k = e->next_pin;
  e->next_pin = (k + 1) % Group::NPIN;
  {
    HOST_TIMER(e, "host_push_pin");
    HIPCHK(hipEventSynchronize(e->pin_ev[k]));
  }
  memcpy(e->pin_avail[k], e->avail.data() + c0, 8 * (size_t)nch);
  HIPCHK(hipMemcpyAsync(e->S.ls + (size_t)LS_AVAIL * e->C + c0, e->pin_avail[k], 8 * nch, hipMemcpyHostToDevice,
                        e->st));
  HIPCHK(hipEventRecord(e->pin_ev[k], e->st));
  return AERO_OK;
}

// Channeliser -> decoder hand-off without a host wait (aero_chan_feed): the
// group's stream waits for the producer's audio (event `ready`), one gather
// launch copies every item into the PCM rings and sets the channels' pushed
// counters, and the producer's stream then waits for that launch before it
// may overwrite the audio.  items: (local channel, device source, samples).
int feed_group(Group *e, const std::vector<std::pair<int, std::pair<const int16_t *, size_t>>> &items,
               hipEvent_t ready, hipStream_t producer) {
  HOST_TIMER(e, "host_push");
  if (items.empty()) return AERO_OK;
  if (int rc = flush_pending_init(e)) return rc;
  for (auto &it : items) {  // keep the ring from overrunning unprocessed samples
    const int c = it.first;
    const long long n = (long long)it.second.second;
    if (n > PCM_CAP / 2) return AERO_E_FULL;
    if (e->avail[c] + n - e->nsamp[c] > PCM_CAP - 2) {
      if (int rc = run_group(e, 0)) return rc;
      if (e->avail[c] + n - e->nsamp[c] > PCM_CAP - 2) return AERO_E_FULL;
    }
  }
  if ((int)items.size() > e->C) return AERO_E_INVALID;
  if (int rc = hostq_flush(e)) return rc;
  int k;
  if (int rc = gather_table(e, k)) return rc;
  if (!e->ev_feed_done) HIPCHK(hipEventCreateWithFlags(&e->ev_feed_done, hipEventDisableTiming));
  long long mx = 0;
  for (size_t i = 0; i < items.size(); i++) {
    const int c = items[i].first;
    const long long n = (long long)items[i].second.second;
    GatherJob &j = e->pin_gjobs[k][i];
    j.src = items[i].second.first;
    j.n = n;
    j.start = e->avail[c];
    j.avail_after = e->avail[c] + n;
    j.c = c;
    j.later = 0;
    e->avail[c] += n;
    if (e->mode == MODE_C8400 && n) e->msg_end[c].push_back(e->avail[c]);  // one message per item
    mx = std::max(mx, n);
  }
  mark_last_jobs(e->pin_gjobs[k], items.size(), e->C);
  HIPCHK(hipMemcpyAsync(e->d_gjobs[k], e->pin_gjobs[k], sizeof(GatherJob) * items.size(), hipMemcpyHostToDevice,
                        e->st));
  HIPCHK(hipEventRecord(e->gjob_ev[k], e->st));
  HIPCHK(hipStreamWaitEvent(e->st, ready, 0));
  const unsigned gx = (unsigned)std::max<long long>(1, std::min<long long>((mx + 255) / 256, 64));
  hipLaunchKernelGGL(pcm_gather_kernel, dim3(gx, (unsigned)items.size()), dim3(256), 0, e->st, e->S.pcm, e->C,
                     (long long)PCM_CAP - 1, e->S.ls + (size_t)LS_AVAIL * e->C, (const GatherJob *)e->d_gjobs[k]);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(e->ev_feed_done, e->st));
  HIPCHK(hipStreamWaitEvent(producer, e->ev_feed_done, 0));
  return AERO_OK;
}

}  // namespace

namespace {

// A new local channel of the group of `mode` (created on first use) for
// engine channel gc; its device state is initialised by flush_pending_init
// the gid of the continuous MSK group serving (bit rate, fs), creating a
// generic-rate group when fs has no fixed one; AERO_E_RATE for rates the
// engine does not serve
int msk_gid(aero_engine *e, int bitrate, int fs, int &gid) {
  const int m = msk_mode(bitrate, fs);
  if (m >= 0) {
    gid = m;
    return AERO_OK;
  }
  const int gm = bitrate == 600 ? MODE_MSKG600 : MODE_MSKG1200;
  int free_gid = -1;
  for (size_t k = MODE_COUNT + 1; k < e->groups.size(); k++) {
    Group *h = e->groups[k].get();
    if (!h) {
      if (free_gid < 0) free_gid = (int)k;  // a retired group's slot
      continue;
    }
    if (h->mode == gm && h->g.fs == fs && (h->nch < h->C || !h->free_slots.empty())) {
      gid = (int)k;
      return AERO_OK;
    }
  }
  std::unique_ptr<Group> g;
  gid = free_gid >= 0 ? free_gid : (int)e->groups.size();
  if (int rc = group_create(e, gm, gid, fs, g)) return rc;
  if (free_gid >= 0)
    e->groups[gid] = std::move(g);
  else
    e->groups.push_back(std::move(g));
  return AERO_OK;
}

int group_add_channel(aero_engine *e, int gid, const aero_channel_cfg &cfg, int gc, int *local) {
  if (!e->groups[gid])
    if (int rc = group_create(e, gid, gid, 0, e->groups[gid])) return rc;
  Group *g = e->groups[gid].get();
  if (!g->free_slots.empty()) {  // a slot an MSK channel moved out of
    if (int rc = flush_pending_init(g)) return rc;
    const int c = g->free_slots.back();
    if (int rc = reset_slot(g, c)) return rc;
    g->free_slots.pop_back();
    g->cfg[c] = cfg;
    g->gch[c] = gc;
    g->avail[c] = g->nsamp[c] = g->hops[c] = 0;
    g->host[c].reset(new PChannelHost(cfg.disable_reassembly != 0));
    g->infofield[c].clear();
    g->soft_hold[c].clear();
    g->hop_hold[c].clear();
    g->pt_hold[c].clear();
    g->blk_hold[c].clear();
    g->frame_hold[c].clear();
    g->soft_seen[c] = 0;
    g->hop_base[c] = 0;
    *local = c;
    return AERO_OK;
  }
  if (g->nch >= g->C) return AERO_E_FULL;
  const int c = g->nch;
  g->nch++;
  g->cfg.push_back(cfg);
  g->gch.push_back(gc);
  g->avail.push_back(0);
  g->nsamp.push_back(0);
  g->hops.push_back(0);
  g->host.emplace_back(new PChannelHost(cfg.disable_reassembly != 0));
  g->infofield.emplace_back();
  g->soft_hold.emplace_back();
  g->hop_hold.emplace_back();
  g->pt_hold.emplace_back();
  g->blk_hold.emplace_back();
  g->frame_hold.emplace_back();
  g->soft_seen.push_back(0);
  g->hop_base.push_back(0);
  g->msg_end.emplace_back();
  g->pre_end.push_back(0);
  g->cunit_hold.emplace_back();
  g->voice_hold.emplace_back();
  g->c_cd.push_back(0);
  g->c_dcd.push_back(0);
  g->c_edges.push_back(0);
  if (g->trace_some) g->trace_mask.resize(g->C, 0);
  *local = c;
  return AERO_OK;
}

// MskDemodulator::dataReceived at another sample rate (decode/mskdemodulator.cpp
// :473-481): setSettings(last_applied_settings with the new Fs) (:94-218) is
// applied to the channel's state, and the channel moves to the group of the
// new rate.  All of its samples so far are demodulated and decoded first (a
// flush of the old group: continuous channels are chunk-invariant, so the
// other channels' outputs do not change).  What setSettings keeps and what
// it resets:
//   kept: mixer_center / mixer2 / st_osc phase pointers, the coarse ring's
//     contents (its pointer restarts), the coarse y history and emptying
//     countdown, msema (created by the ctor only), DiffDecode, the soft bits
//     not yet framed, AeroL, SignalHunter;
//   resized, contents kept: dt (SPS/2 + 1) and delayedsmpl (SPS + 1)
//     (DelayThing::setLength, QVector::resize), pointers restart;
//   reset: frequencies (mixer_center and mixer2 to freq_center 0, st_osc to
//     fb/2 at the new Fs), matched filters, AGC, marg, delayt8, the st
//     resonator (its design follows Fs), mse = 10.
int msk_migrate(aero_engine *e, int ch, uint32_t fs) {
  const int from = e->chmap[ch].first, c = e->chmap[ch].second;
  HIPCHK(hipSetDevice(e->device));
  int to;
  if (int rc = msk_gid(e, msk_bitrate(e->groups[from]->mode), (int)fs, to)) return rc;
  Group *g = e->groups[from].get();
  if (int rc = flush_pending_init(g)) return rc;
  if (int rc = run_group(g, 1)) return rc;
  if (int rc = drain_group(g)) return rc;
  host_wait(e);
  aero_channel_cfg cfg = g->cfg[c];
  cfg.fs = fs;
  int c2;
  if (int rc = group_add_channel(e, to, cfg, ch, &c2)) return rc;
  Group *h = e->groups[to].get();
  if (int rc = flush_pending_init(h)) return rc;
  const int C = g->C, C2 = h->C;
  // scalar state: read the old channel's fields, apply setSettings, write
  std::vector<double> ds(DS_COUNT);
  std::vector<int> is(IS_COUNT);
  std::vector<long long> ls(LS_COUNT);
  HIPCHK(hipMemcpy2D(ds.data(), 8, g->S.ds + c, (size_t)8 * C, 8, DS_COUNT, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy2D(is.data(), 4, g->S.is + c, (size_t)4 * C, 4, IS_COUNT, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy2D(ls.data(), 8, g->S.ls + c, (size_t)8 * C, 8, LS_COUNT, hipMemcpyDeviceToHost));
  const long long n_old = ls[LS_NSAMP], ev_old = ls[LS_EVENTS], zb = ls[LS_ZERO_BEFORE];
  ds[DS_M2_FREQ] = 0;
  ds[DS_M2_STEP] = 0;
  ds[DS_MC_FREQ] = 0;
  ds[DS_MC_STEP] = 0;
  ds[DS_SO_FREQ] = 300;  // st_osc.SetFreq(fb / 2, Fs)
  ds[DS_SO_STEP] = (300.0) * ((double)WTSIZE) / ((float)h->g.fs);
  ds[DS_AGC_SUM] = 0;
  ds[DS_SR_X1] = ds[DS_SR_X2] = ds[DS_SR_Y1] = ds[DS_SR_Y2] = 0;
  ds[DS_MARG_SUM] = 0;
  ds[DS_MSE] = 10.0;
  is[IS_HOPS_DONE] = 0;
  is[IS_MS_OFF] = (int)((is[IS_MS_OFF] + ev_old) % MSK_MSEMA);
  ls[LS_NSAMP] = ls[LS_AVAIL] = ls[LS_FILLED] = 0;
  ls[LS_ZERO_BEFORE] = -(1LL << 62);  // the cleared entries are written as zeros below; the rest is read
  ls[LS_PT_N] = 0;
  ls[LS_EVENTS] = 0;
  HIPCHK(hipMemcpy2D(h->S.ds + c2, (size_t)8 * C2, ds.data(), 8, 8, DS_COUNT, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy2D(h->S.is + c2, (size_t)4 * C2, is.data(), 4, 4, IS_COUNT, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy2D(h->S.ls + c2, (size_t)8 * C2, ls.data(), 8, 8, LS_COUNT, hipMemcpyHostToDevice));
  // rows that carry over (same sizes in both groups)
  HIPCHK(hipMemcpy(h->S.soft + (size_t)c2 * SOFT_RING, g->S.soft + (size_t)c * SOFT_RING, SOFT_RING,
                   hipMemcpyDeviceToDevice));
  HIPCHK(hipMemcpy(h->S.block + (size_t)c2 * 2 * h->g.block, g->S.block + (size_t)c * 2 * g->g.block,
                   (size_t)2 * g->g.block, hipMemcpyDeviceToDevice));
  HIPCHK(hipMemcpy(h->S.overlap + (size_t)c2 * 64, g->S.overlap + (size_t)c * 64, 64, hipMemcpyDeviceToDevice));
  HIPCHK(hipMemcpy(h->S.dl2 + (size_t)c2 * h->g.dl2_len, g->S.dl2 + (size_t)c * g->g.dl2_len, g->g.dl2_len,
                   hipMemcpyDeviceToDevice));
  const size_t ylen = (size_t)(g->g.y_hi - g->g.y_lo + 1);
  HIPCHK(hipMemcpy(h->S.y + c2 * ylen, g->S.y + c * ylen, ylen * 8, hipMemcpyDeviceToDevice));
  HIPCHK(hipMemcpy(h->S.ms + (size_t)c2 * MSK_MSEMA, g->S.ms + (size_t)c * MSK_MSEMA, (size_t)8 * MSK_MSEMA,
                   hipMemcpyDeviceToDevice));
  // dt and delayedsmpl resized with their contents (QVector index = ring slot)
  const int dtn = std::min(g->g.dt_len, h->g.dt_len), dsn = std::min(g->g.dsm_len, h->g.dsm_len);
  HIPCHK(hipMemcpy(h->S.dt + (size_t)c2 * h->g.dt_len, g->S.dt + (size_t)c * g->g.dt_len, (size_t)16 * dtn,
                   hipMemcpyDeviceToDevice));
  HIPCHK(hipMemcpy2D(h->S.dsm + c2, (size_t)16 * C2, g->S.dsm + c, (size_t)16 * C, 16, dsn, hipMemcpyDeviceToDevice));
  // the coarse ring: slot = sample index mod nfft on both sides; entries of
  // samples the AFC zeroed (below zero_before) are written as zeros
  {
    const int nf = g->g.nfft;
    std::vector<uint32_t> ring(nf);
    HIPCHK(hipMemcpy(ring.data(), g->S.cring + (size_t)c * nf, (size_t)4 * nf, hipMemcpyDeviceToHost));
    for (int j = 0; j < nf; j++) {
      const long long smp = (n_old - 1) - (((n_old - 1 - j) % nf + nf) % nf);  // last sample in slot j
      if (smp < zb) ring[j] = 0;  // CIS[0] x 0: the zero a cleared bbcycbuff holds
    }
    HIPCHK(hipMemcpy(h->S.cring + (size_t)c2 * nf, ring.data(), (size_t)4 * nf, hipMemcpyHostToDevice));
  }
  // host state moves with the channel
  h->host[c2] = std::move(g->host[c]);
  g->host[c].reset(new PChannelHost(cfg.disable_reassembly != 0));
  std::swap(h->infofield[c2], g->infofield[c]);
  std::swap(h->soft_hold[c2], g->soft_hold[c]);
  std::swap(h->hop_hold[c2], g->hop_hold[c]);
  std::swap(h->pt_hold[c2], g->pt_hold[c]);
  std::swap(h->blk_hold[c2], g->blk_hold[c]);
  std::swap(h->frame_hold[c2], g->frame_hold[c]);
  h->soft_seen[c2] = g->soft_seen[c];
  h->hop_base[c2] = g->hop_base[c] + n_old;
  if (g->trace_some && g->trace_mask[c]) {
    h->trace_some = true;
    h->trace_mask.resize(h->C, 0);
    h->trace_mask[c2] = 1;
    h->trace_list.push_back(c2);
    g->trace_mask[c] = 0;
    g->trace_list.erase(std::remove(g->trace_list.begin(), g->trace_list.end(), c), g->trace_list.end());
  }
  e->chmap[ch] = {to, c2};
  // the old slot is free for the next channel of that group (it has no
  // samples left: the group ran and drained it above)
  g->gch[c] = -1;
  g->free_slots.push_back(c);
  // a generic-rate group nobody is left in is released (its device pool,
  // stream and pinned buffers); its counters stay in the engine's totals
  if (msk_generic(g->mode) && (int)g->free_slots.size() == g->nch) {
    e->retired_jobs += g->st_jobs.load();
    e->retired_frames += g->st_frames.load();
    e->retired_su_ok += g->st_su_ok.load();
    e->groups[from].reset();
  }
  return AERO_OK;
}

// the group and local index of a continuous channel for a message at rate fs:
// an MSK channel whose group runs at another rate moves first
Group *route_rate(aero_engine *e, int ch, uint32_t fs, int &local, int &rc) {
  rc = AERO_OK;
  Group *g = route(e, ch, local);
  if (!g || g->mode == MODE_OQPSK || g->mode == MODE_C8400 || fs == (uint32_t)g->g.fs)
    return g;  // OQPSK only logs it (:626-628)
  if ((rc = msk_migrate(e, ch, fs))) return nullptr;
  return route(e, ch, local);
}

}  // namespace

extern "C" {

const char *aero_strerror(int rc) {
  switch (rc) {
    case AERO_OK: return "ok";
    case AERO_E_INVALID: return "invalid argument or unsupported configuration";
    case AERO_E_NOMEM: return "out of memory";
    case AERO_E_HIP: return "HIP runtime error";
    case AERO_E_NOGPU: return "no usable gfx950 device";
    case AERO_E_FULL: return "channel table or ring full";
    case AERO_E_RATE: return "sample rate mismatch";
    case AERO_E_DEVICE: return "device error: a demod wave hand-off timed out (outputs invalid)";
    default: return "unknown error";
  }
}

int aero_engine_create(const aero_engine_cfg *cfg, aero_engine **out) {
  if (!cfg || !out || cfg->max_channels <= 0) return AERO_E_INVALID;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= cfg->device) return AERO_E_NOGPU;
  HIPCHK(hipSetDevice(cfg->device));
  std::unique_ptr<aero_engine> e(new aero_engine());
  e->device = cfg->device;
  e->flags = cfg->flags;
  e->max_channels = cfg->max_channels;
  {
    // host threads for the per-frame SU/ACARS work (AERO_HOST_THREADS overrides)
    const char *ev = getenv("AERO_HOST_THREADS");
    const int hw = (int)std::thread::hardware_concurrency();
    int n = ev ? atoi(ev) : std::min(16, std::max(1, hw));
    if (n < 1) n = 1;
    e->hpool.reset(new HostPool(n));
  }
  // every group (continuous and burst) is created on its kind's first
  // aero_channel_open: an engine of burst channels holds no continuous state
  *out = e.release();
  return AERO_OK;
}

void aero_engine_destroy(aero_engine *e) {
  if (!e) return;
  hipSetDevice(e->device);
  for (auto &g : e->groups)
    if (g) (void)drain_group(g.get());
  host_wait(e);
  for (auto &g : e->groups) g.reset();
  for (BurstGroup *b : e->burst)
    if (b) burst_group_destroy(b);
  delete e;
}

int aero_channel_open(aero_engine *e, const aero_channel_cfg *cfg, int *ch_out) {
  if (!e || !cfg || !ch_out) return AERO_E_INVALID;
  if (cfg->burst) {
    // aero-decode --burst: 10500 bps OQPSK at 48 kHz; 600 / 1200 bps MSK run
    // one fb = 1200 demodulator configured for 48 kHz whatever rate the audio
    // is labelled with (decode/decode.cpp:123-132; a mismatch is only logged,
    // burstmskdemodulator.cpp:708-714)
    int kind;
    if (cfg->bitrate == 10500 && cfg->fs == 48000)
      kind = BURST_OQPSK;
    else if ((cfg->bitrate == 600 || cfg->bitrate == 1200) && cfg->fs > 0)
      kind = BURST_MSK;
    else
      return AERO_E_INVALID;
    HIPCHK(hipSetDevice(e->device));
    if (!e->burst[kind]) {
      if (int rc = burst_group_create(e->device, e->flags, e->max_channels, kind, &e->burst[kind])) return rc;
      burst_group_set_pool(e->burst[kind], e->hpool.get());
    }
    int local;
    if (int rc = burst_open(e->burst[kind], (int)cfg->bitrate, cfg->disable_reassembly != 0, &local)) return rc;
    *ch_out = (int)e->chmap.size();
    e->chmap.push_back({MODE_BURST + kind, local});
    return AERO_OK;
  }
  // decode/decode.h:42 validBitRates: 10500 (48 kHz), 600 and 1200 at any
  // rate MSK is served at (12 / 24 kHz as decode/decode.cpp:145); and the C
  // channel, 8400 at 48 kHz (OqpskDemodulator at fb = 8400 + AeroL::DecodeC)
  const bool oq = (cfg->bitrate == 10500 || cfg->bitrate == 8400) && cfg->fs == 48000;
  if (!oq && !(cfg->bitrate == 600 || cfg->bitrate == 1200)) return AERO_E_INVALID;
  if (!oq && (cfg->fs < (uint32_t)MSK_FS_MIN || cfg->fs > (uint32_t)MSK_FS_MAX)) return AERO_E_RATE;
  HIPCHK(hipSetDevice(e->device));
  host_wait(e);  // the host task indexes the per-channel tables
  int gid = MODE_OQPSK;
  if (cfg->bitrate == 8400) {
    gid = GID_C8400;
    if (!e->groups[gid])
      if (int rc = group_create(e, MODE_C8400, gid, 48000, e->groups[gid])) return rc;
  } else if (cfg->bitrate != 10500) {
    if (int rc = msk_gid(e, (int)cfg->bitrate, (int)cfg->fs, gid)) return rc;
  }
  int c;
  if (int rc = group_add_channel(e, gid, *cfg, (int)e->chmap.size(), &c)) return rc;
  *ch_out = (int)e->chmap.size();
  e->chmap.push_back({gid, c});
  return AERO_OK;
}

// burst: one message = one BurstOqpskDemodulator::writeDataSlot call; pieces
// of a long message keep its single message start
int push_burst(aero_engine *e, BurstGroup *bg, int b, const int16_t *pcm, size_t n, bool dev) {
  HIPCHK(hipSetDevice(e->device));
  size_t off = 0;
  while (off < n) {
    const size_t piece = std::min<size_t>(n - off, 16384);
    if (int rc = burst_push(bg, b, pcm + off, piece, dev, off == 0)) return rc;
    off += piece;
  }
  return AERO_OK;
}

int aero_push_pcm(aero_engine *e, int ch, const int16_t *pcm, size_t n, uint32_t fs) {
  BurstGroup *bg;
  const int b = route_burst(e, ch, &bg);
  if (b >= 0) return (pcm || !n) ? push_burst(e, bg, b, pcm, n, false) : AERO_E_INVALID;  // rate only logged (:626-628)
  if (!pcm && n) return AERO_E_INVALID;
  // OQPSK only logs a rate mismatch (oqpskdemodulator.cpp:626-628); the MSK
  // demodulator re-applies its settings at the new rate (mskdemodulator.cpp
  // :473-481): the channel moves to that rate's group (msk_migrate)
  int c, rc;
  Group *g = route_rate(e, ch, fs, c, rc);
  if (rc) return rc;
  if (!g) return AERO_E_INVALID;
  if (!n) return AERO_OK;  // dataReceived with an empty message returns at once (:286-287)
  // a C-channel message is one prefilter block (oqpskdemodulator.cpp:292-324): whole, at most half the ring
  if (g->mode == MODE_C8400 && n > (size_t)PCM_CAP / 2) return AERO_E_INVALID;
  HIPCHK(hipSetDevice(e->device));
  // split so one piece never exceeds the ring
  size_t off = 0;
  while (off < n) {
    const size_t piece = std::min<size_t>(n - off, PCM_CAP / 2);
    int rc = push_common(g, pcm + off, piece, 1, 1, c, false);
    if (rc) return rc;
    off += piece;
  }
  if (g->mode == MODE_C8400) g->msg_end[c].push_back(g->avail[c]);
  return AERO_OK;
}

int aero_push_pcm_dev(aero_engine *e, int ch, const int16_t *pcm, size_t n, uint32_t fs) {
  BurstGroup *bg;
  const int b = route_burst(e, ch, &bg);
  if (b >= 0) return (pcm || !n) ? push_burst(e, bg, b, pcm, n, true) : AERO_E_INVALID;
  if (!pcm && n) return AERO_E_INVALID;
  int c, rc;
  Group *g = route_rate(e, ch, fs, c, rc);
  if (rc) return rc;
  if (!g) return AERO_E_INVALID;
  if (!n) return AERO_OK;
  if (g->mode == MODE_C8400 && n > (size_t)PCM_CAP / 2) return AERO_E_INVALID;
  HIPCHK(hipSetDevice(e->device));
  size_t off = 0;
  while (off < n) {
    const size_t piece = std::min<size_t>(n - off, PCM_CAP / 2);
    int rc = push_common(g, pcm + off, piece, 1, 1, c, true);
    if (rc) return rc;
    off += piece;
  }
  if (g->mode == MODE_C8400) g->msg_end[c].push_back(g->avail[c]);
  return AERO_OK;
}

int aero_push_pcm_batch(aero_engine *e, const int16_t *pcm, size_t n, size_t ld, int nch, int dev) {
  if (!e || !pcm || nch <= 0 || nch > (int)e->chmap.size() || ld < (size_t)nch) return AERO_E_INVALID;
  // channels [0, nch) must be one kind, opened in order (local == engine index)
  const int mode = e->chmap[0].first;
  for (int j = 0; j < nch; j++)
    if (e->chmap[j].first != mode || e->chmap[j].second != j) return AERO_E_INVALID;
  if (mode >= MODE_BURST) {  // one message of n <= 16384 samples per channel
    if (dev && check_dev_ptr(pcm)) return AERO_E_INVALID;
    HIPCHK(hipSetDevice(e->device));
    return burst_push_batch(e->burst[mode - MODE_BURST], pcm, n, ld, nch, dev != 0);
  }
  Group *g = e->groups[mode].get();
  if (g->mode == MODE_C8400 && n > (size_t)PCM_CAP / 2) return AERO_E_INVALID;
  HIPCHK(hipSetDevice(e->device));
  size_t off = 0;
  while (off < n) {
    const size_t piece = std::min<size_t>(n - off, PCM_CAP / 2);
    int rc = push_common(g, pcm + off * ld, piece, ld, nch, 0, dev != 0);
    if (rc) return rc;
    off += piece;
  }
  if (g->mode == MODE_C8400 && n)  // one message per channel
    for (int j = 0; j < nch; j++) g->msg_end[j].push_back(g->avail[j]);
  return AERO_OK;
}

int aero_trace_select(aero_engine *e, const int *ch, int n) {
  if (!e || n < 0 || (n && !ch)) return AERO_E_INVALID;
  for (int i = 0; i < n; i++) {
    int c;
    if (!route(e, ch[i], c)) return AERO_E_INVALID;
  }
  host_wait(e);
  for (auto &g : e->groups) {
    if (!g) continue;
    g->trace_some = n > 0;  // a group with none of the channels keeps none
    g->trace_list.clear();
    g->trace_mask.assign(g->C, 0);
  }
  for (int i = 0; i < n; i++) {
    int c;
    Group *g = route(e, ch[i], c);
    if (!g->trace_mask[c]) g->trace_list.push_back(c);
    g->trace_mask[c] = 1;
  }
  return AERO_OK;
}

int aero_run(aero_engine *e) {
  if (!e) return AERO_E_INVALID;
  return run_impl(e, 0);
}

int aero_flush(aero_engine *e) {
  if (!e) return AERO_E_INVALID;
  return run_impl(e, 1);
}

int aero_pop_softbits(aero_engine *e, int ch, int16_t *dst, size_t cap, size_t *n) {
  BurstGroup *bg;
  const int b = route_burst(e, ch, &bg);
  if (b >= 0) return burst_pop_soft(bg, b, dst, cap, n);
  int c;
  Group *g = route(e, ch, c);
  if (!g) return AERO_E_INVALID;
  return pop_vec(g->soft_hold[c], dst, cap, n);
}

int aero_pop_items(aero_engine *e, int ch, aero_acars_item *dst, size_t cap, size_t *n) {
  BurstGroup *bg;
  const int b = route_burst(e, ch, &bg);
  if (b >= 0) return pop_vec(burst_items(bg, b), dst, cap, n);
  int c;
  Group *g = route(e, ch, c);
  if (!g) return AERO_E_INVALID;
  poll_all(e);
  host_wait(e);
  return pop_vec(g->host[c]->items, dst, cap, n);
}

int aero_pop_items_all(aero_engine *e, aero_acars_item *dst, int *ch, size_t cap, size_t *n) {
  if (!e || (cap && (!dst || !ch))) return AERO_E_INVALID;
  poll_all(e);
  host_wait(e);
  size_t k = 0;
  for (int gc = 0; gc < (int)e->chmap.size() && k < cap; gc++) {
    auto &v = e->chmap[gc].first >= MODE_BURST
                  ? burst_items(e->burst[e->chmap[gc].first - MODE_BURST], e->chmap[gc].second)
                  : e->groups[e->chmap[gc].first]->host[e->chmap[gc].second]->items;
    const size_t m = std::min(cap - k, v.size());
    for (size_t i = 0; i < m; i++) {  // msg bytes past msg_len are left unspecified
      memcpy(&dst[k + i], &v[i], offsetof(aero_acars_item, msg) + v[i].msg_len);
      ch[k + i] = gc;
    }
    v.erase(v.begin(), v.begin() + m);
    k += m;
  }
  if (n) *n = k;
  return AERO_OK;
}

int aero_pop_hops(aero_engine *e, int ch, double *dst, size_t cap_records, size_t *n) {
  BurstGroup *bg;
  const int b = route_burst(e, ch, &bg);
  if (b >= 0) return burst_pop_hops(bg, b, dst, cap_records, n);
  int c;
  Group *g = route(e, ch, c);
  if (!g) return AERO_E_INVALID;
  size_t k = 0;
  int rc = pop_vec(g->hop_hold[c], dst, cap_records * 6, &k);
  if (n) *n = k / 6;
  return rc;
}

int aero_pop_pt(aero_engine *e, int ch, double *dst, size_t cap_records, size_t *n) {
  if (route_burst(e, ch) >= 0) {  // not produced by burst channels
    if (n) *n = 0;
    return AERO_OK;
  }
  int c;
  Group *g = route(e, ch, c);
  if (!g) return AERO_E_INVALID;
  size_t k = 0;
  int rc = pop_vec(g->pt_hold[c], dst, cap_records * 2, &k);
  if (n) *n = k / 2;
  return rc;
}

int aero_pop_blocks(aero_engine *e, int ch, uint8_t *dst, size_t cap, size_t *n) {
  if (route_burst(e, ch) >= 0) {  // not produced by burst channels
    if (n) *n = 0;
    return AERO_OK;
  }
  int c;
  Group *g = route(e, ch, c);
  if (!g) return AERO_E_INVALID;
  host_wait(e);
  return pop_vec(g->blk_hold[c], dst, cap, n);
}

int aero_pop_frames(aero_engine *e, int ch, uint8_t *dst, size_t cap, size_t *n) {
  if (route_burst(e, ch) >= 0) {  // not produced by burst channels
    if (n) *n = 0;
    return AERO_OK;
  }
  int c;
  Group *g = route(e, ch, c);
  if (!g) return AERO_E_INVALID;
  host_wait(e);
  return pop_vec(g->frame_hold[c], dst, cap, n);
}

int aero_pop_c_units(aero_engine *e, int ch, uint8_t *dst, size_t cap, size_t *n) {
  int c;
  Group *g = route(e, ch, c);
  if (!g || g->mode != MODE_C8400) return AERO_E_INVALID;
  host_wait(e);
  auto &v = g->cunit_hold[c];
  const size_t k = std::min(cap, v.size() / 12);
  if (dst && k) memcpy(dst, v.data(), 12 * k);
  v.erase(v.begin(), v.begin() + 12 * k);
  if (n) *n = k;
  return AERO_OK;
}

int aero_pop_voice(aero_engine *e, int ch, uint8_t *dst, size_t cap, size_t *n) {
  int c;
  Group *g = route(e, ch, c);
  if (!g || g->mode != MODE_C8400) return AERO_E_INVALID;
  host_wait(e);
  auto &v = g->voice_hold[c];
  const size_t k = std::min(cap, v.size() / 304);
  if (dst && k) memcpy(dst, v.data(), 304 * k);
  v.erase(v.begin(), v.begin() + 304 * k);
  if (n) *n = k;
  return AERO_OK;
}

int aero_pop_rt_tests(aero_engine *e, int ch, uint8_t *dst, size_t cap, size_t *n) {
  BurstGroup *bg;
  const int b = route_burst(e, ch, &bg);
  if (b < 0) return AERO_E_INVALID;
  return burst_pop_tests(bg, b, dst, cap, n);
}

int aero_pop_rt_packets(aero_engine *e, int ch, uint8_t *dst, size_t cap, size_t *n) {
  BurstGroup *bg;
  const int b = route_burst(e, ch, &bg);
  if (b < 0) return AERO_E_INVALID;
  return burst_pop_packets(bg, b, dst, cap, n);
}

int aero_timing(aero_engine *e, const char *name, double *ms, long *launches) {
  if (!e || !name) return AERO_E_INVALID;
  double tms = 0;
  long tl = 0;
  for (auto &g : e->groups) {
    if (!g) continue;
    ev_collect(g.get());
    auto it = g->timing.find(name);
    if (it != g->timing.end()) {
      tms += it->second.ms;
      tl += it->second.launches;
    }
  }
  for (BurstGroup *b : e->burst) burst_timing(b, name, &tms, &tl);
  if (ms) *ms = tms;
  if (launches) *launches = tl;
  return AERO_OK;
}

void aero_timing_reset(aero_engine *e) {
  if (!e) return;
  for (BurstGroup *b : e->burst) burst_timing_reset(b);
  for (auto &g : e->groups)
    if (g) {
      ev_collect(g.get());
      g->timing.clear();
    }
}

int aero_stat(aero_engine *e, const char *name, uint64_t *value) {
  if (!e || !name || !value) return AERO_E_INVALID;
  host_wait(e);  // counters of frames the host workers are still handling
  uint64_t v = 0;
  const std::string n(name);
  if (n != "rt_tests" && n != "rt_packets" && n != "rt_pass_max" && n != "viterbi_jobs" && n != "frames" &&
      n != "su_crc_ok" && n != "device_bytes" && n != "groups")
    return AERO_E_INVALID;
  if (n == "device_bytes" || n == "groups") {  // continuous groups' device pools, and how many exist
    for (auto &g : e->groups)
      if (g) v += n == "groups" ? 1 : (uint64_t)g->pool_bytes;
    *value = v;
    return AERO_OK;
  }
  if (n == "rt_pass_max") {
    *value = std::max(burst_stat(e->burst[0], 2), burst_stat(e->burst[1], 2));
    return AERO_OK;
  }
  if (n == "rt_tests" || n == "rt_packets") {
    *value = burst_stat(e->burst[0], n == "rt_packets") + burst_stat(e->burst[1], n == "rt_packets");
    return AERO_OK;
  }
  v = n == "viterbi_jobs" ? e->retired_jobs : (n == "frames" ? e->retired_frames : e->retired_su_ok);
  for (auto &g : e->groups) {
    if (!g) continue;
    if (n == "viterbi_jobs")
      v += g->st_jobs.load();
    else if (n == "frames")
      v += g->st_frames.load();
    else
      v += g->st_su_ok.load();
  }
  *value = v;
  return AERO_OK;
}

int aero_channel_stat(aero_engine *e, int ch, const char *name, int64_t *value) {
  if (!e || !name || !value) return AERO_E_INVALID;
  const std::string n(name);
  if (route_burst(e, ch) >= 0) {  // the hunter is disabled in burst mode (decode/decode.cpp:175)
    if (n != "hunter_scans" && n != "freq_center") return AERO_E_INVALID;
    *value = 0;
    return AERO_OK;
  }
  int c;
  Group *g = route(e, ch, c);
  if (!g) return AERO_E_INVALID;
  HIPCHK(hipSetDevice(e->device));
  if (int rc = flush_pending_init(g)) return rc;
  if (n == "hunter_scans") {
    int v = 0;
    HIPCHK(hipMemcpyAsync(g->pin_stat, g->S.is + (size_t)IS_HUNT_SCANS * g->C + c, sizeof(int),
                          hipMemcpyDeviceToHost, g->st));
    HIPCHK(hipStreamSynchronize(g->st));
    memcpy(&v, g->pin_stat, sizeof v);
    *value = v;
  } else if (n == "freq_center") {
    double v = 0;
    HIPCHK(hipMemcpyAsync(g->pin_stat, g->S.ds + (size_t)DS_MC_FREQ * g->C + c, sizeof(double),
                          hipMemcpyDeviceToHost, g->st));
    HIPCHK(hipStreamSynchronize(g->st));
    memcpy(&v, g->pin_stat, sizeof v);
    *value = (int64_t)v;
  } else {
    return AERO_E_INVALID;
  }
  return AERO_OK;
}

int aero_channel_get_events(aero_engine *e, int ch, aero_channel_events *out) {
  if (!e || !out) return AERO_E_INVALID;
  memset(out, 0, sizeof *out);
  BurstGroup *bg;
  const int b = route_burst(e, ch, &bg);
  HIPCHK(hipSetDevice(e->device));
  if (b >= 0) return burst_dcd_edges(bg, b, &out->dcd_edges);
  int c;
  Group *g = route(e, ch, c);
  if (!g) return AERO_E_INVALID;
  if (int rc = flush_pending_init(g)) return rc;
  // two ints and eight doubles into pinned staging, one wait
  int *pi = reinterpret_cast<int *>(g->pin_stat);
  double *pd = reinterpret_cast<double *>(g->pin_stat) + 1;
  HIPCHK(hipMemcpyAsync(pi, g->S.is + (size_t)IS_DCD_EDGES * g->C + c, sizeof(int), hipMemcpyDeviceToHost, g->st));
  HIPCHK(hipMemcpyAsync(pi + 1, g->S.is + (size_t)IS_HUNT_STEPS * g->C + c, sizeof(int), hipMemcpyDeviceToHost,
                        g->st));
  for (int k = 0; k < 8; k++)
    HIPCHK(hipMemcpyAsync(pd + k, g->S.ds + (size_t)(DS_HUNT_FC0 + k) * g->C + c, sizeof(double),
                          hipMemcpyDeviceToHost, g->st));
  HIPCHK(hipStreamSynchronize(g->st));
  out->dcd_edges = pi[0];
  out->hunter_steps = pi[1];
  for (int k = 0; k < 8; k++) out->hunter_fc[k] = pd[k];
  if (g->mode == MODE_C8400) {  // DecodeC's datacd follows the SU CRCs only (host, process_slot)
    host_wait(e);
    out->dcd_edges = g->c_edges[c];
  }
  return AERO_OK;
}

uint64_t aero_samples_processed(aero_engine *e) {
  uint64_t s = 0;
  if (e) {
    for (auto &g : e->groups)
      if (g) s += g->processed;
    for (BurstGroup *b : e->burst) s += burst_processed(b);
  }
  return s;
}

int aero_sync(aero_engine *e) {
  if (!e) return AERO_E_INVALID;
  for (BurstGroup *b : e->burst)
    if (b)
      if (int rc = burst_sync(b)) return rc;
  for (auto &g : e->groups)
    if (g) {
      int rc = drain_group(g.get());
      if (rc) return rc;
    }
  host_wait(e);
  return AERO_OK;
}

int aero_device_math(aero_engine *e, int fn, const double *x, const double *y, double *out, size_t n) {
  if (!e || !x || !y || !out) return AERO_E_INVALID;
  HIPCHK(hipSetDevice(e->device));
  hipStream_t st = nullptr;
  double *d = nullptr;
  HIPCHK(hipMalloc(&d, 3 * n * sizeof(double) + 64));
  HIPCHK(hipMemcpy(d, x, n * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d + n, y, n * 8, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(math_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, fn, d, d + n, d + 2 * n, n);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(st));
  HIPCHK(hipMemcpy(out, d + 2 * n, n * 8, hipMemcpyDeviceToHost));
  HIPCHK(hipFree(d));
  return AERO_OK;
}

}  // extern "C"

// aero_chan_feed's entry into the engine (engine_internal.h)
int aero_engine_feed_dev(aero_engine *e, int nitems, const int *ch, const int16_t *const *src, const size_t *n,
                         const uint32_t *fs, hipEvent_t ready, hipStream_t producer) {
  if (!e || nitems < 0 || (nitems && (!ch || !src || !n || !fs))) return AERO_E_INVALID;
  HIPCHK(hipSetDevice(e->device));
  // per group (gid; a rate change below may add a generic-rate group)
  std::vector<std::vector<std::pair<int, std::pair<const int16_t *, size_t>>>> per(e->groups.size());
  std::vector<uint8_t> queued(e->chmap.size(), 0);  // engine channels with an item in per[]
  auto feed_queued = [&]() -> int {
    for (size_t m = 0; m < per.size(); m++)
      if (!per[m].empty()) {
        if (int rc = feed_group(e->groups[m].get(), per[m], ready, producer)) return rc;
        per[m].clear();
      }
    std::fill(queued.begin(), queued.end(), 0);
    return AERO_OK;
  };
  for (int i = 0; i < nitems; i++) {
    if (!n[i]) continue;
    BurstGroup *bg;
    const int b = route_burst(e, ch[i], &bg);
    if (b >= 0) {  // burst channels keep one message per call (synchronous copy)
      HIPCHK(hipEventSynchronize(ready));
      if (int rc = push_burst(e, bg, b, src[i], n[i], true)) return rc;
      continue;
    }
    int c, rc;
    {
      // a rate change of a channel that already has an item of this call
      // queued: those items go in first, at the old rate (messages are
      // handled in order, MskDemodulator::dataReceived), then it moves
      Group *g0 = route(e, ch[i], c);
      if (g0 && g0->mode != MODE_OQPSK && fs[i] != (uint32_t)g0->g.fs && queued[ch[i]])
        if (int rc2 = feed_queued()) return rc2;
    }
    Group *g = route_rate(e, ch[i], fs[i], c, rc);
    if (rc) return rc;
    if (!g || !src[i]) return AERO_E_INVALID;
    if (per.size() < e->groups.size()) per.resize(e->groups.size());
    per[g->gid].push_back({c, {src[i], n[i]}});
    queued[ch[i]] = 1;
  }
  return feed_queued();
}

// diagnostic builds (AERO_X_STAMPS): the demod's per-section cycle totals
// (loop control, loads+FIR+AGC, hypot+clip, timer, instant+NCO+ring, event
// step, samples) of wave 0; zeros in the product build
extern "C" void aero_x_demod_stamps(unsigned long long *out7) { demod_read_stamps(out7); }
// the coarse kernel's per-section cycle totals over every hop's wave 0
// (9 sections in slots 0-8, the hop count in slot 11)
extern "C" void aero_x_coarse_stamps(unsigned long long *out12) { coarse_read_stamps(out12); }
// the Viterbi kernel's per-section cycle totals over every job (3 sections + job count)
extern "C" void aero_x_viterbi_stamps(unsigned long long *out4) { viterbi_read_stamps(out4); }
// the burst OQPSK demod's per-section cycle totals (AERO_X_BSTAMPS build; burst.hip)
extern "C" void aero_x_burst_stamps(unsigned long long *out16) { burst_read_stamps(out16); }

// host check (tests/test_abi.py): the constants a generic-rate MSK group
// would run with at sample rate fs (msk_gen_consts); iout: sps, d8_old,
// d8_new, start, stop, ilo, ihi, epb, d8_len; dout: fs, sr_b0, sr_b2, sr_a1,
// sr_a2, ee, d8w, d8omw.  AERO_E_RATE for a rate the engine does not serve.
extern "C" int aero_x_msk_rate_consts(int fs, int *iout, double *dout) {
  MskGen m;
  if (!msk_gen_consts(fs, m)) return AERO_E_RATE;
  const int iv[9] = {m.sps, m.d8_old, m.d8_new, m.start, m.stop, m.ilo, m.ihi, m.epb, msk_geom(600, fs).d8_len};
  const double dv[8] = {m.fs, m.sr_b0, m.sr_b2, m.sr_a1, m.sr_a2, m.ee, m.d8w, m.d8omw};
  for (int k = 0; k < 9; k++) iout[k] = iv[k];
  for (int k = 0; k < 8; k++) dout[k] = dv[k];
  return AERO_OK;
}
