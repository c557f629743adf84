/*
 * chan.hip — aero-publish's channeliser on gfx950 (include/aero_chan.h).
 *
 * Publisher::demodData (publish/publisher.cpp:285-306) feeds each CF32 read to
 * the main VFOs; vfo::process (publish/vfo.cpp:154-186) mixes with a 1-second
 * FP32 oscillator queue, half-band decimates k times, hands the result to its
 * sub-VFOs, and each sub-VFO does the same and then USB-demodulates
 * (usb_demod / usb_decimdemod, vfo.cpp:188-258) into int16 audio.
 *
 * Every stage is an elementwise map or a FIR over a stream whose only carried
 * state is a short history, so each runs as one data-parallel launch over all
 * batched reads and all VFOs at once (bit-exact with the sequential code):
 *   mix     out[n] = queue[n] * x[n]                      Oscillator
 *   hb      y[j]   = 11-tap half-band over e[2j-10 .. 2j] HalfBandDecimator
 *   late    w[t]   = N-tap low-pass over z[t*L-N .. t*L-1] fir_decI/Q (1 in 5/6)
 *   usb     u[t]   = w.re[t-62] - hilbert125(w.im)[t]      DelayThing + FIRHilbert
 *   usbfir  y[t]   = N-tap low-pass over u[t-N .. t-1]     fir_usb
 * The half-band's per-read queue copy-back keeps the slots one early
 * (publish/dsp.cpp:163-172): read b's history is read b-1's samples
 * L-12 .. L-2, which hb_kernel gathers directly, so batched reads need no
 * sequential carry.  FIR histories cross batches through the first slots of
 * each stream buffer ("ext" buffers), shifted by shift_kernel after a batch.
 * The only recurrence, the optional DC removal (publisher.cpp:292-296), runs
 * in one lane per arm.
 *
 * These kernels are HBM/launch bound (a few flops per byte); the grid spans
 * reads x tiles x VFOs so one launch per stage level fills the chip.
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <memory>
#include <vector>

#include "../../include/aero_chan.h"
#include "engine_internal.h"
#include "tables_host.h"

using aero::host_pub_hilbert;
using aero::host_pub_low_pass;
using aero::host_pub_osc;
using aero::host_pub_osc_len;

namespace {

#define CHK(x)                                                                         \
  do {                                                                                 \
    hipError_t err__ = (x);                                                            \
    if (err__ != hipSuccess) {                                                         \
      fprintf(stderr, "aero_chan: %s failed: %s\n", #x, hipGetErrorString(err__));     \
      return AERO_E_HIP;                                                               \
    }                                                                                  \
  } while (0)

constexpr int HIL_LEN = 125, HIL_H = HIL_LEN - 1, DLY = (HIL_LEN - 1) / 2;  // vfo.cpp:111-112
constexpr int HB_TILE = 256, MAX_STAGES = 8;                                // hdecimator[8] (vfo.h:63)

// ------------------------------------------------------------------ device
__device__ __forceinline__ float2 cmulf(float2 a, float2 b) {  // GCC's complex<float> product
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}

// Oscillator::_vector after n ticks (oscillator.cpp:24-38): the constructor
// leaves the last queue entry, tick k reads queue[k % length]
__device__ __forceinline__ float2 osc_at(const float2 *q, int len, long long n) {
  return n == 0 ? q[len - 1] : q[n % len];
}

// FIRUpdateAndProcessHalfBandQueue, 11 taps (dsp.cpp:141-146), in its order
__device__ __forceinline__ float hb11(float a0, float a2, float a4, float a5, float a6, float a8, float a10) {
  const float p0 = 0.0060431029837374152f, p2 = -0.049372515458761493f, p4 = 0.29332944952052842f, p5 = 0.5f;
  return 0.0f + (((p0 * (a0 + a10) + p2 * (a2 + a8)) + p4 * (a4 + a6)) + p5 * a5);
}

// double -> int as x86-64 g++ compiles the reference's implicit conversions
// to short / signed char: cvtts?2si (0x80000000 when out of range), low bits
__device__ __forceinline__ int cvtt(double d) {
  return (d > -2147483649.0 && d < 2147483648.0) ? (int)d : (int)0x80000000;
}

struct HbJob {  // one half-band stage (the first one with the NCO mix) of one VFO
  const float2 *in;    // nblk reads of L samples
  float2 *out;         // nblk reads of L/2
  const float2 *hist;  // e[-11..-1] of the first read (already mixed)
  float2 *hist_out;    // the same for the next batch
  const float2 *osc;   // NCO queue, nullptr after the first stage
  long long n0;        // NCO ticks before in[0]
  int osc_len, L;
};

__device__ __forceinline__ float2 hb_in(const HbJob &j, int b, int t) {
  long long i;
  if (t >= 0)
    i = (long long)b * j.L + t;
  else if (b > 0)
    i = (long long)b * j.L - 1 + t;  // previous read's samples L-12 .. L-2
  else
    return j.hist[11 + t];
  float2 v = j.in[i];
  if (j.osc) v = cmulf(osc_at(j.osc, j.osc_len, j.n0 + i), v);
  return v;
}

__global__ __launch_bounds__(HB_TILE) void hb_kernel(const HbJob *jobs, int nblk) {
  const HbJob j = jobs[blockIdx.z];
  const int Lo = j.L >> 1, b = blockIdx.y, j0 = blockIdx.x * HB_TILE;
  if (j0 >= Lo) return;  // uniform per workgroup
  __shared__ float2 e[2 * HB_TILE + 10];
  const int tb = 2 * j0 - 10;
  for (int q = threadIdx.x; q < 2 * HB_TILE + 10; q += HB_TILE) {
    const int t = tb + q;
    e[q] = t < j.L ? hb_in(j, b, t) : make_float2(0.f, 0.f);
  }
  __syncthreads();
  const int o = j0 + threadIdx.x;
  if (o < Lo) {
    const float2 *q = e + 2 * threadIdx.x;  // q[m] = e[2o - 10 + m]
    j.out[(size_t)b * Lo + o] = make_float2(hb11(q[0].x, q[2].x, q[4].x, q[5].x, q[6].x, q[8].x, q[10].x),
                                            hb11(q[0].y, q[2].y, q[4].y, q[5].y, q[6].y, q[8].y, q[10].y));
  }
  if (b == nblk - 1 && blockIdx.x == 0 && threadIdx.x < 11) j.hist_out[threadIdx.x] = hb_in(j, b, j.L - 12 + threadIdx.x);
}

struct MixJob {
  const float2 *in;
  float2 *out;
  const float2 *osc;
  long long n0, n;
  int osc_len;
};

__global__ __launch_bounds__(256) void mix_kernel(const MixJob *jobs) {
  const MixJob j = jobs[blockIdx.y];
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < j.n; i += (long long)gridDim.x * 256)
    j.out[i] = cmulf(osc_at(j.osc, j.osc_len, j.n0 + i), j.in[i]);
}

// demodData's DC removal: avept = avept*(1-1e-6) + 1e-6*x; x -= avept
// (publisher.cpp:292-296), a first-order recurrence per arm, one lane each
__global__ __launch_bounds__(64) void dc_kernel(float2 *x, long long n, float2 *avept) {
  const int lane = threadIdx.x;
  if (lane >= 2) return;
  float *p = reinterpret_cast<float *>(x) + lane;
  float a = lane ? avept->y : avept->x;
#pragma unroll 8
  for (long long i = 0; i < n; i++) {
    const float c = p[2 * i];
    a = a * (1.0f - 0.000001f) + 0.000001f * c;
    p[2 * i] = c - a;
  }
  if (lane)
    avept->y = a;
  else
    avept->x = a;
}

struct UsbJob {
  const float2 *zext;      // late: nlate history + this batch's z
  const float *late_taps;
  int nlate, late;
  float2 *wext;            // HIL_H history + this batch's w
  const float *hil;        // 125 Hilbert taps
  float *uext;             // nusb history + this batch's u
  const float *usb_taps;
  int nusb, n;             // outputs this batch
  int16_t *out;
  float gain;
};

// fir_decI/Q of usb_decimdemod (vfo.cpp:230-256): every input enters the ring,
// the output at t*late covers z[t*late - N .. t*late - 1]
__global__ __launch_bounds__(256) void late_kernel(const UsbJob *jobs) {
  const UsbJob j = jobs[blockIdx.y];
  if (!j.late) return;
  for (int t = blockIdx.x * 256 + threadIdx.x; t < j.n; t += gridDim.x * 256) {
    const float2 *z = j.zext + (size_t)t * j.late;
    float re = 0.f, im = 0.f;
    for (int i = 0; i < j.nlate; i++) {
      const float p = j.late_taps[i];
      re += p * z[i].x;
      im += p * z[i].y;
    }
    j.wext[HIL_H + t] = make_float2(re, im);
  }
}

// usb = delayT(re) - philbert(im) (vfo.cpp:199-212, 234-235), * gain * 32768
__global__ __launch_bounds__(256) void usb_kernel(const UsbJob *jobs) {
  const UsbJob j = jobs[blockIdx.y];
  for (int t = blockIdx.x * 256 + threadIdx.x; t < j.n; t += gridDim.x * 256) {
    const float2 *w = j.wext + t;  // w[i] = sample t - 124 + i
    float h = 0.f;
    for (int i = 0; i < HIL_LEN; i++) h += j.hil[i] * w[i].y;
    const float u = w[HIL_H - DLY].x - h;
    if (j.nusb)
      j.uext[j.nusb + t] = u;
    else
      j.out[t] = (int16_t)cvtt((double)(u * j.gain) * 32768.0);
  }
}

// fir_usb (vfo.cpp:201-204, 237-239): y[t] over u[t - N .. t - 1]
__global__ __launch_bounds__(256) void usbfir_kernel(const UsbJob *jobs) {
  const UsbJob j = jobs[blockIdx.y];
  if (!j.nusb) return;
  for (int t = blockIdx.x * 256 + threadIdx.x; t < j.n; t += gridDim.x * 256) {
    const float *u = j.uext + t;
    float y = 0.f;
    for (int i = 0; i < j.nusb; i++) y += j.usb_taps[i] * u[i];
    j.out[t] = (int16_t)cvtt((double)(y * j.gain) * 32768.0);
  }
}

struct IqJob {
  const float2 *x;
  int8_t *out;
  long long n;
  float scalecomp;
};

// vfo::compress, style 1 (vfo.cpp:262-274): the top nibble of each arm
__global__ __launch_bounds__(256) void compress_kernel(const IqJob *jobs) {
  const IqJob j = jobs[blockIdx.y];
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < j.n; i += (long long)gridDim.x * 256) {
    const float2 c = j.x[i];
    const int re = (int8_t)cvtt((c.x / j.scalecomp) * 128.0f);
    const int im = (int8_t)cvtt((c.y / j.scalecomp) * 128.0f);
    j.out[i] = (int8_t)((re & 0xF0) | ((im & 0xF0) >> 4));
  }
}

struct ShiftJob {  // base[0..h) = base[len .. len + h), len >= h (no overlap)
  float *base;
  long long len;
  int h;
};

__global__ __launch_bounds__(256) void shift_kernel(const ShiftJob *jobs) {
  const ShiftJob s = jobs[blockIdx.y];
  for (int i = threadIdx.x; i < s.h; i += 256) s.base[i] = s.base[s.len + i];
}

// ------------------------------------------------------------------ host
struct Vfo {
  bool main = false, active = false, has_subs = false, publish = false;
  int parent = -1;
  int fs = 0, k = 0, late = 0, out_rate = 0, filterbw = 0, scalecomp = 1;
  int spb = 0;  // input samples per read
  int S = 0;    // output samples per read
  double mixer = 0;
  float gain = 0;
  float2 *osc = nullptr;
  int osc_len = 0;
  long long nmix = 0;
  float2 *hist[2] = {nullptr, nullptr};  // [parity][stage][11]
  float2 *stage[MAX_STAGES] = {};
  float2 *chain = nullptr;  // output of mix + half-bands
  float2 *zext = nullptr, *wext = nullptr;
  float *uext = nullptr, *late_taps = nullptr, *usb_taps = nullptr, *hil = nullptr;
  int nlate = 0, nusb = 0;
  int16_t *out16 = nullptr;
  int8_t *iq = nullptr;
  std::vector<int16_t> host_out;
  std::vector<int8_t> host_iq;
};

}  // namespace

struct aero_chan {
  aero_chan_cfg cfg{};
  int B = 0, bufsplit = 4;
  std::vector<Vfo> mains, subs;
  float2 *in = nullptr, *avept = nullptr;
  int pending = 0, last_nblk = 0, parity = 0;
  hipStream_t st = nullptr;
  hipEvent_t ev_jobs = nullptr, ev_pin = nullptr, ev_in = nullptr, ev_out = nullptr;
  std::vector<void *> dmem;
  char *d_jobs = nullptr, *h_jobs = nullptr;
  size_t jobs_cap = 0;
  float *pin_in = nullptr;
};

namespace {

template <class T>
int dalloc(aero_chan *c, T *&p, size_t n) {
  void *q = nullptr;
  const size_t bytes = std::max<size_t>(n, 1) * sizeof(T);
  if (hipMalloc(&q, bytes) != hipSuccess) return AERO_E_NOMEM;
  c->dmem.push_back(q);
  CHK(hipMemset(q, 0, bytes));
  p = reinterpret_cast<T *>(q);
  return AERO_OK;
}

int upload(aero_chan *c, float *&p, const std::vector<float> &v) {
  if (int rc = dalloc(c, p, v.size())) return rc;
  CHK(hipMemcpy(p, v.data(), v.size() * sizeof(float), hipMemcpyHostToDevice));
  return AERO_OK;
}

int vfo_alloc(aero_chan *c, Vfo &v) {
  const size_t T = (size_t)c->cfg.max_blocks;
  {
    std::vector<float> q(2 * (size_t)host_pub_osc_len(v.fs));
    host_pub_osc(v.fs, v.mixer, q.data());
    float *qd;
    if (int rc = upload(c, qd, q)) return rc;
    v.osc = reinterpret_cast<float2 *>(qd);
    v.osc_len = (int)(q.size() / 2);
  }
  for (int p = 0; p < 2; p++)
    if (int rc = dalloc(c, v.hist[p], (size_t)MAX_STAGES * 11)) return rc;
  const int Lk = v.spb >> v.k;
  if (v.main) {
    if (int rc = dalloc(c, v.chain, T * Lk)) return rc;
    if (v.publish && !v.has_subs)
      if (int rc = dalloc(c, v.iq, T * Lk)) return rc;
  } else {
    std::vector<float> hil(HIL_LEN);
    host_pub_hilbert(HIL_LEN, v.S, hil.data());  // FIRHilbert(125, samplesOut) (vfo.cpp:112)
    if (int rc = upload(c, v.hil, hil)) return rc;
    if (int rc = dalloc(c, v.wext, HIL_H + T * v.S)) return rc;
    std::vector<float> taps(4096);
    if (v.late) {
      const int tr = v.out_rate;  // targetRate after the late division (vfo.cpp:71-79)
      v.nlate = host_pub_low_pass(2, tr * v.late, tr / 2, (double)tr / (v.late - 1), taps.data(), 4096);
      if (v.nlate <= 0 || v.nlate > Lk) return AERO_E_INVALID;
      taps.resize(v.nlate);
      if (int rc = upload(c, v.late_taps, taps)) return rc;
      if (int rc = dalloc(c, v.zext, v.nlate + T * Lk)) return rc;
      v.chain = v.zext + v.nlate;
    } else {
      v.chain = v.wext + HIL_H;
    }
    if (v.filterbw > 0) {  // vfo.cpp:92-102
      taps.assign(4096, 0.f);
      v.nusb = host_pub_low_pass(2, v.out_rate, v.filterbw, (double)v.filterbw / 4, taps.data(), 4096);
      if (v.nusb <= 0 || v.nusb > v.S) return AERO_E_INVALID;
      taps.resize(v.nusb);
      if (int rc = upload(c, v.usb_taps, taps)) return rc;
      if (int rc = dalloc(c, v.uext, v.nusb + T * v.S)) return rc;
    }
    if (int rc = dalloc(c, v.out16, T * v.S)) return rc;
  }
  for (int s = 0; s + 1 < v.k; s++)
    if (int rc = dalloc(c, v.stage[s], T * (size_t)(v.spb >> (s + 1)))) return rc;
  if (v.k > 0) v.stage[v.k - 1] = v.chain;
  return AERO_OK;
}

// a half-band chain of k stages over reads of L samples: every stage input even and >= 12
bool chain_ok(int L, int k) {
  for (int s = 0; s < k; s++) {
    const int Ls = L >> s;
    if (Ls < 12 || (Ls & 1) || (Ls << s) != L) return false;
  }
  return true;
}

size_t align16(size_t x) { return (x + 15) & ~size_t(15); }

int run_impl(aero_chan *c) {
  const int nb = c->pending;
  if (!nb) return AERO_OK;
  const int p = c->parity;
  std::vector<HbJob> hb[2][MAX_STAGES];
  std::vector<MixJob> mix[2];
  std::vector<UsbJob> usb;
  std::vector<IqJob> iq;
  std::vector<ShiftJob> sh;
  auto chain_jobs = [&](Vfo &v, const float2 *in, int side) {
    if (v.k == 0) {
      mix[side].push_back({in, v.chain, v.osc, v.nmix, (long long)nb * v.spb, v.osc_len});
      return;
    }
    for (int s = 0; s < v.k; s++) {
      HbJob j;
      j.in = s == 0 ? in : v.stage[s - 1];
      j.out = v.stage[s];
      j.hist = v.hist[p] + s * 11;
      j.hist_out = v.hist[p ^ 1] + s * 11;
      j.osc = s == 0 ? v.osc : nullptr;
      j.n0 = v.nmix;
      j.osc_len = v.osc_len;
      j.L = v.spb >> s;
      hb[side][s].push_back(j);
    }
  };
  for (auto &m : c->mains)
    if (m.active) chain_jobs(m, c->in, 0);
  for (auto &s : c->subs) {
    if (!s.active) continue;
    chain_jobs(s, c->mains[s.parent].chain, 1);
    UsbJob u{};
    u.zext = s.zext;
    u.late_taps = s.late_taps;
    u.nlate = s.nlate;
    u.late = s.late;
    u.wext = s.wext;
    u.hil = s.hil;
    u.uext = s.uext;
    u.usb_taps = s.usb_taps;
    u.nusb = s.nusb;
    u.n = nb * s.S;
    u.out = s.out16;
    u.gain = s.gain;
    usb.push_back(u);
    if (s.late) sh.push_back({reinterpret_cast<float *>(s.zext), 2LL * nb * (s.spb >> s.k), 2 * s.nlate});
    sh.push_back({reinterpret_cast<float *>(s.wext), 2LL * nb * s.S, 2 * HIL_H});
    if (s.nusb) sh.push_back({s.uext, (long long)nb * s.S, s.nusb});
  }
  for (auto &m : c->mains)
    if (m.active && m.iq) iq.push_back({m.chain, m.iq, (long long)nb * (m.spb >> m.k), (float)m.scalecomp});

  // one job blob per batch: pinned staging -> device
  size_t off = 0;
  std::vector<std::pair<size_t, size_t>> place;  // (offset, bytes) in push order
  auto add = [&](const void *src, size_t bytes) {
    place.push_back({off, bytes});
    off = align16(off + bytes);
    (void)src;
  };
  for (int sd = 0; sd < 2; sd++) {
    add(mix[sd].data(), mix[sd].size() * sizeof(MixJob));
    for (int s = 0; s < MAX_STAGES; s++) add(hb[sd][s].data(), hb[sd][s].size() * sizeof(HbJob));
  }
  add(usb.data(), usb.size() * sizeof(UsbJob));
  add(iq.data(), iq.size() * sizeof(IqJob));
  add(sh.data(), sh.size() * sizeof(ShiftJob));
  if (off > c->jobs_cap) return AERO_E_INVALID;  // sized at create
  CHK(hipEventSynchronize(c->ev_jobs));
  {
    size_t k = 0;
    auto put = [&](const void *src) {
      if (place[k].second) memcpy(c->h_jobs + place[k].first, src, place[k].second);
      k++;
    };
    for (int sd = 0; sd < 2; sd++) {
      put(mix[sd].data());
      for (int s = 0; s < MAX_STAGES; s++) put(hb[sd][s].data());
    }
    put(usb.data());
    put(iq.data());
    put(sh.data());
  }
  CHK(hipMemcpyAsync(c->d_jobs, c->h_jobs, off, hipMemcpyHostToDevice, c->st));
  CHK(hipEventRecord(c->ev_jobs, c->st));
  size_t k = 0;
  auto dptr = [&](size_t i) { return c->d_jobs + place[i].first; };

  if (c->cfg.correct_dc_bias)
    hipLaunchKernelGGL(dc_kernel, dim3(1), dim3(64), 0, c->st, c->in, (long long)nb * c->B, c->avept);
  for (int sd = 0; sd < 2; sd++) {
    if (!mix[sd].empty()) {
      long long mx = 0;
      for (auto &j : mix[sd]) mx = std::max(mx, j.n);
      const int gx = (int)std::min<long long>((mx + 255) / 256, 4096);
      hipLaunchKernelGGL(mix_kernel, dim3(gx, (unsigned)mix[sd].size()), dim3(256), 0, c->st,
                         reinterpret_cast<const MixJob *>(dptr(k)));
    }
    k++;
    for (int s = 0; s < MAX_STAGES; s++, k++) {
      if (hb[sd][s].empty()) continue;
      int tiles = 0;
      for (auto &j : hb[sd][s]) tiles = std::max(tiles, ((j.L >> 1) + HB_TILE - 1) / HB_TILE);
      hipLaunchKernelGGL(hb_kernel, dim3(tiles, nb, (unsigned)hb[sd][s].size()), dim3(HB_TILE), 0, c->st,
                         reinterpret_cast<const HbJob *>(dptr(k)), nb);
    }
  }
  if (!usb.empty()) {
    int mx = 0;
    bool any_late = false, any_fir = false;
    for (auto &u : usb) {
      mx = std::max(mx, u.n);
      any_late |= u.late != 0;
      any_fir |= u.nusb != 0;
    }
    const dim3 g(std::min((mx + 255) / 256, 1024), (unsigned)usb.size());
    const UsbJob *uj = reinterpret_cast<const UsbJob *>(dptr(k));
    if (any_late) hipLaunchKernelGGL(late_kernel, g, dim3(256), 0, c->st, uj);
    hipLaunchKernelGGL(usb_kernel, g, dim3(256), 0, c->st, uj);
    if (any_fir) hipLaunchKernelGGL(usbfir_kernel, g, dim3(256), 0, c->st, uj);
  }
  k++;
  if (!iq.empty()) {
    long long mx = 0;
    for (auto &j : iq) mx = std::max(mx, j.n);
    hipLaunchKernelGGL(compress_kernel, dim3((unsigned)std::min<long long>((mx + 255) / 256, 4096), (unsigned)iq.size()),
                       dim3(256), 0, c->st, reinterpret_cast<const IqJob *>(dptr(k)));
  }
  k++;
  if (!sh.empty())
    hipLaunchKernelGGL(shift_kernel, dim3(1, (unsigned)sh.size()), dim3(256), 0, c->st,
                       reinterpret_cast<const ShiftJob *>(dptr(k)));
  CHK(hipGetLastError());
  for (auto &m : c->mains)
    if (m.active) m.nmix += (long long)nb * m.spb;
  for (auto &s : c->subs)
    if (s.active) s.nmix += (long long)nb * s.spb;
  c->parity ^= 1;
  c->last_nblk = nb;
  c->pending = 0;
  if (c->cfg.flags & AERO_CHAN_F_HOST_OUT) {
    CHK(hipStreamSynchronize(c->st));
    for (auto &s : c->subs) {
      if (!s.active) continue;
      const size_t n = (size_t)nb * s.S, o = s.host_out.size();
      s.host_out.resize(o + n);
      CHK(hipMemcpy(s.host_out.data() + o, s.out16, n * sizeof(int16_t), hipMemcpyDeviceToHost));
    }
    for (auto &m : c->mains) {
      if (!m.active || !m.iq) continue;
      const size_t n = (size_t)nb * (m.spb >> m.k), o = m.host_iq.size();
      m.host_iq.resize(o + n);
      CHK(hipMemcpy(m.host_iq.data() + o, m.iq, n, hipMemcpyDeviceToHost));
    }
  }
  return AERO_OK;
}

template <class T>
int pop_vec(std::vector<T> &v, T *dst, size_t cap, size_t *n) {
  const size_t k = std::min(cap, v.size());
  if (dst && k) memcpy(dst, v.data(), k * sizeof(T));
  if (n) *n = k;
  v.erase(v.begin(), v.begin() + k);
  return AERO_OK;
}

void destroy_impl(aero_chan *c) {
  if (c->st) (void)hipStreamSynchronize(c->st);
  for (void *p : c->dmem) (void)hipFree(p);
  if (c->d_jobs) (void)hipFree(c->d_jobs);
  if (c->h_jobs) (void)hipHostFree(c->h_jobs);
  if (c->pin_in) (void)hipHostFree(c->pin_in);
  if (c->ev_jobs) (void)hipEventDestroy(c->ev_jobs);
  if (c->ev_pin) (void)hipEventDestroy(c->ev_pin);
  if (c->ev_in) (void)hipEventDestroy(c->ev_in);
  if (c->ev_out) (void)hipEventDestroy(c->ev_out);
  if (c->st) (void)hipStreamDestroy(c->st);
}

}  // namespace

extern "C" {

int aero_chan_create(const aero_chan_cfg *cfg, const aero_chan_main *mains, int nmain, const aero_chan_vfo *vfos,
                     int nvfo, aero_chan **out) {
  if (!cfg || !out || nmain < 0 || nmain > 3 || nvfo < 0 || (nmain && !mains) || (nvfo && !vfos) ||
      cfg->max_blocks <= 0)
    return AERO_E_INVALID;
  *out = nullptr;
  const int Fs = cfg->sample_rate;
  if (Fs != 288000 && Fs != 1536000 && Fs != 1920000) return AERO_E_INVALID;  // publisher.h:32
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || cfg->device < 0 || cfg->device >= ndev) return AERO_E_NOGPU;
  CHK(hipSetDevice(cfg->device));
  std::unique_ptr<aero_chan, void (*)(aero_chan *)> c(new aero_chan(), [](aero_chan *p) {
    destroy_impl(p);
    delete p;
  });
  c->cfg = *cfg;
  // four reads a second unless 2*Fs/4 is not a multiple of 512 (publisher.cpp:92-100)
  int buflen;
  if (double((int((2 * Fs) / 4)) % 512) > 0) {
    buflen = int((2 * Fs) / 5);
    c->bufsplit = 5;
  } else {
    buflen = int((2 * Fs) / 4);
  }
  c->B = buflen / 2;
  for (int i = 0; i < nmain; i++) {  // publisher.cpp:115-148
    Vfo v;
    v.main = true;
    v.fs = Fs;
    if (mains[i].out_rate <= 0) return AERO_E_INVALID;
    v.k = Fs / mains[i].out_rate == 1 ? 0 : int(log2(Fs / mains[i].out_rate));
    v.mixer = cfg->center_frequency - mains[i].frequency;
    v.scalecomp = mains[i].compress_scale > 0 ? mains[i].compress_scale : 1;
    v.publish = mains[i].publish != 0;
    v.spb = c->B;
    v.out_rate = (int)(Fs / (pow(2, v.k)));
    v.S = (int)(v.spb / (pow(2, v.k)));
    if (v.k > MAX_STAGES || !chain_ok(v.spb, v.k)) return AERO_E_INVALID;
    c->mains.push_back(v);
  }
  for (int i = 0; i < nvfo; i++) {  // publisher.cpp:151-222
    const aero_chan_vfo &s = vfos[i];
    Vfo v;
    const int vfo_freq = s.frequency + cfg->mix_offset;
    int out_rate = s.out_rate;
    if (out_rate == 0 && s.data_rate > 0) out_rate = s.data_rate == 600 ? 12000 : (s.data_rate == 1200 ? 24000 : 48000);
    if (out_rate <= 0) return AERO_E_INVALID;
    int main_vfo_freq = 0, main_out = Fs, main_idx = -1;
    for (int a = 0; a < nmain; a++) {
      const int diff = (int)std::fabs((cfg->center_frequency - c->mains[a].mixer) - vfo_freq);
      if (diff < c->mains[a].out_rate) {
        main_idx = a;
        main_vfo_freq = (int)c->mains[a].mixer;
        main_out = c->mains[a].out_rate;
        break;
      }
    }
    if (main_idx < 0 && nmain > 0) return AERO_E_INVALID;  // would be fed another main VFO's stream
    int late = 0, k;
    if ((main_out / 48000) == 5) {
      k = int(log2(main_out / (5 * out_rate)));
      late = 5;
    } else if ((main_out / 48000) == 6) {
      k = int(log2(main_out / (6 * out_rate)));
      late = 6;
    } else {
      k = int(log2(Fs / out_rate)) - int(log2(Fs / main_out));
    }
    if (k < 0 || k > MAX_STAGES) return AERO_E_INVALID;
    v.k = k;
    v.late = late;
    v.filterbw = s.filter_bandwidth;
    v.gain = (float)s.gain / 100;
    v.mixer = (cfg->center_frequency - main_vfo_freq) - vfo_freq;
    v.fs = main_out;
    v.parent = main_idx;
    v.spb = main_out / c->bufsplit;
    int targetRate = (int)(v.fs / (pow(2, k)));
    int so = (int)(v.spb / (pow(2, k)));
    if (late) {
      targetRate = targetRate / late;
      so = so / late;
    }
    v.out_rate = targetRate;
    v.S = so;
    v.active = main_idx >= 0 && !s.skip;
    if (main_idx >= 0) {
      Vfo &m = c->mains[main_idx];
      m.has_subs = true;
      // the sub-VFO's read is exactly its main VFO's output read (vfo.cpp:122-126, 154-160)
      if (v.spb != m.S || !chain_ok(v.spb, k)) return AERO_E_INVALID;
      const int Lk = v.spb >> k;
      if (late && (Lk % late || Lk / late != so)) return AERO_E_INVALID;
      if (so < HIL_H) return AERO_E_INVALID;
    }
    c->subs.push_back(v);
  }
  for (auto &m : c->mains) m.active = m.publish && !m.has_subs;
  for (auto &s : c->subs)
    if (s.active) c->mains[s.parent].active = true;
  CHK(hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking));
  CHK(hipEventCreateWithFlags(&c->ev_jobs, hipEventDisableTiming));
  CHK(hipEventCreateWithFlags(&c->ev_pin, hipEventDisableTiming));
  CHK(hipEventCreateWithFlags(&c->ev_in, hipEventDisableTiming));
  CHK(hipEventCreateWithFlags(&c->ev_out, hipEventDisableTiming));
  if (int rc = dalloc(c.get(), c->in, (size_t)cfg->max_blocks * c->B)) return rc;
  if (int rc = dalloc(c.get(), c->avept, 1)) return rc;
  for (auto &m : c->mains)
    if (m.active)
      if (int rc = vfo_alloc(c.get(), m)) return rc;
  for (auto &s : c->subs)
    if (s.active)
      if (int rc = vfo_alloc(c.get(), s)) return rc;
  const size_t nv = c->mains.size() + c->subs.size() + 1;
  c->jobs_cap = 16 * 32 + nv * (MAX_STAGES * sizeof(HbJob) + sizeof(MixJob) + sizeof(UsbJob) + sizeof(IqJob) +
                                3 * sizeof(ShiftJob) + 16 * 16);
  if (hipMalloc(&c->d_jobs, c->jobs_cap) != hipSuccess) return AERO_E_NOMEM;
  if (hipHostMalloc(&c->h_jobs, c->jobs_cap) != hipSuccess) return AERO_E_NOMEM;
  CHK(hipDeviceSynchronize());
  *out = c.release();
  return AERO_OK;
}

void aero_chan_destroy(aero_chan *c) {
  if (!c) return;
  (void)hipSetDevice(c->cfg.device);
  destroy_impl(c);
  delete c;
}

int aero_chan_block_len(aero_chan *c, int *block_len) {
  if (!c || !block_len) return AERO_E_INVALID;
  *block_len = c->B;
  return AERO_OK;
}

int aero_chan_vfo_info(aero_chan *c, int v, int *info) {
  if (!c || !info || v < 0 || v >= (int)c->subs.size()) return AERO_E_INVALID;
  const Vfo &s = c->subs[v];
  info[0] = s.parent;
  info[1] = s.out_rate;
  info[2] = s.S;
  info[3] = s.k;
  info[4] = s.late;
  return AERO_OK;
}

int aero_chan_main_info(aero_chan *c, int m, int *info) {
  if (!c || !info || m < 0 || m >= (int)c->mains.size()) return AERO_E_INVALID;
  const Vfo &v = c->mains[m];
  info[0] = v.out_rate;
  info[1] = v.S;
  info[2] = v.k;
  return AERO_OK;
}

int aero_chan_push(aero_chan *c, const float *iq, size_t nblocks, int dev) {
  if (!c || (!iq && nblocks)) return AERO_E_INVALID;
  CHK(hipSetDevice(c->cfg.device));
  const size_t blk = (size_t)c->B * 2;  // floats per read
  // without host output an implicit batch would overwrite the previous
  // batch's device audio before aero_chan_feed / aero_chan_vfo_output read
  // it: refuse the push whole instead (with host output every batch is kept)
  if (!(c->cfg.flags & AERO_CHAN_F_HOST_OUT) && (size_t)c->pending + nblocks > (size_t)c->cfg.max_blocks)
    return AERO_E_FULL;
  if (dev && nblocks)
    if (int rc = check_dev_ptr(iq)) return rc;
  size_t done = 0;
  while (done < nblocks) {
    if (c->pending == c->cfg.max_blocks)
      if (int rc = run_impl(c)) return rc;
    const size_t nb = std::min<size_t>(nblocks - done, (size_t)(c->cfg.max_blocks - c->pending));
    float *dst = reinterpret_cast<float *>(c->in) + (size_t)c->pending * blk;
    const float *src = iq + done * blk;
    const size_t bytes = nb * blk * sizeof(float);
    if (dev) {
      CHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, c->st));
      CHK(hipEventRecord(c->ev_in, c->st));
      CHK(hipEventSynchronize(c->ev_in));  // the caller's buffer is free again
    } else {
      if (!c->pin_in) {
        if (hipHostMalloc(&c->pin_in, (size_t)c->cfg.max_blocks * blk * sizeof(float)) != hipSuccess) {
          c->pin_in = nullptr;
          return AERO_E_NOMEM;
        }
      }
      CHK(hipEventSynchronize(c->ev_pin));
      memcpy(c->pin_in, src, bytes);
      CHK(hipMemcpyAsync(dst, c->pin_in, bytes, hipMemcpyHostToDevice, c->st));
      CHK(hipEventRecord(c->ev_pin, c->st));
    }
    c->pending += (int)nb;
    done += nb;
  }
  return AERO_OK;
}

int aero_chan_run(aero_chan *c) {
  if (!c) return AERO_E_INVALID;
  CHK(hipSetDevice(c->cfg.device));
  return run_impl(c);
}

int aero_chan_sync(aero_chan *c) {
  if (!c) return AERO_E_INVALID;
  CHK(hipSetDevice(c->cfg.device));
  CHK(hipStreamSynchronize(c->st));
  return AERO_OK;
}

int aero_chan_vfo_output(aero_chan *c, int v, const int16_t **dptr, size_t *n) {
  if (!c || !dptr || !n || v < 0 || v >= (int)c->subs.size()) return AERO_E_INVALID;
  const Vfo &s = c->subs[v];
  *dptr = s.out16;
  *n = s.active ? (size_t)c->last_nblk * s.S : 0;
  return AERO_OK;
}

int aero_chan_pop_audio(aero_chan *c, int v, int16_t *dst, size_t cap, size_t *n) {
  if (!c || v < 0 || v >= (int)c->subs.size()) return AERO_E_INVALID;
  return pop_vec(c->subs[v].host_out, dst, cap, n);
}

int aero_chan_pop_iq(aero_chan *c, int m, int8_t *dst, size_t cap, size_t *n) {
  if (!c || m < 0 || m >= (int)c->mains.size()) return AERO_E_INVALID;
  return pop_vec(c->mains[m].host_iq, dst, cap, n);
}

int aero_chan_feed(aero_chan *c, aero_engine *e, const int *ch) {
  if (!c || !e || !ch) return AERO_E_INVALID;
  CHK(hipSetDevice(c->cfg.device));
  // one gather launch per channel kind, ordered after this batch's audio by
  // an event; the next batch waits for it on this stream (no host wait)
  std::vector<int> chs;
  std::vector<const int16_t *> src;
  std::vector<size_t> n;
  std::vector<uint32_t> fs;
  for (size_t v = 0; v < c->subs.size(); v++) {
    const Vfo &s = c->subs[v];
    if (ch[v] < 0 || !s.active || !c->last_nblk) continue;
    chs.push_back(ch[v]);
    src.push_back(s.out16);
    n.push_back((size_t)c->last_nblk * s.S);
    fs.push_back((uint32_t)s.out_rate);
  }
  if (chs.empty()) return AERO_OK;
  CHK(hipEventRecord(c->ev_out, c->st));
  return aero_engine_feed_dev(e, (int)chs.size(), chs.data(), src.data(), n.data(), fs.data(), c->ev_out, c->st);
}

}  // extern "C"
