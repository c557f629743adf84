/*
 * aero_engine.h — C ABI of the MI355X-native Aero demodulation engine.
 *
 * Drop-in boundary for aero-decode's per-VFO DSP chain.  In the reference
 * (airframesio/aero-cli, decode/) the boundary is a set of Qt signal/slot
 * edges wired in decode/decode.cpp:168-241; each entry point below names the
 * edge it replaces.  Plain pointers and sizes only; no torch/HIP types.
 *
 * Threading: one host thread per engine (the reference runs all DSP on the
 * Qt main thread); push/run/pop on one engine must be serialised by the
 * caller.  Ownership: the caller owns every buffer it passes; the engine
 * copies input before returning and copies output into caller arrays.
 * Errors: 0 = OK, negative = AERO_E_* (aero_strerror).
 */
#ifndef AERO_ENGINE_H
#define AERO_ENGINE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AERO_OK 0
#define AERO_E_INVALID (-1)    /* bad argument / unsupported bit rate      */
#define AERO_E_NOMEM (-2)      /* device or host allocation failed         */
#define AERO_E_HIP (-3)        /* HIP runtime error                        */
#define AERO_E_NOGPU (-4)      /* no gfx950 device / kernels not loadable  */
#define AERO_E_FULL (-5)       /* channel table or PCM ring full           */
#define AERO_E_RATE (-6)       /* sample rate the channel kind does not serve (MSK: outside [12000, 96000] Hz) */
#define AERO_E_DEVICE (-7)     /* a kernel gave up (wave hand-off timeout): the run's outputs are invalid */

/* engine flags */
#define AERO_F_TRACE_PT 0x1    /* keep the rotated pt_qpsk trace (parity tests)      */
#define AERO_F_TRACE_BLOCKS 0x2 /* keep decoded Viterbi blocks (parity tests)         */
#define AERO_F_TIMING 0x4      /* HIP-event timing of every kernel launch            */
#define AERO_F_TRACE_SOFT 0x8  /* keep delivered soft bits for aero_pop_softbits      */
#define AERO_F_TRACE_HOPS 0x10 /* keep per-hop coarse-estimator records              */
#define AERO_F_TRACE_FRAMES 0x20 /* keep per-frame infofield records (aero_pop_frames) */
#define AERO_F_DCD_TICK 0x40   /* continuous OQPSK: run AeroL's 1 s data-carrier-detect
                                  timer (decode/aerol.cpp:900-902, 1043-1058) on the
                                  sample clock, one tick per 48000 input samples, as
                                  the shipped binary's event loop fires it once per
                                  second of real-time audio (decode/main.cpp:106).
                                  Without it the timer never fires: after a lost
                                  message a channel that has synced once searches
                                  for the UW only at the expected frame boundary */

typedef struct aero_engine aero_engine;

typedef struct {
  int device;       /* HIP device ordinal                                   */
  int max_channels; /* channel table size (memory is sized for this)        */
  int flags;        /* AERO_F_*                                              */
} aero_engine_cfg;

typedef struct {
  int bitrate;            /* 10500 (OQPSK), 600 or 1200 (MSK); decode/decode.h:42;
                             8400: the C channel (OqpskDemodulator at fb = 8400 +
                             AeroL::DecodeC, decode/aerol.cpp:2145-2415), outside
                             aero-decode's validBitRates; continuous only, fs 48000 */
  int burst;              /* 1: aero-decode --burst: 10500 bps OQPSK, or
                             600 / 1200 bps MSK (one fb = 1200 demodulator at
                             48 kHz, decode/decode.cpp:123-132)               */
  uint32_t fs;            /* 48000 / 12000 / 24000 for 10500 / 600 / 1200 bps
                             (decode/decode.cpp:145, 152-159); burst MSK takes
                             any rate, the audio is demodulated as 48 kHz
                             (burstmskdemodulator.cpp:708-714 only logs it)   */
  int disable_reassembly; /* 1: items are ACARSfragmentsignal (decode.cpp:233) */
} aero_channel_cfg;

/* ACARSItem (decode/aerol.h:163-197) as a fixed-size POD.  `parsed`
 * (libacars, absent) and the wall-clock time are not produced. */
typedef struct {
  uint32_t aesid;
  uint8_t gesid, qno, refno, seqno;
  uint8_t mode, tak, bi, nonacars;
  uint8_t downlink, valid, hastext, moretocome;
  uint8_t fragment; /* 1 = ACARSfragmentsignal, 0 = ACARSsignal */
  uint8_t label_len, reg_len, pad0;
  char label[4];
  char reg[16];
  uint32_t msg_len;  /* bytes used in msg */
  char msg[3584];    /* Latin-1 text, not NUL-terminated */
} aero_acars_item;

/* Engine lifetime (replaces Decoder::Decoder / ~Decoder, decode/decode.cpp:72-260). */
int aero_engine_create(const aero_engine_cfg *cfg, aero_engine **out);
void aero_engine_destroy(aero_engine *e);

/* Opens one VFO channel: the Decoder ctor's demod + AeroL + hunter wiring
 * (decode/decode.cpp:117-241) for one -t topic.  bitrate 10500 at fs 48000,
 * or 600 / 1200 (MSK) at any fs in [12000, 96000] Hz: 12000, 24000 and
 * 48000 run kernels compiled for the rate, other rates the generic-rate MSK
 * kernels.  AERO_E_INVALID for another bit rate or OQPSK rate, AERO_E_RATE
 * for an MSK rate outside that range. */
int aero_channel_open(aero_engine *e, const aero_channel_cfg *cfg, int *ch_out);

/* One ZMQ message == one call: Decoder::audioReceived ->
 * OqpskDemodulator::dataReceived / MskDemodulator::dataReceived
 * (decode/decode.cpp:352, decode/oqpskdemodulator.cpp:624-630,
 * decode/mskdemodulator.cpp:472-481).  pcm: int16 LE real samples, copied
 * before returning (a continuous channel's message is staged in pinned host
 * memory and reaches the GPU at the next aero_run).  fs: an OQPSK or burst
 * channel only logs a mismatch; a continuous MSK channel re-applies its
 * settings at any rate in [12000, 96000] Hz, keeping the state
 * MskDemodulator::setSettings keeps (decode/mskdemodulator.cpp:94-218), and
 * refuses a rate outside it (AERO_E_RATE, the message is dropped). */
int aero_push_pcm(aero_engine *e, int ch, const int16_t *pcm, size_t n, uint32_t fs);

/* Lockstep batch push for channels [0, nch): pcm is time-major, n samples
 * per channel, sample t of channel c at pcm[t*ld + c].  dev != 0: pcm is a
 * HIP device pointer (inputs already resident in HBM).  Channels [0, nch)
 * must be of one kind (continuous bit rate, burst OQPSK or burst MSK).  For
 * burst channels the batch is one message per channel (at most 16384
 * samples; burst OQPSK output depends on message boundaries,
 * decode/burstoqpskdemodulator.cpp:264).  The channels must have been opened
 * in order into one group (engine channel j is the group's slot j): once an
 * MSK rate change has moved a channel into a slot another channel left, that
 * group no longer qualifies (AERO_E_INVALID; push per channel instead). */
int aero_push_pcm_batch(aero_engine *e, const int16_t *pcm, size_t n, size_t ld, int nch, int dev);

/* aero_push_pcm with pcm a HIP device pointer (e.g. channeliser audio already
 * in HBM, aero_chan.h); the samples are copied before returning. */
int aero_push_pcm_dev(aero_engine *e, int ch, const int16_t *pcm, size_t n, uint32_t fs);

/* Runs the batched kernels for every channel over all pushed samples that
 * complete a coarse-estimate hop; aero_flush also processes the tail. */
int aero_run(aero_engine *e);
int aero_flush(aero_engine *e);

/* Soft bits delivered to AeroL (groups of 32 for OQPSK, 12 for MSK, 0..255;
 * decode/oqpskdemodulator.cpp:534-540, decode/mskdemodulator.cpp:404-407).
 * Needs AERO_F_TRACE_SOFT. */
int aero_pop_softbits(aero_engine *e, int ch, int16_t *dst, size_t cap, size_t *n);

/* ACARSItems emitted on ACARSsignal (or ACARSfragmentsignal with
 * disable_reassembly), in emission order (decode/aerol.cpp:457,522,2127,2142). */
int aero_pop_items(aero_engine *e, int ch, aero_acars_item *dst, size_t cap, size_t *n);

/* Items of every channel in one call (channel order, then emission order);
 * ch[i] receives item i's channel.  For hosts that serve many VFOs from one
 * engine: one call per aero_run instead of one per channel.  Only the first
 * msg_len bytes of each msg are written.
 *
 * aero_run is asynchronous: it enqueues the GPU work and returns.  The pop
 * calls return what has completed so far (in order); aero_flush and
 * aero_sync return only when every pushed sample's outputs are available. */
int aero_pop_items_all(aero_engine *e, aero_acars_item *dst, int *ch, size_t cap, size_t *n);

/* Diagnostics used by the parity tests and the bench.
 * hops: 6 doubles per coarse hop (sample index, estimate, mixer2 Hz,
 * mixer_center Hz, mse, signal). pt: 2 doubles per carrier event.
 * blocks: uint32 count + decoded bits (bytes 0/1) per Viterbi block.
 * frames: 320 bytes per completed frame (312 infofield, u32 len, u32 crc mask);
 * needs AERO_F_TRACE_FRAMES. */
int aero_pop_hops(aero_engine *e, int ch, double *dst, size_t cap_records, size_t *n);
/* Limits the trace collection of continuous channels (soft bits, hops, pt,
 * blocks, frames) to the n channels in ch (n = 0: every channel again), so
 * a parity test can sample a few channels of a full-size batch.  Test
 * support; no reference counterpart. */
int aero_trace_select(aero_engine *e, const int *ch, int n);
int aero_pop_pt(aero_engine *e, int ch, double *dst, size_t cap_records, size_t *n);
int aero_pop_blocks(aero_engine *e, int ch, uint8_t *dst, size_t cap, size_t *n);
int aero_pop_frames(aero_engine *e, int ch, uint8_t *dst, size_t cap, size_t *n);
/* Burst channels (AERO_F_TRACE_FRAMES): every R/T test (uint32 blockptr,
 * uint32 RTChannelDeleaveFECScram result) and every decoded R/T packet
 * (uint32 'R'/'T', uint32 length, the infofield bytes), in order
 * (decode/aerol.h:755-836). */
int aero_pop_rt_tests(aero_engine *e, int ch, uint8_t *dst, size_t cap, size_t *n);

/* C channel (bitrate 8400).  A C-channel message is one prefilter block
 * (decode/oqpskdemodulator.cpp:292-324, output depends on message boundaries):
 * at most 32768 samples per aero_push_pcm (AERO_E_INVALID above).
 * c_units: the 12-byte SUs AeroL::DecodeC emits on Call_progress_Signal
 * (CRC-valid, message 0x30, decode/aerol.cpp:2329-2346), cap / *n in SUs.
 * voice: per decoded frame (Voicesignal, :2394-2402) a 304-byte record: uint32
 * LE AES of the frame's last Call_progress SU (0 = "000000"), then the 300
 * voice bytes (25 frames of 12); cap / *n in records.  Frames (36 SU bytes,
 * CRC mask of the 3 SUs) through aero_pop_frames with AERO_F_TRACE_FRAMES. */
int aero_pop_c_units(aero_engine *e, int ch, uint8_t *dst, size_t cap, size_t *n);
int aero_pop_voice(aero_engine *e, int ch, uint8_t *dst, size_t cap, size_t *n);
int aero_pop_rt_packets(aero_engine *e, int ch, uint8_t *dst, size_t cap, size_t *n);

/* Timing (AERO_F_TIMING): kernel names {"demod","coarse","frame","viterbi"}
 * give summed device milliseconds (HIP events) and launch counts; host
 * sections {"host_push","host_run","host_wait_njobs","host_wait_jobs",
 * "host_frames"} give summed wall milliseconds and entry counts.  Both since
 * the last reset. */
int aero_timing(aero_engine *e, const char *name, double *ms, long *launches);
void aero_timing_reset(aero_engine *e);

/* Counters since creation.  "device_bytes" / "groups": the device pools of
 * the continuous channel groups that exist now and their number (a
 * generic-rate MSK group holds at most 256 channels and is released when its
 * last channel moves to another rate).  Continuous channels: "viterbi_jobs" (blocks
 * the GPU Viterbi decoded and handed back), "frames" (frames delivered to
 * the SU/ACARS host), "su_crc_ok" (SUs whose CRC-16 checked); burst
 * channels: "rt_tests" (RTChannelDeleaveFECScram decodes run),
 * "rt_packets" (R/T packets that passed their CRCs), "rt_pass_max" (the most
 * R/T tests one pass handed to the host; from 256 on they are split over the
 * host threads).  Joins the
 * asynchronous host frame work first.  AERO_E_INVALID for another name. */
int aero_stat(aero_engine *e, const char *name, uint64_t *value);

/* Per-channel state: "hunter_scans" (full SignalHunter scans without a
 * signal, decode/hunter.cpp:31-37 -- aero-decode's --no-signal-exit),
 * "freq_center" (the mixer centre in Hz after the last coarse hop).  Waits
 * for the channel's queued GPU work. */
int aero_channel_stat(aero_engine *e, int ch, const char *name, int64_t *value);

/* Decoder status events of one channel since it opened, for aero-decode's
 * verbose log (Decoder::handleDcdChange / handleNewFreqCenter,
 * decode/decode.cpp:429-439).  dcd_edges: changes of AeroL's data carrier
 * detect as SignalHunter::handleDcd passes them on (decode/hunter.cpp:14-19);
 * they alternate and the first is "no signal => signal".  hunter_steps:
 * SignalHunter::newFreqCenter emissions (decode/hunter.cpp:31-40), with the
 * centre of step k (1-based) in hunter_fc[(k - 1) & 7] for the last eight
 * steps (0 for burst channels: their hunter is disabled, decode/decode.cpp:175).
 * Waits for the channel's queued GPU work. */
typedef struct {
  int64_t dcd_edges;
  int64_t hunter_steps;
  double hunter_fc[8];
} aero_channel_events;
int aero_channel_get_events(aero_engine *e, int ch, aero_channel_events *out);

/* Total input samples demodulated across channels since creation. */
uint64_t aero_samples_processed(aero_engine *e);

/* Synchronise the engine's stream. */
int aero_sync(aero_engine *e);

/* Evaluates the device libm on n inputs (parity test of aero_math.h):
 * fn 0 hypot, 1 atan2, 2 tanh, 3 sin, 4 cos, 5 log10, 6 sqrt, 7 fmod(x,360),
 * 8 division x/y.  x, y, out are host arrays. */
int aero_device_math(aero_engine *e, int fn, const double *x, const double *y, double *out, size_t n);

const char *aero_strerror(int rc);

#ifdef __cplusplus
}
#endif
#endif
