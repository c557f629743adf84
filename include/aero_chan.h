/*
 * aero_chan.h — C ABI of the MI355X channeliser (aero-publish's VFO tree).
 *
 * Replaces the CPU channeliser of airframesio/aero-cli's aero-publish:
 * Publisher::loadSettings (publish/publisher.cpp:55-227) builds main VFOs and
 * their sub-VFOs from the SDRReceiver INI, Publisher::demodData
 * (publish/publisher.cpp:285-306) hands every CF32 read to the main VFOs, and
 * vfo::process (publish/vfo.cpp:154-186) mixes, half-band decimates and
 * USB-demodulates each sub-VFO into int16 audio that ZmqPublisher::publish
 * (publish/zmqpublisher.cpp:61-73) sends to aero-decode.  Here the audio stays
 * in HBM: aero_chan_feed pushes it into aero_engine channels directly.
 *
 * Numerics: FP32, bit-exact with the reference's sample-by-sample code,
 * including the half-band queue copy-back that keeps the wrong slots
 * (publish/dsp.cpp:163-172) and the oscillator's first-sample quirk
 * (publish/oscillator.cpp:12-27).  Errors are the AERO_E_* codes of
 * aero_engine.h.
 */
#ifndef AERO_CHAN_H
#define AERO_CHAN_H

#include <stddef.h>
#include <stdint.h>

#include "aero_engine.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct aero_chan aero_chan;

/* [General] keys of the INI (publish/publisher.cpp:65-113) plus the GPU side */
typedef struct {
  int device;            /* HIP device */
  int sample_rate;       /* 288000, 1536000 or 1920000 (publish/publisher.h:32) */
  int center_frequency;  /* Hz */
  int mix_offset;        /* added to every [vfos] frequency (publisher.cpp:160) */
  int correct_dc_bias;   /* demodData's DC removal (publisher.cpp:292-296) */
  int max_blocks;        /* reads (blocks) batched per aero_chan_run */
  int flags;             /* AERO_CHAN_F_* */
} aero_chan_cfg;

/* one [main_vfos] entry (publisher.cpp:115-148) */
typedef struct {
  int frequency;
  int out_rate;
  int compress_scale;    /* 0: 1 */
  int publish;           /* zmq_address and zmq_topic set: 4-bit IQ output when it has no sub-VFOs */
} aero_chan_main;

/* one [vfos] entry (publisher.cpp:151-222) */
typedef struct {
  int frequency;
  int data_rate;         /* out_rate 0: 600 -> 12000, 1200 -> 24000, other -> 48000 */
  int out_rate;
  int filter_bandwidth;  /* 0: no audio low-pass */
  float gain;            /* INI "gain" (percent) */
  int skip;              /* not computed by this process (multi-GPU sharding) */
} aero_chan_vfo;

#define AERO_CHAN_F_HOST_OUT 0x1 /* keep every output for aero_chan_pop_* */

/* Publisher::loadSettings.  At most 3 main VFOs (VFOsub[3], publisher.h:50);
 * a [vfos] entry that no main VFO covers is refused when main VFOs exist
 * (the reference would feed it another main VFO's stream) and never runs when
 * there are none (as in the reference). */
int aero_chan_create(const aero_chan_cfg *cfg, const aero_chan_main *mains, int nmain, const aero_chan_vfo *vfos,
                     int nvfo, aero_chan **out);
void aero_chan_destroy(aero_chan *c);

/* complex samples per read: buflen / 2 (publisher.cpp:92-100) */
int aero_chan_block_len(aero_chan *c, int *block_len);
/* [vfos] entry v: info5 = {main index (-1: none), output rate, output samples
 * per block, half-band stages, late decimation 0/5/6} */
int aero_chan_vfo_info(aero_chan *c, int v, int *info5);
/* [main_vfos] entry m: info3 = {output rate, output samples per block, half-band stages} */
int aero_chan_main_info(aero_chan *c, int m, int *info3);

/* nblocks whole reads of interleaved CF32 (SOAPY_SDR_CF32, publisher.cpp:254);
 * dev != 0: a HIP device pointer.  Copied before returning.  At most
 * max_blocks reads may be pending between two aero_chan_run calls: a push
 * beyond that returns AERO_E_FULL (nothing of the excess is taken), except
 * with AERO_CHAN_F_HOST_OUT, where the full batch runs first and its
 * outputs are kept for aero_chan_pop_*. */
int aero_chan_push(aero_chan *c, const float *iq, size_t nblocks, int dev);
/* processes the pending reads (asynchronous; aero_chan_sync waits) */
int aero_chan_run(aero_chan *c);
int aero_chan_sync(aero_chan *c);
/* device view of the last batch's int16 audio of [vfos] entry v (valid until
 * the next push/run; call aero_chan_sync before reading it on another stream) */
int aero_chan_vfo_output(aero_chan *c, int v, const int16_t **dptr, size_t *n);
/* AERO_CHAN_F_HOST_OUT: pop the audio of [vfos] entry v / the 4-bit IQ of main VFO m */
int aero_chan_pop_audio(aero_chan *c, int v, int16_t *dst, size_t cap, size_t *n);
int aero_chan_pop_iq(aero_chan *c, int m, int8_t *dst, size_t cap, size_t *n);
/* vfo::transmitData -> ZMQ -> Decoder::audioReceived (vfo.cpp:289-313,
 * decode/decode.cpp:283-366) without the hop: the last batch's audio of every
 * [vfos] entry v with ch[v] >= 0 goes to engine channel ch[v]
 * (aero_push_pcm_dev).  Call once per aero_chan_run. */
int aero_chan_feed(aero_chan *c, aero_engine *e, const int *ch);

#ifdef __cplusplus
}
#endif
#endif
