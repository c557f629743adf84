/*
 * aero_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * C API of the CPU restatement of airframesio/aero-cli's continuous
 * 10500-bps OQPSK decode path (decode/oqpskdemodulator.cpp, decode/DSP.cpp,
 * decode/coarsefreqestimate.cpp, decode/jfft.cpp, decode/hunter.cpp,
 * decode/aerol.cpp, decode/jconvolutionalcodec.cpp + libcorrect).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker.  Nothing in the product path
 * links or calls it.
 *
 * Parity status: see oracle/aero_oracle.cpp header.
 */
#ifndef AERO_ORACLE_H
#define AERO_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_chan oracle_chan;

/* flags */
#define ORACLE_TRACE_PT 1 /* record every rotated pt_qpsk (re,im) */
#define ORACLE_BURST 2    /* burst mode (aero-decode --burst): 10500 OQPSK, 600/1200 MSK */
#define ORACLE_DCD_TICK 4 /* continuous OQPSK: AeroL's 1 s DCD timer (aerol.cpp:900-902,
                             1043-1058) fires after every Fs input samples */

/* bitrate 10500 / 8400 (continuous OQPSK P / C channel), 600 / 1200 (MSK) */
oracle_chan *oracle_create(int bitrate, int flags);
void oracle_destroy(oracle_chan *c);

/* One call == one ZMQ message == OqpskDemodulator::dataReceived
 * (decode/oqpskdemodulator.cpp:624-630). */
int oracle_push(oracle_chan *c, const int16_t *pcm, size_t n);
/* the same with the message's sample rate (Decoder::audioReceived): an MSK
 * channel re-applies its settings at a new rate (mskdemodulator.cpp:473-481) */
int oracle_push_rate(oracle_chan *c, const int16_t *pcm, size_t n, int fs);

/* Soft bits delivered to AeroL (groups of 32, decode/oqpskdemodulator.cpp:534-540). */
size_t oracle_softbits(const oracle_chan *c, uint8_t *dst, size_t cap);
/* burst: delivered soft bits including the -1 start-of-packet markers */
size_t oracle_softbits16(const oracle_chan *c, int16_t *dst, size_t cap);
/* burst: every R/T test (uint32 blockptr, uint32 result code) in order */
size_t oracle_rt_tests(const oracle_chan *c, uint8_t *dst, size_t cap);
/* burst: per decoded R/T packet: uint32 kind ('R'/'T'), uint32 length, infofield bytes */
size_t oracle_rt_packets(const oracle_chan *c, uint8_t *dst, size_t cap);

/* C channel (bitrate 8400, AeroL::DecodeC, decode/aerol.cpp:2145-2415): every
 * CRC-valid Call_progress SU (Call_progress_Signal, 12 bytes each), and per
 * decoded frame a uint32 AES (of the frame's last Call_progress, 0 for
 * "000000") followed by the 300 voice bytes (Voicesignal). */
size_t oracle_c_units(const oracle_chan *c, uint8_t *dst, size_t cap);
size_t oracle_voice(const oracle_chan *c, uint8_t *dst, size_t cap);

/* Per coarse-estimate hop, 6 doubles: sample index, freq_offset_est emitted,
 * mixer2 freq, mixer_center freq (after the slot ran), mse, signal flag. */
size_t oracle_hops(const oracle_chan *c, double *dst, size_t cap_records);

/* Decoder status events (decode/decode.cpp:429-439): *dcd_edges = the data
 * carrier detect changes SignalHunter::handleDcd passes on; returns the
 * number of newFreqCenter emissions and copies their centres (at most cap). */
size_t oracle_events(oracle_chan *c, long long *dcd_edges, double *fc, size_t cap);

/* rotated pt_qpsk trace (2 doubles per carrier event), only with ORACLE_TRACE_PT */
size_t oracle_pt(const oracle_chan *c, double *dst, size_t cap_records);

/* Per decoded P-channel block: 2496 (or 2483 first) decoded bits as bytes 0/1,
 * prefixed by a uint32 count. */
size_t oracle_blocks(const oracle_chan *c, uint8_t *dst, size_t cap);

/* Per completed frame: 320 bytes = up to 312 infofield bytes (zero padded),
 * then uint32 infofield length, then uint32 crc-ok bitmask (26 bits). */
size_t oracle_frames(const oracle_chan *c, uint8_t *dst, size_t cap);

/* ACARSItems as canonical text lines (see tests/aero_items.py). */
size_t oracle_items(const oracle_chan *c, char *dst, size_t cap);

/* libcorrect-ABI restatement (r=1/2, K=7, polys {109,79}). */
size_t oracle_conv_encode(const uint8_t *msg, size_t msg_len, uint8_t *encoded);
size_t oracle_viterbi_decode_soft(const uint8_t *soft, size_t num_encoded_bits,
                                  uint8_t *msg);

/* Known-answer helpers */
uint16_t oracle_crc16_bytes(const uint8_t *bytes, int n);
void oracle_scrambler_bits(int *dst, int n);
void oracle_deinterleave_perm(int N, int *src_index_of_dst);
void oracle_rrc_design(double alpha, int firsize, double fs, double symfreq, double *dst);
void oracle_cis_table(double *dst); /* 19999 x (cos, sin) */
void oracle_twiddles(int nfft, int inverse, double *dst);
void oracle_msk_taps(int sps, double *dst); /* MskDemodulator matched filter, 2*sps taps */

/* raw JFFT-order transform for the FFT parity test (in place, nfft complex) */
void oracle_fft(double *x, int nfft, int inverse);

/* aero-publish channeliser (pub_oracle.cpp).  mains: nmain x {frequency,
 * out_rate, compress_scale, publish}; vfos: nvfo x {frequency, data_rate,
 * out_rate, filter_bandwidth}; gains: the INI "gain" values.  NULL when the
 * configuration is invalid. */
typedef struct oracle_pub oracle_pub;
oracle_pub *oracle_pub_create(int fs, int center, int mix_offset, int dcc, const int *mains, int nmain,
                              const int *vfos, const float *gains, int nvfo);
void oracle_pub_destroy(oracle_pub *o);
int oracle_pub_block_len(const oracle_pub *o);
void oracle_pub_process(oracle_pub *o, const float *iq, int nblocks); /* interleaved CF32 blocks */
size_t oracle_pub_usb(const oracle_pub *o, int v, int16_t *dst, size_t cap);
size_t oracle_pub_iq(const oracle_pub *o, int m, int8_t *dst, size_t cap);
int oracle_pub_info(const oracle_pub *o, int v, int *info7);
int oracle_pub_low_pass(double gain, double fs, double cutoff, double tw, float *dst, int cap);
void oracle_pub_hilbert(int len, int fs, float *dst);
void oracle_pub_osc(double fs, double freq, float *dst); /* (int)fs complex */

#ifdef __cplusplus
}
#endif
#endif
