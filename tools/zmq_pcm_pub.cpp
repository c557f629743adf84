/*
 * zmq_pcm_pub — publishes an int16 PCM file as one VFO topic in
 * aero-publish's wire format ([topic, 5 bytes][u32 LE rate][int16 LE PCM],
 * publish/zmqpublisher.cpp:61-73), the way tools/audio-publisher feeds
 * aero-decode.  Test tool: binds a PUB socket, waits for subscribers, sends
 * the file in messages of --chunk samples, optionally paced.
 *
 *   zmq_pcm_pub --bind tcp://127.0.0.1:6004 --topic VFO01 --rate 48000
 *               --chunk 12000 [--wait-ms 1500] [--pace-ms 0] file.pcm
 */
#include <unistd.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "zmq_dl.h"

using namespace aerohost;

int main(int argc, char **argv) {
  std::string bind = "tcp://127.0.0.1:6004", topic = "VFO01", file;
  uint32_t rate = 48000;
  long chunk = 12000, wait_ms = 1500, pace_ms = 0, tail_ms = 500;
  for (int i = 1; i < argc; i++) {
    std::string a = argv[i];
    auto val = [&]() { return std::string(i + 1 < argc ? argv[++i] : ""); };
    if (a == "--bind") bind = val();
    else if (a == "--topic") topic = val();
    else if (a == "--rate") rate = (uint32_t)atol(val().c_str());
    else if (a == "--chunk") chunk = atol(val().c_str());
    else if (a == "--wait-ms") wait_ms = atol(val().c_str());
    else if (a == "--pace-ms") pace_ms = atol(val().c_str());
    else if (a == "--tail-ms") tail_ms = atol(val().c_str());
    else file = a;
  }
  FILE *f = fopen(file.c_str(), "rb");
  if (!f) {
    fprintf(stderr, "zmq_pcm_pub: cannot open %s\n", file.c_str());
    return 2;
  }
  std::vector<int16_t> pcm;
  int16_t b[4096];
  size_t n;
  while ((n = fread(b, 2, 4096, f)) > 0) pcm.insert(pcm.end(), b, b + n);
  fclose(f);
  const Zmq *z = zmq_load();
  if (!z) return 2;
  void *ctx = z->ctx_new();
  void *pub = z->socket(ctx, ZMQ_PUB_);
  int hwm = 0;  // no drops while the subscriber catches up
  z->setsockopt(pub, ZMQ_SNDHWM_, &hwm, sizeof hwm);
  if (z->bind(pub, bind.c_str()) != 0) {
    fprintf(stderr, "zmq_pcm_pub: bind %s: %s\n", bind.c_str(), z->strerror(z->errno_()));
    return 2;
  }
  usleep((useconds_t)wait_ms * 1000);  // slow-joiner: let SUB sockets connect
  // ZmqPublisher::publish sends the topic as exactly 5 bytes (zmqpublisher.cpp:69)
  std::string t5 = topic;
  t5.resize(5, '\0');
  size_t sent = 0;
  for (size_t off = 0; off < pcm.size(); off += (size_t)chunk) {
    const size_t k = std::min<size_t>((size_t)chunk, pcm.size() - off);
    z->send(pub, t5.data(), 5, ZMQ_SNDMORE_);
    z->send(pub, &rate, 4, ZMQ_SNDMORE_);
    z->send(pub, pcm.data() + off, k * 2, 0);
    sent++;
    if (pace_ms) usleep((useconds_t)pace_ms * 1000);
  }
  usleep((useconds_t)tail_ms * 1000);
  int linger = 2000;
  z->setsockopt(pub, ZMQ_LINGER_, &linger, sizeof linger);
  z->close(pub);
  z->ctx_term(ctx);
  fprintf(stderr, "zmq_pcm_pub: %zu messages, %zu samples\n", sent, pcm.size());
  return 0;
}
