/*
 * zmq_dl.h — the libzmq calls aero-decode / aero-publish make
 * (decode/decode.cpp:95-115, 307-353; publish/zmqpublisher.cpp:10-73),
 * resolved at run time from the image's libzmq.so.5 (conda) so the binaries
 * link against nothing but the engine, libc and libstdc++.
 */
#pragma once
#include <cstddef>

namespace aerohost {

struct Zmq {
  void *(*ctx_new)();
  int (*ctx_term)(void *);
  void *(*socket)(void *, int);
  int (*close)(void *);
  int (*connect)(void *, const char *);
  int (*bind)(void *, const char *);
  int (*setsockopt)(void *, int, const void *, size_t);
  int (*send)(void *, const void *, size_t, int);
  int (*recv)(void *, void *, size_t, int);
  int (*errno_)();
  const char *(*strerror)(int);
};

// loads libzmq (AERO_LIBZMQ, libzmq.so.5, then /opt/conda/lib/libzmq.so.5);
// nullptr with a message on stderr when none loads
const Zmq *zmq_load();

// constants of zmq.h (libzmq 4.x ABI)
constexpr int ZMQ_PUB_ = 1, ZMQ_SUB_ = 2, ZMQ_SUBSCRIBE_ = 6, ZMQ_SNDMORE_ = 2, ZMQ_DONTWAIT_ = 1, ZMQ_LINGER_ = 17,
              ZMQ_SNDHWM_ = 23, ZMQ_RCVHWM_ = 24, ZMQ_RECONNECT_IVL_ = 18, ZMQ_RECONNECT_IVL_MAX_ = 21;

}  // namespace aerohost
