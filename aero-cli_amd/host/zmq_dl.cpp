#include "zmq_dl.h"

#include <dlfcn.h>

#include <cstdio>
#include <cstdlib>

namespace aerohost {

const Zmq *zmq_load() {
  static Zmq z;
  static int state = 0;  // 0 untried, 1 ok, -1 failed
  if (state) return state > 0 ? &z : nullptr;
  const char *cands[] = {getenv("AERO_LIBZMQ"), "libzmq.so.5", "/opt/conda/lib/libzmq.so.5"};
  void *h = nullptr;
  for (const char *c : cands)
    if (c && (h = dlopen(c, RTLD_NOW | RTLD_LOCAL))) break;
  if (!h) {
    fprintf(stderr, "libzmq.so.5 not found (set AERO_LIBZMQ): %s\n", dlerror());
    state = -1;
    return nullptr;
  }
  bool ok = true;
  auto sym = [&](const char *n) {
    void *p = dlsym(h, n);
    if (!p) {
      fprintf(stderr, "libzmq: missing %s\n", n);
      ok = false;
    }
    return p;
  };
  z.ctx_new = (void *(*)())sym("zmq_ctx_new");
  z.ctx_term = (int (*)(void *))sym("zmq_ctx_term");
  z.socket = (void *(*)(void *, int))sym("zmq_socket");
  z.close = (int (*)(void *))sym("zmq_close");
  z.connect = (int (*)(void *, const char *))sym("zmq_connect");
  z.bind = (int (*)(void *, const char *))sym("zmq_bind");
  z.setsockopt = (int (*)(void *, int, const void *, size_t))sym("zmq_setsockopt");
  z.send = (int (*)(void *, const void *, size_t, int))sym("zmq_send");
  z.recv = (int (*)(void *, void *, size_t, int))sym("zmq_recv");
  z.errno_ = (int (*)())sym("zmq_errno");
  z.strerror = (const char *(*)(int))sym("zmq_strerror");
  state = ok ? 1 : -1;
  return ok ? &z : nullptr;
}

}  // namespace aerohost
