/*
 * aero_publish.cpp — drop-in replacement for the reference's aero-publish
 * (publish/main.cpp:12-69, publish/publisher.cpp:13-319,
 * publish/vfo.cpp:57-313, publish/zmqpublisher.cpp:10-73) with the
 * channeliser on the MI355X (include/aero_chan.h).
 *
 * Same command line (-d device, -v, --enable-biast, --enable-dcc, settings
 * INI), same SDRReceiver INI keys, same ZeroMQ output: every [vfos] entry's
 * int16 USB audio on the [General] zmq_address (bound, one shared PUB
 * socket), every main VFO without sub-VFOs that has zmq_address + zmq_topic
 * publishing its compressed IQ on its own (connected) socket, as
 * [topic, 5 bytes][u32 LE rate][payload], main VFOs in INI order and each
 * main's sub-VFOs in INI order after every read.
 *
 * SoapySDR is not in this image, so the device string selects a CF32 source
 * in SoapySDR's key=value syntax instead of a radio:
 *   driver=file,path=<interleaved float32 IQ>[,loop=1][,realtime=1][,start_delay_ms=N]
 * (realtime paces reads at the INI sample rate, as a radio delivers them).
 * Any other driver fails the way SoapySDR::Device::make does.
 */
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "../../include/aero_chan.h"
#include "ini.h"
#include "log.h"
#include "section_timer.h"
#include "zmq_dl.h"

namespace aerohost {
bool g_verbose = false;
}
using namespace aerohost;

namespace {

std::atomic<int> g_running{0};

void on_signal(int sig) {
  if (sig == SIGINT || sig == SIGTERM) g_running.store(0);
}

void on_fatal(int sig) {
  void *bt[64];
  const int n = backtrace(bt, 64);
  fprintf(stderr, "aero-publish: fatal signal %d\n", sig);
  backtrace_symbols_fd(bt, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

const char *kUsage =
    "Usage: aero-publish [options] settings\n"
    "Publish INMARSAT Aero frequency chunks as VFOs over ZMQ\n"
    "\n"
    "Options:\n"
    "  -h, --help               Displays help on commandline options.\n"
    "  --help-all               Displays help including Qt specific options.\n"
    "  -d, --device <device>    SoapySDR device string\n"
    "  -v, --verbose            Show verbose output\n"
    "  --enable-biast           Enable Bias-T\n"
    "  --enable-dcc             Enable DC correction\n"
    "\n"
    "Arguments:\n"
    "  settings                 Path to SDRReceiver compliant satellite settings INI\n"
    "                           file\n";

std::map<std::string, std::string> kwargs(const std::string &s) {  // SoapySDR::KwargsFromString
  std::map<std::string, std::string> kw;
  size_t p = 0;
  while (p <= s.size()) {
    size_t e = s.find(',', p);
    if (e == std::string::npos) e = s.size();
    const std::string item = s.substr(p, e - p);
    const size_t eq = item.find('=');
    if (!item.empty()) kw[item.substr(0, eq)] = eq == std::string::npos ? "" : item.substr(eq + 1);
    p = e + 1;
  }
  return kw;
}

// ZmqPublisher (publish/zmqpublisher.cpp:10-73)
struct Publisher {
  const Zmq *z = nullptr;
  void *ctx = nullptr, *sock = nullptr;
  bool open(const Zmq *zz, void *c, const std::string &addr, bool bind) {
    z = zz;
    ctx = c;
    sock = z->socket(ctx, ZMQ_PUB_);
    if (!sock) return false;
    const int keepalive = 1, cnt = 10, idle = 1, intvl = 1, reconnect = 1000, reconnect_max = 0;
    z->setsockopt(sock, 34 /* ZMQ_TCP_KEEPALIVE */, &keepalive, sizeof keepalive);
    z->setsockopt(sock, 35 /* ZMQ_TCP_KEEPALIVE_CNT */, &cnt, sizeof cnt);
    z->setsockopt(sock, 36 /* ZMQ_TCP_KEEPALIVE_IDLE */, &idle, sizeof idle);
    z->setsockopt(sock, 37 /* ZMQ_TCP_KEEPALIVE_INTVL */, &intvl, sizeof intvl);
    z->setsockopt(sock, ZMQ_RECONNECT_IVL_, &reconnect, sizeof reconnect);
    z->setsockopt(sock, ZMQ_RECONNECT_IVL_MAX_, &reconnect_max, sizeof reconnect_max);
    // AERO_ZMQ_HWM (not in the reference, which keeps ZeroMQ's default 1000):
    // a send queue bound for runs that publish faster than real time (a file
    // source without pacing); 0 = unbounded, nothing is dropped
    if (const char *h = getenv("AERO_ZMQ_HWM")) {
      const int hwm = atoi(h);
      z->setsockopt(sock, ZMQ_SNDHWM_, &hwm, sizeof hwm);
    }
    return (bind ? z->bind(sock, addr.c_str()) : z->connect(sock, addr.c_str())) == 0;
  }
  // the topic goes out as exactly 5 bytes (zmqpublisher.cpp:69), NUL-padded
  void publish(const void *buf, size_t len, const std::string &topic, uint32_t rate) {
    if (!sock || !len) return;
    std::string t5 = topic;
    t5.resize(5, '\0');
    z->send(sock, t5.data(), 5, ZMQ_SNDMORE_);
    z->send(sock, &rate, 4, ZMQ_SNDMORE_);
    z->send(sock, buf, len, 0);
  }
  void close() {
    if (sock) z->close(sock);
    sock = nullptr;
  }
};

}  // namespace

int main(int argc, char **argv) {
  std::string device, settings;
  bool biast = false, dcc = false;
  for (int i = 1; i < argc; i++) {
    std::string a = argv[i];
    if (a == "-h" || a == "--help" || a == "-?" || a == "--help-all") {
      fputs(kUsage, stdout);
      return 0;
    } else if (a == "-v" || a == "--verbose") {
      g_verbose = true;
    } else if (a == "--enable-biast") {
      biast = true;
    } else if (a == "--enable-dcc") {
      dcc = true;
    } else if (a == "-d" || a == "--device") {
      if (i + 1 >= argc) {
        fprintf(stderr, "Missing value after '%s'.\n", a.c_str());
        return 1;
      }
      device = argv[++i];
    } else if (a.rfind("--device=", 0) == 0) {
      device = a.substr(9);
    } else if (a.rfind("-d", 0) == 0 && a.size() > 2) {
      device = a.substr(2);
    } else if (a.size() > 1 && a[0] == '-') {
      fprintf(stderr, "Unknown option '%s'.\n", a.substr(a[1] == '-' ? 2 : 1).c_str());
      return 1;
    } else if (settings.empty()) {
      settings = a;
    }
  }
  if (device.empty()) {
    AH_CRIT("Required device option missing; example: -d driver=rtlsdr");
    return 1;
  }
  if (settings.empty()) {
    AH_CRIT("Required settings path missing; please provide the path to a SDRReceiver compliant settings INI file");
    return 1;
  }
  // Publisher::loadSettings (publisher.cpp:55-227); a failure leaves the
  // publisher stopped and the application completes with status 0
  Ini ini;
  if (access(settings.c_str(), R_OK) != 0 || !ini.load(settings)) {
    AH_CRIT("Provided settings file path either doesn't exist or isn't a file: %s", settings.c_str());
    AH_CRIT("[ERROR] failed to parse and load settings");
    return 0;
  }
  const int Fs = ini.value_int("sample_rate");
  if (Fs == 0) {
    AH_CRIT("Provided sample rate in settings file either doesn't exist or isn't an integer");
    AH_CRIT("[ERROR] failed to parse and load settings");
    return 0;
  }
  if (Fs != 288000 && Fs != 1536000 && Fs != 1920000) {  // validSampleRates (publisher.h:32)
    AH_CRIT("Provided sample rate is not supported: %d", Fs);
    AH_CRIT("[ERROR] failed to parse and load settings");
    return 0;
  }
  const int center = ini.value_int("center_frequency");
  const int mix_offset = ini.value_int("mix_offset");
  const std::string zmq_address = ini.value("zmq_address");
  dcc = dcc || ini.value("correct_dc_bias") == "1";
  biast = biast || ini.value_int("auto_start_biast") == 1;
  const auto mains_ini = ini.array("main_vfos");
  const auto vfos_ini = ini.array("vfos");
  std::vector<aero_chan_main> mains;
  std::vector<std::string> main_addr, main_topic;
  for (auto &m : mains_ini) {
    auto get = [&](const char *k) { auto it = m.find(k); return it == m.end() ? std::string() : it->second; };
    aero_chan_main cm{Ini::to_int(get("frequency")), Ini::to_int(get("out_rate")), Ini::to_int(get("compress_scale")),
                      !get("zmq_address").empty() && !get("zmq_topic").empty()};
    mains.push_back(cm);
    main_addr.push_back(get("zmq_address"));
    main_topic.push_back(get("zmq_topic"));
  }
  std::vector<aero_chan_vfo> vfos;
  std::vector<std::string> topics;
  for (auto &v : vfos_ini) {
    auto get = [&](const char *k) { auto it = v.find(k); return it == v.end() ? std::string() : it->second; };
    vfos.push_back(aero_chan_vfo{Ini::to_int(get("frequency")), Ini::to_int(get("data_rate")),
                                 Ini::to_int(get("out_rate")), Ini::to_int(get("filter_bandwidth")),
                                 Ini::to_float(get("gain")), 0});
    topics.push_back(get("topic"));
  }
  for (size_t m = 0; m < mains.size(); m++)
    AH_DBG("main %zu frequency %d out_rate %d compress_scale %d publish %d", m, mains[m].frequency,
           mains[m].out_rate, mains[m].compress_scale, mains[m].publish);
  for (size_t v = 0; v < vfos.size(); v++)
    AH_DBG("vfo %zu topic %s frequency %d data_rate %d out_rate %d filter_bandwidth %d gain %g", v,
           topics[v].c_str(), vfos[v].frequency, vfos[v].data_rate, vfos[v].out_rate, vfos[v].filter_bandwidth,
           (double)vfos[v].gain);
  // the device: a CF32 source in place of SoapySDR::Device::make
  auto kw = kwargs(device);
  FILE *src = nullptr;
  if (kw["driver"] == "file" && !kw["path"].empty()) src = fopen(kw["path"].c_str(), "rb");
  if (!src) {
    AH_CRIT("[ERROR] failed to find device: %s", device.c_str());
    return 0;
  }
  const bool loop = kw["loop"] == "1", realtime = kw["realtime"] == "1";
  if (biast) AH_DBG("Bias-T requested (no radio: ignored)");
  aero_chan_cfg cfg{0, Fs, center, mix_offset, dcc ? 1 : 0, 1, AERO_CHAN_F_HOST_OUT};
  if (const char *d = getenv("AERO_DEVICE")) cfg.device = atoi(d);
  aero_chan *chan = nullptr;
  if (int rc = aero_chan_create(&cfg, mains.data(), (int)mains.size(), vfos.data(), (int)vfos.size(), &chan)) {
    AH_CRIT("[ERROR] the MI355X channeliser refused these settings: %s", aero_strerror(rc));
    fclose(src);
    return 1;
  }
  int B = 0;
  aero_chan_block_len(chan, &B);
  const Zmq *z = zmq_load();
  if (!z) return 1;
  void *ctx = z->ctx_new();
  // sub-VFOs publish on the shared bound socket (vfo.cpp:128-131), main VFOs
  // without sub-VFOs on their own connected one (:132-136)
  Publisher bound;
  std::vector<Publisher> main_pub(mains.size());
  std::vector<int> parent(vfos.size(), -1), rate(vfos.size(), 0), has_subs(mains.size(), 0);
  for (size_t v = 0; v < vfos.size(); v++) {
    int info[5];
    aero_chan_vfo_info(chan, (int)v, info);
    parent[v] = info[0];
    rate[v] = info[1];
    if (info[0] >= 0) has_subs[info[0]] = 1;
  }
  if (!vfos.empty() && !bound.open(z, ctx, zmq_address, true))
    AH_CRIT("ZeroMQ bind to %s failed: %s", zmq_address.c_str(), z->strerror(z->errno_()));
  for (size_t m = 0; m < mains.size(); m++)
    if (!main_addr[m].empty()) main_pub[m].open(z, ctx, main_addr[m], false);
  g_running.store(1);
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_handler = on_signal;
  sigaction(SIGINT, &sa, nullptr);
  sigaction(SIGTERM, &sa, nullptr);
  signal(SIGHUP, SIG_IGN);
  signal(SIGSEGV, on_fatal);
  signal(SIGABRT, on_fatal);
  if (kw.count("start_delay_ms")) usleep((useconds_t)atoi(kw["start_delay_ms"].c_str()) * 1000);
  AH_DBG("Starting concurrent reader publishing thread");
  std::vector<float> buf((size_t)B * 2);
  std::vector<int16_t> audio;
  std::vector<int8_t> iq;
  const auto t0 = std::chrono::steady_clock::now();
  long long reads = 0;
  int rc_exit = 0;
  aerohost::SectionTimer tm;  // AERO_HOST_TIMING: loop-section totals at exit
  tm.restart();
  while (g_running.load()) {
    size_t got = fread(buf.data(), sizeof(float), buf.size(), src);
    if (got < buf.size()) {
      if (loop && fseek(src, 0, SEEK_SET) == 0) {
        got += fread(buf.data() + got, sizeof(float), buf.size() - got, src);
      }
      if (got < buf.size()) break;  // end of the recording: readStream fails (publisher.cpp:267-271)
    }
    if (realtime) {
      const auto due = t0 + std::chrono::microseconds((long long)(1e6 * (double)reads * B / Fs));
      std::this_thread::sleep_until(due);
    }
    tm.mark("read");
    // Publisher::demodData -> vfo::process -> transmitData
    int rc = aero_chan_push(chan, buf.data(), 1, 0);
    tm.mark("push");
    if (!rc) rc = aero_chan_run(chan);
    tm.mark("run");
    if (!rc) rc = aero_chan_sync(chan);
    tm.mark("sync");
    if (rc) {
      AH_CRIT("channeliser error: %s", aero_strerror(rc));
      rc_exit = 1;
      break;
    }
    for (size_t m = 0; m < mains.size(); m++) {
      if (has_subs[m]) {
        for (size_t v = 0; v < vfos.size(); v++) {
          if (parent[v] != (int)m) continue;
          size_t n = 0;
          audio.resize(1 << 20);
          aero_chan_pop_audio(chan, (int)v, audio.data(), audio.size(), &n);
          tm.mark("pop");
          bound.publish(audio.data(), n * sizeof(int16_t), topics[v], (uint32_t)rate[v]);
          tm.mark("publish");
          tm.count("messages");
        }
      } else if (mains[m].publish) {
        int info[3];
        aero_chan_main_info(chan, (int)m, info);
        iq.resize(1 << 22);
        size_t n = 0;
        aero_chan_pop_iq(chan, (int)m, iq.data(), iq.size(), &n);
        main_pub[m].publish(iq.data(), n, main_topic[m], (uint32_t)info[0]);
      }
    }
    reads++;
    tm.count("reads");
    tm.mark("publish");
  }
  tm.print("aero-publish");
  AH_DBG("reader stopped after %lld reads", reads);
  fclose(src);
  int linger = 2000;
  if (bound.sock) z->setsockopt(bound.sock, ZMQ_LINGER_, &linger, sizeof linger);
  bound.close();
  for (auto &p : main_pub) {
    if (p.sock) z->setsockopt(p.sock, ZMQ_LINGER_, &linger, sizeof linger);
    p.close();
  }
  z->ctx_term(ctx);
  aero_chan_destroy(chan);
  return rc_exit;
}
