/*
 * aero_decode.cpp — drop-in replacement for the reference's aero-decode
 * binary (decode/main.cpp:12-107, decode/decode.cpp:72-471) with the DSP
 * chain on the MI355X engine (include/aero_engine.h).
 *
 * Same command line, same ZeroMQ subscription and wire format
 * ([topic][u32 LE sample rate][int16 LE PCM], receive buffer 192000 bytes,
 * decode/decode.cpp:283-366), same console lines (INF of toOutputFormat,
 * :441-455) and the same forwarders (:368-416, decode/forwarder.cpp).
 * Differences, all deliberate:
 *  - a message longer than the 192000-byte buffer is truncated to it (the
 *    reference copies recvSize bytes out of the 192000-byte buffer);
 *  - on SIGINT / SIGTERM the samples already received are flushed through
 *    the engine and their items printed and forwarded before exit (the
 *    reference's synchronous chain has no tail to flush);
 *  - libacars enrichment (`parsed`) is absent (libacars is not in the image).
 */
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/aero_engine.h"
#include "forwarder.h"
#include "log.h"
#include "output.h"
#include "zmq_dl.h"

namespace aerohost {
bool g_verbose = false;
}
using namespace aerohost;

namespace {

std::atomic<int> g_running{0};

// a crash prints the native stack before the default action (diagnostics)
void on_fatal(int sig) {
  void *bt[64];
  const int n = backtrace(bt, 64);
  fprintf(stderr, "aero-decode: fatal signal %d\n", sig);
  backtrace_symbols_fd(bt, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

void on_signal(int sig) {
  if (sig == SIGINT || sig == SIGTERM) g_running.store(0);  // handleInterrupt / handleTerminate
}

struct Options {
  std::string bitrate, fwd, publisher, station, topic, format;
  bool verbose = false, burst = false, disable_reassembly = false, no_signal_exit = false;
};

const char *kUsage =
    "Usage: aero-decode [options]\n"
    "Demodulate and decode VFOs over ZMQ from SDRReceiver or aero-publish into SatCom ACARS messages\n"
    "\n"
    "Options:\n"
    "  -h, --help                   Displays help on commandline options.\n"
    "  --help-all                   Displays help including Qt specific options.\n"
    "  -b, --bit-rate <bit-rate>    Signal bit rate, valid rates: 600, 1200, 10500\n"
    "  -f, --fwd <fwd>              Forward decoded ACARS messages to a list of\n"
    "                               servers and formats, see --format for allowable\n"
    "                               formats; example: FORMAT1=URL1,FORMAT2=URL2,...\n"
    "  -p, --publisher <publisher>  URL of aero-publish or SDRReceiver publishing\n"
    "                               ZeroMQ server\n"
    "  -s, --station-id <station-id>  Station ID for feeding\n"
    "  -t, --topic <topic>          ZeroMQ VFO topic name\n"
    "  -v, --verbose                Show verbose output\n"
    "  --burst                      Enable burst mode (C-band)\n"
    "  --disable-reassembly         Disable frame reassembly\n"
    "  --format <format>            ACARS format type to display on console; valid:\n"
    "                               jaero, jsondump, text (default)\n"
    "  --no-signal-exit             Exit if no signal is found after a full scan of\n"
    "                               a VFO\n";

// QCommandLineParser (decode/main.cpp:17-51): -x value, -xvalue, --name value,
// --name=value; an unknown option or a missing value ends the program with 1
bool parse_args(int argc, char **argv, Options &o) {
  struct Opt {
    const char *s, *l;
    std::string *val;
    bool *flag;
  } opts[] = {{"b", "bit-rate", &o.bitrate, nullptr},     {"f", "fwd", &o.fwd, nullptr},
              {"p", "publisher", &o.publisher, nullptr},  {"s", "station-id", &o.station, nullptr},
              {"t", "topic", &o.topic, nullptr},          {"v", "verbose", nullptr, &o.verbose},
              {nullptr, "burst", nullptr, &o.burst},      {nullptr, "disable-reassembly", nullptr, &o.disable_reassembly},
              {nullptr, "format", &o.format, nullptr},    {nullptr, "no-signal-exit", nullptr, &o.no_signal_exit}};
  for (int i = 1; i < argc; i++) {
    std::string a = argv[i];
    if (a == "-h" || a == "--help" || a == "-?" || a == "--help-all") {
      fputs(kUsage, stdout);
      exit(0);
    }
    Opt *hit = nullptr;
    std::string inl;
    bool has_inl = false;
    if (a.rfind("--", 0) == 0) {
      std::string name = a.substr(2);
      const size_t eq = name.find('=');
      if (eq != std::string::npos) {
        inl = name.substr(eq + 1);
        has_inl = true;
        name = name.substr(0, eq);
      }
      for (auto &x : opts)
        if (name == x.l) hit = &x;
      if (!hit) {
        fprintf(stderr, "Unknown option '%s'.\n", name.c_str());
        exit(1);
      }
    } else if (a.size() > 1 && a[0] == '-') {
      const std::string name = a.substr(1, 1);
      for (auto &x : opts)
        if (x.s && name == x.s) hit = &x;
      if (!hit) {
        fprintf(stderr, "Unknown option '%s'.\n", name.c_str());
        exit(1);
      }
      if (a.size() > 2) {
        if (hit->val) {
          inl = a.substr(2);
          has_inl = true;
        } else {  // compacted short flags: -v only takes no value
          fprintf(stderr, "Unknown option '%s'.\n", a.substr(2, 1).c_str());
          exit(1);
        }
      }
    } else {
      continue;  // positional arguments are ignored by the reference
    }
    if (hit->flag) {
      *hit->flag = true;
    } else if (has_inl) {
      *hit->val = inl;
    } else if (i + 1 < argc) {
      *hit->val = argv[++i];
    } else {
      fprintf(stderr, "Missing value after '%s'.\n", a.c_str());
      exit(1);
    }
  }
  return true;
}

// sendBuffer + forwarderConsumer (decode/decode.cpp:368-416)
class Forwarders {
 public:
  Forwarders(std::vector<std::unique_ptr<ForwardTarget>> t, ustr station, bool disable_reassembly)
      : targets_(std::move(t)), station_(std::move(station)), dr_(disable_reassembly) {
    th_ = std::thread([this] { loop(); });
  }
  ~Forwarders() { stop(); }
  void push(const aero_acars_item &it, long long ms) {
    std::lock_guard<std::mutex> g(m_);
    q_.push_back({it, ms});
    cv_.notify_all();
  }
  void stop() {  // sends what is queued, then ends the thread
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    if (th_.joinable()) th_.join();
  }

 private:
  void loop() {
    for (auto &t : targets_) t->reconnect();
    for (;;) {
      std::pair<aero_acars_item, long long> it;
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [this] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;
        it = q_.front();
        q_.pop_front();
      }
      for (auto &t : targets_) {
        ustr out;
        if (to_output_format(t->format(), station_, dr_, it.first, it.second, out)) {
          out += u"\n";
          t->send(to_latin1(out));
        }
      }
    }
  }
  std::vector<std::unique_ptr<ForwardTarget>> targets_;
  ustr station_;
  bool dr_;
  std::mutex m_;
  std::condition_variable cv_;
  std::deque<std::pair<aero_acars_item, long long>> q_;
  bool stop_ = false;
  std::thread th_;
};

std::string hostname_upper() {
  char b[256] = {0};
  gethostname(b, sizeof b - 1);
  std::string s = b;
  for (auto &c : s) c = (char)toupper((unsigned char)c);
  return s;
}

}  // namespace

int main(int argc, char **argv) {
  Options o;
  parse_args(argc, argv, o);
  g_verbose = o.verbose;
  if (o.publisher.empty()) {
    AH_CRIT("Required publisher option is missing, example: -p tcp://127.0.0.1:6004");
    return 1;
  }
  if (o.station.empty()) {
    o.station = hostname_upper() + "-AERO-INMARSAT";
    AH_WARN("No station ID provided, using generated default %s", o.station.c_str());
  }
  if (o.topic.empty()) {
    AH_CRIT("Required topic option is missing, example: -t VFO51");
    return 1;
  }
  if (o.format.empty()) o.format = "text";
  const int bitrate = atoi(o.bitrate.c_str());  // QString::toInt: 0 when not a number

  // Decoder::Decoder (decode/decode.cpp:72-115): a bad configuration logs and
  // leaves the decoder stopped; the application then completes with status 0
  if (bitrate != 600 && bitrate != 1200 && bitrate != 10500) {
    AH_CRIT("Unsupported bit rate: %d", bitrate);
    return 0;
  }
  const OutputFormat fmt = parse_output_format(o.format);
  if (fmt == OutputFormat::None) {
    AH_CRIT("Invalid output format provided: %s", o.format.c_str());
    return 0;
  }
  std::vector<std::unique_ptr<ForwardTarget>> targets;
  if (!o.fwd.empty()) {
    size_t s = 0;
    for (;;) {
      const size_t e = o.fwd.find(',', s);
      auto t = ForwardTarget::from_raw(o.fwd.substr(s, e == std::string::npos ? std::string::npos : e - s));
      if (!t) {
        AH_CRIT("Some forwarders configuration may be malformed: %s", o.fwd.c_str());
        return 0;
      }
      targets.push_back(std::move(t));
      if (e == std::string::npos) break;
      s = e + 1;
    }
  }
  const Zmq *z = zmq_load();
  if (!z) return 1;
  void *ctx = z->ctx_new();
  if (!ctx) {
    AH_CRIT("Failed to create new ZeroMQ context, error code = %d", z->errno_());
    return 0;
  }
  void *sub = z->socket(ctx, ZMQ_SUB_);
  if (!sub) {
    AH_CRIT("Failed to create ZeroMQ socket, error code = %d", z->errno_());
    return 0;
  }
  // the engine: one channel, this topic's demodulator + AeroL + hunter
  aero_engine *eng = nullptr;
  const char *dev = getenv("AERO_DEVICE");
  aero_engine_cfg ecfg{dev ? atoi(dev) : 0, 1, 0};
  if (int rc = aero_engine_create(&ecfg, &eng)) {
    AH_CRIT("Failed to create the MI355X demodulation engine: %s", aero_strerror(rc));
    return 1;
  }
  const uint32_t fs_cfg = bitrate == 600 ? 12000 : (bitrate == 1200 ? 24000 : 48000);
  aero_channel_cfg ccfg{bitrate, o.burst ? 1 : 0, fs_cfg, o.disable_reassembly ? 1 : 0};
  int ch = -1;
  if (int rc = aero_channel_open(eng, &ccfg, &ch)) {
    AH_CRIT("Unsupported channel configuration (bit rate %d%s): %s", bitrate, o.burst ? ", burst" : "",
            aero_strerror(rc));
    aero_engine_destroy(eng);
    return 1;
  }
  g_running.store(1);
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_handler = on_signal;
  sigaction(SIGINT, &sa, nullptr);
  sigaction(SIGTERM, &sa, nullptr);
  signal(SIGHUP, SIG_IGN);  // handleHup: nothing to do
  signal(SIGSEGV, on_fatal);
  signal(SIGBUS, on_fatal);
  signal(SIGABRT, on_fatal);
  signal(SIGPIPE, SIG_IGN);

  const ustr station = from_utf8(o.station);
  Forwarders fwd(std::move(targets), station, o.disable_reassembly);
  std::vector<aero_acars_item> items(16);
  // handleACARS (decode/decode.cpp:441-455): console line, then the forwarders
  auto drain = [&]() {
    size_t n = 0;
    do {
      if (aero_pop_items(eng, ch, items.data(), items.size(), &n)) break;
      for (size_t i = 0; i < n; i++) {
        const long long ms = now_ms();
        ustr out;
        if (!to_output_format(fmt, station, o.disable_reassembly, items[i], ms, out)) {
          AH_CRIT("Failed to generate output format!");
          continue;
        }
        AH_INF("%s", to_utf8(out).c_str());
        fwd.push(items[i], ms);
      }
    } while (n == items.size());
  };

  // publisherConsumer (decode/decode.cpp:283-366)
  const int buf_size = 192000;
  std::vector<char> samples(buf_size);
  int rc_exit = 0;
  long long scans_seen = 0, last_check = 0;
  AH_DBG("Connecting to ZMQ endpoint at %s", o.publisher.c_str());
  if (z->connect(sub, o.publisher.c_str()) == -1) {
    AH_CRIT("Failed to connect to publisher, error code: %d; is aero-publish or SDRReceiver running?", -1);
    g_running.store(0);
  } else {
    AH_DBG("Subscribing to ZMQ topic %s", o.topic.c_str());
    if (z->setsockopt(sub, ZMQ_SUBSCRIBE_, o.topic.c_str(), strlen(o.topic.c_str())) == -1) {
      AH_CRIT("Failed to subscribe to %s; error code = %d", o.topic.c_str(), z->errno_());
      g_running.store(0);
    }
  }
  // SignalHunter::noSignalAfterScan -> handleNoSignalAfterFullScan
  // (decode/decode.cpp:418-427), polled about once a second
  auto check_scans = [&]() {
    const long long t = std::chrono::duration_cast<std::chrono::milliseconds>(
                            std::chrono::steady_clock::now().time_since_epoch()).count();
    if (last_check && t - last_check < 1000) return;
    last_check = t;
    int64_t scans = 0;
    if (aero_channel_stat(eng, ch, "hunter_scans", &scans) == AERO_OK && scans > scans_seen) {
      scans_seen = scans;
      AH_WARN("Scanned entire VFO bandwidth and could not find a signal.");
      if (o.no_signal_exit) {
        AH_WARN("Please confirm and verify that the specified topic is correct and that aero-publish is using "
                "correct settings");
        g_running.store(0);
        AH_FATAL("Exiting because of no signal");  // the application then completes (status 0)
      }
    }
  };
  if (g_running.load()) AH_DBG("Listening for samples...");
  while (g_running.load()) {
    int n;
    while ((n = z->recv(sub, nullptr, 0, ZMQ_DONTWAIT_)) < 0 && g_running.load()) {
      usleep(10000);
      check_scans();
    }
    if (!g_running.load()) break;
    unsigned char rate_buf[4];
    n = z->recv(sub, rate_buf, sizeof rate_buf, ZMQ_DONTWAIT_);
    if (n != (int)sizeof rate_buf) continue;
    uint32_t rate;
    memcpy(&rate, rate_buf, 4);
    n = z->recv(sub, samples.data(), buf_size, ZMQ_DONTWAIT_);
    if (!g_running.load()) break;
    if (n < 0) continue;
    const size_t bytes = (size_t)(n < buf_size ? n : buf_size);
    // emit audioReceived -> dataReceived: len/2 int16 samples
    int rc = aero_push_pcm(eng, ch, reinterpret_cast<const int16_t *>(samples.data()), bytes / 2, rate);
    if (rc == AERO_E_RATE) {
      AH_CRIT("Sample rate %u differs from the %u Hz this bit rate's demodulator runs at", rate, fs_cfg);
      continue;
    }
    if (rc || (rc = aero_run(eng))) {
      AH_CRIT("engine error: %s", aero_strerror(rc));
      rc_exit = 1;
      break;
    }
    drain();
    check_scans();
  }
  // the tail of what was received
  if (aero_flush(eng) == AERO_OK) drain();
  fwd.stop();
  aero_engine_destroy(eng);
  z->close(sub);
  z->ctx_term(ctx);
  return rc_exit;
}
