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
 *  - libacars enrichment (`parsed`) is absent (libacars is not in the image);
 *  - a continuous MSK channel re-applies its settings at a message's rate as
 *    MskDemodulator::dataReceived does (decode/mskdemodulator.cpp:473-481)
 *    for 12000, 24000 and 48000 Hz; a message at another rate is dropped
 *    with a CRIT line;
 *  - the verbose DCD / frequency-centre lines (decode/decode.cpp:429-439)
 *    are printed after each engine run, not as the demodulator emits them;
 *  - extension: several -t options decode several topics in one process,
 *    one engine channel per topic (-b / -s once, or once per topic); every
 *    message queued on the socket is pushed before one aero_run;
 *  - AERO_ZMQ_HWM sets the SUB socket's receive high-water mark (0 =
 *    unbounded) for publishers running faster than real time.
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
#include "section_timer.h"
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
  // QCommandLineParser keeps every occurrence of an option: the reference
  // reads value(), the last one; repeated -t / -b / -s select the
  // multi-topic mode (one process, one engine channel per topic)
  std::vector<std::string> bitrate, fwd, publisher, station, topic, format;
  bool verbose = false, burst = false, disable_reassembly = false, no_signal_exit = false;
};

const std::string &last(const std::vector<std::string> &v) {
  static const std::string none;
  return v.empty() ? none : v.back();
}

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
    "                               a VFO\n"
    "\n"
    "Several -t options decode several VFO topics in one process on one engine\n"
    "(-b and -s then given once, or once per topic in the same order).\n";

// QCommandLineParser (decode/main.cpp:17-51): -x value, -xvalue, --name value,
// --name=value; an unknown option or a missing value ends the program with 1
bool parse_args(int argc, char **argv, Options &o) {
  struct Opt {
    const char *s, *l;
    std::vector<std::string> *val;
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
      hit->val->push_back(inl);
    } else if (i + 1 < argc) {
      hit->val->push_back(argv[++i]);
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

// one subscribed VFO topic: its engine channel and what aero-decode keeps
// per Decoder (decode/decode.cpp:72-115)
struct Topic {
  std::string name;
  int bitrate = 0;
  uint32_t fs = 0;
  ustr station;
  int ch = -1;
  bool live = true;               // still decoding (--no-signal-exit stops a topic)
  long long scans_seen = 0;       // SignalHunter full scans reported
  long long dcd_seen = 0, steps_seen = 0;  // status events logged
};

int main(int argc, char **argv) {
  Options o;
  parse_args(argc, argv, o);
  g_verbose = o.verbose;
  if (last(o.publisher).empty()) {
    AH_CRIT("Required publisher option is missing, example: -p tcp://127.0.0.1:6004");
    return 1;
  }
  const std::string publisher = last(o.publisher);
  const bool multi = o.topic.size() > 1;
  if (o.station.empty() || last(o.station).empty()) {
    o.station = {hostname_upper() + "-AERO-INMARSAT"};
    AH_WARN("No station ID provided, using generated default %s", o.station[0].c_str());
  }
  if (last(o.topic).empty()) {
    AH_CRIT("Required topic option is missing, example: -t VFO51");
    return 1;
  }
  const std::string format = o.format.empty() ? std::string("text") : last(o.format);
  // one topic: the reference's last-value semantics; several: -b / -s given
  // once for all topics or once per topic
  std::vector<Topic> topics;
  if (multi) {
    for (const auto *v : {&o.bitrate, &o.station})
      if (v->size() > 1 && v->size() != o.topic.size()) {
        AH_CRIT("With %zu topics, -b and -s are given once or once per topic", o.topic.size());
        return 0;
      }
    for (size_t k = 0; k < o.topic.size(); k++) {
      Topic t;
      t.name = o.topic[k];
      t.bitrate = atoi((o.bitrate.size() > 1 ? o.bitrate[k] : last(o.bitrate)).c_str());
      t.station = from_utf8(o.station.size() > 1 ? o.station[k] : last(o.station));
      topics.push_back(t);
    }
  } else {
    Topic t;
    t.name = last(o.topic);
    t.bitrate = atoi(last(o.bitrate).c_str());  // QString::toInt: 0 when not a number
    t.station = from_utf8(last(o.station));
    topics.push_back(t);
  }

  // Decoder::Decoder (decode/decode.cpp:72-115): a bad configuration logs and
  // leaves the decoder stopped; the application then completes with status 0
  for (auto &t : topics)
    if (t.bitrate != 600 && t.bitrate != 1200 && t.bitrate != 10500) {
      AH_CRIT("Unsupported bit rate: %d", t.bitrate);
      return 0;
    }
  const OutputFormat fmt = parse_output_format(format);
  if (fmt == OutputFormat::None) {
    AH_CRIT("Invalid output format provided: %s", format.c_str());
    return 0;
  }
  const std::string fwd_raw = last(o.fwd);
  std::vector<std::vector<std::unique_ptr<ForwardTarget>>> targets(topics.size());
  if (!fwd_raw.empty()) {
    for (auto &tv : targets) {
      size_t s = 0;
      for (;;) {
        const size_t e = fwd_raw.find(',', s);
        auto t = ForwardTarget::from_raw(fwd_raw.substr(s, e == std::string::npos ? std::string::npos : e - s));
        if (!t) {
          AH_CRIT("Some forwarders configuration may be malformed: %s", fwd_raw.c_str());
          return 0;
        }
        tv.push_back(std::move(t));
        if (e == std::string::npos) break;
        s = e + 1;
      }
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
  // the engine: one channel per topic (its demodulator + AeroL + hunter);
  // every aero_run advances all of them in the same batched launches
  aero_engine *eng = nullptr;
  const char *dev = getenv("AERO_DEVICE");
  // the reference runs Qt's event loop (decode/main.cpp:106), so AeroL's 1 s
  // DCD timer fires (decode/aerol.cpp:900-902): the engine runs it on the
  // sample clock.  AERO_DCD_TICK=0 turns it off (the timer-less behaviour of
  // a reference without an event loop; test support)
  const char *tick = getenv("AERO_DCD_TICK");
  const int eflags = (tick && atoi(tick) == 0) ? 0 : AERO_F_DCD_TICK;
  aero_engine_cfg ecfg{dev ? atoi(dev) : 0, (int)topics.size(), eflags};
  if (int rc = aero_engine_create(&ecfg, &eng)) {
    AH_CRIT("Failed to create the MI355X demodulation engine: %s", aero_strerror(rc));
    return 1;
  }
  for (auto &t : topics) {
    t.fs = t.bitrate == 600 ? 12000 : (t.bitrate == 1200 ? 24000 : 48000);
    aero_channel_cfg ccfg{t.bitrate, o.burst ? 1 : 0, t.fs, o.disable_reassembly ? 1 : 0};
    if (int rc = aero_channel_open(eng, &ccfg, &t.ch)) {
      AH_CRIT("Unsupported channel configuration (bit rate %d%s): %s", t.bitrate, o.burst ? ", burst" : "",
              aero_strerror(rc));
      aero_engine_destroy(eng);
      return 1;
    }
  }
  std::vector<int> topic_of(topics.size());
  for (size_t k = 0; k < topics.size(); k++) topic_of[topics[k].ch] = (int)k;
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

  std::vector<std::unique_ptr<Forwarders>> fwd;
  for (size_t k = 0; k < topics.size(); k++)
    fwd.emplace_back(new Forwarders(std::move(targets[k]), topics[k].station, o.disable_reassembly));
  std::vector<aero_acars_item> items(64);
  std::vector<int> item_ch(items.size());
  // handleACARS (decode/decode.cpp:441-455): console line, then the forwarders
  auto drain = [&]() {
    size_t n = 0;
    do {
      if (aero_pop_items_all(eng, items.data(), item_ch.data(), items.size(), &n)) break;
      for (size_t i = 0; i < n; i++) {
        const int k = topic_of[item_ch[i]];
        const long long ms = now_ms();
        ustr out;
        if (!to_output_format(fmt, topics[k].station, o.disable_reassembly, items[i], ms, out)) {
          AH_CRIT("Failed to generate output format!");
          continue;
        }
        AH_INF("%s", to_utf8(out).c_str());
        fwd[k]->push(items[i], ms);
      }
    } while (n == items.size());
  };

  // publisherConsumer (decode/decode.cpp:283-366)
  const int buf_size = 192000;
  std::vector<char> samples(buf_size);
  int rc_exit = 0;
  AH_DBG("Connecting to ZMQ endpoint at %s", publisher.c_str());
  if (const char *h = getenv("AERO_ZMQ_HWM")) {  // as aero-publish: 0 = unbounded receive queue
    const int hwm = atoi(h);
    z->setsockopt(sub, ZMQ_RCVHWM_, &hwm, sizeof hwm);
  }
  if (z->connect(sub, publisher.c_str()) == -1) {
    AH_CRIT("Failed to connect to publisher, error code: %d; is aero-publish or SDRReceiver running?", -1);
    g_running.store(0);
  } else {
    for (auto &t : topics) {
      AH_DBG("Subscribing to ZMQ topic %s", t.name.c_str());
      if (z->setsockopt(sub, ZMQ_SUBSCRIBE_, t.name.c_str(), strlen(t.name.c_str())) == -1) {
        AH_CRIT("Failed to subscribe to %s; error code = %d", t.name.c_str(), z->errno_());
        g_running.store(0);
        break;
      }
    }
  }
  // in multi-topic mode a log line about one VFO names its topic
  auto tag = [&](const Topic &t) { return multi ? " [" + t.name + "]" : std::string(); };
  // Decoder::handleDcdChange / handleNewFreqCenter (decode/decode.cpp:429-439):
  // verbose only, polled with the scan check (about once a second) and at exit
  auto log_events = [&]() {
    if (!g_verbose) return;
    for (auto &t : topics) {
      aero_channel_events ev;
      if (aero_channel_get_events(eng, t.ch, &ev) != AERO_OK) continue;
      for (long long k = t.dcd_seen + 1; k <= ev.dcd_edges; k++) {
        if (k & 1)
          AH_DBG("Data carrier detected: no signal => signal%s", tag(t).c_str());
        else
          AH_DBG("Data carrier lost: signal => no signal%s", tag(t).c_str());
      }
      t.dcd_seen = ev.dcd_edges;
      for (long long k = std::max(t.steps_seen + 1, (long long)ev.hunter_steps - 7); k <= ev.hunter_steps; k++)
        AH_DBG("Trying frequency center %.1f in search of signal%s", ev.hunter_fc[(k - 1) & 7], tag(t).c_str());
      t.steps_seen = ev.hunter_steps;
    }
  };
  // SignalHunter::noSignalAfterScan -> handleNoSignalAfterFullScan
  // (decode/decode.cpp:418-427), polled about once a second
  long long last_check = 0;
  auto check_scans = [&]() {
    const long long now = std::chrono::duration_cast<std::chrono::milliseconds>(
                              std::chrono::steady_clock::now().time_since_epoch())
                              .count();
    if (last_check && now - last_check < 1000) return;
    last_check = now;
    log_events();
    bool any_live = false;
    for (auto &t : topics) {
      int64_t scans = 0;
      if (t.live && aero_channel_stat(eng, t.ch, "hunter_scans", &scans) == AERO_OK && scans > t.scans_seen) {
        t.scans_seen = scans;
        AH_WARN("Scanned entire VFO bandwidth and could not find a signal.%s", tag(t).c_str());
        if (o.no_signal_exit) {
          AH_WARN("Please confirm and verify that the specified topic is correct and that aero-publish is using "
                  "correct settings%s", tag(t).c_str());
          t.live = false;  // a reference process per topic: this one exits
        }
      }
      any_live |= t.live;
    }
    if (!any_live) {
      g_running.store(0);
      AH_FATAL("Exiting because of no signal");  // the application then completes (status 0)
    }
  };
  if (g_running.load()) AH_DBG("Listening for samples...");
  char tbuf[256];
  aerohost::SectionTimer tm;  // AERO_HOST_TIMING: loop-section totals at exit
  tm.restart();
  while (g_running.load()) {
    int n;
    while ((n = z->recv(sub, tbuf, sizeof tbuf, ZMQ_DONTWAIT_)) < 0 && g_running.load()) {
      usleep(10000);
      check_scans();
    }
    tm.mark("wait");
    if (!g_running.load()) break;
    // every message already queued goes in before one aero_run (the engine
    // re-blocks continuous channels into hop segments, burst channels keep
    // each message's boundaries), at most 256 per run
    int rc = AERO_OK;
    for (int batch = 0; n >= 0 && g_running.load();) {
      unsigned char rate_buf[4];
      const int tlen = n < (int)sizeof tbuf ? n : (int)sizeof tbuf;
      n = z->recv(sub, rate_buf, sizeof rate_buf, ZMQ_DONTWAIT_);
      if (n == (int)sizeof rate_buf) {
        uint32_t rate;
        memcpy(&rate, rate_buf, 4);
        n = z->recv(sub, samples.data(), buf_size, ZMQ_DONTWAIT_);
        if (n >= 0) {
          const size_t bytes = (size_t)(n < buf_size ? n : buf_size);
          // ZMQ's prefix match: the message goes to every topic it matches
          // (one reference process per topic would each receive it)
          for (auto &t : topics) {
            if (!t.live || (int)t.name.size() > tlen || memcmp(tbuf, t.name.data(), t.name.size())) continue;
            // emit audioReceived -> dataReceived: len/2 int16 samples
            tm.mark("recv");
            rc = aero_push_pcm(eng, t.ch, reinterpret_cast<const int16_t *>(samples.data()), bytes / 2, rate);
            tm.mark("push");
            tm.count("messages");
            if (rc == AERO_E_RATE) {
              // the engine re-applies an MSK channel's settings at 12000,
              // 24000 or 48000 Hz (mskdemodulator.cpp:473-481); other rates
              // are dropped
              AH_CRIT("Sample rate %u is not one the MSK demodulator can be set to (12000, 24000, 48000); "
                      "message dropped%s", rate, tag(t).c_str());
              rc = AERO_OK;
            }
            if (rc) break;
          }
        }
      }
      if (rc || ++batch >= 256) break;
      n = z->recv(sub, tbuf, sizeof tbuf, ZMQ_DONTWAIT_);
    }
    tm.mark("recv");
    if (!g_running.load()) break;
    if (rc || (rc = aero_run(eng))) {
      AH_CRIT("engine error: %s", aero_strerror(rc));
      rc_exit = 1;
      break;
    }
    tm.mark("run");
    drain();
    tm.mark("drain");
    check_scans();
    tm.mark("events");
    tm.count("batches");
  }
  // the tail of what was received
  if (aero_flush(eng) == AERO_OK) {
    drain();
    log_events();
  }
  tm.mark("flush");
  tm.print("aero-decode");
  for (auto &f : fwd) f->stop();
  aero_engine_destroy(eng);
  z->close(sub);
  z->ctx_term(ctx);
  return rc_exit;
}
