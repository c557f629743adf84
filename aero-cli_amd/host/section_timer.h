/*
 * section_timer.h — wall-clock totals of a host binary's loop sections
 * (read, push, run, publish, ...), printed as one JSON line on stderr at
 * exit when AERO_HOST_TIMING is set (bench.py --mode c5bin reads them).
 * Diagnostics only: no effect on output.
 */
#pragma once
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <string>

namespace aerohost {

class SectionTimer {
 public:
  SectionTimer() : on_(getenv("AERO_HOST_TIMING") != nullptr) {}
  bool on() const { return on_; }
  // adds the time since the previous mark (or construction) to `name`
  void mark(const char *name) {
    if (!on_) return;
    const auto now = std::chrono::steady_clock::now();
    if (started_) ms_[name] += std::chrono::duration<double, std::milli>(now - last_).count();
    last_ = now;
    started_ = true;
  }
  void restart() {
    if (on_) {
      last_ = std::chrono::steady_clock::now();
      started_ = true;
    }
  }
  void count(const char *name, long long n = 1) {
    if (on_) counts_[name] += n;
  }
  void print(const char *who) const {
    if (!on_) return;
    std::string s = std::string("{\"aero_host_timing\": \"") + who + "\", \"ms\": {";
    bool first = true;
    char buf[96];
    for (auto &kv : ms_) {
      snprintf(buf, sizeof buf, "%s\"%s\": %.3f", first ? "" : ", ", kv.first.c_str(), kv.second);
      s += buf;
      first = false;
    }
    s += "}, \"counts\": {";
    first = true;
    for (auto &kv : counts_) {
      snprintf(buf, sizeof buf, "%s\"%s\": %lld", first ? "" : ", ", kv.first.c_str(), kv.second);
      s += buf;
      first = false;
    }
    s += "}}";
    fprintf(stderr, "%s\n", s.c_str());
  }

 private:
  bool on_, started_ = false;
  std::chrono::steady_clock::time_point last_;
  std::map<std::string, double> ms_;
  std::map<std::string, long long> counts_;
};

}  // namespace aerohost
