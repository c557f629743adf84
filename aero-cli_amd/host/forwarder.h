/*
 * forwarder.h — ForwardTarget (decode/forwarder.h:14-41, decode/forwarder.cpp:20-184):
 * FORMAT=tcp|udp://host:port targets that receive every item in their own
 * output format, reconnecting once on a failed send.
 */
#pragma once
#include <netdb.h>

#include <memory>
#include <string>

#include "output.h"

namespace aerohost {

class ForwardTarget {
 public:
  ForwardTarget(const std::string &scheme, const std::string &host, int port, OutputFormat fmt, std::string url);
  ~ForwardTarget();
  ForwardTarget(const ForwardTarget &) = delete;
  ForwardTarget &operator=(const ForwardTarget &) = delete;

  void reconnect();
  void send(const std::string &data);  // Latin-1 bytes
  OutputFormat format() const { return fmt_; }
  const std::string &url() const { return url_; }

  // ForwardTarget::fromRaw ("FORMAT=URL"); nullptr + a CRIT line when malformed
  static std::unique_ptr<ForwardTarget> from_raw(const std::string &raw);

 private:
  int send_frame(const std::string &data);
  std::string scheme_, host_, url_;
  int port_;
  int connfd_ = -1;
  addrinfo *servinfo_ = nullptr, *activeinfo_ = nullptr;
  OutputFormat fmt_;
};

}  // namespace aerohost
