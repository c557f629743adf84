#include "forwarder.h"

#include <sys/socket.h>
#include <unistd.h>

#include <cctype>
#include <cstring>
#include <vector>

#include "log.h"

namespace aerohost {

ForwardTarget::ForwardTarget(const std::string &scheme, const std::string &host, int port, OutputFormat fmt,
                             std::string url)
    : scheme_(scheme), host_(host), url_(std::move(url)), port_(port), fmt_(fmt) {}

ForwardTarget::~ForwardTarget() {
  if (servinfo_) freeaddrinfo(servinfo_);
  if (connfd_ != -1) ::close(connfd_);
}

// ForwardTarget::reconnect (decode/forwarder.cpp:39-107)
void ForwardTarget::reconnect() {
  AH_DBG("Attempting to connect to forwarder target %s", url_.c_str());
  if (servinfo_) {
    freeaddrinfo(servinfo_);
    servinfo_ = nullptr;
    activeinfo_ = nullptr;
  }
  if (connfd_ != -1) {
    ::close(connfd_);
    connfd_ = -1;
  }
  addrinfo hints;
  memset(&hints, 0, sizeof hints);
  hints.ai_family = AF_INET;
  hints.ai_socktype = scheme_ == "tcp" ? SOCK_STREAM : SOCK_DGRAM;
  const std::string port = std::to_string(port_);
  if (getaddrinfo(host_.c_str(), port.c_str(), &hints, &servinfo_) == 0) {
    for (addrinfo *p = servinfo_; p; p = p->ai_next) {
      connfd_ = ::socket(p->ai_family, p->ai_socktype, p->ai_protocol);
      if (connfd_ == -1) continue;
      if (scheme_ == "tcp" && ::connect(connfd_, p->ai_addr, p->ai_addrlen) == -1) {
        ::close(connfd_);
        connfd_ = -1;
        continue;
      }
      activeinfo_ = p;
      break;
    }
  }
  if (connfd_ == -1)
    AH_DBG("Failed to connect to forwarder target");
  else
    AH_DBG("Connected to forwarder target");
}

// sendFrame (:109-121): strlen() of the payload, so an embedded NUL ends it
int ForwardTarget::send_frame(const std::string &data) {
  const size_t n = strlen(data.c_str());
  if (connfd_ == -1) return -1;
  if (scheme_ == "tcp") return (int)::send(connfd_, data.c_str(), n, MSG_NOSIGNAL);
  if (!activeinfo_) return -1;
  return (int)::sendto(connfd_, data.c_str(), n, 0, activeinfo_->ai_addr, activeinfo_->ai_addrlen);
}

// ForwardTarget::send (:123-150)
void ForwardTarget::send(const std::string &data) {
  AH_DBG("Attempting to send %zu bytes to forwarding target %s", data.size(), url_.c_str());
  if (connfd_ == -1) {
    AH_DBG("Invalid socket detected, attempting reconnect");
    reconnect();
  }
  int w = send_frame(data);
  if (w == -1) {
    reconnect();
    if (connfd_ == -1) {
      AH_DBG("Failed attempt to reconnect to forwarding target during send()");
      return;
    }
    w = send_frame(data);
    if (w == -1) AH_DBG("Failed again to send frame to forwarding target");
  } else {
    AH_DBG("Sent %d to forwarding target", w);
  }
}

// ForwardTarget::fromRaw (:152-184) with QUrl's scheme://host:port parsing
std::unique_ptr<ForwardTarget> ForwardTarget::from_raw(const std::string &raw) {
  if (raw.empty()) return nullptr;
  std::vector<std::string> tok;
  size_t s = 0;
  for (;;) {
    const size_t e = raw.find('=', s);
    tok.push_back(raw.substr(s, e == std::string::npos ? std::string::npos : e - s));
    if (e == std::string::npos) break;
    s = e + 1;
  }
  if (tok.size() != 2) {
    AH_CRIT("Malformed forwarding target syntax: %s", raw.c_str());
    return nullptr;
  }
  const OutputFormat fmt = parse_output_format(tok[0]);
  if (fmt == OutputFormat::None) {
    AH_CRIT("Forwarding target format is invalid: %s", tok[0].c_str());
    return nullptr;
  }
  const std::string &url = tok[1];
  if (url.empty()) {
    AH_CRIT("Forwarding target URL is empty");
    return nullptr;
  }
  const size_t sp = url.find("://");
  std::string scheme = sp == std::string::npos ? "" : url.substr(0, sp);
  for (auto &ch : scheme) ch = (char)tolower((unsigned char)ch);
  const std::string rest = sp == std::string::npos ? url : url.substr(sp + 3);
  if (sp == std::string::npos || scheme.empty() || !isalpha((unsigned char)scheme[0])) {
    AH_CRIT("Forwarding target scheme is unsupported: %s", scheme.c_str());
    return nullptr;
  }
  if (scheme != "tcp" && scheme != "udp") {
    AH_CRIT("Forwarding target scheme is unsupported: %s", scheme.c_str());
    return nullptr;
  }
  // authority = [userinfo@]host[:port], up to the first '/', '?' or '#'
  std::string auth = rest.substr(0, rest.find_first_of("/?#"));
  const size_t at = auth.rfind('@');
  if (at != std::string::npos) auth = auth.substr(at + 1);
  std::string host = auth;
  int port = -1;
  const size_t colon = auth.rfind(':');
  if (colon != std::string::npos && auth.find(']') == std::string::npos) {
    host = auth.substr(0, colon);
    const std::string ps = auth.substr(colon + 1);
    if (ps.empty() || ps.size() > 5 || ps.find_first_not_of("0123456789") != std::string::npos ||
        atoi(ps.c_str()) > 65535) {
      AH_CRIT("Forwarding target URL is invalid: %s", url.c_str());
      return nullptr;
    }
    port = atoi(ps.c_str());
  }
  if (host.empty()) {
    AH_CRIT("Forwarding target URL is missing host");
    return nullptr;
  }
  if (port == -1) {
    AH_CRIT("Forwarding target URL is missing port");
    return nullptr;
  }
  return std::unique_ptr<ForwardTarget>(new ForwardTarget(scheme, host, port, fmt, url));
}

}  // namespace aerohost
