/*
 * host_capi.cpp — C entry to the host's output formatter (libaero_host.so),
 * so the formats can be checked without a GPU or a ZMQ session
 * (tests/test_host_output.py against the Qt-generated fixture).
 */
#include <cstring>

#include "output.h"

using namespace aerohost;

extern "C" {

/* toOutputFormat of one item; fmt 1 text, 2 jaero, 3 jsondump (OutputFormat
 * order).  Writes the UTF-8 line (no newline, NUL-terminated when it fits)
 * and returns its length, or -1 for an unknown format. */
long aero_host_format(int fmt, const char *station_utf8, int disable_reassembly, const aero_acars_item *item,
                      long long ms_since_epoch, char *out, size_t cap) {
  if (fmt < 1 || fmt > 3 || !item) return -1;
  ustr line;
  if (!to_output_format((OutputFormat)fmt, from_utf8(station_utf8 ? station_utf8 : ""), disable_reassembly != 0,
                        *item, ms_since_epoch, line))
    return -1;
  const std::string u = to_utf8(line);
  if (out && cap) {
    const size_t k = u.size() < cap - 1 ? u.size() : cap - 1;
    memcpy(out, u.data(), k);
    out[k] = 0;
  }
  return (long)u.size();
}

/* the Latin-1 bytes a forwarder sends for that line (QString::toLatin1) */
long aero_host_format_latin1(int fmt, const char *station_utf8, int disable_reassembly, const aero_acars_item *item,
                             long long ms_since_epoch, char *out, size_t cap) {
  if (fmt < 1 || fmt > 3 || !item) return -1;
  ustr line;
  if (!to_output_format((OutputFormat)fmt, from_utf8(station_utf8 ? station_utf8 : ""), disable_reassembly != 0,
                        *item, ms_since_epoch, line))
    return -1;
  const std::string l = to_latin1(line);
  if (out && cap) {
    const size_t k = l.size() < cap ? l.size() : cap;
    memcpy(out, l.data(), k);
  }
  return (long)l.size();
}
}
