/*
 * output.cpp — toOutputFormat (decode/output.cpp:12-171) restated over the
 * engine's POD item.  QString semantics (arg chaining, mid, replace, JSON
 * writer) come from qstr.cpp.  Field conversions follow the reference's
 * Qt 6 build: message is Latin-1 text (QString += char, decode/aerol.cpp:450),
 * PLANEREG and TAKstr are QByteArray -> QString (UTF-8), MODE / BI / label
 * characters are QChar(char) (Latin-1).  `parsed` (libacars) is never set.
 */
#include "output.h"

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <ctime>

namespace aerohost {

OutputFormat parse_output_format(const std::string &raw) {
  std::string n;
  for (char c : raw) n.push_back((char)tolower((unsigned char)c));
  if (n == "text") return OutputFormat::Text;
  if (n == "jaero") return OutputFormat::Jaero;
  if (n == "jsondump") return OutputFormat::JsonDump;
  return OutputFormat::None;
}

long long now_ms() {
  if (const char *f = getenv("AERO_DECODE_FIXED_TIME_MS")) return atoll(f);
  return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::system_clock::now().time_since_epoch())
      .count();
}

namespace {

ustr U(const char *s) { return from_latin1(s, strlen(s)); }
ustr qchar(unsigned char c) { return ustr(1, (char16_t)c); }

// QDateTime::toString on the UTC time (only the fields the formats use)
ustr fmt_time(long long ms, bool iso) {
  time_t sec = (time_t)(ms >= 0 ? ms / 1000 : (ms - 999) / 1000);
  struct tm t;
  gmtime_r(&sec, &t);
  char b[64];
  if (iso)  // "yyyy-MM-ddThh:mm:ssZ" (T and Z are literals)
    snprintf(b, sizeof b, "%04d-%02d-%02dT%02d:%02d:%02dZ", t.tm_year + 1900, t.tm_mon + 1, t.tm_mday, t.tm_hour,
             t.tm_min, t.tm_sec);
  else  // "yyyy-MM-dd hh:mm:ss"
    snprintf(b, sizeof b, "%04d-%02d-%02d %02d:%02d:%02d", t.tm_year + 1900, t.tm_mon + 1, t.tm_mday, t.tm_hour,
             t.tm_min, t.tm_sec);
  return U(b);
}

}  // namespace

bool to_output_format(OutputFormat fmt, const ustr &station_id, bool disable_reassembly, const aero_acars_item &item,
                      long long ms, ustr &out) {
  if (fmt == OutputFormat::None) return false;
  // TAKstr (output.cpp:24-27): the TAK byte, "!" for NAK
  std::string takb(1, (char)item.tak);
  if (item.tak == 0x15) takb = "!";
  const ustr tak = from_utf8(takb);
  // label[1], with DEL shown as 'd' (:29-34)
  unsigned char label1 = ' ';
  if (item.label_len > 1) {
    label1 = (unsigned char)item.label[1];
    if (label1 == 127) label1 = 'd';
  }
  const unsigned char label0 = item.label_len > 0 ? (unsigned char)item.label[0] : 0;
  const ustr reg = from_utf8(std::string(item.reg, item.reg_len));
  const ustr msg0 = from_latin1(item.msg, item.msg_len);
  const long long secs = ms >= 0 ? ms / 1000 : (ms - 999) / 1000;

  if (fmt == OutputFormat::JsonDump || fmt == OutputFormat::Jaero) {
    JObj root;
    ustr message = msg0;
    message = qreplace(message, u"\r", u"\n");
    message = qreplace(message, u"\n\n", u"\n");
    if (!message.empty() && message.back() == u'\n') message.pop_back();
    if (!message.empty() && message.front() == u'\n') message.erase(0, 1);
    message = qreplace(message, u"\n", u"\n\t");
    const ustr label = qarg(qarg(u"%1%2", qchar(label0)), qchar(label1));
    if (fmt == OutputFormat::JsonDump) {
      JObj app{{u"name", JVal(ustr(u"aero-decode"))}, {u"ver", JVal(ustr(u"0.0.1"))}};
      root[u"app"] = JVal(app);
      JObj isu, aes, ges;
      aes[u"type"] = JVal(ustr(u"Aircraft Earth Station"));
      aes[u"addr"] = JVal(upper_hex(item.aesid, 6));
      ges[u"type"] = JVal(ustr(u"Ground Earth Station"));
      ges[u"addr"] = JVal(upper_hex(item.gesid, 2));
      if (!item.nonacars) {
        JObj acars;
        acars[u"mode"] = JVal(qchar(item.mode));
        acars[u"ack"] = JVal(tak);
        acars[u"blk_id"] = JVal(qchar(item.bi));
        acars[u"label"] = JVal(label);
        acars[u"reg"] = JVal(reg);
        if (!message.empty()) {
          if (item.downlink) {
            acars[u"msg_num"] = JVal(qmid(message, 0, 3));
            acars[u"msg_num_seq"] = JVal(qmid(message, 3, 1));
            acars[u"flight"] = JVal(qmid(message, 4, 6));
            acars[u"msg_text"] = JVal(qmid(message, 4 + 6));
          } else {
            acars[u"msg_text"] = JVal(message);
          }
        }
        isu[u"acars"] = JVal(acars);
      }
      isu[u"refno"] = JVal(upper_hex(item.refno, 2));
      isu[u"qno"] = JVal(upper_hex(item.qno, 2));
      isu[u"src"] = JVal(item.downlink ? aes : ges);
      isu[u"dst"] = JVal(item.downlink ? ges : aes);
      JObj t{{u"sec", JVal(secs)}, {u"usec", JVal((long long)((ms % 1000) * 1000))}};
      root[u"t"] = JVal(t);
      root[u"isu"] = JVal(isu);
      root[u"station"] = JVal(station_id);
    } else {
      root[u"TIME"] = JVal(secs);
      root[u"TIME_UTC"] = JVal(fmt_time(ms, false));
      root[u"NAME"] = JVal(ustr(u"aero-decode"));
      root[u"NONACARS"] = JVal((bool)item.nonacars);
      root[u"AESID"] = JVal(upper_hex(item.aesid, 6));
      root[u"GESID"] = JVal(upper_hex(item.gesid, 2));
      root[u"QNO"] = JVal(upper_hex(item.qno, 2));
      root[u"REFNO"] = JVal(upper_hex(item.refno, 2));
      root[u"REG"] = JVal(reg);
      if (!item.nonacars) {
        root[u"MODE"] = JVal(qchar(item.mode));
        root[u"TAK"] = JVal(tak);
        root[u"LABEL"] = JVal(label);
        root[u"BI"] = JVal(qchar(item.bi));
      }
    }
    out = from_utf8(json_compact(root));
    return true;
  }
  // Text (output.cpp:131-166)
  ustr message = msg0;
  message = qreplace(message, u"\n", u"\\n");
  message = qreplace(message, u"\r", u"\\r");
  message = qreplace(message, u"\t", u"\\t");
  message = qreplace(message, u"\a", u"\\a");
  out = qarg(qarg(qarg(u"%1 AES:%2 GES:%3", fmt_time(ms, true)), upper_hex(item.aesid, 6)), upper_hex(item.gesid, 6));
  if (!item.nonacars) {
    out += qarg(qarg(qarg(u" [%1] ACK=%2 BLK=%3 ", reg, 7), tak, 1), qchar(item.bi));
    if (disable_reassembly) out += qarg(u"M=%1 ", item.moretocome ? u"1" : u"0");
    out += qarg(qarg(u"LBL=%1%2 ", qchar(label0)), qchar(label1));
    if (!message.empty()) {
      if (item.downlink)
        out += qarg(qarg(qarg(u"MSN=%1 FLT=%2 %3", qmid(message, 0, 4)), qmid(message, 4, 6)), qmid(message, 10));
      else
        out += qarg(u"%1", message);
    }
  }
  return true;
}

}  // namespace aerohost
