/*
 * qstr.h — the few QString behaviours aero-decode's output depends on,
 * restated on std::u16string (UTF-16 code units, as QString holds them):
 * Latin-1 / UTF-8 conversions, QString::arg's lowest-escape substitution
 * (Qt qstring.cpp findArgEscapes / replaceArgEscapes), QString::mid and
 * replace, and QJsonDocument's compact writer (sorted keys, Qt's string
 * escapes).  Used by output.cpp (decode/output.cpp:12-171).
 */
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace aerohost {

using ustr = std::u16string;

ustr from_latin1(const char *s, size_t n);
ustr from_latin1(const std::string &s);
// QString::fromUtf8: one U+FFFD per byte of an invalid sequence
ustr from_utf8(const std::string &s);
std::string to_utf8(const ustr &s);
// QString::toLatin1: '?' for code points above 0xFF
std::string to_latin1(const ustr &s);

// QString::arg(a, fieldWidth, fill): replaces every occurrence of the
// lowest-numbered %n (n = 0..99, optional 'L') with a, padded to
// |fieldWidth| (right-aligned for positive widths); unchanged when the
// string holds no escape
ustr qarg(const ustr &s, const ustr &a, int field_width = 0, char16_t fill = u' ');
ustr qmid(const ustr &s, long pos, long n = -1);
ustr qreplace(const ustr &s, const ustr &before, const ustr &after);
// QString("%1").arg(v, width, base, fill).toUpper() (output.cpp:8-10)
ustr upper_hex(uint64_t v, int width);

// QJsonValue / QJsonObject subset: string, integer, bool, object
struct JVal;
using JObj = std::map<ustr, JVal>;
struct JVal {
  enum Kind { STR, INT, BOOL, OBJ } kind = STR;
  ustr s;
  long long i = 0;
  bool b = false;
  std::shared_ptr<JObj> o;
  JVal() = default;
  JVal(const ustr &v) : kind(STR), s(v) {}
  JVal(long long v) : kind(INT), i(v) {}
  JVal(bool v) : kind(BOOL), b(v) {}
  JVal(const JObj &v) : kind(OBJ), o(std::make_shared<JObj>(v)) {}
};
// QJsonDocument(obj).toJson(QJsonDocument::Compact), as UTF-8
std::string json_compact(const JObj &o);

}  // namespace aerohost
