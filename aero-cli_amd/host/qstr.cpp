/*
 * qstr.cpp — see qstr.h.
 */
#include "qstr.h"

#include <climits>
#include <cstdio>
#include <cstring>

namespace aerohost {

ustr from_latin1(const char *s, size_t n) {
  ustr r;
  r.reserve(n);
  for (size_t i = 0; i < n; i++) r.push_back((char16_t)(unsigned char)s[i]);
  return r;
}

ustr from_latin1(const std::string &s) { return from_latin1(s.data(), s.size()); }

ustr from_utf8(const std::string &s) {
  ustr r;
  const unsigned char *p = (const unsigned char *)s.data();
  const size_t n = s.size();
  size_t i = 0;
  while (i < n) {
    const unsigned c = p[i];
    int len = 0;
    uint32_t cp = 0, minv = 0;
    if (c < 0x80) {
      r.push_back((char16_t)c);
      i++;
      continue;
    } else if ((c & 0xE0) == 0xC0) {
      len = 2, cp = c & 0x1F, minv = 0x80;
    } else if ((c & 0xF0) == 0xE0) {
      len = 3, cp = c & 0x0F, minv = 0x800;
    } else if ((c & 0xF8) == 0xF0) {
      len = 4, cp = c & 0x07, minv = 0x10000;
    }
    bool ok = len > 0 && i + len <= n;
    for (int k = 1; ok && k < len; k++) {
      if ((p[i + k] & 0xC0) != 0x80)
        ok = false;
      else
        cp = (cp << 6) | (p[i + k] & 0x3F);
    }
    if (ok && (cp < minv || cp > 0x10FFFF || (cp >= 0xD800 && cp <= 0xDFFF))) ok = false;
    if (!ok) {
      r.push_back(u'�');
      i++;
      continue;
    }
    if (cp >= 0x10000) {
      cp -= 0x10000;
      r.push_back((char16_t)(0xD800 + (cp >> 10)));
      r.push_back((char16_t)(0xDC00 + (cp & 0x3FF)));
    } else {
      r.push_back((char16_t)cp);
    }
    i += len;
  }
  return r;
}

std::string to_utf8(const ustr &s) {
  std::string r;
  for (size_t i = 0; i < s.size(); i++) {
    uint32_t cp = s[i];
    if (cp >= 0xD800 && cp <= 0xDBFF && i + 1 < s.size() && s[i + 1] >= 0xDC00 && s[i + 1] <= 0xDFFF) {
      cp = 0x10000 + ((cp - 0xD800) << 10) + (s[i + 1] - 0xDC00);
      i++;
    } else if (cp >= 0xD800 && cp <= 0xDFFF) {
      cp = 0xFFFD;
    }
    if (cp < 0x80) {
      r.push_back((char)cp);
    } else if (cp < 0x800) {
      r.push_back((char)(0xC0 | (cp >> 6)));
      r.push_back((char)(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
      r.push_back((char)(0xE0 | (cp >> 12)));
      r.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
      r.push_back((char)(0x80 | (cp & 0x3F)));
    } else {
      r.push_back((char)(0xF0 | (cp >> 18)));
      r.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
      r.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
      r.push_back((char)(0x80 | (cp & 0x3F)));
    }
  }
  return r;
}

std::string to_latin1(const ustr &s) {
  std::string r;
  r.reserve(s.size());
  for (size_t i = 0; i < s.size(); i++) {
    const char16_t c = s[i];
    if (c >= 0xD800 && c <= 0xDBFF && i + 1 < s.size() && s[i + 1] >= 0xDC00 && s[i + 1] <= 0xDFFF) i++;
    r.push_back(c > 0xFF ? '?' : (char)c);
  }
  return r;
}

namespace {
// QChar::digitValue over the code points a Latin-1 message can hold:
// ASCII digits and the superscripts two, three and one (Unicode digits)
int digit_value(char16_t c) {
  if (c >= u'0' && c <= u'9') return c - u'0';
  if (c == 0xB2) return 2;
  if (c == 0xB3) return 3;
  if (c == 0xB9) return 1;
  return -1;
}
}  // namespace

ustr qarg(const ustr &s, const ustr &a, int field_width, char16_t fill) {
  // findArgEscapes
  int min_escape = INT_MAX;
  const size_t n = s.size();
  for (size_t c = 0; c < n;) {
    while (c < n && s[c] != u'%') ++c;
    if (c >= n) break;
    if (++c >= n) break;
    if (s[c] == u'L')
      if (++c >= n) break;
    int escape = digit_value(s[c]);
    if (escape == -1) continue;
    ++c;
    if (c < n) {
      const int nx = digit_value(s[c]);
      if (nx != -1) {
        escape = 10 * escape + nx;
        ++c;
      }
    }
    if (escape < min_escape) min_escape = escape;
  }
  if (min_escape == INT_MAX) return s;  // "QString::arg: Argument missing"
  ustr pad = a;
  const size_t w = (size_t)(field_width < 0 ? -field_width : field_width);
  if (pad.size() < w) {
    if (field_width > 0)
      pad = ustr(w - a.size(), fill) + a;
    else
      pad = a + ustr(w - a.size(), fill);
  }
  // replaceArgEscapes: every occurrence of min_escape, scanning as above
  ustr out;
  for (size_t c = 0; c < n;) {
    const size_t text_start = c;
    while (c < n && s[c] != u'%') ++c;
    out.append(s, text_start, c - text_start);
    if (c >= n) break;
    const size_t escape_start = c;
    if (++c >= n) {
      out.append(s, escape_start, c - escape_start);
      break;
    }
    if (s[c] == u'L')
      if (++c >= n) {
        out.append(s, escape_start, c - escape_start);
        break;
      }
    int escape = digit_value(s[c]);
    if (escape != -1 && c + 1 < n) {
      const int nx = digit_value(s[c + 1]);
      if (nx != -1) {
        escape = 10 * escape + nx;
        ++c;
      }
    }
    if (escape != min_escape) {
      // not ours: copy what was scanned (the digit itself stays for the next pass)
      out.append(s, escape_start, c - escape_start);
      continue;
    }
    ++c;
    out.append(pad);
  }
  return out;
}

ustr qmid(const ustr &s, long pos, long n) {
  const long size = (long)s.size();
  if (pos > size) return ustr();
  if (pos < 0) {
    if (n < 0 || n + pos >= size) return s;
    if (n + pos <= 0) return ustr();
    n += pos;
    pos = 0;
  } else if ((unsigned long)n > (unsigned long)(size - pos)) {
    n = size - pos;
  }
  return s.substr((size_t)pos, (size_t)n);
}

ustr qreplace(const ustr &s, const ustr &before, const ustr &after) {
  if (before.empty()) return s;
  ustr out;
  size_t i = 0;
  for (;;) {
    const size_t j = s.find(before, i);
    if (j == ustr::npos) break;
    out.append(s, i, j - i);
    out.append(after);
    i = j + before.size();
  }
  out.append(s, i, ustr::npos);
  return out;
}

ustr upper_hex(uint64_t v, int width) {
  char b[32];
  snprintf(b, sizeof b, "%0*llX", width, (unsigned long long)v);
  return from_latin1(b, strlen(b));
}

namespace {
// QJsonPrivate::Writer escapedString (Qt 5 qjsonwriter.cpp): ", \ and
// controls below 0x20 escaped (\b \f \n \r \t, else \u00xx lowercase hex),
// everything else as UTF-8
void json_string(std::string &o, const ustr &s) {
  static const char hex[] = "0123456789abcdef";
  o.push_back('"');
  ustr t;
  for (char16_t u : s) {
    if (u < 0x80) {
      if (u < 0x20 || u == 0x22 || u == 0x5c) {
        o.append(to_utf8(t));
        t.clear();
        o.push_back('\\');
        switch (u) {
          case 0x22: o.push_back('"'); break;
          case 0x5c: o.push_back('\\'); break;
          case 0x08: o.push_back('b'); break;
          case 0x0c: o.push_back('f'); break;
          case 0x0a: o.push_back('n'); break;
          case 0x0d: o.push_back('r'); break;
          case 0x09: o.push_back('t'); break;
          default:
            o.push_back('u');
            o.push_back('0');
            o.push_back('0');
            o.push_back(hex[u >> 4]);
            o.push_back(hex[u & 0xF]);
        }
        continue;
      }
    }
    t.push_back(u);
  }
  o.append(to_utf8(t));
  o.push_back('"');
}

void json_obj(std::string &o, const JObj &obj) {
  o.push_back('{');
  bool first = true;
  for (auto &kv : obj) {
    if (!first) o.push_back(',');
    first = false;
    json_string(o, kv.first);
    o.push_back(':');
    const JVal &v = kv.second;
    switch (v.kind) {
      case JVal::STR: json_string(o, v.s); break;
      case JVal::INT: o.append(std::to_string(v.i)); break;
      case JVal::BOOL: o.append(v.b ? "true" : "false"); break;
      case JVal::OBJ: json_obj(o, *v.o); break;
    }
  }
  o.push_back('}');
}
}  // namespace

std::string json_compact(const JObj &o) {
  std::string r;
  json_obj(r, o);
  return r;
}

}  // namespace aerohost
