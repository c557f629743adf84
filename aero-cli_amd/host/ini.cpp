#include "ini.h"

#include <cerrno>
#include <cstdlib>
#include <fstream>

namespace aerohost {

namespace {
std::string trim(const std::string &s) {
  size_t a = 0, b = s.size();
  while (a < b && (s[a] == ' ' || s[a] == '\t' || s[a] == '\r')) a++;
  while (b > a && (s[b - 1] == ' ' || s[b - 1] == '\t' || s[b - 1] == '\r')) b--;
  return s.substr(a, b - a);
}
// QSettings unquotes "..." values
std::string unquote(const std::string &v) {
  if (v.size() >= 2 && v.front() == '"' && v.back() == '"') return v.substr(1, v.size() - 2);
  return v;
}
}  // namespace

bool Ini::load(const std::string &path) {
  std::ifstream f(path);
  if (!f) return false;
  std::string line, cur = "General";
  while (std::getline(f, line)) {
    line = trim(line);
    if (line.empty() || line[0] == ';' || line[0] == '#') continue;
    if (line.front() == '[' && line.back() == ']') {
      cur = trim(line.substr(1, line.size() - 2));
      continue;
    }
    const size_t eq = line.find('=');
    if (eq == std::string::npos) continue;
    std::string k = trim(line.substr(0, eq));
    // QSettings writes the array separator as '\'; '/' reads the same
    for (auto &c : k)
      if (c == '/') c = '\\';
    sec_[cur][k] = unquote(trim(line.substr(eq + 1)));
  }
  return true;
}

std::string Ini::value(const std::string &key, const std::string &group) const {
  auto s = sec_.find(group);
  if (s == sec_.end()) return "";
  auto v = s->second.find(key);
  return v == s->second.end() ? "" : v->second;
}

int Ini::to_int(const std::string &v) {  // QVariant(QString)::toInt: whole text base 10, else 0
  if (v.empty()) return 0;
  char *end = nullptr;
  errno = 0;
  const long r = strtol(v.c_str(), &end, 10);
  if (errno || *end || r > 2147483647L || r < -2147483648L) return 0;
  return (int)r;
}

float Ini::to_float(const std::string &v) {
  if (v.empty()) return 0.f;
  char *end = nullptr;
  const double r = strtod(v.c_str(), &end);
  if (*end) return 0.f;
  return (float)r;
}

int Ini::value_int(const std::string &key, const std::string &group) const { return to_int(value(key, group)); }
float Ini::value_float(const std::string &key, const std::string &group) const {
  return to_float(value(key, group));
}

std::vector<std::map<std::string, std::string>> Ini::array(const std::string &name) const {
  std::vector<std::map<std::string, std::string>> out;
  auto s = sec_.find(name);
  if (s == sec_.end()) return out;
  const int n = to_int(value("size", name));
  for (int i = 1; i <= n; i++) {
    const std::string pre = std::to_string(i) + "\\";
    std::map<std::string, std::string> e;
    for (auto &kv : s->second)
      if (kv.first.compare(0, pre.size(), pre) == 0) e[kv.first.substr(pre.size())] = kv.second;
    out.push_back(e);
  }
  return out;
}

}  // namespace aerohost
