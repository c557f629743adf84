/*
 * ini.h — the part of QSettings(IniFormat) Publisher::loadSettings reads
 * (publish/publisher.cpp:55-227): [General] keys (keys before any section
 * land there) and the main_vfos / vfos arrays (size=N, i\key=value,
 * 1-based), with QVariant::toInt / toFloat conversions (0 on bad text).
 */
#pragma once
#include <map>
#include <string>
#include <vector>

namespace aerohost {

class Ini {
 public:
  bool load(const std::string &path);
  std::string value(const std::string &key, const std::string &group = "General") const;
  int value_int(const std::string &key, const std::string &group = "General") const;
  float value_float(const std::string &key, const std::string &group = "General") const;
  // beginReadArray(name) + setArrayIndex(i): entry i's keys (i from 0)
  std::vector<std::map<std::string, std::string>> array(const std::string &name) const;
  static int to_int(const std::string &v);
  static float to_float(const std::string &v);

 private:
  std::map<std::string, std::map<std::string, std::string>> sec_;
};

}  // namespace aerohost
