/*
 * output.h — aero-decode's console / forwarder formats (decode/output.cpp:12-171,
 * decode/forwarder.cpp:7-18) over the engine's aero_acars_item.
 */
#pragma once
#include <cstdint>
#include <string>

#include "../../include/aero_engine.h"
#include "qstr.h"

namespace aerohost {

enum class OutputFormat { None, Text, Jaero, JsonDump };  // decode/forwarder.h:12

// parseOutputFormat (decode/forwarder.cpp:7-18): case-insensitive
OutputFormat parse_output_format(const std::string &raw);

// toOutputFormat (decode/output.cpp:12-171) at wall time `ms_since_epoch`
// (UTC); returns false for OutputFormat::None.  app_name/app_ver stand for
// QCoreApplication's ("aero-decode", "0.0.1", decode/main.cpp:14-15).
bool to_output_format(OutputFormat fmt, const ustr &station_id, bool disable_reassembly, const aero_acars_item &item,
                      long long ms_since_epoch, ustr &out);

// wall clock in ms; AERO_DECODE_FIXED_TIME_MS=<ms> pins it (tests only)
long long now_ms();

}  // namespace aerohost
