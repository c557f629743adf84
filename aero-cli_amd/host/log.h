/*
 * log.h — common/logger.h's macros: qDebug lines on stderr, colour-tagged
 * except INF; DBG only with -v (gMaxLogVerbosity).
 */
#pragma once
#include <cstdio>

namespace aerohost {
extern bool g_verbose;
}

// the line and its newline under one stream lock (the forwarder thread logs too)
#define AH_INF(...) (flockfile(stderr), fprintf(stderr, __VA_ARGS__), fputc('\n', stderr), funlockfile(stderr))
#define AH_DBG(fmt, ...) \
  (aerohost::g_verbose ? (fprintf(stderr, "\033[1;34m[DEBUG] " fmt "\033[0m\n", ##__VA_ARGS__), 0) : 0)
#define AH_WARN(fmt, ...) fprintf(stderr, "\033[1;33m[WARN] " fmt "\033[0m\n", ##__VA_ARGS__)
#define AH_CRIT(fmt, ...) fprintf(stderr, "\033[1;31m[CRITICAL] " fmt "\033[0m\n", ##__VA_ARGS__)
#define AH_FATAL(fmt, ...) fprintf(stderr, "\033[1;31m[FATAL] " fmt "\033[0m\n", ##__VA_ARGS__)
