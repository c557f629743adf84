// burst_engine.h — the burst-mode group's entry points for engine.hip
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

#include "../../include/aero_engine.h"

namespace aero {

struct BurstGroup;
class HostPool;
enum BurstKind { BURST_OQPSK = 0, BURST_MSK = 1 };  // 10500 OQPSK / 600-1200 MSK (both bit rates in one group)
int burst_group_create(int device, int flags, int max_channels, int kind, BurstGroup **out);
void burst_group_destroy(BurstGroup *g);
int burst_open(BurstGroup *g, int bitrate, bool disable_reassembly, int *local);
int burst_push(BurstGroup *g, int c, const int16_t *pcm, size_t n, bool dev, bool msg_start);
int burst_push_batch(BurstGroup *g, const int16_t *src, size_t n, size_t ld, int nch, bool dev);
int burst_run(BurstGroup *g, int flush);
int burst_sync(BurstGroup *g);
int burst_pop_soft(BurstGroup *g, int c, int16_t *dst, size_t cap, size_t *n);
int burst_pop_hops(BurstGroup *g, int c, double *dst, size_t cap_records, size_t *n);
int burst_pop_tests(BurstGroup *g, int c, uint8_t *dst, size_t cap, size_t *n);
int burst_pop_packets(BurstGroup *g, int c, uint8_t *dst, size_t cap, size_t *n);
std::vector<aero_acars_item> &burst_items(BurstGroup *g, int c);
uint64_t burst_processed(const BurstGroup *g);
uint64_t burst_stat(const BurstGroup *g, int which);  // 0: R/T tests run, 1: R/T packets decoded, 2: most tests of one pass
int burst_dcd_edges(BurstGroup *g, int c, int64_t *edges);  // AeroL datacd changes (waits for the group's work)
void burst_timing(BurstGroup *g, const char *name, double *ms, long *launches);  // adds to *ms / *launches
void burst_timing_reset(BurstGroup *g);
void burst_group_set_pool(BurstGroup *g, HostPool *pool);  // host threads for the R/T tests (the engine's)

}  // namespace aero
