/*
 * engine_internal.h — entry points shared between the engine and the
 * channeliser inside libaero_engine.so (not part of the C ABI).
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/aero_engine.h"

/* Pushes nitems device PCM runs (channel ch[i], src[i], n[i] samples at rate
 * fs[i]) without a host wait: the engine's streams wait for `ready` (recorded
 * on `producer` after the audio was written), one gather launch per channel
 * kind fills the PCM rings, and `producer` then waits for those launches
 * before it may overwrite the sources.  Burst channels take a synchronous
 * per-message copy. */
int aero_engine_feed_dev(aero_engine *e, int nitems, const int *ch, const int16_t *const *src, const size_t *n,
                         const uint32_t *fs, hipEvent_t ready, hipStream_t producer);

/* AERO_E_INVALID (with a message) unless p is a device pointer of this
 * process's HIP runtime */
int check_dev_ptr(const void *p);
