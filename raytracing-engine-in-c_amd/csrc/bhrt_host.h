/*
 * bhrt_host.h -- internals shared by the C host files of libbhrt.so (bhrt_api.c,
 * particles.c). Not installed; hidden visibility.
 */
#ifndef BHRT_HOST_H
#define BHRT_HOST_H

#include "../../include/bhrt_api.h"

/* per-thread error message read back by bhrt_last_error() */
void bhrt_set_err(const char* fmt, ...) __attribute__((format(printf, 1, 2)));

/* BHContextHandle (blackhole_api.c:26-31) */
struct BHContext_t {
    BlackHoleParams blackhole;
    AccretionDiskParams disk;
    SimulationConfig config;
    int disk_enabled;
};

#endif
