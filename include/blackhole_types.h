/* blackhole_types.h -- drop-in name for callers written against the reference engine's headers
 * (include/blackhole_types.h of Klaudiusz321/raytracing-engine-in-c). Everything libbhrt.so provides
 * for the ray-tracing path is declared once, in bhrt_api.h. */
#ifndef BHRT_COMPAT_BLACKHOLE_TYPES_H
#define BHRT_COMPAT_BLACKHOLE_TYPES_H
#include "bhrt_api.h"
#endif
