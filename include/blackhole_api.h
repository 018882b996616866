/* blackhole_api.h -- drop-in name for callers written against the reference engine's headers
 * (include/blackhole_api.h of Klaudiusz321/raytracing-engine-in-c). Everything libbhrt.so provides
 * for the ray-tracing path is declared once, in bhrt_api.h. */
#ifndef BHRT_COMPAT_BLACKHOLE_API_H
#define BHRT_COMPAT_BLACKHOLE_API_H
#include "bhrt_api.h"
#endif
