/* raytracer.h -- drop-in name for callers written against the reference engine's headers
 * (include/raytracer.h of Klaudiusz321/raytracing-engine-in-c). Everything libbhrt.so provides
 * for the ray-tracing path is declared once, in bhrt_api.h. */
#ifndef BHRT_COMPAT_RAYTRACER_H
#define BHRT_COMPAT_RAYTRACER_H
#include "bhrt_api.h"
#endif
