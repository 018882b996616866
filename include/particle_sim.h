/* particle_sim.h -- drop-in name for callers written against the reference engine's headers
 * (include/particle_sim.h of Klaudiusz321/raytracing-engine-in-c). Its types are in
 * bhrt_types.h and its functions in bhrt_api.h. */
#ifndef BHRT_COMPAT_PARTICLE_SIM_H
#define BHRT_COMPAT_PARTICLE_SIM_H
#include "bhrt_api.h"
#endif
