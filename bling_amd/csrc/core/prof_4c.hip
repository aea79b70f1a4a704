// prof_4c.hip -- k_shade_dl (DirectLighting) of feature profile kProfiles[4]
// (core_wave.h), its own unit so the build compiles it beside prof_4.hip.
#ifndef BCR_HUGE_ARGS
#define BCR_HUGE_ARGS 0   // no computed textures: sin / cos arguments are angles (cr_math.h)
#endif
#include "core_wave.h"
BLING_INSTANTIATE_SHADE_DL(4)
