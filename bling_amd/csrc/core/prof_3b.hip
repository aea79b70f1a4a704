// prof_3b.hip -- k_shade<F, false> (depth 0) and k_shade_dl of feature profile kProfiles[3]
// (core_wave.h), its own unit so the build compiles it beside prof_3.hip.
#ifndef BCR_HUGE_ARGS
#define BCR_HUGE_ARGS 0   // no computed textures: sin / cos arguments are angles (cr_math.h)
#endif
#include "core_wave.h"
BLING_INSTANTIATE_SHADE(3, false)
BLING_INSTANTIATE_SHADE_DL(3)
