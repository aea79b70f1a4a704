// prof_1.hip -- kernels of feature profile kProfiles[1] (core_internal.h), compiled as their own unit.
#ifndef BCR_HUGE_ARGS
#define BCR_HUGE_ARGS 0   // no computed textures: sin / cos arguments are angles (cr_math.h)
#endif
#include "core_wave.h"
BLING_INSTANTIATE_PROFILE(1)
