// prof_3.hip -- kernels of feature profile kProfiles[3] (core_internal.h), compiled as their own unit:
// the traversal / compaction pipeline; prof_3a.hip and prof_3b.hip compile its shading kernels.
#ifndef BCR_HUGE_ARGS
#define BCR_HUGE_ARGS 0   // no computed textures: sin / cos arguments are angles (cr_math.h)
#endif
#include "core_wave.h"
BLING_INSTANTIATE_PROFILE_SPLIT(3)
