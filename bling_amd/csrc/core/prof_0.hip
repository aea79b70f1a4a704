// prof_0.hip -- kernels of feature profile kProfiles[0] (core_internal.h), compiled as their own unit.
#include "core_wave.h"
BLING_INSTANTIATE_PROFILE(0)
