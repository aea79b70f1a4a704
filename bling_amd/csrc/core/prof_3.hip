// prof_3.hip -- kernels of feature profile kProfiles[3] (core_internal.h), compiled as their own unit.
#include "core_wave.h"
BLING_INSTANTIATE_PROFILE(3)
