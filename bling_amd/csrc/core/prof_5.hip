// prof_5.hip -- kernels of feature profile kProfiles[5] (core_internal.h), compiled as their own unit:
// the traversal / compaction pipeline; prof_5a / b / c.hip compile its shading kernels.
#include "core_wave.h"
BLING_INSTANTIATE_PROFILE_SPLIT(5)
