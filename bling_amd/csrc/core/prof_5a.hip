// prof_5a.hip -- the fused resolve + shade kernel k_shade<F, true> of feature profile kProfiles[5]
// (core_wave.h), its own unit so the build compiles it beside prof_5.hip.
#include "core_wave.h"
BLING_INSTANTIATE_SHADE(5, true)
