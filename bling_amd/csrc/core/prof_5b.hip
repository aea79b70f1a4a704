// prof_5b.hip -- k_shade<F, false> (depth 0) of feature profile kProfiles[5]
// (core_wave.h), its own unit so the build compiles it beside prof_5.hip.
#include "core_wave.h"
BLING_INSTANTIATE_SHADE(5, false)
