// prof_5c.hip -- k_shade_dl (DirectLighting) of feature profile kProfiles[5]
// (core_wave.h), its own unit so the build compiles it beside prof_5.hip.
#include "core_wave.h"
BLING_INSTANTIATE_SHADE_DL(5)
