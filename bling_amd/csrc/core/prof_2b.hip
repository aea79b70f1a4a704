// prof_2b.hip -- k_shade<F, false> (depth 0) and k_shade_dl of feature profile kProfiles[2]
// (core_wave.h), its own unit so the build compiles it beside prof_2.hip.
#ifndef BCR_HUGE_ARGS
#define BCR_HUGE_ARGS 0   // no computed textures: sin / cos arguments are angles (cr_math.h)
#endif
// The sun-sky profile calls the shared transcendentals out of line, one copy of each instead of one
// per call site (cr_math.h BCR_API): its shading kernel's SGPR spills 782 -> 95 and VGPR spills
// 95 -> 54 at the same three waves, C4 +4.4 % on MI355X; the other profiles measured flat or slower
// with it (C2 +0.5 %, C5 +0.3 %, C3 -1.2 %; profiles/r04_ab_session.txt r04v, r04w).
#ifndef BLING_CR_OUTLINE
#define BLING_CR_OUTLINE 1
#endif
#include "core_wave.h"
BLING_INSTANTIATE_SHADE(2, false)
BLING_INSTANTIATE_SHADE_DL(2)
