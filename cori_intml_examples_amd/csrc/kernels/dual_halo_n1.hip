// dual_halo instantiations for NTC = 1 (see dual_halo_body.h)
#include "dual_halo_body.h"

DUAL_N_DECL(1) { return dual_w<1>(ca, wa, MT, NTT, mtw, tm, wg, cgx, cgy, lds, x, s); }
