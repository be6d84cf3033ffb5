// dual_halo instantiations for NTC = 2 (see dual_halo_body.h)
#include "dual_halo_body.h"

DUAL_N_DECL(2) { return dual_w<2>(ca, wa, MT, NTT, mtw, tm, wg, cgx, cgy, lds, x, s); }
