// dual_halo instantiations for NTC = 4 (see dual_halo_body.h)
#include "dual_halo_body.h"

DUAL_N_DECL(4) { return dual_w<4>(ca, wa, MT, NTT, mtw, tm, wg, cgx, cgy, lds, x, s); }
