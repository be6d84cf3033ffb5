// dual_halo instantiations for NTC = 8 (see dual_halo_body.h)
#include "dual_halo_body.h"

DUAL_N_DECL(8) { return dual_w<8>(ca, wa, MT, NTT, mtw, tm, wg, cgx, cgy, lds, x, s); }
