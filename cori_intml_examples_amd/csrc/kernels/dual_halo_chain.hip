// dual_halo instantiations with a chained first-layer wgrad (DualExtra::ntt2, see args.h):
// the layer-2 backward launch (wgrad || dgrad) whose dgrad workgroups then compute the
// first conv layer's weight gradient over the rows they just produced (one-n-tile dgrad
// blocks, a 16-channel first layer: the RPV stack conv[16, ..]).
#include "dual_halo_body.h"

bool dual_launch_chain(const ConvMMArgs& ca, const WgradArgs& wa, int MT, int NTT, int mtw, int tm, dim3 wg,
                       int cgx, int cgy, size_t lds, const DualExtra& x, hipStream_t s) {
  if (mtw > 4 || x.w2.Cs_in != 4) return false;
#define CH(N_, T_, C_)                                                        \
  if (NTT == N_ && tm == T_ && x.ntt2 == C_) {                              \
    dual_t<1, 4, N_, T_, C_>(ca, wa, MT, wg, cgx, cgy, lds, x, s);           \
    return true;                                                            \
  }
  CH(2, 4, 1) CH(2, 2, 1) CH(2, 1, 1) CH(4, 4, 1) CH(4, 2, 1) CH(4, 1, 1)
#undef CH
  return false;
}
