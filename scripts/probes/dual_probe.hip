// Compile-only probe of the RPV production dual (wgrad || dgrad) kernel instances -- the ones
// the step launches -- for tests/test_kernel_resources.py: ~1 min instead of the ~7 min of
// dual_halo_n1.hip with every instance.  Never linked into the extension.
#include "dual_halo_body.h"

template __global__ void dual_halo_kernel<1, 4, 2, 4, false>(const ConvMMArgs, const WgradArgs, const int, const int,
                                                           const int, const int, const int, const DualExtra);
template __global__ void dual_halo_kernel<1, 4, 4, 4, false>(const ConvMMArgs, const WgradArgs, const int, const int,
                                                           const int, const int, const int, const DualExtra);
template __global__ void dual_halo_kernel<1, 4, 2, 4, true>(const ConvMMArgs, const WgradArgs, const int, const int,
                                                          const int, const int, const int, const DualExtra);
template __global__ void dual_halo_kernel<1, 4, 4, 4, true>(const ConvMMArgs, const WgradArgs, const int, const int,
                                                          const int, const int, const int, const DualExtra);
