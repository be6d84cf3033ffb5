// Horizontal fusion of one conv layer's two independent backward GEMMs:
//   wgrad: dW = im2col(X)^T dY   (wgrad_halo body, few long workgroups: 170-350 at batch 128)
//   dgrad: dX = dY * W^T         (conv_halo body in mode 1, 512 short workgroups)
// Both read the same dY (rebuilt from dP + argmax codes on load) and nothing either writes
// is read by the other, so they run as ONE launch: workgroups [0, n_w) execute the wgrad
// body, the rest the dgrad body.  At batch 128 neither kernel alone fills 256 CUs for long;
// co-scheduled, the dgrad workgroups fill the CUs the wgrad ones leave idle and the step pays
// one kernel boundary (launch ramp + drain + L2 writeback, ~5 us here) instead of two.
// Wgrad workgroups come first: they are the long pole, so they are dispatched first.
// The LDS request is the max of the two bodies' needs.
#include <algorithm>

#include "conv_halo_body.h"
#include "wgrad_halo_body.h"

size_t conv_halo_lds_bytes(const ConvMMArgs& a, int ntc);
size_t wgrad_halo_lds_bytes(const WgradArgs& a, int MT, int NTT);

template <int NTC, int MTW, int NTT>
__global__ __launch_bounds__(256) void dual_halo_kernel(const ConvMMArgs ca, const WgradArgs wa, const int MT,
                                                        const int n_w, const int wgx, const int wgy, const int cgx) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TM = NTC >= 8 ? 2 : 4;
  int id = blockIdx.x;
  if (id < n_w) {
    const int bx = id % wgx;
    id /= wgx;
    wgrad_halo_body<MTW, NTT, false, true>(wa, MT, bx, id % wgy, id / wgy, smem);
  } else {
    id -= n_w;
    conv_halo_body<NTC, TM, 8, false>(ca, id % cgx, id / cgx, smem);
  }
}

template <int NTC, int MTW, int NTT>
static void dual_t(const ConvMMArgs& ca, const WgradArgs& wa, int MT, dim3 wg, int cgx, int cgy, size_t lds,
                   hipStream_t s) {
  auto k = dual_halo_kernel<NTC, MTW, NTT>;
  if (lds > 65536) hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  const int n_w = wg.x * wg.y * wg.z;
  hipLaunchKernelGGL(k, dim3(n_w + cgx * cgy), dim3(256), lds, s, ca, wa, MT, n_w, (int)wg.x, (int)wg.y, cgx);
}

template <int NTC>
static bool dual_w(const ConvMMArgs& ca, const WgradArgs& wa, int MT, int NTT, int mtw, dim3 wg, int cgx, int cgy,
                   size_t lds, hipStream_t s) {
#define C(M_, N_)                                                      \
  if (mtw <= M_ && NTT == N_) {                                        \
    dual_t<NTC, M_, N_>(ca, wa, MT, wg, cgx, cgy, lds, s);             \
    return true;                                                       \
  }
  C(1, 1) C(2, 1) C(4, 1) C(1, 2) C(2, 2) C(4, 2) C(1, 4) C(2, 4) C(4, 4) C(1, 8) C(2, 8)
#undef C
  return false;
}

// Returns false (nothing launched) when the pair is not a supported combination; the caller
// then launches the two kernels separately.
bool launch_dual_halo(const ConvMMArgs& ca, int ntc, const WgradArgs& wa, int MT, int NTT, int splits,
                      hipStream_t s) {
  if (ca.Cs_in == 4 || wa.Cs_in == 4 || ca.KS <= 2) return false;   // 4-channel / tiny-K variants
  const int cgy = (ca.NT + ntc - 1) / ntc;
  const int cgx = ca.B * ((ca.Ho + ca.R - 1) / ca.R);
  const dim3 wg(splits, (wa.NT + NTT - 1) / NTT, (wa.Ktiles + MT - 1) / MT);
  const int mtw = (MT + (wa.bslab ? 1 : 0) + 3) / 4;
  const size_t lds = std::max(conv_halo_lds_bytes(ca, ntc), wgrad_halo_lds_bytes(wa, MT, NTT));
  if (lds > 160 * 1024) return false;
  switch (ntc) {
    case 1: return dual_w<1>(ca, wa, MT, NTT, mtw, wg, cgx, cgy, lds, s);
    case 2: return dual_w<2>(ca, wa, MT, NTT, mtw, wg, cgx, cgy, lds, s);
    case 4: return dual_w<4>(ca, wa, MT, NTT, mtw, wg, cgx, cgy, lds, s);
    case 8: return dual_w<8>(ca, wa, MT, NTT, mtw, wg, cgx, cgy, lds, s);
  }
  return false;
}
