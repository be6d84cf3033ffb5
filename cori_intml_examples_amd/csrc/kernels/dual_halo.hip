// Horizontal fusion of one conv layer's two independent backward GEMMs:
//   wgrad: dW = im2col(X)^T dY   (wgrad_halo body, few long workgroups: 170-350 at batch 128)
//   dgrad: dX = dY * W^T         (conv_halo body in mode 1, 512 short workgroups)
// Both read the same dY (rebuilt from dP + argmax codes on load) and nothing either writes
// is read by the other, so they run as ONE launch: workgroups [0, n_w) execute the wgrad
// body, the rest the dgrad body.  At batch 128 neither kernel alone fills 256 CUs for long;
// co-scheduled, the dgrad workgroups fill the CUs the wgrad ones leave idle and the step pays
// one kernel boundary (launch ramp + drain + L2 writeback, ~5 us here) instead of two.
// Wgrad workgroups come first: they are the long pole, so they are dispatched first.
// The LDS request is the max of the two bodies' needs.  Optionally the launch also carries an
// early bucket's reduction + optimizer (DualExtra) in extra workgroups.
#include <algorithm>

#include "dual_halo_body.h"

size_t conv_halo_lds_bytes(const ConvMMArgs& a, int ntc);
size_t wgrad_halo_lds_bytes(const WgradArgs& a, int MT, int NTT);

// Returns false (nothing launched) when the pair is not a supported combination; the caller
// then launches the two kernels separately.
bool launch_dual_halo(const ConvMMArgs& ca, int ntc, const WgradArgs& wa, int MT, int NTT, int splits,
                      const DualExtra& x, hipStream_t s) {
  if (ca.Cs_in == 4 || wa.Cs_in == 4 || ca.KS <= 2) return false;   // 4-channel / tiny-K variants
  // the dual kernel is built without ablation / diagnostics code and with the dgrad's
  // backward-through epilogue only: anything else runs as two standalone launches
  if (ca.mode != 1 || ca.dbg || wa.dbg || ca.ts || wa.ts || wa.ts2) return false;
  const int cgy = (ca.NT + ntc - 1) / ntc;
  const int cgx = ca.B * ((ca.Ho + ca.R - 1) / ca.R);
  const dim3 wg(splits, (wa.NT + NTT - 1) / NTT, (wa.Ktiles + MT - 1) / MT);
  const int mtw = (MT + (wa.bslab ? 1 : 0) + 3) / 4;
  const size_t lds = std::max(conv_halo_lds_bytes(ca, ntc), wgrad_halo_lds_bytes(wa, MT, NTT));
  if (lds > 160 * 1024 || (x.n_r && lds < 2048)) return false;   // (the reduce body stages <= 2 KB)
  if (x.n_r && x.xp.on && x.xp.mode >= 2 && lds < 4096) return false;   // (+ the exchange's wait word)
  // extras run the exchange's modes 1 (reduce + push) and 4 (owner half) only; a mode-2 table
  // (the unsplit exchange, xchg_split=0) goes to the caller's separate launches
  if (x.n_r && x.xp.on && x.xp.mode != 1 && x.xp.mode != 4) return false;
  // dgrad m-tiles per wave per pass: the TM in {4, 2} that minimises the busiest wave's
  // tile count over the block (ties -> larger TM: more fragment reuse); TM = 1 only when
  // the block has <= 4 tiles (measured: TM 1 loses its fragment reuse on longer blocks)
  const int rows = std::min(ca.R, ca.Ho);
  const int ntiles = ca.pool ? ((rows / 2) * ca.Wp + 3) / 4 : (rows * ca.Wo + 15) / 16;
  int tm = ntc >= 8 ? 2 : 4, best = 1 << 30;
  for (int t : {4, 2, 1}) {
    if (ntc >= 8 && t == 4) continue;
    if (ntc > 2 && t != (ntc >= 8 ? 2 : 4)) continue;
    if (t == 1 && ntiles > 4) continue;
    const int load = t * ((ntiles + 4 * t - 1) / (4 * t));   // tiles of the busiest wave
    if (load < best) { best = load; tm = t; }
  }
  if (ca.tm == 1 || ca.tm == 2 || (ca.tm == 4 && ntc < 8)) tm = ca.tm;   // host override (geometry table)
  switch (ntc) {
    case 1: return dual_launch_n1(ca, wa, MT, NTT, mtw, tm, wg, cgx, cgy, lds, x, s);
    case 2: return dual_launch_n2(ca, wa, MT, NTT, mtw, tm, wg, cgx, cgy, lds, x, s);
    case 4: return dual_launch_n4(ca, wa, MT, NTT, mtw, tm, wg, cgx, cgy, lds, x, s);
    case 8: return dual_launch_n8(ca, wa, MT, NTT, mtw, tm, wg, cgx, cgy, lds, x, s);
  }
  return false;
}
