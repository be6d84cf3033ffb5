// Kernel template + launch dispatch of the dual (wgrad + dgrad) backward launch, shared by
// the per-NTC translation units dual_halo_n*.hip (split so hipcc builds them in parallel).
#pragma once
#include "conv_halo_body.h"
#include "wgrad_halo_body.h"
#include "reduce_body.h"

// XP: the early-bucket workgroups also push their reduced elements to the owners' inboxes
// (XgmiPush, the xGMI data plane's producer push).  A separate instance: compiled into the
// production kernel, that path raised its SGPR spills 165 -> 207 (even as a non-inlined call:
// a call reserves ABI registers for the whole kernel).
template <int NTC, int MTW, int NTT, int TM, bool XP>
__global__ __launch_bounds__(256) void dual_halo_kernel(const ConvMMArgs ca, const WgradArgs wa, const int MT,
                                                        const int n_w, const int wgx, const int wgy, const int cgx,
                                                        const DualExtra x) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int id = blockIdx.x;
  if (x.n_r) {   // early-bucket reduction + optimizer workgroups
    // rfirst 0: the extras last in the grid; 1: first; 2: interleaved -- workgroup e * q of
    // the grid (q = grid / n_r) is extra e, so they dispatch spread among the conv workgroups
    // (interleaving needs q >= 2: with more extras than conv workgroups they go first)
    const bool inter = x.rfirst == 2 && (int)gridDim.x >= 2 * x.n_r;
    const bool first = x.rfirst == 1 || (x.rfirst == 2 && !inter);
    int r;
    if (inter) {
      const int q = (int)gridDim.x / x.n_r, e = id / q;
      r = (id - e * q == 0 && e < x.n_r) ? e : -1;
      if (r < 0) id -= min(x.n_r, e + 1);
    } else {
      r = first ? id : id - (int)gridDim.x + x.n_r;
    }
    if (r >= 0 && r < x.n_r) {
      if constexpr (XP) xgmi_early_block<false>(x.grad, x.rt, x.ro, r, reinterpret_cast<float*>(smem), x.xp);
      else reduce_optim_block_rt(x.grad, x.rt, x.ro, r, reinterpret_cast<float*>(smem));
      return;
    }
    if (first) id -= x.n_r;
  }
  // production bodies only: the dgrad epilogue fixed to backward-through (MODE 1), no
  // ablation / stamp code (launch_dual_halo declines args that ask for them; the executor
  // then runs the two standalone kernels, which keep those switches)
  if (id < n_w) {
    const int bx = id % wgx;
    id /= wgx;
    wgrad_halo_body<MTW, NTT, false, true, false>(wa, MT, bx, id % wgy, id / wgy, smem);
  } else {
    id -= n_w;
    conv_halo_body<NTC, TM, 8, false, 1, false>(ca, id % cgx, id / cgx, smem);
  }
}

template <int NTC, int MTW, int NTT, int TM, bool XP>
static void dual_t(const ConvMMArgs& ca, const WgradArgs& wa, int MT, dim3 wg, int cgx, int cgy, size_t lds,
                   const DualExtra& x, hipStream_t s) {
  auto k = dual_halo_kernel<NTC, MTW, NTT, TM, XP>;
  if (lds > 65536) hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  const int n_w = wg.x * wg.y * wg.z;
  hipLaunchKernelGGL(k, dim3(n_w + cgx * cgy + x.n_r), dim3(256), lds, s, ca, wa, MT, n_w, (int)wg.x, (int)wg.y, cgx,
                     x);
}

// tm: m-tiles per wave per pass of the dgrad body (TM_DEFAULT, or 1 / 2 for NTC <= 2 when
// that evens out the four waves' tile counts on small row blocks).  Producer-push launches
// (x.xp.on) have instances at the default TM only; false = not launched (the caller falls back)
template <int NTC>
static bool dual_w(const ConvMMArgs& ca, const WgradArgs& wa, int MT, int NTT, int mtw, int tm, dim3 wg, int cgx,
                   int cgy, size_t lds, const DualExtra& x, hipStream_t s) {
  constexpr int TMD = NTC >= 8 ? 2 : 4;
  const bool xp = x.n_r && x.xp.on;
#define C(M_, N_)                                                          \
  if (mtw <= M_ && NTT == N_) {                                            \
    if (xp) {                                                              \
      if (tm != TMD && NTC <= 2 && (tm == 1 || tm == 2)) return false;     \
      dual_t<NTC, M_, N_, TMD, true>(ca, wa, MT, wg, cgx, cgy, lds, x, s); \
      return true;                                                         \
    }                                                                      \
    if constexpr (NTC <= 2) {                                              \
      if (tm == 1) { dual_t<NTC, M_, N_, 1, false>(ca, wa, MT, wg, cgx, cgy, lds, x, s); return true; } \
      if (tm == 2) { dual_t<NTC, M_, N_, 2, false>(ca, wa, MT, wg, cgx, cgy, lds, x, s); return true; } \
    }                                                                      \
    dual_t<NTC, M_, N_, TMD, false>(ca, wa, MT, wg, cgx, cgy, lds, x, s);  \
    return true;                                                           \
  }
  C(1, 1) C(2, 1) C(4, 1) C(1, 2) C(2, 2) C(4, 2) C(1, 4) C(2, 4) C(4, 4) C(1, 8) C(2, 8)
#undef C
  return false;
}

#define DUAL_N_DECL(N)                                                                                        \
  bool dual_launch_n##N(const ConvMMArgs& ca, const WgradArgs& wa, int MT, int NTT, int mtw, int tm, dim3 wg, \
                        int cgx, int cgy, size_t lds, const DualExtra& x, hipStream_t s)
DUAL_N_DECL(1);
DUAL_N_DECL(2);
DUAL_N_DECL(4);
DUAL_N_DECL(8);
