// Halo-staged implicit-GEMM convolution for spatial layers (gfx950 MFMA 16x16x32 bf16).
//
// One workgroup = one block of R output rows of one image.  The input rows the block needs
// (R_in = (R-1)*stride + KH rows, full padded width) are staged ONCE into LDS with
// coalesced 16-byte loads -- zero padding, input dilation (dgrad of strided convs) and
// unpool-on-load (dgrad input given as pooled gradient dP + argmax codes) are resolved in
// the staging pass, so the MFMA loop reads A fragments with one ds_read_b128 per k-step
// and never touches global memory.  The workgroup's slice of the fragment-major weight pack
// is staged alongside.  All staging and fragment loads are branch-free (clamped address +
// select), issued in independent batches of 8 so each lane keeps several in flight.
// Epilogues:
//   mode 0 (forward): bias + ReLU (+2x2 max-pool with argmax code, register-local because
//                     a 16-row MFMA tile is 4 windows x 4 positions) (+dropout) -> bf16
//   mode 1 (dgrad):   bwd_through_store into the previous stage (dropout/ReLU masks, dP).
#include "conv_halo_body.h"

template <int NTC, int TM, int KCH, bool CS4>
__global__ __launch_bounds__(256) void conv_halo_kernel(const ConvMMArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  conv_halo_body<NTC, TM, KCH, CS4>(a, blockIdx.x, blockIdx.y, smem);
}

size_t conv_halo_lds_bytes(const ConvMMArgs& a, int ntc) {
  const bool cs4 = a.Cs_in == 4;
  const int ntab = cs4 ? a.KS * 8 : a.KS * 4;
  const int W_in = (a.Wo - 1) * a.stride + a.KW;
  const int R_in = (a.R - 1) * a.stride + a.KH;
  const int TM = (ntc >= 8 || (ntc == 4 && a.tm == 2)) ? 2 : 4;
  const size_t ep_wave = (size_t)TM * 16 * 2 * ntc * 16;   // bytes
  const int XP = (cs4 || !a.xpix) ? a.Cs_in : a.xpix;
  return (size_t)((ntab * 4 + 15) & ~15) + 32 + (size_t)a.KS * ntc * 64 * 16 +
         (((size_t)R_in * W_in * XP + 7) & ~(size_t)7) * 2 + 4 * ep_wave;
}

// TM: m-tiles per wave per pass -- 2 for 8 n-tiles; 4 for fewer, or 2 with 4 n-tiles when the
// host asks (a.tm == 2: half the epilogue staging, 16 KB less LDS per workgroup)
template <int NTC, int KCH, bool CS4>
static void launch_h(const ConvMMArgs& a, int gx, int gy, size_t lds, hipStream_t s) {
  constexpr int TM = NTC >= 8 ? 2 : 4;
  auto k = conv_halo_kernel<NTC, TM, KCH, CS4>;
  if constexpr (NTC == 4) {
    if (a.tm == 2) k = conv_halo_kernel<NTC, 2, KCH, CS4>;
  }
  if (lds > 65536) hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(k, dim3(gx, gy), dim3(256), lds, s, a);
}

template <int NTC>
static void launch_n(const ConvMMArgs& a, int gx, int gy, size_t lds, hipStream_t s) {
  const bool cs4 = a.Cs_in == 4;
  if (a.KS <= 2) {
    if (cs4) launch_h<NTC, 2, true>(a, gx, gy, lds, s);
    else launch_h<NTC, 2, false>(a, gx, gy, lds, s);
  } else {
    if (cs4) launch_h<NTC, 8, true>(a, gx, gy, lds, s);
    else launch_h<NTC, 8, false>(a, gx, gy, lds, s);
  }
}

void launch_conv_halo(const ConvMMArgs& a, int ntc, hipStream_t s) {
  const int gy = (a.NT + ntc - 1) / ntc;
  const int gx = a.B * ((a.Ho + a.R - 1) / a.R);
  const size_t lds = conv_halo_lds_bytes(a, ntc);
  switch (ntc) {
    case 1: launch_n<1>(a, gx, gy, lds, s); break;
    case 2: launch_n<2>(a, gx, gy, lds, s); break;
    case 4: launch_n<4>(a, gx, gy, lds, s); break;
    case 8: launch_n<8>(a, gx, gy, lds, s); break;
    default: break;
  }
}
