// Weight gradient for spatial convolutions, halo-staged (gfx950 MFMA + ds_read_b64_tr_b16).
//
//   dW[k = (tap, ci)][co] = sum_p X[p shifted by tap][ci] * dY[p][co]
//
// A workgroup streams a contiguous run of row-blocks (R output rows of one image each).
// Per block, the input halo rows (all channels) and the dY rows are staged into LDS with
// coalesced, branch-free 16-byte loads in independent batches -- dY is rebuilt on the fly
// from the pooled gradient dP and the forward argmax codes, so the full-resolution gradient
// never exists in HBM.  The MFMA reduction axis (pixels) is the outer axis of both LDS
// images; ds_read_b64_tr_b16 (T10) transposes in the read: each lane supplies the address
// of "its" pixel row, with the tap shift folded into the per-lane address (im2col without
// materialising it).  The bias gradient is one extra MFMA tile with an all-ones A operand.
// Partials: one fp32 slab per split, summed in fixed order by slab_reduce (deterministic).

#include <algorithm>
#include <cstdlib>

#include "wgrad_halo_body.h"

// INSTR: ablation (a.dbg) and diagnostics-stamp (a.ts / a.ts2) code compiled in; the
// production instance (INSTR = false) is launched whenever none of them is asked for -- that
// code's register pressure (SGPRs spilled to VGPR lanes) is then not in the launch
template <int MTW, int NTT, bool CS4, bool PIPE, bool INSTR>
__global__ __launch_bounds__(256) void wgrad_halo_kernel(const WgradArgs a, const int MT) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const size_t lin = blockIdx.x + (size_t)gridDim.x * (blockIdx.y + (size_t)gridDim.y * blockIdx.z);
  if (INSTR && a.ts && threadIdx.x == 0) a.ts[2 * lin] = wall_clock64();
  wgrad_halo_body<MTW, NTT, CS4, PIPE, INSTR>(a, MT, blockIdx.x, blockIdx.y, blockIdx.z, smem);
  if (INSTR && a.ts) {
    __syncthreads();
    if (threadIdx.x == 0) a.ts[2 * lin + 1] = wall_clock64();
  }
}

static bool wh_instr(const WgradArgs& a) { return a.dbg || a.ts || a.ts2; }

size_t wgrad_halo_lds_bytes(const WgradArgs& a, int MT, int NTT) {
  const int W_in = (a.Wo - 1) * a.stride + a.KW;
  const int R_in = (a.R - 1) * a.stride + a.KH;
  const int XP = a.xpix ? a.xpix : a.Cs_in, XR = a.xrow ? a.xrow : W_in;
  const int ldb = a.dyld ? a.dyld : NTT * 16 + 8;
  const size_t x_elems = (size_t)(((R_in * XR * XP) + 7) & ~7);
  const size_t npb32 = (size_t)((a.R * a.Wo + 31) & ~31);
  // (>= the write-through slab squares, 4 x 16 x WH_SQ floats, which reuse the buffer)
  // (+ 64 B of zeros and 64 B of ones: the padding / bias-tile A operands of the fragment reads)
  return std::max<size_t>(x_elems * 2 + npb32 * ldb * 2 + 128 + (size_t)(MT * 4 + 4) * 4, 4 * 16 * WH_SQ * 4);
}

template <int MTW, int NTT, bool CS4>
static void wh_t(const WgradArgs& a, int MT, dim3 grid, size_t lds, hipStream_t s) {
  // few workgroups streaming several blocks each: pipeline their staging; a large grid
  // already hides it with resident workgroups (and keeps the lower VGPR count)
  const bool pipe = grid.x * grid.y * grid.z < 512 && a.blocks_per_split > 1;
  auto k = wh_instr(a) ? (pipe ? wgrad_halo_kernel<MTW, NTT, CS4, true, true> : wgrad_halo_kernel<MTW, NTT, CS4, false, true>)
                       : (pipe ? wgrad_halo_kernel<MTW, NTT, CS4, true, false> : wgrad_halo_kernel<MTW, NTT, CS4, false, false>);
  if (lds > 65536) (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(k, grid, dim3(256), lds, s, a, MT);
}

// MT m-tiles x NTT n-tiles per workgroup; each wave owns ceil((MT+bias)/4) m-tiles
// (MTW <= 4, MTW*NTT <= 16); grid = (splits, n-groups, m-groups)
void launch_wgrad_halo(const WgradArgs& a, int MT, int NTT, int splits, hipStream_t s) {
  const bool cs4 = a.Cs_in == 4;
  dim3 grid(splits, (a.NT + NTT - 1) / NTT, (a.Ktiles + MT - 1) / MT);
  const size_t lds = wgrad_halo_lds_bytes(a, MT, NTT);
  const int mtw = (MT + (a.bslab ? 1 : 0) + 3) / 4;
#define C(M_, N_)                                            \
  if (mtw <= M_ && NTT == N_) {                              \
    if (cs4) wh_t<M_, N_, true>(a, MT, grid, lds, s);     \
    else wh_t<M_, N_, false>(a, MT, grid, lds, s);        \
    return;                                                  \
  }
  C(1, 1) C(2, 1) C(4, 1) C(1, 2) C(2, 2) C(4, 2) C(1, 4) C(2, 4) C(4, 4) C(1, 8) C(2, 8)
#undef C
}

// Workgroups of the (non-pipelined) launch resident at once on the whole device: its
// occupancy (VGPRs, LDS) x the CU count.  The host sizes the split count to ONE such round
// -- a grid past it runs a second, mostly empty round (measured on the RPV first layer:
// 1024 workgroups 16.0 us, 683 workgroups 14.2 us).  0 if the query fails.
int wgrad_halo_resident(const WgradArgs& a, int MT, int NTT, bool bias) {
  const bool cs4 = a.Cs_in == 4;
  const size_t lds = wgrad_halo_lds_bytes(a, MT, NTT);
  const int mtw = (MT + (bias ? 1 : 0) + 3) / 4;
  const void* k = nullptr;
  const bool in = wh_instr(a);
#define C(M_, N_)                                                                                       \
  if (!k && mtw <= M_ && NTT == N_)                                                                     \
    k = cs4 ? (in ? (const void*)wgrad_halo_kernel<M_, N_, true, false, true>                           \
                  : (const void*)wgrad_halo_kernel<M_, N_, true, false, false>)                         \
            : (in ? (const void*)wgrad_halo_kernel<M_, N_, false, false, true>                          \
                  : (const void*)wgrad_halo_kernel<M_, N_, false, false, false>);
  C(1, 1) C(2, 1) C(4, 1) C(1, 2) C(2, 2) C(4, 2) C(1, 4) C(2, 4) C(4, 4) C(1, 8) C(2, 8)
#undef C
  if (!k) return 0;
  int dev = 0, per_cu = 0;
  hipDeviceProp_t prop;
  if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) return 0;
  if (lds > 65536) (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 256, lds) != hipSuccess) return 0;
  return per_cu * prop.multiProcessorCount;
}
