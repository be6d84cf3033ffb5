// Step plumbing kernels:
//   prologue     (K14)       ONE launch per step: batch rows from the device-resident
//                            dataset by the epoch's device permutation (16-byte copies),
//                            the bf16 re-pack of the previous update, and the step
//                            bookkeeping (iteration counter, cursor, LR decay, optimizer
//                            bias-correction scalars) by the last workgroup
//   slab_reduce  (K6/K9 2nd) deterministic fixed-order sum of split partial slabs into the
//                            flat fp32 gradient buffer, remapped to Keras layout
//   optim_update (K13)       ONE multi-tensor launch over the flat buffer: Adam / Nadam /
//                            Adadelta / RMSprop / SGD with Keras 2.2 math, DP averaging
//                            folded in (grad_scale), and the bf16 fragment-major weight
//                            packs the MFMA kernels read scattered out in the same pass
#include <stdexcept>

#include "args.h"
#include "optim_math.h"
#include "reduce_body.h"
#include "step_book.h"

// Batch rows from the device-resident dataset by the epoch's permutation (16-byte copies),
// targets alongside.  `pos0` is the step's cursor (read before the bookkeeping advances it).
__device__ __forceinline__ void gather_block(const GatherArgs& a, const StepState* st, int pos0, int row, int bx,
                                             int gx) {
  const bf16* xs = reinterpret_cast<const bf16*>(st->data_x);
  const float* ys = reinterpret_cast<const float*>(st->data_y);
  const int R = st->data_R, C = st->data_C;
  const int src = step_src_pos(st, pos0 + row);   // (cursor clamped before the permutation)
  const int nvec = R / 8;   // 16-byte vectors per row
  const uint4* s = reinterpret_cast<const uint4*>(xs + (size_t)src * R);
  uint4* d = reinterpret_cast<uint4*>(a.xb + (size_t)row * R);
  if (!a.skip_x) {
    for (int v = bx * 256 + threadIdx.x; v < nvec; v += gx * 256) d[v] = s[v];
    // rows of 4-channel pixels with an odd pixel count end in half a vector (R % 8 == 4)
    if ((R & 7) && bx == 0 && threadIdx.x == 0)
      *reinterpret_cast<uint2*>(a.xb + (size_t)row * R + nvec * 8) =
          *reinterpret_cast<const uint2*>(xs + (size_t)src * R + nvec * 8);
  }
  if (bx == 0 && a.yb && ys)
    for (int c = threadIdx.x; c < C; c += 256) a.yb[(size_t)row * C + c] = ys[(size_t)src * C + c];
}

__global__ __launch_bounds__(256) void slab_reduce_kernel(float* __restrict__ grad, const RedTable tab) {
  __shared__ __attribute__((aligned(16))) float red[512];
  const int blk = blockIdx.x;
  const RedDesc& d = tab.d[red_desc(tab, blk)];
  if (d.vec4) {
    int e;
    float4 g;
    if (slab_reduce_vec4(d, blk, red, e, g)) *reinterpret_cast<float4*>(grad + e) = g;
    return;
  }
  int e;
  float v;
  if (slab_reduce_elem(tab, blk, red, e, v)) grad[e] = v;
}

void launch_slab_reduce(float* grad, int lo, int hi, const RedTable& tab, hipStream_t s) {
  if (tab.nblocks <= 0) return;
  hipLaunchKernelGGL(slab_reduce_kernel, dim3(tab.nblocks), dim3(256), 0, s, grad, tab);
}

// ---------------------------------------------------------------------------------------
// Conv weight packs: one launch over every (fp32 master tensor -> bf16 fragment-major pack)
// descriptor.  A thread writes one 16-byte fragment vector -- 8 consecutive k of one n --
// gathering its 8 sources from the Keras-layout master (the inverse of the pack layout
// pack[((ks*NT+nt)*64+lane)*8+j] = B[32ks+8(lane>>4)+j][16nt+(lane&15)]).  Lanes of a
// wave cover 16 consecutive n, so each gather instruction reads contiguous runs of the
// row-major master.  Padding rows/columns become zeros.  (Dense layers: dense_pack_kernel.)
__device__ __forceinline__ void conv_pack_block(const float* __restrict__ master, bf16* __restrict__ arena,
                                                const PackTable& tab, int blk) {
  int di = 0;
  while (di + 1 < tab.n && blk >= tab.d[di + 1].blk0) ++di;
  const PackDesc& d = tab.d[di];
  const int v = (blk - d.blk0) * 256 + (int)threadIdx.x;
  if (v >= d.nvec) return;
  const int lane = v & 63;
  const int frag = v >> 6;                 // ks * NT + nt
  const int ks = frag / d.NT, nt = frag - ks * d.NT;
  const int k0 = ks * 32 + 8 * (lane >> 4);
  const int n = nt * 16 + (lane & 15);
  const float* w = master + d.src_off;
  // The 8 k of this vector share one tap unless Cs == 4: split the index once, then step
  // the channel -- no per-element divisions.  Loads are unconditional from a clamped
  // address (select afterwards) so all 8 stay in flight.
  int outer = k0 / d.Cs;
  int c = k0 - outer * d.Cs;
  const int KHW = d.KH * d.KW;
  const bool fwd = d.type == PACK_CONV_FWD;
  float vals[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    int cj = c + j, oj = outer;
    if (cj >= d.Cs) { cj -= d.Cs; ++oj; }            // only when Cs == 4
    const int t = fwd ? oj : KHW - 1 - oj;
    const int ci = fwd ? cj : n;
    const int co = fwd ? n : cj;
    const bool ok = oj < KHW && ci < d.Cin && co < d.Cout;
    const long long idx = ((long long)t * d.Cin + ci) * d.Cout + co;
    const float x = w[ok ? idx : 0];
    vals[j] = ok ? x : 0.f;
  }
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = f2bf(vals[j]);
  *reinterpret_cast<bf16x8*>(arena + d.dst_off + (size_t)v * 8) = o;
}

// Dense pair: one workgroup = 32 padded-k rows x 128 n columns of W (Keras [k][n] fp32,
// read once, coalesced rows) staged as bf16 in LDS; it writes the 8 forward-pack fragments
// (8 consecutive k of one n per lane: an LDS column read) and the 8 backward-pack
// fragments (8 consecutive n of one k: one 16-byte LDS row read) the tile covers.  Each
// fragment store is 1 KB contiguous.  Replaces two strided gathers of the master (the
// backward one reading 32-byte pieces of 64 different rows per instruction).
__device__ __forceinline__ void dense_pack_block(const float* __restrict__ master, bf16* __restrict__ arena,
                                                 const PackTable& tab, int blk, bf16 (*tile)[136]) {
  int di = 0;
  while (di + 1 < tab.nd && blk >= tab.dp[di + 1].blk0) ++di;
  const DensePair& d = tab.dp[di];
  const int local = blk - d.blk0;
  const int kt = local / d.ntn, ntile = local - kt * d.ntn;
  const int k0 = kt * 32, n0 = ntile * 128;
  const int t = threadIdx.x;
  const float* w = master + d.src_off;
  // stage: thread -> row (t>>5) + 8*pass, 4 consecutive columns
  const int c4 = (t & 31) * 4;
#pragma unroll
  for (int pass = 0; pass < 4; ++pass) {
    const int row = (t >> 5) + 8 * pass;
    const int k = k0 + row;
    const int oj = k / d.Cs, cj = k - oj * d.Cs;
    const bool kok = cj < d.Cin && oj < d.KHW;
    const long long rbase = (long long)(oj * d.Cin + cj) * d.N;
    float v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n = n0 + c4 + q;
      const bool ok = kok && n < d.N;
      const float x = w[ok ? rbase + n : 0];
      v[q] = ok ? x : 0.f;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) tile[row][c4 + q] = f2bf(v[q]);
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int v = t + 256 * h;
    const int f = v >> 6, l = v & 63;
    // forward fragment (ks = kt, nt = 8*ntile + f)
    const int nt = ntile * 8 + f;
    if (nt < d.NT) {
      bf16x8 o;
      const int col = 16 * f + (l & 15), r0 = 8 * (l >> 4);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = tile[r0 + j][col];
      *reinterpret_cast<bf16x8*>(arena + d.dst_fwd + ((size_t)(kt * d.NT + nt) * 64 + l) * 8) = o;
    }
    // backward fragment (nt' = 2*kt + (f & 1), ks' = 4*ntile + (f >> 1))
    if (d.dst_bwd >= 0) {
      const int ntb = 2 * kt + (f & 1), ksb = 4 * ntile + (f >> 1);
      if (ntb < d.NTb && ksb < d.KSb) {
        const int row = 16 * (f & 1) + (l & 15), col = 32 * (f >> 1) + 8 * (l >> 4);
        *reinterpret_cast<bf16x8*>(arena + d.dst_bwd + ((size_t)(ksb * d.NTb + ntb) * 64 + l) * 8) =
            *reinterpret_cast<const bf16x8*>(&tile[row][col]);
      }
    }
  }
}

// One launch for both: workgroups [0, nblocks) pack conv descriptors, the rest dense pairs.
__global__ __launch_bounds__(256) void pack_kernel(const float* __restrict__ master, bf16* __restrict__ arena,
                                                   const PackTable tab) {
  __shared__ __attribute__((aligned(16))) bf16 tile[32][136];
  if ((int)blockIdx.x >= tab.nblocks) {
    dense_pack_block(master, arena, tab, (int)blockIdx.x - tab.nblocks, tile);
    return;
  }
  conv_pack_block(master, arena, tab, (int)blockIdx.x);
}

void launch_pack(const float* master, bf16* arena, const PackTable& tab, hipStream_t s) {
  const int blocks = tab.nblocks + tab.dblocks;
  if (blocks > 0) hipLaunchKernelGGL(pack_kernel, dim3(blocks), dim3(256), 0, s, master, arena, tab);
}

// ---------------------------------------------------------------------------------------
// Step prologue: ONE launch instead of bookkeeping + gather + pack (three kernel boundaries,
// ~5 us each at this size).  Gather and pack workgroups are independent.  Nothing here
// writes state another prologue workgroup reads: the cursors (st->pos / eval_pos) and the
// stale flag are advanced / cleared by the head kernel later in the step, and workgroup 0
// computes this step's iteration count and optimizer scalars (read only by later kernels).
// (A completion counter instead cost ~15 us: ~1200 same-address atomics serialise.)
__global__ __launch_bounds__(256) void prologue_kernel(const PrologueArgs a, const PackTable tab) {
  __shared__ __attribute__((aligned(16))) bf16 tile[32][136];
  StepState* st = a.sb.st;
  const int b = (int)blockIdx.x;
  if (b < a.gather_blocks) {
    const int row = b / a.gather_gx, bx = b - row * a.gather_gx;
    const int pos0 = a.sb.training ? st->pos : st->eval_pos;
    gather_block(a.ga, st, pos0, row, bx, a.gather_gx);
  } else if (a.pack_mode == 1 || (a.pack_mode == 2 && st->packs_stale)) {
    const int pb = b - a.gather_blocks;
    if (pb >= tab.nblocks) dense_pack_block(a.master, a.arena, tab, pb - tab.nblocks, tile);
    else conv_pack_block(a.master, a.arena, tab, pb);
  }
  if (b == 0 && threadIdx.x == 0) step_bookkeeping(a.sb);
}

void launch_prologue(const PrologueArgs& a, const PackTable& tab, hipStream_t s) {
  const int pack_blocks = a.pack_mode ? tab.nblocks + tab.dblocks : 0;
  hipLaunchKernelGGL(prologue_kernel, dim3(a.gather_blocks + pack_blocks), dim3(256), 0, s, a, tab);
}

int gather_gx(int R) {
  const int nvec = R / 8;
  return max(1, min(8, (nvec + 255) / 256));
}

// ---------------------------------------------------------------------------------------
// Multi-tensor optimizer update over the flat fp32 buffers, 4 elements per thread
// (16-byte loads/stores; the buffers' capacity is a multiple of 64 elements).
// The range [lo, lo + n) is processed in aligned float4 groups from lo & ~3; elements of a
// boundary group outside the range are written back unchanged (no other kernel writes them
// concurrently: the per-bucket optimizer launches of one step are stream-ordered).
// One 8(k) x 128(n) tile of a dense route (kind 2, identity padding): wave w updates the
// 8 x 32 sub-tile at columns 32w.. (lane -> row lane >> 3, 4 columns 4 * (lane & 7)), stages
// the new bf16 weights in its own LDS slice, then writes whole pack vectors: lanes 0..31 one
// forward vector each (8 consecutive k of one n: a column of the slice), lanes 32..63 one
// backward vector each (8 consecutive n of one k: a row segment).  Same per-element math as
// the flat path (bit-identical weights), 16-byte pack stores.
template <int KIND>
__device__ __forceinline__ void optim_tile_block(const OptimArgs& a, int tb, bf16 (*tile)[8][40]) {
  int i = 0;
#pragma unroll
  for (int u = 1; u < 4; ++u)
    if (u < a.ntile && tb >= a.tile_b0[u]) i = u;
  const PackRoute R = a.routes[a.tile_route[i]];
  const int N = R.Cout;
  const int cbn = (N + 127) >> 7;                     // 128-column blocks per row block
  const int t = tb - a.tile_b0[i];
  const int rb = t / cbn, cb = t - rb * cbn;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int col0 = cb * 128 + wave * 32;
  if (col0 >= N) return;                              // wave-uniform (N % 32 == 0)
  const int r = lane >> 3, c4 = (lane & 7) * 4;
  const int row0 = rb * 8;
  const int e = R.lo + (row0 + r) * N + col0 + c4;
  float4 p = *reinterpret_cast<const float4*>(a.p + e);
  const float4 g = *reinterpret_cast<const float4*>(a.g + e);
  float4 s0 = a.s0 ? *reinterpret_cast<const float4*>(a.s0 + e) : float4{0.f, 0.f, 0.f, 0.f};
  float4 s1 = a.s1 ? *reinterpret_cast<const float4*>(a.s1 + e) : float4{0.f, 0.f, 0.f, 0.f};
  const float gs = a.grad_scale;
  opt_update<KIND>(a, a.st, p.x, g.x * gs, &s0.x, &s1.x);
  opt_update<KIND>(a, a.st, p.y, g.y * gs, &s0.y, &s1.y);
  opt_update<KIND>(a, a.st, p.z, g.z * gs, &s0.z, &s1.z);
  opt_update<KIND>(a, a.st, p.w, g.w * gs, &s0.w, &s1.w);
  *reinterpret_cast<float4*>(a.p + e) = p;
  if (a.s0) *reinterpret_cast<float4*>(a.s0 + e) = s0;
  if (a.s1) *reinterpret_cast<float4*>(a.s1 + e) = s1;
  bf16 (*sl)[40] = tile[wave];
  sl[r][c4] = f2bf(p.x);
  sl[r][c4 + 1] = f2bf(p.y);
  sl[r][c4 + 2] = f2bf(p.z);
  sl[r][c4 + 3] = f2bf(p.w);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (lane < 32) {
    if (R.fwd >= 0) {   // column lane: k = row0 .. row0+7 (j = 0..7), n = col0 + lane
      bf16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = sl[j][lane];
      *reinterpret_cast<bf16x8*>(a.arena + R.fwd + frag_off(row0, col0 + lane, R.NT)) = v;
    }
  } else if (R.bwd >= 0) {   // row (lane-32) >> 2, columns 8 * (lane & 3) ..: k' = n, n' = row
    const int rr = (lane - 32) >> 2, cc = ((lane - 32) & 3) * 8;
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(&sl[rr][cc]);
    *reinterpret_cast<bf16x8*>(a.arena + R.bwd + frag_off(col0 + cc, row0 + rr, R.NTb)) = v;
  }
}

// true when element e lies in a route updated by the tile blocks of this launch
__device__ __forceinline__ bool in_tiled_route(const OptimArgs& a, int e) {
  for (int i = 0; i < a.ntile; ++i) {
    const PackRoute& R = a.routes[a.tile_route[i]];
    if (e >= R.lo && e < R.hi) return true;
  }
  return false;
}

template <int KIND>
__global__ __launch_bounds__(256) void optim_kernel(const OptimArgs a) {
  __shared__ __attribute__((aligned(16))) bf16 tile[4][8][40];
  if (a.ntile && (int)blockIdx.x >= a.flat_blocks) {
    optim_tile_block<KIND>(a, (int)blockIdx.x - a.flat_blocks, tile);
    return;
  }
  const int base = a.lo & ~3, end = a.lo + a.n;
  const int e = base + (blockIdx.x * 256 + threadIdx.x) * 4;
  if (e >= end) return;
  // (a tiled route starts and ends on multiples of 4: its float4 groups are all-or-nothing)
  if (a.ntile && in_tiled_route(a, e)) return;
  const StepState* st = a.st;
  float4 p = *reinterpret_cast<const float4*>(a.p + e);
  const float4 g = *reinterpret_cast<const float4*>(a.g + e);
  float4 s0 = a.s0 ? *reinterpret_cast<const float4*>(a.s0 + e) : float4{0.f, 0.f, 0.f, 0.f};
  float4 s1 = a.s1 ? *reinterpret_cast<const float4*>(a.s1 + e) : float4{0.f, 0.f, 0.f, 0.f};
  const float gs = a.grad_scale;
  if (e >= a.lo && e + 4 <= end) {
    opt_update<KIND>(a, st, p.x, g.x * gs, &s0.x, &s1.x);
    opt_update<KIND>(a, st, p.y, g.y * gs, &s0.y, &s1.y);
    opt_update<KIND>(a, st, p.z, g.z * gs, &s0.z, &s1.z);
    opt_update<KIND>(a, st, p.w, g.w * gs, &s0.w, &s1.w);
  } else {
    if (e >= a.lo && e < end) opt_update<KIND>(a, st, p.x, g.x * gs, &s0.x, &s1.x);
    if (e + 1 >= a.lo && e + 1 < end) opt_update<KIND>(a, st, p.y, g.y * gs, &s0.y, &s1.y);
    if (e + 2 >= a.lo && e + 2 < end) opt_update<KIND>(a, st, p.z, g.z * gs, &s0.z, &s1.z);
    if (e + 3 >= a.lo && e + 3 < end) opt_update<KIND>(a, st, p.w, g.w * gs, &s0.w, &s1.w);
  }
  *reinterpret_cast<float4*>(a.p + e) = p;
  if (a.s0) *reinterpret_cast<float4*>(a.s0 + e) = s0;
  if (a.s1) *reinterpret_cast<float4*>(a.s1 + e) = s1;
  if (a.nroutes) {
    if (e >= a.lo && e + 4 <= end) {
      pack_write4(a, e, p);
    } else {
      if (e >= a.lo && e < end) pack_write(a, e, p.x);
      if (e + 1 >= a.lo && e + 1 < end) pack_write(a, e + 1, p.y);
      if (e + 2 >= a.lo && e + 2 < end) pack_write(a, e + 2, p.z);
      if (e + 3 >= a.lo && e + 3 < end) pack_write(a, e + 3, p.w);
    }
  }
  if (a.defer_pack && !a.nroutes && blockIdx.x == 0 && threadIdx.x == 0) a.st->packs_stale = 1;
}

void launch_optim(const OptimArgs& a, const PackTable& tab, hipStream_t s) {
  if (a.n > 0 && !a.pack_only) {
    const int span = a.lo + a.n - (a.lo & ~3);
    const int flat = ((span + 3) / 4 + 255) / 256;
    if (a.ntile && a.flat_blocks != flat) throw std::invalid_argument("optim: flat_blocks mismatch");
    const dim3 grid(flat + (a.ntile ? a.tile_b0[a.ntile] : 0));
    switch (a.kind) {
      case OPT_ADAM: hipLaunchKernelGGL(optim_kernel<OPT_ADAM>, grid, dim3(256), 0, s, a); break;
      case OPT_NADAM: hipLaunchKernelGGL(optim_kernel<OPT_NADAM>, grid, dim3(256), 0, s, a); break;
      case OPT_ADADELTA: hipLaunchKernelGGL(optim_kernel<OPT_ADADELTA>, grid, dim3(256), 0, s, a); break;
      case OPT_RMSPROP: hipLaunchKernelGGL(optim_kernel<OPT_RMSPROP>, grid, dim3(256), 0, s, a); break;
      default: hipLaunchKernelGGL(optim_kernel<OPT_SGD>, grid, dim3(256), 0, s, a); break;
    }
  }
  if (!a.defer_pack || a.pack_only)
    launch_pack(a.p, a.arena, tab, s);    // the MFMA kernels read the bf16 packs
}

// ---------------------------------------------------------------------------------------
// Final slab reduction fused with the optimizer (single GPU: nothing sits between them);
// the body is reduce_optim_block (reduce_body.h), also run by the early-bucket workgroups
// of the dual conv backward launch.
template <int KIND>
__global__ __launch_bounds__(256) void reduce_optim_kernel(float* __restrict__ grad, const RedTable tab,
                                                           const OptimArgs a) {
  __shared__ __attribute__((aligned(16))) float red[512];   // (>= 2 KB: the tiled pack stage)
  reduce_optim_block<KIND, true>(grad, tab, a, blockIdx.x, red);
}

// a data-parallel table launch of its own: the early bucket's reduction + producer push (mode 1)
// or exchange + update (mode 2) when the dual launch that normally carries it declined
// (ablation / stamp args), or the end-of-backward bucket's whole all-reduce + update (mode 3)
__global__ __launch_bounds__(256) void xgmi_early_kernel(float* __restrict__ grad, const RedTable tab,
                                                         const OptimArgs a, const XgmiPush xp) {
  __shared__ __attribute__((aligned(16))) float red[1024];   // (mode 2: the wait word at [1023])
  xgmi_early_block<true>(grad, tab, a, blockIdx.x, red, xp);
}

// the end-of-backward launch of the split exchange: the conv layers' table (mode 3: reduce,
// push, exchange, update) in workgroups [0, nc) and the early range's finish part (mode 5:
// wait for its owners' sums -- pushed by the owner part in an earlier backward launch -- read
// them, update) in workgroups [nc, nc + ne): one launch, no workgroup waits on its own launch
__global__ __launch_bounds__(256) void xgmi_end_kernel(float* __restrict__ grad, const RedTable tc, const OptimArgs a,
                                                       const XgmiPush xc, const RedTable te, const XgmiPush xe, int nc) {
  __shared__ __attribute__((aligned(16))) float red[1024];
  const int b = blockIdx.x;
  if (b < nc) xgmi_early_block<true>(grad, tc, a, b, red, xc);
  else xgmi_early_block<true>(grad, te, a, b - nc, red, xe);
}

// mode 3 with one workgroup per block (xchg_fused_block), and with END the early range's
// finish part (mode 5) in workgroups [nc, grid) -- the optimizer kind a template parameter
template <int KIND, bool END>
__global__ __launch_bounds__(256) void xchg_fused_kernel(float* __restrict__ grad, const RedTable tc, const OptimArgs a,
                                                         const XgmiPush xc, const RedTable te, const XgmiPush xe,
                                                         int nc) {
  __shared__ __attribute__((aligned(16))) float red[1024];
  const int b = blockIdx.x;
  if (!END || b < nc) {
    if (xs_aborted(xc)) return;
    xchg_fused_block<KIND>(grad, tc, a, b, red, xc);
  } else {
    if (xs_aborted(xe)) return;
    xchg_update_block<KIND>(grad, te, a, b - nc, red, xe, 2);
  }
}

template <bool END>
static void launch_fused(float* grad, const RedTable& tc, const OptimArgs& a, const XgmiPush& xc, const RedTable& te,
                         const XgmiPush& xe, int nc, int ne, hipStream_t s) {
  const dim3 g(nc + ne), b(256);
  switch (a.kind) {
    case OPT_ADAM: hipLaunchKernelGGL((xchg_fused_kernel<OPT_ADAM, END>), g, b, 0, s, grad, tc, a, xc, te, xe, nc); break;
    case OPT_NADAM: hipLaunchKernelGGL((xchg_fused_kernel<OPT_NADAM, END>), g, b, 0, s, grad, tc, a, xc, te, xe, nc); break;
    case OPT_ADADELTA:
      hipLaunchKernelGGL((xchg_fused_kernel<OPT_ADADELTA, END>), g, b, 0, s, grad, tc, a, xc, te, xe, nc);
      break;
    case OPT_RMSPROP:
      hipLaunchKernelGGL((xchg_fused_kernel<OPT_RMSPROP, END>), g, b, 0, s, grad, tc, a, xc, te, xe, nc);
      break;
    default: hipLaunchKernelGGL((xchg_fused_kernel<OPT_SGD, END>), g, b, 0, s, grad, tc, a, xc, te, xe, nc); break;
  }
}

// mode 3 goes through the fused kernel when it runs one workgroup per block and has the
// exchange structure (peers, or xchg_p1); looping workgroups (ranks sharing a GPU) and the
// single-GPU reduction keep the generic table kernels
static bool fused_mode3(const XgmiPush& x) { return x.mode == 3 && !x.nx && (x.size > 1 || x.p1); }

void launch_reduce_optim_end(float* grad, const RedTable& tc, const OptimArgs& a, const XgmiPush& xc,
                             const RedTable& te, const XgmiPush& xe, hipStream_t s) {
  const int nc = tc.nblocks <= 0 ? 0 : (xc.nx ? xc.nx : tc.nblocks);
  const int ne = te.nblocks <= 0 ? 0 : (xe.nx ? xe.nx : te.nblocks);
  if (nc + ne == 0) return;
  if (fused_mode3(xc) && !xe.nx) {
    launch_fused<true>(grad, tc, a, xc, te, xe, nc, ne, s);
    return;
  }
  hipLaunchKernelGGL(xgmi_end_kernel, dim3(nc + ne), dim3(256), 0, s, grad, tc, a, xc, te, xe, nc);
}

void launch_reduce_optim(float* grad, const RedTable& tab, const OptimArgs& a, hipStream_t s,
                         const XgmiPush* xp) {
  if (tab.nblocks <= 0) return;
  if (xp && xp->on) {
    const int grid = xp->mode >= 2 && xp->nx ? xp->nx : (xp->mode == 4 ? xp->b_hi - xp->b_lo : tab.nblocks);
    if (grid <= 0) return;
    if (fused_mode3(*xp)) {
      launch_fused<false>(grad, tab, a, *xp, tab, *xp, grid, 0, s);
      return;
    }
    hipLaunchKernelGGL(xgmi_early_kernel, dim3(grid), dim3(256), 0, s, grad, tab, a, *xp);
    return;
  }
  const dim3 g(tab.nblocks), b(256);
  switch (a.kind) {
    case OPT_ADAM: hipLaunchKernelGGL(reduce_optim_kernel<OPT_ADAM>, g, b, 0, s, grad, tab, a); break;
    case OPT_NADAM: hipLaunchKernelGGL(reduce_optim_kernel<OPT_NADAM>, g, b, 0, s, grad, tab, a); break;
    case OPT_ADADELTA: hipLaunchKernelGGL(reduce_optim_kernel<OPT_ADADELTA>, g, b, 0, s, grad, tab, a); break;
    case OPT_RMSPROP: hipLaunchKernelGGL(reduce_optim_kernel<OPT_RMSPROP>, g, b, 0, s, grad, tab, a); break;
    default: hipLaunchKernelGGL(reduce_optim_kernel<OPT_SGD>, g, b, 0, s, grad, tab, a); break;
  }
}
