// Dense forward (K8): Y = act(X W + b) with split-K MFMA partials + a fused epilogue.
//
// M (= batch) is small (64-4096) and K is large (1,152-65,536) for the reference models,
// so a plain MxN tiling leaves most of the 256 CUs idle.  The K axis is split across
// waves (grid covers m-tiles x n-tiles x splits, one 16x16 output tile per wave, A and B
// fragments loaded straight to VGPRs as 16-byte accesses) and partials land in an fp32
// slab; dense_epilogue reduces the splits in fixed order (deterministic) and applies
// bias + ReLU + dropout, writing the bf16 activation the next layer consumes.
//
// The same kernel computes the dense backward dX = dH W^T (mode 1, one split) with the
// bf16 "transposed" pack, routing every output element straight back through the previous
// stage's dropout / ReLU masks (flattened conv dP or hidden-dense dH).
#include "dense_body.h"
#include "step_book.h"

__global__ __launch_bounds__(256) void dense_splitk_kernel(const DenseFwdArgs a) {
  // prologue-free step: this step's bookkeeping (no workgroup of this launch reads its
  // scalars; every later launch of the step does) in an extra LAST workgroup of its own, so
  // its dependent double-precision chain delays no split-K tile
  if (a.book && blockIdx.x == gridDim.x - 1) {
    if (threadIdx.x == 0) step_bookkeeping(a.sb);
    return;
  }
  dense_splitk_body(a, blockIdx.x);
}

// Large-weight path (legacy RPV Dense(512) on a 65,536-wide input: 67 MB of bf16 weights,
// and its dX).  The small-weight kernel above re-reads every weight fragment once per
// 16-row m-tile, which for a weight matrix that does not stay in L2 multiplies the
// dominant HBM stream by M/16.  Here one 512-thread workgroup owns ALL rows of its m-group
// (128) x 8 n-tiles (one per wave) over a K-split:
//   * the activation tile (128 rows x 32 k per k-step) is staged once per workgroup in LDS
//     (one 16-B load per thread per k-step, rows padded to 40 elements for conflict-light
//     fragment reads) and feeds all 8 waves;
//   * each wave streams only its own weight fragments (1 KB coalesced per k-step) straight
//     into VGPRs -- every weight byte crosses HBM once;
//   * DL_KST k-steps per stage, double-buffered in LDS and registers: the next stage's
//     loads (~32 KB per workgroup) are in flight while the current stage's MFMAs run.
namespace {
constexpr int DL_KST = 4;
constexpr int DL_LDA = 40;
constexpr int DL_ROWS = 128;
constexpr long long DL_BIG_BYTES = 8ll << 20;   // weight bytes above which the LDS path is used
}

__global__ __launch_bounds__(512) void dense_lds_kernel(const DenseFwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if (a.book && blockIdx.x == gridDim.x - 1) {   // (as dense_splitk: an extra last workgroup)
    if (threadIdx.x == 0) step_bookkeeping(a.sb);
    return;
  }
  bf16* const As = reinterpret_cast<bf16*>(smem);  // [2][DL_KST][DL_ROWS][DL_LDA]
  constexpr int STG = DL_KST * DL_ROWS * DL_LDA;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 15, g = lane >> 4;
  const int nblocks = (a.NT + 7) / 8, mgroups = (a.M + DL_ROWS - 1) / DL_ROWS;
  // XCD-aware order: workgroup b runs on XCD b % 8, so the n-blocks of one (m-group, K-split)
  // -- which read the same activation slice -- are given consecutive logical indices on ONE
  // XCD and share its L2 (else every n-block's XCD fetches the slice from HBM again)
  const int nwg = (int)gridDim.x - (a.book ? 1 : 0);
  int bid = (int)blockIdx.x;
  if (nwg % 8 == 0 && (nwg / 8) % nblocks == 0) bid = (bid % 8) * (nwg / 8) + bid / 8;
  const int nb = bid % nblocks;
  const int t2 = bid / nblocks;
  const int mg = t2 % mgroups, s = t2 / mgroups;
  const int nt = nb * 8 + wave;
  const int ntc = min(nt, a.NT - 1);
  const int arow = mg * DL_ROWS + (tid >> 2);
  const bool av = arow < a.M;
  const bf16* ap = a.x + (size_t)(av ? arow : 0) * a.Ks + (tid & 3) * 8;
  const int ks_lo = s * a.ks_per_split;
  const int ks_hi = min(a.KS, ks_lo + a.ks_per_split);
  const int nst = (ks_hi - ks_lo + DL_KST - 1) / DL_KST;
  // weights stream to registers TWO stages ahead (three register sets in rotation: ~64 KB of
  // weight loads in flight per workgroup -- one stage ahead left the HBM stream latency-bound);
  // the activation slice goes one stage ahead through LDS (double-buffered)
  bf16x8 ra[DL_KST], w0[DL_KST], w1[DL_KST], w2[DL_KST];
  auto load_w = [&](bf16x8 (&w)[DL_KST], int st) {
#pragma unroll
    for (int kk = 0; kk < DL_KST; ++kk) {
      const int k = ks_lo + st * DL_KST + kk;
      const int ks = k < ks_hi ? k : ks_hi - 1;
      w[kk] = load_bf16x8(a.wpk + ((size_t)(ks * a.NT + ntc) * 64 + lane) * 8);
    }
  };
  auto load_a = [&](int st) {
#pragma unroll
    for (int kk = 0; kk < DL_KST; ++kk) {
      const int k = ks_lo + st * DL_KST + kk;
      const bool kv = k < ks_hi;
      const int ks = kv ? k : ks_hi - 1;
      const int k0 = ks * 32 + (tid & 3) * 8;
      ra[kk] = load_bf16x8_if(kv && av && k0 < a.Ks, ap + ks * 32, a.x);
    }
  };
  auto stash_a = [&](int buf) {
#pragma unroll
    for (int kk = 0; kk < DL_KST; ++kk)
      *reinterpret_cast<bf16x8*>(As + buf * STG + kk * DL_ROWS * DL_LDA + (tid >> 2) * DL_LDA + (tid & 3) * 8) = ra[kk];
  };
  f32x4 acc[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto step = [&](const bf16x8 (&cur)[DL_KST], bf16x8 (&ahead)[DL_KST], int st) {
    const bool more = st + 1 < nst;
    if (more) load_a(st + 1);
    if (st + 2 < nst) load_w(ahead, st + 2);
    const bf16* A = As + (st & 1) * STG;
#pragma unroll
    for (int kk = 0; kk < DL_KST; ++kk) {
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(A + kk * DL_ROWS * DL_LDA + (t * 16 + r) * DL_LDA + 8 * g);
        acc[t] = mfma16(af, cur[kk], acc[t]);
      }
    }
    if (more) stash_a((st & 1) ^ 1);
    __syncthreads();
  };
  if (nst > 0) {
    load_a(0);
    load_w(w0, 0);
    stash_a(0);
  }
  if (nst > 1) load_w(w1, 1);
  __syncthreads();
  for (int st = 0; st < nst; st += 3) {
    step(w0, w2, st);
    if (st + 1 < nst) step(w1, w0, st + 1);
    if (st + 2 < nst) step(w2, w1, st + 2);
  }
  if (a.mode == 1 && a.bt.pCs % 8 == 0) {
    // dX epilogue: the workgroup's 128 rows x 128 columns go through LDS (the operand buffers
    // are dead after the loop's last barrier) so that every thread finishes whole 8-column runs
    // -- one 16-byte load of the saved activation and one 16-byte store per run, 16 threads
    // covering 256 contiguous bytes of a row (the per-element form stored 32-byte pieces)
    constexpr int LDE = 8 * 16 + 4;
    float* ep = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int t = 0; t < 8; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) ep[(t * 16 + g * 4 + j) * LDE + wave * 16 + r] = acc[t][j];
    __syncthreads();
    const BwdThrough& bt = a.bt;
    const uint32_t step = a.st ? (uint32_t)a.st->t : 0u;
    const int width = bt.pH * bt.pW * bt.pCs, pix = bt.pH * bt.pW;
#pragma unroll
    for (int q = 0; q < DL_ROWS * 16 / 512; ++q) {
      const int e = tid + 512 * q, rr = e >> 4, c8 = e & 15;
      const int m = mg * DL_ROWS + rr, n = nb * 128 + c8 * 8;
      if (m >= a.M || n >= width) continue;
      float v[8];
      const f32x4 lo = *reinterpret_cast<const f32x4*>(ep + rr * LDE + c8 * 8);
      const f32x4 hi = *reinterpret_cast<const f32x4*>(ep + rr * LDE + c8 * 8 + 4);
#pragma unroll
      for (int k = 0; k < 4; ++k) { v[k] = lo[k]; v[4 + k] = hi[k]; }
      const int px = n / bt.pCs;
      bwd_through_store8(bt, (size_t)m * pix + px, n - px * bt.pCs, v, step);
    }
    return;
  }
  if (nt >= a.NT) return;
  if (a.mode == 1) {
    const BwdThrough& bt = a.bt;
    const uint32_t step = a.st ? (uint32_t)a.st->t : 0u;
    const int col = nt * 16 + r;
    if (col >= bt.pH * bt.pW * bt.pCs) return;
    const int y = col / (bt.pW * bt.pCs);
    const int rem = col - y * bt.pW * bt.pCs;
    const int x = rem / bt.pCs;
    const int c = rem - x * bt.pCs;
#pragma unroll
    for (int t = 0; t < 8; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = mg * DL_ROWS + t * 16 + g * 4 + j;
        if (m < a.M) bwd_through_store(bt, m, y, x, c, acc[t][j], step);
      }
    return;
  }
  const int ld = a.NT * 16;
  float* out = a.part + (size_t)s * a.M * ld;
#pragma unroll
  for (int t = 0; t < 8; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = mg * DL_ROWS + t * 16 + g * 4 + j;
      if (m < a.M) out[(size_t)m * ld + nt * 16 + r] = acc[t][j];
    }
}

bool dense_big(int NT, int KS) { return (long long)NT * KS * 1024 > DL_BIG_BYTES; }

// Work items per K-split: waves (small path) or workgroups (large-weight path).
int dense_groups(int M, int NT, int KS) {
  if (dense_big(NT, KS)) return ((M + DL_ROWS - 1) / DL_ROWS) * ((NT + 7) / 8);
  return ((M + 15) / 16) * NT;
}

// 64 outputs per workgroup, the 4 waves split the K-splits (independent loads in flight),
// fixed-order LDS combine (deterministic).
__global__ __launch_bounds__(256) void dense_epilogue_kernel(const DenseEpiArgs a) {
  __shared__ float red[256];
  const int l = threadIdx.x & 63, sg = threadIdx.x >> 6;
  const long long idx = (long long)blockIdx.x * 64 + l;
  const bool in = idx < (long long)a.M * a.Ns;
  const int m = in ? (int)(idx / a.Ns) : 0;
  const int n = in ? (int)(idx - (long long)m * a.Ns) : 0;
  float part = 0.f;
  if (in && n < a.N) {
    const size_t stride = (size_t)a.M * a.ldp;
    const float* p = a.part + (size_t)m * a.ldp + n;
    float a0 = 0.f, a1 = 0.f;
    int s = sg;
    for (; s + 4 < a.splits; s += 8) {
      a0 += p[(size_t)s * stride];
      a1 += p[(size_t)(s + 4) * stride];
    }
    for (; s < a.splits; s += 4) a0 += p[(size_t)s * stride];
    part = a0 + a1;
  }
  red[threadIdx.x] = part;
  __syncthreads();
  if (sg != 0 || !in) return;
  float v = 0.f;
  if (n < a.N) {
    v = (red[l] + red[l + 64]) + (red[l + 128] + red[l + 192]);
    if (a.bias) v += a.bias[n];
    if (a.relu) v = fmaxf(v, 0.f);
    if (a.drop_thr) {
      const uint32_t step = a.st ? (uint32_t)a.st->t : 0u;
      v = dropout_keep((uint32_t)(m * a.N + n), a.seed, a.stream_id, step, a.drop_thr) ? v * a.drop_scale : 0.f;
    }
  }
  a.out[idx] = f2bf(v);
}

void launch_dense_fwd(const DenseFwdArgs& a, hipStream_t s) {
  if (dense_big(a.NT, a.KS)) {
    const long long wgs = (long long)dense_groups(a.M, a.NT, a.KS) * a.splits;
    const size_t lds = (size_t)2 * DL_KST * DL_ROWS * DL_LDA * sizeof(bf16);
    hipLaunchKernelGGL(dense_lds_kernel, dim3((unsigned)(wgs + (a.book ? 1 : 0))), dim3(512), lds, s, a);
    return;
  }
  const long long waves = (long long)((a.M + 15) / 16) * a.NT * a.splits;
  hipLaunchKernelGGL(dense_splitk_kernel, dim3((unsigned)((waves + 3) / 4 + (a.book ? 1 : 0))), dim3(256), 0, s, a);
}
void launch_dense_epi(const DenseEpiArgs& a, hipStream_t s) {
  const long long n = (long long)a.M * a.Ns;
  hipLaunchKernelGGL(dense_epilogue_kernel, dim3((unsigned)((n + 63) / 64)), dim3(256), 0, s, a);
}
