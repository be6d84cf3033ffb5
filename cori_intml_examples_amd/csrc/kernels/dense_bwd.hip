// Dense-layer backward on gfx950: the weight gradient dW = X^T dH and the input gradient
// dX = dH W^T (routed through the previous stage's dropout / ReLU masks), designed for the
// reference models' shapes: a large flattened width K (4,096-65,536 features), a small
// output width N (128-512) and a batch M of 128-4,096 rows.
//
// Both GEMMs are tiny in FLOPs (about 0.3 us of MFMA time at batch 1024 for RPV) and are
// bound by load latency, so the kernels are built around keeping loads in flight:
//
// dense_wgrad_kernel<KG, NTT>  (grid: row splits x feature groups x n groups)
//   * a workgroup owns KG*16 features x NTT*16 outputs over a range of batch rows; its four
//     waves take interleaved 32-row chunks and accumulate independently -- each wave stages
//     its chunk in a PRIVATE LDS region, so the chunk loop has no workgroup barrier;
//   * the next chunk's global loads are issued before the current chunk's MFMAs
//     (register double buffer);
//   * both operands have the batch (the reduction axis) outermost, so fragments are read
//     with ds_read_b64_tr_b16 from row-major tiles whose 8-row blocks are each shifted by a
//     further 128 B: the two 32-lane groups of the transposed read then hit disjoint banks;
//   * the bias gradient (column sums of dH) is summed from the dH fragments the MFMAs already
//     read (8 rows per lane), in the feature-group-0 workgroups;
//   * the four waves' partials are summed in fixed order through LDS (deterministic) and
//     stored as coalesced float4 rows of the [split][K][N] slab, the layout slab_reduce reads;
//     with one split that slab IS the Keras gradient, and the kernel can apply the optimizer
//     update to those elements right there (WgradArgs::opt_w), so the layer never enters
//     the end-of-step reduction.
//
// dense_dx_kernel<NTC>  (grid: 64-row groups x n groups)
//   * a wave owns 16 rows x NTC*16 columns: each dH fragment feeds NTC MFMAs;
//   * the result goes through a per-wave LDS tile so every lane finishes with 8 consecutive
//     columns: one 16-byte load of the saved activation (ReLU mask) and one 16-byte store of
//     the gradient per 8 outputs (bwd_through_store8), instead of 2-byte scattered accesses.
//
// dense_bwd_pair_kernel runs both bodies in one launch (they read the same dH and write
// disjoint buffers), the dX workgroups first: they are short and fill the machine while the
// fewer, longer wgrad workgroups run.
#include <algorithm>
#include <stdexcept>

#include "dense_body.h"
#include "optim_math.h"

namespace {
constexpr int DW_LDA = 48;   // A tile row stride (elements): 32 features + pad

__device__ __forceinline__ bf16x4 tr_read4(const bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS_PTR(bf16x4, p));
}

template <int NTT>
struct DwGeom {
  static constexpr int LDB = (NTT * 16 > 32 ? NTT * 16 : 32) + 16;   // dH tile row stride
  static constexpr int A_ELEMS = 32 * DW_LDA + 192;
  static constexpr int B_ELEMS = 32 * LDB + 192;
  static constexpr int WAVE_BYTES = (A_ELEMS + B_ELEMS) * 2;
  static constexpr int LDR = NTT * 16 + 4;                           // fp32 reduce row stride
};

// row r of a staged 32-row tile: each block of 8 rows starts 64 elements (128 B) further on
// than the plain stride puts it, so rows 8g+q of the lane groups g = 0/1 (and 2/3) of a
// transposed read land in opposite bank halves (the blocks never overlap)
__device__ __forceinline__ int dw_row(int r, int ld) { return r * ld + (r >> 3) * 64; }

// the Keras update of one element, optimizer kind chosen at run time (wave-uniform)
__device__ __forceinline__ void dw_opt(const OptimArgs& o, float& p, float g, float* s0, float* s1) {
  switch (o.kind) {
    case OPT_ADAM: opt_update<OPT_ADAM>(o, o.st, p, g, s0, s1); break;
    case OPT_NADAM: opt_update<OPT_NADAM>(o, o.st, p, g, s0, s1); break;
    case OPT_ADADELTA: opt_update<OPT_ADADELTA>(o, o.st, p, g, s0, s1); break;
    case OPT_RMSPROP: opt_update<OPT_RMSPROP>(o, o.st, p, g, s0, s1); break;
    default: opt_update<OPT_SGD>(o, o.st, p, g, s0, s1); break;
  }
}

// fused update of 4 consecutive elements [e, e+4) whose gradient is g; p / s0 / s1 are
// their current values (loaded early by the caller); returns the updated weights
__device__ __forceinline__ f32x4 dw_opt4(const OptimArgs& o, size_t e, const f32x4& g, f32x4 p, f32x4 s0, f32x4 s1) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float pq = p[q], m = s0[q], v = s1[q];
    dw_opt(o, pq, g[q] * o.grad_scale, &m, &v);
    p[q] = pq, s0[q] = m, s1[q] = v;
  }
  *reinterpret_cast<f32x4*>(o.p + e) = p;
  if (o.s0) *reinterpret_cast<f32x4*>(o.s0 + e) = s0;
  if (o.s1) *reinterpret_cast<f32x4*>(o.s1 + e) = s1;
  return p;
}

constexpr int DW_PKLD = 128 + 8;   // bf16 row stride of the updated-weight tile (<= 128 outputs)
}   // namespace

size_t dense_wgrad_lds_bytes(int kg, int ntt) {
  size_t stage = 0, red = 0;
  switch (ntt) {
    case 1: stage = 4 * DwGeom<1>::WAVE_BYTES; red = (size_t)4 * 16 * DwGeom<1>::LDR * 4; break;
    case 2: stage = 4 * DwGeom<2>::WAVE_BYTES; red = (size_t)4 * 16 * DwGeom<2>::LDR * 4; break;
    case 4: stage = 4 * DwGeom<4>::WAVE_BYTES; red = (size_t)4 * 16 * DwGeom<4>::LDR * 4; break;
    default: stage = 4 * DwGeom<8>::WAVE_BYTES; red = (size_t)4 * 16 * DwGeom<8>::LDR * 4; break;
  }
  (void)kg;
  // + the updated-weight bf16 tile of the fused optimizer's pack writes (32 x <= 128)
  return std::max(stage, red + 16 * 128 * 4 + (size_t)32 * DW_PKLD * 2);
}

// LATE: the optimizer state of the fused update is loaded after the chunk loop instead of
// before it (fewer registers live across the MFMAs: 4 waves / SIMD instead of 3 for NTT 4)
template <int KG, int NTT, bool OPT, bool LATE = false>
__device__ __forceinline__ void dense_wgrad_body(const WgradArgs& a, const int bx, const int by, const int bz,
                                                 char* smem) {
  using G = DwGeom<NTT>;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, i = lane & 15, g = lane >> 4;
  bf16* As = reinterpret_cast<bf16*>(smem) + (size_t)wave * (G::A_ELEMS + G::B_ELEMS);
  bf16* Bs = As + G::A_ELEMS;
  const int f0 = by * KG * 16, n0 = bz * NTT * 16;
  const int r_begin = bx * a.px_per_split;
  const int r_end = min(a.P, r_begin + a.px_per_split);
  const int nchunks = max(0, (r_end - r_begin + 31) >> 5);
  const bool do_bias = a.bslab != nullptr && by == 0;

  // per-lane load slots: A pieces (row, 8 features), B pieces (row, 8 outputs)
  bf16x8 ra[KG], rb[NTT];
  auto issue = [&](int c) {
    const int r0 = r_begin + c * 32;
#pragma unroll
    for (int u = 0; u < KG; ++u) {
      const int pc = lane + 64 * u, row = pc / (KG * 2), q = pc - row * (KG * 2);
      const int f = f0 + q * 8;
      ra[u] = load_bf16x8_if(r0 + row < r_end && f < a.Cs_in, a.x + (size_t)(r0 + row) * a.Cs_in + f, a.x);
    }
#pragma unroll
    for (int u = 0; u < NTT; ++u) {
      const int pc = lane + 64 * u, row = pc / (NTT * 2), q = pc - row * (NTT * 2);
      const int n = n0 + q * 8;
      rb[u] = load_bf16x8_if(r0 + row < r_end && n < a.Cs_dy, a.dy + (size_t)(r0 + row) * a.Cs_dy + n, a.dy);
    }
  };
  auto stash = [&]() {
#pragma unroll
    for (int u = 0; u < KG; ++u) {
      const int pc = lane + 64 * u, row = pc / (KG * 2), q = pc - row * (KG * 2);
      *reinterpret_cast<bf16x8*>(As + dw_row(row, DW_LDA) + q * 8) = ra[u];
    }
#pragma unroll
    for (int u = 0; u < NTT; ++u) {
      const int pc = lane + 64 * u, row = pc / (NTT * 2), q = pc - row * (NTT * 2);
      *reinterpret_cast<bf16x8*>(Bs + dw_row(row, G::LDB) + q * 8) = rb[u];
    }
  };

  f32x4 acc[KG][NTT];
  float bsum[NTT];
#pragma unroll
  for (int nt = 0; nt < NTT; ++nt) {
    bsum[nt] = 0.f;
#pragma unroll
    for (int kt = 0; kt < KG; ++kt) acc[kt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  // OPT: the optimizer state of the elements this thread will finalise is loaded now, so
  // its latency hides behind the chunk loop instead of trailing the reduction
  const int ld = a.NT * 16;
  constexpr int C4 = NTT * 4;                                    // float4 per 16-feature row
  constexpr int NQ = (16 * C4 + 255) / 256;                      // float4 per thread per k-tile
  f32x4 op[OPT ? KG : 1][NQ], om[OPT ? KG : 1][NQ], ov[OPT ? KG : 1][NQ];
  auto load_state = [&]() {
    const OptimArgs& o = a.opt;
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kt = 0; kt < KG; ++kt)
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int e = tid + 256 * q, row = e / C4, c4 = e - row * C4;
        const int f = f0 + kt * 16 + row, n = n0 + c4 * 4;
        const bool ok = e < 16 * C4 && f < a.Ktiles * 16 && n < ld;
        const size_t x = ok ? (size_t)a.opt_w + (size_t)f * ld + n : 0;
        op[kt][q] = ok ? *reinterpret_cast<const f32x4*>(o.p + x) : z;
        om[kt][q] = (ok && o.s0) ? *reinterpret_cast<const f32x4*>(o.s0 + x) : z;
        ov[kt][q] = (ok && o.s1) ? *reinterpret_cast<const f32x4*>(o.s1 + x) : z;
      }
  };
  if constexpr (OPT && !LATE) load_state();

  // fragment read rows: lane reads rows 8g + (i>>2) (lo) and +4 (hi), 4 columns at 4*(i&3)
  const int rd = 8 * g + (i >> 2);
  if (wave < nchunks) issue(wave);
  for (int c = wave; c < nchunks; c += 4) {
    stash();
    __builtin_amdgcn_wave_barrier();
    if (c + 4 < nchunks) issue(c + 4);
    bf16x8 afr[KG];
#pragma unroll
    for (int kt = 0; kt < KG; ++kt) {
      const bf16* p = As + dw_row(rd, DW_LDA) + kt * 16 + 4 * (i & 3);
      afr[kt] = __builtin_shufflevector(tr_read4(p), tr_read4(p + 4 * DW_LDA), 0, 1, 2, 3, 4, 5, 6, 7);
    }
#pragma unroll
    for (int nt = 0; nt < NTT; ++nt) {
      const bf16* p = Bs + dw_row(rd, G::LDB) + nt * 16 + 4 * (i & 3);
      const bf16x8 bfr = __builtin_shufflevector(tr_read4(p), tr_read4(p + 4 * G::LDB), 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
      for (int kt = 0; kt < KG; ++kt) acc[kt][nt] = mfma16(afr[kt], bfr, acc[kt][nt]);
      if (do_bias) {   // the lane's 8 rows of column nt*16+i (lane groups summed at the end)
        float s0 = 0.f, s1 = 0.f;
#pragma unroll
        for (int q = 0; q < 4; ++q) { s0 += bf2f(bfr[q]); s1 += bf2f(bfr[4 + q]); }
        bsum[nt] += s0 + s1;
      }
    }
    __builtin_amdgcn_wave_barrier();
  }

  if constexpr (OPT && LATE) load_state();
  // fixed-order cross-wave sum (w0 + w1 + w2 + w3), one 16-feature k-tile per pass
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);                   // [4 waves][16][LDR]
  float* bred = red + 4 * 16 * G::LDR;                           // [4 waves][4 groups][128]
  bf16* pkt = reinterpret_cast<bf16*>(bred + 16 * 128);          // [KG*16][DW_PKLD] updated weights
  const bool packs = OPT && a.pk_fwd >= 0;
  float* slab = a.slab + (size_t)bx * a.Ktiles * 16 * ld;
  if (do_bias) {
#pragma unroll
    for (int nt = 0; nt < NTT; ++nt) bred[(wave * 4 + g) * 128 + nt * 16 + i] = bsum[nt];
  }
#pragma unroll
  for (int kt = 0; kt < KG; ++kt) {
    float* rw = red + wave * 16 * G::LDR;
#pragma unroll
    for (int nt = 0; nt < NTT; ++nt)
#pragma unroll
      for (int j = 0; j < 4; ++j) rw[(4 * g + j) * G::LDR + nt * 16 + i] = acc[kt][nt][j];
    __syncthreads();
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int e = tid + 256 * q;
      if (e >= 16 * C4) break;
      const int row = e / C4, c4 = e - row * C4;
      const int f = f0 + kt * 16 + row, n = n0 + c4 * 4;
      f32x4 s = *reinterpret_cast<const f32x4*>(red + row * G::LDR + c4 * 4);
#pragma unroll
      for (int w = 1; w < 4; ++w) s += *reinterpret_cast<const f32x4*>(red + (w * 16 + row) * G::LDR + c4 * 4);
      if (f < a.Ktiles * 16 && n < ld) {
        if (!(OPT && a.opt_nograd)) *reinterpret_cast<f32x4*>(slab + (size_t)f * ld + n) = s;
        if constexpr (OPT) {
          const f32x4 pn = dw_opt4(a.opt, (size_t)a.opt_w + (size_t)f * ld + n, s, op[kt][q], om[kt][q], ov[kt][q]);
          if (packs) {
            bf16* d = pkt + (kt * 16 + row) * DW_PKLD + c4 * 4;
#pragma unroll
            for (int u = 0; u < 4; ++u) d[u] = f2bf(pn[u]);
          }
        }
      }
    }
    __syncthreads();
  }
  if constexpr (OPT) {
    if (packs && KG * 16 == 32) {
      // whole 16-byte vectors of both packs from the tile (the loop's last barrier published it):
      //   fwd  B[k = feature][n = output]: vector (ks = f0/32, nt, lane) = 8 features of one output
      //   bwd  B[k = output][n = feature]: vector (ksb, ntb, lane)       = 8 outputs of one feature
      bf16* ar = a.opt.arena;
      const int ks = f0 >> 5;
      for (int v = tid; v < NTT * 64; v += 256) {
        const int ntl = v >> 6, lane_ = v & 63, nt = (n0 >> 4) + ntl;
        if (nt >= a.NT) continue;
        bf16x8 w;
#pragma unroll
        for (int j = 0; j < 8; ++j) w[j] = pkt[(8 * (lane_ >> 4) + j) * DW_PKLD + ntl * 16 + (lane_ & 15)];
        *reinterpret_cast<bf16x8*>(ar + a.pk_fwd + ((size_t)(ks * a.pk_NT + nt) * 64 + lane_) * 8) = w;
      }
      if (a.pk_bwd >= 0 && (NTT & 1) == 0) {
        for (int v = tid; v < (NTT / 2) * KG * 64; v += 256) {
          const int lane_ = v & 63, t2 = v >> 6, ntbl = t2 % KG, ksbl = t2 / KG;
          const int ksb = (n0 >> 5) + ksbl, ntb = (f0 >> 4) + ntbl;
          if (n0 + ksbl * 32 >= ld) continue;
          const bf16x8 w = *reinterpret_cast<const bf16x8*>(pkt + (ntbl * 16 + (lane_ & 15)) * DW_PKLD + ksbl * 32 +
                                                            8 * (lane_ >> 4));
          *reinterpret_cast<bf16x8*>(ar + a.pk_bwd + ((size_t)(ksb * a.pk_NTb + ntb) * 64 + lane_) * 8) = w;
        }
      }
    }
  }
  if (do_bias && tid < NTT * 16 && n0 + tid < ld) {
    float b = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) b += bred[q * 128 + tid];     // fixed order: wave-major, group
    a.bslab[(size_t)bx * ld + n0 + tid] = b;
    if (OPT && a.opt_b >= 0) {
      const OptimArgs& o = a.opt;
      const int e = a.opt_b + n0 + tid;
      float p = o.p[e], s0 = o.s0 ? o.s0[e] : 0.f, s1 = o.s1 ? o.s1[e] : 0.f;
      dw_opt(o, p, b * o.grad_scale, &s0, &s1);
      o.p[e] = p;
      if (o.s0) o.s0[e] = s0;
      if (o.s1) o.s1[e] = s1;
    }
  }
  if (OPT && !packs && a.opt.defer_pack && bx == 0 && by == 0 && bz == 0 && tid == 0) a.opt.st->packs_stale = 1;
}

template <int NTC>
__device__ __forceinline__ void dense_dx_body(const DenseFwdArgs& a, const int bx, const int by, char* smem) {
  constexpr int LDE = NTC * 16 + 4;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 15, g = lane >> 4;
  float* ep = reinterpret_cast<float*>(smem) + wave * 16 * LDE;
  const int mt = bx * 4 + wave;
  const int nt0 = by * NTC;
  const int row = mt * 16 + r;
  const bool rv = row < a.M;
  const bf16* xr = a.x + (size_t)(rv ? row : 0) * a.Ks;
  f32x4 acc[NTC];
#pragma unroll
  for (int nt = 0; nt < NTC; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int kb = 0; kb < a.KS; kb += 4) {
    bf16x8 af[4], bfr[4][NTC];
#pragma unroll
    for (int u = 0; u < 4; ++u) {   // independent, branch-free loads
      const int ks = min(kb + u, a.KS - 1);
      const int k0 = ks * 32 + g * 8;
      af[u] = load_bf16x8_if(rv && k0 < a.Ks && kb + u < a.KS, xr + k0, a.x);
#pragma unroll
      for (int nt = 0; nt < NTC; ++nt) {
        const int ntc = min(nt0 + nt, a.NT - 1);
        bfr[u][nt] = load_bf16x8(a.wpk + ((size_t)(ks * a.NT + ntc) * 64 + lane) * 8);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int nt = 0; nt < NTC; ++nt) acc[nt] = mfma16(af[u], bfr[u][nt], acc[nt]);
  }
  // stage [16 rows][NTC*16] fp32, re-read as 8-column runs
#pragma unroll
  for (int nt = 0; nt < NTC; ++nt)
#pragma unroll
    for (int j = 0; j < 4; ++j) ep[(4 * g + j) * LDE + nt * 16 + r] = acc[nt][j];
  __builtin_amdgcn_wave_barrier();
  const BwdThrough& t = a.bt;
  const uint32_t step = a.st ? (uint32_t)a.st->t : 0u;
  const int width = t.pH * t.pW * t.pCs;
  const int pix = t.pH * t.pW;
  constexpr int C8 = NTC * 2;
  for (int e = lane; e < 16 * C8; e += 64) {
    const int rr = e / C8, c8 = e - rr * C8;
    const int m = mt * 16 + rr, n = nt0 * 16 + c8 * 8;
    if (m >= a.M || n >= width) continue;
    float v[8];
    const f32x4 lo = *reinterpret_cast<const f32x4*>(ep + rr * LDE + c8 * 8);
    const f32x4 hi = *reinterpret_cast<const f32x4*>(ep + rr * LDE + c8 * 8 + 4);
#pragma unroll
    for (int k = 0; k < 4; ++k) { v[k] = lo[k]; v[4 + k] = hi[k]; }
    const int px = n / t.pCs;
    bwd_through_store8(t, (size_t)m * pix + px, n - px * t.pCs, v, step);
  }
}

size_t dense_dx_lds_bytes(int ntc) { return (size_t)4 * 16 * (ntc * 16 + 4) * 4; }

// order 0: grid (splits, feature groups, n groups), feature groups fastest.  order 1 / 2: a 1-D
// grid with the n groups of one feature group consecutive -- the workgroups resident together
// then cover whole rows of the [K][N] weight / optimizer-state arrays (contiguous HBM ranges
// instead of one 16 * NTT * 4-byte strip of every row) and share their x slice; order 2 also
// hands each XCD (dispatch round-robins workgroup ids over the 8) a contiguous range of tiles,
// so that x slice is fetched into one L2 (needs a grid that is a multiple of 8)
template <int KG, int NTT, bool OPT, bool LATE = false>
__global__ __launch_bounds__(256, LATE ? 4 : 1) void dense_wgrad_kernel(const WgradArgs a, const int order) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if (order == 0) {
    dense_wgrad_body<KG, NTT, OPT, LATE>(a, blockIdx.x, blockIdx.y, blockIdx.z, smem);
    return;
  }
  const int ny = (a.Ktiles + KG - 1) / KG, nz = (a.NT + NTT - 1) / NTT;
  int id = blockIdx.x;
  if (order == 2) id = (id & 7) * (gridDim.x >> 3) + (id >> 3);
  const int bz = id % nz;
  id /= nz;
  dense_wgrad_body<KG, NTT, OPT, LATE>(a, id / ny, id % ny, bz, smem);
}

template <int NTC>
__global__ __launch_bounds__(256) void dense_dx_kernel(const DenseFwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  dense_dx_body<NTC>(a, blockIdx.x, blockIdx.y, smem);
}

// dX workgroups [0, n_x) first (grid x-major over 64-row groups), then the wgrad ones
template <int KG, int NTT, bool OPT, int NTC>
__global__ __launch_bounds__(256) void dense_bwd_pair_kernel(const WgradArgs wa, const DenseFwdArgs da,
                                                             const int n_x, const int xgx, const int wgx,
                                                             const int wgy) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int id = blockIdx.x;
  if (id < n_x) {
    dense_dx_body<NTC>(da, id % xgx, id / xgx, smem);
  } else {
    id -= n_x;
    const int bx = id % wgx;
    id /= wgx;
    dense_wgrad_body<KG, NTT, OPT>(wa, bx, id % wgy, id / wgy, smem);
  }
}

// Host checks of the shapes the kernels assume (a mismatch would read or write out of range).
static void dense_wgrad_check(const WgradArgs& a, int kg, int ntt, int splits) {
  if (!(kg == 2 && (ntt == 1 || ntt == 2 || ntt == 4 || ntt == 8)))
    throw std::runtime_error("dense_wgrad: unsupported (kg, ntt)");
  if (a.Cs_in % 8 || a.Cs_dy % 8 || a.px_per_split <= 0 || a.px_per_split % 32 ||
      (long long)splits * a.px_per_split < a.P || a.KH != 1 || a.KW != 1)
    throw std::runtime_error("dense_wgrad: geometry");
  if (a.opt_w >= 0 && (splits != 1 || a.opt.p == nullptr || a.opt.st == nullptr || a.opt_w % 4 ||
                       (a.NT * 16) % 4))
    throw std::runtime_error("dense_wgrad: fused optimizer needs one split and float4-aligned rows");
  if (a.pk_fwd >= 0 && (a.opt_w < 0 || a.opt.arena == nullptr || kg != 2 || (a.pk_bwd >= 0 && (ntt & 1)) ||
                        a.Cs_in % 32 || (a.NT * 16) % 32))
    throw std::runtime_error("dense_wgrad: fused pack writes need the fused optimizer, 32-feature tiles and "
                             "32-aligned widths");
}
static void dense_dx_check(const DenseFwdArgs& a, int ntc) {
  if (!(ntc == 1 || ntc == 2 || ntc == 4) || a.mode != 1 || a.splits != 1 || a.bt.pCs % 8 || a.Ks % 8)
    throw std::runtime_error("dense_dx: geometry");
}

static dim3 dense_wgrad_grid(const WgradArgs& a, int kg, int ntt, int splits) {
  return dim3(splits, (a.Ktiles + kg - 1) / kg, (a.NT + ntt - 1) / ntt);
}
static dim3 dense_dx_grid(const DenseFwdArgs& a, int ntc) {
  return dim3((a.M + 63) / 64, (a.NT + ntc - 1) / ntc);
}

#define DW_CASES(X) X(2, 1) X(2, 2) X(2, 4) X(2, 8)

void launch_dense_wgrad(const WgradArgs& a, int kg, int ntt, int splits, hipStream_t s, int order, bool late) {
  dense_wgrad_check(a, kg, ntt, splits);
  dim3 grid = dense_wgrad_grid(a, kg, ntt, splits);
  const unsigned n = grid.x * grid.y * grid.z;
  if (order < 0 || order > 2) throw std::runtime_error("dense_wgrad: order");
  if (order == 2 && n % 8) order = 1;
  if (order) grid = dim3(n);
  const size_t lds = dense_wgrad_lds_bytes(kg, ntt);
  if (late && a.opt_w >= 0 && kg == 2 && ntt == 4) {
    hipLaunchKernelGGL((dense_wgrad_kernel<2, 4, true, true>), grid, dim3(256), lds, s, a, order);
    return;
  }
#define X(KG_, NT_)                                                                         \
  if (kg == KG_ && ntt == NT_) {                                                            \
    if (a.opt_w >= 0) hipLaunchKernelGGL((dense_wgrad_kernel<KG_, NT_, true>), grid, dim3(256), lds, s, a, order); \
    else hipLaunchKernelGGL((dense_wgrad_kernel<KG_, NT_, false>), grid, dim3(256), lds, s, a, order);             \
    return;                                                                                 \
  }
  DW_CASES(X)
#undef X
}

void launch_dense_dx(const DenseFwdArgs& a, int ntc, hipStream_t s) {
  dense_dx_check(a, ntc);
  const dim3 grid = dense_dx_grid(a, ntc);
  const size_t lds = dense_dx_lds_bytes(ntc);
  if (ntc == 1) hipLaunchKernelGGL((dense_dx_kernel<1>), grid, dim3(256), lds, s, a);
  else if (ntc == 2) hipLaunchKernelGGL((dense_dx_kernel<2>), grid, dim3(256), lds, s, a);
  else hipLaunchKernelGGL((dense_dx_kernel<4>), grid, dim3(256), lds, s, a);
}

template <int KG, int NTT, bool OPT, int NTC>
static void pair_l(const WgradArgs& wa, const DenseFwdArgs& da, int splits, size_t lds, hipStream_t s) {
  const dim3 wg = dense_wgrad_grid(wa, KG, NTT, splits), xg = dense_dx_grid(da, NTC);
  const int n_x = xg.x * xg.y, n_w = wg.x * wg.y * wg.z;
  hipLaunchKernelGGL((dense_bwd_pair_kernel<KG, NTT, OPT, NTC>), dim3(n_x + n_w), dim3(256), lds, s, wa, da, n_x,
                     (int)xg.x, (int)wg.x, (int)wg.y);
}

template <int KG, int NTT, bool OPT>
static void pair_t(const WgradArgs& wa, const DenseFwdArgs& da, int ntc, int splits, size_t lds, hipStream_t s) {
  if (ntc == 1) pair_l<KG, NTT, OPT, 1>(wa, da, splits, lds, s);
  else if (ntc == 2) pair_l<KG, NTT, OPT, 2>(wa, da, splits, lds, s);
  else pair_l<KG, NTT, OPT, 4>(wa, da, splits, lds, s);
}

void launch_dense_bwd_pair(const WgradArgs& wa, int kg, int ntt, int splits, const DenseFwdArgs& da, int ntc,
                           hipStream_t s) {
  dense_wgrad_check(wa, kg, ntt, splits);
  dense_dx_check(da, ntc);
  const size_t lds = std::max(dense_wgrad_lds_bytes(kg, ntt), dense_dx_lds_bytes(ntc));
#define X(KG_, NT_)                                   \
  if (kg == KG_ && ntt == NT_) {                      \
    if (wa.opt_w >= 0) pair_t<KG_, NT_, true>(wa, da, ntc, splits, lds, s);  \
    else pair_t<KG_, NT_, false>(wa, da, ntc, splits, lds, s);               \
    return;                                           \
  }
  DW_CASES(X)
#undef X
}
