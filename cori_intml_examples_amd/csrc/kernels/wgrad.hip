// Weight-gradient GEMM on gfx950 MFMA with hardware-transposed LDS reads.
//
//   dW[k][n] = sum_p A[p][k] * dY[p][n]        (p = output pixel, the reduction axis)
//
// In NHWC both operands have the reduction axis (pixels) OUTERMOST, so an MFMA fragment
// (8 consecutive reduction indices per lane) is strided in memory.  Each 32-pixel chunk
// is therefore staged row-major into LDS with 16-byte coalesced loads (im2col rows for A,
// dY rows for B) and read back with ds_read_b64_tr_b16 (CDNA4 T10): one instruction gives
// a lane 4 consecutive pixels of one column, two give the full 8-element fragment.
//
// Split over pixels (grid.x) with one fp32 partial slab per split (deterministic: the
// slabs are summed in fixed order by slab_reduce, no float atomics), over k-tiles
// (grid.y, 4 waves each own k-tiles w, w+4, ...) and over n-tile groups (grid.z).
// Also used for dense layers (1x1 conv over a 1x1 image, pixels = batch rows).
// Bias gradient = column sums of the staged dY tile (grid.y == 0 workgroups).
#include "dense_body.h"

__device__ __forceinline__ bf16x4 tr_read(const bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS_PTR(bf16x4, p));
}

template <int KTW, int NTT, bool CS4>
__device__ __forceinline__ void wgrad_body(const WgradArgs& a, const int bx, const int by, const int bz,
                                           char* smem) {
  const int KT = a.KT;
  const int kt0 = by * KT;
  const int ktn = min(KT, a.Ktiles - kt0);
  const int ntb = bz * NTT;
  const int lda = KT * 16 + 16;
  const int ldb = NTT * 16 + 16;
  bf16* As = reinterpret_cast<bf16*>(smem);
  bf16* Bs = As + 32 * lda;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, i = lane & 15, g = lane >> 4;
  const int HoWo = a.Ho * a.Wo;
  const int KHW = a.KH * a.KW;
  const int NTtot = a.NT;

  f32x4 acc[KTW][NTT];
#pragma unroll
  for (int u = 0; u < KTW; ++u)
#pragma unroll
    for (int v = 0; v < NTT; ++v) acc[u][v] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bacc = 0.f;
  const bool do_bias = a.bslab != nullptr && by == 0;

  const long long p_begin = (long long)bx * a.px_per_split;
  const long long p_end = min((long long)a.P, p_begin + a.px_per_split);
  const int cpr = KT * 2;
  const int cpb = NTT * 2;

  for (long long p0 = p_begin; p0 < p_end; p0 += 32) {
    for (int idx = tid; idx < 32 * cpr; idx += 256) {
      const int pr = idx / cpr, kc = idx - pr * cpr;
      const long long p = p0 + pr;
      bf16x8 v = zero_bf16x8();
      if (p < p_end && kc < ktn * 2) {
        const int pi = (int)p;
        const int b = pi / HoWo;
        const int rem = pi - b * HoWo;
        const int oy = rem / a.Wo, ox = rem - (rem / a.Wo) * a.Wo;
        const int iy0 = oy * a.stride - a.pad_t, ix0 = ox * a.stride - a.pad_l;
        const bf16* xb = a.x + (size_t)b * a.H * a.W * a.Cs_in;
        const int k0 = kt0 * 16 + kc * 8;
        if (!CS4) {
          const int tap = k0 / a.Cs_in;
          const int ci = k0 - tap * a.Cs_in;
          if (tap < KHW) {
            const int ky = tap / a.KW;
            const int iy = iy0 + ky, ix = ix0 + tap - ky * a.KW;
            if (iy >= 0 && iy < a.H && ix >= 0 && ix < a.W)
              v = load_bf16x8(xb + ((size_t)iy * a.W + ix) * a.Cs_in + ci);
          }
        } else {
#pragma unroll
          for (int hh = 0; hh < 2; ++hh) {
            const int tap = (k0 >> 2) + hh;
            if (tap < KHW) {
              const int ky = tap / a.KW;
              const int iy = iy0 + ky, ix = ix0 + tap - ky * a.KW;
              if (iy >= 0 && iy < a.H && ix >= 0 && ix < a.W) {
                const bf16x4 u = load_bf16x4(xb + ((size_t)iy * a.W + ix) * 4);
#pragma unroll
                for (int q = 0; q < 4; ++q) v[hh * 4 + q] = u[q];
              }
            }
          }
        }
      }
      *reinterpret_cast<bf16x8*>(As + pr * lda + kc * 8) = v;
    }
    for (int idx = tid; idx < 32 * cpb; idx += 256) {
      const int pr = idx / cpb, nc = idx - pr * cpb;
      const long long p = p0 + pr;
      const int n0 = (ntb * 16) + nc * 8;
      bf16x8 v = zero_bf16x8();
      if (p < p_end && n0 < a.Cs_dy) v = load_bf16x8(a.dy + (size_t)p * a.Cs_dy + n0);
      *reinterpret_cast<bf16x8*>(Bs + pr * ldb + nc * 8) = v;
    }
    __syncthreads();

    if (do_bias && tid < NTT * 16) {
#pragma unroll 8
      for (int pr = 0; pr < 32; ++pr) bacc += bf2f(Bs[pr * ldb + tid]);
    }

    bf16x8 bfr[NTT];
#pragma unroll
    for (int nt = 0; nt < NTT; ++nt) {
      const bf16* base = Bs + (8 * g + (i >> 2)) * ldb + nt * 16 + 4 * (i & 3);
      const bf16x4 lo = tr_read(base);
      const bf16x4 hi = tr_read(base + 4 * ldb);
      bfr[nt] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    }
#pragma unroll
    for (int u = 0; u < KTW; ++u) {
      const int kt = wave + 4 * u;
      if (kt < ktn) {
        const bf16* base = As + (8 * g + (i >> 2)) * lda + kt * 16 + 4 * (i & 3);
        const bf16x4 lo = tr_read(base);
        const bf16x4 hi = tr_read(base + 4 * lda);
        const bf16x8 afr = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
        for (int nt = 0; nt < NTT; ++nt) acc[u][nt] = mfma16(afr, bfr[nt], acc[u][nt]);
      }
    }
    __syncthreads();
  }

  const int ld = NTtot * 16;
  float* slab = a.slab + (size_t)bx * a.Ktiles * 16 * ld;
#pragma unroll
  for (int u = 0; u < KTW; ++u) {
    const int kt = wave + 4 * u;
    if (kt >= ktn) continue;
#pragma unroll
    for (int nt = 0; nt < NTT; ++nt) {
      if (ntb + nt >= NTtot) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = (kt0 + kt) * 16 + g * 4 + j;
        slab[(size_t)row * ld + (ntb + nt) * 16 + i] = acc[u][nt][j];
      }
    }
  }
  if (do_bias && tid < NTT * 16 && ntb * 16 + tid < ld) a.bslab[(size_t)bx * ld + ntb * 16 + tid] = bacc;
}

template <int KTW, int NTT, bool CS4>
__global__ __launch_bounds__(256) void wgrad_kernel(const WgradArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  wgrad_body<KTW, NTT, CS4>(a, blockIdx.x, blockIdx.y, blockIdx.z, smem);
}

size_t wgrad_lds_bytes(int KT, int NTT) {
  return (size_t)32 * (KT * 16 + 16) * 2 + (size_t)32 * (NTT * 16 + 16) * 2;
}

template <int KTW, int NTT, bool CS4>
static void wl_t(const WgradArgs& a, dim3 grid, size_t lds, hipStream_t s) {
  hipLaunchKernelGGL((wgrad_kernel<KTW, NTT, CS4>), grid, dim3(256), lds, s, a);
}

// ktw in {1,2,4}; ntt in {1,2,4,8}; KT = 4*ktw k-tiles per workgroup
void launch_wgrad(const WgradArgs& a, int ktw, int ntt, int splits, hipStream_t s) {
  const bool cs4 = a.Cs_in == 4;
  const int gy = (a.Ktiles + a.KT - 1) / a.KT;
  const int gz = (a.NT + ntt - 1) / ntt;
  dim3 grid(splits, gy, gz);
  const size_t lds = wgrad_lds_bytes(a.KT, ntt);
#define C2(KW_, NT_)                                          \
  if (ktw == KW_ && ntt == NT_) {                             \
    if (cs4) wl_t<KW_, NT_, true>(a, grid, lds, s);           \
    else wl_t<KW_, NT_, false>(a, grid, lds, s);              \
    return;                                                   \
  }
  C2(1, 1) C2(1, 2) C2(1, 4) C2(1, 8)
  C2(2, 1) C2(2, 2) C2(2, 4) C2(2, 8)
  C2(4, 1) C2(4, 2) C2(4, 4)
#undef C2
}

// Dense backward as ONE launch: the dense wgrad (dW = X^T dH, split over the batch) and the
// dense dX = dH W^T routed through the previous stage's masks are independent GEMMs over
// the same dH, so workgroups [0, n_w) run the wgrad body and the rest the split-K body
// (one kernel boundary instead of two, and the 64 long wgrad workgroups no longer leave
// most CUs idle).
template <int KTW, int NTT>
__global__ __launch_bounds__(256) void dense_bwd_dual_kernel(const WgradArgs wa, const DenseFwdArgs da, const int n_w,
                                                             const int wgx, const int wgy) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int id = blockIdx.x;
  if (id < n_w) {
    const int bx = id % wgx;
    id /= wgx;
    wgrad_body<KTW, NTT, false>(wa, bx, id % wgy, id / wgy, smem);
  } else {
    dense_splitk_body(da, id - n_w);
  }
}

bool dense_big(int NT, int KS);

template <int KTW, int NTT>
static void dd_t(const WgradArgs& wa, const DenseFwdArgs& da, dim3 wg, size_t lds, hipStream_t s) {
  const int n_w = wg.x * wg.y * wg.z;
  const long long waves = (long long)((da.M + 15) / 16) * da.NT * da.splits;
  const int n_d = (int)((waves + 3) / 4);
  hipLaunchKernelGGL((dense_bwd_dual_kernel<KTW, NTT>), dim3(n_w + n_d), dim3(256), lds, s, wa, da, n_w,
                     (int)wg.x, (int)wg.y);
}

// false = unsupported combination (nothing launched): the caller launches both separately
bool launch_dense_bwd_dual(const WgradArgs& wa, int ktw, int ntt, int splits, const DenseFwdArgs& da,
                           hipStream_t s) {
  if (wa.Cs_in == 4 || dense_big(da.NT, da.KS) || da.mode != 1) return false;
  const dim3 wg(splits, (wa.Ktiles + wa.KT - 1) / wa.KT, (wa.NT + ntt - 1) / ntt);
  const size_t lds = wgrad_lds_bytes(wa.KT, ntt);
#define C2(KW_, NT_)                              \
  if (ktw == KW_ && ntt == NT_) {                 \
    dd_t<KW_, NT_>(wa, da, wg, lds, s);           \
    return true;                                  \
  }
  C2(1, 1) C2(1, 2) C2(1, 4) C2(1, 8)
  C2(2, 1) C2(2, 2) C2(2, 4) C2(2, 8)
  C2(4, 1) C2(4, 2) C2(4, 4)
#undef C2
  return false;
}
