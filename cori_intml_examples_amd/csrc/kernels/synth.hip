// K16: device-side parameter initialisers and synthetic data sets on the counter-based RNG
// (common.h rng_u32).  Both are bit-identical to their CPU twins (ops/rng.py init_uniform,
// io/synth.py synth_cpu): every value is a fixed sequence of single fp32 operations, each
// rounded once (no contraction into FMAs, see the pragma), on integers derived from the
// hash -- so a CPU reference model and the GPU model start from the same weights without a
// host round trip, and the bench / HPO engines build their data sets where they train.
//
// Reference: the Keras glorot_uniform / zeros initialisers of every layer of
// /root/reference/rpv.py:42-58 and mnist.py:40-56; the synthetic sets
// stand in for the RPV HDF5 files and MNIST, which the reference downloads and this image
// does not have.
#include <algorithm>

#include "args.h"

namespace {

constexpr uint32_t S_LAB = 1, S_NJ = 2, S_CY = 3, S_CX = 4, S_AMP = 5, S_CH = 6, S_NOISE = 7, S_TPL = 8,
                   S_MCLS = 9, S_MNOISE = 10, S_SHIFT = 11;
constexpr int RPV_JETS = 6;

__device__ __forceinline__ float u01(uint32_t u) { return (float)(u >> 8) * 5.9604644775390625e-8f; }
// floor(u24 * m / 2^24): an unbiased-enough integer in [0, m) for m < 256
__device__ __forceinline__ int uint_below(uint32_t u, int m) { return (int)(((u >> 8) * (uint32_t)m) >> 24); }

__device__ __forceinline__ float bump(int d, float r2inv) {
#pragma clang fp contract(off)
  const float t = fmaxf(1.f - (float)(d * d) * r2inv, 0.f);
  return t * t;
}

}  // namespace

__global__ __launch_bounds__(256) void init_params_kernel(const InitArgs a) {
#pragma clang fp contract(off)
  for (int i = blockIdx.x * 256 + threadIdx.x; i < a.n; i += gridDim.x * 256) {
    float v = 0.f;
    if (a.kind == 1) v = 1.f;
    else if (a.kind == 2) v = (u01(rng_u32((uint32_t)i, a.seed, a.stream, 0u)) * 2.f - 1.f) * a.scale;
    a.p[i] = v;
  }
}

// One workgroup per sample: x[i][y][x][c] (bf16, channels padded to Cs with zeros) and the
// target row y[i][0..ncls) (one-hot for ncls > 1, the 0/1 label for ncls == 1).
__global__ __launch_bounds__(256) void synth_kernel(const SynthArgs a) {
#pragma clang fp contract(off)
  const int il = blockIdx.x, tid = threadIdx.x;
  const uint32_t i = (uint32_t)(a.first + il);
  __shared__ int jy[RPV_JETS], jx[RPV_JETS], jc[RPV_JETS];
  __shared__ float ja[RPV_JETS];
  __shared__ int s_cls;
  int cls = 0;
  float r2inv = 0.f;
  if (a.kind == 1) {
    const bool sig = (rng_u32(i, a.seed, S_LAB, 0u) >> 8) < (1u << 23);
    cls = sig ? 1 : 0;
    r2inv = sig ? (1.f / 9.f) : (1.f / 36.f);
    if (tid < RPV_JETS) {
      const uint32_t un = rng_u32(i, a.seed, S_NJ, 0u);
      const int nj = sig ? 4 + uint_below(un, 3) : 2 + uint_below(un, 2);
      const uint32_t k = i * 8u + (uint32_t)tid;
      jy[tid] = uint_below(rng_u32(k, a.seed, S_CY, 0u), a.H);
      jx[tid] = uint_below(rng_u32(k, a.seed, S_CX, 0u), a.W);
      jc[tid] = uint_below(rng_u32(k, a.seed, S_CH, 0u), a.C);
      ja[tid] = tid < nj ? 0.5f + 2.f * u01(rng_u32(k, a.seed, S_AMP, 0u)) : 0.f;
    }
  } else if (a.kind == 2) {
    cls = uint_below(rng_u32(i, a.seed, S_MCLS, 0u), a.ncls);
    // per-sample translation of the class template by -3..3 pixels in y and x (wrapping)
    const uint32_t us = rng_u32(i, a.seed, S_SHIFT, 0u);
    jy[0] = uint_below(us, 7) - 3;
    jx[0] = (int)((us & 0xFFu) % 7u) - 3;
  } else {
    cls = a.ncls == 1 ? (u01(rng_u32(i, a.seed, S_LAB, 0u)) < 0.5f ? 1 : 0)
                      : uint_below(rng_u32(i, a.seed, S_LAB, 0u), a.ncls);
  }
  if (tid == 0) s_cls = cls;
  __syncthreads();
  cls = s_cls;
  bf16* xo = a.x + (size_t)il * a.H * a.W * a.Cs;
  for (int p = tid; p < a.H * a.W; p += 256) {
    const int y = p / a.W, x = p - y * a.W;
    for (int c = 0; c < a.Cs; ++c) {
      float v = 0.f;
      if (c < a.C) {
        const uint32_t pix = ((i * (uint32_t)a.H + (uint32_t)y) * (uint32_t)a.W + (uint32_t)x) * (uint32_t)a.C + (uint32_t)c;
        if (a.kind == 1) {
          for (int j = 0; j < RPV_JETS; ++j)
            if (jc[j] == c) v = v + (ja[j] * bump(y - jy[j], r2inv)) * bump(x - jx[j], r2inv);
          v = v + 0.05f * u01(rng_u32(pix, a.seed, S_NOISE, 0u));
        } else if (a.kind == 2) {
          // class template: thresholded hash, smoothed with the pixel above and to the left
          // (wrapping, as np.roll(t, 1) in io/datasets.synthetic_mnist)
          const uint32_t tb = (uint32_t)cls * (uint32_t)(a.H * a.W);
          auto tpl = [&](int yy, int xx) -> float {
            return (rng_u32(tb + (uint32_t)(yy * a.W + xx), a.seed, S_TPL, 0u) >> 8) >= 11744051u ? 1.f : 0.f;
          };
          const int ty = (y - jy[0] + 2 * a.H) % a.H, tx = (x - jx[0] + 2 * a.W) % a.W;
          const float sm = ((tpl(ty, tx) + tpl((ty + a.H - 1) % a.H, tx)) + tpl(ty, (tx + a.W - 1) % a.W)) * (1.f / 3.f);
          v = sm + 0.5f * (2.f * u01(rng_u32(pix, a.seed, S_MNOISE, 0u)) - 1.f);
          v = fminf(fmaxf(v, 0.f), 1.f);
        } else {
          v = u01(rng_u32(pix, a.seed, S_NOISE, 0u));
        }
      }
      xo[(size_t)p * a.Cs + c] = f2bf(v);
    }
  }
  if (a.y && tid < a.ncls) a.y[(size_t)il * a.ncls + tid] = a.ncls == 1 ? (float)cls : (tid == cls ? 1.f : 0.f);
}

void launch_init_params(const InitArgs& a, hipStream_t s) {
  if (a.n <= 0) return;
  const int blocks = std::min((a.n + 255) / 256, 4096);
  hipLaunchKernelGGL(init_params_kernel, dim3(blocks), dim3(256), 0, s, a);
}

void launch_synth(const SynthArgs& a, hipStream_t s) {
  if (a.n <= 0) return;
  hipLaunchKernelGGL(synth_kernel, dim3(a.n), dim3(256), 0, s, a);
}
