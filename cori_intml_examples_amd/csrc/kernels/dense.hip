// Dense forward (K8): Y = act(X W + b) with split-K MFMA partials + a fused epilogue.
//
// M (= batch) is small (64-4096) and K is large (1,152-65,536) for the reference models,
// so a plain MxN tiling leaves most of the 256 CUs idle.  The K axis is split across
// waves (grid covers m-tiles x n-tiles x splits, one 16x16 output tile per wave, A and B
// fragments loaded straight to VGPRs as 16-byte accesses) and partials land in an fp32
// slab; dense_epilogue reduces the splits in fixed order (deterministic) and applies
// bias + ReLU + dropout, writing the bf16 activation the next layer consumes.
#include "args.h"

__global__ __launch_bounds__(256) void dense_splitk_kernel(const DenseFwdArgs a) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 15, g = lane >> 4;
  const int mtiles = (a.M + 15) / 16;
  const long long ntot = (long long)mtiles * a.NT * a.splits;
  const long long w = (long long)blockIdx.x * 4 + wave;
  if (w >= ntot) return;
  const int s = (int)(w % a.splits);
  const long long t2 = w / a.splits;
  const int nt = (int)(t2 % a.NT);
  const int mt = (int)(t2 / a.NT);
  const int row = mt * 16 + r;
  const bool rv = row < a.M;
  const bf16* xr = a.x + (size_t)(rv ? row : 0) * a.Ks;
  const int ks_lo = s * a.ks_per_split;
  const int ks_hi = min(a.KS, ks_lo + a.ks_per_split);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int ks = ks_lo; ks < ks_hi; ++ks) {
    const int k0 = ks * 32 + g * 8;
    bf16x8 af = zero_bf16x8();
    if (rv && k0 < a.Ks) af = load_bf16x8(xr + k0);
    const bf16x8 bfr = load_bf16x8(a.wpk + ((size_t)(ks * a.NT + nt) * 64 + lane) * 8);
    acc = mfma16(af, bfr, acc);
  }
  const int ld = a.NT * 16;
  float* out = a.part + (size_t)s * a.M * ld;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = mt * 16 + g * 4 + j;
    if (m < a.M) out[(size_t)m * ld + nt * 16 + r] = acc[j];
  }
}

__global__ __launch_bounds__(256) void dense_epilogue_kernel(const DenseEpiArgs a) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)a.M * a.Ns) return;
  const int m = (int)(idx / a.Ns);
  const int n = (int)(idx - (long long)m * a.Ns);
  float v = 0.f;
  if (n < a.N) {
    const size_t stride = (size_t)a.M * a.ldp;
    const float* p = a.part + (size_t)m * a.ldp + n;
    for (int s = 0; s < a.splits; ++s) v += p[s * stride];
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
  const long long waves = (long long)((a.M + 15) / 16) * a.NT * a.splits;
  hipLaunchKernelGGL(dense_splitk_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s, a);
}

void launch_dense_epi(const DenseEpiArgs& a, hipStream_t s) {
  const long long n = (long long)a.M * a.Ns;
  hipLaunchKernelGGL(dense_epilogue_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a);
}
