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
#include "bwd_through.h"

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
  for (int kb = ks_lo; kb < ks_hi; kb += 8) {
    bf16x8 af[8], bfr[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {   // independent, branch-free loads: 16 in flight per lane
      const int ks = min(kb + u, ks_hi - 1);
      const int k0 = ks * 32 + g * 8;
      af[u] = load_bf16x8_if(rv && k0 < a.Ks && kb + u < ks_hi, xr + k0, a.x);
      bfr[u] = load_bf16x8(a.wpk + ((size_t)(ks * a.NT + nt) * 64 + lane) * 8);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) acc = mfma16(af[u], bfr[u], acc);
  }
  if (a.mode == 1) {
    const BwdThrough& t = a.bt;
    const uint32_t step = a.st ? (uint32_t)a.st->t : 0u;
    const int n = nt * 16 + r;
    const int width = t.pH * t.pW * t.pCs;
    if (n < width) {
      const int y = n / (t.pW * t.pCs);
      const int rem = n - y * t.pW * t.pCs;
      const int x = rem / t.pCs;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = mt * 16 + g * 4 + j;
        if (m < a.M) bwd_through_store(t, m, y, x, rem - x * t.pCs, acc[j], step);
      }
    }
    return;
  }
  const int ld = a.NT * 16;
  float* out = a.part + (size_t)s * a.M * ld;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = mt * 16 + g * 4 + j;
    if (m < a.M) out[(size_t)m * ld + nt * 16 + r] = acc[j];
  }
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
  const long long waves = (long long)((a.M + 15) / 16) * a.NT * a.splits;
  hipLaunchKernelGGL(dense_splitk_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s, a);
}

void launch_dense_epi(const DenseEpiArgs& a, hipStream_t s) {
  const long long n = (long long)a.M * a.Ns;
  hipLaunchKernelGGL(dense_epilogue_kernel, dim3((unsigned)((n + 63) / 64)), dim3(256), 0, s, a);
}
