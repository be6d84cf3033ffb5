// Body of the split-K dense kernel (see dense.hip), as a device function of the block
// index so wgrad.hip can co-schedule the dense backward dX with the dense wgrad.
#pragma once
#include "bwd_through.h"

__device__ __forceinline__ void dense_splitk_body(const DenseFwdArgs& a, const int bx) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 15, g = lane >> 4;
  const int mtiles = (a.M + 15) / 16;
  const long long ntot = (long long)mtiles * a.NT * a.splits;
  const long long w = (long long)bx * 4 + wave;
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
