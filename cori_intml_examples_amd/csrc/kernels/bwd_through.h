// Device helpers for the backward pass.
//
// bwd_through_store: a gradient wrt the previous stage's OUTPUT element (b, y, x, c) is
// multiplied by that stage's (regenerated) dropout mask and ReLU mask (from its saved
// output) and stored AT THE SAME RESOLUTION.  For a max-pooled stage this is dP, the
// gradient at pooled resolution; the full-resolution gradient dY is never materialised:
// consumers rebuild it on load from (dP, argmax code) -- see unpool_load8.
#pragma once
#include "args.h"

__device__ __forceinline__ void bwd_through_store(const BwdThrough& t, int b, int y, int x, int c,
                                                  float g, uint32_t step) {
  if (c >= t.pCs) return;
  const size_t qi = ((size_t)b * t.pH + y) * t.pW + x;
  if (c >= t.pC) {
    g = 0.f;
  } else {
    if (t.drop_thr) {
      const uint32_t idx = (uint32_t)(qi * (size_t)t.pC + c);
      g = dropout_keep(idx, t.seed, t.stream_id, step, t.drop_thr) ? g * t.drop_scale : 0.f;
    }
    if (t.prev_relu) {
      const float a = bf2f(t.prev_out[qi * t.pCs + c]);
      if (!(a > 0.f)) g = 0.f;
    }
  }
  t.dy[qi * t.pCs + c] = f2bf(g);
}

// Vectorised form: 8 consecutive channels [c0, c0+8) of output pixel qi (flat index over
// the previous stage's output grid); one 16-byte load of the saved output, one 16-byte store.
__device__ __forceinline__ void bwd_through_store8(const BwdThrough& t, size_t qi, int c0, const float* g,
                                                   uint32_t step) {
  if (c0 >= t.pCs) return;
  const size_t o = qi * t.pCs + c0;
  bf16x8 prev = zero_bf16x8();
  if (t.prev_relu) prev = load_bf16x8(t.prev_out + o);
  bf16x8 outv;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int c = c0 + k;
    float v = g[k];
    if (c >= t.pC) {
      v = 0.f;
    } else {
      if (t.drop_thr)
        v = dropout_keep((uint32_t)(qi * (size_t)t.pC + c), t.seed, t.stream_id, step, t.drop_thr) ? v * t.drop_scale
                                                                                                  : 0.f;
      if (t.prev_relu && !(bf2f(prev[k]) > 0.f)) v = 0.f;
    }
    outv[k] = f2bf(v);
  }
  if (t.wt) st_wt16(t.dy, (unsigned)(o * 2), __builtin_bit_cast(u32x4, outv));
  else *reinterpret_cast<bf16x8*>(t.dy + o) = outv;
}

// Full-resolution gradient of a max-pooled conv at pixel (y, x), channels [c, c+8), rebuilt
// from the pooled gradient dP [Hp][Wp][Cs] and the forward argmax codes (same layout).
// Pixels outside the 2*Hp x 2*Wp pooled area get no gradient (Keras 'valid' pooling).
// Branch-free: `ok` false (or a pixel outside the pooled area) yields zeros; the loads are
// always issued (from a clamped in-range address) so batches of them stay in flight.
__device__ __forceinline__ bf16x8 unpool_load8(const bf16* dP, const uint8_t* code, int Hp, int Wp, int Cs,
                                               int y, int x, int c, bool ok = true) {
  const int wy = y >> 1, wx = x >> 1;
  ok = ok && wy < Hp && wx < Wp && y >= 0 && x >= 0;
  const size_t o = ok ? ((size_t)wy * Wp + wx) * Cs + c : 0;
  const uint4 raw = *reinterpret_cast<const uint4*>(dP + o);
  const uint2 cw = *reinterpret_cast<const uint2*>(code + o);
  const uint32_t pos = ok ? (uint32_t)(((y & 1) << 1) | (x & 1)) : 0xFFu;
  // per 16-bit lane mask: keep element j iff code byte j == pos
  uint32_t m[4];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t w = h ? cw.y : cw.x;
    const uint32_t k0 = ((w & 0xFF) == pos) ? 0x0000FFFFu : 0u;
    const uint32_t k1 = (((w >> 8) & 0xFF) == pos) ? 0xFFFF0000u : 0u;
    const uint32_t k2 = (((w >> 16) & 0xFF) == pos) ? 0x0000FFFFu : 0u;
    const uint32_t k3 = (((w >> 24) & 0xFF) == pos) ? 0xFFFF0000u : 0u;
    m[2 * h] = k0 | k1;
    m[2 * h + 1] = k2 | k3;
  }
  const uint4 v = {raw.x & m[0], raw.y & m[1], raw.z & m[2], raw.w & m[3]};
  return *reinterpret_cast<const bf16x8*>(&v);
}
