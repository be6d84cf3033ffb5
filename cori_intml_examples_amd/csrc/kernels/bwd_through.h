// Device helper shared by conv_mm (mode 1) and head_fused: route a gradient wrt the
// previous stage's OUTPUT element (b, y, x, c) back through that stage's dropout, ReLU
// and 2x2 max-pool, storing dL/d(pre-activation) of the previous conv/dense.
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
  if (t.prev_pool) {
    const int k = t.prev_code[qi * t.pCs + c];
    const bf16 z = f2bf(0.f), v = f2bf(g);
#pragma unroll
    for (int pos = 0; pos < 4; ++pos) {
      const int yy = 2 * y + (pos >> 1), xx = 2 * x + (pos & 1);
      t.dy[(((size_t)b * t.cH + yy) * t.cW + xx) * t.pCs + c] = (pos == k) ? v : z;
    }
  } else {
    t.dy[qi * t.pCs + c] = f2bf(g);
  }
}
