// Keras-2.2 optimizer update of ONE element (Adam / Nadam / Adadelta / RMSprop / SGD with
// momentum / Nesterov), shared by the multi-tensor optimizer, the fused reduce+optimizer
// and the fused xGMI all-reduce+optimizer kernels.  Per-step scalars (bias-corrected LR,
// Nadam schedule) come from the device StepState written by the step bookkeeping.
#pragma once
#include "args.h"

template <int KIND>
__device__ __forceinline__ void opt_update(const OptimArgs& a, const StepState* st, float& p, float g, float* s0,
                                           float* s1) {
  if (KIND == OPT_ADAM) {
    const float m = a.beta1 * *s0 + (1.f - a.beta1) * g;
    const float v = a.beta2 * *s1 + (1.f - a.beta2) * g * g;
    *s0 = m;
    *s1 = v;
    p -= st->s[0] * m / (sqrtf(v) + a.eps);
  } else if (KIND == OPT_NADAM) {
    const float mc_t = st->s[0], mc_t1 = st->s[1];
    const float gp = g * st->s[2];
    const float m = a.beta1 * *s0 + (1.f - a.beta1) * g;
    const float v = a.beta2 * *s1 + (1.f - a.beta2) * g * g;
    *s0 = m;
    *s1 = v;
    const float mp = m * st->s[3];
    const float vp = v * st->s[4];
    const float mbar = (1.f - mc_t) * gp + mc_t1 * mp;
    p -= st->s[5] * mbar / (sqrtf(vp) + a.eps);
  } else if (KIND == OPT_ADADELTA) {
    const float acc = a.rho * *s0 + (1.f - a.rho) * g * g;
    const float upd = g * sqrtf(*s1 + a.eps) / sqrtf(acc + a.eps);
    *s0 = acc;
    p -= st->s[0] * upd;
    *s1 = a.rho * *s1 + (1.f - a.rho) * upd * upd;
  } else if (KIND == OPT_RMSPROP) {
    const float acc = a.rho * *s0 + (1.f - a.rho) * g * g;
    *s0 = acc;
    p -= st->s[0] * g / (sqrtf(acc) + a.eps);
  } else {   // SGD (+momentum / nesterov)
    const float lr = st->s[0];
    if (a.momentum != 0.f) {
      const float v = a.momentum * *s0 - lr * g;
      *s0 = v;
      p += a.nesterov ? (a.momentum * v - lr * g) : v;
    } else {
      p -= lr * g;
    }
  }
}


// ---------------------------------------------------------------------------------------
// bf16 copies of updated master elements into the fragment packs (routes: PackRoute, args.h).
// Fragment layout: pack[((ks*NT + nt)*64 + lane)*8 + j] = B[k = 32ks + 8(lane>>4) + j][n = 16nt + (lane&15)].
__device__ __forceinline__ long long frag_off(int k, int n, int NT) {
  return (long long)(((k >> 5) * NT + (n >> 4)) * 64 + ((((k >> 3) & 3) << 4) | (n & 15))) * 8 + (k & 7);
}

// element (outer o, inner c) of route R -> fwd (kf, c) and bwd (kb + c, nb) pack coordinates
__device__ __forceinline__ void route_coords(const PackRoute& R, int o, int& kf, int& kb, int& nb) {
  const int tap = o / R.Cin, ci = o - tap * R.Cin;
  kf = tap * R.Cs + ci;
  if (R.kind == 1) { kb = (R.KHW - 1 - tap) * R.Csb; nb = ci; }
  else { kb = 0; nb = kf; }
}

// one element e with its new value p
__device__ __forceinline__ void pack_write(const OptimArgs& a, int e, float p) {
  for (int r = 0; r < a.nroutes; ++r) {            // uniform loop: scalar loads of the route
    const PackRoute R = a.routes[r];
    if (e < R.lo || e >= R.hi) continue;
    const int le = e - R.lo, o = le / R.Cout, c = le - o * R.Cout;
    int kf, kb, nb;
    route_coords(R, o, kf, kb, nb);
    const bf16 v = f2bf(p);
    if (R.fwd >= 0) a.arena[R.fwd + frag_off(kf, c, R.NT)] = v;
    if (R.bwd >= 0) a.arena[R.bwd + frag_off(kb + c, nb, R.NTb)] = v;
  }
}

// four consecutive elements [e, e+4) (e % 4 == 0): one coordinate split when the group is one
// route's row run (Cout % 4 == 0, route start % 4 == 0): four 2-byte forward stores (n .. n+3:
// consecutive lanes of one fragment) and ONE 8-byte backward store (k .. k+3: consecutive j;
// the host sets a backward route only when its k base Csb is a multiple of 4)
__device__ __forceinline__ void pack_write4(const OptimArgs& a, int e, const float4& p) {
  for (int r = 0; r < a.nroutes; ++r) {
    const PackRoute R = a.routes[r];
    if (e + 4 <= R.lo || e >= R.hi) continue;
    if (e < R.lo || e + 4 > R.hi || ((R.Cout | (e - R.lo)) & 3)) {   // straddles / unaligned: per element
      const float v4[4] = {p.x, p.y, p.z, p.w};
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int eu = e + u;
        if (eu < R.lo || eu >= R.hi) continue;
        const int le = eu - R.lo, o = le / R.Cout, c = le - o * R.Cout;
        int kf, kb, nb;
        route_coords(R, o, kf, kb, nb);
        const bf16 v = f2bf(v4[u]);
        if (R.fwd >= 0) a.arena[R.fwd + frag_off(kf, c, R.NT)] = v;
        if (R.bwd >= 0) a.arena[R.bwd + frag_off(kb + c, nb, R.NTb)] = v;
      }
      continue;
    }
    const int le = e - R.lo, o = le / R.Cout, c = le - o * R.Cout;
    int kf, kb, nb;
    route_coords(R, o, kf, kb, nb);
    if (R.fwd >= 0) {
      bf16* d = a.arena + R.fwd + frag_off(kf, c, R.NT);
      d[0] = f2bf(p.x);
      d[8] = f2bf(p.y);
      d[16] = f2bf(p.z);
      d[24] = f2bf(p.w);
    }
    if (R.bwd >= 0) {
      bf16x4 v;
      v[0] = f2bf(p.x); v[1] = f2bf(p.y); v[2] = f2bf(p.z); v[3] = f2bf(p.w);
      *reinterpret_cast<bf16x4*>(a.arena + R.bwd + frag_off(kb + c, nb, R.NTb)) = v;
    }
  }
}
