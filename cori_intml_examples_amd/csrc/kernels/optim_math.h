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

