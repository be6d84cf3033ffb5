// Step bookkeeping (K14 scalars), shared by the prologue kernel (misc.hip) and, in a
// prologue-free step, an extra last workgroup of the step's first dense launch (dense.hip).
#pragma once
#include "args.h"

// Step bookkeeping (one thread): iteration counter, LR decay and the optimizer's
// bias-correction scalars for this step.  (The data cursor is advanced by the head kernel,
// after every prologue workgroup has read it.)
// write_t false: every scalar of step st->t + 1 but the counter itself, which the caller
// advances once no reader of the old count remains
__device__ __forceinline__ void step_bookkeeping(const StepBeginArgs& a, bool write_t = true) {
  StepState* st = a.st;
  if (!a.training) return;
  const int t1 = st->t + 1;
  if (write_t) st->t = t1;
  const double t = (double)t1;
  double base = (double)st->lr;
  const int g = t1 - st->warm_t0 - 1;
  if (g >= 0 && g < st->warm_steps) {
    const double n = (double)st->warm_size;
    base = (double)st->warm_base / n * ((double)(g + 1) / st->warm_spe * (n - 1.0) / st->warm_epochs + 1.0);
  }
  const double lr = base / (1.0 + (double)a.decay * (t - 1.0));
  st->lr_eff = (float)lr;
  switch (a.opt_kind) {
    case OPT_ADAM: {
      const double b1t = pow((double)a.beta1, t), b2t = pow((double)a.beta2, t);
      st->s[0] = (float)(lr * sqrt(1.0 - b2t) / (1.0 - b1t));
      break;
    }
    case OPT_NADAM: {
      const double b1 = a.beta1;
      const double mc_t = b1 * (1.0 - 0.5 * pow(0.96, t * a.schedule_decay));
      const double mc_t1 = b1 * (1.0 - 0.5 * pow(0.96, (t + 1.0) * a.schedule_decay));
      const double ms_new = st->m_schedule * mc_t;
      const double ms_next = ms_new * mc_t1;
      st->m_schedule = ms_new;
      st->s[0] = (float)mc_t;
      st->s[1] = (float)mc_t1;
      st->s[2] = (float)(1.0 / (1.0 - ms_new));
      st->s[3] = (float)(1.0 / (1.0 - ms_next));
      st->s[4] = (float)(1.0 / (1.0 - pow((double)a.beta2, t)));
      st->s[5] = (float)lr;
      break;
    }
    default:
      st->s[0] = (float)lr;
  }
}

