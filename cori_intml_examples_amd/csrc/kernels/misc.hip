// Step plumbing kernels:
//   step_begin   (1 thread)  iteration counter, data cursor, LR decay and the optimizer's
//                            bias-correction scalars for this step (race-free bookkeeping)
//   gather_batch (K14)       batch rows from the device-resident dataset by the epoch's
//                            device permutation (16-byte copies), targets alongside
//   slab_reduce  (K6/K9 2nd) deterministic fixed-order sum of split partial slabs into the
//                            flat fp32 gradient buffer, remapped to Keras layout
//   optim_update (K13)       ONE multi-tensor launch over the flat buffer: Adam / Nadam /
//                            Adadelta / RMSprop / SGD with Keras 2.2 math, DP averaging
//                            folded in (grad_scale), and the bf16 fragment-major weight
//                            packs the MFMA kernels read scattered out in the same pass
#include "args.h"

__global__ void step_begin_kernel(const StepBeginArgs a) {
  if (threadIdx.x != 0) return;
  StepState* st = a.st;
  if (!a.training) {
    st->cur_pos = st->eval_pos;
    st->eval_pos += a.bs;
    return;
  }
  st->t += 1;
  st->cur_pos = st->pos;
  st->pos += a.bs;
  const double t = (double)st->t;
  const double lr = (double)st->lr / (1.0 + (double)a.decay * (t - 1.0));
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

void launch_step_begin(const StepBeginArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(step_begin_kernel, dim3(1), dim3(64), 0, s, a);
}

// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void gather_kernel(const GatherArgs a) {
  const int row = blockIdx.y;
  if (row >= a.bs) return;
  const StepState* st = a.st;
  const bf16* xs = reinterpret_cast<const bf16*>(st->data_x);
  const float* ys = reinterpret_cast<const float*>(st->data_y);
  const int* perm = reinterpret_cast<const int*>(st->perm);
  const int R = st->data_R, C = st->data_C;
  const int pos = st->cur_pos + row;
  int src = (st->use_perm && perm) ? perm[pos] : pos;
  src = min(max(src, 0), st->data_n - 1);
  const int nvec = R / 8;   // 16-byte vectors per row
  const uint4* s = reinterpret_cast<const uint4*>(xs + (size_t)src * R);
  uint4* d = reinterpret_cast<uint4*>(a.xb + (size_t)row * R);
  for (int v = blockIdx.x * 256 + threadIdx.x; v < nvec; v += gridDim.x * 256) d[v] = s[v];
  if (blockIdx.x == 0 && a.yb && ys)
    for (int c = threadIdx.x; c < C; c += 256) a.yb[(size_t)row * C + c] = ys[(size_t)src * C + c];
}

void launch_gather(const GatherArgs& a, hipStream_t s) {
  const int nvec = a.R / 8;
  const int gx = max(1, min(8, (nvec + 255) / 256));
  hipLaunchKernelGGL(gather_kernel, dim3(gx, a.bs), dim3(256), 0, s, a);
}

// ---------------------------------------------------------------------------------------
// Each descriptor owns a contiguous range of workgroups; a workgroup covers E = 256/tpe
// consecutive elements: thread t -> element t % E (consecutive lanes read consecutive
// addresses of one slab: coalesced) and split-lane t / E (the tpe split-lanes of an
// element sum interleaved subsets of the S slabs with independent unrolled loads).  The tpe
// partials are combined through LDS in a fixed order -> bitwise reproducible.
__global__ __launch_bounds__(256) void slab_reduce_kernel(float* __restrict__ grad, const RedTable tab) {
  __shared__ float red[256];
  int di = 0;
  while (di + 1 < tab.n && (int)blockIdx.x >= tab.d[di + 1].blk0) ++di;
  const RedDesc& d = tab.d[di];
  const int tpe = d.tpe;
  const int E = 256 / tpe;
  const int el = (int)threadIdx.x % E;
  const int lane = (int)threadIdx.x / E;
  const int le = ((int)blockIdx.x - d.blk0) * E + el;
  float acc = 0.f;
  const bool in = le < d.numel;
  if (in) {
    size_t src;
    if (d.type == RED_CONVW) {   // keras (ky,kx,ci,co) -> slab[k = tap*Cs + ci][n = co]
      const int co = le % d.Cout;
      const int t2 = le / d.Cout;
      const int ci = t2 % d.Cin;
      const int tap = t2 / d.Cin;
      src = (size_t)(tap * d.Cs + ci) * d.ld + co;
    } else if (d.type == RED_FLATW) {   // keras (k, n) -> slab[padded k][n]
      const int n = le % d.Cout;
      const int k = le / d.Cout;
      src = (size_t)flat_keras_to_padded(k, d.Cin, d.Cs) * d.ld + n;
    } else {   // RED_BIAS / plain: slab[s][le]
      src = (size_t)le;
    }
    const float* p = d.slab + src;
    const size_t st = (size_t)d.stride_s;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int s = lane;
    for (; s + 3 * tpe < d.S; s += 4 * tpe) {
      a0 += p[(size_t)s * st];
      a1 += p[(size_t)(s + tpe) * st];
      a2 += p[(size_t)(s + 2 * tpe) * st];
      a3 += p[(size_t)(s + 3 * tpe) * st];
    }
    for (; s < d.S; s += tpe) a0 += p[(size_t)s * st];
    acc = (a0 + a1) + (a2 + a3);
  }
  if (tpe == 1) {
    if (in) grad[d.dst_off + le] = acc;
    return;
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  if (lane == 0 && in) {
    float sum = 0.f;
    for (int k = 0; k < tpe; ++k) sum += red[k * E + el];
    grad[d.dst_off + le] = sum;
  }
}

void launch_slab_reduce(float* grad, int lo, int hi, const RedTable& tab, hipStream_t s) {
  if (tab.nblocks <= 0) return;
  hipLaunchKernelGGL(slab_reduce_kernel, dim3(tab.nblocks), dim3(256), 0, s, grad, tab);
}

// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void pack_scatter(const PackTable& tab, bf16* arena, int e, float w) {
  for (int di = 0; di < tab.n; ++di) {
    const PackDesc& d = tab.d[di];
    const int le = e - d.src_off;
    if (le < 0 || le >= d.numel) continue;
    int k, n;
    if (d.type == PACK_CONV_FWD || d.type == PACK_CONV_DGRAD) {
      const int co = le % d.Cout;
      const int t2 = le / d.Cout;
      const int ci = t2 % d.Cin;
      const int tap = t2 / d.Cin;
      if (d.type == PACK_CONV_FWD) {
        k = tap * d.Cs + ci;
        n = co;
      } else {
        const int ky = tap / d.KW, kx = tap - (tap / d.KW) * d.KW;
        const int tapf = (d.KH - 1 - ky) * d.KW + (d.KW - 1 - kx);
        k = tapf * d.Cs + co;
        n = ci;
      }
    } else {
      const int nn = le % d.Cout;
      const int kk = le / d.Cout;
      const int kp = flat_keras_to_padded(kk, d.Cin, d.Cs);
      if (d.type == PACK_DENSE_FWD) {
        k = kp;
        n = nn;
      } else {
        k = nn;
        n = kp;
      }
    }
    const int ks = k >> 5, kr = k & 31;
    const int lane = ((kr >> 3) << 4) | (n & 15);
    const size_t dst = (size_t)d.dst_off + ((size_t)(ks * d.NT + (n >> 4)) * 64 + lane) * 8 + (kr & 7);
    arena[dst] = f2bf(w);
  }
}

__global__ __launch_bounds__(256) void optim_kernel(const OptimArgs a, const PackTable tab) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= a.n) return;
  float p = a.p[e];
  if (!a.pack_only) {
    const float g = a.g[e] * a.grad_scale;
    const StepState* st = a.st;
    switch (a.kind) {
      case OPT_ADAM: {
        const float m = a.beta1 * a.s0[e] + (1.f - a.beta1) * g;
        const float v = a.beta2 * a.s1[e] + (1.f - a.beta2) * g * g;
        a.s0[e] = m;
        a.s1[e] = v;
        p -= st->s[0] * m / (sqrtf(v) + a.eps);
        break;
      }
      case OPT_NADAM: {
        const float mc_t = st->s[0], mc_t1 = st->s[1];
        const float gp = g * st->s[2];
        const float m = a.beta1 * a.s0[e] + (1.f - a.beta1) * g;
        const float v = a.beta2 * a.s1[e] + (1.f - a.beta2) * g * g;
        a.s0[e] = m;
        a.s1[e] = v;
        const float mp = m * st->s[3];
        const float vp = v * st->s[4];
        const float mbar = (1.f - mc_t) * gp + mc_t1 * mp;
        p -= st->s[5] * mbar / (sqrtf(vp) + a.eps);
        break;
      }
      case OPT_ADADELTA: {
        const float acc = a.rho * a.s0[e] + (1.f - a.rho) * g * g;
        const float upd = g * sqrtf(a.s1[e] + a.eps) / sqrtf(acc + a.eps);
        a.s0[e] = acc;
        p -= st->s[0] * upd;
        a.s1[e] = a.rho * a.s1[e] + (1.f - a.rho) * upd * upd;
        break;
      }
      case OPT_RMSPROP: {
        const float acc = a.rho * a.s0[e] + (1.f - a.rho) * g * g;
        a.s0[e] = acc;
        p -= st->s[0] * g / (sqrtf(acc) + a.eps);
        break;
      }
      default: {   // SGD (+momentum / nesterov)
        const float lr = st->s[0];
        if (a.momentum != 0.f) {
          const float v = a.momentum * a.s0[e] - lr * g;
          a.s0[e] = v;
          p += a.nesterov ? (a.momentum * v - lr * g) : v;
        } else {
          p -= lr * g;
        }
      }
    }
    a.p[e] = p;
  }
  pack_scatter(tab, a.arena, e, p);
}

void launch_optim(const OptimArgs& a, const PackTable& tab, hipStream_t s) {
  if (a.n <= 0) return;
  hipLaunchKernelGGL(optim_kernel, dim3((a.n + 255) / 256), dim3(256), 0, s, a, tab);
}
