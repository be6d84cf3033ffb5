// The step's last hidden dense layer AND the binary output head in ONE launch (K8 + K12 of
// the RPV training step: Dense(128) + ReLU + Dropout -> Dense(1) + sigmoid + BCE).
//
// Before: a split-K dense launch (partials -> HBM), then a head launch whose 128 one-row
// workgroups reduced the partials (bias, ReLU, dropout) and ran the head -- two launches,
// each a ~3 us boundary plus its own ramp and drain around ~3-5 us of latency-bound work.
//
// Here a workgroup of 16 waves owns one 16-row x 16-column output tile over 1/KH of K: each
// wave reduces a K slice with 16x16x32 MFMAs (A and B fragments loaded straight to VGPRs,
// one batch of 16-byte loads per lane), the 16 wave partials are summed in LDS in fixed wave
// order, and the tile's fp32 partial goes to HBM.  The workgroup then draws an arrival ticket
// for its 16-row group; the LAST of the group's NT*KH workgroups (monotonic counter: no reset
// launch) reads the group's partials back and finishes the dense layer for those 16 rows
// (bias, ReLU, dropout -> the bf16 activation the backward reads) and runs the head with one
// wave per row: logit, sigmoid, Keras BCE + accuracy into the device metrics, and the
// backward's head part (dz, the per-row dW / db slabs, dh through the dense layer's dropout
// and ReLU masks) -- the same formulas, rounding points and per-row slab layout as the head
// kernel's binary fast path (head.hip).  Deterministic: fixed summation orders everywhere.
//
// Hand-off without fences (MI355X_MICROARCH.md, valid forms: stores all sc1 + drained, ONE
// unsharded counter whose last adder is told by its add's return value, loads all sc1): the
// tile partials go out as 16-byte write-through stores, every storing wave drains them
// before the workgroup barrier in front of the ticket, and the last arriver reads them with
// sc1 loads.  (Release / acquire fences around every ticket measured 18.6 us for the launch
// against 13.3 us for the two launches it replaces.)
//
// Step bookkeeping: an extra workgroup computes this step's LR / optimizer scalars at once
// (they are read by later launches only) and the iteration counter and data cursor advance
// only after every reader of the old count in this launch is done -- the last of the row
// groups' heads and that workgroup to add to a second counter advances them.
#include "bwd_through.h"
#include "step_book.h"

#define DH_WAVES 16
#define DH_THREADS (DH_WAVES * 64)
#define DH_MAX_NS 256

namespace {

__device__ __forceinline__ float dh_clip_nan(float q, float lo, float hi) {
  return q != q ? q : fminf(fmaxf(q, lo), hi);
}

__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// 4-byte sc1 load (a relaxed agent-scope atomic load: global_load_dword ... sc1)
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// advance the iteration counter and the data cursor (the last adder to ticket[mgroups])
__device__ __forceinline__ void dh_finish_step(const DenseHeadArgs& A, int mgroups) {
  const DenseFwdArgs& a = A.f;
  StepState* st = A.h.st;
  const unsigned old = __hip_atomic_fetch_add(A.ticket + mgroups, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned n = (unsigned)mgroups + (a.book ? 1u : 0u);
  if (((old + 1u) % n) != 0u || !st) return;
  if (a.book && a.sb.training) st->t += 1;
  if (A.h.training) st->pos += a.M;
  else st->eval_pos += a.M;
  st->packs_stale = 0;
}

}  // namespace

__global__ __launch_bounds__(DH_THREADS) void dense_head_kernel(const DenseHeadArgs A) {
  const DenseFwdArgs& a = A.f;
  const HeadArgs& h = A.h;
  const DenseEpiArgs& e = h.epi;
  __shared__ float red[DH_WAVES][256];
  __shared__ bf16 hs[16][DH_MAX_NS];
  __shared__ float dz_s[16];
  __shared__ int s_last;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 15, g = lane >> 4;
  const int mgroups = (a.M + 15) >> 4;
  const int per_group = a.NT * A.kh;
  const int bx = blockIdx.x;
  if (a.book && bx == (int)gridDim.x - 1) {   // the extra bookkeeping workgroup
    if (tid == 0) {
      step_bookkeeping(a.sb, false);        // every scalar of step t + 1 but t itself
      dh_finish_step(A, mgroups);
    }
    return;
  }
  const int mg = bx / per_group, rem = bx - mg * per_group;
  const int nt = rem % a.NT, kh = rem / a.NT;

  // ---- 1. the tile's K slice: wave `wave` of split kh * 16 + wave
  const int S = DH_WAVES * A.kh, sp = kh * DH_WAVES + wave;
  const int kps = (a.KS + S - 1) / S;
  const int ks_lo = sp * kps, ks_hi = min(a.KS, ks_lo + kps);
  const int row = mg * 16 + r;
  const bool rv = row < a.M;
  const bf16* xr = a.x + (size_t)(rv ? row : 0) * a.Ks;
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
    for (int u = 0; u < 8; ++u)
      if (kb + u < ks_hi) acc = mfma16(af[u], bfr[u], acc);
  }
  *reinterpret_cast<f32x4*>(&red[wave][lane * 4]) = acc;
  __syncthreads();

  // ---- 2. fixed-order sum of the 16 wave partials -> the tile's fp32 partial (thread t:
  //         lane t >> 2's accumulator element t & 3 = row 4 g + j, column r), staged as the
  //         16 x 16 tile so wave 0 writes it as 16-byte write-through stores
  const int ldp = a.NT * 16;
  __shared__ float tile[256];
  if (tid < 256) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < DH_WAVES; ++w) v += red[w][tid];
    const int l2 = tid >> 2, j = tid & 3;
    tile[(4 * (l2 >> 4) + j) * 16 + (l2 & 15)] = v;
  }
  __syncthreads();
  if (tid < 64) {
    const int rl = tid >> 2, c4 = (tid & 3) * 4;
    const int m = mg * 16 + rl;
    if (m < a.M) {
      const u32x4 v = *reinterpret_cast<const u32x4*>(&tile[rl * 16 + c4]);
      st_wt16(a.part, (unsigned)((((size_t)kh * a.M + m) * ldp + nt * 16 + c4) * 4), v);
    }
    drain();                          // the storing wave: its stores complete
  }
  __syncthreads();
  if (tid == 0) {
    const unsigned old = __hip_atomic_fetch_add(A.ticket + mg, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = ((old + 1u) % (unsigned)per_group) == 0u;
  }
  __syncthreads();
  if (!s_last) return;

  // ---- 3. last arriver of row group mg: the dense layer's output rows (bias, ReLU, dropout)
  const StepState* st = h.st;
  // the step's dropout counter: the iteration count advances only after every reader of this
  // launch is done (step 5), so it reads the old count (+1 when the bookkeeping is this launch's)
  const uint32_t step = st ? (uint32_t)st->t + (uint32_t)(a.book ? 1 : 0) : 0u;
  const int m0 = mg * 16;
  for (int i = tid; i < 16 * e.Ns; i += DH_THREADS) {
    const int rl = i / e.Ns, n = i - rl * e.Ns;
    const int m = m0 + rl;
    if (m >= a.M) continue;
    float v = 0.f;
    if (n < e.N) {
      v = 0.f;
      for (int q = 0; q < A.kh; ++q) v += ld_sc1(a.part + ((size_t)q * a.M + m) * ldp + n);
      if (e.bias) v += e.bias[n];
      if (e.relu) v = fmaxf(v, 0.f);
      if (e.drop_thr)
        v = dropout_keep((uint32_t)(m * e.N + n), e.seed, e.stream_id, step, e.drop_thr) ? v * e.drop_scale : 0.f;
    }
    const bf16 hb = f2bf(v);
    hs[rl][n] = hb;
    e.out[(size_t)m * e.Ns + n] = hb;     // saved activation (the backward's ReLU mask)
  }
  __syncthreads();

  // ---- 4. the head, one wave per row: logit (head.hip's lane-strided order + xor tree)
  const int m = m0 + wave;
  const bool live = m < a.M;
  float z = 0.f;
  if (live)
    for (int k = lane; k < h.K; k += 64) z += bf2f(hs[wave][k]) * h.w[k];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) z += __shfl_xor(z, off);
  const float eps = 1e-7f;
  if (live && lane == 0) {
    const float z0 = z + (h.bias ? h.bias[0] : 0.f);
    const float p = 1.f / (1.f + expf(-z0));
    if (h.probs) h.probs[m] = p;
    float dz = 0.f;
    if (h.y) {
      const float* yr = h.yidx ? reinterpret_cast<const float*>(st->data_y) + (size_t)h.yidx[m] * st->data_C
                               : h.y + (size_t)m;
      const float yv = yr[0];
      const float pc = dh_clip_nan(p, eps, 1.f - eps);
      dz = ((p >= eps) && (p <= 1.f - eps)) ? (pc - yv) : 0.f;
      if (h.st) {
        const float lg = logf(pc / (1.f - pc));
        const float ls = fmaxf(lg, 0.f) - lg * yv + log1pf(expf(-fabsf(lg)));
        const float cs = (rintf(p) == yv) ? 1.f : 0.f;
        long long* slot = h.st->metric_slots[m & 15];
        const bool loss_ok = isfinite(ls) && fabsf(ls) < 1073741824.f;
        if (loss_ok) atomicAdd((unsigned long long*)&slot[0], (unsigned long long)llrint((double)ls * 4294967296.0));
        else atomicAdd((unsigned long long*)&slot[3], 1ull);
        atomicAdd((unsigned long long*)&slot[1], (unsigned long long)llrintf(cs));
        atomicAdd((unsigned long long*)&slot[2], 1ull);
      }
    }
    dz_s[wave] = dz * h.inv_bs;
  }
  __syncthreads();
  if (live && h.training) {
    const float dz = dz_s[wave];
    float* ws = h.wslab + (size_t)m * h.K;
    for (int k = lane; k < h.K; k += 64) ws[k] = 0.f + bf2f(hs[wave][k]) * dz;   // (0 + x: as head.hip)
    if (lane == 0 && h.bslab) h.bslab[m] = dz;
    const BwdThrough& t = h.bt;
    for (int c = lane; c < t.pCs; c += 64) {
      float gs = 0.f;
      if (c < t.pC) {
        gs = 0.f + dz * h.w[c];
        if (t.drop_thr) {
          const uint32_t di = (uint32_t)((size_t)m * t.pC + c);
          gs = dropout_keep(di, t.seed, t.stream_id, step, t.drop_thr) ? gs * t.drop_scale : 0.f;
        }
        if (t.prev_relu && !(bf2f(hs[wave][c]) > 0.f)) gs = 0.f;
      }
      t.dy[(size_t)m * t.pCs + c] = f2bf(gs);
    }
  }

  // ---- 5. the last of the row groups (and the bookkeeping workgroup) to finish advances the
  //         iteration counter and the data cursor: every read of the old count is done
  __syncthreads();
  if (tid == 0) dh_finish_step(A, mgroups);
}

int dense_head_blocks(const DenseHeadArgs& a) { return ((a.f.M + 15) / 16) * a.f.NT * a.kh + (a.f.book ? 1 : 0); }

void launch_dense_head(const DenseHeadArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(dense_head_kernel, dim3(dense_head_blocks(a)), dim3(DH_THREADS), 0, s, a);
}
