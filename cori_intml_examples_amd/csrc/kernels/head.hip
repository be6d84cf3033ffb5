// Fused output head (K11 / K12 + the last dense's K8/K9):
//   logits = h W + b  ->  softmax | sigmoid | linear  ->  Keras loss (clipping semantics of
//   categorical_crossentropy / binary_crossentropy) + accuracy,
//   accumulated into device metrics (one int64 fixed-point atomic triple per workgroup,
//   order-independent, no per-batch D2H);
// and in training mode, in the same launch:
//   dz = dL/dlogits / batch, dW / db partial slabs (one per 4-row workgroup, reduced in
//   fixed order by slab_reduce) and dh = dz W^T routed back through the previous stage's
//   dropout / ReLU masks (bwd_through_store: dense dH, or the flattened conv's pooled dP).
// N (classes) <= 16, so the head is a handful of dot products per row: one wave per row,
// K split across the 64 lanes, cross-lane shuffle reductions.
#include "bwd_through.h"

// Keras' probability clip (tf.clip_by_value) propagates a NaN; fminf/fmaxf would replace it
// by a bound and turn a diverged model's loss into a finite value
__device__ __forceinline__ float clip_nan(float q, float lo, float hi) {
  return q != q ? q : fminf(fmaxf(q, lo), hi);
}

#define HEAD_RB 4
#define HEAD_EPI_MAX 1024   // widest previous dense whose epilogue the head absorbs
#define HEAD_W_LDS 2048     // head weights staged in LDS up to this many floats

// dense_epilogue_kernel's value for (m, n): the same 4-way interleaved split order
// (bit-identical), then bias, ReLU, dropout.
__device__ __forceinline__ float dense_epi_value(const DenseEpiArgs& e, int m, int n, uint32_t step) {
  const size_t stride = (size_t)e.M * e.ldp;
  const float* p = e.part + (size_t)m * e.ldp + n;
  float r4[4];
#pragma unroll
  for (int sg = 0; sg < 4; ++sg) {
    float a0 = 0.f, a1 = 0.f;
    int s = sg;
    for (; s + 4 < e.splits; s += 8) {
      a0 += p[(size_t)s * stride];
      a1 += p[(size_t)(s + 4) * stride];
    }
    for (; s < e.splits; s += 4) a0 += p[(size_t)s * stride];
    r4[sg] = a0 + a1;
  }
  float v = (r4[0] + r4[1]) + (r4[2] + r4[3]);
  if (e.bias) v += e.bias[n];
  if (e.relu) v = fmaxf(v, 0.f);
  if (e.drop_thr)
    v = dropout_keep((uint32_t)(m * e.N + n), e.seed, e.stream_id, step, e.drop_thr) ? v * e.drop_scale : 0.f;
  return v;
}

// One split group's partial sum of dense_epi_value (sg in 0..3), its <= 16 loads issued
// together; same summation order as dense_epi_value (bit-identical).
__device__ __forceinline__ float dense_epi_group(const DenseEpiArgs& e, int m, int n, int sg) {
  const size_t stride = (size_t)e.M * e.ldp;
  const float* p = e.part + (size_t)m * e.ldp + n;
  float v[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int sp = sg + 4 * j;
    v[j] = p[(size_t)min(sp, e.splits - 1) * stride];
  }
  // dense_epi_value's loops over the preloaded values: pairs (s, s + 4) while s + 4 < splits,
  // then the remaining s into a0
  float a0 = 0.f, a1 = 0.f;
  int jn = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i)
    if (sg + 8 * i + 4 < e.splits) {
      a0 += v[2 * i];
      a1 += v[2 * i + 1];
      jn = 2 * i + 2;
    }
#pragma unroll
  for (int jj = 0; jj < 16; ++jj)
    if (jj >= jn && sg + 4 * jj < e.splits) a0 += v[jj];
  return a0 + a1;
}

// 16-lane group reductions (lanes 0..15 of a wave; xor offsets < 16 stay inside the group)
__device__ __forceinline__ float grp16_sum(float v) {
#pragma unroll
  for (int off = 8; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}
// max value and its lowest index (the serial loop's strict '>' keeps the first maximum)
__device__ __forceinline__ void grp16_argmax(float& v, int& i) {
#pragma unroll
  for (int off = 8; off > 0; off >>= 1) {
    const float ov = __shfl_xor(v, off);
    const int oi = __shfl_xor(i, off);
    if (ov > v || (ov == v && oi < i)) { v = ov; i = oi; }
  }
}

// Softmax + Keras categorical_crossentropy (clip of the renormalised probabilities) and its
// gradient, lane n = class n.  Same formulas as the serial head path; sums are 16-lane trees.
template <int NM>
__device__ __forceinline__ void softmax_cce_lanes(const HeadArgs& a, const float (&z)[NM], int lane, int row,
                                                  int rw, int N, const float* ysh_row, const float* bsh,
                                                  float* dz_row, float* met_row) {
  const bool live = row < a.M;
  const int n = lane & 15;
  const bool cls = live && lane < 16 && n < N;
  float zn = 0.f;
#pragma unroll
  for (int j = 0; j < NM; ++j)
    if (j == n) zn = z[j];
  zn += bsh[n];
  float mx = cls ? zn : -__builtin_inff();
  int am = cls ? n : 1 << 20;
  grp16_argmax(mx, am);
  const float e = cls ? expf(zn - mx) : 0.f;
  const float s = grp16_sum(e);
  const float p = e / s;
  if (cls && a.probs) a.probs[(size_t)row * N + n] = p;
  float loss = 0.f, dzn = 0.f, correct = 0.f;
  if (a.y) {
    const float eps = 1e-7f;
    const float ps = grp16_sum(cls ? p : 0.f);
    const float yn = cls ? ysh_row[n] : 0.f;
    const float q = p / ps;
    const bool inr = (q >= eps) && (q <= 1.f - eps);
    const float qc = clip_nan(q, eps, 1.f - eps);
    const float ln = cls ? -yn * logf(qc) : 0.f;
    float gn = (cls && inr) ? -yn / qc : 0.f;
    const float gq = grp16_sum(gn * (cls ? q : 0.f));
    gn = (gn - gq) / ps;
    const float pg = grp16_sum(cls ? p * gn : 0.f);
    dzn = cls ? p * (gn - pg) : 0.f;
    loss = grp16_sum(ln);
    float ymx = cls ? yn : -__builtin_inff();
    int ay = cls ? n : 1 << 20;
    grp16_argmax(ymx, ay);
    correct = (live && am == ay) ? 1.f : 0.f;
  }
  if (lane < NM) dz_row[lane] = dzn * a.inv_bs;
  if (lane == 0) {
    met_row[0] = live ? loss : 0.f;
    met_row[1] = correct;
  }
}

#define HEAD_STAMP(i)                                                                 \
  if (a.ts && threadIdx.x == 0) a.ts[(size_t)blockIdx.x * 8 + (i)] = wall_clock64();

template <int RB, int NM>
__global__ __launch_bounds__(256) void head_kernel(const HeadArgs a) {
  __shared__ float dz_s[RB][NM];
  __shared__ float met[RB][2];
  __shared__ bf16 hs[RB][HEAD_EPI_MAX];
  __shared__ float red4[RB == 1 ? 4 : 1][RB == 1 ? HEAD_EPI_MAX : 1];
  __shared__ float wsh[HEAD_W_LDS];      // head weights [K][N] when they fit (read twice below)
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  // head weights -> LDS first: their load overlaps the epilogue's partial-sum loads, and the
  // logit dot and the dH back-projection then read LDS instead of two global round trips
  HEAD_STAMP(0);
  const bool wlds = a.K * a.N <= HEAD_W_LDS;
  if (wlds)
    for (int i = tid; i < a.K * a.N; i += 256) wsh[i] = a.w[i];
  const int row0 = blockIdx.x * RB;
  const int N = a.N;
  const uint32_t step = a.st ? (uint32_t)a.st->t : 0u;
  const int rw = RB == 1 ? 0 : wave;                 // this wave's row slot
  const bool row_wave = RB != 1 || wave == 0;        // RB == 1: wave 0 computes the row
  const int row = row0 + rw;
  const bool fused = a.epi.part != nullptr;
  // the rows' targets and the bias too (read by the serial loss code below)
  __shared__ float ysh[RB][16], bsh[16];
  if (tid < 16) bsh[tid] = (a.bias && tid < a.N) ? a.bias[tid] : 0.f;
  if (tid >= 64 && tid < 64 + RB * 16) {
    const int rl = (tid - 64) >> 4, n = (tid - 64) & 15;
    const int m = row0 + rl;
    const bool ok = a.y && n < a.N && m < a.M;
    // (prologue-free step: the targets' dataset row, recorded by the conv stack)
    const float* yr = a.yidx ? reinterpret_cast<const float*>(a.st->data_y) + (size_t)a.yidx[ok ? m : 0] * a.st->data_C
                             : a.y + (size_t)m * a.N;
    ysh[rl][n] = ok ? yr[n] : 0.f;
  }
  bool done_epi = false;
  if constexpr (RB == 1) {
   if (fused && !a.generic && a.epi.splits <= 32 && a.epi.Ns <= 128) {
    done_epi = true;
    // one row per workgroup, <= 32 splits, <= 128 columns: thread -> column n = tid % 128,
    // split groups sg = tid / 128 and sg + 2; the <= 8 partials of BOTH groups are loaded in
    // one batch (one memory round trip, no clamped duplicates), then summed in
    // dense_epi_value's order (bit-identical)
    const DenseEpiArgs& e = a.epi;
    const int n = tid & 127, sg0 = tid >> 7;
    const bool col = n < e.N;
    const size_t stride = (size_t)e.M * e.ldp;
    const float* p = e.part + (size_t)row0 * e.ldp + (col ? n : 0);
    float v[2][8];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int sp = sg0 + 2 * h + 4 * j;
        v[h][j] = (col && sp < e.splits) ? p[(size_t)sp * stride] : 0.f;
      }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int sg = sg0 + 2 * h;
      float a0 = 0.f, a1 = 0.f;
      int jn = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (sg + 8 * i + 4 < e.splits) {
          a0 += v[h][2 * i];
          a1 += v[h][2 * i + 1];
          jn = 2 * i + 2;
        }
#pragma unroll
      for (int jj = 0; jj < 8; ++jj)
        if (jj >= jn && sg + 4 * jj < e.splits) a0 += v[h][jj];
      if (n < e.Ns) red4[sg][n] = a0 + a1;
    }
    __syncthreads();
    for (int c = tid; c < e.Ns; c += 256) {
      float val = 0.f;
      if (c < e.N) {
        val = (red4[0][c] + red4[1][c]) + (red4[2][c] + red4[3][c]);
        if (e.bias) val += e.bias[c];
        if (e.relu) val = fmaxf(val, 0.f);
        if (e.drop_thr)
          val = dropout_keep((uint32_t)(row0 * e.N + c), e.seed, e.stream_id, step, e.drop_thr) ? val * e.drop_scale
                                                                                                 : 0.f;
      }
      const bf16 hb = f2bf(val);
      hs[0][c] = hb;
      e.out[(size_t)row0 * e.Ns + c] = hb;     // saved activation (ReLU mask of the backward)
    }
    __syncthreads();
   }
   if (fused && !done_epi && a.epi.splits <= 64) {
    done_epi = true;
    // one row per workgroup: the four split groups of every column in parallel (all their
    // loads in flight), combined in dense_epi_value's fixed order
    const DenseEpiArgs& e = a.epi;
    for (int task = tid; task < 4 * e.Ns; task += 256) {
      const int n = task % e.Ns, sg = task / e.Ns;
      red4[sg][n] = n < e.N ? dense_epi_group(e, row0, n, sg) : 0.f;
    }
    __syncthreads();
    for (int n = tid; n < e.Ns; n += 256) {
      float v = 0.f;
      if (n < e.N) {
        v = (red4[0][n] + red4[1][n]) + (red4[2][n] + red4[3][n]);
        if (e.bias) v += e.bias[n];
        if (e.relu) v = fmaxf(v, 0.f);
        if (e.drop_thr)
          v = dropout_keep((uint32_t)(row0 * e.N + n), e.seed, e.stream_id, step, e.drop_thr) ? v * e.drop_scale : 0.f;
      }
      const bf16 hb = f2bf(v);
      hs[0][n] = hb;
      e.out[(size_t)row0 * e.Ns + n] = hb;     // saved activation (ReLU mask of the backward)
    }
    __syncthreads();
   }
  }
  if (fused && !done_epi) {   // previous dense layer's epilogue for this workgroup's rows
    const DenseEpiArgs& e = a.epi;
    const int nr = min(RB, a.M - row0);
    for (int idx = tid; idx < nr * e.Ns; idx += 256) {
      const int rl = idx / e.Ns, n = idx - rl * e.Ns;
      const int m = row0 + rl;
      const bf16 hb = f2bf(n < e.N ? dense_epi_value(e, m, n, step) : 0.f);
      hs[rl][n] = hb;
      e.out[(size_t)m * e.Ns + n] = hb;     // saved activation (ReLU mask of the backward)
    }
    __threadfence_block();
    __syncthreads();
  }
  if (a.st && blockIdx.x == 0 && tid == 0) {
    // advance the data cursor the step prologue gathered from (it must not move while
    // prologue workgroups read it) and mark the weight packs fresh (this step's prologue
    // re-packed them if an optimizer ran; the next optimizer marks them stale again)
    if (a.training) a.st->pos += a.M;
    else a.st->eval_pos += a.M;
    a.st->packs_stale = 0;
  }

  HEAD_STAMP(1);
  if (!fused) __syncthreads();   // (the fused path's barriers already cover wsh / ysh / bsh)
  float z[NM];
#pragma unroll
  for (int n = 0; n < NM; ++n) z[n] = 0.f;
  if (row < a.M && row_wave) {
    const bf16* hr = a.h + (size_t)row * a.Ks;
    for (int k = lane; k < a.K; k += 64) {
      const int kp = a.flat_C ? flat_keras_to_padded(k, a.flat_C, a.flat_Cs) : k;
      const float hv = fused ? bf2f(hs[rw][kp]) : bf2f(hr[kp]);
#pragma unroll
      for (int n = 0; n < NM; ++n)
        if (n < N) z[n] += hv * (wlds ? wsh[k * N + n] : a.w[(size_t)k * N + n]);
    }
  }
  // the NM chains unconditionally (z[n >= N] is 0) and interleaved: 6 dependent cross-lane
  // rounds instead of N guarded chains of 6 (each chain's order is unchanged)
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
#pragma unroll
    for (int n = 0; n < NM; ++n) z[n] += __shfl_xor(z[n], off);
  }
  HEAD_STAMP(7);
  if constexpr (RB == 1 && NM == 1) {
    // Binary head of a fused hidden dense layer (the RPV step): only dz gates the backward,
    // so lane 0 publishes it first; then wave 0 computes the loss / accuracy and the metric
    // atomics (a serial log / exp chain) WHILE waves 1-3 write the dW / db slabs and dh --
    // the loss is off the critical path.  Same formulas and rounding points as below.
    const BwdThrough& t = a.bt;
    if (a.act == 1 && fused && !a.generic && a.training && t.dy && t.prev_out == a.epi.out && t.pH == 1 &&
        t.pW == 1 && N == 1) {
      const float eps = 1e-7f;
      const float z0 = z[0] + bsh[0];
      if (tid == 0) {
        const float p = 1.f / (1.f + expf(-z0));
        if (a.probs) a.probs[row] = p;
        float dz = 0.f;
        if (a.y) {
          const float pc = clip_nan(p, eps, 1.f - eps);
          dz = ((p >= eps) && (p <= 1.f - eps)) ? (pc - ysh[0][0]) : 0.f;
        }
        dz_s[0][0] = dz * a.inv_bs;
      }
      HEAD_STAMP(2);
      __syncthreads();
      HEAD_STAMP(3);
      if (wave == 0) {
        if (tid == 0 && a.y && a.st) {
          const float p = 1.f / (1.f + expf(-z0));
          const float yv = ysh[0][0];
          const float pc = clip_nan(p, eps, 1.f - eps);
          const float lg = logf(pc / (1.f - pc));
          const float ls = fmaxf(lg, 0.f) - lg * yv + log1pf(expf(-fabsf(lg)));
          const float cs = (rintf(p) == yv) ? 1.f : 0.f;
          long long* slot = a.st->metric_slots[blockIdx.x & 15];
          const bool loss_ok = isfinite(ls) && fabsf(ls) < 1073741824.f;
          if (loss_ok) atomicAdd((unsigned long long*)&slot[0], (unsigned long long)llrint((double)ls * 4294967296.0));
          else atomicAdd((unsigned long long*)&slot[3], 1ull);
          atomicAdd((unsigned long long*)&slot[1], (unsigned long long)llrintf(cs));
          atomicAdd((unsigned long long*)&slot[2], 1ull);
        }
        HEAD_STAMP(4);
        return;
      }
      const int t2 = tid - 64;                       // waves 1-3
      const float dz = dz_s[0][0];
      float* ws = a.wslab + (size_t)blockIdx.x * a.K;
      for (int k = t2; k < a.K; k += 192) {
        const int kp = a.flat_C ? flat_keras_to_padded(k, a.flat_C, a.flat_Cs) : k;
        ws[k] = 0.f + bf2f(hs[0][kp]) * dz;      // (0 + x: the serial path's +0 for -0 products)
      }
      if (t2 == 0 && a.bslab) a.bslab[blockIdx.x] = dz;
      if (tid == 64 && a.ts) a.ts[(size_t)blockIdx.x * 8 + 5] = wall_clock64();
      for (int c = t2; c < t.pCs; c += 192) {
        float gs = 0.f;
        if (c < t.pC) {
          gs = 0.f + dz * (wlds ? wsh[c] : a.w[c]);
          if (t.drop_thr) {
            const uint32_t di = (uint32_t)((size_t)row0 * t.pC + c);
            gs = dropout_keep(di, t.seed, t.stream_id, step, t.drop_thr) ? gs * t.drop_scale : 0.f;
          }
          if (t.prev_relu && !(bf2f(hs[0][c]) > 0.f)) gs = 0.f;
        }
        t.dy[(size_t)row0 * t.pCs + c] = f2bf(gs);
      }
      if (tid == 64 && a.ts) a.ts[(size_t)blockIdx.x * 8 + 6] = wall_clock64();
      return;
    }
  }
  if constexpr (NM > 1) {
    if (a.act == 2 && row_wave) {
      // softmax + categorical cross-entropy, one class per lane (lanes 0..15 of the row's
      // wave; every lane holds all logits after the reduction above).  The serial lane-0
      // version spent ~5 us per row in dependent exp / log / divide chains.
      softmax_cce_lanes<NM>(a, z, lane, row, rw, N, &ysh[rw][0], bsh, &dz_s[rw][0], &met[rw][0]);
    }
  }
  if (lane == 0 && row_wave && (NM == 1 || a.act != 2)) {
    float dz[NM];
#pragma unroll
    for (int n = 0; n < NM; ++n) dz[n] = 0.f;
    float loss = 0.f, correct = 0.f;
    if (row < a.M) {
      const float* yr = a.y ? &ysh[rw][0] : nullptr;
      for (int n = 0; n < N; ++n) z[n] += bsh[n];
      const float eps = 1e-7f;
      if (a.act == 1) {
        const float p = 1.f / (1.f + expf(-z[0]));
        if (a.probs) a.probs[row] = p;
        if (yr) {
          const float yv = yr[0];
          const bool inr = (p >= eps) && (p <= 1.f - eps);
          const float pc = clip_nan(p, eps, 1.f - eps);
          const float lg = logf(pc / (1.f - pc));
          loss = fmaxf(lg, 0.f) - lg * yv + log1pf(expf(-fabsf(lg)));
          dz[0] = inr ? (pc - yv) : 0.f;
          correct = (rintf(p) == yv) ? 1.f : 0.f;
        }
      } else if (NM > 1 && a.act == 2) {
        float mx = z[0];
        int am = 0;
        for (int n = 1; n < N; ++n)
          if (z[n] > mx) { mx = z[n]; am = n; }
        float p[NM], s = 0.f;
        for (int n = 0; n < N; ++n) { p[n] = expf(z[n] - mx); s += p[n]; }
        for (int n = 0; n < N; ++n) p[n] /= s;
        if (a.probs)
          for (int n = 0; n < N; ++n) a.probs[(size_t)row * N + n] = p[n];
        if (yr) {
          float ps = 0.f;
          for (int n = 0; n < N; ++n) ps += p[n];
          float gq = 0.f, gn[NM];
          int ay = 0;
          float ymx = yr[0];
          for (int n = 0; n < N; ++n) {
            const float q = p[n] / ps;
            const bool inr = (q >= eps) && (q <= 1.f - eps);
            const float qc = clip_nan(q, eps, 1.f - eps);
            loss -= yr[n] * logf(qc);
            gn[n] = inr ? -yr[n] / qc : 0.f;
            gq += gn[n] * q;
            if (yr[n] > ymx) { ymx = yr[n]; ay = n; }
          }
          float pg = 0.f;
          for (int n = 0; n < N; ++n) { gn[n] = (gn[n] - gq) / ps; pg += p[n] * gn[n]; }
          for (int n = 0; n < N; ++n) dz[n] = p[n] * (gn[n] - pg);
          correct = (am == ay) ? 1.f : 0.f;
        }
      } else {
        if (a.probs)
          for (int n = 0; n < N; ++n) a.probs[(size_t)row * N + n] = z[n];
        if (yr) {
          for (int n = 0; n < N; ++n) {
            const float d = z[n] - yr[n];
            loss += d * d / N;
            dz[n] = 2.f * d / N;
          }
        }
      }
    }
    for (int n = 0; n < NM; ++n) dz_s[rw][n] = dz[n] * a.inv_bs;
    met[rw][0] = loss;
    met[rw][1] = correct;
  }
  HEAD_STAMP(2);
  __syncthreads();
  HEAD_STAMP(3);
  const int rows_here = min(RB, a.M - row0);
  if (tid == 0 && a.y && a.st) {
    float ls = 0.f, cs = 0.f;
    for (int r = 0; r < rows_here; ++r) { ls += met[r][0]; cs += met[r][1]; }
    // per-workgroup sums in a fixed row order, then order-independent integer atomics
    // spread over 16 slots: 128 workgroups on one address serialise at the L2 (~2 us)
    long long* slot = a.st->metric_slots[blockIdx.x & 15];
    // a non-finite loss (diverged trial) or one beyond the fixed-point range (|sum| >= 2^30
    // per workgroup) cannot be converted: count it in the slot's spare word instead, and the
    // host reports the loss as NaN (llrint of NaN/inf is undefined and would read as finite)
    const bool loss_ok = isfinite(ls) && fabsf(ls) < 1073741824.f;
    if (loss_ok) atomicAdd((unsigned long long*)&slot[0], (unsigned long long)llrint((double)ls * 4294967296.0));
    else atomicAdd((unsigned long long*)&slot[3], 1ull);
    atomicAdd((unsigned long long*)&slot[1], (unsigned long long)llrintf(cs));
    atomicAdd((unsigned long long*)&slot[2], (unsigned long long)rows_here);
  }
  HEAD_STAMP(4);
  if (!a.training) return;

  float* ws = a.wslab + (size_t)blockIdx.x * a.K * N;
  for (int idx = tid; idx < a.K * N; idx += 256) {
    const int k = idx / N, n = idx - (idx / N) * N;
    const int kp = a.flat_C ? flat_keras_to_padded(k, a.flat_C, a.flat_Cs) : k;
    float s = 0.f;
    for (int rl = 0; rl < rows_here; ++rl)
      s += (fused ? bf2f(hs[rl][kp]) : bf2f(a.h[(size_t)(row0 + rl) * a.Ks + kp])) * dz_s[rl][n];
    ws[idx] = s;
  }
  if (tid < N && a.bslab) {
    float s = 0.f;
    for (int rl = 0; rl < rows_here; ++rl) s += dz_s[rl][tid];
    a.bslab[(size_t)blockIdx.x * N + tid] = s;
  }
  HEAD_STAMP(5);
  const BwdThrough& t = a.bt;
  if (t.dy) {
    const int width = t.pH * t.pW * t.pCs;
    for (int idx = tid; idx < rows_here * width; idx += 256) {
      const int rl = idx / width;
      const int kp = idx - rl * width;
      const int y = kp / (t.pW * t.pCs);
      const int rem = kp - y * t.pW * t.pCs;
      const int x = rem / t.pCs;
      const int c = rem - x * t.pCs;
      float gs = 0.f;
      if (c < t.pC) {
        const int k = (y * t.pW + x) * t.pC + c;
        for (int n = 0; n < N; ++n) gs += dz_s[rl][n] * (wlds ? wsh[k * N + n] : a.w[(size_t)k * N + n]);
      }
      if (fused && t.prev_out == a.epi.out && t.pH == 1 && t.pW == 1) {
        // the previous stage IS the fused dense layer: its saved output row is in LDS
        if (c >= t.pCs) continue;
        if (c >= t.pC) {
          gs = 0.f;
        } else {
          if (t.drop_thr) {
            const uint32_t idx = (uint32_t)((size_t)(row0 + rl) * t.pC + c);
            gs = dropout_keep(idx, t.seed, t.stream_id, step, t.drop_thr) ? gs * t.drop_scale : 0.f;
          }
          if (t.prev_relu && !(bf2f(hs[rl][c]) > 0.f)) gs = 0.f;
        }
        t.dy[(size_t)(row0 + rl) * t.pCs + c] = f2bf(gs);
        continue;
      }
      bwd_through_store(t, row0 + rl, y, x, c, gs, step);
    }
  }
  HEAD_STAMP(6);
}

// Rows per workgroup: 4 (one wave per row), or 1 when the head also runs the previous dense
// layer's split-K epilogue (a row per workgroup spreads that reduction over 128 workgroups)
int head_rows_per_block(bool fused) { return fused ? 1 : HEAD_RB; }

// NM: class-count bound (1 = the binary sigmoid head: no per-class loops or arrays)
void launch_head(const HeadArgs& a, hipStream_t s) {
  const dim3 g1(a.M), g4((a.M + HEAD_RB - 1) / HEAD_RB);
  if (a.N == 1) {
    if (a.epi.part != nullptr) hipLaunchKernelGGL((head_kernel<1, 1>), g1, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((head_kernel<HEAD_RB, 1>), g4, dim3(256), 0, s, a);
  } else {
    if (a.epi.part != nullptr) hipLaunchKernelGGL((head_kernel<1, 16>), g1, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((head_kernel<HEAD_RB, 16>), g4, dim3(256), 0, s, a);
  }
}
int head_epi_max() { return HEAD_EPI_MAX; }
