// Deterministic slab reduction (and the fused optimizer over it), as device functions of the
// reduction-table block index `blk`: the reduction kernels of misc.hip run one table block per
// workgroup, and the dual conv backward launch (dual_halo_body.h) runs an early bucket's
// table in extra workgroups of its own grid.
#pragma once
#include "args.h"
#include "optim_math.h"

// Each descriptor owns a contiguous range of workgroups; a workgroup covers E = 256/tpe
// consecutive elements: thread t -> element t % E (consecutive lanes read consecutive
// addresses of one slab: coalesced) and split-lane t / E (the tpe split-lanes of an
// element sum interleaved subsets of <= 4 of the S slabs, loads all in flight: the
// reduction is one memory round trip deep however many slabs there are).  The tpe
// partials are combined by a fixed-order LDS tree -> bitwise reproducible.
// Returns true on the thread that holds the final sum of element `dst` (in `val`).
__device__ __forceinline__ bool slab_reduce_elem(const RedTable& tab, int blk, float* red, int& dst, float& val) {
  int di = 0;
  while (di + 1 < tab.n && blk >= tab.d[di + 1].blk0) ++di;
  const RedDesc& d = tab.d[di];
  const int tpe = d.tpe;
  const int E = 256 / tpe;
  const int el = (int)threadIdx.x % E;
  const int lane = (int)threadIdx.x / E;
  const int le = (blk - d.blk0) * E + el;
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
    // 8 independent loads per round (all issued before the first add), fixed summation order
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int s = lane;
    for (; s + 7 * tpe < d.S; s += 8 * tpe) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = p[(size_t)(s + u * tpe) * st];
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u] += v[u];
    }
#pragma unroll
    for (int u = 0; u < 7; ++u)
      if (s + u * tpe < d.S) a[u] += p[(size_t)(s + u * tpe) * st];
    acc = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  }
  dst = d.dst_off + le;
  if (tpe == 1) {
    val = acc;
    return in;
  }
  // fixed-order tree over the tpe split-lanes (bitwise reproducible)
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int off = tpe >> 1; off > 0; off >>= 1) {
    if (lane < off) red[threadIdx.x] += red[threadIdx.x + off * E];
    __syncthreads();
  }
  if (lane != 0 || !in) return false;
  val = red[el];
  return true;
}

// vec4 descriptors (identity layout): thread -> 4 consecutive elements, float4 slab loads in
// fixed split order (the same per-element order as slab_reduce_elem with tpe = 1).
__device__ __forceinline__ int red_desc(const RedTable& tab, int blk) {
  int di = 0;
  while (di + 1 < tab.n && blk >= tab.d[di + 1].blk0) ++di;
  return di;
}

// first element (flat index) of vec4 table block blk
__device__ __forceinline__ int e_block0(const RedDesc& d, int blk) { return d.dst_off + (blk - d.blk0) * 1024; }

__device__ __forceinline__ bool slab_reduce_vec4(const RedDesc& d, int blk, int& e, float4& g) {
  const int le = ((blk - d.blk0) * 256 + (int)threadIdx.x) * 4;
  if (le >= d.numel) return false;
  const float* p = d.slab + le;
  float4 v[8];
#pragma unroll
  for (int s = 0; s < 8; ++s)
    if (s < d.S) v[s] = *reinterpret_cast<const float4*>(p + (size_t)s * d.stride_s);
  float4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};   // a[s % 2], like the scalar path's a[u]
#pragma unroll
  for (int s = 0; s < 8; ++s)
    if (s < d.S) {
      float4& a = (s & 1) ? a1 : a0;
      a.x += v[s].x; a.y += v[s].y; a.z += v[s].z; a.w += v[s].w;
    }
  g = float4{a0.x + a1.x, a0.y + a1.y, a0.z + a1.z, a0.w + a1.w};
  e = d.dst_off + le;
  return true;
}

// Producer push of one finalised gradient element / float4 (XgmiPush; e: flat element, the
// float4 is 4-aligned in the bucket and never straddles an owner chunk: chunk % 4 == 0)
__device__ __forceinline__ void xpush1(const XgmiPush& xp, long long e, float v) {
  const long long idx = e - xp.lo;
  const int j = (int)(idx / xp.chunk);
  if (j != xp.rank) xp.inbox[j][(size_t)xp.rank * xp.chunk + (size_t)(idx - (long long)j * xp.chunk)] = v;
}
__device__ __forceinline__ void xpush4(const XgmiPush& xp, long long e, const float4& v) {
  const long long idx = e - xp.lo;
  const int j = (int)(idx / xp.chunk);
  if (j != xp.rank)
    *reinterpret_cast<float4*>(xp.inbox[j] + (size_t)xp.rank * xp.chunk + (size_t)(idx - (long long)j * xp.chunk)) = v;
}

// Keras update of the elements a table block's thread holds (vec4 descriptor: the float4 at
// e; `mine` false: the thread holds none) -- with the tiled pack writes of a dense route
// (dsc.tile: the workgroup's 1024 updated weights are whole 8-row groups of the route, staged
// as bf16 in LDS -- red: >= 2 KB -- and written as 16-byte vectors).  Every thread of the
// workgroup calls it (it may synchronise the workgroup).
template <int KIND>
__device__ __forceinline__ void update_vec4(const RedDesc& dsc, const OptimArgs& a, int blk, float* red, bool mine,
                                            int e, const float4& g) {
  const PackRoute* tr = nullptr;
  if (a.nroutes && dsc.tile) {
    for (int r = 0; r < a.nroutes; ++r) {           // uniform: the descriptor's route
      const PackRoute& R = a.routes[r];
      if (R.kind == 2 && R.Cin == R.Cs && dsc.dst_off >= R.lo && dsc.dst_off < R.hi) tr = &R;
    }
  }
  bf16* tl = reinterpret_cast<bf16*>(red);
  if (mine) {
    float4 p = *reinterpret_cast<const float4*>(a.p + e);
    float4 s0 = a.s0 ? *reinterpret_cast<const float4*>(a.s0 + e) : float4{0.f, 0.f, 0.f, 0.f};
    float4 s1 = a.s1 ? *reinterpret_cast<const float4*>(a.s1 + e) : float4{0.f, 0.f, 0.f, 0.f};
    const float gs = a.grad_scale;
    opt_update<KIND>(a, a.st, p.x, g.x * gs, &s0.x, &s1.x);
    opt_update<KIND>(a, a.st, p.y, g.y * gs, &s0.y, &s1.y);
    opt_update<KIND>(a, a.st, p.z, g.z * gs, &s0.z, &s1.z);
    opt_update<KIND>(a, a.st, p.w, g.w * gs, &s0.w, &s1.w);
    *reinterpret_cast<float4*>(a.p + e) = p;
    if (a.s0) *reinterpret_cast<float4*>(a.s0 + e) = s0;
    if (a.s1) *reinterpret_cast<float4*>(a.s1 + e) = s1;
    if (tr) {
      bf16x4 v;
      v[0] = f2bf(p.x); v[1] = f2bf(p.y); v[2] = f2bf(p.z); v[3] = f2bf(p.w);
      *reinterpret_cast<bf16x4*>(tl + 4 * threadIdx.x) = v;
    } else if (a.nroutes) {
      pack_write4(a, e, p);
    }
  }
  if (tr) {
    __syncthreads();
    const PackRoute R = *tr;
    const int N = R.Cout, le0 = e_block0(dsc, blk) - R.lo, r0 = le0 / N;
    const int t = threadIdx.x;
    if (t < 128) {          // forward: 8 consecutive rows (k) of column n
      const int gi = t / N, n = t - gi * N;
      if (R.fwd >= 0) {
        bf16x8 v;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = tl[(gi * 8 + j) * N + n];
        *reinterpret_cast<bf16x8*>(a.arena + R.fwd + frag_off(r0 + gi * 8, n, R.NT)) = v;
      }
    } else if (R.bwd >= 0) {  // backward: 8 consecutive columns (n) of row k
      const int v8 = t - 128, per = N >> 3, row = v8 / per, c8 = (v8 - row * per) * 8;
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(tl + row * N + c8);
      *reinterpret_cast<bf16x8*>(a.arena + R.bwd + frag_off(c8, r0 + row, R.NTb)) = v;
    }
  }
}

template <int KIND>
__device__ __forceinline__ void update_elem(const OptimArgs& a, int e, float g) {
  float p = a.p[e];
  float s0 = a.s0 ? a.s0[e] : 0.f, s1 = a.s1 ? a.s1[e] : 0.f;
  opt_update<KIND>(a, a.st, p, g * a.grad_scale, &s0, &s1);
  a.p[e] = p;
  if (a.s0) a.s0[e] = s0;
  if (a.s1) a.s1[e] = s1;
  if (a.nroutes) pack_write(a, e, p);
}

// Reduction + Keras update of table block `blk`: the thread that produces an element's
// gradient writes it and applies the update at once.  `red`: 256 floats of LDS.  xp (grad_only
// tables of the data-parallel step): also push the reduced elements to their owners.
template <int KIND>
__device__ __forceinline__ void reduce_optim_block(float* __restrict__ grad, const RedTable& tab, const OptimArgs& a,
                                                   int blk, float* red, const XgmiPush* xp = nullptr) {
  const RedDesc& dsc = tab.d[red_desc(tab, blk)];
  if (dsc.vec4) {
    int e;
    float4 g;
    const bool mine = slab_reduce_vec4(dsc, blk, e, g);
    if (mine) *reinterpret_cast<float4*>(grad + e) = g;
    if (mine && xp) xpush4(*xp, e, g);
    if (!a.grad_only) update_vec4<KIND>(dsc, a, blk, red, mine, e, g);   // (grad_only: the reduced gradient is all)
  } else {
    int e;
    float g;
    const bool mine = slab_reduce_elem(tab, blk, red, e, g);
    if (mine) grad[e] = g;
    if (mine && xp) xpush1(*xp, e, g);
    if (mine && !a.grad_only) update_elem<KIND>(a, e, g);
  }
  if (a.defer_pack && !a.nroutes && !a.grad_only && blk == 0 && threadIdx.x == 0) a.st->packs_stale = 1;
}

// data-parallel early bucket (a grad_only table): reduction + producer push, no update
__device__ __forceinline__ void reduce_push_block(float* __restrict__ grad, const RedTable& tab, const OptimArgs& a,
                                                  int blk, float* red, const XgmiPush& xp) {
  reduce_optim_block<OPT_SGD>(grad, tab, a, blk, red, &xp);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the pushes complete with this workgroup
}

// the same with the optimizer kind chosen at run time (a workgroup-uniform switch)
__device__ __forceinline__ void reduce_optim_block_rt(float* __restrict__ grad, const RedTable& tab,
                                                      const OptimArgs& a, int blk, float* red) {
  switch (a.kind) {
    case OPT_ADAM: reduce_optim_block<OPT_ADAM>(grad, tab, a, blk, red); break;
    case OPT_NADAM: reduce_optim_block<OPT_NADAM>(grad, tab, a, blk, red); break;
    case OPT_ADADELTA: reduce_optim_block<OPT_ADADELTA>(grad, tab, a, blk, red); break;
    case OPT_RMSPROP: reduce_optim_block<OPT_RMSPROP>(grad, tab, a, blk, red); break;
    default: reduce_optim_block<OPT_SGD>(grad, tab, a, blk, red); break;
  }
}
