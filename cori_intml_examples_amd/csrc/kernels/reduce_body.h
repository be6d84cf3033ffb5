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

__device__ __forceinline__ int red_desc(const RedTable& tab, int blk) {
  int di = 0;
  while (di + 1 < tab.n && blk >= tab.d[di + 1].blk0) ++di;
  return di;
}

// vec4 descriptors (identity layouts: Keras order = slab order): G = 256 / tpe threads each
// own 4 consecutive elements (1024 / tpe per block), their tpe split-lanes sum interleaved
// subsets of the S slabs with float4 loads, 8 in flight -- per element exactly the order of
// slab_reduce_elem (the accumulators a[u], their fixed combine, the lane tree), so the two
// paths agree bit for bit.  `red`: >= 2 KB of LDS (tpe 2: one float4 per element group).
__device__ __forceinline__ int vec4_epb(const RedDesc& d) { return 1024 / d.tpe; }
// first element (flat index) of vec4 table block blk
__device__ __forceinline__ int e_block0(const RedDesc& d, int blk) { return d.dst_off + (blk - d.blk0) * vec4_epb(d); }

__device__ __forceinline__ void add4(float4& a, const float4& b) { a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w; }

__device__ __forceinline__ bool slab_reduce_vec4(const RedDesc& d, int blk, float* red, int& e, float4& g) {
  const int tpe = d.tpe, G = 256 / tpe;
  const int gi = (int)threadIdx.x % G, lane = (int)threadIdx.x / G;
  const int le = ((blk - d.blk0) * G + gi) * 4;
  const bool in = le < d.numel;
  float4 acc = {0.f, 0.f, 0.f, 0.f};
  if (in) {
    const float* p = d.slab + le;
    const size_t st = (size_t)d.stride_s;
    float4 a[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) a[u] = float4{0.f, 0.f, 0.f, 0.f};
    int s = lane;
    for (; s + 7 * tpe < d.S; s += 8 * tpe) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const float4*>(p + (size_t)(s + u * tpe) * st);
#pragma unroll
      for (int u = 0; u < 8; ++u) add4(a[u], v[u]);
    }
    float4 v[7];
#pragma unroll
    for (int u = 0; u < 7; ++u)
      if (s + u * tpe < d.S) v[u] = *reinterpret_cast<const float4*>(p + (size_t)(s + u * tpe) * st);
#pragma unroll
    for (int u = 0; u < 7; ++u)
      if (s + u * tpe < d.S) add4(a[u], v[u]);
    add4(a[0], a[1]); add4(a[2], a[3]); add4(a[4], a[5]); add4(a[6], a[7]);
    add4(a[0], a[2]); add4(a[4], a[6]);
    acc = a[0];
    add4(acc, a[4]);
  }
  e = d.dst_off + le;
  if (tpe == 1) {
    g = acc;
    return in;
  }
  // the scalar path's fixed-order tree over the split-lanes (lane l += lane l + off), one
  // level per round: the upper half's G * off = 128 float4 partials fill the 2 KB of LDS
  float4* r4 = reinterpret_cast<float4*>(red);
  for (int off = tpe >> 1; off > 0; off >>= 1) {
    if (lane >= off && lane < 2 * off) r4[(lane - off) * G + gi] = acc;
    __syncthreads();
    if (lane < off) add4(acc, r4[lane * G + gi]);
    __syncthreads();
  }
  g = acc;
  return lane == 0 && in;
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

// The optimizer state of the elements a thread will update, loaded BEFORE the reduction whose
// result it updates them with: its memory round trip overlaps the slab loads instead of
// following them (~1 us of the reduction launch's latency chain)
struct OptState4 {
  float4 p, s0, s1;
};
struct OptState1 {
  float p, s0, s1;
};
__device__ __forceinline__ OptState4 load_state4(const OptimArgs& a, int e) {
  const float4 z = {0.f, 0.f, 0.f, 0.f};
  return OptState4{*reinterpret_cast<const float4*>(a.p + e), a.s0 ? *reinterpret_cast<const float4*>(a.s0 + e) : z,
                   a.s1 ? *reinterpret_cast<const float4*>(a.s1 + e) : z};
}
__device__ __forceinline__ OptState1 load_state1(const OptimArgs& a, int e) {
  return OptState1{a.p[e], a.s0 ? a.s0[e] : 0.f, a.s1 ? a.s1[e] : 0.f};
}

// Keras update of the elements a table block's thread holds (vec4 descriptor: the float4 at
// e, its state in st; `mine` false: the thread holds none) -- with the tiled pack writes of a dense route
// (dsc.tile: the workgroup's 1024 updated weights are whole 8-row groups of the route, staged
// as bf16 in LDS -- red: >= 2 KB -- and written as 16-byte vectors).  Every thread of the
// workgroup calls it (it may synchronise the workgroup).
template <int KIND>
__device__ __forceinline__ void update_vec4(const RedDesc& dsc, const OptimArgs& a, int blk, float* red, bool mine,
                                            int e, const float4& g, const OptState4& st) {
  const PackRoute* tr = nullptr;
  if (a.nroutes && dsc.tile) {
    for (int r = 0; r < a.nroutes; ++r) {           // uniform: the descriptor's route
      const PackRoute& R = a.routes[r];
      if (R.kind == 2 && R.Cin == R.Cs && dsc.dst_off >= R.lo && dsc.dst_off < R.hi) tr = &R;
    }
  }
  bf16* tl = reinterpret_cast<bf16*>(red);
  if (mine) {
    float4 p = st.p, s0 = st.s0, s1 = st.s1;
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
__device__ __forceinline__ void update_elem(const OptimArgs& a, int e, float g, const OptState1& st) {
  float p = st.p, s0 = st.s0, s1 = st.s1;
  opt_update<KIND>(a, a.st, p, g * a.grad_scale, &s0, &s1);
  a.p[e] = p;
  if (a.s0) a.s0[e] = s0;
  if (a.s1) a.s1[e] = s1;
  if (a.nroutes) pack_write(a, e, p);
}

// Reduction + Keras update of table block `blk`: the thread that produces an element's
// gradient writes it and applies the update at once.  `red`: 256 floats of LDS.  xp (the
// data-parallel step): also push the reduced elements to their owners, and no update.
// PRE: the optimizer state is loaded before the reduction (standalone kernels only: compiled
// into the dual conv launch's extras it made the compiler copy the whole by-value DualExtra
// argument to scratch -- 1.7 KB per lane, the launch 21 -> 90 us)
template <int KIND, bool PRE = false>
__device__ __forceinline__ void reduce_optim_block(float* __restrict__ grad, const RedTable& tab, const OptimArgs& a,
                                                   int blk, float* red, const XgmiPush* xp = nullptr) {
  const RedDesc& dsc = tab.d[red_desc(tab, blk)];
  const bool upd = !a.grad_only && !xp;
  const int t = threadIdx.x;
  if (dsc.vec4) {
    OptState4 st{};
    if (PRE && upd) {   // (slab_reduce_vec4's map: split-lane 0 of element group t % G holds the sum)
      const int G = 256 / dsc.tpe, le = ((blk - dsc.blk0) * G + t % G) * 4;
      if (t < G && le < dsc.numel) st = load_state4(a, dsc.dst_off + le);
    }
    int e;
    float4 g;
    const bool mine = slab_reduce_vec4(dsc, blk, red, e, g);
    if (mine) *reinterpret_cast<float4*>(grad + e) = g;
    if (mine && xp) xpush4(*xp, e, g);
    if (!PRE && mine && upd) st = load_state4(a, e);
    if (upd) update_vec4<KIND>(dsc, a, blk, red, mine, e, g, st);   // (grad_only: the reduced gradient is all)
  } else {
    OptState1 st{};
    if (PRE && upd) {   // (slab_reduce_elem's map: thread t < E holds element t of the block)
      const int E = 256 / dsc.tpe, le = (blk - dsc.blk0) * E + t;
      if (t < E && le < dsc.numel) st = load_state1(a, dsc.dst_off + le);
    }
    int e;
    float g;
    const bool mine = slab_reduce_elem(tab, blk, red, e, g);
    if (mine) grad[e] = g;
    if (mine && xp) xpush1(*xp, e, g);
    if (!PRE && mine && upd) st = load_state1(a, e);
    if (mine && upd) update_elem<KIND>(a, e, g, st);
  }
  if (a.defer_pack && !a.nroutes && upd && blk == 0 && threadIdx.x == 0) a.st->packs_stale = 1;
}

// ---------------------------------------------------------------- xGMI early-bucket exchange
// (XgmiPush, args.h).  The peer buffers are uncached device memory: the protocol is xgmi.hip's
// (payload stores drained, then -- fence 1, the default -- a system-scope release before the
// relaxed system-scope flag store; bounded relaxed polls followed by a system-scope acquire;
// the payload read with sc1 loads) -- see that file's header.
__device__ __forceinline__ unsigned xs_load(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void xs_store(unsigned* p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ bool xs_set_err(int* err, int v) {
  int zero = 0;
  return __hip_atomic_compare_exchange_strong(err, &zero, v, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_SYSTEM);
}
// n (1 or 4) floats at base[idx] of a peer-written buffer (sc1: not from this CU's L1)
__device__ __forceinline__ float4 xs_peer(const float* base, size_t idx, int n) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, 0x7fffffff, 0x00020000);
  if (n == 4) return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, (unsigned)(idx * 4), 0, 16));
  return float4{__builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (unsigned)(idx * 4), 0, 16)), 0.f,
                0.f, 0.f};
}
__device__ __forceinline__ float4 xs_local(const float* p, int n) {
  return n == 4 ? *reinterpret_cast<const float4*>(p) : float4{*p, 0.f, 0.f, 0.f};
}
__device__ __forceinline__ void xs_put(float* p, const float4& v, int n) {
  if (n == 4) *reinterpret_cast<float4*>(p) = v;
  else *p = v.x;
}
// system-scope release before a flag store (XgmiPush::fence 1): the payload stores before it
// are visible to every agent before the flag is (the drain before it already completed them)
__device__ __forceinline__ void xs_release() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ void xs_drain_sync() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}
// Lanes q < size with bit q of `mask` wait until flags[q] >= seq -- bounded in time, with
// xgmi.hip wait_all's failure protocol (a timeout records `phase` and raises every rank's
// sticky abort word; a raised abort word ends the wait as err 3).  Every thread calls it;
// false on failure.  s_ok: one int of LDS no other code of the block touches meanwhile.
__device__ __forceinline__ bool xs_wait(const XgmiPush& x, const unsigned* flags, unsigned mask, unsigned seq,
                                        int phase, int* s_ok) {
  const int t = threadIdx.x;
  if (t == 0) *s_ok = 1;
  __syncthreads();
  if (t < x.size && ((mask >> t) & 1u)) {
    const unsigned long long t0 = wall_clock64();
    while (xs_load(flags + t) < seq) {
      if (xs_load(x.abort_[x.rank])) {
        *s_ok = 0;
        xs_set_err(x.err, 3);
        break;
      }
      if ((long long)(wall_clock64() - t0) > x.timeout_ticks) {
        *s_ok = 0;
        if (xs_set_err(x.err, phase)) {
          x.err[1] = (int)seq;
          x.err[2] = (int)xs_load(flags + t);
          x.err[3] = (int)blockIdx.x * 64 + t;
        }
        for (int j = 0; j < x.size; ++j) xs_store(x.abort_[j], 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    if (x.fence == 1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");        // system-scope acquire
    else __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // (keeps the sc1 loads below the poll)
  }
  __syncthreads();
  return *s_ok != 0;
}

// data-parallel early bucket (a grad_only table), mode 1: reduction + producer push, no
// update; with block flags (exchange), the block's push flag is raised on every peer
__device__ __forceinline__ void reduce_push_block(float* __restrict__ grad, const RedTable& tab, const OptimArgs& a,
                                                  int blk, float* red, const XgmiPush& xp) {
  reduce_optim_block<OPT_SGD>(grad, tab, a, blk, red, &xp);
  if (xp.bflag1[0] == nullptr || xp.size == 1) {   // (no flags / no peers to flag)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the pushes complete with this workgroup
    return;
  }
  const unsigned seq = xp.ctrb[blk] + 1u;
  xs_drain_sync();
  const int t = threadIdx.x;
  if (t < xp.size && t != xp.rank) {
    if (xp.fence == 1) xs_release();
    xs_store(xp.bflag1[t] + (size_t)blk * xp.size + xp.rank, seq);
  }
}

// mode 2: finish the all-reduce of table block `blk` (pushed by mode 1 of an earlier launch on
// every rank) and apply its Keras update.  Element ownership and summation order are the fused
// all-reduce kernel's (owner chunks of x.chunk bucket elements; rows summed in rank order, the
// owner's own row from grad), so the sums are those the end-of-step kernel would produce.
// parts (bit mask): 1 = the OWNER part (wait for every sender's push flag, sum the rows, write
// the own elements' sums to grad, push them into every peer's outbox, raise bflag2); 2 = the
// FINISH part (wait for the block's other owners, read their sums, apply the update, advance
// the block's sequence counter).  Mode 2 / 3 run both in one launch; mode 4 runs the owner
// part in a backward launch and mode 5 the finish part in the end-of-backward launch, so no
// workgroup ever waits on a flag raised in its own launch.  Carried state (mode 3, one block
// per workgroup): `pre` -- the optimizer state loaded before the slab reduction -- and `gin`
// -- this thread's reduced partial, so the owner sum does not re-read it from memory.
template <int KIND>
__device__ __forceinline__ void xchg_update_block(float* __restrict__ grad, const RedTable& tab, const OptimArgs& a, int blk,
                                  float* red, const XgmiPush& x, int parts = 3, const OptState4* pre4 = nullptr,
                                  const OptState1* pre1 = nullptr, const float4* gin = nullptr) {
  const RedDesc& d = tab.d[red_desc(tab, blk)];
  const int P = x.size, me = x.rank, t = threadIdx.x, C = x.chunk;
  const unsigned seq = x.ctrb[blk] + 1u;
  int* s_ok = reinterpret_cast<int*>(red) + 1023;   // (past update_vec4's 2 KB tile stage)
  // the block's elements [b_lo, b_hi) and this thread's n elements at e (the reduce map)
  int b_lo, b_hi, e = 0, n = 0;
  if (d.vec4) {
    b_lo = e_block0(d, blk);
    b_hi = min(b_lo + vec4_epb(d), d.dst_off + d.numel);
    if (t < 256 / d.tpe && b_lo + 4 * t < b_hi) e = b_lo + 4 * t, n = 4;   // (slab_reduce_vec4's map)
  } else {
    const int E = 256 / d.tpe;   // (slab_reduce_elem: thread t < E holds element t)
    b_lo = d.dst_off + (blk - d.blk0) * E;
    b_hi = min(b_lo + E, d.dst_off + d.numel);
    if (t < E && b_lo + t < b_hi) e = b_lo + t, n = 1;
  }
  const int j0 = (int)((b_lo - x.lo) / C), j1 = (int)((b_hi - 1 - x.lo) / C);
  const bool owner = me >= j0 && me <= j1;
  if (parts == 1 && (P == 1 || !owner)) return;   // (mode 4: nothing of this block is mine to sum)
  // (the state the update needs is loaded now: its round trip overlaps the waits)
  OptState4 st4{};
  OptState1 st1{};
  if (parts & 2) {
    if (pre4) st4 = *pre4;
    else if (pre1) st1 = *pre1;
    else if (n == 4) st4 = load_state4(a, e);
    else if (n == 1) st1 = load_state1(a, e);
  }
  const long long ie = (long long)e - x.lo;     // bucket index
  const int own = n ? (int)(ie / C) : -1;
  float4 g = {0.f, 0.f, 0.f, 0.f};
  if (P == 1) {                                 // (no peers: the reduced gradient is final)
    if (n) g = gin ? *gin : xs_local(grad + e, n);
  } else if ((parts & 1) && owner) {
    // the owner part: every sender's row of the block is in my inbox
    if (!xs_wait(x, x.bflag1[me] + (size_t)blk * P, ~(1u << me), seq, 4, s_ok)) return;
    if (own == me) {
      const size_t k = (size_t)(ie - (long long)me * C);
      float4 v[XGMI_MAX_RANKS];
#pragma unroll
      for (int q = 0; q < XGMI_MAX_RANKS; ++q)
        if (q < P) v[q] = q == me ? (gin ? *gin : xs_local(grad + e, n)) : xs_peer(x.inbox[me], (size_t)q * C + k, n);
      g = v[0];
#pragma unroll
      for (int q = 1; q < XGMI_MAX_RANKS; ++q)
        if (q < P) g.x += v[q].x, g.y += v[q].y, g.z += v[q].z, g.w += v[q].w;
      xs_put(grad + e, g, n);
#pragma unroll
      for (int j = 0; j < XGMI_MAX_RANKS; ++j)
        if (j < P && j != me) xs_put(x.outbox[j] + ie, g, n);
    }
    xs_drain_sync();
    if (t < P && t != me) {
      if (x.fence == 1) xs_release();
      xs_store(x.bflag2[t] + (size_t)blk * P + me, seq);
    }
  } else if (n && own == me) {
    g = xs_local(grad + e, n);                  // (mode 5: my own sums, written by the owner part)
  }
  if (!(parts & 2)) return;
  // the other owners' sums of this block's elements are in my outbox
  unsigned need = 0;
  for (int j = j0; j <= j1 && P > 1; ++j)
    if (j != me) need |= 1u << j;
  if (need) {
    if (!xs_wait(x, x.bflag2[me] + (size_t)blk * P, need, seq, 5, s_ok)) return;
    if (n && own != me) {
      g = xs_peer(x.outbox[me], (size_t)ie, n);
      xs_put(grad + e, g, n);
    }
  }
  if (d.vec4) update_vec4<KIND>(d, a, blk, red, n == 4, e, g, st4);
  else if (n) update_elem<KIND>(a, e, g.x, st1);
  if (a.defer_pack && !a.nroutes && blk == 0 && t == 0) a.st->packs_stale = 1;
  if (t == 0) x.ctrb[blk] = seq;
}

// mode 3 with one block per workgroup: the slab reduction, the producer push and the exchange
// of ONE block with the optimizer state loaded before the slab loads and the reduced partial
// kept in registers for the owner sum (no memory round trip between the phases).  Its own
// kernel (misc.hip xchg_fused_kernel, optimizer kind a template parameter): compiled into
// xgmi_early_kernel beside the other modes it made the compiler copy the by-value RedTable /
// XgmiPush arguments to scratch (1.6 KB per lane)
template <int KIND>
__device__ __forceinline__ void xchg_fused_block(float* __restrict__ grad, const RedTable& tab, const OptimArgs& a,
                                                 int blk, float* red, const XgmiPush& x) {
  const RedDesc& dsc = tab.d[red_desc(tab, blk)];
  const int t = threadIdx.x;
  float4 g4 = {0.f, 0.f, 0.f, 0.f};
  if (dsc.vec4) {
    OptState4 st{};
    const int G = 256 / dsc.tpe, le = ((blk - dsc.blk0) * G + t % G) * 4;
    if (t < G && le < dsc.numel) st = load_state4(a, dsc.dst_off + le);
    int e;
    const bool mine = slab_reduce_vec4(dsc, blk, red, e, g4);
    if (mine) *reinterpret_cast<float4*>(grad + e) = g4;
    if (mine && x.size > 1) xpush4(x, e, g4);
    if (x.size > 1) {
      xs_drain_sync();
      if (t < x.size && t != x.rank) {
        if (x.fence == 1) xs_release();
        xs_store(x.bflag1[t] + (size_t)blk * x.size + x.rank, x.ctrb[blk] + 1u);
      }
    }
    __syncthreads();   // (red is reused)
    xchg_update_block<KIND>(grad, tab, a, blk, red, x, 3, &st, nullptr, &g4);
  } else {
    OptState1 st{};
    const int E = 256 / dsc.tpe, le = (blk - dsc.blk0) * E + t;
    if (t < E && le < dsc.numel) st = load_state1(a, dsc.dst_off + le);
    int e;
    float g;
    const bool mine = slab_reduce_elem(tab, blk, red, e, g);
    if (mine) grad[e] = g;
    if (mine && x.size > 1) xpush1(x, e, g);
    if (x.size > 1) {
      xs_drain_sync();
      if (t < x.size && t != x.rank) {
        if (x.fence == 1) xs_release();
        xs_store(x.bflag1[t] + (size_t)blk * x.size + x.rank, x.ctrb[blk] + 1u);
      }
    }
    __syncthreads();
    g4.x = g;
    xchg_update_block<KIND>(grad, tab, a, blk, red, x, 3, nullptr, &st, &g4);
  }
}

// sticky abort (an earlier wait timed out on some rank): true = touch nothing
__device__ __forceinline__ bool xs_aborted(const XgmiPush& x) {
  if (x.size > 1 && xs_load(x.abort_[x.rank])) {
    if (threadIdx.x == 0) xs_set_err(x.err, 3);
    return true;
  }
  return false;
}

// workgroup r of a data-parallel table launch: mode 1 (reduce + push) one table block each;
// mode 2 (exchange + update) and mode 3 (both, one launch: the end-of-backward bucket) one
// block each, or x.nx workgroups looping over the blocks in order (ranks sharing a GPU; mode 3
// then pushes all of its blocks before its first wait); mode 4 / 5: the owner / finish part
// of mode 2 (xchg_update_block), block b_lo + r (mode 4: blocks [b_lo, b_hi) of the table,
// those no part of which this rank owns exit at once).  M3: mode 3 compiled in -- the
// standalone launch only: in the dual conv launch (modes 1 / 2 / 4) its extra code made the
// compiler copy the whole by-value DualExtra argument to scratch (1.7 KB per lane)
template <bool M3>
__device__ __forceinline__ void xgmi_early_block(float* __restrict__ grad, const RedTable& tab, const OptimArgs& a,
                                                 int r, float* red, const XgmiPush& x) {
  if (x.mode == 1) {
    reduce_push_block(grad, tab, a, r, red, x);
    return;
  }
  if (x.size > 1 && xs_load(x.abort_[x.rank])) {   // sticky abort (an earlier wait timed out): touch nothing
    if (threadIdx.x == 0) xs_set_err(x.err, 3);
    return;
  }
  const int step = x.nx ? x.nx : (x.mode == 4 ? x.b_hi - x.b_lo : x.nblk);
  const int b0 = x.mode == 4 ? x.b_lo : 0, b1 = x.mode == 4 ? x.b_hi : x.nblk;
  if constexpr (!M3) {
    // the dual conv launch's extras run modes 1 and 4 only (launch_dual_halo declines the
    // others): the owner half updates nothing, so one instantiation serves every optimizer --
    // the five optimizer kinds of mode 2 compiled in raised the dual kernel's SGPR spills
    for (int b = b0 + r; b < b1; b += step) {
      xchg_update_block<OPT_SGD>(grad, tab, a, b, red, x, 1);
      __syncthreads();
    }
    return;
  }
  const int parts = x.mode == 4 ? 1 : (x.mode == 5 ? 2 : 3);
  if constexpr (M3) {
  if (x.mode == 3 && x.size == 1 && !x.p1) {   // no peers: the single-GPU reduction + update
    for (int b = r; b < x.nblk; b += step) {
      switch (a.kind) {
        case OPT_ADAM: reduce_optim_block<OPT_ADAM>(grad, tab, a, b, red); break;
        case OPT_NADAM: reduce_optim_block<OPT_NADAM>(grad, tab, a, b, red); break;
        case OPT_ADADELTA: reduce_optim_block<OPT_ADADELTA>(grad, tab, a, b, red); break;
        case OPT_RMSPROP: reduce_optim_block<OPT_RMSPROP>(grad, tab, a, b, red); break;
        default: reduce_optim_block<OPT_SGD>(grad, tab, a, b, red); break;
      }
      __syncthreads();
    }
    return;
  }
  if (x.mode == 3) {
    for (int b = r; b < x.nblk; b += step) {
      reduce_push_block(grad, tab, a, b, red, x);
      __syncthreads();
    }
    if (x.size == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  }
  for (int b = b0 + r; b < b1; b += step) {
    switch (a.kind) {
      case OPT_ADAM: xchg_update_block<OPT_ADAM>(grad, tab, a, b, red, x, parts); break;
      case OPT_NADAM: xchg_update_block<OPT_NADAM>(grad, tab, a, b, red, x, parts); break;
      case OPT_ADADELTA: xchg_update_block<OPT_ADADELTA>(grad, tab, a, b, red, x, parts); break;
      case OPT_RMSPROP: xchg_update_block<OPT_RMSPROP>(grad, tab, a, b, red, x, parts); break;
      default: xchg_update_block<OPT_SGD>(grad, tab, a, b, red, x, parts); break;
    }
    __syncthreads();   // (the next block reuses red)
  }
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
