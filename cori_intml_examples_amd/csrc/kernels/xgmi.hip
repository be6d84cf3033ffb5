// Fused data-parallel gradient all-reduce + optimizer over xGMI (SURVEY.md §5.1 item 3:
// small-bucket P2P all-reduce; N7 comm).  Two-shot (reduce-scatter + all-gather) by direct
// peer stores into IPC-mapped uncached device memory, with the Keras update fused into the
// final pass -- ONE kernel on the training stream instead of an RCCL collective plus an
// optimizer launch (a linear HIP graph: no cross-queue edges).  See XgmiArgs (args.h).
//
// Memory model (MI355X_MICROARCH.md "inter-workgroup visibility", cdna_hip_programming.md
// Guideline 16, across GPUs).  The inbox / outbox / flags are UNCACHED device memory (MTYPE UC):
// payload stores go straight to the owning GPU's memory and are acknowledged from there, so
//   producer: payload stores -> every wave s_waitcnt vmcnt(0) -> workgroup barrier ->
//             relaxed system-scope flag store (the drained stores are complete: nothing is left
//             in any cache to write back -- the write-through publish of Guideline 16 R1);
//   consumer: relaxed system-scope poll (bounded) -> acquire -> barrier -> loads.
// a.fence selects the fences around the flags: 1 (default) = system-scope release before every
// flag store + system-scope acquire after every poll -- the HIP memory model's hand-off between
// agents (the release writes back the XCD's L2, the acquire invalidates it); 3 (opt-in,
// INTML_TUNE=xgmi_fence=3) = none, and every load of a peer's payload (inbox / outbox) is an sc1
// buffer load (Guideline 16: a hand-off stored to uncached memory and drained, read with sc1
// loads, needs no fence -- correct for MTYPE UC memory on this ISA, but outside the language
// memory model, so it is not the default until a multi-GPU run shows parity); 2 = an
// agent-scope acquire; 0 = none, plain loads.
#include <cstring>
#include <stdexcept>
#include <string>

#include "args.h"
#include "optim_math.h"

namespace {

__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ unsigned sys_load(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void sys_store(unsigned* p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// first cause wins: a timeout recorded by one workgroup is not overwritten by the abort the
// rank's other workgroups then observe; returns true for the lane that recorded it
__device__ __forceinline__ bool set_err(int* err, int v) {
  int zero = 0;
  return __hip_atomic_compare_exchange_strong(err, &zero, v, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_SYSTEM);
}

// Lanes 0..P-1 of wave 0 each raise flag `slot` of rank `lane` to seq.
__device__ __forceinline__ void signal_all(unsigned* const* flags, int slot, int P, unsigned seq, int fence) {
  drain_stores();
  __syncthreads();
  const int t = threadIdx.x;
  if (t < P) {
    if (fence == 1) {   // (payload in uncached memory is not in any cache: drained stores suffice)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      drain_stores();
    }
    sys_store(flags[t] + slot, seq);
  }
}

// Wait until local flags [base, base + P) all reach seq (lanes 0..P-1 poll one each).
// Bounded in TIME (wall_clock64, 100 MHz), not in polls.  On a timeout the lane records
// `phase` in err and raises the sticky abort word of EVERY rank: a peer that is merely late
// must never match a later step's flags against this step's data, so every later launch on
// every rank exits at its first instruction (the host raises on the error word).  A rank that
// sees the abort word while waiting gives up at once (err 3) instead of waiting out its own
// timeout.  Returns false on either.
__device__ __forceinline__ bool wait_all(const XgmiArgs& a, const unsigned* flags, unsigned seq, int phase) {
  __shared__ int s_ok;
  const int t = threadIdx.x, P = a.size;
  if (t == 0) s_ok = 1;
  __syncthreads();
  if (t < P) {
    const unsigned long long t0 = wall_clock64();
    while (sys_load(flags + t) < seq) {
      if (sys_load(a.abort_[a.rank])) {
        s_ok = 0;
        set_err(a.err, 3);
        break;
      }
      if ((long long)(wall_clock64() - t0) > a.timeout_ticks) {
        s_ok = 0;
        if (set_err(a.err, phase)) {   // diagnostics of the first timeout: what was awaited / seen
          a.err[1] = (int)seq;
          a.err[2] = (int)sys_load(flags + t);
          a.err[3] = (int)blockIdx.x * 64 + t;
        }
        for (int j = 0; j < P; ++j) sys_store(a.abort_[j], 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    if (a.fence == 1) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      drain_stores();
    } else if (a.fence == 2) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      drain_stores();
    } else {   // (3: the payload loads are sc1; this only keeps them below the poll)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
  __syncthreads();
  return s_ok != 0;
}

// 16-byte payload load from a peer-written buffer (wave-uniform base): sc1 (fence 3: bypasses
// this CU's L1, no acquire needed) or plain
__device__ __forceinline__ float4 load_peer4(const float* base, size_t idx, int fence) {
  if (fence == 3) {
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, 0x7fffffff, 0x00020000);
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, (unsigned)(idx * 4), 0, 16));
  }
  return *reinterpret_cast<const float4*>(base + idx);
}

__device__ __forceinline__ float4 load4_guarded(const float* p, long long idx, long long n) {
  if (idx + 4 <= n) return *reinterpret_cast<const float4*>(p + idx);
  float4 v = {0.f, 0.f, 0.f, 0.f};
  if (idx < n) v.x = p[idx];
  if (idx + 1 < n) v.y = p[idx + 1];
  if (idx + 2 < n) v.z = p[idx + 2];
  if (idx + 3 < n) v.w = p[idx + 3];
  return v;
}

// skip_mode 2: bucket elements [skip_lo, skip_hi) were all-reduced and updated inside the
// backward (XgmiPush exchange): no phase touches them
__device__ __forceinline__ bool xchg_done(const XgmiArgs& a, long long e) {
  return a.skip_mode == 2 && e >= a.skip_lo && e < a.skip_hi;
}
__device__ __forceinline__ bool xchg_done4(const XgmiArgs& a, long long e) {
  return a.skip_mode == 2 && e >= a.skip_lo && e + 4 <= a.skip_hi;
}

// grad[idx .. idx+4) = g4 (the reduced SUM) and, in mode 1, the Keras update of those
// parameters with the 1/size average folded in (elements past n, and exchanged ones, skipped)
template <int KIND>
__device__ __forceinline__ void finish4(const XgmiArgs& a, float* __restrict__ grad, long long idx, long long n,
                                        const float4 g4) {
  if (idx >= n) return;
  const OptimArgs& o = a.opt;
  const bool part = a.skip_mode == 2 && idx + 4 > a.skip_lo && idx < a.skip_hi;   // (straddles the range)
  if (idx + 4 <= n && !part) {       // float4 path (idx, C, k multiples of 4: 16-byte aligned)
    *reinterpret_cast<float4*>(grad + idx) = g4;
    if (a.mode == 1) {
      float4 p4 = *reinterpret_cast<const float4*>(o.p + idx);
      float4 m4 = o.s0 ? *reinterpret_cast<const float4*>(o.s0 + idx) : float4{0.f, 0.f, 0.f, 0.f};
      float4 v4 = o.s1 ? *reinterpret_cast<const float4*>(o.s1 + idx) : float4{0.f, 0.f, 0.f, 0.f};
      const float gs = o.grad_scale;
      opt_update<KIND>(o, o.st, p4.x, g4.x * gs, &m4.x, &v4.x);
      opt_update<KIND>(o, o.st, p4.y, g4.y * gs, &m4.y, &v4.y);
      opt_update<KIND>(o, o.st, p4.z, g4.z * gs, &m4.z, &v4.z);
      opt_update<KIND>(o, o.st, p4.w, g4.w * gs, &m4.w, &v4.w);
      *reinterpret_cast<float4*>(o.p + idx) = p4;
      if (o.s0) *reinterpret_cast<float4*>(o.s0 + idx) = m4;
      if (o.s1) *reinterpret_cast<float4*>(o.s1 + idx) = v4;
      if (o.nroutes) pack_write4(o, o.lo + (int)idx, p4);   // o.lo: the bucket's flat start
    }
    return;
  }
  const float gv[4] = {g4.x, g4.y, g4.z, g4.w};
  for (int e = 0; e < (int)min(n - idx, 4LL); ++e) {
    if (xchg_done(a, idx + e)) continue;
    grad[idx + e] = gv[e];
    if (a.mode == 1) {
      float pe = o.p[idx + e];
      float s0 = o.s0 ? o.s0[idx + e] : 0.f, s1 = o.s1 ? o.s1[idx + e] : 0.f;
      opt_update<KIND>(o, o.st, pe, gv[e] * o.grad_scale, &s0, &s1);
      o.p[idx + e] = pe;
      if (o.s0) o.s0[idx + e] = s0;
      if (o.s1) o.s1[idx + e] = s1;
      if (o.nroutes) pack_write(o, o.lo + (int)(idx + e), pe);
    }
  }
}

template <int KIND>
__global__ __launch_bounds__(256) void xgmi_allreduce_kernel(const XgmiArgs a) {
  __shared__ unsigned s_seq;
  __shared__ int s_abort;
  const int w = blockIdx.x, t = threadIdx.x;
  if (t == 0) {
    s_seq = a.ctr[w] + 1u;
    // sticky abort (a rank timed out in an earlier launch): touch nothing, keep the counters
    s_abort = sys_load(a.abort_[a.rank]) != 0u;
    if (s_abort) set_err(a.err, 3);
  }
  __syncthreads();
  if (s_abort) return;
  const unsigned seq = s_seq;
  const int P = a.size, r = a.rank, C = a.chunk;
  const int k0 = w * a.sub, k1 = min(k0 + a.sub, C);
  const long long n = a.n;

  // Every phase first loads all P float4 of a thread into registers, then stores: the
  // compiler cannot reorder loads across stores to possibly-aliasing pointers, and each
  // uncached / remote access costs microseconds, so they must all be in flight together.
  // The owner's own chunk never leaves cached memory: it is not pushed to the own inbox
  // (phase 2 reads it from grad), and its reduced sum + update are written straight to grad
  // in phase 2 (not round-tripped through the own outbox) -- at P = 1 (loopback) the kernel
  // touches no uncached memory besides the flags.
  float* __restrict__ grad = a.grad;

  // 1. push my slice of every OTHER rank's chunk to its owner's inbox row r
  if (P > 1) {
    for (int k = k0 + 4 * t; k < k1; k += 1024) {
      float4 v[XGMI_MAX_RANKS];
#pragma unroll
      for (int j = 0; j < XGMI_MAX_RANKS; ++j)
        if (j < P && j != r) v[j] = load4_guarded(grad, (long long)j * C + k, n);
#pragma unroll
      for (int j = 0; j < XGMI_MAX_RANKS; ++j) {
        const long long e = (long long)j * C + k;
        // (elements the backward already pushed -- XgmiPush -- are in the inbox)
        if (j < P && j != r && !(e >= a.skip_lo && e + 4 <= a.skip_hi))
          *reinterpret_cast<float4*>(a.inbox[j] + (size_t)r * C + k) = v[j];
      }
    }
  }
  signal_all(a.flag1, w * P + r, P, seq, a.fence);

  // 2. reduce my chunk's slice over the P rows in rank order (my own row from grad), push
  //    it to every other rank's outbox, and finish my own chunk in place
  if (!wait_all(a, a.flag1[r] + w * P, seq, 1)) return;
  {
    const float* __restrict__ in = a.inbox[r];
    for (int k = k0 + 4 * t; k < k1; k += 1024) {
      const long long own = (long long)r * C + k;
      if (xchg_done4(a, own)) continue;
      float4 v[XGMI_MAX_RANKS];
#pragma unroll
      for (int q = 0; q < XGMI_MAX_RANKS; ++q)
        if (q < P) v[q] = q == r ? load4_guarded(grad, own, n) : load_peer4(in, (size_t)q * C + k, a.fence);
      float4 s4 = v[0];
#pragma unroll
      for (int q = 1; q < XGMI_MAX_RANKS; ++q)
        if (q < P) { s4.x += v[q].x; s4.y += v[q].y; s4.z += v[q].z; s4.w += v[q].w; }
#pragma unroll
      for (int j = 0; j < XGMI_MAX_RANKS; ++j)
        if (j < P && j != r) *reinterpret_cast<float4*>(a.outbox[j] + (size_t)r * C + k) = s4;
      finish4<KIND>(a, grad, own, n, s4);
    }
  }
  signal_all(a.flag2, w * P + r, P, seq, a.fence);

  // 3. every other chunk's reduced sum is in my outbox: record it and update the parameters
  if (!wait_all(a, a.flag2[r] + w * P, seq, 2)) return;
  if (P > 1) {
    const float* __restrict__ red = a.outbox[r];
    for (int k = k0 + 4 * t; k < k1; k += 1024) {
      float4 g[XGMI_MAX_RANKS];
#pragma unroll
      for (int q = 0; q < XGMI_MAX_RANKS; ++q)
        if (q < P && q != r && !xchg_done4(a, (long long)q * C + k)) g[q] = load_peer4(red, (size_t)q * C + k, a.fence);
#pragma unroll
      for (int q = 0; q < XGMI_MAX_RANKS; ++q)
        if (q < P && q != r && !xchg_done4(a, (long long)q * C + k)) finish4<KIND>(a, grad, (long long)q * C + k, n, g[q]);
    }
  }
  if (a.mode == 1 && a.opt.defer_pack && !a.opt.nroutes && w == 0 && t == 0) a.opt.st->packs_stale = 1;
  if (t == 0) a.ctr[w] = seq;
}

}  // namespace

int xgmi_grid(const XgmiArgs& a) { return (a.chunk + a.sub - 1) / a.sub; }

void launch_xgmi_allreduce(const XgmiArgs& a, hipStream_t s) {
  const dim3 grid(xgmi_grid(a)), block(256);
  switch (a.mode == 1 ? a.opt.kind : -1) {
    case OPT_ADAM: hipLaunchKernelGGL(xgmi_allreduce_kernel<OPT_ADAM>, grid, block, 0, s, a); break;
    case OPT_NADAM: hipLaunchKernelGGL(xgmi_allreduce_kernel<OPT_NADAM>, grid, block, 0, s, a); break;
    case OPT_ADADELTA: hipLaunchKernelGGL(xgmi_allreduce_kernel<OPT_ADADELTA>, grid, block, 0, s, a); break;
    case OPT_RMSPROP: hipLaunchKernelGGL(xgmi_allreduce_kernel<OPT_RMSPROP>, grid, block, 0, s, a); break;
    default: hipLaunchKernelGGL(xgmi_allreduce_kernel<OPT_SGD>, grid, block, 0, s, a); break;
  }
}

// ---------------------------------------------------------------- host: memory + IPC
uintptr_t xgmi_alloc_uncached(size_t bytes, bool finegrained) {
  void* p = nullptr;
  if (hipExtMallocWithFlags(&p, bytes, finegrained ? hipDeviceMallocFinegrained : hipDeviceMallocUncached) !=
          hipSuccess || p == nullptr)
    throw std::runtime_error("hipExtMallocWithFlags(uncached/fine-grained) failed");
  if (hipMemset(p, 0, bytes) != hipSuccess) throw std::runtime_error("hipMemset failed");
  if (hipDeviceSynchronize() != hipSuccess) throw std::runtime_error("hipDeviceSynchronize failed");
  return reinterpret_cast<uintptr_t>(p);
}

void xgmi_free(uintptr_t p) { (void)hipFree(reinterpret_cast<void*>(p)); }

std::string xgmi_ipc_handle(uintptr_t p) {
  hipIpcMemHandle_t h;
  hipError_t e = hipIpcGetMemHandle(&h, reinterpret_cast<void*>(p));
  if (e != hipSuccess) throw std::runtime_error(std::string("hipIpcGetMemHandle: ") + hipGetErrorString(e));
  return std::string(reinterpret_cast<const char*>(&h), sizeof(h));
}

uintptr_t xgmi_ipc_open(const std::string& handle) {
  if (handle.size() != sizeof(hipIpcMemHandle_t)) throw std::invalid_argument("bad IPC handle size");
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle.data(), sizeof(h));
  void* p = nullptr;
  hipError_t e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
  if (e != hipSuccess) throw std::runtime_error(std::string("hipIpcOpenMemHandle: ") + hipGetErrorString(e));
  return reinterpret_cast<uintptr_t>(p);
}

void xgmi_ipc_close(uintptr_t p) { (void)hipIpcCloseMemHandle(reinterpret_cast<void*>(p)); }
