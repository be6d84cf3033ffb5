// Shared definitions for the gfx950 (CDNA4 / MI355X) kernels of cori_intml_examples_amd.
//
// Conventions (see models/plan.py and models/executor_hip.py):
//   * activations are bf16 NHWC with a padded channel stride Cs (multiple of 8; the
//     network input uses Cs = 4): padded channels hold exact zeros;
//   * weights used by MFMA kernels are bf16 "fragment-major" packs produced by the
//     fused optimizer from the fp32 master copy:
//       pack[((ks * NT + nt) * 64 + lane) * 8 + j] = B[k = 32 ks + 8 (lane >> 4) + j]
//                                                     [n = 16 nt + (lane & 15)]
//     i.e. exactly the B-operand fragment of v_mfma_f32_16x16x32_bf16, so a wave
//     loads a whole fragment with one 16-byte access per lane;
//   * all waves are 64 lanes; workgroups are 256 threads (4 waves).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// v_mfma_f32_16x16x16_bf16: lane l holds A[l & 15][k = 4 (l >> 4) + j] / B[k][l & 15], j < 4
__device__ __forceinline__ f32x4 mfma16k16(const bf16x4& a, const bf16x4& b, const f32x4& c) {
  typedef short s16x4 __attribute__((ext_vector_type(4)));
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(s16x4, a), __builtin_bit_cast(s16x4, b), c,
                                                   0, 0, 0);
}

// 16-byte write-through store (vector buffer store, sc1): the line leaves the XCD's L2 with
// the store, so the launch's end-of-kernel release finds none of these bytes dirty (a
// boundary costs ~bytes / 6 TB/s behind a kernel that leaves its output dirty in L2).
// `base` must be wave-uniform; `off` is a byte offset < 2^31.
__device__ __forceinline__ void st_wt16(const void* base, unsigned off, u32x4 v) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 16);
}

__device__ __forceinline__ bf16x8 zero_bf16x8() {
  bf16x8 z;
#pragma unroll
  for (int i = 0; i < 8; ++i) z[i] = (bf16)0.0f;
  return z;
}

__device__ __forceinline__ bf16x8 load_bf16x8(const bf16* p) {
  return *reinterpret_cast<const bf16x8*>(p);
}

// Branch-free masked 16-byte load: always loads (from `safe` when !ok), then zeroes.
__device__ __forceinline__ bf16x8 load_bf16x8_if(bool ok, const bf16* p, const bf16* safe) {
  const uint4 raw = *reinterpret_cast<const uint4*>(ok ? p : safe);
  const uint4 z = {0u, 0u, 0u, 0u};
  const uint4 v = ok ? raw : z;
  return *reinterpret_cast<const bf16x8*>(&v);
}

__device__ __forceinline__ bf16x4 load_bf16x4_if(bool ok, const bf16* p, const bf16* safe) {
  const uint2 raw = *reinterpret_cast<const uint2*>(ok ? p : safe);
  const uint2 z = {0u, 0u};
  const uint2 v = ok ? raw : z;
  return *reinterpret_cast<const bf16x4*>(&v);
}

__device__ __forceinline__ bf16x4 load_bf16x4(const bf16* p) {
  return *reinterpret_cast<const bf16x4*>(p);
}

// Latency-batched staging loop: U independent global loads are issued before the first
// LDS store, so a thread keeps U requests in flight instead of serialising load->store
// round trips (the dominant cost of small, staging-bound kernels).
//   load(idx) -> V      store(idx, V)
// The load functor must be safe for any idx in [0, n) and branch-free (select on a
// validity flag after an unconditional load from a clamped address): a load under an
// `if` makes hipcc wait vmcnt(0) at every branch join, serialising the batch again.
template <int U, typename V, typename L, typename S>
__device__ __forceinline__ void staged_copy_u(int n, int tid, int nthreads, L load, S store) {
  for (int base = tid; base < n; base += nthreads * U) {
    V v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int idx = base + u * nthreads;
      v[u] = load(idx < n ? idx : n - 1);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int idx = base + u * nthreads;
      if (idx < n) store(idx, v[u]);
    }
  }
}

// Unroll depth matched to the work: a batch of U loads costs U address computations per
// thread even when most indices are clamped duplicates, so use the smallest U that still
// covers the range in one pass (uniform branch: n is the same for the whole workgroup).
template <int UMAX, typename V, typename L, typename S>
__device__ __forceinline__ void staged_copy(int n, int tid, int nthreads, L load, S store) {
  const int iters = (n + nthreads - 1) / nthreads;
  if (iters <= 1) staged_copy_u<1, V>(n, tid, nthreads, load, store);
  else if (iters <= 2) staged_copy_u<2, V>(n, tid, nthreads, load, store);
  else if (iters <= 4 || UMAX <= 4) staged_copy_u<(UMAX < 4 ? UMAX : 4), V>(n, tid, nthreads, load, store);
  else staged_copy_u<UMAX, V>(n, tid, nthreads, load, store);
}

// Fast division by a workgroup-uniform runtime divisor d (0 <= x < 2^22): float reciprocal
// estimate + one-step integer correction -- ~6 VALU instead of hipcc's ~30-instruction
// integer division sequence.
struct FastDiv {
  int d;
  float inv;
  __device__ __forceinline__ explicit FastDiv(int dd) : d(dd), inv(1.0f / (float)dd) {}
  __device__ __forceinline__ int div(int x) const {
    int q = (int)((float)x * inv);
    const int r = x - q * d;
    q += (r >= d) ? 1 : 0;
    q -= (r < 0) ? 1 : 0;
    return q;
  }
};

__device__ __forceinline__ float bf2f(bf16 v) { return (float)v; }
__device__ __forceinline__ bf16 f2bf(float v) { return (bf16)v; }

// ---------------------------------------------------------------------------------------
// Counter-based RNG (bit-identical twin of ops/rng.py)
__device__ __forceinline__ uint32_t fmix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x85EBCA6Bu;
  x ^= x >> 13;
  x *= 0xC2B2AE35u;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ uint32_t rng_u32(uint32_t idx, uint32_t seed, uint32_t stream, uint32_t step) {
  uint32_t x = idx ^ (step * 0x9E3779B9u);
  x = fmix32(x ^ seed);
  x = fmix32(x + stream * 0x85EBCA6Bu);
  return x;
}

// keep iff (u >> 8) >= thr ; scale = 1/(1-rate)
__device__ __forceinline__ bool dropout_keep(uint32_t idx, uint32_t seed, uint32_t stream, uint32_t step,
                                             uint32_t thr) {
  return (rng_u32(idx, seed, stream, step) >> 8) >= thr;
}

// ---------------------------------------------------------------------------------------
// Per-step device state, advanced by step_begin<<<1,64>>> at the head of each captured
// training step (race-free scalar bookkeeping: iteration counter, data cursor, LR and
// optimizer bias-correction scalars).
struct StepState {
  int t;          // optimizer iterations completed (Keras `iterations`)
  int pos;        // next data cursor
  int cur_pos;    // (unused; kept for the host-side field offsets)
  int eval_pos;   // cursor for eval / predict steps
  float lr;       // base learning rate (host-written)
  float lr_eff;   // lr after Keras `decay`
  float s[6];     // optimizer scalars for this step (meaning depends on optimizer kind)
  double m_schedule;  // Nadam running product
  // metric accumulators as int64 fixed point (loss in units of 2^-32, correct/count exact):
  // integer atomics commute, so the epoch sums are bit-identical whatever order the head's
  // workgroups retire in (a float/double atomicAdd is order-dependent in its last bits)
  long long metrics[4];  // (unused: see metric_slots)
  // bound dataset (host-written when the executor switches datasets, so captured graphs
  // are dataset-independent): x rows [n][R] bf16, targets [n][C] fp32, epoch permutation
  unsigned long long data_x, data_y, perm;
  int data_n, data_R, data_C, use_perm;
  // "the optimizer updated the master since the weight packs were last written"
  int packs_stale;
  int pad_;
  // device-side LR warmup (Goyal et al. gradual warmup, the Horovod warmup callback's
  // schedule): for 0-based step g = t - warm_t0 - 1 < warm_steps the base LR is
  //   warm_base / size * ((g + 1) / warm_spe * (size - 1) / warm_epochs + 1)
  // instead of the host-written `lr` -- so warmup needs no per-batch host write and runs
  // inside multi-step graph replays.  warm_steps = 0: off.
  int warm_t0, warm_steps, warm_spe, warm_size;
  float warm_base, warm_epochs;
  // metric accumulators spread over METRIC_SLOTS slots (workgroup b adds to slot b % 16):
  // [slot][loss_sum * 2^32, correct_sum, count, spare]; the host sums the slots
  long long metric_slots[16][4];
};

enum OptKind { OPT_SGD = 0, OPT_RMSPROP = 1, OPT_ADADELTA = 2, OPT_ADAM = 3, OPT_NADAM = 4 };

// ---------------------------------------------------------------------------------------
// Pack / unpack descriptors (fp32 master <-> bf16 fragment packs, grad slabs -> master layout)
enum PackType {
  PACK_CONV_FWD = 0,   // B[k=(tap,ci)][n=co] = W[ky][kx][ci][co]
  PACK_CONV_DGRAD = 1, // B[k=(tap',co)][n=ci] = W[KH-1-ky'][KW-1-kx'][ci][co]
  PACK_DENSE_FWD = 2,  // B[k=padded flat][n] = W[k_keras][n]
  PACK_DENSE_BWD = 3,  // B[k=n_dense][n=padded flat] = W[k_keras][k]
};

struct PackDesc {
  int src_off;   // offset of the tensor in the flat master buffer
  int numel;
  int type;
  int KH, KW, Cin, Cout;  // conv dims; dense: KH=Hf, KW=Wf (flatten source), Cin=Cf, Cout=N
  int Cs;        // padded channel stride of the relevant activation (fwd: input; dgrad: output)
  int NT;        // n-tiles of the pack
  int KS;        // 32-wide k-steps of the pack
  long long dst_off;  // element offset in the bf16 pack arena
  int blk0;      // first workgroup of this descriptor in the pack launch
  int nvec;      // 16-byte fragment vectors of the pack (KS * NT * 64)
};

#define MAX_PACK 24

// A dense layer's forward and backward packs, produced together from ONE read of the
// master by 32(k) x 128(n) tiles staged in LDS (dense_pack_kernel).
struct DensePair {
  int src_off;
  int KHW, Cin, Cs, N;     // flatten source grid (H*W), channels, padded channel stride, units
  int KS, NT;              // forward pack: 32-wide k-steps over the padded input, n-tiles over N
  int KSb, NTb;            // backward pack (0 if none): k-steps over N, n-tiles over padded input
  int ntn;                 // 128-column tiles
  int blk0;
  long long dst_fwd, dst_bwd;
};

#define MAX_DENSE_PAIRS 4

struct PackTable {
  int n;
  int nblocks;   // workgroups of the generic pack launch (256 vectors each)
  int nd;        // dense pairs
  int dblocks;   // workgroups of the dense pack launch
  PackDesc d[MAX_PACK];
  DensePair dp[MAX_DENSE_PAIRS];
};

// Dataset row of batch row b of this step: the cursor (training ? pos : eval_pos) + b,
// clamped BEFORE it indexes the permutation (perm holds data_n entries: a cursor run past the
// data set -- a launch replayed on its own, a caller's bad pos -- must not read past it).
__device__ __forceinline__ int step_src_pos(const StepState* st, int pos) {
  const int n = st->data_n;
  pos = min(max(pos, 0), max(n - 1, 0));
  const int* perm = reinterpret_cast<const int*>(st->perm);
  const int src = (st->use_perm && perm) ? perm[pos] : pos;
  return min(max(src, 0), n - 1);
}
__device__ __forceinline__ int step_src_row(const StepState* st, int training, int b) {
  return step_src_pos(st, (training ? st->pos : st->eval_pos) + b);
}

// Dense flatten mapping: keras flat index (h,w,c) over C channels -> padded index over Cs.
__device__ __forceinline__ int flat_keras_to_padded(int k, int C, int Cs) {
  int hw = k / C;
  int c = k - hw * C;
  return hw * Cs + c;
}
