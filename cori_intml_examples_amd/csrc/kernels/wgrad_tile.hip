// Tiled weight gradient for wide convolutions (Cs_in % 32 == 0):
//   dW[k = tap*Cs + c][n] = sum_p X[shift_tap(p)][c] * dY[p][n]      (+ db[n] = sum_p dY[p][n])
//
// wgrad_halo stages an image-row halo with ALL input channels per workgroup and lets each
// workgroup use only one 128-row slice of K, so wide layers re-stage the halo K/128 times.
// Here a workgroup owns a 128(k) x NTC*16(n) output tile and streams a contiguous pixel
// range (split-K over pixels, one fp32 slab per split, reduced in fixed order by
// slab_reduce -> deterministic).  Per stage of 64 pixels it gathers
//   A_s[64 px][128 k]  -- each 8-column chunk is 16 B of one tap-shifted NHWC pixel, and
//   B_s[64 px][NTC*16] -- dY rows, rebuilt from pooled dP + argmax codes when pooled,
// with one batch of independent 16-byte loads, then the four waves (2 x 2 over the tile)
// read MFMA fragments with ds_read_b64_tr_b16: the pixel (reduction) axis is the LDS row
// axis of both images, and the transposed read returns 8 consecutive pixels per lane.
// The bias gradient rides along as an extra m-tile whose A operand is all ones.
#include "bwd_through.h"

namespace {
constexpr int WT_PX = 64;     // pixels per stage (2 MFMA k-steps)
constexpr int WT_MK = 128;    // k rows per workgroup
}

__device__ __forceinline__ bf16x4 tr_read_t(const bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS_PTR(bf16x4, p));
}

template <int NTC>
__global__ __launch_bounds__(256) void wgrad_tile_kernel(const WgradArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int LDA = WT_MK + 8, LDB = NTC * 16 + 8;
  constexpr int NW = NTC / 2;                     // n-tiles per wave
  bf16* as = reinterpret_cast<bf16*>(smem);       // [WT_PX][LDA]
  bf16* bs = as + WT_PX * LDA;                    // [WT_PX][LDB]
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, i = lane & 15, g = lane >> 4;
  const int wm = wave & 1, wn = wave >> 1;
  const int k0 = blockIdx.y * WT_MK;
  const int nt0 = blockIdx.z * NTC;
  const int K = a.Ktiles * 16;
  const int Cs = a.Cs_in, s = a.stride;
  const bool do_bias = a.bslab != nullptr && blockIdx.y == 0 && wm == 0;
  const long long P = (long long)a.B * a.Ho * a.Wo;
  const long long p_begin = (long long)blockIdx.x * a.px_per_split;
  const long long p_end = min(P, p_begin + a.px_per_split);
  const int hw = a.Ho * a.Wo;

  f32x4 acc[4][NW], bacc[NW];
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int v = 0; v < NW; ++v) acc[u][v] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int v = 0; v < NW; ++v) bacc[v] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = f2bf(1.f);

  // this thread's fixed staging columns: A chunk column (k) and B chunk column (n)
  const int acol = (tid & 15) * 8;               // 16 chunks of 8 k per pixel row
  const int ka = k0 + acol;
  const int tapa = ka / Cs;
  const int ca = ka - tapa * Cs;
  const int kya = tapa / a.KW, kxa = tapa - kya * a.KW;
  const bool kok = ka < K && tapa < a.KH * a.KW;
  constexpr int BCH = NTC * 2;                    // 8-channel chunks per dY row
  const int bcol = (tid % BCH) * 8;
  const int nb0 = nt0 * 16 + bcol;
  const bool nok = nb0 < a.Cs_dy;

  // Pixel coordinates of this thread's staging rows, advanced incrementally by WT_PX per
  // stage (no integer division in the loop: the gather would otherwise be VALU-bound).
  constexpr int AR = WT_PX * 16 / 256;            // A rows per thread (4)
  constexpr int BR = WT_PX * BCH / 256;           // B rows per thread (NTC/2)
  const int adv_y = WT_PX / a.Wo, adv_x = WT_PX - (WT_PX / a.Wo) * a.Wo;
  int ab[AR], ay[AR], ax[AR], bb[BR], by[BR], bx[BR];
  auto decompose = [&](long long p, int& b, int& y, int& x) {
    const long long pc = p < P ? p : P - 1;
    b = (int)(pc / hw);
    const int rem = (int)(pc - (long long)b * hw);
    y = rem / a.Wo;
    x = rem - y * a.Wo;
  };
  auto advance = [&](int& b, int& y, int& x) {
    x += adv_x;
    y += adv_y;
    if (x >= a.Wo) { x -= a.Wo; ++y; }
    while (y >= a.Ho) { y -= a.Ho; ++b; }
  };
#pragma unroll
  for (int u = 0; u < AR; ++u) decompose(p_begin + (tid >> 4) + 16 * u, ab[u], ay[u], ax[u]);
#pragma unroll
  for (int u = 0; u < BR; ++u) decompose(p_begin + tid / BCH + (256 / BCH) * u, bb[u], by[u], bx[u]);

  // Two LDS buffers: stage j+1's gather loads are issued before stage j's MFMAs and written
  // to the other buffer after them (one barrier per stage).
  constexpr int STG = WT_PX * (LDA + LDB);        // elements per buffer
  bf16x8 va[AR], vb[BR];
  auto gather = [&](long long pb) {
#pragma unroll
    for (int u = 0; u < AR; ++u) {
      const bool pv = pb + (tid >> 4) + 16 * u < p_end && ab[u] < a.B;
      const int iy = ay[u] * s - a.pad_t + kya, ix = ax[u] * s - a.pad_l + kxa;
      const bool ok = pv && kok && iy >= 0 && ix >= 0 && iy < a.H && ix < a.W;
      va[u] = load_bf16x8_if(ok, a.x + (((size_t)ab[u] * a.H + iy) * a.W + ix) * Cs + ca, a.x);
    }
#pragma unroll
    for (int u = 0; u < BR; ++u) {
      const bool pv = pb + tid / BCH + (256 / BCH) * u < p_end && bb[u] < a.B && nok;
      const int b = pv ? bb[u] : 0;
      if (a.dy_code) {
        const size_t boff = (size_t)b * a.dHp * a.dWp * a.Cs_dy;
        vb[u] = unpool_load8(a.dy + boff, a.dy_code + boff, a.dHp, a.dWp, a.Cs_dy, by[u], bx[u], nb0, pv);
      } else {
        vb[u] = load_bf16x8_if(pv, a.dy + (((size_t)b * a.Ho + by[u]) * a.Wo + bx[u]) * a.Cs_dy + nb0, a.dy);
      }
    }
#pragma unroll
    for (int u = 0; u < AR; ++u) advance(ab[u], ay[u], ax[u]);
#pragma unroll
    for (int u = 0; u < BR; ++u) advance(bb[u], by[u], bx[u]);
  };
  auto stash = [&](int buf) {
    bf16* as_ = as + buf * STG;
    bf16* bs_ = as_ + WT_PX * LDA;
#pragma unroll
    for (int u = 0; u < AR; ++u)
      *reinterpret_cast<bf16x8*>(as_ + ((tid >> 4) + 16 * u) * LDA + acol) = va[u];
#pragma unroll
    for (int u = 0; u < BR; ++u)
      *reinterpret_cast<bf16x8*>(bs_ + (tid / BCH + (256 / BCH) * u) * LDB + bcol) = vb[u];
  };
  auto mma = [&](int buf) {
    const bf16* as_ = as + buf * STG;
    const bf16* bs_ = as_ + WT_PX * LDA;
#pragma unroll
    for (int ks = 0; ks < WT_PX / 32; ++ks) {
      const int P0 = ks * 32 + 8 * g + (i >> 2);
      bf16x8 af[4], bfr[NW];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const bf16* pa = as_ + P0 * LDA + (wm * 4 + u) * 16 + 4 * (i & 3);
        af[u] = __builtin_shufflevector(tr_read_t(pa), tr_read_t(pa + 4 * LDA), 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int v = 0; v < NW; ++v) {
        const bf16* pbp = bs_ + P0 * LDB + (wn * NW + v) * 16 + 4 * (i & 3);
        bfr[v] = __builtin_shufflevector(tr_read_t(pbp), tr_read_t(pbp + 4 * LDB), 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < NW; ++v) acc[u][v] = mfma16(af[u], bfr[v], acc[u][v]);
      if (do_bias) {
#pragma unroll
        for (int v = 0; v < NW; ++v) bacc[v] = mfma16(ones, bfr[v], bacc[v]);
      }
    }
  };
  const int nstage = (int)((p_end - p_begin + WT_PX - 1) / WT_PX);
  if constexpr (NTC <= 4) {          // registers to spare: software-pipelined
    if (nstage > 0) {
      gather(p_begin);
      stash(0);
    }
    __syncthreads();
    for (int st = 0; st < nstage; ++st) {
      const bool more = st + 1 < nstage;
      if (more) gather(p_begin + (long long)(st + 1) * WT_PX);
      mma(st & 1);
      if (more) stash((st & 1) ^ 1);
      __syncthreads();
    }
  } else {                           // 128x128 tile: the prefetch registers would halve occupancy
    for (int st = 0; st < nstage; ++st) {
      gather(p_begin + (long long)st * WT_PX);
      stash(0);
      __syncthreads();
      mma(0);
      __syncthreads();
    }
  }

  // ---- partial slab of this split
  const int ld = a.NT * 16;
  float* slab = a.slab + (size_t)blockIdx.x * K * ld;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int kr = k0 + (wm * 4 + u) * 16 + g * 4;
#pragma unroll
    for (int v = 0; v < NW; ++v) {
      const int n = (nt0 + wn * NW + v) * 16 + i;
      if (n >= ld) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (kr + j < K) slab[(size_t)(kr + j) * ld + n] = acc[u][v][j];
    }
  }
  if (do_bias && g == 0) {
#pragma unroll
    for (int v = 0; v < NW; ++v) {
      const int n = (nt0 + wn * NW + v) * 16 + i;
      if (n < ld) a.bslab[(size_t)blockIdx.x * ld + n] = bacc[v][0];
    }
  }
}

// ------------------------------------------------------------------------------------------
// LDS-DMA path (NTC == 8, unpooled dY): A_s and B_s are [64 px][128] bf16 images with
// 256-B rows filled by global_load_lds_dwordx4 (4 + 4 wave-instructions per wave per stage,
// no VGPR staging, no ds_write), double-buffered with the DMA of stage j+1 in flight during
// stage j's MFMAs.  The DMA destination is lane-linear, so the conflict-avoiding layout is
// produced on the source side: the 16-B chunk c of row R sits at position c ^ h(R),
// h(R) = 2 * ((R & 3) | ((R >> 3) & 1) << 2), which spreads each 32-lane group of a
// ds_read_b64_tr_b16 fragment read (rows 8g + i/4 and 8g + i/4 + 4 share h) over all 64
// banks.  Padding (outside the image, k >= K, n >= Cs_dy, pixels past the split) reads a
// zero buffer.
namespace {
__device__ __forceinline__ int wg_swz(int R) { return ((R & 3) | (((R >> 3) & 1) << 2)) << 1; }
}

// ROWAL: 64 % Wo == 0 and Ho*Wo % 64 == 0 (every legacy / wide layer): a stage is whole
// output rows of ONE image, so each DMA slot's pixel is a lane-constant offset (row, column)
// from a wave-uniform stage base -- the per-stage address math is a few adds and compares
// instead of 64-bit multiply chains (PMC: VALU:MFMA 9.6 and ~250 VALU per 40 MFMAs, mostly
// v_mul_lo / v_mad_u64 at quarter rate, made the generic path VALU-bound).
template <bool ROWAL>
__global__ __launch_bounds__(256) void wgrad_gl_kernel(const WgradArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NTC = 8, NW = 4;
  constexpr int ROWB = 256;                       // bytes per pixel row of either image
  constexpr int IMG = WT_PX * ROWB;               // 16 KB
  constexpr int STG = 2 * IMG;                    // A + B per stage
  const int tid = threadIdx.x, lane = tid & 63, i = lane & 15, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (scalar branches)
  const int wm = wave & 1, wn = wave >> 1;
  const int k0 = blockIdx.y * WT_MK;
  const int nt0 = blockIdx.z * NTC;
  const int K = a.Ktiles * 16;
  const int Cs = a.Cs_in, s = a.stride;
  const bool do_bias = a.bslab != nullptr && blockIdx.y == 0 && wm == 0;
  const long long P = (long long)a.B * a.Ho * a.Wo;
  const long long p_begin = (long long)blockIdx.x * a.px_per_split;
  const long long p_end = min(P, p_begin + a.px_per_split);
  const int hw = a.Ho * a.Wo;
  const bf16* zero = a.zero;

  // this lane's DMA slots, u = 0..3: row R = 16*wave + 4u + g, position i -> source chunk
  // c = i ^ h(R); per u the chunk's (tap, channel) for A and channel for B are fixed.
  int tky[4], tkx[4], tch[4], bn[4];
  bool tok[4], bok[4];
  long long pb_[4];
  int pbb[4], pby[4], pbx[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int R = 16 * wave + 4 * u + g;
    const int c = i ^ wg_swz(R);
    const int k = k0 + 8 * c;
    const int tap = k / Cs;
    tok[u] = k < K && tap < a.KH * a.KW;
    tky[u] = tap / a.KW;
    tkx[u] = tap - tky[u] * a.KW;
    tch[u] = k - tap * Cs;
    bn[u] = nt0 * 16 + 8 * c;
    bok[u] = bn[u] < a.Cs_dy;
    pb_[u] = p_begin + R;
    const long long pc = pb_[u] < P ? pb_[u] : P - 1;
    pbb[u] = (int)(pc / hw);
    const int rem = (int)(pc - (long long)pbb[u] * hw);
    pby[u] = rem / a.Wo;
    pbx[u] = rem - pby[u] * a.Wo;
  }
  const int adv_y = WT_PX / a.Wo, adv_x = WT_PX - (WT_PX / a.Wo) * a.Wo;
  // ROWAL lane constants: slot u's source offsets from the stage's (image, first row) base
  int offA[4], rowA[4], offB[4];
  bool colA[4];
  long long sp = p_begin;                         // stage's first pixel (wave-uniform)
  int sb = 0, sy = 0;                             // its image and output row
  if (ROWAL) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int R = 16 * wave + 4 * u + g;
      const int dyl = R / a.Wo, xl = R - dyl * a.Wo;
      rowA[u] = dyl * s - a.pad_t + tky[u];
      const int ix = xl * s - a.pad_l + tkx[u];
      colA[u] = tok[u] && ix >= 0 && ix < a.W;
      offA[u] = (rowA[u] * a.W + ix) * Cs + tch[u];
      offB[u] = R * a.Cs_dy + bn[u];
    }
    sb = (int)(p_begin / hw);
    sy = (int)(p_begin - (long long)sb * hw) / a.Wo;
  }

  auto issue = [&](int buf) {
    char* as_ = smem + buf * STG;
    char* bs_ = as_ + IMG;
    if (ROWAL) {
      const int left = (int)min((long long)WT_PX, p_end - sp);      // valid pixels of the stage
      const bf16* xb = a.x + ((size_t)sb * a.H + (size_t)sy * s) * a.W * Cs;
      const bf16* yb = a.dy + (size_t)sp * a.Cs_dy;
      const int ys = sy * s;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int R = 16 * wave + 4 * u + g;
        const int iy = ys + rowA[u];
        const bool ok = R < left && colA[u] && iy >= 0 && iy < a.H;
        __builtin_amdgcn_global_load_lds(ok ? xb + offA[u] : zero, as_ + (16 * wave + 4 * u) * ROWB, 16, 0, 0);
        __builtin_amdgcn_global_load_lds(R < left && bok[u] ? yb + offB[u] : zero, bs_ + (16 * wave + 4 * u) * ROWB,
                                         16, 0, 0);
      }
      sp += WT_PX;
      sy += adv_y;
      if (sy >= a.Ho) { sy -= a.Ho; ++sb; }
      return;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool pv = pb_[u] < p_end;
      const int iy = pby[u] * s - a.pad_t + tky[u], ix = pbx[u] * s - a.pad_l + tkx[u];
      const bool ok = pv && tok[u] && iy >= 0 && ix >= 0 && iy < a.H && ix < a.W;
      const bf16* srca = ok ? a.x + (((size_t)pbb[u] * a.H + iy) * a.W + ix) * Cs + tch[u] : zero;
      __builtin_amdgcn_global_load_lds(srca, as_ + (16 * wave + 4 * u) * ROWB, 16, 0, 0);
      const bf16* srcb = pv && bok[u] ? a.dy + (size_t)pb_[u] * a.Cs_dy + bn[u] : zero;
      __builtin_amdgcn_global_load_lds(srcb, bs_ + (16 * wave + 4 * u) * ROWB, 16, 0, 0);
      // advance this slot's pixel by one stage
      pb_[u] += WT_PX;
      pbx[u] += adv_x;
      pby[u] += adv_y;
      if (pbx[u] >= a.Wo) { pbx[u] -= a.Wo; ++pby[u]; }
      while (pby[u] >= a.Ho) { pby[u] -= a.Ho; ++pbb[u]; }
    }
  };

  f32x4 acc[4][NW], bacc[NW];
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int v = 0; v < NW; ++v) acc[u][v] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int v = 0; v < NW; ++v) bacc[v] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = f2bf(1.f);

  // fragment read addresses: rows P0 = 32ks + 8g + i/4 and P0 + 4 (same swizzle), element
  // column 16*tile + 4*(i&3) -> chunk 2*tile + ((i&3)>>1), 8-B half (i&1)
  auto tr_frag = [&](const char* img, int P0, int tile) -> bf16x8 {
    const int pos = (2 * tile + ((i & 3) >> 1)) ^ wg_swz(P0);
    const bf16* p0 = reinterpret_cast<const bf16*>(img + P0 * ROWB + pos * 16 + (i & 1) * 8);
    const bf16* p1 = reinterpret_cast<const bf16*>(img + (P0 + 4) * ROWB + pos * 16 + (i & 1) * 8);
    return __builtin_shufflevector(tr_read_t(p0), tr_read_t(p1), 0, 1, 2, 3, 4, 5, 6, 7);
  };
  auto mma = [&](int buf) {
    const char* as_ = smem + buf * STG;
    const char* bs_ = as_ + IMG;
#pragma unroll
    for (int ks = 0; ks < WT_PX / 32; ++ks) {
      const int P0 = ks * 32 + 8 * g + (i >> 2);
      bf16x8 af[4], bfr[NW];
#pragma unroll
      for (int u = 0; u < 4; ++u) af[u] = tr_frag(as_, P0, wm * 4 + u);
#pragma unroll
      for (int v = 0; v < NW; ++v) bfr[v] = tr_frag(bs_, P0, wn * NW + v);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < NW; ++v) acc[u][v] = mfma16(af[u], bfr[v], acc[u][v]);
      if (do_bias) {
#pragma unroll
        for (int v = 0; v < NW; ++v) bacc[v] = mfma16(ones, bfr[v], bacc[v]);
      }
    }
  };
  const int nstage = (int)((p_end - p_begin + WT_PX - 1) / WT_PX);
  if (nstage > 0) issue(0);
  __syncthreads();
  for (int st = 0; st < nstage; ++st) {
    if (st + 1 < nstage) issue((st & 1) ^ 1);      // buffer last read in stage st-1
    mma(st & 1);
    __syncthreads();                                // vmcnt(0): stage st+1 has landed
  }

  const int ld = a.NT * 16;
  float* slab = a.slab + (size_t)blockIdx.x * K * ld;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int kr = k0 + (wm * 4 + u) * 16 + g * 4;
#pragma unroll
    for (int v = 0; v < NW; ++v) {
      const int n = (nt0 + wn * NW + v) * 16 + i;
      if (n >= ld) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (kr + j < K) slab[(size_t)(kr + j) * ld + n] = acc[u][v][j];
    }
  }
  if (do_bias && g == 0) {
#pragma unroll
    for (int v = 0; v < NW; ++v) {
      const int n = (nt0 + wn * NW + v) * 16 + i;
      if (n < ld) a.bslab[(size_t)blockIdx.x * ld + n] = bacc[v][0];
    }
  }
}

static size_t wgrad_gl_lds_bytes() { return (size_t)2 * 2 * WT_PX * 256; }

size_t wgrad_tile_lds_bytes(int ntc) {
  return (size_t)2 * WT_PX * ((WT_MK + 8) + (ntc * 16 + 8)) * 2;
}

template <int NTC>
static void launch_wt(const WgradArgs& a, hipStream_t s) {
  const long long P = (long long)a.B * a.Ho * a.Wo;
  const int S = (int)((P + a.px_per_split - 1) / a.px_per_split);
  const int gy = (a.Ktiles * 16 + WT_MK - 1) / WT_MK;
  const int gz = (a.NT + NTC - 1) / NTC;
  if (NTC == 8 && a.zero != nullptr && a.dy_code == nullptr) {
    const bool rowal = a.Wo > 0 && WT_PX % a.Wo == 0 && (a.Ho * a.Wo) % WT_PX == 0 && a.px_per_split % WT_PX == 0;
    if (rowal) hipLaunchKernelGGL(wgrad_gl_kernel<true>, dim3(S, gy, gz), dim3(256), wgrad_gl_lds_bytes(), s, a);
    else hipLaunchKernelGGL(wgrad_gl_kernel<false>, dim3(S, gy, gz), dim3(256), wgrad_gl_lds_bytes(), s, a);
  }
  else
    hipLaunchKernelGGL(wgrad_tile_kernel<NTC>, dim3(S, gy, gz), dim3(256), wgrad_tile_lds_bytes(NTC), s, a);
}

void launch_wgrad_tile(const WgradArgs& a, int ntc, hipStream_t s) {
  switch (ntc) {
    case 2: launch_wt<2>(a, s); break;
    case 4: launch_wt<4>(a, s); break;
    case 8: launch_wt<8>(a, s); break;
    default: break;
  }
}
