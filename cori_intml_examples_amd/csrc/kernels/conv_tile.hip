// Tiled implicit-GEMM convolution for wide layers (Cs_in % 32 == 0, large K = KH*KW*Cs_in):
// the legacy RPV model (64..256 channels, Train_rpv.ipynb:205-219) and wide HPO trials.
//
// conv_halo keeps ALL of K's weights in LDS per workgroup, which forces a single 16-channel
// n-tile per workgroup once K is large (every A fragment then feeds one MFMA).  This kernel
// is a classic LDS-blocked GEMM over the whole batch instead:
//   * block tile 128 output rows (pixels over the batch, or 2x2 pool windows x 4 positions)
//     x BN = NTC*16 output channels, 256 threads = 2 x 2 waves, wave tile 64 x BN/2
//     (4 x NTC/2 MFMA 16x16x32 tiles: each A fragment feeds NTC/2 MFMAs, each B fragment 4);
//   * per 32-wide k-step (inside one tap, since Cs_in % 32 == 0) the block stages
//     A_s[128][32] (16 B per lane: 8 channels of one tap-shifted NHWC pixel; zero padding,
//     input dilation for strided dgrad and unpool-on-load from pooled dP + argmax codes are
//     resolved in the gather) and B_s = the fragment-major weight pack slice (1 KB per
//     n-tile, a straight copy) into a double-buffered LDS ring: the global loads of k-step
//     j+1 are in flight while the MFMAs of step j run, one barrier per k-step;
//   * A_s rows are padded to 40 elements so the ds_read_b128 fragment reads of 16 lanes on
//     16 different rows spread over the LDS banks.
// Epilogues are conv_halo's (mode 0: bias/ReLU/pool+argmax/dropout -> bf16 NHWC; mode 1:
// backward-through the previous stage), staged through LDS for 16-byte stores.
#include <type_traits>

#include "bwd_through.h"

namespace {
constexpr int BM = 128;         // rows per block
constexpr int LDA = 40;         // A_s row stride (elements): 32 + 8 pad
constexpr int KST = 2;          // k-steps per pipeline stage (one barrier per stage)
}

template <int NTC>
__global__ __launch_bounds__(256) void conv_tile_kernel(const ConvMMArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NW = NTC / 2;                         // n-tiles per wave
  constexpr int A_EL = BM * LDA;                      // A_s elements per k-step
  constexpr int B_EL = NTC * 64 * 8;                  // B_s elements per k-step
  constexpr int STG_EL = KST * (A_EL + B_EL);         // one LDS buffer = KST k-steps
  bf16* const lds = reinterpret_cast<bf16*>(smem);    // [2][KST][A] [KST][B]
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 15, g = lane >> 4;
  const int wm = wave & 1, wn = wave >> 1;
  const int nt0 = blockIdx.y * NTC;
  const int Cs = a.Cs_in, s = a.stride, dil = a.in_dil;
  const int cps = Cs >> 5;                            // k-steps per tap
  const bool pool = a.mode == 0 && a.pool;
  // Strided dgrad (input dilation dil > 1): output pixels are split into dil x dil parity
  // classes (grid.z); in a class only taps with (o - pad + k) % dil == 0 contribute, so the
  // K loop visits just those (~1/dil^2 of the dense-dilated work).
  const int cy = dil > 1 ? (int)blockIdx.z / dil : 0, cx = dil > 1 ? (int)blockIdx.z % dil : 0;
  const int Hc = dil > 1 ? (a.Ho - cy + dil - 1) / dil : a.Ho;
  const int Wc = dil > 1 ? (a.Wo - cx + dil - 1) / dil : a.Wo;
  const int ky0 = dil > 1 ? ((a.pad_t - cy) % dil + dil) % dil : 0;
  const int kx0 = dil > 1 ? ((a.pad_l - cx) % dil + dil) % dil : 0;
  const int nky = ky0 < a.KH ? (a.KH - ky0 + dil - 1) / dil : 0;
  const int nkx = kx0 < a.KW ? (a.KW - kx0 + dil - 1) / dil : 0;
  const int KS = nky * nkx * cps;                     // k-steps actually visited
  const long long nrows = pool ? (long long)a.B * a.Hp * a.Wp * 4 : (long long)a.B * Hc * Wc;
  const long long row0 = (long long)blockIdx.x * BM;
  if (row0 >= nrows) return;                          // (parity classes differ in size)
  const uint32_t step = a.st ? (uint32_t)a.st->t : 0u;
  const int IH = a.in_code ? a.in_pH : a.H, IW = a.in_code ? a.in_pW : a.W;

  auto row_coords = [&](long long rr, int& b, int& oy, int& ox) {
    if (pool) {
      const long long w = rr >> 2;
      const int q = (int)(rr & 3);
      const int hw = a.Hp * a.Wp;
      b = (int)(w / hw);
      const int rem = (int)(w - (long long)b * hw);
      const int py = rem / a.Wp, px = rem - py * a.Wp;
      oy = 2 * py + (q >> 1);
      ox = 2 * px + (q & 1);
    } else {
      const int hw = Hc * Wc;
      b = (int)(rr / hw);
      const int rem = (int)(rr - (long long)b * hw);
      const int i = rem / Wc, j = rem - i * Wc;
      oy = cy + i * dil;
      ox = cx + j * dil;
    }
  };

  // ---- this thread's two A-gather rows (128 rows x 4 chunks of 8 channels = 512 loads)
  const int ach = tid & 3;                            // 8-channel chunk of the k-step
  int gb[2], gy[2], gx[2];
  bool gv[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const long long row = row0 + (tid >> 2) + 64 * u;
    gv[u] = row < nrows;
    row_coords(gv[u] ? row : 0, gb[u], gy[u], gx[u]);
  }
  // k-step walker: tap (ty, tx) in the class's tap lattice, channel step cstep; per-row
  // input coordinates / validity are recomputed only when the tap changes.
  int wty = 0, wtx = 0, wcs = 0;
  int iyr[2], ixr[2];
  bool okr[2];
  const bf16* rowp[2];
  auto set_tap = [&]() {
    const int ky = ky0 + wty * dil, kx = kx0 + wtx * dil;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      int iy = gy[u] * s - a.pad_t + ky, ix = gx[u] * s - a.pad_l + kx;
      bool ok = gv[u] && iy >= 0 && ix >= 0;
      if (dil > 1) {          // exact: the class guarantees divisibility
        iy /= dil;
        ix /= dil;
      }
      ok = ok && iy < a.H && ix < a.W;
      iyr[u] = iy;
      ixr[u] = ix;
      okr[u] = ok;
      rowp[u] = ok ? a.x + (((size_t)gb[u] * a.H + iy) * a.W + ix) * Cs + 8 * ach : a.x;
    }
  };
  auto next_k = [&]() {
    if (++wcs == cps) {
      wcs = 0;
      if (++wtx == nkx) { wtx = 0; ++wty; }
      set_tap();
    }
  };
  auto pack_ks = [&]() { return ((ky0 + wty * dil) * a.KW + (kx0 + wtx * dil)) * cps + wcs; };
  auto load_a = [&](int u) -> bf16x8 {
    if (a.in_code) {
      const size_t boff = (size_t)gb[u] * IH * IW * Cs;
      return unpool_load8(a.x + boff, a.in_code + boff, IH, IW, Cs, iyr[u], ixr[u], wcs * 32 + 8 * ach, okr[u]);
    }
    return load_bf16x8_if(okr[u], rowp[u] + wcs * 32, a.x);
  };
  // ---- B gather: NTC*64 16-byte fragment vectors per k-step
  constexpr int BV = (NTC * 64 + 255) / 256;
  auto load_b = [&](int ksp, int u) -> bf16x8 {
    const int v = tid + 256 * u;
    const int nt = nt0 + (v >> 6);
    const bool ok = v < NTC * 64 && nt < a.NT;
    return load_bf16x8_if(ok, a.wpk + ((size_t)(ksp * a.NT + nt) * 64 + (v & 63)) * 8, a.wpk);
  };
  f32x4 acc[4][NW];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int n = 0; n < NW; ++n) acc[t][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  // One register stage (KST k-steps) in flight while the previous stage's MFMAs run out of
  // the other LDS buffer.  Loads are unconditional (past the last k-step the walker stays
  // put and the extra results are simply not used): a load under a branch would make
  // hipcc drain vmcnt at the join.
  bf16x8 ra[KST][2], rb[KST][BV];
  int kl = 0;                                         // k-steps issued so far
  auto issue_stage = [&]() {
#pragma unroll
    for (int kk = 0; kk < KST; ++kk) {
#pragma unroll
      for (int u = 0; u < 2; ++u) ra[kk][u] = load_a(u);
      const int kp = pack_ks();
#pragma unroll
      for (int u = 0; u < BV; ++u) rb[kk][u] = load_b(kp, u);
      if (++kl < KS) next_k();
    }
  };
  auto store_stage = [&](int buf) {
    bf16* base = lds + buf * STG_EL;
#pragma unroll
    for (int kk = 0; kk < KST; ++kk) {
#pragma unroll
      for (int u = 0; u < 2; ++u)
        *reinterpret_cast<bf16x8*>(base + kk * A_EL + ((tid >> 2) + 64 * u) * LDA + 8 * ach) = ra[kk][u];
#pragma unroll
      for (int u = 0; u < BV; ++u) {
        const int v = tid + 256 * u;
        if (v < NTC * 64) *reinterpret_cast<bf16x8*>(base + KST * A_EL + kk * B_EL + (size_t)v * 8) = rb[kk][u];
      }
    }
  };
  auto compute_stage = [&](int buf, int nvalid) {
    const bf16* base = lds + buf * STG_EL;
#pragma unroll
    for (int kk = 0; kk < KST; ++kk) {
      if (kk < nvalid) {                              // workgroup-uniform
        const bf16* A = base + kk * A_EL;
        const bf16* Bb = base + KST * A_EL + kk * B_EL;
        bf16x8 af[4], bfr[NW];
#pragma unroll
        for (int t = 0; t < 4; ++t)
          af[t] = *reinterpret_cast<const bf16x8*>(A + ((wm * 4 + t) * 16 + r) * LDA + 8 * g);
#pragma unroll
        for (int n = 0; n < NW; ++n)
          bfr[n] = *reinterpret_cast<const bf16x8*>(Bb + ((size_t)(wn * NW + n) * 64 + lane) * 8);
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int n = 0; n < NW; ++n) acc[t][n] = mfma16(af[t], bfr[n], acc[t][n]);
      }
    }
  };
  const int nst = (KS + KST - 1) / KST;
  if (KS > 0) {
    set_tap();
    issue_stage();
    store_stage(0);
  }
  __syncthreads();
  for (int st = 0; st < nst; ++st) {
    const int cur = st & 1;
    const bool more = st + 1 < nst;
    if (more) issue_stage();                          // next stage's loads fly during the MFMAs
    compute_stage(cur, KS - st * KST);
    if (more) store_stage(cur ^ 1);                   // other buffer: last read one stage ago
    __syncthreads();
  }

  // ---- epilogue through LDS scratch (per wave: [16 rows][NW*16] fp32)
  const int LDC = NW * 16;
  float* ep = reinterpret_cast<float*>(smem) + wave * 16 * LDC;
  const int cbase = (nt0 + wn * NW) * 16;              // first channel of this wave
  const int csh = (a.mode == 1 ? a.bt.pCs : a.Cs_out) - cbase;
  const int C = csh < LDC ? csh : LDC;
  const int cch = C > 0 ? C >> 3 : 0;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const long long tile = (row0 >> 4) + wm * 4 + t;  // global 16-row tile index
    if (tile * 16 >= nrows) break;
    if (pool) {
      bf16* epb = reinterpret_cast<bf16*>(ep);
      uint8_t* epc = reinterpret_cast<uint8_t*>(epb + 4 * LDC);
      const long long q = tile * 4 + g;               // global pool-window index
#pragma unroll
      for (int n = 0; n < NW; ++n) {
        const int ch = cbase + n * 16 + r;
        float best = 0.f;
        int code = 0;
        if (ch < a.N) {
          const float bv = a.bias ? a.bias[ch] : 0.f;
          best = -3.4e38f;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float v = acc[t][n][j] + bv;
            if (a.relu) v = fmaxf(v, 0.f);
            if (v > best) { best = v; code = j; }
          }
          if (a.drop_thr)
            best = dropout_keep((uint32_t)(q * a.N + ch), a.seed, a.stream_id, step, a.drop_thr) ? best * a.drop_scale
                                                                                                : 0.f;
        }
        epb[g * LDC + n * 16 + r] = f2bf(best);
        epc[g * LDC + n * 16 + r] = (uint8_t)code;
      }
      __builtin_amdgcn_wave_barrier();
      const long long nwin = nrows >> 2;
      const int nw = (int)min((long long)4, nwin - tile * 4);
      for (int c = lane; c < nw * cch; c += 64) {
        const int win = c / cch, c8 = c - win * cch;
        const size_t o = (size_t)(tile * 4 + win) * a.Cs_out + cbase + c8 * 8;
        *reinterpret_cast<uint4*>(a.out + o) = *reinterpret_cast<const uint4*>(epb + win * LDC + c8 * 8);
        *reinterpret_cast<uint2*>(a.code + o) = *reinterpret_cast<const uint2*>(epc + win * LDC + c8 * 8);
      }
      __builtin_amdgcn_wave_barrier();
    } else {
#pragma unroll
      for (int n = 0; n < NW; ++n)
#pragma unroll
        for (int j = 0; j < 4; ++j) ep[(g * 4 + j) * LDC + n * 16 + r] = acc[t][n][j];
      __builtin_amdgcn_wave_barrier();
      const int np = (int)min((long long)16, nrows - tile * 16);
      for (int c = lane; c < np * cch; c += 64) {
        const int pr = c / cch, c8 = c - pr * cch;
        size_t m = (size_t)(tile * 16 + pr);
        if (dil > 1) {                                // parity class row -> flat output pixel
          int b, oy, ox;
          row_coords((long long)m, b, oy, ox);
          m = ((size_t)b * a.Ho + oy) * a.Wo + ox;
        }
        float v[8];
        *reinterpret_cast<float4*>(v) = *reinterpret_cast<const float4*>(ep + pr * LDC + c8 * 8);
        *reinterpret_cast<float4*>(v + 4) = *reinterpret_cast<const float4*>(ep + pr * LDC + c8 * 8 + 4);
        const int n0 = cbase + c8 * 8;
        if (a.mode == 1) {
          bwd_through_store8(a.bt, m, n0, v, step);
        } else {
          bf16x8 o;
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const int n = n0 + k;
            float x = 0.f;
            if (n < a.N) {
              x = v[k] + (a.bias ? a.bias[n] : 0.f);
              if (a.relu) x = fmaxf(x, 0.f);
              if (a.drop_thr)
                x = dropout_keep((uint32_t)(m * a.N + n), a.seed, a.stream_id, step, a.drop_thr) ? x * a.drop_scale
                                                                                               : 0.f;
            }
            o[k] = f2bf(x);
          }
          *reinterpret_cast<bf16x8*>(a.out + m * a.Cs_out + n0) = o;
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
}

size_t conv_tile_lds_bytes(int ntc) {
  const size_t stage = (size_t)2 * KST * (BM * LDA + ntc * 64 * 8) * 2;
  const size_t ep = (size_t)4 * 16 * (ntc / 2) * 16 * 4;
  return stage > ep ? stage : ep;
}

template <int NTC>
static void launch_t(const ConvMMArgs& a, hipStream_t s) {
  const bool pool = a.mode == 0 && a.pool;
  const long long nrows = pool ? (long long)a.B * a.Hp * a.Wp * 4 : (long long)a.B * a.Ho * a.Wo;
  const int d = a.in_dil > 1 ? a.in_dil : 1;
  const long long maxrows = pool ? nrows : (long long)a.B * ((a.Ho + d - 1) / d) * ((a.Wo + d - 1) / d);
  const int gx = (int)((maxrows + BM - 1) / BM);
  const int gy = (a.NT + NTC - 1) / NTC;
  hipLaunchKernelGGL(conv_tile_kernel<NTC>, dim3(gx, gy, d * d), dim3(256), conv_tile_lds_bytes(NTC), s, a);
}

void launch_conv_tile(const ConvMMArgs& a, int ntc, hipStream_t s) {
  switch (ntc) {
    case 2: launch_t<2>(a, s); break;
    case 4: launch_t<4>(a, s); break;
    case 8: launch_t<8>(a, s); break;
    default: break;
  }
}
