// Implicit-GEMM convolution on gfx950 MFMA (v_mfma_f32_16x16x32_bf16).
//
//   D[m][n] = sum_k A[m][k] * B[k][n]
//   m = output pixel (b, oy, ox)  -- or, with pooling, 4 pixels of one 2x2 window per
//                                   4 consecutive rows so the max-pool is register-local
//   k = (ky, kx, ci) im2col index, gathered on the fly from NHWC bf16 (16-B loads)
//   n = output channel
//
// One kernel serves:
//   K1/K2/K4  forward conv + bias + ReLU (+2x2 max-pool with argmax code) (+dropout)
//   K3        stride-2 forward (stride param)
//   K5        dgrad: conv of dY with the flipped/transposed pack (input dilation handles
//             strided layers), epilogue routed back through the previous stage's
//             dropout / ReLU / max-pool (bwd_through_store)
//   K9 (dX)   dense backward dX = dH * W^T as a 1x1 conv with a flattened epilogue
//
// Workgroup = 4 waves.  The WG's slice of the fragment-major weight pack (KS x NTC x 1 KiB)
// is staged into LDS once and reused by every m-tile the waves visit (grid-stride loop);
// A fragments go straight global -> VGPR (each lane's 8 k-values are 16 contiguous bytes
// of one NHWC pixel; neighbouring pixels/taps hit L1/L2).
#include "bwd_through.h"

template <int NTC, bool CS4>
__global__ __launch_bounds__(256) void conv_mm_kernel(const ConvMMArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int KS = a.KS;
  const int ntab = CS4 ? KS * 8 : KS * 4;   // 4-wide (CS4) or 8-wide k chunks
  int* tab = reinterpret_cast<int*>(smem);
  const int tab_bytes = (ntab * 4 + 15) & ~15;
  bf16* wl = reinterpret_cast<bf16*>(smem + tab_bytes);
  const int tid = threadIdx.x;
  const int nt0 = blockIdx.y * NTC;

  const int nfrag = KS * NTC * 64;
  for (int i = tid; i < nfrag; i += 256) {
    const int ks = i / (NTC * 64);
    const int rem = i - ks * NTC * 64;
    const int ntl = rem >> 6;
    const int ln = rem & 63;
    bf16x8 v = zero_bf16x8();
    if (nt0 + ntl < a.NT) v = load_bf16x8(a.wpk + ((size_t)(ks * a.NT + nt0 + ntl) * 64 + ln) * 8);
    *reinterpret_cast<bf16x8*>(wl + (size_t)i * 8) = v;
  }
  {
    const int KHW = a.KH * a.KW;
    const int cw = CS4 ? 4 : 8;
    for (int c = tid; c < ntab; c += 256) {
      const int k0 = c * cw;
      const int tap = k0 / a.Cs_in;
      const int ci = k0 - tap * a.Cs_in;
      int e = -1;
      if (tap < KHW) {
        const int ky = tap / a.KW;
        e = (ky << 26) | ((tap - ky * a.KW) << 20) | ci;
      }
      tab[c] = e;
    }
  }
  __syncthreads();

  const int wave = tid >> 6, lane = tid & 63, r = lane & 15, g = lane >> 4;
  const int HoWo = a.Ho * a.Wo;
  const int HpWp = a.Hp * a.Wp;
  const long long nrows = a.pool ? (long long)a.B * HpWp : (long long)a.B * HoWo;
  const long long ntiles = a.pool ? (nrows + 3) / 4 : (nrows + 15) / 16;
  const uint32_t step = a.st ? (uint32_t)a.st->t : 0u;
  const int dil = a.in_dil;

  for (long long tile = (long long)blockIdx.x * 4 + wave; tile < ntiles; tile += (long long)gridDim.x * 4) {
    int b, oy, ox;
    bool rv;
    if (a.pool) {
      const long long w = tile * 4 + (r >> 2);
      rv = w < nrows;
      const int wi = rv ? (int)w : 0;
      b = wi / HpWp;
      const int rem = wi - b * HpWp;
      const int py = rem / a.Wp;
      const int px = rem - py * a.Wp;
      oy = 2 * py + ((r >> 1) & 1);
      ox = 2 * px + (r & 1);
    } else {
      const long long m = tile * 16 + r;
      rv = m < nrows;
      const int mi = rv ? (int)m : 0;
      b = mi / HoWo;
      const int rem = mi - b * HoWo;
      oy = rem / a.Wo;
      ox = rem - oy * a.Wo;
    }
    const int iy0 = oy * a.stride - a.pad_t, ix0 = ox * a.stride - a.pad_l;
    const bf16* xb = a.x + (size_t)b * a.H * a.W * a.Cs_in;

    f32x4 acc[NTC];
#pragma unroll
    for (int nt = 0; nt < NTC; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll 2
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8 af = zero_bf16x8();
      if (rv) {
        if (!CS4) {
          const int e = tab[ks * 4 + g];
          if (e >= 0) {
            int iy = iy0 + (e >> 26), ix = ix0 + ((e >> 20) & 63);
            bool ok = true;
            if (dil > 1) {
              ok = (iy >= 0) && (ix >= 0) && (iy % dil == 0) && (ix % dil == 0);
              iy /= dil;
              ix /= dil;
            }
            ok = ok && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
            if (ok) af = load_bf16x8(xb + ((size_t)iy * a.W + ix) * a.Cs_in + (e & 0xFFFFF));
          }
        } else {
#pragma unroll
          for (int hh = 0; hh < 2; ++hh) {
            const int e = tab[(ks * 4 + g) * 2 + hh];
            if (e >= 0) {
              int iy = iy0 + (e >> 26), ix = ix0 + ((e >> 20) & 63);
              bool ok = true;
              if (dil > 1) {
                ok = (iy >= 0) && (ix >= 0) && (iy % dil == 0) && (ix % dil == 0);
                iy /= dil;
                ix /= dil;
              }
              ok = ok && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
              if (ok) {
                const bf16x4 v = load_bf16x4(xb + ((size_t)iy * a.W + ix) * a.Cs_in);
#pragma unroll
                for (int q = 0; q < 4; ++q) af[hh * 4 + q] = v[q];
              }
            }
          }
        }
      }
#pragma unroll
      for (int nt = 0; nt < NTC; ++nt) {
        const bf16x8 bfr = *reinterpret_cast<const bf16x8*>(wl + ((size_t)(ks * NTC + nt) * 64 + lane) * 8);
        acc[nt] = mfma16(af, bfr, acc[nt]);
      }
    }

    // ------------------------------------------------------------------ epilogues
    if (a.mode == 0) {
      if (a.pool) {
        const long long w = tile * 4 + g;
        if (w < nrows) {
#pragma unroll
          for (int nt = 0; nt < NTC; ++nt) {
            const int n = (nt0 + nt) * 16 + r;
            if (n < a.Cs_out) {
              float best = 0.f;
              int code = 0;
              if (n < a.N) {
                const float bv = a.bias ? a.bias[n] : 0.f;
                best = -3.4e38f;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                  float v = acc[nt][j] + bv;
                  if (a.relu) v = fmaxf(v, 0.f);
                  if (v > best) { best = v; code = j; }
                }
                if (a.drop_thr) {
                  const uint32_t idx = (uint32_t)(w * a.N + n);
                  best = dropout_keep(idx, a.seed, a.stream_id, step, a.drop_thr) ? best * a.drop_scale : 0.f;
                }
              }
              a.out[(size_t)w * a.Cs_out + n] = f2bf(best);
              a.code[(size_t)w * a.Cs_out + n] = (uint8_t)code;
            }
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const long long m = tile * 16 + g * 4 + j;
          if (m >= nrows) continue;
#pragma unroll
          for (int nt = 0; nt < NTC; ++nt) {
            const int n = (nt0 + nt) * 16 + r;
            if (n >= a.Cs_out) continue;
            float v = 0.f;
            if (n < a.N) {
              v = acc[nt][j] + (a.bias ? a.bias[n] : 0.f);
              if (a.relu) v = fmaxf(v, 0.f);
              if (a.drop_thr) {
                const uint32_t idx = (uint32_t)(m * a.N + n);
                v = dropout_keep(idx, a.seed, a.stream_id, step, a.drop_thr) ? v * a.drop_scale : 0.f;
              }
            }
            a.out[(size_t)m * a.Cs_out + n] = f2bf(v);
          }
        }
      }
    } else {
      const BwdThrough& t = a.bt;
      const int flat_w = t.pH * t.pW * t.pCs;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const long long m = tile * 16 + g * 4 + j;
        if (m >= nrows) continue;
#pragma unroll
        for (int nt = 0; nt < NTC; ++nt) {
          const int n = (nt0 + nt) * 16 + r;
          if (!a.flat_out) {
            const int mi = (int)m;
            const int bb = mi / HoWo;
            const int rem = mi - bb * HoWo;
            const int y = rem / a.Wo;
            bwd_through_store(t, bb, y, rem - y * a.Wo, n, acc[nt][j], step);
          } else {
            if (n >= flat_w) continue;
            const int y = n / (t.pW * t.pCs);
            const int rem = n - y * t.pW * t.pCs;
            const int x = rem / t.pCs;
            bwd_through_store(t, (int)m, y, x, rem - x * t.pCs, acc[nt][j], step);
          }
        }
      }
    }
  }
}

template <int NTC, bool CS4>
static void launch_t(const ConvMMArgs& a, int gx, int gy, size_t lds, hipStream_t s) {
  auto k = conv_mm_kernel<NTC, CS4>;
  if (lds > 65536) hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(k, dim3(gx, gy), dim3(256), lds, s, a);
}

size_t conv_mm_lds_bytes(const ConvMMArgs& a, int ntc, bool cs4) {
  const int ntab = cs4 ? a.KS * 8 : a.KS * 4;
  return (size_t)((ntab * 4 + 15) & ~15) + (size_t)a.KS * ntc * 64 * 16;
}

void launch_conv_mm(const ConvMMArgs& a, int ntc, int gx, hipStream_t s) {
  const bool cs4 = a.Cs_in == 4;
  const int gy = (a.NT + ntc - 1) / ntc;
  const size_t lds = conv_mm_lds_bytes(a, ntc, cs4);
#define CASE(N)                                        \
  case N:                                              \
    if (cs4) launch_t<N, true>(a, gx, gy, lds, s);     \
    else launch_t<N, false>(a, gx, gy, lds, s);        \
    break;
  switch (ntc) {
    CASE(1) CASE(2) CASE(4) CASE(8)
    default: break;
  }
#undef CASE
}
