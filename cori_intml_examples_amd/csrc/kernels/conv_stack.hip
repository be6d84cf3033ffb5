// Layer-fused forward of a whole conv stack (gfx950 MFMA 16x16x32 bf16): a workgroup runs
// every Conv2D(+bias +ReLU +2x2 max-pool +dropout) stage of the network for one row band of
// one image, with the activations resident in LDS.
//
// Why: at the reference batch (128) a per-layer conv launch is pure latency -- ~1 GFLOP of
// MFMA work spread over 512 workgroups finishes in < 1 us of math but costs 13-15 us of
// launch ramp, global staging and drain, three times per forward.  The per-image working
// set of the small CNNs this framework targets (RPV: 64x64x3 -> 32x32x16 -> 16x16x32 ->
// 8x8x64; MNIST: 28x28x1 -> 26x26x32 -> 12x12x64) fits the 160 KB LDS of a CDNA4 CU, so
// the stack runs as a single launch: the image band is staged once (zero halo included),
// each layer's output tile is written by the MFMA epilogue straight into the NEXT layer's
// zero-padded halo image in LDS, and only the stage outputs the backward pass and the
// dense layer need (pooled activations + argmax codes) are streamed to global memory with
// 16-byte stores.
//
// Grid = B x splits: workgroup (b, sp) OWNS stage-output rows [own0, own1) of every layer
// (a partition over the splits) and computes conv rows [c0, c1): its owned rows plus the
// halo rows the next layer's range needs (host-computed, ConvStackArgs::rows).  With two
// bands per image the batch-128 launch fills all 256 CUs for ~35% recomputed conv1 rows.
//
// Per layer (8 waves): m-tiles are 16 output pixels (or 4 pooling windows x 4 positions,
// so the 2x2 max-pool is register-local: an MFMA accumulator row group is one window),
// TM m-tiles x NT n-tiles per wave; A fragments are one ds_read_b128 per k-step from the
// halo image (two ds_read_b64 for the 4-channel input), B fragments come from the layer's
// fragment-major weight pack staged in LDS at kernel start.  All LDS traffic goes through
// address-space-3 pointers with 32-bit offsets (generic pointers would turn every access
// into FLAT instructions with 64-bit address math: the epilogue was VALU-bound on that).
// Numerics (bf16 rounding points, dropout counters, argmax codes) are identical to the
// per-layer kernels.
#include "args.h"

#define STACK_THREADS 512
#define STACK_WAVES (STACK_THREADS / 64)
#define LDS __attribute__((address_space(3)))

typedef LDS bf16 lbf16;

// One layer over the workgroup's conv-output rows [c0, c1).  Local conv row y reads rows
// y + roff + ky of the input halo image `in`; stage output row py lands in row py - obase
// of `outimg` (skipped outside [0, OH)); codes are kept for the local stage rows.
template <int NT, int TM, bool CS4>
__device__ __forceinline__ void stack_layer(const ConvStackArgs& A, const StackLayer& L, int b, int c0, int c1,
                                            int roff, const lbf16* in, lbf16* outimg, int obase, int OH, int ol,
                                            int OW, LDS uint8_t* codes, const lbf16* wl, const LDS int* tab,
                                            const lbf16* zl, uint32_t step) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 15, g = lane >> 4;
  const int Wi = L.Wo + L.KW - 1;
  const int Cs = L.Cs_in, Cso = L.Cs_out, Cout = L.Cout, Wp = L.Wp, Wo = L.Wo, KS = L.KS;
  const int Hc = c1 - c0;                       // local conv rows (even when pooled)
  const int p0 = L.pool ? c0 >> 1 : c0;         // first local stage row (global index)
  const bool pool = L.pool, relu = L.relu;
  const uint32_t thr = L.drop_thr, sid = L.stream_id, seed = A.seed;
  const float dscale = L.drop_scale;
  const int nwin = pool ? (Hc >> 1) * Wp : 0;
  const int npix = Hc * Wo;
  const int ntiles = pool ? (nwin + 3) >> 2 : (npix + 15) >> 4;
  const FastDiv fwp(Wp > 0 ? Wp : 1), fwo(Wo);
  // dropout counter bases (uint32 wrap-around == the per-layer kernels' truncated index)
  const uint32_t qb = (uint32_t)(b * L.Hp + p0) * (uint32_t)Wp;     // pooled: window index base
  const uint32_t mb = (uint32_t)(b * L.Ho + c0) * (uint32_t)Wo;     // unpooled: pixel index base
  float bias[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int n = nt * 16 + r;
    bias[nt] = (L.bias && n < Cout) ? L.bias[n] : 0.f;
  }
  for (int tb = wave * TM; tb < ntiles; tb += STACK_WAVES * TM) {
    bool rv[TM];
    int xo[TM];                                   // element offset of the lane's pixel row
#pragma unroll
    for (int t = 0; t < TM; ++t) {
      const int tile = tb + t;
      int ry, rx;
      if (pool) {
        const int w = tile * 4 + (r >> 2);
        rv[t] = w < nwin;
        const int wi = rv[t] ? w : 0;
        const int pyl = fwp.div(wi);
        ry = 2 * pyl + ((r >> 1) & 1);
        rx = 2 * (wi - pyl * Wp) + (r & 1);
      } else {
        const int p = tile * 16 + r;
        rv[t] = p < npix;
        const int pi = rv[t] ? p : 0;
        ry = fwo.div(pi);
        rx = pi - ry * Wo;
      }
      xo[t] = ((ry + roff) * Wi + rx) * Cs;
    }
    f32x4 acc[TM][NT];
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[t][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int KSr = (A.dbg & 1) ? 0 : KS;
#pragma unroll 3
    for (int ks = 0; ks < KSr; ++ks) {
      bf16x8 af[TM];
      if (CS4) {
        const int e0 = tab[(ks * 4 + g) * 2], e1 = tab[(ks * 4 + g) * 2 + 1];
#pragma unroll
        for (int t = 0; t < TM; ++t) {
          const bf16x4 v0 = *reinterpret_cast<const LDS bf16x4*>((rv[t] && e0 >= 0) ? in + xo[t] + e0 : zl);
          const bf16x4 v1 = *reinterpret_cast<const LDS bf16x4*>((rv[t] && e1 >= 0) ? in + xo[t] + e1 : zl);
          af[t] = __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
        }
      } else {
        const int e0 = tab[ks * 4 + g];
#pragma unroll
        for (int t = 0; t < TM; ++t)
          af[t] = *reinterpret_cast<const LDS bf16x8*>((rv[t] && e0 >= 0) ? in + xo[t] + e0 : zl);
      }
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const bf16x8 bfr = *reinterpret_cast<const LDS bf16x8*>(wl + ((ks * NT + nt) * 64 + lane) * 8);
#pragma unroll
        for (int t = 0; t < TM; ++t) acc[t][nt] = mfma16(af[t], bfr, acc[t][nt]);
      }
    }
    if (A.dbg & 2) {
#pragma unroll
      for (int t = 0; t < TM; ++t)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          asm volatile("" ::"v"(acc[t][nt][0]), "v"(acc[t][nt][1]), "v"(acc[t][nt][2]), "v"(acc[t][nt][3]));
      continue;
    }
    // epilogue: straight into the next layer's halo image (and the code plane)
    if (pool) {
#pragma unroll
      for (int t = 0; t < TM; ++t) {
        const int w = (tb + t) * 4 + g;
        if (w >= nwin) continue;
        const int pyl = fwp.div(w), pxl = w - pyl * Wp;
        const int orow = p0 + pyl - obase;
        const bool keep = orow >= 0 && orow < OH;
        const int oo = (orow * OW + pxl + ol) * Cso, co = (pyl * Wp + pxl) * Cso;
        const uint32_t qi = (qb + (uint32_t)w) * (uint32_t)Cout;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const int n = nt * 16 + r;
          if (n >= Cso) continue;
          float best = 0.f;
          int code = 0;
          if (n < Cout) {     // padded channels: value 0 (pre-zeroed image), code 0
            best = -3.4e38f;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              float v = acc[t][nt][j] + bias[nt];
              if (relu) v = fmaxf(v, 0.f);
              if (v > best) { best = v; code = j; }
            }
            if (thr) best = dropout_keep(qi + (uint32_t)n, seed, sid, step, thr) ? best * dscale : 0.f;
            if (keep) outimg[oo + n] = f2bf(best);
          }
          codes[co + n] = (uint8_t)code;
        }
      }
    } else {
#pragma unroll
      for (int t = 0; t < TM; ++t) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int p = (tb + t) * 16 + g * 4 + j;
          if (p >= npix) continue;
          const int yl = fwo.div(p), x = p - yl * Wo;
          const int orow = c0 + yl - obase;
          if (orow < 0 || orow >= OH) continue;
          const int oo = (orow * OW + x + ol) * Cso;
          const uint32_t mi = (mb + (uint32_t)p) * (uint32_t)Cout;
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) {
            const int n = nt * 16 + r;
            if (n >= Cout) continue;
            float v = acc[t][nt][j] + bias[nt];
            if (relu) v = fmaxf(v, 0.f);
            if (thr) v = dropout_keep(mi + (uint32_t)n, seed, sid, step, thr) ? v * dscale : 0.f;
            outimg[oo + n] = f2bf(v);
          }
        }
      }
    }
  }
}

template <int NT, bool CS4>
__device__ __forceinline__ void stack_layer_tm(const ConvStackArgs& A, const StackLayer& L, int b, int c0, int c1,
                                               int roff, const lbf16* in, lbf16* outimg, int obase, int OH, int ol,
                                               int OW, LDS uint8_t* codes, const lbf16* wl, const LDS int* tab,
                                               const lbf16* zl, uint32_t step) {
  constexpr int TM = NT >= 2 ? 2 : 4;
  stack_layer<NT, TM, CS4>(A, L, b, c0, c1, roff, in, outimg, obase, OH, ol, OW, codes, wl, tab, zl, step);
}

__global__ __launch_bounds__(STACK_THREADS) void conv_stack_fwd_kernel(const ConvStackArgs A) {
  extern __shared__ __attribute__((aligned(16))) char smem_[];
  LDS char* smem = (LDS char*)smem_;
  const int tid = threadIdx.x;
  const int b = blockIdx.x / A.splits, sp = blockIdx.x - b * A.splits;
  lbf16* zl = (lbf16*)smem;                                      // 32 B of zeros
  LDS int* tab = (LDS int*)(smem + 32);                          // k-chunk -> halo offset
  lbf16* wlds = (lbf16*)(smem + A.off_w);
  LDS uint8_t* codes = (LDS uint8_t*)(smem + A.off_codes);
  const uint32_t step = A.st ? (uint32_t)A.st->t : 0u;
  if (tid < 8) ((LDS uint32_t*)zl)[tid] = 0u;

  // every layer's weight pack -> LDS (one contiguous run per layer)
  for (int l = 0; l < ((A.dbg & 8) ? 0 : A.n); ++l) {
    const StackLayer& L = A.L[l];
    const int nv = L.KS * L.NT * 64;
    const bf16* src = L.wpk;
    lbf16* dst = wlds + L.w_lds;
    staged_copy<4, bf16x8>(
        nv, tid, STACK_THREADS, [&](int i) { return load_bf16x8(src + (size_t)i * 8); },
        [&](int i, const bf16x8& v) { *reinterpret_cast<LDS bf16x8*>(dst + i * 8) = v; });
  }
  // the image rows layer 0 needs -> its zero-padded halo image
  if (!(A.dbg & 8)) {
    const StackLayer& L = A.L[0];
    lbf16* img = (lbf16*)(smem + A.off_buf[0]);
    const int Hi = A.rows[0][sp][5], Wi = L.Wo + L.KW - 1, Cs = L.Cs_in;
    const int y0 = A.rows[0][sp][4];
    const bf16* x = A.x + (size_t)b * L.H * L.W * Cs;
    if (Cs == 4) {
      const FastDiv fwi(Wi);
      staged_copy<8, bf16x4>(
          Hi * Wi, tid, STACK_THREADS,
          [&](int i) {
            const int hy = fwi.div(i), hx = i - hy * Wi;
            const int iy = y0 + hy, ix = hx - L.pad_l;
            const bool ok = iy >= 0 && ix >= 0 && iy < L.H && ix < L.W;
            return load_bf16x4_if(ok, x + (iy * L.W + ix) * 4, x);
          },
          [&](int i, const bf16x4& v) { *reinterpret_cast<LDS bf16x4*>(img + i * 4) = v; });
    } else {
      const int cpp = Cs >> 3;
      const FastDiv fcpp(cpp), fwi(Wi);
      staged_copy<8, bf16x8>(
          Hi * Wi * cpp, tid, STACK_THREADS,
          [&](int i) {
            const int pix = fcpp.div(i), c = (i - pix * cpp) * 8;
            const int hy = fwi.div(pix), hx = pix - hy * Wi;
            const int iy = y0 + hy, ix = hx - L.pad_l;
            const bool ok = iy >= 0 && ix >= 0 && iy < L.H && ix < L.W;
            return load_bf16x8_if(ok, x + (iy * L.W + ix) * Cs + c, x);
          },
          [&](int i, const bf16x8& v) { *reinterpret_cast<LDS bf16x8*>(img + i * 8) = v; });
    }
  }

  for (int l = 0; l < A.n; ++l) {
    const StackLayer L = A.L[l];      // by value: one batch of scalar loads per layer instead of
    const bool last = l + 1 == A.n;   // a kernarg reload of every field after each barrier
    const int c0 = A.rows[l][sp][0], c1 = A.rows[l][sp][1];
    const int own0 = A.rows[l][sp][2], own1 = A.rows[l][sp][3];
    const int p0 = L.pool ? c0 >> 1 : c0;
    const int roff = c0 - L.pad_t - A.rows[l][sp][4];
    const lbf16* in = (const lbf16*)(smem + ((l & 1) ? A.off_buf[1] : A.off_buf[0]));
    lbf16* out = (lbf16*)(smem + ((l & 1) ? A.off_buf[0] : A.off_buf[1]));
    // where this layer's stage output lands: the next layer's halo image (rows from its
    // first input row), or a compact image of the local stage rows for the last layer
    int obase, OH, ol, OW;
    if (last) {
      obase = p0, OH = L.pool ? (c1 - c0) >> 1 : c1 - c0, ol = 0, OW = L.Wp;
    } else {
      const StackLayer& N = A.L[l + 1];
      obase = A.rows[l + 1][sp][4], OH = A.rows[l + 1][sp][5], ol = N.pad_l, OW = N.Wo + N.KW - 1;
    }
    {
      LDS bf16x8* z = (LDS bf16x8*)out;
      const int nz = (OH * OW * L.Cs_out) >> 3;   // Cs_out % 8 == 0
      const bf16x8 zero8 = zero_bf16x8();
      for (int i = tid; i < nz; i += STACK_THREADS) z[i] = zero8;
      const int Wi = L.Wo + L.KW - 1, KHW = L.KH * L.KW, cw = L.Cs_in == 4 ? 4 : 8;
      const int ntab = L.Cs_in == 4 ? L.KS * 8 : L.KS * 4;
      for (int c = tid; c < ntab; c += STACK_THREADS) {
        const int k0 = c * cw, tap = k0 / L.Cs_in;
        int e = -1;
        if (tap < KHW) {
          const int ky = tap / L.KW;
          e = (ky * Wi + (tap - ky * L.KW)) * L.Cs_in + (k0 - tap * L.Cs_in);
        }
        tab[c] = e;
      }
    }
    __syncthreads();
    const lbf16* wl = wlds + L.w_lds;
#define STACK_ARGS A, L, b, c0, c1, roff, in, out, obase, OH, ol, OW, codes, wl, tab, zl, step
    if (L.Cs_in == 4) {
      switch (L.NT) {
        case 1: stack_layer_tm<1, true>(STACK_ARGS); break;
        case 2: stack_layer_tm<2, true>(STACK_ARGS); break;
        case 3: stack_layer_tm<3, true>(STACK_ARGS); break;
        default: stack_layer_tm<4, true>(STACK_ARGS); break;
      }
    } else {
      switch (L.NT) {
        case 1: stack_layer_tm<1, false>(STACK_ARGS); break;
        case 2: stack_layer_tm<2, false>(STACK_ARGS); break;
        case 3: stack_layer_tm<3, false>(STACK_ARGS); break;
        default: stack_layer_tm<4, false>(STACK_ARGS); break;
      }
    }
#undef STACK_ARGS
    __syncthreads();
    // owned stage rows (+ argmax codes) -> global, 16-byte stores
    if (!(A.dbg & 4)) {
      const int cch = L.Cs_out >> 3;
      const int n = (own1 - own0) * L.Wp * cch;
      const FastDiv fc(cch), fw(L.Wp);
      bf16* gout = L.out + ((size_t)b * L.Hp + own0) * L.Wp * L.Cs_out;
      for (int i = tid; i < n; i += STACK_THREADS) {
        const int pix = fc.div(i), c = (i - pix * cch) * 8;
        const int pyo = fw.div(pix), px = pix - pyo * L.Wp;
        *reinterpret_cast<bf16x8*>(gout + pix * L.Cs_out + c) =
            *reinterpret_cast<const LDS bf16x8*>(out + ((own0 + pyo - obase) * OW + px + ol) * L.Cs_out + c);
      }
      if (L.pool && L.code) {
        const int nb = ((own1 - own0) * L.Wp * L.Cs_out) >> 3;
        unsigned long long* gc =
            reinterpret_cast<unsigned long long*>(L.code + ((size_t)b * L.Hp + own0) * L.Wp * L.Cs_out);
        const LDS unsigned long long* lc = (const LDS unsigned long long*)(codes + (own0 - p0) * L.Wp * L.Cs_out);
        for (int i = tid; i < nb; i += STACK_THREADS) gc[i] = lc[i];
      }
    }
    // (no barrier: the next layer writes `codes` / the other buffer only after its own)
  }
}

void launch_conv_stack_fwd(const ConvStackArgs& a, hipStream_t s) {
  auto k = conv_stack_fwd_kernel;
  if (a.lds_bytes > 65536)
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, a.lds_bytes);
  hipLaunchKernelGGL(k, dim3(a.B * a.splits), dim3(STACK_THREADS), a.lds_bytes, s, a);
}
