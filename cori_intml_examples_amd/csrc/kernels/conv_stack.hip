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
// Per layer (12 waves): m-tiles are 16 output pixels (or 4 pooling windows x 4 positions,
// so the 2x2 max-pool is register-local: an MFMA accumulator row group is one window),
// TM m-tiles x NT n-tiles per wave; A fragments are one ds_read_b128 per k-step from the
// halo image (two ds_read_b64 for the 4-channel input), B fragments come from the layer's
// fragment-major weight pack staged in LDS at kernel start.  All LDS traffic goes through
// address-space-3 pointers with 32-bit offsets (generic pointers would turn every access
// into FLAT instructions with 64-bit address math: the epilogue was VALU-bound on that).
// Numerics (bf16 rounding points, dropout counters, argmax codes) are identical to the
// per-layer kernels.
#include "args.h"

// 12 waves (3 per SIMD): measured 25.4 -> 24.8 us (B=128) and 125.7 -> 115.0 us (B=1024)
// over 8 waves -- the per-layer tile loops are latency-bound, one workgroup per CU (LDS);
// 16 waves would cap the kernel at 128 VGPRs and spill
#define STACK_THREADS 768
#define STACK_WAVES (STACK_THREADS / 64)
#define STACK_TABN 80            // ints per layer's k-offset table (KS <= 18: <= 72 entries)
#define LDS __attribute__((address_space(3)))

typedef LDS bf16 lbf16;

__host__ __device__ __forceinline__ int cdiv(int a, int b) { return (a + b - 1) / b; }

// phase stamp (diagnostics only: A.ts null in production): wall clock per wave, lane 0
#define STACK_STAMP(i)                                                                                   \
  if (TS && A.ts && (threadIdx.x & 63) == 0) {                                                                 \
    unsigned long long* ts_ = A.ts + ((size_t)blockIdx.x * STACK_WAVES + (threadIdx.x >> 6)) * 32 + (i);  \
    ts_[0] = wall_clock64();                                                                             \
    ts_[16] = clock64();                                                                                 \
  }


// One layer over the workgroup's conv-output rows [c0, c1).  Local conv row y reads rows
// y + roff + ky of the input halo image `in`; stage output row py lands in row py - obase
// of `outimg` (skipped outside [0, OH)); codes are kept for the local stage rows.
template <int NT, int TM, bool CS4, int NW = STACK_WAVES>
__device__ __forceinline__ void stack_layer(const ConvStackArgs& A, const StackLayer& L, int b, int c0, int c1,
                                            int roff, const lbf16* in, lbf16* outimg, int obase, int OH, int ol,
                                            int OW, int XPo, LDS uint8_t* codes, const lbf16* wl, const LDS int* tab,
                                            const lbf16* zl, uint32_t step, const LDS float* lb, const int dbg) {
  // OW / XPo: row stride (pixels) / pixel stride (elements) of the output image
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 15, g = lane >> 4;
  const int XR = L.xrow, XP = L.xpix;           // input image layout
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
    bias[nt] = n < Cout ? lb[n] : 0.f;     // staged in LDS at kernel start
  }
  for (int tb = wave * TM; tb < ntiles; tb += NW * TM) {
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
      xo[t] = ((ry + roff) * XR + rx) * XP;
    }
    f32x4 acc[TM][NT];
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[t][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int KSr = (dbg & 1) ? 0 : KS;
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
    if (dbg & 2) {
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
        const int oo = (orow * OW + pxl + ol) * XPo, co = (pyl * Wp + pxl) * Cso;
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
          const int oo = (orow * OW + x + ol) * XPo;
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

// Row-aligned fast path for pooled layers whose pooled width is a multiple of 4 (every
// pooled layer of the RPV / DistTrain_mnist stacks): an m-tile is 4 consecutive pooling
// windows of ONE pooled row, so the tile -> (row, column) split is wave-uniform scalar
// arithmetic and each lane's pixel is a fixed offset from the tile base (no per-lane
// divisions, no per-tile validity selects).  The per-lane tap offsets of every k-step are
// computed once per layer into registers (KS is a template parameter), and the k padding
// beyond the last tap points at the pixel itself -- finite activations times the pack's
// zero rows -- instead of a zero buffer behind a select.  Same k order, rounding points,
// argmax codes and dropout counters as stack_layer (bit-identical).
// K16: 1 = the k16 tail (below) always, 0 = never, -1 = as A.k16 says (generic kernel);
// TS: the diagnostics stamps are compiled in (timeline builds; A.ts may still be null)
template <int NT, int TM, bool CS4, int KS, bool FULL, int K16 = -1, bool TS = true, int NW = STACK_WAVES>
__device__ __forceinline__ void stack_layer_rows(const ConvStackArgs& A, const StackLayer& L, int b, int c0, int c1,
                                                 int roff, const lbf16* in, lbf16* outimg, int obase, int OH, int ol,
                                                 int OW, int XPo, LDS uint8_t* codes, const lbf16* wl, uint32_t step,
                                                 const LDS float* lb, bool stamp) {
  // OW / XPo: row stride (pixels) / pixel stride (elements) of the output image
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 15, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int Wi = L.xrow, Cs = L.xpix;           // input image row / pixel strides
  const int Cso = L.Cs_out, Cout = L.Cout, Wp = L.Wp;
  const int p0 = c0 >> 1;
  const int tpr = Wp >> 2;                      // tiles per pooled row
  const int ntiles = ((c1 - c0) >> 1) * tpr;
  const uint32_t thr = L.drop_thr, sid = L.stream_id, seed = A.seed;
  const float dscale = L.drop_scale;
  const uint32_t qb = (uint32_t)(b * L.Hp + p0) * (uint32_t)Wp;
  // lane -> (window j, sub-pixel dy, dx) of the tile's 2 x 8 conv pixels
  const int lane_px = ((((r >> 1) & 1) * Wi) + 2 * (r >> 2) + (r & 1)) * Cs;
  // per-lane tap offsets of every k-step (k = tap * Cs + c, lanes of group g hold k0 .. k0+7)
  int e0[KS], e1[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int k0 = ks * 32 + g * 8;
    if (CS4) {
      const int t0 = k0 >> 2, t1 = t0 + 1;
      e0[ks] = t0 < 9 ? ((t0 / 3) * Wi + (t0 % 3)) * 4 : 0;
      e1[ks] = t1 < 9 ? ((t1 / 3) * Wi + (t1 % 3)) * 4 : 0;
    } else {
      const int tap = k0 / L.Cs_in, c = k0 - tap * L.Cs_in;
      e0[ks] = tap < 9 ? ((tap / 3) * Wi + (tap % 3)) * Cs + c : 0;
    }
  }
  float bias[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int n = nt * 16 + r;
    bias[nt] = n < Cout ? lb[n] : 0.f;     // staged in LDS at kernel start
  }
  // tile -> (pooled row, first window): scalar shift when tiles-per-row is a power of two
  const bool tpow2 = (tpr & (tpr - 1)) == 0;
  const int tsh = __builtin_ctz(tpr);
  auto trow = [&](int tile) { return tpow2 ? tile >> tsh : tile / tpr; };
  // epilogue lane constants: window g of the tile, channel r of n-tile 0 (output image / codes)
  const int lo_g = g * XPo + r, lc_g = g * Cso + r;
  const uint32_t qlane = (uint32_t)g * (uint32_t)Cout + (uint32_t)r;
  // FULL: Cso == Cout == NT * 16 (no padded channels): no per-lane channel guards
  for (int tb = wave * TM; tb < ntiles; tb += NW * TM) {
    int base[TM];
#pragma unroll
    for (int t = 0; t < TM; ++t) {
      const int tile = min(tb + t, ntiles - 1);   // duplicate of a valid tile: computed, not stored
      const int pyl = trow(tile), wx0 = (tile - pyl * tpr) * 4;
      base[t] = ((2 * pyl + roff) * Wi + 2 * wx0) * Cs + lane_px;
    }
    f32x4 acc[TM][NT];
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[t][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    // software-pipelined k loop: the fragments of k-step ks+1 are requested before the
    // MFMAs of k-step ks issue (sched_barrier pins the order), so LDS latency hides behind
    // the matrix work instead of a wait in front of every MFMA pair
    bf16x8 af[2][TM], bf[2][NT];
    auto load_k = [&](int ks, bf16x8* a, bf16x8* bv) {
#pragma unroll
      for (int t = 0; t < TM; ++t) {
        if (CS4) {
          const bf16x4 v0 = *reinterpret_cast<const LDS bf16x4*>(in + base[t] + e0[ks]);
          const bf16x4 v1 = *reinterpret_cast<const LDS bf16x4*>(in + base[t] + e1[ks]);
          a[t] = __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
        } else {
          a[t] = *reinterpret_cast<const LDS bf16x8*>(in + base[t] + e0[ks]);
        }
      }
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) bv[nt] = *reinterpret_cast<const LDS bf16x8*>(wl + ((ks * NT + nt) * 64 + lane) * 8);
    };
    if constexpr (CS4 && KS == 2 && K16 != 0) {
      if (K16 == 1 || A.k16) {
        // k-step 1 holds only tap 8 (k 32..35): one 16x16x16 MFMA (lane group g holds k
        // 4g..4g+3 of the 16-wide step) on the lane's 8-byte tap-8 read; B = the 32-wide pack
        // vector's first four k of lane (r, 0), zero for g > 0 (k >= 36: no tap)
        load_k(0, af[0], bf[0]);
        bf16x4 a16[TM], b16[NT];
        const bf16x4 z4 = {(bf16)0.f, (bf16)0.f, (bf16)0.f, (bf16)0.f};
#pragma unroll
        for (int t = 0; t < TM; ++t) a16[t] = *reinterpret_cast<const LDS bf16x4*>(in + base[t] + e0[1]);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const bf16x4 w4 = *reinterpret_cast<const LDS bf16x4*>(wl + ((NT + nt) * 64 + r) * 8);
          b16[nt] = g == 0 ? w4 : z4;
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
          for (int t = 0; t < TM; ++t) acc[t][nt] = mfma16(af[0][t], bf[0][nt], acc[t][nt]);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
          for (int t = 0; t < TM; ++t) acc[t][nt] = mfma16k16(a16[t], b16[nt], acc[t][nt]);
        __builtin_amdgcn_sched_barrier(0);
        goto k_done;
      }
    }
    load_k(0, af[0], bf[0]);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (ks + 1 < KS) load_k(ks + 1, af[(ks + 1) & 1], bf[(ks + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int t = 0; t < TM; ++t) acc[t][nt] = mfma16(af[ks & 1][t], bf[ks & 1][nt], acc[t][nt]);
      __builtin_amdgcn_sched_barrier(0);
    }
  k_done:
    if constexpr (TS) {
      if (stamp && tb == wave * TM) {
        asm volatile("" ::"v"(acc[0][0][0]));
        STACK_STAMP(14);
      }
    }
#pragma unroll
    for (int t = 0; t < TM; ++t) {
      const int tile = tb + t;
      if (tile >= ntiles) break;
      const int pyl = trow(tile), wx0 = (tile - pyl * tpr) * 4;
      const int orow = p0 + pyl - obase;
      const bool keep = orow >= 0 && orow < OH;
      if (FULL) {   // scalar tile bases + lane constants: one add per address
        const int ob = (orow * OW + wx0 + ol) * XPo + lo_g, cb = (pyl * Wp + wx0) * Cso + lc_g;
        const uint32_t qt = (qb + (uint32_t)(pyl * Wp + wx0)) * (uint32_t)Cout + qlane;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          // 2x2 max-pool + first-index argmax as a max tree and three equality tests (the
          // serial compare-and-select chain was 3 compares + 6 selects per element)
          float v[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v[j] = acc[t][nt][j] + bias[nt];
            if (L.relu) v[j] = fmaxf(v[j], 0.f);
          }
          float best = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
          const int code = v[0] == best ? 0 : v[1] == best ? 1 : v[2] == best ? 2 : 3;
          if (thr) best = dropout_keep(qt + (uint32_t)(nt * 16), seed, sid, step, thr) ? best * dscale : 0.f;
          if (keep) outimg[ob + nt * 16] = f2bf(best);
          codes[cb + nt * 16] = (uint8_t)code;
        }
        continue;
      }
      const int pxl = wx0 + g;
      const int oo = (orow * OW + pxl + ol) * XPo, co = (pyl * Wp + pxl) * Cso;
      const uint32_t qi = (qb + (uint32_t)(pyl * Wp + pxl)) * (uint32_t)Cout;
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int n = nt * 16 + r;
        if (n >= Cso) continue;
        float best = 0.f;
        int code = 0;
        if (n < Cout) {
          best = -3.4e38f;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float v = acc[t][nt][j] + bias[nt];
            if (L.relu) v = fmaxf(v, 0.f);
            if (v > best) { best = v; code = j; }
          }
          if (thr) best = dropout_keep(qi + (uint32_t)n, seed, sid, step, thr) ? best * dscale : 0.f;
          if (keep) outimg[oo + n] = f2bf(best);
        }
        codes[co + n] = (uint8_t)code;
      }
    }
    if constexpr (TS) {
      if (stamp && tb == wave * TM) STACK_STAMP(15);
    }
  }
}

template <int NT, bool CS4>
__device__ __forceinline__ void stack_layer_tm(const ConvStackArgs& A, const StackLayer& L, int b, int c0, int c1,
                                               int roff, const lbf16* in, lbf16* outimg, int obase, int OH, int ol,
                                               int OW, int XPo, LDS uint8_t* codes, const lbf16* wl, const LDS int* tab,
                                               const lbf16* zl, uint32_t step, const LDS float* lb, const int dbg) {
  constexpr int TM = NT >= 2 ? 2 : 4;
  stack_layer<NT, TM, CS4>(A, L, b, c0, c1, roff, in, outimg, obase, OH, ol, OW, XPo, codes, wl, tab, zl, step, lb,
                           dbg);
}

// the row-aligned fast path applies (pooled, pooled width % 4 == 0, 3x3; ablations off)
__device__ __forceinline__ bool stack_rows_ok(const ConvStackArgs& A, const StackLayer& L) {
  return !(A.dbg & 16) && L.pool && (L.Wp & 3) == 0 && L.KH == 3 && L.KW == 3 && !(A.dbg & 3);
}

// 16 B per lane global -> LDS (M0 + 16 * lane), outside the compiler's wait tracking: the
// caller waits for it itself (s_waitcnt vmcnt(0)) before any LDS read of the destination.
// `ldst` must be wave-uniform.
__device__ __forceinline__ void dma16_untracked(const bf16* gsrc, LDS char* ldst) {
  const uint32_t m0v = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)ldst);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off"
               :: "s"(m0v), "v"(gsrc) : "memory", "m0");
}

// ---------------------------------------------------------------------------------------
// Layer signatures.  The generic kernel picks each layer's body at run time from a table of
// 7 row-aligned and 8 generic instances, keeps every ablation branch (A.dbg) and the k16
// switch live, and carries all of that code's register pressure into every launch (96 SGPRs
// spilled to VGPR lanes).  A SPECIALISED instance is compiled per layer signature of the
// networks that matter (the DistTrain_rpv / DistTrain_mnist stacks): the layer sequence,
// each layer's body and tile shape are template constants, there is no ablation code and
// no generic fallback inside it -- the launcher (launch_conv_stack_fwd) matches the args to
// an instantiated signature on the host and falls back to the generic kernel otherwise.
// A layer code packs:  kind (1 row-aligned, 2 generic) | CS4 << 2 | KS << 3 | NT << 8 |
// TM << 11 | FULL << 14  (stack_code() computes it on the host from the same rules the
// generic kernel applies per band).
constexpr unsigned stack_lc(int kind, bool cs4, int ks, int nt, int tm, bool full) {
  return (unsigned)kind | (cs4 ? 4u : 0u) | ((unsigned)ks << 3) | ((unsigned)nt << 8) | ((unsigned)tm << 11) |
         (full ? (1u << 14) : 0u);
}
template <unsigned C> struct StackLC {
  static constexpr int kind = C & 3;
  static constexpr bool cs4 = (C >> 2) & 1;
  static constexpr int KS = (C >> 3) & 31, NT = (C >> 8) & 7, TM = (C >> 11) & 7;
  static constexpr bool full = (C >> 14) & 1;
};

// one layer of a specialised stack: code C's body, no run-time dispatch
template <unsigned C, bool TS, int NW>
__device__ __forceinline__ void stack_run_code(const ConvStackArgs& A, const StackLayer& L, int b, int c0, int c1,
                                               int roff, const lbf16* in, lbf16* out, int obase, int OH, int ol,
                                               int ORS, int OPS, LDS uint8_t* codes, const lbf16* wl,
                                               const LDS int* tab, const lbf16* zl, uint32_t step,
                                               const LDS float* lb, bool last) {
  using D = StackLC<C>;
  if constexpr (D::kind == 1) {
    stack_layer_rows<D::NT, D::TM, D::cs4, D::KS, D::full, 1, TS, NW>(A, L, b, c0, c1, roff, in, out, obase, OH, ol,
                                                                        ORS, OPS, codes, wl, step, lb, last);
  } else if constexpr (D::kind == 2) {
    stack_layer<D::NT, D::TM, D::cs4, NW>(A, L, b, c0, c1, roff, in, out, obase, OH, ol, ORS, OPS, codes, wl, tab,
                                          zl, step, lb, 0);
  }
}

// SPEC: a specialised instance for the layer codes C0..C3 (0 = no layer); TS: stamps compiled in
// (12-wave instances only: the stamp buffer is indexed by STACK_WAVES); NTH: threads per
// workgroup (768 = 12 waves; 1024 = 16 waves for signatures whose registers fit 128 VGPRs)
template <bool SPEC, bool TS, unsigned C0, unsigned C1, unsigned C2, unsigned C3, int NTH = STACK_THREADS>
__global__ __launch_bounds__(NTH) void conv_stack_kernel(const ConvStackArgs A) {
  static_assert(!TS || NTH == STACK_THREADS, "stamps index NWV waves per workgroup");
  constexpr int NWV = NTH / 64;
  extern __shared__ __attribute__((aligned(16))) char smem_[];
  LDS char* smem = (LDS char*)smem_;
  constexpr int NL = SPEC ? (C0 != 0) + (C1 != 0) + (C2 != 0) + (C3 != 0) : 0;
  // every layer row-aligned: no k-offset tables (only the generic body reads them)
  constexpr bool no_tab = SPEC && StackLC<C0>::kind != 2 && StackLC<C1>::kind != 2 && StackLC<C2>::kind != 2 &&
                          StackLC<C3>::kind != 2;
  const int dbg = SPEC ? 0 : A.dbg;               // ablations: generic kernel only
  const int nlayers = SPEC ? NL : A.n;
  const int tid = threadIdx.x;
  const int b = blockIdx.x / A.splits, sp = blockIdx.x - b * A.splits;
  lbf16* zl = (lbf16*)smem;                                      // 32 B of zeros
  LDS int* tab = (LDS int*)(smem + 32);                          // [layer][STACK_TABN] k-chunk -> halo offset
  lbf16* wlds = (lbf16*)(smem + A.off_w);
  // two argmax-code planes (layer parity): a layer's epilogue writes its plane while slower
  // waves may still copy the previous layer's codes out (no barrier between those phases)
  // (a select, not a 2-entry array: indexed by a non-unrolled layer loop the array went to
  // scratch in the MNIST instances)
  LDS uint8_t* const codes_p0 = (LDS uint8_t*)(smem + A.off_codes);
  LDS uint8_t* const codes_p1 = (LDS uint8_t*)(smem + A.off_codes2);
  const uint32_t step = A.st ? (uint32_t)A.st->t + (uint32_t)A.step_inc : 0u;
  STACK_STAMP(0);
  if (tid < 8) ((LDS uint32_t*)zl)[tid] = 0u;
  // Weight packs -> LDS.  Layer 0's synchronously; the later layers' are loaded into
  // registers now (issued after the image, so waiting for the image does not wait for them)
  // and written to LDS only before layer 1 -- their latency hides behind layer 0.
  constexpr int PF = (4096 + NTH - 1) / NTH;
  // vectors of layers 1, 2, 3 (static indices: the kernarg loads hoist out of the loops)
  const int nv1 = nlayers > 1 ? A.L[1].KS * A.L[1].NT * 64 : 0;
  const int nv2 = nlayers > 2 ? A.L[2].KS * A.L[2].NT * 64 : 0;
  const int nv3 = nlayers > 3 ? A.L[3].KS * A.L[3].NT * 64 : 0;
  // (specialised instances: the launcher checked these geometry conditions on the host)
  const bool prefetch = SPEC ? NL > 1 : !(dbg & 40) && nlayers > 1 && nv1 + nv2 + nv3 <= PF * NTH;
  // Fast prologue (the RPV / MNIST stacks: 4-channel input, one batch of image loads per
  // thread): every global round trip of the staging in ONE batch -- the biases and layer 0's
  // weight pack are loaded first (independent of the image), then the image's dataset row
  // (scalar chain through the cursor and permutation) and its pixels, and only then are all
  // of them stored to LDS.  The sequential form (biases, weights, row lookup, pixels: five
  // dependent round trips) is kept for the other shapes and as the A/B reference (dbg 128).
  LDS float* lbias = (LDS float*)(smem + A.off_bias);
  const int nv0 = A.L[0].KS * A.L[0].NT * 64;
  const int hiwi0 = A.rows[0][sp][5] * (A.L[0].Wo + A.L[0].KW - 1);
  const bool fastpro = SPEC || (!(dbg & (8 | 128)) && prefetch && A.L[0].Cs_in == 4 && nv0 <= NTH &&
                                nlayers * 64 <= NTH && hiwi0 <= 4 * NTH);
  if (fastpro) {
    const StackLayer& L = A.L[0];
    const int bl = min(tid, nlayers * 64 - 1), bc = bl & 63;
    const StackLayer& LB = A.L[bl >> 6];
    const bool bok = tid < nlayers * 64 && LB.bias != nullptr && bc < LB.Cout;
    const float braw = *(bok ? LB.bias + bc : reinterpret_cast<const float*>(L.wpk));
    const bf16x8 wv = load_bf16x8(L.wpk + (size_t)min(tid, nv0 - 1) * 8);
    lbf16* img = (lbf16*)(smem + A.off_buf[0]);
    const int Wi = L.Wo + L.KW - 1, XR = L.xrow, XP = L.xpix, y0 = A.rows[0][sp][4];
    const bf16* x = A.x + (size_t)b * L.H * L.W * 4;
    if (A.from_data) {
      const int src = step_src_row(A.st, A.training, b);
      x = reinterpret_cast<const bf16*>(A.st->data_x) + (size_t)src * A.st->data_R;
      if (sp == 0 && tid == 0 && A.srcidx) A.srcidx[b] = src;
    }
    const FastDiv fwi(Wi);
    bf16x4 iv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = min(tid + u * NTH, hiwi0 - 1);
      const int hy = fwi.div(i), hx = i - hy * Wi;
      const int iy = y0 + hy, ix = hx - L.pad_l;
      const bool ok = iy >= 0 && ix >= 0 && iy < L.H && ix < L.W;
      iv[u] = load_bf16x4_if(ok, x + (iy * L.W + ix) * 4, x);
    }
    if (tid < nlayers * 64) lbias[tid] = bok ? braw : 0.f;
    if (tid < nv0) *reinterpret_cast<LDS bf16x8*>(wlds + L.w_lds + tid * 8) = wv;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = tid + u * NTH;
      if (i < hiwi0) {
        const int hy = fwi.div(i);
        *reinterpret_cast<LDS bf16x4*>(img + (hy * XR + (i - hy * Wi)) * XP) = iv[u];
      }
    }
  } else {
    // biases -> LDS [layer][64] (read by the epilogues: no global load after the prefetch
    // below, which would otherwise make its first use wait for every prefetched vector)
    for (int i = tid; i < nlayers * 64; i += NTH) {
      const StackLayer& L = A.L[i >> 6];
      const int c = i & 63;
      lbias[i] = (L.bias && c < L.Cout) ? L.bias[c] : 0.f;
    }

    for (int l = 0; l < ((dbg & 8) ? 0 : (prefetch ? 1 : nlayers)); ++l) {
      const StackLayer& L = A.L[l];
      const int nv = L.KS * L.NT * 64;
      const bf16* src = L.wpk;
      lbf16* dst = wlds + L.w_lds;
      staged_copy<4, bf16x8>(
          nv, tid, NTH, [&](int i) { return load_bf16x8(src + (size_t)i * 8); },
          [&](int i, const bf16x8& v) { *reinterpret_cast<LDS bf16x8*>(dst + i * 8) = v; });
    }
    // the image rows layer 0 needs -> its zero-padded halo image
    if (!(dbg & 8)) {
      const StackLayer& L = A.L[0];
      lbf16* img = (lbf16*)(smem + A.off_buf[0]);
      const int Hi = A.rows[0][sp][5], Wi = L.Wo + L.KW - 1, Cs = L.Cs_in;
      const int XR = L.xrow, XP = L.xpix;
      const int y0 = A.rows[0][sp][4];
      const bf16* x = A.x + (size_t)b * L.H * L.W * Cs;
      if (A.from_data) {   // straight from the bound dataset: no gather launch
        const int src = step_src_row(A.st, A.training, b);
        x = reinterpret_cast<const bf16*>(A.st->data_x) + (size_t)src * A.st->data_R;
        if (sp == 0 && tid == 0 && A.srcidx) A.srcidx[b] = src;
      }
      if (Cs == 4) {
        const FastDiv fwi(Wi);
        staged_copy<8, bf16x4>(
            Hi * Wi, tid, NTH,
            [&](int i) {
              const int hy = fwi.div(i), hx = i - hy * Wi;
              const int iy = y0 + hy, ix = hx - L.pad_l;
              const bool ok = iy >= 0 && ix >= 0 && iy < L.H && ix < L.W;
              return load_bf16x4_if(ok, x + (iy * L.W + ix) * 4, x);
            },
            [&](int i, const bf16x4& v) {
              const int hy = fwi.div(i);
              *reinterpret_cast<LDS bf16x4*>(img + (hy * XR + (i - hy * Wi)) * XP) = v;
            });
      } else {
        const int cpp = Cs >> 3;
        const FastDiv fcpp(cpp), fwi(Wi);
        staged_copy<8, bf16x8>(
            Hi * Wi * cpp, tid, NTH,
            [&](int i) {
              const int pix = fcpp.div(i), c = (i - pix * cpp) * 8;
              const int hy = fwi.div(pix), hx = pix - hy * Wi;
              const int iy = y0 + hy, ix = hx - L.pad_l;
              const bool ok = iy >= 0 && ix >= 0 && iy < L.H && ix < L.W;
              return load_bf16x8_if(ok, x + (iy * L.W + ix) * Cs + c, x);
            },
            [&](int i, const bf16x8& v) {
              const int pix = fcpp.div(i), c = (i - pix * cpp) * 8;
              const int hy = fwi.div(pix);
              *reinterpret_cast<LDS bf16x8*>(img + (hy * XR + (pix - hy * Wi)) * XP + c) = v;
            });
      }
    }

  }

  // k-chunk -> halo offset tables of every layer (the generic path reads them; the
  // row-aligned path keeps its tap offsets in registers, but a rows_ok layer without an
  // instantiated (KS, NT) falls back to the generic path), all computed once here: the
  // per-layer table phase and its barrier are gone
  for (int l = 0; l < (no_tab ? 0 : nlayers); ++l) {
    const StackLayer& L = A.L[l];
    const int Wi = L.xrow, KHW = L.KH * L.KW, cw = L.Cs_in == 4 ? 4 : 8;
    const int ntab = L.Cs_in == 4 ? L.KS * 8 : L.KS * 4;
    for (int c = tid; c < ntab; c += NTH) {
      const int k0 = c * cw, tap = k0 / L.Cs_in;
      int e = -1;
      if (tap < KHW) {
        const int ky = tap / L.KW;
        e = (ky * Wi + (tap - ky * L.KW)) * L.xpix + (k0 - tap * L.Cs_in);
      }
      tab[l * STACK_TABN + c] = e;
    }
  }

  STACK_STAMP(1);
  __syncthreads();                  // image, layer-0 weights, biases and tables staged

  // The later layers' weight packs -> their LDS slots by LDS-DMA, issued AFTER that barrier
  // so they land during layer 0's tiles: the slots (contiguous, layer 1 first) are not read
  // by layer 0; an explicit vmcnt(0) before layer 0's closing barrier publishes them to
  // layer 1.  The DMA is issued from inline asm: as a builtin the compiler's wait tracking
  // treats it as an LDS store that every later ds_read may alias and puts a vmcnt(0) in
  // front of layer 0's first LDS read (serialising it); register prefetch serialised too
  // (a select on the loaded value waited at once; the live registers spilled).
  // (the DMA source addresses stay live until that wait: overwriting the VGPRs of an
  // outstanding load's address made the compiler wait for it right away)
  const bf16* dma_src[PF];
  if (prefetch) {
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int ntot = nv1 + nv2 + nv3;                 // multiples of 64 vectors per layer
    LDS char* wdst = (LDS char*)(wlds + A.L[1].w_lds);
#pragma unroll
    for (int j = 0; j < PF; ++j) {                  // wave-uniform 64-vector chunks
      const int vb = wave * 64 + j * NTH;
      if (vb >= ntot) break;
      const int v = vb + lane;
      const bf16* src = v < nv1 ? A.L[1].wpk + (size_t)v * 8
                      : v < nv1 + nv2 ? A.L[2].wpk + (size_t)(v - nv1) * 8
                      : A.L[3].wpk + (size_t)(v - nv1 - nv2) * 8;
      dma_src[j] = src;
      dma16_untracked(src, wdst + (size_t)vb * 16);
    }
  }
  for (int l = 0; l < nlayers; ++l) {
    const StackLayer L = A.L[l];      // by value: one batch of scalar loads per layer instead of
    const bool last = l + 1 == nlayers;   // a kernarg reload of every field after each barrier
    const int c0 = A.rows[l][sp][0], c1 = A.rows[l][sp][1];
    const int own0 = A.rows[l][sp][2], own1 = A.rows[l][sp][3];
    const int p0 = L.pool ? c0 >> 1 : c0;
    const int roff = c0 - L.pad_t - A.rows[l][sp][4];
    const lbf16* in = (const lbf16*)(smem + ((l & 1) ? A.off_buf[1] : A.off_buf[0]));
    lbf16* out = (lbf16*)(smem + ((l & 1) ? A.off_buf[0] : A.off_buf[1]));
    // where this layer's stage output lands: the next layer's halo image (rows from its
    // first input row), or a compact image of the local stage rows for the last layer
    // (OW: logical width; ORS / OPS: row stride in pixels / pixel stride in elements of the
    // output image -- the next layer's input layout, dense for the last layer's compact image)
    int obase, OH, ol, OW, ORS, OPS;
    if (last) {
      obase = p0, OH = L.pool ? (c1 - c0) >> 1 : c1 - c0, ol = 0, OW = L.Wp;
      ORS = OW, OPS = L.Cs_out;
    } else {
      const StackLayer& N = A.L[l + 1];
      obase = A.rows[l + 1][sp][4], OH = A.rows[l + 1][sp][5], ol = N.pad_l, OW = N.Wo + N.KW - 1;
      ORS = N.xrow, OPS = N.xpix;
    }
    LDS uint8_t* codes = (l & 1) ? codes_p1 : codes_p0;
    {
      LDS bf16x8* z = (LDS bf16x8*)out;
      const bf16x8 zero8 = zero_bf16x8();
      // The epilogue writes every channel of output rows [wr0, wr1) x columns [ol, ol + Wp)
      // (all channels when Cs_out == Cout); only the rest of the image needs zeros -- at
      // addresses no epilogue store touches, so the zeroing runs beside this layer's tiles
      // (the barrier after them publishes both).  Otherwise the whole image is zeroed first.
      const int nr = L.pool ? (c1 - c0) >> 1 : c1 - c0;
      const int wr0 = max(0, p0 - obase), wr1 = min(OH, p0 - obase + nr);
      // (in 8-channel vectors of the output layout; pixel padding is zeroed with its pixel,
      // row padding past OW is never read)
      const int vpp = OPS >> 3;                             // vectors per pixel (Cs_out % 8 == 0)
      const int nrow = ORS * vpp;                           // vectors per image row
      if (L.Cs_out == L.Cout && wr0 < wr1 && !(dbg & 3)) {
        const int ntop = wr0 * nrow, nbot = (OH - wr1) * nrow;
        const int nside = (OW - L.Wp) * vpp;                // border vectors per written row
        for (int i = tid; i < ntop + nbot; i += NTH) z[i < ntop ? i : wr1 * nrow + (i - ntop)] = zero8;
        if (nside > 0) {
          const int lcols = ol * vpp;
          for (int i = tid; i < (wr1 - wr0) * nside; i += NTH) {
            const int rr = i / nside, c = i - rr * nside;
            z[(wr0 + rr) * nrow + (c < lcols ? c : c + L.Wp * vpp)] = zero8;
          }
        }
      } else {
        const int nz = OH * nrow;
        for (int i = tid; i < nz; i += NTH) z[i] = zero8;
        __syncthreads();                                    // before any epilogue store
      }
    }
    STACK_STAMP(2 + 4 * l);
    const lbf16* wl = wlds + L.w_lds;
#define STACK_ARGS A, L, b, c0, c1, roff, in, out, obase, OH, ol, ORS, OPS, codes, wl, tab + l * STACK_TABN, zl, step, lbias + l * 64
#define ROWS_ARGS A, L, b, c0, c1, roff, in, out, obase, OH, ol, ORS, OPS, codes, wl, step, lbias + l * 64, l == nlayers - 1
    if constexpr (SPEC) {
#define CODE_ARGS A, L, b, c0, c1, roff, in, out, obase, OH, ol, ORS, OPS, codes, wl, tab + l * STACK_TABN, zl, step, \
                  lbias + l * 64, l == nlayers - 1
      if (l == 0) stack_run_code<C0, TS, NWV>(CODE_ARGS);
      else if (l == 1) stack_run_code<C1, TS, NWV>(CODE_ARGS);
      else if (l == 2) stack_run_code<C2, TS, NWV>(CODE_ARGS);
      else stack_run_code<C3, TS, NWV>(CODE_ARGS);
#undef CODE_ARGS
    } else {
    // row-aligned fast path (pooled, pooled width % 4 == 0, 3x3, instantiated KS), else generic
    const bool rows_ok = stack_rows_ok(A, L);
    // TM = 1 when it evens out the waves' tile counts (few tiles per workgroup)
    const int ntl = ((c1 - c0) >> 1) * (L.Wp >> 2);
    const bool tm1 = ntl <= NWV || cdiv(ntl, NWV) < 2 * cdiv(ntl, 2 * NWV);
    const bool full = L.Cs_out == L.Cout && L.Cout == L.NT * 16;
#define ROWS(NT_, TM_, CS4_, KS_)                                                   \
  {                                                                                 \
    if (full) stack_layer_rows<NT_, TM_, CS4_, KS_, true>(ROWS_ARGS);               \
    else stack_layer_rows<NT_, TM_, CS4_, KS_, false>(ROWS_ARGS);                   \
  }
    if (rows_ok && L.Cs_in == 4 && L.KS == 2 && L.NT == 1) ROWS(1, 4, true, 2)
    else if (rows_ok && L.Cs_in == 4 && L.KS == 2 && L.NT == 2) ROWS(2, 2, true, 2)
    else if (rows_ok && L.Cs_in != 4 && L.KS == 5 && L.NT == 2 && tm1) ROWS(2, 1, false, 5)
    else if (rows_ok && L.Cs_in != 4 && L.KS == 5 && L.NT == 2) ROWS(2, 2, false, 5)
    else if (rows_ok && L.Cs_in != 4 && L.KS == 9 && L.NT == 4 && tm1) ROWS(4, 1, false, 9)
    else if (rows_ok && L.Cs_in != 4 && L.KS == 9 && L.NT == 4) ROWS(4, 2, false, 9)
    else if (rows_ok && L.Cs_in != 4 && L.KS == 9 && L.NT == 2) ROWS(2, 2, false, 9)
#undef ROWS
    else if (L.Cs_in == 4) {
      switch (L.NT) {
        case 1: stack_layer_tm<1, true>(STACK_ARGS, dbg); break;
        case 2: stack_layer_tm<2, true>(STACK_ARGS, dbg); break;
        case 3: stack_layer_tm<3, true>(STACK_ARGS, dbg); break;
        default: stack_layer_tm<4, true>(STACK_ARGS, dbg); break;
      }
    } else {
      switch (L.NT) {
        case 1: stack_layer_tm<1, false>(STACK_ARGS, dbg); break;
        case 2: stack_layer_tm<2, false>(STACK_ARGS, dbg); break;
        case 3: stack_layer_tm<3, false>(STACK_ARGS, dbg); break;
        default: stack_layer_tm<4, false>(STACK_ARGS, dbg); break;
      }
    }
    }
#undef STACK_ARGS
#undef ROWS_ARGS
    STACK_STAMP(3 + 4 * l);
    if (l == 0 && prefetch) {
#pragma unroll
      for (int j = 0; j < PF; ++j) asm volatile("" :: "v"(dma_src[j]));
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the untracked DMA
    }
    __syncthreads();
    STACK_STAMP(4 + 4 * l);
    // owned stage rows (+ argmax codes) -> global, 16-byte stores
    if (!(dbg & 4)) {
      const int cch = L.Cs_out >> 3;
      const int n = (own1 - own0) * L.Wp * cch;
      const FastDiv fc(cch), fw(L.Wp);
      bf16* gout = L.out + ((size_t)b * L.Hp + own0) * L.Wp * L.Cs_out;
      // write-through (A.wt): the next launch reads these rows from other XCDs anyway
      const bool wt = A.wt && (L.Cs_out & 15) == 0;
      for (int i = tid; i < n; i += NTH) {
        const int pix = fc.div(i), c = (i - pix * cch) * 8;
        const int pyo = fw.div(pix), px = pix - pyo * L.Wp;
        const u32x4 v = *reinterpret_cast<const LDS u32x4*>(out + ((own0 + pyo - obase) * ORS + px + ol) * OPS + c);
        if (wt) st_wt16(gout, (unsigned)(pix * L.Cs_out + c) * 2u, v);
        else *reinterpret_cast<u32x4*>(gout + pix * L.Cs_out + c) = v;
      }
      if (L.pool && L.code) {
        const int nbytes = (own1 - own0) * L.Wp * L.Cs_out;
        uint8_t* gcb = L.code + ((size_t)b * L.Hp + own0) * L.Wp * L.Cs_out;
        const LDS uint8_t* lcb = codes + (own0 - p0) * L.Wp * L.Cs_out;
        if (wt) {   // 16-byte code vectors (Cs_out % 16 == 0: whole vectors, 16-byte aligned)
          for (int i = tid; i < (nbytes >> 4); i += NTH)
            st_wt16(gcb, (unsigned)i * 16u, *reinterpret_cast<const LDS u32x4*>(lcb + i * 16));
        } else {
          unsigned long long* gc = reinterpret_cast<unsigned long long*>(gcb);
          const LDS unsigned long long* lc = (const LDS unsigned long long*)lcb;
          for (int i = tid; i < (nbytes >> 3); i += NTH) gc[i] = lc[i];
        }
      }
    }
    STACK_STAMP(5 + 4 * l);
    // (no barrier: the next layer writes `codes` / the other buffer only after its own)
  }
}

int conv_stack_threads() { return STACK_THREADS; }
int conv_stack_tabn() { return STACK_TABN; }

// ----------------------------------------------------------------------- host-side dispatch
// Layer l's code as the generic kernel would pick its body (stack_rows_ok, the TM rule per
// band for nw waves, FULL); 0 if the bands disagree on TM (no specialised instance serves them).
static unsigned host_layer_code(const ConvStackArgs& a, int l, int nw) {
  const StackLayer& L = a.L[l];
  const bool rows_ok = !(a.dbg & 19) && L.pool && (L.Wp & 3) == 0 && L.KH == 3 && L.KW == 3;
  const bool full = L.Cs_out == L.Cout && L.Cout == L.NT * 16;
  int tm = 0;
  for (int sp = 0; sp < a.splits; ++sp) {
    const int ntl = ((a.rows[l][sp][1] - a.rows[l][sp][0]) >> 1) * (L.Wp >> 2);
    const bool tm1 = ntl <= nw || cdiv(ntl, nw) < 2 * cdiv(ntl, 2 * nw);
    const int t = tm1 ? 1 : 2;
    if (tm && t != tm) return 0;
    tm = t;
  }
  const bool c4 = L.Cs_in == 4;
  if (rows_ok && c4 && L.KS == 2 && L.NT == 1) return stack_lc(1, true, 2, 1, 4, full);
  if (rows_ok && c4 && L.KS == 2 && L.NT == 2) return stack_lc(1, true, 2, 2, 2, full);
  if (rows_ok && !c4 && L.KS == 5 && L.NT == 2) return stack_lc(1, false, 5, 2, tm, full);
  if (rows_ok && !c4 && L.KS == 9 && L.NT == 4) return stack_lc(1, false, 9, 4, tm, full);
  if (rows_ok && !c4 && L.KS == 9 && L.NT == 2) return stack_lc(1, false, 9, 2, 2, full);
  const int nt = L.NT < 1 ? 1 : (L.NT > 4 ? 4 : L.NT);
  return stack_lc(2, c4, 0, nt, nt >= 2 ? 2 : 4, false);
}

// the specialised instances: the DistTrain_rpv stack (64x64x{1,3} -> conv 16 / 32 / 64, each
// + ReLU + 2x2 pool; the TM of layers 1 and 2 depends on the row bands) and the
// DistTrain_mnist stack (28x28x1 -> conv 32 'valid' unpooled, conv 64 + pool).  The RPV
// stack's all-TM-1 signature also has a 16-wave instance (its 12-wave build needs 120 VGPRs:
// at 16 waves the 128-VGPR cap holds without spills) -- chosen with spec = 2.
#define RPV_L0 stack_lc(1, true, 2, 1, 4, true)
#define RPV_L1(tm) stack_lc(1, false, 5, 2, tm, true)
#define RPV_L2(tm) stack_lc(1, false, 9, 4, tm, true)
#define MN_L0 stack_lc(2, true, 0, 2, 2, false)
#define MN_L1(tm) stack_lc(1, false, 9, 4, tm, true)
typedef void (*StackKernel)(const ConvStackArgs);
struct StackSig { int nth; unsigned c[MAX_STACK]; StackKernel k[2]; };   // k[TS] (k[1] null: no stamp build)
#define SIG(c0, c1, c2, c3) \
  {STACK_THREADS, {c0, c1, c2, c3}, \
   {conv_stack_kernel<true, false, c0, c1, c2, c3>, conv_stack_kernel<true, true, c0, c1, c2, c3>}}
#define SIG16(c0, c1, c2, c3) {1024, {c0, c1, c2, c3}, {conv_stack_kernel<true, false, c0, c1, c2, c3, 1024>, nullptr}}
static const StackSig kStackSigs[] = {
    SIG16(RPV_L0, RPV_L1(1), RPV_L2(1), 0u),
    SIG(RPV_L0, RPV_L1(2), RPV_L2(1), 0u), SIG(RPV_L0, RPV_L1(2), RPV_L2(2), 0u),
    SIG(RPV_L0, RPV_L1(1), RPV_L2(1), 0u), SIG(RPV_L0, RPV_L1(1), RPV_L2(2), 0u),
    SIG(MN_L0, MN_L1(1), 0u, 0u), SIG(MN_L0, MN_L1(2), 0u, 0u),
};
#undef SIG
#undef SIG16

// does signature i serve these args (its layer codes for its wave count, and the
// specialised prologue's geometry conditions -- the generic kernel tests those per launch)
static bool stack_sig_matches(const ConvStackArgs& a, const StackSig& g) {
  const int nth = g.nth, nw = nth / 64;
  for (int l = 0; l < MAX_STACK; ++l) {
    const unsigned c = l < a.n ? host_layer_code(a, l, nw) : 0u;
    if (c == 0u && l < a.n) return false;
    if (c != g.c[l]) return false;
  }
  const int PF = (4096 + nth - 1) / nth;
  int nv_later = 0;
  for (int l = 1; l < a.n; ++l) nv_later += a.L[l].KS * a.L[l].NT * 64;
  const StackLayer& L0 = a.L[0];
  if (L0.Cs_in != 4 || L0.KS * L0.NT * 64 > nth || a.n * 64 > nth || nv_later > PF * nth) return false;
  for (int sp = 0; sp < a.splits; ++sp)
    if (a.rows[0][sp][5] * (L0.Wo + L0.KW - 1) > 4 * nth) return false;
  return true;
}

// 1 + index of the specialised instance serving these args, or 0 (generic kernel).  spec = 1:
// the 12-wave instances; spec = 2: a 16-wave instance first where one matches; a stamp
// request (ts) takes the 12-wave stamp builds.
int conv_stack_variant(const ConvStackArgs& a) {
  if (!a.spec || a.dbg || a.n < 2 || a.n > MAX_STACK) return 0;
  const int nsig = (int)(sizeof(kStackSigs) / sizeof(kStackSigs[0]));
  for (int pass = (a.spec >= 2 && !a.ts) ? 0 : 1; pass < 2; ++pass)
    for (int i = 0; i < nsig; ++i) {
      const bool wide = kStackSigs[i].nth != STACK_THREADS;
      if (wide != (pass == 0)) continue;
      if (stack_sig_matches(a, kStackSigs[i])) return i + 1;
    }
  return 0;
}

void launch_conv_stack_fwd(const ConvStackArgs& a, hipStream_t s) {
  const int v = conv_stack_variant(a);
  StackKernel k = v ? kStackSigs[v - 1].k[a.ts ? 1 : 0] : conv_stack_kernel<false, true, 0u, 0u, 0u, 0u>;
  const int nth = v ? kStackSigs[v - 1].nth : STACK_THREADS;
  if (a.lds_bytes > 65536)
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, a.lds_bytes);
  hipLaunchKernelGGL(k, dim3(a.B * a.splits), dim3(nth), a.lds_bytes, s, a);
}
