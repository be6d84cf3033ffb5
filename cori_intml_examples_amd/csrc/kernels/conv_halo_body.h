// Body of the halo-staged implicit-GEMM conv kernel (see conv_halo.hip for the design),
// as a device function of the block index so dual_halo.hip can co-schedule it with
// the weight-gradient body in one launch.
#pragma once
#include <type_traits>

#include "bwd_through.h"

// NTC n-tiles of the weight slice, TM m-tiles per wave per pass (each A fragment feeds NTC
// MFMAs and each weight fragment TM), KCH k-steps per batch of independent reads.
#define HALO_STAMP(i)                                                                \
  if (INSTR && a.ts && threadIdx.x == 0) a.ts[(size_t)blockIdx.x * 8 + (i)] = wall_clock64();

// MODE: 0 forward / 1 backward-through epilogue fixed at compile time, -1 = a.mode at run time;
// INSTR: the ablation switches (dbg) and diagnostics stamps (a.ts) are compiled in.  The
// co-scheduled dual launch instantiates <.., 1, false>: none of that code (nor the forward
// epilogue) is in its instruction stream or its register allocation.
template <int NTC, int TM, int KCH, bool CS4, int MODE = -1, bool INSTR = true>
__device__ __forceinline__ void conv_halo_body(const ConvMMArgs& a, const int bx, const int by, char* smem) {
  const int dbg = INSTR ? a.dbg : 0;
  const int mode = MODE >= 0 ? MODE : a.mode;
  const int KS = a.KS, R = a.R, s = a.stride, dil = a.in_dil, Cs = a.Cs_in;
  // halo pixel stride (elements): padded by the host's bank-conflict model (lds_layout.py)
  const int XP = (CS4 || !a.xpix) ? Cs : a.xpix;
  const int ntab = CS4 ? KS * 8 : KS * 4;
  int* tab = reinterpret_cast<int*>(smem);
  const int tab_bytes = (ntab * 4 + 15) & ~15;
  bf16* zl = reinterpret_cast<bf16*>(smem + tab_bytes);      // 32 B of zeros
  bf16* wl = zl + 16;
  bf16* xl = wl + (size_t)KS * NTC * 64 * 8;
  const int W_in = (a.Wo - 1) * s + a.KW;
  const int R_in = (R - 1) * s + a.KH;
  const int tid = threadIdx.x;
  const int nrb = (a.Ho + R - 1) / R;
  const int b = bx / nrb;
  const int oy0 = (bx - b * nrb) * R;
  const int nt0 = by * NTC;

  HALO_STAMP(0);
  if (tid < 8) reinterpret_cast<uint32_t*>(zl)[tid] = 0u;
  const bool dbg_stage = !(dbg & 1), dbg_mfma = !(dbg & 2), dbg_store = !(dbg & 4);
  // input halo geometry (staged after the weights: issuing the halo's HBM loads first was
  // measured 3 us slower -- the weights' LDS stores then wait behind them)
  const int hcw = CS4 ? 4 : 8;
  const int hcpp = Cs / hcw;
  const int nch = R_in * W_in * hcpp;
  const int yb = oy0 * s - a.pad_t, xb0 = -a.pad_l;
  const bf16* xbase = a.in_code ? a.x + (size_t)b * a.in_pH * a.in_pW * Cs : a.x + (size_t)b * a.H * a.W * Cs;
  const uint8_t* cbase = a.in_code ? a.in_code + (size_t)b * a.in_pH * a.in_pW * Cs : nullptr;
  const FastDiv fcpp(hcpp), fwin(W_in);
  auto coords = [&](int i, int& c, int& iy, int& ix) -> bool {
    const int pix = fcpp.div(i);
    c = (i - pix * hcpp) * hcw;
    const int r = fwin.div(pix);
    iy = yb + r;
    ix = xb0 + (pix - r * W_in);
    bool ok = iy >= 0 && ix >= 0;
    if (dil > 1) {
      ok = ok && (iy % dil == 0) && (ix % dil == 0);
      iy /= dil;
      ix /= dil;
    }
    return ok && iy < a.H && ix < a.W;
  };
  auto halo8 = [&](int i) {
    int c, iy, ix;
    const bool ok = coords(i, c, iy, ix);
    if (cbase) return unpool_load8(xbase, cbase, a.in_pH, a.in_pW, Cs, iy, ix, c, ok);
    return load_bf16x8_if(ok, xbase + ((size_t)iy * a.W + ix) * Cs + c, xbase);
  };
  // weights -> LDS
  auto wload = [&](int i) {
    const int ks = i / (NTC * 64);   // compile-time power of two
    const int rem = i - ks * NTC * 64;
    const int nt = nt0 + (rem >> 6);
    const bool ok = nt < a.NT;
    return load_bf16x8_if(ok, a.wpk + ((size_t)(ks * a.NT + nt) * 64 + (rem & 63)) * 8, a.wpk);
  };
  auto wstore = [&](int i, const bf16x8& v) { *reinterpret_cast<bf16x8*>(wl + (size_t)i * 8) = v; };
  const int nw = KS * NTC * 64;
  auto build_tab = [&]() {   // k-chunk -> halo offset table
    const int KHW = a.KH * a.KW;
    const int cw = CS4 ? 4 : 8;
    for (int c = tid; c < ntab; c += 256) {
      const int k0 = c * cw;
      const int tap = k0 / Cs;
      int e = -1;
      if (tap < KHW) {
        const int ky = tap / a.KW;
        e = (ky * W_in + (tap - ky * a.KW)) * XP + (k0 - tap * Cs);
      }
      tab[c] = e;
    }
  };
  // Pooled input (dY = unpool(dP, codes)): load each pooled chunk ONCE and expand it into the
  // (up to) four full-resolution halo pixels of its window -- a quarter of the global loads of
  // rebuilding every pixel from its window (unpool_load8 per pixel).
  const bool pooled_in = !CS4 && cbase && dil == 1 && !(dbg & 16);
  const int Ha = 2 * a.in_pH, Wa = 2 * a.in_pW;
  const int y_lo = max(yb, 0), y_hi = min(yb + R_in, Ha);
  const int x_lo = max(xb0, 0), x_hi = min(xb0 + W_in, Wa);
  const bool pin = y_lo < y_hi && x_lo < x_hi;
  const int py0 = y_lo >> 1, npy = pin ? ((y_hi - 1) >> 1) - py0 + 1 : 0;
  const int px0 = x_lo >> 1, npx = pin ? ((x_hi - 1) >> 1) - px0 + 1 : 1;
  const int nq = npy * npx * hcpp;
  const FastDiv fnpx(npx);
  constexpr int UQ = 4;
  // halo pixels outside the pooled area (padding, odd edge) hold zeros: whole rows above /
  // below it and the columns left / right of it -- enumerated directly (the border is a few
  // hundred chunks; testing all R_in x W_in chunks cost two FastDivs each)
  auto zero_border = [&]() {
    const int ntop = min(R_in, max(0, -yb));
    const int nbot = min(R_in - ntop, max(0, yb + R_in - Ha));
    const int lc = min(W_in, max(0, -xb0)), rc = min(W_in - lc, max(0, xb0 + W_in - Wa));
    const int rowch = W_in * hcpp;
    for (int rr = 0; rr < ntop + nbot; ++rr) {         // workgroup-uniform
      const int r = rr < ntop ? rr : R_in - 1 - (rr - ntop);
      for (int i = tid; i < rowch; i += 256) {
        const int px = fcpp.div(i);
        *reinterpret_cast<bf16x8*>(xl + (size_t)(r * W_in + px) * XP + (i - px * hcpp) * 8) = zero_bf16x8();
      }
    }
    const int side = (lc + rc) * hcpp;
    const int nside = (R_in - ntop - nbot) * side;
    for (int i = tid; i < nside; i += 256) {
      const int m = i / side, j = i - m * side;
      const int cp = j / hcpp, ch = j - cp * hcpp;
      const int px = cp < lc ? cp : W_in - rc + (cp - lc);
      *reinterpret_cast<bf16x8*>(xl + (size_t)((ntop + m) * W_in + px) * XP + ch * 8) = zero_bf16x8();
    }
  };
  // one batch of UQ pooled chunks per thread: load (branch-free: clamped index, always loaded)
  // ... and expand into the window's pixels
  uint4 raw[UQ];
  uint2 cwd[UQ];
  int qy[UQ], qx[UQ], qc[UQ];
  auto pq_load = [&](int q0) {
#pragma unroll
    for (int u = 0; u < UQ; ++u) {
      const int q = min(q0 + u * 256, nq - 1);
      const int pp = fcpp.div(q);
      qc[u] = (q - pp * hcpp) * 8;
      const int ry = fnpx.div(pp);
      qy[u] = py0 + ry;
      qx[u] = px0 + (pp - ry * npx);
      const size_t o = ((size_t)qy[u] * a.in_pW + qx[u]) * Cs + qc[u];
      raw[u] = *reinterpret_cast<const uint4*>(xbase + o);
      cwd[u] = *reinterpret_cast<const uint2*>(cbase + o);
    }
  };
  auto pq_expand = [&](int q0) {
#pragma unroll
    for (int u = 0; u < UQ; ++u) {
      if (q0 + u * 256 >= nq) break;
#pragma unroll
      for (int pos = 0; pos < 4; ++pos) {
        const int y = 2 * qy[u] + (pos >> 1), x = 2 * qx[u] + (pos & 1);
        if (y < y_lo || y >= y_hi || x < x_lo || x >= x_hi) continue;
        uint32_t m[4];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const uint32_t w = h ? cwd[u].y : cwd[u].x;
          m[2 * h] = (((w & 0xFF) == (uint32_t)pos) ? 0x0000FFFFu : 0u) |
                     ((((w >> 8) & 0xFF) == (uint32_t)pos) ? 0xFFFF0000u : 0u);
          m[2 * h + 1] = ((((w >> 16) & 0xFF) == (uint32_t)pos) ? 0x0000FFFFu : 0u) |
                         ((((w >> 24) & 0xFF) == (uint32_t)pos) ? 0xFFFF0000u : 0u);
        }
        const uint4 v = {raw[u].x & m[0], raw[u].y & m[1], raw[u].z & m[2], raw[u].w & m[3]};
        *reinterpret_cast<uint4*>(xl + ((size_t)((y - yb) * W_in + (x - xb0)) * XP + qc[u])) = v;
      }
    }
  };
  // One-batch prologue (the co-scheduled dgrad of the RPV / MNIST stacks: the pooled halo is
  // one batch of chunks per thread): the weight vectors' loads go out first, the halo's right
  // behind them, and only then are the weights stored -- their wait (in-order vmcnt) does not
  // cover the halo loads, so the two global round trips overlap instead of running back to
  // back.  (Halo loads issued BEFORE the weights' were measured 3 us slower: the weights'
  // stores then wait behind them.)  dbg 32: the two-phase form (A/B, exact).
  const bool onebatch = dbg_stage && pooled_in && pin && !(dbg & (8 | 32)) && nq <= 256 * UQ && nw <= 8 * 256;
  if (onebatch) {
    auto fused = [&](auto wu) {
      constexpr int WU = decltype(wu)::value;
      bf16x8 wv[WU];
#pragma unroll
      for (int u = 0; u < WU; ++u) wv[u] = wload(min(tid + u * 256, nw - 1));
      pq_load(tid);
#pragma unroll
      for (int u = 0; u < WU; ++u)
        if (tid + u * 256 < nw) wstore(tid + u * 256, wv[u]);
      HALO_STAMP(1);
      build_tab();
      zero_border();
      pq_expand(tid);
    };
    const int wit = (nw + 255) >> 8;
    if (wit <= 2) fused(std::integral_constant<int, 2>{});
    else if (wit <= 4) fused(std::integral_constant<int, 4>{});
    else fused(std::integral_constant<int, 8>{});
  } else {
    if (dbg_stage && !(dbg & 8)) staged_copy<8, bf16x8>(nw, tid, 256, wload, wstore);
    HALO_STAMP(1);
    build_tab();
    // input halo -> LDS
    if (dbg_stage) {
      if (CS4) {
        staged_copy<8, bf16x4>(
            nch, tid, 256,
            [&](int i) {
              int c, iy, ix;
              const bool ok = coords(i, c, iy, ix);
              return load_bf16x4_if(ok, xbase + ((size_t)iy * a.W + ix) * 4, xbase);
            },
            [&](int i, const bf16x4& v) { *reinterpret_cast<bf16x4*>(xl + (size_t)i * 4) = v; });
      } else if (pooled_in) {
        if (!pin) zero_border();
        if (pin) {
          for (int q0 = tid; q0 < nq; q0 += 256 * UQ) {
            pq_load(q0);
            if (q0 == tid) zero_border();               // beside the first batch's loads
                                                        // (threads past nq: after the loop)
            pq_expand(q0);
          }
          if (tid >= nq) zero_border();
        }
      } else {
        staged_copy<8, bf16x8>(nch, tid, 256, halo8, [&](int i, const bf16x8& v) {
          int o = i * 8;
          if (XP != Cs) {
            const int pix = fcpp.div(i);
            o = pix * XP + (i - pix * hcpp) * 8;
          }
          *reinterpret_cast<bf16x8*>(xl + o) = v;
        });
      }
    }
  }
  HALO_STAMP(2);
  __syncthreads();
  HALO_STAMP(3);

  const int wave = tid >> 6, lane = tid & 63, r = lane & 15, g = lane >> 4;
  const int rows = min(R, a.Ho - oy0);
  const int nwin = a.pool ? (rows >> 1) * a.Wp : 0;
  const int npix = rows * a.Wo;
  const int ntiles = a.pool ? (nwin + 3) / 4 : (npix + 15) / 16;
  const uint32_t step = a.st ? (uint32_t)a.st->t : 0u;

  const FastDiv fwp(a.Wp > 0 ? a.Wp : 1), fwo(a.Wo);
  // per-wave epilogue scratch [16 rows][NTC*16] fp32, after the 16-B aligned halo image
  constexpr int EPW = TM * 16 * 2 * NTC * 16 / 4;   // floats per wave: TM*16 rows x LDC bf16
  float* ep = reinterpret_cast<float*>(xl + (((size_t)R_in * W_in * XP + 7) & ~(size_t)7)) + wave * EPW;
  const size_t qbase = ((size_t)b * a.Hp + (oy0 >> 1)) * a.Wp;
  for (int tb = wave * TM; tb < ntiles; tb += 4 * TM) {
    bool rv[TM];
    const bf16* xrow[TM];
#pragma unroll
    for (int t = 0; t < TM; ++t) {
      const int tile = tb + t;
      int ry, rx;
      if (a.pool) {
        const int w = tile * 4 + (r >> 2);
        rv[t] = w < nwin;
        const int wi = rv[t] ? w : 0;
        const int pyl = fwp.div(wi);
        ry = 2 * pyl + ((r >> 1) & 1);
        rx = 2 * (wi - pyl * a.Wp) + (r & 1);
      } else {
        const int p = tile * 16 + r;
        rv[t] = p < npix;
        const int pi = rv[t] ? p : 0;
        ry = fwo.div(pi);
        rx = pi - ry * a.Wo;
      }
      xrow[t] = xl + ((size_t)(ry * s) * W_in + rx * s) * XP;
    }
    f32x4 acc[TM][NTC];
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int nt = 0; nt < NTC; ++nt) acc[t][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    // Fast k loop (kpipe; 8-channel-aligned input with Cs % 32 == 0, the co-scheduled dgrad
    // of the RPV / MNIST stacks): a k-step's tap is wave-uniform (k = 32 ks + 8 g lies in
    // one tap), so its halo offset is scalar arithmetic -- no per-step table lookup, whose
    // LDS round trip the A-fragment reads depended on -- and the loop is software-pipelined:
    // step ks + 1's A / B fragments are requested before step ks's MFMAs issue.  Rows past
    // the block read pixel 0 (finite data, never stored); same k order as the table loop.
    const bool kfast = !CS4 && a.kpipe && (Cs & 31) == 0 && dbg_mfma;
    if (kfast) {
      const int cpk = Cs >> 5;                      // k-steps per tap
      const int g8 = 8 * g;
      auto kbase = [&](int ks) -> int {
        const int tap = ks / cpk;
        const int ky = tap / a.KW;
        return __builtin_amdgcn_readfirstlane((ky * W_in + (tap - ky * a.KW)) * XP + (ks - tap * cpk) * 32);
      };
      bf16x8 af[2][TM], bw[2][NTC];
      auto load_k = [&](int ks, bf16x8* av, bf16x8* bv) {
        const int kb = kbase(ks) + g8;
#pragma unroll
        for (int t = 0; t < TM; ++t) av[t] = *reinterpret_cast<const bf16x8*>(xrow[t] + kb);
#pragma unroll
        for (int nt = 0; nt < NTC; ++nt)
          bv[nt] = *reinterpret_cast<const bf16x8*>(wl + ((size_t)(ks * NTC + nt) * 64 + lane) * 8);
      };
      auto mma_k = [&](const bf16x8* av, const bf16x8* bv) {
#pragma unroll
        for (int nt = 0; nt < NTC; ++nt)
#pragma unroll
          for (int t = 0; t < TM; ++t) acc[t][nt] = mfma16(av[t], bv[nt], acc[t][nt]);
      };
      load_k(0, af[0], bw[0]);
      int ks = 0;
      for (; ks + 2 <= KS; ks += 2) {
        load_k(ks + 1, af[1], bw[1]);
        __builtin_amdgcn_sched_barrier(0);
        mma_k(af[0], bw[0]);
        __builtin_amdgcn_sched_barrier(0);
        if (ks + 2 < KS) load_k(ks + 2, af[0], bw[0]);
        __builtin_amdgcn_sched_barrier(0);
        mma_k(af[1], bw[1]);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (ks < KS) mma_k(af[0], bw[0]);
    }
    for (int kc = 0; kc < ((dbg_mfma && !kfast) ? KS : 0); kc += KCH) {
      int e0[KCH], e1[KCH];
#pragma unroll
      for (int u = 0; u < KCH; ++u) {
        const bool in = kc + u < KS;
        if (CS4) {
          e0[u] = in ? tab[((kc + u) * 4 + g) * 2] : -1;
          e1[u] = in ? tab[((kc + u) * 4 + g) * 2 + 1] : -1;
        } else {
          e0[u] = in ? tab[(kc + u) * 4 + g] : -1;
        }
      }
#pragma unroll
      for (int u = 0; u < KCH; ++u) {
        if (kc + u < KS) {   // wave-uniform
          bf16x8 af[TM];
#pragma unroll
          for (int t = 0; t < TM; ++t) {
            if (!CS4) {
              af[t] = *reinterpret_cast<const bf16x8*>((rv[t] && e0[u] >= 0) ? xrow[t] + e0[u] : zl);
            } else {
              const bf16x4 v0 = *reinterpret_cast<const bf16x4*>((rv[t] && e0[u] >= 0) ? xrow[t] + e0[u] : zl);
              const bf16x4 v1 = *reinterpret_cast<const bf16x4*>((rv[t] && e1[u] >= 0) ? xrow[t] + e1[u] : zl);
              af[t] = __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
            }
          }
#pragma unroll
          for (int nt = 0; nt < NTC; ++nt) {
            const bf16x8 bfr =
                *reinterpret_cast<const bf16x8*>(wl + ((size_t)((kc + u) * NTC + nt) * 64 + lane) * 8);
#pragma unroll
            for (int t = 0; t < TM; ++t) acc[t][nt] = mfma16(af[t], bfr, acc[t][nt]);
          }
        }
      }
    }

    if (tb == 0) {
      asm volatile("" ::"v"(acc[0][0][0]));
      HALO_STAMP(4);
    }
    if (!dbg_store) {
#pragma unroll
      for (int t = 0; t < TM; ++t)
#pragma unroll
        for (int nt = 0; nt < NTC; ++nt)
          asm volatile("" ::"v"(acc[t][nt][0]), "v"(acc[t][nt][1]), "v"(acc[t][nt][2]), "v"(acc[t][nt][3]));
      continue;
    }
    // Epilogue through the wave's LDS scratch: lanes write their MFMA-layout results, then
    // re-read them as 8-channel vectors so every global store is 16 bytes.  The forward
    // epilogue stages all TM tiles of the pass first (final bf16 values + pool codes), so
    // one copy loop writes TM*16 pixels / TM*4 windows with all lanes busy.
    const int LDC = NTC * 16;
    const int csh = (mode == 1 ? a.bt.pCs : a.Cs_out) - nt0 * 16;   // channels this WG owns
    const int C = csh < LDC ? csh : LDC;
    const int cch = C >> 3;                                            // 8-channel chunks
    const FastDiv fcch(cch > 0 ? cch : 1);
    if (mode == 0 && a.pool) {
      bf16* epb = reinterpret_cast<bf16*>(ep);                // [TM*4 windows][LDC]
      uint8_t* epc = reinterpret_cast<uint8_t*>(epb + TM * 4 * LDC);
#pragma unroll
      for (int t = 0; t < TM; ++t) {
        const size_t q = qbase + (tb + t) * 4 + g;
#pragma unroll
        for (int nt = 0; nt < NTC; ++nt) {
          const int n = (nt0 + nt) * 16 + r;
          float best = 0.f;
          int code = 0;
          if (n < a.N) {
            const float bv = a.bias ? a.bias[n] : 0.f;
            best = -3.4e38f;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              float v = acc[t][nt][j] + bv;
              if (a.relu) v = fmaxf(v, 0.f);
              if (v > best) { best = v; code = j; }
            }
            if (a.drop_thr)
              best = dropout_keep((uint32_t)(q * a.N + n), a.seed, a.stream_id, step, a.drop_thr) ? best * a.drop_scale
                                                                                                 : 0.f;
          }
          epb[(t * 4 + g) * LDC + nt * 16 + r] = f2bf(best);
          epc[(t * 4 + g) * LDC + nt * 16 + r] = (uint8_t)code;
        }
      }
      __builtin_amdgcn_wave_barrier();
      const int nw = max(0, min(TM * 4, nwin - tb * 4));
      for (int c = lane; c < nw * cch; c += 64) {
        const int win = fcch.div(c), c8 = c - win * cch;
        const size_t o = (qbase + tb * 4 + win) * a.Cs_out + nt0 * 16 + c8 * 8;
        *reinterpret_cast<uint4*>(a.out + o) = *reinterpret_cast<const uint4*>(epb + win * LDC + c8 * 8);
        *reinterpret_cast<uint2*>(a.code + o) = *reinterpret_cast<const uint2*>(epc + win * LDC + c8 * 8);
      }
      __builtin_amdgcn_wave_barrier();
    } else {
      // unpooled forward and dgrad (mode 1): stage the TM tiles as bf16, then one copy loop
      // The staged rows are XOR-swizzled by 16-byte chunk: chunk c of row q sits at chunk
      // c ^ (((q >> 2) << 1) & (LDC / 8 - 1)).  A store instruction's four lane groups write
      // rows 4 apart, which unswizzled map to the same banks (4-way conflicts at LDC 64).
      bf16* epb = reinterpret_cast<bf16*>(ep);                // [TM*16 pixels][LDC]
      const bool fwd = mode == 0;
      constexpr int CHM = NTC * 2 - 1;                        // chunk-index mask (LDC / 8 - 1)
      // the block is whole output rows: pixel p of the block is output pixel mrow0 + p
      const size_t mrow0 = ((size_t)b * a.Ho + oy0) * a.Wo;
      float bvn[NTC];
#pragma unroll
      for (int nt = 0; nt < NTC; ++nt) {
        const int n = (nt0 + nt) * 16 + r;
        bvn[nt] = (fwd && a.bias && n < a.N) ? a.bias[n] : 0.f;
      }
#pragma unroll
      for (int t = 0; t < TM; ++t) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int q = t * 16 + g * 4 + j;
          const int sw = ((q >> 2) << 1) & CHM;
          size_t m = 0;
          if (fwd && a.drop_thr) {
            const int p = (tb + t) * 16 + g * 4 + j;
            m = mrow0 + (size_t)(p < npix ? p : 0);
          }
#pragma unroll
          for (int nt = 0; nt < NTC; ++nt) {
            const int n = (nt0 + nt) * 16 + r;
            float x = acc[t][nt][j];
            if (fwd) {
              x = 0.f;
              if (n < a.N) {
                x = acc[t][nt][j] + bvn[nt];
                if (a.relu) x = fmaxf(x, 0.f);
                if (a.drop_thr)
                  x = dropout_keep((uint32_t)(m * a.N + n), a.seed, a.stream_id, step, a.drop_thr) ? x * a.drop_scale
                                                                                                 : 0.f;
              }
            }
            const int col = nt * 16 + r;
            epb[q * LDC + (((col >> 3) ^ sw) << 3) + (col & 7)] = f2bf(x);
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
      const int np = max(0, min(TM * 16, npix - tb * 16));
      for (int c = lane; c < np * cch; c += 64) {
        const int pr = fcch.div(c), c8 = c - pr * cch;
        const size_t m = mrow0 + (size_t)(tb * 16 + pr);
        const bf16x8 val = *reinterpret_cast<const bf16x8*>(epb + pr * LDC + ((c8 ^ (((pr >> 2) << 1) & CHM)) << 3));
        if (fwd) {
          *reinterpret_cast<bf16x8*>(a.out + m * a.Cs_out + nt0 * 16 + c8 * 8) = val;
        } else {
          float v[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] = bf2f(val[k]);
          bwd_through_store8(a.bt, m, nt0 * 16 + c8 * 8, v, step);
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
    if (tb == 0) HALO_STAMP(5);
  }
  HALO_STAMP(6);
}

