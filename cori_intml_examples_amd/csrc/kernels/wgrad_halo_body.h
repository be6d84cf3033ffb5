// Body of the halo-staged weight-gradient kernel (see wgrad_halo.hip for the design), as
// a device function of the block index (co-scheduled with dgrad by dual_halo.hip).
#pragma once
#include "bwd_through.h"

// a staged X-halo chunk and its LDS element offset
struct XChunk4 { bf16x4 v; int o; };
struct XChunk8 { bf16x8 v; int o; };

__device__ __forceinline__ bf16x4 tr_read_h(const bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS_PTR(bf16x4, p));
}

// Each wave owns MTW m-tiles (w, w+4, ...) x all NTT n-tiles of the workgroup, so per
// k-step it reads NTT B fragments + MTW A fragments for MTW*NTT MFMAs.
// PIPE: software-pipelined block loop (more VGPRs; pays off for workgroups that stream many
// blocks, not for grids that already hide the latency with many resident workgroups).
#define WH_STAMP(i)                                                                     \
  if (INSTR && a.ts2 && threadIdx.x == 0 && (i) < 16) a.ts2[(size_t)blockIdx.x * 16 + (i)] = wall_clock64();

// image b of the wgrad input: the activation buffer, or (prologue-free step, first layer)
// dataset row xidx[b] of the bound dataset
__device__ __forceinline__ const bf16* wg_xbase(const WgradArgs& a, int b) {
  if (a.xidx) return reinterpret_cast<const bf16*>(a.xst->data_x) + (size_t)a.xidx[b] * a.xst->data_R;
  return a.x + (size_t)b * a.H * a.W * a.Cs_in;
}

// row stride (floats) of a wave's 16x16 write-through staging square: rows 4 apart land
// 16 banks apart (conflict-free lane writes), rows stay 16-byte aligned for the vector read
#define WH_SQ 20

// INSTR: the ablation switches (dbg) and diagnostics stamps (a.ts2) are compiled in (the
// co-scheduled dual launch instantiates false)
template <int MTW, int NTT, bool CS4, bool PIPE, bool INSTR = true>
__device__ __forceinline__ void wgrad_halo_body(const WgradArgs& a, const int MT, const int bx, const int by,
                                                const int bz, char* smem) {
  const int dbg = INSTR ? a.dbg : 0;
  const int R = a.R, s = a.stride, Cs = a.Cs_in;
  const int W_in = (a.Wo - 1) * s + a.KW;
  const int R_in = (R - 1) * s + a.KH;
  const int npb = R * a.Wo;                         // pixels per full block
  const int npb32 = (npb + 31) & ~31;
  // LDS layout (bank-conflict model, models/lds_layout.py): X-halo pixel stride XP and row
  // stride XR (pixels), dY row stride ldb; 0 = dense
  const int XP = a.xpix ? a.xpix : Cs, XR = a.xrow ? a.xrow : W_in;
  const int ldb = a.dyld ? a.dyld : NTT * 16 + 8;   // dY LDS row stride (elements)
  bf16* xl = reinterpret_cast<bf16*>(smem);
  const int x_elems = ((R_in * XR * XP) + 7) & ~7;
  bf16* dyl = xl + x_elems;
  bf16* zl = dyl + (size_t)npb32 * ldb;             // 64 B of zeros
  bf16* ol = zl + 32;                               // 64 B of bf16 ones (the bias tile's A operand)
  int* ktab = reinterpret_cast<int*>(zl + 64);      // [MT*4] halo offsets of k column blocks

  // (wave via readfirstlane: the per-m-tile conditions below are then wave-uniform scalars --
  // as per-lane values they turned the k loop into exec-masked blocks, one lgkmcnt(0) per tile)
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63, i = lane & 15,
            g = lane >> 4;
  const int mt0 = bz * MT;
  const int nt0 = by * NTT;
  const int KHW = a.KH * a.KW;
  const bool do_bias = a.bslab != nullptr && bz == 0;
  const int MTb = MT + (do_bias ? 1 : 0);          // pseudo m-tile MT = bias (ones operand)

  WH_STAMP(0);
  if (tid < 32) reinterpret_cast<uint32_t*>(zl)[tid] = tid < 16 ? 0u : 0x3F803F80u;
  for (int c = tid; c < MT * 4; c += 256) {
    const int k = (mt0 + c / 4) * 16 + 4 * (c & 3);
    const int tap = k / Cs;
    int e = -1;
    if (tap < KHW && mt0 + c / 4 < a.Ktiles) {
      const int ky = tap / a.KW;
      e = (ky * XR + (tap - ky * a.KW)) * XP + (k - tap * Cs);
    }
    ktab[c] = e;
  }
  __syncthreads();
  WH_STAMP(8);

  // per-wave m-tile descriptors (constant over blocks and k-steps).  Wave-uniform state as two
  // scalars -- the wave's valid m-tiles are u < nval, the bias tile is u == ubias -- rather than
  // per-u flag arrays (each a 64-bit lane mask in SGPRs: they pushed the dual kernel's SGPR spills)
  int ko[MTW];
  const int nval = max(0, min(MTW, (MTb - wave + 3) >> 2));
  const int ubias = (do_bias && MT >= wave && ((MT - wave) & 3) == 0) ? (MT - wave) >> 2 : -1;
#pragma unroll
  for (int u = 0; u < MTW; ++u) {
    const int mt = wave + 4 * u;
    ko[u] = (mt < MT) ? ktab[mt * 4 + (i & 3)] : -1;
  }

  f32x4 acc[MTW][NTT];
#pragma unroll
  for (int u = 0; u < MTW; ++u)
#pragma unroll
    for (int v = 0; v < NTT; ++v) acc[u][v] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nrb = (a.Ho + R - 1) / R;
  const int nblocks = a.B * nrb;
  const int blk0 = bx * a.blocks_per_split;
  const int blk1 = min(nblocks, blk0 + a.blocks_per_split);
  const int cw = CS4 ? 4 : 8;
  const int cpp = Cs / cw;
  const int cpr = NTT * 2;
  const int nch_x = R_in * W_in * cpp;              // X-halo chunks per block
  const int nch_y = npb32 * cpr;                    // dY chunks per block
  const FastDiv fcpp(cpp), fwin(W_in), fcpr(cpr), fwo(a.Wo);

  const bool dbg_stage = !(dbg & 1);
  // Pooled dY (dP + argmax codes) over whole even blocks: stage each pooled chunk ONCE and
  // expand it into its 2x2 window's pixel rows in LDS (a quarter of the global loads of a
  // per-pixel unpool; every LDS dY element of the block is written, zeros included).
  const int hw = a.Wo >> 1;
  // (pipelined path only: in the plain path its extra registers cost occupancy -- measured)
  const bool pexp = PIPE && a.dy_code && !(dbg & 16) && (R & 1) == 0 && a.Ho % R == 0 && (a.Wo & 1) == 0 &&
                    npb32 == npb && a.NT % NTT == 0 && a.NT * 16 <= a.Cs_dy && 2 * a.dHp >= a.Ho &&
                    2 * a.dWp >= a.Wo;
  const int nq = (R >> 1) * hw * cpr;               // pooled dY chunks per block
  const FastDiv fhw(hw > 0 ? hw : 1);
  // pooled chunk q of the block starting at conv row oy0 -> global dP offset (in elements)
  auto pq_off = [&](int q, int b, int oy0) -> size_t {
    const int p2 = fcpr.div(q), ch = q - p2 * cpr;
    const int ry = fhw.div(p2);
    const int wy = (oy0 >> 1) + ry, wx = p2 - ry * hw;
    return (((size_t)b * a.dHp + wy) * a.dWp + wx) * a.Cs_dy + nt0 * 16 + ch * 8;
  };
  // write pooled chunk q (dP values v, codes cw) to the 4 pixels of its window
  // ... the same from the chunk's precomputed LDS offset (window's top-left pixel row)
  auto pq_store_at = [&](int dst, const uint4& v, const uint2& cw) {
#pragma unroll
    for (int pos = 0; pos < 4; ++pos) {
      uint32_t m[4];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t w = h ? cw.y : cw.x;
        m[2 * h] = (((w & 0xFF) == (uint32_t)pos) ? 0x0000FFFFu : 0u) |
                   ((((w >> 8) & 0xFF) == (uint32_t)pos) ? 0xFFFF0000u : 0u);
        m[2 * h + 1] = ((((w >> 16) & 0xFF) == (uint32_t)pos) ? 0x0000FFFFu : 0u) |
                       ((((w >> 24) & 0xFF) == (uint32_t)pos) ? 0xFFFF0000u : 0u);
      }
      *reinterpret_cast<uint4*>(dyl + dst + ((pos >> 1) * a.Wo + (pos & 1)) * ldb) =
          uint4{v.x & m[0], v.y & m[1], v.z & m[2], v.w & m[3]};
    }
  };
  auto pq_store = [&](int q, const uint4& v, const uint2& cw) {
    const int p2 = fcpr.div(q), ch = q - p2 * cpr;
    const int ry = fhw.div(p2);
    const int p00 = (2 * ry) * a.Wo + 2 * (p2 - ry * hw);
#pragma unroll
    for (int pos = 0; pos < 4; ++pos) {
      uint32_t m[4];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t w = h ? cw.y : cw.x;
        m[2 * h] = (((w & 0xFF) == (uint32_t)pos) ? 0x0000FFFFu : 0u) |
                   ((((w >> 8) & 0xFF) == (uint32_t)pos) ? 0xFFFF0000u : 0u);
        m[2 * h + 1] = ((((w >> 16) & 0xFF) == (uint32_t)pos) ? 0x0000FFFFu : 0u) |
                       ((((w >> 24) & 0xFF) == (uint32_t)pos) ? 0xFFFF0000u : 0u);
      }
      const int p = p00 + (pos >> 1) * a.Wo + (pos & 1);
      *reinterpret_cast<uint4*>(dyl + (size_t)p * ldb + ch * 8) =
          uint4{v.x & m[0], v.y & m[1], v.z & m[2], v.w & m[3]};
    }
  };

  // MFMA reduction over the staged block's npix pixels
  // per-lane pixel offsets within a 32-pixel k-step (the kperm bijection, see below)
  const int dP0 = ((a.kperm & 1) ? 4 * g : 8 * g) + (i >> 2), dP1 = dP0 + ((a.kperm & 1) ? 16 : 4);
  auto mma_block = [&](const int npix) {
      const int nks = (dbg & 2) ? 0 : (npix + 31) >> 5;
      // Row-aligned fast path (output width % 32 == 0, whole k-steps): a k-step's 32 pixels
      // lie in ONE output row, so the halo offset is a scalar per k-step plus a per-lane
      // constant -- no per-step division or clamping (same pixels, same k order).  One MFMA
      // body for both paths (a second copy doubled the accumulators' AGPRs and halved the
      // occupancy of the dual kernels).
      const bool rowal = (a.Wo & 31) == 0 && (npix & 31) == 0 && !(a.kperm & 2);
      const int la0 = dP0 * s * XP, la1 = dP1 * s * XP;
      int y = 0, x0 = 0;
      // (a row-divisor form of the scalar k-step base -- widths dividing 32, RPV conv2's 16-wide
      // rows -- measured equal, 0.0999-0.1003 vs 0.0999-0.1004 ms/step (profiles/r6_wgrad_ab.txt),
      // and cost the dual kernels SGPR spills: not kept)
      // k-step ks's fragments (the row-aligned path's scalar position (y, x0) advances)
      auto frags = [&](const int ks, bf16x8 (&afr)[MTW], bf16x8 (&bfr)[NTT]) {
        // per-lane pixel rows of the two transposed reads (h = 0, 1).  MFMA k index 8g + j
        // stands for pixel 4g + j (j < 4) / 16 + 4g + j - 4 (j >= 4) of the k-step -- the same
        // bijection for both operands, so a 32-lane half reads 8 CONSECUTIVE pixels (the
        // layout's bank-conflict-free pattern) instead of two runs 8 pixels apart
        const int P0 = ks * 32 + dP0;
        const int P1 = ks * 32 + dP1;
        int off0, off1;
        if (rowal) {
          const int base = __builtin_amdgcn_readfirstlane(((y * s) * XR + x0 * s) * XP);
          if ((x0 += 32) == a.Wo) { x0 = 0; ++y; }
          off0 = base + la0, off1 = base + la1;
        } else {
          const int q0 = min(P0, npix - 1), q1 = min(P1, npix - 1);
          const int y0 = fwo.div(q0), y1 = fwo.div(q1);
          off0 = ((y0 * s) * XR + (q0 - y0 * a.Wo) * s) * XP;
          off1 = ((y1 * s) * XR + (q1 - y1 * a.Wo) * s) * XP;
        }
        const bf16* pbrow = dyl + (size_t)P0 * ldb + 4 * (i & 3);
  #pragma unroll
        for (int v = 0; v < NTT; ++v) {
          const bf16* pb = pbrow + v * 16;
          bfr[v] = __builtin_shufflevector(tr_read_h(pb), tr_read_h(pb + (P1 - P0) * ldb), 0, 1, 2, 3, 4, 5, 6, 7);
        }
  #pragma unroll
        for (int u = 0; u < MTW; ++u) {
          // branch-free: padding k columns read the zero block, the bias tile the ones block
          const bf16* pz = u == ubias ? ol : zl;
          const bf16* pa0 = ko[u] >= 0 ? xl + off0 + ko[u] : pz;
          const bf16* pa1 = ko[u] >= 0 ? xl + off1 + ko[u] : pz;
          afr[u] = __builtin_shufflevector(tr_read_h(pa0), tr_read_h(pa1), 0, 1, 2, 3, 4, 5, 6, 7);
        }
      };
      auto mmas = [&](const bf16x8 (&afr)[MTW], const bf16x8 (&bfr)[NTT]) {
  #pragma unroll
        for (int u = 0; u < MTW; ++u)
          if (u < nval) {
  #pragma unroll
            for (int v = 0; v < NTT; ++v) acc[u][v] = mfma16(afr[u], bfr[v], acc[u][v]);
          }
      };
      for (int ks = 0; ks < nks; ++ks) {
        bf16x8 bfr[NTT], afr[MTW];
        frags(ks, afr, bfr);
        mmas(afr, bfr);
      }
  };

  // Software pipeline over the workgroup's blocks (when one block's staging fits WH_PX + WH_PY
  // chunks per thread): block blk+1's X-halo and dY chunks are loaded into registers while
  // block blk's MFMAs run, and go to LDS after the barrier that retires blk's readers --
  // the staging loads' latency, not the MFMAs, was the per-block cost.
  constexpr int WH_PX = 4, WH_PY = 4;
  if (PIPE && dbg_stage && nch_x <= WH_PX * 256 && (pexp ? nq : nch_y) <= WH_PY * 256) {
    uint4 xr[WH_PX], yr[WH_PY];
    int xa[WH_PX];
    uint2 yc[WH_PY];
    uint32_t yp[WH_PY];
    // Per-lane staging constants, the same for every block: a chunk's halo row / column /
    // channel, its LDS offset and its source offset from the block's first input row (the
    // block only moves the row base), and the pooled dY chunk's source offset from the
    // block's first pooled row and LDS offset -- the per-block fetch is adds and compares,
    // not FastDiv chains.
    int xrow[WH_PX], xoff[WH_PX], qoff[WH_PY], qdst[WH_PY];
    uint32_t xcol = 0;                  // bit u: the chunk's column lies inside the image
#pragma unroll
    for (int u = 0; u < WH_PX; ++u) {
      const int idx = min(tid + u * 256, nch_x - 1);
      const int pix = fcpp.div(idx), c = (idx - pix * cpp) * cw;
      const int r = fwin.div(pix), px = pix - r * W_in;
      const int ix = px - a.pad_l;
      xa[u] = (r * XR + px) * XP + c;
      xrow[u] = r;
      xoff[u] = (r * a.W + ix) * Cs + c;
      if (ix >= 0 && ix < a.W) xcol |= 1u << u;
    }
    if (pexp) {
#pragma unroll
      for (int u = 0; u < WH_PY; ++u) {
        const int q = min(tid + u * 256, nq - 1);
        const int p2 = fcpr.div(q), ch = q - p2 * cpr;
        const int ry = fhw.div(p2), wx = p2 - ry * hw;
        qoff[u] = (ry * a.dWp + wx) * a.Cs_dy + nt0 * 16 + ch * 8;
        qdst[u] = ((2 * ry) * a.Wo + 2 * wx) * ldb + ch * 8;
      }
    }
    auto fetch = [&](const int blk) {
      const int b = blk / nrb, oy0 = (blk - b * nrb) * R;
      const int npix = min(R, a.Ho - oy0) * a.Wo;
      const int yb = oy0 * s - a.pad_t;
      const bf16* xbase = wg_xbase(a, b);
      const bf16* xrow0 = xbase + (ptrdiff_t)yb * a.W * Cs;         // may point before xbase
#pragma unroll
      for (int u = 0; u < WH_PX; ++u) {
        const int iy = yb + xrow[u];
        const bool ok = ((xcol >> u) & 1u) && iy >= 0 && iy < a.H;
        const bf16* src = ok ? xrow0 + xoff[u] : xbase;
        if (CS4) {
          const uint2 v = *reinterpret_cast<const uint2*>(src);
          xr[u] = uint4{ok ? v.x : 0u, ok ? v.y : 0u, 0u, 0u};
        } else {
          const uint4 v = *reinterpret_cast<const uint4*>(src);
          xr[u] = ok ? v : uint4{0u, 0u, 0u, 0u};
        }
      }
      if (pexp) {
        const size_t qb = (((size_t)b * a.dHp + (oy0 >> 1)) * a.dWp) * a.Cs_dy;
#pragma unroll
        for (int u = 0; u < WH_PY; ++u) {
          const size_t o = qb + qoff[u];
          yr[u] = *reinterpret_cast<const uint4*>(a.dy + o);
          yc[u] = *reinterpret_cast<const uint2*>(a.dy_code + o);
        }
        return;
      }
      const size_t boff = (size_t)b * a.dHp * a.dWp * a.Cs_dy;
#pragma unroll
      for (int u = 0; u < WH_PY; ++u) {
        const int idx = min(tid + u * 256, nch_y - 1);
        const int p = fcpr.div(idx);
        const int n0 = nt0 * 16 + (idx - p * cpr) * 8;
        bool ok = p < npix && n0 < a.Cs_dy;
        const int pp = ok ? p : 0;
        const int pyl = fwo.div(pp);
        const int oy = oy0 + pyl, ox = pp - pyl * a.Wo;
        size_t o;
        if (a.dy_code) {   // pooled: dP + argmax code of the window (unpool on commit)
          const int wy = oy >> 1, wx = ox >> 1;
          ok = ok && wy < a.dHp && wx < a.dWp;
          o = ok ? boff + ((size_t)wy * a.dWp + wx) * a.Cs_dy + n0 : 0;
          yc[u] = *reinterpret_cast<const uint2*>(a.dy_code + o);
          yp[u] = ok ? (uint32_t)(((oy & 1) << 1) | (ox & 1)) : 0xFFu;
        } else {
          o = ok ? (((size_t)b * a.Ho + oy) * a.Wo + ox) * a.Cs_dy + n0 : 0;
          yc[u] = uint2{0u, 0u};
          yp[u] = ok ? 0u : 0xFFu;
        }
        yr[u] = *reinterpret_cast<const uint4*>(a.dy + o);
      }
    };
    auto commit = [&]() {
#pragma unroll
      for (int u = 0; u < WH_PX; ++u) {
        const int idx = tid + u * 256;
        if (idx >= nch_x) continue;
        if (CS4) *reinterpret_cast<uint2*>(xl + xa[u]) = uint2{xr[u].x, xr[u].y};
        else *reinterpret_cast<uint4*>(xl + xa[u]) = xr[u];
      }
      if (pexp) {
#pragma unroll
        for (int u = 0; u < WH_PY; ++u)
          if (tid + u * 256 < nq) pq_store_at(qdst[u], yr[u], yc[u]);
        return;
      }
#pragma unroll
      for (int u = 0; u < WH_PY; ++u) {
        const int idx = tid + u * 256;
        if (idx >= nch_y) continue;
        uint4 v = yr[u];
        const uint32_t pos = yp[u];
        if (a.dy_code) {   // keep element j iff its argmax code is this pixel's window position
          uint32_t m[4];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const uint32_t w = h ? yc[u].y : yc[u].x;
            m[2 * h] = (((w & 0xFF) == pos) ? 0x0000FFFFu : 0u) | ((((w >> 8) & 0xFF) == pos) ? 0xFFFF0000u : 0u);
            m[2 * h + 1] =
                ((((w >> 16) & 0xFF) == pos) ? 0x0000FFFFu : 0u) | ((((w >> 24) & 0xFF) == pos) ? 0xFFFF0000u : 0u);
          }
          v = uint4{v.x & m[0], v.y & m[1], v.z & m[2], v.w & m[3]};
        } else if (pos) {
          v = uint4{0u, 0u, 0u, 0u};
        }
        const int p = fcpr.div(idx);
        *reinterpret_cast<uint4*>(dyl + (size_t)p * ldb + (idx - p * cpr) * 8) = v;
      }
    };
    WH_STAMP(9);
    fetch(blk0);
    WH_STAMP(1);
    for (int blk = blk0; blk < blk1; ++blk) {
      const int b = blk / nrb, oy0 = (blk - b * nrb) * R;
      const int npix = min(R, a.Ho - oy0) * a.Wo;
      if (blk != blk0) __syncthreads();   // previous block's readers are done
      commit();
      __syncthreads();
      WH_STAMP(2 + 2 * (blk - blk0));
      fetch(min(blk + 1, blk1 - 1));      // next block's loads fly during this block's MFMAs
      mma_block(npix);
      if (INSTR && a.ts2) asm volatile("" ::"v"(acc[0][0][0]));
      WH_STAMP(3 + 2 * (blk - blk0));
    }
  } else {
    for (int blk = blk0; blk < blk1; ++blk) {
      const int b = blk / nrb;
      const int oy0 = (blk - b * nrb) * R;
      const int rows = min(R, a.Ho - oy0);
      const int npix = rows * a.Wo;
      if (blk != blk0) __syncthreads();   // previous block's readers are done
      if (dbg_stage) {   // X halo
        const int yb = oy0 * s - a.pad_t, xb0 = -a.pad_l;
        const bf16* xbase = wg_xbase(a, b);
        auto coords = [&](int idx, int& c, int& iy, int& ix) -> bool {
          const int pix = fcpp.div(idx);
          c = (idx - pix * cpp) * cw;
          const int r = fwin.div(pix);
          iy = yb + r;
          ix = xb0 + (pix - r * W_in);
          return iy >= 0 && ix >= 0 && iy < a.H && ix < a.W;
        };
        // (the LDS offset rides along with the loaded value: the coordinates are computed
        // once, in the load, instead of again in the store)
        if (CS4) {
          staged_copy<8, XChunk4>(
              nch_x, tid, 256,
              [&](int idx) {
                int c, iy, ix;
                const bool ok = coords(idx, c, iy, ix);
                return XChunk4{load_bf16x4_if(ok, xbase + ((size_t)iy * a.W + ix) * 4, xbase),
                               ((iy - yb) * XR + (ix - xb0)) * XP + c};
              },
              [&](int, const XChunk4& v) { *reinterpret_cast<bf16x4*>(xl + v.o) = v.v; });
        } else {
          staged_copy<8, XChunk8>(
              nch_x, tid, 256,
              [&](int idx) {
                int c, iy, ix;
                const bool ok = coords(idx, c, iy, ix);
                return XChunk8{load_bf16x8_if(ok, xbase + ((size_t)iy * a.W + ix) * Cs + c, xbase),
                               ((iy - yb) * XR + (ix - xb0)) * XP + c};
              },
              [&](int, const XChunk8& v) { *reinterpret_cast<bf16x8*>(xl + v.o) = v.v; });
        }
      }
      if (dbg_stage && pexp) {   // dY rows from pooled chunks, each loaded once
        constexpr int UQ = 4;
        for (int q0 = tid; q0 < nq; q0 += 256 * UQ) {
          uint4 v[UQ];
          uint2 cw[UQ];
#pragma unroll
          for (int u = 0; u < UQ; ++u) {
            const size_t o = pq_off(min(q0 + u * 256, nq - 1), b, oy0);
            v[u] = *reinterpret_cast<const uint4*>(a.dy + o);
            cw[u] = *reinterpret_cast<const uint2*>(a.dy_code + o);
          }
#pragma unroll
          for (int u = 0; u < UQ; ++u)
            if (q0 + u * 256 < nq) pq_store(q0 + u * 256, v[u], cw[u]);
        }
      } else if (dbg_stage) {   // dY rows (rebuilt from pooled dP + codes when the conv is pooled)
        const size_t boff = (size_t)b * a.dHp * a.dWp * a.Cs_dy;
        staged_copy<8, bf16x8>(
            nch_y, tid, 256,
            [&](int idx) {
              const int p = fcpr.div(idx);
              const int n0 = nt0 * 16 + (idx - p * cpr) * 8;
              const bool ok = p < npix && n0 < a.Cs_dy;
              const int pp = ok ? p : 0;
              const int pyl = fwo.div(pp);
              const int oy = oy0 + pyl, ox = pp - pyl * a.Wo;
              if (a.dy_code) return unpool_load8(a.dy + boff, a.dy_code + boff, a.dHp, a.dWp, a.Cs_dy, oy, ox, n0, ok);
              return load_bf16x8_if(ok, a.dy + (((size_t)b * a.Ho + oy) * a.Wo + ox) * a.Cs_dy + n0, a.dy);
            },
            [&](int idx, const bf16x8& v) {
              const int p = fcpr.div(idx);
              *reinterpret_cast<bf16x8*>(dyl + (size_t)p * ldb + (idx - p * cpr) * 8) = v;
            });
      }
      __syncthreads();
      WH_STAMP(2 + 2 * (blk - blk0));
      mma_block(npix);
      if (INSTR && a.ts2) asm volatile("" ::"v"(acc[0][0][0]));
      WH_STAMP(3 + 2 * (blk - blk0));
    }
  }

  const int ld = a.NT * 16;
  float* slab = a.slab + (size_t)bx * a.Ktiles * 16 * ld;
  if (dbg & 4) {
#pragma unroll
    for (int u = 0; u < MTW; ++u)
#pragma unroll
      for (int v = 0; v < NTT; ++v)
        asm volatile("" ::"v"(acc[u][v][0]), "v"(acc[u][v][1]), "v"(acc[u][v][2]), "v"(acc[u][v][3]));
    return;
  }
  // write-through slabs (a.wt): each 16x16 tile goes through a wave-private LDS square and
  // leaves as one 16-byte sc1 store per lane (4 rows x 64 B), so the launch ends with none
  // of its partial bytes dirty in L2; plain form: 4 scalar stores per lane
  float* sq = reinterpret_cast<float*>(smem) + wave * (16 * WH_SQ);
  if (a.wt) __syncthreads();   // the staging images' last readers are done: LDS is scratch
#pragma unroll
  for (int u = 0; u < MTW; ++u) {
    const int mt = wave + 4 * u;
    if (u >= nval) continue;
#pragma unroll
    for (int v = 0; v < NTT; ++v) {
      if (nt0 + v >= a.NT) continue;
      if (u == ubias) {   // bias tile: every row holds the column sums; row 0 lives in lanes 0..15
        if (g == 0) a.bslab[(size_t)bx * ld + (nt0 + v) * 16 + i] = acc[u][v][0];
        continue;
      }
      if (mt0 + mt >= a.Ktiles) continue;
      if (a.wt) {
#pragma unroll
        for (int j = 0; j < 4; ++j) sq[(g * 4 + j) * WH_SQ + i] = acc[u][v][j];
        __builtin_amdgcn_wave_barrier();
        const int row = lane >> 2, c4 = (lane & 3) * 4;
        const u32x4 val = *reinterpret_cast<const u32x4*>(sq + row * WH_SQ + c4);
        const size_t off = (size_t)bx * a.Ktiles * 16 * ld + (size_t)((mt0 + mt) * 16 + row) * ld + (nt0 + v) * 16 + c4;
        st_wt16(a.slab, (unsigned)(off * 4), val);
        __builtin_amdgcn_wave_barrier();
        continue;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
        slab[(size_t)((mt0 + mt) * 16 + g * 4 + j) * ld + (nt0 + v) * 16 + i] = acc[u][v][j];
    }
  }
  WH_STAMP(15);
}

