// Tiled implicit-GEMM convolution for wide layers (Cs_in % 32 == 0, large K = KH*KW*Cs_in):
// the legacy RPV model (64..256 channels, Train_rpv.ipynb:205-219) and wide HPO trials.
//
// conv_halo keeps ALL of K's weights in LDS per workgroup, which forces a single 16-channel
// n-tile per workgroup once K is large (every A fragment then feeds one MFMA).  These
// kernels are LDS-blocked GEMMs over the whole batch instead:
//   * block tile 128 output rows (pixels over the batch, or 2x2 pool windows x 4 positions)
//     x BN = NTC*16 output channels, 256 threads = 2 x 2 waves, wave tile 64 x BN/2
//     (4 x NTC/2 MFMA 16x16x32 tiles: each A fragment feeds NTC/2 MFMAs, each B fragment 4);
//   * a k-step is 32 channels of one tap (Cs_in % 32 == 0): A_s[128][32] holds 8 channels
//     of one tap-shifted NHWC pixel per 16-byte chunk (zero padding and the input dilation
//     of strided dgrad resolved in the gather), B_s is the fragment-major weight pack slice
//     (1 KB per n-tile, a straight copy); the LDS ring is double-buffered, one barrier per
//     stage of 2 k-steps.
//
// Two staging paths:
//   conv_gl_kernel   (default) LDS-DMA: `global_load_lds_dwordx4` writes A and B straight
//                    into LDS with no VGPR round trip and no ds_write pass (which made the
//                    register-staged kernel LDS-store bound: 32 KB of ds_write_b128 per
//                    stage ~ 415 cycles against 512 MFMA cycles).  The DMA destination is
//                    lane-linear, so zero padding comes from pointing a lane's SOURCE at a
//                    zero buffer, and the bank-conflict swizzle of A is applied on the
//                    source side: 64-B rows, chunk c of row r stored at position
//                    c ^ ((-(r>>2)) & 3) within its row, which makes every 16-lane group
//                    of a fragment ds_read_b128 cover all 64 banks once.
//   conv_tile_kernel register-staged, for the unpool-on-load input (dP + argmax codes)
//                    whose gather needs arithmetic; rows padded to 40 elements.
// Epilogues are conv_halo's (mode 0: bias/ReLU/pool+argmax/dropout -> bf16 NHWC; mode 1:
// backward-through the previous stage), staged through LDS for 16-byte stores.
#include <type_traits>

#include "bwd_through.h"

namespace {
constexpr int BM = 128;         // rows per block
constexpr int LDA = 40;         // register path: A_s row stride (elements): 32 + 8 pad
constexpr int KST = 2;          // k-steps per pipeline stage (one barrier per stage)

// Output-row space of one launch: 2x2 pool windows x 4 positions, or the pixels of one
// input-dilation parity class (strided dgrad), or plain pixels.
struct TileRows {
  bool pool;
  int dil, cy, cx, Hc, Wc;
  long long nrows;
  __device__ void coords(const ConvMMArgs& a, long long rr, int& b, int& oy, int& ox) const {
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
  }
};

// Strided dgrad (input dilation dil > 1): output pixels are split into dil x dil parity
// classes (grid.z); in a class only taps with (o - pad + k) % dil == 0 contribute, so the
// K loop visits just those (~1/dil^2 of the dense-dilated work).
struct TapLattice {
  int ky0, kx0, nky, nkx, KS;
};

__device__ __forceinline__ void tile_geometry(const ConvMMArgs& a, TileRows& tr, TapLattice& tl) {
  const int dil = a.in_dil;
  tr.pool = a.mode == 0 && a.pool;
  tr.dil = dil;
  tr.cy = dil > 1 ? (int)blockIdx.z / dil : 0;
  tr.cx = dil > 1 ? (int)blockIdx.z % dil : 0;
  tr.Hc = dil > 1 ? (a.Ho - tr.cy + dil - 1) / dil : a.Ho;
  tr.Wc = dil > 1 ? (a.Wo - tr.cx + dil - 1) / dil : a.Wo;
  tr.nrows = tr.pool ? (long long)a.B * a.Hp * a.Wp * 4 : (long long)a.B * tr.Hc * tr.Wc;
  tl.ky0 = dil > 1 ? ((a.pad_t - tr.cy) % dil + dil) % dil : 0;
  tl.kx0 = dil > 1 ? ((a.pad_l - tr.cx) % dil + dil) % dil : 0;
  tl.nky = tl.ky0 < a.KH ? (a.KH - tl.ky0 + dil - 1) / dil : 0;
  tl.nkx = tl.kx0 < a.KW ? (a.KW - tl.kx0 + dil - 1) / dil : 0;
  tl.KS = tl.nky * tl.nkx * (a.Cs_in >> 5);
}

// k-step walker over the class's tap lattice for this thread's two gather rows; per-row
// input coordinates / validity are recomputed only when the tap changes.
struct Walker {
  int gb[2], gy[2], gx[2];
  bool gv[2];
  int wty, wtx, wcs, cps, chunk;
  int iyr[2], ixr[2];
  bool okr[2];
  const bf16* rowp[2];

  __device__ void init(const ConvMMArgs& a, const TileRows& tr, long long r0, long long r1, int ch) {
    const long long rows[2] = {r0, r1};
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      gv[u] = rows[u] < tr.nrows;
      tr.coords(a, gv[u] ? rows[u] : 0, gb[u], gy[u], gx[u]);
    }
    wty = wtx = wcs = 0;
    cps = a.Cs_in >> 5;
    chunk = ch;
  }
  __device__ void set_tap(const ConvMMArgs& a, const TapLattice& tl) {
    const int dil = a.in_dil;
    const int ky = tl.ky0 + wty * dil, kx = tl.kx0 + wtx * dil;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      int iy = gy[u] * a.stride - a.pad_t + ky, ix = gx[u] * a.stride - a.pad_l + kx;
      bool ok = gv[u] && iy >= 0 && ix >= 0;
      if (dil > 1) {          // exact: the class guarantees divisibility
        iy /= dil;
        ix /= dil;
      }
      ok = ok && iy < a.H && ix < a.W;
      iyr[u] = iy;
      ixr[u] = ix;
      okr[u] = ok;
      rowp[u] = ok ? a.x + (((size_t)gb[u] * a.H + iy) * a.W + ix) * a.Cs_in + 8 * chunk : a.x;
    }
  }
  __device__ void next_k(const ConvMMArgs& a, const TapLattice& tl) {
    if (++wcs == cps) {
      wcs = 0;
      if (++wtx == tl.nkx) { wtx = 0; ++wty; }
      set_tap(a, tl);
    }
  }
  __device__ int pack_ks(const ConvMMArgs& a, const TapLattice& tl) const {
    return ((tl.ky0 + wty * a.in_dil) * a.KW + (tl.kx0 + wtx * a.in_dil)) * cps + wcs;
  }
};

// Shared epilogue: per wave [16 rows][NW*16] through LDS scratch, 16-byte global stores.
// WM: 64-row wave groups of the block (2: 128-row blocks of 4 waves, 4: 256-row blocks of 8)
template <int NTC, int WM = 2>
__device__ __forceinline__ void tile_epilogue(const ConvMMArgs& a, const TileRows& tr, f32x4 (&acc)[4][NTC / 2],
                                              char* smem, long long row0, int nt0, uint32_t step) {
  constexpr int NW = NTC / 2;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 15, g = lane >> 4;
  const int wm = wave % WM, wn = wave / WM;
  const long long nrows = tr.nrows;
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
    if (tr.pool) {
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
      // rows staged with their 16-byte chunks XOR-swizzled by row group: chunk c of row q at
      // c ^ ((q >> 2) * 4 & (chunks - 1)) -- unswizzled, the four lane groups of a store (rows
      // 4 apart, 1-2 KB apart) hit the same banks
      constexpr int CHK = NW * 4 - 1;                 // 16-byte chunks per row - 1
#pragma unroll
      for (int n = 0; n < NW; ++n)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int col = n * 16 + r, sw = (g * 4) & CHK;   // (row g * 4 + j: (row >> 2) == g)
          ep[(g * 4 + j) * LDC + (((col >> 2) ^ sw) << 2) + (col & 3)] = acc[t][n][j];
        }
      __builtin_amdgcn_wave_barrier();
      const int np = (int)min((long long)16, nrows - tile * 16);
      for (int c = lane; c < np * cch; c += 64) {
        const int pr = c / cch, c8 = c - pr * cch;
        size_t m = (size_t)(tile * 16 + pr);
        if (tr.dil > 1) {                             // parity class row -> flat output pixel
          int b, oy, ox;
          tr.coords(a, (long long)m, b, oy, ox);
          m = ((size_t)b * a.Ho + oy) * a.Wo + ox;
        }
        float v[8];
        const int sw = ((pr >> 2) * 4) & CHK;
        *reinterpret_cast<float4*>(v) = *reinterpret_cast<const float4*>(ep + pr * LDC + (((2 * c8) ^ sw) << 2));
        *reinterpret_cast<float4*>(v + 4) = *reinterpret_cast<const float4*>(ep + pr * LDC + (((2 * c8 + 1) ^ sw) << 2));
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
}  // namespace

// ------------------------------------------------------------------------------------------
// LDS-DMA path (NTC 4 or 8).  Per k-step: A = 128 rows x 64 B = 8 wave-instructions (2 per
// wave), B = NTC fragments x 1 KB (NTC/4 per wave).  A ring of GL_NBUF one-k-step buffers
// keeps GL_DIST k-steps of DMA in flight: iteration st waits (counted vmcnt, never 0 in
// the loop) for its own stage-st DMA, passes a raw s_barrier (every wave's stage st has
// landed and every wave has finished computing stage st-1), re-issues the freed buffer
// with stage st+GL_DIST, then runs stage st's MFMAs.  (__syncthreads() would drain vmcnt to
// 0 and serialise the ring: one k-step of latency per k-step, the previous 2-buffer form.)
namespace {
constexpr int GL_NBUF = 4;
constexpr int GL_DIST = GL_NBUF - 1;
}

// NWV waves per block: 4 (128 rows, the 2 x 2 wave grid) or 8 (256 rows, 4 x 2): the larger
// block halves the L2 traffic of the weight operand per MFMA, and with NTC = 16 (all 256
// output channels of a wide layer) the activation taps are fetched once instead of per
// 128-channel half.  PMC: the 128 x 128 form moved ~1.1 GB through L2 per launch (~11 TB/s,
// ~20 % MFMA busy); halving that traffic bought only 1-10 % per legacy launch (conv2 fwd
// 133.8 -> 131.7 us, strided dgrad 85.5 -> 75.8 us; a 5-deep ring: equal): the per-CU
// LDS-DMA rate of the row-gathered A operand (~7.5 B/clk/CU here), not L2 bandwidth, bounds it.
template <int NTC, int NWV, int NBUF = GL_NBUF>
__global__ __launch_bounds__(64 * NWV) void conv_gl_kernel(const ConvMMArgs a) {
  constexpr int DIST = NBUF - 1;
  static_assert(NTC % NWV == 0, "uniform per-wave DMA count needs NTC % NWV == 0");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int BMB = 32 * NWV;                        // rows per block (2 DMA slots of 16 per wave)
  constexpr int WM = BMB / 64;                         // 64-row wave groups
  constexpr int NW = NTC / 2;
  static_assert(NWV / WM == 2, "two n-groups of waves");
  constexpr int A_BYTES = BMB * 64;
  constexpr int STEP_BYTES = A_BYTES + NTC * 1024;
  constexpr int PER_STEP = 2 + NTC / NWV;              // DMA instructions per wave per k-step
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 15, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WM, wn = wave / WM;
  const int nt0 = blockIdx.y * NTC;
  TileRows tr;
  TapLattice tl;
  tile_geometry(a, tr, tl);
  const long long row0 = (long long)blockIdx.x * BMB;
  if (row0 >= tr.nrows) return;                       // (parity classes differ in size)
  const uint32_t step = a.st ? (uint32_t)a.st->t : 0u;
  const int KS = tl.KS;

  // this lane's DMA slots: rows 16*(2*wave+u) + lane/4, LDS position lane&3 holding the
  // swizzled source chunk
  const int chunk = (lane & 3) ^ ((-(lane >> 4)) & 3);
  Walker wk;
  wk.init(a, tr, row0 + 16 * (2 * wave) + (lane >> 2), row0 + 16 * (2 * wave + 1) + (lane >> 2), chunk);
  const bf16* zero = a.zero;

  // issue k-step k (the walker's current position) into ring slot k % GL_NBUF
  auto issue = [&](int k) {
    char* sb = smem + (k % NBUF) * STEP_BYTES;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bf16* src = wk.okr[u] ? wk.rowp[u] + wk.wcs * 32 : zero;
      __builtin_amdgcn_global_load_lds(src, sb + (2 * wave + u) * 1024, 16, 0, 0);
    }
    const int kp = wk.pack_ks(a, tl);
#pragma unroll
    for (int j = 0; j < NTC / NWV; ++j) {            // fragment n = wave + NWV j
      const int n = wave + NWV * j;
      const int nt = min(nt0 + n, a.NT - 1);         // clamped: columns past N are dropped
      __builtin_amdgcn_global_load_lds(a.wpk + ((size_t)(kp * a.NT + nt) * 64 + lane) * 8,
                                       sb + A_BYTES + n * 1024, 16, 0, 0);
    }
    if (k + 1 < KS) wk.next_k(a, tl);
  };

  f32x4 acc[4][NW];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int n = 0; n < NW; ++n) acc[t][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int rsw = (-(r >> 2)) & 3;                     // read-side swizzle of this lane's row

  if (KS > 0) wk.set_tap(a, tl);
#pragma unroll
  for (int k = 0; k < DIST; ++k)
    if (k < KS) issue(k);
  for (int st = 0; st < KS; ++st) {
    // own DMA of stage st retired: later stages issued so far = min(GL_DIST-1, KS-1-st)
    const int later = min(DIST - 1, KS - 1 - st);
    if (later >= 3 && DIST >= 4) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(3 * PER_STEP) : "memory");
    else if (later >= 2) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * PER_STEP) : "memory");
    else if (later == 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(PER_STEP) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (st + DIST < KS) issue(st + DIST);        // slot of stage st-1: free after the barrier
    const char* A = smem + (st % NBUF) * STEP_BYTES;
    const char* Bb = A + A_BYTES;
    bf16x8 af[4], bfr[NW];
#pragma unroll
    for (int t = 0; t < 4; ++t)
      af[t] = *reinterpret_cast<const bf16x8*>(A + ((wm * 4 + t) * 16 + r) * 64 + ((g ^ rsw) << 4));
#pragma unroll
    for (int n = 0; n < NW; ++n)
      bfr[n] = *reinterpret_cast<const bf16x8*>(Bb + ((wn * NW + n) * 64 + lane) * 16);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int n = 0; n < NW; ++n) acc[t][n] = mfma16(af[t], bfr[n], acc[t][n]);
  }
  __syncthreads();                                    // ring reads done before epilogue scratch reuse
  tile_epilogue<NTC, WM>(a, tr, acc, smem, row0, nt0, step);
}

// ------------------------------------------------------------------------------------------
// Halo-staged wide conv (stride 1, Cs_in % 32 == 0, no pool: the legacy model's 32x32 conv3
// forward and dgrad, and its two strided dgrads).  conv_gl gathers the A operand per k-step --
// every input pixel is DMA'd once per TAP, and the per-CU LDS-DMA rate bounds the launch
// (profiles/r3_legacy_ab_big_tiles.txt, r6_legacy_sequence.txt).  Here a block is RB = 256 / Wc
// whole output rows of one image; for each 32-channel chunk the input halo those rows read is
// DMA'd ONCE (double-buffered across chunks) and every tap reads its A fragments from it at a
// tap-shifted offset; only the weight fragments go through the per-k-step ring.
//   strided dgrad (input dilation d > 1): the output pixels split into d x d parity classes
//   (grid.z, as conv_gl); within class (cy, cx) only the taps of one lattice contribute and
//   output pixel (cy + d i, cx + d j) reads input (i + oy0 + ty, j + ox0 + tx) for lattice tap
//   (ty, tx) -- a stride-1 conv on the dilated input's own grid with an nky x nkx kernel, so
//   the same halo scheme applies (the dense-dilated form reads each input pixel ~d^2 KH KW / ...
//   times per chunk, and conv_gl's row gather once per tap).
//   halo LDS layout: flat halo pixel fp = hr * HWd + hc, 64 B per pixel (32 channels), 16-byte
//   chunk c stored at position c ^ ((fp >> 2) & 3) -- any 16 consecutive pixels (an m-tile's
//   rows at any tap shift) then cover all 64 banks once per lane group;
//   k order: chunk-major, tap-minor.
// Waves: 8 = 4 (64-row groups) x 2 (n halves), as conv_gl<NTC, 8>; the epilogue is the shared one.
namespace {
constexpr int HS_NBUF = 4;                 // weight ring slots (3 k-steps of DMA in flight)
constexpr int HS_HALO_INSTR = 3;           // halo DMA instructions per wave per chunk (3 KB)
__host__ __device__ constexpr int hs_halo_bytes(int nwv) { return nwv * HS_HALO_INSTR * 1024; }
__host__ __device__ constexpr int hs_halo_pix(int nwv) { return nwv * HS_HALO_INSTR * 16; }

__device__ __forceinline__ void hs_wait(int n) {   // s_waitcnt vmcnt(min(n, 8)) -- never less
  switch (n) {                                     // than n outstanding is waited for
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
  }
}

// per-launch geometry of the halo-staged conv (one parity class per grid.z)
struct HsGeom {
  int dil, cy, cx, Hc, Wc, RB, ky0, kx0, nky, nkx, oy0, ox0, HWd, HR;
  __host__ __device__ void init(const ConvMMArgs& a, int cls, int rows) {   // rows: block rows
    dil = a.in_dil > 1 ? a.in_dil : 1;
    cy = cls / dil, cx = cls % dil;
    Hc = (a.Ho - cy + dil - 1) / dil, Wc = (a.Wo - cx + dil - 1) / dil;
    RB = Wc > 0 && Wc <= rows ? rows / Wc : 0;
    ky0 = ((a.pad_t - cy) % dil + dil) % dil, kx0 = ((a.pad_l - cx) % dil + dil) % dil;
    nky = ky0 < a.KH ? (a.KH - ky0 + dil - 1) / dil : 0;
    nkx = kx0 < a.KW ? (a.KW - kx0 + dil - 1) / dil : 0;
    oy0 = (cy - a.pad_t + ky0) / dil, ox0 = (cx - a.pad_l + kx0) / dil;   // exact: same parity
    HWd = Wc + (nkx > 0 ? nkx - 1 : 0), HR = RB + (nky > 0 ? nky - 1 : 0);
  }
};
}  // namespace

// NWV waves: 8 (256-row blocks, two per CU) or 16 (512-row blocks: half the weight DMA per MFMA)
// order 1: the n-blocks of one row block get adjacent workgroup ids on ONE XCD (dispatch
// round-robins ids over the 8 XCDs), so the blocks that stage the same input halo share an L2
template <int NTC, int NWV>
__global__ __launch_bounds__(64 * NWV) void conv_hs_kernel(const ConvMMArgs a, const int order) {
  constexpr int WM = NWV / 2, NW = NTC / 2;
  constexpr int B_BYTES = NTC * 1024;
  constexpr int HS_HALO_BYTES = hs_halo_bytes(NWV);
  static_assert(NTC < NWV || NTC % NWV == 0, "uniform weight DMA per wave");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const ring = smem;                             // [HS_NBUF][B_BYTES]
  char* const halo = smem + HS_NBUF * B_BYTES;         // [2][HS_HALO_BYTES]
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 15, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WM, wn = wave / WM;
  HsGeom q;
  q.init(a, (int)blockIdx.z, 32 * NWV);
  const int W = a.W, HWd = q.HWd, RB = q.RB, nkx = q.nkx;
  const int nyb = q.Hc / RB;
  int bxx = (int)blockIdx.x, byy = (int)blockIdx.y;
  if (order == 1) {   // (host: gridDim.x * gridDim.y % 8 == 0)
    const int n = (int)(gridDim.x * gridDim.y);
    int id = bxx + (int)gridDim.x * byy;
    id = (id & 7) * (n >> 3) + (id >> 3);
    byy = id % (int)gridDim.y;
    bxx = id / (int)gridDim.y;
  }
  const int b = bxx / nyb, y0 = (bxx - b * nyb) * RB;
  const int nt0 = byy * NTC;
  const int cps = a.Cs_in >> 5, ntap = q.nky * nkx, KS = ntap * cps;
  const int npix_h = q.HR * HWd;                       // halo pixels per chunk
  const uint32_t step = a.st ? (uint32_t)a.st->t : 0u;
  const bf16* zero = a.zero;
  const bf16* ximg = a.x + (size_t)b * a.H * W * a.Cs_in;
  // weight DMA instructions this wave issues per k-step (NTC 4: waves 0-3 one each)
  const int nbw = NTC >= NWV ? NTC / NWV : (wave < NTC ? 1 : 0);

  // halo chunk c -> buffer c & 1: instruction j of wave w covers flat pixels 16 (w*3 + j) ...
  auto issue_halo = [&](int c) {
    char* hb = halo + (c & 1) * HS_HALO_BYTES;
#pragma unroll
    for (int j = 0; j < HS_HALO_INSTR; ++j) {
      const int ins = wave * HS_HALO_INSTR + j;
      const int fp = ins * 16 + (lane >> 2);
      const int lc = (lane & 3) ^ ((fp >> 2) & 3);       // logical chunk this lane's slot holds
      const int hr = fp / HWd, hc = fp - hr * HWd;
      const int iy = y0 + q.oy0 + hr, ix = q.ox0 + hc;
      const bool ok = fp < npix_h && iy >= 0 && iy < a.H && ix >= 0 && ix < W;
      const bf16* src = ok ? ximg + ((size_t)iy * W + ix) * a.Cs_in + c * 32 + lc * 8 : zero;
      __builtin_amdgcn_global_load_lds(src, hb + ins * 1024, 16, 0, 0);
    }
  };
  // weight fragments of k-step k = (chunk c, lattice tap (ty, tx)) -> ring slot k % HS_NBUF
  auto issue_b = [&](int k, int c, int ty, int tx) {
    const int kp = ((q.ky0 + ty * q.dil) * a.KW + (q.kx0 + tx * q.dil)) * cps + c;
    char* sb = ring + (k % HS_NBUF) * B_BYTES;
#pragma unroll
    for (int j = 0; j < (NTC + NWV - 1) / NWV; ++j) {
      const int n = wave + NWV * j;
      if (n < NTC) {
        const int nt = min(nt0 + n, a.NT - 1);
        __builtin_amdgcn_global_load_lds(a.wpk + ((size_t)(kp * a.NT + nt) * 64 + lane) * 8, sb + n * 1024, 16, 0,
                                         0);
      }
    }
  };
  // k-step walkers (no divisions in the loop): tap-minor, chunk-major
  auto advance = [&](int& c, int& ty, int& tx) {
    if (++tx == nkx) {
      tx = 0;
      if (++ty == q.nky) { ty = 0; ++c; }
    }
  };

  f32x4 acc[4][NW];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int n = 0; n < NW; ++n) acc[t][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  // this lane's output pixel of m-tile t: block row wm * 64 + t * 16 + r -> class pixel (y, x);
  // its halo pixel at lattice tap (0, 0) is (y, x) (the halo starts at the tap-(0, 0) input)
  int fp0[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int pr = wm * 64 + t * 16 + r, y = pr / q.Wc, x = pr - y * q.Wc;
    fp0[t] = y * HWd + x;
  }

  // counted waits: `issued` = this wave's vector-memory instructions so far; pb0..pb2 = the
  // count right after B(st), B(st+1), B(st+2) were issued, phc / phn after H(c) / H(c+1).  Stage
  // st needs B(st) and H(c): it waits until at most issued - max(pb0, phc) remain outstanding.
  int issued = 0, pb0 = 0, pb1 = 0, pb2 = 0, phc = 0, phn = 0;
  int bc = 0, bty = 0, btx = 0;                        // position of the next weight issue
  if (KS > 0) {
    issue_halo(0);
    issued += HS_HALO_INSTR;
    phc = issued;
    issue_b(0, bc, bty, btx);
    advance(bc, bty, btx);
    issued += nbw;
    pb0 = issued;
    if (KS > 1) {
      issue_b(1, bc, bty, btx);
      advance(bc, bty, btx);
      issued += nbw;
    }
    pb1 = issued;
    if (KS > 2) {
      issue_b(2, bc, bty, btx);
      advance(bc, bty, btx);
      issued += nbw;
    }
    pb2 = issued;
  }
  int c = 0, ty = 0, tx = 0;                           // stage st's k-step
  for (int st = 0; st < KS; ++st) {
    hs_wait(issued - max(pb0, phc));
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // (the barrier retired every reader of stage st-1's ring slot and, at tap 0, of chunk c-1's
    // halo buffer: refill them)
    const bool first = ty == 0 && tx == 0, last = ty == q.nky - 1 && tx == nkx - 1;
    if (first && c + 1 < cps) {
      issue_halo(c + 1);
      issued += HS_HALO_INSTR;
      phn = issued;
    }
    if (st + HS_NBUF - 1 < KS) {
      issue_b(st + HS_NBUF - 1, bc, bty, btx);
      advance(bc, bty, btx);
      issued += nbw;
    }
    pb0 = pb1, pb1 = pb2, pb2 = issued;
    if (last) phc = phn;
    const char* Bb = ring + (st % HS_NBUF) * B_BYTES;
    const char* H = halo + (c & 1) * HS_HALO_BYTES;
    const int toff = ty * HWd + tx;
    bf16x8 af[4], bfr[NW];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int fp = fp0[t] + toff;
      af[t] = *reinterpret_cast<const bf16x8*>(H + fp * 64 + ((g ^ ((fp >> 2) & 3)) << 4));
    }
#pragma unroll
    for (int n = 0; n < NW; ++n)
      bfr[n] = *reinterpret_cast<const bf16x8*>(Bb + ((wn * NW + n) * 64 + lane) * 16);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int n = 0; n < NW; ++n) acc[t][n] = mfma16(af[t], bfr[n], acc[t][n]);
    advance(c, ty, tx);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();                                    // ring / halo reads done: epilogue scratch
  TileRows tr;
  tr.pool = false;
  tr.dil = q.dil, tr.cy = q.cy, tr.cx = q.cx, tr.Hc = q.Hc, tr.Wc = q.Wc;
  tr.nrows = (long long)a.B * q.Hc * q.Wc;
  const long long row0 = ((long long)b * q.Hc + y0) * q.Wc;
  tile_epilogue<NTC, WM>(a, tr, acc, smem, row0, nt0, step);
}

// ------------------------------------------------------------------------------------------
// Register-staged path (unpool-on-load input).
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
  TileRows tr;
  TapLattice tl;
  tile_geometry(a, tr, tl);
  const long long row0 = (long long)blockIdx.x * BM;
  if (row0 >= tr.nrows) return;
  const uint32_t step = a.st ? (uint32_t)a.st->t : 0u;
  const int KS = tl.KS, Cs = a.Cs_in;
  const int IH = a.in_code ? a.in_pH : a.H, IW = a.in_code ? a.in_pW : a.W;

  // this thread's two A-gather rows (128 rows x 4 chunks of 8 channels = 512 loads)
  const int ach = tid & 3;
  Walker wk;
  wk.init(a, tr, row0 + (tid >> 2), row0 + (tid >> 2) + 64, ach);
  auto load_a = [&](int u) -> bf16x8 {
    if (a.in_code) {
      const size_t boff = (size_t)wk.gb[u] * IH * IW * Cs;
      return unpool_load8(a.x + boff, a.in_code + boff, IH, IW, Cs, wk.iyr[u], wk.ixr[u], wk.wcs * 32 + 8 * ach,
                          wk.okr[u]);
    }
    return load_bf16x8_if(wk.okr[u], wk.rowp[u] + wk.wcs * 32, a.x);
  };
  // B gather: NTC*64 16-byte fragment vectors per k-step
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
      const int kp = wk.pack_ks(a, tl);
#pragma unroll
      for (int u = 0; u < BV; ++u) rb[kk][u] = load_b(kp, u);
      if (++kl < KS) wk.next_k(a, tl);
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
    wk.set_tap(a, tl);
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
  tile_epilogue<NTC>(a, tr, acc, smem, row0, nt0, step);
}

static size_t epilogue_bytes(int ntc) { return (size_t)4 * 16 * (ntc / 2) * 16 * 4; }

static size_t gl_lds_bytes(int ntc, int nwv = 4, int nbuf = GL_NBUF) {
  const size_t stage = (size_t)nbuf * (32 * nwv * 64 + ntc * 1024);
  const size_t ep = epilogue_bytes(ntc) * nwv / 4;
  return stage > ep ? stage : ep;
}

size_t conv_tile_lds_bytes(int ntc) {
  const size_t stage = (size_t)2 * KST * (BM * LDA + ntc * 64 * 8) * 2;
  const size_t reg = stage > epilogue_bytes(ntc) ? stage : epilogue_bytes(ntc);
  const size_t gl = gl_lds_bytes(ntc);
  return reg > gl ? reg : gl;
}

static long long tile_maxrows(const ConvMMArgs& a) {
  const bool pool = a.mode == 0 && a.pool;
  const long long nrows = pool ? (long long)a.B * a.Hp * a.Wp * 4 : (long long)a.B * a.Ho * a.Wo;
  const int d = a.in_dil > 1 ? a.in_dil : 1;
  return pool ? nrows : (long long)a.B * ((a.Ho + d - 1) / d) * ((a.Wo + d - 1) / d);
}

template <int NTC, int NWV, int NBUF = GL_NBUF>
static void launch_gl(const ConvMMArgs& a, hipStream_t s) {
  const int d = a.in_dil > 1 ? a.in_dil : 1;
  const int gx = (int)((tile_maxrows(a) + 32 * NWV - 1) / (32 * NWV));
  const int gy = (a.NT + NTC - 1) / NTC;
  auto k = conv_gl_kernel<NTC, NWV, NBUF>;
  const size_t lds = gl_lds_bytes(NTC, NWV, NBUF);
  if (lds > 65536) (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(k, dim3(gx, gy, d * d), dim3(64 * NWV), lds, s, a);
}

template <int NTC>
static void launch_t(const ConvMMArgs& a, hipStream_t s) {
  const int d = a.in_dil > 1 ? a.in_dil : 1;
  const int gx = (int)((tile_maxrows(a) + BM - 1) / BM);
  const int gy = (a.NT + NTC - 1) / NTC;
  if constexpr (NTC % 4 == 0) {
    if (a.in_code == nullptr && a.zero != nullptr) {
      launch_gl<NTC, 4>(a, s);
      return;
    }
  }
  hipLaunchKernelGGL(conv_tile_kernel<NTC>, dim3(gx, gy, d * d), dim3(256), conv_tile_lds_bytes(NTC), s, a);
}

// halo-staged path (conv_hs_kernel): the shapes it serves, its LDS bytes and launch.  Every
// parity class must tile into whole (32 * nwv)-row blocks and fit its halo in the DMA slots.
bool conv_hs_ok(const ConvMMArgs& a, int ntc, int nwv) {
  if (!(ntc == 4 || ntc == 8 || ntc == 16) || !(nwv == 8 || nwv == 16) || (nwv == 16 && ntc == 16) || a.zero == nullptr ||
      a.in_code != nullptr || a.stride != 1 || (a.Cs_in & 31) || (a.mode == 0 && a.pool) || a.KH > 3 || a.KW > 3 ||
      a.KS != a.KH * a.KW * (a.Cs_in >> 5))
    return false;
  const int d = a.in_dil > 1 ? a.in_dil : 1;
  if (a.Ho % d || a.Wo % d) return false;
  for (int cls = 0; cls < d * d; ++cls) {
    HsGeom q;
    q.init(a, cls, 32 * nwv);
    if (q.RB == 0 || (32 * nwv) % q.Wc || q.Hc % q.RB || q.HR * q.HWd > hs_halo_pix(nwv)) return false;
  }
  return true;
}

size_t conv_hs_lds_bytes(int ntc, int nwv) {
  const size_t ring = (size_t)HS_NBUF * ntc * 1024 + 2 * hs_halo_bytes(nwv);
  const size_t ep = epilogue_bytes(ntc) * nwv / 4;
  return ring > ep ? ring : ep;
}

template <int NTC, int NWV>
static void launch_hs(const ConvMMArgs& a, hipStream_t s, int order) {
  HsGeom q;
  q.init(a, 0, 32 * NWV);
  const dim3 grid(a.B * (q.Hc / q.RB), (a.NT + NTC - 1) / NTC, q.dil * q.dil);
  if (order != 1 || grid.y < 2 || (grid.x * grid.y) % 8) order = 0;
  const size_t lds = conv_hs_lds_bytes(NTC, NWV);
  auto k = conv_hs_kernel<NTC, NWV>;
  (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(k, grid, dim3(64 * NWV), lds, s, a, order);
}

bool launch_conv_hs(const ConvMMArgs& a, int ntc, hipStream_t s, int nwv, int order) {
  if (!conv_hs_ok(a, ntc, nwv)) return false;
  if (nwv == 16) {   // (no NTC 16 form: 1024 threads leave 128 VGPRs, and its tile spills)
    if (ntc == 8) launch_hs<8, 16>(a, s, order);
    else launch_hs<4, 16>(a, s, order);
  } else {
    if (ntc == 16) launch_hs<16, 8>(a, s, order);
    else if (ntc == 8) launch_hs<8, 8>(a, s, order);
    else launch_hs<4, 8>(a, s, order);
  }
  return true;
}

// ntc: n-tiles per block; big: 256-row blocks of 8 waves (LDS-DMA path only; the host picks
// it when the grid still has >= 512 blocks)
void launch_conv_tile(const ConvMMArgs& a, int ntc, hipStream_t s, bool big, int nbuf) {
  const bool gl = a.in_code == nullptr && a.zero != nullptr;
  // nbuf 3: a 3-slot ring (2 k-steps of DMA in flight) -- 72 KB for the 8-tile big block, so two
  // blocks fit a CU's LDS instead of one
  if (big && gl && ntc == 16) {
    if (nbuf == 3) launch_gl<16, 8, 3>(a, s);
    else launch_gl<16, 8>(a, s);   // (a 5-deep ring measured equal)
    return;
  }
  if (big && gl && ntc == 8) {
    if (nbuf == 3) launch_gl<8, 8, 3>(a, s);
    else launch_gl<8, 8>(a, s);
    return;
  }
  switch (ntc) {
    case 2: launch_t<2>(a, s); break;
    case 4: launch_t<4>(a, s); break;
    case 8: launch_t<8>(a, s); break;
    default: break;
  }
}

// blocks of the big-tile launch for (ntc) -- the host's grid-size rule
long long conv_tile_big_blocks(const ConvMMArgs& a, int ntc) {
  const int d = a.in_dil > 1 ? a.in_dil : 1;
  return ((tile_maxrows(a) + 255) / 256) * ((a.NT + ntc - 1) / ntc) * d * d;
}
