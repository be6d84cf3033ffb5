// Kernel argument structs (shared by the .hip translation units and the pybind11 bindings).
// Pointers are device pointers; Python fills the structs once per (plan, batch size) and
// re-launches them every step (eagerly or under HIP-graph capture).
#pragma once
#include "common.h"

// "Backward through the previous stage": turn dL/d(prev stage output) into dL/d(prev
// pre-activation) = apply the previous stage's dropout mask (regenerated), ReLU mask
// (from its saved output) and 2x2 max-pool routing (from its saved argmax code), writing
// the full-resolution gradient the previous layer's wgrad/dgrad consume.
struct BwdThrough {
  const bf16* prev_out = nullptr;     // saved output of the previous stage [.., pCs]
  const uint8_t* prev_code = nullptr; // saved pool argmax codes
  int prev_relu = 0, prev_pool = 0;
  int pH = 1, pW = 1, pC = 0, pCs = 0;  // previous stage output geometry (post-pool)
  int cH = 1, cW = 1;                   // previous conv's full-resolution grid
  uint32_t drop_thr = 0;
  float drop_scale = 1.f;
  uint32_t seed = 0, stream_id = 0;
  bf16* dy = nullptr;                   // output [B, cH, cW, pCs] (or [B, pH, pW, pCs])
  int wt = 0;                           // dy stored write-through (16-byte sc1 stores; < 2 GB)
};

// Where an updated master element goes in the bf16 fragment packs (pack_write, optim_math.h):
// the optimizer that produces a new weight writes its bf16 copies into the packs the MFMA
// kernels read, so no step needs a separate re-pack pass over the master.  One route per
// packed weight tensor, master range [lo, hi):
//   kind 1, conv  W[tap][ci][co]: fwd pack  k = tap*Cs + ci,            n = co
//                                 dgrad pack k = (KHW-1-tap)*Csb + co,  n = ci
//   kind 2, dense W[k][n] (k = Keras flatten index over Cin channels, padded kp = (k / Cin)*Cs + k % Cin):
//                                 fwd pack  k = kp, n = n;   bwd pack k = n, n = kp
// fwd / bwd: element offsets of the packs in the arena (-1: none); NT / NTb: their n-tiles.
struct PackRoute {
  int lo, hi, kind;
  int KHW, Cin, Cout, Cs, Csb;
  int NT, NTb;
  long long fwd, bwd;
};
#define MAX_ROUTES 8

// Keras optimizer update of a flat fp32 range (optimizer kernels; also fused into the
// reductions / the dense weight-gradient kernel).
struct OptimArgs {
  float* p = nullptr;
  const float* g = nullptr;
  float* s0 = nullptr;
  float* s1 = nullptr;
  int n = 0;                     // elements [lo, lo + n) are updated (lo need not be aligned)
  int lo = 0;
  StepState* st = nullptr;       // read: this step's scalars; written: packs_stale
  int kind = 0;
  float beta1 = 0.9f, beta2 = 0.999f, eps = 1e-7f, rho = 0.95f, momentum = 0.f;
  int nesterov = 0;
  float grad_scale = 1.f;
  int pack_only = 0;
  int defer_pack = 0;            // leave the re-pack to the next step's prologue (marks stale)
  bf16* arena = nullptr;
  // routes (device array, read with workgroup-uniform indices): nroutes > 0 -> every updated
  // weight is also written to its packs (pack_write) and nothing is marked stale
  const PackRoute* routes = nullptr;
  int nroutes = 0;
  // optim_kernel only: dense routes (identity padding, N % 32 == 0, K % 8 == 0) wholly inside
  // [lo, lo + n) updated by 2-D tile blocks after the flat blocks (optim_tile_block: whole
  // 16-byte pack vectors instead of scattered 2-byte stores); the flat blocks skip them
  int ntile = 0, flat_blocks = 0;
  int tile_route[4] = {0, 0, 0, 0}, tile_b0[5] = {0, 0, 0, 0, 0};   // tile_b0[ntile] = tile blocks
  // reduction kernels only: write the reduced gradient and stop (no update, no packs) -- the
  // data-parallel step reduces early buckets' slabs ahead of the all-reduce this way
  int grad_only = 0;
};

// Implicit-GEMM convolution / 1x1 "dense as conv" (fwd, dgrad, dense-dX).
struct ConvMMArgs {
  const bf16* x = nullptr;       // input activations [B, H, W, Cs_in]
  int B = 0, H = 0, W = 0, Cs_in = 0;
  int Ho = 0, Wo = 0;            // GEMM row space = conv output grid
  int KH = 1, KW = 1, stride = 1, pad_t = 0, pad_l = 0, in_dil = 1;
  int KS = 0;                    // number of 32-wide k-steps
  const bf16* wpk = nullptr;     // fragment-major pack
  int NT = 0;                    // n-tiles in the pack
  const float* bias = nullptr;   // fp32 bias (fwd) or null
  int N = 0;                     // valid output channels (fwd)
  int mode = 0;                  // 0: forward epilogue, 1: backward-through-previous-stage
  int flat_out = 0;              // mode 1: GEMM columns are flattened (y, x, c) of prev output
  // forward epilogue
  int relu = 0, pool = 0;
  bf16* out = nullptr;
  int Cs_out = 0, Hp = 0, Wp = 0;
  uint8_t* code = nullptr;
  uint32_t drop_thr = 0;         // 0 = no dropout
  float drop_scale = 1.f;
  uint32_t seed = 0, stream_id = 0;
  const StepState* st = nullptr;
  // backward-through epilogue (mode 1)
  BwdThrough bt;
  // halo-staged spatial kernel: R output rows per workgroup block; input given as a
  // pooled gradient dP [B, in_pH, in_pW, Cs_in] + argmax codes (unpool on load)
  int R = 1;
  const uint8_t* in_code = nullptr;
  int in_pH = 0, in_pW = 0;
  // >= 16 zero bytes in global memory: source of padded / out-of-range rows for the LDS-DMA
  // conv_tile path (set => that path is used when there is no unpool-on-load input)
  const bf16* zero = nullptr;
  int dbg = 0;   // ablation (timing only, wrong results): 1 skip staging, 2 skip MFMA, 4 skip stores,
                 // 8 skip the weight staging only; 16 = per-pixel unpool staging (A/B, exact);
                 // 32 = weights and pooled halo staged in two phases (A/B, exact)
  unsigned long long* ts = nullptr;   // diagnostics: [grid block][8] phase stamps, wave 0 lane 0 (null = off)
  // conv_halo LDS layout: input-halo pixel stride in elements (0 = Cs_in; padded strides
  // break the fragment reads' bank conflicts, models/lds_layout.py)
  int xpix = 0;
  int kpipe = 0;                 // software-pipelined k loop with scalar tap offsets (Cs % 32 == 0)
  int tm = 0;                    // co-scheduled dgrad: m-tiles per wave per pass (0: launch_dual_halo picks)
};

// Layer-fused forward of a conv stack (conv_stack.hip): one workgroup per image, all
// stages' activations in LDS.  Stride-1 convs with optional 2x2 max-pool.
#define MAX_STACK 4
#define MAX_STACK_SPLIT 4
struct StackLayer {
  int H = 0, W = 0, Cs_in = 0;        // input grid and channel stride
  int Ho = 0, Wo = 0, Cout = 0, Cs_out = 0;
  int KH = 3, KW = 3, pad_t = 0, pad_l = 0;
  int KS = 0, NT = 0;                 // k-steps / n-tiles of the forward pack
  int pool = 0, relu = 0;
  int Hp = 0, Wp = 0;                 // stage output grid (pooled, or = Ho, Wo)
  uint32_t drop_thr = 0;
  float drop_scale = 1.f;
  uint32_t stream_id = 0;
  const bf16* wpk = nullptr;          // forward fragment pack (global)
  const float* bias = nullptr;
  bf16* out = nullptr;                // stage output [B][Hp][Wp][Cs_out]
  uint8_t* code = nullptr;            // pool argmax codes, same shape (or null)
  int w_lds = 0;                      // bf16 element offset of the pack inside the LDS weights
  // LDS layout of this layer's INPUT halo image (written by the previous layer's epilogue or
  // staged from the input): pixel stride in elements and row stride in pixels, padded by the
  // host's bank-conflict model (models/lds_layout.py) so the fragment reads are conflict-free
  int xpix = 0, xrow = 0;
};

struct ConvStackArgs {
  const bf16* x = nullptr;            // network input [B][H][W][Cs]
  int B = 0, n = 0;
  uint32_t seed = 0;
  const StepState* st = nullptr;
  int off_w = 0, off_buf[2] = {0, 0}, off_codes = 0, lds_bytes = 0;   // LDS layout (bytes)
  int off_codes2 = 0;                 // second argmax-code plane (odd layers)
  int off_bias = 0;                   // LDS bytes: biases [MAX_STACK][64] fp32
  int dbg = 0;   // ablation (timing only, wrong results): 1 no MFMA loop, 2 no epilogue, 4 no global stores, 8 no staging;
                 // 16 = generic layer path only (A/B of the row-aligned path; results exact)
                 // 32 = all weight packs staged before layer 0 (no LDS-DMA prefetch; A/B, exact)
  int splits = 1;                     // workgroups (row bands) per image
  // per layer, per band: conv-output rows [c0, c1) computed, stage-output rows [own0, own1)
  // stored, input halo image = input rows [ib, ib + ih)
  int rows[MAX_STACK][MAX_STACK_SPLIT][6] = {};
  StackLayer L[MAX_STACK];
  unsigned long long* ts = nullptr;   // diagnostics: per-wave phase stamps [blocks*8][32]: 16 wall, 16 shader clock (null = off)
  // Prologue-free step: from_data = image b is read straight from the bound dataset through
  // the step cursor (training ? pos : eval_pos) and the epoch permutation (step_src_row), and
  // the band-0 workgroup records that dataset row in srcidx[b] for the later kernels of the
  // step (the first layer's wgrad, the head's targets); step_inc = 1: the step bookkeeping
  // runs after this launch, so the dropout counter is st->t + 1
  int from_data = 0, training = 0, step_inc = 0;
  int* srcidx = nullptr;
  // k16: a 4-channel first layer's second k-step (ONLY tap 8: k 32..35 of the 36-wide K)
  // as one v_mfma_f32_16x16x16_bf16 with a single 8-byte A read, instead of a 16x16x32 whose
  // other 28 k are zero weights
  int k16 = 0;
  // wt: stage outputs and argmax codes stored write-through (16-byte sc1 buffer stores)
  int wt = 0;
  // spec: run a specialised (layer-signature) instance when one matches (conv_stack_variant);
  // 0 = always the generic kernel (A/B and the bit-identity tests)
  int spec = 1;
};

// Weight gradient: dW[k][n] = sum_pixels im2col(x)[p][k] * dY[p][n]  (split over pixels)
struct WgradArgs {
  const bf16* x = nullptr;
  int B = 0, H = 0, W = 0, Cs_in = 0;
  int Ho = 0, Wo = 0, KH = 1, KW = 1, stride = 1, pad_t = 0, pad_l = 0;
  int Ktiles = 0;                // 16-wide k tiles over k = tap*Cs_in + ci
  const bf16* dy = nullptr;
  int Cs_dy = 0;
  int NT = 0;                    // 16-wide n tiles
  int P = 0;                     // pixels (B*Ho*Wo)
  int px_per_split = 0;          // multiple of 32
  int KT = 0;                    // k tiles per workgroup (grid.y groups)
  float* slab = nullptr;         // [S][Ktiles*16][NT*16]
  float* bslab = nullptr;        // [S][NT*16] or null
  // halo-staged spatial variant: R output rows per block, blocks_per_split blocks per WG;
  // dY given as pooled gradient dP [B, dHp, dWp, Cs_dy] + codes when dy_code != null
  int R = 1, blocks_per_split = 1;
  const uint8_t* dy_code = nullptr;
  int dHp = 0, dWp = 0;
  // >= 16 zero bytes: LDS-DMA source of padded rows (set => wgrad_tile uses the DMA path
  // when it applies: 8 n-tiles per workgroup, unpooled dY)
  const bf16* zero = nullptr;
  int dbg = 0;   // ablation (timing only): 1 skip staging, 2 skip MFMA, 4 skip slab stores;
                 // 16 = per-pixel unpool staging of pooled dY (A/B, exact)
  unsigned long long* ts = nullptr;   // diagnostics: per-workgroup [start, end] wall clock (null = off)
  unsigned long long* ts2 = nullptr;  // diagnostics: per-workgroup [16] phase stamps (null = off)
  // dense_wgrad with ONE split and the identity layout (slab == the Keras gradient): when
  // opt_w >= 0 the kernel applies `opt` to the weight elements opt_w + f*ld + n (and, with a
  // bias, opt_b + n) as soon as their gradient is final -- no slab reduction for the layer
  OptimArgs opt;
  int opt_w = -1, opt_b = -1;
  // (with opt_w: opt_nograd = 1 skips storing the in-place gradient the update consumed --
  // single-GPU step, nothing reads it; the data-parallel step never fuses the update here)
  int opt_nograd = 0;
  // ... and (pk_fwd >= 0) the updated weights' bf16 copies written into the layer's forward /
  // backward fragment packs (element offsets in opt.arena, their n-tile counts) as whole
  // 16-byte vectors from an LDS tile -- the workgroup's 32 features x NTT*16 outputs are
  // complete pack vectors of both packs, so no re-pack pass is needed for the layer
  long long pk_fwd = -1, pk_bwd = -1;
  int pk_NT = 0, pk_NTb = 0;
  int wt = 0;                    // halo kernels: slabs stored write-through (16-byte sc1 stores; < 2 GB)
  // wgrad_halo LDS layout (models/lds_layout.py picks it with a bank-conflict model; 0 =
  // dense): X-halo pixel stride in elements, X-halo row stride in pixels, dY row stride
  int xpix = 0, xrow = 0, dyld = 0;
  int kperm = 0;                 // bit0: k index 8g+j <-> pixel 4g+j / 16+4g+j-4; bit1: no row-aligned fast path
  // xidx != null: image b of x is dataset row xidx[b] of st->data_x (prologue-free step)
  const int* xidx = nullptr;
  const StepState* xst = nullptr;
};

// Dense forward, split-K partial products: part[s][m][n]
struct StepBeginArgs {
  StepState* st = nullptr;
  int training = 1;
  int bs = 0;
  int opt_kind = 0;
  float beta1 = 0.9f, beta2 = 0.999f, decay = 0.f, schedule_decay = 0.004f;
};

struct DenseFwdArgs {
  const bf16* x = nullptr;
  int M = 0, Ks = 0;             // x is [M][Ks]
  const bf16* wpk = nullptr;
  int NT = 0, KS = 0;            // pack geometry
  int splits = 1, ks_per_split = 0;
  float* part = nullptr;         // [splits][M][NT*16]
  // mode 1 (dense backward dX = dH W^T, splits == 1): route each output element (row m,
  // flattened column n over the previous stage's padded output) through bwd_through_store
  int mode = 0;
  const StepState* st = nullptr;
  BwdThrough bt;
  // book: an extra last workgroup runs the step bookkeeping (step_book.h) -- the training step's first
  // dense launch takes it over when no prologue launch runs (the conv stack before it reads
  // the iteration count as t + 1, see ConvStackArgs::step_inc)
  int book = 0;
  StepBeginArgs sb;
};

// Split-K reduction + bias + activation + dropout -> bf16 [M][Ns]
struct DenseEpiArgs {
  const float* part = nullptr;
  int splits = 1, M = 0, N = 0, Ns = 0, ldp = 0;
  const float* bias = nullptr;
  int relu = 0;
  bf16* out = nullptr;
  uint32_t drop_thr = 0;
  float drop_scale = 1.f;
  uint32_t seed = 0, stream_id = 0;
  const StepState* st = nullptr;
};

// Fused output head: logits = h @ W + b, activation, loss, metrics, and (training)
// dz, dW/db partial slabs and dh_prev (through the previous dense's relu/dropout).
struct HeadArgs {
  const bf16* h = nullptr;       // [M][Ks]
  int M = 0, K = 0, Ks = 0, N = 0;
  int flat_C = 0, flat_Cs = 0;   // flatten mapping of h's columns (keras k -> padded)
  const float* w = nullptr;      // fp32 master kernel [K][N] (keras layout)
  const float* bias = nullptr;
  const float* y = nullptr;      // targets [M][N]
  int act = 0;                   // 0 linear(mse), 1 sigmoid(bce), 2 softmax(cce)
  int training = 0;
  float inv_bs = 1.f;
  StepState* st = nullptr;       // metrics accumulation
  float* probs = nullptr;        // predict mode: [M][N]
  float* wslab = nullptr;        // [nblocks][K][N]
  float* bslab = nullptr;        // [nblocks][N]
  // gradient wrt the previous stage (hidden dense or flattened conv); bt.dy == null: skip
  BwdThrough bt;
  // fused epilogue of the previous dense layer (epi.part != null): the head's workgroup
  // reduces the split-K partials of its rows itself (bias, ReLU, dropout), writes that
  // layer's bf16 output and uses it as h -- one launch instead of two
  DenseEpiArgs epi;
  unsigned long long* ts = nullptr;   // diagnostics: [block][8] phase stamps (null = off)
  // yidx != null: row m's targets are dataset row yidx[m] of st->data_y (prologue-free step)
  const int* yidx = nullptr;
  // A/B + tests: 1 = the generic serial epilogue / loss path even where the fast paths apply
  // (bit-identical results: tests/test_hip_model.py::test_head_fast_paths_bit_identical)
  int generic = 0;
};

struct GatherArgs {
  const bf16* xs = nullptr;      // dataset [Nd][R] bf16
  const float* ys = nullptr;     // [Nd][C]
  const int* perm = nullptr;     // or null (identity / eval)
  const StepState* st = nullptr;
  int bs = 0, R = 0, C = 0, Nd = 0;
  bf16* xb = nullptr;
  float* yb = nullptr;
  int skip_x = 0;                // images read straight from the dataset by the conv stack
};


// One launch opening every step: batch gather (workgroups [0, gather_blocks)), weight
// re-pack of the previous update (the rest; pack_mode 1 always, 2 only if st->packs_stale),
// and the step bookkeeping (workgroup 0; in a prologue-free step, an extra workgroup of the first dense launch).
struct PrologueArgs {
  StepBeginArgs sb;
  GatherArgs ga;
  int gather_gx = 1;             // workgroups per batch row
  int gather_blocks = 0;         // gather_gx * bs
  int pack_mode = 0;             // 0 none, 1 always, 2 if stale
  const float* master = nullptr;
  bf16* arena = nullptr;
};


// Slab reduction descriptors: sum split-partials into the flat fp32 grad buffer in
// Keras layout.
enum RedType { RED_CONVW = 0, RED_BIAS = 1, RED_FLATW = 2 };

struct RedDesc {
  const float* slab;
  long long stride_s;  // elements between consecutive splits
  int S;
  int ld;              // row stride (n) of the slab
  int dst_off, numel, type;
  int KH, KW, Cin, Cout, Cs;   // conv: k = tap*Cs + ci ; flat: C=Cin (channels), Cs
  int tpe;             // threads per element (1..256, power of 2): lanes split the S partials
  int blk0;            // first workgroup of this descriptor in the launch
  int vec4;            // 1: identity layout, 4 consecutive elements per thread (float4 traffic)
  int tile;            // vec4 + a workgroup's 1024 elements are whole 8-row groups (Cout | 128):
                       // the fused optimizer writes its pack route as whole 16-byte vectors
};

#define MAX_RED 16
struct RedTable {
  int n;
  int nblocks;         // total workgroups of the launch
  int pad_[2];
  RedDesc d[MAX_RED];
};

// Producer push (xGMI data plane, P > 1): the thread that finalises an element of the early
// (head / dense) bucket's reduced gradient also stores it straight into its owner's inbox row
// -- phase 1 of the step's fused all-reduce (xgmi.hip) happens inside the backward, behind
// the conv layers still running, and the all-reduce kernel skips those elements.
//
// Exchange (mode 2): a LATER backward launch's extra workgroups finish that bucket's part of
// the all-reduce and apply its update, so the head / dense layers' whole all-reduce + Adam
// runs inside the backward and the fused all-reduce kernel is left with the conv layers:
//   mode 1 (first dual launch): reduce the table block, push each element to its owner's
//          inbox row, raise the block's push flag bflag1[blk][me] on every rank;
//   mode 2 (next dual launch): the owner of a block's elements waits for every sender's push
//          flag, sums the rows in rank order, pushes the sum into every peer's outbox and raises
//          bflag2[blk][me] on every rank; every rank waits for the owners of the block's other
//          elements and reads their sums; then the Keras update of the block (tiled dense
//          pack writes, as the single-GPU early reduction).
// Every wait depends only on other GPUs' earlier launches or on the same block of the same
// launch on another GPU, whose owner part precedes its wait -- no cycle.  Ranks sharing a
// GPU use nx workgroups looping over the blocks in order (a few spinning workgroups cannot
// starve the peers' launches).  Sequence numbers: ctrb[blk] + 1 (ctrb advanced by mode 2).
#define XGMI_MAX_RANKS 8
struct XgmiPush {
  int on = 0, rank = 0, size = 1, chunk = 0;
  long long lo = 0;                      // first flat element of the all-reduce bucket
  float* inbox[XGMI_MAX_RANKS] = {};     // rank j's inbox [P][chunk] (as mapped here)
  int mode = 1;                          // 1 reduce + push (+ block flags), 2 exchange + update,
                                         // 3 both in one launch (the end-of-backward bucket),
                                         // 4 / 5 the owner / finish halves of 2 (reduce_body.h)
  float* outbox[XGMI_MAX_RANKS] = {};    // rank j's outbox [P * chunk] (bucket index)
  unsigned* bflag1[XGMI_MAX_RANKS] = {}; // rank j's per-block push flags [nblk][P] (null: no flags)
  unsigned* bflag2[XGMI_MAX_RANKS] = {}; // rank j's per-block owner-sum flags [nblk][P]
  unsigned* abort_[XGMI_MAX_RANKS] = {}; // rank j's sticky abort word
  unsigned* ctrb = nullptr;              // [nblk] this rank's per-block sequence counters
  int* err = nullptr;                    // the all-reduce's error record (xgmi.hip wait_all)
  long long timeout_ticks = 0;
  int nblk = 0;                          // blocks of the table
  int nx = 0;                            // mode 2: workgroups looping over the blocks (0: one each)
  int p1 = 0;                            // size 1, mode 3: 1 = keep the exchange structure (push /
                                         // flag / re-read: a measurement of its fixed cost); 0 =
                                         // reduce + update in place (no peers: nothing to exchange)
  int b_lo = 0, b_hi = 0;                // mode 4: the table blocks [b_lo, b_hi) its workgroups cover
  int fence = 1;                         // 1: system-scope release before a flag store, acquire after
                                         // a poll (HIP memory model); 3: none (uncached payload:
                                         // drained stores + sc1 loads; opt-in, xgmi.hip header)
};

// Optional extra workgroups of the dual conv backward launch: the fused reduction + optimizer
// of an EARLY bucket (gradients final before that launch, weights no later kernel of the step
// reads), run in n_r workgroups of the same grid (after the conv ones, or before: rfirst).
struct DualExtra {
  RedTable rt;
  OptimArgs ro;
  float* grad = nullptr;
  int n_r = 0, rfirst = 0;
  XgmiPush xp;                   // (ro.grad_only tables) push the reduced elements to their owners
};

// Fused data-parallel all-reduce + optimizer over xGMI peer memory (xgmi.hip).  Every rank
// owns chunk r = [r*chunk, (r+1)*chunk) of the flat gradient.  One launch per step:
//   1. push: workgroup w sends its slice [w*sub, (w+1)*sub) of EVERY chunk j to owner j's
//      inbox row r (remote stores over xGMI), then flags owner j (flag1[w][r] = seq);
//   2. reduce: owner r waits for the P flags of its slice, sums inbox rows 0..P-1 in rank
//      order (deterministic), pushes the sum into every rank's outbox, flags them (flag2);
//   3. update: every rank waits for the P owners' flags and applies the optimizer to the
//      whole reduced gradient (identical inputs -> identical weights on every rank).
// Flags carry a per-workgroup sequence number (ctr[w] + 1), so they never need resetting.
// Communication memory is uncached device memory shared by IPC handles; every wait is
// bounded in time (timeout_ticks) and sets *err instead of hanging.
#define XGMI_MAX_WG 256
struct XgmiArgs {
  int rank = 0, size = 1;
  int n = 0;                     // gradient elements of the bucket (grad points at its start)
  int chunk = 0;                 // elements per owner chunk (multiple of 4)
  int sub = 0;                   // elements per workgroup slice of a chunk (multiple of 4)
  long long timeout_ticks = 0;   // bounded waits: give up after this many wall_clock64 ticks (100 MHz)
  int mode = 1;                  // 0: sum only (reduced gradient -> grad); 1: + optimizer
  int fence = 1;                 // fences around the flags: 1 system release + acquire (default),
                                 // 3 none + sc1 payload loads, 2 agent acquire, 0 none (xgmi.hip)
  // bucket elements [skip_lo, skip_hi) were pushed to their owners already (XgmiPush, in the
  // backward): phase 1 skips every float4 wholly inside; skip_mode 2: they were also
  // all-reduced and updated there (exchange), so no phase touches them
  long long skip_lo = 0, skip_hi = 0;
  int skip_mode = 0;
  float* grad = nullptr;         // local bucket gradient (read in 1, reduced sum written in 2/3)
  float* inbox[XGMI_MAX_RANKS] = {};     // rank j's inbox [P][chunk] (as mapped here)
  float* outbox[XGMI_MAX_RANKS] = {};    // rank j's outbox [P * chunk] = reduced gradient
  unsigned* flag1[XGMI_MAX_RANKS] = {};  // rank j's phase-1 flags [XGMI_MAX_WG][P]
  unsigned* flag2[XGMI_MAX_RANKS] = {};  // rank j's phase-2 flags [XGMI_MAX_WG][P]
  unsigned* abort_[XGMI_MAX_RANKS] = {}; // rank j's sticky abort word (set by any rank that gives up)
  unsigned* ctr = nullptr;       // [XGMI_MAX_WG] local sequence counters
  int* err = nullptr;            // [4]: phase (1, 2) of a timed-out wait, 3 = a peer aborted;
                                 // on a timeout also seq waited for, flag value seen, wg * 64 + peer
  OptimArgs opt;                 // p / s0 / s1 point at the bucket's first element
};

// K16 (synth.hip): parameter initialiser over one flat span -- kind 0 zeros, 1 ones,
// 2 uniform(-scale, scale) from rng_u32(element, seed, stream, 0)
struct InitArgs {
  float* p = nullptr;
  int n = 0, kind = 0;
  float scale = 0.f;
  uint32_t seed = 0, stream = 0;
};

// K16 (synth.hip): synthetic samples [first, first + n) of a data stream -- kind 0 uniform
// [0, 1) pixels, 1 RPV-like jet images, 2 MNIST-like class templates + noise; x bf16
// [n][H][W][Cs] (channels >= C zero), y fp32 [n][ncls] (one-hot, or the 0/1 label)
struct SynthArgs {
  bf16* x = nullptr;
  float* y = nullptr;
  int n = 0, first = 0, H = 0, W = 0, C = 1, Cs = 1, ncls = 1, kind = 0;
  uint32_t seed = 0;
};
