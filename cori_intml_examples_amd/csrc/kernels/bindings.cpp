#include <algorithm>
// pybind11 bindings for the gfx950 kernels.  Argument structs are exposed as Python
// classes (pointer fields take integer device addresses, e.g. tensor.data_ptr()); the
// launch_* functions take the HIP stream as an integer (torch stream.cuda_stream), so
// every launch is capturable into a HIP graph by torch.cuda.graph.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "args.h"

namespace py = pybind11;

void launch_conv_halo(const ConvMMArgs& a, int ntc, hipStream_t s);
size_t conv_halo_lds_bytes(const ConvMMArgs& a, int ntc);
void launch_conv_tile(const ConvMMArgs& a, int ntc, hipStream_t s, bool big, int nbuf);
bool launch_conv_hs(const ConvMMArgs& a, int ntc, hipStream_t s, int nwv, int order);
bool conv_hs_ok(const ConvMMArgs& a, int ntc, int nwv);
long long conv_tile_big_blocks(const ConvMMArgs& a, int ntc);
size_t conv_tile_lds_bytes(int ntc);
void launch_wgrad_tile(const WgradArgs& a, int ntc, hipStream_t s);
size_t wgrad_tile_lds_bytes(int ntc);
void launch_wgrad_halo(const WgradArgs& a, int MT, int NTT, int splits, hipStream_t s);
size_t wgrad_halo_lds_bytes(const WgradArgs& a, int MT, int NTT);
int wgrad_halo_resident(const WgradArgs& a, int MT, int NTT, bool bias);
int head_rows_per_block(bool fused);
int head_epi_max();
void launch_wgrad(const WgradArgs& a, int ktw, int ntt, int splits, hipStream_t s);
size_t wgrad_lds_bytes(int KT, int NTT);
void launch_dense_fwd(const DenseFwdArgs& a, hipStream_t s);
void launch_dense_epi(const DenseEpiArgs& a, hipStream_t s);
int dense_groups(int M, int NT, int KS);
bool dense_big(int NT, int KS);
void launch_head(const HeadArgs& a, hipStream_t s);
bool launch_dual_halo(const ConvMMArgs& ca, int ntc, const WgradArgs& wa, int MT, int NTT, int splits,
                      const DualExtra& x, hipStream_t s);
bool launch_dense_bwd_dual(const WgradArgs& wa, int ktw, int ntt, int splits, const DenseFwdArgs& da,
                           hipStream_t s);
void launch_dense_wgrad(const WgradArgs& a, int kg, int ntt, int splits, hipStream_t s, int order, bool late);
size_t dense_wgrad_lds_bytes(int kg, int ntt);
void launch_dense_dx(const DenseFwdArgs& a, int ntc, hipStream_t s);
void launch_dense_bwd_pair(const WgradArgs& wa, int kg, int ntt, int splits, const DenseFwdArgs& da, int ntc,
                           hipStream_t s);
void launch_conv_stack_fwd(const ConvStackArgs& a, hipStream_t s);
void launch_init_params(const InitArgs& a, hipStream_t s);
void launch_synth(const SynthArgs& a, hipStream_t s);
int conv_stack_threads();
int conv_stack_variant(const ConvStackArgs& a);
int conv_stack_tabn();
void launch_prologue(const PrologueArgs& a, const PackTable& tab, hipStream_t s);
int gather_gx(int R);
void launch_slab_reduce(float* grad, int lo, int hi, const RedTable& tab, hipStream_t s);
void launch_reduce_optim_end(float* grad, const RedTable& tc, const OptimArgs& a, const XgmiPush& xc,
                             const RedTable& te, const XgmiPush& xe, hipStream_t s);
void launch_reduce_optim(float* grad, const RedTable& tab, const OptimArgs& a, hipStream_t s,
                         const XgmiPush* xp = nullptr);
void launch_optim(const OptimArgs& a, const PackTable& tab, hipStream_t s);
void launch_pack(const float* master, bf16* arena, const PackTable& tab, hipStream_t s);
int xgmi_grid(const XgmiArgs& a);
void launch_xgmi_allreduce(const XgmiArgs& a, hipStream_t s);
uintptr_t xgmi_alloc_uncached(size_t bytes, bool finegrained);
void xgmi_free(uintptr_t p);
std::string xgmi_ipc_handle(uintptr_t p);
uintptr_t xgmi_ipc_open(const std::string& handle);
void xgmi_ipc_close(uintptr_t p);

static hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

#define RW(cls, f) .def_readwrite(#f, &cls::f)
#define PTR(cls, f)                                                                   \
  .def_property(                                                                      \
      #f, [](const cls& o) { return reinterpret_cast<uintptr_t>(o.f); },              \
      [](cls& o, uintptr_t v) { o.f = reinterpret_cast<decltype(o.f)>(v); })

static void check_last(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// host-side checks of an early-bucket xGMI push / exchange (XgmiPush, args.h) against its
// reduction table: every pointer the device code dereferences, the block count its flags are
// indexed by, and float4 groups that never straddle an owner chunk
// slab partials per split-lane the automatic split-lane choice of RedTable.add aims at
// (INTML_TUNE red_lanes; set before the tables are built)
static int g_red_lanes = 16;

static void check_xgmi_push(const XgmiPush& x, const RedTable& t, const OptimArgs& a) {
  if (x.size < 1 || x.size > XGMI_MAX_RANKS || x.rank < 0 || x.rank >= x.size || x.chunk <= 0 || x.chunk % 4)
    throw std::invalid_argument("xgmi push: ranks / chunk");
  if (x.mode < 1 || x.mode > 5) throw std::invalid_argument("xgmi push: mode");
  if (x.mode == 4 && (x.b_lo < 0 || x.b_hi > t.nblocks || x.b_lo > x.b_hi))
    throw std::invalid_argument("xgmi push: mode-4 block range");
  if (x.size == 1 && x.mode == 1 && !x.bflag1[0]) throw std::invalid_argument("xgmi push: nothing to push");
  if ((x.mode == 1) != (a.grad_only != 0))
    throw std::invalid_argument("xgmi push: mode 1 needs a grad_only table, mode 2 an updating one");
  const bool flags = x.mode >= 2 || x.bflag1[0] != nullptr;
  for (int j = 0; j < x.size; ++j) {
    if (!x.inbox[j]) throw std::invalid_argument("xgmi push: inbox");
    if (flags && !x.bflag1[j]) throw std::invalid_argument("xgmi push: block flags");
    if (x.mode >= 2 && (!x.outbox[j] || !x.bflag2[j] || !x.abort_[j])) throw std::invalid_argument("xgmi push: peers");
  }
  if (flags && (!x.ctrb || x.nblk != t.nblocks)) throw std::invalid_argument("xgmi push: block counters / nblk");
  if (x.mode >= 2 && (!x.err || x.timeout_ticks <= 0 || x.nx < 0)) throw std::invalid_argument("xgmi push: err / timeout");
  for (int i = 0; i < t.n; ++i) {
    const RedDesc& d = t.d[i];
    if (d.dst_off < x.lo || d.dst_off + (long long)d.numel > x.lo + (long long)x.chunk * x.size)
      throw std::invalid_argument("xgmi push: table outside the bucket");
    if (d.vec4 && ((d.dst_off - x.lo) % 4 || d.numel % 4)) throw std::invalid_argument("xgmi push: float4 alignment");
  }
}

PYBIND11_MODULE(_kernels, m) {
  m.doc() = "cori_intml_examples_amd gfx950 HIP kernels";

  py::class_<BwdThrough>(m, "BwdThrough")
      .def(py::init<>())
      PTR(BwdThrough, prev_out) PTR(BwdThrough, prev_code) RW(BwdThrough, prev_relu)
      RW(BwdThrough, prev_pool) RW(BwdThrough, pH) RW(BwdThrough, pW) RW(BwdThrough, pC)
      RW(BwdThrough, pCs) RW(BwdThrough, cH) RW(BwdThrough, cW) RW(BwdThrough, drop_thr)
      RW(BwdThrough, drop_scale) RW(BwdThrough, seed) RW(BwdThrough, stream_id) PTR(BwdThrough, dy) RW(BwdThrough, wt);

  py::class_<ConvMMArgs>(m, "ConvMMArgs")
      .def(py::init<>())
      PTR(ConvMMArgs, x) RW(ConvMMArgs, B) RW(ConvMMArgs, H) RW(ConvMMArgs, W) RW(ConvMMArgs, Cs_in)
      RW(ConvMMArgs, Ho) RW(ConvMMArgs, Wo) RW(ConvMMArgs, KH) RW(ConvMMArgs, KW) RW(ConvMMArgs, stride)
      RW(ConvMMArgs, pad_t) RW(ConvMMArgs, pad_l) RW(ConvMMArgs, in_dil) RW(ConvMMArgs, KS)
      PTR(ConvMMArgs, wpk) RW(ConvMMArgs, NT) PTR(ConvMMArgs, bias) RW(ConvMMArgs, N) RW(ConvMMArgs, mode)
      RW(ConvMMArgs, flat_out) RW(ConvMMArgs, relu) RW(ConvMMArgs, pool) PTR(ConvMMArgs, out)
      RW(ConvMMArgs, Cs_out) RW(ConvMMArgs, Hp) RW(ConvMMArgs, Wp) PTR(ConvMMArgs, code)
      RW(ConvMMArgs, drop_thr) RW(ConvMMArgs, drop_scale) RW(ConvMMArgs, seed) RW(ConvMMArgs, stream_id)
      PTR(ConvMMArgs, st) RW(ConvMMArgs, bt) RW(ConvMMArgs, R) PTR(ConvMMArgs, in_code) PTR(ConvMMArgs, zero)
      RW(ConvMMArgs, in_pH) RW(ConvMMArgs, in_pW) RW(ConvMMArgs, dbg) PTR(ConvMMArgs, ts) RW(ConvMMArgs, xpix) RW(ConvMMArgs, kpipe) RW(ConvMMArgs, tm);

  py::class_<WgradArgs>(m, "WgradArgs")
      .def(py::init<>())
      PTR(WgradArgs, x) RW(WgradArgs, B) RW(WgradArgs, H) RW(WgradArgs, W) RW(WgradArgs, Cs_in)
      RW(WgradArgs, Ho) RW(WgradArgs, Wo) RW(WgradArgs, KH) RW(WgradArgs, KW) RW(WgradArgs, stride)
      RW(WgradArgs, pad_t) RW(WgradArgs, pad_l) RW(WgradArgs, Ktiles) PTR(WgradArgs, dy)
      RW(WgradArgs, Cs_dy) RW(WgradArgs, NT) RW(WgradArgs, P) RW(WgradArgs, px_per_split)
      RW(WgradArgs, KT) PTR(WgradArgs, slab) PTR(WgradArgs, bslab) RW(WgradArgs, R)
      RW(WgradArgs, blocks_per_split) PTR(WgradArgs, dy_code) PTR(WgradArgs, zero) RW(WgradArgs, dHp) RW(WgradArgs, dWp)
      RW(WgradArgs, dbg) PTR(WgradArgs, ts) PTR(WgradArgs, ts2) RW(WgradArgs, opt) RW(WgradArgs, opt_w)
      RW(WgradArgs, opt_b) RW(WgradArgs, xpix) RW(WgradArgs, xrow) RW(WgradArgs, dyld) RW(WgradArgs, kperm)
      PTR(WgradArgs, xidx) PTR(WgradArgs, xst) RW(WgradArgs, pk_fwd) RW(WgradArgs, pk_bwd) RW(WgradArgs, pk_NT)
      RW(WgradArgs, pk_NTb) RW(WgradArgs, wt) RW(WgradArgs, opt_nograd);

  py::class_<DenseFwdArgs>(m, "DenseFwdArgs")
      .def(py::init<>())
      PTR(DenseFwdArgs, x) RW(DenseFwdArgs, M) RW(DenseFwdArgs, Ks) PTR(DenseFwdArgs, wpk)
      RW(DenseFwdArgs, NT) RW(DenseFwdArgs, KS) RW(DenseFwdArgs, splits) RW(DenseFwdArgs, ks_per_split)
      PTR(DenseFwdArgs, part) RW(DenseFwdArgs, mode) PTR(DenseFwdArgs, st) RW(DenseFwdArgs, bt)
      RW(DenseFwdArgs, book) RW(DenseFwdArgs, sb);

  py::class_<DenseEpiArgs>(m, "DenseEpiArgs")
      .def(py::init<>())
      PTR(DenseEpiArgs, part) RW(DenseEpiArgs, splits) RW(DenseEpiArgs, M) RW(DenseEpiArgs, N)
      RW(DenseEpiArgs, Ns) RW(DenseEpiArgs, ldp) PTR(DenseEpiArgs, bias) RW(DenseEpiArgs, relu)
      PTR(DenseEpiArgs, out) RW(DenseEpiArgs, drop_thr) RW(DenseEpiArgs, drop_scale)
      RW(DenseEpiArgs, seed) RW(DenseEpiArgs, stream_id) PTR(DenseEpiArgs, st);

  py::class_<HeadArgs>(m, "HeadArgs")
      .def(py::init<>())
      PTR(HeadArgs, h) RW(HeadArgs, M) RW(HeadArgs, K) RW(HeadArgs, Ks) RW(HeadArgs, N)
      RW(HeadArgs, flat_C) RW(HeadArgs, flat_Cs) PTR(HeadArgs, w) PTR(HeadArgs, bias) PTR(HeadArgs, y)
      RW(HeadArgs, act) RW(HeadArgs, training) RW(HeadArgs, inv_bs) PTR(HeadArgs, st) PTR(HeadArgs, probs)
      PTR(HeadArgs, wslab) PTR(HeadArgs, bslab) RW(HeadArgs, bt) RW(HeadArgs, epi) PTR(HeadArgs, ts)
      PTR(HeadArgs, yidx) RW(HeadArgs, generic);


  py::class_<GatherArgs>(m, "GatherArgs")
      .def(py::init<>())
      PTR(GatherArgs, xs) PTR(GatherArgs, ys) PTR(GatherArgs, perm) PTR(GatherArgs, st)
      RW(GatherArgs, bs) RW(GatherArgs, R) RW(GatherArgs, C) RW(GatherArgs, Nd) PTR(GatherArgs, xb)
      PTR(GatherArgs, yb) RW(GatherArgs, skip_x);

  py::class_<StepBeginArgs>(m, "StepBeginArgs")
      .def(py::init<>())
      PTR(StepBeginArgs, st) RW(StepBeginArgs, training) RW(StepBeginArgs, bs) RW(StepBeginArgs, opt_kind)
      RW(StepBeginArgs, beta1) RW(StepBeginArgs, beta2) RW(StepBeginArgs, decay)
      RW(StepBeginArgs, schedule_decay);

  py::class_<StackLayer>(m, "StackLayer")
      .def(py::init<>())
      RW(StackLayer, H) RW(StackLayer, W) RW(StackLayer, Cs_in) RW(StackLayer, Ho) RW(StackLayer, Wo)
      RW(StackLayer, Cout) RW(StackLayer, Cs_out) RW(StackLayer, KH) RW(StackLayer, KW) RW(StackLayer, pad_t)
      RW(StackLayer, pad_l) RW(StackLayer, KS) RW(StackLayer, NT) RW(StackLayer, pool) RW(StackLayer, relu)
      RW(StackLayer, Hp) RW(StackLayer, Wp) RW(StackLayer, drop_thr) RW(StackLayer, drop_scale)
      RW(StackLayer, stream_id) PTR(StackLayer, wpk) PTR(StackLayer, bias) PTR(StackLayer, out)
      PTR(StackLayer, code) RW(StackLayer, w_lds) RW(StackLayer, xpix) RW(StackLayer, xrow);

  py::class_<ConvStackArgs>(m, "ConvStackArgs")
      .def(py::init<>())
      PTR(ConvStackArgs, x) RW(ConvStackArgs, B) RW(ConvStackArgs, n) RW(ConvStackArgs, seed)
      PTR(ConvStackArgs, st) RW(ConvStackArgs, dbg) RW(ConvStackArgs, off_w) RW(ConvStackArgs, off_codes) RW(ConvStackArgs, off_codes2) RW(ConvStackArgs, lds_bytes)
      .def("set_buf_offsets", [](ConvStackArgs& a, int b0, int b1) { a.off_buf[0] = b0; a.off_buf[1] = b1; })
      RW(ConvStackArgs, splits) PTR(ConvStackArgs, ts) RW(ConvStackArgs, off_bias)
      RW(ConvStackArgs, from_data) RW(ConvStackArgs, training) RW(ConvStackArgs, step_inc) PTR(ConvStackArgs, srcidx) RW(ConvStackArgs, k16) RW(ConvStackArgs, wt) RW(ConvStackArgs, spec)
      .def("set_rows", [](ConvStackArgs& a, int l, int sp, int c0, int c1, int o0, int o1, int ib, int ih) {
        if (l < 0 || l >= MAX_STACK || sp < 0 || sp >= MAX_STACK_SPLIT) throw std::out_of_range("conv stack rows");
        const int v[6] = {c0, c1, o0, o1, ib, ih};
        for (int i = 0; i < 6; ++i) a.rows[l][sp][i] = v[i];
      })
      .def("set_layer", [](ConvStackArgs& a, int i, const StackLayer& l) {
        if (i < 0 || i >= MAX_STACK) throw std::out_of_range("conv stack layer index");
        a.L[i] = l;
      });

  py::class_<InitArgs>(m, "InitArgs")
      .def(py::init<>())
      PTR(InitArgs, p) RW(InitArgs, n) RW(InitArgs, kind) RW(InitArgs, scale) RW(InitArgs, seed) RW(InitArgs, stream);
  py::class_<SynthArgs>(m, "SynthArgs")
      .def(py::init<>())
      PTR(SynthArgs, x) PTR(SynthArgs, y) RW(SynthArgs, n) RW(SynthArgs, first) RW(SynthArgs, H) RW(SynthArgs, W)
      RW(SynthArgs, C) RW(SynthArgs, Cs) RW(SynthArgs, ncls) RW(SynthArgs, kind) RW(SynthArgs, seed);
  m.def("init_params", [](const InitArgs& a, uintptr_t s) { launch_init_params(a, S(s)); check_last("init_params"); });
  m.def("synth", [](const SynthArgs& a, uintptr_t s) { launch_synth(a, S(s)); check_last("synth"); });

  py::class_<PrologueArgs>(m, "PrologueArgs")
      .def(py::init<>())
      RW(PrologueArgs, sb) RW(PrologueArgs, ga) RW(PrologueArgs, gather_gx) RW(PrologueArgs, gather_blocks)
      RW(PrologueArgs, pack_mode) PTR(PrologueArgs, master) PTR(PrologueArgs, arena);

  py::class_<OptimArgs>(m, "OptimArgs")
      .def(py::init<>())
      PTR(OptimArgs, p) PTR(OptimArgs, g) PTR(OptimArgs, s0) PTR(OptimArgs, s1) RW(OptimArgs, n) RW(OptimArgs, lo)
      PTR(OptimArgs, st) RW(OptimArgs, kind) RW(OptimArgs, beta1) RW(OptimArgs, beta2) RW(OptimArgs, eps)
      RW(OptimArgs, rho) RW(OptimArgs, momentum) RW(OptimArgs, nesterov) RW(OptimArgs, grad_scale)
      RW(OptimArgs, grad_only)
      RW(OptimArgs, pack_only) RW(OptimArgs, defer_pack) PTR(OptimArgs, arena) PTR(OptimArgs, routes)
      RW(OptimArgs, nroutes) RW(OptimArgs, ntile) RW(OptimArgs, flat_blocks)
      .def("set_tile", [](OptimArgs& a, int i, int route, int b0) {
        if (i < 0 || i > 4) throw std::out_of_range("optim tile index");
        if (i < 4) a.tile_route[i] = route;
        a.tile_b0[i] = b0;
      });

  py::class_<PackTable>(m, "PackTable")
      .def(py::init([]() { PackTable t; memset(&t, 0, sizeof(t)); return t; }))
      .def_readonly("n", &PackTable::n)
      .def("add", [](PackTable& t, int src_off, int numel, int type, int KH, int KW, int Cin, int Cout,
                      int Cs, int NT, long long dst_off) {
        if (type == PACK_DENSE_FWD || type == PACK_DENSE_BWD) {
          // dense packs go to the tiled pair kernel: FWD opens a pair, BWD completes it
          if (type == PACK_DENSE_FWD) {
            if (t.nd >= MAX_DENSE_PAIRS) throw std::runtime_error("PackTable: too many dense layers");
            DensePair& p = t.dp[t.nd++];
            p.src_off = src_off; p.KHW = KH * KW; p.Cin = Cin; p.Cs = Cs; p.N = Cout;
            p.KS = (int)(((long long)KH * KW * Cs + 31) / 32); p.NT = NT;
            p.KSb = 0; p.NTb = 0; p.dst_fwd = dst_off; p.dst_bwd = -1;
          } else {
            if (t.nd == 0 || t.dp[t.nd - 1].src_off != src_off)
              throw std::runtime_error("PackTable: dense BWD pack must follow its FWD pack");
            DensePair& p = t.dp[t.nd - 1];
            p.KSb = (Cout + 31) / 32; p.NTb = NT; p.dst_bwd = dst_off;
          }
          t.dblocks = 0;
          for (int i = 0; i < t.nd; ++i) {
            DensePair& p = t.dp[i];
            const int ncols = std::max(p.NT * 16, p.KSb * 32);
            p.ntn = (ncols + 127) / 128;
            p.blk0 = t.dblocks;
            t.dblocks += p.KS * p.ntn;
          }
          return;
        }
        if (t.n >= MAX_PACK) throw std::runtime_error("PackTable full");
        PackDesc& d = t.d[t.n++];
        d.src_off = src_off; d.numel = numel; d.type = type; d.KH = KH; d.KW = KW; d.Cin = Cin;
        d.Cout = Cout; d.Cs = Cs; d.NT = NT; d.dst_off = dst_off;
        long long krows;   // k extent of the pack
        if (type == PACK_CONV_FWD || type == PACK_CONV_DGRAD) krows = (long long)KH * KW * Cs;
        else if (type == PACK_DENSE_FWD) krows = (long long)KH * KW * Cs;
        else krows = Cout;
        d.KS = (int)((krows + 31) / 32);
        d.nvec = d.KS * NT * 64;
        d.blk0 = t.nblocks;
        t.nblocks += (d.nvec + 255) / 256;
      });

  py::class_<RedTable>(m, "RedTable")
      .def(py::init([]() { RedTable t; memset(&t, 0, sizeof(t)); return t; }))
      .def_readonly("n", &RedTable::n)
      .def_readonly("nblocks", &RedTable::nblocks)
      .def("owned_blocks", [](const RedTable& t, long long lo, int chunk, int rank) {
        // [b_lo, b_hi): the table blocks some element of which falls in owner chunk `rank` of
        // the bucket starting at flat element lo (the blocks a mode-4 launch must cover) --
        // the element map of reduce_body.h (vec4: 1024 / tpe elements per block, else 256 / tpe)
        int b_lo = t.nblocks, b_hi = 0;
        const long long c_lo = lo + (long long)rank * chunk, c_hi = c_lo + chunk;
        for (int i = 0; i < t.n; ++i) {
          const RedDesc& d = t.d[i];
          const int epb = d.vec4 ? 1024 / d.tpe : 256 / d.tpe;
          const int nb = (d.numel + epb - 1) / epb;
          for (int k = 0; k < nb; ++k) {
            const long long e0 = d.dst_off + (long long)k * epb, e1 = std::min<long long>(e0 + epb, d.dst_off + d.numel);
            if (e0 < c_hi && e1 > c_lo) b_lo = std::min(b_lo, d.blk0 + k), b_hi = std::max(b_hi, d.blk0 + k + 1);
          }
        }
        return b_hi > b_lo ? std::make_pair(b_lo, b_hi) : std::make_pair(0, 0);
      })
      .def("add", [](RedTable& t, uintptr_t slab, long long stride_s, int S, int ld, int dst_off, int numel,
                      int type, int KH, int KW, int Cin, int Cout, int Cs, int tpe) {
        if (t.n >= MAX_RED) throw std::runtime_error("RedTable full");
        RedDesc& d = t.d[t.n++];
        d.slab = reinterpret_cast<const float*>(slab); d.stride_s = stride_s; d.S = S; d.ld = ld;
        d.dst_off = dst_off; d.numel = numel; d.type = type; d.KH = KH; d.KW = KW; d.Cin = Cin;
        d.Cout = Cout; d.Cs = Cs;
        // a flattened dense or conv kernel with unpadded channels and slab rows of exactly Cout
        // columns IS the Keras layout (so is a bias): 4 consecutive elements per thread, float4
        // traffic (an explicit tpe keeps the scalar path)
        const bool ident = type == RED_BIAS || ((type == RED_FLATW || type == RED_CONVW) && Cin == Cs && ld == Cout);
        d.vec4 = (ident && numel % 4 == 0 && dst_off % 4 == 0 && stride_s % 4 == 0 && tpe <= 0) ? 1 : 0;
        d.tile = (d.vec4 && type == RED_FLATW && 1024 % Cout == 0 && (1024 / Cout) % 8 == 0 && numel % 1024 == 0)
                     ? 1 : 0;
        // threads per element (power of 2, <= 64): E = 256 / tpe consecutive elements per
        // workgroup keep each slab-row read >= 16 contiguous bytes; each thread sums its
        // S / tpe partials 8 independent loads at a time
        if (d.vec4) {
          // split-lanes as the scalar path (~S/16 partials per thread); tiled dense blocks
          // need the 1024-element map (tpe 1)
          d.tpe = 1;
          while (d.tpe < 64 && d.tpe * g_red_lanes < S) d.tpe *= 2;
          if (d.tpe > 1) d.tile = 0;
        } else if (tpe > 0) {
          if (tpe > 256 || (tpe & (tpe - 1))) throw std::invalid_argument("tpe: power of 2 <= 256");
          d.tpe = tpe;
        } else {
          d.tpe = 1;                                    // ~S/16 partials per thread (sweep:
          while (d.tpe < 64 && d.tpe * g_red_lanes < S) d.tpe *= 2;   // scripts/red_sweep.py)
        }
        d.blk0 = t.nblocks;
        const int epb = d.vec4 ? 1024 / d.tpe : 256 / d.tpe;
        t.nblocks += (numel + epb - 1) / epb;
      }, py::arg("slab"), py::arg("stride_s"), py::arg("S"), py::arg("ld"), py::arg("dst_off"), py::arg("numel"),
      py::arg("type"), py::arg("KH"), py::arg("KW"), py::arg("Cin"), py::arg("Cout"), py::arg("Cs"), py::arg("tpe") = -1);

  m.attr("STEP_STATE_BYTES") = (int)sizeof(StepState);
  m.def("set_red_lanes", [](int n) {
    if (n < 1 || n > 256) throw std::invalid_argument("red_lanes: 1..256");
    g_red_lanes = n;
  });
  static_assert(sizeof(PackRoute) == 56 && offsetof(PackRoute, fwd) == 40, "PackRoute layout (models/plan routes)");
  m.attr("PACK_ROUTE_BYTES") = (int)sizeof(PackRoute);
  m.attr("MAX_ROUTES") = MAX_ROUTES;
  m.attr("STEP_STATE_METRICS_OFFSET") = (int)offsetof(StepState, metric_slots);
  m.attr("STEP_STATE_METRIC_SLOTS") = 16;
  m.attr("STEP_STATE_MSCHED_OFFSET") = (int)offsetof(StepState, m_schedule);
  m.attr("STEP_STATE_LR_OFFSET") = (int)offsetof(StepState, lr);
  m.attr("STEP_STATE_WARM_OFFSET") = (int)offsetof(StepState, warm_t0);
  m.attr("STEP_STATE_DATA_OFFSET") = (int)offsetof(StepState, data_x);
  m.attr("STEP_STATE_DATAN_OFFSET") = (int)offsetof(StepState, data_n);

  m.def("wgrad_lds_bytes", &wgrad_lds_bytes);
  m.def("conv_halo_lds_bytes", &conv_halo_lds_bytes);
  m.def("wgrad_halo_lds_bytes", &wgrad_halo_lds_bytes);
  m.def("wgrad_halo_resident", &wgrad_halo_resident);
  m.def("head_rows_per_block", &head_rows_per_block, py::arg("fused") = false);
  m.def("conv_tile_lds_bytes", &conv_tile_lds_bytes);
  m.def("conv_tile", [](const ConvMMArgs& a, int ntc, uintptr_t s, bool big, int nbuf) {
    launch_conv_tile(a, ntc, S(s), big, nbuf); check_last("conv_tile"); }, py::arg("a"), py::arg("ntc"), py::arg("s"),
    py::arg("big") = false, py::arg("nbuf") = 4);
  m.def("conv_tile_big_blocks", &conv_tile_big_blocks);
  m.def("conv_hs_ok", &conv_hs_ok, py::arg("a"), py::arg("ntc"), py::arg("nwv") = 8);
  m.def("conv_hs", [](const ConvMMArgs& a, int ntc, uintptr_t s, int nwv, int order) {
    const bool ok = launch_conv_hs(a, ntc, S(s), nwv, order); check_last("conv_hs"); return ok; },
    py::arg("a"), py::arg("ntc"), py::arg("s"), py::arg("nwv") = 8, py::arg("order") = 0,
    "halo-staged wide conv (stride 1 or the parity classes of a strided dgrad, whole-row blocks of "
    "32 * nwv rows); false (nothing launched) for other shapes");
  m.def("wgrad_tile_lds_bytes", &wgrad_tile_lds_bytes);
  m.def("wgrad_tile", [](const WgradArgs& a, int ntc, uintptr_t s) {
    launch_wgrad_tile(a, ntc, S(s)); check_last("wgrad_tile"); });
  m.def("conv_halo", [](const ConvMMArgs& a, int ntc, uintptr_t s) {
    launch_conv_halo(a, ntc, S(s)); check_last("conv_halo"); });
  m.def("wgrad_halo", [](const WgradArgs& a, int MT, int NTT, int splits, uintptr_t s) {
    launch_wgrad_halo(a, MT, NTT, splits, S(s)); check_last("wgrad_halo"); });
  m.def("wgrad", [](const WgradArgs& a, int ktw, int ntt, int splits, uintptr_t s) {
    launch_wgrad(a, ktw, ntt, splits, S(s)); check_last("wgrad"); });
  m.def("dense_fwd", [](const DenseFwdArgs& a, uintptr_t s) { launch_dense_fwd(a, S(s)); check_last("dense_fwd"); });
  m.def("dense_groups", &dense_groups, "work items per K-split of dense_fwd for (M, NT, KS)");
  m.def("dense_big", &dense_big, "dense_fwd uses the large-weight LDS path for (NT, KS)");
  m.def("dense_epi", [](const DenseEpiArgs& a, uintptr_t s) { launch_dense_epi(a, S(s)); check_last("dense_epi"); });
  m.def("head", [](const HeadArgs& a, uintptr_t s) { launch_head(a, S(s)); check_last("head"); });
  m.def("prologue", [](const PrologueArgs& a, const PackTable& t, uintptr_t s) {
    launch_prologue(a, t, S(s)); check_last("prologue"); });
  m.def("gather_gx", &gather_gx);
  m.def("head_epi_max", &head_epi_max);
  m.def("reduce_optim_end", [](uintptr_t grad, const RedTable& tc, const OptimArgs& a, uintptr_t s,
                               const XgmiPush& xc, const RedTable& te, const XgmiPush& xe) {
    if (!xc.on || !xe.on || xc.mode != 3 || xe.mode != 5) throw std::invalid_argument("reduce_optim_end: modes 3 + 5");
    check_xgmi_push(xc, tc, a);
    check_xgmi_push(xe, te, a);
    launch_reduce_optim_end(reinterpret_cast<float*>(grad), tc, a, xc, te, xe, S(s)); check_last("reduce_optim_end"); },
    "the end-of-backward table (mode 3) and the early range's finish part (mode 5) in one launch");
  m.def("reduce_optim", [](uintptr_t grad, const RedTable& t, const OptimArgs& a, uintptr_t s, const XgmiPush* xp) {
    if (xp && xp->on) check_xgmi_push(*xp, t, a);
    launch_reduce_optim(reinterpret_cast<float*>(grad), t, a, S(s), xp); check_last("reduce_optim"); },
    py::arg("grad"), py::arg("t"), py::arg("a"), py::arg("s"), py::arg("xp") = nullptr);
  m.def("dense_bwd_dual", [](const WgradArgs& wa, int ktw, int ntt, int splits, const DenseFwdArgs& da, uintptr_t s) {
    const bool ok = launch_dense_bwd_dual(wa, ktw, ntt, splits, da, S(s));
    check_last("dense_bwd_dual");
    return ok;
  });
  m.def("dense_wgrad", [](const WgradArgs& a, int kg, int ntt, int splits, uintptr_t s, int order, bool late) {
    launch_dense_wgrad(a, kg, ntt, splits, S(s), order, late); check_last("dense_wgrad"); }, py::arg("a"),
    py::arg("kg"), py::arg("ntt"), py::arg("splits"), py::arg("s"), py::arg("order") = 0, py::arg("late") = false);
  m.def("dense_wgrad_lds_bytes", &dense_wgrad_lds_bytes);
  m.def("dense_dx", [](const DenseFwdArgs& a, int ntc, uintptr_t s) {
    launch_dense_dx(a, ntc, S(s)); check_last("dense_dx"); });
  m.def("dense_bwd_pair", [](const WgradArgs& wa, int kg, int ntt, int splits, const DenseFwdArgs& da, int ntc,
                             uintptr_t s) {
    launch_dense_bwd_pair(wa, kg, ntt, splits, da, ntc, S(s)); check_last("dense_bwd_pair"); });
  m.def(
      "dual_halo",
      [](const ConvMMArgs& ca, int ntc, const WgradArgs& wa, int MT, int NTT, int splits, uintptr_t s,
         const RedTable* rt, const OptimArgs* ro, uintptr_t rgrad, int rfirst, const XgmiPush* xp) {
        DualExtra x;
        if (rt && ro && rt->nblocks > 0) {
          x.rt = *rt, x.ro = *ro, x.grad = reinterpret_cast<float*>(rgrad);
          x.n_r = rt->nblocks, x.rfirst = rfirst;
          if (xp && xp->on) {
            check_xgmi_push(*xp, *rt, *ro);
            x.xp = *xp;
            if (xp->mode >= 2 && xp->nx) x.n_r = xp->nx;   // (workgroups looping over the blocks)
            else if (xp->mode == 4) x.n_r = xp->b_hi - xp->b_lo;   // (the blocks it may own a part of)
            if (xp->mode == 3 || xp->mode == 5) throw std::invalid_argument("dual_halo: exchange modes 1 / 2 / 4 only");
            // (mode 2: launch_dual_halo declines it -- the caller runs the three launches apart)
          }
        }
        const bool ok = launch_dual_halo(ca, ntc, wa, MT, NTT, splits, x, S(s));
        check_last("dual_halo");
        return ok;
      },
      py::arg("ca"), py::arg("ntc"), py::arg("wa"), py::arg("MT"), py::arg("NTT"), py::arg("splits"), py::arg("s"),
      py::arg("rt") = nullptr, py::arg("ro") = nullptr, py::arg("rgrad") = 0, py::arg("rfirst") = 0,
      py::arg("xp") = nullptr,
      "dual wgrad + dgrad launch; with (rt, ro, rgrad) it also runs that table's reduction + optimizer");
  m.attr("MAX_STACK") = MAX_STACK;
  m.attr("MAX_STACK_SPLIT") = MAX_STACK_SPLIT;
  m.attr("STACK_THREADS") = conv_stack_threads();
  m.attr("STACK_TABN") = conv_stack_tabn();
  m.def("conv_stack_variant", &conv_stack_variant);
  m.def("conv_stack_fwd", [](const ConvStackArgs& a, uintptr_t s) {
    launch_conv_stack_fwd(a, S(s)); check_last("conv_stack_fwd"); });
  m.def("slab_reduce", [](uintptr_t grad, int lo, int hi, const RedTable& t, uintptr_t s) {
    launch_slab_reduce(reinterpret_cast<float*>(grad), lo, hi, t, S(s)); check_last("slab_reduce"); });
  m.def("optim", [](const OptimArgs& a, const PackTable& t, uintptr_t s) { launch_optim(a, t, S(s)); check_last("optim"); });
  m.def("pack", [](uintptr_t master, uintptr_t arena, const PackTable& t, uintptr_t s) {
    launch_pack(reinterpret_cast<const float*>(master), reinterpret_cast<bf16*>(arena), t, S(s)); check_last("pack"); });

  // fused xGMI all-reduce + optimizer (xgmi.hip)
  m.attr("XGMI_MAX_RANKS") = XGMI_MAX_RANKS;
  m.attr("XGMI_MAX_WG") = XGMI_MAX_WG;
  py::class_<XgmiPush>(m, "XgmiPush")
      .def(py::init<>())
      RW(XgmiPush, on) RW(XgmiPush, rank) RW(XgmiPush, size) RW(XgmiPush, chunk) RW(XgmiPush, lo)
      RW(XgmiPush, mode) RW(XgmiPush, nblk) RW(XgmiPush, nx) RW(XgmiPush, p1) RW(XgmiPush, fence) RW(XgmiPush, b_lo) RW(XgmiPush, b_hi) RW(XgmiPush, timeout_ticks)
      PTR(XgmiPush, ctrb) PTR(XgmiPush, err)
      .def("set_inbox", [](XgmiPush& x, int j, uintptr_t p) {
        if (j < 0 || j >= XGMI_MAX_RANKS) throw std::out_of_range("peer index");
        x.inbox[j] = reinterpret_cast<float*>(p);
      })
      .def("set_peer", [](XgmiPush& x, int j, uintptr_t inbox, uintptr_t outbox, uintptr_t bf1, uintptr_t bf2,
                          uintptr_t ab) {
        if (j < 0 || j >= XGMI_MAX_RANKS) throw std::out_of_range("peer index");
        x.inbox[j] = reinterpret_cast<float*>(inbox);
        x.outbox[j] = reinterpret_cast<float*>(outbox);
        x.bflag1[j] = reinterpret_cast<unsigned*>(bf1);
        x.bflag2[j] = reinterpret_cast<unsigned*>(bf2);
        x.abort_[j] = reinterpret_cast<unsigned*>(ab);
      });
  py::class_<XgmiArgs>(m, "XgmiArgs")
      .def(py::init<>())
      RW(XgmiArgs, skip_lo) RW(XgmiArgs, skip_hi) RW(XgmiArgs, skip_mode)
      RW(XgmiArgs, rank) RW(XgmiArgs, size) RW(XgmiArgs, n) RW(XgmiArgs, chunk) RW(XgmiArgs, sub)
      RW(XgmiArgs, timeout_ticks) RW(XgmiArgs, mode) RW(XgmiArgs, fence) PTR(XgmiArgs, grad) PTR(XgmiArgs, ctr) PTR(XgmiArgs, err)
      RW(XgmiArgs, opt)
      .def("set_peer", [](XgmiArgs& a, int j, uintptr_t inbox, uintptr_t outbox, uintptr_t f1, uintptr_t f2,
                          uintptr_t ab) {
        if (j < 0 || j >= XGMI_MAX_RANKS) throw std::out_of_range("peer index");
        a.inbox[j] = reinterpret_cast<float*>(inbox);
        a.outbox[j] = reinterpret_cast<float*>(outbox);
        a.flag1[j] = reinterpret_cast<unsigned*>(f1);
        a.flag2[j] = reinterpret_cast<unsigned*>(f2);
        a.abort_[j] = reinterpret_cast<unsigned*>(ab);
      });
  m.def("xgmi_grid", &xgmi_grid);
  m.def("xgmi_allreduce", [](const XgmiArgs& a, uintptr_t s) {
    if (a.size < 1 || a.size > XGMI_MAX_RANKS || a.rank < 0 || a.rank >= a.size) throw std::invalid_argument("xgmi ranks");
    if (a.chunk % 4 || a.sub % 4 || a.sub <= 0 || (long long)a.chunk * a.size < a.n) throw std::invalid_argument("xgmi geometry");
    if (xgmi_grid(a) > XGMI_MAX_WG) throw std::invalid_argument("xgmi grid > XGMI_MAX_WG");
    for (int j = 0; j < a.size; ++j)
      if (!a.inbox[j] || !a.outbox[j] || !a.flag1[j] || !a.flag2[j] || !a.abort_[j])
        throw std::invalid_argument("xgmi peer not set");
    if (!a.grad || !a.ctr || !a.err || (a.mode == 1 && (!a.opt.p || !a.opt.st))) throw std::invalid_argument("xgmi null pointer");
    if (a.timeout_ticks <= 0) throw std::invalid_argument("xgmi timeout_ticks must be > 0");
    launch_xgmi_allreduce(a, S(s));
    check_last("xgmi_allreduce");
  });
  m.def("xgmi_alloc_uncached", &xgmi_alloc_uncached, py::arg("bytes"), py::arg("finegrained") = false);
  m.def("xgmi_free", &xgmi_free);
  m.def("xgmi_ipc_handle", [](uintptr_t p) { return py::bytes(xgmi_ipc_handle(p)); });
  m.def("xgmi_ipc_open", [](py::bytes h) { return xgmi_ipc_open(std::string(h)); });
  m.def("xgmi_ipc_close", &xgmi_ipc_close);
}
