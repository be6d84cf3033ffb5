"""HIP / gfx950 backend: executes a Plan with the hand-written CDNA4 kernels.

One training step is a fixed sequence of ~15-20 launches (SURVEY.md §2.7 "fused op
boundaries"), captured once per batch size into a HIP graph and replayed:

  prologue(gather + re-pack + bookkeeping) -> conv_mm(fwd) x C -> [dense split-K + epilogue] x D -> head
  -> [wgrad(dense) + conv_mm(dX, bwd-through)] x D -> [wgrad(conv) + conv_mm(dgrad,
  bwd-through)] x C -> slab_reduce (per DP bucket) -> [RCCL all-reduce] -> optim

Activations are bf16 NHWC with channel strides padded to 8 (input: 4); weights live in
ONE fp32 master buffer (Keras layout) and are mirrored into bf16 fragment-major packs by
the optimizer kernel; gradients land in ONE flat fp32 buffer via deterministic slab
reductions.  Metrics accumulate on the device; the host syncs once per epoch.
"""
from __future__ import annotations

import gc
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from ..ops.hip import kernels
from ..ops.rng import keep_threshold
from ..utils.env import env_flag, tune
from .executor_base import DeviceData, Executor, prepare_targets
from .hip_geometry import GeometryMixin, cdiv, r8  # noqa: F401  (cdiv: re-exported for tests)
from .plan import Plan

BF16 = torch.bfloat16
OPT_KIND = {"sgd": 0, "rmsprop": 1, "adadelta": 2, "adam": 3, "nadam": 4}
PACK_CONV_FWD, PACK_CONV_DGRAD, PACK_DENSE_FWD, PACK_DENSE_BWD = 0, 1, 2, 3
RED_CONVW, RED_BIAS, RED_FLATW = 0, 1, 2


@dataclass
class Src:
    """An activation buffer feeding the next stage (for flatten mapping / bwd-through)."""
    kind: str            # 'input' | 'conv' | 'dense'
    idx: int
    C: int               # logical channels (flatten mapping)
    Cs: int              # padded channel stride
    H: int = 1
    W: int = 1

    @property
    def width(self):
        return self.H * self.W * self.Cs


@dataclass
class ConvGeo:
    i: int
    H: int
    W: int
    Cin: int
    Cs_in: int
    Ho: int
    Wo: int
    Cout: int
    Cs_out: int
    Hp: int
    Wp: int
    KH: int
    KW: int
    stride: int
    pad_t: int
    pad_l: int
    pool: bool
    relu: bool
    rate: float
    stream: int
    KS: int = 0
    NT: int = 0
    KSd: int = 0
    NTd: int = 0
    pack_fwd: int = 0
    pack_dgrad: int = -1


@dataclass
class DenseGeo:
    j: int
    src: Src
    K: int
    N: int
    Ns: int
    relu: bool
    rate: float
    stream: int
    KS: int = 0
    NT: int = 0
    KSb: int = 0
    NTb: int = 0
    pack_fwd: int = 0
    pack_bwd: int = -1


def splice_bucket_launches(launches, inserts, per_bucket):
    """Insert each bucket's launches into the step's launch list.

    ``inserts``: (launch index after which bucket k's partial slabs are final, k);
    ``per_bucket``: [(name pattern, factory k -> fn(stream), stream tag)] appended, in
    order, at that point (slab reduction, then all-reduce / optimizer on the comm stream).
    Returns (new launch list, bucket_ready[k] = index just past bucket k's launches)."""
    out, ready, pos = [], [0] * len(inserts), 0
    for at, k in sorted(inserts):
        out.extend(launches[pos:at])
        pos = at
        for pat, make, tag in per_bucket:
            fn = make(k)
            if fn is not None:          # a factory returns None for buckets it does not apply to
                out.append((pat % k, fn, tag))
        ready[k] = len(out)
    out.extend(launches[pos:])
    return out, ready


def defer_after_readers(launches, pattern, spans, readers):
    """Move each bucket's comm-stream optimizer (launch name ``pattern % k``) behind the
    last launch that reads a bf16 pack of a parameter in bucket k's span ``spans[k]``.

    The optimizer writes the packs of the weights it updates (pack routes), and a
    comm-stream launch forks after everything issued on main before it: a bucket whose
    slabs are final before a later dgrad / dense-dX launch reads the same layer's pack
    (wide convs have no dual launch, so their dgrad runs after the wgrad) must not update
    that pack while the reader runs.  ``readers``: [(launch name, param lo, param hi)].
    Returns the new launch list (the all-reduce stays where it was, so it still overlaps)."""
    out = list(launches)
    for k, (lo, hi) in enumerate(spans):
        names = [it[0] for it in out]
        name = pattern % k
        if name not in names:
            continue
        at = names.index(name)
        rd = {rn for rn, rlo, rhi in readers if rlo < hi and rhi > lo}
        last = max((i for i, n in enumerate(names) if n in rd), default=-1)
        if last > at:
            item = out.pop(at)
            out.insert(last, item)          # (the pop shifted the reader to last - 1)
    return out


def stream_program(tags, comm=True):
    """The stream schedule of a launch sequence, as a list of ops:
    ("run", stream, i)  launch i on "main" / "comm";
    ("wait", dst, src)  make stream dst wait for everything issued so far on src.

    'main' launches (any tag other than 'comm': 'side' marks the launches that only feed a
    slab reduction) run in order on the current stream.  'comm' launches fork the comm
    stream after everything issued so far (the bucket's slab reduction) -- RCCL and the
    bucket's optimizer run there while main continues the backward -- and the comm stream
    is joined back into main at the end.  ``comm=False``: comm launches run in order on main
    (a linear graph)."""
    ops, used = [], False
    for i, tag in enumerate(tags):
        if tag == "comm" and comm:
            ops.append(("wait", "comm", "main"))
            ops.append(("run", "comm", i))
            used = True
        else:
            ops.append(("run", "main", i))
    if used:
        ops.append(("wait", "main", "comm"))
    return ops


def check_bucket_cover(spans, numel):
    """Bucket (lo, hi) spans must tile [0, numel) exactly: disjoint, no gap, nothing left
    out (every gradient is reduced, all-reduced and updated exactly once)."""
    sp = sorted(spans)
    if not sp or sp[0][0] != 0 or sp[-1][1] != numel or any(a[1] != b[0] for a, b in zip(sp, sp[1:])):
        raise AssertionError("gradient buckets %s do not tile [0, %d)" % (spans, numel))


class HipExecutor(Executor):
    def __init__(self, plan: Plan, store, optimizer, seed: int):
        super().__init__(plan, store, optimizer, seed)
        self.K = kernels()
        self.K.set_red_lanes(int(tune("red_lanes", 16)))   # slab partials per reduction split-lane
        self.device = store.device
        if self.device.type != "cuda":
            raise RuntimeError("HipExecutor needs a GPU device")
        torch.cuda.set_device(self.device)
        self.use_graphs = env_flag("INTML_GRAPHS", True)
        self.state = torch.zeros(self.K.STEP_STATE_BYTES, dtype=torch.uint8, device=self.device)
        self._st_i32 = self.state.view(torch.int32)
        self._st_f32 = self.state.view(torch.float32)
        self._st_f64 = self.state.view(torch.float64)
        self._st_i64 = self.state.view(torch.int64)
        self._st_f64[self.K.STEP_STATE_MSCHED_OFFSET // 8] = 1.0
        base = getattr(optimizer, "_base_optimizer", optimizer)
        self.opt = base
        n_slots = getattr(base, "n_slots", 0)
        self.slots = [torch.zeros(store.capacity, dtype=torch.float32, device=self.device) for _ in range(n_slots)]
        self._build_geometry()
        self._build_packs()
        self._plans: Dict[Tuple[int, str], "BatchPlan"] = {}
        self._lr_host = None
        self._expected_pos = None
        self._bound_data = None
        self._bound_ref = None
        self._use_perm = None
        self._perm_obj = None
        self._perm_buf = None
        self._metrics_prev = (0.0, 0.0, 0.0)
        self.grad_scale = 1.0
        self.params_changed()

    # ------------------------------------------------------------------ geometry
    def _build_geometry(self):
        p = self.plan
        H0, W0, C0 = (p.input_shape + (1, 1))[:3] if len(p.input_shape) == 3 else (1, 1, p.input_shape[0])
        if len(p.input_shape) == 1:
            H0, W0, C0 = 1, 1, p.input_shape[0]
        self.in_C = C0
        self.in_Cs = 4 if C0 <= 4 else r8(C0)
        self.in_H, self.in_W = H0, W0
        self.convs: List[ConvGeo] = []
        src = Src("input", 0, C0, self.in_Cs, H0, W0)
        H, W, Cin, Cs_in = H0, W0, C0, self.in_Cs
        for i, cs in enumerate(p.convs):
            Ho, Wo, Cout = cs.conv_shape
            Hp, Wp, _ = cs.out_shape
            pt, _, pl, _ = cs.pads
            kh, kw = cs.conv.kernel_size
            g = ConvGeo(i, H, W, Cin, Cs_in, Ho, Wo, Cout, r8(Cout), Hp, Wp, kh, kw, cs.stride, pt, pl,
                        cs.pool is not None, cs.relu, cs.rate, cs.stream)
            g.KS = cdiv(kh * kw * Cs_in, 32)
            g.NT = cdiv(Cout, 16)
            if i > 0:
                g.KSd = cdiv(kh * kw * g.Cs_out, 32)
                g.NTd = cdiv(Cin, 16)
            self.convs.append(g)
            H, W, Cin, Cs_in = Hp, Wp, Cout, g.Cs_out
            src = Src("conv", i, Cout, g.Cs_out, Hp, Wp)
        self.denses: List[DenseGeo] = []
        for j, ds in enumerate(p.denses):
            g = DenseGeo(j, src, ds.K, ds.N, r8(ds.N), ds.relu, ds.rate, ds.stream)
            if g.K != src.H * src.W * src.C:
                raise ValueError("dense %d input width mismatch" % j)
            g.KS = cdiv(src.width, 32)
            g.NT = cdiv(ds.N, 16)
            if j > 0 or self.convs:
                g.KSb = cdiv(g.Ns, 32)
                g.NTb = cdiv(src.width, 16)
            self.denses.append(g)
            src = Src("dense", j, ds.N, g.Ns)
        self.head_src = src
        hd = p.head
        if hd.K != src.H * src.W * src.C:
            raise ValueError("head input width mismatch")
        if hd.N > 16:
            raise NotImplementedError("output layers wider than 16 units")
        self.head_act = {None: 0, "sigmoid": 1, "softmax": 2}[hd.activation]

    def _build_packs(self):
        K = self.K
        st = self.store
        self.pack_descs = []          # descriptor tuples, for per-bucket pack tables

        class _Tab:
            def __init__(self, outer):
                self.t, self.outer = K.PackTable(), outer

            def add(self, *d):
                self.t.add(*d)
                self.outer.pack_descs.append(d)

        tab = _Tab(self)
        off = 0

        def alloc(ks, nt):
            nonlocal off
            o = off
            off += ks * nt * 64 * 8
            return o

        for g, cs in zip(self.convs, self.plan.convs):
            sp = st.spec(cs.conv, "kernel")
            g.pack_fwd = alloc(g.KS, g.NT)
            tab.add(sp.offset, sp.numel, PACK_CONV_FWD, g.KH, g.KW, g.Cin, g.Cout, g.Cs_in, g.NT, g.pack_fwd)
            if g.i > 0:
                g.pack_dgrad = alloc(g.KSd, g.NTd)
                tab.add(sp.offset, sp.numel, PACK_CONV_DGRAD, g.KH, g.KW, g.Cin, g.Cout, g.Cs_out, g.NTd,
                        g.pack_dgrad)
        for g, ds in zip(self.denses, self.plan.denses):
            sp = st.spec(ds.dense, "kernel")
            g.pack_fwd = alloc(g.KS, g.NT)
            tab.add(sp.offset, sp.numel, PACK_DENSE_FWD, g.src.H, g.src.W, g.src.C, g.N, g.src.Cs, g.NT, g.pack_fwd)
            if g.KSb:
                g.pack_bwd = alloc(g.KSb, g.NTb)
                tab.add(sp.offset, sp.numel, PACK_DENSE_BWD, g.src.H, g.src.W, g.src.C, g.N, g.src.Cs, g.NTb, g.pack_bwd)
        self.pack_table = tab.t
        self.arena = torch.zeros(max(off, 8), dtype=BF16, device=self.device)
        # pack routes (PackRoute, args.h): the optimizer writes every updated weight's bf16
        # copies into these packs itself, so a training step needs no re-pack pass
        routes = []
        for g, cs in zip(self.convs, self.plan.convs):
            sp = st.spec(cs.conv, "kernel")
            bwd = g.pack_dgrad if g.i > 0 and g.Cs_out % 4 == 0 else -1
            routes.append((sp.offset, sp.offset + sp.numel, 1, g.KH * g.KW, g.Cin, g.Cout, g.Cs_in,
                           g.Cs_out if g.i > 0 else 0, g.NT, g.NTd if g.i > 0 else 0, g.pack_fwd, bwd))
        for g, ds in zip(self.denses, self.plan.denses):
            sp = st.spec(ds.dense, "kernel")
            routes.append((sp.offset, sp.offset + sp.numel, 2, g.src.H * g.src.W, g.src.C, g.N, g.src.Cs, 0,
                           g.NT, g.NTb if g.KSb else 0, g.pack_fwd, g.pack_bwd if g.KSb else -1))
        # (a dense layer whose optimizer runs inside its wgrad kernel writes its packs there
        # too -- WgradArgs.pk_fwd -- or is not fused: see BatchPlan._build_args)
        self.routes_ok = bool(routes) and len(routes) <= K.MAX_ROUTES and tune("opt_packs", True)
        self.routes = None
        self.route_list = routes
        if self.routes_ok:
            words = K.PACK_ROUTE_BYTES // 4
            arr = np.zeros(len(routes) * words, dtype=np.int32)
            a64 = arr.view(np.int64)
            for r, rt in enumerate(routes):
                arr[r * words:r * words + 10] = rt[:10]
                a64[r * words // 2 + 5] = rt[10]
                a64[r * words // 2 + 6] = rt[11]
            self.routes = torch.from_numpy(arr).to(self.device)

    # ------------------------------------------------------------------ params / optimizer
    def _optim_args(self, pack_only: bool, defer_pack: bool = False):
        K = self.K
        a = K.OptimArgs()
        a.p = self.store.master.data_ptr()
        a.g = self.store.grad.data_ptr()
        if self.slots:
            a.s0 = self.slots[0].data_ptr()
        if len(self.slots) > 1:
            a.s1 = self.slots[1].data_ptr()
        a.n = self.store.numel
        a.st = self.state.data_ptr()
        o = self.opt
        a.kind = OPT_KIND[o.kind]
        a.beta1 = getattr(o, "beta_1", 0.9)
        a.beta2 = getattr(o, "beta_2", 0.999)
        a.eps = getattr(o, "epsilon", 1e-7)
        a.rho = getattr(o, "rho", 0.95)
        a.momentum = getattr(o, "momentum", 0.0)
        a.nesterov = int(getattr(o, "nesterov", False))
        a.grad_scale = self.grad_scale
        a.pack_only = int(pack_only)
        a.defer_pack = int(defer_pack)
        a.arena = self.arena.data_ptr()
        if self.routes is not None and not pack_only:
            a.routes = self.routes.data_ptr()
            a.nroutes = self.routes.numel() * 4 // K.PACK_ROUTE_BYTES
        return a

    def tile_routes(self, a):
        """optim_kernel launches: the dense routes wholly inside [a.lo, a.lo + a.n) (identity
        padding, N % 32 == 0, K % 8 == 0) are updated by 2-D tile blocks that write whole
        16-byte pack vectors (the flat blocks' scattered 2-byte pack stores cost the legacy
        model's 33.5M-weight dense layer ~190 us per update)."""
        if self.routes is None or not tune("opt_tiles", True):
            return a
        span = a.lo + a.n - (a.lo & ~3)
        flat = cdiv(cdiv(span, 4), 256)
        b0 = i = 0
        for r, rt in enumerate(self.route_list):
            lo, hi, kind, _khw, cin, n, cs = rt[:7]
            k = (hi - lo) // n
            if (kind != 2 or cin != cs or n % 32 or k % 8 or lo % 4 or lo < a.lo or hi > a.lo + a.n
                    or i == 4 or rt[10] < 0):
                continue
            a.set_tile(i, r, b0)
            b0 += (k // 8) * cdiv(n, 128)
            i += 1
        if i:
            a.set_tile(i, 0, b0)
            a.ntile, a.flat_blocks = i, flat
        return a

    def params_changed(self):
        self.K.optim(self._optim_args(True), self.pack_table, torch.cuda.current_stream().cuda_stream)

    def optimizer_state(self):
        return [s[:self.store.numel] for s in self.slots]

    def set_optimizer_state(self, iterations, slots):
        self.opt.iterations = int(iterations)
        self._st_i32[0] = int(iterations)
        for dst, src in zip(self.slots, slots):
            dst[:self.store.numel].copy_(torch.as_tensor(src, device=self.device).reshape(-1))

    def m_schedule_value(self) -> float:
        return float(self._st_f64[self.K.STEP_STATE_MSCHED_OFFSET // 8])

    def set_m_schedule(self, v: float) -> None:
        self._st_f64[self.K.STEP_STATE_MSCHED_OFFSET // 8] = float(v)

    def set_lr_warmup(self, t0, steps, spe, size, epochs, base):
        super().set_lr_warmup(t0, steps, spe, size, epochs, base)
        w = self.lr_warmup or (0, 0, 1, 1, 1.0, 0.0)
        o = self.K.STEP_STATE_WARM_OFFSET
        self._st_i32[o // 4:o // 4 + 4] = torch.tensor(w[:4], dtype=torch.int32)
        # StepState order: warm_base, warm_epochs
        self._st_f32[o // 4 + 4:o // 4 + 6] = torch.tensor([w[5], w[4]], dtype=torch.float32)

    def _sync_lr(self):
        lr = float(self.opt.lr)
        if lr != self._lr_host:
            self._st_f32[self.K.STEP_STATE_LR_OFFSET // 4] = lr
            self._lr_host = lr

    # ------------------------------------------------------------------ data
    def upload(self, x, y):
        if x is None:
            return None
        x = np.asarray(x)
        if tuple(x.shape[1:]) != tuple(self.plan.input_shape):
            raise ValueError("input shape %s != model input %s" % (x.shape[1:], self.plan.input_shape))
        n = x.shape[0]
        xt = torch.as_tensor(np.ascontiguousarray(x, dtype=np.float32)).to(self.device, non_blocking=False)
        xt = xt.reshape(n, self.in_H, self.in_W, self.in_C)
        xs = torch.zeros(n, self.in_H, self.in_W, self.in_Cs, dtype=BF16, device=self.device)
        xs[..., :self.in_C] = xt.to(BF16)
        del xt
        yt = None
        if y is not None:
            yt = torch.as_tensor(prepare_targets(y, self.plan)).to(self.device)
        else:
            yt = torch.zeros(n, self.plan.head.N, dtype=torch.float32, device=self.device)
        return DeviceData(xs.reshape(n, -1), yt, n)

    def _bind_data(self, data: DeviceData, perm: Optional[torch.Tensor]):
        K = self.K
        key = (id(data), data.x.data_ptr(), data.y.data_ptr())
        if self._bound_data != key or self._bound_ref is not data:
            self._bound_ref = data     # keep alive: its id / memory must not be recycled while bound
            o = K.STEP_STATE_DATA_OFFSET // 8
            self._st_i64[o] = data.x.data_ptr()
            self._st_i64[o + 1] = data.y.data_ptr()
            on = K.STEP_STATE_DATAN_OFFSET // 4
            self._st_i32[on] = data.n
            self._st_i32[on + 1] = data.x.shape[1]
            self._st_i32[on + 2] = data.y.shape[1]
            self._bound_data = key
            self._perm_obj = None
        if perm is not None and perm is not self._perm_obj:
            # (a DP rank's epoch slice of the sampler permutation is shorter than the data set)
            m = min(int(perm.numel()), data.n)
            if self._perm_buf is None or self._perm_buf.numel() < max(data.n, 1):
                self._perm_buf = torch.empty(max(data.n, 1), dtype=torch.int32, device=self.device)
            self._perm_buf[:m].copy_(perm[:m].to(device=self.device, dtype=torch.int32))
            self._st_i64[K.STEP_STATE_DATA_OFFSET // 8 + 2] = self._perm_buf.data_ptr()
            self._perm_obj = perm
        use = 1 if perm is not None else 0
        if use != self._use_perm:     # host->device writes only on change (each is a copy + sync point)
            self._st_i32[K.STEP_STATE_DATAN_OFFSET // 4 + 3] = use
            self._use_perm = use

    # ------------------------------------------------------------------ steps
    def _plan_for(self, bs: int, mode: str) -> "BatchPlan":
        key = (bs, mode)
        bp = self._plans.get(key)
        if bp is None:
            bp = BatchPlan(self, bs, mode)
            self._plans[key] = bp
        return bp

    def train_step(self, data, perm, pos, bs):
        self.train_steps(data, perm, pos, bs, 1)

    def train_steps(self, data, perm, pos, bs, k):
        """k consecutive full training steps over batches [pos, pos + k*bs) of ``perm``
        (one graph replay; the caller guarantees no host-side change between them)."""
        self._sync_lr()
        self._bind_data(data, perm)
        if self._expected_pos != pos:
            self._st_i32[1] = pos
        bp = self._plan_for(bs, "train")
        bp.run(k)
        self._expected_pos = pos + k * bs
        self.opt.iterations += k

    def _set_eval_pos(self, pos, bs):
        if getattr(self, "_expected_eval_pos", None) != pos:
            self._st_i32[3] = pos
        self._expected_eval_pos = pos + bs

    def eval_step(self, data, pos, bs):
        self._bind_data(data, None)
        self._set_eval_pos(pos, bs)
        self._plan_for(bs, "eval").run()

    def predict_step(self, data, pos, bs):
        self._bind_data(data, None)
        self._set_eval_pos(pos, bs)
        bp = self._plan_for(bs, "predict")
        bp.run()
        out = bp.probs.clone()
        return out

    # ------------------------------------------------------------------ metrics
    def _metrics(self):
        # int64 fixed point (StepState::metric_slots [16][4]): loss in units of 2^-32, counts
        # exact; integer sums over the slots are order-independent
        o = self.K.STEP_STATE_METRICS_OFFSET // 8
        v = self.state.view(torch.int64)[o:o + 4 * self.K.STEP_STATE_METRIC_SLOTS].view(-1, 4).sum(0).tolist()
        # v[3] counts head workgroups whose loss was non-finite or out of fixed-point range:
        # the loss is then NaN (sticky until reset_metrics), never a finite garbage value
        return [v[0] / 4294967296.0 if v[3] == 0 else float("nan"), float(v[1]), float(v[2])]

    def reset_metrics(self):
        o = self.K.STEP_STATE_METRICS_OFFSET // 8
        self._st_f64[o:o + 4 * self.K.STEP_STATE_METRIC_SLOTS].zero_()
        self._metrics_prev = (0.0, 0.0, 0.0)

    def read_metrics(self):
        ls, cs, n = self._metrics()
        self._metrics_prev = (ls, cs, n)
        n1 = max(n, 1.0)
        return ls / n1, cs / n1, int(n)

    def last_batch_metrics(self):
        ls, cs, n = self._metrics()
        pl, pc, pn = self._metrics_prev
        self._metrics_prev = (ls, cs, n)
        dn = max(n - pn, 1.0)
        return (ls - pl) / dn, (cs - pc) / dn   # NaN propagates once the flag is set

    def synchronize(self):
        torch.cuda.synchronize(self.device)


class BatchPlan(GeometryMixin):
    """Buffers + prepared kernel argument structs for one (batch size, mode); records the
    launch sequence and replays it from a HIP graph."""

    def __init__(self, ex: HipExecutor, bs: int, mode: str):
        self.ex, self.bs, self.mode = ex, bs, mode
        self.training = mode == "train"
        K = ex.K
        dev = ex.device
        self.graph = None
        self.multi_graphs: Dict[int, torch.cuda.CUDAGraph] = {}   # k -> graph of k steps
        self.dp_graphs = None
        # (a second compute stream for the weight gradients and a per-bucket early optimizer
        # stream were measured slower on one MI355X and removed: docs/ARCHITECTURE.md §6)
        self.optim_fused = False           # set by _build_reduce
        self.early_red = {}                # dual launch name -> (RedTable, span): set by _build_reduce
        # Native RCCL data plane: the bucket all-reduces are part of the launch sequence (on
        # their own comm stream) and captured with the rest of the step into ONE HIP graph.
        red = ex.reducer
        self.comm_in_graph = (self.training and red is not None and getattr(red, "capturable", False)
                              and red.active and tune("comm_capture", True))
        # tune comm_fork=0: the captured all-reduces stay on the main stream (a linear graph:
        # no cross-queue edges, whose graph-launch cost is several us each, but no overlap)
        # (default: fork only when there is more than one bucket to overlap; set in _build_reduce)
        self.comm_fork = None
        self.comm_stream = None
        # ... and each bucket's optimizer update follows its all-reduce on the comm stream (the
        # 1/size average folded in), so the dense bucket's update overlaps the conv backward and
        # only the last bucket's (small) update is on the step's tail
        self.optim_on_comm = self.comm_in_graph and tune("dp_optim_on_comm", True)
        z = lambda *s, dt=BF16: torch.zeros(*s, dtype=dt, device=dev)
        self.xb = z(bs, ex.in_H * ex.in_W * ex.in_Cs)
        self.yb = z(bs, ex.plan.head.N, dt=torch.float32)
        self.conv_out, self.conv_code, self.conv_dy = [], [], []
        for g in ex.convs:
            self.conv_out.append(z(bs, g.Hp, g.Wp, g.Cs_out))
            self.conv_code.append(z(bs, g.Hp, g.Wp, g.Cs_out, dt=torch.uint8) if g.pool else None)
            # gradient wrt the stage OUTPUT resolution (pooled dP for pooled convs; the
            # full-resolution dY is rebuilt on load from dP + codes, never stored)
            self.conv_dy.append(z(bs, g.Hp, g.Wp, g.Cs_out) if self.training else None)
        self.dense_out, self.dense_part, self.dense_dh = [], [], []
        self.dense_splits = []
        for g in ex.denses:
            self.dense_out.append(z(bs, g.Ns))
            if K.dense_big(g.NT, g.KS):
                # large weights: ~256 workgroups (one per CU) of >= 8 k-steps; each owns
                # 128 rows x 8 n-tiles, so every weight byte streams from HBM once
                splits = max(1, min(cdiv(tune("dense_big_wgs", 256), K.dense_groups(bs, g.NT, g.KS)),
                                    cdiv(g.KS, tune("dense_big_minks", 8))))
            else:
                # ~2048 16x16-tile waves: latency-bound small layers want parallelism
                splits = max(1, min(g.KS, tune("dense_waves", 2048) // max(1, K.dense_groups(bs, g.NT, g.KS))))
            kps = cdiv(g.KS, splits)
            splits = cdiv(g.KS, kps)
            self.dense_splits.append((splits, kps))
            self.dense_part.append(z(splits, bs, g.NT * 16, dt=torch.float32))
            self.dense_dh.append(z(bs, g.Ns) if self.training else None)
        hd = ex.plan.head
        self.head_blocks = cdiv(bs, K.head_rows_per_block(False))   # re-set below if the head fuses the epilogue
        head_slab_blocks = cdiv(bs, K.head_rows_per_block(True))
        self.probs = z(bs, hd.N, dt=torch.float32) if mode == "predict" else None
        if self.training:
            self.head_wslab = z(head_slab_blocks, hd.K, hd.N, dt=torch.float32)
            self.head_bslab = z(head_slab_blocks, hd.N, dt=torch.float32)
        self._build_args()

    # ---------------------------------------------------------------- helpers
    def step_inputs(self):
        """(x [bs, R] bf16, y [bs, C] fp32) of this plan's last step: the gathered batch
        buffers, or -- prologue-free step -- the dataset rows the conv stack recorded."""
        if self.srcidx is None:
            return self.xb, self.yb
        d = self.ex._bound_ref
        idx = self.srcidx.long()
        return d.x[idx], d.y[idx]

    def _src_buf(self, src: Src):
        if src.kind == "input":
            return self.xb
        if src.kind == "conv":
            return self.conv_out[src.idx]
        return self.dense_out[src.idx]

    def _bt_for(self, src: Src):
        """BwdThrough args routing a gradient wrt ``src``'s output back into its layer."""
        K, ex = self.ex.K, self.ex
        bt = K.BwdThrough()
        if src.kind == "input":
            return None
        if src.kind == "conv":
            g = ex.convs[src.idx]
            bt.prev_out = self.conv_out[g.i].data_ptr()
            if g.pool:
                bt.prev_code = self.conv_code[g.i].data_ptr()
            bt.prev_relu, bt.prev_pool = int(g.relu), int(g.pool)
            bt.pH, bt.pW, bt.pC, bt.pCs = g.Hp, g.Wp, g.Cout, g.Cs_out
            bt.cH, bt.cW = g.Ho, g.Wo
            rate, stream = g.rate, g.stream
            bt.dy = self.conv_dy[g.i].data_ptr()
        else:
            g = ex.denses[src.idx]
            bt.prev_out = self.dense_out[g.j].data_ptr()
            bt.prev_relu, bt.prev_pool = int(g.relu), 0
            bt.pH, bt.pW, bt.pC, bt.pCs = 1, 1, g.N, g.Ns
            bt.cH, bt.cW = 1, 1
            rate, stream = g.rate, g.stream
            bt.dy = self.dense_dh[g.j].data_ptr()
        if rate > 0:
            bt.drop_thr = keep_threshold(rate)
            bt.drop_scale = 1.0 / (1.0 - rate)
        bt.seed, bt.stream_id = ex.seed, stream
        # write-through gradient stores (16-byte sc1; byte offsets < 2 GB)
        dyb = self.conv_dy[g.i] if src.kind == "conv" else self.dense_dh[g.j]
        bt.wt = int(bool(int(tune("wt", 7)) & 2) and dyb.numel() * 2 < (1 << 31))
        return bt

    def _build_args(self):
        ex, K, bs = self.ex, self.ex.K, self.bs
        st_ptr = ex.state.data_ptr()
        store = ex.store
        training = self.training
        self.launches = []          # list of (name, callable(stream))

        # step begin
        sb = K.StepBeginArgs()
        sb.st = st_ptr
        sb.training = int(training)
        sb.bs = bs
        o = ex.opt
        sb.opt_kind = OPT_KIND[o.kind]
        sb.beta1 = getattr(o, "beta_1", 0.9)
        sb.beta2 = getattr(o, "beta_2", 0.999)
        sb.decay = getattr(o, "initial_decay", 0.0)
        sb.schedule_decay = getattr(o, "schedule_decay", 0.004)
        ga = K.GatherArgs()
        ga.st = st_ptr
        ga.bs = bs
        ga.R = self.xb.shape[1]
        ga.xb = self.xb.data_ptr()
        ga.yb = self.yb.data_ptr()
        # one prologue launch: gather + the previous update's weight re-pack (training: always,
        # except with per-bucket optimizers that pack themselves; eval/predict: only if an
        # optimizer ran since the last pack) + the step bookkeeping
        stack = self._conv_stack_args(training) if tune("conv_stack", True) else None
        # Prologue-free step (conv stack + a hidden dense layer + optimizer-written packs): the
        # stack reads its images straight from the dataset through the cursor and permutation
        # (recording each image's dataset row for the first layer's wgrad and the head's
        # targets), the optimizer keeps the bf16 packs current, and the first dense launch runs
        # the step bookkeeping -- the step has no prologue launch
        self.pro_free = bool(stack is not None and ex.denses and ex.routes_ok and tune("pro_free", True))
        self.srcidx = None
        if self.pro_free:
            self.srcidx = torch.zeros(max(bs, 1), dtype=torch.int32, device=ex.device)
            stack.from_data, stack.training, stack.step_inc = 1, int(training), int(training)
            stack.srcidx = self.srcidx.data_ptr()
        pa = K.PrologueArgs()
        pa.sb, pa.ga = sb, ga
        pa.gather_gx = 1 if ga.skip_x else K.gather_gx(ga.R)
        pa.gather_blocks = pa.gather_gx * bs
        pa.pack_mode = 1 if training else 2
        pro_dbg = tune("pro_dbg", 0)          # timing ablation only: 1 no re-pack, 2 no gather
        if pro_dbg == 1:
            pa.pack_mode = 0
        elif pro_dbg == 2:
            pa.gather_blocks = 0
        pa.master = store.master.data_ptr()
        pa.arena = ex.arena.data_ptr()
        if training and ex.routes_ok:
            pa.pack_mode = 0          # the optimizer writes the packs itself (pack routes)
        if not self.pro_free:
            self.launches.append(("prologue", lambda s, a=pa: K.prologue(a, ex.pack_table, s)))

        # ---------------- forward convs
        if stack is not None:
            self.stack_args = stack
            self.launches.append(("conv_stack_fwd", lambda s, a=stack: K.conv_stack_fwd(a, s)))
        x_buf, H, W, Cs = self.xb, ex.in_H, ex.in_W, ex.in_Cs
        for g, cs in zip(ex.convs, ex.plan.convs):
            if stack is not None:
                break
            a = K.ConvMMArgs()
            a.x = x_buf.data_ptr()
            a.B, a.H, a.W, a.Cs_in = bs, g.H, g.W, g.Cs_in
            a.Ho, a.Wo = g.Ho, g.Wo
            a.KH, a.KW, a.stride, a.pad_t, a.pad_l, a.in_dil = g.KH, g.KW, g.stride, g.pad_t, g.pad_l, 1
            a.KS = g.KS
            a.wpk = ex.arena.data_ptr() + 2 * g.pack_fwd
            a.NT = g.NT
            a.bias = store.view(cs.conv, "bias").data_ptr() if cs.conv.use_bias else 0
            a.N = g.Cout
            a.mode = 0
            a.relu, a.pool = int(g.relu), int(g.pool)
            a.out = self.conv_out[g.i].data_ptr()
            a.Cs_out, a.Hp, a.Wp = g.Cs_out, g.Hp, g.Wp
            if g.pool:
                a.code = self.conv_code[g.i].data_ptr()
            if training and g.rate > 0:
                a.drop_thr = keep_threshold(g.rate)
                a.drop_scale = 1.0 / (1.0 - g.rate)
            a.seed, a.stream_id, a.st = ex.seed, g.stream, st_ptr
            self.launches.append(("conv_fwd%d" % g.i, self._conv_launch(a, g.NT, g.pool)))
            x_buf = self.conv_out[g.i]

        # ---------------- forward denses
        head_epi = None
        for g, ds in zip(ex.denses, ex.plan.denses):
            splits, kps = self.dense_splits[g.j]
            a = K.DenseFwdArgs()
            a.x = self._src_buf(g.src).data_ptr()
            a.M, a.Ks = bs, g.src.width
            a.wpk = ex.arena.data_ptr() + 2 * g.pack_fwd
            a.NT, a.KS = g.NT, g.KS
            a.splits, a.ks_per_split = splits, kps
            a.part = self.dense_part[g.j].data_ptr()
            if self.pro_free and g.j == 0 and training:
                a.book, a.sb = 1, sb      # this step's bookkeeping (the stack read t + 1)
            self.launches.append(("dense_fwd%d" % g.j, lambda s, a=a: K.dense_fwd(a, s)))
            last_fwd = (len(self.launches) - 1, a, g)
            e = K.DenseEpiArgs()
            e.part = a.part
            e.splits, e.M, e.N, e.Ns, e.ldp = splits, bs, g.N, g.Ns, g.NT * 16
            e.bias = store.view(ds.dense, "bias").data_ptr() if ds.dense.use_bias else 0
            e.relu = int(g.relu)
            e.out = self.dense_out[g.j].data_ptr()
            if training and g.rate > 0:
                e.drop_thr = keep_threshold(g.rate)
                e.drop_scale = 1.0 / (1.0 - g.rate)
            e.seed, e.stream_id, e.st = ex.seed, g.stream, st_ptr
            if (g.j == len(ex.denses) - 1 and ex.head_src.kind == "dense" and g.Ns <= K.head_epi_max()
                    and tune("fuse_head", True)):
                # the head launch (one row per workgroup, the row's split groups in parallel)
                # reduces this layer's partials itself: one kernel boundary fewer
                head_epi = e
                self.head_blocks = cdiv(bs, K.head_rows_per_block(True))
            else:
                self.launches.append(("dense_epi%d" % g.j, lambda s, e=e: K.dense_epi(e, s)))

        # ---------------- head
        hd = ex.plan.head
        h = K.HeadArgs()
        src = ex.head_src
        h.h = self._src_buf(src).data_ptr()
        h.M, h.K, h.Ks, h.N = bs, hd.K, src.width, hd.N
        h.flat_C, h.flat_Cs = src.C, src.Cs
        h.w = store.view(hd.dense, "kernel").data_ptr()
        h.bias = store.view(hd.dense, "bias").data_ptr() if hd.dense.use_bias else 0
        h.y = self.yb.data_ptr() if self.mode != "predict" else 0
        if self.pro_free and h.y:
            h.yidx = self.srcidx.data_ptr()      # targets straight from the dataset rows
        h.act = ex.head_act
        if head_epi is not None:
            h.epi = head_epi
        h.training = int(training)
        h.generic = int(tune("head_generic", False))
        h.inv_bs = 1.0 / bs
        h.st = st_ptr
        if self.probs is not None:
            h.probs = self.probs.data_ptr()
        if training:
            h.wslab = self.head_wslab.data_ptr()
            h.bslab = self.head_bslab.data_ptr()
            bt = self._bt_for(src)
            if bt is not None:
                h.bt = bt
        # (a fused dense layer + head launch -- 16-wave K-slice tiles, the last arriving workgroup
        # of each row group running the head -- measured 15.6 us against 13.3 us for the split-K
        # dense launch + this head launch at RPV B=128, and was removed in round 5)
        self.launches.append(("head", lambda s, a=h: K.head(a, s)))
        if not training:
            return

        # ---------------- backward
        self.red_groups = []       # (lo, hi, [desc tuples]) in backward order
        self.pack_readers = []     # (launch name, param lo, hi): backward launches reading a layer's pack
        self.red_ready = []        # launch count after which each group's partial slabs are final
        hw = store.spec(hd.dense, "kernel")
        descs = [(self.head_wslab.data_ptr(), hd.K * hd.N, self.head_blocks, hd.N, hw.offset, hw.numel,
                  RED_BIAS, 0, 0, 0, 0, 0)]
        lo, hi = hw.offset, hw.offset + hw.numel
        if hd.dense.use_bias:
            hb = store.spec(hd.dense, "bias")
            descs.append((self.head_bslab.data_ptr(), hd.N, self.head_blocks, hd.N, hb.offset, hb.numel,
                          RED_BIAS, 0, 0, 0, 0, 0))
            hi = max(hi, hb.offset + hb.numel)
        self.red_groups.append((lo, hi, descs))
        self._add_group_reduce()
        self.wgrad_slabs = []
        self.dense_fused_opt = []          # (WgradArgs, params) updated inside dense_wgrad
        # opt-in: the dense layer's optimizer update inside its (one-split) wgrad kernel.  Measured
        # slower on RPV at batch 128: the 128 wgrad workgroups move the layer's 14 MB of optimizer
        # state at per-CU bandwidth (wgrad 6.1 -> 9.7 us) while the end-of-step reduction, which
        # spreads it over thousands of workgroups, only drops 10.8 -> 8.2 us
        # dense_opt: "auto" (default) = only layers whose gradient is written in place (> 16 MB,
        # the legacy model's 33.5M-weight Dense(512)): their update moves ~1 GB either way, and
        # fusing it saves the gradient's own write + re-read (legacy 1.269 -> 1.238 ms/step,
        # profiles/r4c_ab_legacy.txt); "1" = every one-split layer; "0" = off
        dense_opt = str(tune("dense_opt", "auto")).lower()
        self.dense_opt_ok = (ex.reducer is None and tune("fuse_optim", True)
                             and dense_opt not in ("0", "false", "off", "no"))
        self.dense_opt_all = dense_opt in ("1", "true", "on", "yes")

        for g, ds in reversed(list(zip(ex.denses, ex.plan.denses))):
            xin = self._src_buf(g.src)
            sp = store.spec(ds.dense, "kernel")
            # Unpadded flatten source and N % 16 == 0: the single-split slab IS the Keras
            # (in, out) layout, so the wgrad kernel writes the gradient buffer directly and
            # the slab round trip disappears (the dense kernel is most of the model's bytes).
            direct = (g.src.C == g.src.Cs and g.N % 16 == 0 and g.src.width % 16 == 0
                      and g.src.width * g.N * 4 > (16 << 20))     # small layers keep split-K slabs
            direct_ptr = (store.grad.data_ptr() + 4 * sp.offset) if direct else None
            # dense_bwd.hip kernels (per-wave pipelined wgrad, vectorised dX epilogue) where the
            # 8-element alignment they assume holds; the generic wgrad / split-K path otherwise
            bwd2 = tune("dense_bwd2", True) and g.src.width % 8 == 0 and g.Ns % 8 == 0
            fused_opt = False
            if bwd2:
                wa, cfg, slab, bslab = self._dense_wgrad_args(xin, g.src.width, self.dense_dh[g.j], g.Ns, g.N, bs,
                                                              ds.dense.use_bias, direct_ptr)
                # one split + identity layout: the kernel's fixed-order sum IS the Keras
                # gradient -- write it in place and apply the optimizer there (single GPU,
                # fused-optimizer step), so the layer skips the end-of-step reduction
                fused_opt = (self.dense_opt_ok and (self.dense_opt_all or direct)
                             and cfg[2] == 1 and g.src.C == g.src.Cs and g.N % 16 == 0 and sp.offset % 4 == 0)
                # with optimizer-written packs the kernel must write this layer's packs itself
                pk_ok = (cfg[0] == 2 and g.src.width % 32 == 0 and g.N % 32 == 0
                         and (not g.KSb or cfg[1] % 2 == 0))
                if fused_opt and ex.routes_ok and not pk_ok:
                    fused_opt = False
                if fused_opt:
                    grad = store.grad.data_ptr()
                    wa.slab = grad + 4 * sp.offset
                    wa.opt = ex._optim_args(False, defer_pack=True)
                    wa.opt_w = sp.offset
                    # the gradient the update consumed is not stored (134 MB of writes for the
                    # legacy Dense(512): 1.107 -> 1.097 ms/step, with dw_order 1.101 -> 1.086,
                    # profiles/r6_dense_wgrad_ab.txt) -- this layer's gradient is then not
                    # readable through the store (store.view(..., grad=True)); opt_nograd=0 keeps it
                    wa.opt_nograd = int(tune("opt_nograd", True))
                    if ex.routes_ok:
                        wa.pk_fwd, wa.pk_NT = g.pack_fwd, g.NT
                        wa.pk_bwd, wa.pk_NTb = (g.pack_bwd, g.NTb) if g.KSb else (-1, 0)
                    if ds.dense.use_bias:
                        wa.bslab = grad + 4 * store.spec(ds.dense, "bias").offset
                        wa.opt_b = store.spec(ds.dense, "bias").offset
                # grid order 1: the n groups of one feature group consecutive (whole rows of the
                # weight / optimizer-state arrays per resident wave of workgroups; legacy -5 us)
                dw_order = int(tune("dw_order", 1))
                dw_late = bool(tune("dw_late", True))     # 4 waves / SIMD: legacy 1.070 -> 1.059 ms
                wl = lambda s, a=wa, c=cfg, o=dw_order, l=dw_late: K.dense_wgrad(a, c[0], c[1], c[2], s, o, l)
            else:
                wa, cfg, slab, bslab = self._wgrad_args(
                    xin, 1, 1, g.src.width, 1, 1, 1, 1, 1, 0, 0, self.dense_dh[g.j], g.Ns, g.N, bs,
                    ds.dense.use_bias, direct=direct_ptr)
                wl = lambda s, a=wa, c=cfg: K.wgrad(a, c[0], c[1], c[2], s)
            self.launches.append(("wgrad_dense%d" % g.j, wl, "side"))
            w_at = len(self.launches) - 1
            S, ld = cfg[2], g.NT * 16
            descs = [] if (direct or fused_opt) else [(slab.data_ptr(), wa.Ktiles * 16 * ld, S, ld, sp.offset,
                                                        sp.numel, RED_FLATW, 0, 0, g.src.C, g.N, g.src.Cs)]
            lo, hi = sp.offset, sp.offset + sp.numel
            if ds.dense.use_bias:
                bp_ = store.spec(ds.dense, "bias")
                if not fused_opt:
                    descs.append((bslab.data_ptr(), ld, S, ld, bp_.offset, bp_.numel, RED_BIAS, 0, 0, 0, 0, 0))
                hi = max(hi, bp_.offset + bp_.numel)
            if fused_opt:
                self.dense_fused_opt.append((wa, hi - lo))
            self.red_groups.append((lo, hi, descs))
            self._add_group_reduce()
            if g.KSb:
                a = K.DenseFwdArgs()
                a.x = self.dense_dh[g.j].data_ptr()
                a.M, a.Ks = bs, g.Ns
                a.wpk = ex.arena.data_ptr() + 2 * g.pack_bwd
                a.NT, a.KS = g.NTb, g.KSb
                a.splits, a.ks_per_split = 1, g.KSb
                a.mode = 1
                a.st = st_ptr
                a.bt = self._bt_for(g.src)
                dname = "dense_dx%d" % g.j
                ntc = self._dense_dx_ntc(a) if (bwd2 and a.bt.pCs % 8 == 0 and a.Ks % 8 == 0
                                               and not K.dense_big(a.NT, a.KS)) else 0
                if fused_opt:
                    # the wgrad's fused optimizer rewrites this layer's backward pack: its dX (that
                    # pack's reader) runs first, as a launch of its own on the same stream -- never
                    # in one launch with it (dense_bwd_pair: dX workgroups would read a pack the
                    # wgrad workgroups are rewriting)
                    fn = ((lambda s, a=a, n=ntc: K.dense_dx(a, n, s)) if ntc else (lambda s, a=a: K.dense_fwd(a, s)))
                    self.launches[w_at] = (self.launches[w_at][0], self.launches[w_at][1], "main")
                    self.launches.insert(w_at, (dname, fn, "main"))
                    self.red_ready[-1] += 1
                elif tune("dual_dense", True):
                    # one launch for the dense wgrad and dX (independent GEMMs over dH), in the
                    # wgrad's slot (its slabs are final after it)
                    dname = "dense_bwd%d" % g.j
                    if ntc:
                        fn = lambda s, a=a, w=wa, c=cfg, n=ntc: K.dense_bwd_pair(w, c[0], c[1], c[2], a, n, s)
                    elif bwd2:
                        fn = lambda s, a=a, w=wa, c=cfg: (K.dense_wgrad(w, c[0], c[1], c[2], s), K.dense_fwd(a, s))
                    else:
                        fn = lambda s, a=a, w=wa, c=cfg: self._dense_dual(w, c, a, s)
                    self.launches[w_at] = (dname, fn, "main")
                elif ntc:
                    self.launches.append((dname, lambda s, a=a, n=ntc: K.dense_dx(a, n, s)))
                else:
                    self.launches.append((dname, lambda s, a=a: K.dense_fwd(a, s)))
                self.pack_readers.append((dname, sp.offset, sp.offset + sp.numel))

        for g, cs in reversed(list(zip(ex.convs, ex.plan.convs))):
            xin = self.xb if g.i == 0 else self.conv_out[g.i - 1]
            if self._wide(g.Cs_in, g.KS, g.NT):
                wa, cfg, slab, bslab = self._wgrad_tile_args(xin, g, bs, cs.conv.use_bias)
                self.launches.append(("wgrad_conv%d" % g.i, lambda s, a=wa, c=cfg: K.wgrad_tile(a, c[0], s),
                                      "side"))
            else:
                wa, cfg, slab, bslab = self._wgrad_halo_args(xin, g, bs, cs.conv.use_bias)
                if g.i == 0 and self.pro_free:      # the images the stack read from the dataset
                    wa.xidx, wa.xst = self.srcidx.data_ptr(), st_ptr
                self.launches.append(("wgrad_conv%d" % g.i,
                                      lambda s, a=wa, c=cfg: K.wgrad_halo(a, c[0], c[1], c[2], s), "side"))
            w_at = len(self.launches) - 1
            sp = store.spec(cs.conv, "kernel")
            S, ld = cfg[2], g.NT * 16
            descs = [(slab.data_ptr(), wa.Ktiles * 16 * ld, S, ld, sp.offset, sp.numel, RED_CONVW,
                      g.KH, g.KW, g.Cin, g.Cout, g.Cs_in)]
            lo, hi = sp.offset, sp.offset + sp.numel
            if cs.conv.use_bias:
                bp_ = store.spec(cs.conv, "bias")
                descs.append((bslab.data_ptr(), ld, S, ld, bp_.offset, bp_.numel, RED_BIAS, 0, 0, 0, 0, 0))
                hi = max(hi, bp_.offset + bp_.numel)
            self.red_groups.append((lo, hi, descs))
            self._add_group_reduce()
            if g.i > 0:
                prev = ex.convs[g.i - 1]
                a = K.ConvMMArgs()
                a.x = self.conv_dy[g.i].data_ptr()
                a.B, a.H, a.W, a.Cs_in = bs, g.Ho, g.Wo, g.Cs_out
                if g.pool:      # dY rebuilt on load from pooled dP + argmax codes
                    a.in_code = self.conv_code[g.i].data_ptr()
                    a.in_pH, a.in_pW = g.Hp, g.Wp
                a.Ho, a.Wo = g.H, g.W            # == prev stage output grid
                a.KH, a.KW, a.stride = g.KH, g.KW, 1
                a.pad_t, a.pad_l, a.in_dil = g.KH - 1 - g.pad_t, g.KW - 1 - g.pad_l, g.stride
                a.KS = g.KSd
                a.wpk = ex.arena.data_ptr() + 2 * g.pack_dgrad
                a.NT = g.NTd
                a.mode, a.flat_out = 1, 0
                a.st = st_ptr
                a.bt = self._bt_for(Src("conv", prev.i, prev.Cout, prev.Cs_out, prev.Hp, prev.Wp))
                a.tm = tune("dgrad_tm%d" % g.i, 0)      # co-scheduled dgrad m-tiles per wave per pass
                a.dbg = tune("dgrad_dbg", 0)            # A/B switches (ConvMMArgs::dbg; exact ones only)
                dname = "dgrad_conv%d" % g.i
                dual = (tune("dual_halo", True)
                        and not self._wide(g.Cs_in, g.KS, g.NT) and not self._wide(a.Cs_in, a.KS, g.NTd))
                if dual:
                    # one launch for the layer's wgrad and dgrad (independent GEMMs sharing dY):
                    # replaces the wgrad launch in place (its slabs are final after it)
                    ntc = self._halo_cfg(a, g.NTd, False, dual=True)
                    dname = "wgrad_dgrad_conv%d" % g.i
                    self.launches[w_at] = (dname, lambda s, a=a, n=ntc, w=wa, c=cfg, nm=dname: self._dual(a, n, w, c, s, nm),
                                           "main")
                else:
                    self.launches.append((dname, self._conv_launch(a, g.NTd, False)))
                self.pack_readers.append((dname, sp.offset, sp.offset + sp.numel))
        self._build_reduce()

    def _add_group_reduce(self):
        """Record where the group just appended has its partial slabs final."""
        self.red_ready.append(len(self.launches))

    def _build_reduce(self):
        """Merge per-layer slab groups (backward order) into buckets -- the DP reducer's
        buckets, or the same 1 MiB bucketing without DP (dense layer first, then convs) --
        and insert one reduction launch per bucket right after its last group's wgrad, on
        the side stream, so the dense bucket's reduction overlaps the conv backward."""
        ex, K = self.ex, self.ex.K
        groups = [(lo, hi) for lo, hi, _ in self.red_groups]
        reducer = ex.reducer
        dp_early = []
        self.early_push, self.pushed, self.early_xchg, self.exchanged = {}, None, {}, False
        self.bucket_xchg, self.xchg_end, self.xchg_fin = {}, None, None
        if reducer is not None:
            bucket_groups = reducer.configure(groups)
            # one bucket at the end of the backward (the adaptive plan for gradients <= 16 MB):
            # the groups final before the first dual launch (head, dense -- the single-GPU
            # step's early bucket) are REDUCED early there (grad_only: no update), so the
            # end-of-backward reduction ahead of the all-reduce only has the conv layers' slabs
            # left (the update stays behind the all-reduce)
            # one rank (the N = 1 data-parallel step): nothing to exchange -- the early groups
            # are reduced AND updated in that launch, as on a single GPU (xchg_p1: keep the
            # exchange structure, to measure its fixed cost)
            solo = reducer.size == 1 and getattr(reducer, "xgmi", None) is not None and not tune("xchg_p1", False)
            if len(bucket_groups) == 1 and self.comm_in_graph and tune("dp_early", True):
                dp_early = self._early_groups(grad_only=not solo)
                if solo and self.early_red:
                    self.pushed = next(iter(self.early_red.values()))[1]
                    self.exchanged = True
                # producer push (xGMI plane): the early groups' reduced gradient goes straight to
                # its owners' inboxes from the launch that reduces it, inside the backward, and
                # the fused all-reduce kernel skips those elements in its phase 1
                # ... and (exchange) the NEXT dual launch finishes that range's all-reduce and
                # applies its update in extra workgroups of its own, so the fused kernel after
                # the backward is left with the conv layers only
                if tune("xgmi_push", True) and not solo:
                    # every early table would start at block-flag slot 0 (fbase) and the pushed /
                    # exchanged range is ONE span: _early_groups caps them at one dual launch
                    assert len(self.early_red) <= 1, "exchange: one early table per step (flag slots, pushed range)"
                    for nm, (tab_, (elo, ehi), go) in self.early_red.items():
                        if not go:
                            continue
                        # (xchg_at=end: the exchange as a launch of its own after the end-of-
                        # backward reduction instead of extra workgroups of the next dual launch)
                        at_end = tune("xchg_at", "dual") == "end"
                        nxt = (("end" if at_end else self._xchg_launch(nm, elo, ehi))
                               if tune("xgmi_xchg", True) else None)
                        # split exchange (default): the owner half (wait for the senders, sum,
                        # push the sums back: mode 4) in extra workgroups of the next dual launch,
                        # covering only the table blocks this rank owns part of (none at one
                        # rank), and the finish half (wait for the other owners, update: mode 5)
                        # beside the end-of-backward table in ONE launch -- every wait is on a
                        # flag raised in an EARLIER launch, and no conv-sized workgroup holds a
                        # CU slot for the update (xchg_split=0: both halves in the dual launch)
                        if nxt and not at_end and tune("xchg_split", True):
                            trip = reducer.exchange_args(elo, ehi, tab_.nblocks, table=tab_)
                            if trip is not None:
                                self.early_push[nm] = trip[0]
                                if trip[1].b_hi > trip[1].b_lo:
                                    self.early_xchg[nxt] = (tab_, trip[1])
                                self.xchg_fin = (tab_, trip[2])
                                self.pushed, self.exchanged = (elo, ehi), True
                                continue
                        pair = reducer.exchange_args(elo, ehi, tab_.nblocks) if nxt else None
                        if pair is not None:
                            self.early_push[nm] = pair[0]
                            if at_end:
                                self.xchg_end = (tab_, pair[1])
                            else:
                                self.early_xchg[nxt] = (tab_, pair[1])
                            self.pushed, self.exchanged = (elo, ehi), True
                            continue
                        xp = reducer.push_args(elo, ehi)
                        if xp is not None:
                            self.early_push[nm], self.pushed = xp, (elo, ehi)
        else:
            # single stream, no all-reduce to overlap: ONE reduction launch at the end of the
            # backward (each launch boundary costs ~5 us here), if the descriptors fit a table
            ndesc = sum(len(d) for _, _, d in self.red_groups)
            one = ndesc <= tune("red_desc_max", 16)       # (RedTable capacity, MAX_RED)
            limit = 1 << 62 if one else int(os.environ.get("INTML_BUCKET_BYTES", 1 << 20))
            # ... with the optimizer fused into it when its table covers every parameter
            covered = sum(d[5] for _, _, ds in self.red_groups for d in ds)
            covered += sum(n for _, n in self.dense_fused_opt)
            self.optim_fused = one and covered == ex.store.numel and tune("fuse_optim", True)
            if not self.optim_fused:
                # the step ends with a full optimizer launch after all: the dense layers keep
                # writing their gradient in place, but leave the update -- and the bf16 pack
                # writes that go with it -- to it, so they also store the gradient it reads
                for wa, _ in self.dense_fused_opt:
                    wa.opt_w, wa.opt_b = -1, -1
                    wa.pk_fwd, wa.pk_bwd = -1, -1
                    wa.opt_nograd = 0
                self.dense_fused_opt = []
            early = self._early_groups() if self.optim_fused else []
            bucket_groups, cur, nb = [], [], 0
            for gi, (lo, hi) in enumerate(groups):
                if gi in early:
                    continue
                cur.append(gi)
                nb += (hi - lo) * 4
                if nb >= limit:
                    bucket_groups.append(cur)
                    cur, nb = [], 0
            if cur:
                bucket_groups.append(cur)
        self.bucket_tables = []
        inserts = []                       # (launch index to insert after, bucket)
        for k, bg in enumerate(bucket_groups):
            tab = K.RedTable()
            # longest reductions (most slabs) first: their workgroups dispatch first and their
            # memory round trips overlap the many short ones instead of trailing the launch
            for d in sorted((d for i in bg if i not in dp_early for d in self.red_groups[i][2]),
                            key=lambda d: -d[2]):
                tab.add(*d)
            lo = min(self.red_groups[i][0] for i in bg)
            hi = max(self.red_groups[i][1] for i in bg)
            self.bucket_tables.append((lo, hi, tab))
            inserts.append((max(self.red_ready[i] for i in bg), k))
        extra = []
        xk = getattr(reducer, "xgmi_bucket", None) if self.comm_in_graph else None
        # xGMI exchange of the end-of-backward table too (XgmiPush mode 3): its launch reduces the
        # conv layers' slabs, pushes them to their owners, finishes their all-reduce and applies
        # the update -- with the early range exchanged inside the backward, the whole step's
        # all-reduce + optimizer then runs in table launches and the fused kernel is not launched
        self.bucket_xchg = {}
        if xk is not None and tune("xgmi_xchg", True) and (self.exchanged or not dp_early):
            blo, bhi, btab = self.bucket_tables[xk]
            rlo, rhi = reducer.buckets[xk]
            early_n = (self.pushed[1] - self.pushed[0]) if self.exchanged else 0
            tab_n = sum(self.red_groups[i][1] - self.red_groups[i][0]
                        for i in bucket_groups[xk] if i not in dp_early)
            if btab.nblocks > 0 and early_n + tab_n == rhi - rlo:
                # (the early table's flag slots [0, its nblocks) -- one early table, asserted above)
                fb = sum(t.nblocks for t in {id(t): t for t in [e[0] for e in self.early_xchg.values()]
                                             + ([self.xchg_end[0]] if self.xchg_end else [])
                                             + ([self.xchg_fin[0]] if self.xchg_fin else [])}.values())
                x3 = reducer.exchange_args(blo, bhi, btab.nblocks, fbase=fb, fused=True)
                if x3 is not None:
                    self.bucket_xchg[xk] = x3
        if self.comm_in_graph:
            rccl_buckets = [k for k in range(len(bucket_groups)) if k != xk]
            # fork the comm stream only when an RCCL bucket has later backward work to overlap
            fork = tune("comm_fork", "")
            self.comm_fork = ((fork not in ("0", "false", "False")) if fork
                              else any(k < len(bucket_groups) - 1 for k in rccl_buckets))
            if self.comm_fork:
                self.comm_stream = torch.cuda.Stream(device=ex.device)
            if xk is not None:
                self.optim_on_comm = True
            extra.append(("allreduce_b%d", lambda k: None if k == xk else
                          (lambda s: reducer.launch(k, ex.store.grad, s)), "comm"))
            if self.optim_on_comm:
                extra.append(("optim_b%d", lambda k: None if k == xk else
                              (lambda s: self._launch_optim_comm(k, s)), "comm"))
            # the xGMI bucket: all-reduce + Keras update in one kernel on the main stream
            # (xchg_at=end: the early range's exchange + update after the end-of-backward reduction)
            extra.append(("xchg_early_b%d", lambda k: None if (k != xk or self.xchg_end is None) else
                          (lambda s: K.reduce_optim(ex.store.grad.data_ptr(), self.xchg_end[0],
                                                    ex._optim_args(False, defer_pack=True), s, self.xchg_end[1])),
                          "main"))
            # (the split exchange's finish half rides in the end-of-backward table launch; a launch
            # of its own only when that table is not exchanged)
            extra.append(("xchg_fin_b%d", lambda k: None if (k != xk or self.xchg_fin is None
                                                            or k in self.bucket_xchg) else
                          (lambda s: K.reduce_optim(ex.store.grad.data_ptr(), self.xchg_fin[0],
                                                    ex._optim_args(False, defer_pack=True), s, self.xchg_fin[1])),
                          "main"))
            extra.append(("xgmi_allreduce_optim_b%d", lambda k: None if (k != xk or k in self.bucket_xchg) else
                          (lambda s: reducer.launch_fused(ex.store.grad, ex._optim_args(False, defer_pack=True), s,
                                                          pushed=getattr(self, "pushed", None),
                                                          exchanged=getattr(self, "exchanged", False))),
                          "main"))
        self.launches, self.bucket_ready = splice_bucket_launches(
            self.launches, inserts,
            [("reduce_b%d", lambda k: (lambda s: self._launch_bucket_reduce(k, s)), "side")] + extra)
        if self.comm_in_graph and self.optim_on_comm:
            # a comm-stream optimizer writes its layers' packs: never while a later
            # main-stream launch (a wide conv's separate dgrad) still reads one of them
            self.launches = defer_after_readers(self.launches, "optim_b%d",
                                                [(lo, hi) for lo, hi, _ in self.bucket_tables],
                                                self.pack_readers)
        spans = [(lo, hi) for lo, hi, _ in self.bucket_tables]
        # (data parallel: every early reduction lies inside its all-reduce bucket's span)
        if reducer is None:
            spans += [e[1] for e in (self.early_red or {}).values()]
        check_bucket_cover(spans, ex.store.numel)

    def _early_groups(self, grad_only: bool = False):
        """Single-GPU fused-optimizer step: slab groups whose gradients are final before a dual
        conv backward launch (the head and dense layers before the first one) are reduced and
        updated by extra workgroups OF that launch (DualExtra) instead of in the end-of-step
        reduction -- their latency-bound reduce + update overlaps the conv backward.  Only
        groups no later launch reads the weights of (pack readers), as one contiguous
        parameter span.  Sets
        self.early_red = {launch name: (RedTable, (lo, hi), grad_only)}; returns the groups
        assigned.  grad_only (data-parallel step): reduction only -- no update, no pack
        writes, so later pack readers do not matter."""
        self.early_red = {}
        if not tune("early_reduce", True):
            return []
        names = [it[0] for it in self.launches]
        # only the FIRST dual launch carries a bucket: every dual launch carrying the previous
        # layer's bucket (conv2's in dual conv1, ...) measured 3% slower on RPV (conv2's
        # many-split slabs stretch dual conv1's tail by ~3 us, more than the reduction sheds)
        # (the step's last wgrad launch -- the first conv layer's -- carrying the other conv
        # layers' reductions as extra workgroups measured 2-3 us slower on RPV and MNIST:
        # profiles/r3_s2_early_wgrad_ab.txt)
        duals = [i for i, nm in enumerate(names) if nm.startswith("wgrad_dgrad_conv")][:1]
        # (the step's last launch -- the first conv layer's halo wgrad -- reducing + updating the
        # earlier conv layers' slabs in its own workgroups' tails measured slower too: RPV
        # 1.121M -> 1.071M img/s, legacy 103.4k -> 94.7k; profiles/r4_ab_rpv.txt)
        taken = []
        for t in duals:
            late_readers = [] if grad_only else [(rlo, rhi) for nm, rlo, rhi in self.pack_readers
                                                 if nm not in names[:t]]
            grp = [gi for gi in range(len(self.red_groups)) if gi not in taken and self.red_ready[gi] <= t
                   and not any(rlo < self.red_groups[gi][1] and rhi > self.red_groups[gi][0]
                               for rlo, rhi in late_readers)]
            if not grp:
                continue
            lo = min(self.red_groups[gi][0] for gi in grp)
            hi = max(self.red_groups[gi][1] for gi in grp)
            descs = [d for gi in grp for d in self.red_groups[gi][2]]
            if (sum(self.red_groups[gi][1] - self.red_groups[gi][0] for gi in grp) != hi - lo
                    or not descs or len(descs) > 16):
                continue                                   # not one contiguous span / table
            tab = self.ex.K.RedTable()
            for d in sorted(descs, key=lambda d: -d[2]):
                tab.add(*d)
            self.early_red[names[t]] = (tab, (lo, hi), grad_only)
            taken += grp
        return taken

    def _xchg_launch(self, name, lo, hi):
        """The dual launch after ``name`` that can run the exchange (all-reduce finish + update)
        of the early range [lo, hi): the next dual backward launch, provided no launch from it
        on reads the range's bf16 packs (the update rewrites them).  None if there is none."""
        names = [it[0] for it in self.launches]
        i = names.index(name)
        nxt = [j for j in range(i + 1, len(names)) if names[j].startswith("wgrad_dgrad_conv")]
        if not nxt:
            return None
        later = set(names[nxt[0]:])
        if any(nm in later and rlo < hi and rhi > lo for nm, rlo, rhi in self.pack_readers):
            return None
        return names[nxt[0]]

    def _launch_optim_comm(self, k, stream):
        """Keras update of bucket k's parameters on the comm stream after its all-reduce;
        it writes the bf16 packs of the weights it updates (pack routes), so the launch list
        places it behind the last backward launch reading one of them (defer_after_readers)."""
        ex = self.ex
        lo, hi, _ = self.bucket_tables[k]
        a = ex._optim_args(False, defer_pack=True)   # built at capture time: grad_scale = 1/size
        a.lo, a.n = lo, hi - lo
        ex.tile_routes(a)
        if getattr(self, "_no_packs", None) is None:
            self._no_packs = ex.K.PackTable()
        ex.K.optim(a, self._no_packs, stream.cuda_stream if hasattr(stream, "cuda_stream") else stream)

    # ---------------------------------------------------------------- execution
    def _run_seq(self, lo: int = 0, hi: Optional[int] = None):
        """Launch [lo, hi) on the streams ``stream_program`` assigns (concurrent chains that
        join main at the end)."""
        items = self.launches[lo:hi]
        skip = tune("skip", "")          # timing ablation only (wrong results): "name/name"
        if skip:
            drop = set(skip.split("/"))
            items = [it for it in items if it[0] not in drop]
        tags = [it[2] if len(it) > 2 else "main" for it in items]
        streams = {"main": torch.cuda.current_stream(), "comm": self.comm_stream}
        for op in stream_program(tags, comm=self.comm_stream is not None):
            if op[0] == "wait":
                streams[op[1]].wait_stream(streams[op[2]])
                continue
            _, sname, i = op
            st = streams[sname]
            # comm launches take the Stream (RCCL wrappers use it as a context); others the handle
            items[i][1](st if tags[i] == "comm" else st.cuda_stream)

    def _launch_bucket_reduce(self, k, s):
        lo, hi, tab = self.bucket_tables[k]
        ex = self.ex
        xp = (getattr(self, "bucket_xchg", None) or {}).get(k)
        fin = getattr(self, "xchg_fin", None)
        if xp is not None and fin is not None:   # + the early range's exchange finish (mode 5)
            ex.K.reduce_optim_end(ex.store.grad.data_ptr(), tab, ex._optim_args(False, defer_pack=True), s, xp,
                                  fin[0], fin[1])
        elif xp is not None:     # reduction + all-reduce (exchange) + Keras update in one launch
            ex.K.reduce_optim(ex.store.grad.data_ptr(), tab, ex._optim_args(False, defer_pack=True), s, xp)
        elif self.optim_fused:     # gradient reduction + Keras update in one launch (re-pack deferred)
            ex.K.reduce_optim(ex.store.grad.data_ptr(), tab, ex._optim_args(False, defer_pack=True), s)
        else:
            ex.K.slab_reduce(ex.store.grad.data_ptr(), lo, hi, tab, s)

    def _launch_optim(self):
        ex = self.ex
        # the re-pack of the updated weights is done by the next step's prologue launch
        ex.K.optim(ex.tile_routes(ex._optim_args(False, defer_pack=True)), ex.pack_table,
                   torch.cuda.current_stream().cuda_stream)

    def _body(self, with_optim: bool):
        self._run_seq()
        if self.training and with_optim and not self.optim_fused and not self.optim_on_comm:
            self._launch_optim()

    def _dp_segments(self):
        """[(launch_lo, launch_hi, bucket)]: segment k ends with the slab reduction that
        completes bucket k; a trailing (lo, hi, None) segment holds any later launches."""
        segs, lo = [], 0
        for k, ready in enumerate(self.bucket_ready):
            segs.append((lo, ready, k))
            lo = ready
        if lo < len(self.launches):
            segs.append((lo, len(self.launches), None))
        return segs

    def _run_segment(self, lo, hi, k):
        self._run_seq(lo, hi)

    def run(self, k: int = 1):
        """Run ``k`` consecutive steps.  Step bookkeeping (data cursor, iteration count, LR,
        dropout counter) is device-resident, so k steps are ONE graph of k back-to-back step
        bodies: the inter-graph launch gap is paid once per k steps."""
        ex = self.ex
        dp = self.training and ex.reducer is not None and ex.reducer.active
        if dp:
            ex.grad_scale = 1.0 / ex.reducer.size
        if not dp or self.comm_in_graph:
            # single launch sequence; with the native RCCL engine it includes the bucket
            # all-reduces on the comm stream (one graph replay per DP step / k steps)
            if not ex.use_graphs:
                for _ in range(k):
                    self._body(with_optim=True)
            elif k == 1:
                if self.graph is None:
                    self.graph = self._capture(lambda: self._body(with_optim=True))
                self.graph.replay()
            else:
                g = self.multi_graphs.get(k)
                if g is None:
                    def body_k():
                        for _ in range(k):
                            self._body(with_optim=True)
                    g = self.multi_graphs[k] = self._capture(body_k)
                g.replay()
            if dp:
                ex.reducer.after_step()
            return
        for _ in range(k):
            self._run_dp_segmented()

    def _run_dp_segmented(self):
        ex = self.ex
        # Data parallel, torch.distributed data plane: each bucket's all-reduce is issued
        # between graph segments as soon as its slab reduction is done, so RCCL moves the
        # dense bucket over xGMI while the conv backward runs; the fused optimizer (with the
        # 1/size average folded in) runs after the last wait.
        segs = self._dp_segments()
        if ex.use_graphs and self.dp_graphs is None:
            self.dp_graphs = [self._capture(lambda a=lo, b=hi, k=k: self._run_segment(a, b, k))
                              for lo, hi, k in segs]
            self.dp_graphs.append(self._capture(self._launch_optim))
        for j, (lo, hi, k) in enumerate(segs):
            if ex.use_graphs:
                self.dp_graphs[j].replay()
            else:
                self._run_segment(lo, hi, k)
            if k is not None:
                ex.reducer.start(k, ex.store.grad)
        ex.reducer.finish()
        if ex.use_graphs:
            self.dp_graphs[-1].replay()
        else:
            self._launch_optim()

    def _capture(self, fn):
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(device=self.ex.device)
        s.wait_stream(torch.cuda.current_stream())
        # no Python GC inside the capture: collecting an unreachable plan of another model
        # destroys its graphs/events, which HIP forbids while a stream is capturing (abort)
        gc_was = gc.isenabled()
        gc.collect()
        gc.disable()
        try:
            # thread-local capture mode: RCCL / watchdog threads may query events meanwhile
            with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                fn()
        finally:
            if gc_was:
                gc.enable()
        torch.cuda.current_stream().wait_stream(s)
        return g
