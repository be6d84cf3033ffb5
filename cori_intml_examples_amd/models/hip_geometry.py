"""Per-launch geometry of the HIP backend's BatchPlan: the layer-fused conv stack's row
bands and LDS layout, the halo conv / wgrad / tiled / dense kernels' tile, split and block
choices, and the launch helpers that dispatch between them.  A mixin of
executor_hip.BatchPlan (split out of it to keep the step-program logic and the geometry
apart); every method reads the plan's executor (``self.ex``) and batch size."""
from __future__ import annotations

import torch

from ..ops.rng import keep_threshold
from ..utils.env import tune
from . import lds_layout


def cdiv(a, b):
    return -(-a // b)


def r8(x):
    return cdiv(x, 8) * 8


def _pow2_le(x, cap):
    p = 1
    while p * 2 <= min(x, cap):
        p *= 2
    return p


class GeometryMixin:
    LDS_LIMIT = 160 * 1024

    def _conv_stack_args(self, training: bool):
        """ConvStackArgs for the layer-fused forward (one workgroup per image, activations in
        LDS), or None when the conv stack does not qualify: stride-1 convs, <= 64 output
        channels, <= MAX_STACK layers, and the per-image working set within the LDS."""
        ex, K = self.ex, self.ex.K
        convs = ex.convs
        if not convs or len(convs) > K.MAX_STACK:
            return None
        for g in convs:
            if g.stride != 1 or g.NT > 4 or g.Cs_out % 8 or (g.Cs_in != 4 and g.Cs_in % 8):
                return None

        # row bands per image: enough workgroups to cover the 256 CUs at small batches
        want = tune("stack_splits", 0) or cdiv(256, self.bs)
        splits = max(1, min(K.MAX_STACK_SPLIT, want))
        while splits > 1 and self._stack_rows(convs, splits) is None:
            splits -= 1
        rows = self._stack_rows(convs, splits)
        if rows is None:
            return None
        layout = self._stack_layout(convs, rows, splits)
        if layout is None:
            return None
        off_w, w_off, off_b0, off_b1, off_codes, lds, off_bias = layout
        n = len(convs)
        a = K.ConvStackArgs()
        a.x = self.xb.data_ptr()
        a.B, a.n, a.seed, a.st = self.bs, n, ex.seed, ex.state.data_ptr()
        a.off_w, (a.off_codes, a.off_codes2), a.lds_bytes = off_w, off_codes, lds
        a.off_bias = off_bias
        a.dbg = tune("stack_dbg", 0)
        a.k16 = int(tune("stack_k16", True))
        a.wt = int(bool(int(tune("wt", 7)) & 1))      # write-through stage outputs / codes
        # a layer-signature-specialised instance when one matches (conv_stack.hip kStackSigs):
        # 1 = 12-wave instances, 2 (default: +0.4 %, profiles/r5e_ab.txt) = a 16-wave instance first
        # where one exists, 0 = generic
        a.spec = int(tune("stack_spec", 2))
        a.set_buf_offsets(off_b0, off_b1)
        a.splits = splits
        for l in range(n):
            for sp in range(splits):
                a.set_rows(l, sp, *rows[l][sp])
        store = ex.store
        lay = self._stack_img_layouts(convs)
        for i, (g, cs) in enumerate(zip(convs, ex.plan.convs)):
            L = K.StackLayer()
            L.H, L.W, L.Cs_in = g.H, g.W, g.Cs_in
            L.Ho, L.Wo, L.Cout, L.Cs_out = g.Ho, g.Wo, g.Cout, g.Cs_out
            L.KH, L.KW, L.pad_t, L.pad_l = g.KH, g.KW, g.pad_t, g.pad_l
            L.KS, L.NT = g.KS, g.NT
            L.pool, L.relu = int(g.pool), int(g.relu)
            L.Hp, L.Wp = g.Hp, g.Wp
            if training and g.rate > 0:
                L.drop_thr = keep_threshold(g.rate)
                L.drop_scale = 1.0 / (1.0 - g.rate)
            L.stream_id = g.stream
            L.wpk = ex.arena.data_ptr() + 2 * g.pack_fwd
            L.bias = store.view(cs.conv, "bias").data_ptr() if cs.conv.use_bias else 0
            L.out = self.conv_out[i].data_ptr()
            if g.pool:
                L.code = self.conv_code[i].data_ptr()
            L.w_lds = w_off[i]
            L.xpix, L.xrow = lay[i]
            a.set_layer(i, L)
        self.stack_splits = splits
        return a

    @staticmethod
    def _stack_rows(convs, splits):
        """Per layer, per row band: (c0, c1, own0, own1, ib, ih) = conv-output rows computed,
        stage-output rows stored, and the input halo image's first input row and row count.
        Bands own an even partition of every layer's stage rows; each band computes its
        owned rows plus what the next layer's computed rows read (halo), walking the stack
        backwards.  A layer's input image spans both the rows its conv reads and the rows the
        previous layer stores from it.  None if a band would own no rows."""
        n = len(convs)
        rows = [[None] * splits for _ in range(n)]
        for sp in range(splits):
            need = None                       # stage-output rows of layer l needed downstream
            for l in range(n - 1, -1, -1):
                g = convs[l]
                P = 2 if g.pool else 1
                own = (sp * g.Hp // splits, (sp + 1) * g.Hp // splits)
                if own[1] <= own[0]:
                    return None
                lo, hi = own
                if need is not None:
                    lo, hi = min(lo, need[0]), max(hi, need[1])
                lo, hi = max(lo, 0), min(hi, g.Hp)
                c0, c1 = lo * P, hi * P
                rows[l][sp] = [c0, c1, own[0], own[1], c0 - g.pad_t, c1 - c0 + g.KH - 1]
                need = (max(c0 - g.pad_t, 0), min(c1 - 1 - g.pad_t + g.KH, g.H))
            for l in range(1, n):             # image of layer l also holds layer l-1's stored rows
                r, o0, o1 = rows[l][sp], rows[l - 1][sp][2], rows[l - 1][sp][3]
                ib0, ie0 = r[4], r[4] + r[5]
                r[4] = min(ib0, o0)
                r[5] = max(ie0, o1) - r[4]
        return [[tuple(r) for r in layer] for layer in rows]

    def _stack_layout(self, convs, rows, splits):
        """LDS byte layout: zeros + per-layer k-offset tables | biases | all weight packs | two
        ping-pong halo images | two code planes.  None if it exceeds the CU's LDS."""
        def a16(v):
            return (v + 15) & ~15

        n = len(convs)
        lay = self._stack_img_layouts(convs)
        ntab = max((g.KS * 8 if g.Cs_in == 4 else g.KS * 4) for g in convs)
        tabn = self.ex.K.STACK_TABN
        if ntab > tabn:
            return None
        off_bias = 32 + a16(4 * tabn * self.ex.K.MAX_STACK)         # [layer][STACK_TABN] tables
        off_w = off_bias + 4 * 64 * self.ex.K.MAX_STACK      # biases [layer][64] fp32
        w_off, welems = [], 0
        for g in convs:
            w_off.append(welems)
            welems += g.KS * g.NT * 64 * 8
        bufs, codes = [0, 0], 16
        for l, g in enumerate(convs):
            P = 2 if g.pool else 1
            for sp in range(splits):
                c0, c1, _, _, _, ih = rows[l][sp]
                bufs[l & 1] = max(bufs[l & 1], ih * lay[l][1] * lay[l][0])
                if g.pool:
                    codes = max(codes, (c1 - c0) // 2 * g.Wp * g.Cs_out)
                if l == n - 1:
                    bufs[n & 1] = max(bufs[n & 1], (c1 - c0) // P * g.Wp * g.Cs_out)
        off_b0 = off_w + a16(2 * welems)
        off_b1 = off_b0 + a16(2 * bufs[0])
        off_codes = off_b1 + a16(2 * bufs[1])
        off_codes2 = off_codes + a16(codes)          # two code planes (layer parity)
        lds = off_codes2 + a16(codes)
        if lds > self.LDS_LIMIT:
            return None
        return off_w, w_off, off_b0, off_b1, (off_codes, off_codes2), lds, off_bias

    @staticmethod
    def _stack_img_layouts(convs):
        """(xpix, xrow) of each stack layer's input halo image (lds_layout.stack_layout; dense
        when the tune switch lds_layout is off)."""
        out = []
        for g in convs:
            Wi = g.Wo + g.KW - 1
            rows_path = g.pool and g.Wp % 4 == 0 and g.KH == 3 and g.KW == 3
            if tune("lds_layout", True):
                out.append(lds_layout.stack_layout(g.Cs_in, Wi, g.Wo, bool(rows_path), g.KS))
            else:
                out.append((g.Cs_in, Wi))
        return out

    @staticmethod
    def _wide(Cs_in: int, KS: int, NT: int) -> bool:
        """Wide layer: conv_halo would have to keep all of K's weights in LDS for fewer
        n-tiles than a 128-channel tile needs -> use the tiled whole-batch GEMM kernels."""
        return Cs_in % 32 == 0 and KS * min(NT, 8) > 64

    def _cu_count(self):
        """Compute units of the executor's device (256 on MI355X; CPU / no device: 256)."""
        if getattr(self, "_ncu", None) is None:
            try:
                self._ncu = int(torch.cuda.get_device_properties(self.ex.device).multi_processor_count)
            except Exception:          # noqa: BLE001
                self._ncu = 256
        return self._ncu

    def _zero_buf(self):
        """Zero bytes for the LDS-DMA kernels: padded rows read from here (DMA cannot zero-fill)."""
        if getattr(self, "_zero16", None) is None:
            self._zero16 = torch.zeros(64, dtype=torch.bfloat16, device=self.ex.device)
        return self._zero16

    def _conv_launch(self, a, NT, pool):
        K = self.ex.K
        if self._wide(a.Cs_in, a.KS, NT):
            ntc = 8 if NT > 4 else (4 if NT > 2 else 2)
            if K.conv_tile_lds_bytes(ntc) > 150 * 1024:
                raise NotImplementedError("conv tile LDS")
            big = False
            if tune("conv_glds", True):
                a.zero = self._zero_buf().data_ptr()
                # 256-row / 8-wave blocks (all 256 channels of a wide layer per block: NTC 16)
                # when the grid keeps >= 512 blocks: half the L2 traffic per MFMA
                if tune("conv_big", True) and a.in_code == 0:
                    for nb in ((16, 8) if NT >= 16 else (8,)):
                        if NT >= nb and K.conv_tile_big_blocks(a, nb) >= tune("conv_big_min", 512):
                            ntc, big = nb, True
                            break
                # stride-1 layers (and the parity classes of a strided dgrad) with whole-row
                # blocks: the halo-staged kernel (each input pixel DMA'd once per 32-channel
                # chunk instead of once per tap)
                # (8 n-tiles per block: 116 VGPRs and 80 KB of LDS -- two blocks per CU; the
                # all-256-channel NTC 16 block, one per CU, measured no faster than conv_gl;
                # a 64-channel strided dgrad takes 4-tile blocks)
                hs = int(tune("conv_hs_ntc", 8))
                if NT < hs:
                    hs = 4 if NT >= 4 and a.in_dil > 1 else 0
                dil_ok = a.in_dil <= 1 or tune("conv_hs_dil", True)
                if tune("conv_hs", True) and hs and dil_ok:
                    # 16 waves / 512-row blocks where the shape tiles into them (half the weight
                    # DMA per MFMA), else 8 waves / 256 rows
                    for wv in ((16, 8) if tune("conv_hs_wv", 8) == 16 else (8,)):
                        if K.conv_hs_ok(a, hs, wv):
                            # (1: the n-blocks of a row block adjacent on one XCD -- legacy conv3
                            # forward 103.0 -> 101.6 us, profiles/r6_conv_hs_order_ab.txt)
                            o = int(tune("conv_hs_order", 1))
                            return lambda s, a=a, n=hs, w=wv, o=o: K.conv_hs(a, n, s, w, o)
            nbuf = int(tune("conv_gl_nbuf", 3))
            return lambda s, a=a, n=ntc, b=big, nb=nbuf: K.conv_tile(a, n, s, b, nb)
        ntc = self._halo_cfg(a, NT, pool)
        if not a.tm:
            # 4-tile blocks: two m-tiles per wave per pass -- half the epilogue staging LDS, four
            # workgroups per CU instead of three (legacy first conv 37.7 -> 26.8 us,
            # profiles/r6_halo_tm_ab.txt); halo_tm=4 restores the four-tile pass
            a.tm = int(tune("halo_tm", 2))
        return lambda s, a=a, n=ntc: K.conv_halo(a, n, s)

    def _dense_dual(self, wa, cfg, da, s):
        K = self.ex.K
        if not K.dense_bwd_dual(wa, cfg[0], cfg[1], cfg[2], da, s):   # unsupported combination
            K.wgrad(wa, cfg[0], cfg[1], cfg[2], s)
            K.dense_fwd(da, s)

    def _dual(self, a, ntc, wa, cfg, s, name=None):
        K, ex = self.ex.K, self.ex
        early = (self.early_red or {}).get(name)
        xp = (getattr(self, "early_push", None) or {}).get(name)   # producer push (xGMI plane)
        # exchange (xGMI plane): this launch finishes an earlier launch's pushed range -- its
        # all-reduce + Keras update in extra workgroups (XgmiPush mode 2)
        xe = (getattr(self, "early_xchg", None) or {}).get(name)
        kw = {}
        if early is not None:   # this launch also carries an early bucket's reduction (+ optimizer)
            kw.update(rt=early[0], ro=self._early_ro(early), rgrad=ex.store.grad.data_ptr(),
                      rfirst=int(tune("early_rfirst", 0)))   # (0: last in the grid, 1: first, 2: interleaved)
            if xp is not None:
                kw["xp"] = xp
        elif xe is not None:
            kw.update(rt=xe[0], ro=ex._optim_args(False, defer_pack=True), rgrad=ex.store.grad.data_ptr(), xp=xe[1],
                      rfirst=int(tune("xchg_rfirst", 1)))   # (dispatched first: their waits overlap the convs)
        ok = K.dual_halo(a, ntc, wa, cfg[0], cfg[1], cfg[2], s, **kw)
        if not ok:   # unsupported combination
            K.wgrad_halo(wa, cfg[0], cfg[1], cfg[2], s)
            K.conv_halo(a, ntc, s)
            if "rt" in kw:
                K.reduce_optim(kw["rgrad"], kw["rt"], kw["ro"], s, kw.get("xp"))

    def _early_ro(self, early):
        """OptimArgs of an early reduction table: the Keras update, or (data-parallel step,
        early[2]) the reduction only -- the update follows the all-reduce."""
        ro = self.ex._optim_args(False, defer_pack=True)
        ro.grad_only = int(early[2])
        return ro

    def _halo_cfg(self, a, NT, pool, dual=False):
        """Pick n-tiles per workgroup (weight LDS slice) and R output rows per block: the
        largest block that still leaves >= `want` workgroups (a dgrad co-scheduled with its
        wgrad in one launch wants fewer, longer workgroups: each stages the whole weight
        slice, and the launch should fit the CUs in one wave)."""
        want = tune("dgrad_min_wgs", 256) if dual else tune("halo_min_wgs", 512)
        KS = a.KS
        # co-scheduled dgrad: one n-tile per workgroup and whole-image blocks (measured on the
        # RPV stack: each workgroup stages half the weights, the launch fits the CUs in one wave)
        ntc = tune("dgrad_ntc", 1) if dual else 8
        while ntc > 1 and (ntc > NT or KS * ntc > 64):
            ntc //= 2
        if KS * ntc > 96:
            raise NotImplementedError("conv K too large for the LDS weight stage (KS=%d)" % KS)
        Wo, Ho = a.Wo, a.Ho
        W_in = (Wo - 1) * a.stride + a.KW
        step = 2 if pool else 1
        a.kpipe = int(tune("conv_kpipe", True))
        gy = cdiv(NT, ntc)

        def rows(XP):
            # Balanced blocks: the fewest row blocks per image (c) that satisfy the limits, each
            # cdiv(Ho, c) rows -- not the largest R with a short remainder block.  Measured on
            # MNIST's 26-row dgrad (co-scheduled with its wgrad): 15 + 11-row blocks 156 us/step,
            # 13 + 13 125 us; the RPV layers divide evenly and are unchanged.
            for c in range(1, Ho + 1):
                R = cdiv(cdiv(Ho, c), step) * step
                if R * Wo > 512:
                    continue
                halo = ((R - 1) * a.stride + a.KH) * W_in * XP * 2
                if halo + KS * ntc * 1024 > 80 * 1024:
                    continue
                if a.B * cdiv(Ho, R) * gy < want:
                    continue         # too few workgroups: more, smaller blocks
                return R
            return step

        best = rows(a.Cs_in)
        if tune("lds_layout", True) and a.Cs_in % 8 == 0:
            # the bank-conflict-free pixel stride, unless its larger halo costs block rows
            xp = lds_layout.conv_layout(a.Cs_in, W_in, Wo, bool(pool), a.KH, a.KW)
            if xp != a.Cs_in and rows(xp) >= best:
                a.xpix = xp
        a.R = best
        lds = self.ex.K.conv_halo_lds_bytes(a, ntc)
        if lds > 150 * 1024:
            raise NotImplementedError("conv halo stage too large (%d bytes)" % lds)
        return ntc

    def _wgrad_tile_args(self, xin, g, bs, bias):
        """Tiled wgrad for wide convs: 128(k) x ntc*16(n) tiles, split-K over pixel ranges."""
        K, dev = self.ex.K, self.ex.device
        a = K.WgradArgs()
        a.x = xin.data_ptr()
        a.B, a.H, a.W, a.Cs_in = bs, g.H, g.W, g.Cs_in
        a.Ho, a.Wo, a.KH, a.KW, a.stride, a.pad_t, a.pad_l = g.Ho, g.Wo, g.KH, g.KW, g.stride, g.pad_t, g.pad_l
        a.Ktiles = cdiv(g.KH * g.KW * g.Cs_in, 16)
        a.dy = self.conv_dy[g.i].data_ptr()
        a.Cs_dy = g.Cs_out
        if g.pool:
            a.dy_code = self.conv_code[g.i].data_ptr()
            a.dHp, a.dWp = g.Hp, g.Wp
        a.NT = g.NT
        ntc = 8 if g.NT > 4 else (4 if g.NT > 2 else 2)
        ntc = min(ntc, tune("wgrad_tile_ntc", ntc))
        if tune("conv_glds", True):
            a.zero = self._zero_buf().data_ptr()
        P = bs * g.Ho * g.Wo
        a.P = P
        tiles = cdiv(a.Ktiles * 16, 128) * cdiv(g.NT, ntc)
        per_split_bytes = a.Ktiles * 16 * g.NT * 16 * 4
        # split count: as many workgroups as fit the machine AT ONCE (64 KB of LDS each: two per
        # CU), never one more -- a grid a few workgroups past a whole number of residency
        # waves runs a second wave for them and nearly doubles the launch (legacy conv3 wgrad
        # 113 us at 486 workgroups, 185 us at 522; profiles/r6_wgrad_splits_ab.txt).  The
        # reduction's slab bytes halve with it (end-of-step reduce + Adam 54 -> 35 us).
        slots = tune("wgrad_tile_fill", 1) * self._cu_count() * 2
        wgs = tune("wgrad_tile_wgs", 0)
        S = max(1, min(cdiv(wgs, tiles) if wgs else max(1, slots // tiles),
                       (tune("wgrad_tile_slab_mb", 64) << 20) // per_split_bytes, cdiv(P, 256)))
        a.px_per_split = cdiv(cdiv(P, S), 64) * 64
        S = cdiv(P, a.px_per_split)
        slab = torch.zeros(S, a.Ktiles * 16, g.NT * 16, dtype=torch.float32, device=dev)
        bslab = torch.zeros(S, g.NT * 16, dtype=torch.float32, device=dev) if bias else None
        a.slab = slab.data_ptr()
        a.bslab = bslab.data_ptr() if bslab is not None else 0
        self.wgrad_slabs.append((slab, bslab))
        return a, (ntc, None, S), slab, bslab

    def _wgrad_halo_args(self, xin, g, bs, bias):
        K, dev = self.ex.K, self.ex.device
        a = K.WgradArgs()
        a.x = xin.data_ptr()
        a.B, a.H, a.W, a.Cs_in = bs, g.H, g.W, g.Cs_in
        a.Ho, a.Wo, a.KH, a.KW, a.stride, a.pad_t, a.pad_l = g.Ho, g.Wo, g.KH, g.KW, g.stride, g.pad_t, g.pad_l
        a.Ktiles = cdiv(g.KH * g.KW * g.Cs_in, 16)
        a.dy = self.conv_dy[g.i].data_ptr()
        a.Cs_dy = g.Cs_out
        if g.pool:
            a.dy_code = self.conv_code[g.i].data_ptr()
            a.dHp, a.dWp = g.Hp, g.Wp
        NT = g.NT
        a.NT = NT
        a.P = bs * g.Ho * g.Wo
        NTT = _pow2_le(NT, 8)
        # each wave owns <= 4 m-tiles x NTT n-tiles (<= 16 accumulator tiles)
        mt_cap = (8 if NTT == 8 else 16) - (1 if bias else 0)
        MT = max(1, min(a.Ktiles, mt_cap))
        MT = cdiv(a.Ktiles, cdiv(a.Ktiles, MT))        # balance the m-groups
        # rows per block: ~256 pixels (the first layer, a standalone launch: ~512), at most 8
        # rows (measured best at batch 128 for the RPV and MNIST stacks; RPV first layer
        # 512 px = 8 rows: +0.2-0.5 %, profiles/r4m_ab_rpv.txt, r4n_ab_rpv.txt), bounded LDS
        W_in = (g.Wo - 1) * g.stride + g.KW
        px = tune("wgrad_block_px%d" % g.i, tune("wgrad_block_px", 512 if g.i == 0 else 256))
        R = max(1, min(g.Ho, px // max(1, g.Wo), tune("wgrad_max_rows%d" % g.i, tune("wgrad_max_rows", 8))))
        # prefer the largest R whose block staging fits the kernel's register pipeline
        # (<= 4 X-halo and 4 dY chunks per thread, wgrad_halo_body.h WH_PX / WH_PY)
        cpp = g.Cs_in // (4 if g.Cs_in == 4 else 8)

        def fits(r):
            w_in = (g.Wo - 1) * g.stride + g.KW
            nch_x = ((r - 1) * g.stride + g.KH) * w_in * cpp
            nch_y = cdiv(r * g.Wo, 32) * 32 * NTT * 2
            return nch_x <= 1024 and nch_y <= 1024
        for r in range(R, 0, -1):
            if fits(r) or not tune("wgrad_fit%d" % g.i, True):
                R = r
                break
        # LDS layout from the bank-conflict model (pixel / row strides of the X halo, dY rows)
        a.kperm = int(tune("wgrad_perm", True)) | (0 if tune("wgrad_fast", True) else 2)
        if tune("lds_layout", True):
            a.xpix, a.xrow, a.dyld = lds_layout.wgrad_layout(g.Cs_in, W_in, g.Wo, NTT, g.KH, g.KW, g.stride,
                                                             a.Ktiles, bool(a.kperm & 1))
        XP, XR = (a.xpix or g.Cs_in), (a.xrow or W_in)
        while R > 1 and (((R - 1) * g.stride + g.KH) * XR * XP * 2 > 64 * 1024):
            R -= 1
        a.R = R
        nblocks = bs * cdiv(g.Ho, R)
        groups = cdiv(NT, NTT) * cdiv(a.Ktiles, MT)
        per_split_bytes = a.Ktiles * 16 * NT * 16 * 4
        s_budget = max(1, (tune("wgrad_slab_mb", 8) << 20) // per_split_bytes)
        # splits: one round of resident workgroups (occupancy x CUs), not more -- the
        # latency-bound blocks then all stream concurrently instead of a second thin round
        cap = (tune("wgrad_splits%d" % g.i, 0) or tune("wgrad_splits", 0) or K.wgrad_halo_resident(a, MT, NTT, bool(bias))
               or 768)
        S = max(1, min(nblocks, s_budget, max(1, cap // groups)))
        bps = cdiv(nblocks, S)
        S = cdiv(nblocks, bps)
        a.blocks_per_split = bps
        lds = K.wgrad_halo_lds_bytes(a, MT, NTT)
        if lds > 150 * 1024:
            raise NotImplementedError("wgrad halo stage too large (%d bytes)" % lds)
        slab = torch.zeros(S, a.Ktiles * 16, NT * 16, dtype=torch.float32, device=dev)
        bslab = torch.zeros(S, NT * 16, dtype=torch.float32, device=dev) if bias else None
        a.slab = slab.data_ptr()
        a.bslab = bslab.data_ptr() if bslab is not None else 0
        # write-through slabs (16-byte sc1 stores, byte offsets < 2 GB)
        a.wt = int(bool(int(tune("wt", 7)) & 4) and slab.numel() * 4 < (1 << 31))
        self.wgrad_slabs.append((slab, bslab))
        return a, (MT, NTT, S), slab, bslab

    def _wgrad_args(self, xin, H, W, Cs_in, Ho, Wo, KH, KW, stride, pad_t, pad_l, dy, Cs_dy, N, bs, bias,
                    direct=None):
        K, dev = self.ex.K, self.ex.device
        a = K.WgradArgs()
        a.x = xin.data_ptr()
        a.B, a.H, a.W, a.Cs_in = bs, H, W, Cs_in
        a.Ho, a.Wo, a.KH, a.KW, a.stride, a.pad_t, a.pad_l = Ho, Wo, KH, KW, stride, pad_t, pad_l
        if not (Cs_in == 4 or Cs_in % 8 == 0):
            raise NotImplementedError("wgrad needs Cs_in == 4 or a multiple of 8 (got %d)" % Cs_in)
        a.Ktiles = cdiv(KH * KW * Cs_in, 16)
        a.dy = dy.data_ptr()
        a.Cs_dy = Cs_dy
        NT = cdiv(N, 16)
        a.NT = NT
        P = bs * Ho * Wo
        a.P = P
        ntt = _pow2_le(NT, 8)
        ktw = 4 if ntt <= 4 else 2
        while ktw > 1 and 4 * (ktw // 2) >= a.Ktiles:
            ktw //= 2
        if ntt == 8 and ktw == 4:
            ktw = 2
        a.KT = 4 * ktw
        gy = cdiv(a.Ktiles, a.KT)
        gz = cdiv(NT, ntt)
        per_split_bytes = a.Ktiles * 16 * NT * 16 * 4
        s_budget = max(1, (4 << 20) // per_split_bytes)
        S = 1 if direct else max(1, min(512 // max(1, gy * gz), s_budget, cdiv(P, 32)))
        pps = cdiv(cdiv(P, S), 32) * 32
        S = cdiv(P, pps)
        a.px_per_split = pps
        slab = None if direct else torch.zeros(S, a.Ktiles * 16, NT * 16, dtype=torch.float32, device=dev)
        bslab = torch.zeros(S, NT * 16, dtype=torch.float32, device=dev) if bias else None
        a.slab = direct if direct else slab.data_ptr()
        a.bslab = bslab.data_ptr() if bslab is not None else 0
        self.wgrad_slabs.append((slab, bslab))
        return a, (ktw, ntt, S), slab, bslab

    def _dense_wgrad_args(self, xin, width, dh, Ns, N, bs, bias, direct=None):
        """Dense weight gradient on dense_wgrad_kernel: KG*16 features x NTT*16 outputs per
        workgroup, the batch split into row ranges of >= 128 rows (one 32-row chunk per wave)
        until the launch has ~256 workgroups or the partial slabs reach their byte budget."""
        K, dev = self.ex.K, self.ex.device
        a = K.WgradArgs()
        a.x = xin.data_ptr()
        a.B, a.H, a.W, a.Cs_in = bs, 1, 1, width
        a.Ho, a.Wo = 1, 1
        a.Ktiles = cdiv(width, 16)
        a.dy = dh.data_ptr()
        a.Cs_dy = Ns
        NT = cdiv(N, 16)
        a.NT = NT
        a.P = bs
        # (at most 4 n-tiles: twice the workgroups of 8 -- RPV +0.6 %, MNIST +1.2 %,
        # profiles/r4s_ab_rpv.txt, r4s_ab_mnist.txt)
        ntt = _pow2_le(NT, min(8, tune("dw_ntt", 4)))
        kg = 2
        groups = cdiv(a.Ktiles, kg) * cdiv(NT, ntt)
        per_split_bytes = a.Ktiles * 16 * NT * 16 * 4
        s_budget = max(1, (tune("dw_slab_mb", 8) << 20) // per_split_bytes)
        S = 1 if direct else max(1, min(s_budget, cdiv(tune("dw_min_wgs", 256), groups),
                                        cdiv(bs, 128)))
        pps = cdiv(cdiv(bs, S), 32) * 32
        S = cdiv(bs, pps)
        a.px_per_split = pps
        slab = None if direct else torch.zeros(S, a.Ktiles * 16, NT * 16, dtype=torch.float32, device=dev)
        bslab = torch.zeros(S, NT * 16, dtype=torch.float32, device=dev) if bias else None
        a.slab = direct if direct else slab.data_ptr()
        a.bslab = bslab.data_ptr() if bslab is not None else 0
        self.wgrad_slabs.append((slab, bslab))
        return a, (kg, ntt, S), slab, bslab

    @staticmethod
    def _dense_dx_ntc(a):
        """n-tiles per wave of dense_dx_kernel: the most A-fragment reuse that still leaves
        >= tune dx_min_wgs workgroups (4 waves x 16 rows each)."""
        if tune("dx_ntc", 0):
            return tune("dx_ntc", 0)
        # (256: the RPV dense dX at 2 n-tiles per wave, 256 workgroups -- 3 us faster than
        # 512 one-tile workgroups, profiles/r4p_ab_rpv.txt)
        want = tune("dx_min_wgs", 256)
        for ntc in (4, 2):
            if cdiv(a.M, 64) * cdiv(a.NT, ntc) >= want:
                return ntc
        return 1

