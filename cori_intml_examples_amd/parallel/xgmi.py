"""Fused data-parallel gradient all-reduce + optimizer over xGMI peer memory.

SURVEY.md §5.1 item 3 (the small-bucket latency path) and N7 (comm): for a fused gradient
bucket of a few MB -- the RPV model's whole 2.2 MB gradient -- one kernel on the training
stream does a two-shot all-reduce by direct stores into the peers' IPC-mapped uncached
device memory (xGMI links are point-to-point: every rank talks to every other rank at
once) and applies the Keras update to the reduced gradient in its final pass
(``csrc/kernels/xgmi.hip``).  Compared to RCCL + a separate optimizer launch this keeps the
step ONE linear HIP graph and removes a launch; each rank moves 2 x (P-1)/P of the
gradient over its links.

Reference call site it replaces: Horovod's fused gradient all-reduce behind
``hvd.DistributedOptimizer`` (``rpv.py:63-65``).

Safety: setup (uncached allocation, IPC handle exchange over the gloo control plane,
mapping) and a numeric self-test against closed-form sums run at construction; every rank
votes and the path is used only if ALL ranks pass (else the caller keeps RCCL).  Every
in-kernel wait is bounded in time (``timeout_s``: min(INTML_DP_TIMEOUT, 120) s by default)
and reports through an error word (``check()``), never a hang; a rank that gives up raises
a sticky abort word on every rank, so no later launch anywhere can pair this step's flags
with another step's data (every later launch exits at once and the host raises).

A bucket is any flat range [lo, hi) of the gradient: ``launch(grad_ptr, ..)`` takes the
bucket's first element and the optimizer arguments are offset to it (``offset_optim``).
"""
from __future__ import annotations

import os
from typing import Callable, List, Optional

import torch

from ..ops.hip import kernels
from ..utils.env import tune

_FLAG_WORDS = 256 * 8          # XGMI_MAX_WG x XGMI_MAX_RANKS
XCHG_MAX_BLOCKS = 4096         # early-bucket exchange: table blocks with flags (x XGMI_MAX_RANKS)
_TICKS_PER_S = 100_000_000     # wall_clock64 (s_memrealtime) runs at 100 MHz on gfx950


def default_timeout_s() -> float:
    return min(float(os.environ.get("INTML_DP_TIMEOUT", 600)), 120.0)


def offset_optim(opt, lo: int):
    """OptimArgs whose parameter / slot pointers start at flat element ``lo`` (a bucket);
    ``opt.lo`` records that start (the kernel's pack routes are in absolute elements)."""
    opt.lo = lo
    if lo:
        for f in ("p", "s0", "s1"):
            v = getattr(opt, f)
            if v:
                setattr(opt, f, v + 4 * lo)
    return opt


def _align(x: int, a: int) -> int:
    return (x + a - 1) // a * a


def geometry(n: int, size: int, max_wg: int = 256):
    """(chunk, sub, grid): owner chunk and per-workgroup slice lengths (multiples of 4) for
    an n-element gradient over `size` ranks; ~1024 elements (one float4 per thread) per
    workgroup slice, at most max_wg workgroups."""
    chunk = _align(max(1, -(-n // size)), 4)
    grid = max(1, min(max_wg, -(-chunk // 1024)))
    sub = _align(-(-chunk // grid), 4)
    grid = -(-chunk // sub)
    return chunk, sub, grid


class XgmiAllreduce:
    """One communicator-like object per (process group, gradient size).  Collective:
    every rank must construct it, in the same order."""

    def __init__(self, rank: int, size: int, n: int, device: torch.device,
                 allgather: Callable[[object], List[object]], timeout_s: Optional[float] = None,
                 max_wg: Optional[int] = None):
        K = kernels()
        self.K, self.rank, self.size, self.n, self.device = K, rank, size, n, device
        if size > K.XGMI_MAX_RANKS:
            raise ValueError("xgmi all-reduce supports at most %d ranks" % K.XGMI_MAX_RANKS)
        self.chunk, self.sub, self.grid = geometry(n, size, min(max_wg or K.XGMI_MAX_WG, K.XGMI_MAX_WG))
        words = self.chunk * size
        # layout (bytes): flag1 | flag2 | abort word | block flags 1 | block flags 2 (the early
        # bucket's exchange, XgmiPush) | inbox [P][chunk] fp32 | outbox [P*chunk] fp32
        self.off_f1, self.off_f2 = 0, 4 * _FLAG_WORDS
        self.off_ab = self.off_f2 + 4 * _FLAG_WORDS
        self.off_bf1 = _align(self.off_ab + 256, 256)
        self.off_bf2 = self.off_bf1 + 4 * XCHG_MAX_BLOCKS * 8
        self.off_in = _align(self.off_bf2 + 4 * XCHG_MAX_BLOCKS * 8, 256)
        self.off_out = _align(self.off_in + 4 * words, 256)
        self.nbytes = _align(self.off_out + 4 * words, 4096)
        self.buf = 0
        self._opened: List[int] = []
        err = None
        torch.cuda.set_device(device)
        try:
            self.buf = K.xgmi_alloc_uncached(self.nbytes, tune("xgmi_mem", "uncached") == "finegrained")
            handle = K.xgmi_ipc_handle(self.buf)
        except Exception as e:        # noqa: BLE001 -- reported through the vote below
            err, handle = "setup: %s" % e, b""
        handles = allgather(handle)
        bases = []
        if err is None:
            try:
                for j, h in enumerate(handles):
                    if j == rank:
                        bases.append(self.buf)
                    elif not h:
                        raise RuntimeError("rank %d has no IPC handle" % j)
                    else:
                        p = K.xgmi_ipc_open(h)
                        self._opened.append(p)
                        bases.append(p)
            except Exception as e:    # noqa: BLE001
                err = "ipc: %s" % e
        self.ctr = torch.zeros(K.XGMI_MAX_WG, dtype=torch.int32, device=device)
        self.ctrb = torch.zeros(XCHG_MAX_BLOCKS, dtype=torch.int32, device=device)   # exchange blocks
        self.shared = False            # ranks share a GPU (set by the reducer): looping exchange WGs
        self.err = torch.zeros(4, dtype=torch.int32, device=device)   # code, seq, seen, wg*64+peer
        a = K.XgmiArgs()
        a.rank, a.size, a.n, a.chunk, a.sub = rank, size, n, self.chunk, self.sub
        self.timeout_s = float(timeout_s or default_timeout_s())
        a.timeout_ticks = int(self.timeout_s * _TICKS_PER_S)
        a.ctr, a.err = self.ctr.data_ptr(), self.err.data_ptr()
        # 1 (default): system-scope release + acquire around every flag (the HIP memory model;
        # the fence-free form 3 -- sc1 payload loads only -- stays opt-in until a
        # multi-GPU run shows parity); 2: agent-scope acquire; 0: none (xgmi.hip header)
        a.fence = int(tune("xgmi_fence", 1))
        if err is None:
            for j, b in enumerate(bases):
                a.set_peer(j, b + self.off_in, b + self.off_out, b + self.off_f1, b + self.off_f2, b + self.off_ab)
        self.bases = bases if err is None else []
        self.args = a
        self.setup_error = err

    # ------------------------------------------------------------------ launches
    def push_args(self, lo: int = 0, mode: int = 1, nblk: int = 0, fbase: int = 0, blocks=None):
        """XgmiPush for the kernels that finalise part of this all-reduce's bucket inside the
        backward (the early head / dense reduction).  mode 1: they store each reduced element
        straight into its owner's inbox row -- phase 1 of the all-reduce, overlapping the rest
        of the backward; with ``nblk`` (the table's blocks) they also raise per-block flags for
        an exchange.  mode 2 (the exchange, a later backward launch): the owners sum the rows
        and send the sums back, and every rank applies the update -- the range's whole
        all-reduce + optimizer inside the backward (args.h XgmiPush); mode 3: both in one
        launch (the end-of-backward bucket's table).  ``lo``: the bucket's first flat element;
        ``fbase``: the table's first block-flag slot (tables of one step use disjoint slots);
        mode 4 / 5 (the split exchange): the owner half of mode 2 in a backward launch over the
        table ``blocks`` = (b_lo, b_hi) this rank owns part of, and the finish half (waits for
        the other owners + update) in the end-of-backward launch.  None past the flag capacity, or at size 1 without an exchange
        (nothing to push; at size 1 the exchange is the range's update in the later launch --
        the same structure, no peer traffic)."""
        if not self.bases or fbase + nblk > XCHG_MAX_BLOCKS or (self.size < 2 and not nblk):
            return None
        fo = 4 * fbase * self.size             # byte offset of the table's flag rows
        x = self.K.XgmiPush()
        x.on, x.rank, x.size, x.chunk, x.lo = 1, self.rank, self.size, self.chunk, int(lo)
        x.mode = mode
        for j, b in enumerate(self.bases):
            if nblk:
                x.set_peer(j, b + self.off_in, b + self.off_out, b + self.off_bf1 + fo, b + self.off_bf2 + fo,
                           b + self.off_ab)
            else:
                x.set_inbox(j, b + self.off_in)
        if nblk:
            x.nblk, x.ctrb, x.err = nblk, self.ctrb.data_ptr() + 4 * fbase, self.err.data_ptr()
            x.timeout_ticks = self.args.timeout_ticks
            # ranks sharing a GPU: a few workgroups looping over the blocks (one per block would
            # let one rank's spinning workgroups fill the CUs its peers' launches need);
            # xchg_nx (A/B): as many looping workgroups on separate GPUs too
            x.nx = int(tune("xgmi_xchg_wg", 4)) if self.shared else int(tune("xchg_nx", 0))
            x.nx = x.nx if mode >= 2 else 0
            if mode == 4:
                x.b_lo, x.b_hi = blocks if blocks is not None else (0, nblk)
                if x.nx:
                    x.nx = min(x.nx, max(1, x.b_hi - x.b_lo))
            x.p1 = int(tune("xchg_p1", False))
            x.fence = 3 if self.args.fence == 3 else 1    # the exchange: release/acquire or none
        return x

    def launch(self, grad: int, stream: int, opt=None, skip=(0, 0), exchanged: bool = False) -> None:
        """Enqueue the fused all-reduce on `stream` (capturable): the reduced SUM lands in
        `grad`; with `opt` (OptimArgs, grad_scale = 1/size) the Keras update follows.
        ``skip``: bucket-relative element range already pushed by the backward (push_args);
        ``exchanged``: ... and also all-reduced and updated there (mode-2 exchange)."""
        a = self.args
        a.skip_lo, a.skip_hi = int(skip[0]), int(skip[1])
        a.skip_mode = 2 if exchanged else 0
        a.grad = grad
        if opt is not None:
            a.mode, a.opt = 1, opt
        else:
            a.mode = 0
        self.K.xgmi_allreduce(a, stream)

    def check(self) -> None:
        """Raise if a wait in an earlier launch timed out (a peer died or hung)."""
        e = self.err.tolist()
        if e[0]:
            raise RuntimeError(describe_error(*e))

    def _skew(self, it: int) -> None:
        """A rank-dependent device-side busy delay before launch ``it`` of a stressed self-test
        (0-40 us, different on every rank and launch): back-to-back launches then meet their
        peers out of phase, so a flag seen before its payload -- an ordering bug -- shows up
        as a wrong sum instead of hiding behind lockstep timing."""
        cyc = ((it * 7 + self.rank * 13) % 5) * 20000
        if cyc:
            try:
                torch.cuda._sleep(cyc)
            except Exception:         # noqa: BLE001 -- (no delay kernel: unskewed)
                pass

    def selftest(self, stress: Optional[int] = None) -> Optional[str]:
        """Closed-form data (exact in fp32) through the two-shot kernel and the exchange
        protocol; None if correct on this rank.  Two synchronised launches, then ``stress``
        (default: up to 64, bounded to 256 MB of buffers) back-to-back launches on distinct
        buffers with rank-dependent busy delays in front of each (``_skew``), every result
        checked after one synchronisation."""
        if self.setup_error:
            return self.setup_error
        n, P, r = self.n, self.size, self.rank
        idx = torch.arange(n, device=self.device, dtype=torch.float32)
        pat = torch.remainder(idx, 97.0) * 0.25
        stream = torch.cuda.current_stream(self.device).cuda_stream
        for it in range(2):
            g = pat * float(r + 1 + it)
            self.launch(g.data_ptr(), stream)
            torch.cuda.synchronize(self.device)
            if int(self.err[0].item()):
                return "selftest: " + describe_error(*self.err.tolist())
            want = pat * float(sum(q + 1 + it for q in range(P)))
            if not torch.equal(g, want):
                bad = int((g != want).sum())
                return "selftest: %d of %d elements wrong" % (bad, n)
        if stress is None:
            stress = int(tune("xgmi_selftest_stress", 64))
        k = max(0, min(int(stress), (256 << 20) // max(1, 4 * n)))
        if k:
            gs = []
            for it in range(k):
                g = pat * float(r + 1 + (it % 11))
                self._skew(it)
                self.launch(g.data_ptr(), stream)
                gs.append(g)
            torch.cuda.synchronize(self.device)
            if int(self.err[0].item()):
                return "stressed selftest: " + describe_error(*self.err.tolist())
            for it, g in enumerate(gs):
                want = pat * float(sum(q + 1 + (it % 11) for q in range(P)))
                if not torch.equal(g, want):
                    return "stressed selftest: launch %d of %d: %d of %d elements wrong" % (
                        it, k, int((g != want).sum()), n)
            del gs
        return self._xchg_selftest(stress=min(k, 16))

    def _xchg_selftest(self, stress: int = 0) -> Optional[str]:
        """The exchange protocol the training step uses (XgmiPush mode 3: per-block flags,
        owner sums pushed back through the outboxes) on a closed-form table -- a float4 and a
        split-lane descriptor over a window straddling the first owner boundary -- as mode 3 (one
        launch) and as the split exchange (modes 1 -> 4 -> 5, three launches), twice each (the
        block sequence numbers advance), then ``stress`` more launches back to back alternating
        the two, with rank-dependent delays (``_skew``); every rank must read back the exact sums.  The
        geometry is training's (one workgroup per block on separate GPUs, looping workgroups
        when ranks share one: ``shared``).  Uses the top block-flag slots, which no training
        table reaches."""
        K, P, r, dev = self.K, self.size, self.rank, self.device
        lo = max(0, min(self.n, self.chunk) - 2048) // 4 * 4
        hi = min(self.n, lo + 4096) // 4 * 4
        nv = (hi - lo) // 64 * 64                        # float4 descriptor: Cout 16 x Cin rows
        nb = min(hi - lo - nv, 256)                      # split-lane descriptor
        if nv < 64:
            return None                                  # (a bucket too small to matter)
        S, tpe = 4, 2
        stream = torch.cuda.current_stream(self.device).cuda_stream
        st = torch.zeros(K.STEP_STATE_BYTES, dtype=torch.uint8, device=dev)   # lr 0: the update is a no-op
        p = torch.zeros(self.n, dtype=torch.float32, device=dev)
        ramp = lambda m: torch.remainder(torch.arange(m, device=dev, dtype=torch.float32), 7.0) * 0.25
        def launch(it, split=False):
            f = float(r + 1 + it)
            sv = torch.stack([ramp(nv) * f * (s + 1) for s in range(S)])
            sb = torch.stack([ramp(max(nb, 1)) * f * (s + 1) for s in range(S)])
            tab = K.RedTable()
            tab.add(sv.data_ptr(), nv, S, 16, lo, nv, 2, 1, 1, nv // 16, 16, nv // 16, -1)   # RED_FLATW, float4
            if nb:
                tab.add(sb.data_ptr(), max(nb, 1), S, nb, lo + nv, nb, 1, 1, 1, 1, nb, nb, tpe)   # RED_BIAS
            a = K.OptimArgs()
            a.p, a.n, a.st, a.kind = p.data_ptr(), self.n, st.data_ptr(), 0
            g = torch.zeros(self.n, dtype=torch.float32, device=dev)
            if split:
                # the split exchange the training step runs: mode 1 (reduce + push, a grad-only
                # table), mode 4 (owner half, the blocks this rank owns part of), mode 5 (finish
                # half) -- three launches, in the flag slots below mode 3's
                fb = XCHG_MAX_BLOCKS - 2 * tab.nblocks
                own = tuple(tab.owned_blocks(0, self.chunk, r)) if P > 1 else (0, 0)
                x1 = self.push_args(0, mode=1, nblk=tab.nblocks, fbase=fb)
                x4 = self.push_args(0, mode=4, nblk=tab.nblocks, fbase=fb, blocks=own)
                x5 = self.push_args(0, mode=5, nblk=tab.nblocks, fbase=fb)
                if x1 is None or x4 is None or x5 is None:
                    return None
                a.grad_only = 1
                K.reduce_optim(g.data_ptr(), tab, a, stream, x1)
                a.grad_only = 0
                K.reduce_optim(g.data_ptr(), tab, a, stream, x4)
                K.reduce_optim(g.data_ptr(), tab, a, stream, x5)
                return g, (sv, sb)
            xp = self.push_args(0, mode=3, nblk=tab.nblocks, fbase=XCHG_MAX_BLOCKS - tab.nblocks)
            if xp is None:
                return None
            K.reduce_optim(g.data_ptr(), tab, a, stream, xp)
            return g, (sv, sb)            # (the slabs stay alive until the check)

        def check(g, it, what):
            k = sum(q + 1 + it for q in range(P)) * S * (S + 1) / 2
            want = torch.cat([ramp(nv), ramp(nb)[:nb]]) * k
            if not torch.equal(g[lo:lo + nv + nb], want):
                bad = int((g[lo:lo + nv + nb] != want).sum())
                return "%s: %d of %d elements wrong" % (what, bad, nv + nb)
            return None

        for it in range(4):
            out = launch(it, split=it >= 2)
            if out is None:
                return "exchange selftest: no flag slots"
            torch.cuda.synchronize(self.device)
            if int(self.err[0].item()):
                return "exchange selftest: " + describe_error(*self.err.tolist())
            why = check(out[0], it, "exchange selftest")
            if why:
                return why
        outs = []
        for it in range(4, 4 + stress):
            self._skew(it)
            outs.append(launch(it, split=bool(it & 1)))
        if outs:
            torch.cuda.synchronize(self.device)
            if int(self.err[0].item()):
                return "stressed exchange selftest: " + describe_error(*self.err.tolist())
            for it, out in enumerate(outs, start=4):
                why = check(out[0], it, "stressed exchange selftest (launch %d)" % it)
                if why:
                    return why
        return None

    def close(self) -> None:
        torch.cuda.synchronize(self.device)
        for p in self._opened:
            try:
                self.K.xgmi_ipc_close(p)
            except Exception:         # noqa: BLE001
                pass
        self._opened = []
        if self.buf:
            self.K.xgmi_free(self.buf)
            self.buf = 0


def describe_error(e: int, seq: int = 0, seen: int = 0, where: int = 0) -> str:
    if e == 3:
        return "xgmi all-reduce: aborted (a peer rank timed out waiting; peer dead or hung)"
    return ("xgmi all-reduce: phase-%d wait timed out (peer rank dead or hung): workgroup %d waited for "
            "rank %d's flag to reach %d, saw %d" % (e, where // 64, where % 64, seq, seen))


def create(rank: int, size: int, n: int, device: torch.device, allgather,
           timeout_s: Optional[float] = None, max_wg: Optional[int] = None,
           shared: bool = False) -> Optional[XgmiAllreduce]:
    """Build + self-test collectively; returns the object only if EVERY rank passed both
    the setup and the (stressed) self-test (same decision on every rank: the votes are
    gathered).  ``shared``: the ranks share a GPU -- set BEFORE the self-test, so it runs the
    exchange geometry (looping workgroups) that training will use."""
    x, why = None, None
    try:
        x = XgmiAllreduce(rank, size, n, device, allgather, timeout_s=timeout_s, max_wg=max_wg)
        x.shared = bool(shared)
        why = x.setup_error
    except Exception as e:            # noqa: BLE001
        why = "error: %s" % e
    bad = [(i, v) for i, v in enumerate(allgather(why)) if v]
    if not bad:
        limit = x.args.timeout_ticks
        x.args.timeout_ticks = min(limit, 5 * _TICKS_PER_S)    # a broken path fails the test fast
        try:
            why = x.selftest()
        except Exception as e:        # noqa: BLE001
            why = "selftest error: %s" % e
        x.args.timeout_ticks = limit
        bad = [(i, v) for i, v in enumerate(allgather(why)) if v]
    if bad:
        if x is not None:
            try:
                x.close()
            except Exception:         # noqa: BLE001
                pass
        if rank == 0:
            import sys
            print("[xgmi] fused all-reduce disabled, using RCCL: %s" % bad, file=sys.stderr, flush=True)
        return None
    return x
