"""LDS layouts of the conv kernels' staged images, chosen by an LDS bank-conflict model.

gfx950 LDS (MI355X_MICROARCH.md §LDS): 64 banks x 4 B; a wave64 access is serviced in
fixed lane groups (``ds_read_b128``: four groups of 16 lanes {0-3,12-15,20-27}, ...;
``ds_read_b64`` / ``ds_read_b64_tr_b16``: two halves of 32), one LDS cycle per group when
its lanes hit distinct banks, +1 cycle per extra distinct address on a bank.  The conv
kernels read MFMA fragments whose lane -> (pixel, channel chunk) map is fixed by the MFMA
operand layout; with dense NHWC images (pixel stride = channel stride, 64 / 128 B for 32 /
64 channels) several lanes of a group land on the same banks -- PMC counted 41-54 % of the
LDS-active cycles of the dual backward launch as bank conflicts (profiles/r2_v13_pmc.txt).

This module replays each kernel's fragment-read address pattern (the same per-lane
formulas the kernels use) and picks, per geometry, the cheapest layout among a few
candidates: a padded pixel stride (``xpix``), a padded image row (``xrow``) and the dY row
stride of the weight-gradient kernel (``dyld``).  The wgrad kernel also permutes which pixel
each MFMA k index stands for (the reduction order is free, both operands use the same
bijection): k = 8g + j <-> pixel 4g + j (j < 4), 16 + 4g + j - 4 (j >= 4), so a 32-lane half
reads 8 consecutive pixels instead of two runs 8 apart.  ``scripts/lds_banks.py`` prints the
model's tables.
"""
from __future__ import annotations

import functools
from typing import Iterable, List, Sequence, Tuple

_B128 = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
         list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32)),
         list(range(32, 36)) + list(range(44, 48)) + list(range(52, 60)),
         list(range(36, 44)) + list(range(48, 52)) + list(range(60, 64))]
_HALVES = [list(range(0, 32)), list(range(32, 64))]
GROUPS = {"b128": (_B128, 16), "b64": (_HALVES, 8), "tr_b64": (_HALVES, 8)}


def cycles(addrs: Sequence[int], kind: str) -> int:
    """LDS cycles of one wave-instruction with per-lane byte addresses ``addrs``."""
    groups, width = GROUPS[kind]
    tot = 0
    for grp in groups:
        per_bank = {}
        for ln in grp:
            w0 = addrs[ln] // 4
            for d in range(width // 4):
                per_bank.setdefault((w0 + d) % 64, set()).add(w0 + d)
        tot += max(len(v) for v in per_bank.values())
    return tot


def wgrad_pixel(g: int, j: int, perm: bool = True) -> int:
    """Pixel (within a 32-pixel k-step) of MFMA k index 8g + j in the weight-gradient kernel
    (wgrad_halo_body.h mma_block; perm=False: the identity, pixel 8g + j)."""
    if not perm:
        return 8 * g + j
    return 4 * g + j if j < 4 else 16 + 4 * g + (j - 4)


def _taps(KH: int, KW: int) -> List[Tuple[int, int]]:
    return [(ky, kx) for ky in range(KH) for kx in range(KW)]


# ------------------------------------------------------------------ access patterns
def wgrad_x_cost(Cs: int, xpix: int, xrow: int, Wo: int, KH: int = 3, KW: int = 3,
                 stride: int = 1, ktiles: int = 3, perm: bool = True) -> float:
    """Average cycles of the X-halo (A operand) transposed reads: lane (i, g) reads 4
    channels (8 B) of pixel P(g, (i >> 2) + 4 * sec) shifted by the tap of its k row group."""
    res = []
    KHW = KH * KW
    for mt in range(ktiles):
        for sec in (0, 1):
            addrs = []
            for ln in range(64):
                i, g = ln & 15, ln >> 4
                P = wgrad_pixel(g, (i >> 2) + 4 * sec, perm)
                k = mt * 16 + 4 * (i & 3)
                tap = min(k // Cs, KHW - 1)
                ky, kx = tap // KW, tap % KW
                c = k - (k // Cs) * Cs if k // Cs < KHW else 0
                y, x = P // Wo, P % Wo
                q = (y * stride + ky) * xrow + x * stride + kx
                addrs.append((q * xpix + c) * 2)
            res.append(cycles(addrs, "tr_b64"))
    return sum(res) / len(res)


def wgrad_dy_cost(ntt: int, dyld: int, perm: bool = True) -> float:
    """Average cycles of the dY-row (B operand) transposed reads of n-tile 0."""
    res = []
    for sec in (0, 1):
        addrs = []
        for ln in range(64):
            i, g = ln & 15, ln >> 4
            P = wgrad_pixel(g, (i >> 2) + 4 * sec, perm)
            addrs.append((P * dyld + 4 * (i & 3)) * 2)
        res.append(cycles(addrs, "tr_b64"))
    return sum(res) / len(res)


def conv_a_cost(Cs: int, xpix: int, xrow: int, Wo: int, pool: bool, KH: int = 3, KW: int = 3) -> float:
    """Average cycles of the implicit-GEMM A-fragment reads of conv_halo_body (fwd / dgrad):
    lane (r, g) reads the 8-channel chunk g of the k-step's tap of its pixel (16 consecutive
    output pixels, or 4 pooling windows x 2 x 2 when pooled): ds_read_b128."""
    res = []
    nch = max(1, Cs // 8)
    for (ky, kx) in _taps(KH, KW)[:4]:
        for x0 in (0, 16):
            if x0 + 16 > Wo:
                continue
            addrs = []
            for ln in range(64):
                r, g = ln & 15, ln >> 4
                if pool:
                    dy, dx = (r >> 1) & 1, r & 1
                    y, x = dy, x0 // 2 * 2 + 2 * (r >> 2) + dx
                else:
                    y, x = 0, x0 + r
                q = (y + ky) * xrow + x + kx
                addrs.append((q * xpix + 8 * (g % nch)) * 2)
            res.append(cycles(addrs, "b128"))
    return sum(res) / max(1, len(res))


# ------------------------------------------------------------------ pickers
def _cands(base: int, pads: Iterable[int]) -> List[int]:
    return sorted({base + p for p in pads})


@functools.lru_cache(maxsize=256)
def wgrad_layout(Cs: int, W_in: int, Wo: int, ntt: int, KH: int = 3, KW: int = 3, stride: int = 1,
                 ktiles: int = 3, perm: bool = True) -> Tuple[int, int, int]:
    """(xpix, xrow, dyld) for wgrad_halo_body: the X-halo pixel / row strides and the dY row
    stride with the fewest modelled LDS cycles (ties: the smallest footprint)."""
    best = None
    for xpix in _cands(Cs, (0, 8, 16) if Cs >= 8 else (0, 4)):
        if (xpix * 2) % 8:
            continue                   # 8-byte aligned pixels (transposed 8-byte reads)
        for xrow in range(W_in, W_in + 17):
            c = wgrad_x_cost(Cs, xpix, xrow, Wo, KH, KW, stride, ktiles, perm)
            key = (c, xpix * xrow)
            if best is None or key < best[0]:
                best = (key, xpix, xrow)
    dbest = None
    for dyld in _cands(ntt * 16, (0, 8, 16, 24)):
        c = wgrad_dy_cost(ntt, dyld, perm)
        if dbest is None or (c, dyld) < dbest[0]:
            dbest = ((c, dyld), dyld)
    return best[1], best[2], dbest[1]


@functools.lru_cache(maxsize=256)
def conv_layout(Cs: int, W_in: int, Wo: int, pool: bool, KH: int = 3, KW: int = 3) -> int:
    """Pixel stride (elements) of conv_halo_body's input halo image (row stride = W_in)."""
    if Cs < 8:
        return Cs
    best = None
    for xpix in _cands(Cs, (0, 8, 16)):
        c = conv_a_cost(Cs, xpix, W_in, Wo, pool, KH, KW)
        if best is None or (c, xpix) < best[0]:
            best = ((c, xpix), xpix)
    return best[1]


def stack_cs4_cost(xrow: int, Wo: int, pool: bool, KS: int = 2, KW: int = 3) -> float:
    """First stack layer (4-channel pixels, 8 B): an A fragment is two ds_read_b64, taps
    t0 = 8 ks + 2g and t0 + 1 of the lane's pixel (pooled tile: 4 windows x 2 x 2)."""
    res = []
    for ks in range(KS):
        for x0 in (0, 8):
            for second in (0, 1):
                addrs = []
                for ln in range(64):
                    r, g = ln & 15, ln >> 4
                    if pool:
                        y, x = (r >> 1) & 1, x0 + 2 * (r >> 2) + (r & 1)
                    else:
                        y, x = 0, x0 + r
                    t = 8 * ks + 2 * g + second
                    off = (t // KW) * xrow + t % KW if t < 9 else 0
                    addrs.append(((y * xrow + x) + off) * 4 * 2)
                res.append(cycles(addrs, "b64"))
    return sum(res) / len(res)


@functools.lru_cache(maxsize=256)
def stack_layout(Cs: int, W_in: int, Wo: int, pool: bool, KS: int = 2) -> Tuple[int, int]:
    """(xpix, xrow) of a conv-stack layer's input halo image (conv_stack.hip): fewest modelled
    LDS cycles of its fragment reads, ties to the smallest footprint."""
    best = None
    for xpix in ((4,) if Cs == 4 else _cands(Cs, (0, 8, 16))):
        for xrow in range(W_in, W_in + 17):
            c = (stack_cs4_cost(xrow, Wo, pool, KS) if Cs == 4 else conv_a_cost(Cs, xpix, xrow, Wo, pool))
            key = (c, xpix * xrow)
            if best is None or key < best[0]:
                best = (key, xpix, xrow)
    return best[1], best[2]
