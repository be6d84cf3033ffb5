"""Standalone numerics check of dense_bwd.hip's dense_wgrad kernel against torch fp32:
slab[s] summed over splits vs X^T dH, bias slab vs column sums of dH, over a sweep of
(rows, width, N, KG, NTT, splits).  GPU only.

    python scripts/dense_bwd_check.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cori_intml_examples_amd.ops.hip import kernels as load_kernels  # noqa: E402


def cdiv(a, b):
    return (a + b - 1) // b


def check(M, width, N, kg, ntt, S, dev):
    K = load_kernels()
    torch.manual_seed(M * 7 + width + N)
    Ns = cdiv(N, 8) * 8
    x = torch.randn(M, width, device=dev).to(torch.bfloat16)
    dh = torch.zeros(M, Ns, device=dev, dtype=torch.bfloat16)
    dh[:, :N] = torch.randn(M, N, device=dev).to(torch.bfloat16)
    NT = cdiv(N, 16)
    Ktiles = cdiv(width, 16)
    pps = cdiv(cdiv(M, S), 32) * 32
    S = cdiv(M, pps)
    slab = torch.full((S, Ktiles * 16, NT * 16), float("nan"), device=dev)
    bslab = torch.full((S, NT * 16), float("nan"), device=dev)
    a = K.WgradArgs()
    a.x, a.B, a.H, a.W, a.Cs_in = x.data_ptr(), M, 1, 1, width
    a.Ho, a.Wo = 1, 1
    a.Ktiles, a.dy, a.Cs_dy, a.NT, a.P = Ktiles, dh.data_ptr(), Ns, NT, M
    a.px_per_split = pps
    a.slab, a.bslab = slab.data_ptr(), bslab.data_ptr()
    K.dense_wgrad(a, kg, ntt, S, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ref = x.float().t() @ dh.float()[:, :N]
    got = slab.sum(0)[:width, :N]
    bref = dh.float()[:, :N].sum(0)
    bgot = bslab.sum(0)[:N]
    e = ((got - ref).abs().max() / ref.abs().max()).item()
    eb = ((bgot - bref).abs().max() / bref.abs().max()).item()
    bad = (got - ref).abs() > 1e-2 * ref.abs().max()
    where = ""
    if bad.any():
        rows = bad.any(1).nonzero().flatten().tolist()
        cols = bad.any(0).nonzero().flatten().tolist()
        where = " bad rows %s.. (%d) cols %s.. (%d)" % (rows[:8], len(rows), cols[:8], len(cols))
    ok = e < 1e-3 and eb < 1e-3
    print("M=%5d width=%5d N=%4d kg=%d ntt=%d S=%d  wgrad %.2e  bias %.2e  %s%s" %
          (M, width, N, kg, ntt, S, e, eb, "ok" if ok else "FAIL", where), flush=True)
    return ok


def probe(kg, ntt, dev, dbg=0):
    """X = I (32 rows x 16 features): slab[f][n] = dH[f][n]; dH = row id, then column id."""
    K = load_kernels()
    M, width, N = 32, 16, ntt * 16
    x = torch.eye(M, width, device=dev).to(torch.bfloat16)
    for name, dh in (("row", torch.arange(M, device=dev)[:, None].expand(M, N)),
                     ("col", torch.arange(N, device=dev)[None, :].expand(M, N))):
        dh = dh.float().to(torch.bfloat16).contiguous()
        slab = torch.full((1, 16 * kg if kg == 1 else 16, N), float("nan"), device=dev)
        slab = torch.full((1, 16, N), float("nan"), device=dev)
        a = K.WgradArgs()
        a.x, a.B, a.H, a.W, a.Cs_in = x.data_ptr(), M, 1, 1, width
        a.Ho, a.Wo = 1, 1
        a.Ktiles, a.dy, a.Cs_dy, a.NT, a.P = 1, dh.data_ptr(), N, ntt, M
        a.px_per_split = 32
        a.slab, a.bslab = slab.data_ptr(), 0
        a.dbg = dbg
        K.dense_wgrad(a, kg, ntt, 1, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        got = slab[0].cpu()
        want = dh.float()[:16].cpu()
        bad = (got != want)
        print("probe kg=%d ntt=%d dbg=%d dH=%s: %d / %d wrong" % (kg, ntt, dbg, name, bad.sum().item(), got.numel()))
        if bad.any():
            idx = bad.nonzero()[:12].tolist()
            print("   ", [(r, c, got[r, c].item(), want[r, c].item()) for r, c in idx])


def main():
    dev = torch.device("cuda", 0)
    if len(sys.argv) > 1 and sys.argv[1] == "probe":
        for dbg in (0, 1, 2, 3):
            for kg, ntt in ((2, 8), (2, 2)):
                probe(kg, ntt, dev, dbg)
        return
    ok = True
    for (M, width, N) in [(40, 256, 128), (128, 4096, 128), (64, 96, 24), (1024, 4096, 128), (200, 512, 40)]:
        for kg in (2,):
            ntt = min(8, 1 << (cdiv(N, 16).bit_length() - 1))
            for S in (1, 2):
                ok &= check(M, width, N, kg, ntt, S, dev)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
