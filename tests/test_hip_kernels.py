"""Per-kernel numerics: every HIP kernel of a captured training step is checked against
a plain fp32 PyTorch reference computed FROM THE SAME bf16 INPUTS the kernel saw (the
step's saved activations, codes and gradients), so bf16 rounding of upstream values does
not blur the comparison.
"""
import numpy as np
import pytest
import torch

from cori_intml_examples_amd.ops import reference as R
from cori_intml_examples_amd.ops.rng import dropout_keep
from cori_intml_examples_amd.utils import set_random_seed

from test_hip_model import _build, _data

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-12)


def _step(kind, drop, cin, hw=16, n=40, opt="SGD"):
    set_random_seed(99)
    m = _build(kind, "cuda", opt=opt, drop=drop, cin=cin, hw=hw)
    ex = m._executor
    x, y = _data(m, n, seed=4)
    d = ex.upload(x, y)
    w_before = m.store.master.clone()
    ex.train_step(d, torch.arange(n, device=ex.device), 0, n)
    torch.cuda.synchronize()
    bp = ex._plans[(n, "train")]
    return m, ex, bp, w_before


def _f(t):
    return t.detach().float().cpu()


def _w(m, w_before, layer, short):
    s = m.store.spec(layer, short)
    return w_before[s.offset:s.offset + s.numel].view(s.shape).cpu()


def _bf(t):
    return t.to(torch.bfloat16).float()


def _mask(numel, rate, seed, stream, step):
    return dropout_keep(numel, rate, seed, stream, step).float() / (1.0 - rate)


def _full_dy(bp, g):
    """Full-resolution dY of conv stage g, rebuilt from the saved pooled dP + codes
    (what the kernels do on load)."""
    dp = _f(bp.conv_dy[g.i])[..., :g.Cout]
    if not g.pool:
        return dp
    code = bp.conv_code[g.i].cpu()[..., :g.Cout]
    return R.maxpool2x2_backward(dp, code, (g.Ho, g.Wo))


CASES = [("rpv", 0.0, 1), ("rpv", 0.3, 3), ("mnist", 0.4, 1), ("odd", 0.25, 2), ("strided", 0.0, 3),
         ("wide", 0.2, 3), ("wide_strided", 0.0, 3)]
# The benchmarked geometries at the benchmarked batch (bench.py --model rpv / mnist / rpv_legacy):
# RPV 64x64x3 B=128 takes the 2-band conv_stack split and the pipelined 256-px wgrad_halo
# blocks; MNIST 28x28x1 conv 32-64; the legacy widths 64-128(s2)-256-256(s2) with the
# K = 65,536 split-K dense.  (kind, drop, cin, hw, n)
BENCH_CASES = [("rpv_bench", 0.2, 3, 64, 128), ("mnist_bench", 0.4, 1, 28, 128), ("legacy", 0.0, 1, 64, 128)]
ALL = [c + (16, 40) for c in CASES] + BENCH_CASES


@pytest.mark.parametrize("kind,drop,cin,hw,n", ALL)
def test_conv_forward(kind, drop, cin, hw, n):
    m, ex, bp, wb = _step(kind, drop, cin, hw, n)
    step = int(ex._st_i32[0].item())
    x = _f(bp.step_inputs()[0]).view(bp.bs, ex.in_H, ex.in_W, ex.in_Cs)[..., :ex.in_C]
    for g, cs in zip(ex.convs, ex.plan.convs):
        w = _bf(_w(m, wb, cs.conv, "kernel"))
        b = _w(m, wb, cs.conv, "bias")
        z = R.conv2d(x, w, b, cs.stride, cs.conv.padding)
        r = torch.relu(z) if g.relu else z
        if g.pool:
            r, code = R.maxpool2x2(r)
        if g.rate > 0:
            r = r * _mask(r.numel(), g.rate, ex.seed, g.stream, step).view(r.shape)
        got = _f(bp.conv_out[g.i])
        assert _rel(got[..., :g.Cout], r) < 1e-2, "conv %d fwd" % g.i
        assert float(got[..., g.Cout:].abs().max() if g.Cs_out > g.Cout else 0) == 0.0
        x = got[..., :g.Cout]


@pytest.mark.parametrize("kind,drop,cin,hw,n", ALL)
def test_conv_wgrad_and_bias(kind, drop, cin, hw, n):
    m, ex, bp, wb = _step(kind, drop, cin, hw, n)
    for g, cs in zip(ex.convs, ex.plan.convs):
        if g.i == 0:
            x = _f(bp.step_inputs()[0]).view(bp.bs, ex.in_H, ex.in_W, ex.in_Cs)[..., :ex.in_C]
        else:
            pg = ex.convs[g.i - 1]
            x = _f(bp.conv_out[g.i - 1])[..., :pg.Cout]
        dy = _full_dy(bp, g)
        w = _w(m, wb, cs.conv, "kernel")
        _, dw, db = R.conv2d_backward(x, w, dy, cs.stride, cs.conv.padding, need_dx=False)
        gw = m.store.view(cs.conv, "kernel", grad=True).cpu()
        gb = m.store.view(cs.conv, "bias", grad=True).cpu()
        assert _rel(gw, dw) < 5e-3, "conv %d wgrad %.3g" % (g.i, _rel(gw, dw))
        assert _rel(gb, db) < 5e-3, "conv %d bias grad" % g.i


@pytest.mark.parametrize("kind,drop,cin,hw,n", ALL)
def test_conv_dgrad_bwd_through(kind, drop, cin, hw, n):
    m, ex, bp, wb = _step(kind, drop, cin, hw, n)
    step = int(ex._st_i32[0].item())
    for g, cs in zip(ex.convs, ex.plan.convs):
        if g.i == 0:
            continue
        pg = ex.convs[g.i - 1]
        dy = _full_dy(bp, g)
        w = _bf(_w(m, wb, cs.conv, "kernel"))
        xin = _f(bp.conv_out[g.i - 1])[..., :pg.Cout]
        dx, _, _ = R.conv2d_backward(xin, w, dy, cs.stride, cs.conv.padding)
        if pg.rate > 0:
            dx = dx * _mask(dx.numel(), pg.rate, ex.seed, pg.stream, step).view(dx.shape)
        if pg.relu:
            dx = dx * (xin > 0).float()
        got = _f(bp.conv_dy[pg.i])[..., :pg.Cout]    # pooled-resolution dP of the prev stage
        assert _rel(got, dx) < 1e-2, "dgrad into conv %d: %.3g" % (pg.i, _rel(got, dx))


@pytest.mark.parametrize("kind,drop,cin,hw,n", ALL)
def test_dense_and_head(kind, drop, cin, hw, n, monkeypatch):
    # (the legacy Dense(512) applies its update inside its wgrad kernel and by default does not
    # store the gradient it consumed: keep it here so the gradient can be checked)
    monkeypatch.setenv("INTML_TUNE", "opt_nograd=0")
    m, ex, bp, wb = _step(kind, drop, cin, hw, n)
    step = int(ex._st_i32[0].item())

    def src_val(src):
        if src.kind == "input":
            return _f(bp.step_inputs()[0]).view(bp.bs, ex.in_H, ex.in_W, ex.in_Cs)[..., :ex.in_C].reshape(bp.bs, -1)
        if src.kind == "conv":
            g = ex.convs[src.idx]
            return _f(bp.conv_out[src.idx])[..., :g.Cout].reshape(bp.bs, -1)
        g = ex.denses[src.idx]
        return _f(bp.dense_out[src.idx])[:, :g.N]

    for g, ds in zip(ex.denses, ex.plan.denses):
        a = src_val(g.src)
        w, b = _bf(_w(m, wb, ds.dense, "kernel")), _w(m, wb, ds.dense, "bias")
        z = a @ w + b
        r = torch.relu(z) if g.relu else z
        if g.rate > 0:
            r = r * _mask(r.numel(), g.rate, ex.seed, g.stream, step).view(r.shape)
        got = _f(bp.dense_out[g.j])
        assert _rel(got[:, :g.N], r) < 1e-2, "dense %d fwd" % g.j
        # weight grad of this dense from its saved input and saved dh
        dh = _f(bp.dense_dh[g.j])[:, :g.N]
        gw = m.store.view(ds.dense, "kernel", grad=True).cpu()
        assert _rel(gw, a.t() @ dh) < 5e-3, "dense %d wgrad" % g.j
        assert _rel(m.store.view(ds.dense, "bias", grad=True).cpu(), dh.sum(0)) < 5e-3
        if g.src.kind == "conv" and g.KSb:
            # dX of a dense fed by a flattened conv: dH W^T through that conv's dropout / ReLU
            # masks, stored as its (pooled-resolution) output gradient -- dense_dx_kernel, or
            # dense_lds_kernel's LDS-staged epilogue for the legacy 65,536-wide layer
            pg = ex.convs[g.src.idx]
            xin = _f(bp.conv_out[pg.i])[..., :pg.Cout]
            dx = (dh @ w.t()).reshape(xin.shape)
            if pg.rate > 0:
                dx = dx * _mask(dx.numel(), pg.rate, ex.seed, pg.stream, step).view(dx.shape)
            if pg.relu:
                dx = dx * (xin > 0).float()
            got = _f(bp.conv_dy[pg.i])[..., :pg.Cout]
            assert _rel(got, dx) < 1e-2, "dense %d dX into conv %d: %.3g" % (g.j, pg.i, _rel(got, dx))
    # head: grads from the saved head input
    hd = ex.plan.head
    a = src_val(ex.head_src)
    w, b = _w(m, wb, hd.dense, "kernel"), _w(m, wb, hd.dense, "bias")
    z = a @ w + b
    y = _f(bp.step_inputs()[1])
    if hd.activation == "sigmoid":
        _, dz, _ = R.sigmoid_bce(z.reshape(-1), y.reshape(-1))
        dz = dz.reshape(-1, 1)
    else:
        _, dz, _ = R.softmax_cce(z, y)
    dz = dz / bp.bs
    gw = m.store.view(hd.dense, "kernel", grad=True).cpu()
    assert _rel(gw, a.t() @ dz) < 5e-3
    assert _rel(m.store.view(hd.dense, "bias", grad=True).cpu(), dz.sum(0)) < 5e-3


@pytest.mark.parametrize("kind,drop,cin", [("wide", 0.2, 3), ("wide_strided", 0.0, 3)])
def test_wide_convs_on_big_tiles(kind, drop, cin, monkeypatch):
    """The 256-row / 8-wave LDS-DMA conv blocks (conv_gl_kernel<NTC, 8>), which the legacy
    bench shapes take on grid size alone, forced onto the small wide cases: forward, dgrad
    (plain and input-dilated) and the pooled epilogue against the fp32 reference."""
    monkeypatch.setenv("INTML_TUNE", "conv_big_min=1")
    test_conv_forward(kind, drop, cin, 16, 40)
    test_conv_dgrad_bwd_through(kind, drop, cin, 16, 40)


@pytest.mark.parametrize("tune_s", ["conv_hs_wv=16,halo_tm=4", "conv_hs_dil=0,conv_gl_nbuf=4", "conv_hs=0", "conv_hs_order=0"])
def test_legacy_conv_variants(tune_s, monkeypatch):
    """The legacy bench shapes through each conv kernel form the executor can pick: the
    halo-staged conv in 512-row / 16-wave blocks (conv3, the strided dgrads' parity classes),
    the per-tap LDS-DMA gather with the 4-slot ring for the strided dgrads, and no halo-staged
    conv at all -- forward and dgrad against the fp32 reference."""
    monkeypatch.setenv("INTML_TUNE", tune_s)
    test_conv_forward("legacy", 0.0, 1, 64, 128)
    test_conv_dgrad_bwd_through("legacy", 0.0, 1, 64, 128)
