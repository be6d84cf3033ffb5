"""dense_bwd.hip: the per-wave pipelined dense weight-gradient kernel against a plain torch
fp32 reference (every split / tile-width variant the executor picks, odd batch tails and
N not a multiple of 16), and the opt-in fused optimizer path (INTML_TUNE=dense_opt=1) against the
default end-of-step reduction."""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

gpu = pytest.mark.gpu


def cdiv(a, b):
    return (a + b - 1) // b


def _wgrad(K, x, dh, N, S, order=0):
    dev = x.device
    M, width = x.shape
    NT, Ktiles = cdiv(N, 16), cdiv(width, 16)
    ntt = min(8, 1 << (NT.bit_length() - 1))
    pps = cdiv(cdiv(M, S), 32) * 32
    S = cdiv(M, pps)
    slab = torch.full((S, Ktiles * 16, NT * 16), float("nan"), device=dev)
    bslab = torch.full((S, NT * 16), float("nan"), device=dev)
    a = K.WgradArgs()
    a.x, a.B, a.H, a.W, a.Cs_in = x.data_ptr(), M, 1, 1, width
    a.Ho, a.Wo = 1, 1
    a.Ktiles, a.dy, a.Cs_dy, a.NT, a.P = Ktiles, dh.data_ptr(), dh.shape[1], NT, M
    a.px_per_split = pps
    a.slab, a.bslab = slab.data_ptr(), bslab.data_ptr()
    K.dense_wgrad(a, 2, ntt, S, torch.cuda.current_stream().cuda_stream, order)
    torch.cuda.synchronize()
    return slab.sum(0)[:width, :N], bslab.sum(0)[:N]


@gpu
@pytest.mark.parametrize("order", [0, 1, 2])
@pytest.mark.parametrize("M,width,N,S", [(40, 256, 128, 1), (128, 4096, 128, 1), (1024, 4096, 128, 2),
                                         (64, 96, 24, 1), (200, 512, 40, 2), (128, 9216, 128, 1)])
def test_dense_wgrad_matches_fp32(M, width, N, S, order):
    from cori_intml_examples_amd.ops.hip import kernels
    K = kernels()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(M + width + N)
    Ns = cdiv(N, 8) * 8
    x = torch.randn(M, width, generator=g).to(torch.bfloat16).to(dev)
    dh = torch.zeros(M, Ns, dtype=torch.bfloat16, device=dev)
    dh[:, :N] = torch.randn(M, N, generator=g).to(torch.bfloat16).to(dev)
    # order 1 / 2: the 1-D grid orders (n groups of a feature group consecutive; XCD ranges)
    gw, gb = _wgrad(K, x, dh, N, S, order)
    ref = x.float().t() @ dh.float()[:, :N]
    bref = dh.float()[:, :N].sum(0)
    assert torch.isfinite(gw).all() and torch.isfinite(gb).all()
    assert ((gw - ref).abs().max() / ref.abs().max()).item() < 1e-4
    assert ((gb - bref).abs().max() / bref.abs().max()).item() < 1e-4


@gpu
def test_dense_fused_optimizer_matches_reduction(monkeypatch):
    """INTML_TUNE=dense_opt=1 (optimizer applied inside the one-split dense wgrad) ends a few Adam
    steps where the default path (update in the end-of-step reduction) does: same gradient,
    same per-element update; only fp contraction may differ (Adam turns a last-ulp
    difference of a near-zero gradient into up to a full lr step, hence the distribution
    bound)."""
    from cori_intml_examples_amd.apps import zoo
    from cori_intml_examples_amd.io.datasets import synthetic_rpv
    kw = dict(conv_sizes=[16, 32, 64], fc_sizes=[128], dropout=0.0, optimizer="Adam", lr=1e-3, device="cuda:0")
    x, y, _ = synthetic_rpv(256, channels=3, seed=3)
    np.random.seed(1)
    torch.manual_seed(1)
    w0 = zoo.rpv_cnn((64, 64, 3), use_horovod=False, **kw).get_weights()
    out = {}
    for flag in ("0", "1"):
        monkeypatch.setenv("INTML_TUNE", "dense_opt=" + flag)
        m = zoo.rpv_cnn((64, 64, 3), use_horovod=False, **kw)
        m.set_weights(w0)
        for i in range(2):
            m.train_on_batch(x[i * 128:(i + 1) * 128], y[i * 128:(i + 1) * 128])
        torch.cuda.synchronize()
        plan = next(iter(m._executor._plans.values()))
        out[flag] = (np.concatenate([w.ravel() for w in m.get_weights()]), len(plan.dense_fused_opt))
    assert out["0"][1] == 0 and out["1"][1] == 1, "fused path not taken / taken by default"
    d = np.abs(out["1"][0] - out["0"][0])
    assert np.quantile(d, 0.999) < 1e-5 and d.max() < 2e-3, (np.quantile(d, 0.999), d.max())


@gpu
@pytest.mark.parametrize("extra", ["", ",dw_late=1,dw_order=2"])
def test_dense_fused_optimizer_writes_packs_legacy(monkeypatch, extra):
    """Legacy RPV (Dense(512) on a flattened 16384-wide input: its gradient is written in
    place) with the optimizer fused into the dense wgrad (dense_opt=auto, the default): the kernel
    also writes the layer's forward / backward bf16 packs from its updated-weight tile, and
    the layer's dX (the backward pack's reader) runs as a launch BEFORE it -- so after a few
    steps (a) the packs equal a full re-pack of the master bit for bit and (b) the weights
    match the unfused path (update in the end-of-step optimizer) within Adam's last-ulp bound."""
    from cori_intml_examples_amd.apps import zoo
    rs = np.random.RandomState(4)
    x = torch.tensor(rs.rand(96, 32, 32, 3).astype(np.float32)).to(torch.bfloat16).float().numpy()
    y = (rs.rand(96) > 0.5).astype(np.float32)
    np.random.seed(2)
    torch.manual_seed(2)
    w0 = zoo.rpv_legacy_cnn((32, 32, 3), lr=1e-3, device="cuda:0").get_weights()
    out = {}
    for flag in ("auto", "0"):
        # (extra: the late optimizer-state load form at 4 waves / SIMD, the XCD-ranged grid order)
        monkeypatch.setenv("INTML_TUNE", "dense_opt=" + flag + extra)
        m = zoo.rpv_legacy_cnn((32, 32, 3), lr=1e-3, device="cuda:0")
        m.set_weights(w0)
        for i in range(3):
            m.train_on_batch(x[i * 32:(i + 1) * 32], y[i * 32:(i + 1) * 32])
        torch.cuda.synchronize()
        ex = m._executor
        plan = next(iter(ex._plans.values()))
        arena = ex.arena.clone()
        ex.params_changed()                  # full re-pack from the master
        torch.cuda.synchronize()
        names = [it[0] for it in plan.launches]
        out[flag] = (np.concatenate([w.ravel() for w in m.get_weights()]), len(plan.dense_fused_opt),
                     bool(plan.optim_fused), torch.equal(arena, ex.arena), names)
    assert out["auto"][1] == 1 and out["0"][1] == 0, "fused path not taken by default / taken with dense_opt=0"
    assert out["auto"][3], "packs written by the fused dense optimizer differ from a re-pack"
    nm = out["auto"][4]
    assert "dense_dx0" in nm and nm.index("dense_dx0") < nm.index("wgrad_dense0"), nm
    d = np.abs(out["auto"][0] - out["0"][0])
    assert np.quantile(d, 0.999) < 1e-5 and d.max() < 3e-3, (np.quantile(d, 0.999), d.max())
