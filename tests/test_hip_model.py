"""HIP (gfx950) kernels vs the fp32 PyTorch reference, at whole-step granularity.

Every kernel of the fused step is exercised: gather, conv_mm forward (valid / same /
strided, pooled / unpooled, dropout), dense split-K + epilogue, the fused head (sigmoid-BCE,
softmax-CCE), wgrad (conv + dense), dgrad / dense-dX with the bwd-through epilogue,
slab_reduce and the fused optimizers + weight packing.  Tolerances reflect bf16
activations/weights against an fp32 reference.
"""
import numpy as np
import pytest
import torch

from cori_intml_examples_amd import Conv2D, Dense, Dropout, Flatten, Input, MaxPooling2D, Model, Sequential
from cori_intml_examples_amd.apps import zoo
from cori_intml_examples_amd.utils import set_random_seed

pytestmark = pytest.mark.gpu


def _build(kind, device, opt="Adam", drop=0.0, cin=1, hw=16):
    # the benchmarked geometries, built by the zoo exactly as bench.py builds them
    if kind == "rpv_bench":       # DistTrain_rpv: 64x64x3, conv[16,32,64] fc[128]
        return zoo.rpv_cnn((hw, hw, cin), conv_sizes=[16, 32, 64], fc_sizes=[128], dropout=drop,
                           optimizer=opt, lr=1e-3, device=device)
    if kind == "mnist_bench":     # DistTrain_mnist: 28x28x1, conv 32-64, fc 128
        return zoo.mnist_cnn(32, 64, 128, dropout=drop, optimizer=opt, lr=1e-3,
                             input_shape=(hw, hw, cin), device=device)
    if kind == "legacy":          # Train_rpv legacy: 64-128(s2)-256-256(s2), dense K = 65,536
        return zoo.rpv_legacy_cnn((hw, hw, cin), optimizer=opt, lr=1e-3, device=device)
    if kind == "mnist":
        m = Sequential(device=device)
        m.add(Conv2D(8, (3, 3), activation="relu", input_shape=(hw, hw, cin)))
        m.add(Conv2D(16, (3, 3), activation="relu"))
        m.add(MaxPooling2D((2, 2)))
        m.add(Dropout(drop))
        m.add(Flatten())
        m.add(Dense(32, activation="relu"))
        m.add(Dropout(drop))
        m.add(Dense(10, activation="softmax"))
        m.compile(optimizer=opt, loss="categorical_crossentropy", metrics=["accuracy"])
        return m
    if kind == "rpv":
        inp = Input(shape=(hw, hw, cin))
        h = inp
        for c in (16, 32, 64):
            h = Conv2D(c, (3, 3), activation="relu", padding="same")(h)
            h = MaxPooling2D((2, 2))(h)
        h = Dropout(drop)(h)
        h = Flatten()(h)
        h = Dense(128, activation="relu")(h)
        h = Dropout(drop)(h)
        out = Dense(1, activation="sigmoid")(h)
        m = Model(inp, out, name="RPVClassifier", device=device)
        m.compile(optimizer=opt, loss="binary_crossentropy", metrics=["accuracy"])
        return m
    if kind == "odd":     # odd channel counts, odd pooled grid, two hidden denses
        inp = Input(shape=(hw + 3, hw + 1, cin))
        h = Conv2D(5, (3, 3), activation="relu", padding="same")(inp)
        h = MaxPooling2D((2, 2))(h)
        h = Conv2D(12, (3, 3), activation="relu")(h)
        h = MaxPooling2D((2, 2))(h)
        h = Flatten()(h)
        h = Dense(20, activation="relu")(h)
        h = Dropout(drop)(h)
        h = Dense(9, activation="relu")(h)
        out = Dense(3, activation="softmax")(h)
        m = Model(inp, out, device=device)
        m.compile(optimizer=opt, loss="categorical_crossentropy", metrics=["accuracy"])
        return m
    if kind == "strided":
        inp = Input(shape=(hw, hw, cin))
        h = Conv2D(16, (3, 3), activation="relu", strides=1, padding="same")(inp)
        h = Conv2D(32, (3, 3), activation="relu", strides=2, padding="same")(h)
        h = Conv2D(32, (3, 3), activation="relu", strides=1, padding="same")(h)
        h = Conv2D(48, (3, 3), activation="relu", strides=2, padding="same")(h)
        h = Flatten()(h)
        h = Dense(64, activation="relu")(h)
        out = Dense(1, activation="sigmoid")(h)
        m = Model(inp, out, device=device)
        m.compile(optimizer=opt, loss="binary_crossentropy", metrics=["accuracy"])
        return m
    if kind == "wide":     # 64->128 pooled conv + its dgrad/wgrad take the tiled (wide) kernels
        inp = Input(shape=(hw, hw, cin))
        h = inp
        for c in (32, 64, 128):
            h = Conv2D(c, (3, 3), activation="relu", padding="same")(h)
            h = MaxPooling2D((2, 2))(h)
        h = Dropout(drop)(h)
        h = Flatten()(h)
        h = Dense(32, activation="relu")(h)
        out = Dense(1, activation="sigmoid")(h)
        m = Model(inp, out, device=device)
        m.compile(optimizer=opt, loss="binary_crossentropy", metrics=["accuracy"])
        return m
    if kind == "wide_strided":     # legacy-RPV-like strided wide convs (input-dilated dgrad)
        inp = Input(shape=(hw, hw, cin))
        h = Conv2D(32, (3, 3), activation="relu", strides=1, padding="same")(inp)
        h = Conv2D(64, (3, 3), activation="relu", strides=2, padding="same")(h)
        h = Conv2D(64, (3, 3), activation="relu", strides=1, padding="same")(h)
        h = Conv2D(96, (3, 3), activation="relu", strides=2, padding="same")(h)
        h = Flatten()(h)
        h = Dense(32, activation="relu")(h)
        out = Dense(1, activation="sigmoid")(h)
        m = Model(inp, out, device=device)
        m.compile(optimizer=opt, loss="binary_crossentropy", metrics=["accuracy"])
        return m
    raise ValueError(kind)


def _pair(kind, **kw):
    set_random_seed(1234)
    g = _build(kind, "cuda", **kw)
    set_random_seed(1234)
    c = _build(kind, "cpu", **kw)
    assert g._seed == c._seed
    for a, b in zip(g.get_weights(), c.get_weights()):
        np.testing.assert_array_equal(a, b)
    return g, c


def _data(model, n, seed=0):
    rs = np.random.RandomState(seed)
    shape = model.input_shape[1:]
    x = rs.rand(n, *shape).astype(np.float32)
    # quantise to bf16 so both backends see identical inputs
    x = torch.tensor(x).to(torch.bfloat16).float().numpy()
    nout = model.output_shape[-1]
    if nout == 1:
        y = (rs.rand(n) > 0.5).astype(np.float32)
    else:
        y = np.eye(nout, dtype=np.float32)[rs.randint(0, nout, n)]
    return x, y


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-12)


def _one_step(g, c, x, y):
    for m in (g, c):
        ex = m._executor
        d = ex.upload(x, y)
        ex.reset_metrics()
        perm = torch.arange(d.n, device=ex.device)
        ex.train_step(d, perm, 0, d.n)
    torch.cuda.synchronize()
    gg = g.store.grad[:g.store.numel].cpu().numpy()
    cg = c.store.grad[:c.store.numel].numpy()
    return gg, cg


@pytest.mark.parametrize("kind,drop,cin,hw,n", [
    ("rpv", 0.0, 1, 16, 48), ("rpv", 0.3, 3, 16, 48), ("mnist", 0.0, 1, 16, 48), ("mnist", 0.4, 1, 16, 48),
    ("odd", 0.25, 2, 16, 48), ("strided", 0.0, 3, 16, 48), ("wide", 0.2, 3, 16, 48), ("wide_strided", 0.0, 3, 16, 48),
    ("rpv_bench", 0.2, 3, 64, 128), ("mnist_bench", 0.4, 1, 28, 128)])
def test_grads_match_reference(kind, drop, cin, hw, n):
    g, c = _pair(kind, drop=drop, cin=cin, hw=hw)
    x, y = _data(g, n)
    gg, cg = _one_step(g, c, x, y)
    # end-to-end vs a pure-fp32 reference: bf16 activations flip near-tied max-pool
    # argmaxes / near-zero ReLU masks, so deep-layer gradients (first conv) drift most;
    # the per-kernel tests (test_hip_kernels.py) check each kernel tightly.
    for s in g.store.specs:
        a = gg[s.offset:s.offset + s.numel]
        b = cg[s.offset:s.offset + s.numel]
        err = _rel(a, b)
        cos = float(np.dot(a, b) / max(np.linalg.norm(a) * np.linalg.norm(b), 1e-30))
        assert err < 0.35 and cos > 0.95, "%s: grad rel err %.3g cos %.4f" % (s.name, err, cos)
    lg, ag, _ = g._executor.read_metrics()
    lc, ac, _ = c._executor.read_metrics()
    assert abs(lg - lc) < 2e-2 * max(1.0, abs(lc))


@pytest.mark.parametrize("kind,drop,cin,hw,n", [
    ("rpv_bench", 0.2, 3, 64, 128), ("mnist_bench", 0.4, 1, 28, 128), ("rpv", 0.3, 3, 16, 48),
    ("odd", 0.25, 2, 16, 48)])
def test_grads_match_bf16_reference(kind, drop, cin, hw, n, monkeypatch):
    """Whole-step gradients at the bench shapes against the bf16-FAITHFUL CPU oracle
    (executor_ref with ref_bf16: the same bf16 storage points as the HIP step, fp32
    everywhere else): every weight / bias gradient within the per-kernel tests' standard
    (relative error < 5e-2, cosine > 0.995).  What remains is fp32 summation
    order and the rare max-pool argmax tie it flips."""
    monkeypatch.setenv("INTML_TUNE", "ref_bf16=1")
    g, c = _pair(kind, drop=drop, cin=cin, hw=hw)
    assert c._executor.emulate_bf16
    x, y = _data(g, n)
    gg, cg = _one_step(g, c, x, y)
    worst = []
    for s in g.store.specs:
        a = gg[s.offset:s.offset + s.numel]
        b = cg[s.offset:s.offset + s.numel]
        err = _rel(a, b)
        cos = float(np.dot(a, b) / max(np.linalg.norm(a) * np.linalg.norm(b), 1e-30))
        worst.append((err, cos, s.name))
        assert err < 5e-2 and cos > 0.995, "%s: grad rel err %.3g cos %.6f" % (s.name, err, cos)
    lg, ag, _ = g._executor.read_metrics()
    lc, ac, _ = c._executor.read_metrics()
    assert abs(lg - lc) < 1e-3 * max(1.0, abs(lc)) and ag == ac, (lg, lc, ag, ac)
    print("worst grad rel err %.3g (cos %.6f) at %s" % max(worst))


@pytest.mark.parametrize("opt", ["Adam", "Nadam", "Adadelta", "SGD", "RMSprop"])
def test_optimizer_kernel_matches_keras_math(opt):
    """Fused optimizer kernel vs Keras-2.2 update math applied to the SAME gradients,
    over 3 steps (exercises slot state, bias correction, Nadam's schedule)."""
    from cori_intml_examples_amd.ops import reference as R
    set_random_seed(5)
    g = _build("rpv", "cuda", opt=opt)
    ex = g._executor
    o = ex.opt
    x, y = _data(g, 96, seed=3)
    d = ex.upload(x, y)
    n = g.store.numel
    w = g.store.master[:n].cpu().clone().double()
    s0 = torch.zeros(n, dtype=torch.float64)
    s1 = torch.zeros(n, dtype=torch.float64)
    msched = 1.0
    lr = float(o.lr)
    for t in range(1, 4):
        ex.train_step(d, torch.arange(d.n, device=ex.device), 32 * (t - 1), 32)
        torch.cuda.synchronize()
        gr = g.store.grad[:n].cpu().double()
        if opt == "Adam":
            R.adam_update(w, gr, s0, s1, t, lr, o.beta_1, o.beta_2, o.epsilon)
        elif opt == "Nadam":
            msched = R.nadam_update(w, gr, s0, s1, t, lr, msched, o.beta_1, o.beta_2, o.epsilon, o.schedule_decay)
        elif opt == "Adadelta":
            R.adadelta_update(w, gr, s0, s1, lr, o.rho, o.epsilon)
        elif opt == "SGD":
            R.sgd_update(w, gr, s0, lr)
        else:
            R.rmsprop_update(w, gr, s0, lr, o.rho, o.epsilon)
        got = g.store.master[:n].cpu().double()
        assert float((got - w).abs().max()) < 2e-5 * max(1.0, lr * 100), (opt, t)
    # bf16 pack mirrors the fp32 master after the update
    bp = ex._plans[(32, "train")]
    assert ex.arena.abs().sum().item() > 0


def test_predict_and_evaluate_match():
    g, c = _pair("mnist")
    x, y = _data(g, 77, seed=5)
    pg = g.predict(x, batch_size=32)
    pc = c.predict(x, batch_size=32)
    assert pg.shape == pc.shape == (77, 10)
    assert np.abs(pg - pc).max() < 2e-2
    eg = g.evaluate(x, y, batch_size=32, verbose=0)
    ec = c.evaluate(x, y, batch_size=32, verbose=0)
    assert abs(eg[0] - ec[0]) < 2e-2 * max(1, ec[0])


def test_fit_learns_and_graph_replay_consistent():
    from cori_intml_examples_amd.io.datasets import synthetic_mnist
    x, y, xt, yt = synthetic_mnist(4096, 512, rows=16, cols=16)
    set_random_seed(7)
    g = _build("mnist", "cuda", opt="Adadelta")
    h = g.fit(x, y, batch_size=128, epochs=3, verbose=0, validation_data=(xt, yt))
    assert h.history["val_acc"][-1] > 0.8
    assert h.history["loss"][-1] < h.history["loss"][0]


def test_multiple_steps_track_reference():
    g, c = _pair("rpv", opt="Adam", drop=0.2, cin=3)
    x, y = _data(g, 256, seed=11)
    for m in (g, c):
        ex = m._executor
        d = ex.upload(x, y)
        perm = torch.arange(d.n, device=ex.device)
        for k in range(4):
            ex.train_step(d, perm, 64 * k, 64)
    torch.cuda.synchronize()
    wg = g.store.master[:g.store.numel].cpu().numpy()
    wc = c.store.master[:c.store.numel].numpy()
    assert _rel(wg, wc) < 1e-2


def test_multi_step_graph_matches_single_steps():
    """train_steps(k) replays ONE graph of k step bodies (device-resident cursor, step
    counter, LR, dropout counter): bit-identical to k single-step replays, including the
    metric accumulators and a following single step."""
    set_random_seed(21)
    a = _build("rpv", "cuda", opt="Adam", drop=0.2, cin=3)
    set_random_seed(21)
    b = _build("rpv", "cuda", opt="Adam", drop=0.2, cin=3)
    x, y = _data(a, 640, seed=4)
    res = []
    for m, chunks in ((a, [1, 1, 1, 1, 1]), (b, [4, 1])):
        ex = m._executor
        d = ex.upload(x, y)
        perm = torch.randperm(d.n, generator=torch.Generator().manual_seed(3)).to(ex.device)
        ex.reset_metrics()
        pos = 0
        for k in chunks:
            ex.train_steps(d, perm, pos, 128, k)
            pos += 128 * k
        torch.cuda.synchronize()
        res.append((m.store.master[:m.store.numel].cpu().numpy(), ex.read_metrics(), int(m.optimizer.iterations)))
    np.testing.assert_array_equal(res[0][0], res[1][0])
    assert res[0][1] == res[1][1] and res[0][2] == res[1][2] == 5


@pytest.mark.parametrize("kind,drop,cin,hw", [("rpv", 0.2, 3, 64), ("rpv", 0.0, 1, 16), ("mnist", 0.4, 1, 28),
                                              ("odd", 0.25, 2, 16)])
def test_conv_stack_forward_matches_per_layer(kind, drop, cin, hw, monkeypatch):
    """The layer-fused forward (one workgroup per image, activations in LDS) produces the
    per-layer kernels' stage outputs and argmax codes bit for bit (same k order, bf16
    rounding points and dropout counters), and hence the same training step."""
    outs = []
    for flag in ("1", "0"):
        monkeypatch.setenv("INTML_TUNE", "conv_stack=" + flag)
        set_random_seed(33)
        m = _build(kind, "cuda", opt="Adam", drop=drop, cin=cin, hw=hw)
        x, y = _data(m, 96, seed=8)
        ex = m._executor
        d = ex.upload(x, y)
        perm = torch.arange(d.n, device=ex.device)
        ex.train_step(d, perm, 0, 96)
        torch.cuda.synchronize()
        bp = ex._plans[(96, "train")]
        names = [it[0] for it in bp.launches]
        outs.append(([t.clone() for t in bp.conv_out], [c.clone() if c is not None else None for c in bp.conv_code],
                     m.store.master[:m.store.numel].clone(), names))
    (o1, c1, w1, n1), (o0, c0, w0, n0) = outs
    assert "conv_stack_fwd" in n1 and "conv_stack_fwd" not in n0
    for i, (a, b) in enumerate(zip(o1, o0)):
        assert torch.equal(a, b), "stage %d output differs (max %g)" % (i, (a.float() - b.float()).abs().max())
    for a, b in zip(c1, c0):
        if a is not None:
            assert torch.equal(a, b)
    assert torch.equal(w1, w0)


def test_device_lr_warmup_matches_host_schedule():
    """The LR warmup evaluated by the device step bookkeeping (fit() keeps multi-step graph
    replays) gives the weights of writing each step's warmup LR from the host before every
    batch (one step per replay)."""
    from cori_intml_examples_amd import optim
    from cori_intml_examples_amd.models.executor_base import warmup_lr
    from cori_intml_examples_amd.parallel import callbacks as hcb
    from cori_intml_examples_amd.parallel import dist
    from cori_intml_examples_amd.train import callbacks as cbks
    orig = dist.size
    dist.size = lambda: 4
    try:
        set_random_seed(9)
        a = _build("rpv", "cuda", opt="SGD")
        w0 = a.get_weights()
        set_random_seed(9)
        b = _build("rpv", "cuda", opt="SGD")
        b.set_weights(w0)
        x, y = _data(a, 16 * 32, seed=2)
        a.fit(x, y, batch_size=32, epochs=3, verbose=0, shuffle=False, callbacks=[hcb.LearningRateWarmupCallback(2)])
        lr0 = float(optim.get_value(b.optimizer.lr))
        step = {"g": 0}

        def begin(bi, logs):
            g = step["g"]
            optim.set_value(b.optimizer.lr, warmup_lr(g, 16, 4, 2.0, lr0) if g < 32 else lr0)
            step["g"] += 1
        b.fit(x, y, batch_size=32, epochs=3, verbose=0, shuffle=False,
              callbacks=[cbks.LambdaCallback(on_batch_begin=begin)])
    finally:
        dist.size = orig
    assert (32, "train") in a._executor._plans
    assert a._executor._plans[(32, "train")].multi_graphs, "warmup must not force one step per replay"
    for wa, wb in zip(a.get_weights(), b.get_weights()):
        np.testing.assert_allclose(wa, wb, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("kind", ["rpv", "mnist"])
def test_nonfinite_loss_reads_nan(kind):
    """A diverged model (a NaN weight) reports loss / val_loss NaN, never a finite value: the
    head kernel's int64 fixed-point metric sum cannot carry a NaN, so it counts non-finite
    workgroups in a flag word and the host returns NaN.  The FoM of such a
    history is NaN (ranked worst), and finite epochs before the divergence still win."""
    from cori_intml_examples_amd.hpo.evaluator import figure_of_merit
    set_random_seed(5)
    m = _build(kind, "cuda", opt="Adam", cin=1, hw=16 if kind == "rpv" else 28)
    x, y = _data(m, 64, seed=2)
    h = m.fit(x, y, batch_size=32, epochs=1, validation_data=(x, y), verbose=0)
    assert np.isfinite(h.history["loss"][0]) and np.isfinite(h.history["val_loss"][0])
    w = m.get_weights()
    w[-2] = w[-2].copy()
    w[-2].flat[0] = np.nan                        # head kernel weight
    m.set_weights(w)
    ev = m.evaluate(x, y, verbose=0)
    assert np.isnan(ev[0]), ev
    h2 = m.fit(x, y, batch_size=32, epochs=1, validation_data=(x, y), verbose=0)
    assert np.isnan(h2.history["loss"][0]) and np.isnan(h2.history["val_loss"][0]), h2.history
    assert np.isnan(figure_of_merit(h2.history["val_loss"]))
    assert figure_of_merit(h.history["val_loss"] + h2.history["val_loss"]) == h.history["val_loss"][0]


@pytest.mark.parametrize("kind,drop,cin,hw,opt", [("rpv", 0.2, 3, 64, "Adam"), ("mnist", 0.4, 1, 28, "Nadam"),
                                                  ("odd", 0.25, 2, 16, "Adadelta")])
def test_prologue_free_step_matches_prologue(kind, drop, cin, hw, opt, monkeypatch):
    """The prologue-free step (the conv stack reads its images through the device cursor and
    permutation, the optimizer writes the bf16 packs through its pack routes, the first dense
    launch runs the step bookkeeping) trains bit-identically to the step with a prologue
    launch (gather + re-pack + bookkeeping) -- weights, metrics, iteration count, dropout
    counters over a multi-step graph -- and leaves the packs equal to a full re-pack."""
    res = []
    for tv in ("pro_free=1,opt_packs=1", "pro_free=0,opt_packs=0"):
        monkeypatch.setenv("INTML_TUNE", tv)
        set_random_seed(44)
        m = _build(kind, "cuda", opt=opt, drop=drop, cin=cin, hw=hw)
        x, y = _data(m, 320, seed=9)
        ex = m._executor
        d = ex.upload(x, y)
        perm = torch.randperm(d.n, generator=torch.Generator().manual_seed(5)).to(ex.device)
        ex.reset_metrics()
        ex.train_steps(d, perm, 0, 64, 3)
        ex.train_step(d, perm, 192, 64)
        torch.cuda.synchronize()
        names = [it[0] for it in ex._plans[(64, "train")].launches]
        arena = ex.arena.clone()
        ex.params_changed()                      # full re-pack from the master
        torch.cuda.synchronize()
        res.append((m.store.master[:m.store.numel].clone(), ex.read_metrics(), int(m.optimizer.iterations),
                    names, arena, ex.arena.clone()))
    (w1, m1, i1, n1, a1, r1), (w0, m0, i0, n0, a0, r0) = res
    assert "prologue" not in n1 and "prologue" in n0
    assert torch.equal(w1, w0)
    assert m1 == m0 and i1 == i0 == 4
    assert torch.equal(a1, r1), "optimizer-written packs differ from a re-pack of the master"
    assert torch.equal(r1, r0)     # (a0 is one update behind: the prologue re-packs at step start)


@pytest.mark.parametrize("kind,cin,tiled", [("odd", 2, False), ("rpv", 3, False), ("rpv", 3, True)])
def test_optimizer_pack_routes_match_repack(kind, cin, tiled):
    """optim_kernel (the DP path's optimizer) with pack routes writes exactly the bf16 packs a
    full re-pack of its updated master produces, for models with conv fwd + dgrad packs and
    dense fwd + bwd packs: per-element and float4 route paths (odd channel counts, unaligned
    ranges) and the 2-D tile blocks of a dense route (whole-range launch), whose weights
    equal the flat path's bit for bit."""
    outs = []
    for use_tiles in ((False, True) if tiled else (False,)):
        set_random_seed(45)
        m = _build(kind, "cuda", opt="Adam", drop=0.0, cin=cin, hw=16)
        ex = m._executor
        assert ex.routes is not None
        g = torch.randn(ex.store.capacity, generator=torch.Generator().manual_seed(7)) * 1e-2
        ex.store.grad.copy_(g.to(ex.device))
        a = ex._optim_args(False, defer_pack=True)
        ranges = ((0, ex.store.numel),) if use_tiles else ((0, ex.store.numel // 3), (ex.store.numel // 3, ex.store.numel))
        for lo, hi in ranges:
            a.lo, a.n = lo, hi - lo
            if use_tiles:
                ex.tile_routes(a)
                assert a.ntile == 1
            ex.K.optim(a, ex.pack_table, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        written = ex.arena.clone()
        ex.params_changed()
        torch.cuda.synchronize()
        assert torch.equal(written, ex.arena)
        outs.append(m.store.master.clone())
    if tiled:
        assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("kind,drop,cin,hw,opt", [("rpv", 0.2, 3, 64, "Adam"), ("mnist", 0.4, 1, 28, "Nadam")])
def test_head_fast_paths_bit_identical(kind, drop, cin, hw, opt, monkeypatch):
    """The head kernel's fast paths (one-round-trip split-K epilogue loads; the binary head's
    dz published before its loss, with the loss / metric atomics on wave 0 while waves 1-3
    write the slabs and dh) train bit-identically to the generic serial path: weights,
    metrics and iteration count over a multi-step graph."""
    res = []
    for tv in ("head_generic=0", "head_generic=1"):
        monkeypatch.setenv("INTML_TUNE", tv)
        set_random_seed(46)
        m = _build(kind, "cuda", opt=opt, drop=drop, cin=cin, hw=hw)
        x, y = _data(m, 512, seed=10)
        ex = m._executor
        d = ex.upload(x, y)
        perm = torch.randperm(d.n, generator=torch.Generator().manual_seed(6)).to(ex.device)
        ex.reset_metrics()
        ex.train_steps(d, perm, 0, 128, 3)
        torch.cuda.synchronize()
        res.append((m.store.master[:m.store.numel].clone(), ex.read_metrics(), int(m.optimizer.iterations)))
    (w1, m1, i1), (w0, m0, i0) = res
    assert torch.equal(w1, w0)
    assert m1 == m0 and i1 == i0 == 3


@pytest.mark.parametrize("kind,drop,cin,hw", [("rpv", 0.2, 3, 64), ("rpv", 0.0, 1, 16)])
def test_stack_k16_tail_bit_identical(kind, drop, cin, hw, monkeypatch):
    """The conv stack's 4-channel first layer with its tap-8 k-step as a 16x16x16 MFMA
    (stack_k16) computes exactly what the 16x16x32 k-step over zero-padded weights does:
    whole training steps bit-identical."""
    res = []
    for tv in ("stack_k16=1", "stack_k16=0"):
        monkeypatch.setenv("INTML_TUNE", tv)
        set_random_seed(48)
        m = _build(kind, "cuda", opt="Adam", drop=drop, cin=cin, hw=hw)
        x, y = _data(m, 256, seed=12)
        ex = m._executor
        d = ex.upload(x, y)
        perm = torch.randperm(d.n, generator=torch.Generator().manual_seed(8)).to(ex.device)
        ex.reset_metrics()
        ex.train_steps(d, perm, 0, 128, 2)
        torch.cuda.synchronize()
        res.append((m.store.master[:m.store.numel].clone(), ex.read_metrics()))
    assert torch.equal(res[0][0], res[1][0]) and res[0][1] == res[1][1]


@pytest.mark.parametrize("kind,drop,cin,hw", [("rpv", 0.2, 3, 64), ("mnist", 0.3, 1, 28)])
def test_stack_fast_prologue_bit_identical(kind, drop, cin, hw, monkeypatch):
    """The conv stack's one-batch prologue (biases, layer-0 weights, the image's dataset row
    and pixels loaded together before any LDS store) stages exactly what the sequential
    prologue (stack_dbg=128) does: whole training steps bit-identical."""
    res = []
    for tv in ("stack_dbg=0", "stack_dbg=128"):
        monkeypatch.setenv("INTML_TUNE", tv)
        set_random_seed(49)
        m = _build(kind, "cuda", opt="Adam", drop=drop, cin=cin, hw=hw)
        x, y = _data(m, 256, seed=13)
        ex = m._executor
        d = ex.upload(x, y)
        perm = torch.randperm(d.n, generator=torch.Generator().manual_seed(9)).to(ex.device)
        ex.reset_metrics()
        ex.train_steps(d, perm, 0, 128, 2)
        torch.cuda.synchronize()
        res.append((m.store.master[:m.store.numel].clone(), ex.read_metrics()))
    assert torch.equal(res[0][0], res[1][0]) and res[0][1] == res[1][1]


@pytest.mark.parametrize("kind,drop,cin,hw", [("rpv_bench", 0.2, 3, 64), ("rpv_bench", 0.0, 1, 64),
                                               ("mnist_bench", 0.3, 1, 28)])
def test_conv_stack_specialised_bit_identical(kind, drop, cin, hw, monkeypatch):
    """The layer-signature-specialised conv stack instances (compile-time layer bodies and
    tile shapes, no ablation code: conv_stack.hip kStackSigs) train exactly like the generic
    kernel on the DistTrain_rpv / DistTrain_mnist stacks -- and the launcher really picks a
    specialised instance for them (conv_stack_variant > 0)."""
    res = []
    for tv in ("stack_spec=2", "stack_spec=1", "stack_spec=0"):
        monkeypatch.setenv("INTML_TUNE", tv)
        set_random_seed(55)
        m = _build(kind, "cuda", opt="Adam", drop=drop, cin=cin, hw=hw)
        x, y = _data(m, 256, seed=19)
        ex = m._executor
        d = ex.upload(x, y)
        perm = torch.randperm(d.n, generator=torch.Generator().manual_seed(16)).to(ex.device)
        ex.reset_metrics()
        ex.train_steps(d, perm, 0, 128, 2)
        torch.cuda.synchronize()
        plan = ex._plans[(128, "train")]
        stack = [f for it in plan.launches if it[0] == "conv_stack_fwd" for f in (it[1].__defaults__ or ())
                 if hasattr(f, "spec")]
        assert len(stack) == 1
        res.append((m.store.master[:m.store.numel].clone(), ex.read_metrics(), ex.K.conv_stack_variant(stack[0])))
    assert res[0][2] > 0 and res[1][2] > 0 and res[2][2] == 0, [r[2] for r in res]
    for r in res[:2]:
        assert torch.equal(r[0], res[2][0]) and r[1] == res[2][1]


@pytest.mark.parametrize("kind,drop,cin,hw", [("rpv", 0.2, 3, 64), ("mnist", 0.3, 1, 28)])
def test_write_through_stores_bit_identical(kind, drop, cin, hw, monkeypatch):
    """Write-through (16-byte sc1) stores of the stage outputs / argmax codes (wt & 1), the
    backward gradients dP / dH (wt & 2) and the weight-gradient slabs (wt & 4, through a
    wave-private LDS square) store exactly the plain stores' bytes: whole training steps
    bit-identical."""
    res = []
    for tv in ("wt=7", "wt=0"):
        monkeypatch.setenv("INTML_TUNE", tv)
        set_random_seed(50)
        m = _build(kind, "cuda", opt="Adam", drop=drop, cin=cin, hw=hw)
        x, y = _data(m, 256, seed=14)
        ex = m._executor
        d = ex.upload(x, y)
        perm = torch.randperm(d.n, generator=torch.Generator().manual_seed(10)).to(ex.device)
        ex.reset_metrics()
        ex.train_steps(d, perm, 0, 128, 2)
        torch.cuda.synchronize()
        res.append((m.store.master[:m.store.numel].clone(), ex.read_metrics()))
    assert torch.equal(res[0][0], res[1][0]) and res[0][1] == res[1][1]


@pytest.mark.parametrize("kind,drop,cin,hw", [("rpv", 0.2, 3, 64), ("mnist", 0.3, 1, 28)])
def test_dgrad_onebatch_prologue_bit_identical(kind, drop, cin, hw, monkeypatch):
    """The dgrad's one-batch prologue (weight and pooled-halo loads in flight together,
    conv_halo_body.h) stages exactly what the two-phase form (dgrad_dbg=32) does: whole training
    steps bit-identical.  (The A/B switch lives in the standalone dgrad kernel only -- the
    co-scheduled dual kernel is built without it -- so both arms run standalone launches.)"""
    res = []
    for tv in ("dual_halo=0,dgrad_dbg=0", "dual_halo=0,dgrad_dbg=32"):
        monkeypatch.setenv("INTML_TUNE", tv)
        set_random_seed(51)
        m = _build(kind, "cuda", opt="Adam", drop=drop, cin=cin, hw=hw)
        x, y = _data(m, 256, seed=15)
        ex = m._executor
        d = ex.upload(x, y)
        perm = torch.randperm(d.n, generator=torch.Generator().manual_seed(12)).to(ex.device)
        ex.reset_metrics()
        ex.train_steps(d, perm, 0, 128, 2)
        torch.cuda.synchronize()
        res.append((m.store.master[:m.store.numel].clone(), ex.read_metrics()))
    assert torch.equal(res[0][0], res[1][0]) and res[0][1] == res[1][1]


def test_fused_dense_optimizer_falls_back(monkeypatch):
    """A dense layer that took the in-wgrad optimizer path (dense_opt=1: every one-split layer)
    in a step whose end-of-step reduction cannot fuse the optimizer (more slab descriptors than
    the table holds; forced here with red_desc_max=1) falls back to the full optimizer launch:
    its wgrad then stores the gradient and writes no packs, and the step trains exactly like
    the same fallback step without the dense fusion (it used to throw 'fused pack
    writes need the fused optimizer' on every launch)."""
    res = []
    for tv in ("dense_opt=1,red_desc_max=1", "dense_opt=0,red_desc_max=1"):
        monkeypatch.setenv("INTML_TUNE", tv)
        set_random_seed(54)
        m = _build("rpv_bench", "cuda", opt="Adam", drop=0.2, cin=3, hw=64)
        x, y = _data(m, 256, seed=18)
        ex = m._executor
        d = ex.upload(x, y)
        perm = torch.randperm(d.n, generator=torch.Generator().manual_seed(15)).to(ex.device)
        ex.reset_metrics()
        ex.train_steps(d, perm, 0, 128, 2)
        torch.cuda.synchronize()
        plan = ex._plans[(128, "train")]
        assert not plan.optim_fused and not plan.dense_fused_opt
        arena = ex.arena.clone()
        ex.params_changed()                      # full re-pack from the master
        torch.cuda.synchronize()
        assert torch.equal(arena, ex.arena), "packs differ from a re-pack of the master"
        res.append((m.store.master[:m.store.numel].clone(), ex.read_metrics()))
    assert torch.equal(res[0][0], res[1][0]) and res[0][1] == res[1][1]


@pytest.mark.parametrize("kind,drop,cin,hw", [("rpv_bench", 0.2, 3, 64), ("mnist_bench", 0.3, 1, 28)])
def test_dual_launch_matches_standalone(kind, drop, cin, hw, monkeypatch):
    """The co-scheduled wgrad || dgrad launch (production bodies only: dgrad epilogue fixed to
    backward-through, no ablation / stamp code) computes exactly what the two standalone kernels
    it fuses compute: with the head / dense layers' reduction + update at the end of the step in
    both arms (early_reduce=0), whole training steps are bit-identical.  (With the default early
    reduction riding in the dual launch, the update of those layers runs in a different kernel
    instance -- fp32 last-bit differences, test_dual_launch_early_reduce_close.)"""
    res = []
    for tv in ("dual_halo=1,early_reduce=0", "dual_halo=0,early_reduce=0"):
        monkeypatch.setenv("INTML_TUNE", tv)
        set_random_seed(56)
        m = _build(kind, "cuda", opt="Adam", drop=drop, cin=cin, hw=hw)
        x, y = _data(m, 256, seed=20)
        ex = m._executor
        d = ex.upload(x, y)
        perm = torch.randperm(d.n, generator=torch.Generator().manual_seed(17)).to(ex.device)
        ex.reset_metrics()
        ex.train_steps(d, perm, 0, 128, 2)
        torch.cuda.synchronize()
        names = [it[0] for it in ex._plans[(128, "train")].launches]
        res.append((m.store.master[:m.store.numel].clone(), ex.read_metrics(), names))
    assert any(n.startswith("wgrad_dgrad_conv") for n in res[0][2])
    d = (res[0][0] - res[1][0]).abs()
    assert torch.equal(res[0][0], res[1][0]) and res[0][1] == res[1][1], (float(d.max()), int((d > 0).sum()),
                                                                           res[0][1], res[1][1])


def test_dual_launch_early_reduce_close(monkeypatch):
    """Default step (dual launches carrying the head / dense reduction + Adam in extra
    workgroups) vs standalone launches with one end-of-step reduction: the same training to
    fp32 last-bit level (measured max |dw| ~4e-9), identical metrics."""
    res = []
    for tv in ("dual_halo=1", "dual_halo=0"):
        monkeypatch.setenv("INTML_TUNE", tv)
        set_random_seed(57)
        m = _build("rpv_bench", "cuda", opt="Adam", drop=0.2, cin=3, hw=64)
        x, y = _data(m, 256, seed=21)
        ex = m._executor
        d = ex.upload(x, y)
        perm = torch.randperm(d.n, generator=torch.Generator().manual_seed(18)).to(ex.device)
        ex.reset_metrics()
        ex.train_steps(d, perm, 0, 128, 2)
        torch.cuda.synchronize()
        res.append((m.store.master[:m.store.numel].clone(), ex.read_metrics()))
    assert float((res[0][0] - res[1][0]).abs().max()) < 1e-6 and res[0][1] == res[1][1]


def test_dense_dx_tiles_agree(monkeypatch):
    """The dense layer's dX at 1, 2 and 4 n-tiles per wave (dense_bwd_pair / dense_dx: the
    tile only changes which wave computes an output, not its k order) trains the same: SGD
    weights after 2 steps agree to fp32 reordering level."""
    res = []
    for tv in ("dx_ntc=1", "dx_ntc=2", "dx_ntc=4"):
        monkeypatch.setenv("INTML_TUNE", tv)
        set_random_seed(53)
        m = _build("rpv_bench", "cuda", opt="SGD", drop=0.0, cin=3, hw=64)
        x, y = _data(m, 256, seed=17)
        ex = m._executor
        d = ex.upload(x, y)
        perm = torch.randperm(d.n, generator=torch.Generator().manual_seed(14)).to(ex.device)
        ex.reset_metrics()
        ex.train_steps(d, perm, 0, 128, 2)
        torch.cuda.synchronize()
        res.append(m.store.master[:m.store.numel].clone())
    for r in res[1:]:
        assert (r - res[0]).abs().max().item() < 1e-5
