"""Framework semantics on the CPU reference backend (SURVEY.md §4.2/§4.3 "Framework
tests"): summary goldens, Keras 2.2 fit/evaluate/predict behaviour, optimizer math,
callbacks, the dropout RNG twin, and gradients of the explicit backward vs autograd."""
import io
import contextlib

import numpy as np
import pytest
import torch

from cori_intml_examples_amd import optim
from cori_intml_examples_amd.apps import zoo
from cori_intml_examples_amd.io.datasets import synthetic_mnist, synthetic_rpv
from cori_intml_examples_amd.models import (Conv2D, Dense, Dropout, Flatten, Input, MaxPooling2D, Model,
                                            Sequential)
from cori_intml_examples_amd.ops import reference as R
from cori_intml_examples_amd.ops.rng import dropout_keep, keep_threshold, rng_u32
from cori_intml_examples_amd.train import callbacks as cbks
from cori_intml_examples_amd.utils import set_random_seed

GOLDEN_SUMMARY = """\
_________________________________________________________________
Layer (type)                 Output Shape              Param #
=================================================================
conv2d_1 (Conv2D)            (None, 26, 26, 32)        320
_________________________________________________________________
conv2d_2 (Conv2D)            (None, 24, 24, 64)        18496
_________________________________________________________________
max_pooling2d_1 (MaxPooling2 (None, 12, 12, 64)        0
_________________________________________________________________
dropout_1 (Dropout)          (None, 12, 12, 64)        0
_________________________________________________________________
flatten_1 (Flatten)          (None, 9216)              0
_________________________________________________________________
dense_1 (Dense)              (None, 128)               1179776
_________________________________________________________________
dropout_2 (Dropout)          (None, 128)               0
_________________________________________________________________
dense_2 (Dense)              (None, 10)                1290
=================================================================
Total params: 1,199,882
Trainable params: 1,199,882
Non-trainable params: 0
_________________________________________________________________
"""


def _summary(m):
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        m.summary()
    return buf.getvalue()


def test_summary_golden_mnist():
    m = zoo.mnist_cnn(h1=32, h2=64, h3=128, dropout=0.25, dropout2=0.5, device="cpu")
    got = _summary(m).splitlines()
    # DistTrain_mnist.ipynb summary output, verbatim (Keras pads table rows to 65 columns)
    assert [l.rstrip() for l in got] == GOLDEN_SUMMARY.splitlines()
    assert got[1] == "Layer (type)                 Output Shape              Param #   "
    assert got[3] == "conv2d_1 (Conv2D)            (None, 26, 26, 32)        320       "


def test_param_count_goldens():
    assert zoo.mnist_cnn(32, 64, 128, device="cpu").count_params() == 1199882
    assert zoo.mnist_cnn(4, 8, 32, device="cpu").count_params() == 37562
    assert zoo.rpv_cnn((64, 64, 1), [16, 32, 64], [128], device="cpu").count_params() == 547841
    assert zoo.rpv_legacy_cnn((64, 64, 1), device="cpu").count_params() == 34515201
    s = _summary(zoo.rpv_cnn((64, 64, 1), [16, 32, 64], [128], device="cpu"))
    assert " (InputLayer)         (None, 64, 64, 1)         0" in s


def test_functional_and_sequential_api():
    inp = Input(shape=(8, 8, 1))
    h = Conv2D(2, (3, 3), padding="same", activation="relu")(inp)
    h = MaxPooling2D()(h)
    h = Flatten()(h)
    out = Dense(1, activation="sigmoid")(h)
    m = Model(inputs=inp, outputs=out, name="RPVClassifier", device="cpu")
    assert m.name == "RPVClassifier" and m.output_shape == (None, 1)
    assert [l.name for l in m.layers] == ["input_1", "conv2d_1", "max_pooling2d_1", "flatten_1", "dense_1"]
    s = Sequential(device="cpu")
    with pytest.raises(ValueError):
        s.add(Dense(3))                          # first layer needs an input_shape
    with pytest.raises(RuntimeError):
        m.fit(np.zeros((2, 8, 8, 1)), np.zeros(2))   # not compiled
    m.compile("adam", "binary_crossentropy", metrics=["accuracy"])
    assert m.metrics_names == ["loss", "acc"]
    assert m.get_config()["layers"][1]["inbound_nodes"] == [[["input_1", 0, 0, {}]]]


def test_fit_semantics_history_validation_split():
    x, y, _, _ = synthetic_mnist(600, 10, rows=12, cols=12)
    m = zoo.mnist_cnn(4, 8, 16, dropout=0.1, optimizer="Adam", input_shape=(12, 12, 1), device="cpu")
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        h = m.fit(x, y, batch_size=64, epochs=2, validation_split=0.17, verbose=2)
    out = buf.getvalue()
    # validation_split takes the LAST fraction (DistHPO_mnist.ipynb:293: 60000 -> 49800 / 10200)
    assert "Train on 498 samples, validate on 102 samples" in out
    assert "Epoch 1/2" in out and " - loss: " in out and " - val_acc: " in out
    assert sorted(h.history) == ["acc", "loss", "val_acc", "val_loss"] and h.epoch == [0, 1]
    ev = m.evaluate(x[498:], y[498:], verbose=0)
    assert ev[0] == pytest.approx(h.history["val_loss"][-1], rel=1e-6)
    p = m.predict(x[:7])
    assert p.shape == (7, 10) and np.allclose(p.sum(1), 1, atol=1e-5)
    assert m.predict_classes(x[:7]).shape == (7,)
    assert h.history["loss"][1] < h.history["loss"][0]


def test_history_lr_and_callbacks_order():
    x, y, _ = synthetic_rpv(96, size=16, seed=1)
    m = zoo.rpv_cnn((16, 16, 1), [4, 4, 4], [8], optimizer="Adam", device="cpu")
    seen = []
    lam = cbks.LambdaCallback(on_epoch_end=lambda e, logs: seen.append(dict(logs)))
    rl = cbks.ReduceLROnPlateau(patience=0, factor=0.5, min_delta=10.0, verbose=0)   # always "plateaus"
    h = m.fit(x, y, batch_size=32, epochs=3, validation_data=(x[:32], y[:32]), verbose=0, callbacks=[rl, lam])
    assert "lr" in h.history and h.history["lr"][0] == pytest.approx(0.001)
    assert h.history["lr"][-1] < h.history["lr"][0]
    assert optim.get_value(m.optimizer.lr) == pytest.approx(h.history["lr"][-1] * 0.5)
    assert "lr" in seen[0]                        # later callbacks see the lr key (rpv.py:94-98)
    es = cbks.EarlyStopping(monitor="val_loss", patience=0, min_delta=10.0)
    h2 = m.fit(x, y, batch_size=32, epochs=5, validation_data=(x[:32], y[:32]), verbose=0, callbacks=[es])
    assert len(h2.epoch) == 2


def test_lr_warmup_callback_matches_per_batch_schedule():
    """The device/executor-evaluated warmup gives exactly the weights of writing
    lr * (1/size) * ((g+1)/spe * (size-1)/W + 1) into the optimizer before every batch
    (the Horovod callback's per-batch behaviour), and keeps fit() on multi-step replays."""
    from cori_intml_examples_amd.parallel import callbacks as hcb
    from cori_intml_examples_amd.parallel import dist
    from cori_intml_examples_amd.models.executor_base import warmup_lr

    x, y, _ = synthetic_rpv(64, size=16, seed=1)
    orig = dist.size
    dist.size = lambda: 4                          # pretend 4 ranks: warmup lr/4 -> lr
    try:
        m = zoo.rpv_cnn((16, 16, 1), [4, 4, 4], [8], dropout=0.0, optimizer="SGD", lr=0.004, device="cpu")
        w0 = m.get_weights()
        cb = hcb.LearningRateWarmupCallback(2)
        assert not cbks.CallbackList([cb]).batch_begin_needed
        h = m.fit(x, y, batch_size=16, epochs=3, verbose=0, shuffle=False, callbacks=[cb])
        wa = m.get_weights()

        m2 = zoo.rpv_cnn((16, 16, 1), [4, 4, 4], [8], dropout=0.0, optimizer="SGD", lr=0.004, device="cpu")
        m2.set_weights(w0)
        step = {"g": 0}

        def begin(b, logs):
            g = step["g"]
            optim.set_value(m2.optimizer.lr, warmup_lr(g, 4, 4, 2.0, 0.004) if g < 8 else 0.004)
            step["g"] += 1
        m2.fit(x, y, batch_size=16, epochs=3, verbose=0, shuffle=False,
               callbacks=[cbks.LambdaCallback(on_batch_begin=begin)])
        wb = m2.get_weights()
    finally:
        dist.size = orig
    for a, b in zip(wa, wb):
        np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-7)
    # epoch logs carry the LR of the epoch's last step; after warmup the full LR
    assert h.history["lr"][0] == pytest.approx(0.004 / 4 * (4 / 4 * 3 / 2 + 1))
    assert h.history["lr"][1] == pytest.approx(0.004)
    assert optim.get_value(m.optimizer.lr) == pytest.approx(0.004)


def test_lr_warmup_resume_continues_absolute_ramp():
    """A fit() resumed at initial_epoch continues the warmup ramp where it stands (the ramp is
    anchored at epoch 0, as Horovod's callback uses the absolute epoch): epochs 0-2 in one
    run end on the weights of epoch 0, then a resumed fit(initial_epoch=1) -- not a restart
    of the ramp from lr/size.  Momentum correction with a momentum optimizer is refused."""
    from cori_intml_examples_amd.parallel import callbacks as hcb
    from cori_intml_examples_amd.parallel import dist

    x, y, _ = synthetic_rpv(64, size=16, seed=1)
    orig = dist.size
    dist.size = lambda: 4
    try:
        m = zoo.rpv_cnn((16, 16, 1), [4, 4, 4], [8], dropout=0.0, optimizer="SGD", lr=0.004, device="cpu")
        w0 = m.get_weights()
        m.fit(x, y, batch_size=16, epochs=3, verbose=0, shuffle=False, callbacks=[hcb.LearningRateWarmupCallback(2)])
        wa = m.get_weights()
        m2 = zoo.rpv_cnn((16, 16, 1), [4, 4, 4], [8], dropout=0.0, optimizer="SGD", lr=0.004, device="cpu")
        m2.set_weights(w0)
        m2.fit(x, y, batch_size=16, epochs=1, verbose=0, shuffle=False, callbacks=[hcb.LearningRateWarmupCallback(2)])
        optim.set_value(m2.optimizer.lr, 0.004)        # what a checkpoint of the run would hold
        m2.fit(x, y, batch_size=16, epochs=3, initial_epoch=1, verbose=0, shuffle=False,
               callbacks=[hcb.LearningRateWarmupCallback(2)])
        wb = m2.get_weights()
        m3 = zoo.rpv_cnn((16, 16, 1), [4, 4, 4], [8], dropout=0.0, optimizer=optim.SGD(lr=0.004, momentum=0.9),
                         device="cpu")
        with pytest.raises(NotImplementedError):
            m3.fit(x, y, batch_size=16, epochs=1, verbose=0, callbacks=[hcb.LearningRateWarmupCallback(2)])
        m3.fit(x, y, batch_size=16, epochs=1, verbose=0,
               callbacks=[hcb.LearningRateWarmupCallback(2, momentum_correction=False)])
        # no ramp -> nothing for momentum correction to do: warmup_epochs=0 (what
        # apps.rpv.train_model always adds) and a resume past the window both train
        m3.fit(x, y, batch_size=16, epochs=1, verbose=0, callbacks=[hcb.LearningRateWarmupCallback(0)])
        m3.fit(x, y, batch_size=16, epochs=3, initial_epoch=2, verbose=0,
               callbacks=[hcb.LearningRateWarmupCallback(2)])
    finally:
        dist.size = orig
    for a, b in zip(wa, wb):
        np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-7)


def test_optimizer_closed_form_single_step():
    torch.manual_seed(0)
    p0, g = torch.randn(50), torch.randn(50)
    # Adam step 1: p -= lr * sqrt(1-b2)/(1-b1) * m/(sqrt(v)+eps), m=(1-b1)g, v=(1-b2)g^2
    p, m, v = p0.clone(), torch.zeros(50), torch.zeros(50)
    R.adam_update(p, g, m, v, 1, 0.001)
    lr_t = 0.001 * np.sqrt(1 - 0.999) / (1 - 0.9)
    exp = p0 - lr_t * (0.1 * g) / (torch.sqrt(0.001 * g * g) + 1e-7)
    assert torch.allclose(p, exp, atol=1e-6)
    # Adadelta: a = (1-rho) g^2; upd = g sqrt(eps)/sqrt(a+eps); p -= lr upd
    p, a, d = p0.clone(), torch.zeros(50), torch.zeros(50)
    R.adadelta_update(p, g, a, d, 1.0)
    upd = g * np.sqrt(1e-7) / torch.sqrt(0.05 * g * g + 1e-7)
    assert torch.allclose(p, p0 - upd, atol=1e-6) and torch.allclose(d, 0.05 * upd * upd, atol=1e-9)
    # SGD momentum / nesterov
    p, mom = p0.clone(), torch.zeros(50)
    R.sgd_update(p, g, mom, 0.1, momentum=0.9, nesterov=True)
    assert torch.allclose(p, p0 + 0.9 * (-0.1 * g) - 0.1 * g, atol=1e-6)
    # optimizer objects: Keras defaults and name lookup (rpv.py:62 getattr(optimizers, name)(lr=lr))
    assert getattr(optim, "Adadelta")().lr.get() == 1.0 and optim.get("nadam").lr.get() == 0.002
    assert optim.get("Adam").get_config()["beta_2"] == 0.999


def test_model_training_matches_closed_form_adam():
    """Two full training steps on the CPU backend == Keras Adam math on autograd gradients."""
    x, y, _ = synthetic_rpv(32, size=8, seed=4)
    m = zoo.rpv_cnn((8, 8, 1), [2, 2, 2], [4], dropout=0.0, optimizer="Adam", lr=0.01, device="cpu")
    ws = [torch.tensor(w, dtype=torch.float64, requires_grad=True) for w in m.get_weights()]
    mom = [torch.zeros_like(w) for w in ws]
    vel = [torch.zeros_like(w) for w in ws]

    def loss_fn(ws):
        a = torch.tensor(x, dtype=torch.float64)
        for i in range(3):
            a = R.conv2d(a, ws[2 * i], ws[2 * i + 1], 1, "same").relu()
            a = torch.nn.functional.max_pool2d(a.permute(0, 3, 1, 2), 2).permute(0, 2, 3, 1)
        a = a.reshape(a.shape[0], -1)
        a = (a @ ws[6] + ws[7]).relu()
        z = (a @ ws[8] + ws[9]).reshape(-1)
        p = torch.sigmoid(z).clamp(1e-7, 1 - 1e-7)
        yt = torch.tensor(y, dtype=torch.float64)
        return -(yt * torch.log(p) + (1 - yt) * torch.log(1 - p)).mean()

    for t in (1, 2):
        ws_ = [w.detach().clone().requires_grad_(True) for w in ws]
        loss = loss_fn(ws_)
        gs = torch.autograd.grad(loss, ws_)
        lr_t = 0.01 * np.sqrt(1 - 0.999 ** t) / (1 - 0.9 ** t)
        new = []
        for w, g, mo, ve in zip(ws_, gs, mom, vel):
            mo.mul_(0.9).add_(0.1 * g)
            ve.mul_(0.999).add_(0.001 * g * g)
            new.append((w - lr_t * mo / (ve.sqrt() + 1e-7)).detach())
        ws = new
        out = m.train_on_batch(x, y)
        assert out[0] == pytest.approx(float(loss), rel=1e-4)
    for a, b in zip(m.get_weights(), ws):
        np.testing.assert_allclose(a, b.numpy(), rtol=0, atol=2e-5)


def test_dropout_rng_twin_properties():
    idx = torch.arange(100000, dtype=torch.int64)
    u = rng_u32(idx, seed=7, stream=1, step=3)
    assert u.dtype == torch.int64 and int(u.min()) >= 0 and int(u.max()) < 2 ** 32
    keep = dropout_keep(100000, 0.2, seed=7, stream=1, step=3)
    assert abs(float(keep.float().mean()) - 0.8) < 0.01
    assert not torch.equal(keep, dropout_keep(100000, 0.2, seed=7, stream=1, step=4))   # new mask per step
    assert torch.equal(keep, dropout_keep(100000, 0.2, seed=7, stream=1, step=3))       # reproducible
    assert keep_threshold(0.0) == 0


def test_cpu_plumbing_config_mnist_learns():
    """BASELINE.json's "MNIST 3-layer CNN single-process fit() on CPU (plumbing)" config."""
    x, y, xt, yt = synthetic_mnist(2000, 500)
    m = zoo.mnist_cnn(8, 16, 32, dropout=0.25, optimizer="Adadelta", device="cpu")
    h = m.fit(x, y, batch_size=128, epochs=2, validation_data=(xt, yt), verbose=0)
    assert h.history["val_acc"][-1] > 0.5


def test_profiling_hooks_and_resume(tmp_path):
    from cori_intml_examples_amd.models import load_model
    from cori_intml_examples_amd.utils.profiling import StepTimer, ThroughputLogger, trace
    x, y, _ = synthetic_rpv(64, size=16, seed=1)
    m = zoo.rpv_cnn((16, 16, 1), [4, 4, 4], [8], device="cpu")
    tl = ThroughputLogger()
    with trace(str(tmp_path / "t.json")):
        h = m.fit(x, y, batch_size=16, epochs=2, verbose=0, callbacks=[tl])
    assert (tmp_path / "t.json").exists()
    assert h.history["img_per_sec"][0] > 0 and len(tl.history) == 2
    assert h.history["img_per_sec_node"] == h.history["img_per_sec"]      # single process
    timer = StepTimer()
    with timer.region("eval"):
        m.evaluate(x, y, verbose=0)
    assert timer.summary()["eval"]["calls"] == 1
    # checkpoint / resume: reload and continue from epoch 2 (Keras initial_epoch)
    p = str(tmp_path / "ck.h5")
    m.save(p)
    m2 = load_model(p)
    h2 = m2.fit(x, y, batch_size=16, epochs=3, initial_epoch=2, verbose=0)
    assert h2.epoch == [2] and m2.optimizer.iterations == m.optimizer.iterations + 4


def test_reference_bf16_mode_runs_and_stays_close(monkeypatch):
    """executor_ref's bf16-faithful mode (the HIP step's storage roundings; the GPU tests'
    tight whole-step oracle): finite gradients within bf16 noise of the fp32 reference."""
    import torch
    x, y, _ = synthetic_rpv(32, size=16, seed=3)
    grads = []
    for tv in ("ref_bf16=0", "ref_bf16=1"):
        monkeypatch.setenv("INTML_TUNE", tv)
        set_random_seed(7)
        m = zoo.rpv_cnn((16, 16, 1), [4, 8, 8], [16], dropout=0.2, optimizer="Adam", lr=1e-3, device="cpu")
        assert m._executor.emulate_bf16 == (tv == "ref_bf16=1")
        ex = m._executor
        d = ex.upload(torch.tensor(x).to(torch.bfloat16).float().numpy(), y)
        ex.train_step(d, torch.arange(d.n), 0, d.n)
        grads.append(m.store.grad[:m.store.numel].clone())
    a, b = grads
    assert torch.isfinite(b).all() and not torch.equal(a, b)
    assert float((a - b).norm() / a.norm()) < 0.1
