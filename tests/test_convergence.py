"""Convergence equivalence at the benchmark geometry (VERDICT r2 "pin convergence, not only
single-step numerics").

The bf16 HIP training step must TRAIN like the fp32 reference over hundreds of steps, not
only match it for one: a learnable synthetic set (RPV: signal events carry more, narrower
jets; MNIST: class templates + noise), the benchmark's model / batch / optimizer, the same
initial weights, shuffle order and dropout masks (counter-based RNG shared by both
backends), 2 epochs x 16k samples.  The HIP ``val_loss`` must land within 5 % of the fp32
CPU reference's and both must beat chance clearly.  A 2-rank data-parallel run at the same
global batch (gloo data plane, both ranks on GPU 0) must land in the same band.

Reference: DistTrain_rpv.ipynb:267-300 (Adam, B=128, conv[16,32,64] fc[128], dropout 0.2),
DistTrain_mnist.ipynb:294-317 (32-64-128, Adadelta).  Parity with the reference's own
accuracies (0.9834 RPV, 0.9932 MNIST) needs their datasets and stays unpinned.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from cori_intml_examples_amd.apps import zoo
from cori_intml_examples_amd.io.datasets import synthetic_mnist, synthetic_rpv
from cori_intml_examples_amd.utils import set_random_seed

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

N_TRAIN, N_VALID, EPOCHS = 16384, 4096, 2
LABEL_NOISE = 0.1       # flipped labels: the loss plateaus near H(0.1) = 0.33 nats (RPV) instead
#                         of -> 0, so a 5 % band compares training, not rounding of ~1e-4 losses
OUT = os.path.join(ROOT, "gpurun_out")


class _Progress:
    """Epoch lines into gpurun_out/ (a long CPU reference run must not look silent)."""

    def __init__(self, tag):
        self.tag = tag

    def __call__(self, epoch, logs):
        if os.path.isdir(OUT):
            with open(os.path.join(OUT, "convergence_progress.txt"), "a") as f:
                f.write("%s epoch %d %s\n" % (self.tag, epoch, json.dumps({k: float(v) for k, v in logs.items()})))


def _rpv(device, w0=None):
    set_random_seed(11)
    m = zoo.rpv_cnn((64, 64, 3), conv_sizes=[16, 32, 64], fc_sizes=[128], dropout=0.2, optimizer="Adam",
                    lr=1e-3, device=device)
    if w0 is not None:
        m.set_weights(w0)
    return m


def _mnist(device, w0=None):
    set_random_seed(12)
    m = zoo.mnist_cnn(32, 64, 128, 0.25, 0.5, optimizer="Adadelta", lr=1.0, device=device)
    if w0 is not None:
        m.set_weights(w0)
    return m


def _fit(m, x, y, xv, yv, tag, bs=128, seed=5):
    from cori_intml_examples_amd.train import callbacks as cbks
    np.random.seed(seed)          # fit()'s shuffle order
    h = m.fit(x, y, batch_size=bs, epochs=EPOCHS, validation_data=(xv, yv), verbose=0,
              callbacks=[cbks.LambdaCallback(on_epoch_end=_Progress(tag))])
    return h.history


def _data(kind):
    rs = np.random.RandomState(31)
    if kind == "rpv":
        x, y, _ = synthetic_rpv(N_TRAIN + N_VALID, channels=3, seed=21)
        flip = rs.rand(len(y)) < LABEL_NOISE
        y = np.where(flip, 1.0 - y, y).astype(np.float32)
        return x[:N_TRAIN], y[:N_TRAIN], x[N_TRAIN:], y[N_TRAIN:]
    x, y, xv, yv = synthetic_mnist(N_TRAIN, N_VALID, seed=22)
    for t in (y, yv):
        flip = rs.rand(len(t)) < LABEL_NOISE
        lab = np.where(flip, rs.randint(0, 10, len(t)), t.argmax(1))
        t[:] = np.eye(10, dtype=np.float32)[lab]
    return x, y, xv, yv


@pytest.mark.timeout(900)
@pytest.mark.parametrize("kind", ["rpv", "mnist"])
def test_bf16_step_converges_like_fp32_reference(kind, tmp_path):
    build = _rpv if kind == "rpv" else _mnist
    x, y, xv, yv = _data(kind)
    ref = build("cpu")
    w0 = ref.get_weights()
    h_ref = _fit(ref, x, y, xv, yv, kind + " fp32-ref")
    hip = build("cuda:0", w0)
    h_hip = _fit(hip, x, y, xv, yv, kind + " hip")
    chance = np.log(2.0) if kind == "rpv" else np.log(10.0)
    vr, vh = h_ref["val_loss"][-1], h_hip["val_loss"][-1]
    rec = {"kind": kind, "ref": h_ref, "hip": h_hip}
    # evidence for the record (profiles/ is copied from gpurun_out by the round scripts)
    out = OUT
    if os.path.isdir(out):
        with open(os.path.join(out, "convergence_%s.json" % kind), "w") as f:
            json.dump(rec, f)
    assert vr < 0.75 * chance and vh < 0.75 * chance, rec      # both learned (noise floor ~0.5 chance)
    assert abs(vh - vr) <= 0.05 * vr, rec                       # same training, within 5 %
    assert abs(h_hip["val_acc"][-1] - h_ref["val_acc"][-1]) < 0.02, rec
    # DP: 2 ranks x 64 = the same global batch of 128, both on GPU 0: the RCCL-free xGMI plane
    # (NativeGradReducer, fused all-reduce + optimizer kernel in the step graph)
    np.savez(tmp_path / "data.npz", x=x, y=y, xv=xv, yv=yv)
    np.savez(tmp_path / "w0.npz", *w0)
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, PYTHONPATH=ROOT, INTML_DEVICE="cuda:0")
    for k in ("WORLD_SIZE", "RANK", "INTML_COMM", "INTML_DP_BACKEND"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "tests", "convergence_dp_worker.py"), kind, str(tmp_path)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    dp = json.load(open(tmp_path / "dp0.json"))
    rec["dp2"] = dp
    if os.path.isdir(out):
        with open(os.path.join(out, "convergence_%s.json" % kind), "w") as f:
            json.dump(rec, f)
    assert dp["reducer"] == "NativeGradReducer" and "xgmi" in dp["data_plane"], dp
    assert dp["val_loss"][-1] < 0.75 * chance, rec
    assert abs(dp["val_loss"][-1] - vr) <= 0.10 * vr, rec       # different sampling: wider band
