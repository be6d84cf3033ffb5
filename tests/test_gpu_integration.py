"""GPU integration: checkpoint round-trip from the HIP executor, the train_rpv CLI on a
GPU, a farm engine pinned to the GPU, and the HIP data-parallel step with 2 ranks."""
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _flat(m):
    return np.concatenate([w.reshape(-1) for w in m.get_weights()])


def test_checkpoint_roundtrip_gpu(tmp_path):
    from cori_intml_examples_amd.apps import zoo
    from cori_intml_examples_amd.io.datasets import synthetic_rpv
    from cori_intml_examples_amd.models import load_model
    x, y, _ = synthetic_rpv(256, channels=3, seed=1)
    for opt in ("Adam", "Nadam"):
        m = zoo.rpv_cnn((64, 64, 3), [16, 32, 64], [128], dropout=0.2, optimizer=opt, device="cuda:0")
        assert type(m._executor).__name__ == "HipExecutor"
        m.fit(x, y, batch_size=64, epochs=1, verbose=0)
        p = str(tmp_path / ("m_%s.h5" % opt))
        m.save(p)
        m2 = load_model(p)
        assert type(m2._executor).__name__ == "HipExecutor"
        np.testing.assert_array_equal(_flat(m), _flat(m2))
        for a, b in zip(m._executor.optimizer_state(), m2._executor.optimizer_state()):
            assert bool((a == b).all())
        assert m.evaluate(x, y, verbose=0) == m2.evaluate(x, y, verbose=0)
        m2._executor.seed = m._executor.seed
        m.train_on_batch(x[:64], y[:64])
        m2.train_on_batch(x[:64], y[:64])
        np.testing.assert_allclose(_flat(m), _flat(m2), rtol=0, atol=1e-6)


def test_train_rpv_cli_gpu():
    env = dict(os.environ, PYTHONPATH=ROOT)
    env.pop("INTML_DEVICE", None)
    r = subprocess.run([sys.executable, "-m", "cori_intml_examples_amd.apps.train_rpv", "--n-train", "4096",
                        "--n-valid", "1024", "--n-epochs", "2", "--batch-size", "128", "--fom", "best",
                        "--channels", "3"], env=env, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "FoM:" in r.stdout and "Total params: 547,841" not in r.stdout   # 3-channel first conv
    assert "Total params: 548,129" in r.stdout


def _gpu_trial(n):
    import torch
    from cori_intml_examples_amd.apps.mlextras import IPyParallelLogger
    from cori_intml_examples_amd.apps.zoo import rpv_cnn
    from cori_intml_examples_amd.io.datasets import synthetic_rpv
    x, y, _ = synthetic_rpv(n, channels=3, seed=2)
    m = rpv_cnn((64, 64, 3), [16, 32, 64], [128], dropout=0.2)
    h = m.fit(x, y, batch_size=128, epochs=2, validation_split=0.25, verbose=0, callbacks=[IPyParallelLogger()])
    return {"device": str(m.device), "executor": type(m._executor).__name__, "hist": h.history,
            "visible": os.environ.get("HIP_VISIBLE_DEVICES"), "gpus": torch.cuda.device_count()}


def test_farm_engine_on_gpu():
    import cloudpickle
    cloudpickle.register_pickle_by_value(sys.modules[__name__])
    from cori_intml_examples_amd import farm
    cl = farm.start_cluster(1, cluster_id="gpu_pytest_%d" % os.getpid(), gpus=[0], timeout=300)
    try:
        with cl.client() as c:
            ar = c.load_balanced_view().apply(_gpu_trial, 1024)
            out = ar.get(600)
            assert out["executor"] == "HipExecutor" and out["device"].startswith("cuda")
            assert out["visible"] == "0" and out["gpus"] == 1
            assert len(out["hist"]["val_loss"]) == 2
            assert ar.data["status"] == "Ended Training"
    finally:
        cl.stop()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_hip_data_parallel_two_ranks(tmp_path):
    """2 ranks on GPU 0 through train_on_batch and fit() on the native reducer (ranks sharing
    a GPU select the RCCL-free xGMI plane themselves; no gloo override)."""
    env = dict(os.environ, PYTHONPATH=ROOT)
    for k in ("INTML_DEVICE", "INTML_DP_BACKEND", "INTML_COMM"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "dp_worker_gpu.py"), str(tmp_path)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    reps = [json.load(open(tmp_path / ("rank%d.json" % i))) for i in range(2)]
    assert reps[0]["w1"] == reps[1]["w1"] and reps[0]["wf"] == reps[1]["wf"]       # lockstep
    assert reps[0]["val_loss"] == reps[1]["val_loss"]
    assert reps[0]["rel_diff"] < 0.05, reps[0]["rel_diff"]      # bf16 half-batches vs one global batch
    for rep in reps:
        assert rep["reducer"] == "NativeGradReducer" and "xgmi" in rep["data_plane"], rep


def test_nested_hpo_dp_evaluation_gpu(tmp_path):
    """Nested HPO x DP (CrayHPO_rpv.ipynb:62-64,145-151): one Evaluator evaluation that is a
    2-rank torch.distributed.run train_rpv job on GPU through fit().  With >= 2 GPUs the slot
    is two distinct GPUs and the job votes on RCCL (numeric self-test); on a 1-GPU box both
    ranks share GPU 0 (the slot names it twice) and run the RCCL-free xGMI plane.  Either way
    the gradients go through the native captured reducer (NativeGradReducer)."""
    import torch
    from cori_intml_examples_amd import hpo
    n = torch.cuda.device_count()
    slots = [[0, 1]] if n >= 2 else [[0, 0]]
    ev = hpo.Evaluator("python -m cori_intml_examples_amd.apps.train_rpv --synthetic --n-epochs 1 "
                       "--n-train 2048 --n-valid 512 --fom best", gpus_per_eval=2, slots=slots,
                       timeout=240, cwd=ROOT, log_dir=str(tmp_path))
    foms = ev.evaluate([["--lr", "0.001"]])
    rec = ev.history[0]
    out = open(sorted(tmp_path.glob("eval*.out"))[0]).read()
    plane = "xgmi, ranks share GPU 0" if n < 2 else "rccl over 2 GPUs"
    assert rec["ok"] and np.isfinite(foms[0]), "%s: rc %s\n%s" % (plane, rec["rc"], out[-3000:])
    assert "rank 0/2" in out, out[-2000:]
    assert "gradient reducer NativeGradReducer:%s" % ("xgmi" if n < 2 else "rccl") in out, out[-2000:]


def test_train_rpv_cli_four_ranks_one_gpu(tmp_path):
    """The train_rpv CLI (train_rpv.py:37,55-79) as a 4-rank torchrun job through fit() on ONE
    GPU: the ranks select the RCCL-free xGMI plane (the fused all-reduce + Adam kernel, captured
    into the step graph), linear LR scaling, Horovod callbacks; every rank prints the same FoM."""
    env = dict(os.environ, PYTHONPATH=ROOT, HIP_VISIBLE_DEVICES="0")
    for k in ("INTML_DEVICE", "INTML_DP_BACKEND", "INTML_COMM", "WORLD_SIZE", "RANK"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           "-m", "cori_intml_examples_amd.apps.train_rpv", "--synthetic", "--n-epochs", "2",
           "--n-train", "4096", "--n-valid", "1024", "--lr-scaling", "linear", "--fom", "best"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=400, cwd=ROOT)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    # (four ranks print concurrently: their "FoM:" lines may interleave at the word level)
    import re
    foms = [float(v) for v in re.findall(r"FoM:\s*(\d[\d.eE+-]*\d)", r.stdout)]
    assert r.stdout.count("FoM:") == 4 and foms and len(set(foms)) == 1 and np.isfinite(foms[0]), out[-3000:]
    assert "gradient reducer NativeGradReducer:xgmi" in out, out[-3000:]
    assert "rank 3/4" in out, out[-2000:]


def test_dist_train_px_engines_gpu():
    """DistTrain_rpv through %%px on farm engines (DistTrain_mnist.ipynb:148,294-317,494):
    two engines pinned to GPU 0, hvd.init() inside the engines turns them into one 2-rank
    data-parallel job (engines sharing a GPU run the RCCL-free xGMI plane: the controller
    says so in their environment, so every rank picks the same plane), the HIP executor
    trains on the GPU through the native reducer and both engines end in lockstep."""
    from cori_intml_examples_amd import farm
    from cori_intml_examples_amd.farm import magics
    cl = farm.start_cluster(2, cluster_id="gpu_px_%d" % os.getpid(), gpus=[0, 0], timeout=300)
    try:
        with cl.client() as c:
            ar = magics.px(
                "import numpy as np\n"
                "from cori_intml_examples_amd.parallel import hvd\n"
                "from cori_intml_examples_amd.apps.rpv import build_model, train_model\n"
                "from cori_intml_examples_amd.io.datasets import synthetic_rpv\n"
                "hvd.init()\n"
                "x, y, _ = synthetic_rpv(2048, channels=1, seed=3)\n"
                "xv, yv, _ = synthetic_rpv(512, channels=1, seed=4)\n"
                "model = build_model(x.shape[1:], conv_sizes=[16, 32, 64], fc_sizes=[128], dropout=0.2,\n"
                "                    optimizer='Adam', lr=0.001 * hvd.size(), use_horovod=True)\n"
                "history = train_model(model, x, y, xv, yv, batch_size=128, n_epochs=2, use_horovod=True, verbose=0)\n"
                "wsum = float(sum(np.abs(w).sum() for w in model.get_weights()))\n"
                "dev = str(model.device); ex = type(model._executor).__name__; world = hvd.size()\n"
                "red = type(model._executor.reducer).__name__; plane = history.data_plane\n",
                client=c, verbose=False, block=True)
            dv = c[:]
            assert dv.pull("world") == [2, 2]
            assert dv.pull("red") == ["NativeGradReducer"] * 2, dv.pull("plane")
            assert all("xgmi" in p for p in dv.pull("plane")), dv.pull("plane")
            assert dv.pull("ex") == ["HipExecutor"] * 2 and all(d.startswith("cuda") for d in dv.pull("dev"))
            ws = dv.pull("wsum")
            assert ws[0] == ws[1], ws                                   # lockstep weights
            vl = dv.pull("history.history['val_loss']")
            assert len(vl[0]) == 2 and vl[0] == vl[1] and np.all(np.isfinite(vl[0])), vl
    finally:
        cl.stop()


def test_farm_engines_distinct_gpus_remapped(monkeypatch):
    """farm engines pinned to DISTINCT GPU indices (the one-engine-per-GPU layout
    of an 8-GPU node: no shared-GPU environment, every engine a one-rank-per-node RCCL
    candidate), rehearsed on one card by remapping the indices to GPU 0 only in the engines'
    HIP_VISIBLE_DEVICES.  %%px + hvd.init() over the two engines must come up collectively --
    RCCL refuses two ranks on one physical device, so the phased bring-up votes both ranks onto
    the RCCL-free plane -- and train in lockstep."""
    from cori_intml_examples_amd import farm
    from cori_intml_examples_amd.farm import magics
    monkeypatch.setenv("INTML_FARM_GPU_REMAP", "*:0")
    monkeypatch.setenv("INTML_RCCL_INIT_TIMEOUT", "30")
    cl = farm.start_cluster(2, cluster_id="gpu_remap_%d" % os.getpid(), gpus=[0, 1], timeout=300)
    try:
        with cl.client() as c:
            ar = magics.px(
                "import os\n"
                "import numpy as np\n"
                "from cori_intml_examples_amd.parallel import hvd\n"
                "from cori_intml_examples_amd.apps.rpv import build_model, train_model\n"
                "from cori_intml_examples_amd.io.datasets import synthetic_rpv\n"
                "shared_env = os.environ.get('INTML_COMM')\n"
                "st = hvd.init()\n"
                "x, y, _ = synthetic_rpv(1024, channels=1, seed=3)\n"
                "model = build_model(x.shape[1:], conv_sizes=[8, 16, 16], fc_sizes=[32], dropout=0.2,\n"
                "                    optimizer='Adam', lr=0.001 * hvd.size(), use_horovod=True)\n"
                "history = train_model(model, x, y, None, None, batch_size=64, n_epochs=2, use_horovod=True, verbose=0)\n"
                "wsum = float(sum(np.abs(w).sum() for w in model.get_weights()))\n"
                "world = hvd.size(); plane = history.data_plane; note = st.plane\n"
                "checks = [r['identical'] for r in history.dp_consistency]\n",
                client=c, verbose=False, block=True)
            dv = c[:]
            assert dv.pull("shared_env") == [None, None]          # the distinct-GPU environment
            assert dv.pull("world") == [2, 2]
            ws = dv.pull("wsum")
            assert ws[0] == ws[1], (ws, dv.pull("plane"), dv.pull("note"))
            assert dv.pull("checks") == [[True, True], [True, True]], dv.pull("checks")
            assert all("NativeGradReducer" in p for p in dv.pull("plane")), dv.pull("plane")
    finally:
        cl.stop()
