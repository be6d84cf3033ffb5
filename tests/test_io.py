"""Native HDF5 module, RPV dataset files and Keras-HDF5 checkpoints (CPU).

Checks the layout of SURVEY.md Appendix B.1/B.2 and that save -> load round-trips the
weights, the optimizer slots and the step counter exactly (``rpv.py:100-101``,
``DistHPO_mnist.ipynb:540-542``)."""
import json
import os

import numpy as np
import pytest

from cori_intml_examples_amd.apps import zoo
from cori_intml_examples_amd.io import keras_h5
from cori_intml_examples_amd.io.datasets import load_dataset, load_file, make_synthetic_rpv_dir, synthetic_rpv
from cori_intml_examples_amd.io.h5 import H5File
from cori_intml_examples_amd.models import Sequential, load_model
from cori_intml_examples_amd.models.layers import Conv2D, Dense, Dropout, Flatten, MaxPooling2D
from cori_intml_examples_amd.train.callbacks import ModelCheckpoint


def test_h5lite_datasets_and_attrs(tmp_path):
    p = str(tmp_path / "a.h5")
    a = np.arange(60, dtype=np.float32).reshape(10, 3, 2)
    with H5File(p, "w") as f:
        f.create_group("g/h")
        f.write_dataset("g/h/x:0", a)
        f.write_dataset("ints", np.arange(5, dtype=np.int64))
        f.write_dataset("bytes", np.arange(7, dtype=np.uint8), gzip=4)
        f.attrs("/")["s"] = "héllo"
        f.attrs("g")["names"] = ["a", "bb", "ccc"]
        f.attrs("g/h")["num"] = np.asarray([1.5, 2.5])
        f.attrs("g/h")["scalar"] = np.asarray(3, dtype=np.int64)
    with H5File(p) as f:
        assert "g/h/x:0" in f and "nope" not in f
        assert f.kind("g") == "group" and f.kind("g/h/x:0") == "dataset"
        assert f.shape("g/h/x:0") == (10, 3, 2)
        np.testing.assert_array_equal(f.read_dataset("g/h/x:0"), a)
        np.testing.assert_array_equal(f.read_dataset("g/h/x:0", 4), a[:4])
        np.testing.assert_array_equal(f.read_dataset("g/h/x:0", 3, start=8), a[8:])
        np.testing.assert_array_equal(f.read_dataset("ints"), np.arange(5))
        np.testing.assert_array_equal(f.read_dataset("bytes"), np.arange(7, dtype=np.uint8))
        assert f.attrs("/")["s"] == "héllo"
        assert f.attrs("g")["names"] == ["a", "bb", "ccc"]
        np.testing.assert_array_equal(f.attrs("g/h")["num"], [1.5, 2.5])
        assert int(f.attrs("g/h")["scalar"]) == 3
        assert sorted(f.keys("/")) == ["bytes", "g", "ints"]
        with pytest.raises(KeyError):
            f.attrs("g")["missing"]
    with pytest.raises(RuntimeError):
        H5File(str(tmp_path / "missing.h5"))


def test_rpv_files_partial_read(tmp_path):
    d = make_synthetic_rpv_dir(str(tmp_path / "rpv"), 40, 20, 10, seed=3)
    with H5File(os.path.join(d, "train.h5")) as f:
        assert f.shape("all_events/hist") == (40, 64, 64)       # rpv.py:21 layout (no channel axis)
        assert f.shape("all_events/y") == (40,) and f.shape("all_events/weight") == (40,)
    x, y, w = load_file(os.path.join(d, "train.h5"), 25)
    assert x.shape == (25, 64, 64, 1) and y.shape == (25,) and w.shape == (25,)
    x0, y0, w0 = synthetic_rpv(40, seed=3)
    np.testing.assert_array_equal(x, x0[:25])
    np.testing.assert_array_equal(y, y0[:25])
    (xt, yt, wt), (xv, yv, wv), (xs, ys, ws) = load_dataset(d, 30, 20, 5)
    assert len(xt) == 30 and len(xv) == 20 and len(xs) == 5


def _small_rpv(opt):
    return zoo.rpv_cnn((16, 16, 1), conv_sizes=[4, 8, 8], fc_sizes=[16], optimizer=opt, device="cpu")


@pytest.mark.parametrize("opt", ["Adam", "Nadam", "Adadelta", "SGD", "RMSprop"])
def test_checkpoint_roundtrip_and_resume(tmp_path, opt):
    x, y, _ = synthetic_rpv(64, size=16, seed=1)
    m = _small_rpv(opt)
    m.fit(x, y, batch_size=16, epochs=1, verbose=0, shuffle=False)
    p = str(tmp_path / "m.h5")
    m.save(p)
    m2 = load_model(p)
    assert type(m2.optimizer).__name__ == opt
    assert m2.optimizer.iterations == m.optimizer.iterations == 4
    for a, b in zip(m.get_weights(), m2.get_weights()):
        np.testing.assert_array_equal(a, b)
    for a, b in zip(m._executor.optimizer_state(), m2._executor.optimizer_state()):
        np.testing.assert_array_equal(a.numpy(), b.numpy())
    assert m.evaluate(x, y, verbose=0) == m2.evaluate(x, y, verbose=0)
    # one more identical step on both (dropout masks depend on the model seed: align it)
    m2._executor.seed = m._executor.seed
    m.train_on_batch(x[:16], y[:16])
    m2.train_on_batch(x[:16], y[:16])
    for a, b in zip(m.get_weights(), m2.get_weights()):
        np.testing.assert_allclose(a, b, rtol=0, atol=1e-6)


def test_checkpoint_layout_matches_keras(tmp_path):
    m = Sequential(device="cpu")
    m.add(Conv2D(4, (3, 3), activation="relu", input_shape=(12, 12, 1)))
    m.add(MaxPooling2D(pool_size=(2, 2)))
    m.add(Dropout(0.25))
    m.add(Flatten())
    m.add(Dense(10, activation="softmax"))
    m.compile(loss="categorical_crossentropy", optimizer="Adam", metrics=["accuracy"])
    p = str(tmp_path / "s.h5")
    m.save(p)
    with H5File(p) as f:
        root = f.attrs("/")
        assert root["keras_version"] == "2.2.4" and root["backend"] == "tensorflow"
        mc = json.loads(root["model_config"])
        assert mc["class_name"] == "Sequential"
        assert [l["class_name"] for l in mc["config"]["layers"]] == ["Conv2D", "MaxPooling2D", "Dropout",
                                                                      "Flatten", "Dense"]
        tc = json.loads(root["training_config"])
        assert tc["optimizer_config"]["class_name"] == "Adam" and tc["loss"] == "categorical_crossentropy"
        assert f.attrs("model_weights")["layer_names"] == ["conv2d_1", "max_pooling2d_1", "dropout_1",
                                                           "flatten_1", "dense_1"]
        assert f.attrs("model_weights/conv2d_1")["weight_names"] == ["conv2d_1/kernel:0", "conv2d_1/bias:0"]
        assert f.attrs("model_weights/dropout_1")["weight_names"] == []
        assert f.shape("model_weights/conv2d_1/conv2d_1/kernel:0") == (3, 3, 1, 4)
        assert f.shape("model_weights/dense_1/dense_1/kernel:0") == (100, 10)
        wn = f.attrs("optimizer_weights")["weight_names"]
        assert wn[0] == "Adam/iterations:0" and len(wn) == 1 + 3 * 4


def test_save_load_weights_and_checkpoint_callback(tmp_path):
    x, y, _ = synthetic_rpv(32, size=16, seed=2)
    m = _small_rpv("Adam")
    p = str(tmp_path / "ck_{epoch:02d}.h5")
    m.fit(x, y, batch_size=16, epochs=2, verbose=0, validation_split=0.25,
          callbacks=[ModelCheckpoint(p)])
    assert os.path.exists(str(tmp_path / "ck_01.h5")) and os.path.exists(str(tmp_path / "ck_02.h5"))
    assert not [n for n in os.listdir(tmp_path) if n.startswith(".")]      # no temp files left
    w = str(tmp_path / "w.h5")
    m.save_weights(w)
    m2 = _small_rpv("Adam")
    m2.load_weights(w)
    for a, b in zip(m.get_weights(), m2.get_weights()):
        np.testing.assert_array_equal(a, b)
    m3 = keras_h5.load_model(str(tmp_path / "ck_02.h5"))
    for a, b in zip(m.get_weights(), m3.get_weights()):
        np.testing.assert_array_equal(a, b)
