"""Model zoo: the three CNN families the reference trains.

  M1 ``mnist_cnn``      Conv(h1,valid)-Conv(h2)-MaxPool-Dropout-Flatten-Dense(h3)-Dropout-
                         Dense(10,softmax)  (mnist.py:44-59, DistTrain_mnist.ipynb:294-304)
  M2 ``rpv_cnn``        [Conv(c,same)+ReLU, MaxPool] x n - Dropout - Flatten -
                         [Dense(f)+ReLU, Dropout] x m - Dense(1, sigmoid)   (rpv.py:38-72)
  M3 ``rpv_legacy_cnn`` strided 4-conv + Dense(512) RPV model (Train_rpv.ipynb:205-219)
"""
from __future__ import annotations

from ..models import Conv2D, Dense, Dropout, Flatten, Input, MaxPooling2D, Model, Sequential
from .. import optim as optimizers


def _opt(optimizer, lr, use_horovod):
    if isinstance(optimizer, str):
        opt = getattr(optimizers, optimizer)(lr=lr) if lr is not None else optimizers.get(optimizer)
    else:
        opt = optimizer
    if use_horovod:
        from ..parallel import hvd
        opt = hvd.DistributedOptimizer(opt)
    return opt


def mnist_cnn(h1=4, h2=8, h3=32, dropout=0.5, dropout2=None, optimizer="Adadelta", lr=None,
              n_classes=10, input_shape=(28, 28, 1), use_horovod=False, device=None):
    m = Sequential(device=device)
    m.add(Conv2D(h1, (3, 3), activation="relu", input_shape=input_shape))
    m.add(Conv2D(h2, (3, 3), activation="relu"))
    m.add(MaxPooling2D(pool_size=(2, 2)))
    m.add(Dropout(dropout))
    m.add(Flatten())
    m.add(Dense(h3, activation="relu"))
    m.add(Dropout(dropout if dropout2 is None else dropout2))
    m.add(Dense(n_classes, activation="softmax"))
    m.compile(optimizer=_opt(optimizer, lr, use_horovod), loss="categorical_crossentropy",
              metrics=["accuracy"])
    return m


def rpv_cnn(input_shape, conv_sizes=(8, 16, 32), fc_sizes=(64,), dropout=0.5, optimizer="Adam", lr=0.001,
            use_horovod=False, device=None):
    inputs = Input(shape=input_shape)
    h = inputs
    for c in conv_sizes:
        h = Conv2D(c, kernel_size=(3, 3), activation="relu", padding="same")(h)
        h = MaxPooling2D(pool_size=(2, 2))(h)
    h = Dropout(dropout)(h)
    h = Flatten()(h)
    for f in fc_sizes:
        h = Dense(f, activation="relu")(h)
        h = Dropout(dropout)(h)
    outputs = Dense(1, activation="sigmoid")(h)
    model = Model(inputs=inputs, outputs=outputs, name="RPVClassifier", device=device)
    model.compile(optimizer=_opt(optimizer, lr, use_horovod), loss="binary_crossentropy", metrics=["accuracy"])
    return model


def rpv_legacy_cnn(input_shape=(64, 64, 1), optimizer="Adam", lr=None, h1=64, h2=128, h3=256, h4=256, h5=512,
                   use_horovod=False, device=None):
    inputs = Input(shape=input_shape)
    h = Conv2D(h1, kernel_size=(3, 3), activation="relu", strides=1, padding="same")(inputs)
    h = Conv2D(h2, kernel_size=(3, 3), activation="relu", strides=2, padding="same")(h)
    h = Conv2D(h3, kernel_size=(3, 3), activation="relu", strides=1, padding="same")(h)
    h = Conv2D(h4, kernel_size=(3, 3), activation="relu", strides=2, padding="same")(h)
    h = Flatten()(h)
    h = Dense(h5, activation="relu")(h)
    outputs = Dense(1, activation="sigmoid")(h)
    model = Model(inputs=inputs, outputs=outputs, name="RPVClassifier", device=device)
    model.compile(optimizer=_opt(optimizer, lr, use_horovod), loss="binary_crossentropy", metrics=["accuracy"])
    return model
