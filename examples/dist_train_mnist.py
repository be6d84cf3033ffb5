"""DistTrain_mnist workflow: SPMD data-parallel MNIST over the farm's engines (%%px).

Each engine is one rank on one MI355X; ``hvd.init()`` inside the px cell joins them into
one RCCL job (engine id == rank == GPU).  Same recipe as the notebook: 32-64-128 CNN,
``Adadelta(1.0 * hvd.size())`` + DistributedOptimizer, broadcast of the initial state,
batch 128, validation on the test set; afterwards every rank reports the same test score
(the reference's consistency check, ``DistTrain_mnist.ipynb:526-527``).
"""
import argparse

from common import connect, farm_args
from cori_intml_examples_amd.farm.magics import px


def main():
    p = farm_args(argparse.ArgumentParser(description=__doc__))
    p.add_argument("--epochs", type=int, default=8)
    p.add_argument("--batch-size", type=int, default=128)
    p.add_argument("--n-train", type=int, default=60000)
    a = p.parse_args()
    c, cl = connect(a)
    try:
        print("engines:", c.ids)
        px("""
import cori_intml_examples_amd.compat as _c; _c.install()
import keras, horovod.keras as hvd
from keras.models import Sequential
from keras.layers import Conv2D, MaxPooling2D, Dropout, Flatten, Dense
from cori_intml_examples_amd.apps.mnist import load_data
hvd.init()
print('rank', hvd.rank(), 'of', hvd.size())
""", client=c)
        px("""
x_train, y_train, x_test, y_test = load_data(n_train=%d)
x_train, y_train = x_train[:%d], y_train[:%d]
model = Sequential()
model.add(Conv2D(32, kernel_size=(3, 3), activation='relu', input_shape=(28, 28, 1)))
model.add(Conv2D(64, (3, 3), activation='relu'))
model.add(MaxPooling2D(pool_size=(2, 2)))
model.add(Dropout(0.25))
model.add(Flatten())
model.add(Dense(128, activation='relu'))
model.add(Dropout(0.5))
model.add(Dense(10, activation='softmax'))
opt = hvd.DistributedOptimizer(keras.optimizers.Adadelta(1.0 * hvd.size()))
model.compile(loss='categorical_crossentropy', optimizer=opt, metrics=['accuracy'])
if hvd.rank() == 0:
    model.summary()
history = model.fit(x_train, y_train, batch_size=%d, epochs=%d, verbose=2,
                    callbacks=[hvd.callbacks.BroadcastGlobalVariablesCallback(0)],
                    validation_data=(x_test, y_test))
score = model.evaluate(x_test, y_test, verbose=0)
print('Test loss:', score[0], 'Test accuracy:', score[1])
""" % (a.n_train, a.n_train, a.n_train, a.batch_size, a.epochs), client=c)
        scores = c[:].get("score")
        print("per-rank test scores:", scores)
        assert all(s == scores[0] for s in scores), "ranks diverged"
    finally:
        c.close()
        if cl:
            cl.stop()


if __name__ == "__main__":
    main()
