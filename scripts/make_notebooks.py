"""Generate ``notebooks/*.ipynb``: the reference's 11 workflow notebooks rebuilt on this
framework.  The cell text below is the source of truth; run

    python scripts/make_notebooks.py

after editing it.  Every notebook reads its problem sizes from ``NB_*`` environment
variables (defaults = the reference's sizes) so ``tests/test_notebooks.py`` executes all of
them headless at tiny sizes (``cori_intml_examples_amd.utils.nbrun``)."""
import json
import os
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "notebooks")


def md(s):
    return ("markdown", textwrap.dedent(s).strip("\n"))


def code(s):
    return ("code", textwrap.dedent(s).strip("\n"))


SIZES = code('''
    # Problem sizes: the reference's values by default; NB_* environment variables shrink
    # them (the headless CI run uses tiny ones).  NB_CPU=1 runs everything on CPU engines.
    import os
    def nb(name, default, cast=int):
        return cast(os.environ.get('NB_' + name, default))
    cpu_only = nb('CPU', 0) == 1
''')

FARM = code('''
    # Connect to the farm: a cluster started by examples/startCluster.sh (pass its id in
    # INTML_CLUSTER_ID), or start one here -- in Jupyter: %ipcluster -n 8
    import cori_intml_examples_amd.compat as compat; compat.install()
    import ipyparallel as ipp
    from cori_intml_examples_amd.farm import magics
    cluster_id = os.environ.get('INTML_CLUSTER_ID')
    if cluster_id is None:
        cluster_id = 'nb_%d' % os.getpid()
        magics.ipcluster('-n %d -J %s%s' % (n_engines, cluster_id, ' --cpu' if cpu_only else ''))
        __nb_cleanup__ = magics.stop_clusters
    c = ipp.Client(timeout=60, cluster_id=cluster_id)
    magics.set_client(c)
    print('Worker IDs:', c.ids)
''')

NOTEBOOKS = {}

NOTEBOOKS["DistTrain_mnist"] = [
    md('''
    # Distributed training: MNIST CNN, data parallel over the farm's engines
    One engine per MI355X; `hvd.init()` inside a `%%px` cell joins the engines into one
    data-parallel job (the gradient all-reduce runs on RCCL / the fused xGMI kernel over the
    GPUs' xGMI links).  Same recipe as the reference's `DistTrain_mnist`: 32-64-128 CNN,
    Adadelta with the learning rate scaled by the number of ranks, state broadcast from rank
    0, batch 128 per rank, the test set as validation data.
    '''),
    SIZES,
    code('''
    n_engines = nb('ENGINES', 8)
    batch_size = 128
    n_epochs = nb('EPOCHS', 8)
    n_train = nb('N_TRAIN', 60000)
    '''),
    FARM,
    code('''
    c[:].push(dict(batch_size=batch_size, n_epochs=n_epochs, n_train=n_train))
    '''),
    code('''
    %%px
    import cori_intml_examples_amd.compat as compat; compat.install()
    import keras
    import horovod.keras as hvd
    from keras.models import Sequential
    from keras.layers import Conv2D, MaxPooling2D, Dropout, Flatten, Dense
    from cori_intml_examples_amd.apps.mnist import load_data
    hvd.init()
    print('rank', hvd.rank(), 'of', hvd.size())
    '''),
    code('''
    %%px
    x_train, y_train, x_test, y_test = load_data(n_train=n_train)
    x_train, y_train = x_train[:n_train], y_train[:n_train]
    print('x_train shape:', x_train.shape, 'x_test shape:', x_test.shape)
    '''),
    code('''
    %%px
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
    '''),
    code('''
    %%px
    callbacks = [hvd.callbacks.BroadcastGlobalVariablesCallback(0)]
    history = model.fit(x_train, y_train, batch_size=batch_size, epochs=n_epochs, verbose=2,
                        callbacks=callbacks, validation_data=(x_test, y_test))
    '''),
    code('''
    %%px
    score = model.evaluate(x_test, y_test, verbose=0)
    print('Test loss:', score[0])
    print('Test accuracy:', score[1])
    '''),
    code('''
    # every rank holds the same weights: identical test scores
    scores = c[:].get('score')
    print(scores)
    assert all(s == scores[0] for s in scores)
    '''),
]

NOTEBOOKS["DistTrain_rpv"] = [
    md('''
    # Distributed training: ATLAS RPV calorimeter-image classifier
    Data-parallel RPV CNN ([16, 32, 64] convolutions, [128] dense) over the farm's engines,
    Adam with `lr = 0.001 * size`, batch 128 per rank; then the histories are pulled back and
    the test set is scored (accuracy, purity, efficiency), as in `DistTrain_rpv`.
    Synthetic events of the RPV schema are used when the HDF5 files are absent.
    '''),
    SIZES,
    code('''
    n_engines = nb('ENGINES', 8)
    input_dir = os.environ.get('RPV_DATA_DIR', 'data/atlas-rpv-images')
    n_train, n_valid, n_test = nb('N_TRAIN', 64000), nb('N_VALID', 32000), nb('N_TEST', 32000)
    conv_sizes, fc_sizes, dropout, optimizer = [16, 32, 64], [128], 0.2, 'Adam'
    batch_size, n_epochs = 128, nb('EPOCHS', 4)
    '''),
    FARM,
    code('''
    c[:].push(dict(input_dir=input_dir, n_train=n_train, n_valid=n_valid, n_test=n_test,
                   conv_sizes=conv_sizes, fc_sizes=fc_sizes, dropout=dropout, optimizer=optimizer,
                   batch_size=batch_size, n_epochs=n_epochs))
    '''),
    code('''
    %%px
    import cori_intml_examples_amd.compat as compat; compat.install()
    import horovod.keras as hvd
    from cori_intml_examples_amd.apps.rpv import load_dataset, build_model, train_model
    hvd.init()
    train, valid, test = load_dataset(input_dir, n_train, n_valid, n_test, synthetic=True)
    train_input, train_labels, train_weights = train
    valid_input, valid_labels, valid_weights = valid
    test_input, test_labels, test_weights = test
    print('train shape:', train_input.shape, 'Mean label:', train_labels.mean())
    '''),
    code('''
    %%px
    model = build_model(train_input.shape[1:], conv_sizes=conv_sizes, fc_sizes=fc_sizes, dropout=dropout,
                        optimizer=optimizer, lr=0.001 * hvd.size(), use_horovod=True)
    if hvd.rank() == 0:
        model.summary()
    history = train_model(model, train_input=train_input, train_labels=train_labels,
                          valid_input=valid_input, valid_labels=valid_labels,
                          batch_size=batch_size, n_epochs=n_epochs, use_horovod=True, verbose=2)
    '''),
    code('''
    epochs = c[0].get('history.epoch')
    histories = c[:].get('history.history')
    print('epochs:', epochs)
    print('rank-0 val_loss:', histories[0]['val_loss'])
    '''),
    code('''
    %%px
    test_output = model.predict(test_input).squeeze(-1)
    test_score = model.evaluate(test_input, test_labels, verbose=0)
    '''),
    code('''
    from cori_intml_examples_amd.apps.rpv import classification_report
    test_output = c[0].get('test_output')
    test_labels, test_weights = c[0].get('test_labels'), c[0].get('test_weights')
    print('Unweighted:', classification_report(test_labels, test_output))
    print('Weighted:  ', classification_report(test_labels, test_output, test_weights))
    '''),
]

NOTEBOOKS["Train_rpv"] = [
    md('''
    # Single-GPU RPV training (legacy 34.5M-parameter model)
    The reference's `Train_rpv` notebook on one GPU: load the RPV events, build the legacy
    strided CNN, train with Adam and report test metrics and per-epoch times.
    '''),
    SIZES,
    code('''
    import time
    import numpy as np
    import cori_intml_examples_amd.compat as compat; compat.install()
    from cori_intml_examples_amd.apps.rpv import load_dataset, train_model, classification_report
    from cori_intml_examples_amd.apps.zoo import rpv_legacy_cnn
    input_dir = os.environ.get('RPV_DATA_DIR', 'data/atlas-rpv-images')
    n_train, n_valid, n_test = nb('N_TRAIN', 64000), nb('N_VALID', 32000), nb('N_TEST', 32000)
    device = 'cpu' if cpu_only else None
    '''),
    code('''
    %%time
    train, valid, test = load_dataset(input_dir, n_train, n_valid, n_test, synthetic=True)
    print('train shape:', train[0].shape, 'valid shape:', valid[0].shape, 'test shape:', test[0].shape)
    '''),
    code('''
    model = rpv_legacy_cnn(train[0].shape[1:], device=device)
    model.summary()
    '''),
    code('''
    t0 = time.time()
    history = train_model(model, train[0], train[1], valid[0], valid[1], batch_size=128,
                          n_epochs=nb('EPOCHS', 4), verbose=2)
    print('%.1f us/sample' % ((time.time() - t0) / (len(history.epoch) * len(train[0])) * 1e6))
    '''),
    code('''
    test_output = model.predict(test[0], batch_size=1024).squeeze(-1)
    print('Unweighted:', classification_report(test[1], test_output))
    print('Weighted:  ', classification_report(test[1], test_output, test[2]))
    '''),
]

_HPO_MNIST_SPACE = code('''
    import numpy as np
    np.random.seed(0)
    h1 = np.random.choice([4, 8, 16, 32, 64], size=n_hpo_trials)
    h2 = np.random.choice([4, 8, 16, 32, 64], size=n_hpo_trials)
    h3 = np.random.choice([8, 16, 32, 64, 128], size=n_hpo_trials)
    dropout = np.random.rand(n_hpo_trials)
    optimizer = np.random.choice(['Adadelta', 'Adam', 'Nadam'], size=n_hpo_trials)
    for i in range(n_hpo_trials):
        print('Trial %i: %i-%i-%i dropout %.3f %s' % (i, h1[i], h2[i], h3[i], dropout[i], optimizer[i]))
''')

_BUILD_TRAIN_MNIST = code('''
    def build_and_train(h1, h2, h3, dropout, optimizer, n_epochs, n_train, checkpoint_file=None, verbose=0):
        """One trial on one engine (imports inside: the function is shipped to the engines)."""
        from cori_intml_examples_amd.apps.mnist import load_data, build_model
        from cori_intml_examples_amd.apps.mlextras import IPyParallelLogger
        from cori_intml_examples_amd.train.callbacks import ModelCheckpoint
        x_train, y_train, _, _ = load_data(n_train=n_train)
        model = build_model(h1=int(h1), h2=int(h2), h3=int(h3), dropout=float(dropout), optimizer=str(optimizer))
        callbacks = [IPyParallelLogger()]
        if checkpoint_file is not None:
            callbacks.append(ModelCheckpoint(checkpoint_file))
        history = model.fit(x_train[:n_train], y_train[:n_train], batch_size=128, epochs=n_epochs,
                            validation_split=0.17, callbacks=callbacks, verbose=verbose)
        return history.history
''')

NOTEBOOKS["DistHPO_mnist"] = [
    md('''
    # Distributed random-search HPO: MNIST
    32 random trials of the MNIST CNN (layer widths, dropout, optimizer), load-balanced over
    the farm's engines (one trial per MI355X at a time), then the best trial's checkpoint is
    reloaded and scored on the test set -- the reference's `DistHPO_mnist`.
    '''),
    SIZES,
    code('''
    import tempfile
    n_engines = nb('ENGINES', 8)
    n_hpo_trials = nb('TRIALS', 32)
    n_epochs = nb('EPOCHS', 16)
    n_train = nb('N_TRAIN', 60000)
    checkpoint_dir = tempfile.mkdtemp(prefix='mnist_hpo_')
    '''),
    _HPO_MNIST_SPACE,
    FARM,
    _BUILD_TRAIN_MNIST,
    code('''
    lv = c.load_balanced_view()
    results = [lv.apply(build_and_train, h1[i], h2[i], h3[i], dropout[i], optimizer[i], n_epochs, n_train,
                        checkpoint_file=os.path.join(checkpoint_dir, 'model_%i.h5' % i))
               for i in range(n_hpo_trials)]
    '''),
    code('''
    lv.wait(results)
    print('Tasks completed: %i / %i' % (sum(ar.ready() for ar in results), len(results)))
    histories = [ar.get() for ar in results]
    runtimes = np.array([(ar.completed - ar.started).total_seconds() for ar in results])
    print('runtime per trial: mean %.1f s' % runtimes.mean())
    '''),
    code('''
    best_scores = np.array([max(h['val_acc']) for h in histories])
    for i in best_scores.argsort()[::-1][:5]:
        print('trial %i: %i-%i-%i dropout %.3f %s  best val_acc %.4f' %
              (i, h1[i], h2[i], h3[i], dropout[i], optimizer[i], best_scores[i]))
    '''),
    code('''
    import keras
    from cori_intml_examples_amd.apps.mnist import load_data
    _, _, x_test, y_test = load_data(n_train=n_train)
    i = best_scores.argmax()
    model = keras.models.load_model(os.path.join(checkpoint_dir, 'model_%i.h5' % i))
    score = model.evaluate(x_test, y_test, verbose=0)
    print('Best model test loss %.4f accuracy %.4f' % (score[0], score[1]))
    '''),
]

_RPV_SPACE = code('''
    import numpy as np
    np.random.seed(0)
    h1 = np.random.choice([4, 8, 16, 32, 64], size=n_hpo_trials)
    h2 = np.random.choice([4, 8, 16, 32, 64], size=n_hpo_trials)
    h3 = np.random.choice([8, 16, 32, 64, 128], size=n_hpo_trials)
    conv_sizes = np.stack([h1, h2, h3], axis=1)
    fc_sizes = np.random.choice([32, 64, 128, 256], size=(n_hpo_trials, 1))
    lr = np.random.choice([0.0001, 0.001, 0.01], size=n_hpo_trials)
    dropout = np.random.rand(n_hpo_trials)
    optimizer = np.random.choice(['Adadelta', 'Adam', 'Nadam'], size=n_hpo_trials)
''')

_BUILD_TRAIN_RPV = code('''
    def build_and_train(input_dir, n_train, n_valid, conv_sizes, fc_sizes, dropout, optimizer, lr,
                        batch_size, n_epochs, checkpoint_file=None, verbose=0):
        """One RPV trial on one engine; streams its epochs to the notebook."""
        from cori_intml_examples_amd.apps.rpv import build_model, train_model, load_dataset
        from cori_intml_examples_amd.apps.mlextras import IPyParallelLogger
        train, valid, _ = load_dataset(input_dir, n_train, n_valid, 0, synthetic=True)
        model = build_model(train[0].shape[1:], conv_sizes=[int(v) for v in conv_sizes],
                            fc_sizes=[int(v) for v in fc_sizes], dropout=float(dropout),
                            optimizer=str(optimizer), lr=float(lr))
        history = train_model(model, train[0], train[1], valid[0], valid[1], batch_size=batch_size,
                              n_epochs=n_epochs, checkpoint_file=checkpoint_file,
                              callbacks=[IPyParallelLogger()], verbose=verbose)
        return history.history
''')

_RPV_ANALYSIS = [
    code('''
    best_scores = np.array([max(h['val_acc']) for h in histories])
    for i in best_scores.argsort()[::-1][:5]:
        print('trial %i conv %s fc %s dropout %.3f opt %s lr %.4f: best val_acc %.4f' %
              (i, conv_sizes[i], fc_sizes[i], dropout[i], optimizer[i], lr[i], best_scores[i]))
    '''),
    code('''
    import keras
    from cori_intml_examples_amd.apps.rpv import load_dataset, classification_report
    _, _, (test_input, test_labels, test_weights) = load_dataset(input_dir, 0, 0, n_test, synthetic=True)
    i = best_scores.argmax()
    model = keras.models.load_model(os.path.join(checkpoint_dir, 'model_%i.h5' % i))
    test_output = model.predict(test_input).squeeze(-1)
    print('Unweighted:', classification_report(test_labels, test_output))
    print('Weighted:  ', classification_report(test_labels, test_output, test_weights))
    '''),
]

NOTEBOOKS["DistHPO_rpv"] = [
    md('''
    # Distributed random-search HPO: RPV classifier
    Conv / dense widths, learning rate, dropout and optimizer sampled at random; trials are
    load-balanced over the farm; per-trial runtimes, the top-5 and a test evaluation of the
    best checkpoint -- the reference's `DistHPO_rpv`.
    '''),
    SIZES,
    code('''
    import tempfile
    n_engines = nb('ENGINES', 8)
    input_dir = os.environ.get('RPV_DATA_DIR', 'data/atlas-rpv-images')
    n_train, n_valid, n_test = nb('N_TRAIN', 64000), nb('N_VALID', 32000), nb('N_TEST', 32000)
    n_hpo_trials = nb('TRIALS', 32)
    batch_size, n_epochs = 64, nb('EPOCHS', 16)
    checkpoint_dir = tempfile.mkdtemp(prefix='rpv_hpo_')
    '''),
    _RPV_SPACE,
    FARM,
    _BUILD_TRAIN_RPV,
    code('''
    lv = c.load_balanced_view()
    results = []
    for i in range(n_hpo_trials):
        results.append(lv.apply(build_and_train, input_dir, n_train, n_valid, conv_sizes=conv_sizes[i],
                                fc_sizes=fc_sizes[i], dropout=dropout[i], optimizer=optimizer[i], lr=lr[i],
                                batch_size=batch_size, n_epochs=n_epochs,
                                checkpoint_file=os.path.join(checkpoint_dir, 'model_%i.h5' % i)))
    lv.wait(results)
    histories = [ar.get() for ar in results]
    runtimes = np.array([(ar.completed - ar.started).total_seconds() for ar in results])
    print('Tasks completed: %i / %i, runtime per trial mean %.1f s' % (len(histories), n_hpo_trials, runtimes.mean()))
    '''),
] + _RPV_ANALYSIS

NOTEBOOKS["DistWidgetHPO_mnist"] = [
    md('''
    # Random-search HPO with a live dashboard: MNIST
    `ParamSpanWidget` submits one trial per parameter row, streams every epoch
    (`IPyParallelLogger`) into a table and per-trial training curves, and offers Stop /
    Restart per trial; in Jupyter with ipywidgets/bqplot it renders the interactive widget,
    headless it renders text.  The reference's analysis cells after the widget (broken there:
    `psw.model_runs`) work on `psw.results`.
    '''),
    SIZES,
    code('''
    from functools import partial
    n_engines = nb('ENGINES', 8)
    n_hpo_trials = nb('TRIALS', 8)
    n_epochs = nb('EPOCHS', 16)
    n_train = nb('N_TRAIN', 60000)
    '''),
    _HPO_MNIST_SPACE,
    FARM,
    _BUILD_TRAIN_MNIST,
    code('''
    from cori_intml_examples_amd.widgets import ModelPlot, ParamSpanWidget
    train_func = partial(build_and_train, n_epochs=n_epochs, n_train=n_train)
    plot_func = partial(ModelPlot, y=['loss', 'acc', 'val_loss', 'val_acc'], x='epoch', xlim=[0, n_epochs])
    hpo_params = dict(h1=h1, h2=h2, h3=h3, dropout=dropout, optimizer=optimizer)
    psw = ParamSpanWidget(compute_func=train_func, vis_func=plot_func, params=hpo_params, ipp_cluster_id=cluster_id)
    psw.submit_computations()
    psw
    '''),
    code('''
    psw.wait()
    print(psw.render())
    '''),
    code('''
    histories = [ar.get() for ar in psw.model_runs]
    best_scores = np.array([max(h['val_acc']) for h in histories])
    i = best_scores.argmax()
    print('best trial %i: %i-%i-%i dropout %.3f %s  val_acc %.4f' %
          (i, h1[i], h2[i], h3[i], dropout[i], optimizer[i], best_scores[i]))
    '''),
]

NOTEBOOKS["DistWidgetHPO_rpv"] = [
    md('''
    # Random-search HPO with a live dashboard: RPV classifier
    RPV trials (conv / dense widths, dropout, optimizer, learning rate) streamed live to the
    dashboard -- per-engine GPU / HBM use included -- then the analysis that was broken in
    the reference's `DistWidgetHPO_rpv`: best / worst trial, top-5 and a test evaluation of
    the best checkpoint.
    '''),
    SIZES,
    code('''
    import tempfile
    from functools import partial
    n_engines = nb('ENGINES', 8)
    input_dir = os.environ.get('RPV_DATA_DIR', 'data/atlas-rpv-images')
    n_train, n_valid, n_test = nb('N_TRAIN', 64000), nb('N_VALID', 32000), nb('N_TEST', 32000)
    n_hpo_trials = nb('TRIALS', 8)
    batch_size, n_epochs = 64, nb('EPOCHS', 16)
    checkpoint_dir = tempfile.mkdtemp(prefix='rpv_widget_hpo_')
    '''),
    _RPV_SPACE,
    FARM,
    code('''
    def build_and_train(input_dir, n_train, n_valid, conv_sizes, fc_sizes, dropout, optimizer, lr,
                        batch_size, n_epochs, trial_index, checkpoint_dir, verbose=0):
        from cori_intml_examples_amd.apps.rpv import build_model, train_model, load_dataset
        from cori_intml_examples_amd.apps.mlextras import IPyParallelLogger
        train, valid, _ = load_dataset(input_dir, n_train, n_valid, 0, synthetic=True)
        model = build_model(train[0].shape[1:], conv_sizes=[int(v) for v in conv_sizes],
                            fc_sizes=[int(v) for v in fc_sizes], dropout=float(dropout),
                            optimizer=str(optimizer), lr=float(lr))
        history = train_model(model, train[0], train[1], valid[0], valid[1], batch_size=batch_size,
                              n_epochs=n_epochs, callbacks=[IPyParallelLogger()], verbose=verbose,
                              checkpoint_file=os.path.join(checkpoint_dir, 'model_%i.h5' % trial_index))
        return history.history
    '''),
    code('''
    from cori_intml_examples_amd.widgets import ModelPlot, ParamSpanWidget
    train_func = partial(build_and_train, input_dir=input_dir, n_train=n_train, n_valid=n_valid,
                         batch_size=batch_size, n_epochs=n_epochs, checkpoint_dir=checkpoint_dir)
    plot_func = partial(ModelPlot, y=['loss', 'acc', 'val_loss', 'val_acc'], x='epoch', xlim=[0, n_epochs],
                        xlabel='epochs', ylabel='training metrics')
    hpo_params = dict(conv_sizes=list(conv_sizes), fc_sizes=list(fc_sizes), dropout=dropout, optimizer=optimizer,
                      lr=lr, trial_index=list(range(n_hpo_trials)))
    psw = ParamSpanWidget(compute_func=train_func, vis_func=plot_func, params=hpo_params, ipp_cluster_id=cluster_id)
    psw.submit_computations()
    psw
    '''),
    code('''
    psw.wait()
    print(psw.render())
    histories = [ar.get() for ar in psw.model_runs]
    last_scores = np.array([h['val_acc'][-1] for h in histories])
    '''),
    code('''
    best_scores = np.array([max(h['val_acc']) for h in histories])
    for name, i in (('best', best_scores.argmax()), ('worst', best_scores.argmin())):
        print('%s: trial %i conv %s fc %s dropout %.3f opt %s lr %.4f: last val_acc %.4f best %.4f' %
              (name, i, conv_sizes[i], fc_sizes[i], dropout[i], optimizer[i], lr[i], last_scores[i], best_scores[i]))
    '''),
] + _RPV_ANALYSIS[1:]

NOTEBOOKS["CrayHPO_mnist"] = [
    md('''
    # Genetic HPO (Cray-HPO style): MNIST
    `hpo.Params` / `hpo.Evaluator` / `hpo.genetic.Optimizer`: every evaluation runs the MNIST
    training CLI on one GPU slot of the node and reports its figure of merit; demes evolve
    with migration and the per-generation log is written -- the reference's `CrayHPO_mnist`
    (whose `train.py` was missing; `apps.train_mnist` is that script).
    '''),
    SIZES,
    code('''
    import sys
    import cori_intml_examples_amd.compat as compat; compat.install()
    import crayai.hpo as hpo
    params = hpo.Params([['--h1', 16, (4, 64)],
                         ['--h2', 32, (4, 64)],
                         ['--h3', 64, (8, 128)],
                         ['--dropout', 0.5, (0., 1.)],
                         ['--optimizer', 'Adadelta', ['Adadelta', 'Adam', 'Nadam']]])
    n_epochs, n_train = nb('EPOCHS', 8), nb('N_TRAIN', 60000)
    cmd = '%s -m cori_intml_examples_amd.apps.train_mnist --epochs %d --n-train %d' % (sys.executable, n_epochs, n_train)
    evaluator = hpo.Evaluator(cmd, verbose=True, **({'cpu_slots': 2, 'gpus': []} if cpu_only else {}))
    print(evaluator)
    '''),
    code('''
    optimizer = hpo.genetic.Optimizer(evaluator, generations=nb('GENERATIONS', 16), num_demes=nb('DEMES', 4),
                                      pop_size=nb('POP', 4), mutation_rate=0.05, crossover_rate=0.33,
                                      verbose=True, log_fn='mnist_hpo.log')
    best = optimizer.optimize(params)
    print('best FoM', optimizer.best_fom, best)
    '''),
    code('''
    print(open('mnist_hpo.log').read()[:2000])
    '''),
]

NOTEBOOKS["CrayHPO_rpv"] = [
    md('''
    # Genetic HPO over data-parallel RPV trainings (HPO x DP)
    Each evaluation is itself a data-parallel `train_rpv` run over `gpus_per_eval` MI355X
    (one rank per GPU, its own RCCL communicator), several evaluations at a time on the
    node -- the reference's `CrayHPO_rpv` ran 8 concurrent 4-node Horovod evaluations.
    '''),
    SIZES,
    code('''
    import sys
    import cori_intml_examples_amd.compat as compat; compat.install()
    import crayai.hpo as hpo
    gpus_per_eval = nb('GPUS_PER_EVAL', 4)
    train_args = os.environ.get('NB_TRAIN_ARGS', '')
    cmd = '%s -m cori_intml_examples_amd.apps.train_rpv --n-epochs %d --fom best %s' % (
        sys.executable, nb('EPOCHS', 4), train_args)
    evaluator = hpo.Evaluator(cmd, gpus_per_eval=gpus_per_eval, verbose=True,
                              **({'cpu_slots': 2, 'gpus': []} if cpu_only else {}))
    print(evaluator)
    '''),
    code('''
    params = hpo.Params([['--h1', 16, (4, 64)],
                         ['--h2', 32, (4, 64)],
                         ['--h3', 64, (8, 128)],
                         ['--h4', 128, (32, 256)],
                         ['--dropout', 0.2, (0., 1.)],
                         ['--optimizer', 'Adam', ['Adam', 'Nadam', 'Adadelta']],
                         ['--lr', 0.001, [0.1, 0.01, 0.001, 0.0001, 0.00001]]])
    optimizer = hpo.genetic.Optimizer(evaluator, generations=nb('GENERATIONS', 4), num_demes=nb('DEMES', 4),
                                      pop_size=nb('POP', 8), mutation_rate=0.05, crossover_rate=0.33,
                                      verbose=True, log_fn='rpv_hpo.log')
    '''),
    code('''
    %%time
    best = optimizer.optimize(params)
    print('best FoM', optimizer.best_fom, best)
    '''),
    code('''
    import glob
    for f in sorted(glob.glob('Deme*_rpv_hpo.log'))[:2]:
        print(f, open(f).read()[:500])
    '''),
]

NOTEBOOKS["GridSearchCV_mnist"] = [
    md('''
    # k-fold grid search with the scikit-learn wrapper: MNIST
    `KerasClassifier(build_fn)` + `GridSearchCV` over layer widths and dropout, 3 folds --
    the reference's `GridSearchCV_mnist`.
    '''),
    SIZES,
    code('''
    import pandas as pd
    import cori_intml_examples_amd.compat as compat; compat.install()
    from keras.wrappers.scikit_learn import KerasClassifier
    from sklearn.model_selection import GridSearchCV
    from cori_intml_examples_amd.apps.mnist import load_data
    from cori_intml_examples_amd.apps.zoo import mnist_cnn
    n_train, n_epochs = nb('N_TRAIN', 40000), nb('EPOCHS', 16)
    x_train, y_train, x_test, y_test = load_data(n_train=n_train)
    x_train, y_train = x_train[:n_train], y_train[:n_train]
    def build_model(h1=4, h2=8, h3=32, dropout=0.5):
        return mnist_cnn(h1=h1, h2=h2, h3=h3, dropout=dropout, optimizer='Adadelta',
                         device='cpu' if cpu_only else None)
    '''),
    code('''
    param_grid = dict(h1=[8, 16, 32], h2=[16, 32], h3=[16, 32], dropout=[0., 0.25, 0.5])
    if os.environ.get('NB_SMALL_GRID'):
        param_grid = dict(h1=[8, 16], dropout=[0.25])
    gs = GridSearchCV(KerasClassifier(build_fn=build_model, batch_size=128, epochs=n_epochs, verbose=0),
                      param_grid, cv=3, verbose=2)
    gs.fit(x_train, y_train)
    '''),
    code('''
    res = pd.DataFrame(gs.cv_results_)
    print(res[['params', 'mean_test_score', 'std_test_score', 'mean_fit_time']].to_string())
    print('best:', gs.best_params_, 'test accuracy:', gs.best_estimator_.score(x_test, y_test))
    '''),
]

NOTEBOOKS["HPO_mnist"] = [
    md('''
    # Serial random-search HPO: MNIST
    The single-process version of the random search (one trial after the other in this
    kernel, on one GPU) -- the reference's `HPO_mnist`.
    '''),
    SIZES,
    code('''
    import numpy as np
    import cori_intml_examples_amd.compat as compat; compat.install()
    from cori_intml_examples_amd.apps.mnist import load_data, build_model
    n_hpo_trials, n_epochs, n_train = nb('TRIALS', 16), nb('EPOCHS', 16), nb('N_TRAIN', 60000)
    x_train, y_train, x_test, y_test = load_data(n_train=n_train)
    np.random.seed(0)
    h1 = np.random.choice([4, 8, 16, 32, 64], size=n_hpo_trials)
    h2 = np.random.choice([4, 8, 16, 32, 64], size=n_hpo_trials)
    h3 = np.random.choice([8, 16, 32, 64, 128], size=n_hpo_trials)
    dropout = np.random.rand(n_hpo_trials)
    '''),
    code('''
    histories, models = [], []
    for i in range(n_hpo_trials):
        print('Trial %i: %i-%i-%i dropout %.3f' % (i, h1[i], h2[i], h3[i], dropout[i]))
        model = build_model(h1=int(h1[i]), h2=int(h2[i]), h3=int(h3[i]), dropout=float(dropout[i]),
                            device='cpu' if cpu_only else None)
        h = model.fit(x_train[:n_train], y_train[:n_train], batch_size=128, epochs=n_epochs,
                      validation_split=0.17, verbose=0)
        histories.append(h.history)
        models.append(model)
    '''),
    code('''
    best_scores = np.array([max(h['val_acc']) for h in histories])
    i = best_scores.argmax()
    score = models[i].evaluate(x_test, y_test, verbose=0)
    print('best trial %i val_acc %.4f, test loss %.4f accuracy %.4f' % (i, best_scores[i], score[0], score[1]))
    '''),
]


def write(name, cells):
    nb = {"cells": [], "metadata": {"kernelspec": {"display_name": "Python 3", "language": "python",
                                                   "name": "python3"},
                                    "language_info": {"name": "python"}},
          "nbformat": 4, "nbformat_minor": 4}
    for kind, src in cells:
        lines = src.split("\n")
        source = [l + "\n" for l in lines[:-1]] + [lines[-1]]
        cell = {"cell_type": kind, "metadata": {}, "source": source}
        if kind == "code":
            cell.update(execution_count=None, outputs=[])
        nb["cells"].append(cell)
    path = os.path.join(OUT, name + ".ipynb")
    with open(path, "w") as f:
        json.dump(nb, f, indent=1)
        f.write("\n")
    return path


def main():
    os.makedirs(OUT, exist_ok=True)
    for name, cells in NOTEBOOKS.items():
        print("wrote", write(name, cells))


if __name__ == "__main__":
    main()
