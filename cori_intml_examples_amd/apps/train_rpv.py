"""Distributed RPV classifier training CLI (``train_rpv.py:1-85``): the batch job
(``batch_scripts/train_rpv.sh``) and the HPO evaluator command
(``CrayHPO_rpv.ipynb:145``).  Same flags and defaults as ``train_rpv.py:16-31``; prints
the ``FoM: <float>`` line the HPO evaluators parse (``train_rpv.py:76-79``).

One rank per GPU:

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m cori_intml_examples_amd.apps.train_rpv --lr-scaling linear --fom best

Extra flags (not in the reference): ``--synthetic`` (auto-enabled when ``--input-dir``
has no ``train.h5``: synthetic events of the RPV schema), ``--channels``, ``--seed``,
``--verbose``, ``--shard`` / ``--replicate`` (data-parallel sampling: each rank reads a
disjoint shard, or -- the reference's semantics -- the full dataset with its own shuffle).
"""
from __future__ import annotations

import argparse
import os
import socket
import sys


def build_parser():
    p = argparse.ArgumentParser(description="RPV calorimeter-image CNN: data-parallel training on MI355X "
                                            "(one rank per GPU), prints the HPO figure of merit")
    # no site-specific default: $RPV_DATA_DIR, else ./data/atlas-rpv-images (synthetic if absent)
    p.add_argument("--input-dir", default=os.environ.get("RPV_DATA_DIR", os.path.join("data", "atlas-rpv-images")))
    p.add_argument("--n-train", type=int, default=64000)
    p.add_argument("--n-valid", type=int, default=32000)
    p.add_argument("--n-test", type=int, default=0)
    p.add_argument("--h1", type=int, default=16)
    p.add_argument("--h2", type=int, default=32)
    p.add_argument("--h3", type=int, default=64)
    p.add_argument("--h4", type=int, default=128)
    p.add_argument("--dropout", type=float, default=0.2)
    p.add_argument("--lr", type=float, default=0.001)
    p.add_argument("--lr-scaling", choices=["linear"])
    p.add_argument("--optimizer", default="Adam")
    p.add_argument("--batch-size", type=int, default=64)
    p.add_argument("--n-epochs", type=int, default=4)
    p.add_argument("--fom", choices=["best", "last"])
    # extensions
    p.add_argument("--synthetic", action="store_true")
    p.add_argument("--channels", type=int, default=1)
    p.add_argument("--seed", type=int, default=None)
    p.add_argument("--verbose", type=int, default=2)
    g = p.add_mutually_exclusive_group()
    g.add_argument("--shard", dest="shard", action="store_true", default=None)
    g.add_argument("--replicate", dest="shard", action="store_false")
    return p


def main(argv=None):
    args = build_parser().parse_args(argv)
    from ..parallel import hvd
    from ..utils import set_random_seed
    from .rpv import build_model, load_dataset, train_model

    st = hvd.init(shard_data=args.shard)
    print("[train_rpv] rank %d/%d (local %d) on %s, data plane %s" % (
        hvd.rank(), hvd.size(), hvd.local_rank(), socket.gethostname(),
        st.plane or ("rccl" if st.comm is not None else st.backend)))
    if args.seed is not None:
        set_random_seed(args.seed + hvd.rank())

    synthetic = args.synthetic or not os.path.exists(os.path.join(args.input_dir, "train.h5"))
    if synthetic and not args.synthetic:
        print("input dir %s has no train.h5: using synthetic RPV events" % args.input_dir)
    train_data, valid_data, test_data = load_dataset(args.input_dir, args.n_train, args.n_valid, args.n_test,
                                                     synthetic=synthetic, channels=args.channels)
    train_input, train_labels, _ = train_data
    valid_input, valid_labels, _ = valid_data
    test_input, test_labels, _ = test_data
    print("train shape:", train_input.shape, "Mean label:", train_labels.mean())
    print("valid shape:", valid_input.shape, "Mean label:", valid_labels.mean())
    if args.n_test > 0:
        print("test shape: ", test_input.shape, "Mean label:", test_labels.mean())

    lr = args.lr * hvd.size() if args.lr_scaling == "linear" else args.lr
    model = build_model(train_input.shape[1:], conv_sizes=[args.h1, args.h2, args.h3], fc_sizes=[args.h4],
                        dropout=args.dropout, optimizer=args.optimizer, lr=lr, use_horovod=True)
    if hvd.rank() == 0:
        model.summary()

    print("[train_rpv] %d epochs, batch %d per rank, lr %g" % (args.n_epochs, args.batch_size, lr))
    history = train_model(model, train_input=train_input, train_labels=train_labels, valid_input=valid_input,
                          valid_labels=valid_labels, batch_size=args.batch_size, n_epochs=args.n_epochs,
                          verbose=args.verbose, use_horovod=True)
    if hvd.rank() == 0 and getattr(history, "data_plane", None):
        print("[train_rpv] gradient reducer %s" % history.data_plane)
    if args.fom in ("best", "last"):
        from ..hpo.evaluator import figure_of_merit
        # one write per line: the ranks share the launcher's pipe, and print's separate writes
        # of "FoM:" and the value interleave across ranks
        sys.stdout.write("FoM: %s\n" % figure_of_merit(history.history["val_loss"], args.fom))
        sys.stdout.flush()
    sys.stdout.flush()

    if hvd.rank() == 0 and args.n_test > 0:
        score = model.evaluate(test_input, test_labels, verbose=2)
        print("Test loss:", score[0])
        print("Test accuracy:", score[1])
    hvd.shutdown()
    return history


if __name__ == "__main__":
    main()
