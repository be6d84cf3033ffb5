"""``python train_rpv.py [flags]`` -- distributed RPV training with the FoM protocol.
Under torchrun each rank drives one MI355X over RCCL."""
import _path  # noqa: F401
from cori_intml_examples_amd.apps.train_rpv import main

if __name__ == "__main__":
    main()
