"""``import ipcluster_magics`` registers ``%ipcluster`` (and ``%%px``) in IPython."""
import _path  # noqa: F401
from cori_intml_examples_amd.farm.magics import ipcluster, load_ipython_extension, px  # noqa: F401
