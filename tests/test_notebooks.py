"""Every workflow notebook (``notebooks/*.ipynb``, the reference's 11 drivers rebuilt on
this framework) executes headless end to end at tiny sizes on CPU engines, through the
notebook runner (``utils/nbrun.py``: ``%%px`` -> farm, ``%%time``, line magics).  The
notebooks on disk must also match their generator (``scripts/make_notebooks.py``)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NB = os.path.join(ROOT, "notebooks")

TINY = {"NB_CPU": "1", "NB_ENGINES": "2", "NB_EPOCHS": "1", "NB_N_TRAIN": "256", "NB_N_VALID": "64",
        "NB_N_TEST": "64", "NB_TRIALS": "2", "NB_GENERATIONS": "1", "NB_DEMES": "2", "NB_POP": "2",
        "NB_GPUS_PER_EVAL": "2", "NB_SMALL_GRID": "1",
        "NB_TRAIN_ARGS": "--n-train 128 --n-valid 64 --batch-size 32 --h1 4 --h2 4 --h3 8 --h4 16"}

NOTEBOOKS = ["DistTrain_mnist", "DistTrain_rpv", "Train_rpv", "DistHPO_mnist", "DistHPO_rpv",
             "DistWidgetHPO_mnist", "DistWidgetHPO_rpv", "CrayHPO_mnist", "CrayHPO_rpv", "GridSearchCV_mnist",
             "HPO_mnist"]


def test_notebooks_match_generator(tmp_path):
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_notebooks", os.path.join(ROOT, "scripts", "make_notebooks.py"))
    mk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mk)
    assert sorted(mk.NOTEBOOKS) == sorted(NOTEBOOKS)
    mk.OUT = str(tmp_path)
    for name, cells in mk.NOTEBOOKS.items():
        fresh = json.load(open(mk.write(name, cells)))
        on_disk = json.load(open(os.path.join(NB, name + ".ipynb")))
        assert fresh == on_disk, "%s.ipynb is stale: run python scripts/make_notebooks.py" % name


def test_translate_magics():
    from cori_intml_examples_amd.utils.nbrun import translate
    assert translate("%%px\nx = 1").startswith("__nb_px__('x = 1', targets='all', block=True)")
    assert "targets=[0, 1]" in translate("%%px --targets 0:2\nx = 1")
    assert "Wall time" in translate("%%time\ny = 2")
    assert translate("%matplotlib notebook\nz = 3") == "pass\nz = 3"
    assert translate("%%bash\nls", skip_shell=True) == ""


@pytest.mark.parametrize("name", NOTEBOOKS)
def test_notebook_runs_headless(name, tmp_path):
    env = dict(os.environ, INTML_DEVICE="cpu", OMP_NUM_THREADS="2", PYTHONPATH=ROOT, **TINY)
    env.pop("INTML_CLUSTER_ID", None)
    r = subprocess.run([sys.executable, "-m", "cori_intml_examples_amd.utils.nbrun",
                        os.path.join(NB, name + ".ipynb")], env=env, capture_output=True, text=True,
                       timeout=900, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "notebook finished" in r.stdout
