"""Host sanitizers over the native C++ that parses user files (SURVEY.md §5 race / memory
error detection): the HDF5 module built with AddressSanitizer + UBSan runs the HDF5 tests.

The child process preloads the ASan runtime (prepended to any existing preload list) and
swaps the sanitized ``_h5lite`` in for the in-tree one before the package imports it; any
ASan/UBSan report aborts the child.  CPU only -- GPU sanitizers are not available."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import importlib.util, sys
spec = importlib.util.spec_from_file_location("cori_intml_examples_amd._h5lite", sys.argv[1])
mod = importlib.util.module_from_spec(spec)
spec.loader.exec_module(mod)
sys.modules["cori_intml_examples_amd._h5lite"] = mod
import cori_intml_examples_amd.io.h5 as h5
import pytest
rc = pytest.main([sys.argv[2], "-q", "-x", "-p", "no:cacheprovider", "-m", "not gpu",
                  "-k", "h5lite or rpv_files or save or load or checkpoint or strings"])
assert getattr(h5, "_MOD", mod) is mod, "the tests did not use the sanitized module"
print("SANITIZED_MODULE", mod.__file__)
sys.exit(int(rc))
"""


def _gcc_lib(name):
    gcc = shutil.which("g++")
    if not gcc:
        return None
    p = subprocess.run([gcc, "-print-file-name=" + name], capture_output=True, text=True).stdout.strip()
    return os.path.realpath(p) if os.path.isabs(p) and os.path.exists(p) else None


def test_h5lite_under_asan_ubsan(tmp_path):
    from cori_intml_examples_amd import _build
    rt = _gcc_lib("libasan.so")
    if rt is None:
        pytest.skip("no gcc ASan runtime")
    so = _build.build_h5_sanitized(str(tmp_path / "san"))
    if so is None:
        pytest.skip("libhdf5 headers not found")
    env = dict(os.environ)
    # the ASan runtime first; then the compiler's own libstdc++ (the module's rpath would
    # otherwise pull in the older copy next to libhdf5, which lacks symbols -O2 -g references)
    pre = [rt] + [p for p in [_gcc_lib("libstdc++.so")] if p]
    env["LD_PRELOAD"] = " ".join(pre + ([env["LD_PRELOAD"]] if env.get("LD_PRELOAD") else []))
    # leaks: CPython's interned objects are reported at exit; memory errors are what we want
    env["ASAN_OPTIONS"] = "detect_leaks=0:abort_on_error=1:halt_on_error=1"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    r = subprocess.run([sys.executable, "-c", CHILD, so, os.path.join(ROOT, "tests", "test_io.py")],
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    assert "ERROR: AddressSanitizer" not in out and "runtime error:" not in out, out[-4000:]
    assert r.returncode == 0, out[-4000:]
    assert "SANITIZED_MODULE " + so in out and " passed" in out, out[-2000:]
