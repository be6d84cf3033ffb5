"""Native build driver: hipcc (gfx950) for the HIP kernels, g++ for the host-only C++.

    python -m cori_intml_examples_amd._build          # incremental
    python -m cori_intml_examples_amd._build --clean

Outputs live IN-TREE next to this file (``_kernels*.so``, ``_h5lite*.so``) so they travel
with the repository snapshot to the GPU box.  No hipify, no torch JIT cache.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "build")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
ARCH = os.environ.get("INTML_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
HDF5_ROOT = os.environ.get("INTML_HDF5_ROOT", "/opt/conda")


def _py_includes():
    import pybind11
    return ["-I" + sysconfig.get_paths()["include"], "-I" + pybind11.get_include()]


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed: %s\n%s\n%s" % (" ".join(cmd), r.stdout, r.stderr))
    return r


def kernels_so_path():
    return os.path.join(HERE, "_kernels" + EXT)


def h5_so_path():
    return os.path.join(HERE, "_h5lite" + EXT)


def build_kernels(verbose=False, jobs=8):
    kdir = os.path.join(CSRC, "kernels")
    headers = glob.glob(os.path.join(kdir, "*.h"))
    srcs = sorted(glob.glob(os.path.join(kdir, "*.hip"))) + [os.path.join(kdir, "bindings.cpp")]
    os.makedirs(BUILD, exist_ok=True)
    # -amdgpu-mfma-vgpr-form: MFMA accumulators in arch VGPRs.  The default AGPR form made the
    # register allocator rotate accumulators between AGPR sets through VGPR copies at every
    # loop back-edge (thousands of v_accvgpr_read/write per kernel: ~90 VALU per 40 MFMAs in
    # wgrad_gl's k loop); the VGPR form has none, and equal or higher occupancy for every
    # kernel here (conv_gl<8> 2 -> 4 waves/SIMD, conv_halo 2 -> 4, wgrad_gl 2 -> 3).
    flags = ["-O3", "-fPIC", "-std=c++17", "--offload-arch=" + ARCH, "-I" + kdir,
             "-Wno-unused-result", "-munsafe-fp-atomics", "-mllvm", "-amdgpu-mfma-vgpr-form"]
    objs, jobs_list = [], []
    # a change of the compile flags rebuilds every object (timestamps alone would miss it)
    stamp = os.path.join(BUILD, "kernel_flags.txt")
    flag_txt = " ".join(flags)
    stale_flags = not os.path.exists(stamp) or open(stamp).read() != flag_txt
    for src in srcs:
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        objs.append(obj)
        if stale_flags or _newer(obj, [src] + headers):
            extra = _py_includes() if src.endswith(".cpp") else []
            lang = ["-x", "hip"] if src.endswith(".hip") else []
            jobs_list.append([HIPCC] + flags + extra + lang + ["-c", src, "-o", obj])
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        list(ex.map(lambda c: _run(c, verbose), jobs_list))
    with open(stamp, "w") as f:
        f.write(flag_txt)
    out = kernels_so_path()
    if jobs_list or _newer(out, objs):
        _run([HIPCC, "-shared", "-fPIC", "--offload-arch=" + ARCH, "-o", out] + objs, verbose)
    return out


def build_h5(verbose=False):
    src = os.path.join(CSRC, "io", "h5lite.cpp")
    out = h5_so_path()
    if not os.path.exists(src):
        return None
    inc, lib = os.path.join(HDF5_ROOT, "include"), os.path.join(HDF5_ROOT, "lib")
    if not os.path.exists(os.path.join(inc, "hdf5.h")):
        if verbose:
            print("libhdf5 headers not found under %s; skipping _h5lite" % HDF5_ROOT)
        return None
    if _newer(out, [src]):
        cxx = shutil.which("g++") or "c++"
        _run([cxx, "-O2", "-shared", "-fPIC", "-std=c++17", src, "-o", out, "-I" + inc] + _py_includes()
             + ["-L" + lib, "-Wl,-rpath," + lib, "-lhdf5"], verbose)
    return out


def build_h5_sanitized(out_dir, verbose=False):
    """Host-sanitizer build of the HDF5 module (AddressSanitizer + UndefinedBehaviorSanitizer,
    aborting on the first report) into ``out_dir/_h5lite<EXT>``.  The module reads
    user-supplied checkpoint and dataset files, so it is the C++ that gets sanitized;
    ``tests/test_sanitizers.py`` runs the HDF5 round-trip tests against it in a child process
    with the ASan runtime preloaded.  Returns the path, or None without libhdf5."""
    src = os.path.join(CSRC, "io", "h5lite.cpp")
    inc, lib = os.path.join(HDF5_ROOT, "include"), os.path.join(HDF5_ROOT, "lib")
    if not os.path.exists(os.path.join(inc, "hdf5.h")):
        return None
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.join(out_dir, "_h5lite" + EXT)
    cxx = shutil.which("g++") or "c++"
    _run([cxx, "-O2", "-g", "-shared", "-fPIC", "-std=c++17", "-fno-omit-frame-pointer",
          "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", src, "-o", out,
          "-I" + inc] + _py_includes()
         # libhdf5 by path, no -L: a -L into the conda tree would resolve the sanitizer
         # runtimes to its older copies instead of the compiler's own
         + [os.path.join(lib, "libhdf5.so"), "-Wl,-rpath," + lib], verbose)
    return out


def comm_so_path():
    return os.path.join(HERE, "_comm" + EXT)


def build_comm(verbose=False):
    """RCCL data-plane engine.  Links librccl.so.1 (same SONAME as the copy PyTorch loads,
    so one RCCL instance serves the process)."""
    src = os.path.join(CSRC, "comm", "engine.cpp")
    out = comm_so_path()
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    if _newer(out, [src]):
        _run([HIPCC, "-O2", "-shared", "-fPIC", "-std=c++17", "-x", "hip", "--offload-arch=" + ARCH,
              src, "-o", out, "-I" + os.path.join(rocm, "include")] + _py_includes()
             + ["-L" + os.path.join(rocm, "lib"), "-lrccl", "-lpthread"], verbose)
    return out


def build_all(verbose=False):
    outs = [build_kernels(verbose), build_comm(verbose)]
    h5 = build_h5(verbose)
    if h5:
        outs.append(h5)
    return outs


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    if a.clean:
        shutil.rmtree(BUILD, ignore_errors=True)
        for p in (kernels_so_path(), h5_so_path(), comm_so_path()):
            if os.path.exists(p):
                os.remove(p)
    for o in build_all(a.verbose):
        print("built", o)


if __name__ == "__main__":
    main()
