"""Compiler resource report of the production dual backward kernels (CPU: hipcc cross-compiles
gfx950): no scratch -- a by-value kernel argument taken by reference in a non-inlined call, or
a mode compiled into the dual kernel's extras, made the compiler copy the whole 1.7 KB
DualExtra argument to scratch for every lane (the dual launch ran 18 -> 87-107 us,
docs/ARCHITECTURE.md §10) -- and the spill / register counts the round-5 kernels reach."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"), reason="no hipcc")
@pytest.mark.skipif(os.environ.get("INTML_SLOW_TESTS") != "1",
                    reason="~7 min device compile: INTML_SLOW_TESTS=1 (run with every kernel change)")
def test_dual_kernels_no_scratch():
    import kernel_resources as KR
    rows = KR.report(os.path.join(KR.KDIR, "dual_halo_n1.hip"))
    assert rows, "no kernels reported"
    dual = [r for r in rows if r["name"].startswith("_Z16dual_halo_kernel")]
    assert dual and all(r.get("scratch", 0) == 0 for r in dual), [(r["name"], r.get("scratch")) for r in dual if r.get("scratch")]
    # the RPV production instances (NTC 1, 4 m-tiles, 2 / 4 n-tiles, TM 4, no push): 2 waves /
    # SIMD, SGPR spills at most the round-5 level
    prod = [r for r in dual if r["name"].startswith(("_Z16dual_halo_kernelILi1ELi4ELi2ELi4ELb0E",
                                                     "_Z16dual_halo_kernelILi1ELi4ELi4ELi4ELb0E"))]
    assert prod and all(r.get("occ", 0) >= 2 and r.get("sgpr_spill", 0) <= 170 for r in prod), prod
