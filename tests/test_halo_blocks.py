"""Row-block choice of the conv halo / co-scheduled dgrad launches (CPU: host-side planning
only; the kernels module's host helpers load without a GPU).

Balanced blocks (``BatchPlan._halo_cfg``): the fewest row blocks per image that satisfy the
pixel / LDS / workgroup-count limits, each ``cdiv(Ho, c)`` rows -- e.g. MNIST's 26-row dgrad
as 13 + 13 rows, not 15 + 11 (measured 76.7 -> 46.6 us for that launch)."""
import types

import pytest

K = pytest.importorskip("cori_intml_examples_amd._kernels")
from cori_intml_examples_amd.models.executor_hip import BatchPlan, cdiv  # noqa: E402


def _cfg(Ho, Wo, Cs_in, KS, NT, B=128, pool=False, dual=True):
    a = K.ConvMMArgs()
    a.B, a.H, a.W, a.Cs_in = B, Ho, Wo, Cs_in
    a.Ho, a.Wo, a.KH, a.KW, a.stride = Ho, Wo, 3, 3, 1
    a.pad_t, a.pad_l, a.in_dil = 1, 1, 1
    a.KS, a.NT = KS, NT
    me = types.SimpleNamespace(ex=types.SimpleNamespace(K=K))
    ntc = BatchPlan._halo_cfg(me, a, NT, pool, dual=dual)
    return a.R, ntc


@pytest.mark.parametrize("Ho,Wo,Cs_in,KS,NT,want_R", [
    (26, 26, 64, 18, 2, 13),     # MNIST conv2 dgrad (26x26x64 -> 32): 13 + 13
    (16, 16, 64, 18, 2, 16),     # RPV conv3 dgrad: whole 16-row image
    (32, 32, 32, 9, 1, 16),      # RPV conv2 dgrad: two 16-row halves
])
def test_balanced_rows(Ho, Wo, Cs_in, KS, NT, want_R):
    R, _ = _cfg(Ho, Wo, Cs_in, KS, NT)
    assert R == want_R
    # balanced: R is the even split of the image over its block count
    assert R == cdiv(Ho, cdiv(Ho, R))
    assert R * Wo <= 512


def test_rows_respect_min_workgroups():
    # a tiny batch must split images into more blocks to reach the workgroup floor
    R_big, _ = _cfg(26, 26, 64, 18, 2, B=128)
    R_small, _ = _cfg(26, 26, 64, 18, 2, B=8)
    assert R_small < R_big
    assert 8 * cdiv(26, R_small) * 2 >= 256 or R_small == 1
