"""Row-band plan of the layer-fused conv-stack forward (BatchPlan._stack_rows), CPU-only:
every stage-output row is stored by exactly one band, each band computes what it stores
plus every row its next layer reads, and the band ranges respect the pool pairing."""
from types import SimpleNamespace

import pytest

from cori_intml_examples_amd.models.executor_hip import BatchPlan


def _geo(H, KH, pad_t, pool, Ho=None):
    Ho = H - KH + 1 + 2 * pad_t if Ho is None else Ho
    Hp = Ho // 2 if pool else Ho
    return SimpleNamespace(H=H, KH=KH, pad_t=pad_t, pool=pool, Ho=Ho, Hp=Hp)


RPV = [_geo(64, 3, 1, True), _geo(32, 3, 1, True), _geo(16, 3, 1, True)]
MNIST = [_geo(28, 3, 0, False), _geo(26, 3, 0, True)]
ODD = [_geo(19, 3, 1, True), _geo(9, 3, 0, True)]


@pytest.mark.parametrize("convs", [RPV, MNIST, ODD], ids=["rpv", "mnist", "odd"])
@pytest.mark.parametrize("splits", [1, 2, 3, 4])
def test_stack_rows_cover_and_nest(convs, splits):
    rows = BatchPlan._stack_rows(convs, splits)
    if rows is None:
        assert splits > 1
        return
    n = len(convs)
    for l, g in enumerate(convs):
        P = 2 if g.pool else 1
        owned = []
        for sp in range(splits):
            c0, c1, o0, o1, ib, ih = rows[l][sp]
            assert 0 <= c0 < c1 <= g.Ho and c0 % P == 0 and c1 % P == 0
            assert c0 // P <= o0 < o1 <= c1 // P            # stores only what it computes
            owned.extend(range(o0, o1))
            if l > 0:                                        # inputs come from the band's previous layer
                p0, p1 = rows[l - 1][sp][:2]
                Pp = 2 if convs[l - 1].pool else 1
                need0, need1 = max(c0 - g.pad_t, 0), min(c1 - g.pad_t + g.KH - 1, g.H)
                assert p0 // Pp <= need0 and need1 <= p1 // Pp
                assert ib <= c0 - g.pad_t and c1 - g.pad_t + g.KH - 1 <= ib + ih   # conv reads inside the image
                po0, po1 = rows[l - 1][sp][2:4]
                assert ib <= po0 and po1 <= ib + ih                               # stored rows inside it
        assert owned == list(range(g.Hp))                   # exact partition
    assert len(rows) == n


def test_rpv_two_bands_recompute_is_bounded():
    rows = BatchPlan._stack_rows(RPV, 2)
    conv1 = [r[1] - r[0] for r in rows[0]]
    assert sum(conv1) <= 1.5 * 64                           # < 50% extra conv1 rows for 2 bands
