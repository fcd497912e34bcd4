"""Host logic of the placement-aware input buffers (ScanContext.workspace(placed=True)), without a GPU: the device
buffers and the calibration ratio are stand-ins, the retry / selection / release rules are the library's."""
import pytest

from dataplug_amd.scan import _lib
from dataplug_amd.scan import device as sdev


class FakeBuf:
    live = []

    def __init__(self, ctx, nbytes):
        if ctx.fail_after is not None and len(FakeBuf.live) >= ctx.fail_after:
            raise _lib.DPScanError(2, "out of device memory")
        self.ctx, self.nbytes, self.ptr = ctx, int(nbytes), 0x1000 * (len(FakeBuf.live) + 1)
        FakeBuf.live.append(self)

    def free(self):
        FakeBuf.live.remove(self)


@pytest.fixture
def ctx(monkeypatch):
    FakeBuf.live = []
    monkeypatch.setattr(sdev, "DeviceBuffer", FakeBuf)
    c = sdev.ScanContext.__new__(sdev.ScanContext)
    c._bufs, c._pinned, c.placements, c._timing_on = {}, {}, [], False
    c.fail_after = None
    ratios = []
    monkeypatch.setattr(sdev.ScanContext, "placement_ratio", lambda self, buf, nbytes=None: ratios.pop(0))
    return c, ratios


def test_fast_first_candidate_kept(ctx):
    c, ratios = ctx
    ratios += [1.09]
    b = c.workspace("input", 1 << 30, placed=True)
    assert c.placements == [[1.09]] and FakeBuf.live == [b]


def test_slow_candidates_replaced_and_released(ctx):
    c, ratios = ctx
    ratios += [1.18, 1.16, 1.10]
    b = c.workspace("input", 1 << 30, placed=True)
    assert c.placements == [[1.18, 1.16, 1.10]]
    assert FakeBuf.live == [b]                       # the slow ones were held while trying, then freed


def test_all_slow_keeps_the_best(ctx):
    c, ratios = ctx
    ratios += [1.19, 1.15, 1.17, 1.2, 1.16]
    b = c.workspace("input", 1 << 30, placed=True)
    assert len(c.placements[0]) == sdev.PLACEMENT_TRIES and FakeBuf.live == [b]
    assert b.ptr == 0x2000                           # the second candidate (1.15)


def test_out_of_memory_keeps_the_best_so_far(ctx):
    c, ratios = ctx
    ratios += [1.19, 1.16]
    c.fail_after = 2
    b = c.workspace("input", 1 << 30, placed=True)
    assert c.placements == [[1.19, 1.16]] and FakeBuf.live == [b] and b.ptr == 0x2000


def test_out_of_memory_on_the_first_candidate_raises(ctx):
    c, _ = ctx
    c.fail_after = 0
    with pytest.raises(_lib.DPScanError):
        c.workspace("input", 1 << 30, placed=True)
    assert "input" not in c._bufs


def test_sizes_outside_the_probed_band_are_not_probed(ctx):
    c, ratios = ctx
    c.workspace("small", sdev.PLACEMENT_MIN - 1, placed=True)
    c.workspace("large", sdev.PLACEMENT_MAX + 1, placed=True)
    c.workspace("unplaced", 1 << 30)
    assert c.placements == [] and len(FakeBuf.live) == 3


def test_growth_reprobes_and_frees_the_old_buffer(ctx):
    c, ratios = ctx
    ratios += [1.09, 1.2, 1.1]
    a = c.workspace("input", 1 << 30, placed=True)
    assert c.workspace("input", 1 << 29, placed=True) is a
    b = c.workspace("input", 2 << 30, placed=True)
    assert b is not a and FakeBuf.live == [b] and c.placements == [[1.09], [1.2, 1.1]]
