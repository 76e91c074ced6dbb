"""The library/package layout guard (ops._check_layout), CPU only.

Round 5's GPU log gpurun_out/r05/h/tests.log (8 passed, ~190 failed, then
``Fatal Python error: Aborted`` in a backward) came from a library built with
the save layout that still held the ``feat`` segment (32 KiB per 32-sample
block, between h8 and hdir) while ops.py already sized save buffers without
it: every training forward wrote hdir, dir PE and the ReLU masks past the end
of the caller-sized buffer.  The guard compares the library's block sizes
(nr_layout_query 3 / 4) with the package's before the first save buffer is
sized; these tests drive its raise path with a stand-in library."""
import pytest

from nerf_pl_amd import ops


class _FakeLib:
    def __init__(self, save, grad, abi=ops.ABI_REVISION):
        self._v = {3: save, 4: grad, 9: abi}

    def nr_layout_query(self, what):
        return self._v[what]


@pytest.fixture
def fresh_guard(monkeypatch):
    monkeypatch.setattr(ops, "_LAYOUT_OK", False)
    return monkeypatch


@pytest.mark.parametrize("save_delta,grad_delta", [(32 * 256, 0), (0, 32 * 256), (-1, 0), (0, 4)])
def test_layout_mismatch_raises(fresh_guard, save_delta, grad_delta):
    fake = _FakeLib(ops.SAVE_PER_BLOCK + save_delta, ops.GRAD_PER_BLOCK + grad_delta)
    fresh_guard.setattr(ops, "lib", lambda: fake)
    with pytest.raises(RuntimeError, match="rebuild the library"):
        ops.save_floats(1000)
    assert ops._LAYOUT_OK is False          # a failed check is not remembered as passed


def test_layout_match_passes_once(fresh_guard):
    calls = []

    class Counting(_FakeLib):
        def nr_layout_query(self, what):
            calls.append(what)
            return super().nr_layout_query(what)

    fake = Counting(ops.SAVE_PER_BLOCK, ops.GRAD_PER_BLOCK)
    fresh_guard.setattr(ops, "lib", lambda: fake)
    n = ops.save_floats(1000)
    assert n == ops.n_blocks(1000) * ops.SAVE_PER_BLOCK + ops.SAVE_STATS + ops.STAT_SEGS * ops.n_blocks(1000)
    ops.save_floats(5)
    assert calls == [3, 4, 9]               # queried once per process


def test_r05_layout_is_rejected(fresh_guard):
    """the exact r05 pair: a library with the feat segment, the package without"""
    r05_lib_save = ops.BLK * (64 + 8 * 256 + 256 + 128 + 32) + 9 * 256
    fresh_guard.setattr(ops, "lib", lambda: _FakeLib(r05_lib_save, ops.GRAD_PER_BLOCK))
    with pytest.raises(RuntimeError):
        ops.save_floats(128)


def test_abi_revision_mismatch_raises(fresh_guard):
    """a revision-1 library (every nr_wgrad* gradient final, no
    nr_wgrad_dir_feat follow-up) is refused"""
    fresh_guard.setattr(ops, "lib", lambda: _FakeLib(ops.SAVE_PER_BLOCK, ops.GRAD_PER_BLOCK, 1))
    with pytest.raises(RuntimeError, match="ABI"):
        ops.save_floats(128)


def test_built_library_matches_package():
    """the in-tree library itself (no GPU call: nr_layout_query is host code)"""
    from nerf_pl_amd._lib import lib
    assert lib().nr_layout_query(9) == ops.ABI_REVISION
    assert (lib().nr_layout_query(3), lib().nr_layout_query(4)) == (ops.SAVE_PER_BLOCK,
                                                                   ops.GRAD_PER_BLOCK)
