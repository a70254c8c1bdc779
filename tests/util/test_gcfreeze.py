"""``utils/gcfreeze.py``: the pre-loop heap leaves the collector's scans during a training loop
and comes back after it; cycles created inside are still collected."""
import gc
import weakref

import pytest

from imitation_amd.utils import gcfreeze


class _Node:
    pass


def test_frozen_heap_freezes_and_restores():
    base = gc.get_freeze_count()
    with gcfreeze.frozen_heap():
        inside = gc.get_freeze_count()
        assert inside > base
        with gcfreeze.frozen_heap():  # nested: no second freeze
            assert gc.get_freeze_count() == inside
        assert gc.get_freeze_count() == inside
    assert gc.get_freeze_count() == base


def test_cycles_created_inside_are_collected():
    with gcfreeze.frozen_heap():
        a, b = _Node(), _Node()
        a.other, b.other = b, a
        ref = weakref.ref(a)
        del a, b
        gc.collect()
        assert ref() is None


def test_cycles_from_before_are_collected_after():
    a, b = _Node(), _Node()
    a.other, b.other = b, a
    ref = weakref.ref(a)
    with gcfreeze.frozen_heap():
        del a, b
        gc.collect()
        assert ref() is not None  # frozen: not scanned while the loop runs
    gc.collect()
    assert ref() is None


def test_exception_unfreezes_and_knob_disables(monkeypatch):
    base = gc.get_freeze_count()

    @gcfreeze.during
    def boom():
        assert gc.get_freeze_count() > base
        raise RuntimeError("x")

    with pytest.raises(RuntimeError):
        boom()
    assert gc.get_freeze_count() == base
    monkeypatch.setenv("IMITATION_AMD_GC_FREEZE", "0")
    with gcfreeze.frozen_heap():
        assert gc.get_freeze_count() == base
