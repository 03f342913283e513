"""Host-side argument checks of the Python mirror that need no GPU: a caller's `out` rows for the
coalescing entry points are written in place by the engine, so they must match the operand exactly
(an undersized or converted `out` would otherwise take an out-of-bounds write or lose
the result)."""
import numpy as np
import pytest

from fedtree_amd.paillier import _check_out


def test_out_rows_accepted_when_exact():
    a = np.zeros((4, 128), np.uint32)
    assert _check_out(a, (4, 128), "add_shared") is a


@pytest.mark.parametrize("bad", [np.zeros((3, 128), np.uint32), np.zeros((4, 128), np.int32),
                                 np.zeros((4, 256), np.uint32)[:, ::2], np.zeros(4 * 128, np.uint32),
                                 [[0] * 128] * 4])
def test_out_rows_rejected(bad):
    with pytest.raises(ValueError):
        _check_out(bad, (4, 128), "add_shared")


def test_readonly_out_rejected():
    a = np.zeros((4, 128), np.uint32)
    a.flags.writeable = False
    with pytest.raises(ValueError):
        _check_out(a, (4, 128), "add_shared")
