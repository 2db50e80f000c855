"""GN host-side helpers that need no GPU (foto/gn.py)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "optical-flow-optimal-transport_amd"))
from foto import gn  # noqa: E402


def test_outputs_are_disjoint_contiguous_views_of_one_array():
    """u, v, m come back as three views of one allocation (one 7.4 MB array at 640x480, which
    numpy backs with huge pages): each C-contiguous float64 of n values, none overlapping, in
    the order the C ABI writes them."""
    for n in (1, 4, 307200):
        u, v, m = gn._outputs(n)
        for a in (u, v, m):
            assert a.dtype == np.float64 and a.size == n and a.flags.c_contiguous and a.flags.writeable
        assert not np.shares_memory(u, v) and not np.shares_memory(v, m) and not np.shares_memory(u, m)
        assert u.base is v.base is m.base
        base = u.base
        u[:] = 1.0
        v[:] = 2.0
        m[:] = 3.0
        np.testing.assert_array_equal(base, np.repeat([1.0, 2.0, 3.0], n))
