"""Rules of the flattened max-min system (System::flatten_maxmin, lmm_system.cpp), CPU only.

lmm_solve's init (maxmin.cpp:509-540) makes a variable active through an enabled element of weight > 0 on a
listed constraint that passes the bound test (bound > bound * prec, :523-525): the *members*.  Since round 4
the flattened system also lists every listed constraint a member has such an element on whatever its bound
(the device init starts those dead, as the reference's init leaves them out of cnst_light_tab), so that a
bound crossing the test keeps the structure.  These tests pin the two halves of that rule
on the host flatten (`lmm_flat_export`), on random API scripts with zero-bound constraints, FATPIPE, zero
weights, duplicate elements, concurrency staging, frees and updates: the member set is exactly the one of
the part-test-only rule, every flattened constraint carries a member's element, and the extra constraints
are exactly the ones that fail the bound test.  The device flatten equals this one bit for bit
(tests/test_gpu_resident.py), and the solve on it equals the oracle's (tests/test_gpu_parity.py).
"""
import numpy as np
import pytest

from simgrid_amd import lmm as L
from simgrid_amd import multi as M
from tests import lmm_cases as K
from tests.golden.make_c2_full_sample import part_only


def _flat(seed, **kw):
    ops = K.random_script(seed, n_cnst=40, n_var=150, zero_bound_p=0.25, **kw)
    s, _, _ = K.replay(L, ops)
    return M.export_flat(s)


@pytest.mark.parametrize("seed", range(12))
@pytest.mark.parametrize("kw", [{}, {"conc_limits": True, "frees": 10, "penalty_updates": 10, "bound_updates": 10}],
                         ids=["plain", "staged"])
def test_members_and_superset_constraints(seed, kw):
    prec = L.get_precision()
    f = _flat(seed, **kw)
    nv, nc = len(f.penalty), len(f.cbound)
    part = f.cbound > f.cbound * prec
    rows = np.repeat(np.arange(nv), np.diff(f.var_ptr))
    # every member has an element on a constraint that passes the bound test
    has_part = np.zeros(nv, bool)
    np.logical_or.at(has_part, rows, part[f.cnst_idx])
    assert has_part.all()
    # every flattened constraint carries an element of a member (and only members are flattened)
    assert np.array_equal(np.unique(f.cnst_idx), np.arange(nc))
    assert np.all(f.weight > 0)
    # the part-test-only filter keeps the same members in the same order: the extra constraints add
    # elements to members' rows, never a member
    old, keep = part_only(f, prec)
    assert np.array_equal(keep, part)
    assert np.array_equal(old.var_ids, f.var_ids) and len(old.penalty) == nv
    assert np.all(np.diff(old.var_ptr) >= 1)


def test_superset_rule_is_exercised():
    """Across the scripts, some flattened constraints fail the bound test (zero bounds with members on them):
    the rule above is not vacuous."""
    prec = L.get_precision()
    extra = 0
    for seed in range(12):
        f = _flat(seed)
        extra += int(np.count_nonzero(~(f.cbound > f.cbound * prec)))
    assert extra > 0
