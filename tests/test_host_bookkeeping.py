"""Host-side System bookkeeping of the product (simgrid_amd.lmm) vs the oracle — CPU only.

Concurrency staging decides which variables are enabled (integer work): it must be identical.
Checked: element lists per constraint (print() order), weights, concurrency current/max/limit,
variable_set order, active_constraint_set order, penalties after staging.
"""
import pytest

from oracle import pyoracle as O
from simgrid_amd import lmm as L
from tests import lmm_cases as K


def same_structure(ps, os_, pcs, ocs, pvs, ovs):
    for k in ocs:
        assert pcs[k].concurrency() == ocs[k].concurrency(), k
        pe = [(e[0], e[1], e[3]) for e in pcs[k].elements()]
        oe = [(e[0], e[1], e[3]) for e in ocs[k].elements()]
        assert pe == oe, k
        assert pcs[k].is_shared() == ocs[k].is_shared()
    for k in ovs:
        assert pvs[k].get_penalty() == ovs[k].get_penalty(), k
        assert pvs[k].get_number_of_constraint() == ovs[k].get_number_of_constraint()
    assert [v.rank for v in ps.variables()] == [v.rank for v in os_.variables()]
    assert [c.rank for c in ps.active_constraints()] == [c.rank for c in os_.active_constraints()]


@pytest.mark.parametrize("klass,runs", [(0, 10), (1, 5), (2, 1)])
def test_maxmin_bench_staging_matches_oracle(klass, runs):
    for run in range(runs):
        ps, os_ = L.System(False), O.System(False)
        pc, pv, a, b = ps.gen_maxmin_bench(klass, run)
        oc, ov, a2, b2 = os_.gen_maxmin_bench(klass, run)
        assert (a, b) == (a2, b2)
        same_structure(ps, os_, dict(enumerate(pc)), dict(enumerate(oc)), dict(enumerate(pv)), dict(enumerate(ov)))


@pytest.mark.parametrize("seed", range(12))
def test_random_scripts_with_limits_frees_updates(seed):
    ops = K.random_script(seed, conc_limits=True, frees=10, penalty_updates=15, bound_updates=10)
    ps, pcs, pvs = K.replay(L, ops)
    os_, ocs, ovs = K.replay(O, ops)
    same_structure(ps, os_, pcs, ocs, pvs, ovs)


@pytest.mark.parametrize("seed", range(4))
def test_selective_mode_bookkeeping(seed):
    ops = K.random_script(100 + seed, conc_limits=True, frees=5, penalty_updates=5)
    ps, pcs, pvs = K.replay(L, ops, selective=True)
    os_, ocs, ovs = K.replay(O, ops, selective=True)
    same_structure(ps, os_, pcs, ocs, pvs, ovs)
    assert ps.modified and os_.modified


@pytest.mark.parametrize("M", [L, O], ids=["product", "oracle"])
def test_free_staged_variable_with_duplicate_elements(M):
    # The reference re-enables such a variable inside its own free and double-erases it (UB).
    # Both implementations define it as "a freed variable is never re-enabled".
    s = M.System(False)
    c = s.constraint_new(None, 5.0)
    c.set_concurrency_limit(2)
    a = s.variable_new(None, 1.0, -1.0, 2)
    s.expand(c, a, 1.0)
    s.expand(c, a, 1.0)  # a holds the two slots
    b = s.variable_new(None, 1.0, -1.0, 2)
    b.set_concurrency_share(2)
    s.expand(c, b, 1.0)  # no slack: b is staged (weight 0)
    s.expand(c, b, 1.0)  # second element of b on c, b disabled
    assert b.get_penalty() == 0.0
    s.variable_free(b)  # must not re-enable b while freeing it
    assert c.concurrency()[0] == 2
    s.variable_free(a)
    assert c.concurrency()[0] == 0 and c.elements() == []


@pytest.mark.parametrize("seed", range(60))
def test_dense_frees_and_duplicates(seed):
    ops = K.random_script(seed, conc_limits=(seed % 2 == 0), frees=3 + seed % 7, penalty_updates=4, bound_updates=4,
                          dup_p=0.4)
    a = K.replay(L, ops)
    b = K.replay(O, ops)
    same_structure(a[0], b[0], a[1], b[1], a[2], b[2])


def test_variable_free_all_empties_system():
    ops = K.random_script(7, conc_limits=True)
    ps, pcs, _ = K.replay(L, ops)
    ps.variable_free_all()
    assert ps.variables() == []
    for c in pcs.values():
        assert c.elements() == []
        assert c.concurrency()[0] == 0


def test_too_many_constraints_is_reported():
    s = L.System(False)
    c1, c2 = s.constraint_new(None, 1.0), s.constraint_new(None, 1.0)
    v = s.variable_new(None, 1.0, -1.0, 1)
    s.expand(c1, v, 1.0)
    with pytest.raises(L.LmmError, match="Too much constraints"):
        s.expand(c2, v, 1.0)
