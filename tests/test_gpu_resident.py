"""Resident mode on the GPU: HBM mirror + delta log + device flatten.

Parity bar: the device flatten must build, BIT FOR BIT, the very arrays the host flatten uploads (dense
constraint ids in list order, dense variables ascending, CSC by a stable sort) — checked by downloading
both flattened systems from HBM (lmmhip_flat_download) step after step of random mutations (flows
ending and starting, penalty / bound moves, staging).  Values are then compared with the parity
tolerance of tests/lmm_cases.py against the host-flatten solve and the oracle, and in selective (Lazy)
mode the modified-action lists must be identical.  Max-min systems are resident by default
(maxmin/resident:yes): the host-flatten twin of each test is switched to set_resident(False).
"""
import random

import numpy as np
import pytest

from oracle import pyoracle as O
from simgrid_amd import lmm as L
from tests import lmm_cases as K
from tests.test_resident import step_ops

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if L.device_count() == 0:
        pytest.fail("no HIP device visible: the GPU tests must run on the MI355X")


def _values(vs):
    return {k: v.get_value() for k, v in vs.items()}


def _flat_equal(fa, fb):
    for k in fb:
        assert fa[k].dtype == fb[k].dtype and np.array_equal(fa[k], fb[k]), k


def _flat_equal_fair(fa, fb):
    """FairBottleneck flattens: CSR and metadata bit for bit; each constraint's CSC elements as a set.  The
    host flatten hands each constraint's elements in the reference's enabled-list order (System::flatten_fair,
    for the element-by-element remaining update of lmm_fb_kernels.hpp:fbk_update_seq); the device flatten of
    resident mode keeps them in ascending variable order."""
    for k in fb:
        if k not in ("csc_v", "csc_w"):
            assert fa[k].dtype == fb[k].dtype and np.array_equal(fa[k], fb[k]), k
    cp = fb["cnst_ptr"].astype(np.int64)
    for c in range(len(cp) - 1):
        ea = sorted(zip(fa["csc_v"][cp[c]:cp[c + 1]].tolist(), fa["csc_w"][cp[c]:cp[c + 1]].tolist()))
        eb = sorted(zip(fb["csc_v"][cp[c]:cp[c + 1]].tolist(), fb["csc_w"][cp[c]:cp[c + 1]].tolist()))
        assert ea == eb, c


def _split_solve(s):
    s.prepare()
    f = s.device_flat()
    s.device_solve()
    s.fetch()
    return f


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("selective", [False, True])
def test_resident_steps_bit_identical(seed, selective):
    ops = K.random_script(seed, n_cnst=40, n_var=150, conc_limits=seed % 2 == 1, frees=10, penalty_updates=10,
                          bound_updates=10)
    a, csa, vsa = K.replay(L, ops, selective)
    a.set_resident(True)
    b, csb, vsb = K.replay(L, ops, selective)
    b.set_resident(False)
    o, cso, vso = K.replay(O, ops, selective)
    rng = random.Random(7 + seed)
    next_var = 10000
    for step in range(6):
        fa = _split_solve(a)
        fb = _split_solve(b)
        o.solve()
        _flat_equal(fa, fb)
        worst, bad = K.compare_values(vsa, vsb)
        assert not bad, (step, worst, bad[:5])
        worst, bad = K.compare_values(vsa, vso)
        assert not bad, (step, worst, bad[:5])
        if selective:
            assert [v.h for v in a.modified_actions()] == [v.h for v in b.modified_actions()]
            a.clear_modified_actions()
            b.clear_modified_actions()
        st = a.last_stats()
        assert st["n_var"] == b.last_stats()["n_var"] and st["nnz"] == b.last_stats()["nnz"]
        if step > 0:  # only the logged records travel after the first (full) ship
            assert 0 < st["delta_records"] < len(vsa) * 4 + 200
        more, next_var = step_ops(rng, csa, vsa, next_var)
        K.replay(L, more, sys_=a, cs=csa, vs=vsa)
        K.replay(L, more, sys_=b, cs=csb, vs=vsb)
        K.replay(O, more, sys_=o, cs=cso, vs=vso)


@pytest.mark.parametrize("klass,run", [(0, r) for r in range(10)] + [(1, r) for r in range(5)])
def test_resident_maxmin_bench_goldens(klass, run):
    """maxmin_bench small/medium (golden-pinned systems, heavy concurrency staging) through resident mode."""
    a = L.System(False)
    a.set_resident(True)
    _, va, _, _ = a.gen_maxmin_bench(klass, run)
    b = L.System(False)
    b.set_resident(False)
    _, vb, _, _ = b.gen_maxmin_bench(klass, run)
    _flat_equal(_split_solve(a), _split_solve(b))
    for x, y in zip(va, vb):
        assert K.close(x.get_value(), y.get_value())


def test_resident_synthetic_churn():
    """A 2e4 x 2e5 x 8 synthetic system, then churn steps driven through the API: resident equals the
    host flatten bit for bit and ships only the logged records."""
    nC, nV = 20000, 200000
    a = L.System(False)
    a.set_resident(True)
    va = a.gen_synthetic(nC, nV, k=8, seed=3, penalty_mix=1, bounded_permille=100, fatpipe_permille=50)
    b = L.System(False)
    b.set_resident(False)
    vb = b.gen_synthetic(nC, nV, k=8, seed=3, penalty_mix=1, bounded_permille=100, fatpipe_permille=50)
    rng = np.random.default_rng(5)
    for step in range(3):
        _flat_equal(_split_solve(a), _split_solve(b))
        xa, xb = a.values_of(va), b.values_of(vb)
        assert np.all(np.abs(xa - xb) <= np.maximum(K.ABS_TOL, K.REL_TOL * np.abs(xb))), step
        if step:
            assert a.last_stats()["delta_records"] < 20000
        for i in rng.choice(nV, 500, replace=False):
            p = float(rng.choice([0.0, 0.5, 1.0, 2.0]))
            a.update_variable_penalty(L.Variable(a, int(va[i])), p)
            b.update_variable_penalty(L.Variable(b, int(vb[i])), p)
        for c in rng.choice(nC, 100, replace=False):
            bnd = float(rng.uniform(0.5, 10.0))
            a.update_constraint_bound(L.Constraint(a, int(c)), bnd)
            b.update_constraint_bound(L.Constraint(b, int(c)), bnd)


@pytest.mark.parametrize("seed", range(4))
def test_resident_fair_bottleneck_flatten(seed):
    """FairBottleneck inputs built on the device (flatten_fair's rules: no bound test, zero-weight FATPIPE
    flag, CSC chunks) equal the host flatten's bit for bit, over mutation steps.  Flatten only: these
    systems mix zero weights, zero bounds and FATPIPE, on which the reference's bottleneck_solve need not
    terminate (tests/test_gpu_parity.py)."""
    ops = K.random_script(100 + seed, n_cnst=40, n_var=150, zero_w_p=0.1, fatpipe_p=0.2)
    a, csa, vsa = K.replay(L, ops, kind=1)
    a.set_resident(True)
    b, csb, vsb = K.replay(L, ops, kind=1)
    rng = random.Random(seed)
    next_var = 5000
    for step in range(4):
        a.prepare()
        b.prepare()
        _flat_equal_fair(a.device_flat(), b.device_flat())
        more, next_var = step_ops(rng, csa, vsa, next_var)
        K.replay(L, more, sys_=a, cs=csa, vs=vsa)
        K.replay(L, more, sys_=b, cs=csb, vs=vsb)


@pytest.mark.parametrize("seed", range(4))
def test_resident_fair_bottleneck_steps(seed):
    """FairBottleneck::solve through the device flatten on terminating systems (no FATPIPE, no zero
    weight; zero bounds allowed): flattened inputs bit-identical, values within tolerance, steps."""
    ops = K.random_script(200 + seed, n_cnst=40, n_var=150, zero_w_p=0.0, fatpipe_p=0.0, zero_bound_p=0.05)
    a, csa, vsa = K.replay(L, ops, kind=1)
    a.set_resident(True)
    b, csb, vsb = K.replay(L, ops, kind=1)
    rng = random.Random(seed)
    next_var = 5000
    for step in range(4):
        _flat_equal_fair(_split_solve(a), _split_solve(b))
        worst, bad = K.compare_values(vsa, vsb)
        assert not bad, (step, worst, bad[:5])
        more, next_var = step_ops(rng, csa, vsa, next_var, unshare_p=0.0)
        more = [op for op in more if not (op[0] == "expand_add" and op[3] == 0.0)]
        K.replay(L, more, sys_=a, cs=csa, vs=vsa)
        K.replay(L, more, sys_=b, cs=csb, vs=vsb)


def test_resident_switches_solver_kind():
    """lmm_solve() on a FairBottleneck system is the max-min solver (maxmin.hpp:447): the device flatten
    follows the kind of each call."""
    ops = K.random_script(7, n_cnst=20, n_var=60, zero_w_p=0.0, fatpipe_p=0.0)
    a, _, vsa = K.replay(L, ops, kind=1)
    a.set_resident(True)
    b, _, vsb = K.replay(L, ops, kind=1)
    for call in ("solve", "lmm_solve", "solve"):
        getattr(a, call)()
        getattr(b, call)()
        worst, bad = K.compare_values(vsa, vsb)
        assert not bad, (call, worst, bad[:5])


def test_resident_refresh_path_bounds_and_penalties():
    """Steps that only move penalties (staying > 0), variable bounds and constraint bounds (staying > 0)
    keep the structure: the device flatten takes the refresh path (dense penalties / bounds rewritten,
    structure reused) and must still equal the host flatten bit for bit."""
    import ctypes as ct

    ops = K.random_script(21, n_cnst=50, n_var=300, conc_limits=False)
    a, csa, vsa = K.replay(L, ops)
    a.set_resident(True)
    b, csb, vsb = K.replay(L, ops)
    b.set_resident(False)
    rng = random.Random(4)
    _flat_equal(_split_solve(a), _split_solve(b))
    nref = ct.c_int64()
    for step in range(4):
        live = [k for k in sorted(vsa) if vsa[k].get_penalty() > 0]
        for k in rng.sample(live, 20):
            p = rng.choice([0.5, 1.5, 3.0])
            a.update_variable_penalty(vsa[k], p)
            b.update_variable_penalty(vsb[k], p)
        for k in rng.sample(live, 10):
            bd = round(rng.uniform(0.05, 3.0), 3)
            a.update_variable_bound(vsa[k], bd)
            b.update_variable_bound(vsb[k], bd)
        for k in rng.sample([k for k in sorted(csa) if csa[k].get_bound() > 0], 5):
            bd = round(rng.uniform(0.5, 20.0), 3)
            a.update_constraint_bound(csa[k], bd)
            b.update_constraint_bound(csb[k], bd)
        _flat_equal(_split_solve(a), _split_solve(b))
        worst, bad = K.compare_values(vsa, vsb)
        assert not bad, (step, worst, bad[:5])
        L._check_hip(L.lib().lmmhip_res_refreshes(a.device_ctx(), ct.byref(nref)))
        assert nref.value == step + 1
    # a structural step (a new flow) goes back to the full rebuild
    v = a.variable_new(None, 1.0, -1.0, 2)
    a.expand(csa[0], v, 1.0)
    w = b.variable_new(None, 1.0, -1.0, 2)
    b.expand(csb[0], w, 1.0)
    _flat_equal(_split_solve(a), _split_solve(b))
    L._check_hip(L.lib().lmmhip_res_refreshes(a.device_ctx(), ct.byref(nref)))
    assert nref.value == 4


def _counters(s):
    import ctypes as ct

    n, x = ct.c_int64(), ct.c_int64()
    L._check_hip(L.lib().lmmhip_res_refreshes(s.device_ctx(), ct.byref(n)))
    L._check_hip(L.lib().lmmhip_res_cross_refreshes(s.device_ctx(), ct.byref(x)))
    return n.value, x.value


def test_resident_refresh_path_part_crossings():
    """A constraint bound crossing the part test (maxmin.cpp:523-525) keeps the flattened structure unless it
    changes the member set (every listed constraint a member lies on is flattened whatever its bound; the
    solver's init starts the failing ones dead): the device decides (rs_cross_check) and the result must
    equal the host flatten bit for bit, and the values the oracle's, on both outcomes.
    c0 .. c3 (bound 1), v0 on c0 + c1, v1 on c1 only, v2 on c2 + c3, v3 (bound 0.25) on c1 + c2."""
    ops = [("cnst", i, 1.0) for i in range(4)]
    ops += [("var", 0, 1.0, -1.0, 2), ("var", 1, 1.0, -1.0, 1), ("var", 2, 2.0, -1.0, 2), ("var", 3, 1.0, 0.25, 2)]
    ops += [("expand", 0, 0, 1.0), ("expand", 1, 0, 2.0), ("expand", 1, 1, 1.0), ("expand", 2, 2, 1.0),
            ("expand", 3, 2, 0.5), ("expand", 1, 3, 1.0), ("expand", 2, 3, 1.0)]
    a, csa, vsa = K.replay(L, ops)
    a.set_resident(True)
    b, csb, vsb = K.replay(L, ops)
    b.set_resident(False)
    o, cso, vso = K.replay(O, ops)
    # (bounds set this step, refresh path expected, with part-test crossings)
    steps = [
        ({0: 0.0}, True, True),              # v0 keeps c1
        ({0: 2.0}, True, True),              # c0 back: its only enabled element is v0's, a member
        ({1: 0.0}, False, False),            # v1 only lies on c1: it leaves the member set
        ({3: 5.0}, True, False),             # no crossing (c1 flattened though failing the part test)
        ({1: 1.0}, False, False),            # v1 (an outsider of c1 at the last flatten) joins again
        ({2: 0.0, 3: 0.0}, False, False),    # v2 loses both of its constraints in one step
        ({2: 0.0, 3: 4.0}, False, False),    # v2 joins again through c3
        ({1: 0.0, 0: 3.0}, False, False),    # v1 and v3 leave (v3's c2 is still at 0)
        ({2: 0.0, 0: 5.0}, True, False),     # no crossing
        ({1: 1.0}, False, False),            # v1 and v3 join again
        ({0: 0.0}, True, True),              # v0 keeps c1
    ]
    _flat_equal(_split_solve(a), _split_solve(b))
    o.solve()
    for step, (bounds, refresh, cross) in enumerate(steps):
        n0, x0 = _counters(a)
        for k, bd in bounds.items():
            a.update_constraint_bound(csa[k], bd)
            b.update_constraint_bound(csb[k], bd)
            o.update_constraint_bound(cso[k], bd)
        _flat_equal(_split_solve(a), _split_solve(b))
        o.solve()
        worst, bad = K.compare_values(vsa, vsb)
        assert not bad, (step, worst, bad[:5])
        worst, bad = K.compare_values(vsa, vso)
        assert not bad, (step, worst, bad[:5])
        n1, x1 = _counters(a)
        assert (n1 - n0, x1 - x0) == (int(refresh), int(cross)), (step, bounds)


def test_resident_refresh_path_zero_bound_churn():
    """The C2 generator's bounds (~1/1000 of the constraints at 0) under random constraint-bound updates drawn
    from the same law, so that steps cross the part test both ways: the device flatten equals the host
    flatten and the values agree at every step, and most crossing steps stay on the refresh path."""
    nC, nV = 20000, 200000
    a = L.System(False)
    a.set_resident(True)
    va = a.gen_synthetic(nC, nV, k=8, seed=11)
    b = L.System(False)
    b.set_resident(False)
    vb = b.gen_synthetic(nC, nV, k=8, seed=11)
    rng = np.random.default_rng(9)
    _flat_equal(_split_solve(a), _split_solve(b))
    n0, x0 = _counters(a)
    zero = 0
    for step in range(6):
        ids = rng.choice(nC, 400, replace=False)
        bnds = 10.0 * rng.integers(0, 1001, len(ids)) / 1001.0
        bnds[:2] = 0.0  # at least two crossings (or zero-to-zero moves) per step
        zero += int(np.count_nonzero(bnds == 0))
        for c, bd in zip(ids, bnds):
            a.update_constraint_bound(L.Constraint(a, int(c)), float(bd))
            b.update_constraint_bound(L.Constraint(b, int(c)), float(bd))
        _flat_equal(_split_solve(a), _split_solve(b))
        xa, xb = a.values_of(va), b.values_of(vb)
        assert np.all(np.abs(xa - xb) <= np.maximum(K.ABS_TOL, K.REL_TOL * np.abs(xb))), step
    n1, x1 = _counters(a)
    assert n1 - n0 == 6 and x1 - x0 >= 5, (n1 - n0, x1 - x0, zero)
