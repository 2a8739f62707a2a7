"""Resident mode, host half: the delta log.

In resident mode the device holds a mirror of the System's element / variable / constraint records
(lmmhip_res_apply) and every mutation (maxmin.cpp:205-323, 703-888: expand, expand_add, variable_new
/ variable_free, update_variable_{penalty,bound}, update_constraint_bound, unshare, and the
concurrency staging they trigger) must log the records it touched.  These tests keep a shadow mirror
that is fed ONLY the drained delta log and check it against a full dump of the host tables after
random mutation sequences — exactly the state the device flatten reads (slab of every live variable,
every variable and constraint record).  No GPU needed: the log is drained instead of shipped.
"""
import random

import numpy as np
import pytest

from simgrid_amd import lmm as L
from tests import lmm_cases as K


class Shadow:
    def __init__(self):
        self.e_cnst = np.zeros(0, np.int32)
        self.e_w = np.zeros(0)
        self.e_fl = np.zeros(0, np.uint8)
        self.v_eb = np.zeros(0, np.int64)
        self.v_n = np.zeros(0, np.int32)
        self.v_p = np.zeros(0)
        self.v_b = np.zeros(0)
        self.c_b = np.zeros(0)
        self.c_fl = np.zeros(0, np.uint8)

    @staticmethod
    def _grow(a, n):
        if len(a) >= n:
            return a
        b = np.zeros(n, a.dtype)
        b[: len(a)] = a
        return b

    def apply(self, d):
        nE, nV, nC = d["totals"]
        for k in ("e_cnst", "e_w", "e_fl"):
            setattr(self, k, self._grow(getattr(self, k), nE))
        for k in ("v_eb", "v_n", "v_p", "v_b"):
            setattr(self, k, self._grow(getattr(self, k), nV))
        for k in ("c_b", "c_fl"):
            setattr(self, k, self._grow(getattr(self, k), nC))
        self.e_cnst[d["e_id"]] = d["e_cnst"]
        self.e_w[d["e_id"]] = d["e_w"]
        self.e_fl[d["e_id"]] = d["e_fl"]
        self.v_eb[d["v_id"]] = d["v_eb"]
        self.v_n[d["v_id"]] = d["v_n"]
        self.v_p[d["v_id"]] = d["v_p"]
        self.v_b[d["v_id"]] = d["v_b"]
        self.c_b[d["c_id"]] = d["c_b"]
        self.c_fl[d["c_id"]] = d["c_fl"]


def full_dump(s):
    s.set_resident(True)  # whole system pending
    sh = Shadow()
    sh.apply(s.drain_deltas())
    return sh


def assert_same_device_view(a, b):
    """What the device flatten reads: every variable / constraint record and the live slabs."""
    assert len(a.v_n) == len(b.v_n) and len(a.c_b) == len(b.c_b)
    np.testing.assert_array_equal(a.v_n, b.v_n)
    np.testing.assert_array_equal(a.v_p, b.v_p)
    np.testing.assert_array_equal(a.v_b, b.v_b)
    np.testing.assert_array_equal(a.c_b, b.c_b)
    np.testing.assert_array_equal(a.c_fl, b.c_fl)
    for v in np.nonzero(b.v_n > 0)[0]:  # the slabs the device reads (-1 = dead)
        assert a.v_eb[v] == b.v_eb[v]
        sl = slice(int(b.v_eb[v]), int(b.v_eb[v] + b.v_n[v]))
        np.testing.assert_array_equal(a.e_cnst[sl], b.e_cnst[sl])
        np.testing.assert_array_equal(a.e_w[sl], b.e_w[sl])
        np.testing.assert_array_equal(a.e_fl[sl], b.e_fl[sl])


def step_ops(rng, cs, vs, next_var, n_new=8, n_free=6, n_pen=6, n_bound=6, max_el=5, unshare_p=0.3):
    """One simulation step's worth of mutations on an existing replayed system (op tuples of
    tests/lmm_cases.replay): flows end, flows start, penalties / bounds move."""
    ops = []
    alive = sorted(vs)
    for v in rng.sample(alive, min(n_free, len(alive))):
        ops.append(("free", v))
        alive.remove(v)
    ckeys = sorted(cs)
    for i in range(n_new):
        v = next_var + i
        k = rng.randint(1, max_el)
        ops.append(("var", v, rng.choice([1.0, 2.0, 0.5]), -1.0 if rng.random() < 0.7 else round(rng.uniform(0.1, 3), 3),
                    k + 2))
        picked = rng.sample(ckeys, min(k, len(ckeys)))
        for c in picked:
            ops.append(("expand", c, v, round(rng.uniform(0.05, 2.0), 4)))
        if rng.random() < 0.3:
            ops.append(("expand_add", picked[0], v, round(rng.uniform(0.0, 1.0), 4)))
        alive.append(v)
    for _ in range(n_pen):
        ops.append(("penalty", rng.choice(alive), rng.choice([0.0, 1.0, 2.0, 3.0])))
    for _ in range(n_bound):
        if rng.random() < 0.5:
            ops.append(("vbound", rng.choice(alive), round(rng.uniform(0.05, 3.0), 3)))
        else:
            ops.append(("cbound", rng.choice(ckeys), round(rng.uniform(0.5, 20.0), 3)))
    if rng.random() < unshare_p:
        ops.append(("unshare", rng.choice(ckeys)))
    return ops, next_var + n_new


def test_resident_flag_and_full_pending():
    s = L.System(False)
    assert s.resident()  # max-min systems start resident (maxmin/resident:yes)
    assert not L.System(False, L.System.FAIR_BOTTLENECK).resident()  # FairBottleneck keeps the host flatten
    s.set_resident(False)
    assert not s.resident()
    s.set_resident(True)
    assert s.resident()
    assert s.pending_deltas() == (-1, -1, -1)
    _, vs, _, _ = s.gen_maxmin_bench(0, 0)
    d = s.drain_deltas()
    assert d["totals"][1] == 10 and len(d["v_id"]) == 10 and len(d["c_id"]) == 10
    assert s.pending_deltas() == (0, 0, 0)
    s.update_variable_bound(vs[3], 2.5)
    assert s.pending_deltas() == (0, 1, 0)
    d = s.drain_deltas()
    assert list(d["v_id"]) == [vs[3].h] and d["v_b"][0] == 2.5
    s.set_resident(False)
    with pytest.raises(L.LmmError):
        s.drain_deltas()


@pytest.mark.parametrize("seed", range(8))
@pytest.mark.parametrize("selective", [False, True])
def test_delta_log_reproduces_tables(seed, selective):
    rng = random.Random(1000 + seed)
    ops = K.random_script(seed, n_cnst=25, n_var=60, conc_limits=seed % 2 == 0, frees=5, penalty_updates=5,
                          bound_updates=5)
    s = L.System(selective)
    s.set_resident(True)
    s, cs, vs = K.replay(L, ops, sys_=s)
    sh = Shadow()
    sh.apply(s.drain_deltas())
    next_var = 1000
    for _ in range(6):
        more, next_var = step_ops(rng, cs, vs, next_var)
        K.replay(L, more, sys_=s, cs=cs, vs=vs)
        sh.apply(s.drain_deltas())
        assert_same_device_view(sh, full_dump(s))
        sh = full_dump(s)  # full_dump re-armed the log; continue from a full mirror


def test_staging_moves_are_logged():
    """Concurrency staging (maxmin.cpp:804-843) moves elements between the enabled / disabled lists of
    constraints the mutation never named: those moves must be in the log too."""
    s = L.System(False)
    s.set_resident(True)
    c = s.constraint_new(None, 10.0)
    c.set_concurrency_limit(2)
    vs = []
    for _ in range(4):
        v = s.variable_new(None, 1.0, -1.0, 2)
        s.expand(c, v, 1.0)
        vs.append(v)
    sh = Shadow()
    sh.apply(s.drain_deltas())
    s.variable_free(vs[0])  # frees a slot: a staged variable gets enabled
    sh.apply(s.drain_deltas())
    assert_same_device_view(sh, full_dump(s))


def test_config_flags():
    """--cfg-style flags (lmm_config_set): the solver selector the reference lacks, resident default."""
    assert L.config_get("maxmin/solver") == "hip-auto"
    L.config_set("maxmin/solver:hip-rounds")
    assert L.config_get("maxmin/solver") == "hip-rounds"
    L.config_set("maxmin/solver:hip")
    assert L.config_get("maxmin/solver") == "hip-auto"
    with pytest.raises(L.LmmError, match="no CPU solver"):
        L.config_set("maxmin/solver:cpu")
    with pytest.raises(L.LmmError, match="unknown key"):
        L.config_set("maxmin/nope:1")
    L.config_set("maxmin/resident:no")
    try:
        assert not L.System(False).resident()
    finally:
        L.config_set("maxmin/resident:yes")
    assert L.System(False).resident()
    L.config_set("maxmin/precision:1e-6")
    assert L.get_precision() == 1e-6
    L.config_set("maxmin/precision:1e-5")


def test_opaque_ids():
    """Constraint / Variable ids (maxmin.hpp:395, :404): borrowed Resource* / Action* handed back by
    get_id() and by the modified set (maxmin.cpp:536-538)."""
    s = L.System(True)
    c = s.constraint_new(0x1000, 3.0)
    v = s.variable_new(0x2000, 1.0, -1.0, 1)
    w = s.variable_new(None, 1.0, -1.0, 1)
    s.expand(c, v, 1.0)
    s.expand(c, w, 1.0)
    assert c.get_id() == 0x1000 and v.get_id() == 0x2000 and w.get_id() is None
