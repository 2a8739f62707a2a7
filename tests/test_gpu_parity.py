"""GPU parity: the HIP solver (through the C ABI) vs the oracle and the reference's goldens.

Tolerances are those of tests/lmm_cases.py: per variable
|x_gpu - x_oracle| <= max(1e-9, 1e-6 |x_oracle|); goldens +-1.5e-6 (%f printing); saturated
constraint sets identical.
"""
import json
import os

import numpy as np
import pytest

from oracle import pyoracle as O
from simgrid_amd import lmm as L
from tests import lmm_cases as K

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if L.device_count() == 0:
        pytest.fail("no HIP device visible: the GPU tests must run on the MI355X")


# ---- reference unit tests (maxmin_test.cpp) -------------------------------------------------
@pytest.mark.parametrize("kat", K.MAXMIN_TEST_KATS, ids=lambda f: f.__name__)
def test_maxmin_test_kats(kat):
    s, expect = kat(L)
    for v, x in expect:
        assert abs(v.get_value() - x) < 1e-5  # double_equals(value, expected, sg_maxmin_precision)
        assert abs(v.get_value() - x) < 1e-12


@pytest.mark.parametrize("case", [K.lmm_usage_test1, K.lmm_usage_test2])
def test_lmm_usage_cases(case):
    s, expect = case(L)
    for v, x in expect:
        assert abs(v.get_value() - x) < 1e-12


def test_lmm_usage_test3_vs_oracle():
    _, pv = K.lmm_usage_test3(L)
    _, ov = K.lmm_usage_test3(O)
    for a, b in zip(pv, ov):
        assert K.close(a.get_value(), b.get_value())


# ---- golden vectors (maxmin_bench tesh) -----------------------------------------------------
@pytest.mark.parametrize("name,klass", [("small", 0), ("medium", 1)])
def test_maxmin_bench_goldens(name, klass):
    with open(os.path.join(GOLD, f"maxmin_bench_{name}.json")) as f:
        d = json.load(f)
    for r in d["runs"]:
        s = L.System(False)
        cs, vs, a, b = s.gen_maxmin_bench(klass, r["run"])
        assert (a, b) == (r["check_start"], r["check_solve"])
        s.solve()
        for rk, (pen, val) in r["values"].items():
            v = vs[int(rk) - 1]
            assert abs(v.get_penalty() - pen) <= K.GOLDEN_TOL
            assert abs(v.get_value() - val) <= K.GOLDEN_TOL, (name, r["run"], rk, v.get_value(), val)
        # the constraint equations' sums stay within bounds (print()'s assertion, maxmin.cpp:470)
        for c in cs:
            assert not (c.get_usage() - c.get_bound() > c.get_bound() * 1e-5)


@pytest.mark.parametrize("name,klass,runs", [("small", 0, 10), ("medium", 1, 5)])
def test_maxmin_bench_vs_oracle_tight(name, klass, runs):
    for run in range(runs):
        ps, os_ = L.System(False), O.System(False)
        pc, pv, _, _ = ps.gen_maxmin_bench(klass, run)
        oc, ov, _, _ = os_.gen_maxmin_bench(klass, run)
        ps.solve()
        os_.solve()
        worst, bad = K.compare_values(dict(enumerate(pv)), dict(enumerate(ov)))
        assert not bad, bad[:5]
        assert K.saturated(ps, dict(enumerate(pc)), 1e-5) == K.saturated(os_, dict(enumerate(oc)), 1e-5)


def test_maxmin_bench_big_vs_oracle():
    ps, os_ = L.System(False), O.System(False)
    _, pv, a, b = ps.gen_maxmin_bench(2, 0)
    _, ov, _, _ = os_.gen_maxmin_bench(2, 0)
    assert (a, b) == (807, 812)  # maxmin_bench_large.tesh
    ps.solve()
    os_.solve()
    worst, bad = K.compare_values(dict(enumerate(pv)), dict(enumerate(ov)))
    assert not bad, bad[:5]


# ---- random systems: penalties, bounds, FATPIPE, duplicates, zero bounds, staging ----------
@pytest.mark.parametrize("seed", range(40))
def test_random_maxmin_vs_oracle(seed):
    ops = K.random_script(seed, conc_limits=(seed % 2 == 0), frees=3, penalty_updates=4, bound_updates=4)
    ps, pcs, pvs = K.replay(L, ops)
    os_, ocs, ovs = K.replay(O, ops)
    ps.solve()
    os_.solve()
    worst, bad = K.compare_values(pvs, ovs)
    assert not bad, bad[:5]
    assert K.saturated(ps, pcs, 1e-5) == K.saturated(os_, ocs, 1e-5)


# The reference's bottleneck_solve does not terminate on some inputs: a variable dropped from the
# list keeps its last mu_ (possibly 0, e.g. after sitting on a zero-bound constraint) and FATPIPE
# constraints take min(usage, w*mu) over ALL enabled elements (fair_bottleneck.cpp:118-125), so their
# remaining never decreases again and their other variables grow forever.  The oracle hangs there
# too, so the random FairBottleneck systems avoid {zero-bound + FATPIPE} and zero weights; the
# product reports LMMHIP_E_NOCONVERGE instead of hanging (test below).
# FATPIPE systems can need millions of reference rounds (remaining shrinks geometrically); these
# seeds need <= 3000 (oracle last_rounds, scanned offline) so the device round budget covers them.
FB_FATPIPE_SEEDS = [0, 1, 3, 5, 6, 7, 9, 10, 12, 13, 15, 16, 17, 22, 23, 25, 30, 33, 37, 44]


@pytest.mark.parametrize("seed", range(20))
@pytest.mark.parametrize("variant", ["fatpipe", "zero_bounds"])
def test_random_fair_bottleneck_vs_oracle(seed, variant):
    if variant == "fatpipe":
        seed = FB_FATPIPE_SEEDS[seed]
    kw = dict(zero_bound_p=0.0, fatpipe_p=0.1) if variant == "fatpipe" else dict(zero_bound_p=0.05, fatpipe_p=0.0)
    ops = K.random_script(1000 + seed, conc_limits=(seed % 3 == 0), frees=2, bound_updates=3, zero_w_p=0.0, **kw)
    ps, pcs, pvs = K.replay(L, ops, kind=L.System.FAIR_BOTTLENECK)
    os_, ocs, ovs = K.replay(O, ops, kind=O.System.FAIR_BOTTLENECK)
    ps.solve()
    os_.solve()
    worst, bad = K.compare_values(pvs, ovs)
    assert not bad, bad[:5]


@pytest.mark.parametrize("kat", K.FB_TESH_KATS, ids=lambda f: f.__name__)
def test_fair_bottleneck_tesh_kats(kat):
    """FairBottleneck on the device vs the answers the reference's L07 tesh files print (the same KATs
    pin the oracle in tests/test_oracle.py)."""
    _, expect = kat(L)
    assert not K.check_fb_kat(expect)


def test_fair_bottleneck_nonterminating_input_is_reported():
    s = L.System(False, L.System.FAIR_BOTTLENECK)
    z = s.constraint_new(None, 0.0)  # zero-bound: its variable leaves the list with mu = 0
    f = s.constraint_new(None, 5.0)
    f.unshare()
    a = s.variable_new(None, 1.0, -1.0, 2)
    b = s.variable_new(None, 1.0, -1.0, 1)
    s.expand(z, a, 1.0)
    s.expand(f, a, 1.0)
    s.expand(f, b, 1.0)
    with pytest.raises(L.LmmError, match="round guard"):
        s.solve()


def test_resolve_after_mutations():
    # solve / mutate / solve again: the device state is fully re-initialised per solve
    ops = K.random_script(77, frees=0)
    ps, pcs, pvs = K.replay(L, ops)
    os_, ocs, ovs = K.replay(O, ops)
    for step in range(4):
        ps.solve()
        os_.solve()
        _, bad = K.compare_values(pvs, ovs)
        assert not bad, (step, bad[:5])
        more = K.random_script(500 + step, n_cnst=0, n_var=0, frees=0)  # empty
        upd = [("penalty", k, 2.0) for k in list(ovs)[step::7]] + [("vbound", k, 0.3) for k in list(ovs)[1 + step::9]]
        upd += [("cbound", k, 5.0 + step) for k in list(ocs)[step::5]] + [("free", k) for k in list(ovs)[2 + step::11]]
        K.replay(L, more + upd, sys_=ps, cs=pcs, vs=pvs)
        K.replay(O, more + upd, sys_=os_, cs=ocs, vs=ovs)


@pytest.mark.parametrize("seed", range(6))
def test_selective_update_vs_oracle(seed):
    ops = K.random_script(300 + seed, n_cnst=40, n_var=50, max_el=3, frees=0)
    ps, pcs, pvs = K.replay(L, ops, selective=True)
    os_, ocs, ovs = K.replay(O, ops, selective=True)
    for step in range(3):
        ps.solve()
        os_.solve()
        _, bad = K.compare_values(pvs, ovs)
        assert not bad, (step, bad[:5])
        assert sorted(v.rank for v in ps.modified_actions()) == sorted(v.rank for v in os_.modified_actions())
        ps.clear_modified_actions()
        os_.clear_modified_actions()
        keys = sorted(ovs)
        upd = [("vbound", keys[(step * 13 + seed) % len(keys)], 0.2 + step), ("cbound", step * 3 + 1, 3.0 + step)]
        K.replay(L, upd, sys_=ps, cs=pcs, vs=pvs)
        K.replay(O, upd, sys_=os_, cs=ocs, vs=ovs)


def test_edge_cases():
    # empty system
    s = L.System(False)
    s.solve()
    # constraints only, variables without constraints, disabled variables, zero-bound constraint
    s = L.System(False)
    c0 = s.constraint_new(None, 0.0)
    c1 = s.constraint_new(None, 4.0)
    a = s.variable_new(None, 1.0, -1.0, 2)
    b = s.variable_new(None, 0.0, -1.0, 1)  # disabled
    lone = s.variable_new(None, 1.0)  # no constraint
    s.expand(c0, a, 1.0)  # ignored: bound <= bound*prec (maxmin.cpp:524)
    s.expand(c1, a, 2.0)
    s.expand(c1, b, 1.0)
    s.solve()
    assert abs(a.get_value() - 2.0) < 1e-12
    assert b.get_value() == 0.0 and lone.get_value() == 0.0
    # bounded variable below its share
    s = L.System(False)
    c = s.constraint_new(None, 10.0)
    x = s.variable_new(None, 1.0, 1.5)
    y = s.variable_new(None, 1.0)
    s.expand(c, x, 1.0)
    s.expand(c, y, 1.0)
    s.solve()
    assert abs(x.get_value() - 1.5) < 1e-12 and abs(y.get_value() - 8.5) < 1e-12


def test_batched_medium_systems_vs_oracle():
    n = 32
    ps = [L.System(False) for _ in range(n)]
    pvs = [p.gen_maxmin_bench(1, i)[1] for i, p in enumerate(ps)]
    L.solve_batch(ps)
    for i in range(n):
        o = O.System(False)
        _, ov, _, _ = o.gen_maxmin_bench(1, i)
        o.solve()
        _, bad = K.compare_values(dict(enumerate(pvs[i])), dict(enumerate(ov)))
        assert not bad, (i, bad[:5])


@pytest.mark.parametrize("variant", ["plain", "stress"])
def test_synthetic_midsize_vs_oracle(variant):
    # C2-style generator at a size the O(R*L) oracle finishes in seconds
    kw = dict(penalty_mix=1, bounded_permille=100, fatpipe_permille=50) if variant == "stress" else {}
    ps, os_ = L.System(False), O.System(False)
    pv = ps.gen_synthetic(2000, 20000, 8, seed=3, **kw)
    ov = os_.gen_synthetic(2000, 20000, 8, seed=3, **kw)
    ps.solve()
    os_.solve()
    x = ps.values_of(pv)
    y = os_.values_of(ov, len(pv))
    tol = np.maximum(K.ABS_TOL, K.REL_TOL * np.abs(y))
    assert np.all(np.abs(x - y) <= tol), float(np.max(np.abs(x - y)))


def saturated_dense(f, x, prec):
    """Saturated constraints (maxmin.cpp print()'s test, `bound - usage <= bound * prec`) of the flattened
    system `f` (multi.export_flat) under the dense variable values `x`: usage = sum (FATPIPE: max) of w x."""
    rows = np.repeat(np.arange(len(f.penalty)), np.diff(f.var_ptr))
    wx = f.weight * x[rows]
    use = np.bincount(f.cnst_idx, weights=wx, minlength=len(f.cbound))
    fat = (f.cflags & 1).astype(bool)
    if fat.any():
        mx = np.zeros(len(f.cbound))
        np.maximum.at(mx, f.cnst_idx, wx)
        use = np.where(fat, mx, use)
    return np.flatnonzero(~(f.cbound - use > f.cbound * prec))


@pytest.mark.parametrize("variant", ["plain", "stress"])
def test_synthetic_c2_tenth_vs_oracle(variant):
    """The C2 generator at 1/10 scale (1e5 x 1e6 x 8, the bench's CPU-baseline sample: ~45k sequential
    reference rounds, maxmin.cpp:560-680) on the device against the oracle: every variable within
    K.ABS_TOL / K.REL_TOL and the same saturated constraint set."""
    from simgrid_amd import multi as M

    kw = dict(penalty_mix=1, bounded_permille=100, fatpipe_permille=50) if variant == "stress" else {}
    ps, os_ = L.System(False), O.System(False)
    pv = ps.gen_synthetic(100_000, 1_000_000, 8, seed=1, **kw)
    ov = os_.gen_synthetic(100_000, 1_000_000, 8, seed=1, **kw)
    f = M.export_flat(ps)
    ps.solve()
    os_.solve()
    x = ps.values_of(pv)
    y = os_.values_of(ov, len(pv))
    assert ps.last_stats()["n_var"] > 900_000
    tol = np.maximum(K.ABS_TOL, K.REL_TOL * np.abs(y))
    diff = np.abs(x - y)
    assert np.all(diff <= tol), (float(diff.max()), int(np.count_nonzero(diff > tol)))
    # dense variable i of the flat system is host variable f.var_ids[i]; the generator made pv in order
    pos = np.searchsorted(pv, f.var_ids) if np.all(np.diff(pv) > 0) else None
    assert pos is not None and np.array_equal(pv[pos], f.var_ids)
    prec = L.get_precision()
    np.testing.assert_array_equal(saturated_dense(f, x[pos], prec), saturated_dense(f, y[pos], prec))


@pytest.mark.slow
def test_synthetic_full_size_certificate():
    """C2 at full size (1e6 x 1e7 x 8): too big for the O(R*L) oracle, so check size-independent
    max-min properties: feasibility of every constraint and the bottleneck certificate (each
    variable with x > 0 has a saturated constraint on which its level x*p is maximal)."""
    s = L.System(False)
    vids = s.gen_synthetic(1_000_000, 10_000_000, 8, seed=1)
    s.solve()
    st = s.last_stats()
    assert st["n_var"] > 9_000_000 and st["rounds"] > 0
    x = s.values_of(vids)
    assert np.all(np.isfinite(x)) and np.all(x >= 0)
    assert np.count_nonzero(x) > 0.99 * len(x)
    excess, n_inf, n_unb = s.check_certificate()
    assert n_inf == 0 and excess <= 1e-5, (excess, n_inf)
    assert n_unb == 0, n_unb


@pytest.mark.parametrize("variant", ["plain", "stress"])
def test_synthetic_certificate_matches_oracle_certificate(variant):
    # the certificate itself is validated on a size where the oracle runs: both solutions pass it
    kw = dict(penalty_mix=1, bounded_permille=100, fatpipe_permille=50) if variant == "stress" else {}
    ps = L.System(False)
    ps.gen_synthetic(5000, 50000, 8, seed=5, **kw)
    ps.solve()
    excess, n_inf, n_unb = ps.check_certificate()
    assert n_inf == 0 and n_unb == 0, (excess, n_inf, n_unb)


def test_c_client_drives_a_solve():
    """tests/c/abi_drive.c: a plain C client of include/lmm/lmm_system.h + lmm_hip.h solves the
    maxmin_test.cpp:17-42 system and the exec-ptask L07 system on the device."""
    import subprocess

    from tests.test_abi import build_c_drive

    r = subprocess.run([build_c_drive()], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "abi_drive: ok" in r.stdout


@pytest.mark.slow
@pytest.mark.timeout(600)
@pytest.mark.parametrize("variant", ["plain", "stress"])
def test_synthetic_full_size_vs_oracle_sample(variant):
    """C2 at FULL size (1e6 x 1e7 x 8, seed 1) against the oracle's own solve of the same system, made once in
    the build container (tests/golden/make_c2_full_sample.py; the O(rounds x constraints) reference loop,
    maxmin.cpp:560-680): a fixed random sample of 1e5 variables within K.ABS_TOL / K.REL_TOL, and the
    saturated-constraint set (maxmin.cpp print()'s test over every constraint) identical bit for bit.
    `stress`: the bench's --variant stress system (5 % FATPIPE constraints, 10 % bounded variables, penalties
    {1, 2, 4}; make_c2_full_sample.py --stress)."""
    import os

    from simgrid_amd import multi as M
    from tests.golden.make_c2_full_sample import STRESS_KW, flat_sha256, saturated_bits

    name = "c2_full_sample.npz" if variant == "plain" else "c2_stress_full_sample.npz"
    path = os.path.join(os.path.dirname(__file__), "golden", name)
    if not os.path.exists(path):
        pytest.skip(f"{name} not generated (tests/golden/make_c2_full_sample.py)")
    fx = np.load(path)
    s = L.System(False)
    vids = s.gen_synthetic(1_000_000, 10_000_000, 8, seed=1, **(STRESS_KW if variant == "stress" else {}))
    f = M.export_flat(s)
    assert flat_sha256(f) == str(fx["csr_sha256"]), "not the system the oracle solved"
    assert np.array_equal(f.var_ids, vids)
    s.solve()
    x = s.values_of(vids)
    idx, y = fx["sample_idx"], fx["sample_x"]
    tol = np.maximum(K.ABS_TOL, K.REL_TOL * np.abs(y))
    diff = np.abs(x[idx] - y)
    assert np.all(diff <= tol), (float(diff.max()), int(np.count_nonzero(diff > tol)))
    got = saturated_bits(f, x, L.get_precision())
    assert np.array_equal(got, fx["sat_bits"]), int(np.count_nonzero(np.unpackbits(got) != np.unpackbits(fx["sat_bits"])))
