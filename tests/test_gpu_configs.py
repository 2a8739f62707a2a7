"""Parity at the BASELINE.json configurations' own sizes, not scaled-down stand-ins.

* C3: all 4096 maxmin_bench "medium" systems (maxmin_bench.cpp:110-116, seeds 1..4096), both as one
  disjoint-union system (bench.py --workload c3) and as 4096 systems through lmm_solve_batch, against
  the oracle system by system (seeds 1..5 are also golden-pinned in test_gpu_parity.py).
* C4: 1e5 LV08 flows on the 4096-host fat tree 3;16,16,16;1,16,16;1,1,1 against the oracle.
* C5: FairBottleneck with L07 flows on the dragonfly 8,4;16,3;8,2;4 — 1e6 flows against the oracle, and
  at the full 1e7 flows the size-independent properties of bottleneck_solve's fixed point
  (fair_bottleneck.cpp:59-145): every value finite and > 0, every shared constraint feasible, every
  variable stopped by an erased constraint or its bound; plus agreement with the variable-sharded
  device solve (multi.py), which reduces in a different order.
Tolerances: tests/lmm_cases.py.
"""
import numpy as np
import pytest

from oracle import pyoracle as O
from simgrid_amd import lmm as L
from simgrid_amd import multi as M
from tests import lmm_cases as K

pytestmark = pytest.mark.gpu

C4_PLATFORM = dict(topology=L.FAT_TREE, topo_parameters="3;16,16,16;1,16,16;1,1,1", loopback_bw=1e8)
C5_PLATFORM = dict(topology=L.DRAGONFLY, topo_parameters="8,4;16,3;8,2;4", loopback_bw=1e9, limiter_bw=2e8)


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if L.device_count() == 0:
        pytest.fail("no HIP device visible: the GPU tests must run on the MI355X")


@pytest.fixture(scope="module")
def c3_oracle():
    """Oracle values of the 4096 medium systems (one disjoint-union system: identical per system)."""
    o = O.System(False)
    vs = []
    for i in range(4096):
        vs.extend(o.gen_maxmin_bench(1, i)[1])
    o.solve()
    return np.array([v.get_value() for v in vs])


@pytest.fixture(scope="module")
def c3_oracle_saturated():
    """The oracle's saturated set of the 4096 medium systems (SURVEY.md A.6 through Constraint::get_usage,
    maxmin.cpp:948-961): (system, constraint position) pairs."""
    out = set()
    for i in range(4096):
        o = O.System(False)
        cs = o.gen_maxmin_bench(1, i)[0]
        o.solve()
        out |= {(i, k) for k in K.saturated(o, dict(enumerate(cs)), L.get_precision())}
    return out


def _sat_dense(f, x, prec):
    """Saturated constraints (NOT double_positive(bound - get_usage(), bound * prec), with get_usage =
    sum, FATPIPE max, of w x over the constraint's elements, maxmin.cpp:948-961 / :470-480) of the flattened system
    `f` under dense values `x`, as a boolean per dense constraint."""
    rows = np.repeat(np.arange(len(f.penalty)), np.diff(f.var_ptr))
    wx = f.weight * x[rows]
    use = np.bincount(f.cnst_idx, weights=wx, minlength=len(f.cbound))
    fat = (f.cflags & 1).astype(bool)
    if fat.any():
        mx = np.zeros(len(f.cbound))
        np.maximum.at(mx, f.cnst_idx, wx)
        use = np.where(fat, mx, use)
    return ~(f.cbound - use > f.cbound * prec)


def _close(x, y):
    tol = np.maximum(K.ABS_TOL, K.REL_TOL * np.abs(y))
    bad = np.nonzero(~(np.abs(x - y) <= tol))[0]
    return bad, (float(np.max(np.abs(x - y))) if len(x) else 0.0)


def test_c3_disjoint_union_vs_oracle(c3_oracle, c3_oracle_saturated):
    s = L.System(False)
    ids, cs = [], {}
    for i in range(4096):
        c, v, _, _ = s.gen_maxmin_bench(1, i)
        ids.extend(x.h for x in v)
        cs.update({(i, k): ck for k, ck in enumerate(c)})
    f = M.export_flat(s)
    s.solve()
    x = s.values_of(np.array(ids, np.int64))
    bad, worst = _close(x, c3_oracle)
    assert len(bad) == 0, (len(bad), worst)
    assert s.last_stats()["n_var"] > 100_000
    # the same saturated set: through the drop-in Constraint::get_usage of every constraint, and the
    # device's own (mm_saturated) against the oracle's values on the flattened system
    assert K.saturated(s, cs, L.get_precision()) == c3_oracle_saturated
    pos = {int(h): j for j, h in enumerate(ids)}
    y = c3_oracle[[pos[int(h)] for h in f.var_ids]]
    np.testing.assert_array_equal(s.device_saturated(), _sat_dense(f, y, L.get_precision()))


def test_c3_solve_batch_vs_oracle(c3_oracle):
    ps = [L.System(False) for _ in range(4096)]
    ids = [np.array([v.h for v in p.gen_maxmin_bench(1, i)[1]], np.int64) for i, p in enumerate(ps)]
    L.solve_batch(ps)
    x = np.concatenate([p.values_of(i) for p, i in zip(ps, ids)])
    bad, worst = _close(x, c3_oracle)
    assert len(bad) == 0, (len(bad), worst)


def test_c3_device_batch_vs_oracle_and_global_engine(c3_oracle, monkeypatch):
    """bench.py --workload c3: the 4096 systems as one block-diagonal upload (multi.DeviceBatch,
    lmmhip_set_batch) solved by the LDS kernel (one workgroup per system), against the oracle, against
    the global engine on the same upload (LMMHIP_BATCH=0), and run to run."""
    ps = [L.System(False) for _ in range(4096)]
    hid = [np.array([v.h for v in p.gen_maxmin_bench(1, i)[1]], np.int64) for i, p in enumerate(ps)]
    b = M.DeviceBatch(ps)
    b.solve()
    x = b.values()
    b.solve()
    assert b.values().tobytes() == x.tobytes()  # deterministic
    rounds = b.stats()["rounds"]
    # dense order of system i -> oracle order (its variables in creation order)
    y = c3_oracle
    xo = np.zeros(len(y))  # variables outside the solved system (disabled by staging) stay at 0
    k = 0
    for i in range(4096):
        pos = {int(h): j for j, h in enumerate(b.var_ids[i])}
        for h in hid[i]:
            j = pos.get(int(h))
            if j is not None:
                xo[k] = x[b.var_off[i] + j]
            k += 1
    bad, worst = _close(xo, y)
    assert len(bad) == 0, (len(bad), worst)
    # the same saturated set: the batch kernel's device set against the oracle's values on the
    # concatenated flattened systems
    yd = np.zeros(b.n_var)
    k = 0
    for i in range(4096):
        pos = {int(h): j for j, h in enumerate(hid[i])}
        for j, h in enumerate(b.var_ids[i]):
            yd[b.var_off[i] + j] = y[k + pos[int(h)]]
        k += len(hid[i])
    prec = L.get_precision()
    sat_b = b.saturated()
    np.testing.assert_array_equal(sat_b, _sat_dense(b.flat(), yd, prec))
    monkeypatch.setenv("LMMHIP_BATCH", "0")
    b.solve()
    xg = b.values()
    bad, worst = _close(x, xg)
    assert len(bad) == 0, (len(bad), worst)
    np.testing.assert_array_equal(b.saturated(), sat_b)  # the global engine: the same set
    assert 0 < rounds <= 64
    b.close()


def test_c3_batch_goldens():
    """The LDS batch kernel on the golden-pinned medium seeds 1..5 (maxmin_bench_medium.tesh)."""
    import json
    import os

    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "maxmin_bench_medium.json")) as f:
        d = json.load(f)
    ps, vs = [], []
    for r in d["runs"]:
        ps.append(L.System(False))
        vs.append(ps[-1].gen_maxmin_bench(1, r["run"])[1])
    L.solve_batch(ps)  # lmm_solve_batch declares the batch: the LDS kernel
    for r, vv in zip(d["runs"], vs):
        for rk, (pen, val) in r["values"].items():
            got = vv[int(rk) - 1].get_value()
            assert abs(got - val) <= K.GOLDEN_TOL, (r["run"], rk, got, val)


def test_c4_full_size_vs_oracle():
    p = dict(model=L.LV08, n_flows=100_000, seed=1, **C4_PLATFORM)
    s, o = L.System(False), O.System(False)
    pc, vs = s.gen_platform_flows(L.platform_params(**p))
    oc, ov = o.gen_platform_flows(O.platform_params(**p))
    f = M.export_flat(s)
    s.solve()
    o.solve()
    x, y = s.values_of(vs), o.values_of(ov, len(vs))
    bad, worst = _close(x, y)
    assert len(bad) == 0, (len(bad), worst)
    assert np.all(y > 0)
    # the same saturated set (maxmin.cpp:948-961 / :470-480): every link through the drop-in
    # Constraint::get_usage, and the device's own (mm_saturated) against the oracle's values on the flattened system
    prec = L.get_precision()
    sat_p = K.saturated(s, {k: L.Constraint(s, int(c)) for k, c in enumerate(pc)}, prec)
    sat_o = K.saturated(o, dict(enumerate(oc)), prec)
    assert sat_p == sat_o and len(sat_o) > 0, (len(sat_p ^ sat_o), len(sat_o))
    pos = {int(h): j for j, h in enumerate(vs)}
    yd = y[[pos[int(h)] for h in f.var_ids]]
    np.testing.assert_array_equal(s.device_saturated(), _sat_dense(f, yd, prec))
    excess, infeasible, unbottlenecked = s.check_certificate()
    assert infeasible == 0 and unbottlenecked == 0, (excess, infeasible, unbottlenecked)


@pytest.fixture(scope="module")
def c5_1e6_oracle():
    p = dict(model=L.L07, n_flows=1_000_000, seed=1, **C5_PLATFORM)
    o = O.System(False, O.System.FAIR_BOTTLENECK)
    _, ov = o.gen_platform_flows(O.platform_params(**p))
    o.solve()
    return p, o.values_of(ov, p["n_flows"])


# LMMHIP_FB_LONG: shared constraints with at least this many elements chain increments precomputed by fbk_acc,
# shorter ones compute them inside the chain (fb_chain_pull); the C5 1e6 system's longest holds ~1.6e4
# w3: the long chains over 3 workgroups (each then takes many of them) instead of the default 128
@pytest.mark.parametrize("longmin", ["default", "0", "4096", "1000000000", "4096w3"])
def test_c5_1e6_flows_vs_oracle(c5_1e6_oracle, longmin, monkeypatch):
    if longmin.endswith("w3"):
        monkeypatch.setenv("LMMHIP_FB_LONG", longmin[:-2])
        monkeypatch.setenv("LMMHIP_FB_LONGWG", "3")
    elif longmin != "default":
        monkeypatch.setenv("LMMHIP_FB_LONG", longmin)
    p, y = c5_1e6_oracle
    s = L.System(False, L.System.FAIR_BOTTLENECK)
    _, vs = s.gen_platform_flows(L.platform_params(**p))
    s.solve()
    x = s.values_of(vs)
    bad, worst = _close(x, y)
    assert len(bad) == 0, (len(bad), worst)
    # one context, elements in the reference's list order: the same floating-point operations in the
    # same order as bottleneck_solve -> the same bytes
    assert x.tobytes() == y.tobytes(), int(np.count_nonzero(x != y))


def fb_fixed_point_violations(flat, x, erased, prec=1e-5):
    """Size-independent properties of bottleneck_solve's result on the solved (flattened) system.
    Returns (non-finite / non-positive values, infeasible shared constraints, unstopped variables)."""
    nv, nc = len(flat["pen"]), len(flat["cbound"])
    vp = flat["var_ptr"].astype(np.int64)
    rows = np.repeat(np.arange(nv), np.diff(vp))
    bad_x = int(np.count_nonzero(~np.isfinite(x) | ~(x > 0)))
    use = np.bincount(flat["csr_c"], weights=flat["csr_w"] * x[rows], minlength=nc)
    shared = (flat["cflags"] & 1) == 0
    b = flat["cbound"]
    # consumption is over-counted by the frozen variables' stale increments (fair_bottleneck.cpp:111-116),
    # so the real usage stays within the bound up to the double_update clamp (sg_maxmin_precision)
    infeasible = int(np.count_nonzero(shared & (use > b + np.maximum(prec, 1e-9 * b))))
    stopped_by_cnst = np.zeros(nv, bool)
    np.logical_or.at(stopped_by_cnst, rows, erased[flat["csr_c"]])
    vb = flat["vbound"]
    at_bound = (vb > 0) & (x == vb)  # fair_bottleneck.cpp:101: exact
    unstopped = int(np.count_nonzero(~(stopped_by_cnst | at_bound)))
    return bad_x, infeasible, unstopped


@pytest.mark.slow
def test_c5_full_size_fixed_point_properties():
    s = L.System(False, L.System.FAIR_BOTTLENECK)
    s.gen_platform_flows(L.platform_params(model=L.L07, n_flows=10_000_000, seed=1, **C5_PLATFORM),
                         want_vars=False)
    s.solve()
    st = s.last_stats()
    assert st["n_var"] == 10_000_000 and st["rounds"] > 0
    flat = s.device_flat()
    x = s.device_values()
    erased = s.device_saturated()
    bad_x, infeasible, unstopped = fb_fixed_point_violations(flat, x, erased)
    assert (bad_x, infeasible, unstopped) == (0, 0, 0)


@pytest.mark.slow
@pytest.mark.timeout(600)
def test_c5_full_size_vs_oracle_sample():
    """C5 at FULL size (1e7 L07 flows on the dragonfly, seed 1) against the oracle's own FairBottleneck solve of
    the same system, made once in the build container (tests/golden/make_c5_full_sample.py): the flattened
    system hashes to the one the fixture was made from, and a fixed random sample of 1e5 flows is equal BYTE for
    byte — the one-context solve runs the reference's floating-point operations in the reference's element
    order (fair_bottleneck.cpp:23-153), so not a tolerance but the same bits."""
    import os

    from tests.golden.make_c5_full_sample import flat_sha256

    fx = np.load(os.path.join(os.path.dirname(__file__), "golden", "c5_full_sample.npz"))
    s = L.System(False, L.System.FAIR_BOTTLENECK)
    _, vs = s.gen_platform_flows(L.platform_params(model=L.L07, n_flows=int(fx["n_flows"]), seed=1, **C5_PLATFORM))
    f = M.export_flat(s)
    assert flat_sha256(f) == str(fx["flat_sha256"]), "not the system the oracle solved"
    del f
    s.solve()
    x = s.values_of(vs)
    idx, y = fx["sample_idx"], fx["sample_x"]
    assert x[idx].tobytes() == y.tobytes(), (int(np.count_nonzero(x[idx] != y)), s.last_stats()["rounds"],
                                             int(fx["oracle_rounds"]))
    assert bool(np.all(x > 0)) == bool(fx["all_positive"])


def test_c5_fixed_point_properties_hold_on_the_oracle_solution():
    """The property check itself, validated where the oracle runs: the oracle's values pass it."""
    p = dict(model=L.L07, n_flows=20_000, seed=3, **C5_PLATFORM)
    s, o = L.System(False, L.System.FAIR_BOTTLENECK), O.System(False, O.System.FAIR_BOTTLENECK)
    _, vs = s.gen_platform_flows(L.platform_params(**p))
    _, ov = o.gen_platform_flows(O.platform_params(**p))
    s.solve()
    o.solve()
    x_host = s.values_of(vs)  # before export_flat: a flatten resets the host values (fair_bottleneck.cpp:30)
    flat = s.device_flat()
    erased = s.device_saturated()
    assert fb_fixed_point_violations(flat, s.device_values(), erased) == (0, 0, 0)
    # the oracle's values in the device's dense order (host ids of the dense variables: lmm_flat_export)
    pos = {int(h): k for k, h in enumerate(vs)}
    y = o.values_of(ov, len(vs))
    y_dense = y[[pos[int(h)] for h in M.export_flat(s).var_ids]]
    assert fb_fixed_point_violations(flat, y_dense, erased) == (0, 0, 0)
    bad, worst = _close(x_host, y)
    assert len(bad) == 0, (len(bad), worst)
    assert x_host.tobytes() == y.tobytes()  # bit-identical (fbk_update_seq, reference element order)


@pytest.mark.parametrize("parts", [2, 3, 8])
def test_c5_sharded_matches_single_context(parts):
    """The constraint-owner sharded FairBottleneck (multi.FbShardPlan: counts all-reduced, mu and the owned
    remaining values all-gathered, each owner chaining its constraints in the reference's element order)
    against the single-context solve of the same 1e6-flow system: the same bytes."""
    from tests.test_gpu_multi import device_shard_maker
    from tests.test_multi import sharded_fb_values

    s = L.System(False, L.System.FAIR_BOTTLENECK)
    _, vs = s.gen_platform_flows(L.platform_params(model=L.L07, n_flows=1_000_000, seed=2, **C5_PLATFORM))
    f = M.export_flat(s)
    s.solve()
    want = s.values_of(f.var_ids)
    shards = []
    x, _ = sharded_fb_values(f, M.LocalExchange(), parts, device_shard_maker(shards), device=True)
    for sh in shards:
        sh.close()
    assert x.tobytes() == want.tobytes(), int(np.count_nonzero(x != want))
