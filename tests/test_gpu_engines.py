"""Max-min engines and determinism on the device.

* The persistent engine (ONE cooperative launch per solve, lmm_persist_kernels.hpp) and the multi-launch
  round engine run the same phase bodies: their values must be identical bit for bit.
* System::lmm_solve is sequential and bit-reproducible in the reference (maxmin.cpp:601-606); the device
  sums a round's decrements as fixed-point integers (CstRec in lmm_dev.hpp), so two solves of the same
  system must give identical bytes too.
* The stream ABI: lmmhip_ctx_set_stream(0) is the legacy null stream (torch's default stream), so a
  FairBottleneck solve sharded on torch's default stream is ordered and correct.
"""
import numpy as np
import pytest

from oracle import pyoracle as O
from simgrid_amd import lmm as L
from simgrid_amd import multi as M
from tests import lmm_cases as K

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if L.device_count() == 0:
        pytest.fail("no HIP device visible: the GPU tests must run on the MI355X")


def _synthetic(nc, nv, seed, stress):
    kw = dict(penalty_mix=1, bounded_permille=100, fatpipe_permille=50) if stress else {}

    def build(s):
        return s.gen_synthetic(nc, nv, 8, seed=seed, **kw)
    return build


def _bench(klass, run):
    def build(s):
        return np.array([v.h for v in s.gen_maxmin_bench(klass, run)[1]], dtype=np.int64)
    return build


def _platform(n_flows, seed):
    def build(s):
        _, vs = s.gen_platform_flows(L.platform_params(topology=L.FAT_TREE, topo_parameters="3;8,8,8;1,8,4;1,1,2",
                                                       loopback_bw=1e9, model=L.LV08, n_flows=n_flows, seed=seed))
        return vs
    return build


def _values(build, engine):
    s = L.System(False)
    ids = build(s)
    s.set_engine(engine)
    s.solve()
    return s.values_of(ids), s.last_stats()["rounds"]


CASES = {
    "synthetic_2e3x2e4": _synthetic(2000, 20000, 3, False),
    "synthetic_2e3x2e4_stress": _synthetic(2000, 20000, 3, True),
    "synthetic_2e4x2e5": _synthetic(20000, 200000, 7, False),
    "synthetic_1e5x1e6_stress": _synthetic(100000, 1000000, 11, True),
    "medium_run3": _bench(1, 3),
    "small_run7": _bench(0, 7),
    "big_run0": _bench(2, 0),
    "fattree_lv08_5000": _platform(5000, 2),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_frontier_engine_bit_identical(name):
    """The frontier engine (votes registered at their target, lmm_frontier_kernels.hpp) takes the same
    decisions as the round engine: identical values bit for bit and the same number of rounds."""
    xf, rf = _values(CASES[name], L.System.ENGINE_FRONTIER)
    xr, rr = _values(CASES[name], L.System.ENGINE_ROUNDS)
    assert rf == rr
    assert xf.tobytes() == xr.tobytes(), float(np.max(np.abs(xf - xr)))


def _launches(s):
    """Per-slot kernel launches of the last solve (lmmhip_stats.kernel_launches: 2 vote / persistent, 4 saturation,
    5 update)."""
    import ctypes as ct

    st = L.LmmhipStats()
    assert L.lib().lmmhip_get_stats(s.device_ctx(), ct.byref(st)) == 0
    return list(st.kernel_launches)


@pytest.mark.parametrize("name", sorted(CASES))
def test_engines_bit_identical(name):
    xp, rp = _values(CASES[name], L.System.ENGINE_PERSISTENT)
    xr, rr = _values(CASES[name], L.System.ENGINE_ROUNDS)
    assert rp == rr
    assert xp.tobytes() == xr.tobytes(), float(np.max(np.abs(xp - xr)))


@pytest.mark.parametrize("engine", [0, 1])
def test_persistent_engine_vs_oracle(engine):
    ps, os_ = L.System(False), O.System(False)
    pv = ps.gen_synthetic(2000, 20000, 8, seed=9, penalty_mix=1, bounded_permille=100, fatpipe_permille=50)
    ov = os_.gen_synthetic(2000, 20000, 8, seed=9, penalty_mix=1, bounded_permille=100, fatpipe_permille=50)
    ps.set_engine(engine)
    ps.solve()
    os_.solve()
    x, y = ps.values_of(pv), os_.values_of(ov, len(pv))
    assert np.all(np.abs(x - y) <= np.maximum(K.ABS_TOL, K.REL_TOL * np.abs(y))), float(np.max(np.abs(x - y)))


@pytest.mark.parametrize("engine", [0, 1])
def test_run_to_run_identical_stress(engine):
    """The 2e3 x 2e4 stress system (penalties {1,2,4}, 10 % bounded, 5 % FATPIPE) solved twice."""
    a, _ = _values(_synthetic(2000, 20000, 3, True), engine)
    b, _ = _values(_synthetic(2000, 20000, 3, True), engine)
    assert a.tobytes() == b.tobytes()


def test_run_to_run_identical_resolve_same_system():
    s = L.System(False)
    ids = s.gen_synthetic(20000, 200000, 8, seed=5, penalty_mix=1, bounded_permille=100, fatpipe_permille=50)
    s.solve()
    a = s.values_of(ids)
    for _ in range(3):
        s.solve()
        assert s.values_of(ids).tobytes() == a.tobytes()


def test_run_to_run_identical_c3_batch():
    """A C3-style batch of maxmin_bench medium systems (disjoint union) solved twice."""
    out = []
    for _ in range(2):
        ps = [L.System(False) for _ in range(256)]
        vs = [p.gen_maxmin_bench(1, i)[1] for i, p in enumerate(ps)]
        L.solve_batch(ps)
        out.append(np.array([v.get_value() for vv in vs for v in vv]))
    assert out[0].tobytes() == out[1].tobytes()


def test_fb_sharded_on_torch_default_stream():
    """lmmhip_ctx_set_stream(0) = the legacy null stream: shards on torch's default stream are ordered
    with the torch-side exchanges of fb_solve_sharded (handle 0 used to mean "own stream")."""
    import torch

    from tests.test_gpu_multi import device_shard_maker
    from tests.test_multi import fb_pair, oracle_dense_values, sharded_fb_values

    s, o, ovars = fb_pair()
    f = M.export_flat(s)
    shards = []
    stream = torch.cuda.default_stream()
    x, _ = sharded_fb_values(f, M.LocalExchange(), 2, device_shard_maker(shards, stream), device=True,
                             stream=stream)
    for sh in shards:
        sh.close()
    want = oracle_dense_values(o, ovars, f)
    assert x.tobytes() == want.tobytes()


def test_fb_device_shards_over_gloo():
    """DistExchange on gloo with device-resident exchange buffers (the all-reduce and the all-gathers copy
    through the CPU): a world-1 gloo group in this process."""
    import os

    import torch.distributed as dist

    from tests.test_gpu_multi import device_shard_maker
    from tests.test_multi import fb_pair, oracle_dense_values, sharded_fb_values

    s, o, ovars = fb_pair(seed=6)
    f = M.export_flat(s)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29561")
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        shards = []
        x, _ = sharded_fb_values(f, M.DistExchange(), 2, device_shard_maker(shards), device=True)
        for sh in shards:
            sh.close()
    finally:
        dist.destroy_process_group()
    want = oracle_dense_values(o, ovars, f)
    assert x.tobytes() == want.tobytes()


@pytest.mark.parametrize("stress", [False, True])
def test_round_engine_variants_bit_identical(stress, monkeypatch):
    """The round engine's vote / ready variants give the same bytes on the C2/10 system (1e5 x 1e6 x 8):
    (LMMHIP_CREC, LMMHIP_RDQ, LMMHIP_VOTE_BITS) — the packed row records, the ready constraints listed by the update
    and the vote (no mm_ready pass), and the vote's filter on the change stamps instead of the LDS bitmap.  (The
    target-ordered rows, the saturation's row retirement and the ready candidates as records were measured slower
    on every configuration and removed in round 6)"""
    out = []
    for crec, rdq, bits in (("0", "0", "1"), ("1", "0", "1"), ("1", "1", "1"), ("1", "1", "0")):
        monkeypatch.setenv("LMMHIP_CREC", crec)
        monkeypatch.setenv("LMMHIP_RDQ", rdq)
        monkeypatch.setenv("LMMHIP_VOTE_BITS", bits)
        out.append(_values(_synthetic(100000, 1000000, 1, stress), L.System.ENGINE_ROUNDS))
    for o in out[1:]:
        assert out[0][1] == o[1]
        assert out[0][0].tobytes() == o[0].tobytes(), float(np.max(np.abs(out[0][0] - o[0])))


def test_persistent_engine_concurrent_contexts_and_torch():
    """The persistent engine's grid barriers need all its workgroups co-resident.  Two Systems (two contexts,
    two streams) solving at the same time from two host threads, and a solve while torch matmuls run on
    another stream, must return the round engine's values: persistent launches are serialised per device,
    and a barrier timeout (a grid that could not become co-resident) re-runs the solve on the round engine
    instead of failing."""
    import threading

    import torch

    build = _platform(5000, 2)
    ref, _ = _values(build, L.System.ENGINE_ROUNDS)
    systems = []
    for _ in range(2):
        s = L.System(False)
        ids = build(s)
        s.set_engine(L.System.ENGINE_PERSISTENT)
        systems.append((s, ids))
    out, errs = [None, None], []

    def run(k):
        try:
            s, ids = systems[k]
            for _ in range(4):
                s.solve()
            out[k] = s.values_of(ids)
        except Exception as e:  # noqa: BLE001 (reported below)
            errs.append(repr(e))

    th = [threading.Thread(target=run, args=(k,)) for k in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=100)
    assert not errs, errs
    for k in range(2):
        assert out[k] is not None and out[k].tobytes() == ref.tobytes()
    assert systems[0][0].engine_fallbacks() == 0 and systems[1][0].engine_fallbacks() == 0
    # a persistent solve while torch kernels occupy the chip from another stream
    s, ids = systems[0]
    side = torch.cuda.Stream()
    a = torch.randn(4096, 4096, device="cuda")
    with torch.cuda.stream(side):
        for _ in range(30):
            a = torch.tanh(a @ a * 1e-3)
    s.solve()
    torch.cuda.synchronize()
    assert s.values_of(ids).tobytes() == ref.tobytes()


def test_persistent_rendezvous_deadline_falls_back_fast():
    """A persistent solve whose grid cannot become co-resident — half the CUs held for 2 s by a kernel of another
    process (tests/c/occupy_run.py, tests/c/occupy.hip: the one-process-per-GPU deployment's neighbour) — closes
    its launch rendezvous after LMMHIP_PERSIST_RDV_MS (20 ms) and re-runs on the round engine on the free CUs
    (lmm_persist_kernels.hpp bar_rdv, lmm_hip.hip solve_maxmin_persist): the values are the round engine's bytes,
    one fallback is counted, the solve returns well within the 2 s the CUs stay held (< 0.5 s), and the next solve
    of the context takes the round engine directly (cooldown) instead of waiting again."""
    import os
    import subprocess
    import sys
    import time

    build = _platform(5000, 2)
    ref, _ = _values(build, L.System.ENGINE_ROUNDS)
    s = L.System(False)
    ids = build(s)
    s.set_engine(L.System.ENGINE_PERSISTENT)
    s.set_resident(False)  # (host flatten: prepare / device_solve / fetch re-solve the unchanged system)
    s.prepare()
    s.device_solve()
    s.fetch()
    assert s.engine_fallbacks() == 0 and s.values_of(ids).tobytes() == ref.tobytes()
    script = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c", "occupy_run.py")
    p = subprocess.Popen([sys.executable, script, "0", "2.0"], stdout=subprocess.PIPE, text=True)
    try:
        line = p.stdout.readline()
        assert line.startswith("RUNNING"), line
        t0 = time.time()
        t = time.perf_counter()
        s.device_solve()  # (the system is unchanged: System::solve would not run the solver again)
        wall = time.perf_counter() - t
        s.fetch()
        vals, fb = s.values_of(ids), s.engine_fallbacks()
        t = time.perf_counter()
        s.device_solve()  # cooldown: the round engine directly
        wall2 = time.perf_counter() - t
        s.fetch()
        vals2, fb2 = s.values_of(ids), s.engine_fallbacks()
        held = time.time() - t0 < 1.5 and p.poll() is None
        assert p.wait(timeout=60) == 0
    finally:
        if p.poll() is None:
            p.kill()
    assert vals.tobytes() == ref.tobytes() and vals2.tobytes() == ref.tobytes()
    assert held, "the CUs were released before the solves ended: the check is void"
    assert fb == 1 and fb2 == 1, (fb, fb2, wall, wall2)
    assert wall < 0.5 and wall2 < 0.5, (wall, wall2)


def test_frontier_duplicate_elements_on_a_high_degree_constraint():
    """A constraint holding two elements of each of its 40,000 variables (cdup, as a route crossing a link twice
    or a flow's cross-traffic element on its own link): the frontier engine's CSR -> CSC map (fr_c2s) counts a
    variable's earlier occurrences over the run of equal ids only, so the first solve stays fast (ADVICE r04:
    the full rescan was O(degree^2) in one wave), and the values equal the round engine's bit for bit."""
    import time

    def build(s):
        big = s.constraint_new(None, 1e6)
        vs = []
        for i in range(40_000):
            c = s.constraint_new(None, 1.0 + (i % 97))
            v = s.variable_new(None, 1.0 + (i % 3), -1.0, 3)
            s.expand(big, v, 1.0)
            s.expand(c, v, 1.0)
            s.expand(big, v, 0.05 * (1 + i % 5))
            vs.append(v.h)
        return np.array(vs, dtype=np.int64)

    s = L.System(False)
    ids = build(s)
    s.set_engine(L.System.ENGINE_FRONTIER)
    t = time.perf_counter()
    s.solve()
    first = time.perf_counter() - t
    xf = s.values_of(ids)
    xr, _ = _values(build, L.System.ENGINE_ROUNDS)
    assert xf.tobytes() == xr.tobytes(), float(np.max(np.abs(xf - xr)))
    assert first < 2.0, first



def _hint_steps(s, ids, step):
    """Mutations of the round-hint test: step 1 bounds a third of the variables tightly (early bound fixes: a
    different round count), step 2 lifts them again (the first system back)."""
    if step == 0:
        return
    for h in ids[::3]:
        s.update_variable_bound(L.Variable(s, int(h)), 1e-4 if step == 1 else -1.0)


@pytest.mark.parametrize("engine", [L.System.ENGINE_ROUNDS, L.System.ENGINE_FRONTIER])
def test_round_hint_other_round_counts_bit_identical(engine):
    """The chunked polls end a chunk where the previous solve of the context ended (round_hint_chunk, lmm_hip.hip):
    a solve that takes more or fewer rounds than the previous one must still give a fresh context's bytes."""
    build = _synthetic(20000, 200000, 5, False)
    s = L.System(False)
    ids = build(s)
    s.set_engine(engine)
    rounds = []
    for step in (0, 1, 2, 1):
        _hint_steps(s, ids, step)
        s.solve()
        x, r = s.values_of(ids), s.last_stats()["rounds"]
        f = L.System(False)  # fresh context: the same system, no hint
        fids = build(f)
        for k in range(1, step + 1 if step < 2 else 3):
            _hint_steps(f, fids, k)
        f.set_engine(engine)
        f.solve()
        xf, rf = f.values_of(fids), f.last_stats()["rounds"]
        assert r == rf, (step, r, rf)
        assert x.tobytes() == xf.tobytes(), (step, float(np.max(np.abs(x - xf))))
        rounds.append(r)
    assert len(set(rounds)) > 1, rounds  # (the hint was wrong at least once)
