"""Multi-GPU layer (simgrid_amd/multi.py) on CPU: partitioning, connected components,
and world-size-2 gloo runs of the component-sharded solve and of the next-event all-reduce.  The
per-rank sub-solves run in the oracle here (no GPU); tests/test_gpu_multi.py runs them on the device.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from oracle import pyoracle as O
from simgrid_amd import lmm as L
from simgrid_amd import multi as M
from tests.lmm_cases import ABS_TOL, REL_TOL


def oracle_solve_flat(f, kind):
    """Rebuild a flattened system in the oracle and solve it (test stand-in for the device)."""
    o = O.System(False, kind)
    cs = []
    for b, fl in zip(f.cbound, f.cflags):
        c = o.constraint_new(None, float(b))
        if fl & 1:
            c.unshare()
        if fl & 2:  # an enabled zero-weight element the flat does not list (FATPIPE usage clamp)
            o.expand(c, o.variable_new(None, 1.0, -1.0, 1), 0.0)
        cs.append(c)
    vs = []
    for i in range(len(f.penalty)):
        lo, hi = int(f.var_ptr[i]), int(f.var_ptr[i + 1])
        v = o.variable_new(None, float(f.penalty[i]), float(f.vbound[i]), hi - lo)
        for j in range(lo, hi):
            o.expand(cs[int(f.cnst_idx[j])], v, float(f.weight[j]))
        vs.append(v)
    o.solve()
    return np.array([v.get_value() for v in vs])


def build_pair(kind):
    """The same multi-component system in the product (host side only) and in the oracle."""
    s, o = L.System(False, kind), O.System(False, kind)
    ovars = []
    if kind == 0:
        for run in range(6):  # six independent maxmin_bench "medium" systems
            s.gen_maxmin_bench(1, run)
            ovars += o.gen_maxmin_bench(1, run)[1]
    p = dict(topology=L.DRAGONFLY, topo_parameters="2,1;2,2;3,1;2", policy=L.SHARED, n_flows=60,
             model=L.LV08 if kind == 0 else L.L07)
    for seed in (1, 2):  # two disjoint platforms
        s.gen_platform_flows(L.platform_params(seed=seed, **p))
        _, ov = o.gen_platform_flows(O.platform_params(seed=seed, **p))
        ovars += [O.Variable(o, ov[i]) for i in range(60)]
    return s, o, ovars


def test_balanced_blocks():
    assert M.balanced_blocks([5, 1, 1, 1, 5, 1, 1, 1], 3) == [0, 3, 6, 8]
    assert M.balanced_blocks([1] * 10, 4) == [0, 3, 6, 9, 10]
    assert M.balanced_blocks([3], 2) == [0, 1, 1]
    rng = np.random.default_rng(1)
    for _ in range(20):
        w = rng.integers(1, 100, size=int(rng.integers(1, 40)))
        b = M.balanced_blocks(w, 3)
        assert b[0] == 0 and b[-1] == len(w) and all(x <= y for x, y in zip(b, b[1:]))
        worst = max(int(w[lo:hi].sum()) for lo, hi in zip(b, b[1:]))
        assert worst <= max(int(w.max()), -(-int(w.sum()) // 3) + int(w.max()))


def test_pack_components():
    owner = M.pack_components([10, 3, 3, 3, 1], 2)
    load = np.bincount(owner, weights=[10, 3, 3, 3, 1], minlength=2)
    assert sorted(load) == [10, 10]


@pytest.mark.parametrize("kind", [0, 1])
def test_components_and_single_rank_sharded_solve(kind):
    s, o, ovars = build_pair(kind)
    f = M.export_flat(s)
    var_lab, cnst_lab, n = M.components_host(f)
    assert n >= (8 if kind == 0 else 2)
    # every element joins a variable to a constraint of its own component
    rows = np.repeat(np.arange(len(f.penalty)), np.diff(f.var_ptr))
    assert np.all(var_lab[rows] == cnst_lab[f.cnst_idx])
    x = M.solve_components(f, kind, M.LocalExchange(), oracle_solve_flat, M.components_host)
    o.solve()
    want = np.array([ovars[int(i)].get_value() for i in f.var_ids])
    assert np.all(np.abs(x - want) <= np.maximum(ABS_TOL, REL_TOL * np.abs(want)))


def _free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def _worker(rank, world, port, kind, out_dir):
    import torch.distributed as dist

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        ex = M.DistExchange()
        s, _, _ = build_pair(kind)
        f = M.export_flat(s)
        x = M.solve_components(f, kind, ex, oracle_solve_flat, M.components_host)
        date = M.next_event_date([0.5, 0.25][rank] if rank < 2 else -1.0, ex)
        none = M.next_event_date(-1.0, ex)
        np.save(os.path.join(out_dir, f"x{rank}.npy"), x)
        np.save(os.path.join(out_dir, f"d{rank}.npy"), np.array([date, none]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind", [0, 1])
def test_gloo_world2_component_sharded_solve(kind, tmp_path):
    mp.spawn(_worker, args=(2, _free_port(), kind, str(tmp_path)), nprocs=2, join=True)
    s, o, ovars = build_pair(kind)
    f = M.export_flat(s)
    o.solve()
    want = np.array([ovars[int(i)].get_value() for i in f.var_ids])
    for r in range(2):
        x = np.load(tmp_path / f"x{r}.npy")
        assert np.all(np.abs(x - want) <= np.maximum(ABS_TOL, REL_TOL * np.abs(want)))
        assert list(np.load(tmp_path / f"d{r}.npy")) == [0.25, -1.0]


def test_batch_block_partition():
    weights = [O.System(False).gen_maxmin_bench(1, i) and 1 for i in range(5)]
    got = {}
    for rank in range(2):
        ex = M.LocalExchange()
        ex.rank, ex.world = rank, 2

        def build(i):
            o = O.System(False)
            o.gen_maxmin_bench(1, i)
            return o

        mine = M.solve_batch_block(build, 5, weights, ex, solve=lambda systems: [o.solve() for o in systems])
        got.update({i: rank for i in mine})
    assert sorted(got) == list(range(5)) and set(got.values()) == {0, 1}


# ---- variable-sharded FairBottleneck ----------------------------------------------------------

def fb_pair(seed=4):
    """A FairBottleneck system: L07 flows on the example dragonfly (FATPIPE loopbacks included)."""
    s, o = L.System(False, 1), O.System(False, 1)
    p = dict(topology=L.DRAGONFLY, topo_parameters="3,4;4,3;5,1;2", loopback_bw=1e8, limiter_bw=1.5e8,
             model=L.L07, n_flows=400, seed=seed)
    s.gen_platform_flows(L.platform_params(**p))
    _, ov = o.gen_platform_flows(O.platform_params(**p))
    return s, o, [O.Variable(o, ov[i]) for i in range(400)]


def sharded_fb_values(f, exchange, local_parts, make_shard, device=False, stream=None):
    """Values of the constraint-owner sharded FairBottleneck (multi.FbShardPlan over world x local_parts
    shards, this rank's `local_parts` of them made by make_shard(plan, p, gather)), dense order of `f`."""
    plan = M.FbShardPlan(f, exchange.world * local_parts)
    gather = M.FbGather(plan, device=device, stream=stream)
    parts = range(exchange.rank * local_parts, (exchange.rank + 1) * local_parts)
    shards = [make_shard(plan, p, gather) for p in parts]
    M.fb_solve_sharded(shards, exchange, gather)
    x = np.zeros(len(f.penalty))
    for sh in shards:
        x[sh.idx] = sh.values()
    return exchange.sum(x), shards


def numpy_shard(plan, p, gather):
    from tests.fb_shard_model import NumpyFbShard

    return NumpyFbShard(plan, p, gather, L.get_precision())


def oracle_dense_values(o, ovars, f):
    o.solve()
    return np.array([ovars[int(i)].get_value() for i in f.var_ids])


@pytest.mark.parametrize("local_parts", [1, 3])
def test_fb_sharded_single_process(local_parts):
    s, o, ovars = fb_pair()
    f = M.export_flat(s)
    x, _ = sharded_fb_values(f, M.LocalExchange(), local_parts, numpy_shard)
    want = oracle_dense_values(o, ovars, f)
    # the owners chain each constraint's increments in the reference's element order: the same bytes
    assert x.tobytes() == want.tobytes(), int(np.count_nonzero(x != want))


def test_fb_plan_layout():
    """Every element of the system is owned exactly once, in its constraint's reference order."""
    s, _, _ = fb_pair()
    f = M.export_flat(s)
    assert sorted(f.csc_order.tolist()) == list(range(len(f.cnst_idx)))
    assert np.all(np.diff(f.cnst_idx[f.csc_order]) >= 0)
    plan = M.FbShardPlan(f, 3)
    rows = np.repeat(np.arange(len(f.penalty)), np.diff(f.var_ptr))
    got = []
    for p in range(3):
        oc, optr, ovar, ow = plan.owned(p)
        for i, c in enumerate(oc):
            for pos, w in zip(ovar[optr[i]:optr[i + 1]], ow[optr[i]:optr[i + 1]]):
                got.append((int(c), int(pos), float(w)))
    want = [(int(f.cnst_idx[e]), int(plan.vpos[rows[e]]), float(f.weight[e])) for e in f.csc_order]
    assert got == want
    assert len(set(plan.vpos.tolist())) == len(f.penalty) and plan.vpos.max() < plan.mu_len
    assert len(set(plan.cpos.tolist())) == len(f.cbound) and plan.cpos.max() < plan.rem_len


def _fb_worker(rank, world, port, out_dir, seed):
    import torch.distributed as dist

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        s, _, _ = fb_pair(seed)
        f = M.export_flat(s)
        ex = M.DistExchange()
        x, shards = sharded_fb_values(f, ex, 2, numpy_shard)
        np.save(os.path.join(out_dir, f"fb{rank}.npy"), x)
        # bytes this rank put on the wire with the delta exchange of mu vs. the full all-gather every round
        M.FB_DELTA = False
        ex_full = M.DistExchange()
        x_full, _ = sharded_fb_values(f, ex_full, 2, numpy_shard)
        M.FB_DELTA = True
        assert x_full.tobytes() == x.tobytes()
        np.save(os.path.join(out_dir, f"wire{rank}.npy"), np.array([ex.wire_bytes, ex_full.wire_bytes,
                                                                    shards[0].rounds]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("seed", [4, 7])
def test_gloo_world2_fb_sharded(tmp_path, seed):
    """Two gloo ranks x two numpy shards each: counts all-reduced, mu and owned remaining all-gathered;
    the values are the oracle's, byte for byte."""
    mp.spawn(_fb_worker, args=(2, _free_port(), str(tmp_path), seed), nprocs=2, join=True)
    s, o, ovars = fb_pair(seed)
    f = M.export_flat(s)
    want = oracle_dense_values(o, ovars, f)
    for r in range(2):
        x = np.load(tmp_path / f"fb{r}.npy")
        assert x.tobytes() == want.tobytes(), (r, int(np.count_nonzero(x != want)))
        wire, full, rounds = np.load(tmp_path / f"wire{r}.npy")
        assert rounds >= 2 and 0 < wire < full, (wire, full, rounds)  # rounds > 0 ship listed mu only
