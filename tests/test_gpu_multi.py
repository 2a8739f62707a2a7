"""Component-sharded solve on the device (simgrid_amd/multi.py): every component of a multi-component
system solved through the lmmhip_* ABI on its own context, compared with the oracle's solve of the
whole system.  One process (LocalExchange); the cross-rank path is covered on gloo in test_multi.py."""
import numpy as np
import pytest

from simgrid_amd import multi as M
from tests.lmm_cases import ABS_TOL, REL_TOL
from tests.test_multi import build_pair

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kind", [0, 1])
def test_device_component_sharded_solve(kind):
    s, o, ovars = build_pair(kind)
    f = M.export_flat(s)
    for world in (1, 3):  # pretend to be every rank of a 3-rank job in turn
        x = np.zeros(len(f.penalty))
        for rank in range(world):
            ex = M.LocalExchange()
            ex.rank, ex.world = rank, world
            x += M.solve_components(f, kind, ex)
        o.solve()
        want = np.array([ovars[int(i)].get_value() for i in f.var_ids])
        assert np.all(np.abs(x - want) <= np.maximum(ABS_TOL, REL_TOL * np.abs(want))), world


def device_shard_maker(shards, stream=None):
    def make(plan, p, gather):
        sh = M.DeviceFbShard(plan, p, gather, stream=stream)
        shards.append(sh)
        return sh

    return make


@pytest.mark.parametrize("local_parts", [1, 2, 3])
def test_device_fb_sharded(local_parts):
    """Constraint-owner sharded FairBottleneck (lmmhip_fb_shard_*): `local_parts` device shards in this
    process, counts summed and mu / remaining gathered between the phases; the oracle's values, byte for
    byte."""
    from tests.test_multi import fb_pair, oracle_dense_values, sharded_fb_values

    s, o, ovars = fb_pair()
    f = M.export_flat(s)
    shards = []
    x, _ = sharded_fb_values(f, M.LocalExchange(), local_parts, device_shard_maker(shards), device=True)
    for sh in shards:
        sh.close()
    want = oracle_dense_values(o, ovars, f)
    assert x.tobytes() == want.tobytes(), int(np.count_nonzero(x != want))


def canonical(var_lab, cnst_lab):
    """Labels renamed by first occurrence over [variables, constraints] (the device's own numbering:
    components in the order of their smallest node)."""
    lab = np.concatenate([var_lab, cnst_lab]).astype(np.int64)
    _, first, inv = np.unique(lab, return_index=True, return_inverse=True)
    rank = np.empty(len(first), np.int64)
    rank[np.argsort(first, kind="stable")] = np.arange(len(first))
    return rank[inv]


def component_systems():
    from simgrid_amd import lmm as L

    out = [("medium+dragonfly maxmin", build_pair(0)[0]), ("dragonfly L07", build_pair(1)[0])]
    s = L.System(False)  # C4-style: LV08 flows on the fat tree (one giant component + idle links)
    s.gen_platform_flows(L.platform_params(model=L.LV08, n_flows=20_000, seed=3, topology=0,
                                           topo_parameters="3;16,16,16;1,16,16;1,1,1", loopback_bw=1e8))
    out.append(("fat tree LV08", s))
    s = L.System(False)  # sparse random: many small components (k = 1 and 2 elements per variable)
    s.gen_synthetic(50_000, 30_000, 1, seed=4)
    s.gen_synthetic(50_000, 20_000, 2, seed=5)
    out.append(("sparse synthetic", s))
    return out


def test_device_components_match_scipy():
    """lmmhip_components (device union-find) against scipy's connected_components on the same flattened
    systems: identical labels up to renaming (the device numbering is scipy's renamed by first occurrence)."""
    for name, s in component_systems():
        f = M.export_flat(s)
        dv, dc, dn = M.device_components(f)
        hv, hc, hn = M.components_host(f)
        assert dn == hn, (name, dn, hn)
        assert np.array_equal(np.concatenate([dv, dc]), canonical(hv, hc)), name
        sv, sc, sn = s.components()  # the System's own device flatten, no export
        assert sn == dn and np.array_equal(sv, dv) and np.array_equal(sc, dc), name


def _gloo_worker(rank, world, port, kind, out_dir):
    import os

    import torch
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        s, _, _ = build_pair(kind)
        f = M.export_flat(s)
        x = M.solve_components(f, kind, M.DistExchange())  # device labels, device sub-solves
        np.save(os.path.join(out_dir, f"x{rank}.npy"), x)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind", [0, 1])
def test_gloo_world2_device_components(kind, tmp_path):
    """The component-sharded solve of test_multi.py's gloo world-2 run with the product path on both ranks:
    components labelled on the device, each rank's share solved on the device."""
    import torch.multiprocessing as mp

    from tests.test_multi import _free_port

    mp.spawn(_gloo_worker, args=(2, _free_port(), kind, str(tmp_path)), nprocs=2, join=True)
    s, o, ovars = build_pair(kind)
    f = M.export_flat(s)
    o.solve()
    want = np.array([ovars[int(i)].get_value() for i in f.var_ids])
    for r in range(2):
        x = np.load(tmp_path / f"x{r}.npy")
        assert np.all(np.abs(x - want) <= np.maximum(ABS_TOL, REL_TOL * np.abs(want))), r


def test_rccl_world1_exchange_paths():
    """RCCL itself (torch.distributed's "nccl" backend = RCCL on ROCm), in a world-size-1 group on this GPU:
    DistExchange's device branch — all_reduce and all_gather_into_tensor of device tensors on the shard
    stream, ordered with the solver's kernels through lmmhip_ctx_set_stream — drives the constraint-owner
    sharded FairBottleneck (2 local shards) to the oracle's bytes, and the component-sharded max-min solve and
    the next-event all-reduce(MIN) to the LocalExchange results."""
    import torch
    import torch.distributed as dist

    from tests.test_multi import _free_port, fb_pair, oracle_dense_values, sharded_fb_values

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)
    try:
        ex = M.DistExchange()
        assert ex.device.type == "cuda"
        s, o, ovars = fb_pair(seed=6)
        f = M.export_flat(s)
        shards = []
        x, _ = sharded_fb_values(f, ex, 2, device_shard_maker(shards), device=True)
        for sh in shards:
            sh.close()
        want = oracle_dense_values(o, ovars, f)
        assert x.tobytes() == want.tobytes(), int(np.count_nonzero(x != want))
        s2, _, _ = build_pair(0)
        f2 = M.export_flat(s2)
        xr = M.solve_components(f2, 0, ex)
        xl = M.solve_components(f2, 0, M.LocalExchange())
        assert xr.tobytes() == xl.tobytes()
        assert M.next_event_date(0.25, ex) == 0.25 and M.next_event_date(-1.0, ex) == -1.0
    finally:
        dist.destroy_process_group()
