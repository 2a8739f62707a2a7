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
