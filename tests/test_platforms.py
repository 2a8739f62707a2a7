"""Cluster platforms and flow generators (simgrid_amd/csrc/lmm_platforms.hpp), CPU only.

The reference's tesh files print no fat-tree / dragonfly route, so routing parity with the reference is
unpinned: routes are checked here against an independent Python restatement of the hop structure
FatTreeZone.cpp:62-129 / DragonflyZone.cpp:238-336 produce (route lengths per host pair, latencies,
LV08 penalties and TCP-gamma bounds), and the product's generator (simgrid_amd/csrc/lmm_platforms.hpp) is
checked to build exactly the system the oracle's own restatement of the zones and flow models builds
(oracle/platforms.py, replayed through the oracle's System API; it shares no code with the product).  The
GPU-vs-oracle solves on these systems (tests/test_gpu_platforms.py, test_gpu_configs.py C4 / C5) therefore
check the product's generator too.
"""
import math
from collections import defaultdict

import pytest

from oracle import pyoracle as O
from simgrid_amd import lmm as L
from tests.test_host_bookkeeping import same_structure

# examples/platforms/cluster_fat_tree.xml and cluster_dragonfly.xml (bw 125MBps, lat 50us, SPLITDUPLEX)
FAT_TREE = dict(topology=L.FAT_TREE, topo_parameters="2;4,4;1,2;1,2", loopback_bw=1e8)
DRAGONFLY = dict(topology=L.DRAGONFLY, topo_parameters="3,4;4,3;5,1;2", loopback_bw=1e8, limiter_bw=1.5e8)
BW, LAT, GAMMA = 1.25e8, 5e-5, 4194304.0


def test_platform_sizes():
    # 16 host loopbacks + 32 cables x SPLITDUPLEX
    assert L.platform_size(L.platform_params(**FAT_TREE)) == (80, 16)
    # 120 loopbacks + 120 limiters + 60 routers x 2 nodes x 2 + green 12 x 10 x 2 + black 3 x 6 x 5 x 2 + blue 3 x 2
    assert L.platform_size(L.platform_params(**DRAGONFLY)) == (906, 120)
    # SHARED cables are one link each
    assert L.platform_size(L.platform_params(topology=L.FAT_TREE, topo_parameters="2;4,4;1,2;1,2",
                                             policy=L.SHARED)) == (32, 16)


@pytest.mark.parametrize("kw", [
    dict(topology=L.FAT_TREE, topo_parameters="2;4;1,2;1,2"),          # wrong vector length
    dict(topology=L.FAT_TREE, topo_parameters="2;4,4;1,2"),            # 3 parts
    dict(topology=L.FAT_TREE, topo_parameters="x;4,4;1,2;1,2"),        # levels not a number
    dict(topology=L.DRAGONFLY, topo_parameters="3;4,3;5,1;2"),         # level with one element
    dict(topology=7, topo_parameters="2;4,4;1,2;1,2"),                 # unknown topology
    # a fat-tree node with both a loopback and a limiter (FatTreeZone.cpp:446-462, network_cm02.cpp:99)
    dict(topology=L.FAT_TREE, topo_parameters="2;4,4;1,2;1,2", loopback_bw=1e8, limiter_bw=1e8),
])
def test_bad_parameters_are_reported(kw):
    with pytest.raises(L.LmmError):
        L.platform_size(L.platform_params(**kw))


def elements_by_var(s, cs):
    """var rank -> [(constraint index, weight)] over the generated constraints."""
    out = defaultdict(list)
    for i, c in enumerate(cs):
        for rank, w, _, _ in L.Constraint(s, int(c)).elements():
            out[rank].append((i, w))
    return out


def l07_flows(kw, n, seed):
    s = L.System(False, L.System.FAIR_BOTTLENECK)
    p = L.platform_params(model=L.L07, n_flows=n, seed=seed, **kw)
    cs, vs = s.gen_platform_flows(p)
    n_links, n_hosts = L.platform_size(p)
    assert len(cs) == n_links + n_hosts
    per_var = elements_by_var(s, cs)
    for vid in vs:
        v = L.Variable(s, int(vid))
        els = per_var[v.rank]
        hosts = [i - n_links for i, w in els if i >= n_links]
        links = [(i, w) for i, w in els if i < n_links]
        assert all(w == 0.0 for i, w in els if i >= n_links)          # CPUs at weight 0
        assert len(hosts) == 2 and len({w for _, w in links}) == 1     # one size on every link
        yield v, hosts[0], hosts[1], len(links), links[0][1]


def fat_tree_links(src, dst):
    # hosts share a leaf switch iff label[1] = position // 4 matches: up + down, else up, up, down, down
    return 1 if src == dst else 2 if src // 4 == dst // 4 else 4


def test_fat_tree_l07_routes():
    n = 0
    for v, a, b, nl, size in l07_flows(FAT_TREE, 400, 3):
        if a == b:  # expand order cannot tell src from dst
            assert nl == 1 and v.get_bound() == -1.0      # loopback, latency 0: no TCP bound
            continue
        assert nl == fat_tree_links(a, b)
        assert math.isclose(v.get_bound(), GAMMA / (2 * nl * LAT * size), rel_tol=1e-12)
        assert v.get_penalty() == 1.0
        n += 1
    assert n > 300


def dragonfly_links(src, dst, C=4, B=5, N=2):
    """Unique links of the minimal route (DragonflyZone.cpp:238-336), limiters included."""
    if src == dst:
        return 1
    co = lambda r: (r // (C * B * N), r % (C * B * N) // (B * N), r % (B * N) // N)  # noqa: E731
    my, tg = co(src), co(dst)
    n, cur = 4, my  # node->router, src limiter, dst limiter, router->node
    if tg != my:
        if tg[0] != my[0]:
            if cur[2] != tg[0]:
                n, cur = n + 1, (my[0], my[1], tg[0])
            if cur[1] != 0:
                n, cur = n + 1, (my[0], 0, tg[0])
            n, cur = n + 1, (tg[0], 0, my[0])
        if tg[2] != cur[2]:
            n, cur = n + 1, (tg[0], 0, tg[2])   # the reference lands in chassis 0 here
        if tg[1] != cur[1]:
            n += 1
    return n


def test_dragonfly_l07_routes():
    seen = set()
    for v, a, b, nl, size in l07_flows(DRAGONFLY, 600, 5):
        # the route is not symmetric: accept either direction, but it must be one of them
        assert nl in (dragonfly_links(a, b), dragonfly_links(b, a)), (a, b, nl)
        if a != b:
            lat = (nl - 2) * LAT  # limiters carry no latency
            assert math.isclose(v.get_bound(), GAMMA / (2 * lat * size), rel_tol=1e-12)
        seen.add(nl)
    assert len(seen) >= 5  # local, intra-chassis, intra-group and inter-group routes all occur


@pytest.mark.parametrize("model", [L.LV08, L.CM02])
def test_fat_tree_network_flows(model):
    s = L.System(False)
    p = L.platform_params(model=model, n_flows=300, seed=2, **FAT_TREE)
    cs, vs = s.gen_platform_flows(p)
    factor, weight_s = (0.97, 20537.0) if model == L.LV08 else (1.0, 0.0)
    counts = set()
    for vid in vs:
        v = L.Variable(s, int(vid))
        n = v.get_number_of_constraint()
        counts.add(n)
        assert n in (2, 4, 8)  # route + back route: loopback / same leaf / through a level-2 switch
        hops = n // 2
        if n == 2:
            assert v.get_penalty() == 1.0 and v.get_bound() == -1.0
        else:
            lat = hops * LAT
            assert math.isclose(v.get_penalty(), lat + hops * weight_s / BW, rel_tol=1e-12)
            assert math.isclose(v.get_bound(), GAMMA / (2 * lat), rel_tol=1e-12)
    assert counts == {2, 4, 8}
    bounds = sorted({L.Constraint(s, int(c)).get_bound() for c in cs})
    assert bounds == [factor * 1e8, factor * BW]
    shared = [L.Constraint(s, int(c)).is_shared() for c in cs]
    assert shared.count(False) == 16  # the loopbacks are FATPIPE


def test_crosstraffic_off():
    s = L.System(False)
    cs, vs = s.gen_platform_flows(L.platform_params(model=L.LV08, n_flows=100, seed=2, crosstraffic=False,
                                                    **FAT_TREE))
    assert {L.Variable(s, int(v)).get_number_of_constraint() for v in vs} <= {1, 2, 4}


@pytest.mark.parametrize("plat,model,kind", [
    (FAT_TREE, L.LV08, 0), (FAT_TREE, L.CM02, 0), (FAT_TREE, L.L07, 1),
    (DRAGONFLY, L.LV08, 0), (DRAGONFLY, L.L07, 1), (DRAGONFLY, L.CM02, 0),
    (dict(topology=L.DRAGONFLY, topo_parameters="2,1;2,2;3,1;2", policy=L.SHARED), L.LV08, 0),
    (dict(topology=L.DRAGONFLY, topo_parameters="3,4;4,3;5,1;2", policy=L.FATPIPE), L.L07, 1),
    # three levels, switch limiters on the routes, no back route
    (dict(topology=L.FAT_TREE, topo_parameters="3;4,4,4;1,4,2;1,1,2", limiter_bw=1e8), L.LV08, 0),
    (dict(topology=L.FAT_TREE, topo_parameters="3;4,4,4;1,4,2;1,1,2", limiter_bw=1e8, crosstraffic=False),
     L.CM02, 0),
    # the C4 / C5 platforms of bench.py (fewer flows)
    (dict(topology=L.FAT_TREE, topo_parameters="3;16,16,16;1,16,16;1,1,1", loopback_bw=1e9), L.LV08, 0),
    (dict(topology=L.DRAGONFLY, topo_parameters="8,4;16,3;8,2;4", loopback_bw=1e9, limiter_bw=2e8), L.L07, 1),
])
def test_product_and_oracle_build_the_same_system(plat, model, kind):
    ps, os_ = L.System(False, kind), O.System(False, kind)
    pc, pv = ps.gen_platform_flows(L.platform_params(model=model, n_flows=200, seed=3, **plat))
    oc, ov = os_.gen_platform_flows(O.platform_params(model=model, n_flows=200, seed=3, **plat))
    assert len(pc) == len(oc) and len(pv) == len(ov)
    same_structure(ps, os_, {i: L.Constraint(ps, int(c)) for i, c in enumerate(pc)}, dict(enumerate(oc)),
                   {i: L.Variable(ps, int(v)) for i, v in enumerate(pv)},
                   {i: O.Variable(os_, ov[i]) for i in range(len(pv))})
    for i in range(len(pv)):
        assert L.Variable(ps, int(pv[i])).get_bound() == O.Variable(os_, ov[i]).get_bound()
        assert L.Variable(ps, int(pv[i])).get_penalty() == O.Variable(os_, ov[i]).get_penalty()


@pytest.mark.parametrize("kw", [
    dict(topology=L.FAT_TREE, topo_parameters="2;4;1,2;1,2"),
    dict(topology=L.DRAGONFLY, topo_parameters="3;4,3;5,1;2"),
    dict(topology=7, topo_parameters="2;4,4;1,2;1,2"),
    dict(topology=L.FAT_TREE, topo_parameters="2;4,4;1,2;1,2", loopback_bw=1e8, limiter_bw=1e8),
])
def test_oracle_restatement_rejects_bad_parameters(kw):
    with pytest.raises(ValueError):
        O.System(False).gen_platform_flows(O.platform_params(**kw))


def test_dragonfly_coords_pinned_to_reference_tesh():
    """DragonflyZone::rankId_to_coords (DragonflyZone.cpp:26-35) and the host count of cluster_dragonfly.xml
    ("3,4;4,3;5,1;2", hosts node-0 .. node-119), against the 120 host lines and 120 `rank: (group, chassis, blade,
    node)` lines s4u-routing-get-clusters.tesh prints for it (tests/golden/dragonfly_coords.json): the product's
    coordinates through the C ABI (lmm_platform_dragonfly_coords) and the oracle's restatement (oracle/platforms.py)."""
    import json
    import os

    import numpy as np

    from oracle import platforms as PL

    fx = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "dragonfly_coords.json")))
    assert fx["topo_parameters"] == DRAGONFLY["topo_parameters"] and len(fx["coords"]) == 120
    want = np.array(fx["coords"], dtype=np.int64)
    assert want[:, 0].tolist() == list(range(120))  # one line per rank, in rank order
    lo, hi = (int(x) for x in fx["radical"].split("-"))
    assert fx["hosts"] == [f"node-{i}.simgrid.org" for i in range(lo, hi + 1)]
    p = L.platform_params(**DRAGONFLY)
    assert L.platform_size(p)[1] == len(fx["hosts"]) == 120
    got = L.dragonfly_coords(p)
    assert got.tolist() == want[:, 1:].tolist()
    op = O.params_dict(O.platform_params(**DRAGONFLY))
    plat = PL.make_platform(op)
    assert plat.n_hosts == 120 and PL.platform_size(op)[1] == 120
    oc = np.stack(plat.coords(np.arange(120)), axis=1)
    assert oc.tolist() == want[:, 1:].tolist()
    # and the other topologies are refused
    with pytest.raises(L.LmmError, match="not a dragonfly"):
        L.dragonfly_coords(L.platform_params(**FAT_TREE))
