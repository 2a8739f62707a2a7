"""GPU parity on cluster-platform systems (SURVEY.md §8 f3 and configs C4 / C5 at test scale): flows on
fat trees and dragonflies (lmm_platforms.hpp) solved by the HIP path, compared with the oracle's solve
of the same system.  Tolerance as everywhere (tests/lmm_cases.py): |x - x_ref| <= max(1e-9, 1e-6 |x_ref|).
"""
import numpy as np
import pytest

from oracle import pyoracle as O
from simgrid_amd import lmm as L
from tests.lmm_cases import ABS_TOL, REL_TOL

pytestmark = pytest.mark.gpu

EX_FAT_TREE = dict(topology=L.FAT_TREE, topo_parameters="2;4,4;1,2;1,2", loopback_bw=1e8)
EX_DRAGONFLY = dict(topology=L.DRAGONFLY, topo_parameters="3,4;4,3;5,1;2", loopback_bw=1e8, limiter_bw=1.5e8)
BIG_FAT_TREE = dict(topology=L.FAT_TREE, topo_parameters="3;8,8,8;1,8,4;1,1,2", loopback_bw=1e9)
BIG_DRAGONFLY = dict(topology=L.DRAGONFLY, topo_parameters="4,2;4,2;8,1;4", loopback_bw=1e9, limiter_bw=2e8)

CASES = [
    ("fat_tree_lv08", EX_FAT_TREE, L.LV08, 0, 2000),
    ("fat_tree_cm02_shared", dict(EX_FAT_TREE, policy=L.SHARED), L.CM02, 0, 2000),
    ("fat_tree_l07", EX_FAT_TREE, L.L07, 1, 2000),
    ("dragonfly_lv08", EX_DRAGONFLY, L.LV08, 0, 3000),
    ("dragonfly_l07", EX_DRAGONFLY, L.L07, 1, 3000),
    ("big_fat_tree_lv08", BIG_FAT_TREE, L.LV08, 0, 20000),
    ("big_dragonfly_l07", BIG_DRAGONFLY, L.L07, 1, 20000),
    ("big_dragonfly_lv08_no_crosstraffic", dict(BIG_DRAGONFLY, crosstraffic=False), L.LV08, 0, 20000),
]


@pytest.mark.parametrize("name,plat,model,kind,n", CASES, ids=[c[0] for c in CASES])
def test_platform_flows_match_oracle(name, plat, model, kind, n):
    s, o = L.System(False, kind), O.System(False, kind)
    _, vs = s.gen_platform_flows(L.platform_params(model=model, n_flows=n, seed=11, **plat))
    _, ov = o.gen_platform_flows(O.platform_params(model=model, n_flows=n, seed=11, **plat))
    s.solve()
    o.solve()
    got, want = s.values_of(vs), o.values_of(ov, n)
    tol = np.maximum(ABS_TOL, REL_TOL * np.abs(want))
    bad = np.nonzero(np.abs(got - want) > tol)[0]
    assert len(bad) == 0, (name, len(bad), [(int(i), got[i], want[i]) for i in bad[:5]])
    assert np.all(want > 0)  # every flow gets a share
    if kind == 0:
        excess, infeasible, unbottlenecked = s.check_certificate()
        assert infeasible == 0 and unbottlenecked == 0, (excess, infeasible, unbottlenecked)


@pytest.mark.parametrize("model", [0, 1], ids=["cm02", "lv08"])
def test_wifi_flows_device_match_oracle(model):
    """WIFI access points (lmm_wifi_link_new / lmm_communicate_ex, network_cm02.cpp:239-260, 383-420): the HIP
    solve of tests/test_wifi.py's two-AP system equals the oracle's, and stations alone on an AP get the closed
    form 1 / Σ 1/r_i (the slowest station sets everyone's rate)."""
    from tests.test_wifi import build_wifi

    s, o = L.System(False), O.System(False)
    (pv, _), (ov, _) = build_wifi(s, "product", model), build_wifi(o, "oracle", model)
    s.solve()
    o.solve()
    got, want = np.array([v.get_value() for v in pv]), np.array([v.get_value() for v in ov])
    tol = np.maximum(ABS_TOL, REL_TOL * np.abs(want))
    assert np.all(np.abs(got - want) <= tol), (got, want)
    assert np.all(want > 0)
    s1 = L.System(False)
    ap = s1.wifi_link_new(model)
    vs = [s1.communicate(model, [(ap, 0.0, 0.0, (r, -1.0))], paid=True)[0] for r in (54e6, 54e6, 6e6)]
    s1.solve()
    bf = 0.97 if model == 1 else 1.0
    for v in vs:
        assert v.get_value() == pytest.approx(bf * (1.0 / bf) / (2 / 54e6 + 1 / 6e6), rel=1e-9)


def test_reference_dragonfly_coords_and_flows_on_device():
    """The reference's cluster_dragonfly.xml ("3,4;4,3;5,1;2", 120 hosts), pinned by s4u-routing-get-clusters.tesh
    (tests/golden/dragonfly_coords.json): the library loaded on the GPU box reproduces every `rank: (group, chassis,
    blade, node)` line (DragonflyZone.cpp:26-35) and the host count, and LV08 flows between hosts of different groups
    (the blue links the coordinates route over) and of one blade solve on the device to the oracle's values and
    saturated set."""
    import json
    import os

    fx = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "dragonfly_coords.json")))
    want = np.array(fx["coords"], dtype=np.int64)[:, 1:]
    p = dict(model=L.LV08, n_flows=4000, seed=5, **EX_DRAGONFLY)
    assert L.dragonfly_coords(L.platform_params(**p)).tolist() == want.tolist()
    assert L.platform_size(L.platform_params(**p))[1] == len(fx["hosts"]) == 120
    s, o = L.System(False), O.System(False)
    pc, vs = s.gen_platform_flows(L.platform_params(**p))
    oc, ov = o.gen_platform_flows(O.platform_params(**p))
    s.solve()
    o.solve()
    got, ref = s.values_of(vs), o.values_of(ov, len(vs))
    tol = np.maximum(ABS_TOL, REL_TOL * np.abs(ref))
    assert np.all(np.abs(got - ref) <= tol), float(np.max(np.abs(got - ref)))
    from tests.lmm_cases import saturated

    prec = L.get_precision()
    sat_p = saturated(s, {k: L.Constraint(s, int(c)) for k, c in enumerate(pc)}, prec)
    assert sat_p == saturated(o, dict(enumerate(oc)), prec) and len(sat_p) > 0
