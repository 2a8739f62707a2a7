"""WIFI access points in the flow builder (NetworkCm02Model::communicate's WIFI rates,
network_cm02.cpp:239-260; NetworkWifiLink, network_cm02.cpp:383-420).  No tesh of the reference exercises WIFI, so
this row's parity is against the oracle's restatement (oracle/platforms.py) and the closed form of the one case
the model is known for — stations sharing an access point all get the same rate, set by the slowest (Σ x / r_i
<= 1 with equal penalties).  CPU only: host bookkeeping and the oracle solve; the device solve of the same
systems is tests/test_gpu_platforms.py::test_wifi_flows_device_match_oracle."""
import pytest

from oracle import platforms as PL
from oracle import pyoracle as O

CM02, LV08 = 0, 1
GAMMA = 4194304.0


def _product():
    from simgrid_amd import lmm as L

    return L


def build_wifi(sys, backend, model, paid=True):
    """Two access points (stations at 54, 54 and 6 Mb/s on AP 1; 11 and 54 Mb/s on AP 2) joined by a wired
    backbone; flows station -> station across the APs (AP 1 weighs the source's rate: the destination is not
    associated with it; AP 2 the destination's), one flow station -> a wired host and one wired host -> station.
    backend: 'product' (lmm_wifi_link_new / lmm_communicate_ex) or 'oracle'.  Returns (flow variables, the
    constraints)."""
    if backend == "product":
        ap1, ap2 = sys.wifi_link_new(model), sys.wifi_link_new(model)
        bb, wired = sys.link_new(model, 1.25e8), sys.link_new(model, 1e7)
        comm = lambda route, **kw: sys.communicate(model, route, tcp_gamma=GAMMA, paid=paid, **kw)[0]
    else:
        ap1, ap2 = PL.wifi_link_new(sys, model), PL.wifi_link_new(sys, model)
        bb, wired = PL.link_new(sys, model, 1.25e8), PL.link_new(sys, model, 1e7)
        comm = lambda route, **kw: PL.communicate(sys, model, route, tcp_gamma=GAMMA, paid=paid, **kw)[0]
    r1, r2 = [54e6, 54e6, 6e6], [11e6, 54e6]
    bbl, wl = (bb, 1.25e8, 5e-5), (wired, 1e7, 1e-4)
    flows = []
    for i, a in enumerate(r1):  # AP 1 station i -> AP 2 station i % 2
        flows.append(comm([(ap1, 0.0, 0.0, (a, -1.0)), bbl, (ap2, 0.0, 0.0, (-1.0, r2[i % 2]))]))
    flows.append(comm([(ap1, 0.0, 0.0, (r1[2], -1.0)), bbl, wl]))  # AP 1 slow station -> wired host
    flows.append(comm([wl, bbl, (ap2, 0.0, 0.0, (-1.0, r2[1]))]))  # wired host -> AP 2 fast station
    flows.append(comm([(ap1, 0.0, 0.0, (r1[0], r1[1]))]))          # two stations of AP 1: the source's rate
    return flows, [ap1, ap2, bb, wired]


@pytest.mark.parametrize("model", [CM02, LV08])
@pytest.mark.parametrize("paid", [False, True])
def test_wifi_communicate_product_equals_oracle(model, paid):
    """lmm_communicate_ex and the oracle's communicate build the same system: weights 1 / rate on the access
    points (source rate, else destination rate), the AP's bound bf * (1 / bf), its bandwidth 1 / bf in the
    weight_S penalty and latency 0 in the route latency."""
    L = _product()
    ps, os_ = L.System(False), O.System(False)
    (pv, pc), (ov, oc) = build_wifi(ps, "product", model, paid), build_wifi(os_, "oracle", model, paid)
    assert [v.get_penalty() for v in pv] == [v.get_penalty() for v in ov]
    assert [v.get_bound() for v in pv] == [v.get_bound() for v in ov]
    assert [c.get_bound() for c in pc] == [c.get_bound() for c in oc]
    pe = [sorted((e[1], e[3]) for e in c.elements()) for c in pc]
    oe = [sorted((e[1], e[3]) for e in c.elements()) for c in oc]
    assert pe == oe
    assert sorted(w for w, _ in pe[0]) == sorted([1 / 54e6, 1 / 54e6, 1 / 6e6, 1 / 6e6, 1 / 54e6])


def test_wifi_weights_and_errors():
    """The element weights of network_cm02.cpp:249-262, the AP's bound, and the two assertions as errors:
    a back route (crosstraffic) with a WIFI link, and neither station associated."""
    L = _product()
    for backend in ("product", "oracle"):
        sys = L.System(False) if backend == "product" else O.System(False)
        ap = sys.wifi_link_new(LV08) if backend == "product" else PL.wifi_link_new(sys, LV08)
        wl = sys.link_new(LV08, 1e7) if backend == "product" else PL.link_new(sys, LV08, 1e7)
        assert ap.get_bound() == 0.97 * (1.0 / 0.97)
        comm = (lambda r, **kw: sys.communicate(LV08, r, **kw)) if backend == "product" else \
            (lambda r, **kw: PL.communicate(sys, LV08, r, **kw))
        _, info = comm([(ap, 123.0, 9.0, (6e6, 54e6)), (wl, 1e7, 1e-4)], paid=True)
        # the AP's latency is 0 and its bandwidth 1 / 0.97 whatever the caller passed
        assert info["lat_current"] == 1e-4
        assert info["sharing_penalty"] == 1e-4 + 20537.0 / (1.0 / 0.97) + 20537.0 / 1e7
        ws = sorted(e[1] for e in ap.elements())
        assert ws == [1.0 / 6e6]
        comm([(ap, 0.0, 0.0, (-1.0, 11e6))])
        assert sorted(e[1] for e in ap.elements()) == sorted([1.0 / 6e6, 1.0 / 11e6])
        err = L.LmmError if backend == "product" else ValueError
        with pytest.raises(err, match="Cross-traffic"):
            comm([(ap, 0.0, 0.0, (6e6, -1.0))], back=[wl])
        # the assertion tests the configuration, not the back route (network_cm02.cpp:242): crosstraffic on with an
        # empty back route fails too, and a back route is no error once the caller says crosstraffic is off
        with pytest.raises(err, match="Cross-traffic"):
            comm([(ap, 0.0, 0.0, (6e6, -1.0))], back=[], crosstraffic=True)
        comm([(ap, 0.0, 0.0, (6e6, -1.0))], back=[], crosstraffic=False)
        with pytest.raises(err, match="not associated"):
            comm([(ap, 0.0, 0.0, (-1.0, -1.0))])
        if backend == "product":  # (a rate of 0 would weigh 1 / 0: refused)
            with pytest.raises(err, match="WIFI rate"):
                comm([(ap, 0.0, 0.0, (0.0, 6e6))])


def test_wifi_oracle_closed_form():
    """Stations sharing one access point with nothing else limiting get one rate, 1 / Σ 1/r_i (the slowest
    station drags the others down): the oracle's solve of three flows at 54, 54 and 6 Mb/s."""
    s = O.System(False)
    ap = PL.wifi_link_new(s, CM02)
    vs = [PL.communicate(s, CM02, [(ap, 0.0, 0.0, (r, -1.0))], paid=True)[0] for r in (54e6, 54e6, 6e6)]
    s.solve()
    want = 1.0 / (2 / 54e6 + 1 / 6e6)
    for v in vs:
        assert v.get_value() == pytest.approx(want, rel=1e-12)
