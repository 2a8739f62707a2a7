"""examples/s4u/app-pingpong replayed on the oracle (CPU): the LV08 / CM02 flow model and both model-side step
paths (LAZY: Model::next_occuring_event_lazy + ActionHeap; FULL: next_occuring_event_full +
update_actions_state_full) against the reference's tesh (tests/pingpong_scenario.py, fixture
tests/golden/pingpong.json).  The device replay is tests/test_gpu_step.py::test_pingpong_device_*.

Also: the product's one-communication builder (lmm_communicate, lmm_platforms.hpp `communicate` — the code
that builds C4's flows) and the oracle's restatement (oracle/platforms.py `communicate`) build the same LMM
system; that needs no GPU (host bookkeeping + flat export)."""
import pytest

from tests import pingpong_scenario as PP


@pytest.mark.parametrize("run", sorted(PP.RUNS))
def test_pingpong_oracle_matches_reference_tesh(run):
    """Every logged line (clock to 6 decimals, actor, message) of s4u-app-pingpong.tesh's run `run`: LV08 Lazy
    and Full 0.019014 / 150.178356, CM02 0.001462 / 145.639041."""
    out, _ = PP.run_pingpong(PP.PingOracle(), run)
    assert out == PP.expected(run)


def test_pingpong_dates_closed_form():
    """The dates the replay produces are the closed form of the flow model: the latency (13.01 x 1.461517 ms
    for LV08) then size / (0.97 x 7.20975e6 / 1.05) per message."""
    for run, (lf, bf) in {"lv08_lazy": (13.01, 0.97), "lv08_full": (13.01, 0.97), "cm02_lazy": (1.0, 1.0)}.items():
        _, e = PP.run_pingpong(PP.PingOracle(), run)
        lat, bw = 1.461517e-3 * lf, 7.20975e6 * bf / 1.05
        t1 = lat + 1.0 / bw
        assert e.now == pytest.approx(t1 + lat + 1e9 / bw, rel=1e-12), run


@pytest.mark.parametrize("model", [PP.CM02, PP.LV08])
def test_communicate_product_equals_oracle_restatement(model):
    """lmm_communicate (product, lmm_platforms.hpp) and oracle/platforms.py's communicate build the same
    variable (penalty unpaid 0 / paid sharing penalty, TCP-gamma and rate bounds, 1.0 + 0.05 elements) on the
    same links; the returned action parameters are equal bit for bit."""
    from oracle import platforms as PL
    from oracle import pyoracle as O
    from simgrid_amd import lmm as L

    links = [(7.20975e6, 1.461517e-3), (1.25e8, 5e-5), (41.279125e6, 59.904e-6)]
    for rate in (-1.0, 1e5, 1e12):
        for paid in (False, True):
            ps, os_ = L.System(False), O.System(False)
            pc = [ps.link_new(model, bw) for bw, _ in links]
            oc = [PL.link_new(os_, model, bw) for bw, _ in links]
            pv, pi = ps.communicate(model, [(c, bw, lat) for c, (bw, lat) in zip(pc, links)], pc[::-1], rate,
                                    4194304.0, paid)
            ov, oi = PL.communicate(os_, model, [(c, bw, lat) for c, (bw, lat) in zip(oc, links)], oc[::-1], rate,
                                    4194304.0, paid)
            assert pi == oi, (model, rate, paid)
            assert pv.get_penalty() == ov.get_penalty() and pv.get_bound() == ov.get_bound()
            assert [c.get_bound() for c in pc] == [c.get_bound() for c in oc]
            pe = sorted((e[1], e[3], cid) for cid, c in enumerate(pc) for e in c.elements())
            oe = sorted((e[1], e[3], cid) for cid, c in enumerate(oc) for e in c.elements())
            assert pe == oe, (model, rate, paid)
