"""Step glue on the device (simgrid_amd/step.py, lmm_step_kernels.hpp) against oracle/step_oracle.py,
bit for bit: every action is independent element-wise IEEE arithmetic in the same order."""
import numpy as np
import pytest

from oracle import step_oracle as S
from simgrid_amd import lmm as L
from simgrid_amd import multi as M
from simgrid_amd import step as D

pytestmark = pytest.mark.gpu


def random_actions(rng, n, n_dense):
    vi = rng.integers(-1, n_dense, size=n).astype(np.int32)
    st = dict(remains=rng.choice([0.0, 1e-9, 1.0, 5.0, 1e3], size=n) * rng.random(n),
              max_duration=np.where(rng.random(n) < 0.3, rng.random(n) * 2, -1.0),
              latency=np.where(rng.random(n) < 0.3, rng.random(n) * 1e-3, 0.0),
              penalty=np.where(rng.random(n) < 0.2, 0.0, 1.0),
              sharing_penalty=rng.random(n) + 0.5,
              flags=rng.choice([0, 0, 0, S.ACT_NO_CNST, S.ACT_SUSPENDED], size=n).astype(np.uint8))
    return vi, st


@pytest.mark.parametrize("model", [D.MODEL_CPU, D.MODEL_CM02, D.MODEL_L07])
def test_step_glue_matches_oracle(model):
    rng = np.random.default_rng(model + 1)
    s = L.System(False)
    s.gen_maxmin_bench(2, 0)
    f = M.export_flat(s)
    s.solve()
    x = np.array(s.values_of(f.var_ids))
    vi, st = random_actions(rng, 5000, len(x))
    acts = D.DeviceActions(s.device_ctx(), vi, **st)
    ost = {k: list(v) for k, v in st.items()}
    values = [x[i] if i >= 0 else 0.0 for i in vi]
    lat_term = model != D.MODEL_CPU
    for step in range(6):
        got = acts.next_occuring_event(with_latency=lat_term)
        want = S.next_occuring_event_full(values, ost["remains"], ost["max_duration"],
                                          ost["latency"] if lat_term else None)
        assert got == want, (step, got, want)
        delta = want if want > 0 else 0.01
        nev = acts.update_actions_state(model, delta, 1e-5, 1e-5)
        ev = S.update_actions_state_full(model, values, ost, delta, 1e-5, 1e-5)
        dev = acts.state()
        assert nev == sum(e != 0 for e in ev)
        assert list(dev["events"]) == ev
        for k in ("remains", "max_duration", "latency", "penalty"):
            assert np.array_equal(dev[k], np.array(ost[k])), (step, k)


@pytest.mark.parametrize("model", [D.MODEL_CPU, D.MODEL_CM02])
def test_lazy_glue_matches_heap_oracle(model):
    """LAZY models: device (date, type) arrays + min-reduction vs the oracle's real heap, bit for bit,
    over steps of modified sets, completion dates, pops and latency hats."""
    rng = np.random.default_rng(11 + model)
    s = L.System(False)
    s.gen_maxmin_bench(2, 1)
    f = M.export_flat(s)
    s.solve()
    x = np.array(s.values_of(f.var_ids))
    n = 6000
    vi, st = random_actions(rng, n, len(x))
    st["flags"] = np.where(rng.random(n) < 0.05, S.ACT_NOT_STARTED, 0).astype(np.uint8)
    lat_hat = (rng.random(n) < 0.2) if model == D.MODEL_CM02 else np.zeros(n, bool)
    lz = dict(last_update=np.zeros(n), last_value=np.where(rng.random(n) < 0.5, rng.random(n), 0.0),
              start_time=np.zeros(n), date=np.where(lat_hat, rng.random(n) * 1e-3, 0.0),
              heap_type=np.where(lat_hat, S.HEAP_LATENCY, S.HEAP_UNSET).astype(np.uint8))
    acts = D.DeviceActions(s.device_ctx(), vi, **st)
    acts.lazy_init(**lz)
    ost = {k: list(v) for k, v in st.items() if k in ("remains", "max_duration", "penalty", "flags")}
    ost.update({k: list(v) for k, v in lz.items()})
    ost["date"] = [d if h else float("inf") for d, h in zip(ost["date"], ost["heap_type"])]
    O = S.LazyModel(model, ost)
    values = [x[i] if i >= 0 else 0.0 for i in vi]
    # a modified action the loop does not skip must get a date (else DIE_IMPOSSIBLE, Model.cpp:96):
    # share > 0 or a max duration
    dated = np.array([values[i] > 0 or st["max_duration"][i] != S.NO_MAX_DURATION or st["penalty"][i] <= 0
                      or st["flags"][i] & S.ACT_NOT_STARTED or lat_hat[i] for i in range(n)])
    now, pops = 0.0, 0
    for step in range(10):
        modified = rng.permutation(np.nonzero(dated)[0])[: n // 3]
        nfin = acts.lazy_update(model, now, modified, 1e-5, 1e-5)
        want_ev, want_fin = O.next_occuring_event_lazy(values, now, [int(i) for i in modified], 1e-5, 1e-5)
        got_ev = acts.next_occuring_event_lazy(now)
        assert nfin == len(want_fin) and got_ev == want_ev, (step, got_ev, want_ev)
        if got_ev < 0:
            break
        now = now + got_ev
        ids, evs = acts.lazy_due(model, now, 1e-5)
        want = sorted(O.update_actions_state_lazy(now, 1e-5))
        assert list(zip(ids.tolist(), evs.tolist())) == want, step
        pops += len(want)
        dev, lzs = acts.state(), acts.lazy_state()
        for k in ("remains", "max_duration"):
            assert np.array_equal(dev[k], np.array(ost[k])), (step, k)
        for k in ("last_update", "last_value", "date"):
            assert np.array_equal(lzs[k], np.array(ost[k])), (step, k)
        assert np.array_equal(lzs["heap_type"], np.array(ost["heap_type"], np.uint8)), step
    assert pops > 0


@pytest.mark.parametrize("variant,name", [(1, "surf_usage"), (2, "surf_usage2")])
def test_surf_usage_device_matches_reference_tesh(variant, name):
    """The device step glue (act_lazy_update / act_lazy_min / act_lazy_due, lmm_step_kernels.hpp) over the HIP
    lmm solve replays teshsuite/surf/<name> (Cas01 + CM02, both LAZY, two_hosts_profiles.xml): every
    next-event date and every done / failed action of the reference's tesh (tests/surf_scenario.py)."""
    from tests import surf_scenario as SC

    assert SC.run_surf_usage(SC.DeviceBackend(), variant) == SC.expected(name)


@pytest.mark.parametrize("run", ["lv08_lazy", "lv08_full", "cm02_lazy"])
def test_pingpong_device_matches_reference_tesh(run):
    """examples/s4u/app-pingpong on the device: both communications built by lmm_communicate (the flow code of
    the C4 platforms, lmm_platforms.hpp), solved by the HIP solver, stepped by the device glue — act_next_event
    / act_update in Full mode, act_lazy_update / act_lazy_min / act_lazy_due in Lazy mode — print the tesh's
    lines: LV08 Lazy and Full 0.019014 / 150.178356, CM02 0.001462 / 145.639041 (tests/pingpong_scenario.py)."""
    from tests import pingpong_scenario as PP

    out, _ = PP.run_pingpong(PP.PingDevice(), run)
    assert out == PP.expected(run)


def test_pingpong_device_dates_equal_oracle():
    """The device replay's final clock equals the oracle replay's bit for bit in every configuration (the solve
    of a one-flow system and the element-wise step glue are exact)."""
    from tests import pingpong_scenario as PP

    for run in PP.RUNS:
        _, ed = PP.run_pingpong(PP.PingDevice(), run)
        _, eo = PP.run_pingpong(PP.PingOracle(), run)
        assert ed.now == eo.now, run
