"""Step-glue restatement (oracle/step_oracle.py) on hand-computed cases (CPU).  The device kernels are
compared with it bit for bit in tests/test_gpu_step.py."""
import pytest

from oracle import step_oracle as S


def test_next_event_min_of_remaining_time_duration_latency():
    # remains / value, 0 for a finished one, max duration, latency
    assert S.next_occuring_event_full([2.0, 4.0], [10.0, 4.0], [-1.0, -1.0]) == 1.0
    assert S.next_occuring_event_full([2.0, 0.0], [0.0, 4.0], [-1.0, -1.0]) == 0.0
    assert S.next_occuring_event_full([0.0, 0.0], [1.0, 4.0], [-1.0, 3.0]) == 3.0
    assert S.next_occuring_event_full([0.0], [1.0], [-1.0]) == -1.0
    assert S.next_occuring_event_full([0.0], [1.0], [-1.0], latency=[0.5]) == 0.5
    assert S.next_occuring_event_full([1.0], [1.0], [-1.0], latency=[0.0]) == 1.0


def state(**kw):
    st = dict(remains=[10.0], max_duration=[-1.0], latency=[0.0], penalty=[1.0], sharing_penalty=[1.0], flags=[0])
    st.update({k: [v] for k, v in kw.items()})
    return st


def test_cpu_update_and_finish():
    st = state()
    assert S.update_actions_state_full(0, [2.0], st, 4.0, 1e-5, 1e-5) == [0]
    assert st["remains"] == [2.0]
    assert S.update_actions_state_full(0, [2.0], st, 1.0, 1e-5, 1e-5) == [S.EV_FINISHED]
    assert st["remains"] == [0.0]
    st = state(max_duration=2.0)  # max duration reached
    assert S.update_actions_state_full(0, [0.0], st, 2.0, 1e-5, 1e-5) == [S.EV_FINISHED]
    st = state(remains=0.0, penalty=0.0)  # a disabled action does not finish on remains
    assert S.update_actions_state_full(0, [0.0], st, 1.0, 1e-5, 1e-5) == [0]


def test_cm02_latency_then_transfer():
    st = state(latency=0.5, penalty=0.0, sharing_penalty=3.0)
    assert S.update_actions_state_full(1, [0.0], st, 0.25, 1e-5, 1e-5) == [0]
    assert st["latency"] == [0.25] and st["penalty"] == [0.0]
    assert S.update_actions_state_full(1, [0.0], st, 0.25, 1e-5, 1e-5) == [S.EV_LATENCY_PAID]
    assert st["latency"] == [0.0] and st["penalty"] == [3.0]
    st = state(flags=S.ACT_NO_CNST)  # no link: completes at once
    assert S.update_actions_state_full(1, [0.0], st, 0.1, 1e-5, 1e-5) == [S.EV_FINISHED]
    st = state(latency=0.5, penalty=0.0, flags=S.ACT_SUSPENDED)  # suspended: penalty kept
    assert S.update_actions_state_full(1, [0.0], st, 1.0, 1e-5, 1e-5) == [0]


def test_l07_latency_sets_penalty_one():
    st = state(latency=0.5, penalty=0.0)
    assert S.update_actions_state_full(2, [0.0], st, 1.0, 1e-5, 1e-5) == [S.EV_LATENCY_PAID]
    assert st["penalty"] == [1.0] and st["latency"] == [0.0]


# ---- LAZY models (oracle.step_oracle.LazyModel: a real heap) ----
def lazy_state(n, **kw):
    st = dict(remains=[10.0] * n, max_duration=[-1.0] * n, penalty=[1.0] * n, flags=[0] * n,
              last_update=[0.0] * n, last_value=[0.0] * n, start_time=[0.0] * n, date=[0.0] * n,
              heap_type=[S.HEAP_UNSET] * n)
    st.update(kw)
    return st


def test_lazy_completion_dates_and_pop():
    # two flows at shares 2 and 1 from t=0: remaining 10 -> complete at 5 and 10
    m = S.LazyModel(1, lazy_state(2))
    ev, fin = m.next_occuring_event_lazy([2.0, 1.0], 0.0, [0, 1], 1e-5, 1e-5)
    assert ev == 5.0 and fin == []
    assert m.update_actions_state_lazy(5.0, 1e-5) == [(0, S.EV_FINISHED)]
    # at t=5 flow 1 is re-solved (now alone: share 2): it has 5 left -> completes at 7.5
    ev, fin = m.next_occuring_event_lazy([0.0, 2.0], 5.0, [1], 1e-5, 1e-5)
    assert m.st["remains"][1] == 5.0 and ev == 2.5
    assert m.update_actions_state_lazy(7.5, 1e-5) == [(1, S.EV_FINISHED)]
    assert m.next_occuring_event_lazy([0.0, 0.0], 7.5, [], 1e-5, 1e-5)[0] == -1.0


def test_lazy_max_duration_latency_hat_and_skips():
    st = lazy_state(4, max_duration=[3.0, -1.0, -1.0, -1.0], heap_type=[0, S.HEAP_LATENCY, 0, 0],
                    date=[0.0, 0.25, 0.0, 0.0], penalty=[1.0, 1.0, 0.0, 1.0], flags=[0, 0, 0, S.ACT_NOT_STARTED])
    m = S.LazyModel(1, st)
    ev, _ = m.next_occuring_event_lazy([1.0, 1.0, 1.0, 1.0], 0.0, [0, 1, 2, 3], 1e-5, 1e-5)
    # 0: max duration 3 < 10 -> max_duration hat; 1: latency hat untouched; 2: bogus penalty; 3: not started
    assert st["heap_type"] == [S.HEAP_MAX_DURATION, S.HEAP_LATENCY, 0, 0] and st["date"][0] == 3.0
    assert ev == 0.25
    assert m.update_actions_state_lazy(0.25, 1e-5) == [(1, S.EV_LATENCY_PAID)]
    assert st["last_update"][1] == 0.25


def test_lazy_pop_is_the_prefix_within_precision():
    """The device pops the SET {d : |d - now| < prec} once the top qualifies; the heap pops a prefix."""
    import random

    rng = random.Random(3)
    for _ in range(200):
        n = 30
        dates = [round(rng.uniform(0.99, 1.01), rng.choice([3, 5, 6, 7])) for _ in range(n)]
        st = lazy_state(n, date=list(dates), heap_type=[S.HEAP_NORMAL] * n)
        now = rng.choice(dates) + rng.choice([0.0, 4e-6, -4e-6, 2e-5])
        got = sorted(S.LazyModel(0, st).update_actions_state_lazy(now, 1e-5))
        top = min(dates)
        want = [(i, S.EV_FINISHED) for i, d in enumerate(dates) if abs(d - now) < 1e-5] if abs(top - now) < 1e-5 else []
        assert got == want


@pytest.mark.parametrize("variant,name", [(1, "surf_usage"), (2, "surf_usage2")])
def test_surf_usage_oracle_matches_reference_tesh(variant, name):
    """The step oracle (step_oracle.LazyModel over the LMM oracle) replays teshsuite/surf/<name>: Cas01 + CM02,
    both LAZY, on two_hosts_profiles.xml with its speed / state profiles — every next-event date (0.2, 0.200016,
    1, 7.32, 10 ... 130, 132.5) and every done / failed action of the reference's tesh (tests/surf_scenario.py,
    fixture tests/golden/surf_usage.json)."""
    from tests import surf_scenario as SC

    assert SC.run_surf_usage(SC.OracleBackend(), variant) == SC.expected(name)


def test_surf_usage_profiles_restated():
    """Profile::from_string's event list (Profile.cpp:65-100): deltas to the next event, LOOPAFTER + first date."""
    from tests import surf_scenario as SC

    pr = SC.golden()["profiles"]
    assert SC.profile_from_string(pr["trace_B.txt"]) == [[0.0, -1.0], [10.0, 1.0], [10.0, 0.8], [10.0, 0.4]]
    assert SC.profile_from_string(pr["trace_A_failure.txt"]) == [[1.0, -1.0], [1.0, -1.0], [9.0, 1.0]]
