"""Step-glue restatement (oracle/step_oracle.py) on hand-computed cases (CPU).  The device kernels are
compared with it bit for bit in tests/test_gpu_step.py."""
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
