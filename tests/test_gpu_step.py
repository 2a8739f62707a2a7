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
