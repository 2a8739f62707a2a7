"""Model-side step glue on the device: the action state of a model (remains, max
duration, latency) kept in HBM next to the solver's values, with the two per-step passes of a FULL-update
model run as kernels (lmm_step_kernels.hpp) through the lmmhip_* step ABI:

* `next_occuring_event` — Model::next_occuring_event_full (Model.cpp:103-129), plus the latency term of
  NetworkModel (network_interface.cpp:57-70) and HostL07Model (ptask_L07.cpp:69-82);
* `update_actions_state` — update_actions_state_full of CpuModel (cpu_interface.cpp:37-51),
  NetworkCm02Model (network_cm02.cpp:128-163) and HostL07Model (ptask_L07.cpp:84-118);
* LAZY models (the default, sg_config.cpp:252): `lazy_update` (the loop of
  Model::next_occuring_event_lazy over lmm_solve's modified actions, Model.cpp:46-94),
  `next_occuring_event_lazy` (heap top - now) and `lazy_due` (update_actions_state_lazy) over an
  ActionHeap kept as per-action (date, type) arrays in HBM.

Only the events (finished actions, paid latencies) go back to the host, which then does what the
reference does with them: Action::finish, update_variable_penalty (and, for L07, updateBound).  With
several GPUs, the step date is multi.next_event_date over the ranks' `next_occuring_event`.
"""
import ctypes as ct

import numpy as np

from simgrid_amd import lmm

MODEL_CPU, MODEL_CM02, MODEL_L07 = 0, 1, 2
EV_FINISHED, EV_LATENCY_PAID = 1, 2
ACT_NO_CNST, ACT_SUSPENDED, ACT_NOT_STARTED = 1, 2, 4
HEAP_UNSET, HEAP_LATENCY, HEAP_MAX_DURATION, HEAP_NORMAL = 0, 1, 2, 3  # ActionHeap::Type
NO_MAX_DURATION = -1.0
SURF_PRECISION = 1e-5  # --cfg=surf/precision default


def dense_index(flat_var_ids, action_vars):
    """Dense (device) index of each action's variable id, -1 when the variable is not solved."""
    pos = {int(v): i for i, v in enumerate(flat_var_ids)}
    return np.array([pos.get(int(v), -1) for v in action_vars], dtype=np.int32)


def _p(a, t):
    return a.ctypes.data_as(ct.POINTER(t))


class DeviceActions:
    """The actions of one model on the device context `ctx` (System.device_ctx() or a multi shard)."""

    def __init__(self, ctx, var_index, remains, max_duration=None, latency=None, penalty=None,
                 sharing_penalty=None, flags=None):
        n = len(var_index)
        self.ctx, self.n, self.L = ctx, n, lmm.lib()

        def arr(a, default, dtype=np.float64):
            return np.ascontiguousarray(np.full(n, default) if a is None else a, dtype=dtype)

        vi = arr(var_index, -1, np.int32)
        rem = arr(remains, 0.0)
        md = arr(max_duration, NO_MAX_DURATION)
        lat = arr(latency, 0.0)
        pen = arr(penalty, 1.0)
        sp = arr(sharing_penalty, 1.0)
        fl = arr(flags, 0, np.uint8)
        self._check(self.L.lmmhip_actions_upload(ctx, n, _p(vi, ct.c_int32), _p(rem, ct.c_double),
                                                 _p(md, ct.c_double), _p(lat, ct.c_double), _p(pen, ct.c_double),
                                                 _p(sp, ct.c_double), _p(fl, ct.c_uint8)))

    def _check(self, rc):
        if rc != 0:
            raise lmm.LmmError(self.L.lmmhip_last_error().decode())

    def next_occuring_event(self, with_latency=False):
        out = ct.c_double()
        self._check(self.L.lmmhip_next_event_full(self.ctx, int(with_latency), ct.byref(out)))
        return out.value

    def update_actions_state(self, model, delta, maxmin_precision=None, surf_precision=SURF_PRECISION):
        mp = lmm.get_precision() if maxmin_precision is None else maxmin_precision
        n = ct.c_int64()
        self._check(self.L.lmmhip_update_actions_full(self.ctx, model, delta, mp, surf_precision, ct.byref(n)))
        return n.value

    def state(self):
        """remains, max_duration, latency, penalty, events (numpy copies)."""
        out = [np.empty(self.n) for _ in range(4)] + [np.empty(self.n, np.uint8)]
        self._check(self.L.lmmhip_actions_download(self.ctx, *[_p(a, ct.c_double) for a in out[:4]],
                                                   _p(out[4], ct.c_uint8)))
        return dict(zip(("remains", "max_duration", "latency", "penalty", "events"), out))

    # ---- LAZY models ----
    def lazy_init(self, last_update=None, last_value=None, start_time=None, date=None, heap_type=None):
        n = self.n

        def arr(a, default, dtype=np.float64):
            return np.ascontiguousarray(np.full(n, default) if a is None else a, dtype=dtype)

        lu, lv, st = arr(last_update, 0.0), arr(last_value, 0.0), arr(start_time, 0.0)
        dt, ht = arr(date, 0.0), arr(heap_type, HEAP_UNSET, np.uint8)
        self._check(self.L.lmmhip_actions_lazy_upload(self.ctx, _p(lu, ct.c_double), _p(lv, ct.c_double),
                                                      _p(st, ct.c_double), _p(dt, ct.c_double), _p(ht, ct.c_uint8)))

    def lazy_update(self, model, now, modified, maxmin_precision=None, surf_precision=SURF_PRECISION):
        mp = lmm.get_precision() if maxmin_precision is None else maxmin_precision
        mod = np.ascontiguousarray(modified, dtype=np.int32)
        n = ct.c_int64()
        self._check(self.L.lmmhip_actions_lazy_update(self.ctx, model, now, mp, surf_precision, len(mod),
                                                      _p(mod, ct.c_int32), ct.byref(n)))
        return n.value

    def next_occuring_event_lazy(self, now):
        out = ct.c_double()
        self._check(self.L.lmmhip_next_event_lazy(self.ctx, now, ct.byref(out)))
        return out.value

    def lazy_due(self, model, now, surf_precision=SURF_PRECISION):
        """Popped actions (ascending index) and their events."""
        ids, ev = np.empty(self.n, np.int32), np.empty(self.n, np.uint8)
        k = ct.c_int64()
        self._check(self.L.lmmhip_actions_lazy_due(self.ctx, model, now, surf_precision, _p(ids, ct.c_int32),
                                                   _p(ev, ct.c_uint8), self.n, ct.byref(k)))
        return ids[: k.value].copy(), ev[: k.value].copy()

    def lazy_state(self):
        out = [np.empty(self.n) for _ in range(3)] + [np.empty(self.n, np.uint8)]
        self._check(self.L.lmmhip_actions_lazy_download(self.ctx, *[_p(a, ct.c_double) for a in out[:3]],
                                                        _p(out[3], ct.c_uint8)))
        return dict(zip(("last_update", "last_value", "date", "heap_type"), out))
