"""ORACLE — TEST INFRASTRUCTURE ONLY.  Pure-Python restatement of the model-side step passes the device
runs in simgrid_amd/csrc/lmm_step_kernels.hpp (small cases; one action at a time, in the reference's
order of operations).  Imported by tests/ only."""
import math

NO_MAX_DURATION = -1.0  # Action.hpp:17
EV_FINISHED, EV_LATENCY_PAID = 1, 2
ACT_NO_CNST, ACT_SUSPENDED = 1, 2


def double_update(v, d, prec):  # surf_interface.hpp:34-42
    v -= d
    return 0.0 if v < prec else v


def next_occuring_event_full(values, remains, max_duration, latency=None):
    """Model::next_occuring_event_full (Model.cpp:103-129); with `latency`, the network / ptask term
    (network_interface.cpp:57-70, ptask_L07.cpp:69-82).  -1 = no event."""
    mn = -1.0
    for i, value in enumerate(values):
        if value > 0:
            value = remains[i] / value if remains[i] > 0 else 0.0
            if mn < 0 or value < mn:
                mn = value
        if max_duration[i] >= 0 and (mn < 0 or max_duration[i] < mn):
            mn = max_duration[i]
    if latency is not None:
        for lat in latency:
            if lat > 0:
                mn = lat if mn < 0 else min(mn, lat)
    return mn


def update_actions_state_full(model, values, st, delta, maxmin_prec, surf_prec):
    """In place on st = dict(remains, max_duration, latency, penalty, sharing_penalty, flags) lists;
    returns the per-action event codes.  model 0 = CpuModel (cpu_interface.cpp:37-51), 1 = CM02
    (network_cm02.cpp:128-163), 2 = L07 (ptask_L07.cpp:84-118)."""
    events = []
    rprec = maxmin_prec * surf_prec  # Action::update_remains (Action.cpp:199-202)
    for i, value in enumerate(values):
        ev = 0
        rem, md, lat, pen = st["remains"][i], st["max_duration"][i], st["latency"][i], st["penalty"][i]
        fl = st["flags"][i]
        if model == 1:
            deltap = delta
            if lat > 0:
                if lat > deltap:
                    lat = double_update(lat, deltap, surf_prec)
                    deltap = 0.0
                else:
                    deltap = double_update(deltap, lat, surf_prec)
                    lat = 0.0
                if lat <= 0.0 and not fl & ACT_SUSPENDED:
                    pen = st["sharing_penalty"][i]
                    ev |= EV_LATENCY_PAID
            if fl & ACT_NO_CNST:
                rem = double_update(rem, rem, rprec)
        elif model == 2:
            if lat > 0:
                lat = double_update(lat, delta, surf_prec) if lat > delta else 0.0
                if lat <= 0.0 and not fl & ACT_SUSPENDED:
                    pen = 1.0
                    ev |= EV_LATENCY_PAID
        rem = double_update(rem, value * delta, rprec)
        if md != NO_MAX_DURATION:  # Action::update_max_duration (Action.cpp:194-198)
            md = double_update(md, delta, surf_prec)
        if (rem <= 0 and pen > 0) or (md != NO_MAX_DURATION and md <= 0):
            ev |= EV_FINISHED
        st["remains"][i], st["max_duration"][i], st["latency"][i], st["penalty"][i] = rem, md, lat, pen
        events.append(ev)
    assert all(not math.isnan(x) for x in st["remains"])
    return events
