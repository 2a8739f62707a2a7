"""TEST INFRASTRUCTURE ONLY: the reference's surf_usage scenario as a tiny surf engine.

teshsuite/surf/surf_usage/surf_usage.cpp and surf_usage2/surf_usage2.cpp run, on
examples/platforms/two_hosts_profiles.xml, a Cas01 CPU model and a CM02 network model (both LAZY, the
defaults: cpu_cas01.cpp:20, network_cm02.cpp's "network/optim") under the compound host model, with a speed
and a state profile on "Cpu A", a speed profile on "Cpu B", two 1000-flop executions, a 7.32-s sleep and a
150-B communication.  Their tesh files print every next-event date and every done / failed action: the
reference's own known answer for the model-side step glue (Model::next_occuring_event_lazy, Model.cpp:40-101;
update_actions_state_lazy, cpu_interface.cpp:25-35 / network_cm02.cpp:103-126) on top of lmm_solve.

This module restates the pieces of the reference that the scenario exercises, over a pluggable backend:
  * profiles and the future event set: Profile::from_string / next (Profile.cpp:47-110), FutureEvtSet
    (FutureEvtSet.cpp), surf_presolve (surf_c_bindings.cpp:22-43), surf_solve (surf_c_bindings.cpp:45-148);
  * the CPU: CpuCas01::execution_start / sleep / apply_event / on_speed_change (cpu_cas01.cpp:104-207),
    CpuCas01Action (cpu_cas01.cpp:212-227);
  * the network: NetworkCm02Model::communicate (network_cm02.cpp:165-274) with cross-traffic (default on,
    network_interface.cpp) and the CM02 factors (latency / bandwidth factor 1, weight-S 0);
  * the host model: HostCLM03Model::next_occuring_event (host_clm03.cpp:34-52).
The per-model LAZY step passes (the part SURVEY.md §8 f1/f2 moves to the device) are the backend's:
  * OracleBackend — oracle/pyoracle.py's System (the LMM oracle) + oracle/step_oracle.LazyModel (a real heap);
  * DeviceBackend — simgrid_amd.lmm.System (HIP solve) + simgrid_amd.step.DeviceActions (lmm_step_kernels.hpp).
"""
import heapq
import os

SURF_PREC = 1e-5     # surf/precision default
MAXMIN_PREC = 1e-5   # maxmin/precision default
TCP_GAMMA = 4194304.0  # network/TCP-gamma default
NO_MAX_DURATION = -1.0
MODEL_CPU, MODEL_NET = 0, 1  # step_oracle / lmm_step_kernels model codes (CpuModel / NetworkCm02Model)

# ---- the platform of examples/platforms/two_hosts_profiles.xml (its data, restated) ----
PLATFORM = {
    "hosts": [("Cpu A", 10.0, "trace_A.txt", "trace_A_failure.txt"), ("Cpu B", 10.0, "trace_B.txt", None)],
    "link": ("LinkA", 10e6, 0.2),  # 10MBps, 200ms; the route Cpu A -> Cpu B (and back, symmetric Full routing)
}
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "surf_usage.json")


def golden():
    """tests/golden/surf_usage.json (tests/golden/make_surf_usage.py): the profiles' text and the tesh lines."""
    import json
    with open(GOLDEN) as f:
        return json.load(f)


def profile_from_string(text):
    """Profile::from_string (Profile.cpp:65-100): a fake first event (0, -1), then each event's date_ holds
    the delta to the next one; the last one's date_ is LOOPAFTER + the first event's date (or -1)."""
    ev = [[0.0, -1.0]]
    period = -1.0
    for line in text.replace("\r", "\n").split("\n"):
        val = line.strip()
        if not val or val[0] in "#%":
            continue
        w = val.split()
        if w[0] in ("PERIODICITY", "LOOPAFTER"):
            period = float(w[1])
            continue
        date, value = float(w[0]), float(w[1])
        ev[-1][0] = date - ev[-1][0]
        ev.append([date, value])
    ev[-1][0] = period + ev[0][0] if period > 0 else -1.0
    return ev


class ProfileEvent:
    def __init__(self, profile, resource, kind):
        self.profile, self.resource, self.kind, self.idx = profile, resource, kind, 0


class FutureEvtSet:
    """FutureEvtSet.cpp: a min-heap of (date, event); pop_leq advances the event's profile (Profile::next)."""

    def __init__(self):
        self.h, self.seq = [], 0

    def add(self, date, ev):
        heapq.heappush(self.h, (date, self.seq, ev))
        self.seq += 1

    def next_date(self):
        return self.h[0][0] if self.h else -1.0

    def pop_leq(self, date):
        if not self.h or self.h[0][0] > date:
            return None
        ev_date, _, ev = heapq.heappop(self.h)
        d, value = ev.profile[ev.idx]
        if ev.idx < len(ev.profile) - 1:  # Profile::next (Profile.cpp:47-62)
            self.add(ev_date + d, ev)
            ev.idx += 1
        elif d > 0:  # loop
            self.add(ev_date + d, ev)
            ev.idx = 1
        return ev, value


class Action:
    STARTED, FAILED, FINISHED = "started", "failed", "finished"

    def __init__(self, model, cost, now):
        self.model, self.remains, self.start_time = model, cost, now
        self.state = Action.STARTED
        self.max_duration = NO_MAX_DURATION
        self.sharing_penalty = 1.0  # Action::sharing_penalty_ default
        self.last_update, self.last_value = 0.0, 0.0
        self.date, self.heap_type = float("inf"), 0  # ActionHeap entry (0 = unset)
        self.var = None
        self.finish_time = -1.0
        self.alive = True


HEAP_UNSET, HEAP_LATENCY, HEAP_MAX_DURATION, HEAP_NORMAL = 0, 1, 2, 3


class Model:
    """One LAZY resource model: its lmm System (selective update), its actions, the modified-set additions
    that bypass lmm (CpuCas01::sleep pushes its action there itself, cpu_cas01.cpp:193-196)."""

    def __init__(self, kind, backend):
        self.kind, self.backend = kind, backend
        self.sys = backend.new_system()
        self.actions = []
        self.extra_modified = []

    def started(self):
        return [a for a in self.actions if a.alive and a.state == Action.STARTED]

    def extract(self, state):
        return [a for a in self.actions if a.alive and a.state == state]

    def next_occuring_event(self, now):
        """Model::next_occuring_event_lazy (Model.cpp:40-101)."""
        mod = self.backend.solve(self)
        for a in self.extra_modified:
            if a.alive and a not in mod:
                mod.append(a)
        self.extra_modified = []
        for a in self.backend.lazy_update(self, mod, now):  # update_remains_lazy finished them (network)
            self.finish(a, now)
        tops = [a.date for a in self.actions if a.alive and a.heap_type != HEAP_UNSET]
        return min(tops) - now if tops else -1.0

    def update_actions_state(self, now):
        """CpuModel / NetworkCm02Model::update_actions_state_lazy."""
        for a, ev in self.backend.lazy_due(self, now):
            if ev == 2:  # latency hat paid: the variable gets its sharing penalty (network_cm02.cpp:112-116)
                self.sys.update_variable_penalty(a.var, a.sharing_penalty)
            else:
                self.finish(a, now)

    @staticmethod
    def finish(a, now):  # Action::finish (Action.cpp:40-45)
        a.finish_time, a.remains, a.state = now, 0.0, Action.FINISHED

    def unref(self, a):  # Action::~Action (Action.cpp:30-38)
        a.alive = False
        self.sys.variable_free(a.var)
        a.heap_type, a.date = HEAP_UNSET, float("inf")
        if a in self.extra_modified:
            self.extra_modified.remove(a)


class Engine:
    def __init__(self, backend):
        self.backend, self.now = backend, 0.0
        self.cpu = Model(MODEL_CPU, backend)
        self.net = Model(MODEL_NET, backend)
        self.models = [self.cpu, self.net]  # all_existing_models order: cpu (pm), network; host/vm add no work
        self.fes = FutureEvtSet()
        self.hosts = {}
        profiles = golden()["profiles"]
        for name, speed, speed_file, state_file in PLATFORM["hosts"]:
            h = dict(name=name, peak=speed, scale=1.0, on=True)
            h["cnst"] = self.cpu.sys.constraint_new(self._rid(), 1 * speed)  # CpuCas01: core * speed_per_pstate[0]
            self.hosts[name] = h
            for fname, kind in ((speed_file, "speed"), (state_file, "state")):
                if fname:  # Profile::schedule: the profile's event enters the set at 0
                    self.fes.add(0.0, ProfileEvent(profile_from_string(profiles[fname]), h, kind))
        lname, bw, lat = PLATFORM["link"]
        self.link = dict(name=lname, bw=bw, lat=lat)
        self.link["cnst"] = self.net.sys.constraint_new(self._rid(), 1.0 * bw)  # sg_bandwidth_factor (CM02: 1)
        self.presolve()

    _next_id = [1]

    def _rid(self):
        self._next_id[0] += 1
        return self._next_id[0]

    # ---- resources (cpu_cas01.cpp) ----
    def is_used(self, res):
        return self.cpu.sys.constraint_used(res["cnst"])

    def apply_event(self, ev, value):
        h = ev.resource
        if ev.kind == "speed":  # CpuCas01::apply_event + on_speed_change (cpu_cas01.cpp:102-129)
            h["scale"] = value
            self.cpu.sys.update_constraint_bound(h["cnst"], 1 * h["scale"] * h["peak"])
            for a in self.cpu.actions:
                if a.alive and a.host is h:
                    self.cpu.sys.update_variable_bound(a.var, 1 * h["scale"] * h["peak"])
        else:  # state event (cpu_cas01.cpp:130-154)
            if value > 0:
                h["on"] = True
            else:
                h["on"] = False
                for a in self.cpu.actions:
                    if a.alive and a.host is h and a.state == Action.STARTED:
                        a.finish_time, a.state = self.now, Action.FAILED

    # ---- actions ----
    def _cpu_action(self, h, cost):  # CpuCas01Action (cpu_cas01.cpp:212-227)
        a = Action(self.cpu, cost, self.now)
        a.host = h
        if not h["on"]:
            a.state = Action.FAILED
        a.var = self.cpu.sys.variable_new(self._aid(a, self.cpu), 1.0, 1 * h["scale"] * h["peak"], 1)
        a.last_update = self.now
        self.cpu.sys.expand(h["cnst"], a.var, 1.0)
        self.cpu.actions.append(a)
        return a

    def _aid(self, a, model):
        a.id = self._rid()
        self.backend.register(model, a)
        return a.id

    def execution_start(self, host, size):
        return self._cpu_action(self.hosts[host], size)

    def sleep(self, host, duration):  # CpuCas01::sleep (cpu_cas01.cpp:176-200)
        if duration > 0:
            duration = max(duration, SURF_PREC)
        a = self._cpu_action(self.hosts[host], 1.0)
        a.max_duration = duration  # set_max_duration: LAZY -> off the heap (not in it yet)
        a.heap_type, a.date = HEAP_UNSET, float("inf")
        self.cpu.sys.update_variable_penalty(a.var, 0.0)
        self.cpu.extra_modified.insert(0, a)
        return a

    def communicate(self, src, dst, size, rate):  # NetworkCm02Model::communicate (network_cm02.cpp:165-274)
        route, back = [self.link], [self.link]  # Full routing, symmetric
        latency = sum(l["lat"] for l in route)
        a = Action(self.net, size, self.now)
        a.sharing_penalty = latency
        a.latency = latency
        a.rate = rate
        a.last_update = self.now
        a.lat_current = a.latency
        a.latency *= 1.0  # latency factor (CM02: 1)
        n = len(route) + len(back)
        if a.latency > 0:
            a.var = self.net.sys.variable_new(self._aid(a, self.net), 0.0, -1.0, n)
            a.date, a.heap_type = a.latency + a.last_update, HEAP_LATENCY
        else:
            a.var = self.net.sys.variable_new(self._aid(a, self.net), 1.0, -1.0, n)
        if a.rate < 0:
            self.net.sys.update_variable_bound(a.var, TCP_GAMMA / (2.0 * a.lat_current) if a.lat_current > 0 else -1.0)
        else:
            self.net.sys.update_variable_bound(a.var, min(a.rate, TCP_GAMMA / (2.0 * a.lat_current))
                                               if a.lat_current > 0 else a.rate)
        for l in route:
            self.net.sys.expand(l["cnst"], a.var, 1.0)
        for l in back:  # cross-traffic: 5 % of the bandwidth backwards
            self.net.sys.expand(l["cnst"], a.var, 0.05)
        self.net.actions.append(a)
        return a

    # ---- surf_c_bindings.cpp ----
    def presolve(self):  # surf_presolve (surf_c_bindings.cpp:22-43): events at time 0, values >= 0 only
        while self.fes.next_date() != -1.0 and self.fes.next_date() <= self.now:
            d = self.fes.next_date()
            while True:
                r = self.fes.pop_leq(d)
                if r is None:
                    break
                if r[1] >= 0:
                    self.apply_event(*r)
        for m in self.models:
            m.update_actions_state(self.now)

    def host_next(self):  # HostCLM03Model::next_occuring_event (host_clm03.cpp:34-52)
        res = self.cpu.next_occuring_event(self.now)
        net = self.net.next_occuring_event(self.now)
        if res < 0 or (net >= 0 and net < res):
            res = net
        return res

    def solve(self):  # surf_solve(-1) (surf_c_bindings.cpp:45-148)
        time_delta = -1.0
        phy = self.host_next()
        if (time_delta < 0 or phy < time_delta) and phy >= 0:
            time_delta = phy
        m = self.cpu.next_occuring_event(self.now)  # the loop over the other models: the CPU model again
        if (time_delta < 0 or m < time_delta) and m >= 0:
            time_delta = m
        while True:
            d = self.fes.next_date()
            if d < 0 or d > self.now + time_delta:
                break
            while True:
                r = self.fes.pop_leq(d)
                if r is None:
                    break
                ev, value = r
                if self.is_used(ev.resource):
                    time_delta = d - self.now
                start, self.now = self.now, d
                self.apply_event(ev, value)
                self.now = start
        if time_delta < 0:
            return -1.0
        self.now = self.now + time_delta
        for mdl in self.models:
            mdl.update_actions_state(self.now)
        return time_delta


def run_surf_usage(backend, variant=1):
    """surf_usage.cpp (variant 1) / surf_usage2.cpp (variant 2): the (clock, message) lines they log."""
    e = Engine(backend)
    out = []

    def log(msg):
        out.append(("%.6f" % e.now, msg))
    a = e.execution_start("Cpu A", 1000.0)
    b = e.execution_start("Cpu B", 1000.0)
    c = e.sleep("Cpu B", 7.32)
    if variant == 1:
        for name, act in (("actionA", a), ("actionB", b), ("actionC", c)):
            log(f"{name} state: " + ("SURF_ACTION_RUNNING" if act.state == Action.STARTED else "?"))
    e.communicate("Cpu A", "Cpu B", 150.0, -1.0)
    e.solve()
    while True:
        log("Next Event : %g" % e.now)
        running = False
        if variant == 1:
            for mdl, what in ((e.cpu, "CPU"), (e.net, "Network")):
                for act in mdl.extract(Action.FAILED):
                    log(f"   {what} Failed action")
                    mdl.unref(act)
                for act in mdl.extract(Action.FINISHED):
                    log(f"   {what} Done action")
                    mdl.unref(act)
            running = bool(e.net.started() or e.cpu.started())
        else:
            for mdl in e.models:
                running |= bool(mdl.started())
                for st in (Action.FAILED, Action.FINISHED):
                    for act in mdl.extract(st):
                        log("   * Done Action")
                        mdl.unref(act)
        if not (running and e.solve() >= 0.0):
            break
    if variant == 2:
        log("Simulation Terminated")
    return out


def expected(name):
    """The surf_test/INFO lines of teshsuite/surf/<name>/<name>.tesh: (clock "%.6f", message)."""
    return [tuple(x) for x in golden()["expected"][name]]


# ---- backends ----
class OracleBackend:
    """The LMM oracle (oracle/pyoracle.py) + step_oracle.LazyModel per call (a real heap)."""

    def __init__(self):
        from oracle import pyoracle as O
        from oracle import step_oracle as S
        self.O, self.S = O, S
        self.by_var = {}

    def new_system(self):
        return self.O.System(True)

    def register(self, model, a):
        pass

    def solve(self, model):
        model.sys.solve()
        for a in model.actions:
            if a.alive:
                self.by_var[a.var.h] = a
        mod = []
        for v in model.sys.modified_actions():
            a = self.by_var.get(v.h)
            if a is not None and a.alive and a not in mod:
                mod.append(a)
        model.sys.clear_modified_actions()
        model.values = {id(a): a.var.get_value() for a in model.actions if a.alive}
        return mod

    def _lazy(self, model):
        acts = [a for a in model.actions if a.alive]
        st = dict(remains=[a.remains for a in acts], max_duration=[a.max_duration for a in acts],
                  penalty=[a.sharing_penalty for a in acts],
                  flags=[0 if a.state == Action.STARTED else self.S.ACT_NOT_STARTED for a in acts],
                  last_update=[a.last_update for a in acts], last_value=[a.last_value for a in acts],
                  start_time=[a.start_time for a in acts], date=[a.date for a in acts],
                  heap_type=[a.heap_type for a in acts])
        return acts, st, self.S.LazyModel(model.kind, st)

    @staticmethod
    def _back(acts, st):
        for i, a in enumerate(acts):
            a.remains, a.max_duration = st["remains"][i], st["max_duration"][i]
            a.last_update, a.last_value = st["last_update"][i], st["last_value"][i]
            a.date, a.heap_type = st["date"][i], st["heap_type"][i]

    def lazy_update(self, model, mod, now):
        acts, st, lm = self._lazy(model)
        idx = {id(a): i for i, a in enumerate(acts)}
        values = [model.values.get(id(a), 0.0) for a in acts]
        _, fin = lm.next_occuring_event_lazy(values, now, [idx[id(a)] for a in mod], MAXMIN_PREC, SURF_PREC)
        self._back(acts, st)
        return [acts[i] for i in fin]

    def lazy_due(self, model, now):
        acts, st, lm = self._lazy(model)
        out = lm.update_actions_state_lazy(now, SURF_PREC)
        self._back(acts, st)
        return [(acts[i], ev) for i, ev in out]


class DeviceBackend:
    """simgrid_amd.lmm.System (the HIP solver, selective update) + the device step glue per call
    (simgrid_amd.step.DeviceActions: act_lazy_update / act_lazy_min / act_lazy_due)."""

    def __init__(self):
        from simgrid_amd import lmm as L
        from simgrid_amd import multi as M
        from simgrid_amd import step as D
        self.L, self.M, self.D = L, M, D
        self.by_id = {}

    def new_system(self):
        return self.L.System(True)

    def register(self, model, a):
        self.by_id[a.id] = a

    def solve(self, model):
        # the dense index of every action's variable in the flattened system this solve runs on
        f = self.M.export_flat(model.sys) if model.sys.modified else None
        model.sys.lmm_solve()
        pos = {} if f is None else {int(v): i for i, v in enumerate(f.var_ids)}
        model.vidx = {id(a): pos.get(int(a.var.h), -1) for a in model.actions if a.alive}
        mod = []
        for aid in model.sys.modified_action_ids():
            a = self.by_id.get(aid)
            if a is not None and a.alive and a not in mod:
                mod.append(a)
        model.sys.clear_modified_actions()
        return mod

    def _acts(self, model):
        import numpy as np
        acts = [a for a in model.actions if a.alive]
        D = self.D
        vi = np.array([model.__dict__.get("vidx", {}).get(id(a), -1) for a in acts], np.int32)
        da = D.DeviceActions(model.sys.device_ctx(), vi, remains=[a.remains for a in acts],
                             max_duration=[a.max_duration for a in acts],
                             penalty=[a.sharing_penalty for a in acts],
                             flags=[0 if a.state == Action.STARTED else D.ACT_NOT_STARTED for a in acts])
        da.lazy_init(last_update=[a.last_update for a in acts], last_value=[a.last_value for a in acts],
                     start_time=[a.start_time for a in acts], date=[a.date for a in acts],
                     heap_type=[a.heap_type for a in acts])
        return acts, da

    @staticmethod
    def _back(acts, da):
        st, lz = da.state(), da.lazy_state()
        for i, a in enumerate(acts):
            a.remains, a.max_duration = float(st["remains"][i]), float(st["max_duration"][i])
            a.last_update, a.last_value = float(lz["last_update"][i]), float(lz["last_value"][i])
            a.date, a.heap_type = float(lz["date"][i]), int(lz["heap_type"][i])

    def lazy_update(self, model, mod, now):
        acts, da = self._acts(model)
        if not acts:
            return []
        idx = {id(a): i for i, a in enumerate(acts)}
        da.lazy_update(model.kind, now, [idx[id(a)] for a in mod], MAXMIN_PREC, SURF_PREC)
        ev = da.state()["events"]
        self._back(acts, da)
        return [a for i, a in enumerate(acts) if idx[id(a)] in {idx[id(m)] for m in mod} and ev[i] & 1]

    def lazy_due(self, model, now):
        acts, da = self._acts(model)
        if not acts:
            return []
        top = da.next_occuring_event_lazy(now)
        if top < 0 or not abs(top) < SURF_PREC:  # the top is not due: nothing pops (act_lazy_due's contract)
            return []
        ids, evs = da.lazy_due(model.kind, now, SURF_PREC)
        self._back(acts, da)
        return [(acts[int(i)], int(e)) for i, e in zip(ids, evs)]
