#!/usr/bin/env python
"""Simulation-step timing of the two solve paths on one system (GPU box):

  host    : System::solve() = host flatten_maxmin + full upload + device solve + fetch
  resident: System::solve() = delta-log ship + device flatten + device solve + fetch

Each step first mutates the system through the API (untimed: that is the simulation's own work):
`--pen` penalty updates (0 / 0.5 / 1 / 2: flows pausing, resuming, changing priority) and `--cb`
constraint-bound updates.  Prints one JSON line per path with the per-phase wall times.
usage: python scripts/resident_steps.py [--cnst N] [--vars N] [--steps K] [--pen P] [--cb B]
"""
import argparse
import ctypes as ct
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simgrid_amd import lmm as L  # noqa: E402


def run(resident, a):
    s = L.System(False)
    t0 = time.perf_counter()
    vs = s.gen_synthetic(a.cnst, a.vars, k=8, seed=1)
    gen_s = time.perf_counter() - t0
    s.set_resident(resident)
    rng = np.random.default_rng(9)
    rows = []
    for step in range(a.steps + 1):
        if step:
            for i in rng.choice(a.vars, a.pen, replace=False):
                s.update_variable_penalty(L.Variable(s, int(vs[i])), float(rng.choice([0.5, 1.0, 2.0])))
            for c in rng.choice(a.cnst, a.cb, replace=False):
                s.update_constraint_bound(L.Constraint(s, int(c)), float(rng.uniform(0.5, 10.0)))
        t = time.perf_counter()
        s.solve()
        wall = (time.perf_counter() - t) * 1e3
        st = s.last_stats()
        nref = ct.c_int64(-1)
        if resident:
            L._check_hip(L.lib().lmmhip_res_refreshes(s.device_ctx(), ct.byref(nref)))
        rows.append(dict(step=step, wall_ms=wall, flatten_ms=st["flatten_ms"], upload_ms=st["upload_ms"],
                         device_ms=st["device_ms"], fetch_ms=st["fetch_ms"], delta_records=st["delta_records"],
                         n_var=st["n_var"], refreshes=nref.value))
        print(json.dumps(dict(path="resident" if resident else "host", **rows[-1])), file=sys.stderr, flush=True)
    x = s.values_of(vs)
    steady = rows[1:]
    med = lambda k: float(np.median([r[k] for r in steady]))  # noqa: E731
    return dict(path="resident" if resident else "host", cnst=a.cnst, vars=a.vars, steps=a.steps,
                pen_updates=a.pen, cbound_updates=a.cb, gen_s=round(gen_s, 2), first_solve_ms=round(rows[0]["wall_ms"], 2),
                step_wall_ms=round(med("wall_ms"), 2), step_host_ms=round(med("flatten_ms"), 2),
                step_upload_or_devflatten_ms=round(med("upload_ms"), 2), step_device_ms=round(med("device_ms"), 2),
                step_fetch_ms=round(med("fetch_ms"), 2), delta_records=int(med("delta_records")),
                vars_per_s=round(a.vars / (med("wall_ms") / 1e3), 1)), x


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cnst", type=int, default=1000000)
    ap.add_argument("--vars", type=int, default=10000000)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--pen", type=int, default=10000)
    ap.add_argument("--cb", type=int, default=1000)
    ap.add_argument("--resident-only", action="store_true")
    a = ap.parse_args()
    res, xr = run(True, a)
    print(json.dumps(res), flush=True)
    if a.resident_only:
        return
    host, xh = run(False, a)
    print(json.dumps(host), flush=True)
    # parity tolerance of tests/lmm_cases.py (fp64 decrement atomics: last bits vary run to run)
    worst = float(np.max(np.abs(xr - xh) / np.maximum(1e-3, np.abs(xh)))) if len(xh) else 0.0
    assert np.all(np.abs(xr - xh) <= np.maximum(1e-9, 1e-6 * np.abs(xh))), "resident and host paths disagree"
    print(json.dumps(dict(values_within_tolerance=True, worst_rel_diff=worst,
                          step_speedup=round(host["step_wall_ms"] / res["step_wall_ms"], 2))))


if __name__ == "__main__":
    main()
