#!/usr/bin/env python3
"""Dependency depth D of the reference's saturation order vs the device's round count (VERDICT r05 Next #1a).

The oracle (oracle/lmm_oracle.cpp, the restatement of maxmin.cpp:502-693) solves the system with `depth_on`: every
saturation event (a minimal-ratio constraint fixing its variables, :583) and every bound fix (:587-589, its own
node) gets a level = 1 + the deepest event that fixed a variable of its constraint(s) in an EARLIER sequential
round; D = the deepest level.  No exact schedule that saturates a constraint only once its own variables' fates are
known can take fewer than D rounds: if b fixed a variable of c before c saturated, b's round precedes c's on the
device too (the device reproduces the reference's events, values and saturated set).  With --device the same
system is solved on the GPU and every variable's device round (lmmhip_get_var_rounds) is compared with the level of
the event that fixed it: device round + 1 - level = the rounds the local-minimum schedule waited beyond the
dependency bound for that variable.

usage: python scripts/depth.py [--device] [--systems c4,c2_100,c2_10] --out profiles/r06_depth.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

C4 = dict(topo_parameters="3;16,16,16;1,16,16;1,1,1", loopback_bw=1e8)


def build(mod, name):
    """(system, variable handles) of one named system, built by module `mod` (oracle or product)."""
    if name.startswith("c2_"):
        div = int(name[3:])
        s = mod.System(False)
        vs = s.gen_synthetic(1_000_000 // div, 10_000_000 // div, 8, seed=1, want_vars=True)
        return s, vs
    if name == "c2":
        s = mod.System(False)
        return s, s.gen_synthetic(1_000_000, 10_000_000, 8, seed=1, want_vars=True)
    assert name == "c4"
    s = mod.System(False)
    _, vs = s.gen_platform_flows(mod.platform_params(topology=mod.FAT_TREE, model=mod.LV08, n_flows=100_000, seed=1,
                                                     **C4))
    return s, vs


def oracle_side(name):
    from oracle import pyoracle as O
    O.set_precision(1e-5)
    o, vs = build(O, name)
    o.set_depth(True)
    t = time.time()
    o.solve()
    dt = time.time() - t
    D, nsat, nbound, hist, bhist = o.depth_stats()
    lv, rd, by = o.variable_depth(vs)
    vals = o.values_of(vs, len(vs)) if hasattr(o, "values_of") else None
    res = {"sequential_rounds": int(o.last_rounds), "D": int(D), "saturation_events": int(nsat),
           "bound_fix_events": int(nbound), "oracle_solve_s": round(dt, 2),
           "saturations_per_level": hist.tolist(), "bound_fixes_per_level": bhist.tolist(),
           "variables": len(vs), "variables_fixed_by_bound": int(np.sum((by == 0) & (lv >= 0))),
           "variables_never_fixed": int(np.sum(lv < 0))}
    del o
    return res, lv, vals


def device_side(name, lv, ovals):
    import torch  # noqa: F401

    from simgrid_amd import lmm as L
    L.set_precision(1e-5)
    s, vs = build(L, name)
    s.set_resident(False)
    s.prepare()
    s.device_solve()
    st = s.last_stats()
    r = s.device_var_rounds().astype(np.int64)  # 1 + round, dense order
    x = s.device_values()
    res = {"device_rounds": int(st["rounds"]), "device_ms": round(float(st["device_ms"]), 3),
           "device_variables": int(len(r))}
    if len(r) == len(lv):
        ok = lv >= 1
        gap = r[ok] - lv[ok]  # (round + 1) - level: 0 = fixed in the first round the dependencies allow
        res["per_variable_wait_beyond_depth"] = {
            "mean": round(float(gap.mean()), 3), "p50": int(np.percentile(gap, 50)), "p90": int(np.percentile(gap, 90)),
            "p99": int(np.percentile(gap, 99)), "max": int(gap.max()), "min": int(gap.min()),
            "share_at_zero": round(float(np.mean(gap == 0)), 4)}
        if ovals is not None:
            res["alignment_check_max_abs_value_diff"] = float(np.max(np.abs(x - ovals)))
    del s
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--systems", default="c4,c2_100,c2_10")
    ap.add_argument("--device", action="store_true")
    ap.add_argument("--out", required=True)
    args = ap.parse_args()
    out = {"definition": __doc__.split("usage:")[0].strip(), "systems": {}}
    if os.path.exists(args.out):
        out = json.load(open(args.out))
    for name in args.systems.split(","):
        res, lv, vals = oracle_side(name)
        print(name, {k: v for k, v in res.items() if "per_level" not in k}, flush=True)
        if args.device:
            dres = device_side(name, lv, vals)
            res.update(dres)
            print(name, dres, flush=True)
        out["systems"].setdefault(name, {}).update(res)
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
