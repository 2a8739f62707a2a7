"""How many variable values a drop-in C2 step changes (bench.py's mutations: 1e4 penalties, 1e3 constraint bounds
per step): the share of slots whose value differs from the previous solve's, bit for bit.  Measurement for the
value path's delta transfer.  Run on the GPU: python scripts/changed_values.py"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simgrid_amd import lmm  # noqa: E402


def main():
    nc, nv = 1_000_000, 10_000_000
    s = lmm.System(False)
    vs = s.gen_synthetic(nc, nv, 8, seed=1)
    s.solve()
    prev = s.values_of(vs)
    rng = np.random.default_rng(9)
    out = []
    for step in range(3):
        for i in rng.choice(nv, 10_000, replace=False):
            s.update_variable_penalty(lmm.Variable(s, int(vs[i])), float(rng.choice([0.5, 1.0, 2.0])))
        for c in rng.choice(nc, 1_000, replace=False):
            s.update_constraint_bound(lmm.Constraint(s, int(c)), float(rng.uniform(0.5, 10.0)))
        s.solve()
        x = s.values_of(vs)
        ch = x != prev
        rel = np.abs(x - prev) / np.maximum(np.abs(prev), 1e-300)
        out.append({"step": step, "changed": int(ch.sum()), "share": float(ch.mean()),
                    "changed_rel_gt_1e-9": int((rel > 1e-9).sum()), "rounds": s.last_stats()["rounds"]})
        print(json.dumps(out[-1]), flush=True)
        prev = x


if __name__ == "__main__":
    main()
