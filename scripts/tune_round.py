#!/usr/bin/env python
"""Launch-width sweep of the max-min round kernels on one resident C2 system (GPU box).

Builds the system once, then for each (LMMHIP_UPD_BLOCKS, LMMHIP_READY_BLOCKS, LMMHIP_SAT_BLOCKS)
setting runs `--reps` device solves (inputs resident in HBM) and prints the median HIP-event time.
usage: python scripts/tune_round.py [--cnst N] [--vars N] [--reps R]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simgrid_amd import lmm as L  # noqa: E402

CONFIGS = [(0, 0, 0), (1024, 0, 0), (512, 0, 0), (0, 0, 1024), (0, 0, 512), (0, 1024, 0), (0, 512, 0),
           (1024, 1024, 1024), (512, 512, 512), (0, 0, 256)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cnst", type=int, default=1000000)
    ap.add_argument("--vars", type=int, default=10000000)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    s = L.System(False)
    vs = s.gen_synthetic(a.cnst, a.vars, k=8, seed=1)
    s.prepare()
    s.device_solve()
    ref = None
    for upd, rdy, sat in CONFIGS:
        os.environ["LMMHIP_UPD_BLOCKS"], os.environ["LMMHIP_READY_BLOCKS"], os.environ["LMMHIP_SAT_BLOCKS"] = (
            str(upd), str(rdy), str(sat))
        t = []
        for _ in range(a.reps):
            s.device_solve()
            t.append(s.last_stats()["device_ms"])
        s.fetch()
        x = s.values_of(vs)
        if ref is None:
            ref = x
        ok = bool(np.all(np.abs(x - ref) <= np.maximum(1e-9, 1e-6 * np.abs(ref))))
        print(json.dumps(dict(upd=upd, ready=rdy, sat=sat, ms=round(float(np.median(t)), 3),
                              min_ms=round(min(t), 3), rounds=s.last_stats()["rounds"], values_ok=ok)), flush=True)


if __name__ == "__main__":
    main()
