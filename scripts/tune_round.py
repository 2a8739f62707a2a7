#!/usr/bin/env python
"""Sweep of the max-min solve's tuning knobs on one resident C2 system (GPU box).

Builds the system once, then for each setting of the launch widths (--sweep widths:
LMMHIP_UPD/READY/SAT_BLOCKS) or of the compaction cadence (--sweep cadence: LMMHIP_COMPACT_EVERY,
LMMHIP_COMPACT_PCT, LMMHIP_CLIST_EVERY) runs `--reps` device solves (inputs resident in HBM) and
prints the median HIP-event time.
usage: python scripts/tune_round.py [--cnst N] [--vars N] [--reps R] [--sweep widths|cadence]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simgrid_amd import lmm as L  # noqa: E402

KNOBS = ("LMMHIP_UPD_BLOCKS", "LMMHIP_READY_BLOCKS", "LMMHIP_SAT_BLOCKS", "LMMHIP_COMPACT_EVERY",
         "LMMHIP_COMPACT_PCT", "LMMHIP_CLIST_EVERY")
DEFAULT = (0, 0, 0, 32, 75, 8)
WIDTHS = [(0, 0, 0), (1024, 0, 0), (512, 0, 0), (0, 0, 1024), (0, 0, 512), (0, 1024, 0), (0, 512, 0),
          (1024, 1024, 1024), (512, 512, 512), (0, 0, 256)]
CADENCE = [(16, 75, 8), (32, 75, 8), (16, 50, 8), (32, 50, 8), (8, 75, 8), (24, 60, 8), (16, 75, 16),
           (16, 75, 4), (12, 85, 8)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cnst", type=int, default=1000000)
    ap.add_argument("--vars", type=int, default=10000000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--sweep", choices=("widths", "cadence"), default="widths")
    a = ap.parse_args()
    configs = [w + DEFAULT[3:] for w in WIDTHS] if a.sweep == "widths" else [DEFAULT[:3] + c for c in CADENCE]
    s = L.System(False)
    vs = s.gen_synthetic(a.cnst, a.vars, k=8, seed=1)
    s.prepare()
    s.device_solve()
    ref = None
    for cfg in configs:
        for k, v in zip(KNOBS, cfg):
            os.environ[k] = str(v)
        t = []
        for _ in range(a.reps):
            s.device_solve()
            t.append(s.last_stats()["device_ms"])
        s.fetch()
        x = s.values_of(vs)
        if ref is None:
            ref = x
        ok = bool(np.all(np.abs(x - ref) <= np.maximum(1e-9, 1e-6 * np.abs(ref))))
        print(json.dumps(dict(zip(KNOBS, cfg), ms=round(float(np.median(t)), 3),
                              min_ms=round(min(t), 3), rounds=s.last_stats()["rounds"], values_ok=ok)), flush=True)


if __name__ == "__main__":
    main()
