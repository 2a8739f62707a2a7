"""Per-round regression of kernel launch times against the work profile (bench.py --profile-json)."""
import json
import sys

import numpy as np

d = json.load(open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_c2.json"))
slot = np.array(d["launch_slot"]); rnd = np.array(d["launch_round"]); ms = np.array(d["launch_ms"])
a = np.array(d["alive_vars"]); rv = np.array(d["reeval_vars"])
for sl, name in [(2, "vote"), (3, "ready"), (4, "sat"), (5, "upd"), (6, "compact/done")]:
    sel = (slot == sl) & (rnd >= 0) & (rnd < len(a))
    r = rnd[sel]; t = ms[sel] * 1000
    X = np.stack([np.ones(len(r)), a[r] / 1e6, rv[np.minimum(r, len(rv) - 1)] / 1e5], 1)
    if not len(t):
        continue
    coef, *_ = np.linalg.lstsq(X, t, rcond=None)
    print(f"{name:12s} us = {coef[0]:6.1f} + {coef[1]:6.2f}/M alive + {coef[2]:6.2f}/100k reeval   total {t.sum()/1000:.2f} ms"
          f"  (r0 {t[0]:.0f} us, n={len(t)})")
