"""Collect the same-box A/B lines of round-5 GPU scripts (gpurun_out/<prefix>_<tag>.json: bench.py JSON lines) into
one profile summary: python scripts/collect_ab.py <out.json> <prefix> [<prefix> ...]"""
import glob
import json
import os
import sys


def main():
    out, prefixes = sys.argv[1], sys.argv[2:]
    res = {}
    for pre in prefixes:
        for p in sorted(glob.glob(os.path.join("gpurun_out", f"{pre}_*.json"))):
            try:
                d = json.loads(open(p).read().strip().splitlines()[-1])
            except (OSError, ValueError, IndexError):
                continue
            row = {"ms_per_step": d.get("ms_per_step"), "workload": d.get("config", {}).get("workload")}
            drop = d.get("config", {}).get("dropin_step")
            if drop:
                row["dropin_step"] = drop
            res[os.path.basename(p)[:-5]] = row
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    for k, v in res.items():
        print(k, v["ms_per_step"], (v.get("dropin_step") or {}).get("solve_step_ms", ""))


if __name__ == "__main__":
    main()
