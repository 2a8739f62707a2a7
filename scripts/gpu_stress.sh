#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --variant stress --steps 5 --warmup 1 --no-cpu-baseline --dropin-steps 0 \
  --profile-json gpurun_out/prof_c2s.json > gpurun_out/bench_c2s.json 2> gpurun_out/bench_c2s.log || { echo "rc=$?"; exit 1; }
python - <<'PY'
import json, numpy as np
d = json.load(open("gpurun_out/prof_c2s.json"))
print(json.load(open("gpurun_out/bench_c2s.json"))["ms_per_step"], d["rounds"])
print({k: (v["launches"], round(v["total_ms"], 2), round(v["avg_us"], 1)) for k, v in d["per_kernel"].items()})
sl = np.array(d["launch_slot"]); rd = np.array(d["launch_round"]); ms = np.array(d["launch_ms"])
av = np.array(d["alive_vars"]); rv = np.array(d["reeval_vars"])
for r in [0, 1, 2, 5, 10, 50, 100, 150, 190, 210]:
    if r < len(av):
        print(r, av[r], rv[r], " ".join("%d:%.1f" % (k, 1000 * ms[(sl == k) & (rd == r)].sum()) for k in (2, 3, 4, 5, 6)))
PY
