#!/bin/bash
# Perf-only iteration (no parity suite): C2 profiled line, C4 line, optional extra command in $EXTRA.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --dropin-steps 0 --profile-json gpurun_out/prof_c2.json \
  > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.log || { echo "c2 rc=$?"; tail -5 gpurun_out/bench_c2.log; exit 1; }
timeout -k 10 200 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.log || { echo "c4 rc=$?"; exit 1; }
timeout -k 10 200 python bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.log || { echo "c3 rc=$?"; exit 1; }
python - <<'PY'
import json
for w in ("c2", "c4", "c3"):
    print(w, json.load(open(f"gpurun_out/bench_{w}.json"))["ms_per_step"])
d = json.load(open("gpurun_out/prof_c2.json"))
print({k: (v["launches"], round(v["total_ms"], 2), round(v["avg_us"], 1)) for k, v in d["per_kernel"].items()})
PY
