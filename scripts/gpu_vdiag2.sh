#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
LMMHIP_VOTE_DIAG=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --dropin-steps 0 \
  --profile-json gpurun_out/prof_c2_vdiag.json > gpurun_out/bench_c2_vdiag.json 2> gpurun_out/bench_c2_vdiag.log || { echo "vdiag rc=$?"; exit 1; }
python - <<'PY'
import json, numpy as np
d = json.load(open("gpurun_out/prof_c2_vdiag.json"))
sl = np.array(d["launch_slot"]); rd = np.array(d["launch_round"]); ms = np.array(d["launch_ms"])
bm = (sl == 7) & (rd >= 1000000); fo = (sl == 7) & (rd < 1000000)
print({k: (v["launches"], round(v["total_ms"], 2), round(v["avg_us"], 1)) for k, v in d["per_kernel"].items()})
print("bitmap-only avg us", 1000 * ms[bm].mean(), "filter-only avg us", 1000 * ms[fo].mean())
for r in [1, 2, 5, 10, 50, 100, 150, 190, 210]:
    print(r, "bm %.1f filt %.1f vote %.1f" % (1000 * ms[bm & (rd == r + 1000000)].sum(), 1000 * ms[fo & (rd == r)].sum(),
                                            1000 * ms[(sl == 2) & (rd == r)].sum()))
PY
