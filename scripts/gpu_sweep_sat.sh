#!/bin/bash
# Launch-width sweep of mm_sat_scan on C2 (LMMHIP_SAT_BLOCKS; 0 = grid_for(alive constraints)).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for sb in ${SWEEP:-0 1280 1024 512}; do
  LMMHIP_SAT_BLOCKS=$sb timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --dropin-steps 0 \
    --profile-json gpurun_out/prof_c2_sat$sb.json > gpurun_out/bench_c2_sat$sb.json 2> gpurun_out/bench_c2_sat$sb.log || { echo "sb=$sb rc=$?"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/prof_c2_sat$sb.json'));print($sb, json.load(open('gpurun_out/bench_c2_sat$sb.json'))['ms_per_step'], {k:round(v['avg_us'],1) for k,v in d['per_kernel'].items()})"
done
