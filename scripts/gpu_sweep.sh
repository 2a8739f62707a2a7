#!/bin/bash
# Generic C2 knob sweep: SWEEP_VAR=<env name> SWEEP="v1 v2 ..." (one bench line + per-kernel averages each).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in $SWEEP; do
  env $SWEEP_VAR=$v timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --dropin-steps 0 \
    --profile-json gpurun_out/prof_sw_$v.json > gpurun_out/bench_sw_$v.json 2> gpurun_out/bench_sw_$v.log || { echo "$v rc=$?"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/prof_sw_$v.json'));print('$SWEEP_VAR=$v', json.load(open('gpurun_out/bench_sw_$v.json'))['ms_per_step'], {k:round(v['avg_us'],1) for k,v in d['per_kernel'].items()})"
done
