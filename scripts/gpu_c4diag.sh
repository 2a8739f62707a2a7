#!/bin/bash
# C4 diagnostics: persistent-engine barrier timestamps and the per-launch profile of the round engine.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/diag_r2.py c4 > gpurun_out/diag_c4.log 2>&1 || { echo "c4 rc=$?"; exit 1; }
timeout -k 10 200 python bench.py --workload c4 --steps 5 --warmup 1 --no-cpu-baseline --profile-json gpurun_out/prof_c4.json \
  > gpurun_out/bench_c4p.json 2> gpurun_out/bench_c4p.log || { echo "c4p rc=$?"; exit 1; }
