#!/bin/bash
# Round-2 profiling call: per-phase persistent-engine breakdown on C4, C2 per-launch profile, rocprofv3
# trace + PMC passes (scripts/profile.sh).  Each GPU step under its own limit; stop at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python scripts/diag_r2.py c4 > gpurun_out/diag_c4.log 2>&1 || { echo "STOP diag c4"; tail gpurun_out/diag_c4.log; exit 1; }
tail -2 gpurun_out/diag_c4.log
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --dropin-steps 0 --profile-json gpurun_out/prof_c2.json \
  > gpurun_out/bench_c2_prof.json 2> gpurun_out/bench_c2_prof.log || { echo "STOP c2 prof"; tail gpurun_out/bench_c2_prof.log; exit 1; }
bash scripts/profile.sh
