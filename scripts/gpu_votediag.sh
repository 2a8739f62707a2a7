#!/bin/bash
# Vote-phase diagnostics on C2: per-round filter-only / bitmap-only launches (LMMHIP_VOTE_DIAG), and the
# persistent engine's barrier profile on C2.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
LMMHIP_VOTE_DIAG=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --dropin-steps 0 \
  --profile-json gpurun_out/prof_c2_vdiag.json > gpurun_out/bench_c2_vdiag.json 2> gpurun_out/bench_c2_vdiag.log || { echo "vdiag rc=$?"; exit 1; }
LMMHIP_ENGINE=persistent timeout -k 10 300 python -u scripts/diag_r2.py c2 > gpurun_out/diag_c2.log 2>&1 || { echo "c2 rc=$?"; exit 1; }
