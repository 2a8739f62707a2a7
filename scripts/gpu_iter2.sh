#!/bin/bash
# Iteration check on the GPU box: engines + parity + full-size configs, then C2 (profiled) and C4 lines.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_engines.py tests/test_gpu_parity.py tests/test_gpu_configs.py \
  -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_iter.log
if [ $rc -ne 0 ]; then echo "STOP pytest rc=$rc"; tail -30 gpurun_out/pytest_iter.log; exit $rc; fi
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --dropin-steps 0 --profile-json gpurun_out/prof_c2.json \
  > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.log || { echo "c2 rc=$?"; tail -5 gpurun_out/bench_c2.log; exit 1; }
cat gpurun_out/bench_c2.json
timeout -k 10 200 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.log || { echo "c4 rc=$?"; exit 1; }
cat gpurun_out/bench_c4.json
timeout -k 10 200 python -u scripts/diag_r2.py c4 > gpurun_out/diag_c4.log 2>&1 || { echo "c4diag rc=$?"; exit 1; }
