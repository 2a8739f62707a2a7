#!/bin/bash
# Round 6, last build: the frontier kernels without the removed variants' template paths (persistent-frontier
# relaxed accesses, LMMHIP_FR_SATOLD, LMMHIP_FR_MFEARLY).  Frontier / engine / C4 tests and two C4 lines on it, then
# the counter passes of scripts/gpu_r06_final.sh 3 (FETCH / WRITE of C3-C5, request counts of C2 / C4 / C5).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_engines.py tests/test_gpu_configs.py -k "frontier or c4 or engine" \
  -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06_tests_q.log 2>&1 \
  || { tail -30 gpurun_out/r06_tests_q.log; exit 1; }
tail -n 2 gpurun_out/r06_tests_q.log
for pass in 1 2; do
  timeout -k 10 200 python bench.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/abq_c4_$pass.out \
    2> gpurun_out/abq_c4_$pass.log || { echo "STOP c4 $pass"; tail -20 gpurun_out/abq_c4_$pass.log; exit 1; }
  tail -c 150 gpurun_out/abq_c4_$pass.out; echo
done
scripts/gpu_r06_final.sh 3
