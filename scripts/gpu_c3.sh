#!/bin/bash
mkdir -p gpurun_out
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 600 $PT tests/test_gpu_configs.py -k c3 > gpurun_out/pytest_c3.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_c3.log
case $rc in 124|134|137|139) echo "STOP rc=$rc"; exit $rc;; esac
timeout -k 10 300 python bench.py --workload c3 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.log || { echo "c3 bench failed"; exit 1; }
