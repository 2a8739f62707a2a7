#!/bin/bash
# batch kernel + engines + configs, then C3/C4 benches (quick)
mkdir -p gpurun_out
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 600 $PT tests/test_gpu_engines.py tests/test_gpu_configs.py > gpurun_out/pytest_r2b.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_r2b.log
case $rc in 124|134|137|139) echo "STOP rc=$rc"; exit $rc;; esac
timeout -k 10 300 python bench.py --workload c3 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.log || { echo "c3 bench failed"; exit 1; }
LMMHIP_BATCH=0 timeout -k 10 300 python bench.py --workload c3 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c3_global.json 2> gpurun_out/bench_c3_global.log || { echo "c3g bench failed"; exit 1; }
timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.log || { echo "c4 bench failed"; exit 1; }
