#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 600 $PT tests/test_gpu_configs.py -k c3 tests/test_gpu_engines.py -k "c3 or batch" > gpurun_out/pytest_c3.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_c3.log
if [ $rc -ne 0 ]; then echo "STOP pytest rc=$rc"; tail -20 gpurun_out/pytest_c3.log; exit $rc; fi
timeout -k 10 300 python bench.py --workload c3 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.log || { echo "c3 bench failed"; exit 1; }
python -c "import json; print('c3', json.load(open('gpurun_out/bench_c3.json'))['ms_per_step'])"
tail -2 gpurun_out/pytest_c3.log
