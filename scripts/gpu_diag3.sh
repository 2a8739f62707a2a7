#!/bin/bash
mkdir -p gpurun_out
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 600 $PT tests/test_gpu_configs.py -k "c5_1e6 or oracle_solution" tests/test_gpu_parity.py -k "fair or c5" > gpurun_out/pytest_fb.log 2>&1; echo "fb rc=$?" >> gpurun_out/pytest_fb.log
timeout -k 10 200 python -u scripts/diag_r2.py c4 > gpurun_out/diag_c4.log 2>&1 || { echo "c4 rc=$?"; exit 1; }
timeout -k 10 300 python -u scripts/diag_r2.py c2 > gpurun_out/diag_c2.log 2>&1 || { echo "c2 rc=$?"; exit 1; }
