#!/bin/bash
mkdir -p gpurun_out
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 600 $PT tests/test_gpu_engines.py > gpurun_out/pytest_engines.log 2>&1 || { echo "engines failed"; exit 1; }
timeout -k 10 200 python -u scripts/diag_r2.py c4 > gpurun_out/diag_c4.log 2>&1 || { echo "c4 rc=$?"; exit 1; }
timeout -k 10 300 python -u scripts/diag_r2.py c2 > gpurun_out/diag_c2.log 2>&1 || { echo "c2 rc=$?"; exit 1; }
cp gpurun_out/persist_c2.json gpurun_out/persist_c2_agent.json; cp gpurun_out/persist_c4.json gpurun_out/persist_c4_agent.json
LMMHIP_PERSIST_SYSFENCE=1 timeout -k 10 200 python -u scripts/diag_r2.py c4 > gpurun_out/diag_c4s.log 2>&1 || { echo "c4s rc=$?"; exit 1; }
LMMHIP_PERSIST_SYSFENCE=1 timeout -k 10 300 python -u scripts/diag_r2.py c2 > gpurun_out/diag_c2s.log 2>&1 || { echo "c2s rc=$?"; exit 1; }
