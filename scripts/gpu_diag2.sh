#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/diag_r2.py c5rounds 1000000 > gpurun_out/diag_c5r.log 2>&1 || { echo "c5r rc=$?"; exit 1; }
timeout -k 10 200 python -u scripts/diag_r2.py c4 > gpurun_out/diag_c4.log 2>&1 || { echo "c4 rc=$?"; exit 1; }
timeout -k 10 300 python -u scripts/diag_r2.py c2 > gpurun_out/diag_c2.log 2>&1 || { echo "c2 rc=$?"; exit 1; }
