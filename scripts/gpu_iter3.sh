#!/bin/bash
# Parity suite (engines, parity, configs) then the C2 stress and plain lines.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_engines.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_platforms.py tests/test_gpu_resident.py \
  -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_iter.log
if [ $rc -ne 0 ]; then echo "STOP pytest rc=$rc"; tail -30 gpurun_out/pytest_iter.log; exit $rc; fi
tail -2 gpurun_out/pytest_iter.log
bash scripts/gpu_stress.sh || exit 1
bash scripts/gpu_perf.sh || exit 1
