#!/bin/bash
# Round 5: the new GPU tests first (pingpong replay on the device, the persistent rendezvous deadline), then
# every -m gpu test.  Each step under its own limit; stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_engines.py -k "pingpong or rendezvous or tail_handoff or duplicate" -x -v \
  -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r05_new_tests.log 2>&1; rc=$?
tail -n 30 gpurun_out/r05_new_tests.log
if [ $rc -ne 0 ]; then echo "STOP new tests rc=$rc"; exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/r05_pytest_gpu.log 2>&1; rc=$?
tail -n 5 gpurun_out/r05_pytest_gpu.log
if [ $rc -ne 0 ]; then echo "STOP pytest rc=$rc"; tail -n 60 gpurun_out/r05_pytest_gpu.log; exit $rc; fi
echo done
