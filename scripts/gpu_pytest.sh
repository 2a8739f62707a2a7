#!/bin/bash
# One GPU-box pytest session (run through gpurun): the given pytest selection, each test under a
# thread timeout, log in gpurun_out/pytest_sel.log.  usage: scripts/gpu_pytest.sh <pytest args...>
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread "$@" \
  > gpurun_out/pytest_sel.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_sel.log
tail -5 gpurun_out/pytest_sel.log
exit $rc
