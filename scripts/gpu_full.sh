#!/bin/bash
# Full GPU verification (through gpurun): every -m gpu test, smoke(), then the default bench line (C2).
# Each step under its own limit; stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -n 3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then echo "STOP pytest rc=$rc"; grep -E "FAIL|Error" gpurun_out/pytest_gpu.log | head -20; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
cat gpurun_out/smoke.log; if [ $rc -ne 0 ]; then echo "STOP smoke rc=$rc"; exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.log; rc=$?
cat gpurun_out/bench_default.json; if [ $rc -ne 0 ]; then echo "STOP bench rc=$rc"; tail -20 gpurun_out/bench_default.log; exit $rc; fi
