#!/bin/bash
# Round-2 GPU session: the engine / determinism tests first, then the parity suite (optionally filtered),
# then short benches of C2 and C4 on both engines.  Stops at the first GPU fault / abort / timeout.
# usage: scripts/gpu_r2.sh [pytest -k expression]
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 600 $PT tests/test_gpu_engines.py > gpurun_out/pytest_engines.log 2>&1
rc=$?; echo "engines rc=$rc" >> gpurun_out/pytest_engines.log
if [ $rc -ne 0 ]; then echo "STOP after engine tests rc=$rc"; exit $rc; fi
timeout -k 10 900 $PT tests -m gpu ${1:+-k "$1"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if fatal $rc; then echo "STOP after pytest rc=$rc"; exit $rc; fi
for eng in persistent rounds; do
  LMMHIP_ENGINE=$eng timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline \
    > gpurun_out/bench_c2_$eng.json 2> gpurun_out/bench_c2_$eng.log
  rc=$?; echo "bench c2 $eng rc=$rc" >> gpurun_out/bench_c2_$eng.log
  if [ $rc -ne 0 ]; then echo "STOP after bench c2 $eng rc=$rc"; exit $rc; fi
  LMMHIP_ENGINE=$eng timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline \
    > gpurun_out/bench_c4_$eng.json 2> gpurun_out/bench_c4_$eng.log
  rc=$?; echo "bench c4 $eng rc=$rc" >> gpurun_out/bench_c4_$eng.log
  if [ $rc -ne 0 ]; then echo "STOP after bench c4 $eng rc=$rc"; exit $rc; fi
done
timeout -k 10 200 python -u scripts/diag_r2.py c4 > gpurun_out/diag_c4.log 2>&1 || { echo "diag c4 rc=$?"; exit 1; }
timeout -k 10 300 python -u scripts/diag_r2.py c2 > gpurun_out/diag_c2.log 2>&1 || { echo "diag c2 rc=$?"; exit 1; }
exit 0
