#!/bin/bash
# One GPU-box session: parity tests, smoke, bench.  Stops at the first GPU fault / abort / timeout.
# usage: scripts/gpu_check.sh [pytest-args...]
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider "$@" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if fatal $rc; then echo "STOP after pytest rc=$rc"; exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.build(); g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> gpurun_out/smoke.log
if fatal $rc; then echo "STOP after smoke rc=$rc"; exit $rc; fi
timeout -k 10 300 python bench.py --cnst 100000 --vars 1000000 --steps 3 --warmup 1 --no-cpu-baseline \
  --profile-json gpurun_out/prof_small.json > gpurun_out/bench_small.json 2> gpurun_out/bench_small.log
rc=$?; echo "bench_small rc=$rc" >> gpurun_out/bench_small.log
if [ $rc -ne 0 ]; then echo "STOP after bench_small rc=$rc"; exit $rc; fi
timeout -k 10 600 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --profile-json gpurun_out/prof_full.json \
  > gpurun_out/bench_full.json 2> gpurun_out/bench_full.log
rc=$?; echo "bench_full rc=$rc" >> gpurun_out/bench_full.log
exit $rc
