#!/bin/bash
# One optimisation iteration on the GPU box: parity suite, then the C2 bench with the per-launch
# profile.  Stops at the first GPU fault / abort / timeout.  usage: scripts/gpu_iter.sh [pytest -k expr]
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
K="${1:-}"
timeout -k 10 700 python -m pytest tests -m gpu -x -q -p no:cacheprovider ${K:+-k "$K"} > gpurun_out/pytest_iter.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_iter.log
if [ $rc -ne 0 ]; then echo "STOP pytest rc=$rc"; tail -30 gpurun_out/pytest_iter.log; exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --profile-json gpurun_out/prof_c2.json \
  > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.log; rc=$?
echo "bench rc=$rc" >> gpurun_out/bench_c2.log
if fatal $rc; then echo "STOP bench rc=$rc"; exit $rc; fi
cat gpurun_out/bench_c2.json
exit $rc
