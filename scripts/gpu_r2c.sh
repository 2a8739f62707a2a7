#!/bin/bash
# Round-2 checkpoint on the GPU box: full parity suite, then the C2 line (with per-launch profile) and the
# C3/C4/C5 lines.  Every GPU step has its own limit; the script stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then echo "STOP pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log; exit $rc; fi
timeout -k 10 400 python bench.py --profile-json gpurun_out/prof_c2.json > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.log; rc=$?
echo "c2 rc=$rc" >> gpurun_out/bench_c2.log
if [ $rc -ne 0 ]; then echo "STOP c2 rc=$rc"; tail -20 gpurun_out/bench_c2.log; exit $rc; fi
cat gpurun_out/bench_c2.json
for w in c3 c4 c5; do
  timeout -k 10 400 python bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.log
  rc=$?; echo "$w rc=$rc" >> gpurun_out/bench_$w.log
  if [ $rc -ne 0 ]; then echo "STOP $w rc=$rc"; tail -20 gpurun_out/bench_$w.log; exit $rc; fi
  cat gpurun_out/bench_$w.json
done
