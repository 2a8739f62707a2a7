#!/bin/bash
# Round 5, final code: the C4 / C5 kernel traces and bench lines again (the frontier and FairBottleneck sources
# changed after the first r05 evidence pass), then the persistent-frontier and LPT bit-identity tests.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
PARTS="c4 c5" scripts/profile.sh || exit $?
for w in c4 c5; do
  timeout -k 10 400 python bench.py --workload $w --steps 10 --warmup 2 > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.log
  rc=$?; if [ $rc -ne 0 ]; then echo "STOP $w rc=$rc"; tail -20 gpurun_out/bench_$w.log; exit $rc; fi
  tail -1 gpurun_out/bench_$w.json | cut -c1-200
done
timeout -k 10 500 python -u -m pytest tests/test_gpu_engines.py tests/test_gpu_configs.py -k "frontier or c4 or c5_1e6" -x -q \
  -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/final_tests.log 2>&1; rc=$?
tail -n 3 gpurun_out/final_tests.log
exit $rc
