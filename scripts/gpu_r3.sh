#!/bin/bash
# Round-3 iteration call (gpurun): selected GPU tests, then bench lines of the given workloads, then (DIAG=1)
# the C4 bench under rocprofv3 with the native crash backtrace (scripts/segv_trace.c).  Each step under its
# own limit; stops at the first failure.  usage: TESTS="..." WL="c5 c4" DIAG=1 scripts/gpu_r3.sh
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_r3.log 2>&1; rc=$?
  tail -n 3 gpurun_out/pytest_r3.log
  if [ $rc -ne 0 ]; then echo "STOP pytest rc=$rc"; grep -E "FAIL|Error" gpurun_out/pytest_r3.log | head -20; exit $rc; fi
fi
for w in $WL; do
  timeout -k 10 400 python bench.py --workload $w --steps 10 --warmup 2 ${BENCH_ARGS:---no-cpu-baseline} \
    > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.log; rc=$?
  if [ $rc -ne 0 ]; then echo "STOP $w rc=$rc"; tail -n 20 gpurun_out/bench_$w.log; exit $rc; fi
  cat gpurun_out/bench_$w.json
done
if [ -n "$DIAG" ]; then
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
  LMM_SEGV_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rp_trace_c4 \
    -o run -- python3 bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/rp_trace_c4.log 2>&1
  rc=$?; echo "trace c4 rc=$rc" >> gpurun_out/rp_trace_c4.log; tail -n 40 gpurun_out/rp_trace_c4.log
  exit $rc
fi
