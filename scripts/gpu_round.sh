#!/bin/bash
# Round-end evidence on the GPU box: parity suite, smoke, default C2 bench line (with the CPU
# baseline), the other §8(d) configs, then the rocprofv3 trace + PMC passes.  Every GPU step has its
# own limit and the script stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then echo "STOP pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log; exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc" >> gpurun_out/smoke.log
if [ $rc -ne 0 ]; then echo "STOP smoke rc=$rc"; tail -30 gpurun_out/smoke.log; exit $rc; fi
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.log; rc=$?
echo "bench rc=$rc" >> gpurun_out/bench_default.log
if [ $rc -ne 0 ]; then echo "STOP bench rc=$rc"; tail -20 gpurun_out/bench_default.log; exit $rc; fi
cat gpurun_out/bench_default.json
bash scripts/gpu_configs.sh || exit $?
# rocprofv3 evidence: scripts/profile.sh (its own gpurun call)
