#!/bin/bash
# Round 6, last change (64-round chunks under the round hint, round engine): engine bit-identity tests (all engines,
# the wrong-hint test), the full-size C2 plain / stress samples against the oracle, smoke, the default bench line.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_engines.py "tests/test_gpu_parity.py::test_synthetic_full_size_vs_oracle_sample" \
  -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06_tests_x.log 2>&1 \
  || { tail -30 gpurun_out/r06_tests_x.log; exit 1; }
tail -n 2 gpurun_out/r06_tests_x.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -n 1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.log \
  || { tail -20 gpurun_out/bench_default.log; exit 1; }
tail -c 300 gpurun_out/bench_default.json
