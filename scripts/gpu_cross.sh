#!/bin/bash
# Resident refresh path across part-test crossings: resident + parity tests first, then every -m gpu test,
# then the default bench line (drop-in steps included) with the crossing check on and off.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_parity.py -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/pytest_cross.log 2>&1; rc=$?
tail -n 3 gpurun_out/pytest_cross.log
if [ $rc -ne 0 ]; then echo "STOP pytest rc=$rc"; grep -E "FAILED|Error|error" gpurun_out/pytest_cross.log | head -20; tail -n 40 gpurun_out/pytest_cross.log; exit $rc; fi
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  --deselect tests/test_gpu_parity.py::test_synthetic_full_size_vs_oracle_sample \
  > gpurun_out/pytest_gpu_all.log 2>&1; rc=$?
tail -n 3 gpurun_out/pytest_gpu_all.log
if [ $rc -ne 0 ]; then echo "STOP pytest-all rc=$rc"; grep -E "FAILED|Error|error" gpurun_out/pytest_gpu_all.log | head -20; tail -n 40 gpurun_out/pytest_gpu_all.log; exit $rc; fi
line() {
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 400 python bench.py "$@" --steps 5 --warmup 1 --no-cpu-baseline \
    > gpurun_out/x_$tag.json 2> gpurun_out/x_$tag.log; local rc=$?
  if [ $rc -ne 0 ]; then echo "STOP $tag rc=$rc"; tail -n 20 gpurun_out/x_$tag.log; exit $rc; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/x_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'], json.dumps(d['config'].get('dropin_step')))"
}
line dropin_cross LMMHIP_RES_CROSS=1 --
line dropin_nocross LMMHIP_RES_CROSS=0 --
echo done
