#!/bin/bash
# Round engine with / without the saturation's row retirement: engine bit-identity tests, C2 lines, C2 stress.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_engines.py tests/test_gpu_parity.py -x -q -p no:cacheprovider \
  -k "not full_size" --timeout 200 --timeout-method thread > gpurun_out/rt_pytest.log 2>&1; rc=$?
tail -n 1 gpurun_out/rt_pytest.log
if [ $rc -ne 0 ]; then echo "STOP pytest rc=$rc"; tail -n 40 gpurun_out/rt_pytest.log; exit $rc; fi
line() {
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py "$@" --steps 5 --warmup 1 --no-cpu-baseline --dropin-steps 0 \
    > gpurun_out/rt_$tag.json 2> gpurun_out/rt_$tag.log; local rc=$?
  if [ $rc -ne 0 ]; then echo "STOP $tag rc=$rc"; tail -n 20 gpurun_out/rt_$tag.log; exit $rc; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/rt_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'])"
}
line c2_retire LMMHIP_RETIRE=1 --
line c2_noretire LMMHIP_RETIRE=0 --
line c2_retire_b LMMHIP_RETIRE=1 --
line c2_noretire_b LMMHIP_RETIRE=0 --
line c2s_retire LMMHIP_RETIRE=1 -- --variant stress
line c2s_noretire LMMHIP_RETIRE=0 -- --variant stress
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --dropin-steps 0 \
  --profile-json gpurun_out/rt_c2prof.json > /dev/null 2> gpurun_out/rt_c2prof.log || { echo "STOP prof"; exit 1; }
echo done
