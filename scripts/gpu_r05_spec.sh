#!/bin/bash
# Round 5: the frontier kernels' loads issued with the keys (LMMHIP_FR_SPEC, removed after this measurement): bit identity, then the C4 A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
LMMHIP_FR_SPEC=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_engines.py tests/test_gpu_configs.py \
  -k "frontier_engine_bit or c4" -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/spec_tests.log 2>&1; rc=$?
tail -n 4 gpurun_out/spec_tests.log
if [ $rc -ne 0 ]; then echo "STOP tests rc=$rc"; exit $rc; fi
line() {  # line <tag> <env...> -- <bench args>
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py "$@" --steps 20 --warmup 2 --no-cpu-baseline \
    > gpurun_out/spec_$tag.json 2> gpurun_out/spec_$tag.log; local rc=$?
  if [ $rc -ne 0 ]; then echo "STOP $tag rc=$rc"; tail -n 20 gpurun_out/spec_$tag.log; exit $rc; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/spec_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'])"
}
for pass in a b c; do
line c4_base_$pass LMMHIP_FR_SPEC=0 -- --workload c4
line c4_spec_$pass LMMHIP_FR_SPEC=1 -- --workload c4
done
echo done
