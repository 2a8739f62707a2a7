#!/bin/bash
# Round 5: the batch (LDS) kernel's loads in flight (LMMHIP_BATCH_V, removed after this measurement): the C3 tests per variant, then the C3 A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in 1 2; do
  LMMHIP_BATCH_V=$v timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -k "c3" -x -v -p no:cacheprovider \
    --timeout 200 --timeout-method thread > gpurun_out/bv_tests_$v.log 2>&1; rc=$?
  tail -n 3 gpurun_out/bv_tests_$v.log
  if [ $rc -ne 0 ]; then echo "STOP tests $v rc=$rc"; exit $rc; fi
done
line() {  # line <tag> <env...> -- <bench args>
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py "$@" --steps 50 --warmup 5 --no-cpu-baseline \
    > gpurun_out/bv_$tag.json 2> gpurun_out/bv_$tag.log; local rc=$?
  if [ $rc -ne 0 ]; then echo "STOP $tag rc=$rc"; tail -n 20 gpurun_out/bv_$tag.log; exit $rc; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/bv_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'])"
}
for pass in a b; do
line v0_$pass LMMHIP_BATCH_V=0 -- --workload c3
line v1_$pass LMMHIP_BATCH_V=1 -- --workload c3
line v2_$pass LMMHIP_BATCH_V=2 -- --workload c3
done
echo done
