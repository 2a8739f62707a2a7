#!/bin/bash
# Round 5: the frontier engine's rounds in one persistent launch (LMMHIP_FR_PERSIST): bit identity first, then the
# C4 A/B (same box) against the multi-launch frontier, over the persistent grid size.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_engines.py -k "frontier_persistent or frontier_engine_bit" -x -v \
  -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/frp_tests.log 2>&1; rc=$?
tail -n 25 gpurun_out/frp_tests.log
if [ $rc -ne 0 ]; then echo "STOP tests rc=$rc"; exit $rc; fi
line() {  # line <tag> <env...> -- <bench args>
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py "$@" --steps 20 --warmup 2 --no-cpu-baseline \
    > gpurun_out/frp_$tag.json 2> gpurun_out/frp_$tag.log; local rc=$?
  if [ $rc -ne 0 ]; then echo "STOP $tag rc=$rc"; tail -n 20 gpurun_out/frp_$tag.log; exit $rc; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/frp_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'])"
}
for pass in a b; do
line c4_base_$pass LMMHIP_FR_PERSIST=0 -- --workload c4
line c4_frp_$pass LMMHIP_FR_PERSIST=1 -- --workload c4
line c4_frp64_$pass LMMHIP_FR_PERSIST=1 LMMHIP_FRP_GRID=64 -- --workload c4
line c4_frp32_$pass LMMHIP_FR_PERSIST=1 LMMHIP_FRP_GRID=32 -- --workload c4
line c4_frp128_$pass LMMHIP_FR_PERSIST=1 LMMHIP_FRP_GRID=128 -- --workload c4
done
echo done
