#!/bin/bash
# Round 5: the vote filter's packed words (LMMHIP_PKF, removed after this measurement: DESIGN.md §6 "Round 5"): bit identity, then the C2 / C2-stress A/B on one box.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_engines.py -k "target_ordered" -x -v -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/pkf_tests.log 2>&1; rc=$?
tail -n 6 gpurun_out/pkf_tests.log
if [ $rc -ne 0 ]; then echo "STOP tests rc=$rc"; exit $rc; fi
line() {  # line <tag> <env...> -- <bench args>
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py "$@" --steps 10 --warmup 2 --no-cpu-baseline --dropin-steps 0 \
    > gpurun_out/pkf_$tag.json 2> gpurun_out/pkf_$tag.log; local rc=$?
  if [ $rc -ne 0 ]; then echo "STOP $tag rc=$rc"; tail -n 20 gpurun_out/pkf_$tag.log; exit $rc; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/pkf_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'])"
}
for pass in a b; do
line c2_base_$pass LMMHIP_PKF=0 --
line c2_pkf2_$pass LMMHIP_PKF=2 --
done
line st_base LMMHIP_PKF=0 -- --variant stress
line st_pkf2 LMMHIP_PKF=2 -- --variant stress
echo done
