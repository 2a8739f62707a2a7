#!/bin/bash
# Round 5: resident tests (refresh path with the touched-variable list), then the drop-in C2 step with and without
# the list (same box), then the C4 frontier knobs.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_step.py -x -v -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/r05_resident_tests.log 2>&1; rc=$?
tail -n 3 gpurun_out/r05_resident_tests.log
if [ $rc -ne 0 ]; then echo "STOP tests rc=$rc"; grep -E "^E |Error" gpurun_out/r05_resident_tests.log | head -30; exit $rc; fi
line() {  # line <tag> <env...> -- <bench args>
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py "$@" --steps 3 --warmup 1 --no-cpu-baseline --dropin-steps 5 \
    > gpurun_out/rf_$tag.json 2> gpurun_out/rf_$tag.log; local rc=$?
  if [ $rc -ne 0 ]; then echo "STOP $tag rc=$rc"; tail -n 20 gpurun_out/rf_$tag.log; exit $rc; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/rf_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'], d['config']['dropin_step'])"
}
line vl1 LMMHIP_RES_VLIST=1 --
line vl0 LMMHIP_RES_VLIST=0 --
line vl1b LMMHIP_RES_VLIST=1 --
scripts/gpu_r05_c4.sh || exit $?
echo done
