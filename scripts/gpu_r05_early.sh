#!/bin/bash
# Round 5: the drop-in solve's early value snapshot (System::solve_and_fetch, lmmhip_res_early_*; removed after
# this measurement, DESIGN.md §6 "Round 5"): the resident
# tests (bit identity with the sliced fetch), then the C2 drop-in step A/B on one box over the trigger share.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_resident.py -k early -x -v -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/early_tests.log 2>&1; rc=$?
tail -n 8 gpurun_out/early_tests.log
if [ $rc -ne 0 ]; then echo "STOP tests rc=$rc"; exit $rc; fi
line() {  # line <tag> <env...> -- <bench args>
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py "$@" --steps 3 --warmup 1 --no-cpu-baseline --dropin-steps 6 \
    > gpurun_out/early_$tag.json 2> gpurun_out/early_$tag.log; local rc=$?
  if [ $rc -ne 0 ]; then echo "STOP $tag rc=$rc"; tail -n 20 gpurun_out/early_$tag.log; exit $rc; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/early_$tag.json').read().strip().splitlines()[-1]); x=d['config']['dropin_step']; print('$tag', d['ms_per_step'], x['solve_step_ms'], x['value_scatter_ms'], x['device_solve_ms'])"
}
for pass in a b; do
line off_$pass LMM_EARLY_FETCH=0 --
line f10_$pass LMM_EARLY_FRAC=0.10 --
line f20_$pass LMM_EARLY_FRAC=0.20 --
line f30_$pass LMM_EARLY_FRAC=0.30 --
done
echo done
