#!/bin/bash
# Round 5: resident tests (device flatten + sliced fetch == host path), then the drop-in C2 step with 1 / 32 / 64
# fetch slices (same box), then the request passes for the roofline.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_resident.py -x -v -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/r05_resident_tests.log 2>&1; rc=$?
tail -n 4 gpurun_out/r05_resident_tests.log
if [ $rc -ne 0 ]; then echo "STOP tests rc=$rc"; grep -E "^E |Error" gpurun_out/r05_resident_tests.log | head -30; exit $rc; fi
line() {  # line <tag> <env...> -- <bench args>
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py "$@" --steps 3 --warmup 1 --no-cpu-baseline --dropin-steps 5 \
    > gpurun_out/fx_$tag.json 2> gpurun_out/fx_$tag.log; local rc=$?
  if [ $rc -ne 0 ]; then echo "STOP $tag rc=$rc"; tail -n 20 gpurun_out/fx_$tag.log; exit $rc; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/fx_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'], d['config']['dropin_step'])"
}
line s1 LMM_FETCH_SLICES=1 --
line s32 LMM_FETCH_SLICES=32 --
line s8 LMM_FETCH_SLICES=8 --
line s64 LMM_FETCH_SLICES=64 --
PARTS="trace req" scripts/profile.sh || exit $?
echo done
