#!/bin/bash
# Round 5: C4 frontier knobs (big-constraint chunk threshold / waves), same box, after the frontier bit-identity tests.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
LMMHIP_FR_BIGCH=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_engines.py -k "frontier" -x -v -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/r05_c4_tests.log 2>&1; rc=$?
tail -n 3 gpurun_out/r05_c4_tests.log
if [ $rc -ne 0 ]; then echo "STOP tests rc=$rc"; grep -E "^E |Error" gpurun_out/r05_c4_tests.log | head -30; exit $rc; fi
line() {  # line <tag> <env...> -- <bench args>
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py --workload c4 "$@" --steps 20 --warmup 3 --no-cpu-baseline \
    > gpurun_out/c4ab_$tag.json 2> gpurun_out/c4ab_$tag.log; local rc=$?
  if [ $rc -ne 0 ]; then echo "STOP $tag rc=$rc"; tail -n 20 gpurun_out/c4ab_$tag.log; exit $rc; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/c4ab_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'])"
}
for pass in a b; do
line base_$pass LMMHIP_FR_BIGCH=16 --
line ch8_$pass LMMHIP_FR_BIGCH=8 --
line ch4_$pass LMMHIP_FR_BIGCH=4 --
line ch2_$pass LMMHIP_FR_BIGCH=2 --
line ch4w8_$pass LMMHIP_FR_BIGCH=4 LMMHIP_FR_BIGW=8 --
line ch4w32_$pass LMMHIP_FR_BIGCH=4 LMMHIP_FR_BIGW=32 --
done
echo done
