#!/bin/bash
# Round 5: C5 with shorter shared constraints streaming fbk_acc's increments (LMMHIP_FB_STREAM), bit-identity first.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py -k "c5_1e6_flows" -x -v -p no:cacheprovider \
  --timeout 600 --timeout-method thread > gpurun_out/r05_c5_tests.log 2>&1; rc=$?
tail -n 3 gpurun_out/r05_c5_tests.log
if [ $rc -ne 0 ]; then echo "STOP tests rc=$rc"; grep -E "^E |Error" gpurun_out/r05_c5_tests.log | head -30; exit $rc; fi
line() {  # line <tag> <env...> -- <bench args>
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py --workload c5 "$@" --steps 10 --warmup 2 --no-cpu-baseline \
    > gpurun_out/c5st_$tag.json 2> gpurun_out/c5st_$tag.log; local rc=$?
  if [ $rc -ne 0 ]; then echo "STOP $tag rc=$rc"; tail -n 20 gpurun_out/c5st_$tag.log; exit $rc; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/c5st_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'])"
}
for pass in a b; do
line base_$pass LMMHIP_FB_ENV=0 --
line s4096_$pass LMMHIP_FB_STREAM=4096 --
line s1024_$pass LMMHIP_FB_STREAM=1024 --
line s256_$pass LMMHIP_FB_STREAM=256 --
line s64_$pass LMMHIP_FB_STREAM=64 --
done
echo done
