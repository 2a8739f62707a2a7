#!/bin/bash
# Round 5: FairBottleneck long chains longest first from a queue (LMMHIP_FB_LPT): C5 1e6 byte-equality with the
# oracle in every mode, then the C5 A/B (same box) over the mode and the long-chain workgroups.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -k "c5_1e6" -x -v -p no:cacheprovider --timeout 200 \
  --timeout-method thread > gpurun_out/lpt_tests.log 2>&1; rc=$?
tail -n 14 gpurun_out/lpt_tests.log
if [ $rc -ne 0 ]; then echo "STOP tests rc=$rc"; exit $rc; fi
line() {  # line <tag> <env...> -- <bench args>
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py "$@" --steps 10 --warmup 2 --no-cpu-baseline \
    > gpurun_out/lpt_$tag.json 2> gpurun_out/lpt_$tag.log; local rc=$?
  if [ $rc -ne 0 ]; then echo "STOP $tag rc=$rc"; tail -n 20 gpurun_out/lpt_$tag.log; exit $rc; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/lpt_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'])"
}
for pass in a b; do
line base_$pass LMMHIP_FB_LPT=0 -- --workload c5
line lpt_$pass LMMHIP_FB_LPT=1 -- --workload c5
line lpt256_$pass LMMHIP_FB_LPT=1 LMMHIP_FB_LONGWG=256 -- --workload c5
line lpt64_$pass LMMHIP_FB_LPT=1 LMMHIP_FB_LONGWG=64 -- --workload c5
line lpt_l8k_$pass LMMHIP_FB_LPT=1 LMMHIP_FB_LONG=8192 LMMHIP_FB_LONGWG=256 -- --workload c5
line lpt_l32k_$pass LMMHIP_FB_LPT=1 LMMHIP_FB_LONG=32768 -- --workload c5
done
echo done
