#!/bin/bash
# Every -m gpu test (one process), then C4 lines (frontier with 16-register re-votes, without, persistent).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_all.log 2>&1; rc=$?
tail -n 3 gpurun_out/pytest_gpu_all.log
if [ $rc -ne 0 ]; then echo "STOP pytest rc=$rc"; grep -E "FAILED|Error|error" gpurun_out/pytest_gpu_all.log | head -20; tail -n 30 gpurun_out/pytest_gpu_all.log; exit $rc; fi
line() {
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py "$@" --steps 10 --warmup 2 --no-cpu-baseline --dropin-steps 0 \
    > gpurun_out/t_$tag.json 2> gpurun_out/t_$tag.log; local rc=$?
  if [ $rc -ne 0 ]; then echo "STOP $tag rc=$rc"; tail -n 20 gpurun_out/t_$tag.log; exit $rc; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/t_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'])"
}
line c4_fr16 LMMHIP_ENGINE=frontier -- --workload c4
line c4_fr8 LMMHIP_ENGINE=frontier LMMHIP_FR_R16=0 -- --workload c4
line c4_persist LMMHIP_ENGINE=persistent -- --workload c4
echo done
