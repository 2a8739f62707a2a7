#!/bin/bash
# Round 5: the new tests (pingpong replay on the device, persistent rendezvous deadline, tail hand-off
# bit-identity, frontier duplicates), then C2 with the tail hand-off at several thresholds (same box).
# Each step under its own limit; stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_engines.py \
  -k "pingpong or rendezvous or tail_handoff or duplicate" -x -v -p no:cacheprovider --timeout 120 \
  --timeout-method thread > gpurun_out/r05_new_tests.log 2>&1; rc=$?
tail -n 8 gpurun_out/r05_new_tests.log
if [ $rc -ne 0 ]; then echo "STOP new tests rc=$rc"; grep -E "^E |Error" gpurun_out/r05_new_tests.log | head -30; exit $rc; fi
line() {  # line <tag> <env...> -- <bench args>
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py "$@" --steps 10 --warmup 2 --no-cpu-baseline --dropin-steps 0 \
    > gpurun_out/tl_$tag.json 2> gpurun_out/tl_$tag.log; local rc=$?
  if [ $rc -ne 0 ]; then echo "STOP $tag rc=$rc"; tail -n 20 gpurun_out/tl_$tag.log; exit $rc; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/tl_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'])"
}
for pass in a b; do
line c2_off_$pass LMMHIP_TAIL_ROWS=0 --
line c2_2m_$pass LMMHIP_TAIL_ROWS=2000000 --
line c2_1m_$pass LMMHIP_TAIL_ROWS=1000000 --
line c2_500k_$pass LMMHIP_TAIL_ROWS=500000 --
line c2_250k_$pass LMMHIP_TAIL_ROWS=250000 --
done
line c2_3m LMMHIP_TAIL_ROWS=3000000 --
line c2_2m_fr LMMHIP_TAIL_ROWS=2000000 LMMHIP_TAIL_ENGINE=3 --
line c2_500k_fr LMMHIP_TAIL_ROWS=500000 LMMHIP_TAIL_ENGINE=3 --
echo done
