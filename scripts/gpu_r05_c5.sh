#!/bin/bash
# Round 5: C5 levers on the mu gathers (same box): the increments streamed from fbk_acc's per-element copy for
# every shared constraint (LMMHIP_FB_LONG=0) or the long ones only (default / 4096), the locality order off; then
# the FETCH_SIZE pass of the default and of FB_LONG=0.
cd "$GRAFT_REPO_ROOT" || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
line() {  # line <tag> <env...> -- <bench args>
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py --workload c5 "$@" --steps 10 --warmup 2 --no-cpu-baseline \
    > gpurun_out/c5ab_$tag.json 2> gpurun_out/c5ab_$tag.log; local rc=$?
  if [ $rc -ne 0 ]; then echo "STOP $tag rc=$rc"; tail -n 20 gpurun_out/c5ab_$tag.log; exit $rc; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/c5ab_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'])"
}
for pass in a b; do
line base_$pass LMMHIP_FB_ENV=0 --
line long0_$pass LMMHIP_FB_LONG=0 --
line long4k_$pass LMMHIP_FB_LONG=4096 --
done
for v in base long0; do
  if [ $v = long0 ]; then E="LMMHIP_FB_LONG=0"; else E="LMMHIP_FB_ENV=0"; fi
  env $E timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/c5pmc_$v -o run \
    -- python3 bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c5pmc_$v.log 2>&1 || { echo "STOP pmc $v"; exit 1; }
done
echo done
