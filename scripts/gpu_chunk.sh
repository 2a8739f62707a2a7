#!/bin/bash
# A/B of the rounds queued per termination poll (LMMHIP_CHUNK_MAX) on C4 (frontier engine) and C2 (rounds).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
line() {
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py "$@" --steps 20 --warmup 3 --no-cpu-baseline --dropin-steps 0 \
    > gpurun_out/ch_$tag.json 2> gpurun_out/ch_$tag.log; local rc=$?
  if [ $rc -ne 0 ]; then echo "STOP $tag rc=$rc"; tail -n 20 gpurun_out/ch_$tag.log; exit $rc; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/ch_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'])"
}
for rep in a b; do
  line c4_16_$rep LMMHIP_CHUNK_MAX=16 -- --workload c4
  line c4_8_$rep LMMHIP_CHUNK_MAX=8 -- --workload c4
  line c4_4_$rep LMMHIP_CHUNK_MAX=4 -- --workload c4
done
for rep in a b; do
  line c2_16_$rep LMMHIP_CHUNK_MAX=16 --
  line c2_8_$rep LMMHIP_CHUNK_MAX=8 --
  line c2_4_$rep LMMHIP_CHUNK_MAX=4 --
done
echo done
