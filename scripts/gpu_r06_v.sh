#!/bin/bash
# Round 6: C2 mid-solve chunk length under the round hint (LMMHIP_CHUNK_MAX 32 = default, 48, 64): with no returning
# rounds after the last one, longer chunks cost only the list / compaction cadence.  Same box.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.out" 2> "gpurun_out/$name.log"
  local rc=$?
  tail -c 100 "gpurun_out/$name.out"; echo
  if [ $rc -ne 0 ]; then echo "STOP $name rc=$rc"; tail -20 "gpurun_out/$name.log"; exit $rc; fi
}
B="python bench.py --no-cpu-baseline --steps 10 --warmup 2 --dropin-steps 0"
for pass in 1 2; do
  step abv_c2_32_$pass 200 $B
  step abv_c2_48_$pass 200 env LMMHIP_CHUNK_MAX=48 $B
  step abv_c2_64_$pass 200 env LMMHIP_CHUNK_MAX=64 $B
done
echo done
