#!/bin/bash
# Round 6: C2 chunk length 32 (default) against 64 under the round hint, plain and stress, interleaved on one box.
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
for pass in 1 2 3; do
  step abw_c2_64_$pass 200 env LMMHIP_CHUNK_MAX=64 $B
  step abw_c2_32_$pass 200 $B
done
step abw_c2s_64 200 env LMMHIP_CHUNK_MAX=64 $B --variant stress
step abw_c2s_32 200 $B --variant stress
echo done
