#!/bin/bash
# Round 6: C2 with the round-count hint, the short tail chunks kept (default) or dropped (LMMHIP_HINT_NOTAIL=1, removed
# after this A/B: profiles/r06_ab.json pass T),
# against the hint off; C2 plain and stress, same box.
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
  step abt_c2_nohint_$pass 200 env LMMHIP_ROUND_HINT=0 $B
  step abt_c2_hint_$pass 200 $B
  step abt_c2_notail_$pass 200 env LMMHIP_HINT_NOTAIL=1 $B
  step abt_c2s_hint_$pass 200 $B --variant stress
  step abt_c2s_notail_$pass 200 env LMMHIP_HINT_NOTAIL=1 $B --variant stress
done
echo done
