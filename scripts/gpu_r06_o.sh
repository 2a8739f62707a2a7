#!/bin/bash
# Round 6: host pacing by progress words written by the first vote workgroup (round engine LMMHIP_MM_AHEAD, frontier
# LMMHIP_FR_AHEAD, FairBottleneck LMMHIP_FB_PACE) instead of a control-word copy kernel + event per chunk; the round
# engine's termination test moves into the vote (mm_round_done).  Engine / configuration / parity tests, then same-box
# A/B against the chunked polls (knob = 0).
# (LMMHIP_MM_AHEAD and LMMHIP_FR_AHEAD were removed after this A/B: profiles/r06_ab.json pass O; LMMHIP_FB_PACE stays)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.out" 2> "gpurun_out/$name.log"
  local rc=$?
  tail -c 200 "gpurun_out/$name.out"; echo
  if [ $rc -ne 0 ]; then echo "STOP $name rc=$rc"; tail -20 "gpurun_out/$name.log"; exit $rc; fi
}
timeout -k 10 900 python -u -m pytest tests/test_gpu_engines.py tests/test_gpu_configs.py tests/test_gpu_parity.py \
  -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06_tests_o.log 2>&1 \
  || { tail -30 gpurun_out/r06_tests_o.log; exit 1; }
tail -n 2 gpurun_out/r06_tests_o.log
B="python bench.py --no-cpu-baseline"
for pass in 1 2; do
  step abo_c2_old_$pass 200 env LMMHIP_MM_AHEAD=0 $B --steps 10 --warmup 2 --dropin-steps 0
  step abo_c2_new_$pass 200 $B --steps 10 --warmup 2 --dropin-steps 0
  step abo_c4_old_$pass 200 env LMMHIP_FR_AHEAD=0 $B --workload c4 --steps 20 --warmup 3
  step abo_c4_new_$pass 200 $B --workload c4 --steps 20 --warmup 3
  step abo_c4_a2_$pass 200 env LMMHIP_FR_AHEAD=2 $B --workload c4 --steps 20 --warmup 3
  step abo_c4_a5_$pass 200 env LMMHIP_FR_AHEAD=5 $B --workload c4 --steps 20 --warmup 3
  step abo_c5_old_$pass 200 env LMMHIP_FB_PACE=0 $B --workload c5 --steps 10 --warmup 2
  step abo_c5_new_$pass 200 $B --workload c5 --steps 10 --warmup 2
done
step abo_c2s_old 200 env LMMHIP_MM_AHEAD=0 $B --steps 10 --warmup 2 --dropin-steps 0 --variant stress
step abo_c2s_new 200 $B --steps 10 --warmup 2 --dropin-steps 0 --variant stress
echo done
