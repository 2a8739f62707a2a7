#!/bin/bash
# Round 6: the frontier's termination word written by fr_vote itself (no mm_ctl_out per chunk) and the FairBottleneck
# rounds paced by fbk_share's progress words; the round engine's loop refactored (same launches).  Engine /
# configuration / parity tests, then same-box A/B against abl/n0 (the previous commit's build).
# (the frontier done word was removed after this A/B: profiles/r06_ab.json pass P)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.out" 2> "gpurun_out/$name.log"
  local rc=$?
  tail -c 120 "gpurun_out/$name.out"; echo
  if [ $rc -ne 0 ]; then echo "STOP $name rc=$rc"; tail -20 "gpurun_out/$name.log"; exit $rc; fi
}
timeout -k 10 900 python -u -m pytest tests/test_gpu_engines.py tests/test_gpu_configs.py tests/test_gpu_parity.py -k "c4 or c5 or frontier or fair or fb or bottleneck" \
  -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06_tests_p.log 2>&1 \
  || { tail -30 gpurun_out/r06_tests_p.log; exit 1; }
tail -n 2 gpurun_out/r06_tests_p.log
B="python bench.py --no-cpu-baseline"
O="env LMM_AMD_LIB=abl/n0/liblmm_amd.so"
for pass in 1 2; do
  step abp_c4_old_$pass 200 $O $B --workload c4 --steps 20 --warmup 3
  step abp_c4_new_$pass 200 $B --workload c4 --steps 20 --warmup 3
  step abp_c5_old_$pass 200 $O $B --workload c5 --steps 10 --warmup 2
  step abp_c5_new_$pass 200 $B --workload c5 --steps 10 --warmup 2
  step abp_c2_old_$pass 200 $O $B --steps 10 --warmup 2 --dropin-steps 0
  step abp_c2_new_$pass 200 $B --steps 10 --warmup 2 --dropin-steps 0
done
echo done
