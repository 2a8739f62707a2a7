#!/bin/bash
# Round 6: single-address atomics drained after a grid's last wave — the init's unread alive count (8,192 atomics on one
# word per solve), the FairBottleneck work counters (one word per counter: 8,192 atomics per fb_var_inc launch, now over
# 64 slots), the saturation's per-task CTL_LASTR stores (now the update's); and the vote's ready constraints in one
# segment per vote workgroup instead of a returning add per workgroup on one queue word (LMMHIP_VOTE_SEG).  Tests, then
# same-box A/B against abl/n0 (new0: LMMHIP_VOTE_SEG=0).
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
  -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06_tests_n.log 2>&1 \
  || { tail -30 gpurun_out/r06_tests_n.log; exit 1; }
tail -n 2 gpurun_out/r06_tests_n.log
for pass in 1 2; do
  step abn_c2_n0_$pass 200 env LMM_AMD_LIB=abl/n0/liblmm_amd.so python bench.py --steps 10 --warmup 2 --no-cpu-baseline --dropin-steps 0
  step abn_c2_new0_$pass 200 env LMMHIP_VOTE_SEG=0 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --dropin-steps 0
  step abn_c2_new_$pass 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --dropin-steps 0
  step abn_c4_n0_$pass 200 env LMM_AMD_LIB=abl/n0/liblmm_amd.so python bench.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline
  step abn_c4_new_$pass 200 python bench.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline
  step abn_c5_n0_$pass 200 env LMM_AMD_LIB=abl/n0/liblmm_amd.so python bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline
  step abn_c5_new_$pass 200 python bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline
done
