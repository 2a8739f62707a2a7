#!/bin/bash
# Round 6: chunk ends planned from the previous solve's round count (round engine and frontier; LMMHIP_ROUND_HINT=0:
# off) — a solve as long as the previous one runs no returning rounds after its last.  Engine / configuration /
# parity tests, then same-box A/B against the knob off.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.out" 2> "gpurun_out/$name.log"
  local rc=$?
  tail -c 100 "gpurun_out/$name.out"; echo
  if [ $rc -ne 0 ]; then echo "STOP $name rc=$rc"; tail -20 "gpurun_out/$name.log"; exit $rc; fi
}
timeout -k 10 900 python -u -m pytest tests/test_gpu_engines.py tests/test_gpu_configs.py -x -v -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/r06_tests_r.log 2>&1 || { tail -30 gpurun_out/r06_tests_r.log; exit 1; }
tail -n 2 gpurun_out/r06_tests_r.log
B="python bench.py --no-cpu-baseline"
for pass in 1 2; do
  step abr_c4_old_$pass 200 env LMMHIP_ROUND_HINT=0 $B --workload c4 --steps 20 --warmup 3
  step abr_c4_new_$pass 200 $B --workload c4 --steps 20 --warmup 3
  step abr_c2_old_$pass 200 env LMMHIP_ROUND_HINT=0 $B --steps 10 --warmup 2 --dropin-steps 0
  step abr_c2_new_$pass 200 $B --steps 10 --warmup 2 --dropin-steps 0
done
step abr_c2s_old 200 env LMMHIP_ROUND_HINT=0 $B --steps 10 --warmup 2 --dropin-steps 0 --variant stress
step abr_c2s_new 200 $B --steps 10 --warmup 2 --dropin-steps 0 --variant stress
echo done
