#!/bin/bash
# Round 6: with a round-count hint the frontier's chunks grow to LMMHIP_HINT_CHUNK_MAX rounds (default 32; 8 = the
# unhinted cap).  Frontier tests, then same-box C4 A/B over the cap and against the hint off.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.out" 2> "gpurun_out/$name.log"
  local rc=$?
  tail -c 100 "gpurun_out/$name.out"; echo
  if [ $rc -ne 0 ]; then echo "STOP $name rc=$rc"; tail -20 "gpurun_out/$name.log"; exit $rc; fi
}
timeout -k 10 900 python -u -m pytest tests/test_gpu_engines.py tests/test_gpu_configs.py -k "frontier or c4" -x -v \
  -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06_tests_s.log 2>&1 \
  || { tail -30 gpurun_out/r06_tests_s.log; exit 1; }
tail -n 2 gpurun_out/r06_tests_s.log
B="python bench.py --no-cpu-baseline --workload c4 --steps 20 --warmup 3"
for pass in 1 2 3; do
  step abs_c4_nohint_$pass 200 env LMMHIP_ROUND_HINT=0 $B
  step abs_c4_cap8_$pass 200 env LMMHIP_HINT_CHUNK_MAX=8 $B
  step abs_c4_cap16_$pass 200 env LMMHIP_HINT_CHUNK_MAX=16 $B
  step abs_c4_cap32_$pass 200 $B
  step abs_c4_cap64_$pass 200 env LMMHIP_HINT_CHUNK_MAX=64 $B
done
echo done
