#!/bin/bash
# Round 6: the frontier's slot / floor fills folded into fr_init_vars, and under a round hint the first chunk as long
# as the others (LMMHIP_HINT_CHUNK0; 2 = the short first chunk).  Frontier / engine tests, then same-box C4 A/B
# against abl/n0 (the previous commit's build).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.out" 2> "gpurun_out/$name.log"
  local rc=$?
  tail -c 100 "gpurun_out/$name.out"; echo
  if [ $rc -ne 0 ]; then echo "STOP $name rc=$rc"; tail -20 "gpurun_out/$name.log"; exit $rc; fi
}
timeout -k 10 900 python -u -m pytest tests/test_gpu_engines.py tests/test_gpu_configs.py -k "frontier or c4 or hint" \
  -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06_tests_u.log 2>&1 \
  || { tail -30 gpurun_out/r06_tests_u.log; exit 1; }
tail -n 2 gpurun_out/r06_tests_u.log
B="python bench.py --no-cpu-baseline --workload c4 --steps 20 --warmup 3"
for pass in 1 2 3; do
  step abu_c4_n0_$pass 200 env LMM_AMD_LIB=abl/n0/liblmm_amd.so $B
  step abu_c4_c02_$pass 200 env LMMHIP_HINT_CHUNK0=2 $B
  step abu_c4_new_$pass 200 $B
done
echo done
