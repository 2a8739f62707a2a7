#!/bin/bash
# Round 6, fifth GPU pass: the batched saturation with 32-element chunks (LMMHIP_SATQ_CW=32: a mid-solve chunk's
# claimed variables over twice the waves) against the batch with 64-element chunks and mm_saturate_q; its bit-identity
# and C2 parity first.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.out" 2> "gpurun_out/$name.log"
  local rc=$?
  tail -c 200 "gpurun_out/$name.out"; echo
  if [ $rc -ne 0 ]; then echo "STOP $name rc=$rc"; tail -20 "gpurun_out/$name.log"; exit $rc; fi
}
echo "== tests (batch 4, cw 32)"
LMMHIP_SATQ_BATCH=4 LMMHIP_SATQ_CW=32 timeout -k 10 400 python -u -m pytest tests/test_gpu_engines.py tests/test_gpu_parity.py \
  -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06_tests_e.log 2>&1 \
  || { tail -30 gpurun_out/r06_tests_e.log; exit 1; }
tail -n 2 gpurun_out/r06_tests_e.log
for pass in 1 2; do
  step abe_c2_q_$pass 200 env LMMHIP_SATQ_BATCH=0 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --dropin-steps 0
  step abe_c2_b64_$pass 200 env LMMHIP_SATQ_BATCH=4 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --dropin-steps 0
  step abe_c2_b32_$pass 200 env LMMHIP_SATQ_BATCH=4 LMMHIP_SATQ_CW=32 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --dropin-steps 0
done
step abe_c2s_q 200 env LMMHIP_SATQ_BATCH=0 python bench.py --variant stress --steps 10 --warmup 2 --no-cpu-baseline --dropin-steps 0
step abe_c2s_b32 200 env LMMHIP_SATQ_BATCH=4 LMMHIP_SATQ_CW=32 python bench.py --variant stress --steps 10 --warmup 2 --no-cpu-baseline --dropin-steps 0
step prof_c2e 200 env LMMHIP_SATQ_BATCH=4 LMMHIP_SATQ_CW=32 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --dropin-steps 0 --profile-json gpurun_out/r06_prof_c2e.json
