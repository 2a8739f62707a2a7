#!/bin/bash
# Round 6, fourth GPU pass: batched saturation (LMMHIP_SATQ_BATCH = M ready tasks' first chunks at a time) and the
# frontier saturation's chunk width (LMMHIP_FR_SATCW) — correctness first (engine bit-identity and C2 / C4 parity
# with the levers on), then same-box A/B, then the C2 anatomy with the batched saturation.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.out" 2> "gpurun_out/$name.log"
  local rc=$?
  tail -c 200 "gpurun_out/$name.out"; echo
  if [ $rc -ne 0 ]; then echo "STOP $name rc=$rc"; tail -20 "gpurun_out/$name.log"; exit $rc; fi
}
for lever in LMMHIP_SATQ_BATCH=4 LMMHIP_FR_SATCW=16; do
  echo "== tests ($lever)"
  env $lever timeout -k 10 500 python -u -m pytest tests/test_gpu_engines.py tests/test_gpu_parity.py \
    "tests/test_gpu_configs.py::test_c4_full_size_vs_oracle" -x -v -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/r06_tests_d_${lever%%=*}.log 2>&1 || { tail -30 gpurun_out/r06_tests_d_${lever%%=*}.log; exit 1; }
  tail -n 2 gpurun_out/r06_tests_d_${lever%%=*}.log
done
for pass in 1 2; do
  for m in 0 2 4; do
    step abd_c2_b${m}_$pass 200 env LMMHIP_SATQ_BATCH=$m python bench.py --steps 10 --warmup 2 --no-cpu-baseline --dropin-steps 0
  done
  for cw in 64 32 16; do
    step abd_c4_w${cw}_$pass 200 env LMMHIP_FR_SATCW=$cw python bench.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline --dropin-steps 0
  done
done
for m in 0 4; do
  step abd_c2s_b$m 200 env LMMHIP_SATQ_BATCH=$m python bench.py --variant stress --steps 10 --warmup 2 --no-cpu-baseline --dropin-steps 0
done
step prof_c2d 200 env LMMHIP_SATQ_BATCH=4 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --dropin-steps 0 --profile-json gpurun_out/r06_prof_c2d.json
step anat_c2d 200 env LMMHIP_SATQ_BATCH=4 LMM_AMD_LIB=simgrid_amd/_anat/liblmm_amd.so python scripts/anatomy.py \
  --rounds 70,71,200,201 --product-profile gpurun_out/r06_prof_c2d.json --out gpurun_out/r06_c2_round_anatomy_d.json \
  --raw gpurun_out/r06_anat_c2d.npz
