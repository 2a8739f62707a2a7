#!/bin/bash
# Round 6, third GPU pass: same-box A/B (abl/base = round-5 code, abl/pipe = + saturation pipelining + wave-level
# vote queue, product = + workgroup-level vote queue), the C2 anatomy of the product build (saturation grid at 4
# workgroups per CU, the stamped build's occupancy), then the engine bit-identity, C2 parity and config tests.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.out" 2> "gpurun_out/$name.log"
  local rc=$?
  tail -c 200 "gpurun_out/$name.out"; echo
  if [ $rc -ne 0 ]; then echo "STOP $name rc=$rc"; tail -20 "gpurun_out/$name.log"; exit $rc; fi
}
for pass in 1 2; do
  for v in base pipe new; do
    lib=abl/$v/liblmm_amd.so; [ $v = new ] && lib=simgrid_amd/_lib/liblmm_amd.so
    step abc_c2_${v}_$pass 200 env LMM_AMD_LIB=$lib python bench.py --steps 10 --warmup 2 --no-cpu-baseline --dropin-steps 0
  done
done
for v in base new; do
  lib=abl/$v/liblmm_amd.so; [ $v = new ] && lib=simgrid_amd/_lib/liblmm_amd.so
  step abc_c2s_$v 200 env LMM_AMD_LIB=$lib python bench.py --variant stress --steps 10 --warmup 2 --no-cpu-baseline --dropin-steps 0
done
step prof_c2c 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --dropin-steps 0 --profile-json gpurun_out/r06_prof_c2c.json
step anat_c2c 200 env LMMHIP_SAT_BLOCKS=1024 LMM_AMD_LIB=simgrid_amd/_anat/liblmm_amd.so python scripts/anatomy.py \
  --rounds 70,71,200,201 --product-profile gpurun_out/r06_prof_c2c.json --out gpurun_out/r06_c2_round_anatomy_c.json \
  --raw gpurun_out/r06_anat_c2c.npz
echo "== tests"
timeout -k 10 700 python -u -m pytest tests/test_gpu_engines.py tests/test_gpu_parity.py tests/test_gpu_configs.py \
  tests/test_gpu_platforms.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/r06_tests_c.log 2>&1; rc=$?
tail -n 4 gpurun_out/r06_tests_c.log
exit $rc
