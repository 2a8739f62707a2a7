#!/bin/bash
# Round 6: the frontier saturation's pushes aggregated per constraint in LDS (LMMHIP_FR_AGG) and the FairBottleneck
# chain / increment kernels' loads issued before their stores — frontier bit-identity, C4 / C5 oracle tests, then
# same-box A/B (C4: FR_AGG 0 / 1; C5: abl/tie, the build before the FB changes), then the C4 anatomy.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.out" 2> "gpurun_out/$name.log"
  local rc=$?
  tail -c 200 "gpurun_out/$name.out"; echo
  if [ $rc -ne 0 ]; then echo "STOP $name rc=$rc"; tail -20 "gpurun_out/$name.log"; exit $rc; fi
}
timeout -k 10 700 python -u -m pytest tests/test_gpu_engines.py tests/test_gpu_configs.py tests/test_gpu_platforms.py \
  -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06_tests_i.log 2>&1 \
  || { tail -30 gpurun_out/r06_tests_i.log; exit 1; }
tail -n 2 gpurun_out/r06_tests_i.log
C4="--workload c4 --steps 20 --warmup 3 --no-cpu-baseline"
C5="--workload c5 --steps 10 --warmup 2 --no-cpu-baseline"
for pass in 1 2; do
  step abi_c4_ag0_$pass 200 env LMMHIP_FR_AGG=0 python bench.py $C4
  step abi_c4_ag1_$pass 200 python bench.py $C4
  step abi_c5_tie_$pass 200 env LMM_AMD_LIB=abl/tie/liblmm_amd.so python bench.py $C5
  step abi_c5_new_$pass 200 python bench.py $C5
done
step prof_c4i 200 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline --profile-json gpurun_out/r06_prof_c4i.json
step anat_c4i 200 env LMM_AMD_LIB=simgrid_amd/_anat/liblmm_amd.so python scripts/anatomy.py --workload c4 \
  --rounds 30,31,70,71 --product-profile gpurun_out/r06_prof_c4i.json --out gpurun_out/r06_c4_round_anatomy_i.json \
  --raw gpurun_out/r06_anat_c4i.npz
