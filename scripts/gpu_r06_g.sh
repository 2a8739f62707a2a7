#!/bin/bash
# Round 6: the tied constraints' exact ratios loaded together (vote_row / fr_revote) and the frontier saturation's
# deferred pushes (LMMHIP_FR_DEFER, FrDefer) — engine bit-identity, C2 parity and C4 oracle tests with both on, then
# same-box A/B against abl/prev (the build before them) on C2 and C4, then the C4 anatomy of the new build.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.out" 2> "gpurun_out/$name.log"
  local rc=$?
  tail -c 200 "gpurun_out/$name.out"; echo
  if [ $rc -ne 0 ]; then echo "STOP $name rc=$rc"; tail -20 "gpurun_out/$name.log"; exit $rc; fi
}
timeout -k 10 600 python -u -m pytest tests/test_gpu_engines.py tests/test_gpu_parity.py \
  "tests/test_gpu_configs.py::test_c4_full_size_vs_oracle" tests/test_gpu_platforms.py -x -v -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/r06_tests_g.log 2>&1 || { tail -30 gpurun_out/r06_tests_g.log; exit 1; }
tail -n 2 gpurun_out/r06_tests_g.log
for pass in 1 2; do
  step abg_c2_prev_$pass 200 env LMM_AMD_LIB=abl/prev/liblmm_amd.so python bench.py --steps 10 --warmup 2 --no-cpu-baseline --dropin-steps 0
  step abg_c2_new_$pass 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --dropin-steps 0
  step abg_c4_prev_$pass 200 env LMM_AMD_LIB=abl/prev/liblmm_amd.so python bench.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline
  step abg_c4_nodf_$pass 200 env LMMHIP_FR_DEFER=0 python bench.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline
  step abg_c4_new_$pass 200 python bench.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline
done
step abg_c2s_prev 200 env LMM_AMD_LIB=abl/prev/liblmm_amd.so python bench.py --variant stress --steps 10 --warmup 2 --no-cpu-baseline --dropin-steps 0
step abg_c2s_new 200 python bench.py --variant stress --steps 10 --warmup 2 --no-cpu-baseline --dropin-steps 0
step prof_c4g 200 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline --profile-json gpurun_out/r06_prof_c4g.json
step anat_c4g 200 env LMM_AMD_LIB=simgrid_amd/_anat/liblmm_amd.so python scripts/anatomy.py --workload c4 \
  --rounds 30,31,70,71 --product-profile gpurun_out/r06_prof_c4g.json --out gpurun_out/r06_c4_round_anatomy_g.json \
  --raw gpurun_out/r06_anat_c4g.npz
