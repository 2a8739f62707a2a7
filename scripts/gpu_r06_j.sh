#!/bin/bash
# Round 6: the small systems' frontier saturation with 16 claimed-row elements per lane per pass (LMMHIP_FR_SATU16: a
# C4 chunk's pushes in one pass) — frontier bit-identity and C4 oracle tests, then same-box A/B, then the C4 anatomy.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.out" 2> "gpurun_out/$name.log"
  local rc=$?
  tail -c 200 "gpurun_out/$name.out"; echo
  if [ $rc -ne 0 ]; then echo "STOP $name rc=$rc"; tail -20 "gpurun_out/$name.log"; exit $rc; fi
}
timeout -k 10 500 python -u -m pytest tests/test_gpu_engines.py "tests/test_gpu_configs.py::test_c4_full_size_vs_oracle" \
  tests/test_gpu_platforms.py tests/test_gpu_step.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/r06_tests_j.log 2>&1 || { tail -30 gpurun_out/r06_tests_j.log; exit 1; }
tail -n 2 gpurun_out/r06_tests_j.log
C4="--workload c4 --steps 20 --warmup 3 --no-cpu-baseline"
for pass in 1 2 3; do
  step abj_c4_u8_$pass 200 env LMMHIP_FR_SATU16=0 python bench.py $C4
  step abj_c4_u16_$pass 200 python bench.py $C4
done
step prof_c4j 200 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline --profile-json gpurun_out/r06_prof_c4j.json
step anat_c4j 200 env LMM_AMD_LIB=simgrid_amd/_anat/liblmm_amd.so python scripts/anatomy.py --workload c4 \
  --rounds 30,31,70,71 --product-profile gpurun_out/r06_prof_c4j.json --out gpurun_out/r06_c4_round_anatomy_j.json \
  --raw gpurun_out/r06_anat_c4j.npz
