#!/bin/bash
# Round 6: C4 levers from the round anatomy — the frontier ready test in one dependent level with the ready
# constraints' ratio / CSC range / duplicate flag stashed in LDS, the re-vote's floor read before its slot store, and
# fr_update's state loads issued with the keys (LMMHIP_FR_UPDSPEC).  Tests first, then same-box A/B against abl/prev
# (before the tie loads) and abl/tie (tie loads, deferral off), then the C4 anatomy.
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
  > gpurun_out/r06_tests_h.log 2>&1 || { tail -30 gpurun_out/r06_tests_h.log; exit 1; }
tail -n 2 gpurun_out/r06_tests_h.log
C4="--workload c4 --steps 20 --warmup 3 --no-cpu-baseline"
for pass in 1 2; do
  step abh_c4_prev_$pass 200 env LMM_AMD_LIB=abl/prev/liblmm_amd.so python bench.py $C4
  step abh_c4_tie_$pass 200 env LMM_AMD_LIB=abl/tie/liblmm_amd.so LMMHIP_FR_DEFER=0 python bench.py $C4
  step abh_c4_nous_$pass 200 env LMMHIP_FR_UPDSPEC=0 python bench.py $C4
  step abh_c4_new_$pass 200 python bench.py $C4
done
step abh_c2_new_1 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --dropin-steps 0
step prof_c4h 200 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline --profile-json gpurun_out/r06_prof_c4h.json
step anat_c4h 200 env LMM_AMD_LIB=simgrid_amd/_anat/liblmm_amd.so python scripts/anatomy.py --workload c4 \
  --rounds 30,31,70,71 --product-profile gpurun_out/r06_prof_c4h.json --out gpurun_out/r06_c4_round_anatomy_h.json \
  --raw gpurun_out/r06_anat_c4h.npz
