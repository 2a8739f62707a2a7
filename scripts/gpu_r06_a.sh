#!/bin/bash
# Round 6, first GPU pass on the pruned build: the default C2 line, the product build's per-launch profile (HIP
# events), the round anatomy of rounds 70/71 (mid-solve) and 200/201 (tail) on the LMM_ANAT diagnostic build, then
# the whole -m gpu suite.  Every GPU step under its own time limit; the first failure ends the call.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.out" 2> "gpurun_out/$name.log"
  local rc=$?
  tail -c 600 "gpurun_out/$name.out"; echo
  if [ $rc -ne 0 ]; then echo "STOP $name rc=$rc"; tail -20 "gpurun_out/$name.log"; exit $rc; fi
}
step bench_c2 400 python bench.py --steps 20 --warmup 2 --cpu-reps 1 --dropin-steps 2
step prof_c2 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --dropin-steps 0 --profile-json gpurun_out/r06_prof_c2.json
step anat_c2 300 env LMM_AMD_LIB=simgrid_amd/_anat/liblmm_amd.so python scripts/anatomy.py --rounds 70,71,200,201 \
  --product-profile gpurun_out/r06_prof_c2.json --out gpurun_out/r06_c2_round_anatomy.json
echo "== pytest"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/r06_pytest_gpu.log 2>&1; rc=$?
tail -n 5 gpurun_out/r06_pytest_gpu.log
exit $rc
