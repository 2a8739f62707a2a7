#!/bin/bash
# Round 6: fr_vote's first queue entry loaded with the queue count (one dependent level less per re-vote, small systems)
# — frontier bit-identity and C4 oracle tests, then same-box A/B against abl/h (the build before it), then C4 anatomy.
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
  > gpurun_out/r06_tests_l.log 2>&1 || { tail -30 gpurun_out/r06_tests_l.log; exit 1; }
tail -n 2 gpurun_out/r06_tests_l.log
C4="--workload c4 --steps 20 --warmup 3 --no-cpu-baseline"
for pass in 1 2 3; do
  step abl_c4_h_$pass 200 env LMM_AMD_LIB=abl/h/liblmm_amd.so python bench.py $C4
  step abl_c4_new_$pass 200 python bench.py $C4
done
