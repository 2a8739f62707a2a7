#!/bin/bash
# Round 5: two C2 latency levers A/B (same box), builds loaded with LMM_AMD_LIB from build_ab/:
#   sqs  (LMM_SATQ_SPEC=1): the saturation loads a candidate's ratio, CSC range and duplicate flag with its key and
#        vote count (one dependent level less);
#   vpre (LMM_VOTE_PRE=1): the vote issues its first filter step's row loads before the bitmap copy into LDS;
#   both.
# (make OUT=../../build_ab/<tag> EXTRA_HIPFLAGS=-D...), then the engine bit-identity tests with the combined build.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
line() {  # line <tag> <env...>
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --dropin-steps 0 \
    > gpurun_out/sp_$tag.json 2> gpurun_out/sp_$tag.log; local rc=$?
  if [ $rc -ne 0 ]; then echo "STOP $tag rc=$rc"; tail -n 20 gpurun_out/sp_$tag.log; exit $rc; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/sp_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'])"
}
for pass in a b; do
  line base_$pass LMMHIP_X=0
  for t in sqs vpre both; do
    line ${t}_$pass LMM_AMD_LIB=$GRAFT_REPO_ROOT/build_ab/$t/liblmm_amd.so
  done
done
LMM_AMD_LIB=$GRAFT_REPO_ROOT/build_ab/both/liblmm_amd.so timeout -k 10 540 python -u -m pytest tests/test_gpu_engines.py \
  tests/test_gpu_parity.py -k "bit_identical or c2 or synthetic" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  > gpurun_out/sp_tests.log 2>&1; rc=$?
tail -n 3 gpurun_out/sp_tests.log
exit $rc
