#!/bin/bash
# Iteration call: core parity tests, then per variant C2 / C4 bench lines, the C2 per-launch profile and
# the C4 persistent phase breakdown.  A variant is "NAME=VAL,NAME2=VAL2" environment settings ("-" =
# defaults; LMM_AMD_LIB=path selects another build).  Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_engines.py tests/test_gpu_parity.py} -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1; rc=$?
tail -n 2 gpurun_out/pytest_ab.log
if [ $rc -ne 0 ]; then echo "STOP pytest rc=$rc"; tail -n 30 gpurun_out/pytest_ab.log; exit $rc; fi
fi
i=0
for v in "$@"; do
  i=$((i+1))
  envs=""; [ "$v" != "-" ] && envs=$(echo "$v" | tr ',' ' ')
  for w in ${WL:-c2 c4}; do
    env $envs timeout -k 10 300 python bench.py --workload $w --steps 5 --warmup 1 --no-cpu-baseline --dropin-steps 0 \
      > gpurun_out/ab_${i}_$w.json 2> gpurun_out/ab_${i}_$w.log; rc=$?
    if [ $rc -ne 0 ]; then echo "STOP $v $w rc=$rc"; tail -n 20 gpurun_out/ab_${i}_$w.log; exit $rc; fi
  done
  [ -n "$NOPROF" ] && { python3 scripts/ab_summary.py "$v" $i; continue; }
  if [ -z "$NOC2PROF" ]; then
  env $envs timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --dropin-steps 0 \
    --profile-json gpurun_out/ab_${i}_c2prof.json > /dev/null 2> gpurun_out/ab_${i}_c2prof.log; rc=$?
  if [ $rc -ne 0 ]; then echo "STOP $v c2prof rc=$rc"; tail -n 20 gpurun_out/ab_${i}_c2prof.log; exit $rc; fi
  fi
  env $envs timeout -k 10 200 python scripts/diag_r2.py c4 > gpurun_out/ab_${i}_diag.log 2>&1; rc=$?
  if [ $rc -ne 0 ]; then echo "STOP $v diag rc=$rc"; tail -n 20 gpurun_out/ab_${i}_diag.log; exit $rc; fi
  python3 scripts/ab_summary.py "$v" $i
done
