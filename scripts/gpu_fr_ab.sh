#!/bin/bash
# One GPU call: frontier bit-identity tests, C5 bit-identity tests (renumbered FairBottleneck), then C2 frontier
# variants (environment knobs) beside the round engine, C4 frontier vs persistent, C5 renumbered vs not, and a
# clean per-launch profile of the default frontier solve.  Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_engines.py -k "frontier" -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/ab_pytest_fr.log 2>&1; rc=$?
tail -n 1 gpurun_out/ab_pytest_fr.log
if [ $rc -ne 0 ]; then echo "STOP pytest rc=$rc"; tail -n 40 gpurun_out/ab_pytest_fr.log; exit $rc; fi
if [ -z "$NOC5" ]; then
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py -k "c5" -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/ab_pytest_c5.log 2>&1; rc=$?
tail -n 1 gpurun_out/ab_pytest_c5.log
if [ $rc -ne 0 ]; then echo "STOP pytest c5 rc=$rc"; tail -n 40 gpurun_out/ab_pytest_c5.log; exit $rc; fi
fi
line() {  # line <tag> <env...> -- <bench args>
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py "$@" --steps 5 --warmup 1 --no-cpu-baseline --dropin-steps 0 \
    > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.log; local rc=$?
  if [ $rc -ne 0 ]; then echo "STOP $tag rc=$rc"; tail -n 20 gpurun_out/ab_$tag.log; exit $rc; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/ab_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'])"
}
line c2_rounds LMMHIP_ENGINE=rounds --
line c2_fr LMMHIP_ENGINE=frontier --
line c2_fr_mflate LMMHIP_ENGINE=frontier LMMHIP_FR_MFEARLY=0 --
line c2_fr_sat256 LMMHIP_ENGINE=frontier LMMHIP_FR_SATB=256 --
line c2_fr_satold LMMHIP_ENGINE=frontier LMMHIP_FR_SATOLD=1 --
line c4_persist LMMHIP_ENGINE=persistent -- --workload c4
line c4_fr LMMHIP_ENGINE=frontier -- --workload c4
if [ -z "$NOC5" ]; then
line c5_renum LMMHIP_FB_RENUM=1 -- --workload c5
line c5_norenum LMMHIP_FB_RENUM=0 -- --workload c5
fi
LMMHIP_ENGINE=frontier timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --dropin-steps 0 \
  --profile-json gpurun_out/ab_fr_c2prof.json > /dev/null 2> gpurun_out/ab_fr_c2prof.log; rc=$?
if [ $rc -ne 0 ]; then echo "STOP c2prof rc=$rc"; tail -n 20 gpurun_out/ab_fr_c2prof.log; exit $rc; fi
echo done
