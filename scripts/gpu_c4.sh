#!/bin/bash
# C4 iteration: frontier variants vs the persistent engine, and a per-launch profile of the frontier solve.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_engines.py -k "frontier" -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/c4_pytest_fr.log 2>&1; rc=$?
tail -n 1 gpurun_out/c4_pytest_fr.log
if [ $rc -ne 0 ]; then echo "STOP pytest rc=$rc"; tail -n 40 gpurun_out/c4_pytest_fr.log; exit $rc; fi
line() {
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py "$@" --steps 10 --warmup 2 --no-cpu-baseline --dropin-steps 0 \
    > gpurun_out/c4_$tag.json 2> gpurun_out/c4_$tag.log; local rc=$?
  if [ $rc -ne 0 ]; then echo "STOP $tag rc=$rc"; tail -n 20 gpurun_out/c4_$tag.log; exit $rc; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/c4_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'])"
}
line persist LMMHIP_ENGINE=persistent -- --workload c4
line fr LMMHIP_ENGINE=frontier -- --workload c4
line fr_early LMMHIP_ENGINE=frontier LMMHIP_FR_MFEARLY=1 -- --workload c4
line fr_satold LMMHIP_ENGINE=frontier LMMHIP_FR_SATOLD=1 -- --workload c4
line rounds LMMHIP_ENGINE=rounds -- --workload c4
line c2_fr LMMHIP_ENGINE=frontier --
LMMHIP_ENGINE=frontier timeout -k 10 300 python bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline \
  --profile-json gpurun_out/c4_fr_prof.json > /dev/null 2> gpurun_out/c4_fr_prof.log; rc=$?
if [ $rc -ne 0 ]; then echo "STOP prof rc=$rc"; tail -n 20 gpurun_out/c4_fr_prof.log; exit $rc; fi
echo done
