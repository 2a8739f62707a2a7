#!/bin/bash
# Packed row records (LMMHIP_CREC=1) A/B: bit-identity tests, then C2 / C2 stress lines and a profile.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_engines.py -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread -k "target_ordered" > gpurun_out/pytest_crec.log 2>&1; rc=$?
tail -n 2 gpurun_out/pytest_crec.log
if [ $rc -ne 0 ]; then echo "STOP pytest rc=$rc"; grep -E "FAILED|Error|error" gpurun_out/pytest_crec.log | head -20; tail -n 30 gpurun_out/pytest_crec.log; exit $rc; fi
line() {
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py "$@" --steps 10 --warmup 2 --no-cpu-baseline --dropin-steps 0 \
    > gpurun_out/cr_$tag.json 2> gpurun_out/cr_$tag.log; local rc=$?
  if [ $rc -ne 0 ]; then echo "STOP $tag rc=$rc"; tail -n 20 gpurun_out/cr_$tag.log; exit $rc; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/cr_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'])"
}
for rep in a b; do
  line c2_base_$rep LMMHIP_CREC=0 --
  line c2_crec_$rep LMMHIP_CREC=1 --
done
line c2s_base LMMHIP_CREC=0 -- --variant stress
line c2s_crec LMMHIP_CREC=1 -- --variant stress
LMMHIP_CREC=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --dropin-steps 0 \
  --profile-json gpurun_out/cr_c2prof.json > /dev/null 2> gpurun_out/cr_c2prof.log || { echo "STOP prof"; exit 1; }
LMMHIP_CREC=0 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --dropin-steps 0 \
  --profile-json gpurun_out/cr_c2prof0.json > /dev/null 2> gpurun_out/cr_c2prof0.log || { echo "STOP prof0"; exit 1; }
echo done
