#!/bin/bash
# Ready queues instead of the mm_ready pass (LMMHIP_RDQ=1): bit-identity and oracle tests with it, then C2 /
# C2 stress lines both ways and a per-launch profile.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_engines.py -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread -k "target_ordered" > gpurun_out/pytest_rdq.log 2>&1; rc=$?
tail -n 2 gpurun_out/pytest_rdq.log
if [ $rc -ne 0 ]; then echo "STOP pytest rc=$rc"; grep -E "FAILED|Error|error|assert" gpurun_out/pytest_rdq.log | head -20; exit $rc; fi
LMMHIP_RDQ=1 LMMHIP_ENGINE=rounds timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread -k "not full_size and not c5 and not fb and not fair" \
  > gpurun_out/pytest_rdq2.log 2>&1; rc=$?
tail -n 2 gpurun_out/pytest_rdq2.log
if [ $rc -ne 0 ]; then echo "STOP pytest2 rc=$rc"; grep -E "FAILED|Error|error|assert" gpurun_out/pytest_rdq2.log | head -20; exit $rc; fi
line() {
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py "$@" --steps 10 --warmup 2 --no-cpu-baseline --dropin-steps 0 \
    > gpurun_out/rq_$tag.json 2> gpurun_out/rq_$tag.log; local rc=$?
  if [ $rc -ne 0 ]; then echo "STOP $tag rc=$rc"; tail -n 20 gpurun_out/rq_$tag.log; exit $rc; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/rq_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'])"
}
for rep in a b; do
  line c2_base_$rep LMMHIP_RDQ=0 --
  line c2_rdq_$rep LMMHIP_RDQ=1 --
done
line c2s_base LMMHIP_RDQ=0 -- --variant stress
line c2s_rdq LMMHIP_RDQ=1 -- --variant stress
LMMHIP_RDQ=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --dropin-steps 0 \
  --profile-json gpurun_out/rq_c2prof.json > /dev/null 2> gpurun_out/rq_c2prof.log || { echo "STOP prof"; exit 1; }
echo done
