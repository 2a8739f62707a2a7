#!/bin/bash
# Vote bitmap copy into LDS: the default build (staggered start per workgroup, 2 loads in flight) against
# builds in simgrid_amd/_lib_* (4 in flight; the plain copy), after the engine tests of the default build.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_engines.py -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/pytest_bits.log 2>&1; rc=$?
tail -n 2 gpurun_out/pytest_bits.log
if [ $rc -ne 0 ]; then echo "STOP pytest rc=$rc"; grep -E "FAILED|Error|error" gpurun_out/pytest_bits.log | head -20; exit $rc; fi
line() {
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py "$@" --steps 10 --warmup 2 --no-cpu-baseline --dropin-steps 0 \
    > gpurun_out/bt_$tag.json 2> gpurun_out/bt_$tag.log; local rc=$?
  if [ $rc -ne 0 ]; then echo "STOP $tag rc=$rc"; tail -n 20 gpurun_out/bt_$tag.log; exit $rc; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/bt_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'])"
}
for rep in a b; do
  line s1u2_$rep X=1 --
  line s1u4_$rep LMM_AMD_LIB=simgrid_amd/_lib_s1u4/liblmm_amd.so --
  line s0u1_$rep LMM_AMD_LIB=simgrid_amd/_lib_s0u1/liblmm_amd.so --
done
line s1u2_stress X=1 -- --variant stress
line s0u1_stress LMM_AMD_LIB=simgrid_amd/_lib_s0u1/liblmm_amd.so -- --variant stress
echo done
