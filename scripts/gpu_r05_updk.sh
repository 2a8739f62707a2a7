#!/bin/bash
# Round 5: C2 update-kernel groups per wave step A/B (same box): the in-tree build (LMM_UPD_K 2) against builds
# with 4 / 1 groups of 64 constraints in flight per wave (make OUT=../../build_ab/uk4 EXTRA_HIPFLAGS=-DLMM_UPD_K=4),
# and K=4 with 2 update workgroups per CU (LMMHIP_UPDQ_BLOCKS=512).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
line() {  # line <tag> <env...> -- <bench args>
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py "$@" --steps 10 --warmup 2 --no-cpu-baseline --dropin-steps 0 \
    > gpurun_out/bk_$tag.json 2> gpurun_out/bk_$tag.log; local rc=$?
  if [ $rc -ne 0 ]; then echo "STOP $tag rc=$rc"; tail -n 20 gpurun_out/bk_$tag.log; exit $rc; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/bk_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'])"
}
for pass in a b; do
line base_$pass LMMHIP_X=0 --
for t in uk4 uk1; do
line ${t}_$pass LMM_AMD_LIB=$GRAFT_REPO_ROOT/build_ab/$t/liblmm_amd.so --
done
line uk4u512_$pass LMM_AMD_LIB=$GRAFT_REPO_ROOT/build_ab/uk4/liblmm_amd.so LMMHIP_UPDQ_BLOCKS=512 --
done
echo done
