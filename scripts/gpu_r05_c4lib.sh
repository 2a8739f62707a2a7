#!/bin/bash
# Round 5: C4 with the frontier kernels before / after their per-workgroup refactor (fr_*_blk, commit 79ab1d6): the
# pre-refactor build (build_ab/liblmm_pre_frp.so, built from 53adac9) against the current one, same box.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
line() {  # line <tag> <env...> -- <bench args>
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py "$@" --steps 20 --warmup 2 --no-cpu-baseline \
    > gpurun_out/c4lib_$tag.json 2> gpurun_out/c4lib_$tag.log; local rc=$?
  if [ $rc -ne 0 ]; then echo "STOP $tag rc=$rc"; tail -n 20 gpurun_out/c4lib_$tag.log; exit $rc; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/c4lib_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'])"
}
for pass in a b c; do
line pre_$pass LMM_AMD_LIB=$GRAFT_REPO_ROOT/build_ab/liblmm_pre_frp.so -- --workload c4
line cur_$pass LMMHIP_X=0 -- --workload c4
done
line c5pre LMM_AMD_LIB=$GRAFT_REPO_ROOT/build_ab/liblmm_pre_frp.so -- --workload c5
line c5cur LMMHIP_X=0 -- --workload c5
echo done
