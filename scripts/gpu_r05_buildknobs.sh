#!/bin/bash
# Round 5: C2 build knobs A/B (same box): the in-tree build against builds with other vote-filter rows in flight
# (LMM_KFILT 4 / 16), saturation element batches (LMM_KSATU 2 / 8) and bitmap loads in flight (LMM_BITS_UNROLL 1),
# loaded with LMM_AMD_LIB from build_ab/ (built here by scripts: make EXTRA_HIPFLAGS=-D...).
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
for t in kf4 kf16 su2 su8 bu1; do
line ${t}_$pass LMM_AMD_LIB=$GRAFT_REPO_ROOT/build_ab/lib_$t.so --
done
done
echo done
