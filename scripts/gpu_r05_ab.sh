#!/bin/bash
# Round 5 same-box A/B of round-engine knobs on C2 (and its stress variant), after the bit-identity test.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_engines.py -k "target_ordered" -x -v -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/r05_ab_tests.log 2>&1; rc=$?
tail -n 4 gpurun_out/r05_ab_tests.log
if [ $rc -ne 0 ]; then echo "STOP tests rc=$rc"; grep -E "^E |Error" gpurun_out/r05_ab_tests.log | head -30; exit $rc; fi
line() {  # line <tag> <env...> -- <bench args>
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py "$@" --steps 10 --warmup 2 --no-cpu-baseline --dropin-steps 0 \
    > gpurun_out/ab5_$tag.json 2> gpurun_out/ab5_$tag.log; local rc=$?
  if [ $rc -ne 0 ]; then echo "STOP $tag rc=$rc"; tail -n 20 gpurun_out/ab5_$tag.log; exit $rc; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/ab5_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'])"
}
for pass in a b; do
line base_$pass LMMHIP_SATENT=0 --
line ent_$pass LMMHIP_SATENT=1 --
line nobits_$pass LMMHIP_VOTE_BITS=0 --
done
line base_stress LMMHIP_SATENT=0 -- --variant stress
line ent_stress LMMHIP_SATENT=1 -- --variant stress
echo done
