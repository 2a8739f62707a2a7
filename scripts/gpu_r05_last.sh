#!/bin/bash
# Round 5, last code (C2 grid defaults of ec5385b): every -m gpu test, smoke, then the default bench line
# (the driver's arguments), then the saturation grid cap re-swept (env knob, same box).  Each step under its own limit; stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 840 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/r05_pytest_gpu.log 2>&1; rc=$?
tail -n 3 gpurun_out/r05_pytest_gpu.log
if [ $rc -ne 0 ]; then echo "STOP pytest rc=$rc"; tail -n 60 gpurun_out/r05_pytest_gpu.log; exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" >> gpurun_out/r05_pytest_gpu.log 2>&1; rc=$?
tail -n 1 gpurun_out/r05_pytest_gpu.log
if [ $rc -ne 0 ]; then echo "STOP smoke rc=$rc"; exit $rc; fi
timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_default.json 2> gpurun_out/bench_default.log; rc=$?
tail -1 gpurun_out/bench_default.json | cut -c1-300
if [ $rc -ne 0 ]; then echo "STOP bench rc=$rc"; tail -n 20 gpurun_out/bench_default.log; exit $rc; fi
# the end-of-solve chunk knobs around the default (5 % of the variables, 4 rounds per chunk)
# (earlier in the round: the saturation grid cap LMMHIP_SAT_BLOCKS 1024 / 1536 re-swept here, default stayed)
line() {  # line <tag> <env...>
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --dropin-steps 0 \
    > gpurun_out/se_$tag.json 2> gpurun_out/se_$tag.log; local rc=$?
  if [ $rc -ne 0 ]; then echo "STOP $tag rc=$rc"; tail -n 20 gpurun_out/se_$tag.log; exit $rc; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/se_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'])"
}
for pass in a b; do
  line base_$pass LMMHIP_X=0
  line t2_$pass LMMHIP_CHUNK_TAIL=2
  line p10_$pass LMMHIP_CHUNK_TAIL_PCT=10
  line p2_$pass LMMHIP_CHUNK_TAIL_PCT=2
done
echo done
