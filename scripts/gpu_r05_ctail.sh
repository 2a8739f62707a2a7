#!/bin/bash
# Round 5: short chunks near the end of the C2 solve (fewer no-op rounds queued after the last one), same box:
# LMMHIP_CHUNK_TAIL_ROWS / LMMHIP_CHUNK_TAIL_CNST thresholds with LMMHIP_CHUNK_TAIL rounds per chunk, against off;
# then the engine bit-identity and C2 parity tests with the knob on at every size.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
line() {  # line <tag> <env...>
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --dropin-steps 0 \
    > gpurun_out/ct_$tag.json 2> gpurun_out/ct_$tag.log; local rc=$?
  if [ $rc -ne 0 ]; then echo "STOP $tag rc=$rc"; tail -n 20 gpurun_out/ct_$tag.log; exit $rc; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/ct_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'], d['config']['device_rounds'])"
}
for pass in a b; do
  line base_$pass LMMHIP_X=0
  line r5e5c4_$pass LMMHIP_CHUNK_TAIL_ROWS=500000 LMMHIP_CHUNK_TAIL=4
  line r1e6c4_$pass LMMHIP_CHUNK_TAIL_ROWS=1000000 LMMHIP_CHUNK_TAIL=4
  line r1e6c8_$pass LMMHIP_CHUNK_TAIL_ROWS=1000000 LMMHIP_CHUNK_TAIL=8
  line r2e6c8_$pass LMMHIP_CHUNK_TAIL_ROWS=2000000 LMMHIP_CHUNK_TAIL=8
  line c2e4c4_$pass LMMHIP_CHUNK_TAIL_CNST=20000 LMMHIP_CHUNK_TAIL=4
  line c1e5c4_$pass LMMHIP_CHUNK_TAIL_CNST=100000 LMMHIP_CHUNK_TAIL=4
done
LMMHIP_CHUNK_TAIL_ROWS=100000000 LMMHIP_CHUNK_TAIL=4 timeout -k 10 540 python -u -m pytest tests/test_gpu_engines.py \
  tests/test_gpu_parity.py -k "bit_identical or c2 or synthetic" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  > gpurun_out/ct_tests.log 2>&1; rc=$?
tail -n 3 gpurun_out/ct_tests.log
exit $rc
