#!/bin/bash
# Round 5, after the end-of-solve chunks: the chunk cap and the compaction cadence re-checked (env knobs, same box).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
line() {  # line <tag> <env...>
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --dropin-steps 0 \
    > gpurun_out/cd_$tag.json 2> gpurun_out/cd_$tag.log; local rc=$?
  if [ $rc -ne 0 ]; then echo "STOP $tag rc=$rc"; tail -n 20 gpurun_out/cd_$tag.log; exit $rc; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/cd_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'], d['config']['device_rounds'])"
}
for pass in a b; do
  line base_$pass LMMHIP_X=0
  line cm64_$pass LMMHIP_CHUNK_MAX=64
  line ce32_$pass LMMHIP_COMPACT_EVERY=32
  line ce64_$pass LMMHIP_COMPACT_EVERY=64
done
echo done
